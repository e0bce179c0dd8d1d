"""Benchmark / parity-harness helpers shared by bench.py, __graft_entry__.smoke(),
tests/ and tools/.  Not part of the product (syncr_amd never imports this)."""
