"""Generate the committed golden fixtures under tests/golden/.

Provenance: the reference (Rust + the absent `rollsum ^0.3` crate) cannot be
built or run in this environment, so expected outputs come from
the CPU restatement in oracle/bup_oracle.c -- formulation (i), the literal
Bup state machine driven like compute_file_chunks / chunk_data -- and are only
written after formulation (ii) (closed form + head fix-up) agrees on every
case.  Inputs are stored as recipes (generator + seed), not raw bytes.

Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import oracle as O  # noqa: E402

M = 1 << 20


# ---------------------------------------------------------------------------
# input recipes (shared with tests/golden_inputs.py)
# ---------------------------------------------------------------------------
sys.path.insert(0, os.path.dirname(HERE))
from golden_inputs import make_input  # noqa: E402


def both_modes(data, bits, max_chunk, cap):
    prod = O.chunk_production(data, bits, max_chunk, cap) if cap else O.chunk_ideal(data, bits, max_chunk)
    cf = O.chunk_closed_form(data, bits, max_chunk, cap)
    assert np.array_equal(prod, cf), "formulations (i) and (ii) disagree"
    return prod


def case(name, recipe, bits, max_chunk, cap, note=""):
    data = make_input(recipe)
    ends = both_modes(data, bits, max_chunk, cap)
    return {"name": name, "recipe": recipe, "len": int(data.size), "chunk_bits": bits,
            "max_chunk": max_chunk, "read_cap": cap, "n_chunks": int(ends.size),
            "ends": [int(e) for e in ends], "note": note}


def main():
    cases = []
    PROD, IDEAL = O.TOKIO_READ_CAP, 0
    B, MX = O.CHUNK_BITS, O.MAX_CHUNK_SIZE
    # SURVEY Appendix A KATs (bits 20, MAX 16 MiB)
    cases.append(case("empty_prod", {"kind": "bytes", "hex": ""}, B, MX, PROD,
                      "tests/chunking_test.rs:37-43; file_operations.rs:746-747"))
    cases.append(case("small_prod", {"kind": "bytes", "hex": b"small".hex()}, B, MX, PROD,
                      "tests/protocol_list_test.rs:305-322 -> [(0,5)]"))
    for cap, tag in ((PROD, "prod"), (IDEAL, "ideal")):
        cases.append(case(f"xorshift64M_{tag}", {"kind": "xorshift", "seed": 88172645463325252, "n": 64 * M},
                          B, MX, cap, "SURVEY App. A KAT 4: 81 chunks, (0,1001954),(1001954,132287),..."))
        cases.append(case(f"xorshift64M_zero3M_{tag}",
                          {"kind": "xorshift", "seed": 88172645463325252, "n": 64 * M, "zero": [0, 3 * M]},
                          B, MX, cap, "SURVEY App. A KAT 5: ideal 76 / production 78 chunks"))
        cases.append(case(f"const_A_50M_{tag}", {"kind": "const", "byte": 65, "n": 50 * M}, B, MX, cap,
                          "SURVEY App. A KAT 3 / protocol_list_test.rs:360-378: ideal 4, production 25"))
        cases.append(case(f"const_X_100000_{tag}", {"kind": "const", "byte": 88, "n": 100000}, B, MX, cap,
                          "tests/protocol_list_test.rs:381-400"))
    cases.append(case("xorshift256M_ideal", {"kind": "xorshift", "seed": 88172645463325252, "n": 256 * M},
                      B, MX, IDEAL, "SURVEY App. A: 328 chunks"))
    # tests/chunking_test.rs inputs at its own CHUNK_BITS=13, MAX=(1<<13)*16 (:7-8), ideal semantics
    tb, tm = 13, (1 << 13) * 16
    for nm in ("deterministic", "small_file", "empty_file", "large_file", "content_shifting_1",
               "content_shifting_2", "boundaries", "binary_data", "identical_blocks", "from_file",
               "offset_progression", "modification_1", "modification_2"):
        cases.append(case(f"chunking_test_{nm}", {"kind": "chunking_test", "name": nm}, tb, tm, IDEAL,
                          "tests/chunking_test.rs input, bits 13 / MAX 128 KiB"))
    # production semantics on the same inputs (what compute_file_chunks would do with bits 13)
    for nm in ("large_file", "boundaries", "binary_data"):
        cases.append(case(f"chunking_test_{nm}_prod_b13", {"kind": "chunking_test", "name": nm}, tb, tm,
                          64 * 1024, "read_cap 64 KiB < MAX: read-boundary cuts"))
    # random data at several chunk_bits, both modes, small caps to force read-boundary cuts
    for bits in (8, 11, 13, 16, 17, 20, 24):
        for cap in (0, 3000, 65536):
            mx = max(256, (1 << bits) * 4)
            cases.append(case(f"xorshift_b{bits}_cap{cap}",
                              {"kind": "xorshift", "seed": 1000 + bits, "n": 3 * M + 12345},
                              bits, mx, cap, "random bytes"))
    # adversarial: inputs on which skipping the chunk-head fix-up changes the cuts
    found = 0
    for seed in range(1, 4000):
        if found >= 12:
            break
        bits = 9 + seed % 4
        rec = {"kind": "xorshift", "seed": 7_000_000 + seed, "n": 40000}
        d = make_input(rec)
        mx = (1 << bits) * 8
        cap = [0, 4096, 777][seed % 3]
        good = O.chunk_production(d, bits, mx, cap) if cap else O.chunk_ideal(d, bits, mx)
        bad = O.chunk_no_head_fixup(d, bits, mx, cap)
        if not np.array_equal(good, bad):
            cases.append(case(f"adversarial_head_{found}", rec, bits, mx, cap,
                              "head fix-up changes the cuts (chunk-local != file-global in [s, s+62])"))
            found += 1
    assert found >= 4, "no adversarial head cases found"

    with open(os.path.join(HERE, "kat_cases.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "oracle": "oracle/bup_oracle.c",
                   "cases": cases}, f, separators=(",", ":"))

    # 1024 x 1 MiB corpus files (production == ideal here)
    lens = np.full(1024, M, np.uint64)
    buf, offs = O.corpus_fill(lens)
    ends = O.chunk_batch(buf, offs, lens, mode=O.MODE_PRODUCTION)
    ends_cf = O.chunk_batch(buf, offs, lens, mode=O.MODE_CLOSED_FORM)
    ends_id = O.chunk_batch(buf, offs, lens, mode=O.MODE_IDEAL)
    for a, b, c in zip(ends, ends_cf, ends_id):
        assert np.array_equal(a, b) and np.array_equal(a, c)
    with open(os.path.join(HERE, "corpus_uniform_1024x1MiB.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "files": 1024, "file_len": M,
                   "seed_rule": "xorshift64 seed 0x9E3779B97F4A7C15*(i+1), 64 outputs discarded",
                   "chunk_bits": 20, "max_chunk": MX, "read_cap": PROD,
                   "ends": [[int(x) for x in e] for e in ends]}, f, separators=(",", ":"))
    print(f"{len(cases)} KAT cases, {sum(len(e) for e in ends)} corpus cuts")


if __name__ == "__main__":
    main()
