#!/usr/bin/env python3
"""One-screen summary of a bench.py JSON line (the last line of the file).

    python tools/bench_summary.py gpurun_out/<tag>_bench.json
"""
import json
import sys


def main():
    d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    r = d["roofline"]
    print("value", d["value"], "ms", d["ms_per_step"], "frac", r["frac"], "kernel", r.get("kernel"),
          "traffic", r.get("traffic"), "hashed", (d.get("hashed") or {}).get("value"))
    print("parity", json.dumps(d["parity"].get("summary")))
    for k in ("uniform1k", "dedup", "dense", "dense1", "ingest", "ingest_files", "ingest_zero_copy", "shim_per_file",
              "shim_walk", "h2d_probe"):
        v = d.get(k) or {}
        if v:
            print(k, {x: v.get(x) for x in ("value", "ms_per_step", "scan_ms", "scan_frac", "step_frac", "dense_ms",
                                            "resolve_ms", "frac_of_h2d", "vs_cpu_one_thread", "latency_us", "in_walk_order",
                                            "host_stage_seconds", "error") if x in v},
                  "pipelined", {x: (v.get("pipelined") or {}).get(x) for x in ("ms_per_step", "step_frac")}
                  if v.get("pipelined") else None,
                  "parity_mism", (v.get("parity") or {}).get("mismatches"))
    s8 = d.get("shard8") or {}
    print("shard8", {x: s8.get(x) for x in ("mean_step_frac", "mean_scan_frac", "max_ms_per_step", "projected_value",
                                            "error")})
    p8 = s8.get("pipelined") or {}
    print("shard8.pipelined", {x: p8.get(x) for x in ("mean_step_frac", "max_ms_per_step", "projected_value")})
    for sh in s8.get("shards", []):
        print("   ", {x: sh.get(x) for x in ("shard", "ms_per_step", "scan_ms", "step_frac", "dense_ms", "resolve_ms")})
    print("sustained", (d.get("sustained") or {}).get("value"), "pipelined", (d.get("pipelined") or {}).get("value"))
    print("legs_seconds", d.get("legs_seconds"))


if __name__ == "__main__":
    main()
