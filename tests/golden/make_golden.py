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


# ---------------------------------------------------------------------------
# head fix-up cases at the PRODUCTION parameters (chunk_bits 20, MAX 16 MiB,
# read caps 2 MiB and 0).  A fresh Bup per chunk (file_operations.rs:748) means
# the 63 positions after a chunk start s see a window zeroed before s, unlike
# the stream-global digest G.  Random data at bits 20 has a head event once per
# ~16 000 cuts, so the cases are built, not searched for (SURVEY App. A kinds):
#   (a) a chunk-local hit at p in [s, s+62] -- the next cut is p+1, a head-hit
#       cut whose own chunk starts with a fresh window again;
#   (b) a G-hit at p in [s+1, s+62] that is NOT chunk-local -- a scan that
#       skipped the head fix-up would cut at p+1.
# s is a content cut (a G-hit), the 2 MiB read-boundary cut after a constant
# prefix (production), or a forced MAX cut (ideal).  Bytes are planted by
# solving the last two window bytes (weights 2 and 1) for the W target, as
# benchlib/workloads.py periodic_pattern does, and checking S.
# ---------------------------------------------------------------------------
W_TARGET = 0x17BF        # (124992 + W) & 0xffff == 0xffff
S_TARGET = 15            # (1984 + S) & 0xf == 0xf (1984 = 124 * 16)


def bup_hit(window, bits=20) -> bool:
    """Exact Bup edge test for the bytes of a window, oldest first (bytes
    before it read as 0): s1 = 1984 + S, s2 = 124992 + W, weight = age + 1."""
    b = np.asarray(window, np.int64)
    S = int(b.sum())
    W = int((np.arange(b.size, 0, -1) * b).sum())
    dg = ((((1984 + S) & 0xFFFF) << 16) | ((124992 + W) & 0xFFFF)) & 0xFFFFFFFF
    mask = (1 << bits) - 1
    return (dg & mask) == mask


def solve_tail(rng, b: np.ndarray, weights: np.ndarray, free: np.ndarray):
    """Re-draw the bytes b[free] (not the last two) until the last two bytes
    (weights 2, 1) can make W = W_TARGET and S = S_TARGET mod 16; returns b."""
    for _ in range(20000):
        b[free] = rng.integers(0, 256, free.size)
        rest_w = int((weights[:-2] * b[:-2]).sum())
        rest_s = int(b[:-2].sum())
        t = (W_TARGET - rest_w) % 65536                       # 2 x1 + x0 = t, 0 <= x0, x1 < 256
        if t > 765:
            continue
        for x1 in range(max(0, (t - 255 + 1) // 2), min(255, t // 2) + 1):
            x0 = t - 2 * x1
            if 0 <= x0 < 256 and (rest_s + x1 + x0) % 16 == S_TARGET:
                b[-2], b[-1] = x1, x0
                return b
    raise RuntimeError("no solution")


def plant_local(rng, d, s, L):
    """(a): bytes d[s : s+L] whose chunk-local window hits at p = s+L-1 and
    nowhere before it in the chunk."""
    for _ in range(1000):
        b = solve_tail(rng, np.zeros(L, np.int64), np.arange(L, 0, -1), np.arange(L - 2))
        if all(not bup_hit(b[:k + 1]) for k in range(L - 1)) and bup_hit(b):
            d[s:s + L] = b
            return s + L - 1
    raise RuntimeError("plant_local")


def plant_global(rng, d, s, p):
    """(b): re-draw d[s : p+1] so that the stream-global 64-byte window at p
    hits, no chunk-local position in [s, s+62] hits, and no G-hit lies in
    [s, p) (so only the head fix-up tells the true walk from a wrong one)."""
    assert s + 8 <= p <= s + 62
    for _ in range(1000):
        w = d[p - 63:p + 1].astype(np.int64)
        free = np.arange(64 - (p - s + 1), 62)                   # window slots of bytes s .. p-2
        w = solve_tail(rng, w, np.arange(64, 0, -1), free)
        d[p - 63:p + 1] = w
        ok = bup_hit(d[p - 63:p + 1]) and not bup_hit(d[s:p + 1])
        ok = ok and all(not bup_hit(d[s:q + 1]) for q in range(s, min(s + 63, d.size)))
        ok = ok and all(not bup_hit(d[q - 63:q + 1]) for q in range(s, p))
        if ok:
            return p
    raise RuntimeError("plant_global")


def first_content_cut(d, cap):
    ends = O.chunk_production(d, 20, O.MAX_CHUNK_SIZE, cap) if cap else O.chunk_ideal(d, 20, O.MAX_CHUNK_SIZE)
    for e in ends.tolist():
        if not (cap and e % cap == 0) and e % O.MAX_CHUNK_SIZE and e + 200 < d.size:
            return int(e)
    raise RuntimeError("no content cut")


def production_head_cases():
    out = []
    MX = O.MAX_CHUNK_SIZE
    rng = np.random.default_rng(4242)

    def emit(name, rec, d, cap, note):
        patch = [[int(a), d[a:b].tobytes().hex()] for a, b in spans]
        rec = dict(rec, patch=patch)
        c = case(name, rec, 20, MX, cap, note)
        data = make_input(rec)
        assert np.array_equal(data, d)
        bad = O.chunk_no_head_fixup(data, 20, MX, cap)
        assert not np.array_equal(np.array(c["ends"], np.uint64), bad), name + ": fix-up does not matter"
        out.append(c)

    for cap, tag in ((O.TOKIO_READ_CAP, "prod"), (0, "ideal")):
        for k, (kind, arg) in enumerate((("a", 63), ("a", 7), ("a", 33), ("b", 62), ("b", 20), ("aa", 45),
                                        ("ab", 50))):
            for seed in range(9_100_000 + 1000 * k + (0 if cap else 500), 9_100_000 + 1000 * k + 1000):
                rec = {"kind": "xorshift", "seed": seed, "n": 5 * M + 333}
                d = make_input(rec)
                s = first_content_cut(d, cap)
                if kind == "b":                          # the bytes before s must leave the W target reachable
                    try:
                        plant_global(rng, d.copy(), s, s + arg)
                    except RuntimeError:
                        continue
                break
            spans = []
            if kind[0] == "a":
                p = plant_local(rng, d, s, arg)
                spans.append((s, p + 1))
                assert (p + 1) in (O.chunk_production(d, 20, MX, cap) if cap else O.chunk_ideal(d, 20, MX)).tolist()
                if kind == "aa":                              # a head-hit cut followed by another
                    p2 = plant_local(rng, d, p + 1, 29)
                    spans.append((p + 1, p2 + 1))
                elif kind == "ab":                            # a head-hit cut followed by kind (b)
                    p2 = plant_global(rng, d, p + 1, p + 1 + 40)
                    spans.append((p2 - 63, p2 + 1))
            else:
                p = plant_global(rng, d, s, s + arg)
                spans.append((p - 63, p + 1))
            emit(f"adversarial_head_b20_{tag}_content_{kind}{arg}", rec, d, cap,
                 f"bits 20 / 16 MiB, read_cap {cap}: kind ({kind}) planted after the content cut at {s}")
    # after the 2 MiB read-boundary cut of a constant prefix (production grid point)
    for k, (kind, arg) in enumerate((("a", 63), ("a", 12), ("b", 62), ("b", 24))):
        rec = {"kind": "xorshift", "seed": 9_200_000 + k, "n": 6 * M + 77, "fill": [[0, 2 * M, 0x41]]}
        d = make_input(rec)
        s = 2 * M
        spans = []
        if kind == "a":
            p = plant_local(rng, d, s, arg)
            spans.append((s, p + 1))
        else:
            p = plant_global(rng, d, s, s + arg)
            spans.append((p - 63, p + 1))
        emit(f"adversarial_head_b20_prod_readcap_{kind}{arg}", rec, d, O.TOKIO_READ_CAP,
             f"bits 20 / 16 MiB / 2 MiB reads: kind ({kind}) planted after the read-boundary cut at {s}")
    # after a forced MAX cut (ideal semantics: 16 MiB of constant bytes)
    for k, (kind, arg) in enumerate((("a", 50), ("b", 50))):
        rec = {"kind": "xorshift", "seed": 9_300_000 + k, "n": MX + M + 5, "fill": [[0, MX, 0x58]]}
        d = make_input(rec)
        s = MX
        spans = []
        if kind == "a":
            p = plant_local(rng, d, s, arg)
            spans.append((s, p + 1))
        else:
            p = plant_global(rng, d, s, s + arg)
            spans.append((p - 63, p + 1))
        emit(f"adversarial_head_b20_ideal_max_{kind}{arg}", rec, d, 0,
             f"bits 20 / 16 MiB, ideal: kind ({kind}) planted after the MAX cut at {s}")
    return out


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
    cases.extend(production_head_cases())

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
