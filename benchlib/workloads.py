"""Synthetic workloads of BASELINE.json's configs and the
per-file sharding used across GPUs.

  uniform1k  config 2: 1024 x 1 MiB random files
  zipf10k    config 3: 10 000 Zipf(1.5) files, 4 KiB..128 MiB (9.73 GiB)
             config 4: the SAME corpus LPT-sharded per file across N GPUs
             ("strong"), or N such corpora, one per GPU ("weak")
  dedup      config 5: 1000 single-edit variants of one 32 MiB random base
  dense      adversarial: the zipf10k table with periodic / constant files

Every random byte comes from the per-file xorshift64 stream of SURVEY §8d
(file i: seed 0x9E3779B97F4A7C15*(i+1), 64 outputs discarded), generated on
the device (syncr_cdc_gen_corpus) or on the host (oracle orc_corpus_fill) --
the same bytes either way, so golden digests computed on the CPU
(tests/golden/make_corpus_digests.py) check GPU results at full size.
"""
from __future__ import annotations

import heapq

import numpy as np

M = 1 << 20
ZIPF_SEED = 20251212


def zipf_sizes(n: int = 10000, seed: int = ZIPF_SEED) -> np.ndarray:
    """size_i = min(4 KiB * Z_i, 128 MiB), Z = rng.zipf(1.5)."""
    z = np.random.default_rng(seed).zipf(1.5, n).astype(np.float64)
    return np.minimum(4096.0 * z, float(128 * M)).astype(np.uint64)


# --workload dense: the zipf10k file table with adversarial contents in some
# files (the reference's own tests chunk constant data,
# tests/chunking_test.rs:95-108, and 50 MiB of 'A',
# tests/protocol_list_test.rs:360-378).  Kind per corpus index i:
DENSE_PERIODIC, DENSE_CONSTANT = 5, 11          # i % 16 == 5: 64-byte period; i % 16 == 11: one byte value


def dense_kind(i: int) -> int:
    """0 random, 1 periodic (a 64-byte pattern that hits at bits 20 once per
    period: a candidate every 64 bytes, 288 per scan tile = dense tiles), 2
    constant byte (never hits: forced MAX / read-cap cuts only)."""
    r = i % 16
    return 1 if r == DENSE_PERIODIC else (2 if r == DENSE_CONSTANT else 0)


def periodic_pattern(seed: int = ZIPF_SEED) -> np.ndarray:
    """64 bytes whose periodic extension hits the Bup edge test at chunk_bits
    20 (S = sum of the window = 15 mod 16 and W = sum of (age+1)*byte = 0x17BF
    mod 2^16) at the phase where the window is exactly the
    pattern (age 0 = pattern[63]).  Built by fixing 62 random bytes and solving
    the last two (weights 1 and 2) for the W target, then checking S."""
    rng = np.random.default_rng(seed)
    w = np.arange(64, 0, -1, dtype=np.int64)          # pattern[k] has age 63-k: weight 64-k
    for _ in range(1 << 20):
        p = rng.integers(0, 256, 64).astype(np.int64)
        rest = int((w[:62] * p[:62]).sum())
        t = (0x17BF - rest) % 65536                   # W = 0x17BF mod 2^16: (124992 + W) & 0xffff == 0xffff
        for x1 in range(256):                          # pattern[62]: weight 2, pattern[63]: weight 1
            x0 = t - 2 * x1
            if 0 <= x0 < 256:
                p[62], p[63] = x1, x0
                S = int(p.sum())
                if (1984 + S) % 16 == 15 and ((124992 + int((w * p).sum())) & 0xFFFF) == 0xFFFF:
                    return p.astype(np.uint8)
    raise RuntimeError("no periodic pattern found")


def dense_file(i: int, n: int, pat: np.ndarray | None = None) -> np.ndarray | None:
    """Bytes of dense-workload file with corpus index i and size n, or None for
    a random file (its bytes are the corpus stream)."""
    k = dense_kind(i)
    if k == 0:
        return None
    if k == 1:
        return np.resize(periodic_pattern() if pat is None else pat, n)
    return np.full(n, i & 0xFF, np.uint8)


# --workload dedup: one 32 MiB random base (corpus file
# DEDUP_BASE_INDEX of the xorshift stream, so the device generates it) and
# 1000 variants, each one edit of 1..256 bytes at a uniform offset: 50 %
# overwrite, 25 % insert, 25 % delete (seeded).
DEDUP_BASE = 32 * M
DEDUP_BASE_INDEX = 1_000_003
DEDUP_FILES = 1000


def dedup_plan(n: int = DEDUP_FILES, seed: int = ZIPF_SEED):
    """(kind, pos, len, inserted bytes, file size) of the dedup corpus's variants."""
    rng = np.random.default_rng(seed)
    plan = []
    for _ in range(n):
        pos = int(rng.integers(0, DEDUP_BASE))
        ln = int(rng.integers(1, 257))
        kind = ("overwrite", "overwrite", "insert", "delete")[int(rng.integers(0, 4))]
        ins = rng.integers(0, 256, ln, dtype=np.uint8)
        d = min(ln, DEDUP_BASE - pos)
        size = DEDUP_BASE + (ln if kind == "insert" else (-d if kind == "delete" else 0))
        plan.append((kind, pos, ln, ins, size))
    return plan


def dedup_pieces(entry) -> list[tuple[str, int, int]]:
    """A variant as consecutive pieces ("base", src offset, n) / ("ins", 0, n):
    the copies that build it from the base and the edit's bytes."""
    kind, pos, ln, _, _ = entry
    if kind == "overwrite":
        k = max(0, min(ln, DEDUP_BASE - pos))
        return [("base", 0, pos), ("ins", 0, k), ("base", pos + k, DEDUP_BASE - pos - k)]
    if kind == "insert":
        return [("base", 0, pos), ("ins", 0, ln), ("base", pos, DEDUP_BASE - pos)]
    d = min(ln, DEDUP_BASE - pos)
    return [("base", 0, pos), ("base", pos + d, DEDUP_BASE - pos - d)]


def dedup_file(base: np.ndarray, entry) -> np.ndarray:
    """One variant's bytes (host), from the same pieces the device copies."""
    ins = entry[3]
    parts = [base[o:o + n] if src == "base" else ins[:n] for src, o, n in dedup_pieces(entry)]
    return np.concatenate(parts) if parts else np.zeros(0, np.uint8)


def dedup_shift(entry) -> int:
    kind, pos, ln, _, _ = entry
    return ln if kind == "insert" else (-min(ln, DEDUP_BASE - pos) if kind == "delete" else 0)


DENSE1_BYTES = 128 * M                 # the adversarial single file (bench --workload dense1, the dense1 leg)
WORKLOADS = ("zipf10k", "uniform1k", "uniform2k", "uniform4k", "dense", "big1", "dense1", "dedup")


def workload(name: str, world: int, scaling: str = "strong"):
    """Global file table (sizes, corpus indices, description) for `world` GPUs.

    scaling "strong": ONE file set (config 3's 10 000 files for zipf10k)
    sharded per file across the ranks -- BASELINE config 4.  "weak": `world`
    copies of the file set with distinct corpus indices, one share per rank."""
    if name in ("zipf10k", "dense"):
        one = zipf_sizes()
        desc = "SURVEY §8d config 3: 10 000 Zipf(1.5) files, 4 KiB-128 MiB, 9.73 GiB"
        if name == "dense":
            desc = ("adversarial: the zipf10k file table; files i%16==5 are a 64-byte period that hits at "
                    "chunk_bits 20 every 64 bytes (dense tiles, long serial resolve chains), files i%16==11 are "
                    "one constant byte (no hits: MAX / read-cap cuts), the rest random")
    elif name == "big1":
        one = np.full(1, 128 * M, np.uint64)
        desc = "diagnostic: one 128 MiB file (the longest resolve walk of zipf10k)"
    elif name == "dense1":
        one = np.full(1, DENSE1_BYTES, np.uint64)
        desc = "diagnostic: one 128 MiB periodic-64 file (2 M chained cuts: the dense workload's longest walk)"
    elif name == "dedup":
        one = np.array([p[4] for p in dedup_plan()], np.uint64)
        desc = ("SURVEY §8d config 5: 1000 files, each one 1-256 byte edit (50 % overwrite, 25 % insert, "
                "25 % delete) of one random 32 MiB base, ~32 GiB (boundary stability in `dedup`)")
    elif name == "uniform1k":
        one = np.full(1024, M, np.uint64)
        desc = "SURVEY §8d config 2: 1024 x 1 MiB files"
    elif name in ("uniform2k", "uniform4k"):
        n = 2048 if name == "uniform2k" else 4096
        one = np.full(n, M, np.uint64)
        desc = f"diagnostic: {n} x 1 MiB files (batch-size sweep between uniform1k and zipf10k)"
    else:
        raise SystemExit(f"unknown workload {name}")
    if scaling not in ("strong", "weak"):
        raise SystemExit(f"unknown scaling {scaling}")
    if world > 1:
        if scaling == "strong":
            desc += (f"; ONE file set LPT-sharded per file across {world} GPUs (strong scaling"
                     + ("; BASELINE config 4)" if name == "zipf10k" else ")"))
        else:
            desc += (f"; {world} file sets with distinct seeds, one share per GPU (weak scaling: fixed work per "
                     "GPU)")
    sizes = one if scaling == "strong" else np.tile(one, world)
    return sizes, np.arange(sizes.size, dtype=np.uint64), desc


def lpt_shard(sizes: np.ndarray, world: int) -> list[np.ndarray]:
    """Longest-processing-time-first assignment of files to ranks."""
    order = np.argsort(-sizes.astype(np.int64), kind="stable")
    heap = [(0, r) for r in range(world)]
    parts: list[list[int]] = [[] for _ in range(world)]
    for i in order.tolist():
        load, r = heapq.heappop(heap)
        parts[r].append(i)
        heapq.heappush(heap, (load + int(sizes[i]), r))
    return [np.array(sorted(p), dtype=np.int64) for p in parts]


def offsets_of(lens: np.ndarray) -> np.ndarray:
    offs = np.zeros_like(lens)
    if lens.size:
        offs[1:] = np.cumsum(lens)[:-1]
    return offs
