// cdc_kernels.hip -- gfx950 (MI355X, CDNA4) kernels of the Bup CDC engine.
//
// Replaces the per-byte scan of rollsum::Bup::find_chunk_edge as driven by
// compute_file_chunks (reference src/protocol/file_operations.rs:721-788).
//
// Decomposition (DESIGN.md "Algorithm"):
//   G(p)  = digest hit at p with the rolling window zeroed before the FILE
//           start: s1 = 1984 + S, s2 = 124992 + W (S = sum of the last 64
//           bytes, W = sum (age+1)*byte).  Position-local, so it is computed
//           for every byte in parallel (cdc_scan_kernel, HBM-bound).
//   A chunk starting at s sees G exactly for p >= s+63; the 63 head positions
//   need the window zeroed before s: a "head fix-up", precomputed per
//   candidate (first chunk-local hit in [e+1, e+63]) or rolled on demand.
//   Candidates are compacted into one sorted array (dense -> prefix ->
//   gather), then cdc_resolve_kernel walks compute_file_chunks' loop for each
//   file (one lane per file) applying MAX_CHUNK_SIZE and the tokio read cap.
#include <mutex>
#include <set>


#include "../../include/syncr_cdc.h"
#include "cdc_internal.h"
#include "lds_dma.h"

namespace cdc {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u16x2 as_u16x2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }

// Exact Bup edge test from window sums (digest = (s1<<16) | (s2 & 0xffff)).
__device__ __forceinline__ bool hit_exact(uint32_t S, uint32_t W, uint32_t mask) {
    const uint32_t dg = ((1984u + S) << 16) | ((124992u + W) & 0xffffu);
    return (dg & mask) == mask;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t u = __shfl_up(v, off);
        if (lane >= off) v += u;
    }
    return v;
}

// Whole-wave shifts by one lane as DPP moves (wave_shr:1 / wave_shl:1), not
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Output stores of candidate words and cuts; nt (Tables::nt_out, dev A/B
// SYNCR_CDC_NT_OUT=1): non-temporal.  Nothing re-reads them through this XCD's
// L2 before the end-of-kernel release, so streaming them past it looked free; the
// same-process A/B (order alternated, 8 rounds) says otherwise: dense1 0.2099 vs
// 0.2145 ms per step, dense 2.099 vs 2.090, shard8 / uniform1k within noise
// (profiles/r05_nt_stores_ab.jsonl).  The product stores plainly.
__device__ __forceinline__ void st_u64(uint64_t *p, uint64_t v, uint32_t nt) {
    if (nt) __builtin_nontemporal_store(v, p);
    else *p = v;
}
__device__ __forceinline__ void st_cut(DevCut *p, const DevCut &v, uint32_t nt) {
    if (nt) {
        const u32x4 w = {(uint32_t)v.offset, (uint32_t)(v.offset >> 32), v.len, v.file};
        __builtin_nontemporal_store(w, (u32x4 *)p);
    } else {
        *p = v;
    }
}

// The scans' tile / segment wait and their work grab.  Their DMAs are inline asm
// (LDS-DMA with M0), which hipcc's waitcnt tracking cannot see, so
//  - the wait is the builtin (tracked: hipcc then adds no vmcnt(0) of its own for
//    loads it believes pending across the loop -- a landing-time stall behind the
//    DMAs just issued), and the empty statement after it is the definition of the
//    grab's result `pend` for hipcc;
//  - the grab is an asm atomic of lane 0, exec set inside the statement (`on` 0:
//    no lane), run at every tile / segment so `pend` has one definition per
//    iteration and no join copy reads its register before it returned.  hipcc's
//    atomicAdd waited for the result at once (the atomic optimizer spreads it over
//    the lanes), i.e. for the DMAs issued just before it.
// Invariant (hipcc cannot see it): between the asm atomic and the next
// vmcnt(0) no instruction may read, copy or spill `pend`'s register, or the
// scan reads a stale work index.  tests/test_codeobj.py disassembles the product
// code object and checks every path from each grab to its wait, and that the
// scans spill no VGPRs; a compiler update that breaks it fails that test.
__device__ __forceinline__ void wait_all_pend(uint32_t &pend) {
    __builtin_amdgcn_s_waitcnt(0x0F70);                               // vmcnt(0)
    asm volatile("" : "+v"(pend) : : "memory");
}
__device__ __forceinline__ void grab_async(uint32_t &pend, uint32_t *ctr_word0, uint32_t on) {
    const uint32_t gm = __builtin_amdgcn_readfirstlane(on);
    uint32_t keep_lo, keep_hi;
    asm volatile("s_mov_b32 %1, exec_lo\n\t"
                 "s_mov_b32 %2, exec_hi\n\t"
                 "s_mov_b32 exec_lo, %3\n\t"
                 "s_mov_b32 exec_hi, 0\n\t"
                 "global_atomic_add %0, %4, %5, %6 offset:%7 sc0\n\t"
                 "s_mov_b32 exec_lo, %1\n\t"
                 "s_mov_b32 exec_hi, %2"
                 : "+v"(pend), "=&s"(keep_lo), "=&s"(keep_hi)
                 : "s"(gm), "v"(0u), "v"(1u), "s"(ctr_word0), "i"(CTR_CANDS_HI * 4)
                 : "memory");
}

// ds_bpermute round trips through the LDS unit: lane l gets lane l-1's value
// (up1; lane 0 gets 0) or lane l+1's (down1; lane 63 gets 0).  All lanes active.
__device__ __forceinline__ uint32_t up1(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t down1(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xf, 0xf, false);
}

__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src), hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t shfl_up64(uint64_t v, int d) {
    const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)v, d), hi = (uint32_t)__shfl_up((int)(uint32_t)(v >> 32), d);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t k) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)k);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)k);
    return ((uint64_t)hi << 32) | lo;
}

// tv = a*b + c on packed u16 pairs, pinned to ONE v_pk_mad_u16: left to itself
// hipcc re-associates two dependent mads into mul + mad + add (3 VOP3P).
__device__ __forceinline__ u16x2 pk_mad(uint32_t a, uint32_t b_uniform, u16x2 c) {
    uint32_t r;
    asm("v_pk_mad_u16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(b_uniform), "v"(as_u32(c)));
    return as_u16x2(r);
}

// min of the low 16-bit halves of three registers.  Plain C, not
// inline asm: the operands come straight from MFMA results, and only
// compiler-visible instructions get the MFMA -> VALU wait states.
__device__ __forceinline__ uint32_t min3_lo16(uint32_t a, uint32_t b, uint32_t c) {
    const unsigned short x = (unsigned short)a, y = (unsigned short)b, z = (unsigned short)c;
    return __builtin_elementwise_min(__builtin_elementwise_min(x, y), z);
}

// Scalar (s_load) read of wave-uniform, kernel-invariant metadata.  A vector
// load here would be waited with vmcnt(0), draining the in-flight tile DMA.
__device__ __forceinline__ uint64_t sload_u64(const void *p) {
    const uint64_t a = (uint64_t)p;
    // readfirstlane returns int: go through uint32_t so the low half is not sign-extended
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    const uint64_t u = ((uint64_t)hi << 32) | (uint64_t)lo;
    uint64_t v;
    asm volatile("s_nop 4\n\ts_load_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(u) : "memory");
    return v;
}

// development timeline of the scan (Tables::dbg, SYNCR_CDC_TRACE=1): lane 0
// stores a value; compiled out of the product library, a no-op without tracing
#ifdef SYNCR_CDC_DEV
#define SCAN_STAMP(T, slot, v) do { if ((T).dbg && lane == 0) (T).dbg[(slot)] = (v); } while (0)
#else
#define SCAN_STAMP(T, slot, v) do { } while (0)
#endif

// Device-clock scan timing (Tables::tscan / tacc): the first blocks dispatched stamp
// the entry (a launch's blocks start within ~1 us of each other), every wave
// that worked stamps its exit; non-returning atomics, nothing waits on them.
__device__ __forceinline__ void scan_time_entry(const Tables &T) {
    if (T.tacc && blockIdx.x < 8u && threadIdx.x == 0)
        __hip_atomic_fetch_max(&T.tscan[0], ~0ull - wall_clock64(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void scan_time_exit(const Tables &T, int lane) {
    if (T.tacc && lane == 0)
        __hip_atomic_fetch_max(&T.tscan[1], (uint64_t)wall_clock64(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// (the resolve, after the scan on the same stream) the launch's scan time into the sums
__device__ __forceinline__ void scan_time_account(const Tables &T) {
    if (T.tacc && blockIdx.x == 0 && threadIdx.x == 0) {
        const uint64_t t0 = __hip_atomic_load(&T.tscan[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t e = __hip_atomic_load(&T.tscan[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t b = ~0ull - t0;
        if (t0 && e > b) {
            T.tacc[0] += e - b;
            T.tacc[1] += 1;
        }
    }
}

__device__ __forceinline__ void record(uint32_t *wcount, uint32_t *wlist, uint32_t rel) {
    const uint32_t idx = atomicAdd(wcount, 1u);
    if (idx < (uint32_t)LISTCAP) wlist[idx] = rel;
}

// ---------------------------------------------------------------------------
// One tile of RUNS x RUN bytes.  The wave copies its two runs' bytes (plus the
// 64-byte warm-up before each) from the LDS landing buffer into registers, so
// the buffer can take the next tile's DMA while this tile is rolled.
// Lane l rolls runs l and l+64 as the two 16-bit halves of packed registers.
// Per byte pair: 1 v_perm_b32 builds the pair (A_j, B_j) once -- it is the new
// byte at j and the dropped byte at j+64 -- then
//   S += x - d      two VOP2 32-bit ops (carry-free: each half < 2^15, S >= d)
//   tv = S*k + tv; tv = d*(-64k) + tv   two v_pk_mad_u16
//   acc = min(acc, tv)                  one v_pk_min_u16
// tv = ((s2+1)*k) mod 2^16 is zero exactly when the s2 half of the mask test
// passes; a zero in a 16-byte group's minimum triggers an exact re-walk of
// that group (s1 half of the test included).
// ---------------------------------------------------------------------------
template <int RUN>
__device__ __forceinline__ uint32_t pair_at(const uint32_t (&A)[(HALO + RUN) / 4],
                                            const uint32_t (&B)[(HALO + RUN) / 4], int j) {
    return __builtin_amdgcn_perm(B[j >> 2], A[j >> 2], 0x0C040C00u + (uint32_t)(j & 3) * 0x00010001u);
}

// Dirty-group side slots (LDS, per wave): a lane whose 16-byte group minimum
// hits zero stores that group's bytes and entry state here; they are re-walked
// exactly after the roll.  Overflow hands the tile to the exact dense pass.
constexpr int DIRTYCAP = 16;
struct DirtySlot {             // 80 bytes
    uint4 xa, da, xb, db;      // new / dropped bytes of the group, runs A and B
    uint32_t S0, T0;           // packed state before the group
    uint32_t rel;              // tile-relative position of the group's first byte (run A)
    uint32_t flags;            // bit0: check A, bit1: check B
};

// Closed-form state before run position 16q (the window is the 64 bytes
// A/B words q..q+15; weights 64..1, oldest first): the packed s1 sums and
// the packed mask-test values tv.
template <int RUN>
__device__ __forceinline__ void window_state(const uint32_t (&A)[(HALO + RUN) / 4],
                                             const uint32_t (&B)[(HALO + RUN) / 4], const KParams &P,
                                             int q, uint32_t &S, u16x2 &Tv) {
    uint32_t SA = 0, WA = 0, SB = 0, WB = 0;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        const uint32_t w = 0x3D3E3F40u - 0x04040404u * (uint32_t)m;
        SA = __builtin_amdgcn_udot4(A[q + m], 0x01010101u, SA, false);
        WA = __builtin_amdgcn_udot4(A[q + m], w, WA, false);
        SB = __builtin_amdgcn_udot4(B[q + m], 0x01010101u, SB, false);
        WB = __builtin_amdgcn_udot4(B[q + m], w, WB, false);
    }
    S = SA | (SB << 16);
    const uint32_t tA = ((124993u + WA) * P.k) & 0xffffu;
    const uint32_t tB = ((124993u + WB) * P.k) & 0xffffu;
    Tv = as_u16x2(tA | (tB << 16));
}

// ROLL2: the same values with single-op dependency chains per byte pair:
// V = S - 64 d (one v_pk_mad_u16 off the T chain), then T += k V (one
// v_pk_mad_u16 on it), instead of two dependent v_pk_mad_u16 on T.
// The 16-byte group checks are two compares into lane masks each; the run
// has no branch until its end, where a wave with any dirty group recomputes
// each dirty group's entry state in closed form (window_state, from the
// bytes still in registers) and hands it to the side slots.  (A branch per
// group cost 4 more VALU per group to materialise the flags and split the
// run into basic blocks the scheduler could not interleave across.)
template <int RUN, bool ROLL2 = false, bool NOWARM = false>
__device__ __forceinline__ void roll_fast(const uint32_t (&A)[(HALO + RUN) / 4],
                                          const uint32_t (&B)[(HALO + RUN) / 4], const KParams &P,
                                          int lane, bool recA, bool recB, uint32_t *dcount,
                                          DirtySlot *dslots) {
    constexpr int NG = RUN / 16;
    uint32_t S;
    u16x2 Tv;
    if constexpr (NOWARM) {                 // development timing ablation: no closed-form warm-up
        S = 0u;
        Tv = as_u16x2(P.kk);
    } else {
        window_state<RUN>(A, B, P, 0, S, Tv);
    }
    const uint32_t want = (recA ? 1u : 0u) | (recB ? 2u : 0u);
    bool zg[NG];
    bool anyz = false;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        u16x2 acc = as_u16x2(0xffffffffu);
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
            const int i = g * 16 + jj;
            const uint32_t x = pair_at<RUN>(A, B, HALO + i), d = pair_at<RUN>(A, B, i);
            S = S + x - d;
            if constexpr (ROLL2) {
                const u16x2 V = pk_mad(d, 0xFFC0FFC0u, as_u16x2(S));   // S - 64 d (mod 2^16 per half)
                Tv = pk_mad(as_u32(V), P.kk, Tv);                       // T += k (S - 64 d)
            } else {
                Tv = pk_mad(S, P.kk, Tv);
                Tv = pk_mad(d, P.kmv, Tv);
            }
            acc = __builtin_elementwise_min(acc, Tv);
        }
        const uint32_t a = as_u32(acc);
        zg[g] = (recA && (a & 0xffffu) == 0u) || (recB && (a >> 16) == 0u);
        anyz = anyz || zg[g];
    }
    if (__builtin_expect(__ballot(anyz) != 0ull, 0)) {
        // more dirty groups than side slots (low-entropy / periodic data): the
        // tile goes to the exact dense pass anyway, so capture none of them
        // (each capture is a closed-form window_state of 64 v_dot4)
        uint32_t tot = 0;
#pragma unroll
        for (int g = 0; g < NG; ++g) tot += (uint32_t)__builtin_popcountll(__ballot(zg[g]));
        if (tot > (uint32_t)DIRTYCAP) {
            if (lane == 0) *dcount = tot;
            return;
        }
#pragma unroll
        for (int g = 0; g < NG; ++g) {
            if (zg[g]) {
                const uint32_t idx = atomicAdd(dcount, 1u);
                if (idx < (uint32_t)DIRTYCAP) {
                    uint32_t S0;
                    u16x2 T0;
                    window_state<RUN>(A, B, P, 4 * g, S0, T0);
                    DirtySlot &ds = dslots[idx];
                    ds.xa = make_uint4(A[16 + 4 * g], A[17 + 4 * g], A[18 + 4 * g], A[19 + 4 * g]);
                    ds.da = make_uint4(A[4 * g], A[1 + 4 * g], A[2 + 4 * g], A[3 + 4 * g]);
                    ds.xb = make_uint4(B[16 + 4 * g], B[17 + 4 * g], B[18 + 4 * g], B[19 + 4 * g]);
                    ds.db = make_uint4(B[4 * g], B[1 + 4 * g], B[2 + 4 * g], B[3 + 4 * g]);
                    ds.S0 = S0;
                    ds.T0 = as_u32(T0);
                    ds.rel = (uint32_t)(lane * RUN + g * 16);
                    ds.flags = want;         // the re-walk tests both halves exactly
                }
            }
        }
    }
}

#ifdef SYNCR_CDC_DEV
// The round-2 roll (development A/B only, SYNCR_CDC_ABLATE=10): a branch per
// 16-byte group that materialises the group's flags and captures its entry
// state in registers.
template <int RUN>
__device__ __forceinline__ void roll_branchy(const uint32_t (&A)[(HALO + RUN) / 4],
                                             const uint32_t (&B)[(HALO + RUN) / 4], const KParams &P,
                                             int lane, uint32_t *dcount, DirtySlot *dslots) {
    uint32_t S;
    u16x2 Tv;
    window_state<RUN>(A, B, P, 0, S, Tv);
#pragma unroll
    for (int g = 0; g < RUN / 16; ++g) {
        const uint32_t S0 = S;
        const u16x2 T0 = Tv;
        u16x2 acc = as_u16x2(0xffffffffu);
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
            const int i = g * 16 + jj;
            const uint32_t x = pair_at<RUN>(A, B, HALO + i), d = pair_at<RUN>(A, B, i);
            S = S + x - d;
            const u16x2 V = pk_mad(d, 0xFFC0FFC0u, as_u16x2(S));
            Tv = pk_mad(as_u32(V), P.kk, Tv);
            acc = __builtin_elementwise_min(acc, Tv);
        }
        const uint32_t a = as_u32(acc);
        const uint32_t zf = (((a & 0xffffu) == 0u) ? 1u : 0u) | (((a >> 16) == 0u) ? 2u : 0u);
        const bool z = zf != 0u;
        if (__builtin_expect(__ballot(z) != 0ull, 0)) {
            if (z) {
                const uint32_t idx = atomicAdd(dcount, 1u);
                if (idx < (uint32_t)DIRTYCAP) {
                    DirtySlot &ds = dslots[idx];
                    ds.xa = make_uint4(A[16 + 4 * g], A[17 + 4 * g], A[18 + 4 * g], A[19 + 4 * g]);
                    ds.da = make_uint4(A[4 * g], A[1 + 4 * g], A[2 + 4 * g], A[3 + 4 * g]);
                    ds.xb = make_uint4(B[16 + 4 * g], B[17 + 4 * g], B[18 + 4 * g], B[19 + 4 * g]);
                    ds.db = make_uint4(B[4 * g], B[1 + 4 * g], B[2 + 4 * g], B[3 + 4 * g]);
                    ds.S0 = S0;
                    ds.T0 = as_u32(T0);
                    ds.rel = (uint32_t)(lane * RUN + g * 16);
                    ds.flags = zf;
                }
            }
        }
    }
}
#endif

// Exact re-walk of the dirty groups (one lane per slot, bytes from LDS).
template <int RUN>
__device__ __forceinline__ void rewalk_dirty(const KParams &P, int lane, uint32_t nd,
                                             const DirtySlot *dslots, int64_t lim_rel,
                                             uint32_t *wcount, uint32_t *wlist) {
    if ((uint32_t)lane >= nd) return;
    const DirtySlot &ds = dslots[lane];
    const uint8_t *xa = (const uint8_t *)&ds.xa, *da = (const uint8_t *)&ds.da;
    const uint8_t *xb = (const uint8_t *)&ds.xb, *db = (const uint8_t *)&ds.db;
    const u16x2 kk = as_u16x2(P.kk), km = as_u16x2(P.kmv);
    uint32_t s = ds.S0;
    u16x2 t = as_u16x2(ds.T0);
    const uint32_t fl = ds.flags;
    const uint32_t relA = ds.rel, relB = ds.rel + 64u * RUN;
    for (int jj = 0; jj < 16; ++jj) {
        const uint32_t x = (uint32_t)xa[jj] | ((uint32_t)xb[jj] << 16);
        const uint32_t d = (uint32_t)da[jj] | ((uint32_t)db[jj] << 16);
        s = s + x - d;
        t = as_u16x2(s) * kk + t;
        t = as_u16x2(d) * km + t;
        if ((fl & 1u) && t.x == 0 && ((1984u + (s & 0xffffu)) & P.m1) == P.m1 && (int64_t)(relA + jj) < lim_rel)
            record(wcount, wlist, relA + jj);
        if ((fl & 2u) && t.y == 0 && ((1984u + (s >> 16)) & P.m1) == P.m1 && (int64_t)(relB + jj) < lim_rel)
            record(wcount, wlist, relB + jj);
    }
}

// Dense-list slots are handed to a wave DENSE_CHUNK at a time: one atomic on
// the list counter per 8 dense tiles of a wave instead of per tile (periodic
// data makes tens of thousands of dense tiles, and a single counter serialises
// them: the scan of the dense workload ran 0.2 ms longer than random data's).
// A chunk's unused slots stay DENSE_HOLE, which the dense pass and the gather
// skip.
constexpr uint32_t DENSE_CHUNK = 8;
constexpr uint32_t DENSE_HOLE = 0xffffffffu;
struct DenseSlots {
    uint32_t lo = 0, hi = 0;       // the wave's unused slots [lo, hi) (wave-uniform)
};

// The product scan defers its dense tiles' list slots: a wave keeps up to
// DPEND dense tiles in a register (lane i: the i-th) and takes their slots with
// one atomic when the register is full or the wave ends.  Taking slots at the
// tile (DenseSlots, 8 at a time) put a returning atomic on one counter in the
// roll loop: its wait also drained the next tile's DMA, and on all-dense data
// (dense1) the grid's first grabs queued on that one address (scan 81 us for
// 128 MiB, 13 us per tile; tools/scan_timeline.py).  No slot is left unused.
constexpr uint32_t DPEND = 64;
struct DensePend {
    uint32_t tile = 0;             // lane i < n: the wave's i-th pending dense tile
    uint32_t n = 0;                // (wave-uniform)
};
__device__ __forceinline__ void dense_pend_flush(const Tables &T, DensePend &dp, int lane) {
    if (dp.n == 0u) return;
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(&T.ctr[CTR_DENSE], dp.n);
    base = (uint32_t)__builtin_amdgcn_readfirstlane(base);
    if ((uint32_t)lane < dp.n) {
        const uint32_t idx = base + (uint32_t)lane;
        if (idx < T.dense_cap) {
            T.dense_list[idx] = dp.tile;
            T.tile_meta[dp.tile] = DENSE_BIT | idx;
        } else {
            T.tile_meta[dp.tile] = DENSE_BIT | 0x7fffffffu;
        }
    }
    if (lane == 0 && base + dp.n > T.dense_cap) atomicOr(&T.ctr[CTR_FLAGS], FLAG_DENSE_OVERFLOW);
    dp.n = 0u;
}
__device__ __forceinline__ void dense_mark(const Tables &T, uint32_t tile, int lane, DensePend &dp) {
    if ((uint32_t)lane == dp.n) dp.tile = tile;
    if (++dp.n == DPEND) dense_pend_flush(T, dp, lane);
}
__device__ __forceinline__ void dense_mark(const Tables &T, uint32_t tile, int lane, DenseSlots &ds) {
    if (ds.lo == ds.hi) {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(&T.ctr[CTR_DENSE], DENSE_CHUNK);
        base = (uint32_t)__builtin_amdgcn_readfirstlane(base);
        ds.lo = base;
        ds.hi = base + DENSE_CHUNK;
        if ((uint32_t)lane < DENSE_CHUNK && base + (uint32_t)lane < T.dense_cap)
            T.dense_list[base + (uint32_t)lane] = DENSE_HOLE;
    }
    const uint32_t idx = ds.lo++;
    if (lane == 0) {
        if (idx < T.dense_cap) {
            T.dense_list[idx] = tile;
            T.tile_meta[tile] = DENSE_BIT | idx;
        } else {
            T.tile_meta[tile] = DENSE_BIT | 0x7fffffffu;
            atomicOr(&T.ctr[CTR_FLAGS], FLAG_DENSE_OVERFLOW);
        }
    }
}

// Publish this tile's candidates (sorted, with head fix-ups) or mark it dense.
template <class DS>
__device__ __forceinline__ void publish_tile(const uint8_t *__restrict__ data, const KParams &P,
                                             const Tables &T, uint32_t tile, int64_t t0,
                                             uint32_t *wlist, uint32_t *wcount, int lane,
                                             bool force_dense, DS &ds) {
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    // LDS-typed read: a generic (flat) read would wait vmcnt(0) on the tile DMA.
    const uint32_t n = __builtin_amdgcn_readfirstlane(
        __hip_atomic_load((__attribute__((address_space(3))) uint32_t *)wcount, __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_WAVEFRONT));
    if (n == 0u && !force_dense) return;
    if (lane == 0) atomicOr(&T.nonempty[tile >> 6], 1ull << (tile & 63));
    if (n > (uint32_t)LISTCAP || force_dense) {
        dense_mark(T, tile, lane, ds);
        return;
    }
    const uint32_t e = (uint32_t)lane < n ? wlist[lane] : 0xffffffffu;
    uint32_t rank = 0;
    for (uint32_t m = 0; m < n; ++m) rank += wlist[m] < e;
    if ((uint32_t)lane < n) {
        // head fix-ups are computed by cdc_fix_kernel: a global load here would
        // be waited with vmcnt, which drains the in-flight tile DMA
        T.slots[(size_t)tile * LISTCAP + rank] = make_uint2(e, 0u);
    }
    if (lane == 0) {
        T.tile_meta[tile] = n;
        atomicAdd(&T.super_cnt[tile >> 6], n);
        atomicAdd(&T.coarse[(tile >> 12) * COARSE_STRIDE], n);
    }
}

// DMA of tile `tile`'s bytes [tile*TILE - HALO, tile*TILE + TILE) into the
// wave's LDS landing buffer (BUF = HALO + TILE bytes).
template <int BUF, int TILE, bool NT>
__device__ __forceinline__ void issue_buf(const uint8_t *data, uint64_t span, uint32_t tile,
                                          uint32_t lds_buf, int lane) {
    constexpr int NDMA = (BUF + 1023) / 1024;
    const int64_t base = (int64_t)tile * TILE - HALO;
    if (base >= 0 && (uint64_t)base + BUF <= span) {      // interior tile: SGPR base + lane*16
        const uint64_t b = (uint64_t)(data + base);
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
        const uint64_t ub = ((uint64_t)hi << 32) | lo;
#pragma unroll
        for (int i = 0; i < NDMA; ++i) {
            if (i < NDMA - 1 || i * 1024 + lane * 16 < BUF)
                dma16_s<NT>((uint32_t)lane * 16u, ub + (uint64_t)i * 1024u, lds_buf + (uint32_t)(i * 1024));
        }
        return;
    }
    // Edge tiles: out-of-range vectors are clamped to a valid one; their bytes
    // only feed positions outside [0, span) or before a file start (never recorded).
    const int64_t last = (int64_t)((span - 1) & ~15ull);
#pragma unroll
    for (int i = 0; i < NDMA; ++i) {
        const int off = i * 1024 + lane * 16;
        int64_t g = base + off;
        g = g < 0 ? 0 : (g > last ? last : g);
        if (i < NDMA - 1 || off < BUF) dma16<NT>(data + g, lds_buf + (uint32_t)(i * 1024));
    }
}

template <int RUN, bool NT>
__device__ __forceinline__ void issue_tile(const uint8_t *data, uint64_t span, uint32_t tile,
                                           uint32_t lds_buf, int lane) {
    issue_buf<buf_bytes(RUN), tile_bytes(RUN), NT>(data, span, tile, lds_buf, lane);
}

// ---------------------------------------------------------------------------
// Scan kernel: persistent, one wave per block, one LDS landing buffer.  Per
// tile: wait for its DMA, copy the runs into registers, hand the buffer to the
// next tile's DMA, then roll.  The DMA latency hides under the rolling of this
// tile and under the other resident waves.  The scan knows nothing about files:
// it computes G over the batch as one continuous stream.
// ---------------------------------------------------------------------------
// MODE bits 0-1: 0 is exact; 1 (staging only) and 2 (no DMA) are timing-only
// ablations, instantiated only in the development library.  Bit 2:
// non-temporal tile loads.  Bit 3: dynamic tile groups.  Bit 4: ROLL2.
// The product's scan: non-temporal tile loads (4) + dynamic tile groups (8) +
// single-op dependency chains in the roll (16; same process, zipf10k: scan
// 1.591 vs 1.640 ms, profiles/r02_ab_roll2.log).
// Bit 7 (development A/B only, SYNCR_CDC_ABLATE=11): a tile with more dirty
// groups than side slots is passed exactly by the scan wave itself
// (scan_dense_tile), with no separate dense launch.  Inlined, the pass raises
// the scan to 256 VGPRs (one wave per SIMD); out of line it needs 384 B of
// scratch per lane and 254 VGPRs; the product keeps the separate launch.
constexpr int SCAN_PRODUCT_MODE = 4 | 8 | 16;
// Small batches do not use the dynamic groups: a group of 8 tiles is ~46 us of
// one wave's roll, and below ~80-100 tiles per wave the last groups' imbalance
// costs more than the dynamic grab recovers (profiles/r02_ab_schedule.log).
// They run the CU schedule (cdc_scan_kernel<..., WPB = 8>, round 4): the static
// stride they used before left a SIMD's slow wave alone at the end (per-wave
// ends 113-229 us on uniform1k, profiles/r04b_*), the CU schedule ends every
// wave within ~30 us (profiles/r04d_*, r04f_*).  scan_dynamic() picks.
constexpr int SCAN_STATIC_MODE = 4 | 16;
constexpr uint32_t SCAN_DYN_MIN_TILES_PER_WAVE = 96;
__host__ __device__ constexpr bool scan_dynamic(uint32_t ntiles, uint32_t grid) {
    return (uint64_t)ntiles >= (uint64_t)grid * SCAN_DYN_MIN_TILES_PER_WAVE;
}
// The product's choice (round 4): stream tiles (cdc_scan_st_kernel) from 24 tiles
// (3 stream tiles) per wave, the CU schedule below.  Same-process A/B against the
// CU schedule (profiles/r04_stream_tile_shards_ab.jsonl): config 4's shards at
// N = 8 / 4 / 2 (35 / 69 / 138 tiles per wave) 0.259 vs 0.264, 0.486 vs 0.505,
// 0.881 vs 0.913 ms; uniform1k (28 per wave) 0.207 vs 0.211 once the next-ST
// grab moved off the launch contention (profiles/r04_stream_tile_uniform1k_ab.jsonl;
// 0.224 vs 0.217 before it).
constexpr uint32_t SCAN_ST_MIN_TILES_PER_WAVE = 24;
__host__ __device__ constexpr bool scan_stream_tiles(uint32_t ntiles, uint32_t grid) {
    return (uint64_t)ntiles >= (uint64_t)grid * SCAN_ST_MIN_TILES_PER_WAVE;
}

// MODE bit 5: ask for 3 waves per SIMD (VGPRs <= 168; development A/B only).
// MODE bit 6: the round-2 roll with a branch per group (development A/B only)
// WPB > 1 (the CU schedule): one workgroup of WPB waves per CU, each wave with
// its own LDS region as above.  The CU takes groups of CU_GROUP consecutive
// tiles -- its first group is its block index, later ones come from one global
// counter (T.sched, SCHED_SCAN_GROUP), fetched a group ahead -- and its waves take the group's
// tiles one at a time from an LDS counter.  The two waves of a SIMD do not run
// at the same speed (per-wave rates differ up to 2x with the same mean on every
// XCC, SE, CU and SIMD, tools/scan_timeline.py): a static share per wave ends
// with the slow waves alone on their SIMDs, a global counter per tile costs a
// fabric round trip per tile; the LDS counter balances a CU's waves for ~100
// cycles per tile and the group counter balances the CUs.
constexpr uint32_t CU_GROUP = 32;            // tiles per group
constexpr uint32_t CU_NSLOT = 8;             // group ring in LDS (local group j in slot j % CU_NSLOT)
template <int RUN>                           // (below: the scan wave's own exact pass over a dense tile)
__device__ __forceinline__ void scan_dense_tile(const uint8_t *__restrict__ data, const KParams &P,
                                                const Tables &T, uint32_t tile, int64_t t0, int lane);
template <int RUN, int MODE, int WPB = 1>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu((MODE & 32) ? 3 : 1)))
void cdc_scan_kernel(const uint8_t *__restrict__ data, KParams P, Tables T) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int BUF = buf_bytes(RUN);
    constexpr int TILE = tile_bytes(RUN);
    constexpr int NQ = (HALO + RUN) / 16;
    constexpr bool CUS = WPB > 1;
    const int lane = threadIdx.x & 63;
    const uint32_t wid = CUS ? (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : 0u;
    uint8_t *wl = smem + wid * (uint32_t)lds_wave_bytes(RUN);
    scan_time_entry(T);
    // CU schedule state after the waves' regions: the local tile counter, then
    // the group ring (u64: local group index << 32 | global group id + 1)
    typedef __attribute__((address_space(3))) uint32_t lds_u32;
    typedef __attribute__((address_space(3))) uint64_t lds_u64;
    lds_u32 *cu_next = (lds_u32 *)(smem + WPB * lds_wave_bytes(RUN));
    lds_u64 *cu_grp = (lds_u64 *)(smem + WPB * lds_wave_bytes(RUN) + 16);
    if constexpr (CUS) {
        if (threadIdx.x == 0) {
            *cu_next = (uint32_t)WPB;                                  // k < WPB: the waves' first tiles
            // LDS is not cleared between workgroups: a slot left by an earlier
            // launch on this CU can hold the very tag a wave waits for, so every
            // slot starts with a tag no group has
            for (uint32_t j = 2; j < CU_NSLOT; ++j) cu_grp[j] = ~0ull;
            cu_grp[0] = (uint64_t)blockIdx.x + 1;                     // group 0: the block's own
            const uint32_t g1 = gridDim.x + atomicAdd(&T.sched[SCHED_SCAN_GROUP * COARSE_STRIDE], 1u);
            cu_grp[1] = (1ull << 32) | ((uint64_t)g1 + 1);
        }
        __syncthreads();
    }
    DirtySlot *dslots = (DirtySlot *)(wl + BUF);                     // this wave's side slots and list
    uint32_t *wlist = (uint32_t *)(wl + BUF + DIRTYCAP * sizeof(DirtySlot));
    uint32_t *wcount = wlist + LISTCAP;
    uint32_t *dcount = wcount + 1;
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr(wl));
    const uint32_t stride = gridDim.x;
    // MODE bit 3 (DYN, the product; SYNCR_CDC_ABLATE=4 = static stride): dynamic groups of DG tiles.  Group k covers tiles
    // (k / G) * G * DG + (k % G) + i * G, i < DG (G = grid): the waves still
    // sweep the batch together as with the static stride, but a wave that
    // runs faster takes more groups.  A wave's first group is its block
    // index; later ones come from a counter (CTR_CANDS_HI is free until the
    // prefix kernel writes it), grabbed at a group's first tile so the atomic
    // completes under the roll.
    constexpr bool DYN = (MODE & 8) != 0 && !CUS;
    // zipf10k A/B (same process): groups of 4 -> 2.07 ms (one counter serialises ~69 M grabs/s), 8 -> 1.601,
    // 16 -> 1.635, 24 -> 1.651, 32 -> 1.633, 64 -> 1.669, static stride 1.657-1.694
    constexpr uint32_t DG = 8;
    auto gbase = [&](uint32_t k) { return (k / stride) * stride * DG + (k % stride); };
    uint32_t tile = blockIdx.x;
    if (!CUS && tile >= T.ntiles) return;
    const int64_t span = (int64_t)T.span;
    // CU schedule: a prefetch of local group pf_j's id is pending from this wave
    // (issued when the wave took the first tile of group pf_j - 1); it is stored
    // at the wave's next landing wait or when the wave exits, before the wave
    // itself ever waits for a group id, so no wave waits on a wave that waits
    bool pf_pending = false;
    uint32_t pf_j = 0, pf_v = 0;
    auto pf_store = [&]() {
        if (pf_pending) {
            const uint32_t g = gridDim.x + (uint32_t)__builtin_amdgcn_readfirstlane(pf_v);
            if (lane == 0)
                __hip_atomic_store(&cu_grp[pf_j % CU_NSLOT], ((uint64_t)pf_j << 32) | ((uint64_t)g + 1),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            pf_pending = false;
        }
    };
    // Group g covers the tiles (g / NB) * NB * CU_GROUP + g % NB + i * NB, i <
    // CU_GROUP (NB = the grid): the CUs sweep the batch together, each wave a
    // tile NB apart from its CU's others.  A group whose first tile lies past
    // the batch ends the CU's work (later groups start later); a tile past the
    // batch inside an earlier group is skipped.
    const uint32_t NB = gridDim.x;
    auto gtile = [&](uint32_t g, uint32_t i) -> uint64_t {
        return (uint64_t)(g / NB) * NB * CU_GROUP + g % NB + (uint64_t)i * NB;
    };
    // the tile of local index k (group j = k / CU_GROUP, id from the ring; the
    // wave's own pending prefetch is stored before it ever waits on the ring),
    // T.ntiles when the CU has no tile left, 0xffffffff for a skipped index
    auto cu_tile = [&](uint32_t k) -> uint32_t {
        const uint32_t j = k / CU_GROUP;
        uint64_t v = __hip_atomic_load(&cu_grp[j % CU_NSLOT], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if ((uint32_t)(v >> 32) != j) {
            if (pf_pending) {
                wait_vmcnt<0>();
                pf_store();
            }
            const uint64_t dl = wall_clock64() + 100000000ull;      // ~1 s: bounded, never a hang
            while ((uint32_t)(v >> 32) != j) {
                __builtin_amdgcn_s_sleep(2);
                v = __hip_atomic_load(&cu_grp[j % CU_NSLOT], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (wall_clock64() > dl) {
                    if (lane == 0) atomicOr(&T.ctr[CTR_FLAGS], FLAG_SCHED_STUCK);
                    return T.ntiles;
                }
            }
        }
        const uint32_t g = (uint32_t)v - 1u;
        if (gtile(g, 0) >= T.ntiles) return T.ntiles;
        const uint64_t t = gtile(g, k % CU_GROUP);
        return t < T.ntiles ? (uint32_t)t : 0xffffffffu;
    };
    // local index k taken: the first tile of group j fetches group j+1's id
    auto cu_took = [&](uint32_t k) {
        if (k % CU_GROUP == 0u) {
            if (pf_pending) {                                        // (one prefetch in flight per wave)
                wait_vmcnt<0>();
                pf_store();
            }
            if (lane == 0) pf_v = atomicAdd(&T.sched[SCHED_SCAN_GROUP * COARSE_STRIDE], 1u);
            pf_pending = true;
            pf_j = k / CU_GROUP + 1;
        }
    };
    if constexpr (CUS) {
        tile = (uint32_t)min<uint64_t>(gtile(blockIdx.x, wid), (uint64_t)T.ntiles);
        if (tile >= T.ntiles) {                                      // (skipped or past the batch: tiny batch)
            if (gtile(blockIdx.x, 0) >= T.ntiles) return;
            for (;;) {                                               // a later tile of the CU, if any
                uint32_t k = 0;
                if (lane == 0) k = __hip_atomic_fetch_add(cu_next, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                k = (uint32_t)__builtin_amdgcn_readfirstlane(k);
                cu_took(k);
                tile = cu_tile(k);
                if (tile != 0xffffffffu) break;
            }
            if (tile >= T.ntiles) {
                if (pf_pending) {
                    wait_vmcnt<0>();
                    pf_store();
                }
                return;
            }
        }
    }
    const uint32_t wslot = blockIdx.x * WPB + wid;                 // timeline slot of this wave (dev)
    const bool stamp = wslot < (uint32_t)DBG_SCAN_N;
    if (stamp) SCAN_STAMP(T, DBG_SCAN + 4 * wslot, wall_clock64());
    issue_tile<RUN, (MODE & 4) != 0>(data, T.span, tile, lds0, lane);
    uint32_t gj = 0, pend = 0;
    DensePend dslots_alloc;
#ifdef SYNCR_CDC_DEV
    uint32_t ntile_done = 0;
#endif
    for (uint32_t next; tile < T.ntiles; tile = next) {
        bool grabbed = false;
        uint32_t gjn = 0;
        if constexpr (DYN) {
            if (gj + 1 < DG && tile + stride < T.ntiles) {
                next = tile + stride;
                gjn = gj + 1;
            } else {
                if (gj == 0) {                                       // group ends at its first tile (last round)
                    grab_async(pend, T.ctr, 1u);
                    grabbed = true;                                  // (no second grab below: it would drop a group)
                }
                wait_all_pend(pend);                                 // the grab
                next = gbase(stride + (uint32_t)__builtin_amdgcn_readfirstlane(pend));
                gjn = 0;
            }
        } else if constexpr (!CUS) {
            next = tile + stride;
        }
        const int64_t t0 = (int64_t)tile * TILE;
        if (lane == 0) { *wcount = 0u; *dcount = 0u; }
        if constexpr (DYN) wait_all_pend(pend);                      // this tile has landed (and the group grab)
        else wait_vmcnt<0>();
        uint32_t nk = 0;
        if constexpr (CUS) {                                         // the CU's next tile (read after the runs)
            pf_store();
            if (lane == 0) nk = __hip_atomic_fetch_add(cu_next, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
#ifdef SYNCR_CDC_DEV
        if (stamp && ntile_done == 0) SCAN_STAMP(T, DBG_SCAN + 4 * wslot + 1, wall_clock64());
        if (wslot < (uint32_t)DBG_TILE_W && ntile_done < (uint32_t)DBG_TILE_N)
            SCAN_STAMP(T, DBG_TILE + DBG_TILE_N * wslot + ntile_done, wall_clock64());
        ++ntile_done;
#endif
        uint32_t A[NQ * 4], B[NQ * 4];
        {
            const uint4 *la = (const uint4 *)(wl + lane * RUN);          // = run start - 64
            const uint4 *lb = (const uint4 *)(wl + (lane + 64) * RUN);
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                if ((MODE & 512) != 0 && q < HALO / 16) {         // development timing ablation: no halo
                    A[4 * q + 0] = A[4 * q + 1] = A[4 * q + 2] = A[4 * q + 3] = 0u;
                    B[4 * q + 0] = B[4 * q + 1] = B[4 * q + 2] = B[4 * q + 3] = 0u;
                    continue;
                }
                const uint4 a = la[q], b = lb[q];
                A[4 * q + 0] = a.x; A[4 * q + 1] = a.y; A[4 * q + 2] = a.z; A[4 * q + 3] = a.w;
                B[4 * q + 0] = b.x; B[4 * q + 1] = b.y; B[4 * q + 2] = b.z; B[4 * q + 3] = b.w;
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");           // runs are in registers
        if constexpr (CUS) {
            uint32_t k = (uint32_t)__builtin_amdgcn_readfirstlane(nk);
            for (;;) {
                cu_took(k);
                next = cu_tile(k);
                if (next != 0xffffffffu) break;
                if (lane == 0) k = __hip_atomic_fetch_add(cu_next, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                k = (uint32_t)__builtin_amdgcn_readfirstlane(k);
            }
        }
        if (next < T.ntiles && (MODE & 3) != 2) issue_tile<RUN, (MODE & 4) != 0>(data, T.span, next, lds0, lane);
        if constexpr (DYN) {
            grab_async(pend, T.ctr, (gj == 0 && !grabbed) ? 1u : 0u);  // read at the group's last tile
            gj = gjn;
        }
        if constexpr ((MODE & 3) == 1) {                                   // diagnostics: staging only
#pragma unroll
            for (int q = 0; q < NQ * 4; ++q) asm volatile("" ::"v"(A[q]), "v"(B[q]));
            continue;
        }
        const int64_t lim_rel = span - t0;                           // positions >= span are not bytes
#ifdef SYNCR_CDC_DEV
        if constexpr ((MODE & 64) != 0) roll_branchy<RUN>(A, B, P, lane, dcount, dslots); else
#endif
        roll_fast<RUN, (MODE & 16) != 0, (MODE & 256) != 0>(A, B, P, lane, true, true, dcount, dslots);
        if constexpr ((MODE & 3) == 2) continue;                          // diagnostics: rolling only
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        const uint32_t nd = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load((__attribute__((address_space(3))) uint32_t *)dcount, __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_WAVEFRONT));
        if constexpr ((MODE & 128) != 0) {                          // dense tile: exact pass right here
            if (__builtin_expect(nd > (uint32_t)DIRTYCAP, 0)) {
                scan_dense_tile<RUN>(data, P, T, tile, t0, lane);
                continue;
            }
        }
        if (nd && nd <= (uint32_t)DIRTYCAP) rewalk_dirty<RUN>(P, lane, nd, dslots, lim_rel, wcount, wlist);
        publish_tile(data, P, T, tile, t0, wlist, wcount, lane, nd > (uint32_t)DIRTYCAP, dslots_alloc);
    }
    dense_pend_flush(T, dslots_alloc, lane);
    if constexpr (CUS) {
        if (pf_pending) {                                            // readers may wait for it
            wait_vmcnt<0>();
            pf_store();
        }
    }
    scan_time_exit(T, lane);
#ifdef SYNCR_CDC_DEV
    if (stamp) {
        // where the wave ran: HW_ID (wave, SIMD, CU, SH, SE) and the XCC id
        uint32_t hwid, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)\n\ts_getreg_b32 %1, hwreg(HW_REG_XCC_ID)"
                     : "=s"(hwid), "=s"(xcc));
        SCAN_STAMP(T, DBG_SCAN + 4 * wslot + 2, wall_clock64());
        SCAN_STAMP(T, DBG_SCAN + 4 * wslot + 3,
                   (uint64_t)ntile_done | ((uint64_t)hwid << 32) | ((uint64_t)(xcc & 0xf) << 28));
    }
#endif
}

// ---------------------------------------------------------------------------
// Stream-tile scan (round 4): the rolling window carries over between segments.
//
// The warm-up of every 144-byte run of cdc_scan_kernel (64 v_dot4 for S and W
// of the 64 bytes before it, 64 v_perm for their pairs, 208 bytes of LDS read
// per 144 rolled) is ~13 % of the roll's VALU work, and in the shader-clock dip
// the scan is VALU / energy bound: the same scan without warm-up and halo ran
// 8-10 % faster in the driver's window (timing-only ablations,
// profiles/r04a_dip_ablation.jsonl).  A stream tile (ST) is 8 consecutive tiles
// (147 456 bytes) cut into 128 STREAMS of ST_SEGS segments of 128 bytes (stream
// s = bytes [1152 s, 1152 (s + 1)) of the ST; lane l owns streams l and l + 64,
// packed as in roll_fast).  Iteration g rolls segment g of every stream: its
// bytes land in LDS by LDS-DMA, one whole 128-byte line per stream (segments are
// line-aligned: a 144-byte segment straddled lines, and the nt policy re-read
// the shared lines from HBM, 1.7x slower); the window's state (S, T) and the
// 64 packed byte pairs it drops next (Pd) stay in registers from segment g - 1.
// Only segment 0 warms up (closed form) from the 64 bytes before each stream,
// loaded into registers an iteration ahead.  Tile t of the ST = streams
// 16 t .. 16 t + 15 = one 18 432-byte tile of the batch: the bookkeeping is the
// scan's, each tile's candidates collected over the segments and published
// when the ST ends.  LDS: piece q (16 B) of stream s sits at 16-byte slot
// 8 s + (q ^ (s & 7)) (an XOR swizzle: a lane-stride of 128 B would put every
// lane of a ds_read_b128 group in the same banks).  A dirty group is captured
// right after it is rolled, from the packed pairs it added and dropped (still
// in registers then) and its entry state.
// ---------------------------------------------------------------------------
constexpr int ST_RUN = 128;                   // bytes per segment and stream (ST_SEGS of them: 1152-byte streams)
constexpr int ST_LISTCAP = 32;                // candidate slots per tile (more: dense); 16 from 36 segments
__host__ __device__ constexpr int st_listcap(int segs) { return segs >= 36 ? 16 : ST_LISTCAP; }
constexpr int ST_DIRTYCAP = 6;                // side slots per segment
// ST geometry by segments per stream: 9 (1152-byte streams, 16 per batch tile, 8
// tiles per ST) or 18 (2304-byte streams, 16 tiles per ST: half the stream
// starts, so half the warm-ups, halo re-reads and ST switches per byte)
__host__ __device__ constexpr int st_tiles(int segs) { return segs * 8 / 9; }
static_assert(16 * ST_SEGS * ST_RUN == tile_bytes(DEFAULT_RUN), "16 streams of 9 segments = one batch tile");
static_assert(st_tiles(ST_SEGS) == ST_TILES && st_tiles(18) == 16 && st_tiles(27) == 24 && st_tiles(36) == 32,
              "ST geometry");
struct DirtySlotST {                          // 144 bytes
    uint32_t dp[16];                          // dropped bytes, packed pairs (run A low, run B high)
    uint32_t xp[16];                          // new bytes, packed pairs
    uint32_t S0, T0;                          // packed state before the group
    uint32_t relA;                            // ST-relative position of the group's first byte, run A
    uint32_t pad;
};
static_assert(sizeof(DirtySlotST) == 144, "slot size");
__host__ __device__ constexpr int st_lds_bytes(int segs) {
    return RUNS * ST_RUN + ST_DIRTYCAP * (int)sizeof(DirtySlotST) + st_tiles(segs) * st_listcap(segs) * 4 +
           st_tiles(segs) * 4 + 16;
}

__device__ __forceinline__ uint32_t xpair32(const uint32_t (&XA)[ST_RUN / 4], const uint32_t (&XB)[ST_RUN / 4], int j) {
    return __builtin_amdgcn_perm(XB[j >> 2], XA[j >> 2], 0x0C040C00u + (uint32_t)(j & 3) * 0x00010001u);
}

// Publish one tile's list (n candidates, tile-relative positions) or mark it dense.
template <class DS>
__device__ __forceinline__ void publish_list(const Tables &T, uint32_t tile, const uint32_t *list, uint32_t n,
                                             int lane, bool force_dense, DS &ds, uint32_t cap = ST_LISTCAP) {
    if (n == 0u && !force_dense) return;
    if (lane == 0) atomicOr(&T.nonempty[tile >> 6], 1ull << (tile & 63));
    if (n > cap || force_dense) {
        dense_mark(T, tile, lane, ds);
        return;
    }
    const uint32_t e = (uint32_t)lane < n ? list[lane] : 0xffffffffu;
    uint32_t rank = 0;
    for (uint32_t m = 0; m < n; ++m) rank += list[m] < e;
    if ((uint32_t)lane < n) T.slots[(size_t)tile * LISTCAP + rank] = make_uint2(e, 0u);
    if (lane == 0) {
        T.tile_meta[tile] = n;
        atomicAdd(&T.super_cnt[tile >> 6], n);
        atomicAdd(&T.coarse[(tile >> 12) * COARSE_STRIDE], n);
    }
}

template <int MODE, int SEGS = ST_SEGS>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2)))
void cdc_scan_st_kernel(const uint8_t *__restrict__ data, KParams P, Tables T) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int RUN = ST_RUN;
    constexpr int NW = RUN / 4;                  // words per segment and run
    constexpr int NG = RUN / 16;                 // 16-byte groups per segment
    constexpr int TILES = st_tiles(SEGS);        // batch tiles per ST
    constexpr uint32_t L = SEGS * ST_RUN;        // stream bytes
    constexpr int LC = st_listcap(SEGS);         // candidate slots per tile in LDS
    constexpr uint32_t STB = RUNS * L;           // ST bytes
    constexpr int NDMA = RUNS * RUN / 1024;      // DMA instructions per segment (8 streams each)
    const int lane = threadIdx.x;
    uint8_t *wl = smem;
    DirtySlotST *dslots = (DirtySlotST *)(smem + RUNS * RUN);
    uint32_t *tlist = (uint32_t *)(smem + RUNS * RUN + ST_DIRTYCAP * sizeof(DirtySlotST));
    uint32_t *tcnt = tlist + TILES * LC;
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr(wl));
    const uint32_t nst = T.nst;
    // the grid size in a register for the loop (read from the dispatch packet by a
    // scalar load and an lgkmcnt(0) wait at every segment otherwise)
    uint32_t grid = gridDim.x;
    asm volatile("" : "+s"(grid));
    const bool multi = nst > grid;                 // more STs than waves: the counter hands out the rest
    const int64_t span = (int64_t)T.span;
    // DMA instruction i, lane l fills slot 64 i + l = stream 8 i + l / 8, physical piece l % 8,
    // which holds logical piece (l % 8) ^ ((l / 8) & 7): a per-lane offset fixed for the kernel
    const uint32_t dmaoff = ((uint32_t)lane >> 3) * L + ((((uint32_t)lane & 7u) ^ (((uint32_t)lane >> 3) & 7u)) << 4);
    // this lane's stream (l) reads its piece q at byte 128 l + 16 (q ^ (l & 7)); stream l + 64 at + 8192
    const uint32_t rbase = (uint32_t)lane * RUN, rsw = ((uint32_t)lane & 7u) << 4;
    auto issue_seg = [&](uint32_t st, uint32_t g) {
        const uint64_t b0 = (uint64_t)st * STB + (uint64_t)g * RUN;
        if ((uint64_t)st * STB + STB <= (uint64_t)span) {            // whole ST inside the batch
#pragma unroll
            for (int i = 0; i < NDMA; ++i) {
                const uint64_t sb = (uint64_t)(data + b0 + (uint64_t)i * 8u * L);
                const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)sb);
                const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(sb >> 32));
                dma16_s<(MODE & 4) != 0>(dmaoff, ((uint64_t)hi << 32) | lo, lds0 + 1024u * (uint32_t)i);
            }
        } else {                                 // the batch's last ST: clamp (bytes past it are never recorded)
            const int64_t last = (int64_t)((span - 1) & ~15ll);
#pragma unroll
            for (int i = 0; i < NDMA; ++i) {
                uint32_t o = dmaoff;
                asm volatile("" : "+v"(o));          // keep the 16 lane addresses out of the hot loop's registers
                int64_t a = (int64_t)b0 + (int64_t)i * 8 * L + o;
                a = a > last ? last : a;
                dma16<(MODE & 4) != 0>(data + a, lds0 + 1024u * (uint32_t)i);
            }
        }
    };
    // the 64 bytes before each of this lane's two streams (the stream's warm-up)
    uint32_t HA[16], HB[16];
    auto load_halo = [&](uint32_t st) {
        const int64_t sa = (int64_t)st * STB + (int64_t)lane * L - 64, sbb = sa + 64 * (int64_t)L;
        if (st != 0u && (uint64_t)st * STB + STB <= (uint64_t)span) {
            // (wave-uniform) every halo of the ST lies inside the batch: no per-load bounds
            // (the checked form below is ~50 VALU per ST)
            const uint4 *pa = (const uint4 *)(data + sa), *pb = (const uint4 *)(data + sbb);
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const uint4 va = pa[m], vb = pb[m];
                HA[4 * m] = va.x; HA[4 * m + 1] = va.y; HA[4 * m + 2] = va.z; HA[4 * m + 3] = va.w;
                HB[4 * m] = vb.x; HB[4 * m + 1] = vb.y; HB[4 * m + 2] = vb.z; HB[4 * m + 3] = vb.w;
            }
            return;
        }
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            uint4 va, vb;
            const int64_t a = sa + 16 * m, b = sbb + 16 * m;
            if (a >= 0 && a + 16 <= span) va = *(const uint4 *)(data + a); else va = make_uint4(0, 0, 0, 0);
            if (b >= 0 && b + 16 <= span) vb = *(const uint4 *)(data + b); else vb = make_uint4(0, 0, 0, 0);
            HA[4 * m] = va.x; HA[4 * m + 1] = va.y; HA[4 * m + 2] = va.z; HA[4 * m + 3] = va.w;
            HB[4 * m] = vb.x; HB[4 * m + 1] = vb.y; HB[4 * m + 2] = vb.z; HB[4 * m + 3] = vb.w;
        }
    };
    scan_time_entry(T);
    if (blockIdx.x >= nst) return;
    uint32_t st = blockIdx.x;
    const bool stamp = blockIdx.x < (uint32_t)DBG_SCAN_N;              // timeline slot (dev)
    if (stamp) SCAN_STAMP(T, DBG_SCAN + 4 * blockIdx.x, wall_clock64());
#ifdef SYNCR_CDC_DEV
    uint32_t nst_done = 0, seg_done = 0;
#endif
    issue_seg(st, 0);
    load_halo(st);
    uint32_t pend = 0, nextst = 0;
    uint32_t nth = 0;                              // this wave's STs so far (wave-uniform)
    DensePend dslots_alloc;
    // (a ping-pong of two carried arrays, segments unrolled in pairs to drop the 64 moves
    // below, measured slower: 3 copies of the roll overflow the instruction cache)
    uint32_t Pd[64];                               // packed pairs the window drops at positions 0..63
    uint32_t Sc = 0;                               // carried state
    u16x2 Tc = as_u16x2(0u);
    uint32_t dmark = 0;                            // tiles (bit t) holding a dirty group no slot took
    for (;;) {
#pragma unroll 1
        for (uint32_t g = 0; g < (uint32_t)SEGS; ++g) {
            const bool first = g == 0u;
            if (first && lane < TILES) tcnt[lane] = 0u;
            uint32_t have = 0;                                       // dirty slots taken (wave-uniform)
#ifdef SYNCR_CDC_DEV
            // every segment of the first DBG_TILE_W waves: arrival at the wait (bit 55) and
            // landing (unit switches vs. steady segments; processing vs. waiting)
            if (blockIdx.x < (uint32_t)DBG_TILE_W && seg_done + 1 < (uint32_t)DBG_TILE_N)
                SCAN_STAMP(T, DBG_TILE + DBG_TILE_N * blockIdx.x + seg_done,
                           wall_clock64() | ((uint64_t)g << 56) | (1ull << 55));
#endif
            wait_all_pend(pend);                                     // segment g landed (and, at 0, the halo)
#ifdef SYNCR_CDC_DEV
            if (stamp && first && nst_done == 0) SCAN_STAMP(T, DBG_SCAN + 4 * blockIdx.x + 1, wall_clock64());
            if (blockIdx.x < (uint32_t)DBG_TILE_W && seg_done + 1 < (uint32_t)DBG_TILE_N)
                SCAN_STAMP(T, DBG_TILE + DBG_TILE_N * blockIdx.x + seg_done + 1, wall_clock64() | ((uint64_t)g << 56));
            seg_done += 2;
#endif
            if (first) {                                             // warm-up from the halo (closed form)
                uint32_t SA = 0, WA = 0, SB = 0, WB = 0;
#pragma unroll
                for (int m = 0; m < 16; ++m) {
                    const uint32_t w = 0x3D3E3F40u - 0x04040404u * (uint32_t)m;
                    SA = __builtin_amdgcn_udot4(HA[m], 0x01010101u, SA, false);
                    WA = __builtin_amdgcn_udot4(HA[m], w, WA, false);
                    SB = __builtin_amdgcn_udot4(HB[m], 0x01010101u, SB, false);
                    WB = __builtin_amdgcn_udot4(HB[m], w, WB, false);
                }
                Sc = SA | (SB << 16);
                Tc = as_u16x2((((124993u + WA) * P.k) & 0xffffu) | ((((124993u + WB) * P.k) & 0xffffu) << 16));
#pragma unroll
                for (int j = 0; j < 64; ++j)
                    Pd[j] = __builtin_amdgcn_perm(HB[j >> 2], HA[j >> 2], 0x0C040C00u + (uint32_t)(j & 3) * 0x00010001u);
            }
            uint32_t XA[NW], XB[NW];
#pragma unroll
            for (int q = 0; q < NW / 4; ++q) {
                const uint32_t off = rbase + (((uint32_t)q << 4) ^ rsw);
                const uint4 a = *(const uint4 *)(wl + off), b = *(const uint4 *)(wl + off + 64u * RUN);
                XA[4 * q + 0] = a.x; XA[4 * q + 1] = a.y; XA[4 * q + 2] = a.z; XA[4 * q + 3] = a.w;
                XB[4 * q + 0] = b.x; XB[4 * q + 1] = b.y; XB[4 * q + 2] = b.z; XB[4 * q + 3] = b.w;
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");       // segment in registers: buffer free
            bool more = true;
            if (g + 1 < (uint32_t)SEGS) {
                issue_seg(st, g + 1);
                // the next ST comes from a counter, grabbed behind the next segment's DMAs and
                // late in the ST (a wave that binds its next ST early can be a slow one holding
                // the batch's last ST): at segment 7, in a wave's first ST at 4 + blockIdx.x % 4
                // (grabbing at segment 0 before its landing wait put every wave of the grid on
                // one address at launch: the first segment landed 18.7 us after entry, median,
                // tools/scan_timeline.py)
            } else {
                nextst = multi ? grid + (uint32_t)__builtin_amdgcn_readfirstlane(pend) : nst;
                more = nextst < nst;
                if (more) {
                    issue_seg(nextst, 0);
                    load_halo(nextst);
                }
            }
            // the ST grab (grab_async): lane 0 at 4 + blockIdx % 4 in a wave's first ST,
            // at SEGS - 2 in later ones; read at the ST's last segment after its wait
            grab_async(pend, T.ctr, (g == (nth == 0u ? 4u + (blockIdx.x & 3u) : (uint32_t)SEGS - 2u) &&
                                     multi) ? 1u : 0u);
            // ---- roll segment g: positions 0..63 drop Pd, later ones this segment's own pairs
            const int64_t lim_rel = span - (int64_t)st * STB;         // ST-relative positions >= lim: not bytes
            const uint32_t relA0 = (uint32_t)lane * L + g * RUN;
            uint32_t S = Sc;
            u16x2 Tv = Tc;
            // positions 64..127 go straight into Pd as the next segment's dropped pairs:
            // Pd[j - 64] was last read as position j - 64's (no carry copies after the
            // segment: those were 64 moves per segment, 7 % of the kernel's VALU)
            static_assert(RUN == 128, "two halves of 64 pairs");
            uint32_t xl[64];                                           // pairs of positions 0..63
#pragma unroll
            for (int gg = 0; gg < NG; ++gg) {
                const uint32_t S0 = S;
                const u16x2 T0 = Tv;
                u16x2 acc = as_u16x2(0xffffffffu);
#pragma unroll
                for (int jj = 0; jj < 16; ++jj) {
                    const int j = gg * 16 + jj;
                    const uint32_t x = xpair32(XA, XB, j);
                    const uint32_t d = j < 64 ? Pd[j < 64 ? j : 0] : xl[j >= 64 ? j - 64 : 0];
                    if (j < 64) xl[j < 64 ? j : 0] = x;
                    else Pd[j >= 64 ? j - 64 : 0] = x;
                    S = S + x - d;
                    const u16x2 V = pk_mad(d, 0xFFC0FFC0u, as_u16x2(S));
                    Tv = pk_mad(as_u32(V), P.kk, Tv);
                    acc = __builtin_elementwise_min(acc, Tv);
                }
                const uint32_t a = as_u32(acc);
                // (two ballots of plain compares: one of their OR went through a 0/1
                // VGPR and a compare; the lane's own bit and the marks below are
                // derived inside the rare branch, not per group)
                const uint64_t bz = __builtin_amdgcn_ballot_w64((a & 0xffffu) == 0u) |
                                    __builtin_amdgcn_ballot_w64(a < 0x10000u);
                if (__builtin_expect(bz != 0ull, 0)) {
                    const uint32_t nz = (uint32_t)__builtin_popcountll(bz);
                    uint64_t bzs = bz;
                    asm volatile("" : "+s"(bzs));            // (else folded back to the lane's condition, kept live per group)
                    const bool z = ((bzs >> lane) & 1ull) != 0ull;
                    if (have + nz > (uint32_t)ST_DIRTYCAP) {
                        // no room for this group's dirty streams: their tiles go to the dense
                        // pass (the tiles of the dirty groups of this lane's two streams;
                        // the marks are applied when the ST is published)
                        constexpr uint32_t TB = (uint32_t)tile_bytes(DEFAULT_RUN);
                        uint32_t ga = relA0 + 16u * (uint32_t)gg;              // the group's ST-relative position
                        asm volatile("" : "+v"(ga));                            // (computed here, not per segment)
                        dmark |= ((a & 0xffffu) == 0u ? 1u << (ga / TB) : 0u) |
                                 ((a >> 16) == 0u ? 1u << ((ga + 64u * L) / TB) : 0u);
                    } else {
                        if (z) {                                           // slot: have + rank among z lanes
                            const uint32_t idx = have + __builtin_amdgcn_mbcnt_hi(
                                (uint32_t)(bz >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bz, 0u));
                            DirtySlotST &ds = dslots[idx];
#pragma unroll
                            for (int jj = 0; jj < 16; ++jj) {
                                const int j = gg * 16 + jj;
                                ds.dp[jj] = j < 64 ? Pd[j < 64 ? j : 0] : xl[j >= 64 ? j - 64 : 0];
                                ds.xp[jj] = j < 64 ? xl[j < 64 ? j : 0] : Pd[j >= 64 ? j - 64 : 0];
                            }
                            ds.S0 = S0;
                            ds.T0 = as_u32(T0);
                            ds.relA = relA0 + 16u * (uint32_t)gg;
                        }
                        have += nz;
                    }
                }
            }
            Sc = S;
            Tc = Tv;
            // ---- exact re-walk of the captured groups
            if (__builtin_expect(have != 0u, 0)) {
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");     // the slots' LDS writes
                const uint32_t nd = have;
                if ((uint32_t)lane < nd) {
                    const DirtySlotST &ds = dslots[lane];
                    const u16x2 kk = as_u16x2(P.kk), km = as_u16x2(P.kmv);
                    uint32_t s = ds.S0;
                    u16x2 t = as_u16x2(ds.T0);
                    const uint32_t relA = ds.relA, relB = ds.relA + 64u * L;
                    constexpr uint32_t TB = (uint32_t)tile_bytes(DEFAULT_RUN);
                    for (int jj = 0; jj < 16; ++jj) {
                        const uint32_t x = ds.xp[jj];
                        const uint32_t d = ds.dp[jj];
                        s = s + x - d;
                        t = as_u16x2(s) * kk + t;
                        t = as_u16x2(d) * km + t;
                        if (t.x == 0 && ((1984u + (s & 0xffffu)) & P.m1) == P.m1 && (int64_t)(relA + jj) < lim_rel) {
                            const uint32_t p = relA + jj, tt = p / TB;
                            const uint32_t idx = atomicAdd(&tcnt[tt], 1u) & 0x7fffffffu;
                            if (idx < (uint32_t)LC) tlist[tt * LC + idx] = p - tt * TB;
                        }
                        if (t.y == 0 && ((1984u + (s >> 16)) & P.m1) == P.m1 && (int64_t)(relB + jj) < lim_rel) {
                            const uint32_t p = relB + jj, tt = p / TB;
                            const uint32_t idx = atomicAdd(&tcnt[tt], 1u) & 0x7fffffffu;
                            if (idx < (uint32_t)LC) tlist[tt * LC + idx] = p - tt * TB;
                        }
                    }
                }
            }
            if (g + 1 == (uint32_t)SEGS) {                           // the ST's tiles are complete: publish
                if (__builtin_expect(__ballot(dmark != 0u) != 0ull, 0)) {   // tiles with unrecorded dirty groups
                    uint32_t m = 0;
#pragma unroll
                    for (int t = 0; t < TILES; ++t)
                        if (__ballot((dmark >> t) & 1u)) m |= 1u << t;
                    if (lane < TILES && ((m >> lane) & 1u)) atomicOr(&tcnt[lane], 0x80000000u);
                    dmark = 0u;
                }
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                // the ST's tile counts in one LDS read (lane t: tile t), then only the tiles
                // with candidates or a dense mark (random data: none) -- one LDS round trip
                // per tile was ~0.6 us of every ST switch
                static_assert(TILES <= 64, "one lane per tile");
                const uint32_t cl = (uint32_t)lane < (uint32_t)TILES
                                        ? __hip_atomic_load((__attribute__((address_space(3))) uint32_t *)&tcnt[lane],
                                                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT)
                                        : 0u;
                uint64_t todo = __builtin_amdgcn_ballot_w64(cl != 0u);
                while (todo) {
                    const uint32_t t = (uint32_t)__builtin_ctzll(todo);
                    todo &= todo - 1ull;
                    const uint32_t tile = st * TILES + t;
                    if (tile >= T.ntiles) break;
                    const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)cl, (int)t);
                    publish_list(T, tile, tlist + t * LC, c & 0x7fffffffu, lane, (c >> 31) != 0u,
                                 dslots_alloc, (uint32_t)LC);
                }
                __builtin_amdgcn_wave_barrier();
            }
            if (!more) {
                dense_pend_flush(T, dslots_alloc, lane);
                scan_time_exit(T, lane);
#ifdef SYNCR_CDC_DEV
                if (stamp) {
                    uint32_t hwid, xcc;
                    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)\n\ts_getreg_b32 %1, hwreg(HW_REG_XCC_ID)"
                                 : "=s"(hwid), "=s"(xcc));
                    SCAN_STAMP(T, DBG_SCAN + 4 * blockIdx.x + 2, wall_clock64());
                    SCAN_STAMP(T, DBG_SCAN + 4 * blockIdx.x + 3,
                               (uint64_t)(TILES * (nst_done + 1u)) | ((uint64_t)hwid << 32) | ((uint64_t)(xcc & 0xf) << 28));
                }
#endif
                return;
            }
        }
        st = nextst;
        ++nth;
#ifdef SYNCR_CDC_DEV
        ++nst_done;
#endif
    }
}

// ---------------------------------------------------------------------------
// Three-waves-per-SIMD scan (cdc_scan3_kernel, RUN = W3_RUN = 96).
//
// At two waves per SIMD a wave issues a VALU instruction at most every ~8
// cycles, so the roll's 2 VOP2 + 4 VOP3(P) per byte pair cost 3.85 / 6.05
// SIMD-cycles each; at three waves they cost 2.72 / 4.70
// (profiles/r02_ubench_valu.log): 32 -> 24 SIMD-cycles per 128 bytes, which
// keeps the scan above the HBM read ceiling even at the 1.7 GHz the part
// drops to when a scan load starts.  Three waves need
// <= 168 VGPRs and <= 13.6 KB of LDS per wave:
//   - a 12 KB tile (128 runs x 96 B): 12 waves x 12.35 KB keep the same
//     148 KB per CU of tile bytes in flight as 8 waves x 18.5 KB;
//   - dirty 16-byte groups keep no bytes in LDS or registers: the roll only
//     records their positions; after the roll each dirty slot's lane re-reads
//     the group's 80 bytes of both runs from HBM (the same clamped 16-byte
//     pieces the tile DMA read) behind the next tile's DMA, and the next
//     iteration's landing wait covers them, so the exact re-walk (closed-form
//     entry state + 16 exact steps) and the tile's publication happen one
//     iteration late without draining anything.
// ---------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ void window_state_n(const uint32_t (&A)[N], const uint32_t (&B)[N], const KParams &P,
                                               uint32_t &S, u16x2 &Tv) {
    uint32_t SA = 0, WA = 0, SB = 0, WB = 0;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        const uint32_t w = 0x3D3E3F40u - 0x04040404u * (uint32_t)m;
        SA = __builtin_amdgcn_udot4(A[m], 0x01010101u, SA, false);
        WA = __builtin_amdgcn_udot4(A[m], w, WA, false);
        SB = __builtin_amdgcn_udot4(B[m], 0x01010101u, SB, false);
        WB = __builtin_amdgcn_udot4(B[m], w, WB, false);
    }
    S = SA | (SB << 16);
    const uint32_t tA = ((124993u + WA) * P.k) & 0xffffu;
    const uint32_t tB = ((124993u + WB) * P.k) & 0xffffu;
    Tv = as_u16x2(tA | (tB << 16));
}

// The ROLL2 roll of one tile-lane; zg[g] = the 16-byte group g of run A or B
// has a zero mask-test value (a superset of its edges).
template <int RUN>
__device__ __forceinline__ void roll_flags(const uint32_t (&A)[(HALO + RUN) / 4],
                                           const uint32_t (&B)[(HALO + RUN) / 4], const KParams &P,
                                           bool (&zg)[RUN / 16]) {
    uint32_t S;
    u16x2 Tv;
    window_state<RUN>(A, B, P, 0, S, Tv);
#pragma unroll
    for (int g = 0; g < RUN / 16; ++g) {
        u16x2 acc = as_u16x2(0xffffffffu);
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
            const int i = g * 16 + jj;
            const uint32_t x = pair_at<RUN>(A, B, HALO + i), d = pair_at<RUN>(A, B, i);
            S = S + x - d;
            const u16x2 V = pk_mad(d, 0xFFC0FFC0u, as_u16x2(S));   // S - 64 d (mod 2^16 per half)
            Tv = pk_mad(as_u32(V), P.kk, Tv);                       // T += k (S - 64 d)
            acc = __builtin_elementwise_min(acc, Tv);
        }
        const uint32_t a = as_u32(acc);
        zg[g] = (a & 0xffffu) == 0u || (a >> 16) == 0u;
    }
}

// One 16-byte piece of the batch at g, clamped as issue_buf clamps an edge
// tile's pieces (so the re-walk sees exactly the bytes the roll saw).
__device__ __forceinline__ uint4 reread_piece(const uint8_t *data, int64_t g, int64_t last) {
    g = g < 0 ? 0 : (g > last ? last : g);
    return *(const uint4 *)(data + g);
}

// Exact re-walk of one dirty group from its re-read bytes: ra / rb = bytes
// [rel - 64, rel + 16) of runs A and B (tile-relative rel, rel + 64 RUN).
template <int RUN>
__device__ __forceinline__ void rewalk_reread(const KParams &P, uint32_t relA, const uint4 (&ra)[5],
                                              const uint4 (&rb)[5], int64_t lim_rel, uint32_t *wcount,
                                              uint32_t *wlist) {
    uint32_t A[20], B[20];
#pragma unroll
    for (int m = 0; m < 5; ++m) {
        A[4 * m] = ra[m].x; A[4 * m + 1] = ra[m].y; A[4 * m + 2] = ra[m].z; A[4 * m + 3] = ra[m].w;
        B[4 * m] = rb[m].x; B[4 * m + 1] = rb[m].y; B[4 * m + 2] = rb[m].z; B[4 * m + 3] = rb[m].w;
    }
    uint32_t s;
    u16x2 t;
    window_state_n<20>(A, B, P, s, t);
    const u16x2 kk = as_u16x2(P.kk), km = as_u16x2(P.kmv);
    const uint32_t relB = relA + 64u * RUN;
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) {
        const uint32_t sel = 0x0C040C00u + (uint32_t)(jj & 3) * 0x00010001u;
        const uint32_t x = __builtin_amdgcn_perm(B[16 + (jj >> 2)], A[16 + (jj >> 2)], sel);
        const uint32_t d = __builtin_amdgcn_perm(B[jj >> 2], A[jj >> 2], sel);
        s = s + x - d;
        t = as_u16x2(s) * kk + t;
        t = as_u16x2(d) * km + t;
        if (t.x == 0 && ((1984u + (s & 0xffffu)) & P.m1) == P.m1 && (int64_t)(relA + jj) < lim_rel)
            record(wcount, wlist, relA + jj);
        if (t.y == 0 && ((1984u + (s >> 16)) & P.m1) == P.m1 && (int64_t)(relB + jj) < lim_rel)
            record(wcount, wlist, relB + jj);
    }
}

// MODE bit 2: non-temporal tile loads; bit 3: dynamic tile groups; bit 1
// (development library only): no tile DMA after the first (roll timing).
template <int RUN, int MODE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3)))
void cdc_scan3_kernel(const uint8_t *__restrict__ data, KParams P, Tables T) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int TILE = tile_bytes(RUN);
    constexpr int NQ = (HALO + RUN) / 16;
    constexpr int NG = RUN / 16;
    constexpr bool NT = (MODE & 4) != 0;
    constexpr bool DYN = (MODE & 8) != 0;
    const int lane = threadIdx.x;
    uint8_t *wl = smem;
    uint32_t *drel = (uint32_t *)(smem + buf_bytes(RUN));
    uint32_t *wlist = drel + DIRTYCAP3;
    uint32_t *wcount = wlist + LISTCAP;
    uint32_t *dcount = wcount + 1;
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr(wl));
    const uint32_t stride = gridDim.x;
    // dynamic groups as in cdc_scan_kernel; 12 tiles of 12 KB per grab keep
    // the counter below its ~69 M grabs/s
    constexpr uint32_t DG = 12;
    auto gbase = [&](uint32_t k) { return (k / stride) * stride * DG + (k % stride); };
    uint32_t tile = blockIdx.x;
    if (tile >= T.ntiles) return;
    const int64_t span = (int64_t)T.span;
    const int64_t last = (int64_t)((T.span - 1) & ~15ull);
    issue_tile<RUN, NT>(data, T.span, tile, lds0, lane);
    if (lane == 0) { *wcount = 0u; *dcount = 0u; }
    uint32_t gj = 0, pend = 0;
    DenseSlots dslots_alloc;
    // the previous tile's dirty groups: count, tile, this lane's slot and bytes
    uint32_t pnd = 0, ptile = 0, prel = 0;
    uint4 ra[5], rb[5];
    for (uint32_t next; tile < T.ntiles; tile = next) {
        bool grabbed = false;
        uint32_t gjn = 0;
        if constexpr (DYN) {
            if (gj + 1 < DG && tile + stride < T.ntiles) {
                next = tile + stride;
                gjn = gj + 1;
            } else {
                if (gj == 0) {
                    if (lane == 0) pend = atomicAdd(&T.ctr[CTR_CANDS_HI], 1u);
                    grabbed = true;
                }
                wait_vmcnt<0>();                                     // the grab
                next = gbase(stride + (uint32_t)__builtin_amdgcn_readfirstlane(pend));
                gjn = 0;
            }
        } else {
            next = tile + stride;
        }
        const int64_t t0 = (int64_t)tile * TILE;
        wait_vmcnt<0>();                         // this tile has landed, and the previous tile's re-reads
        if (pnd) {
            const int64_t pt0 = (int64_t)ptile * TILE;
            if ((uint32_t)lane < pnd) rewalk_reread<RUN>(P, prel, ra, rb, span - pt0, wcount, wlist);
            publish_tile(data, P, T, ptile, pt0, wlist, wcount, lane, false, dslots_alloc);
            if (lane == 0) *wcount = 0u;
        }
        uint32_t A[NQ * 4], B[NQ * 4];
        {
            const uint4 *la = (const uint4 *)(wl + lane * RUN);          // = run start - 64
            const uint4 *lb = (const uint4 *)(wl + (lane + 64) * RUN);
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const uint4 a = la[q], b = lb[q];
                A[4 * q + 0] = a.x; A[4 * q + 1] = a.y; A[4 * q + 2] = a.z; A[4 * q + 3] = a.w;
                B[4 * q + 0] = b.x; B[4 * q + 1] = b.y; B[4 * q + 2] = b.z; B[4 * q + 3] = b.w;
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");           // runs are in registers
        if (next < T.ntiles && (MODE & 2) == 0) issue_tile<RUN, NT>(data, T.span, next, lds0, lane);
        if constexpr (DYN) {
            if (gj == 0 && !grabbed && lane == 0) pend = atomicAdd(&T.ctr[CTR_CANDS_HI], 1u);
            gj = gjn;
        }
        bool zg[NG];
        roll_flags<RUN>(A, B, P, zg);
        bool anyz = false;
#pragma unroll
        for (int g = 0; g < NG; ++g) anyz = anyz || zg[g];
        pnd = 0;
        if (__builtin_expect(__ballot(anyz) != 0ull, 0)) {
#pragma unroll
            for (int g = 0; g < NG; ++g) {
                if (zg[g]) {
                    const uint32_t idx = atomicAdd(dcount, 1u);
                    if (idx < (uint32_t)DIRTYCAP3) drel[idx] = (uint32_t)(lane * RUN + g * 16);
                }
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            const uint32_t nd = __builtin_amdgcn_readfirstlane(
                __hip_atomic_load((__attribute__((address_space(3))) uint32_t *)dcount, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WAVEFRONT));
            if ((uint32_t)lane < nd && (uint32_t)lane < (uint32_t)DIRTYCAP3) prel = drel[lane];
            __builtin_amdgcn_wave_barrier();
            if (lane == 0) *dcount = 0u;
            if (nd > (uint32_t)DIRTYCAP3) {
                publish_tile(data, P, T, tile, t0, wlist, wcount, lane, true, dslots_alloc);    // exact dense pass
            } else {
                pnd = nd;
                ptile = tile;
                if ((uint32_t)lane < nd) {
                    const int64_t ga = t0 + (int64_t)prel - HALO, gb = ga + 64 * RUN;
#pragma unroll
                    for (int m = 0; m < 5; ++m) {
                        ra[m] = reread_piece(data, ga + 16 * m, last);
                        rb[m] = reread_piece(data, gb + 16 * m, last);
                    }
                }
            }
        }
    }
    if (pnd) {
        wait_vmcnt<0>();
        const int64_t pt0 = (int64_t)ptile * TILE;
        if ((uint32_t)lane < pnd) rewalk_reread<RUN>(P, prel, ra, rb, span - pt0, wcount, wlist);
        publish_tile(data, P, T, ptile, pt0, wlist, wcount, lane, false, dslots_alloc);
    }
}

#ifdef SYNCR_CDC_DEV
#include "dev/scan_mfma.inc"
#endif  // SYNCR_CDC_DEV

// File starts: the scan treats the batch as ONE byte stream, so its G is exact
// for p >= f+63 inside a file starting at f.  The 63 head positions of a file
// are the resolve's head scan at s = 0 (a fresh window at f, exactly as after
// any cut), so file starts need no kernel of their own.
// Head fix-ups, computed before the resolve so its serial walk never waits
// on byte loads: of every candidate e (first chunk-local hit in [e+1, e+63])
// and of every read-boundary grid point (first chunk-local hit in
// [p, min(p+63, file end)), stored as offset + 1).
// Head fix-ups, two per thread as the 16-bit halves of packed registers (the
// scan's trick): item k of the launch (a candidate, or past the candidates a
// read-boundary grid point) rolls its 63 bytes from a zeroed window:
//   S += x; T += k S                    (T = ((s2 + 1) k) mod 2^16, s2 = 124992 + W)
//   Z = ((S + 1985) & m1) | T           zero iff the digest test passes
//   acc = 2 acc + sat(1 - Z)            16-position hit masks, first position in bit 15
// and the first hit is the leading one of the 63-bit mask (clz).  A T-only pass
// (min of T over the 63 positions: 2 VALU per item-byte) runs first; only items
// with a zero T (any at all: 63 / 2^16 at bits >= 16, 63 / 2^bits below) take
// the exact pass (~3.5 VALU per item-byte).  The dense workload has a
// candidate every 64 bytes (7.5 M per launch).
// (Fusing fix-ups into the dense and gather launches -- no separate launch --
// measured 8 us SLOWER per step on zipf10k: the per-lane serial fix-ups
// lengthen the gather's critical path; profiles/r02_ab_run_fusefix.log.)
// known = the fix-up the dense pass already stored with a candidate (CAND_KNOWN), else ~0u
__device__ __forceinline__ void fix_item(const Tables &T, uint64_t n, uint64_t i, uint64_t &a, uint32_t &cnt,
                                         uint32_t &known, uint32_t &dec) {
    known = ~0u;
    dec = 0u;                                             // bit 0: link decided (CAND_LDEC), bit 1: its value
    if (i < n) {                                          // a candidate e: chunk starts at e + 1
        const uint64_t w = T.cand[i];
        a = (w & CAND_POS_MASK) + 1;
        cnt = (uint32_t)min<uint64_t>(63ull, T.span > a ? T.span - a : 0ull);
        if (w & CAND_KNOWN) {
            known = (uint32_t)(w >> 48) & 0xffu;
            cnt = 0u;
            if (w & CAND_LDEC) dec = 1u | ((w & CAND_LINK) ? 2u : 0u);
        }
    } else if (i < n + T.ngrid) {                         // a grid point p: chunk starts at p, ends by the file's end
        a = T.gpos[i - n];
        const uint64_t end = T.gend[i - n];
        cnt = (uint32_t)min<uint64_t>(63ull, end > a ? end - a : 0ull);
    } else {
        a = 0;
        cnt = 0;
    }
}

__device__ __forceinline__ void fix_load(const uint8_t *__restrict__ data, uint64_t span, uint64_t a, uint32_t cnt,
                                         uint32_t (&w)[16]) {
    if (cnt && a + 64 <= span) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            uint4 v;
            __builtin_memcpy(&v, data + a + 16 * i, 16);
            w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            uint32_t x = 0;
            for (int b = 0; b < 4; ++b)
                if ((uint32_t)(4 * i + b) < cnt) x |= (uint32_t)data[a + 4 * i + b] << (8 * b);
            w[i] = x;
        }
    }
}

// first hit among the first cnt of 63 positions from the four 16-position masks of one half
__device__ __forceinline__ uint32_t fix_first(uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3, uint32_t cnt) {
    uint64_t m = ((uint64_t)m0 << 48) | ((uint64_t)m1 << 32) | ((uint64_t)m2 << 16) | (uint64_t)m3;
    m &= cnt ? ~0ull << (64 - cnt) : 0ull;
    return m ? (uint32_t)__builtin_clzll(m) + 1u : 0u;
}

// bits x0..x31 to the even bit positions of a 64-bit word
__device__ __forceinline__ uint64_t spread32(uint32_t x) {
    uint64_t v = x;
    v = (v | (v << 16)) & 0x0000FFFF0000FFFFull;
    v = (v | (v << 8)) & 0x00FF00FF00FF00FFull;
    v = (v | (v << 4)) & 0x0F0F0F0F0F0F0F0Full;
    v = (v | (v << 2)) & 0x3333333333333333ull;
    v = (v | (v << 1)) & 0x5555555555555555ull;
    return v;
}

// Head fix-ups of two items (A: the low halves, B: the high halves): the first
// chunk-local hit among the first nA / nB of the 63 bytes in A[] / B[], + 1, or 0.
__device__ __forceinline__ void fix_pair(const uint32_t (&A)[16], const uint32_t (&B)[16], uint32_t nA, uint32_t nB,
                                         const KParams &P, uint32_t &fA, uint32_t &fB) {
    const uint32_t m1x2 = P.m1 | (P.m1 << 16);
    const uint32_t t0 = ((124993u * P.k) & 0xffffu) * 0x00010001u;   // T of an empty window, both halves
    fA = 0u;
    fB = 0u;
    // fast pass: only T (the s2 test, exact for masks of <= 16 bits and the rarer half of
    // wider ones) -- 4 VALU per position pair; a zero T anywhere sends the item to the
    // exact pass (P(some T == 0 in 63) = 63 / 2^16 per item at bits >= 16)
    {
        uint32_t S = 0;
        u16x2 Tv = as_u16x2(t0), mn = as_u16x2(0xffffffffu);
#pragma unroll
        for (int k = 0; k < 63; ++k) {
            const uint32_t x = __builtin_amdgcn_perm(B[k >> 2], A[k >> 2], 0x0C040C00u + (uint32_t)(k & 3) * 0x00010001u);
            S += x;
            Tv = pk_mad(S, P.kk, Tv);
            mn = __builtin_elementwise_min(mn, Tv);
        }
        const uint32_t m = as_u32(mn);
        if (__builtin_expect((m & 0xffffu) == 0u || (m >> 16) == 0u, 0)) {
            uint32_t acc[4];
            S = 0;
            Tv = as_u16x2(t0);
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                uint32_t mm = 0;
#pragma unroll
                for (int jj = 0; jj < 16; ++jj) {
                    const int k = 16 * g + jj;
                    if (k < 63) {
                        const uint32_t x = __builtin_amdgcn_perm(B[k >> 2], A[k >> 2],
                                                                 0x0C040C00u + (uint32_t)(k & 3) * 0x00010001u);
                        S += x;                                       // halves < 2^15: no carry
                        Tv = pk_mad(S, P.kk, Tv);                     // T += k S
                        const uint32_t U = as_u32(as_u16x2(S) + (u16x2){(unsigned short)1985, (unsigned short)1985});
                        const uint32_t Z = (U & m1x2) | as_u32(Tv);
                        uint32_t h;
                        asm volatile("v_pk_sub_u16 %0, %1, %2 clamp" : "=v"(h) : "s"(0x00010001u), "v"(Z));
                        mm = as_u32(pk_mad(mm, 0x00020002u, as_u16x2(h)));   // mm = 2 mm + h
                    } else {
                        mm = as_u32(pk_mad(mm, 0x00020002u, as_u16x2(0u)));  // position 63: none
                    }
                }
                acc[g] = mm;
            }
            fA = fix_first(acc[0] & 0xffffu, acc[1] & 0xffffu, acc[2] & 0xffffu, acc[3] & 0xffffu, nA);
            fB = fix_first(acc[0] >> 16, acc[1] >> 16, acc[2] >> 16, acc[3] >> 16, nB);
        }
    }
}

__global__ __launch_bounds__(256) void cdc_fix_kernel(const uint8_t *__restrict__ data, KParams P,
                                                      Tables T) {
    const uint64_t total = (uint64_t)T.ctr[CTR_CANDS_LO] | ((uint64_t)T.ctr[CTR_CANDS_HI] << 32);
    const uint64_t n = total < T.cand_cap ? total : T.cand_cap;
    const uint64_t items = n + T.ngrid;
    for (uint64_t q = (uint64_t)blockIdx.x * 256 + threadIdx.x; 2 * q < items; q += (uint64_t)gridDim.x * 256) {
        uint64_t aA, aB;
        uint32_t nA, nB, kA, kB, dA, dB;
        fix_item(T, n, 2 * q, aA, nA, kA, dA);
        fix_item(T, n, 2 * q + 1, aB, nB, kB, dB);
        uint32_t fA = 0u, fB = 0u;
        if (__ballot(nA != 0u || nB != 0u)) {             // (candidates of the dense pass's tiles come known)
            uint32_t A[16], B[16];
            fix_load(data, T.span, aA, nA, A);
            fix_load(data, T.span, aB, nB, B);
            fix_pair(A, B, nA, nB, P, fA, fB);
        }
        if (kA != ~0u) fA = kA;
        if (kB != ~0u) fB = kB;
        // chain links (CAND_LINK): empty fix-up, next candidate 64 .. gapmax past
        // (a dense tile's candidates come with theirs decided, CAND_LDEC, but the last)
        const uint64_t gapmax = T.gapmax;
        bool lA = (dA & 2u) != 0u, lB = (dB & 2u) != 0u;
        if (T.linkw && !dA && 2 * q + 1 < n) {
            const uint64_t d = aB - aA;                       // positions 2q+1 and 2q
            lA = fA == 0u && d >= 64u && d <= gapmax;
        }
        if (T.linkw && !dB && 2 * q + 2 < n) {
            const uint64_t d = (T.cand[2 * q + 2] & CAND_POS_MASK) - (aB - 1);
            lB = fB == 0u && d >= 64u && d <= gapmax;
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint64_t i = 2 * q + (uint64_t)h;
            const uint32_t f = h ? fB : fA;
            if (i < n && !(h ? dB : dA))                      // (a decided word is complete already)
                st_u64(&T.cand[i], ((h ? aB : aA) - 1) | ((uint64_t)f << 48) | CAND_KNOWN |
                                       ((h ? lB : lA) ? CAND_LINK : 0ull), T.nt_out);
            else if (i >= n && i < items) T.gfix[i - n] = (uint8_t)f;
        }
        // the wave's 128 consecutive candidates (lane l: 2l, 2l+1) as two link words
        if (T.linkw) {
        const unsigned long long E = __ballot(lA), O = __ballot(lB);
        const uint64_t q0 = q - (threadIdx.x & 63u);
        if ((threadIdx.x & 63u) == 0u && 2 * q0 < n) {
            T.linkw[q0 / 32] = spread32((uint32_t)E) | (spread32((uint32_t)O) << 1);
            T.linkw[q0 / 32 + 1] = spread32((uint32_t)(E >> 32)) | (spread32((uint32_t)(O >> 32)) << 1);
        }
        }
    }
}

#ifdef SYNCR_CDC_DEV
#include "dev/dense_generic.inc"
#endif  // SYNCR_CDC_DEV

// Exact packed roll of one dense tile-lane (runs lane and lane+64 in the two
// 16-bit halves, as roll_fast): every position's full digest test.  Per byte
// pair:
//   S += x - d; V = S - 64 d; T += k V           as in the scan (4 ops)
//   Z = ((S + 1985) & m1) | T                    zero iff both halves of the
//        digest test pass: (s1 & m1) == m1 <=> ((s1 + 1) & m1) == 0 for the
//        low-bit mask m1 = mask >> 16, s1 = 1984 + S; T = ((s2+1) k) mod 2^16
//   h = sat(1 - Z); acc = 2 acc + h              (v_pk_sub_u16 clamp, v_pk_mad_u16)
// so each run's 16-position group ends as a 16-bit hit mask (first position
// in bit 15; one v_bfrev per group puts both runs' masks in bitmap order).
// ~9.4 VALU per byte pair against ~27 for the byte-at-a-time exact roll.
// put(g, r): r = group g's masks, run A in the high half, run B in the low;
// positions at or past `lim` (tile-relative) are masked off.  Returns the
// lane's hit count.
template <int RUN, class Put>
__device__ __forceinline__ uint32_t dense_roll(const uint32_t (&A)[(HALO + RUN) / 4],
                                               const uint32_t (&B)[(HALO + RUN) / 4], const KParams &P,
                                               int lane, int64_t lim, Put put) {
    constexpr int NG = RUN / 16;
    const uint32_t m1x2 = P.m1 | (P.m1 << 16);
    uint32_t S;
    u16x2 Tv;
    window_state<RUN>(A, B, P, 0, S, Tv);
    uint32_t cnt = 0;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        uint32_t acc = 0;
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
            const int i = g * 16 + jj;
            const uint32_t x = pair_at<RUN>(A, B, HALO + i), d = pair_at<RUN>(A, B, i);
            S = S + x - d;
            const u16x2 V = pk_mad(d, 0xFFC0FFC0u, as_u16x2(S));      // S - 64 d
            Tv = pk_mad(as_u32(V), P.kk, Tv);                         // T += k (S - 64 d)
            const uint32_t U = as_u32(as_u16x2(S) + (u16x2){(unsigned short)1985, (unsigned short)1985});
            const uint32_t Z = (U & m1x2) | as_u32(Tv);
            uint32_t h;
            asm volatile("v_pk_sub_u16 %0, %1, %2 clamp" : "=v"(h) : "s"(0x00010001u), "v"(Z));
            acc = as_u32(pk_mad(acc, 0x00020002u, as_u16x2(h)));      // acc = 2 acc + h
        }
        uint32_t r = __builtin_bitreverse32(acc);    // lo half: run B's mask, hi half: run A's
        if (lim < (int64_t)tile_bytes(RUN)) {
            const int64_t pa = (int64_t)lane * RUN + 16 * g, pb = pa + 64 * RUN;
            const int64_t na = lim - pa, nb = lim - pb;
            const uint32_t ma = na >= 16 ? 0xffffu : (na <= 0 ? 0u : (1u << na) - 1u);
            const uint32_t mb = nb >= 16 ? 0xffffu : (nb <= 0 ? 0u : (1u << nb) - 1u);
            r &= (ma << 16) | mb;
        }
        cnt += (uint32_t)__builtin_popcount(r);
        put(g, r);
    }
    return cnt;
}

// The scan wave's own exact pass over a tile with more dirty groups than side
// slots (low-entropy / periodic data): no separate dense launch.  The runs are
// re-read from memory (the landing buffer already holds the next tile, and
// keeping the roll's registers alive for this rare path would cost the scan
// its second wave per SIMD); bytes outside [0, span) read as zero.  The bitmap
// words go straight to dense_bits (halfword stores); the tile joins the dense
// list that cdc_gather_kernel expands.
template <int RUN>
__device__ __forceinline__ void load_runs(const uint8_t *__restrict__ data, int64_t span, int64_t t0, int lane,
                                          uint32_t (&A)[(HALO + RUN) / 4], uint32_t (&B)[(HALO + RUN) / 4]) {
    constexpr int NQ = (HALO + RUN) / 16;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int64_t g0 = t0 + (int64_t)(lane + 64 * h) * RUN - HALO;
        uint32_t *dst = h ? B : A;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int64_t g = g0 + 16 * q;
            uint4 v;
            if (g >= 0 && g + 16 <= span) {
                v = *(const uint4 *)(data + g);
            } else {
                uint32_t w4[4] = {0u, 0u, 0u, 0u};
                for (int b = 0; b < 16; ++b)
                    if (g + b >= 0 && g + b < span) w4[b >> 2] |= (uint32_t)data[g + b] << (8 * (b & 3));
                v = make_uint4(w4[0], w4[1], w4[2], w4[3]);
            }
            dst[4 * q] = v.x; dst[4 * q + 1] = v.y; dst[4 * q + 2] = v.z; dst[4 * q + 3] = v.w;
        }
    }
}

template <int RUN>
__device__ __forceinline__ void scan_dense_tile(const uint8_t *__restrict__ data, const KParams &P,
                                                const Tables &T, uint32_t tile, int64_t t0, int lane) {
    constexpr int NG = RUN / 16;
    uint32_t idx = 0;
    if (lane == 0) {
        atomicOr(&T.nonempty[tile >> 6], 1ull << (tile & 63));
        idx = atomicAdd(&T.ctr[CTR_DENSE], 1u);
    }
    idx = (uint32_t)__builtin_amdgcn_readfirstlane(idx);
    if (idx >= T.dense_cap) {                            // the host re-runs with a bigger list
        if (lane == 0) {
            T.tile_meta[tile] = DENSE_BIT | 0x7fffffffu;
            atomicOr(&T.ctr[CTR_FLAGS], FLAG_DENSE_OVERFLOW);
        }
        return;
    }
    uint32_t A[(HALO + RUN) / 4], B[(HALO + RUN) / 4];
    load_runs<RUN>(data, (int64_t)T.span, t0, lane, A, B);
    uint16_t *bm = (uint16_t *)(T.dense_bits + (size_t)idx * (tile_bytes(RUN) / 32));
    uint32_t cnt = dense_roll<RUN>(A, B, P, lane, (int64_t)T.span - t0, [&](int g, uint32_t r) {
        bm[lane * NG + g] = (uint16_t)(r >> 16);
        bm[(lane + 64) * NG + g] = (uint16_t)r;
    });
    for (int off = 32; off >= 1; off >>= 1) cnt += __shfl_xor(cnt, off);
    if (lane == 0) {
        T.dense_list[idx] = tile;
        T.dense_cnt[idx] = cnt;
        T.tile_meta[tile] = DENSE_BIT | idx;
        atomicAdd(&T.super_cnt[tile >> 6], cnt);
        atomicAdd(&T.coarse[(tile >> 12) * COARSE_STRIDE], cnt);
        atomicAdd(&T.split[SPL_DENSE_TILES], 1u);
    }
}

// Dense tiles, packed (the product's dense pass): the scan's own two-stage
// pipeline -- a wave's tile lands in its LDS buffer by LDS-DMA, is copied to
// registers (lane l: runs l and l+64 with their warm-up bytes), and the next
// dense tile's DMA is issued at once, so it lands while this one is rolled by
// dense_roll.  Edge tiles clamp out-of-range pieces like the scan (their bytes
// only feed positions outside [0, span), which are masked, or before a file's
// 63rd byte, which the resolve never reads).  The bitmap halfwords go straight
// to dense_bits.
__device__ __forceinline__ uint32_t sload_u32(const uint32_t *p) {
    const uint64_t a = (uint64_t)p;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    const uint64_t u = ((uint64_t)hi << 32) | (uint64_t)lo;
    uint32_t v;
    asm volatile("s_nop 4\n\ts_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(u) : "memory");
    return v;
}

// Head fix-ups of a dense tile's candidates from its bytes in the dense pass's
// LDS buffer (see cdc_dense_packed_kernel): round k takes each lane's k-th
// candidate of run A and of run B (rr: the roll's group masks, run A high), loads
// the 63 bytes after each from LDS (17 aligned words + v_alignbyte) and rolls
// them as the halves of packed registers (fix_pair).  Candidate ranks in the
// tile: run order (runs 0..63 are the lanes' A, 64..127 their B), then position.
// Returns false (nothing stored) when the tile is past FIXCAP candidates or a
// run past FIX_RMAX.
template <int RUN>
__device__ __forceinline__ bool dense_fixups(const uint8_t *dbuf, const KParams &P, const Tables &T,
                                             const uint32_t (&rr)[RUN / 16], uint32_t cnt, uint32_t idx, int64_t t0,
                                             int lane) {
    constexpr int NG = RUN / 16;
    uint32_t cA = 0, cB = 0;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        cA += (uint32_t)__builtin_popcount(rr[g] >> 16);
        cB += (uint32_t)__builtin_popcount(rr[g] & 0xffffu);
    }
    uint32_t mx = cA > cB ? cA : cB;
    for (int off = 32; off >= 1; off >>= 1) {
        const uint32_t o = (uint32_t)__shfl_xor((int)mx, off);
        mx = o > mx ? o : mx;
    }
    mx = (uint32_t)__builtin_amdgcn_readfirstlane(mx);
    if (cnt > FIXCAP || mx > FIX_RMAX) return false;
    const uint32_t iA = wave_incl_scan(cA, lane), iB = wave_incl_scan(cB, lane);
    const uint32_t totA = (uint32_t)__builtin_amdgcn_readlane((int)iA, 63);
    const uint32_t preA = iA - cA, preB = totA + iB - cB;
    // the runs' masks, position j of the run = bit j
    uint64_t a0 = 0, a1 = 0, b0 = 0, b1 = 0;
    uint32_t a2 = 0, b2 = 0;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        const uint64_t ha = rr[g] >> 16, hb = rr[g] & 0xffffu;
        if (g < 4) { a0 |= ha << (16 * g); b0 |= hb << (16 * g); }
        else if (g < 8) { a1 |= ha << (16 * (g - 4)); b1 |= hb << (16 * (g - 4)); }
        else { a2 |= (uint32_t)ha << (16 * (g - 8)); b2 |= (uint32_t)hb << (16 * (g - 8)); }
    }
    auto take = [](uint64_t &m0, uint64_t &m1, uint32_t &m2) -> int {
        if (m0) { const int o = __builtin_ctzll(m0); m0 &= m0 - 1; return o; }
        if (m1) { const int o = 64 + __builtin_ctzll(m1); m1 &= m1 - 1; return o; }
        if (m2) { const int o = 128 + __builtin_ctz(m2); m2 &= m2 - 1; return o; }
        return -1;
    };
    uint8_t *fx = T.dense_fix + (size_t)idx * FIXCAP;
    uint16_t *ps = T.dense_pos + (size_t)idx * FIXCAP;
    const int64_t span = (int64_t)T.span;
    auto window = [&](int run, int o, uint32_t &n, uint32_t (&w)[16]) {
        const uint32_t rel = (uint32_t)(run * RUN + o + 1);              // tile-relative chunk start
        const uint32_t off = o < 0 ? 0u : (uint32_t)HALO + rel;         // its LDS byte
        const int64_t left = span - (t0 + (int64_t)rel);
        n = o < 0 ? 0u : (uint32_t)(left >= 63 ? 63 : (left > 0 ? left : 0));
        const uint32_t *src = (const uint32_t *)(dbuf + (off & ~3u));
        const uint32_t sh = off & 3u;
        uint32_t W[17];
#pragma unroll
        for (int i = 0; i < 17; ++i) W[i] = src[i];
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = __builtin_amdgcn_alignbyte(W[i + 1], W[i], sh);
    };
    for (uint32_t k = 0; k < mx; ++k) {
        const int oA = take(a0, a1, a2), oB = take(b0, b1, b2);
        uint32_t XA[16], XB[16], nA, nB, fA, fB;
        window(lane, oA, nA, XA);
        window(lane + 64, oB, nB, XB);
        fix_pair(XA, XB, nA, nB, P, fA, fB);
        if (oA >= 0) {
            fx[preA + k] = (uint8_t)fA;
            ps[preA + k] = (uint16_t)(lane * RUN + oA);
        }
        if (oB >= 0) {
            fx[preB + k] = (uint8_t)fB;
            ps[preB + k] = (uint16_t)((lane + 64) * RUN + oB);
        }
    }
    return true;
}

// FUSE (the product, round 4): the head fix-ups of the tile's candidates are
// computed here, from the tile's bytes still in LDS, and stored by rank
// (dense_fix, DENSE_FIXED in dense_cnt); cdc_gather_kernel writes them into the
// candidates (CAND_KNOWN) and cdc_fix_kernel skips them.  The fix kernel had
// re-read 63 bytes per candidate from HBM (0.40 GB per launch of the dense
// workload, 0.84x its periodic bytes: profiles/r04jdense_pmc_traffic.json).
// The buffer then holds 80 bytes past the tile (the windows of its last
// candidates), and the next tile's DMA is issued after the fix-ups: the
// other wave of the SIMD covers its latency.  A tile with more than FIXCAP
// candidates, or a run with more than FIX_RMAX, keeps the separate fix-ups
// (the rounds below go by the fullest run: ~0.4 us per round).
template <int RUN, bool FUSE>
__global__ __launch_bounds__(64) void cdc_dense_packed_kernel(const uint8_t *__restrict__ data, KParams P,
                                                              Tables T) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dbuf[];   // [HALO + tile (+ DENSE_TAIL)]
    constexpr int TILE = tile_bytes(RUN), NQ = (HALO + RUN) / 16, NG = RUN / 16;
    constexpr int BUFD = dense_buf_bytes(RUN, FUSE);
    const int lane = threadIdx.x;
    if (blockIdx.x < (uint32_t)DBG_NDW) SCAN_STAMP(T, DBG_DW + 2 * blockIdx.x, wall_clock64());
    const uint32_t nd = min(sload_u32(&T.ctr[CTR_DENSE]), T.dense_cap);
    // Block b takes the contiguous list range [b*per, (b+1)*per): the list is
    // in scan order, so a grid stride over it put the whole grid's coarse
    // atomics on the one or two counters of the scan's window (dense workload:
    // 248 vs 152 us); contiguous ranges spread them over the batch, and a
    // wave adds its consecutive tiles' counts to a coarse counter once.
    const uint32_t per = (nd + gridDim.x - 1) / gridDim.x;
    uint32_t idx = blockIdx.x * per;
    const uint32_t iend = min(nd, idx + per);
    if (idx >= iend) return;
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr(dbuf));
    const int64_t span = (int64_t)T.span;
    // unused slots of the scan waves' chunks (DENSE_HOLE) are skipped
    uint32_t tile = sload_u32(&T.dense_list[idx]);
    while (tile == DENSE_HOLE) {
        if (++idx >= iend) return;
        tile = sload_u32(&T.dense_list[idx]);
    }
    uint32_t cur_c = tile >> 12, acc_c = 0, ndone = 0;
    // (dev timeline: the first DBG_DT_N tiles of the first DBG_DT_W blocks)
    const bool dstamp = blockIdx.x < (uint32_t)DBG_DT_W;
#define DENSE_STAMP(k, j) do { if (dstamp && (k) < (uint32_t)DBG_DT_N) \
        SCAN_STAMP(T, DBG_DT + 4 * (DBG_DT_N * blockIdx.x + (k)) + (j), wall_clock64()); } while (0)
    DENSE_STAMP(0u, 0);
    issue_buf<BUFD, TILE, true>(data, T.span, tile, lds0, lane);
    for (uint32_t next; idx < iend; idx = next) {
        next = idx + 1;
        uint32_t ntile = DENSE_HOLE;
        while (next < iend && (ntile = sload_u32(&T.dense_list[next])) == DENSE_HOLE) ++next;
        wait_vmcnt<0>();                                          // this tile has landed
        DENSE_STAMP(ndone, 1);
        uint32_t A[NQ * 4], B[NQ * 4];
        {
            const uint4 *la = (const uint4 *)(dbuf + lane * RUN);          // = run start - 64
            const uint4 *lb = (const uint4 *)(dbuf + (lane + 64) * RUN);
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const uint4 a = la[q], b = lb[q];
                A[4 * q + 0] = a.x; A[4 * q + 1] = a.y; A[4 * q + 2] = a.z; A[4 * q + 3] = a.w;
                B[4 * q + 0] = b.x; B[4 * q + 1] = b.y; B[4 * q + 2] = b.z; B[4 * q + 3] = b.w;
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");            // runs are in registers
        if (!FUSE && next < iend) issue_buf<BUFD, TILE, true>(data, T.span, ntile, lds0, lane);
        const int64_t t0 = (int64_t)tile * TILE;
        uint16_t *bm = (uint16_t *)(T.dense_bits + (size_t)idx * (TILE / 32));
        uint32_t rr[NG];
        uint32_t cnt = dense_roll<RUN>(A, B, P, lane, span - t0, [&](int g, uint32_t r) {
            if constexpr (!FUSE) {
                bm[lane * NG + g] = (uint16_t)(r >> 16);
                bm[(lane + 64) * NG + g] = (uint16_t)r;
            }
            rr[g] = r;
        });
        for (int off = 32; off >= 1; off >>= 1) cnt += __shfl_xor(cnt, off);
        DENSE_STAMP(ndone, 2);
        bool fixed = false;
        if constexpr (FUSE) {
            // a tile whose fix-ups are stored gets its candidates as a position list
            // (dense_pos, 2 B per candidate) instead of the bitmap (TILE / 8 bytes)
            fixed = dense_fixups<RUN>(dbuf, P, T, rr, cnt, idx, t0, lane);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");        // the fix-ups' LDS reads are done
            DENSE_STAMP(ndone, 3);
            if (next < iend) {
                DENSE_STAMP(ndone + 1u, 0);
                issue_buf<BUFD, TILE, true>(data, T.span, ntile, lds0, lane);
            }
            if (!fixed) {
#pragma unroll
                for (int g = 0; g < NG; ++g) {
                    bm[lane * NG + g] = (uint16_t)(rr[g] >> 16);
                    bm[(lane + 64) * NG + g] = (uint16_t)rr[g];
                }
            }
        }
        if ((tile >> 12) != cur_c) {
            if (lane == 0 && acc_c) atomicAdd(&T.coarse[cur_c * COARSE_STRIDE], acc_c);
            cur_c = tile >> 12;
            acc_c = 0;
        }
        acc_c += cnt;
        ++ndone;
        if (lane == 0) {
            T.dense_cnt[idx] = cnt | (fixed ? DENSE_FIXED : 0u);
            atomicAdd(&T.super_cnt[tile >> 6], cnt);
        }
        tile = ntile;
    }
    if (lane == 0 && acc_c) atomicAdd(&T.coarse[cur_c * COARSE_STRIDE], acc_c);
    if (lane == 0) atomicAdd(&T.split[SPL_DENSE_TILES], ndone);     // real tiles, for the stats
    if (blockIdx.x < (uint32_t)DBG_NDW) SCAN_STAMP(T, DBG_DW + 2 * blockIdx.x + 1, wall_clock64() | ((uint64_t)ndone << 56));
#undef DENSE_STAMP
}

// Compact every tile's candidates into T.cand in position order (one wave per
// 64-tile group; empty groups exit on their bitset word).  A sparse tile's
// lane copies its slot list; the wave then walks the group's dense tiles
// together: 64 bitmap words at a time, a wave prefix of their popcounts gives
// each lane its output run.
// The exclusive prefix of the candidate counts before 64-tile group w, from
// the counts per 4096 tiles (coarse) and per 64 tiles (super_cnt): two wave
// reductions instead of a separate one-block prefix launch.  Every wave of the
// gather computes its own word's prefix; the resolve reads super_off.
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, off), hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), off);
        v += ((uint64_t)hi << 32) | lo;
    }
    return v;
}

__device__ __forceinline__ uint64_t word_prefix(const Tables &T, uint32_t w, int lane) {
    const uint32_t c = w >> 6;
    uint64_t a = 0;
    for (uint32_t k = (uint32_t)lane; k < c; k += 64) a += T.coarse[k * COARSE_STRIDE];
    const uint32_t f = 64 * c + (uint32_t)lane;
    if (f < w) a += T.super_cnt[f];
    return readlane64(wave_sum64(a), 0);
}

// A nonempty tile's candidate count for the compaction and its tile_meta (DENSE_BIT |
// dense index, else 0 or the count).
__device__ __forceinline__ uint32_t tile_cands_of(const Tables &T, uint32_t m, uint32_t &meta) {
    meta = m;
    if (meta & DENSE_BIT) {
        const uint32_t idx = meta & ~DENSE_BIT;
        return (!T.dense_off && idx < T.dense_cap) ? T.dense_cnt[idx] & ~DENSE_FIXED : 0u;
    }
    return meta;
}
__device__ __forceinline__ uint32_t tile_cands(const Tables &T, uint32_t tile, uint32_t &meta) {
    return tile_cands_of(T, T.tile_meta[tile], meta);
}

// Dense tiles are expanded by the blocks past the word blocks, one wave per
// dense tile (grid-stride over the dense list): a word of 64 dense tiles on
// one wave was 64 dependent bitmap passes (dense1: 330 us for 2.1 M candidates).
__device__ __forceinline__ void gather_dense(const Tables &T, int lane, uint32_t wid, uint32_t nw_waves) {
    if (T.dense_off) return;                                 // (no blocks are launched for it then)
    const uint32_t nd = min(T.ctr[CTR_DENSE], T.dense_cap);
    const uint32_t nw = T.tile / 32;
    for (uint32_t idx = wid; idx < nd; idx += nw_waves) {
        const uint32_t tile = T.dense_list[idx];
        if (tile == DENSE_HOLE) continue;                        // an unused slot of a wave's chunk
        const uint32_t w = tile >> 6;
        // this tile's output offset: its word's prefix of per-tile counts
        const unsigned long long bits = T.nonempty[w];
        const uint32_t tl = w * 64 + (uint32_t)lane;
        uint32_t c = 0;
        if ((bits >> lane) & 1ull) {
            uint32_t meta;
            c = tile_cands(T, tl, meta);
        }
        const uint32_t incl = wave_incl_scan(c, lane);
        const uint32_t j = tile & 63u;
        const uint64_t tb = word_prefix(T, w, lane) + (uint32_t)__builtin_amdgcn_readlane((int)(incl - c), (int)j);
        const uint32_t tc = (uint32_t)__builtin_amdgcn_readlane((int)c, (int)j);
        if (!tc || tb + tc > T.cand_cap) continue;                // overflow: flagged by prefix, re-run
        const uint32_t *bm = T.dense_bits + (size_t)idx * nw;
        const uint64_t t0 = (uint64_t)tile * T.tile;
        if (T.dense_cnt[idx] & DENSE_FIXED) {
            // the dense pass stored rank r's position and head fix-up (dense_pos / dense_fix)
            const uint16_t *ps = T.dense_pos + (size_t)idx * FIXCAP;
            const uint8_t *fx = T.dense_fix + (size_t)idx * FIXCAP;
            // and, with chain links on, each candidate's link but the tile's last
            // (its next candidate is in another tile: cdc_fix_kernel decides it)
            for (uint32_t r = (uint32_t)lane; r < tc; r += 64) {
                const uint32_t p = ps[r], f = fx[r];
                uint64_t lk = 0;
                if (T.linkw && r + 1 < tc) {
                    const uint32_t d = (uint32_t)ps[r + 1] - p;
                    lk = CAND_LDEC | ((f == 0u && d >= 64u && (uint64_t)d <= T.gapmax) ? CAND_LINK : 0ull);
                }
                st_u64(&T.cand[tb + r], (t0 + p) | ((uint64_t)f << 48) | CAND_KNOWN | lk, T.nt_out);
            }
            continue;
        }
        uint64_t o = tb;
        for (uint32_t b0 = 0; b0 < nw; b0 += 64) {
            const uint32_t wi = b0 + (uint32_t)lane;
            uint32_t m = wi < nw ? bm[wi] : 0u;
            const uint32_t pc = (uint32_t)__builtin_popcount(m);
            const uint32_t ic = wave_incl_scan(pc, lane);
            uint64_t q = o + (ic - pc);
            while (m) {
                st_u64(&T.cand[q++], t0 + wi * 32u + (uint32_t)__builtin_ctz(m), T.nt_out);
                m &= m - 1;
            }
            o += (uint32_t)__builtin_amdgcn_readlane((int)ic, 63);
        }
    }
}

__global__ __launch_bounds__(256) void cdc_gather_kernel(Tables T) {
    const uint32_t w = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const uint32_t wblocks = (T.nwords + 3) / 4;
    if (blockIdx.x >= wblocks) {
        gather_dense(T, lane, (blockIdx.x - wblocks) * 4 + (threadIdx.x >> 6), (gridDim.x - wblocks) * 4);
        return;
    }
    if (w >= T.nwords) return;
    if (w == 0) {                                             // the total (fix-ups, resolve, fetch)
        uint64_t a = 0;
        for (uint32_t k = (uint32_t)lane; k < T.ncoarse; k += 64) a += T.coarse[k * COARSE_STRIDE];
        const uint64_t total = readlane64(wave_sum64(a), 0);
        if (lane == 0) {
            T.super_off[T.nwords] = total;
            T.ctr[CTR_CANDS_LO] = (uint32_t)total;
            T.ctr[CTR_CANDS_HI] = (uint32_t)(total >> 32);
            if (total > T.cand_cap) T.ctr[CTR_FLAGS] |= FLAG_CAND_OVERFLOW;
        }
    }
    // the word's bits and its tiles' metas are loaded with the prefix's counts (one round
    // trip, not three: the super_off store kept them behind the prefix)
    const uint32_t tile = w * 64 + lane;
    const unsigned long long bits = T.nonempty[w];
    const uint32_t m0 = T.tile_meta[tile < T.ntiles ? tile : 0u];
    const uint64_t pre = word_prefix(T, w, lane);
    if (lane == 0) T.super_off[w] = pre;
    if (!bits) return;
    const bool has = (bits >> lane) & 1ull;
    uint32_t meta = 0, c = 0;
    if (has) c = tile_cands_of(T, m0, meta);
    const uint32_t incl = wave_incl_scan(c, lane);
    const uint64_t base = pre + (incl - c);
    const bool dense = has && (meta & DENSE_BIT) && c;
    if (has && c && !dense && base + c <= T.cand_cap) {   // overflow is flagged by prefix; host re-runs
        const uint64_t t0 = (uint64_t)tile * T.tile;
        const uint2 *sl = T.slots + (size_t)tile * LISTCAP;
        for (uint32_t j = 0; j < c; ++j) st_u64(&T.cand[base + j], t0 + sl[j].x, T.nt_out);   // fix-up: cdc_fix_kernel
    }
    (void)dense;                                               // dense tiles: gather_dense
}

// Compaction and head fix-ups in one launch, for launches with no dense pass and
// no chain links (random data, the common case: cdc_gather_kernel followed by
// cdc_fix_kernel otherwise).  A word wave computes its 64 tiles' output offsets as
// the gather does, stages the word's candidates (word-relative positions, in
// order) in LDS 128 at a time, and rolls their head fix-ups two per lane as
// cdc_fix_kernel does: every candidate is written once, complete (CAND_KNOWN).
// The blocks past the word blocks compute the read-boundary grid points' fix-ups.
// One dependent launch fewer per step: on small batches (BASELINE config 4's
// per-rank shards, 1 GiB) the chain of short post-scan launches is ~10 % of a step.
__global__ __launch_bounds__(256) void cdc_gather_fix_kernel(const uint8_t *__restrict__ data, KParams P,
                                                             Tables T) {
    __shared__ uint32_t lpos[4][128];
    const uint32_t wv = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const uint32_t wblocks = (T.nwords + 3) / 4;
    if (blockIdx.x >= wblocks) {                              // grid points, two per lane
        const uint32_t nthr = (gridDim.x - wblocks) * 256;
        for (uint64_t q = (uint64_t)(blockIdx.x - wblocks) * 256 + threadIdx.x; 2 * q < T.ngrid; q += nthr) {
            uint64_t a[2] = {0, 0};
            uint32_t n[2] = {0, 0};
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint64_t i = 2 * q + (uint64_t)h;
                if (i < T.ngrid) {
                    a[h] = T.gpos[i];
                    const uint64_t end = T.gend[i];
                    n[h] = (uint32_t)min<uint64_t>(63ull, end > a[h] ? end - a[h] : 0ull);
                }
            }
            uint32_t A[16], B[16], fA = 0u, fB = 0u;
            fix_load(data, T.span, a[0], n[0], A);
            fix_load(data, T.span, a[1], n[1], B);
            fix_pair(A, B, n[0], n[1], P, fA, fB);
            T.gfix[2 * q] = (uint8_t)fA;
            if (2 * q + 1 < T.ngrid) T.gfix[2 * q + 1] = (uint8_t)fB;
        }
        return;
    }
    const uint32_t w = blockIdx.x * 4 + wv;
    if (w >= T.nwords) return;
    if (w == 0) {                                             // the total (resolve, fetch)
        uint64_t a = 0;
        for (uint32_t k = (uint32_t)lane; k < T.ncoarse; k += 64) a += T.coarse[k * COARSE_STRIDE];
        const uint64_t total = readlane64(wave_sum64(a), 0);
        if (lane == 0) {
            T.super_off[T.nwords] = total;
            T.ctr[CTR_CANDS_LO] = (uint32_t)total;
            T.ctr[CTR_CANDS_HI] = (uint32_t)(total >> 32);
            if (total > T.cand_cap) T.ctr[CTR_FLAGS] |= FLAG_CAND_OVERFLOW;
        }
    }
    const uint32_t tile = w * 64 + (uint32_t)lane;
    const unsigned long long bits = T.nonempty[w];                 // (loaded with the prefix's counts)
    const uint32_t m0 = T.tile_meta[tile < T.ntiles ? tile : 0u];
    const uint64_t pre = word_prefix(T, w, lane);
    if (lane == 0) T.super_off[w] = pre;
    if (!bits) return;
    const bool has = (bits >> lane) & 1ull;
    uint32_t meta = 0, c = 0;
    if (has) c = tile_cands_of(T, m0, meta);                 // (dense_off: a dense tile counts 0; fetch re-runs)
    if (meta & DENSE_BIT) c = 0u;
    const uint32_t incl = wave_incl_scan(c, lane);
    const uint32_t ctot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    const uint32_t b0 = incl - c;                             // this tile's first word-relative index
    const uint64_t wbase = (uint64_t)w * 64u * T.tile;
    const uint32_t trel = (uint32_t)lane * T.tile;           // this tile's offset in the word
    const uint2 *sl = T.slots + (size_t)tile * LISTCAP;
    for (uint32_t k0 = 0; k0 < ctot; k0 += 128) {
        // stage positions k0 .. k0 + 127 of the word's ordered candidates
        if (c && b0 < k0 + 128 && b0 + c > k0) {
            for (uint32_t j = 0; j < c; ++j) {
                const uint32_t i = b0 + j;
                if (i >= k0 && i < k0 + 128) lpos[wv][i - k0] = trel + sl[j].x;
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        uint64_t a[2] = {0, 0};
        uint32_t n[2] = {0, 0};
        bool in[2] = {false, false};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t i = k0 + 2u * (uint32_t)lane + (uint32_t)h;
            if (i < ctot) {
                in[h] = true;
                a[h] = wbase + lpos[wv][2 * lane + h] + 1;      // a candidate e: the chunk starts at e + 1
                n[h] = (uint32_t)min<uint64_t>(63ull, T.span > a[h] ? T.span - a[h] : 0ull);
            }
        }
        uint32_t fA = 0u, fB = 0u;
        if (__ballot(in[0])) {
            uint32_t A[16], B[16];
            fix_load(data, T.span, a[0], n[0], A);
            fix_load(data, T.span, a[1], n[1], B);
            fix_pair(A, B, n[0], n[1], P, fA, fB);
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint64_t o = pre + k0 + 2u * (uint32_t)lane + (uint32_t)h;
            if (in[h] && o < T.cand_cap) st_u64(&T.cand[o], (a[h] - 1) | ((uint64_t)(h ? fB : fA) << 48) | CAND_KNOWN, T.nt_out);
        }
        __builtin_amdgcn_wave_barrier();                       // (the staging is reused)
    }
}

// ---------------------------------------------------------------------------
// Resolve: one lane per file walks compute_file_chunks' loop over the sorted
// candidate array.
// ---------------------------------------------------------------------------
// First chunk-local hit in [a, b) for a chunk starting at a (b - a <= 63);
// all loads issued up front (no early exit in the load stream).
__device__ uint64_t head_scan(const uint8_t *data, uint64_t a, uint64_t b, uint32_t mask) {
    const uint32_t n = (uint32_t)(b - a);
    uint32_t x[63];
#pragma unroll
    for (uint32_t k = 0; k < 63; ++k) x[k] = k < n ? data[a + k] : 0u;
    uint32_t S = 0, W = 0;
    uint64_t hit = NONE;
#pragma unroll
    for (uint32_t k = 0; k < 63; ++k) {
        S += x[k];
        W += S;
        if (hit == NONE && k < n && hit_exact(S, W, mask)) hit = a + k;
    }
    return hit;
}

// The next launch's zeroed block (and this launch's hash counters), written by
// the resolve kernel's threads instead of a memset packet before the next scan.
__device__ __forceinline__ void zero_next(const Tables &T) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x, nthr = gridDim.x * blockDim.x;
    if (T.znext)
        for (uint32_t k = tid; k < T.znext_vec; k += nthr) T.znext[k] = make_uint4(0u, 0u, 0u, 0u);
    if (T.hzero && tid < (uint32_t)B3C_WORDS) T.hzero[tid] = 0ull;
    if (T.hzero && tid < B3_SHARDS) T.hzero[(tid + 1) * B3_SHARD_STRIDE] = 0ull;
}

__global__ __launch_bounds__(64) void cdc_resolve_kernel(const uint8_t *__restrict__ data, KParams P,
                                                         Tables T) {
    scan_time_account(T);
    zero_next(T);
    const uint32_t kf = blockIdx.x * 64 + threadIdx.x;
    if (kf >= T.nfiles) return;
    const uint32_t i = T.order[kf];
    const ulonglong2 fr = T.ofile[kf];                          // {foff, flen} of file i
    const uint64_t F = fr.y, g0 = fr.x;
    DevCut *out = T.cuts + T.cut_base[i];
    const uint32_t cap = T.cut_cap[i];
    const uint64_t MAX = P.max_chunk;
    const uint64_t CAP = P.read_cap ? P.read_cap : ~0ull;
    const uint64_t total = (uint64_t)T.ctr[CTR_CANDS_LO] | ((uint64_t)T.ctr[CTR_CANDS_HI] << 32);
    const uint64_t ncand = min(total, T.cand_cap);
    // first candidate at or after the file start
    uint64_t j = 0;
    if (F) {
        const uint32_t w = (uint32_t)((g0 / T.tile) >> 6);
        uint64_t lo = T.super_off[w], hi = min(T.super_off[w + 1], ncand);
        while (lo < hi) {
            const uint64_t mid = lo + ((hi - lo) >> 1);
            if ((T.cand[mid] & CAND_POS_MASK) < g0) lo = mid + 1; else hi = mid;
        }
        j = lo;
    }
    uint64_t cv = j < ncand ? T.cand[j] : NONE;         // current candidate word
    uint64_t cnt = 0;
    // compute_file_chunks (file_operations.rs:737-784): R = bytes buffered.
    uint64_t R = min(min(F, MAX), CAP);                   // first read :738
    uint64_t s = 0;
    int head = 2;            // 1: fix known, 2: unknown (head scan; also at the file start)
    uint32_t fix = 0;
    while (s < R) {                                       // n = R - s > 0  :747
        const uint64_t lim = R;                           // endofs = min(MAX, n) :749-752
        uint64_t e = NONE;
        bool known = false;
        uint32_t cfix = 0;
        uint64_t from = s + 63;                           // stream G applies from here
        {
            uint64_t hh = NONE;
            if (head == 1) {
                if (fix) hh = s - 1 + fix;
            } else {
                const uint64_t h = head_scan(data, g0 + s, g0 + min(s + 63, lim), P.mask);
                if (h != NONE) hh = h - g0;
            }
            if (hh != NONE && hh < lim) e = hh;           // chunk-local head hit
        }
        if (e == NONE && from < lim) {
            const uint64_t a = g0 + from, b = g0 + lim;
            while (j < ncand && (cv & CAND_POS_MASK) < a) {
                ++j;
                cv = j < ncand ? T.cand[j] : NONE;
            }
            if (j < ncand && (cv & CAND_POS_MASK) < b) {
                e = (cv & CAND_POS_MASK) - g0;
                known = (cv & CAND_KNOWN) != 0;
                cfix = (uint32_t)(cv >> 48) & 0xffu;
            }
        }
        uint64_t cut;                                     // edge or endofs :754-755
        if (e != NONE) { cut = e + 1; head = known ? 1 : 2; fix = cfix; }
        else { cut = lim; head = 2; }
        if (cnt < cap) {
            DevCut d;
            d.offset = s;
            d.len = (uint32_t)(cut - s);
            d.file = i;
            st_cut(out + cnt, d, T.nt_out);
        }
        ++cnt;
        s = cut;                                          // copy_within :771
        uint64_t rd = MAX - (R - s);                      // f.read(&mut buf[n..]) :776
        rd = min(rd, CAP);
        rd = min(rd, F - R);
        R += rd;
    }
    T.counts[i] = cnt;
    if (cnt > cap) atomicOr(&T.ctr[CTR_FLAGS], FLAG_CUT_OVERFLOW);
}

// ---------------------------------------------------------------------------
// Resolve, one WAVE per file (default).  The wave holds a window of 64
// consecutive sorted candidates (one coalesced load); the next candidate at
// or after `a` is the first set bit of a ballot.  An unknown head fix-up is one
// coalesced 63-byte load plus two wave prefix sums (S, then W).  All control
// state is wave-uniform, so the serial compute_file_chunks walk costs a few
// scalar/vector ops per cut instead of a dependent memory round trip.
// ---------------------------------------------------------------------------

// First index in [lo, hi) whose candidate position is >= key (cand sorted), by
// 64 probes per round: two or three dependent loads for a 64-tile group.
__device__ __forceinline__ uint64_t wave_lower_bound(const uint64_t *cand, uint64_t lo, uint64_t hi, uint64_t key,
                                                     int lane) {
    if (lo > hi) lo = hi;
    while (hi - lo > 64) {
        const uint64_t n = hi - lo;
        const uint64_t idx = lo + n * (uint64_t)(lane + 1) / 65;          // 64 increasing probes in [lo, hi)
        const uint32_t c = (uint32_t)__builtin_popcountll(__ballot((cand[idx] & CAND_POS_MASK) < key));
        const uint64_t nlo = c ? lo + n * c / 65 + 1 : lo;               // past the last probe below key
        const uint64_t nhi = c < 64 ? lo + n * (c + 1) / 65 : hi;         // the first probe at or above key
        lo = nlo;
        hi = nhi;
    }
    const uint64_t idx = lo + (uint64_t)lane;
    const uint64_t r = lo + (uint64_t)__builtin_popcountll(__ballot(idx < hi && (cand[idx] & CAND_POS_MASK) < key));
    return readlane64(r, 0);                     // wave-uniform to the compiler
}

// SplitSeg fields written by another wave are read with agent-scope atomic
// loads: a plain load with a wave-uniform address may be a scalar load through
// the scalar cache, which the acquire does not make coherent (stale fields
// from an earlier launch were read that way).
__device__ __forceinline__ uint32_t seg_ld(const uint32_t &f) {
    return (uint32_t)__builtin_amdgcn_readfirstlane(
        __hip_atomic_load(&f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ uint64_t seg_ld(const uint64_t &f) {
    const uint64_t v = __hip_atomic_load(&f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
}

// Wall-clock budget of a wave's waits on other waves (s_memrealtime, constant rate).
struct Patience {
    uint64_t deadline;
    __device__ __forceinline__ explicit Patience(uint64_t ticks)
        : deadline(ticks ? wall_clock64() + ticks : 0ull) {}
    __device__ __forceinline__ bool spent() const { return deadline == 0ull || wall_clock64() > deadline; }
};

// development timeline (Tables::dbg, SYNCR_CDC_TRACE=1): lane 0 stamps wall_clock64
#ifdef SYNCR_CDC_DEV
#define DBG_STAMP(T, slot) do { if ((T).dbg && lane == 0) (T).dbg[(slot)] = wall_clock64(); } while (0)
#define DBG_MIN(T, slot) do { if ((T).dbg && lane == 0) atomicMax((unsigned long long *)&(T).dbg[(slot)], \
                                  ~(unsigned long long)wall_clock64()); } while (0)     /* stored inverted */
#define DBG_MAX(T, slot) do { if ((T).dbg && lane == 0) atomicMax((unsigned long long *)&(T).dbg[(slot)], \
                                  (unsigned long long)wall_clock64()); } while (0)
#else
#define DBG_STAMP(T, slot) do { } while (0)
#define DBG_MIN(T, slot) do { } while (0)
#define DBG_MAX(T, slot) do { } while (0)
#endif

__device__ __forceinline__ unsigned long long *split_pub(const Tables &T) {
    return reinterpret_cast<unsigned long long *>(&T.split[SPL_PUB64]);
}

// Split setup by the walker of an eligible file (Tables::n_elig): when the file
// holds >= 2 SPLIT_SEGC candidates, reserve and initialise the SplitSeg records
// of its boundaries 1 .. nseg-1 (boundary k = its k * SPLIT_SEGC-th candidate)
// for the extra resolve waves to walk.  Returns the record of boundary 1 and
// the segment count (nseg = 0: not split).  Every eligible walker then counts
// itself in the SPL_PUB64 count exactly once, after its reservation.
__device__ __forceinline__ void split_setup(const KParams &P, const Tables &T, uint32_t i, uint64_t F, uint64_t g0,
                                            uint64_t ncand, int lane, uint32_t &first, uint32_t &nseg) {
    first = 0;
    nseg = 0;
    if (!P.resolve_nosplit && F && F <= 0xFFFFFF00ull && T.seg_cap) {
        const uint32_t w0 = (uint32_t)((g0 / T.tile) >> 6), w1 = (uint32_t)(((g0 + F - 1) / T.tile) >> 6);
        const uint64_t a0 = T.super_off[w0], a1 = T.super_off[w0 + 1], b0 = T.super_off[w1], b1 = T.super_off[w1 + 1];
        const uint64_t SEGC = T.seg_segc;
        if (b1 - a0 >= 2ull * SEGC) {                             // upper bound on the file's candidates
            const uint64_t j0 = wave_lower_bound(T.cand, min(a0, ncand), min(a1, ncand), g0, lane);
            const uint64_t j1 = wave_lower_bound(T.cand, min(b0, ncand), min(b1, ncand), g0 + F, lane);
            const uint64_t ns = j1 > j0 ? (j1 - j0) / SEGC : 0;
            if (ns >= 2 && ns < 0x10000ull) {
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(&T.split[SPL_RESERVED], (uint32_t)ns - 1u);
                base = (uint32_t)__builtin_amdgcn_readfirstlane(base);
                const bool fits = (uint64_t)base + ns - 1 <= (uint64_t)T.seg_cap;
                const uint64_t MAX = P.max_chunk;
                for (uint32_t r = (uint32_t)lane; r + 1 < (uint32_t)ns; r += 64) {
                    const uint32_t q = base + r;
                    if (q >= T.seg_cap) continue;
                    SplitSeg &g = T.segs[q];
                    g.k = 0;                                          // unusable unless it fits
                    if (fits) {
                        const uint64_t cidx = j0 + (uint64_t)(r + 1) * SEGC;
                        const uint64_t s0 = (T.cand[cidx] & CAND_POS_MASK) - g0 + 1;
                        g.cidx = cidx;
                        g.out_off = 0;
                        g.file = i;
                        g.k = r + 1;
                        g.s0 = (uint32_t)s0;
                        g.R0 = (uint32_t)min(F, s0 + MAX);
                        g.first = base;
                        g.nseg = (uint32_t)ns;
                        g.res = seg_res(SEG_PENDING, 0u, 0u);
                        g.verdict = 0;
                        g.run_pre = 0;
                        g.run_len = 0;
                    }
                }
                __threadfence();
                for (uint32_t r = (uint32_t)lane; r + 1 < (uint32_t)ns; r += 64)
                    if (base + r < T.seg_cap)
                        __hip_atomic_store(&T.segs[base + r].ready, T.epoch, __ATOMIC_RELEASE,
                                           __HIP_MEMORY_SCOPE_AGENT);
                if (fits) {                                       // (uniform again after the lane loops)
                    first = (uint32_t)__builtin_amdgcn_readfirstlane(base);
                    nseg = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)ns);
                }
            }
        }
    }
    // (a reservation precedes the fence before the records' ready stores, so it
    // is ordered before this count)
    if (lane == 0) atomicAdd(split_pub(T), (nseg ? 1ull << 32 : 0ull) + 1ull);
}

// The walk of one file, in file-relative offsets of type Off (uint32_t for
// files below 4 GiB: every comparison and min stays in the scalar unit, which
// has no 64-bit unsigned compare).  Per window lane: wr = candidate position
// relative to the file (below the file -> 0, at/after its end or none -> OMAX;
// monotone, so the window stays sorted), wk = head fix-up | known << 8.
// Cuts are gathered into two VGPRs (lane k = k-th cut of a batch of 64) and
// stored 64 at a time.
//
// Split walks (Off = uint32_t): `elig` = the walker of an eligible file (it may
// split the file, then adopts segment walks at its boundaries); spec >= 0 = the
// walk of segment record `spec`, from that segment's start state into scratch,
// until it lands on a later boundary with that boundary's start state (link),
// reaches the file end, or passes two boundaries without landing (abort).
template <typename Off, int PF, bool SPLIT>
__device__ __forceinline__ void resolve_walk(const uint8_t *__restrict__ data, const KParams &P,
                                             const Tables &T, uint32_t i, uint64_t F, uint64_t g0, int lane,
                                             bool elig, uint32_t spec, const uint64_t *ring) {
    constexpr Off OMAX = (Off)~(Off)0;
    // SPLIT = false: a launch without split workers (no segment records, no
    // run skips, no deferral): the random-data walk, without the long-walk
    // machinery's registers
    const bool is_spec = SPLIT && spec != SPLIT_END;
    DevCut *out = is_spec ? T.seg_cuts + (uint64_t)spec * T.seg_scap : T.cuts + T.cut_base[i];
    uint64_t cap = is_spec ? (uint64_t)T.seg_scap : (uint64_t)T.cut_cap[i];
    // runs deferred to the copy launch (only while it runs: split workers
    // launched); a segment walk defers at most one, its scratch skipping it
    const bool defer = SPLIT && T.runs_cap && !P.resolve_nosplit;
    uint32_t run_pre = 0, run_len = 0;
    const Off Fo = (Off)F;
    const Off MAX = (Off)min<uint64_t>(P.max_chunk, (uint64_t)OMAX);
    const Off CAP = P.read_cap ? (Off)min<uint64_t>(P.read_cap, (uint64_t)OMAX) : OMAX;
    const uint64_t total = (uint64_t)T.ctr[CTR_CANDS_LO] | ((uint64_t)T.ctr[CTR_CANDS_HI] << 32);
    const uint64_t ncand = min(total, T.cand_cap);
    // split state: the file's remaining boundaries are records [brec, bend);
    // sb = the next one's start (OMAX: none)
    uint32_t brec = 0, bend = 0;
    const bool dbgw = elig && T.order[0] == i;              // (development timeline: the largest file)
    (void)dbgw;
    if (dbgw) DBG_STAMP(T, DBG_W_ENTRY);
    if (SPLIT && elig) {
        uint32_t first, nseg;
        split_setup(P, T, i, F, g0, ncand, lane, first, nseg);
        if (dbgw) DBG_STAMP(T, DBG_W_SETUP);
        if (nseg) {
            brec = first;
            bend = first + nseg - 1;
        }
    }
    if (is_spec) {
        brec = spec + 1;
        bend = seg_ld(T.segs[spec].first) + seg_ld(T.segs[spec].nseg) - 1;
    }
    if constexpr (sizeof(Off) != 4) bend = 0;
    Off sb = OMAX;
    uint64_t sbi = NONE;                     // the next boundary's candidate index (run skips stop there)
    auto load_bnd = [&]() {
        sb = brec < bend ? (Off)seg_ld(T.segs[brec].s0) : OMAX;
        sbi = brec < bend ? seg_ld(T.segs[brec].cidx) : NONE;
    };
    load_bnd();
    uint64_t wb = is_spec ? seg_ld(T.segs[spec].cidx)
                          : (F ? T.super_off[(uint32_t)((g0 / T.tile) >> 6)] : 0);   // the file's 64-tile group
    if (!is_spec && F) {
        // a group crowded with another file's candidates (a periodic file before
        // this one in the same 64 tiles, 1.1 MiB): start at the file's own first
        // candidate instead of sliding through them a window at a time (dense
        // workload: up to 288 slides, ~150 us, for a random file's walker)
        const uint64_t ge = min(T.super_off[(uint32_t)((g0 / T.tile) >> 6) + 1], ncand);
        if (ge > wb && ge - wb > 128u) wb = wave_lower_bound(T.cand, wb, ge, g0, lane);
    }
    Off wr = OMAX;
    uint32_t wk = 0, nx = 64;
    // Candidate windows stream through the wave's LDS ring of PF slots (ring:
    // PF x 64 words) by LDS-DMA, two dword DMAs per 64-candidate window, PF-1
    // windows ahead of the one in use.  Completion is tracked by hand: a window
    // has 2 (PF-1) DMAs issued after it, so s_waitcnt vmcnt(2 (PF-1)) retires it
    // (vector-memory operations retire in issue order; other loads and stores in
    // between only make that wait stricter).  No register ever holds an
    // in-flight window: a register ring rotated at each slide made hipcc wait
    // vmcnt(0) at the rotation, one HBM round trip per 64 candidates.  Indices
    // are clamped (entries past ncand are masked when the window is consumed).
    const uint32_t ring0 = (uint32_t)__builtin_amdgcn_readfirstlane(lds_addr(ring));
    uint32_t rh = 0;                                  // slot of the current window
    auto issue = [&](uint64_t b, uint32_t slot) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint64_t k = b + (uint64_t)((64 * h + lane) >> 1);   // dword 64h + lane of the window
            const uint8_t *src = (const uint8_t *)(T.cand + (k < ncand ? k : 0)) + ((lane & 1) << 2);
            dma4(src, (uint32_t)__builtin_amdgcn_readfirstlane(ring0 + slot * 512u + (uint32_t)h * 256u));
        }
    };
    auto prime = [&]() {                              // the windows from wb on, slots 0 .. PF-1
        wait_vmcnt<0>();                              // (no older DMA may still land in a slot)
#pragma unroll
        for (int k = 0; k < PF; ++k) issue(wb + 64ull * k, (uint32_t)k);
        rh = 0;
    };
    auto cur = [&]() -> uint64_t {                    // this lane's word of the current window
        wait_vmcnt<2 * (PF - 1)>();
        return ring[rh * 64u + (uint32_t)lane];
    };
    auto slide = [&]() {                              // the current window has been consumed
        issue(wb + 64ull * PF, rh);
        wb += 64;
        rh = (rh + 1u) & (uint32_t)(PF - 1);
    };
    prime();
    auto load_window = [&]() {
        const uint64_t raw = cur();
        const uint64_t c = wb + (uint64_t)lane < ncand ? raw : NONE;
        wr = OMAX;
        wk = 0;
        if (c != NONE) {
            const uint64_t p = c & CAND_POS_MASK;
            wr = p < g0 ? (Off)0 : (p - g0 >= F ? OMAX : (Off)(p - g0));
            wk = (uint32_t)((c >> 48) & 0xffu) | ((c & CAND_KNOWN) ? 0x100u : 0u) | ((c & CAND_LINK) ? 0x200u : 0u);
        }
        // nx: window index of the first candidate >= this lane's + 64, where the
        // search resumes after a cut at it with no head hit (64 = past the window)
        const Off key = wr == OMAX ? OMAX : (Off)(wr + 64);
        if constexpr (sizeof(Off) == 4) {
            // dense windows (periodic data: a candidate every 64 bytes): every
            // lane's answer is the next lane, found with one shuffle instead of
            // six dependent ones.  (nx of a lane past the file is never read.)
            const Off up = (Off)down1((uint32_t)wr);
            if (__ballot(lane == 63 || up >= key) == ~0ull) {
                nx = (uint32_t)lane + 1u;
                return;
            }
        }
        uint32_t idx = 0;
#pragma unroll
        for (uint32_t st = 32; st >= 1; st >>= 1) {
            Off pv;
            if constexpr (sizeof(Off) == 4) {
                pv = (Off)__shfl((int)wr, (int)(idx + st - 1));
            } else {
                const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)wr, (int)(idx + st - 1));
                const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)((uint64_t)wr >> 32), (int)(idx + st - 1));
                pv = (Off)(((uint64_t)hi << 32) | lo);
            }
            if (pv < key) idx += st;
        }
        nx = idx;
    };
    auto rl = [&](Off v, uint32_t k) -> Off {                // readlane of an Off
        if constexpr (sizeof(Off) == 4) {
            return (Off)__builtin_amdgcn_readlane((int)v, (int)k);
        } else {
            const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)k);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), (int)k);
            return (Off)(((uint64_t)hi << 32) | lo);
        }
    };
    load_window();
    // head hits at this file's read-boundary grid points (lane k: k * read_cap)
    const uint64_t CAPv = P.read_cap;
    const bool grid = T.ngrid && CAPv && F;
    uint64_t gb = 0;
    uint32_t gf = 0;
    if (grid) {
        gb = T.gbase[i];
        if ((uint64_t)lane * CAPv < F) gf = T.gfix[gb + lane];
    }
    // gathered cuts: lane k of (bo, bl) = cut (cnt & ~63) + k, valid from slot bstart
    // (the slots below it were written directly by a burst, see below)
    Off bo = 0;
    uint32_t bl = 0;
    Off cnt = 0;             // cuts so far (< F + 1, so Off is wide enough)
    uint32_t bstart = 0;
    auto flush = [&](uint32_t n) {
        const uint64_t k = (uint64_t)(cnt - n) + (uint64_t)lane;   // cnt already counts these n cuts
        if ((uint32_t)lane >= bstart && (uint32_t)lane < n && k < cap) {
            DevCut d;
            d.offset = (uint64_t)bo;
            d.len = bl;
            d.file = i;
            st_cut(out + k, d, T.nt_out);
        }
    };
    Off R = min(min(Fo, MAX), CAP);                          // first read (file_operations.rs:738)
    Off s = 0;
    int head = 2;            // 1: fix known, 2: unknown (head scan / grid; also at the file start)
    uint32_t fix = 0;
    int jlast = -1;          // window index of the candidate the last cut was made at
    // a cut at window lane 0's candidate, buffer full (a segment's start state)
    auto start_at_lane0 = [&](Off s0, Off R0) {
        s = s0;
        R = R0;
        const uint32_t k0 = (uint32_t)__builtin_amdgcn_readlane((int)wk, 0);
        head = (k0 & 0x100u) ? 1 : 2;
        fix = k0 & 0xffu;
        jlast = 0;
    };
    if (is_spec) start_at_lane0((Off)seg_ld(T.segs[spec].s0), (Off)seg_ld(T.segs[spec].R0));
    uint32_t link = SPLIT_END;          // segment walk: the record it linked at / SPLIT_END / SPLIT_ABORT
    while (s < R) {                                          // :747
        if (SPLIT && s >= sb) {
            // at or past boundary brec: a landing with the boundary's start state
            // links (segment walk) or adopts the boundary's segment walk (file walker)
            bool stop = false;
            while (s >= sb) {
                if (s == sb && R == (Off)seg_ld(T.segs[brec].R0)) {
                    if (is_spec) {
                        link = brec;
                        stop = true;
                        break;
                    }
                    // Adopt the chain of done segment walks that starts here, 64
                    // records per memory round trip: lane k reads record brec + k's
                    // result word (cuts, link, status in one atomic load, so no
                    // acquire is needed: the cuts themselves are read only by the
                    // copy launch), and the chain brec -> link -> ... is followed on
                    // lane indices; a chain that leaves the block continues with the
                    // next block at once, without walking.  A segment a worker is
                    // walking right now ends soon: wait for it (bounded) rather than
                    // walk it again.
                    bool moved = false;
#ifdef SYNCR_CDC_DEV
                    uint32_t nblk = 0;
                    if (dbgw && T.dbg) nblk = (uint32_t)T.dbg[DBG_W_NBLK];
#endif
                    for (;;) {
#ifdef SYNCR_CDC_DEV
                        if (dbgw && nblk < DBG_MAXBLK / 2) DBG_STAMP(T, DBG_W_BLK + 2 * nblk);
#endif
                        const uint32_t rq = brec + (uint32_t)lane;
                        uint64_t rs = rq < bend ? __hip_atomic_load(&T.segs[rq].res, __ATOMIC_RELAXED,
                                                                     __HIP_MEMORY_SCOPE_AGENT) : 0ull;
                        uint32_t st0 = (uint32_t)__builtin_amdgcn_readlane((int)seg_res_status(rs), 0);
                        if (st0 == SEG_WALKING) {
                            const Patience pat(P.split_patience);
                            while (st0 == SEG_WALKING && !pat.spent()) {
                                __builtin_amdgcn_s_sleep(2);
                                rs = rq < bend ? __hip_atomic_load(&T.segs[rq].res, __ATOMIC_RELAXED,
                                                                   __HIP_MEMORY_SCOPE_AGENT) : 0ull;
                                st0 = (uint32_t)__builtin_amdgcn_readlane((int)seg_res_status(rs), 0);
                            }
                        }
                        if (st0 != SEG_DONE) break;
                        // (atomic results are divergent to the compiler: readlane keeps the
                        // walk state in scalar registers)
                        const uint32_t stv = seg_res_status(rs), nn = seg_res_n(rs), lkv = seg_res_link(rs);
                        // the usual chain links each record to the next one (periodic
                        // data): that prefix is one ballot; the rest (a jump, the chain's
                        // end) is followed lane by lane
                        const unsigned long long nextm =
                            __ballot(stv == SEG_DONE && lkv == rq + 1u && rq + 1u < bend);
                        const uint32_t run = ~nextm ? (uint32_t)__builtin_ctzll(~nextm) : 64u;
                        unsigned long long adopted = run >= 64u ? ~0ull : ((1ull << run) - 1ull);
                        uint32_t cur = run, last = brec + run;
                        for (; cur < 64u;) {                       // chain order = increasing lanes
                            if ((uint32_t)__builtin_amdgcn_readlane((int)stv, (int)cur) != SEG_DONE) {
                                last = brec + cur;                 // not done: the walk goes on here
                                break;
                            }
                            const uint32_t lk = (uint32_t)__builtin_amdgcn_readlane((int)lkv, (int)cur);
                            if (lk != SPLIT_END && (lk <= brec + cur || lk >= bend)) {   // (never)
                                last = brec + cur;
                                break;
                            }
                            adopted |= 1ull << cur;
                            last = lk;
                            if (lk == SPLIT_END || lk - brec >= 64u) break;
                            cur = lk - brec;
                        }
                        if (!adopted) break;
                        const uint32_t pend = (uint32_t)cnt & 63u;   // gathered cuts before the adopted ones
                        if (pend > bstart) flush(pend);
                        const bool mine = (adopted >> lane) & 1ull;
                        const uint32_t incl = wave_incl_scan(mine ? nn : 0u, lane);
                        if (mine) {
                            T.segs[rq].out_off = (uint64_t)cnt + (incl - nn);
                            T.segs[rq].verdict = 1u;
                        }
                        cnt += (Off)(uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
                        if (lane == 0) atomicAdd(&T.split[SPL_ADOPTED], (uint32_t)__builtin_popcountll(adopted));
                        bstart = (uint32_t)cnt & 63u;              // slots below: the copy kernel's
                        moved = true;
                        brec = last;
#ifdef SYNCR_CDC_DEV
                        if (dbgw && nblk < DBG_MAXBLK / 2) {
                            DBG_STAMP(T, DBG_W_BLK + 2 * nblk + 1);
                            ++nblk;
                            if (lane == 0 && T.dbg) T.dbg[DBG_W_NBLK] = nblk;
                        }
#endif
                        if (last == SPLIT_END) break;
                    }
                    if (moved) {
                        if (brec == SPLIT_END) {
                            stop = true;
                            break;
                        }
                        // at boundary brec with its start state: walk on from there
                        load_bnd();
                        wb = seg_ld(T.segs[brec].cidx);
                        prime();
                        load_window();
                        start_at_lane0(sb, (Off)seg_ld(T.segs[brec].R0));
                        continue;
                    }
                }
                ++brec;                                            // passed without adopting
                if (is_spec && brec > spec + 2) {                  // two boundaries without a landing
                    link = SPLIT_ABORT;
                    stop = true;
                    break;
                }
                load_bnd();
            }
            if (stop) break;
        }
        if constexpr (sizeof(Off) == 4) {
            // Chained windows (periodic / low-entropy data), whole windows at a
            // time.  With the reference's buffer full (R = min(F, s + MAX)) and
            // the last cut made at a candidate whose head fix-up is known to be
            // empty (head 1, fix 0), the next cut is the next candidate c if
            // c >= s + 63 (file_operations.rs:754-755 with the fix-up), and
            // then c < R holds whenever c - (s - 1) <= MAX; if that gap is also
            // <= CAP the buffer is full again after the cut (:776:
            // R' = min(F, R + min(MAX - (R - s'), CAP)) = min(F, s' + MAX)).  So
            // lane l of the window continues the chain iff its predecessor
            // (lane l-1, or the last cut for the first lane) has a known empty
            // fix-up and l's candidate lies 64 .. min(MAX, CAP) bytes past it:
            // one ballot finds the run, its cuts are stored one per lane, and a
            // used-up window slides to the next (loaded PF windows ahead).  Cuts
            // stop at the first landing at or past the next split boundary.
            if (head == 1 && fix == 0 && jlast >= 0 && !P.resolve_noburst &&
                (uint64_t)R == min<uint64_t>((uint64_t)Fo, (uint64_t)s + (uint64_t)MAX)) {
                const Off gapmax = CAP < MAX ? CAP : MAX;
                for (;;) {
                    // Run skip: when the chain continues through the rest of this
                    // window, find where it ends from the link words (4096
                    // candidates per load) instead of window by window, write the
                    // run's cuts with independent loads/stores, and re-seat the
                    // window ring at the run's last cut.  The run stops at the next
                    // split boundary's candidate (a landing there is decided above)
                    // and at the file's last candidate.
                    if (SPLIT && T.linkw && !P.no_skip && ncand && __ballot((uint32_t)lane >= (uint32_t)jlast && !(wk & 0x200u)) == 0ull) {
                        const uint64_t ci = wb + (uint64_t)jlast;               // the last cut's candidate
                        uint64_t lim = ncand - 1;
                        if (sbi < lim) lim = sbi;
                        const uint64_t w0 = ci >> 6, wi = w0 + (uint64_t)lane;
                        uint64_t word = wi <= (lim >> 6) ? T.linkw[wi] : 0ull;
                        if (lane == 0) word |= (1ull << (ci & 63u)) - 1ull;     // below ci: not looked at
                        const unsigned long long hz = __ballot(~word != 0ull);
                        uint64_t z = (w0 + 64u) * 64u - 1u;                    // 4096 links, all set
                        if (hz) {
                            const uint32_t fl = (uint32_t)__builtin_ctzll(hz);
                            z = (w0 + fl) * 64u + (uint64_t)__builtin_ctzll(~readlane64(word, fl));
                        }
                        if (z > lim) z = lim;
                        uint64_t cz = z > ci ? T.cand[z] : 0ull;
                        if (z > ci && (cz & CAND_POS_MASK) >= g0 + F) {         // past the file: its last candidate
                            z = wave_lower_bound(T.cand, ci + 1, z + 1, g0 + F, lane) - 1;
                            cz = T.cand[z];
                        }
                        if (z > ci) {
                            const uint32_t pend = (uint32_t)cnt & 63u;      // gathered cuts before the run
                            if (pend > bstart) flush(pend);
                            const uint64_t L = z - ci;
                            bool deferred = false;
                            if (defer && (is_spec ? run_len == 0u && L < 0xffffffffull
                                                  : (uint64_t)cnt + L <= cap)) {
                                uint32_t q = 0;
                                if (lane == 0) q = atomicAdd(&T.split[SPL_RUNS], 1u);
                                q = (uint32_t)__builtin_amdgcn_readfirstlane(q);
                                if (q < T.runs_cap) {
                                    if (lane == 0) {
                                        RunJob j;
                                        j.out = is_spec ? (uint64_t)cnt : T.cut_base[i] + (uint64_t)cnt;
                                        j.a = ci + 1;
                                        j.n = (uint32_t)L;
                                        j.file = i;
                                        j.rec = is_spec ? spec : SPLIT_END;
                                        j.pad = 0;
                                        T.runs[q] = j;
                                    }
                                    deferred = true;
                                    if (is_spec) {                           // scratch skips the run
                                        run_pre = (uint32_t)cnt;
                                        run_len = (uint32_t)L;
                                        out -= L;
                                        cap += L;
                                    }
                                }
                            }
                            for (uint64_t k0 = ci + 1; !deferred && k0 <= z; k0 += 256u) {
                                uint64_t pk[4], pp[4];
#pragma unroll
                                for (int u = 0; u < 4; ++u) {
                                    const uint64_t k = k0 + 64u * u + (uint64_t)lane;
                                    const uint64_t kk = k <= z ? k : z;
                                    pk[u] = T.cand[kk] & CAND_POS_MASK;
                                    pp[u] = T.cand[kk - 1] & CAND_POS_MASK;
                                }
#pragma unroll
                                for (int u = 0; u < 4; ++u) {
                                    const uint64_t k = k0 + 64u * u + (uint64_t)lane;
                                    const uint64_t idx = (uint64_t)cnt + (k - ci - 1);
                                    if (k <= z && idx < cap) {
                                        DevCut d;
                                        d.offset = pp[u] + 1 - g0;
                                        d.len = (uint32_t)(pk[u] - pp[u]);
                                        d.file = i;
                                        st_cut(out + idx, d, T.nt_out);
                                    }
                                }
                            }
                            cnt += (Off)(z - ci);
                            bstart = (uint32_t)cnt & 63u;
                            s = (Off)((cz & CAND_POS_MASK) - g0 + 1);
                            R = (Off)min<uint64_t>((uint64_t)Fo, (uint64_t)s + (uint64_t)MAX);
                            head = (cz & CAND_KNOWN) ? 1 : 2;
                            fix = (uint32_t)(cz >> 48) & 0xffu;
                            wb = z;                                          // window ring at the last cut
                            prime();
                            load_window();
                            jlast = 0;
                            if (s >= R || s >= sb || head != 1 || fix != 0) break;
                        }
                    }
                    if (jlast == 63) {                               // window used up: slide
                        if (wb + 64 >= ncand) break;
                        slide();
                        load_window();
                        jlast = -1;
                    }
                    const Off up = (Off)up1((uint32_t)wr);
                    const uint32_t kup = up1(wk);
                    const bool first = lane == jlast + 1;
                    const Off pw = first ? (Off)(s - 1) : up;      // the cut before this lane's
                    const bool plink = first || (kup & 0x1ffu) == 0x100u;
                    const bool ok = lane > jlast && plink && wr != OMAX && wr >= (Off)(pw + 64) &&
                                    (Off)(wr - pw) <= gapmax;
                    const unsigned long long run = __ballot(ok) >> (jlast + 1);   // jlast + 1 <= 63
                    const uint32_t n0 = ~run ? (uint32_t)__builtin_ctzll(~run) : (uint32_t)(63 - jlast);
                    if (!n0) break;
                    uint32_t lastl = (uint32_t)jlast + n0;
                    const unsigned long long past =
                        __ballot(lane > jlast && (uint32_t)lane <= lastl && (Off)(wr + 1) >= sb);
                    if (past) lastl = (uint32_t)__builtin_ctzll(past);
                    const uint32_t n = lastl - (uint32_t)jlast;
                    const uint32_t pend = (uint32_t)cnt & 63u;      // gathered cuts before these
                    if (pend > bstart) flush(pend);
                    if (lane > jlast && (uint32_t)lane <= lastl) {
                        const uint64_t idx = (uint64_t)cnt + (uint64_t)(lane - jlast - 1);
                        if (idx < cap) {
                            DevCut d;
                            d.offset = (uint64_t)pw + 1;
                            d.len = (uint32_t)(wr - pw);
                            d.file = i;
                            st_cut(out + idx, d, T.nt_out);
                        }
                    }
                    cnt += (Off)n;
                    bstart = (uint32_t)cnt & 63u;
                    s = rl(wr, lastl) + 1;
                    R = (Off)min<uint64_t>((uint64_t)Fo, (uint64_t)s + (uint64_t)MAX);
                    const uint32_t k = (uint32_t)__builtin_amdgcn_readlane((int)wk, (int)lastl);
                    head = (k & 0x100u) ? 1 : 2;
                    fix = k & 0xffu;
                    jlast = (int)lastl;
                    if (lastl < 63u || s >= R || s >= sb || head != 1 || fix != 0) break;
                }
                if (s >= R) break;
                if (s >= sb) continue;                              // the boundary first
            }
        }
        if constexpr (sizeof(Off) == 4) {
            // Burst of chained hops: while every cut lands on a window candidate
            // with no head hit after it (fix 0), the next cut is the candidate
            // nx[] names, if it lies below the read limit.  Those iterations of
            // the loop below reduce to a chain through the window, found here
            // in O(log 64) wave steps instead of one scalar hop per cut:
            //   * list ranking by pointer jumping over f = nx (64 = the chain
            //     ends: past the window, fix-up unknown or non-zero, no candidate);
            //   * lane j lies on the chain from jlast iff f^(r[jlast]-r[j])(jlast) == j;
            //   * the read limit after the m-th cut of the chain is
            //     R_m = min(F, s_m + MAX, R_{m-1} + CAP)  (file_operations.rs:776)
            //         = min(F, m*CAP + min(R_0, min_{i<=m} (s_i + MAX - i*CAP))),
            //     a prefix minimum over the chain's lanes; the chain is cut
            //     short at its first candidate at or past the limit before it.
            // The cuts are then written in parallel (one lane per cut).
            if (head == 1 && fix == 0 && jlast >= 0 && !P.resolve_noburst) {
                uint64_t mk = 0;
                const Off s0 = s, n0 = cnt;
                int j = jlast;
                uint32_t f = (wk & 0x1ffu) == 0x100u ? nx : 64u;
                if (wr == OMAX || f <= (uint32_t)lane) f = 64u;     // past the file / unsorted (overflow re-run)
                // fast path: a chain of consecutive lanes (nx[j] == j + 1, periodic
                // data) ending in the window or at a lane whose chain ends
                const unsigned long long contig = __ballot(f == (uint32_t)lane + 1u);   // f == 64 at lane 63: end
                const unsigned long long fromj = contig >> j;
                const uint32_t run = ~fromj ? (uint32_t)__builtin_ctzll(~fromj) : 64u - (uint32_t)j;
                const uint32_t last = (uint32_t)j + run;            // reached; its own f is not last + 1
                const uint32_t flast = last < 64u ? (uint32_t)__builtin_amdgcn_readlane((int)f, (int)last) : 64u;
                unsigned long long pm;
                const bool chain_contig = flast >= 64u;             // pm = lanes j+1 .. last
                if (chain_contig) {
                    const unsigned long long upto = last >= 63u ? ~0ull : ((2ull << last) - 1ull);   // lanes <= last
                    const unsigned long long thru = j >= 63 ? ~0ull : ((2ull << j) - 1ull);          // lanes <= j
                    pm = upto & ~thru;
                } else {
                    uint32_t rk = f < 64u ? 1u : 0u, nxt = f;
                    uint32_t J[6];                                  // J[k] = f^(2^k)
#pragma unroll
                    for (int k = 0; k < 6; ++k) {
                        J[k] = nxt;
                        const int src = (int)(nxt & 63u);
                        const uint32_t rn = (uint32_t)__shfl((int)rk, src), nn = (uint32_t)__shfl((int)nxt, src);
                        if (nxt < 64u) { rk += rn; nxt = nn; }
                    }
                    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)rk, j);
                    const uint32_t t = r0 - rk;                     // hops from jlast to this lane, if on the chain
                    const bool cand = lane > j && rk <= r0;
                    uint32_t x = (uint32_t)j;
#pragma unroll
                    for (int k = 0; k < 6; ++k) {
                        const uint32_t jx = (uint32_t)__shfl((int)J[k], (int)(x & 63u));
                        if (((t >> k) & 1u) && x < 64u) x = jx;
                    }
                    pm = __ballot(cand && x == (uint32_t)lane);
                }
                const bool on = (pm >> lane) & 1ull;
                Off wup = 0;                                        // the previous lane's candidate
                if (pm) {
                    const unsigned long long lt = lane ? (~0ull >> (64 - lane)) : 0ull;
                    const int64_t capv = (int64_t)CAP, maxv = (int64_t)MAX;
                    const int64_t m = on ? (int64_t)__builtin_popcountll(pm & lt) + 1 : 0;
                    int64_t a = on ? (int64_t)wr + 1 + maxv - m * capv : INT64_MAX;
                    const int64_t R0 = (int64_t)R, Fv = (int64_t)Fo;
                    const unsigned long long below = pm & lt;
                    int64_t Rm, Rprev, wprev;
                    // consecutive chain lanes whose candidates are less than CAP apart
                    // (periodic data): a_m falls with m, so the prefix minimum is a_m
                    // itself and R_{m-1} follows from the previous lane's candidate --
                    // one shuffle instead of the 6-step scan and two more shuffles
                    wup = (Off)up1((uint32_t)wr);
                    const bool mono = chain_contig &&
                                      __ballot(on && below && (int64_t)wr - (int64_t)wup >= capv) == 0ull;
                    if (mono) {
                        const int64_t B = a < R0 ? a : R0;
                        Rm = m * capv + B;
                        if (Rm > Fv) Rm = Fv;
                        if (below) {
                            const int64_t ap = (int64_t)wup + 1 + maxv - (m - 1) * capv;
                            Rprev = (m - 1) * capv + (ap < R0 ? ap : R0);
                            if (Rprev > Fv) Rprev = Fv;
                            wprev = (int64_t)wup;
                        } else {
                            Rprev = R0;
                            wprev = (int64_t)s - 1;
                        }
                    } else {
#pragma unroll
                        for (int off = 1; off < 64; off <<= 1) {    // inclusive prefix minimum
                            const int64_t u = (int64_t)shfl_up64((uint64_t)a, off);
                            if (lane >= off && u < a) a = u;
                        }
                        const int64_t B = a < R0 ? a : R0;
                        Rm = m * capv + B;
                        if (Rm > Fv) Rm = Fv;
                        const int pl = below ? 63 - __builtin_clzll(below) : 0;
                        // shuffles with every lane active: under a per-lane condition the
                        // source lane (the chain's first lane has no predecessor) would be
                        // inactive and read back as 0
                        const int64_t Rsh = (int64_t)shfl64((uint64_t)Rm, pl);
                        const int64_t wsh = (int64_t)(Off)__shfl((int)wr, pl);
                        Rprev = below ? Rsh : R0;
                        wprev = below ? wsh : (int64_t)s - 1;
                    }
                    const bool ok = on && (int64_t)wr < Rprev && (int64_t)wr >= wprev + 64;
                    const unsigned long long bad = __ballot(on && !ok);
                    mk = bad ? pm & ((1ull << __builtin_ctzll(bad)) - 1ull) : pm;
                    if (mk) {                                      // stop at the next split boundary
                        const unsigned long long past = __ballot(((mk >> lane) & 1ull) && (Off)(wr + 1) >= sb);
                        if (past) {
                            const uint32_t fl = (uint32_t)__builtin_ctzll(past);
                            mk &= fl >= 63u ? ~0ull : ((2ull << fl) - 1ull);
                        }
                    }
                    if (mk) {
                        j = 63 - __builtin_clzll(mk);
                        s = rl(wr, (uint32_t)j) + 1;                 // cut = edge + 1 (:754-755, :771)
                        R = (Off)readlane64((uint64_t)Rm, (uint32_t)j);
                    }
                }
                if (mk) {
                    cnt += (Off)__builtin_popcountll(mk);
                    jlast = j;
                    const uint32_t k = (uint32_t)__builtin_amdgcn_readlane((int)wk, j);
                    head = (k & 0x100u) ? 1 : 2;
                    fix = k & 0xffu;
                    const uint32_t pend = (uint32_t)n0 & 63u;        // gathered cuts before the burst
                    if (pend > bstart) {
                        const Off keep = cnt;
                        cnt = n0;
                        flush(pend);
                        cnt = keep;
                    }
                    const uint64_t below = (lane ? (~0ull >> (64 - lane)) : 0ull) & mk;
                    const uint32_t pl = below ? 63u - (uint32_t)__builtin_clzll(below) : 0u;
                    // a consecutive chain's previous cut lane is the previous lane
                    const Off pw = chain_contig ? wup : (Off)__shfl((int)wr, (int)pl);
                    if ((mk >> lane) & 1ull) {
                        const Off st = below ? pw + 1 : s0;
                        const uint64_t idx = (uint64_t)n0 + (uint64_t)__builtin_popcountll(below);
                        if (idx < cap) {
                            DevCut d;
                            d.offset = (uint64_t)st;
                            d.len = (uint32_t)(wr + 1 - st);
                            d.file = i;
                            st_cut(out + idx, d, T.nt_out);
                        }
                    }
                    bstart = (uint32_t)cnt & 63u;
                }
                if (s >= R) break;
                if (s >= sb) continue;                              // the boundary first
            }
        }
        const Off lim = R;                                   // :749-752
        Off e = OMAX;
        bool known = false;
        uint32_t cfix = 0;
        const Off from = s + 63;                             // stream G applies from here
        bool done = false;
        if (head == 1 && fix == 0 && jlast >= 0) {           // chained candidate: one table hop
            const uint32_t jn = (uint32_t)__builtin_amdgcn_readlane((int)nx, jlast);
            if (jn < 64) {
                const Off c = rl(wr, jn);
                // trusted only if it moves forward: after a candidate overflow the
                // (discarded, re-run) launch sees unwritten, unsorted entries and
                // the walk must still terminate; the ballot search always does
                if (c >= from) {
                    jlast = -1;
                    if (c < lim) {
                        const uint32_t k = (uint32_t)__builtin_amdgcn_readlane((int)wk, (int)jn);
                        e = c;
                        known = (k & 0x100u) != 0;
                        cfix = k & 0xffu;
                        jlast = (int)jn;
                    }
                    done = true;
                }
            }
        }
        if (!done) {
            jlast = -1;
            Off hh = OMAX;
            if (head == 1) {
                if (fix) hh = s - 1 + fix;
            } else {
                bool tab = false;
                if (grid) {                                  // a read-boundary grid point: precomputed
                    const uint64_t k = (uint64_t)s / CAPv;
                    if (k * CAPv == (uint64_t)s) {
                        const uint32_t f = k < 64 ? (uint32_t)__builtin_amdgcn_readlane((int)gf, (int)k)
                                                  : (uint32_t)T.gfix[gb + k];
                        if (f) hh = s + (Off)(f - 1);
                        tab = true;
                    }
                }
                if (!tab) {                                  // wave head scan of [s, min(s+63, lim))
                    const uint32_t n = (uint32_t)min<uint64_t>(63ull, (uint64_t)(lim - s));
                    const uint32_t x = (uint32_t)lane < n ? data[g0 + (uint64_t)s + lane] : 0u;
                    const uint32_t S = wave_incl_scan(x, lane);
                    const uint32_t W = wave_incl_scan(S, lane);
                    const unsigned long long m = __ballot((uint32_t)lane < n && hit_exact(S, W, P.mask));
                    if (m) hh = s + (Off)__builtin_ctzll(m);
                }
            }
            if (hh != OMAX && hh < lim) e = hh;
            if (e == OMAX && from < lim) {
                for (;;) {
                    const unsigned long long m = __ballot(wr >= from);
                    if (m) {
                        const uint32_t j = (uint32_t)__builtin_ctzll(m);
                        const Off c = rl(wr, j);
                        if (c < lim) {
                            const uint32_t k = (uint32_t)__builtin_amdgcn_readlane((int)wk, (int)j);
                            e = c;
                            known = (k & 0x100u) != 0;
                            cfix = k & 0xffu;
                            jlast = (int)j;
                        }
                        break;
                    }
                    if (wb + 64 >= ncand) break;             // whole window below `from`: slide
                    slide();
                    load_window();
                }
            }
        }
        Off cut;                                             // :754-755
        if (e != OMAX) { cut = e + 1; head = known ? 1 : 2; fix = cfix; }
        else { cut = lim; head = 2; }
        const uint32_t slot = (uint32_t)cnt & 63u;
        if ((uint32_t)lane == slot) {                        // gather: lane `slot` keeps this cut
            bo = s;
            bl = (uint32_t)(cut - s);
        }
        ++cnt;
        if (__builtin_expect(slot == 63u, 0)) { flush(64); bstart = 0; }
        s = cut;                                             // :771
        // :776, kept in the scalar unit (hipcc otherwise fuses the mins into a
        // VALU v_min3 plus a readfirstlane round trip on this serial path)
        Off rd = MAX - (R - s);
        rd = min(rd, CAP);
        if constexpr (sizeof(Off) == 4) asm volatile("" : "+s"(rd));
        rd = min(rd, (Off)(Fo - R));
        R += rd;
    }
    if (cnt & 63u) flush((uint32_t)(cnt & 63u));
    // Retire the ring's outstanding LDS-DMAs before the walk ends: a wave must
    // not end (and its workgroup's LDS be handed to another) with DMA writes
    // into it still in flight.
    wait_vmcnt<0>();
    if (is_spec) {
        // the result in one word: a file walker needs nothing else of the record
        // (the scratch cuts are read only by the copy launch), so no release fence
        const uint32_t st = (link == SPLIT_ABORT || (uint64_t)cnt > cap) ? SEG_ABORTED : SEG_DONE;
        if (lane == 0) {
            T.segs[spec].run_pre = run_pre;                 // read by the copy launch only
            T.segs[spec].run_len = run_len;
            __hip_atomic_store(&T.segs[spec].res,
                               seg_res(st, link, (uint32_t)min<uint64_t>((uint64_t)cnt, 0xffffffffull)),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (st == SEG_DONE) atomicAdd(&T.split[SPL_WALKED], 1u);
        }
        return;
    }
    if (dbgw) DBG_STAMP(T, DBG_W_END);
    if (lane == 0) {
        T.counts[i] = (uint64_t)cnt;
        if ((uint64_t)cnt > cap) atomicOr(&T.ctr[CTR_FLAGS], FLAG_CUT_OVERFLOW);
    }
    if (SPLIT && elig && bend) {                             // adoptions before the done count
        __threadfence();
        if (lane == 0) atomicAdd(&T.split[SPL_DONE], 1u);
    }
}

// The extra resolve waves (split workers): walk segments as the file walkers
// publish them.  They never hold up a file walker (which walks a segment itself
// when that segment's walk is not done), and the only thing they wait for is a
// file walker publishing its segments.  File-walker blocks have the lower
// block indices and are dispatched first, but the programming model does not
// promise it, so every wait is bounded: past KParams::split_patience of wall
// clock (~100 ms; 0 with SYNCR_CDC_FLAG_SPLIT_NOWAIT) the worker gives up,
// counts itself in SPL_GIVEUP and stops -- the segments it would have walked
// stay pending and their file walkers walk them, so a give-up costs time,
// never correctness.  Adopted segments' cuts are copied by a separate launch
// (cdc_split_copy_kernel), so no wave ever waits for the walkers to finish.
// Polls are relaxed: an agent-scope acquire invalidates the XCD's L2 on gfx950,
// so it is taken once, only before reading what another wave published.
__device__ __forceinline__ uint32_t ld_relaxed(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t ld64_relaxed(const unsigned long long *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t give_up(const Tables &T, int lane) {
    if (lane == 0) atomicAdd(&T.split[SPL_GIVEUP], 1u);
    return SPLIT_END;
}

// The next segment record to walk, or SPLIT_END once every eligible walker has
// published and the queue is empty (or the worker ran out of patience).
// A worker's first record is its own index (no atomic: a thousand workers
// incrementing one counter at once held up every file walker's first loads by
// ~10-20 us); later ones come from the queue counter, past the first nwork.
__device__ __forceinline__ uint32_t split_next(const KParams &P, const Tables &T, int lane, uint32_t first,
                                               uint32_t nwork) {
    const Patience pat(P.split_patience);
    if (P.split_patience == 0ull) return give_up(T, lane);           // SYNCR_CDC_FLAG_SPLIT_NOWAIT
    uint32_t q = first;
    if (q == SPLIT_END) {
        if (lane == 0) q = nwork + atomicAdd(&T.split[SPL_HEAD], 1u);
        q = (uint32_t)__builtin_amdgcn_readfirstlane(q);
    } else {
        __builtin_amdgcn_s_sleep(32);                                // the walkers publish after ~5-10 us
    }
    // exponential backoff between polls: a thousand waves polling one word at
    // full rate queue up in front of the file walkers' own loads
    uint32_t nap = 1;
    for (;;) {
        if (q < min(ld_relaxed(&T.split[SPL_RESERVED]), T.seg_cap)) break;
        if ((uint32_t)ld64_relaxed(split_pub(T)) >= T.n_elig) {
            // every reservation precedes its walker's count (split_setup); a stale
            // read here only leaves a segment to its file's walker
            if (q < min(ld_relaxed(&T.split[SPL_RESERVED]), T.seg_cap)) break;
            return SPLIT_END;
        }
        if (pat.spent()) return give_up(T, lane);
        for (uint32_t k = 0; k < nap; ++k) __builtin_amdgcn_s_sleep(8);
        nap = nap < 16u ? 2u * nap : 16u;
    }
    while (ld_relaxed(&T.segs[q].ready) != T.epoch) {                 // not a stale record
        if (pat.spent()) return give_up(T, lane);                     // record q stays pending
        __builtin_amdgcn_s_sleep(4);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");        // the record's fields
    return q;
}

template <int PF>
__device__ void split_worker(const uint8_t *__restrict__ data, const KParams &P, const Tables &T, int lane,
                             const uint64_t *ring, uint32_t widx, uint32_t nwork) {
    for (uint32_t first = widx;; first = SPLIT_END) {
        const uint32_t q = split_next(P, T, lane, first, nwork);
        if (q == SPLIT_END) break;
        if (seg_ld(T.segs[q].k) == 0u) continue;
        const uint32_t i = seg_ld(T.segs[q].file);
        if (lane == 0)
            __hip_atomic_store(&T.segs[q].res, seg_res(SEG_WALKING, 0u, 0u), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        if (q < DBG_NREC) DBG_STAMP(T, DBG_REC + 2 * q);
        resolve_walk<uint32_t, PF, true>(data, P, T, i, T.flen[i], T.foff[i], lane, false, q, ring);
        if (q < DBG_NREC) DBG_STAMP(T, DBG_REC + 2 * q + 1);
    }
}

// After the resolve launch (so after every walker): copy the cuts of every
// segment walk a file walker adopted into that file's output, and expand the
// deferred runs.  PARTS waves per record / run (up to 3 x 4096 cuts: one wave
// each left most of the grid idle), U1 16-byte loads in flight per lane (dev A/B:
// SYNCR_CDC_ABLATE=18: U1 8).  The units of both kinds form ONE grid-
// stride range (a wave of the usual grid takes one unit, not one of each), and a
// run's candidate loads go out with its record / file loads: a wave's chain is
// two dependent load rounds and its stores (dense1: the last of 4096 waves ended
// 33 us after the launch when each wave walked one record unit, then one run
// unit, each four dependent rounds deep; profiles/r05_dense1_resolve_copy_timeline.txt).
template <uint32_t COPY_PARTS, int U1>
__device__ __forceinline__ void copy_record_part(const Tables &T, uint32_t q, uint32_t part, int lane) {
    const SplitSeg &g = T.segs[q];
    if (g.k == 0u || g.verdict != 1u || g.ready != T.epoch) return;    // not adopted (or a stale record)
    const uint32_t i = g.file;
    const uint64_t o = g.out_off, rl = g.run_len, rp = g.run_pre, nr = seg_res_n(g.res);
    const uint64_t n = nr > rl ? nr - rl : 0ull;                      // scratch cuts
    const uint64_t per = ((n + COPY_PARTS - 1) / COPY_PARTS + 255) & ~255ull;
    const uint64_t a = (uint64_t)part * per, e = min(n, a + per);
    if (a >= e) return;
    const DevCut *src = T.seg_cuts + (uint64_t)q * T.seg_scap;
    for (uint64_t t = a + (uint64_t)lane; t < e; t += 64u * U1) {
        DevCut v[U1];
#pragma unroll
        for (int u = 0; u < U1; ++u)
            if (t + 64u * u < e) v[u] = src[t + 64u * u];
        const uint64_t cap = T.cut_cap[i];                          // (issued with the block's loads)
        DevCut *dst = T.cuts + T.cut_base[i];
#pragma unroll
        for (int u = 0; u < U1; ++u) {
            const uint64_t tt = t + 64u * u, d = o + tt + (tt < rp ? 0u : rl);
            if (tt < e && d < cap) st_cut(dst + d, v[u], T.nt_out);
        }
    }
}

// Deferred run r, part `part`: cut k starts right after candidate k-1 (file-relative).
template <uint32_t COPY_PARTS>
__device__ __forceinline__ void expand_run_part(const Tables &T, uint32_t r, uint32_t part, int lane) {
    const RunJob j = T.runs[r];
    const uint32_t i = j.file;
    const uint64_t per = (((uint64_t)j.n + COPY_PARTS - 1) / COPY_PARTS + 255) & ~255ull;
    const uint64_t a = (uint64_t)part * per, e = min((uint64_t)j.n, a + per);
    if (a >= e) return;
    // one load per cut: the previous candidate comes from the lane before (DPP) or
    // the previous 64 (readlane); eight 64-candidate blocks in flight, issued with the
    // record / file loads below
    constexpr int U = 8;
    for (uint64_t t0 = a; t0 < e; t0 += 64u * U) {
        uint64_t pk[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t k = j.a + min(t0 + 64u * u + (uint64_t)lane, (uint64_t)j.n - 1);
            pk[u] = T.cand[k] & CAND_POS_MASK;
        }
        const uint64_t before = T.cand[j.a + t0 - 1] & CAND_POS_MASK;     // the cut before this block
        bool ok = true;
        uint64_t rel = j.out - T.cut_base[i];                            // slot within the file's output
        if (j.rec != SPLIT_END) {
            const SplitSeg &g = T.segs[j.rec];
            ok = g.k != 0u && g.verdict == 1u && g.ready == T.epoch;
            rel = g.out_off + j.out;
        }
        const uint64_t cap = T.cut_cap[i], g0 = T.foff[i];
        if (!ok) return;                                             // (wave-uniform)
        DevCut *dst = T.cuts + T.cut_base[i] + rel;
        const uint64_t lim = cap > rel ? cap - rel : 0ull;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t up = ((uint64_t)up1((uint32_t)(pk[u] >> 32)) << 32) | up1((uint32_t)pk[u]);
            const uint64_t pp = lane ? up : (u ? readlane64(pk[u - 1], 63) : before);
            const uint64_t tt = t0 + 64u * u + (uint64_t)lane;
            if (tt < e && tt < lim) {
                DevCut d;
                d.offset = pp + 1 - g0;
                d.len = (uint32_t)(pk[u] - pp);
                d.file = i;
                st_cut(dst + tt, d, T.nt_out);
            }
        }
    }
}

template <uint32_t COPY_PARTS, int U1>
__global__ __launch_bounds__(256) void cdc_split_copy_kernel(Tables T) {
    const int lane = threadIdx.x & 63;
    const uint32_t wid = blockIdx.x * 4u + (threadIdx.x >> 6), nw = gridDim.x * 4u;
    const uint32_t nsplit = (uint32_t)(*split_pub(T) >> 32);
    const uint32_t nruns = T.runs_cap ? min(T.split[SPL_RUNS], T.runs_cap) : 0u;
    if (nsplit == 0u && nruns == 0u) return;                  // nothing split or deferred
    if (blockIdx.x == 0 && threadIdx.x < 64) DBG_STAMP(T, DBG_COPY_START);
#ifdef SYNCR_CDC_DEV
    const uint64_t dbg_t0 = wall_clock64();
#endif
    const uint32_t nrec = nsplit ? min(T.split[SPL_RESERVED], T.seg_cap) : 0u;
    // units [0, n1): scratch cuts of every adopted segment walk (its deferred run, if
    // any, leaves a gap of run_len slots after its first run_pre cuts); [n1, n1 + n2):
    // the deferred runs
    const uint32_t n1 = nrec * COPY_PARTS, n2 = nruns * COPY_PARTS;
    for (uint32_t w = wid; w < n1 + n2; w += nw) {
        if (w < n1)
            copy_record_part<COPY_PARTS, U1>(T, w / COPY_PARTS, w % COPY_PARTS, lane);
        else
            expand_run_part<COPY_PARTS>(T, (w - n1) / COPY_PARTS, (w - n1) % COPY_PARTS, lane);
    }
#ifdef SYNCR_CDC_DEV
    if (wid < (uint32_t)DBG_NCW) {
        SCAN_STAMP(T, DBG_CW + 2 * wid, wall_clock64());
        SCAN_STAMP(T, DBG_CW + 2 * wid + 1, dbg_t0);
    }
#endif
}

// One wave per file; files below 4 GiB walk in 32-bit offsets.  Blocks past
// the file walkers' (launched only when a file is eligible) are split workers.
// (Their walk is a separate inlined copy: sharing one with the file walkers
// made the file walk spill scalar registers.)
template <int PF, bool SPLIT>
__global__ __launch_bounds__(256) void cdc_resolve_wave_kernel(const uint8_t *__restrict__ data,
                                                               KParams P, Tables T) {
    const int lane = threadIdx.x & 63;
    __shared__ uint64_t rings[4 * PF * 64];                     // each wave's candidate-window ring
    const uint64_t *ring = rings + (threadIdx.x >> 6) * (PF * 64);
    if (blockIdx.x == 0 && threadIdx.x < 64) DBG_STAMP(T, DBG_RES_START);   // (one wave: no contention)
    scan_time_account(T);
    zero_next(T);
    if (blockIdx.x == 0 && threadIdx.x < 64) DBG_STAMP(T, 6);
    const uint32_t nmain = (T.nfiles + 3u) / 4u, nwork = gridDim.x - nmain;
    // split workers take the FIRST blocks when P.split_first: a grid larger than
    // the resident set dispatched them last, after the file walkers of the big
    // files had published their segments and waited (their waits are bounded,
    // and the file walkers never wait on a worker that has not started)
    const uint32_t b = P.split_first ? (blockIdx.x >= nwork ? blockIdx.x - nwork : nmain + blockIdx.x) : blockIdx.x;
    if (SPLIT && b >= nmain) {
        const uint32_t widx = __builtin_amdgcn_readfirstlane((b - nmain) * 4u + (threadIdx.x >> 6));
        split_worker<PF>(data, P, T, lane, ring, widx, 4u * nwork);
        return;
    }
    const uint32_t kf = __builtin_amdgcn_readfirstlane(b * 4 + (threadIdx.x >> 6));
    if (kf >= T.nfiles) return;
    const uint32_t i = T.order[kf];
    const ulonglong2 fr = T.ofile[kf];                          // {foff, flen} of file i
    const uint64_t F = fr.y, g0 = fr.x;
    const bool elig = kf < T.n_elig;
    if (kf == 0) DBG_STAMP(T, 7);
    if (F <= 0xFFFFFF00ull) {
        resolve_walk<uint32_t, PF, SPLIT>(data, P, T, i, F, g0, lane, elig, SPLIT_END, ring);
        if (kf < DBG_NFW) DBG_STAMP(T, DBG_FW + kf);
    } else {
        if (elig && lane == 0) atomicAdd(split_pub(T), 1ull);            // counted, never split
        resolve_walk<uint64_t, PF, SPLIT>(data, P, T, i, F, g0, lane, false, SPLIT_END, ring);
    }
}

// ---------------------------------------------------------------------------
// Synthetic corpus generator (bench/tests): xorshift64 with GF(2) jump-ahead
// so every thread writes its own 4 KiB segment of some file.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t gf2_apply(const uint64_t *cols, uint64_t x) {
    uint64_t y = 0;
    for (int b = 0; b < 64; ++b)
        if ((x >> b) & 1ull) y ^= cols[b];
    return y;
}

__global__ __launch_bounds__(256) void cdc_gen_kernel(uint8_t *__restrict__ base,
                                                      const uint64_t *__restrict__ foff,
                                                      const uint64_t *__restrict__ flen,
                                                      const uint64_t *__restrict__ findex,
                                                      const uint64_t *__restrict__ seg_prefix,
                                                      uint32_t nfiles, uint64_t nseg,
                                                      uint64_t first_index,
                                                      const uint64_t *__restrict__ jump) {
    const uint64_t sid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (sid >= nseg) return;
    uint32_t lo = 0, hi = nfiles;                         // last i with seg_prefix[i] <= sid
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (seg_prefix[mid] <= sid) lo = mid; else hi = mid;
    }
    const uint32_t i = lo;
    const uint64_t start = (sid - seg_prefix[i]) * (uint64_t)GEN_SEG;
    const uint64_t n = min<uint64_t>((uint64_t)GEN_SEG, flen[i] - start);
    const uint64_t fidx = findex ? findex[i] : first_index + i;
    uint64_t x = 0x9E3779B97F4A7C15ull * (fidx + 1);
    const uint64_t steps = 64 + start;
    for (int k = 0; k < GEN_JUMPS; ++k)
        if ((steps >> k) & 1ull) x = gf2_apply(jump + k * 64, x);
    uint8_t *p = base + foff[i] + start;
    uint64_t j = 0;
    for (; j < n && ((uintptr_t)(p + j) & 3u); ++j) {   // head to 4-byte alignment
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        p[j] = (uint8_t)(x >> 32);
    }
    for (; j + 4 <= n; j += 4) {
        uint32_t wv = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            x ^= x << 13; x ^= x >> 7; x ^= x << 17;
            wv |= (uint32_t)(uint8_t)(x >> 32) << (8 * b);
        }
        *(uint32_t *)(p + j) = wv;
    }
    for (; j < n; ++j) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        p[j] = (uint8_t)(x >> 32);
    }
}

// ---------------------------------------------------------------------------
// A small copy group in one dispatch (cdc_internal.h CopyList): the grid strides
// over each segment in turn, 16-byte words where both sides are 16-aligned.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void cdc_copy_kernel(CopyList L) {
    const uint64_t tid = (uint64_t)blockIdx.x * 256u + threadIdx.x, nthr = (uint64_t)gridDim.x * 256u;
    for (uint32_t k = 0; k < L.n; ++k) {
        const uint32_t *src = (const uint32_t *)L.seg[k].src;
        uint32_t *dst = (uint32_t *)L.seg[k].dst;
        const uint64_t nw = L.seg[k].bytes >> 2;
        uint64_t head = 0;                                    // words done as 16-byte vectors
        if (!src) {                                           // a zero fill
            if (((uintptr_t)dst & 15u) == 0) {
                const uint64_t nv = nw >> 2;
                for (uint64_t i = tid; i < nv; i += nthr) ((uint4 *)dst)[i] = make_uint4(0u, 0u, 0u, 0u);
                head = 4 * nv;
            }
            for (uint64_t i = head + tid; i < nw; i += nthr) dst[i] = 0u;
            continue;
        }
        if ((((uintptr_t)src | (uintptr_t)dst) & 15u) == 0) {
            const uint64_t nv = nw >> 2;
            for (uint64_t i = tid; i < nv; i += nthr) ((uint4 *)dst)[i] = ((const uint4 *)src)[i];
            head = 4 * nv;
        }
        for (uint64_t i = head + tid; i < nw; i += nthr) dst[i] = src[i];
    }
}

hipError_t launch_copy(const CopyList &l, uint64_t total_bytes, hipStream_t s) {
    if (!l.n) return hipSuccess;
    const uint64_t want = (total_bytes / 16 + 255) / 256;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(want, 1), 64);
    hipLaunchKernelGGL(cdc_copy_kernel, dim3(blocks), dim3(256), 0, s, l);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Streaming-read probe (roofline denominator): the best rate this
// part reaches reading bytes once, with nothing else to do.  Each lane keeps
// UNR 16-byte loads in flight per iteration (grid-stride over 64 KiB blocks so
// a workgroup's loads are contiguous); the XOR of everything read is stored
// only if it equals an impossible sentinel, so the loads cannot be dropped and
// nothing is written.  NT selects the non-temporal policy (as the scan uses).
// ---------------------------------------------------------------------------

template <bool NT>
__global__ __launch_bounds__(256) void cdc_read_probe_kernel(const u32x4 *__restrict__ src, uint64_t nvec,
                                                             uint32_t *__restrict__ sink) {
    constexpr int UNR = 16;                               // 256 lanes x 16 x 16 B = 64 KiB per block step
    u32x4 acc = {0u, 0u, 0u, 0u};
    const uint64_t step = (uint64_t)gridDim.x * 256 * UNR;
    for (uint64_t b = (uint64_t)blockIdx.x * 256 * UNR; b < nvec; b += step) {
        u32x4 v[UNR];
        if (b + 256 * UNR <= nvec) {
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                const u32x4 *p = src + b + u * 256 + threadIdx.x;
                if constexpr (NT) v[u] = __builtin_nontemporal_load(p); else v[u] = *p;
            }
        } else {
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                const uint64_t k = b + u * 256 + threadIdx.x;
                v[u] = k < nvec ? src[k] : u32x4{0u, 0u, 0u, 0u};
            }
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) acc ^= v[u];
    }
    const uint32_t r = acc.x ^ acc.y ^ acc.z ^ acc.w;
    if (r == 0x5EC7E7u && acc.x == 0xC0FFEEu && acc.y == 0xFACADEu) sink[blockIdx.x] = r;
}

hipError_t launch_read_probe(const uint8_t *d, uint64_t bytes, bool nt, uint32_t grid, uint32_t *sink,
                             hipStream_t s) {
    const uint64_t nvec = bytes / 16;
    if (!nvec) return hipSuccess;
    if (nt)
        hipLaunchKernelGGL(cdc_read_probe_kernel<true>, dim3(grid), dim3(256), 0, s, (const u32x4 *)d, nvec, sink);
    else
        hipLaunchKernelGGL(cdc_read_probe_kernel<false>, dim3(grid), dim3(256), 0, s, (const u32x4 *)d, nvec, sink);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Scan instances.  The product library carries exactly one: RUN = DEFAULT_RUN,
// non-temporal tile loads, dynamic tile groups (MODE 12).  The development
// library (-DSYNCR_CDC_DEV, libsyncr_cdc_dev.so, tools/ only) adds the other
// RUN sizes, the static-stride and timing-only ablations and the MFMA scan,
// selected by environment variables that the product never reads.
// ---------------------------------------------------------------------------
// The CU schedule: one workgroup of SCAN_CU_WAVES waves per CU (grid = the
// per-wave grid / SCAN_CU_WAVES), plus the LDS tile counter.
constexpr int SCAN_CU_WAVES = 8;
// The stream-tile scan with the geometry st_segs() picks for this launch.
static void launch_st(uint32_t grid, const uint8_t *d, const KParams &p, const Tables &t, hipStream_t s) {
#ifdef SYNCR_CDC_DEV
    switch (st_segs(grid, p, t)) {
    case 18:
        hipLaunchKernelGGL((cdc_scan_st_kernel<4, 18>), dim3(grid), dim3(64), st_lds_bytes(18), s, d, p, t);
        return;
    case 27:
        hipLaunchKernelGGL((cdc_scan_st_kernel<4, 27>), dim3(grid), dim3(64), st_lds_bytes(27), s, d, p, t);
        return;
    case 36:
        hipLaunchKernelGGL((cdc_scan_st_kernel<4, 36>), dim3(grid), dim3(64), st_lds_bytes(36), s, d, p, t);
        return;
    default:
        break;
    }
#endif
    hipLaunchKernelGGL((cdc_scan_st_kernel<4, ST_SEGS>), dim3(grid), dim3(64), st_lds_bytes(ST_SEGS), s, d, p, t);
}

// The > 64 KB dynamic-LDS attribute is set once per (kernel instance, device), under
// a lock: multi-device ingest opens and launches handles from several threads.
template <int RUN, int MODE>
static hipError_t launch_scan_cu(uint32_t wave_grid, const uint8_t *d, const KParams &p, const Tables &t,
                                 hipStream_t s) {
    const size_t lds = (size_t)SCAN_CU_WAVES * lds_wave_bytes(RUN) + 16 + 8 * CU_NSLOT;
    const void *f = (const void *)&cdc_scan_kernel<RUN, MODE, SCAN_CU_WAVES>;
    {
        static std::mutex mu;
        static std::set<int> done;                 // devices whose attribute is set
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return e;
        std::lock_guard<std::mutex> g(mu);
        if (!done.count(dev)) {
            e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
            done.insert(dev);
        }
    }
    uint32_t grid = (wave_grid + SCAN_CU_WAVES - 1) / SCAN_CU_WAVES;
    hipLaunchKernelGGL((cdc_scan_kernel<RUN, MODE, SCAN_CU_WAVES>), dim3(grid), dim3(64 * SCAN_CU_WAVES), lds, s,
                       d, p, t);
    return hipGetLastError();
}

#ifdef SYNCR_CDC_DEV
#include "dev/scan_launch_dev.inc"
#else   // product: one exact scan instance
bool scan_supported(ScanGeom g) { return g.kind == SCAN_VALU && g.param == DEFAULT_RUN; }
int scan_tile_bytes(ScanGeom) { return tile_bytes(DEFAULT_RUN); }
int scan_lds_bytes(ScanGeom) { return lds_wave_bytes(DEFAULT_RUN); }
static const void *scan_kernel_ptr(ScanGeom) { return (const void *)&cdc_scan_kernel<DEFAULT_RUN, SCAN_PRODUCT_MODE>; }
bool scan_dense_inline(ScanGeom, const KParams &) { return false; }

static hipError_t launch_scan_kernel(ScanGeom g, uint32_t grid, const uint8_t *d, const KParams &p, const Tables &t,
                                     hipStream_t s) {
    if (!scan_supported(g)) return hipErrorInvalidValue;
    const int kind = scan_kind(g, grid, p, t);
    grid = grid < t.ntiles ? grid : t.ntiles;
    if (kind == SYNCR_CDC_SCAN_TILES)             // the handle's last batch was dense-heavy: tiles
        hipLaunchKernelGGL((cdc_scan_kernel<DEFAULT_RUN, SCAN_PRODUCT_MODE>), dim3(grid), dim3(64),
                           lds_wave_bytes(DEFAULT_RUN), s, d, p, t);
    else if (kind == SYNCR_CDC_SCAN_STREAM_TILES) // >= 3 stream tiles per wave (§4.6)
        launch_st(grid, d, p, t, s);
    else                                          // small batch: the CU schedule (per-wave static shares end
        return launch_scan_cu<DEFAULT_RUN, SCAN_STATIC_MODE>(grid, d, p, t, s);   // with the slow waves alone)
    return hipGetLastError();
}
#endif

// Segments per stream of the stream-tile scan (see st_tiles): 9 in the product.
// Longer streams read fewer halo lines (27 segments: traffic 1.027x against
// 1.07x, profiles/r05_v1_pmc_traffic.json) but ran slower once the hot loop lost
// its split-round branches: same-process A/B in the driver's condition, zipf10k
// scan 1.652 ms (9) vs 1.667 (27), and the sustained rate of round 4's 9-segment
// code 6002-6030 GiB/s vs 5822-5847 with 27 on the same boxes
// (profiles/r05_st_segments_ab.jsonl, r05_zipf10k_bisect_traces.json).  Small
// batches lose more (coarser last grabs: uniform1k 0.228 / 0.243 ms at 9 / 18).
// (The dev library's KParams::st_segs forces one of 9 / 18 / 27 / 36.)
int st_segs(uint32_t grid, const KParams &p, const Tables &t) {
    (void)grid;
    (void)t;
#ifdef SYNCR_CDC_DEV
    if (p.st_segs == 18u || p.st_segs == 27u || p.st_segs == 36u) return (int)p.st_segs;
#else
    (void)p;
#endif
    return ST_SEGS;
}

// The scan launch of do_launch; e0 / e1 (may be null): HIP events recorded around it.
hipError_t launch_scan(ScanGeom g, uint32_t grid, const uint8_t *d, const KParams &p, const Tables &t,
                       hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    if (!t.ntiles) return hipSuccess;
    hipError_t e = e0 ? hipEventRecord(e0, s) : hipSuccess;
    if (e == hipSuccess) e = launch_scan_kernel(g, grid, d, p, t, s);
    if (e == hipSuccess && e1) e = hipEventRecord(e1, s);
    return e;
}

// The product's choice between its three exact scans (the dev library's
// variants, other geometries and ablations report SYNCR_CDC_SCAN_DEV).
int scan_kind(ScanGeom g, uint32_t grid, const KParams &p, const Tables &t) {
    if (!t.ntiles) return SYNCR_CDC_SCAN_NONE;
    if (g.kind != SCAN_VALU || g.param != DEFAULT_RUN || p.ablate != 0u || !p.nt) return SYNCR_CDC_SCAN_DEV;
    grid = grid < t.ntiles ? grid : t.ntiles;
    if (p.scan_tiles && scan_dynamic(t.ntiles, grid)) return SYNCR_CDC_SCAN_TILES;
    if (!p.scan_tiles && scan_stream_tiles(t.ntiles, grid)) return SYNCR_CDC_SCAN_STREAM_TILES;
    return SYNCR_CDC_SCAN_CU;
}

int scan_blocks_per_cu(ScanGeom g) {
    int n = 0;
    const void *f = scan_kernel_ptr(g);
    if (!f || hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, 64, scan_lds_bytes(g)) != hipSuccess)
        return 1;
    return n > 0 ? n : 1;
}

hipError_t launch_post(const uint8_t *d, const KParams &p, const Tables &t, hipStream_t s, bool dense_inline,
                       uint32_t scan_grid) {
    if (!t.ntiles) return hipSuccess;
    uint32_t dblocks = t.dense_cap < 2048u ? (t.dense_cap ? t.dense_cap : 1u) : 2048u;
    if (p.dense_blocks) dblocks = p.dense_blocks;                  // (development A/B)
    if (dense_inline) {
        // (development A/B) the scan passed its dense tiles itself
    } else if (t.dense_off) {
        // no dense tile seen yet on this handle: no dense launch (fetch re-runs if needed)
    } else if (t.tile == (uint32_t)tile_bytes(DEFAULT_RUN)) {
        if (p.dense_fuse)
            hipLaunchKernelGGL((cdc_dense_packed_kernel<DEFAULT_RUN, true>), dim3(dblocks), dim3(64),
                               dense_buf_bytes(DEFAULT_RUN, true), s, d, p, t);
        else
            hipLaunchKernelGGL((cdc_dense_packed_kernel<DEFAULT_RUN, false>), dim3(dblocks), dim3(64),
                               dense_buf_bytes(DEFAULT_RUN, false), s, d, p, t);
    } else {                                          // other scan geometries (development library)
#ifdef SYNCR_CDC_DEV
        hipLaunchKernelGGL(cdc_dense_kernel, dim3(dblocks), dim3(64), HALO + t.tile, s, d, p, t);
#endif
    }
    // + up to 2048 blocks (one wave per dense tile) that expand dense tiles; they
    // exit at once when there are none.  (256 blocks left ~33 serial tile
    // expansions per wave on the dense workload: 0.2 ms.)
    // No dense pass, no chain links: compaction and fix-ups in one launch when its
    // blocks fit one round on the device (4 per CU at its 119 VGPRs = scan_grid / 2).
    // Past that each extra round repeats the word waves' chain of dependent loads: on
    // zipf10k (2216 word blocks) it ran 26 us against 9.6 + 8.8 us for the two
    // kernels (profiles/r05_zipf10k_bisect_traces.json).
    const uint32_t gblocks = std::min<uint32_t>((t.ngrid + 511) / 512, 1024u);
    const uint32_t fused_blocks = (t.nwords + 3) / 4 + gblocks;
    if (t.dense_off && !t.linkw && !dense_inline && fused_blocks <= std::max(scan_grid / 2u, 1u)) {
        hipLaunchKernelGGL(cdc_gather_fix_kernel, dim3(fused_blocks), dim3(256), 0, s, d, p, t);
        return hipGetLastError();
    }
    const uint32_t dgb = t.dense_off ? 0u : std::min<uint32_t>((t.dense_cap + 3) / 4, 2048u);
    hipLaunchKernelGGL(cdc_gather_kernel, dim3((t.nwords + 3) / 4 + dgb), dim3(256), 0, s, t);
    const uint64_t want = (t.cand_cap + t.ngrid + 511) / 512;       // two items per thread
    const uint32_t blocks = (uint32_t)(want < 2048 ? (want ? want : 1) : 2048);
    hipLaunchKernelGGL(cdc_fix_kernel, dim3(blocks), dim3(256), 0, s, d, p, t);
    return hipGetLastError();
}

bool resolve_splits(const KParams &p, const Tables &t) {
    return t.nfiles && !p.resolve_lane && t.n_elig && t.seg_cap && !p.resolve_nosplit;
}

hipError_t launch_resolve(const uint8_t *d, const KParams &p, const Tables &t, hipStream_t s) {
    if (!t.nfiles) return hipSuccess;           // (do_launch then memsets the next block itself)
    if (p.resolve_lane)
        hipLaunchKernelGGL(cdc_resolve_kernel, dim3((t.nfiles + 63) / 64), dim3(64), 0, s, d, p, t);
    else {
        const bool split = resolve_splits(p, t);
        const dim3 grid((t.nfiles + 3) / 4 + (split ? t.split_blocks : 0u));
#ifdef SYNCR_CDC_DEV
        if (p.resolve_pf && p.resolve_pf != RESOLVE_PF) {           // (development A/B: SYNCR_CDC_RESOLVE_PF)
            switch (p.resolve_pf) {
                case 2: hipLaunchKernelGGL((cdc_resolve_wave_kernel<2, true>), grid, dim3(256), 0, s, d, p, t); break;
                case 4: hipLaunchKernelGGL((cdc_resolve_wave_kernel<4, true>), grid, dim3(256), 0, s, d, p, t); break;
                case 8: hipLaunchKernelGGL((cdc_resolve_wave_kernel<8, true>), grid, dim3(256), 0, s, d, p, t); break;
                case 16: hipLaunchKernelGGL((cdc_resolve_wave_kernel<16, true>), grid, dim3(256), 0, s, d, p, t); break;
                case 32: hipLaunchKernelGGL((cdc_resolve_wave_kernel<32, true>), grid, dim3(256), 0, s, d, p, t); break;
                default: return hipErrorInvalidValue;
            }
        } else
#endif
        if (split)
            hipLaunchKernelGGL((cdc_resolve_wave_kernel<RESOLVE_PF, true>), grid, dim3(256), 0, s, d, p, t);
        else
            hipLaunchKernelGGL((cdc_resolve_wave_kernel<RESOLVE_PF, false>), grid, dim3(256), 0, s, d, p, t);
        if (split && p.ablate == 18u)          // (dev A/B: 8 blocks of 64 cuts in flight per lane)
            hipLaunchKernelGGL((cdc_split_copy_kernel<8, 8>), dim3(1024), dim3(256), 0, s, t);
        else if (split)
            hipLaunchKernelGGL((cdc_split_copy_kernel<8, 4>), dim3(1024), dim3(256), 0, s, t);
    }
    return hipGetLastError();
}

hipError_t launch_gen(uint8_t *d_base, const uint64_t *d_foff, const uint64_t *d_flen,
                      const uint64_t *d_findex, const uint64_t *d_seg_prefix, uint32_t nfiles,
                      uint64_t nseg, uint64_t first_index, const uint64_t *d_jump, hipStream_t s) {
    if (!nseg) return hipSuccess;
    hipLaunchKernelGGL(cdc_gen_kernel, dim3((uint32_t)((nseg + 255) / 256)), dim3(256), 0, s,
                       d_base, d_foff, d_flen, d_findex, d_seg_prefix, nfiles, nseg, first_index, d_jump);
    return hipGetLastError();
}

}  // namespace cdc
