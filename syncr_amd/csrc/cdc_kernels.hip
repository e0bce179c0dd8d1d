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
//   cdc_resolve_kernel then walks the cuts of each file serially (one lane per
//   file) applying MAX_CHUNK_SIZE and the tokio read-cap lookahead.
#include "cdc_internal.h"

namespace cdc {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u16x2 as_u16x2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }

// Exact Bup edge test from window sums (digest = (s1<<16) | (s2 & 0xffff)).
__device__ __forceinline__ bool hit_exact(uint32_t S, uint32_t W, uint32_t mask) {
    const uint32_t dg = ((1984u + S) << 16) | ((124992u + W) & 0xffffu);
    return (dg & mask) == mask;
}

// first index i in [lo, hi) with a[i] >= key (serial, per lane)
__device__ __forceinline__ uint32_t lower_bound_serial(const uint64_t *a, uint32_t lo, uint32_t hi,
                                                       int64_t key) {
    while (lo < hi) {
        const uint32_t mid = lo + ((hi - lo) >> 1);
        if ((int64_t)a[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// ---------------------------------------------------------------------------
// Slow path: one run rolled byte by byte with file-start resets.  Used for the
// (rare) runs whose windows straddle a file start.  `byte(q)` reads global
// position q; positions before `q0` are treated as outside the window.
// ---------------------------------------------------------------------------
template <class ByteFn, class HitFn>
__device__ __forceinline__ void roll_with_resets(ByteFn byte, int64_t rs, int len,
                                                 const uint64_t *fstart, uint32_t lo, uint32_t hi,
                                                 uint32_t mask, HitFn on_hit) {
    const int64_t q0 = rs - 64;
    uint32_t j = lower_bound_serial(fstart, lo, hi, q0);
    int64_t next = j < hi ? (int64_t)fstart[j] : INT64_MAX;
    int64_t g = q0;                       // window floor: bytes < g read as 0
    uint32_t S = 0, W = 0;
    for (int64_t q = q0; q < rs + len; ++q) {
        if (q == next) {                  // fresh Bup at a file start
            S = 0; W = 0; g = q;
            ++j;
            next = j < hi ? (int64_t)fstart[j] : INT64_MAX;
        }
        const uint32_t x = byte(q);
        const uint32_t d = (q - 64 >= g) ? byte(q - 64) : 0u;
        S += x - d;
        W += S - 64u * d;
        if (q >= rs && hit_exact(S, W, mask)) on_hit(q);
    }
}

// First chunk-local hit in [e+1, e+63] for a chunk starting at e+1, as e+k -> k
// (0 = none).  Bytes before e+1 are outside the fresh window, so no drops.
__device__ __forceinline__ uint32_t head_fix(const uint8_t *data, uint64_t span, uint64_t e,
                                             uint32_t mask) {
    uint32_t S = 0, W = 0;
    for (uint32_t k = 1; k <= 63; ++k) {
        const uint64_t q = e + k;
        if (q >= span) break;
        S += data[q];
        W += S;
        if (hit_exact(S, W, mask)) return k;
    }
    return 0;
}

__device__ __forceinline__ void record(uint32_t *wcount, uint32_t *wlist, uint32_t rel) {
    const uint32_t idx = atomicAdd(wcount, 1u);
    if (idx < (uint32_t)LISTCAP) wlist[idx] = rel;
}

// ---------------------------------------------------------------------------
// Scan kernel.  One wave = one tile of 18 KiB.  Staging: coalesced 16-B loads
// of [t0-64, t0+TILE) into the wave's LDS region.  Rolling: lane l holds the
// 208-byte windows of runs l and l+64 in 104 VGPRs and rolls both as packed
// u16 pairs: per byte pair 2 v_perm_b32 + 4 packed integer ops + 1 v_pk_min.
// tv = ((s2+1)*k) mod 2^16 is zero exactly when the s2 half of the mask test
// passes; the group minimum of tv flags the rare 16-byte groups that are
// re-walked exactly (s1 half of the test included).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256, 2) void cdc_scan_kernel(const uint8_t *__restrict__ data,
                                                          KParams P, Tables T) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const uint32_t tile = blockIdx.x * WAVES + wave;
    if (tile >= T.ntiles) return;                         // whole wave
    uint8_t *wl = smem + wave * LDS_WAVE;                 // [0,64) halo, [64, 64+TILE) tile
    uint32_t *wlist = (uint32_t *)(wl + HALO + TILE);
    uint32_t *wcount = wlist + LISTCAP;
    const int64_t t0 = (int64_t)tile * TILE;
    const int64_t span = (int64_t)T.span;
    const uint2 trange = T.tile_range[tile];

    // ---- stage [t0-64, t0+TILE) -> LDS (1156 x 16 B) ----
    constexpr int NV = (HALO + TILE) / 16;
    constexpr int NIT = (NV + 63) / 64;
    {
        uint4 v[NIT];
        const bool interior = (t0 >= HALO) && (t0 + TILE <= span);
        if (interior) {
            const uint4 *src = (const uint4 *)(data + t0 - HALO);
#pragma unroll
            for (int it = 0; it < NIT; ++it) {
                const int vi = it * 64 + lane;
                v[it] = (it < NIT - 1 || vi < NV) ? src[vi] : make_uint4(0, 0, 0, 0);
            }
        } else {
#pragma unroll
            for (int it = 0; it < NIT; ++it) {
                const int vi = it * 64 + lane;
                const int64_t g = t0 - HALO + (int64_t)vi * 16;
                uint4 r = make_uint4(0, 0, 0, 0);
                if (vi < NV && g >= 0 && g < span) {
                    if (g + 16 <= span) {
                        r = *(const uint4 *)(data + g);
                    } else {
                        uint32_t w[4] = {0, 0, 0, 0};
                        for (int b = 0; b < 16 && g + b < span; ++b)
                            w[b >> 2] |= (uint32_t)data[g + b] << (8 * (b & 3));
                        r = make_uint4(w[0], w[1], w[2], w[3]);
                    }
                }
                v[it] = r;
            }
        }
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
            const int vi = it * 64 + lane;
            if (it < NIT - 1 || vi < NV) *(uint4 *)(wl + vi * 16) = v[it];
        }
    }
    if (lane == 0) *wcount = 0u;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");

    // ---- which of my runs straddle a file start (rare) ----
    const int64_t rsA = t0 + (int64_t)lane * RUN;
    const int64_t rsB = t0 + (int64_t)(lane + 64) * RUN;
    bool slowA = false, slowB = false;
    if (trange.y > trange.x) {                            // wave-uniform
        uint32_t j = lower_bound_serial(T.fstart, trange.x, trange.y, rsA - 62);
        slowA = j < trange.y && (int64_t)T.fstart[j] <= rsA + RUN - 1;
        j = lower_bound_serial(T.fstart, trange.x, trange.y, rsB - 62);
        slowB = j < trange.y && (int64_t)T.fstart[j] <= rsB + RUN - 1;
    }
    const int64_t lim_rel = span - t0;                    // positions >= span are not bytes
    const bool recA = !slowA, recB = !slowB;

    // ---- fast path: both runs packed ----
    {
        uint32_t A[52], B[52];
        const uint4 *la = (const uint4 *)(wl + lane * RUN);          // = run start - 64
        const uint4 *lb = (const uint4 *)(wl + (lane + 64) * RUN);
#pragma unroll
        for (int q = 0; q < 13; ++q) {
            const uint4 a = la[q], b = lb[q];
            A[4 * q + 0] = a.x; A[4 * q + 1] = a.y; A[4 * q + 2] = a.z; A[4 * q + 3] = a.w;
            B[4 * q + 0] = b.x; B[4 * q + 1] = b.y; B[4 * q + 2] = b.z; B[4 * q + 3] = b.w;
        }
        // closed-form window sums at run start - 1 (weights 64..1, oldest first)
        uint32_t SA = 0, WA = 0, SB = 0, WB = 0;
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            const uint32_t w = 0x3D3E3F40u - 0x04040404u * (uint32_t)m;
            SA = __builtin_amdgcn_udot4(A[m], 0x01010101u, SA, false);
            WA = __builtin_amdgcn_udot4(A[m], w, WA, false);
            SB = __builtin_amdgcn_udot4(B[m], 0x01010101u, SB, false);
            WB = __builtin_amdgcn_udot4(B[m], w, WB, false);
        }
        u16x2 S = as_u16x2(SA | (SB << 16));
        const uint32_t tA = ((124993u + WA) * P.k) & 0xffffu;
        const uint32_t tB = ((124993u + WB) * P.k) & 0xffffu;
        u16x2 Tv = as_u16x2(tA | (tB << 16));
        const u16x2 kk = as_u16x2(P.kk), km = as_u16x2(P.kmv);
        const uint8_t *ba = wl + lane * RUN, *bb = wl + (lane + 64) * RUN;

#pragma unroll
        for (int g = 0; g < RUN / 16; ++g) {
            const u16x2 S0 = S, T0 = Tv;
            u16x2 acc = as_u16x2(0xffffffffu);
#pragma unroll
            for (int jj = 0; jj < 16; ++jj) {
                const int i = g * 16 + jj;
                const uint32_t sel = 0x0C040C00u + (uint32_t)(i & 3) * 0x00010001u;
                const u16x2 x = as_u16x2(__builtin_amdgcn_perm(B[16 + (i >> 2)], A[16 + (i >> 2)], sel));
                const u16x2 d = as_u16x2(__builtin_amdgcn_perm(B[i >> 2], A[i >> 2], sel));
                S = S + x - d;
                Tv = S * kk + Tv;
                Tv = d * km + Tv;
                acc = __builtin_elementwise_min(acc, Tv);
            }
            const uint32_t a = as_u32(acc);
            const bool z = ((a & 0xffffu) == 0u) | ((a >> 16) == 0u);
            if (__builtin_expect(__ballot(z) != 0ull, 0)) {
                if (z) {
                    // exact re-walk of this 16-byte group (bytes re-read from LDS)
                    u16x2 s = S0, t = T0;
                    for (int jj = 0; jj < 16; ++jj) {
                        const int i = g * 16 + jj;
                        const u16x2 x = {ba[64 + i], bb[64 + i]};
                        const u16x2 d = {ba[i], bb[i]};
                        s = s + x - d;
                        t = s * kk + t;
                        t = d * km + t;
                        const int rA = lane * RUN + i, rB = (lane + 64) * RUN + i;
                        if (recA && t.x == 0 && ((1984u + s.x) & P.m1) == P.m1 && rA < lim_rel)
                            record(wcount, wlist, (uint32_t)rA);
                        if (recB && t.y == 0 && ((1984u + s.y) & P.m1) == P.m1 && rB < lim_rel)
                            record(wcount, wlist, (uint32_t)rB);
                    }
                }
            }
        }
    }

    // ---- slow path for runs straddling a file start ----
    if (slowA || slowB) {
        const uint8_t *wlc = wl;
        auto byte = [&](int64_t q) -> uint32_t { return wlc[q - t0 + HALO]; };
        if (slowA)
            roll_with_resets(byte, rsA, RUN, T.fstart, trange.x, trange.y, P.mask, [&](int64_t q) {
                if (q - t0 < lim_rel) record(wcount, wlist, (uint32_t)(q - t0));
            });
        if (slowB)
            roll_with_resets(byte, rsB, RUN, T.fstart, trange.x, trange.y, P.mask, [&](int64_t q) {
                if (q - t0 < lim_rel) record(wcount, wlist, (uint32_t)(q - t0));
            });
    }

    // ---- publish this tile's candidates (sorted) ----
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    const uint32_t n = __builtin_amdgcn_readfirstlane(*(volatile uint32_t *)wcount);
    if (n == 0u) return;
    if (lane == 0) {
        atomicOr(&T.nonempty[tile >> 6], 1ull << (tile & 63));
        atomicAdd(&T.ctr[CTR_CANDS], n);
    }
    if (n > (uint32_t)LISTCAP) {
        if (lane == 0) {
            const uint32_t idx = atomicAdd(&T.ctr[CTR_DENSE], 1u);
            if (idx < T.dense_cap) {
                T.dense_list[idx] = tile;
                T.tile_meta[tile] = DENSE_BIT | idx;
            } else {
                T.tile_meta[tile] = DENSE_BIT | 0x7fffffffu;
                atomicOr(&T.ctr[CTR_FLAGS], FLAG_DENSE_OVERFLOW);
            }
        }
        return;
    }
    const uint32_t e = (uint32_t)lane < n ? wlist[lane] : 0xffffffffu;
    uint32_t rank = 0;
    for (uint32_t m = 0; m < n; ++m) rank += wlist[m] < e;
    if ((uint32_t)lane < n) {
        const uint32_t fix = head_fix(data, T.span, (uint64_t)t0 + e, P.mask);
        T.slots[(size_t)tile * LISTCAP + rank] = make_uint2(e, fix);
    }
    if (lane == 0) T.tile_meta[tile] = n;
}

// ---------------------------------------------------------------------------
// Dense tiles (more than LISTCAP candidates, i.e. adversarial / low-entropy
// data at small chunk_bits): recompute G for the whole tile into a bitmap.
// Lane l covers 288 positions = 9 bitmap words.  Grid-stride over the list.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void cdc_dense_kernel(const uint8_t *__restrict__ data,
                                                       KParams P, Tables T) {
    const uint32_t nd = min(T.ctr[CTR_DENSE], T.dense_cap);
    const int lane = threadIdx.x;
    for (uint32_t idx = blockIdx.x; idx < nd; idx += gridDim.x) {
        const uint32_t tile = T.dense_list[idx];
        const int64_t t0 = (int64_t)tile * TILE;
        const int64_t rs = t0 + (int64_t)lane * DENSE_LANE_BYTES;
        const int64_t span = (int64_t)T.span;
        uint32_t words[DENSE_LANE_BYTES / 32];
#pragma unroll
        for (int w = 0; w < DENSE_LANE_BYTES / 32; ++w) words[w] = 0u;
        auto byte = [&](int64_t q) -> uint32_t { return (q >= 0 && q < span) ? data[q] : 0u; };
        const uint32_t lo = lower_bound_serial(T.fstart, 0, T.nstarts, rs - 64);
        const uint32_t hi = lower_bound_serial(T.fstart, lo, T.nstarts, rs + DENSE_LANE_BYTES);
        roll_with_resets(byte, rs, DENSE_LANE_BYTES, T.fstart, lo, hi, P.mask, [&](int64_t q) {
            if (q < span) {
                const int r = (int)(q - rs);
                words[r >> 5] |= 1u << (r & 31);
            }
        });
        uint32_t *out = T.dense_bits + (size_t)idx * DENSE_WORDS + lane * (DENSE_LANE_BYTES / 32);
#pragma unroll
        for (int w = 0; w < DENSE_LANE_BYTES / 32; ++w) out[w] = words[w];
    }
}

// ---------------------------------------------------------------------------
// Resolve: one lane per file walks compute_file_chunks' loop over candidates.
// ---------------------------------------------------------------------------
struct Cand {
    uint64_t pos;
    uint32_t fix;
    bool fix_known;
};

// First G-candidate with global position in [a, b).
__device__ bool find_cand(const Tables &T, uint64_t a, uint64_t b, Cand *c) {
    if (a >= b) return false;
    uint32_t t = (uint32_t)(a / TILE);
    const uint32_t tl = (uint32_t)((b - 1) / TILE);
    while (t <= tl) {
        uint32_t w = t >> 6;
        unsigned long long bits = T.nonempty[w] & (~0ull << (t & 63));
        while (!bits) {
            ++w;
            if ((w << 6) > tl) return false;
            bits = T.nonempty[w];
        }
        t = (w << 6) + (uint32_t)__builtin_ctzll(bits);
        if (t > tl) return false;
        const uint32_t meta = T.tile_meta[t];
        const uint64_t tb = (uint64_t)t * TILE;
        if (meta & DENSE_BIT) {
            const uint32_t idx = meta & ~DENSE_BIT;
            if (idx < T.dense_cap) {              // else: overflowed, host re-runs
                const uint32_t *bm = T.dense_bits + (size_t)idx * DENSE_WORDS;
                const uint32_t r0 = a > tb ? (uint32_t)(a - tb) : 0u;
                const uint32_t r1 = (uint32_t)min<uint64_t>(b - tb, (uint64_t)TILE);
                for (uint32_t wi = r0 >> 5; (wi << 5) < r1; ++wi) {
                    uint32_t m = bm[wi];
                    if ((wi << 5) < r0) m &= ~0u << (r0 & 31);
                    if (m) {
                        const uint32_t r = (wi << 5) + (uint32_t)__builtin_ctz(m);
                        if (r >= r1) return false;
                        c->pos = tb + r;
                        c->fix = 0;
                        c->fix_known = false;
                        return true;
                    }
                }
            }
        } else {
            const uint2 *sl = T.slots + (size_t)t * LISTCAP;
            for (uint32_t j = 0; j < meta; ++j) {
                const uint2 v = sl[j];
                const uint64_t p = tb + v.x;
                if (p >= a) {
                    if (p >= b) return false;
                    c->pos = p;
                    c->fix = v.y;
                    c->fix_known = true;
                    return true;
                }
            }
        }
        ++t;
    }
    return false;
}

// First chunk-local hit in [a, b) for a chunk starting at a (b - a <= 63).
__device__ uint64_t head_scan(const uint8_t *data, uint64_t a, uint64_t b, uint32_t mask) {
    uint32_t S = 0, W = 0;
    for (uint64_t q = a; q < b; ++q) {
        S += data[q];
        W += S;
        if (hit_exact(S, W, mask)) return q;
    }
    return NONE;
}

__global__ __launch_bounds__(64) void cdc_resolve_kernel(const uint8_t *__restrict__ data,
                                                         KParams P, Tables T) {
    const uint32_t k = blockIdx.x * 64 + threadIdx.x;
    if (k >= T.nfiles) return;
    const uint32_t i = T.order[k];
    const uint64_t F = T.flen[i], g0 = T.foff[i];
    DevCut *out = T.cuts + T.cut_base[i];
    const uint32_t cap = T.cut_cap[i];
    const uint64_t MAX = P.max_chunk;
    const uint64_t CAP = P.read_cap ? P.read_cap : ~0ull;
    uint64_t cnt = 0;
    // compute_file_chunks (file_operations.rs:737-784): R = bytes buffered.
    uint64_t R = min(min(F, MAX), CAP);                   // first read :738
    uint64_t s = 0;
    int head = 0;            // 0: file start (G is chunk-local), 1: fix known, 2: unknown
    uint32_t fix = 0;
    while (s < R) {                                       // n = R - s > 0  :747
        const uint64_t lim = R;                           // endofs = min(MAX, n) :749-752
        Cand c;
        bool found = false, known = false;
        uint32_t cfix = 0;
        uint64_t e = NONE;
        if (head == 0) {
            if (find_cand(T, g0 + s, g0 + lim, &c)) { e = c.pos - g0; found = true; known = c.fix_known; cfix = c.fix; }
        } else {
            uint64_t hh = NONE;
            if (head == 1) {
                if (fix) hh = s - 1 + fix;
            } else {
                const uint64_t hb = min(s + 63, lim);
                const uint64_t h = head_scan(data, g0 + s, g0 + hb, P.mask);
                if (h != NONE) hh = h - g0;
            }
            if (hh != NONE && hh < lim) {
                e = hh; found = true; known = false;      // chunk-local head hit
            } else if (s + 63 < lim && find_cand(T, g0 + s + 63, g0 + lim, &c)) {
                e = c.pos - g0; found = true; known = c.fix_known; cfix = c.fix;
            }
        }
        uint64_t cut;                                     // edge or endofs :754-755
        if (found) { cut = e + 1; head = known ? 1 : 2; fix = cfix; }
        else { cut = lim; head = 2; }
        if (cnt < cap) {
            DevCut d;
            d.offset = s;
            d.len = (uint32_t)(cut - s);
            d.file = i;
            out[cnt] = d;
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
    for (uint64_t j = 0; j < n; ++j) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        p[j] = (uint8_t)(x >> 32);
    }
}

// ---------------------------------------------------------------------------
hipError_t launch_scan(const uint8_t *d, const KParams &p, const Tables &t, hipStream_t s) {
    if (!t.ntiles) return hipSuccess;
    const uint32_t blocks = (t.ntiles + WAVES - 1) / WAVES;
    hipLaunchKernelGGL(cdc_scan_kernel, dim3(blocks), dim3(64 * WAVES), LDS_BLOCK, s, d, p, t);
    return hipGetLastError();
}

hipError_t launch_dense(const uint8_t *d, const KParams &p, const Tables &t, hipStream_t s) {
    if (!t.ntiles || !t.dense_cap) return hipSuccess;
    const uint32_t blocks = t.dense_cap < 2048u ? t.dense_cap : 2048u;
    hipLaunchKernelGGL(cdc_dense_kernel, dim3(blocks), dim3(64), 0, s, d, p, t);
    return hipGetLastError();
}

hipError_t launch_resolve(const uint8_t *d, const KParams &p, const Tables &t, hipStream_t s) {
    if (!t.nfiles) return hipSuccess;
    hipLaunchKernelGGL(cdc_resolve_kernel, dim3((t.nfiles + 63) / 64), dim3(64), 0, s, d, p, t);
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
