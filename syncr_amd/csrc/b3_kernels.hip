// b3_kernels.hip -- gfx950 BLAKE3 of every chunk of a launch.
//
// Replaces the per-chunk hash of compute_file_chunks:
//     let hash_binary = util::hash_binary(&buf[..count]);   src/protocol/file_operations.rs:757
//     util::hash_binary(buf) = *blake3::hash(buf).as_bytes()  src/util.rs:57-59
// so a launch yields complete ChunkInfo{hash, offset, size} (src/protocol/types.rs:24-29).
//
// BLAKE3 splits a chunk of `len` bytes into 1 KiB leaves (16 blocks of 64 B,
// compressed in sequence) whose chaining values (CVs) are merged in a
// left-balanced binary tree of PARENT compressions; the last compression of
// the root gets the ROOT flag.  Leaves are independent; a lane TASK is
// LPL consecutive leaves (contiguous bytes; LPL = B3_LANE_LEAVES, or 1 on a
// launch of at most B3_SMALL_SPAN bytes: HashTables::lpl_log):
//   b3_items_kernel  one block per 256 files (per part of their cut list): a chunk of T <= 64 tasks goes to packed
//                    class c = ceil(log2 T) (64 >> c chunks share a wave, each
//                    in an aligned run of 2^c lanes); a bigger chunk becomes
//                    ceil(T / 64) group items plus a tree entry;
//   b3_leaf_kernel   persistent waves pull wave items (group items first, then
//                    packed classes 6..0): each lane compresses its task's
//                    leaves, folds them into one subtree CV, then the lanes of
//                    each chunk merge by shuffles -> the hash of a packed chunk,
//                    or one CV per group item;
//   b3_tree_kernel   one wave per multi-item chunk merges its group CVs.
// Any aligned power-of-two run of leaves (or the run's tail) is a subtree of
// the left-balanced tree, so these partial merges are the tree's own nodes.
//
// Compute bound: 7 rounds x 8 G x 12 integer ops per 64-byte block
// (~10.5 VALU ops per byte); the 1 byte/byte HBM read is not the limit.
#include "cdc_internal.h"
#include "lds_dma.h"

namespace cdc {

namespace {

constexpr uint32_t B3_START = 1u, B3_END = 2u, B3_PARENT = 4u, B3_ROOT = 8u;
constexpr uint32_t IV0 = 0x6A09E667u, IV1 = 0xBB67AE85u, IV2 = 0x3C6EF372u, IV3 = 0xA54FF53Au,
                   IV4 = 0x510E527Fu, IV5 = 0x9B05688Cu, IV6 = 0x1F83D9ABu, IV7 = 0x5BE0CD19u;

// message word schedule: SCHED[r][k] = index of the original word used at
// position k of round r (the spec permutes the message between rounds)
struct Sched {
    uint8_t s[7][16];
};
constexpr uint8_t PERM[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
constexpr Sched make_sched() {
    Sched t{};
    for (int k = 0; k < 16; ++k) t.s[0][k] = (uint8_t)k;
    for (int r = 1; r < 7; ++r)
        for (int k = 0; k < 16; ++k) t.s[r][k] = t.s[r - 1][PERM[k]];
    return t;
}
constexpr Sched SCHED = make_sched();

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_rotateright32(x, n); }

#define B3_G(a, b, c, d, mx, my)      \
    do {                              \
        v[a] = v[a] + v[b] + (mx);    \
        v[d] = rotr(v[d] ^ v[a], 16); \
        v[c] = v[c] + v[d];           \
        v[b] = rotr(v[b] ^ v[c], 12); \
        v[a] = v[a] + v[b] + (my);    \
        v[d] = rotr(v[d] ^ v[a], 8);  \
        v[c] = v[c] + v[d];           \
        v[b] = rotr(v[b] ^ v[c], 7);  \
    } while (0)

// cv <- first half of compress(cv, m, counter, blen, flags) (the chaining value
// / the 32-byte hash when flags has ROOT)
__device__ __forceinline__ void compress(uint32_t cv[8], const uint32_t m[16], uint32_t counter,
                                         uint32_t blen, uint32_t flags) {
    uint32_t v[16] = {cv[0], cv[1], cv[2], cv[3], cv[4], cv[5], cv[6], cv[7],
                      IV0,   IV1,   IV2,   IV3,   counter, 0u, blen, flags};
#pragma unroll
    for (int r = 0; r < 7; ++r) {
        const uint8_t *s = SCHED.s[r];
        B3_G(0, 4, 8, 12, m[s[0]], m[s[1]]);
        B3_G(1, 5, 9, 13, m[s[2]], m[s[3]]);
        B3_G(2, 6, 10, 14, m[s[4]], m[s[5]]);
        B3_G(3, 7, 11, 15, m[s[6]], m[s[7]]);
        B3_G(0, 5, 10, 15, m[s[8]], m[s[9]]);
        B3_G(1, 6, 11, 12, m[s[10]], m[s[11]]);
        B3_G(2, 7, 8, 13, m[s[12]], m[s[13]]);
        B3_G(3, 4, 9, 14, m[s[14]], m[s[15]]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) cv[i] = v[i] ^ v[i + 8];
}
#undef B3_G

__device__ __forceinline__ void set_iv(uint32_t cv[8]) {
    cv[0] = IV0; cv[1] = IV1; cv[2] = IV2; cv[3] = IV3;
    cv[4] = IV4; cv[5] = IV5; cv[6] = IV6; cv[7] = IV7;
}

// x <- parent(x, r): a PARENT node over two child CVs (counter 0, 64 bytes)
__device__ __forceinline__ void parent(uint32_t x[8], const uint32_t r[8], uint32_t extra) {
    uint32_t m[16];
#pragma unroll
    for (int k = 0; k < 8; ++k) { m[k] = x[k]; m[8 + k] = r[k]; }
    set_iv(x);
    compress(x, m, 0u, 64u, B3_PARENT | extra);
}

// Merge the CVs held by lanes 0..m-1 (level pairing, the last node of an odd
// level is promoted) into lane 0.  `root`: this is the whole tree, so the
// final merge gets ROOT.  m, root are wave-uniform.
__device__ __forceinline__ void wave_merge(uint32_t x[8], uint32_t m, bool root, int lane) {
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        if (m > d) {                               // wave-uniform
            uint32_t r[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) r[k] = (uint32_t)__shfl_down((int)x[k], d);
            const bool act = ((uint32_t)lane & (2 * d - 1)) == 0 && (uint32_t)lane + d < m;
            if (act) parent(x, r, (root && m <= 2 * d) ? B3_ROOT : 0u);
        }
    }
}

// The 16 message words of the 64 bytes at batch offset p, bytes at or past
// `valid` (< 64 only on a chunk's last block) read as zero.  p has any
// alignment: gfx950 global loads are unaligned-capable (hipcc itself emits
// global_load_dwordx4 for a byte-aligned 16-byte memcpy).
template <bool NT>
__device__ __forceinline__ void load_block(const uint8_t *__restrict__ data, uint64_t span, uint64_t p,
                                           uint32_t valid, uint32_t m[16]) {
    if (p + 64 <= span) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            v4u v;
            if constexpr (NT) {
                v4u t;
                __builtin_memcpy(&t, data + p + 16 * i, 16);
                v = __builtin_nontemporal_load(&t);
            } else {
                __builtin_memcpy(&v, data + p + 16 * i, 16);
            }
            m[4 * i] = v.x; m[4 * i + 1] = v.y; m[4 * i + 2] = v.z; m[4 * i + 3] = v.w;
        }
    } else {                                   // the batch's last bytes: guarded byte loads
        // one 32-bit limit (no per-byte 64-bit compares: this rare path sets
        // the kernel's peak register count); the bytes past it are zero
        const uint32_t lim = (uint32_t)min<uint64_t>(valid, span > p ? span - p : 0ull);
        const uint8_t *src = data + p;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            uint32_t w = 0;
            for (int b = 0; b < 4; ++b)
                if ((uint32_t)(4 * k + b) < lim) w |= (uint32_t)src[4 * k + b] << (8 * b);
            m[k] = w;
        }
        return;
    }
    // only a task's last block can be partial: a wave-uniform branch keeps the
    // compiler from if-converting the masking into the full-block path
    if (__builtin_expect(__ballot(valid < 64) != 0ull, 0)) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int c = (int)valid - 4 * k;
            const uint32_t keep = c >= 4 ? 0xffffffffu : (c <= 0 ? 0u : (1u << (8 * c)) - 1u);
            m[k] &= keep;
        }
    }
}

__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t u = (uint32_t)__shfl_up((int)v, off);
        if (lane >= off) v += u;
    }
    return v;
}

__device__ __forceinline__ uint64_t bcast64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// cnt[key]++ for every active lane, returning each lane's old value, with one
// LDS atomic per distinct key of the wave instead of one per lane: a block of
// 64-byte chunks (periodic data: millions per file) otherwise serialises all
// 256 threads on the same class counter (18.4 ms for the dense workload's
// 7.4 M chunks).  Works under divergence: only active lanes take part.
__device__ __forceinline__ uint32_t agg_inc(uint32_t *cnt, uint32_t key) {
    const uint32_t lane = threadIdx.x & 63u;
    const unsigned long long below = lane ? (~0ull >> (64u - lane)) : 0ull;
    uint32_t res = 0;
    unsigned long long rem = __ballot(1);
    while (rem) {
        const int leader = __builtin_ctzll(rem);
        const uint32_t k = (uint32_t)__builtin_amdgcn_readlane((int)key, leader);
        const unsigned long long m = __ballot(key == k);
        uint32_t base = 0;
        if ((int)lane == leader) base = atomicAdd(&cnt[k], (uint32_t)__builtin_popcountll(m));
        base = (uint32_t)__builtin_amdgcn_readlane((int)base, leader);
        if (key == k) res = base + (uint32_t)__builtin_popcountll(m & below);
        rem &= ~m;
    }
    return res;
}

__device__ __forceinline__ uint32_t chunk_leaves(uint32_t len) { return len ? (len + 1023u) >> 10 : 1u; }
__device__ __forceinline__ uint32_t chunk_tasks(uint32_t len, uint32_t lpl_log) {
    return (chunk_leaves(len) + (1u << lpl_log) - 1u) >> lpl_log;
}
__device__ __forceinline__ uint32_t ceil_log2(uint32_t t) { return t <= 1 ? 0u : 32u - __builtin_clz(t - 1); }

}  // namespace

// ---------------------------------------------------------------------------
// One block per 256 files and per part of their cuts: the group's cuts form
// one flat list (a block scan of the per-file counts) and a block takes its
// part of it (~16384 output slots per part, host-planned from the caps), so
// every thread has work whatever the file sizes and a file of millions of
// chunks is planned by many blocks.
// Packed chunks are appended to their class list; a big chunk gets its group
// items (slot << 24 | group, contiguous per chunk) and a tree entry {slot,
// first item}.  When its task count T is not a multiple of 64 the last item
// is a placeholder (B3_TAIL set; skipped by the group loop) and the T % 64
// tail tasks are a unit in the class list of their size (B3_TAIL | item).  Slots are handed out by LDS atomics in two passes (count, then
// place) so the global counters see one atomic per list per block.  A file
// whose cuts overflowed its output slots is skipped (the host re-launches).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void b3_items_kernel(Tables T, HashTables H) {
    constexpr int NL = B3_CLASSES + 3;                   // lists: classes, group items, trees, pieces
    constexpr int LIST_ITEMS = B3_CLASSES, LIST_TREES = B3_CLASSES + 1, LIST_PIECES = B3_CLASSES + 2;
    __shared__ uint32_t cnt[NL];
    __shared__ uint64_t gbase[NL];
    __shared__ uint32_t foff[257];                       // exclusive prefix of cut counts
    __shared__ uint64_t fbase[256];                      // cut_base of the block's files
    __shared__ uint32_t wsum[4];
    const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
    // block = (file group, part of its cut list, parts): see upload_cut_tables
    const uint64_t ibk = H.iblocks[blockIdx.x];
    const uint32_t grp = (uint32_t)(ibk >> 40), part = (uint32_t)((ibk >> 20) & 0xfffffu),
                   parts = (uint32_t)(ibk & 0xfffffu);
    const uint32_t i = grp * 256 + t;
    uint32_t nc = 0;
    if (i < T.nfiles) {
        const uint64_t n = T.counts[i];
        if (n <= T.cut_cap[i]) nc = (uint32_t)n;
        fbase[t] = T.cut_base[i];
    }
    if (t < NL) cnt[t] = 0;
    const uint32_t incl = wave_incl_scan_u32(nc, (int)lane);
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    uint32_t before = 0;
    for (uint32_t k = 0; k < w; ++k) before += wsum[k];
    foff[t + 1] = before + incl;
    if (t == 0) foff[0] = 0;
    __syncthreads();
    const uint32_t all = foff[256];
    const uint32_t qbeg = (uint32_t)((uint64_t)all * part / parts), total = (uint32_t)((uint64_t)all * (part + 1) / parts);
    // a unit of r tasks (first task k0) whose r is not a power of two becomes
    // popcount(r) pieces, the binary digits of r largest first
    auto put_pieces = [&](bool place, uint64_t slot, uint32_t k0, uint32_t r, uint64_t &pbase) {
        const uint32_t np = (uint32_t)__builtin_popcount(r);
        const uint32_t lpc = atomicAdd(&cnt[LIST_PIECES], np);
        pbase = place ? gbase[LIST_PIECES] + lpc : 0ull;
        uint32_t off = k0, p = 0;
        for (int b = 6; b >= 0; --b) {
            if (!((r >> b) & 1u)) continue;
            const uint32_t li = atomicAdd(&cnt[b], 1u);
            if (place) {
                const uint64_t pi = pbase + p;
                const uint64_t idx = gbase[b] + li;
                if (pi < H.pieces_cap) {
                    H.pieces[pi] = make_ulonglong2(slot, off);
                    if (idx < H.packed_cap) H.packed[b * H.packed_cap + idx] = B3_PIECE | pi;
                } else {
                    atomicOr((unsigned long long *)&H.ctr[B3C_FLAGS], 2ull);
                }
            }
            off += 1u << b;
            ++p;
        }
        return np;
    };
    auto one = [&](bool place, uint64_t slot, uint32_t len) {
        {
            const uint32_t tk = chunk_tasks(len, H.lpl_log);
            if (tk <= 64) {
                if ((tk & (tk - 1)) == 0 || H.nosplit) {  // one unit: the whole chunk
                    const uint32_t c = ceil_log2(tk);
                    const uint32_t li = agg_inc(cnt, c);
                    if (place) {
                        const uint64_t idx = gbase[c] + li;
                        if (idx < H.packed_cap) H.packed[c * H.packed_cap + idx] = slot;
                    }
                } else {                                 // pieces, folded (with ROOT) by the tree kernel
                    uint64_t pb = 0;
                    const uint32_t np = put_pieces(place, slot, 0u, tk, pb);
                    const uint32_t lt = agg_inc(cnt, LIST_TREES);
                    if (place) {
                        const uint64_t ti = gbase[LIST_TREES] + lt;
                        if (ti < H.trees_cap) {
                            H.trees[ti] = make_ulonglong2(slot, ~0ull);
                            H.tpieces[ti] = (pb << 8) | np;
                        }
                    }
                }
            } else {                                     // big chunk: full group items + tail unit
                const uint32_t tail = tk % 64, ng = tk / 64 + (tail ? 1u : 0u);
                const uint32_t li = atomicAdd(&cnt[LIST_ITEMS], ng);
                const uint32_t lt = atomicAdd(&cnt[LIST_TREES], 1u);
                const bool split = tail && (tail & (tail - 1)) != 0 && !H.nosplit;
                const uint32_t c = ceil_log2(tail);
                const uint32_t lp = (tail && !split) ? atomicAdd(&cnt[c], 1u) : 0u;
                uint64_t pb = 0;
                const uint32_t np = split ? put_pieces(place, slot, (ng - 1) * 64u, tail, pb) : 0u;
                if (place) {
                    const uint64_t first = gbase[LIST_ITEMS] + li;
                    if (first + ng <= H.items_cap) {
                        for (uint32_t g = 0; g < ng; ++g)   // the tail's entry is a placeholder
                            H.items[first + g] = (slot << 24) | g | (tail && g + 1 == ng ? B3_TAIL : 0ull);
                        if (tail && !split) {
                            const uint64_t idx = gbase[c] + lp;
                            if (idx < H.packed_cap) H.packed[c * H.packed_cap + idx] = B3_TAIL | (first + ng - 1);
                        }
                    } else {
                        atomicOr((unsigned long long *)&H.ctr[B3C_FLAGS], 1ull);
                    }
                    const uint64_t ti = gbase[LIST_TREES] + lt;
                    if (ti < H.trees_cap) {
                        H.trees[ti] = make_ulonglong2(slot, first);
                        H.tpieces[ti] = (pb << 8) | np;
                    }
                }
            }
        }
    };
    // A thread's cuts are visited UNROLL at a time with their lengths loaded
    // first: one HBM round trip per UNROLL cuts instead of per cut (a block
    // holding one periodic file has millions of cuts: 16 ms of serial
    // round trips per pass before).
    constexpr int UNROLL = 16;
    auto visit = [&](bool place) {
        for (uint32_t q0 = qbeg + t; q0 < total; q0 += 256u * UNROLL) {
            uint64_t slots[UNROLL];
            uint32_t lens[UNROLL];
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) {
                const uint32_t q = q0 + 256u * (uint32_t)u;
                slots[u] = 0;
                lens[u] = 0;
                if (q < total) {
                    uint32_t lo = 0, hi = 256;           // last f with foff[f] <= q
                    while (hi - lo > 1) {
                        const uint32_t mid = (lo + hi) >> 1;
                        if (foff[mid] <= q) lo = mid; else hi = mid;
                    }
                    slots[u] = fbase[lo] + (q - foff[lo]);
                    lens[u] = T.cuts[slots[u]].len;
                }
            }
#pragma unroll
            for (int u = 0; u < UNROLL; ++u)
                if (q0 + 256u * (uint32_t)u < total) one(place, slots[u], lens[u]);
        }
    };
    visit(false);                                        // pass 1: count per list
    __syncthreads();
    if (t < NL) {
        const uint32_t gi = t < B3_CLASSES ? B3C_PK0 + t
                          : (t == LIST_ITEMS ? B3C_ITEMS : (t == LIST_TREES ? B3C_TREES : B3C_PIECES));
        gbase[t] = cnt[t] ? atomicAdd((unsigned long long *)&H.ctr[gi], (unsigned long long)cnt[t]) : 0ull;
        cnt[t] = 0;
    }
    __syncthreads();
    visit(true);                                         // pass 2: place
}

// ---------------------------------------------------------------------------
// Loader kinds of the leaf kernel (template parameter LD): per-lane global
// loads (LD_PLAIN, development A/B only), the cooperative LDS-DMA loader one
// 64-byte block per task per issue round (LD_COOP64), or two blocks (one
// 128-byte run) per task per round (LD_PAIR).
constexpr int LD_PLAIN = 0, LD_PAIR = 2;
[[maybe_unused]] constexpr int LD_COOP64 = 1;   // (development library only)

// ---------------------------------------------------------------------------
// Cooperative block loader (COOP): the wave steps through block index t in
// lockstep (t < wave max of the tasks' block counts).  Block t+1 of all 64
// tasks is fetched by four global_load_lds_dwordx4: instruction i moves one
// 16-byte piece of each of tasks 16i..16i+15, so every instruction reads 16
// contiguous 64-byte runs instead of 64 scattered 16-byte pieces.  Task q's
// block lands at slot + 64 q with its pieces rotated by (q >> 2) & 3, which
// makes the owner's four ds_read_b128 bank-conflict free.  Bytes past the
// chunk (a task's last block) are zeroed by the owner; pieces that would read
// past the batch end are not DMA'd but loaded byte by byte by the owner.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src), hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src);
    return ((uint64_t)hi << 32) | lo;
}

//
// LD_PAIR: blocks t, t+1 (t even) of all 64 tasks are fetched together by
// eight instructions (instruction i: tasks 8i..8i+7, one 128-byte run each),
// into an 8 KiB slot (task q at slot + 128 q, 16-byte pieces of each 64-byte
// half rotated by (q >> 1) & 3).  A 128-byte run at a line-aligned task start
// is one L2 line, read once; the 64-byte rounds touch every line in two
// consecutive rounds, and the second touch misses L2 for a third of the
// lines (profiles/r02_fetch_calibration.json: 1.34x the input bytes).
// The next pair is issued once block t+1 is in registers, so it lands under
// block t+1's compression, as the single-block round lands under block t's.
template <bool NT, int ABLATE, int LD, uint32_t LPL>
__device__ __forceinline__ void leaf_blocks_coop(const uint8_t *__restrict__ data, uint64_t span, uint32_t stage,
                                                 uint32_t *stage_ptr, int lane, bool act, uint64_t tp,
                                                 uint32_t nbytes, uint32_t nblk, uint32_t nl, uint32_t nleaves,
                                                 uint32_t j0, bool task_root, bool uni, uint64_t tp0,
                                                 uint32_t x[8]) {
    // leaf CVs are folded as they complete (left-balanced pairing of <= 4
    // leaves): x = leaf 0, then node(0,1); y = leaf 2, then node(2,3)
    static_assert(LPL == 1 || LPL == 4, "lane tasks of 1 or 4 leaves");
    constexpr uint32_t TASK = 1024u * LPL;                    // bytes per lane task
    uint32_t y[8];
    // piece at task byte ps (multiple of 16) is DMA'd iff ps < plim: inside the
    // chunk's task and 16 bytes inside the batch
    const uint32_t plim = act ? (uint32_t)min<uint64_t>(nbytes, span >= tp + 16 ? span - tp - 15 : 0ull) : 0u;
    uint32_t tmax = nblk;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) tmax = max(tmax, (uint32_t)__shfl_xor((int)tmax, o));
    tmax = (uint32_t)__builtin_amdgcn_readfirstlane((int)tmax);
    // the piece sources are re-derived from the owners' registers at every
    // issue (ds_bpermute): holding four 64-bit sources and limits across the
    // compression cost 5 -> 4 waves/SIMD
    constexpr bool PAIR = LD == LD_PAIR;
    auto issue = [&](uint32_t t) {           // PAIR: t is even, blocks t and t+1
        if constexpr (PAIR) {
            if (uni) {
                // a group item inside the batch (wave-uniform): task q starts at
                // tp0 + TASK q, so instruction i's source is the SGPR base
                // tp0 + 64 t + 8 TASK i plus a per-lane offset fixed for the item
                // ((q >> 1) & 3 == (lane >> 4) & 3 for every i) -- no shuffles, no
                // per-piece branch; pieces past a partial last task are fetched
                // from inside the batch and overwritten by the owner's fix-up
                const uint32_t pos = (uint32_t)lane & 7u;
                const uint32_t pc = (pos & 4u) | ((pos & 3u) ^ (((uint32_t)lane >> 4) & 3u));
                const uint32_t voff = ((uint32_t)lane >> 3) * TASK + pc * 16u;
                const uint64_t b = (uint64_t)(data + tp0) + (uint64_t)t * 64u;
#pragma unroll
                for (int i = 0; i < 8; ++i) dma16_s<NT>(voff, b + 8ull * TASK * (uint64_t)i, stage + (uint32_t)i * 1024u);
                return;
            }
        }
        // opaque copies: keep the shuffles here instead of hoisted out of the loop
        uint32_t tl = (uint32_t)tp, th = (uint32_t)(tp >> 32), pl = plim;
        asm volatile("" : "+v"(tl), "+v"(th), "+v"(pl));
        if constexpr (PAIR) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int q = 8 * i + (lane >> 3);
                const uint32_t pos = (uint32_t)lane & 7u;                     // 16-byte position in the run
                const uint32_t pc = (pos & 4u) | ((pos & 3u) ^ (((uint32_t)q >> 1) & 3u));   // piece moved
                const uint32_t ps = t * 64u + pc * 16u;
                const uint32_t l = (uint32_t)__shfl((int)pl, q);
                const uint64_t src = ((uint64_t)(uint32_t)__shfl((int)th, q) << 32) | (uint32_t)__shfl((int)tl, q);
                if (ps < l) dma16<NT>(data + src + ps, stage + (uint32_t)i * 1024u);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int q = 16 * i + (lane >> 2);
                const uint32_t pc = ((uint32_t)lane & 3u) ^ (((uint32_t)q >> 2) & 3u);   // piece this lane moves
                const uint32_t ps = t * 64u + pc * 16u;
                const uint32_t l = (uint32_t)__shfl((int)pl, q);
                const uint64_t src = ((uint64_t)(uint32_t)__shfl((int)th, q) << 32) | (uint32_t)__shfl((int)tl, q);
                if (ps < l) dma16<NT>(data + src + ps, stage + (uint32_t)i * 1024u);
            }
        }
    };
    const uint32_t rot = PAIR ? (((uint32_t)lane >> 1) & 3u) : (((uint32_t)lane >> 2) & 3u);
    uint8_t *const mine0 = (uint8_t *)stage_ptr + lane * (PAIR ? 128 : 64);
    if (ABLATE != 2 && tmax) issue(0);
#pragma unroll
    for (uint32_t jj = 0; jj < LPL; ++jj) {
        if (16 * jj < tmax) {                                    // uniform
            uint32_t cv[8];
            set_iv(cv);
            const uint32_t lbu = min(16u, tmax - 16 * jj);             // uniform blocks of this leaf
            const uint32_t lb = nblk > 16 * jj ? min(16u, nblk - 16 * jj) : 0u;   // this lane's
            for (uint32_t b = 0; b < lbu; ++b) {
                const uint32_t t = 16 * jj + b;
                const uint32_t off = t * 64;
                const uint32_t vb = nbytes > off ? min(64u, nbytes - off) : 0u;
                uint32_t m[16];
                if constexpr (ABLATE == 2) {               // timing only: no loads
    #pragma unroll
                    for (int q = 0; q < 16; ++q) m[q] = (uint32_t)lane * 0x9E3779B9u + q + off;
                } else {
                    uint8_t *const mine = mine0 + (PAIR ? (t & 1u) * 64u : 0u);
                    if (!PAIR || (t & 1u) == 0u) wait_vmcnt<0>();     // block t has landed
                    // bytes of my block that are past the chunk or were not DMA'd
                    const uint32_t dma_end = plim > off ? min(64u, (plim - off + 15u) & ~15u) : 0u;
                    const uint32_t fix = min(vb, dma_end);
                    if (__builtin_expect(__ballot(b < lb && fix < 64u) != 0ull, 0)) {
                        if (b < lb) {
    #pragma unroll 1
                            for (uint32_t q = fix; q < 64u; ++q) {
                                const uint8_t v = q < vb ? data[tp + off + q] : (uint8_t)0;
                                mine[(((q >> 4) ^ rot) << 4) | (q & 15u)] = v;
                            }
                        }
                    }
    #pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const uint4 v = *(const uint4 *)(mine + ((((uint32_t)i) ^ rot) << 4));
                        m[4 * i] = v.x; m[4 * i + 1] = v.y; m[4 * i + 2] = v.z; m[4 * i + 3] = v.w;
                    }
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");     // slot free for block t+1
                    if (PAIR) {
                        if ((t & 1u) && t + 1 < tmax) issue(t + 1);
                    } else if (t + 1 < tmax) {
                        issue(t + 1);
                    }
                }
                if (b < lb) {
                    uint32_t fl = (b == 0 ? B3_START : 0u) | (b + 1 == lb ? B3_END : 0u);
                    if (b + 1 == lb && nleaves == 1) fl |= B3_ROOT;
                    if constexpr (ABLATE == 1) {           // timing only: loads, no compression
    #pragma unroll
                        for (int q = 0; q < 8; ++q) cv[q] ^= m[q] + m[q + 8] + fl;
                    } else {
                        compress(cv, m, j0 + jj, vb, fl);
                    }
                }
            }
            if (jj < nl) {
                if (jj == 0) {
    #pragma unroll
                    for (int q = 0; q < 8; ++q) x[q] = cv[q];
                } else if (jj == 1) {
                    parent(x, cv, (task_root && nl == 2) ? B3_ROOT : 0u);
                } else if (jj == 2) {
    #pragma unroll
                    for (int q = 0; q < 8; ++q) y[q] = cv[q];
                } else {
                    parent(y, cv, 0u);
                }
            }
        }
    }
    if (LPL > 2 && nl > 2) parent(x, y, task_root ? B3_ROOT : 0u);
}

// ---------------------------------------------------------------------------
// Cross-lane merges by quads (MQ).  The shuffle merge (one `parent` per level
// with the whole wave issuing a full compression for 64 / 2d active lanes)
// spends 6 x 688 VALU instructions on the 63 parents of a group item.  Here a
// parent is computed by four lanes, one per column of the state: the column
// G, three quad rotations (DPP quad_perm), the diagonal G, three rotations
// back -- 30 instructions per round instead of 96 -- so the 16 parents of a
// level take one pass of the wave (level 1: two).  Node CVs live in the
// wave's LDS slot, compacted per level: node n of a level at byte 36 n (the
// 4-byte pad spreads the quads over the banks), so the two children of parent
// p are the 72 bytes at 72 p and parent p becomes node p of the next level.
// A lane's message words are read from LDS at per-lane addresses fixed for
// the whole merge (quad p = lane >> 2 always reads message p; lane i of the
// quad needs words SCHED[r][2i, 2i+1, 8+2i, 9+2i] of round r).  All LDS reads
// of a pass precede its writes in program order, and a wave's LDS accesses
// complete in order, so the in-place compaction needs no barrier.
// ---------------------------------------------------------------------------
constexpr uint32_t mq_off(int r, int s, int i) {          // byte offset of the word in its 72-byte message
    const int k = s < 2 ? 2 * i + s : 8 + 2 * i + (s - 2);
    const uint32_t w = SCHED.s[r][k];
    return w < 8 ? 4 * w : 4 * w + 4;
}
constexpr uint32_t mq_pack(int r, int s) {                // the four lanes' offsets, one byte each
    return mq_off(r, s, 0) | (mq_off(r, s, 1) << 8) | (mq_off(r, s, 2) << 16) | (mq_off(r, s, 3) << 24);
}

template <int CTRL>
__device__ __forceinline__ uint32_t quad_perm(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false);
}
constexpr int QP_NEXT1 = 0x39, QP_NEXT2 = 0x4E, QP_NEXT3 = 0x93;   // lane i <- lane (i+1|2|3) & 3

#define MQ_G(a, b, c, d, mx, my)      \
    do {                              \
        a = a + b + (mx);             \
        d = rotr(d ^ a, 16);          \
        c = c + d;                    \
        b = rotr(b ^ c, 12);          \
        a = a + b + (my);             \
        d = rotr(d ^ a, 8);           \
        c = c + d;                    \
        b = rotr(b ^ c, 7);           \
    } while (0)

// Merge the lanes' CVs x of each unit (aligned runs of dmax lanes, dmax > 1,
// wave-uniform; node km of a unit is at lane U + km) into the unit's CV, left
// in x of every lane of the unit.  km, mm, act, root as in b3_leaf_body.
__device__ __forceinline__ void merge_quads(uint32_t *slot_ptr, int lane, uint32_t dmax, bool act, uint32_t km,
                                            uint32_t mm, bool root, uint32_t x[8]) {
    uint8_t *const lds = (uint8_t *)slot_ptr;
    // opaque copies: the per-lane tables below are loop-invariant, and hoisted
    // out of the wave-item loop they would stay live through the block loop
    // (153 VGPRs, 3 waves/SIMD)
    uint32_t i = (uint32_t)lane & 3u, q = (uint32_t)lane >> 2;
    asm volatile("" : "+v"(i), "+v"(q));
#pragma unroll
    for (int k = 0; k < 8; ++k) *(uint32_t *)(lds + lane * 36 + 4 * k) = x[k];     // level-1 nodes
    uint32_t ad[7][4];                                    // this lane's message word addresses (pass 0)
#pragma unroll
    for (int r = 0; r < 7; ++r)
#pragma unroll
        for (int s = 0; s < 4; ++s) ad[r][s] = q * 72u + __builtin_amdgcn_ubfe(mq_pack(r, s), 8u * i, 8u);
    const uint32_t ivA = i == 0 ? IV0 : (i == 1 ? IV1 : (i == 2 ? IV2 : IV3));
    const uint32_t ivB = i == 0 ? IV4 : (i == 1 ? IV5 : (i == 2 ? IV6 : IV7));
    const uint32_t dfix = i == 2 ? 64u : 0u;              // v[12..14] = counter 0, 0, block length 64
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        if (d >= dmax) break;                             // uniform
        // parent p of this level merges the nodes at lanes 2pd and (2p+1)d; the
        // left child's lane knows whether it merges (1), is promoted (2) or is
        // not a node; bit 3: ROOT
        const uint32_t code = !act ? 0u : (km + d < mm ? (1u | ((root && mm <= 2 * d) ? B3_ROOT : 0u)) : 2u);
#pragma unroll
        for (uint32_t pass = 0; pass < 2; ++pass) {
            if (pass == 1 && d != 1) break;               // 32 parents only at level 1
            const uint32_t p = q + 16u * pass;
            const uint32_t L = 2u * p * d;
            const uint32_t c = (uint32_t)__shfl((int)code, (int)(L & 63u));
            const uint32_t my = L < 64u ? c : 0u;
            if (__ballot(my != 0u) == 0ull) continue;
            const uint32_t pb = pass * 1152u;             // messages 16..31
            // promoted node: words i, 4+i of the left child (read before any write)
            const uint32_t c0 = *(const uint32_t *)(lds + pb + q * 72u + 4u * i);
            const uint32_t c1 = *(const uint32_t *)(lds + pb + q * 72u + 16u + 4u * i);
            uint32_t a = ivA, b = ivB, cc = ivA, dd = i == 3 ? (B3_PARENT | (my & B3_ROOT)) : dfix;
#pragma unroll
            for (int r = 0; r < 7; ++r) {
                const uint32_t m0 = *(const uint32_t *)(lds + pb + ad[r][0]);
                const uint32_t m1 = *(const uint32_t *)(lds + pb + ad[r][1]);
                const uint32_t m2 = *(const uint32_t *)(lds + pb + ad[r][2]);
                const uint32_t m3 = *(const uint32_t *)(lds + pb + ad[r][3]);
                MQ_G(a, b, cc, dd, m0, m1);                                   // column i
                b = quad_perm<QP_NEXT1>(b);
                cc = quad_perm<QP_NEXT2>(cc);
                dd = quad_perm<QP_NEXT3>(dd);
                MQ_G(a, b, cc, dd, m2, m3);                                   // diagonal i
                b = quad_perm<QP_NEXT3>(b);
                cc = quad_perm<QP_NEXT2>(cc);
                dd = quad_perm<QP_NEXT1>(dd);
            }
            __builtin_amdgcn_wave_barrier();
            if (my) {
                const bool merge = (my & 1u) != 0u;
                *(uint32_t *)(lds + p * 36u + 4u * i) = merge ? (a ^ cc) : c0;
                *(uint32_t *)(lds + p * 36u + 16u + 4u * i) = merge ? (b ^ dd) : c1;
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    // the unit's CV: node U / dmax of the last level
    const uint32_t node = (uint32_t)lane >> __builtin_ctz(dmax);
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = *(const uint32_t *)(lds + node * 36u + 4 * k);
}
#undef MQ_G

// ---------------------------------------------------------------------------
// Persistent waves pull wave items: the group items of big chunks first, then
// the packed classes 6..0.  Per lane: a chunk slot, its task k (leaves
// LPL*k .. LPL*k+LPL-1) and the merge geometry of that chunk within the wave.
// ---------------------------------------------------------------------------
template <bool NT, int ABLATE, int LD, bool MQ, uint32_t LPL>
__device__ __forceinline__ void b3_leaf_body(const uint8_t *__restrict__ data, const Tables &T,
                                             const HashTables &H) {
    constexpr uint32_t LG = LPL == 1 ? 0u : 2u;                 // == H.lpl_log (the host launches this instance)
    const int lane = threadIdx.x & 63;
    constexpr bool COOP = LD != LD_PLAIN;
    constexpr uint32_t SLOT = LD == LD_PAIR ? 2048 : 1024;       // words: per-wave staging slot (8 / 4 KiB)
    __shared__ __attribute__((aligned(16))) uint32_t stage_mem[COOP ? 4 * SLOT : 1];
    uint32_t *stage_ptr = stage_mem + (COOP ? (threadIdx.x >> 6) * SLOT : 0);
    const uint32_t stage = (uint32_t)__builtin_amdgcn_readfirstlane(lds_addr(stage_ptr));
    const uint64_t nbig = min(H.ctr[B3C_ITEMS], H.items_cap);
    // Wave items are dealt by B3_SHARDS counters 4 KiB apart (shard k: items
    // k, k + S, k + 2S, ...; a block starts on shard blockIdx % S and moves on
    // when it is spent).  One counter made it the limit on many tiny chunks: one
    // address takes ~70 M atomics/s, and a wave item of class 0 or 1 (64 or 32
    // chunks of <= 4 KiB) can be one compression per lane (dense1: 2.1 M 64-byte
    // chunks = 33 K wave items = 0.45 ms of grabs on one counter).
    uint64_t npk[B3_CLASSES], total = nbig;
#pragma unroll
    for (int c = 0; c < B3_CLASSES; ++c) {
        npk[c] = min(H.ctr[B3C_PK0 + c], H.packed_cap);
        total += (npk[c] + (64u >> c) - 1) >> (6 - c);          // waves of class c
    }
    uint32_t shard = blockIdx.x % B3_SHARDS, spent = 0;
    for (;;) {
        unsigned long long *const sc = (unsigned long long *)&H.ctr[(shard + 1) * B3_SHARD_STRIDE];
        uint64_t j = 0;
        if (lane == 0) {
            // a shard other than the block's own is looked at first (a load: no
            // atomic on a counter that is already past its last item)
            j = spent ? __hip_atomic_load(sc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
            if (shard + j * B3_SHARDS < total) j = atomicAdd(sc, 1ull);
        }
        j = bcast64(j);
        const uint64_t w = shard + j * B3_SHARDS;
        if (w >= total) {                                        // this shard is spent: the next one
            if (++spent == B3_SHARDS) break;
            shard = (shard + 1) % B3_SHARDS;
            continue;
        }
        // per-lane geometry
        bool valid;
        uint64_t slot = 0;
        uint32_t k;              // task index within the chunk
        uint32_t km, mm;         // merge index / node count of this lane's unit in this wave
        uint32_t dmax;           // merge levels: lanes per unit in this wave (uniform)
        bool root;               // this unit is the whole chunk (its merge gets ROOT)
        const bool group = w < nbig;                             // uniform
        uint64_t out_item = w;                                   // group item / tail: its gcv slot; piece: index
        bool tail = false, piece = false;
        uint32_t k0 = 0;                                         // first task of this unit
        if (group) {                                             // 64 tasks of a big chunk
            const uint64_t code = H.items[w];
            if (code & B3_TAIL) continue;                        // placeholder: hashed as a packed unit
            slot = code >> 24;
            k0 = ((uint32_t)code & 0xffffffu) * 64;
            k = k0 + (uint32_t)lane;
            km = (uint32_t)lane;
            mm = 64;
            valid = true;
            dmax = 64;
            root = false;                                        // b3_tree_kernel finishes
        } else {                                                 // packed units
            uint64_t r = w - nbig;
            int c = B3_CLASSES - 1;
            for (; c > 0; --c) {                                 // uniform
                const uint64_t wc = (npk[c] + (64u >> c) - 1) >> (6 - c);
                if (r < wc) break;
                r -= wc;
            }
            const uint64_t idx = r * (64u >> c) + ((uint32_t)lane >> c);
            k = (uint32_t)lane & ((1u << c) - 1u);
            km = k;
            valid = idx < npk[c];
            piece = false;
            if (valid) {
                const uint64_t code = H.packed[c * H.packed_cap + idx];
                tail = (code & B3_TAIL) != 0;
                piece = (code & B3_PIECE) != 0;
                if (tail) {                                      // T % 64 tail tasks of a big chunk
                    out_item = code & ~B3_TAIL;
                    const uint64_t ic = H.items[out_item] & ~B3_TAIL;
                    slot = ic >> 24;
                    k0 = ((uint32_t)ic & 0xffffffu) * 64;
                } else if (piece) {                              // 2^c tasks of a split unit
                    out_item = code & ~B3_PIECE;
                    const ulonglong2 pd = H.pieces[out_item];
                    slot = pd.x;
                    k0 = (uint32_t)pd.y;
                } else {
                    slot = code;
                }
            }
            mm = 0;
            dmax = 1u << c;
            root = !tail && !piece;
        }
        uint32_t len = 0;
        uint64_t cstart = 0;
        if (valid) {
            const DevCut cu = T.cuts[slot];
            len = cu.len;
            cstart = T.foff[cu.file] + cu.offset;                // batch offset of the chunk
            if (!group) {
                k += k0;
                mm = min(dmax, chunk_tasks(len, LG) - k0);       // a piece before the last one is full
            }
        }
        // where the unit's CV goes, fixed before the block loop (slot and
        // out_item then need not stay live through it)
        uint32_t *const dst = root ? H.hashes + slot * 8 : (piece ? H.pcv : H.gcv) + out_item * 8;
        const uint32_t nleaves = chunk_leaves(len);
        const uint32_t j0 = k * LPL;
        const bool act = valid && j0 < nleaves;
        const uint64_t lane_off = (uint64_t)j0 << 10;            // chunk-relative byte offset
        const uint32_t nbytes = act ? (uint32_t)min<uint64_t>(1024ull * LPL, len - lane_off) : 0u;
        const uint32_t nblk = act ? (nbytes ? (nbytes + 63) >> 6 : 1u) : 0u;
        const uint32_t nl = (nblk + 15) >> 4;                    // leaves of this task
        const bool task_root = root && mm == 1;                  // the task is the whole chunk
        uint32_t x[8];
        if constexpr (COOP) {
            // uniform fast loader: a group item whose 64 tasks (64 LPL KiB) lie inside the batch
            const uint64_t tp0 = group ? bcast64(cstart + (uint64_t)k0 * (1024u * LPL)) : 0ull;
            const bool uni = group && tp0 + 64ull * 1024u * LPL + 16u <= T.span && !H.nouni;
            leaf_blocks_coop<NT, ABLATE, LD, LPL>(data, T.span, stage, stage_ptr, lane, act, cstart + lane_off, nbytes,
                                         nblk, nl, nleaves, j0, task_root, uni, tp0, x);
        } else {
            uint32_t lc[LPL][8];                                 // leaf CVs
            // block t of the task (t < nblk) is at task offset 64*t; the next
            // block's loads are issued before the current block is compressed
            auto fetch = [&](uint32_t t, uint32_t m[16]) {
                const uint32_t off = t * 64;
                const uint32_t vb = nbytes > off ? min(64u, nbytes - off) : 0u;
                if constexpr (ABLATE == 2) {               // timing only: no loads
#pragma unroll
                    for (int q = 0; q < 16; ++q) m[q] = (uint32_t)lane * 0x9E3779B9u + q + off;
                } else {
                    load_block<NT>(data, T.span, cstart + lane_off + off, vb, m);
                }
            };
            uint32_t m[16];
            if (nblk) fetch(0, m);
#pragma unroll
            for (uint32_t jj = 0; jj < LPL; ++jj) {
                if (jj >= nl) continue;
                uint32_t cv[8];
                set_iv(cv);
                const uint32_t tb = jj * 16;
                const uint32_t lb = min(16u, nblk - tb);               // blocks of this leaf
                for (uint32_t b = 0; b < lb; ++b) {
                    const uint32_t t = tb + b;
                    uint32_t mn[16];
                    const bool more = t + 1 < nblk;
                    if (more) fetch(t + 1, mn);
                    const uint32_t off = t * 64;
                    const uint32_t vb = nbytes > off ? min(64u, nbytes - off) : 0u;
                    uint32_t fl = (b == 0 ? B3_START : 0u) | (b + 1 == lb ? B3_END : 0u);
                    if (b + 1 == lb && nleaves == 1) fl |= B3_ROOT;
                    if constexpr (ABLATE == 1) {           // timing only: loads, no compression
#pragma unroll
                        for (int q = 0; q < 8; ++q) cv[q] ^= m[q] + m[q + 8] + fl;
                    } else {
                        compress(cv, m, j0 + jj, vb, fl);
                    }
                    if (more) {
#pragma unroll
                        for (int q = 0; q < 16; ++q) m[q] = mn[q];
                    }
                }
#pragma unroll
                for (int q = 0; q < 8; ++q) lc[jj][q] = cv[q];
            }
            // fold the task's leaves (left-balanced level pairing); ROOT when the
            // task is the whole chunk.
#pragma unroll
            for (uint32_t d = 1; d < LPL; d <<= 1)
#pragma unroll
                for (uint32_t i = 0; i + d < LPL; i += 2 * d)
                    if (i + d < nl) parent(lc[i], lc[i + d], (task_root && nl <= 2 * d) ? B3_ROOT : 0u);
#pragma unroll
            for (int q = 0; q < 8; ++q) x[q] = lc[0][q];
        }
        // merge the tasks of each chunk (runs of 2^c lanes, or the 64 lanes of a group)
        if constexpr (MQ && COOP) {
            if (dmax > 1) merge_quads(stage_ptr, lane, dmax, act, km, mm, root, x);
        } else {
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
            if (d < dmax) {                                      // uniform
                uint32_t r[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) r[q] = (uint32_t)__shfl_down((int)x[q], d);
                if (act && (km & (2 * d - 1)) == 0 && km + d < mm)
                    parent(x, r, (root && mm <= 2 * d) ? B3_ROOT : 0u);
            }
        }
        }
        if (act && km == 0) {
            *(uint4 *)dst = make_uint4(x[0], x[1], x[2], x[3]);
            *(uint4 *)(dst + 4) = make_uint4(x[4], x[5], x[6], x[7]);
        }
    }
}

// ---------------------------------------------------------------------------
// One wave per multi-item chunk: merge its item CVs (batches of 64 aligned
// nodes are complete subtrees; results are written back in place).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void b3_tree_kernel(Tables T, HashTables H) {
    const int lane = threadIdx.x & 63;
    const uint64_t ntrees = min(H.ctr[B3C_TREES], H.trees_cap);
    for (uint64_t w = blockIdx.x * 4ull + (threadIdx.x >> 6); w < ntrees; w += gridDim.x * 4ull) {
        const ulonglong2 e = H.trees[w];
        const uint64_t slot = e.x;
        const bool small = e.y == ~0ull;                 // a split packed chunk: pieces only
        uint32_t n = small ? 1u : (chunk_tasks(T.cuts[slot].len, H.lpl_log) + 63) / 64;
        const uint64_t tp = H.tpieces[w];
        const uint32_t np = (uint32_t)(tp & 0xffu);
        if (np) {
            // fold the pieces right to left (each left piece is a complete left
            // subtree of the rest): the unit's CV, or the chunk's hash
            const uint64_t pb = tp >> 8;
            uint32_t x[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) x[q] = H.pcv[(pb + np - 1) * 8 + q];
            for (int p = (int)np - 2; p >= 0; --p) {
                uint32_t l[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) l[q] = H.pcv[(pb + (uint32_t)p) * 8 + q];
                parent(l, x, (small && p == 0) ? B3_ROOT : 0u);
#pragma unroll
                for (int q = 0; q < 8; ++q) x[q] = l[q];
            }
            if (lane == 0) {
                uint32_t *dst = small ? H.hashes + slot * 8 : H.gcv + (e.y + n - 1) * 8;   // the tail's item
                *(uint4 *)dst = make_uint4(x[0], x[1], x[2], x[3]);
                *(uint4 *)(dst + 4) = make_uint4(x[4], x[5], x[6], x[7]);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");   // the tail CV is read below
        }
        if (small) continue;
        uint32_t *nodes = H.gcv + e.y * 8;
        while (n > 1) {
            const uint32_t nb = (n + 63) / 64;
            for (uint32_t b = 0; b < nb; ++b) {
                const uint32_t k = b * 64 + (uint32_t)lane;
                uint32_t x[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                if (k < n) {
                    const uint4 a = *(const uint4 *)(nodes + k * 8);
                    const uint4 c = *(const uint4 *)(nodes + k * 8 + 4);
                    x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
                    x[4] = c.x; x[5] = c.y; x[6] = c.z; x[7] = c.w;
                }
                wave_merge(x, min(64u, n - b * 64), n <= 64, lane);
                // reads of this batch before the in-place write (one wave: CU-local ordering)
                if (n > 64) __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
                if (lane == 0) {
                    uint32_t *dst = n <= 64 ? H.hashes + slot * 8 : nodes + b * 8;
                    *(uint4 *)dst = make_uint4(x[0], x[1], x[2], x[3]);
                    *(uint4 *)(dst + 4) = make_uint4(x[4], x[5], x[6], x[7]);
                }
            }
            if (n > 64) __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");   // level visible to the wave
            n = nb;
        }
    }
}

template <bool NT, int ABLATE, int LD, bool MQ, uint32_t LPL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void b3_leaf_kernel(const uint8_t *__restrict__ data, Tables T, HashTables H) {
    b3_leaf_body<NT, ABLATE, LD, MQ, LPL>(data, T, H);
}

// The persistent grid: every resident slot, but no more blocks (4 waves each)
// than the launch can have wave items.  That bound is known on the host before
// the item planner runs -- group items <= items_cap, and every packed class
// list holds at most packed_cap entries, a chunk giving at most 7 (a whole unit,
// or the binary pieces of its task count) -- and on a small batch it keeps the
// 4096 waves of a full grid from each probing the work counters on their way
// out (~0.1 ms for a one-file batch: the per-file call site, round 6).
static uint32_t leaf_blocks(int device, const void *kernel, const HashTables &ht) {
    int cus = 0, per = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0)
        cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, 256, 0) != hipSuccess || per <= 0) per = 1;
    const uint64_t max_items = ht.items_cap + 7ull * ht.packed_cap + (uint64_t)B3_CLASSES;
    return (uint32_t)std::max<uint64_t>(1ull, std::min<uint64_t>((uint64_t)cus * (uint64_t)per, (max_items + 3) / 4));
}

template <bool NT, int AB, int CO, bool MQ = false, uint32_t LPL = B3_LANE_LEAVES>
static void launch_leaf(int device, const uint8_t *d, const Tables &t, const HashTables &ht, hipStream_t s) {
    const uint32_t blocks = leaf_blocks(device, (const void *)&b3_leaf_kernel<NT, AB, CO, MQ, LPL>, ht);
    hipLaunchKernelGGL((b3_leaf_kernel<NT, AB, CO, MQ, LPL>), dim3(blocks), dim3(256), 0, s, d, t, ht);
}

#ifdef SYNCR_CDC_DEV
// development library only: per-lane loads, non-temporal loads and the
// timing-only ablations (loads only / no loads), selected by SYNCR_B3_* variables
// (with 4-leaf lane tasks: the host plans those variants with lpl_log 2)
template <int CO, bool MQ = false>
static hipError_t launch_leaf_v(int device, const uint8_t *d, const Tables &t, const HashTables &ht, hipStream_t s) {
    if (ht.lpl_log != 2) return hipErrorInvalidValue;
    switch (ht.ablate * 2 + (ht.nt ? 1 : 0)) {
        case 0: launch_leaf<false, 0, CO, MQ>(device, d, t, ht, s); break;
        case 1: launch_leaf<true, 0, CO, MQ>(device, d, t, ht, s); break;
        case 2: launch_leaf<false, 1, CO, MQ>(device, d, t, ht, s); break;
        case 3: launch_leaf<true, 1, CO, MQ>(device, d, t, ht, s); break;
        case 4: case 5: launch_leaf<true, 2, CO, MQ>(device, d, t, ht, s); break;
        default: return hipErrorInvalidValue;
    }
    return hipSuccess;
}
#endif

hipError_t launch_hash(int device, const uint8_t *d, const Tables &t, const HashTables &ht, hipStream_t s) {
    hipError_t e = hipSuccess;
    if (!t.hzero) e = hipMemsetAsync(ht.ctr, 0, B3_CTR_BYTES, s);   // else: the resolve zeroed them
    if (e != hipSuccess) return e;
    if (!t.nfiles) return hipSuccess;
    hipLaunchKernelGGL(b3_items_kernel, dim3(ht.n_iblocks), dim3(256), 0, s, t, ht);
#ifdef SYNCR_CDC_DEV
    if (ht.coop == 3 && !ht.ablate && !ht.nt && ht.lpl_log == 0) launch_leaf<false, 0, LD_PAIR, true, 1>(device, d, t, ht, s);
    else e = ht.coop == 3   ? launch_leaf_v<LD_PAIR, true>(device, d, t, ht, s)
        : ht.coop == 2 ? launch_leaf_v<LD_PAIR>(device, d, t, ht, s)
        : ht.coop == 1 ? launch_leaf_v<LD_COOP64>(device, d, t, ht, s)
                       : launch_leaf_v<LD_PLAIN>(device, d, t, ht, s);
    if (e != hipSuccess) return e;
#else
    // the one exact product instance: two blocks per loader round (zipf10k, same
    // process: leaf HBM reads 1.34x -> 1.255x of the input, time within 0.5 %)
    // and quad-parallel cross-lane merges (leaf 4.157 -> 4.068 ms, same process);
    // 1-leaf lane tasks on a small launch (cdc_internal.h, B3_SMALL_SPAN)
    if (ht.lpl_log == 0) launch_leaf<false, 0, LD_PAIR, true, 1>(device, d, t, ht, s);
    else launch_leaf<false, 0, LD_PAIR, true, B3_LANE_LEAVES>(device, d, t, ht, s);
#endif
    const uint64_t want = (ht.trees_cap + 3) / 4;
    const uint32_t blocks = (uint32_t)(want < 4096 ? (want ? want : 1) : 4096);
    hipLaunchKernelGGL(b3_tree_kernel, dim3(blocks), dim3(256), 0, s, t, ht);
    return hipGetLastError();
}

}  // namespace cdc
