// Internal layout shared by the HIP kernels (cdc_kernels.hip) and the C ABI
// (cdc_api.cpp).  Not part of the public interface (include/syncr_cdc.h).
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

namespace cdc {

// ---- scan geometry (see DESIGN.md "Scan kernel") -------------------------
// A wave owns one tile of RUNS runs x RUN bytes; lane l rolls runs l and l+64
// as the two 16-bit halves of packed registers.  RUN/16 is odd so the
// per-lane ds_read_b128 of a run is bank-conflict free.
constexpr int RUN = 144;                 // bytes rolled per (lane, half)
constexpr int RUNS = 128;                // runs per wave tile
constexpr int TILE = RUN * RUNS;         // 18432 bytes per wave tile
constexpr int HALO = 64;                 // window warm-up bytes before the tile
constexpr int WAVES = 4;                 // waves (tiles) per 256-thread block
constexpr int LISTCAP = 64;              // candidate slots per tile
constexpr int LDS_WAVE = HALO + TILE + LISTCAP * 4 + 16;   // 18768 B, 16-aligned
constexpr int LDS_BLOCK = LDS_WAVE * WAVES;                // 75072 B -> 2 blocks/CU
constexpr uint32_t DENSE_BIT = 0x80000000u;
constexpr int DENSE_WORDS = TILE / 32;   // bitmap words per dense tile (576)
constexpr int DENSE_LANE_BYTES = TILE / 64;  // 288 positions per lane in the dense pass
constexpr uint64_t NONE = ~0ull;

// ctr[] words (zeroed by the per-launch memset)
enum { CTR_DENSE = 0, CTR_FLAGS = 1, CTR_CANDS = 2, CTR_PAD = 3 };
enum { FLAG_DENSE_OVERFLOW = 1u, FLAG_CUT_OVERFLOW = 2u };

struct KParams {
    uint32_t bits;     // chunk_bits
    uint32_t mask;     // (1<<bits)-1
    uint32_t m1;       // s1 mask for bits>16 (0 otherwise)
    uint32_t kk;       // packed (k,k), k = 2^(16-min(bits,16))
    uint32_t kmv;      // packed (-64k mod 2^16) x2
    uint32_t k;        // scalar k
    uint64_t max_chunk;
    uint64_t read_cap; // 0 = unlimited (ideal semantics)
};

struct DevCut {        // == syncr_cut
    uint64_t offset;
    uint32_t len;
    uint32_t file;
};

struct Tables {
    uint64_t span;                 // bytes [0, span) of d_bytes are addressable
    uint32_t ntiles;
    uint32_t nstarts;              // non-empty files (sorted starts)
    const uint64_t *fstart;        // [nstarts] sorted file starts
    const uint2 *tile_range;       // [ntiles] {lo, hi} into fstart: starts in [t0-63, t0+TILE)
    uint32_t nfiles;
    const uint64_t *foff, *flen;   // [nfiles] file table (caller order)
    const uint32_t *order;         // [nfiles] resolve order (largest first)
    const uint64_t *cut_base;      // [nfiles] first output slot per file
    const uint32_t *cut_cap;       // [nfiles] output slots per file
    uint32_t *tile_meta;           // [ntiles] count or DENSE_BIT|pool index (valid iff nonempty bit)
    uint2 *slots;                  // [ntiles*LISTCAP] {tile-relative pos, head fix-up}
    unsigned long long *nonempty;  // [ceil(ntiles/64)] tile has >=1 candidate
    uint32_t *ctr;                 // [4]
    uint32_t *dense_list;          // [dense_cap] tile ids
    uint32_t dense_cap;
    uint32_t *dense_bits;          // [dense_cap*DENSE_WORDS] candidate bitmaps
    DevCut *cuts;                  // [sum cut_cap]
    uint64_t *counts;              // [nfiles]
};

// launchers (cdc_kernels.hip)
hipError_t launch_scan(const uint8_t *d_bytes, const KParams &p, const Tables &t, hipStream_t s);
hipError_t launch_dense(const uint8_t *d_bytes, const KParams &p, const Tables &t, hipStream_t s);
hipError_t launch_resolve(const uint8_t *d_bytes, const KParams &p, const Tables &t, hipStream_t s);
hipError_t launch_gen(uint8_t *d_base, const uint64_t *d_foff, const uint64_t *d_flen,
                      const uint64_t *d_findex, const uint64_t *d_seg_prefix, uint32_t nfiles,
                      uint64_t nseg, uint64_t first_index, const uint64_t *d_jump, hipStream_t s);
constexpr int GEN_SEG = 4096;     // bytes generated per thread
constexpr int GEN_JUMPS = 48;     // xorshift jump matrices M^(2^k), k < 48

}  // namespace cdc
