// Internal layout shared by the HIP kernels (cdc_kernels.hip) and the C ABI
// (cdc_api.cpp).  Not part of the public interface (include/syncr_cdc.h).
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

namespace cdc {

// ---- scan geometry (see DESIGN.md "Scan kernel") -------------------------
// A wave owns a tile of RUNS runs x RUN bytes; lane l rolls runs l and l+64 as
// the two 16-bit halves of packed registers.  RUN/16 is odd so that the
// per-lane ds_read_b128 of a run is bank-conflict free.  RUN is a template
// parameter of the scan kernel (tuned on MI355X).
constexpr int RUNS = 128;                // runs per wave tile
constexpr int HALO = 64;                 // window warm-up bytes before the tile
constexpr int LISTCAP = 64;              // candidate slots per tile
constexpr uint32_t DENSE_BIT = 0x80000000u;
// dense pass with fused head fix-ups (cdc_dense_packed_kernel<RUN, true>): up to
// FIXCAP fix-ups per dense tile, by candidate rank, in Tables::dense_fix (and the
// candidates' positions in Tables::dense_pos: no bitmap); a tile whose fix-ups are
// there has DENSE_FIXED in its dense_cnt word.  The LDS
// buffer holds DENSE_TAIL bytes past the tile (the last candidates' windows).
constexpr uint32_t FIXCAP = 1024;
constexpr uint32_t FIX_RMAX = 6;
constexpr uint32_t DENSE_FIXED = 0x80000000u;
constexpr int DENSE_TAIL = 80;
// Tables::coarse keeps one counter per 128-byte line: the waves of a launch
// work through a window of nearby tiles, so their atomics meet on a few
// counters, and counters sharing a line serialise in one L2 channel.
constexpr uint32_t COARSE_STRIDE = 32;
constexpr uint64_t NONE = ~0ull;
// Work counters zeroed per launch, one per 128-byte line (Tables::sched):
// SCHED_SCAN_GROUP is the CU scan schedule's group counter, SCHED_DENSE_CHUNK
// the dense pass's list-chunk counter.
constexpr uint32_t SCHED_REGIONS = 4;
enum { SCHED_SCAN_GROUP = 0, SCHED_DENSE_CHUNK = 1 };
constexpr int DEFAULT_RUN = 144;

// MFMA scan (cdc_scan_mfma_kernel): a wave tile is 32 streams x NB blocks of
// 32 bytes; W for a 32-position block is a Toeplitz product of the block and
// its two predecessors (three v_mfma_i32_32x32x32_i8).
constexpr int MF_STREAMS = 32;
constexpr int DEFAULT_NB = 10;
__host__ __device__ constexpr int mf_tile_bytes(int nb) { return 1024 * nb; }
__host__ __device__ constexpr int mf_buf_bytes(int nb) { return HALO + 1024 * nb; }
// landing buffers (2: tile t+1 in flight while tile t is filtered; 1: the
// buffer is recycled as soon as the tile is in registers) + candidate list
__host__ __device__ constexpr int mf_lds_bytes(int nb, int nbuf) { return nbuf * mf_buf_bytes(nb) + LISTCAP * 4 + 16; }

// Scan geometry: kind 0 = packed-u16 VALU roll (param = RUN bytes per lane
// run), kind 1 = MFMA Toeplitz filter (param = NB blocks per stream).
enum { SCAN_VALU = 0, SCAN_MFMA = 1 };
enum { MFV_SINGLE = 1, MFV_NOPIPE = 2 };   // MFMA scan variants (ScanGeom::var)
struct ScanGeom {
    int kind;
    int param;
    int var;     // MFMA: MFV_* bits
};

__host__ __device__ constexpr int tile_bytes(int run) { return run * RUNS; }
__host__ __device__ constexpr int buf_bytes(int run) { return HALO + run * RUNS; }
__host__ __device__ constexpr int dense_buf_bytes(int run, bool fuse) { return buf_bytes(run) + (fuse ? DENSE_TAIL : 0); }
// LDS per wave: one tile landing buffer + 16 dirty-group slots (80 B) +
// candidate list + counters
__host__ __device__ constexpr int lds_wave_bytes(int run) { return buf_bytes(run) + 16 * 80 + LISTCAP * 4 + 16; }
// Three-waves-per-SIMD scan (cdc_scan3_kernel, RUN = W3_RUN): the landing
// buffer + DIRTYCAP3 dirty-group positions (their bytes are re-read from HBM,
// not kept in LDS) + candidate list + counters.  12 waves x 12 880 B <= 160 KiB.
constexpr int W3_RUN = 96;
constexpr int DIRTYCAP3 = 64;
__host__ __device__ constexpr bool run_is_w3(int run) { return run == W3_RUN; }
__host__ __device__ constexpr int lds3_wave_bytes(int run) { return buf_bytes(run) + DIRTYCAP3 * 4 + LISTCAP * 4 + 16; }
__host__ __device__ constexpr int scan_lds_for_run(int run) {
    return run_is_w3(run) ? lds3_wave_bytes(run) : lds_wave_bytes(run);
}

// ---- stream-tile scan (cdc_scan_st_kernel) --------------------------------
// A stream tile (ST) is ST_TILES consecutive batch tiles cut into 128 streams
// of ST_SEGS segments (st_segs(); 18 / 27 / 36 in the dev library), handed out
// whole from a counter.  (Round 5 measured handing the
// batch's last round out in segment-range parts, to end the waves closer
// together, and a raised issue priority for the last round's late waves: both
// null or slower -- DESIGN.md §4.1 -- and removed, with the extra branches and
// runtime loop bounds they put in the hot loop.)
constexpr int ST_TILES = 8;                   // batch tiles per ST
constexpr int ST_SEGS = 9;                    // segments per stream

// ctr[] words (zeroed by the per-launch memset)
enum { CTR_DENSE = 0, CTR_FLAGS = 1, CTR_CANDS_LO = 2, CTR_CANDS_HI = 3 };
// FLAG_SCHED_STUCK: a scan wave gave up waiting (~1 s) for its CU's next group
// id -- cannot happen by construction; fetch reports SYNCR_CDC_EIO if it does
enum { FLAG_DENSE_OVERFLOW = 1u, FLAG_CUT_OVERFLOW = 2u, FLAG_CAND_OVERFLOW = 4u, FLAG_SCHED_STUCK = 8u };

// compacted candidate: bits 0..47 global position, 48..55 head fix-up (0..63),
// bit 63 = fix-up known
constexpr uint64_t CAND_POS_MASK = (1ull << 48) - 1;
constexpr uint64_t CAND_KNOWN = 1ull << 63;
// chain link (cdc_fix_kernel): a cut at this candidate, with the reference's
// buffer full, implies a cut at the next candidate -- its head fix-up is empty
// and the next candidate lies 64 .. min(MAX, read_cap) bytes past it (one file
// or not: the resolve bounds runs by its file).  Tables::linkw holds the same
// bits 64 candidates per word.
constexpr uint64_t CAND_LINK = 1ull << 62;
// the word's CAND_LINK bit is final (set with it by the compaction for a dense
// tile's candidates but its last, whose next candidate lies in another tile):
// cdc_fix_kernel neither recomputes nor rewrites such a complete word
constexpr uint64_t CAND_LDEC = 1ull << 61;

struct KParams {
    uint32_t bits;     // chunk_bits
    uint32_t mask;     // (1<<bits)-1
    uint32_t m1;       // s1 mask for bits>16 (0 otherwise)
    uint32_t kk;       // packed (k,k), k = 2^(16-min(bits,16))
    uint32_t kmv;      // packed (-64k mod 2^16) x2
    uint32_t k;        // scalar k
    uint64_t max_chunk;
    uint64_t read_cap; // 0 = unlimited (ideal semantics)
    uint32_t ablate;   // development library only (SYNCR_CDC_ABLATE): scan variants / timing-only ablations
    uint32_t nt;       // 1: non-temporal tile loads (SYNCR_CDC_NT=1)
    uint32_t resolve_lane;  // 1: lane-per-file resolve (SYNCR_CDC_FLAG_RESOLVE_LANE); 0: wave-per-file
    uint32_t resolve_noburst;  // 1: no burst of chained hops in the wave resolve (SYNCR_CDC_FLAG_RESOLVE_NOBURST)
    uint32_t resolve_nosplit;  // 1: no split walks of long files (SYNCR_CDC_FLAG_RESOLVE_NOSPLIT)
    uint64_t split_patience;   // wall-clock ticks a split worker waits for file walkers (0: none,
                               //   SYNCR_CDC_FLAG_SPLIT_NOWAIT)
    uint32_t split_first;      // 1: split workers take the resolve grid's first blocks (dev A/B: SYNCR_CDC_SPLIT_FIRST)
    uint32_t no_skip;          // 1: no run skips in the resolve walk (dev A/B: SYNCR_CDC_NOSKIP)
    uint32_t scan_tiles;       // 1: the last fetched launch of the handle was dense-heavy: scan by tiles
                               //   (dynamic groups) instead of stream tiles (cdc_kernels.hip launch_scan)
    uint32_t dense_fuse;       // 1: the dense pass computes its candidates' head fix-ups (product; dev A/B:
                               //   SYNCR_CDC_DENSE_FUSE=0)
    uint32_t resolve_pf;       // development library only (SYNCR_CDC_RESOLVE_PF): candidate windows
                               //   the resolve walk loads ahead (0: RESOLVE_PF)
    uint32_t st_segs;          // (dev A/B: SYNCR_CDC_ST_SEGS) 9 / 18 / 27 / 36 segments per stream forced; 0: st_segs()
    uint32_t nt_out;           // 1: candidate words and cuts are stored non-temporally (dev A/B:
                               //   SYNCR_CDC_NT_OUT=1; product 0); Tables::nt_out carries it to the kernels
    uint32_t dense_blocks;     // (dev A/B: SYNCR_CDC_DENSE_BLOCKS) dense-pass grid forced; 0: the product's
};
constexpr int RESOLVE_PF = 8;  // product: candidate windows in the resolve walk's LDS ring (PF-1 ahead)

// ---- split walks of long files (wave resolve) -------------
// A file whose walk would be long (>= 2 SPLIT_SEGC candidates) is cut into
// segments of SPLIT_SEGC candidates.  Segment k >= 1 is walked speculatively by
// an extra resolve wave from the state "a cut at its first candidate c, buffer
// full": s = c + 1, R = min(F, s + MAX).  A walk whose own cut lands on
// segment b's start with exactly that R continues identically to segment b's
// walk (the walk's future is a function of (s, R) only), so the file's walker
// adopts segment b's cuts and jumps to where that walk linked in turn.
constexpr uint32_t SPLIT_SEGC = 8192;                   // candidates per segment (default; Tables::seg_segc; 4096 before run skips)
__host__ __device__ constexpr uint32_t split_scap(uint32_t segc) { return 3 * segc + 64; }   // scratch cuts per walk
constexpr uint64_t SPLIT_MIN_BYTES = 256ull << 10;       // smaller files never split
constexpr uint32_t SPLIT_BLOCKS = 256;                  // extra resolve blocks (4 waves each; default)
constexpr uint32_t SPLIT_END = 0xffffffffu;             // SplitSeg::link: walked to the file end
constexpr uint32_t SPLIT_ABORT = 0xfffffffeu;           // (segment walk state: gave up)
// split[] words: a 64-bit count (split files << 32 | eligible walkers
// published), so one relaxed read gives both; segment records reserved;
// queue head; split walkers done; worker give-ups; segments walked by workers;
// segments adopted by file walkers; deferred runs; dense tiles the dense pass
// rolled (ctr[CTR_DENSE] counts list slots: the product's deferred DensePend
// slots leave no holes; only the dev library's DenseSlots scans pad 8-slot
// chunks with DENSE_HOLE)
enum { SPL_PUB64 = 0, SPL_RESERVED = 2, SPL_HEAD = 3, SPL_DONE = 4, SPL_GIVEUP = 5, SPL_WALKED = 6,
       SPL_ADOPTED = 7, SPL_RUNS = 8, SPL_DENSE_TILES = 9, SPL_WORDS = 10 };
struct SplitSeg {            // 64 bytes
    uint64_t cidx;           // candidate index of the segment's first candidate
    uint64_t out_off;        // adopted: first cut slot within the file's output
    uint32_t file;           // file index
    uint32_t k;              // boundary number within the file (>= 1); 0: unusable record
    uint32_t s0, R0;         // walk state at the segment start
    uint32_t first, nseg;    // record of the file's boundary 1; the file's segment count
    uint64_t res;            // the walk's result in one word (seg_res): cuts n, link, status --
                             //   one atomic load gives a file walker all it needs of a record
    uint32_t verdict;        // 1: adopted by the file's walker
    uint32_t ready;          // == Tables::epoch: initialised in this launch (release)
    uint32_t run_pre, run_len;   // the walk's deferred run (RunJob): its cuts sit after run_pre
                                 //   scratch cuts; run_len 0 = none
};
// A run of chained cuts the resolve walk deferred to the copy launch (cuts at
// candidates a .. a+n-1, each starting after the previous candidate): the walk
// only counts them.  rec == SPLIT_END: `out` is the absolute output slot of the
// first; else `out` is the slot within segment walk `rec`'s cuts, placed when a
// file walker adopts that walk.
struct RunJob {
    uint64_t out;
    uint64_t a;
    uint32_t n, file, rec, pad;
};
enum { SEG_PENDING = 0, SEG_DONE = 1, SEG_ABORTED = 2, SEG_WALKING = 3 };
// res = n << 32 | link (30 bits; SPLIT_END / SPLIT_ABORT keep their low 30) << 2 | status
__host__ __device__ constexpr uint64_t seg_res(uint32_t status, uint32_t link, uint32_t n) {
    return ((uint64_t)n << 32) | ((uint64_t)(link & 0x3fffffffu) << 2) | (uint64_t)status;
}
__host__ __device__ constexpr uint32_t seg_res_status(uint64_t r) { return (uint32_t)r & 3u; }
__host__ __device__ constexpr uint32_t seg_res_n(uint64_t r) { return (uint32_t)(r >> 32); }
__host__ __device__ constexpr uint32_t seg_res_link(uint64_t r) {
    return ((uint32_t)(r >> 2) & 0x3fffffffu) >= 0x3ffffffeu ? ((uint32_t)(r >> 2) | 0xc0000000u)
                                                             : ((uint32_t)(r >> 2) & 0x3fffffffu);
}
static_assert(sizeof(SplitSeg) == 64, "SplitSeg is one 64-byte record");

struct DevCut {        // == syncr_cut
    uint64_t offset;
    uint32_t len;
    uint32_t file;
};

struct Tables {
    uint64_t span;                 // bytes [0, span) of d_bytes are addressable
    uint32_t ntiles;
    uint32_t tile;                 // bytes per tile (scan_tile_bytes)
    uint32_t nwords;               // ceil(ntiles / 64)
    uint32_t nstarts;              // non-empty files (sorted starts)
    const uint64_t *fstart;        // [nstarts] sorted file starts
    uint32_t nfiles;
    const uint64_t *foff, *flen;   // [nfiles] file table (caller order)
    const uint32_t *order;         // [nfiles] resolve order (largest first)
    const ulonglong2 *ofile;       // [nfiles] {foff, flen} of order[k], in resolve order (read beside
                                   //   order[k]: one dependent load less at every file walker's start)
    const uint64_t *cut_base;      // [nfiles] first output slot per file
    const uint32_t *cut_cap;       // [nfiles] output slots per file
    uint32_t *tile_meta;           // [ntiles] count or DENSE_BIT|pool index (valid iff nonempty bit)
    uint2 *slots;                  // [ntiles*LISTCAP] {tile-relative pos, head fix-up}
    unsigned long long *nonempty;  // [nwords] tile has >=1 candidate        (zeroed per launch)
    uint32_t *super_cnt;           // [nwords] candidates per 64-tile group   (zeroed per launch)
    uint32_t *coarse;              // [ncoarse * COARSE_STRIDE] candidates per 64 groups (4096 tiles),
                                   // one counter per 128-byte line (zeroed per launch)
    uint32_t ncoarse;
    uint64_t *super_off;           // [nwords+1] exclusive prefix of super_cnt (written by the gather)
    uint32_t *ctr;                 // [4]                                      (zeroed per launch)
    uint32_t *dense_list;          // [dense_cap] tile ids
    uint32_t *dense_cnt;           // [dense_cap] candidates per dense tile
    uint32_t dense_cap;
    uint32_t *dense_bits;          // [dense_cap * tile/32] candidate bitmaps
    uint8_t *dense_fix;            // [dense_cap * FIXCAP] head fix-ups of dense tiles' candidates, by rank
    uint16_t *dense_pos;           // [dense_cap * FIXCAP] their tile-relative positions (DENSE_FIXED tiles)
    uint64_t *cand;                // [cand_cap] compacted sorted candidates
    uint64_t *linkw;               // [cand_cap / 64 + 4] CAND_LINK bits, 64 candidates per word (cdc_fix_kernel)
    uint64_t cand_cap;
    DevCut *cuts;                  // [sum cut_cap]
    uint64_t *counts;              // [nfiles]
    // read-boundary grid (production semantics): while the reference's buffer
    // is not saturated its reads end at multiples of read_cap from the file
    // start, so cuts forced there start chunks at those offsets; their head
    // hits are precomputed by cdc_fix_kernel instead of rolled by the resolve
    uint32_t ngrid;
    const uint64_t *gpos;          // [ngrid] batch offset of grid point (file start + k * read_cap)
    const uint64_t *gend;          // [ngrid] batch offset of that file's end
    uint8_t *gfix;                 // [ngrid] first chunk-local hit in [p, p+63): offset + 1, 0 = none
    const uint64_t *gbase;         // [nfiles] first grid index of each file
    // split walks of long files
    uint32_t n_elig;               // order[0 .. n_elig): files of >= SPLIT_MIN_BYTES (largest first)
    uint32_t seg_cap;              // SplitSeg records
    SplitSeg *segs;                // [seg_cap]
    DevCut *seg_cuts;              // [seg_cap * seg_scap]
    uint32_t seg_segc, seg_scap;   // candidates per segment, scratch cuts per segment walk
    uint32_t split_blocks;         // extra resolve blocks (split workers)
    uint32_t *split;               // [SPL_WORDS] counters                    (zeroed per launch)
    uint32_t dense_off;            // 1: no dense pass this launch (the handle has not seen a dense tile);
                                   //   the compaction counts dense tiles as empty and fetch re-runs if any
    uint32_t *sched;               // [SCHED_REGIONS * COARSE_STRIDE] work counters (SCHED_*), one per
                                   //   128-byte line (zeroed per launch)
    RunJob *runs;                  // [runs_cap] deferred runs (only while split workers run)
    uint32_t runs_cap;
    uint32_t epoch;                // this launch's id (!= 0, unique in the process): SplitSeg::ready
    // The per-launch counters above (ctr, nonempty, super_cnt, split) live in one
    // of two zeroed blocks, alternating by launch.  The resolve kernel zeroes the
    // OTHER block for the next launch (and the hash counters of this launch),
    // so a step needs no memset packet (cdc_api.cpp do_launch).
    uint4 *znext;                  // [znext_vec] the next launch's block (nullptr: none)
    uint32_t znext_vec;
    uint64_t *hzero;               // [B3C_WORDS] + shards: hash counters of this launch (hashed launches), or nullptr
    uint64_t *dbg;                 // development library only (SYNCR_CDC_TRACE=1): [DBG_WORDS] resolve
                                   //   timeline (wall_clock64 stamps, DBG_*), else nullptr
    uint32_t nst;                  // stream-tile scan: STs of the batch (launch geometry)
    uint32_t nt_out;               // KParams::nt_out: non-temporal stores of candidate words and cuts
    uint64_t gapmax;               // chain links: the next candidate at most min(MAX, read_cap) past
    // scan timing by the device clock (syncr_cdc_set_timing mode 4; null: off): the scan's
    // waves stamp wall_clock64 -- tscan[0] = ~0 - the earliest entry, tscan[1] = the
    // latest exit (atomic max, zeroed per launch) -- and the resolve adds exit - entry
    // to tacc[0] and 1 to tacc[1] (the handle's running sums).  No queue packets.
    uint64_t *tscan;
    uint64_t *tacc;
};
// dev timeline slots: resolve entry (min over waves), end (max); the largest
// split file's walker: entry, after split setup, adoption blocks (start, end),
// walk end; split workers: record q < DBG_NREC walk start / end; copy kernel
// scan timeline: per scan wave (block) w < DBG_SCAN_N: entry, first tile landed,
// exit, tiles rolled (DBG_SCAN + 4 w ...); per-tile ends of waves < DBG_TILE_W
// (DBG_TILE + DBG_TILE_N w + k, k-th tile)
enum { DBG_RES_START = 0, DBG_RES_END = 1, DBG_W_ENTRY = 2, DBG_W_SETUP = 3, DBG_W_END = 4, DBG_W_NBLK = 5,
       DBG_W_BLK = 8, DBG_MAXBLK = 120, DBG_COPY_START = 248, DBG_COPY_END = 249, DBG_REC = 256,
       DBG_NREC = 1024, DBG_FW = DBG_REC + 2 * DBG_NREC, DBG_NFW = 1024, DBG_SCAN = DBG_FW + DBG_NFW,
       DBG_SCAN_N = 4096, DBG_TILE = DBG_SCAN + 4 * DBG_SCAN_N, DBG_TILE_W = 16, DBG_TILE_N = 128,
       DBG_CW = DBG_TILE + DBG_TILE_W * DBG_TILE_N, DBG_NCW = 4096,   // split copy waves: end, start
       DBG_DW = DBG_CW + 2 * DBG_NCW, DBG_NDW = 2048,                  // dense-pass waves: entry, end | tiles << 56
       DBG_DT = DBG_DW + 2 * DBG_NDW, DBG_DT_W = 16, DBG_DT_N = 16,    // their first tiles: issue, landed, rolled, fixed
       DBG_WORDS = DBG_DT + 4 * DBG_DT_W * DBG_DT_N };

// ---- BLAKE3 of every chunk (b3_kernels.hip) -------------------------------
// A lane TASK is LPL consecutive 1 KiB leaves of one chunk: LPL = B3_LANE_LEAVES
// on a big launch, 1 on a launch of at most B3_SMALL_SPAN bytes whose max_chunk
// is at most 64 MiB (a lane's leaves
// are compressed in sequence, 16 blocks each: a 4-leaf task is ~80 us of one
// wave, so on a small batch -- one file of the per-file call site, an 8 KiB
// file included -- the leaf kernel's time is that one task; 1-leaf tasks cut it
// ~4x, and give a small batch 4x the group items to spread over the waves; a
// big launch keeps 4 leaves per lane: a quarter of the cross-lane merges).  A chunk
// of T <= 64 tasks is PACKED: class c = ceil(log2 T), 64 >> c such units per
// wave, each in an aligned run of 2^c lanes.  A chunk of T > 64 tasks (a BIG
// chunk) is floor(T / 64) GROUP items of 64 tasks (one wave each) plus, when
// T % 64 != 0, a TAIL unit of the last T % 64 tasks packed like a small chunk;
// b3_tree_kernel merges the items' and the tail's subtree CVs.  A unit whose
// task count r is not a power of two (a small chunk or a tail) is split into
// PIECES by the binary digits of r, largest first -- exactly the subtrees of
// BLAKE3's left-balanced tree -- so each piece fills its 2^c lanes; the tree
// kernel folds the piece CVs right to left.
constexpr uint32_t B3_LANE_LEAVES = 4;                      // 1 KiB leaves per lane task (big launches)
constexpr uint64_t B3_SMALL_SPAN = 1ull << 30;              // launches up to this many bytes: 1 leaf per task
constexpr int B3_CLASSES = 7;                               // packed classes: <= 1, 2, 4, ..., 64 tasks
constexpr uint64_t B3_TAIL = 1ull << 63;                  // packed entry: tail unit
constexpr uint64_t B3_PIECE = 1ull << 62;                 // packed entry: piece (index into pieces[])
constexpr uint32_t B3_MAX_PIECES = 7;                     // popcount of a task count <= 127
constexpr uint64_t B3_ITEMS_CUTS = 2048;                  // output slots per b3_items_kernel block (dense1: 1024 blocks)
enum { B3C_ITEMS = 0, B3C_TREES = 1, B3C_NEXT = 2, B3C_FLAGS = 3, B3C_PK0 = 4, B3C_PIECES = 4 + B3_CLASSES,
       B3C_WORDS = 5 + B3_CLASSES };
// The leaf kernel's work counters: B3_SHARDS of them, 4 KiB apart (different
// memory channels: each takes its own atomics), after the B3C_WORDS counters in
// the same buffer: shard k at ctr[(k + 1) * B3_SHARD_STRIDE].  Zeroed with them.
constexpr uint32_t B3_SHARDS = 8, B3_SHARD_STRIDE = 512;
constexpr uint64_t B3_CTR_BYTES = (uint64_t)(B3_SHARDS + 1) * B3_SHARD_STRIDE * 8;

struct HashTables {
    uint64_t *ctr;                 // [B3C_WORDS] + the leaf's shard counters (zeroed per hashed launch)
    uint64_t *items;               // [items_cap] slot << 24 | group (| B3_TAIL: tail placeholder)
    uint64_t items_cap;
    uint64_t *packed;              // [B3_CLASSES * packed_cap] by packed class: a chunk slot, or
    uint64_t packed_cap;           //   B3_TAIL | its placeholder item for a big chunk's tail unit
    ulonglong2 *trees;             // [trees_cap] {slot, first item or ~0} of big and of split chunks
    uint64_t *tpieces;             // [trees_cap] first piece << 8 | pieces (0: none) of each tree
    uint64_t trees_cap;
    ulonglong2 *pieces;            // [pieces_cap] {slot, first task}: a piece's chunk and position
    uint32_t *pcv;                 // [pieces_cap * 8] CV of each piece
    uint64_t pieces_cap;
    uint32_t lpl_log;              // log2 of the leaves per lane task: 2 (B3_LANE_LEAVES) or 0 (small launch)
    uint32_t nosplit;              // dev A/B only (SYNCR_B3_SPLIT=0): one unit per power-of-two class, no pieces
    uint32_t nouni;                // dev A/B only (SYNCR_B3_UNI=0): group items use the per-task loader
    uint32_t *gcv;                 // [items_cap * 8] subtree CV of each item (or tail placeholder)
    uint32_t *hashes;              // [sum cut_cap * 8] BLAKE3 of each cut slot
    uint32_t ablate;               // timing-only (SYNCR_B3_ABLATE): 1 = loads only, 2 = no loads
    uint32_t nt;                   // 1: non-temporal chunk loads (SYNCR_B3_NT)
    const uint64_t *iblocks;       // [n_iblocks] b3_items_kernel blocks: group << 40 | part << 20 | parts
    uint32_t n_iblocks;
    uint32_t coop;                 // 3 (product): cooperative LDS-DMA loader, two blocks per round, quad
                                   //   merges; 2: shuffle merges (SYNCR_B3_LOAD=pair); 1: one block per
                                   //   round (=coop); 0: per-lane loads (=plain)
};

// launchers (cdc_kernels.hip)
bool scan_supported(ScanGeom g);
int scan_tile_bytes(ScanGeom g);
int scan_lds_bytes(ScanGeom g);
int scan_blocks_per_cu(ScanGeom g);
// e0 / e1 (may be null): HIP events recorded on s right before and after the scan kernel
hipError_t launch_scan(ScanGeom g, uint32_t grid, const uint8_t *d_bytes, const KParams &p, const Tables &t,
                       hipStream_t s, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);
bool scan_dense_inline(ScanGeom g, const KParams &p);      // the scan passes dense tiles itself
// Which scan kernel launch_scan runs for this launch (SYNCR_CDC_SCAN_* of include/syncr_cdc.h):
// the one decision, reported through syncr_cdc_last_scan so callers never restate it.
int scan_kind(ScanGeom g, uint32_t grid, const KParams &p, const Tables &t);
int st_segs(uint32_t grid, const KParams &p, const Tables &t);   // stream-tile geometry of a launch
hipError_t launch_post(const uint8_t *d_bytes, const KParams &p, const Tables &t, hipStream_t s, bool dense_inline,
                       uint32_t scan_grid);
hipError_t launch_resolve(const uint8_t *d_bytes, const KParams &p, const Tables &t, hipStream_t s);
bool resolve_splits(const KParams &p, const Tables &t);   // launch_resolve starts split workers
// A small copy group (cdc_api.cpp upload / download) as one dispatch: each
// segment's bytes (a multiple of 4) from src to dst, either side device memory
// or the handle's pinned, device-visible staging.  A hipMemcpyAsync per table is
// one blit dispatch each (~2 us of GPU and ~5 us of API time): a one-file batch
// moved ~20 tables that way per round trip.
constexpr int COPY_MAX = 14;
struct CopySeg {
    const void *src;               // nullptr: zero-fill dst
    void *dst;
    uint64_t bytes;
};
struct CopyList {
    CopySeg seg[COPY_MAX];
    uint32_t n;
};
hipError_t launch_copy(const CopyList &l, uint64_t total_bytes, hipStream_t s);
hipError_t launch_gen(uint8_t *d_base, const uint64_t *d_foff, const uint64_t *d_flen,
                      const uint64_t *d_findex, const uint64_t *d_seg_prefix, uint32_t nfiles,
                      uint64_t nseg, uint64_t first_index, const uint64_t *d_jump, hipStream_t s);
hipError_t launch_read_probe(const uint8_t *d_bytes, uint64_t bytes, bool nt, uint32_t grid, uint32_t *sink,
                             hipStream_t s);
hipError_t launch_hash(int device, const uint8_t *d_bytes, const Tables &t, const HashTables &ht,
                       hipStream_t s);
constexpr int GEN_SEG = 4096;     // bytes generated per thread
constexpr int GEN_JUMPS = 48;     // xorshift jump matrices M^(2^k), k < 48

}  // namespace cdc
