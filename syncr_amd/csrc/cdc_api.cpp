// cdc_api.cpp -- C ABI of the MI355X CDC engine (declared in include/syncr_cdc.h).
//
// Replaces the scan half of compute_file_chunks (reference
// src/protocol/file_operations.rs:721-788): the caller hands over file bytes,
// gets (offset, size) per chunk back.  No C++ exception crosses this boundary.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <map>
#include <mutex>
#include <cstdlib>
#include <cstring>
#include <new>
#include <numeric>
#include <vector>

#include "../../include/syncr_cdc.h"
#include "cdc_internal.h"
#include <cstdio>

using namespace cdc;

namespace {

// A device allocation owned by its holder: released by its destructor, so a
// buffer added to syncr_cdc can never be missed by syncr_cdc_close.
struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() { release(); }
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap && p) return hipSuccess;
        if (p) { (void)hipFree(p); p = nullptr; cap = 0; }
        size_t want = std::max<size_t>(bytes, 256);
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T> T *as() const { return static_cast<T *>(p); }
};

// Pinned host staging for a handle's small table uploads and result
// downloads.  A synchronous hipMemcpy from pageable memory costs ~20 us; a
// one-file batch made ~20 of them (plan's tables, fetch's counters, counts,
// cuts and hashes): ~0.45 ms of a ~0.5 ms per-file round trip (rocprofv3 HIP
// trace of the per-file call site, round 6).  A CopyGroup goes through this
// buffer on the handle's stream and is waited for once: up to KCOPY_MAX bytes as
// one cdc_copy_kernel dispatch that reads (upload) or writes (download) the
// buffer across PCIe -- coherent memory, so nothing of it is cached on the
// device -- else one hipMemcpyAsync per table; groups above STAGE_MAX use plain
// hipMemcpy (large tables and results: the runtime stages those itself, and the
// buffer stays small).
struct HostStage {
    uint8_t *p = nullptr;
    uint8_t *d = nullptr;               // the same memory, as the device addresses it
    size_t cap = 0;
    HostStage() = default;
    HostStage(const HostStage &) = delete;
    HostStage &operator=(const HostStage &) = delete;
    ~HostStage() {
        if (p) (void)hipHostFree(p);
    }
    hipError_t ensure(size_t n) {
        if (n <= cap && p) return hipSuccess;
        const size_t want = std::max<size_t>(n, std::max<size_t>(64u << 10, 2 * cap));
        uint8_t *q = nullptr, *qd = nullptr;
        hipError_t e = hipHostMalloc((void **)&q, want, hipHostMallocCoherent | hipHostMallocPortable);
        if (e != hipSuccess) return e;
        if ((e = hipHostGetDevicePointer((void **)&qd, q, 0)) != hipSuccess) {
            (void)hipHostFree(q);
            return e;
        }
        if (p) (void)hipHostFree(p);
        p = q;
        d = qd;
        cap = want;
        return hipSuccess;
    }
};
constexpr size_t STAGE_MAX = 4u << 20;
constexpr size_t KCOPY_MAX = 256u << 10;

// copies of one group: (device, host, bytes); host buffers stay valid until
// upload() / download() returns.  An upload item without a host side zero-fills
// its device range (no staging).
struct CopyGroup {
    struct Item {
        void *dev;
        void *host;
        size_t n, off;
    };
    std::vector<Item> items;
    size_t total = 0;
    void add(void *dev, const void *host, size_t n) {
        if (!n) return;
        items.push_back({dev, const_cast<void *>(host), n, total});
        total += (n + 15) & ~size_t(15);
    }
    void zero(void *dev, size_t n) {
        if (n) items.push_back({dev, nullptr, n, 0});
    }
};

constexpr int NPHASE = 4;            // scan, dense+compaction, resolve, hash

struct PendingTiming {
    hipEvent_t ev[NPHASE + 1];
    int nev;
};

}  // namespace

struct syncr_cdc {
    int device = 0;
    syncr_cdc_params params{};
    KParams kp{};
    hipStream_t stream = nullptr;
    hipEvent_t scan_done = nullptr;     // recorded after each launch's scan (scan_order)
    bool serial_scans = false;          // order scans of same-device handles (dev lib: SYNCR_CDC_SERIAL=1)
    // scan kernel and tile geometry: the packed-u16 VALU roll (north_star: integer
    // work, no MFMA).  Other geometries and the MFMA Toeplitz variant exist only
    // in the development library.
    ScanGeom geom{SCAN_VALU, DEFAULT_RUN, 0};
    uint32_t scan_grid = 0;         // persistent scan grid (CUs x resident blocks)

    // plan
    bool planned = false;
    uint32_t nfiles = 0, nstarts = 0, ntiles = 0, nwords = 0;
    uint64_t span = 0;
    uint32_t dense_cap = 0;
    uint64_t cand_cap = 0;
    uint64_t total_cut_cap = 0;
    std::vector<uint64_t> h_foff, h_flen, h_cut_base;
    std::vector<uint32_t> h_cut_cap;
    DevBuf fstart, foff, flen, order, ofile, cut_base, cut_cap, tile_meta, slots, zeroed,
        dense_list, dense_cnt, dense_bits, dense_fix, dense_pos, super_off, cand, linkw, cuts, counts;
    // BLAKE3 of every chunk (launch_hashed)
    bool hash_on = false;
    uint32_t b3_lpl_log = 2;           // leaves per lane task of the planned launch (log2; upload_cut_tables)
    uint32_t b3_lpl = 0;               // dev A/B only (SYNCR_B3_LPL=1|4): force it; 0 = by span
    uint32_t b3_ablate = 0, b3_nt = 0, b3_coop = 3, b3_nosplit = 0, b3_nouni = 0;     // dev A/B knobs; coop 3 = the product (LD_PAIR + quad merges)
    uint64_t items_cap = 0, trees_cap = 0;
    DevBuf hctr, items, trees, gcv, hashes, packed, tpieces, pieces, pcv, iblocks;
    uint32_t n_iblocks = 0;
    uint64_t pieces_cap = 0;
    // read-boundary grid (Tables::gpos...): production semantics only
    uint32_t ngrid = 0;
    DevBuf gpos, gend, gfix, gbase;
    // split walks of long files (Tables::segs...): files order[0 .. n_elig) may split
    uint32_t n_elig = 0, seg_cap = 0;
    uint32_t split_segc = SPLIT_SEGC, split_blocks = SPLIT_BLOCKS;   // (development library: SYNCR_CDC_SPLIT_*)
    DevBuf segs, seg_cuts, runs;
    uint32_t runs_cap = 0;
    DevBuf dbg;                         // development library: resolve timeline (SYNCR_CDC_TRACE=1)
    // split only when walks can be long: the last launch fetched held >= 64 Ki
    // candidates at >= 1 per 16 KiB (random data: ~1 per MiB, so never;
    // periodic or low-entropy data: thousands per MiB).  Off until a fetch has
    // seen that, so the common case launches no split workers at all.
    bool split_hint = false;
    // the dense pass runs only once a fetched launch of this handle held a dense
    // tile (low-entropy / periodic data); until then its launch is skipped, and a
    // launch that turns out to hold dense tiles is re-run by fetch with it
    bool dense_hint = false, last_dense_off = false;
    bool dense_heavy = false;           // the last fetched launch had >= 1 % dense tiles (scan choice)

    // two per-launch zeroed blocks (Tables::znext): launch k uses block zpar; the
    // resolve of launch k zeroes the other one for launch k+1
    uint32_t zpar = 0, zlast = 0;
    bool zclean[2] = {false, false};

    // the fetched launch's results on the host: valid from its first fetch until
    // the next plan or launch, so the count-then-fetch pattern (cap 0 for the
    // total, then the caller's buffer: syncr_ingest's complete()) waits for the
    // device once; a small launch's cut slots and hashes come down with its
    // counters in that same wait
    struct FetchCache {
        bool valid = false, cuts = false;
        uint32_t ctr[4];
        std::vector<uint64_t> counts;
        uint32_t sp[SPL_WORDS];
        std::vector<DevCut> all;
        uint64_t hc[B3C_WORDS];
        std::vector<uint8_t> hs;
    } fc;

    // launch
    bool launched = false;
    const uint8_t *last_bytes = nullptr;
    hipStream_t last_stream = nullptr;  // stream of the last launch (nullptr: none since open)
    hipEvent_t xstream_ev = nullptr;    // orders a launch after the previous one on another stream
    hipEvent_t up_ev = nullptr;         // the plan's table upload on `stream` (not waited for by plan)
    bool up_pending = false;            // hstage may still be read by that upload
    uint64_t stats[4] = {0, 0, 0, 0};
    uint64_t scan_info[4] = {SYNCR_CDC_SCAN_NONE, 0, 0, 0};   // syncr_cdc_last_scan
    uint64_t reruns = 0;                // capacity re-runs of the last fetch
    bool split_launched = false;        // the last launch started split workers
    uint64_t split_stats[6] = {0, 0, 0, 0, 0, 0};

    // host-path staging
    DevBuf stage;
    HostStage hstage;                   // pinned: CopyGroup uploads / downloads
    std::vector<uint64_t> h_iblocks;    // b3_items_kernel block table (kept for its upload)

    // timing
    bool timing = false;
    bool timing_scan_only = false;            // set_timing(h, 2, 3 or 4): the scan only
    bool timing_clock = false;                // set_timing(h, 4): by the device clock (no events)
    DevBuf tacc;                              // [sum of scan ticks, launches] (timing_clock)
    uint64_t wall_khz = 100000;               // the device clock's rate
    std::vector<PendingTiming> pending;
    double ms[NPHASE] = {0, 0, 0, 0};
    uint64_t timed_launches = 0;
};

namespace {

int32_t hip_err(hipError_t e) {
    if (e == hipSuccess) return SYNCR_CDC_OK;
#ifdef SYNCR_CDC_DEV
    fprintf(stderr, "syncr_cdc (dev): HIP error %d: %s\n", (int)e, hipGetErrorString(e));
#endif
    if (e == hipErrorOutOfMemory) return SYNCR_CDC_ENOMEM;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return SYNCR_CDC_ENODEV;
    return SYNCR_CDC_EIO;
}

#define CHECK_HIP(x)                                  \
    do {                                              \
        hipError_t e_ = (x);                          \
        if (e_ != hipSuccess) return hip_err(e_);     \
    } while (0)

int32_t validate_params(const syncr_cdc_params *p) {
    if (!p) return SYNCR_CDC_EINVAL;
    if (p->chunk_bits < 1 || p->chunk_bits > 31) return SYNCR_CDC_EINVAL;
    if (p->flags & ~(uint32_t)(SYNCR_CDC_FLAG_RESOLVE_LANE | SYNCR_CDC_FLAG_RESOLVE_NOBURST |
                               SYNCR_CDC_FLAG_RESOLVE_NOSPLIT | SYNCR_CDC_FLAG_SPLIT_NOWAIT))
        return SYNCR_CDC_EINVAL;
    if (p->max_chunk < 1 || p->max_chunk > 0xffffffffull) return SYNCR_CDC_EINVAL;
    return SYNCR_CDC_OK;
}

KParams make_kparams(const syncr_cdc_params &p) {
    KParams k{};
    k.bits = p.chunk_bits;
    k.mask = (uint32_t)((1ull << p.chunk_bits) - 1);
    k.m1 = p.chunk_bits > 16 ? (uint32_t)((1u << (p.chunk_bits - 16)) - 1) : 0u;
    const uint32_t kk = 1u << (16 - std::min<uint32_t>(p.chunk_bits, 16));
    k.k = kk;
    k.kk = (kk & 0xffffu) | ((kk & 0xffffu) << 16);
    const uint32_t km = (0u - 64u * kk) & 0xffffu;
    k.kmv = km | (km << 16);
    k.max_chunk = p.max_chunk;
    k.read_cap = p.read_cap;
    k.nt = 1;              // tile bytes are read once: non-temporal loads
    k.nt_out = 0;          // candidate words / cuts: plain stores (non-temporal: dev A/B, no faster)
    k.dense_blocks = 0;
    // exact alternative resolves, for cross-checks (include/syncr_cdc.h)
    k.resolve_lane = (p.flags & SYNCR_CDC_FLAG_RESOLVE_LANE) ? 1u : 0u;
    k.resolve_noburst = (p.flags & SYNCR_CDC_FLAG_RESOLVE_NOBURST) ? 1u : 0u;
    k.resolve_nosplit = (p.flags & SYNCR_CDC_FLAG_RESOLVE_NOSPLIT) ? 1u : 0u;
    return k;
}

// Output slots reserved per file: 16x the expected chunk count plus slack; a
// file that needs more is re-resolved with its exact count (fetch()).
// host -> device, complete on return
// the group as one copy dispatch: small, few tables, whole 4-byte words
bool one_dispatch(const CopyGroup &g) {
    if (g.total > KCOPY_MAX || g.items.size() > (size_t)COPY_MAX) return false;
    size_t zeros = 0;
    for (const auto &it : g.items) {
        if (it.n & 3u) return false;
        if (!it.host) zeros += it.n;
    }
    return zeros <= KCOPY_MAX;
}

// the staging buffer is free: a plan's upload left in flight has completed
hipError_t stage_free(syncr_cdc *h) {
    if (!h->up_pending) return hipSuccess;
    const hipError_t e = hipEventSynchronize(h->up_ev);
    if (e == hipSuccess) h->up_pending = false;
    return e;
}

// wait = false (plan): the copy is left in flight on the handle's stream, and
// do_launch orders a launch on another stream after it (up_ev)
hipError_t upload(syncr_cdc *h, const CopyGroup &g, bool wait = true) {
    if (g.items.empty()) return hipSuccess;
    hipError_t e = stage_free(h);
    if (e != hipSuccess) return e;
    if (g.total > STAGE_MAX || (e = h->hstage.ensure(std::max<size_t>(g.total, 16))) != hipSuccess) {
        for (const auto &it : g.items) {
            e = it.host ? hipMemcpy(it.dev, it.host, it.n, hipMemcpyHostToDevice) : hipMemset(it.dev, 0, it.n);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    for (const auto &it : g.items)
        if (it.host) memcpy(h->hstage.p + it.off, it.host, it.n);
    if (one_dispatch(g)) {
        CopyList l{};
        uint64_t bytes = 0;
        for (const auto &it : g.items) {
            l.seg[l.n++] = CopySeg{it.host ? h->hstage.d + it.off : nullptr, it.dev, it.n};
            bytes += it.n;
        }
        if ((e = launch_copy(l, bytes, h->stream)) != hipSuccess) return e;
    } else {
        for (const auto &it : g.items) {
            e = it.host ? hipMemcpyAsync(it.dev, h->hstage.p + it.off, it.n, hipMemcpyHostToDevice, h->stream)
                        : hipMemsetAsync(it.dev, 0, it.n, h->stream);
            if (e != hipSuccess) return e;
        }
    }
    if (wait) return hipStreamSynchronize(h->stream);
    if (!h->up_ev) e = hipEventCreateWithFlags(&h->up_ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(h->up_ev, h->stream);
    if (e != hipSuccess) {              // no event to order by: complete the copy here instead
        (void)hipStreamSynchronize(h->stream);
        return e;
    }
    h->up_pending = true;
    return hipSuccess;
}

// device -> host, complete on return (the caller has waited for the kernels
// that wrote the device side)
hipError_t download(syncr_cdc *h, const CopyGroup &g) {
    if (g.items.empty()) return hipSuccess;
    hipError_t e = stage_free(h);
    if (e != hipSuccess) return e;
    if (g.total > STAGE_MAX || (e = h->hstage.ensure(g.total)) != hipSuccess) {
        for (const auto &it : g.items)
            if ((e = hipMemcpy(it.host, it.dev, it.n, hipMemcpyDeviceToHost)) != hipSuccess) return e;
        return hipSuccess;
    }
    if (one_dispatch(g)) {
        CopyList l{};
        for (const auto &it : g.items) l.seg[l.n++] = CopySeg{it.dev, h->hstage.d + it.off, it.n};
        if ((e = launch_copy(l, g.total, h->stream)) != hipSuccess) return e;
    } else {
        for (const auto &it : g.items)
            if ((e = hipMemcpyAsync(h->hstage.p + it.off, it.dev, it.n, hipMemcpyDeviceToHost, h->stream)) !=
                hipSuccess)
                return e;
    }
    if ((e = hipStreamSynchronize(h->stream)) != hipSuccess) return e;
    for (const auto &it : g.items) memcpy(it.host, h->hstage.p + it.off, it.n);
    return hipSuccess;
}

uint32_t default_cut_cap(uint64_t len, uint32_t bits) {
    const uint32_t sh = bits > 4 ? bits - 4 : 0;
    uint64_t c = (len >> sh) + 8;
    return (uint32_t)std::min<uint64_t>(c, 0xffffffffull);
}

// the per-launch zeroed block: ctr[4] | nonempty[nwords] (u64) | super_cnt[nwords] (u32) |
// coarse[ncoarse * COARSE_STRIDE] (u32, 128-byte aligned) | split[SPL_WORDS]
uint32_t ncoarse(const syncr_cdc *h) { return (h->nwords + 63) / 64; }
size_t coarse_offset(const syncr_cdc *h) { return (16 + (size_t)h->nwords * 12 + 127) & ~size_t(127); }
size_t split_ctr_offset(const syncr_cdc *h) {
    return coarse_offset(h) + (size_t)ncoarse(h) * COARSE_STRIDE * 4;
}
size_t sched_offset(const syncr_cdc *h) { return (split_ctr_offset(h) + SPL_WORDS * 4 + 127) & ~size_t(127); }
uint32_t st_tiles_of(int segs) { return (uint32_t)segs * 8u / 9u; }
size_t tscan_offset(const syncr_cdc *h) { return sched_offset(h) + (size_t)SCHED_REGIONS * COARSE_STRIDE * 4; }
size_t zeroed_bytes(const syncr_cdc *h) { return tscan_offset(h) + 128; }
size_t zstride(const syncr_cdc *h) { return (zeroed_bytes(h) + 255) & ~size_t(255); }
uint8_t *zblock(const syncr_cdc *h, uint32_t par) { return h->zeroed.as<uint8_t>() + par * zstride(h); }

Tables make_tables(syncr_cdc *h) {
    Tables t{};
    t.span = h->span;
    t.ntiles = h->ntiles;
    t.tile = (uint32_t)scan_tile_bytes(h->geom);
    t.nwords = h->nwords;
    t.nstarts = h->nstarts;
    t.fstart = h->fstart.as<uint64_t>();
        t.nfiles = h->nfiles;
    t.foff = h->foff.as<uint64_t>();
    t.flen = h->flen.as<uint64_t>();
    t.order = h->order.as<uint32_t>();
    t.ofile = h->ofile.as<ulonglong2>();
    t.cut_base = h->cut_base.as<uint64_t>();
    t.cut_cap = h->cut_cap.as<uint32_t>();
    t.tile_meta = h->tile_meta.as<uint32_t>();
    t.slots = h->slots.as<uint2>();
    uint8_t *zb = zblock(h, h->zpar);
    t.ctr = reinterpret_cast<uint32_t *>(zb);
    t.nonempty = reinterpret_cast<unsigned long long *>(zb + 16);
    t.super_cnt = reinterpret_cast<uint32_t *>(zb + 16 + (size_t)h->nwords * 8);
    t.coarse = reinterpret_cast<uint32_t *>(zb + coarse_offset(h));
    t.ncoarse = ncoarse(h);
    t.super_off = h->super_off.as<uint64_t>();
    t.dense_list = h->dense_list.as<uint32_t>();
    t.dense_cnt = h->dense_cnt.as<uint32_t>();
    t.dense_cap = h->dense_cap;
    t.dense_bits = h->dense_bits.as<uint32_t>();
    t.dense_fix = h->dense_fix.as<uint8_t>();
    t.dense_pos = h->dense_pos.as<uint16_t>();
    t.cand = h->cand.as<uint64_t>();
    // chain links only while the handle splits (periodic / low-entropy data):
    // random data never chains, and its fix-ups skip the link work
    t.linkw = h->split_hint ? h->linkw.as<uint64_t>() : nullptr;
    t.cand_cap = h->cand_cap;
    t.cuts = h->cuts.as<DevCut>();
    t.counts = h->counts.as<uint64_t>();
    t.ngrid = h->ngrid;
    t.gpos = h->gpos.as<uint64_t>();
    t.gend = h->gend.as<uint64_t>();
    t.gfix = h->gfix.as<uint8_t>();
    t.gbase = h->gbase.as<uint64_t>();
    t.n_elig = h->split_hint ? h->n_elig : 0u;
    t.seg_cap = h->seg_cap;
    t.segs = h->segs.as<SplitSeg>();
    t.seg_cuts = h->seg_cuts.as<DevCut>();
    t.seg_segc = h->split_segc;
    t.seg_scap = split_scap(h->split_segc);
    t.split_blocks = h->split_blocks;
    t.runs = h->runs.as<RunJob>();
    t.runs_cap = (h->n_elig && h->seg_cap) ? h->runs_cap : 0u;     // deferral only when the copy launch runs
    t.split = reinterpret_cast<uint32_t *>(zb + split_ctr_offset(h));
    t.sched = reinterpret_cast<uint32_t *>(zb + sched_offset(h));
    t.nst = (h->ntiles + ST_TILES - 1) / ST_TILES;   // do_launch sets the launch's geometry
    t.tscan = reinterpret_cast<uint64_t *>(zb + tscan_offset(h));
    t.nt_out = h->kp.nt_out;
    t.gapmax = (h->kp.read_cap && h->kp.read_cap < h->kp.max_chunk) ? h->kp.read_cap : h->kp.max_chunk;
    t.tacc = (h->timing && h->timing_clock) ? h->tacc.as<uint64_t>() : nullptr;
    t.znext = reinterpret_cast<uint4 *>(zblock(h, h->zpar ^ 1u));
    t.znext_vec = (uint32_t)(zstride(h) / 16);
    t.hzero = nullptr;
    t.dbg = h->dbg.p ? h->dbg.as<uint64_t>() : nullptr;
    t.dense_off = (!h->dense_hint && !scan_dense_inline(h->geom, h->kp)) ? 1u : 0u;
    // SplitSeg records outlive a launch: a record is ready for this launch only
    // when its ready word holds this launch's id (records are zeroed when allocated)
    static std::atomic<uint32_t> epochs{0};
    uint32_t ep;
    while ((ep = ++epochs) == 0u) {}
    t.epoch = ep;
    return t;
}

int32_t upload_cut_tables(syncr_cdc *h, CopyGroup *into = nullptr) {
    h->h_cut_base.resize(h->nfiles);
    uint64_t acc = 0;
    for (uint32_t i = 0; i < h->nfiles; i++) {
        h->h_cut_base[i] = acc;
        acc += h->h_cut_cap[i];
    }
    h->total_cut_cap = acc;
    // BLAKE3 lane tasks: 1 leaf on a small launch, B3_LANE_LEAVES otherwise
    // (cdc_internal.h).  A chunk of len bytes is ceil(leaves / (64 LPL)) group
    // items (the last may be a tail placeholder), so a file needs at most
    // ceil(F / group bytes) + (its cuts) of them
    // (a chunk is at most max_chunk: with 1-leaf tasks one of 64 MiB is 1024 group
    // items for b3_tree_kernel's single wave to merge, 4x its 4-leaf count)
    const bool variant = h->b3_coop != 3 || h->b3_ablate || h->b3_nt;    // dev loaders: 4-leaf instances only
    const bool small = h->span <= B3_SMALL_SPAN && h->kp.max_chunk <= (64ull << 20);
    h->b3_lpl_log = (h->b3_lpl ? h->b3_lpl == 1 : small) && !variant ? 0u : 2u;
    const uint64_t gbytes = (1024ull * 64ull) << h->b3_lpl_log;
    uint64_t icap = 0;
    for (uint32_t i = 0; i < h->nfiles; i++) icap += (h->h_flen[i] + gbytes - 1) / gbytes + h->h_cut_cap[i];
    h->items_cap = std::max<uint64_t>(icap, 1);
    h->trees_cap = std::max<uint64_t>(acc, 1);
    CHECK_HIP(h->hctr.ensure(B3_CTR_BYTES));
    CHECK_HIP(h->items.ensure(h->items_cap * 8));
    CHECK_HIP(h->trees.ensure(h->trees_cap * 16));
    CHECK_HIP(h->gcv.ensure(h->items_cap * 32));
    CHECK_HIP(h->hashes.ensure(std::max<uint64_t>(acc, 1) * 32));
    CHECK_HIP(h->packed.ensure((size_t)B3_CLASSES * std::max<uint64_t>(acc, 1) * 8));
    // pieces: at most popcount(63) = 6 per chunk (a split unit has under 64 tasks)
    h->pieces_cap = std::max<uint64_t>(6 * acc, 1);
    CHECK_HIP(h->tpieces.ensure(h->trees_cap * 8));
    CHECK_HIP(h->pieces.ensure(h->pieces_cap * 16));
    CHECK_HIP(h->pcv.ensure(h->pieces_cap * 32));
    // b3_items_kernel blocks: each group of 256 files is split into parts of
    // ~B3_ITEMS_CUTS of its output slots, so one file with millions of chunks
    // (periodic data) is planned by many blocks, not one
    std::vector<uint64_t> &ib = h->h_iblocks;
    ib.clear();
    for (uint32_t g = 0; g * 256u < h->nfiles; g++) {
        uint64_t caps = 0;
        for (uint32_t i = g * 256u; i < std::min<uint32_t>(h->nfiles, g * 256u + 256u); i++) caps += h->h_cut_cap[i];
        const uint64_t parts = std::min<uint64_t>(std::max<uint64_t>((caps + B3_ITEMS_CUTS - 1) / B3_ITEMS_CUTS, 1), 0xfffff);
        for (uint64_t k = 0; k < parts; k++) ib.push_back(((uint64_t)g << 40) | (k << 20) | parts);
    }
    h->n_iblocks = (uint32_t)ib.size();
    CHECK_HIP(h->iblocks.ensure(std::max<size_t>(ib.size(), 1) * 8));
    CHECK_HIP(h->cut_base.ensure(std::max<size_t>(h->nfiles, 1) * 8));
    CHECK_HIP(h->cut_cap.ensure(std::max<size_t>(h->nfiles, 1) * 4));
    CHECK_HIP(h->cuts.ensure(std::max<uint64_t>(acc, 1) * sizeof(DevCut)));
    CopyGroup own;
    CopyGroup &g = into ? *into : own;
    g.add(h->iblocks.p, ib.data(), ib.size() * 8);
    g.add(h->cut_base.p, h->h_cut_base.data(), h->nfiles * 8ull);
    g.add(h->cut_cap.p, h->h_cut_cap.data(), h->nfiles * 4ull);
    if (!into) CHECK_HIP(upload(h, own));
    return SYNCR_CDC_OK;
}

HashTables make_hash_tables(syncr_cdc *h) {
    HashTables t{};
    t.ctr = h->hctr.as<uint64_t>();
    t.items = h->items.as<uint64_t>();
    t.items_cap = h->items_cap;
    t.trees = h->trees.as<ulonglong2>();
    t.trees_cap = h->trees_cap;
    t.tpieces = h->tpieces.as<uint64_t>();
    t.pieces = h->pieces.as<ulonglong2>();
    t.pcv = h->pcv.as<uint32_t>();
    t.pieces_cap = h->pieces_cap;
    t.gcv = h->gcv.as<uint32_t>();
    t.hashes = h->hashes.as<uint32_t>();
    t.packed = h->packed.as<uint64_t>();
    t.packed_cap = std::max<uint64_t>(h->total_cut_cap, 1);
    t.ablate = h->b3_ablate;
    t.nt = h->b3_nt;
    t.coop = h->b3_coop;
    t.iblocks = h->iblocks.as<uint64_t>();
    t.n_iblocks = h->n_iblocks;
    t.lpl_log = h->b3_lpl_log;
    t.nosplit = h->b3_nosplit;
    t.nouni = h->b3_nouni;
    return t;
}

int32_t ensure_dense(syncr_cdc *h, uint32_t cap) {
    h->dense_cap = cap;
    CHECK_HIP(h->dense_list.ensure(std::max<size_t>(cap, 1) * 4));
    CHECK_HIP(h->dense_cnt.ensure(std::max<size_t>(cap, 1) * 4));
    CHECK_HIP(h->dense_bits.ensure(std::max<size_t>(cap, 1) * (size_t)(scan_tile_bytes(h->geom) / 32) * 4));
    CHECK_HIP(h->dense_fix.ensure(std::max<size_t>(cap, 1) * (size_t)FIXCAP));
    CHECK_HIP(h->dense_pos.ensure(std::max<size_t>(cap, 1) * (size_t)FIXCAP * 2));
    return SYNCR_CDC_OK;
}

// Split-walk records and scratch, only while the handle splits (split_hint):
// a file splits into segments of split_segc of its candidates, so
// cand_cap / split_segc records cover every split file.
int32_t ensure_split(syncr_cdc *h) {
    h->seg_cap = 0;
    if (h->n_elig && h->split_hint) {
        const uint64_t segs = std::min<uint64_t>(h->cand_cap / h->split_segc + 8, 0xffffffull);
        CHECK_HIP(h->segs.ensure(segs * sizeof(SplitSeg)));
        CHECK_HIP(hipMemset(h->segs.p, 0, segs * sizeof(SplitSeg)));     // no ready word from other memory
        CHECK_HIP(h->seg_cuts.ensure(segs * split_scap(h->split_segc) * sizeof(DevCut)));
        const uint64_t runs = std::min<uint64_t>(h->cand_cap / 64 + 1024, 0xffffffull);
        CHECK_HIP(h->runs.ensure(runs * sizeof(RunJob)));
        h->runs_cap = (uint32_t)runs;
        h->seg_cap = (uint32_t)segs;
    }
    return SYNCR_CDC_OK;
}

int32_t ensure_cand(syncr_cdc *h, uint64_t cap) {
    h->cand_cap = cap;
    CHECK_HIP(h->cand.ensure(std::max<uint64_t>(cap, 1) * 8));
    CHECK_HIP(h->linkw.ensure((cap / 64 + 4) * 8));
    return ensure_split(h);
}

void drain_timing(syncr_cdc *h) {
    for (auto &pt : h->pending) {
        (void)hipEventSynchronize(pt.ev[pt.nev - 1]);
        for (int k = 0; k + 1 < pt.nev; k++) {
            float f = 0.f;
            if (hipEventElapsedTime(&f, pt.ev[k], pt.ev[k + 1]) == hipSuccess) h->ms[k] += f;
        }
        for (int k = 0; k < pt.nev; k++) (void)hipEventDestroy(pt.ev[k]);
        h->timed_launches++;
    }
    h->pending.clear();
}

// Scan ordering between handles of one device.  The scan is a persistent grid
// sized to fill every CU (scan_grid = CUs x resident blocks), so two scans in
// flight on two streams cannot co-reside: they contend for the same slots and
// HBM, and the later one's waves start piecemeal as the earlier one's retire.
// With several handles on one device (the ingest pipeline's slots, bench.py's
// pipelined segment) each launch's scan could wait for the scan most recently
// enqueued on that device by ANOTHER handle, so that only the short
// compaction / fix-up / resolve / hash tail of one batch overlaps the next
// batch's scan (round 1: two unordered scans in flight made the step 13 %
// slower than one, BENCH_r01.json `pipelined`).  The product no longer orders
// them (round 6): the persistent scan grids hand the CUs over as the first
// scan's last stream tiles end, so the next batch's scan fills the first one's
// tail.  Two batches in flight, same process (tools/pipe_ab.py,
// profiles/r06v_pipe_ab/): config 4's shards 0.686 -> 0.734 of 8 TB/s per step,
// uniform1k 0.661 -> 0.716, zipf10k 0.823 -> 0.827, dense 0.652 -> 0.656; the
// development library restores the order with SYNCR_CDC_SERIAL=1.
struct ScanOrder {
    std::mutex mu;
    const syncr_cdc *owner = nullptr;   // handle whose scan was enqueued last
    hipEvent_t ev = nullptr;            // its scan_done event
    std::atomic<int> open{0};           // handles open on the device: ordering only when > 1
};
ScanOrder &scan_order(int device) {
    static std::mutex reg_mu;
    static std::map<int, ScanOrder> reg;   // std::map: node addresses are stable
    std::lock_guard<std::mutex> g(reg_mu);
    return reg[device];
}

int32_t do_launch(syncr_cdc *h, const uint8_t *d_bytes, hipStream_t s) {
    CHECK_HIP(hipSetDevice(h->device));
    h->fc.valid = false;
    KParams kp = h->kp;
    kp.scan_tiles = h->dense_heavy ? 1u : 0u;
    Tables t = make_tables(h);
    PendingTiming pt{};
    pt.nev = h->timing_scan_only ? 2 : h->hash_on ? 5 : 4;
    if (h->timing && !h->timing_clock) {
        if (h->pending.size() >= 256) drain_timing(h);
        // timing only: no system-scope release (a cache writeback + invalidate per
        // event would stall the queue and perturb the kernels being timed)
        for (int k = 0; k < pt.nev; k++) CHECK_HIP(hipEventCreateWithFlags(&pt.ev[k], hipEventDisableSystemFence));
    }
    // All launches of a handle share its tables (counter blocks, candidate
    // list, cuts, hash work lists).  On the same stream they are ordered; when
    // the caller switches streams, this launch first waits for everything
    // enqueued on the previous launch's stream (an event recorded there now),
    // so no two launches of one handle ever overlap -- and the block the
    // previous resolve zeroed (zclean) is zero by the time this scan starts.
    if (h->last_stream && s != h->last_stream) {
        if (!h->xstream_ev)
            CHECK_HIP(hipEventCreateWithFlags(&h->xstream_ev, hipEventDisableTiming | hipEventDisableSystemFence));
        CHECK_HIP(hipEventRecord(h->xstream_ev, h->last_stream));
        CHECK_HIP(hipStreamWaitEvent(s, h->xstream_ev, 0));
    }
    // the plan's tables (uploaded on the handle's stream, not waited for)
    if (h->up_pending && s != h->stream) CHECK_HIP(hipStreamWaitEvent(s, h->up_ev, 0));
    const uint32_t par = h->zpar;
    if (!h->zclean[par]) CHECK_HIP(hipMemsetAsync(zblock(h, par), 0, zeroed_bytes(h), s));
    h->zclean[par] = false;
    if (h->hash_on && t.nfiles) t.hzero = h->hctr.as<uint64_t>();     // zeroed by the resolve
    ScanOrder &so = scan_order(h->device);
    const bool order = h->serial_scans && so.open.load() > 1;          // another handle on this device
    if (order) {
        std::lock_guard<std::mutex> g(so.mu);        // held: the owner cannot close its event meanwhile
        if (so.owner && so.owner != h) CHECK_HIP(hipStreamWaitEvent(s, so.ev, 0));
    }
#ifdef SYNCR_CDC_DEV
    if (t.dbg) CHECK_HIP(hipMemsetAsync(t.dbg, 0, DBG_WORDS * sizeof(uint64_t), s));
#endif
    // HIP events (timing modes 1, 2 and 3) are marker packets around the kernels: each
    // costs queue idle (an event pair ~18 us of a 1 GiB batch's ~0.3 ms step,
    // profiles/r05c_*_trace_shard8); mode 4 times the scan by the device clock instead
    const bool events = h->timing && !h->timing_clock;
    const bool bound = events && t.ntiles;           // the pair around the scan: launch_scan records it
    if (events && !bound) CHECK_HIP(hipEventRecord(pt.ev[0], s));
    {
        const int kind = scan_kind(h->geom, h->scan_grid, kp, t);
        const uint64_t waves = std::min<uint64_t>(h->scan_grid, t.ntiles);
        h->scan_info[0] = (uint64_t)kind;
        h->scan_info[1] = t.ntiles;
        h->scan_info[2] = kind == SYNCR_CDC_SCAN_NONE ? 0u : waves;
        h->scan_info[3] = 0;
        // stream tiles: STs of the launch's geometry
        const int segs = kind == SYNCR_CDC_SCAN_STREAM_TILES ? st_segs(h->scan_grid, kp, t) : ST_SEGS;
        t.nst = (h->ntiles + st_tiles_of(segs) - 1) / st_tiles_of(segs);
        if (kind == SYNCR_CDC_SCAN_STREAM_TILES) h->scan_info[3] = (uint64_t)segs;
    }
    CHECK_HIP(launch_scan(h->geom, h->scan_grid, d_bytes, kp, t, s, bound ? pt.ev[0] : nullptr,
                          bound ? pt.ev[1] : nullptr));
    if (events && !bound) CHECK_HIP(hipEventRecord(pt.ev[1], s));
    if (order) {
        std::lock_guard<std::mutex> g(so.mu);
        CHECK_HIP(hipEventRecord(h->scan_done, s));
        so.owner = h;
        so.ev = h->scan_done;
    }
    // an event record costs ~6 us of queue idle: the scan-only mode has only the
    // two bound to the scan dispatch (no markers); the phase mode adds markers
    const bool phases = events && !h->timing_scan_only;
    CHECK_HIP(launch_post(d_bytes, kp, t, s, scan_dense_inline(h->geom, kp), h->scan_grid));
    h->last_dense_off = t.dense_off != 0u;
    if (phases) CHECK_HIP(hipEventRecord(pt.ev[2], s));
    CHECK_HIP(launch_resolve(d_bytes, kp, t, s));
    h->split_launched = resolve_splits(kp, t);
    if (t.nfiles) h->zclean[par ^ 1u] = true;        // the resolve zeroed the next launch's block
    h->zlast = par;
    h->zpar = par ^ 1u;
    if (phases) CHECK_HIP(hipEventRecord(pt.ev[3], s));
    if (h->hash_on) {
        CHECK_HIP(launch_hash(h->device, d_bytes, t, make_hash_tables(h), s));
        if (phases) CHECK_HIP(hipEventRecord(pt.ev[4], s));
    }
    if (events) h->pending.push_back(pt);
    h->launched = true;
    h->last_bytes = d_bytes;
    h->last_stream = s;
    return SYNCR_CDC_OK;
}

}  // namespace

extern "C" {

int32_t syncr_cdc_abi_version(void) { return SYNCR_CDC_ABI_VERSION; }

const char *syncr_cdc_strerror(int32_t code) {
    switch (code) {
        case SYNCR_CDC_OK: return "ok";
        case SYNCR_CDC_EINVAL: return "invalid argument";
        case SYNCR_CDC_ENOMEM: return "out of memory";
        case SYNCR_CDC_ERANGE: return "output capacity too small";
        case SYNCR_CDC_ENODEV: return "no HIP device";
        case SYNCR_CDC_EIO: return "HIP runtime error";
        case SYNCR_CDC_ESTATE: return "call out of order";
        case SYNCR_CDC_ENOENT: return "no such entry";
        case SYNCR_CDC_EBUSY: return "locked by another handle";
        default: return "unknown error";
    }
}

void syncr_cdc_default_params(syncr_cdc_params *p) {
    if (!p) return;
    p->chunk_bits = 20;                 // src/chunking.rs:7
    p->flags = 0;
    p->max_chunk = (1ull << 20) * 16;   // src/chunking.rs:10-13
    p->read_cap = 2ull * 1024 * 1024;   // tokio File::read cap (file_operations.rs:738,776)
}

int32_t syncr_cdc_device_count(int32_t *n) {
    if (!n) return SYNCR_CDC_EINVAL;
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) { *n = 0; return SYNCR_CDC_ENODEV; }
    *n = c;
    return SYNCR_CDC_OK;
}

int32_t syncr_cdc_open(int32_t device, const syncr_cdc_params *p, syncr_cdc **out) {
    if (!out) return SYNCR_CDC_EINVAL;
    *out = nullptr;
    syncr_cdc_params prm;
    if (p) prm = *p; else syncr_cdc_default_params(&prm);
    int32_t rc = validate_params(&prm);
    if (rc) return rc;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return SYNCR_CDC_ENODEV;
    if (device < 0 || device >= ndev) return SYNCR_CDC_ENODEV;
    CHECK_HIP(hipSetDevice(device));
    syncr_cdc *h = new (std::nothrow) syncr_cdc();
    if (!h) return SYNCR_CDC_ENOMEM;
    h->device = device;
    h->params = prm;
    h->kp = make_kparams(prm);
    {   // split workers wait at most ~100 ms of wall clock for file walkers (cdc_kernels.hip split_next)
        int khz = 0;
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess || khz <= 0)
            khz = 100000;
        h->kp.split_patience = (prm.flags & SYNCR_CDC_FLAG_SPLIT_NOWAIT) ? 0ull : 100ull * (uint64_t)khz;
        h->wall_khz = (uint64_t)khz;
    }
    h->kp.dense_fuse = 1u;                      // dense pass computes its candidates' head fix-ups
#ifdef SYNCR_CDC_DEV
    // Development library only (libsyncr_cdc_dev.so, used by tools/): variants
    // and timing-only ablations chosen by environment variables.  The product
    // library reads no environment at all, so no stray variable can change its
    // results.
    if (const char *a = getenv("SYNCR_CDC_ABLATE")) h->kp.ablate = (uint32_t)atoi(a);  // timing-only
    if (const char *nt = getenv("SYNCR_CDC_NT")) h->kp.nt = (uint32_t)atoi(nt);
    if (const char *rs = getenv("SYNCR_CDC_RESOLVE")) {
        h->kp.resolve_lane = strcmp(rs, "lane") == 0;
        h->kp.resolve_noburst = strcmp(rs, "noburst") == 0;
        h->kp.resolve_nosplit = strcmp(rs, "nosplit") == 0;
    }
    if (const char *a = getenv("SYNCR_CDC_SERIAL")) h->serial_scans = atoi(a) != 0;
    if (const char *a = getenv("SYNCR_CDC_RESOLVE_PF")) h->kp.resolve_pf = (uint32_t)atoi(a);      // A/B only
    if (const char *a = getenv("SYNCR_CDC_SPLIT_FIRST")) h->kp.split_first = (uint32_t)atoi(a) != 0; // A/B only
    if (const char *a = getenv("SYNCR_CDC_NOSKIP")) h->kp.no_skip = atoi(a) != 0;                    // A/B only
    if (const char *a = getenv("SYNCR_CDC_DENSE_FUSE")) h->kp.dense_fuse = atoi(a) != 0;           // A/B only
    if (const char *a = getenv("SYNCR_CDC_ST_SEGS")) h->kp.st_segs = (uint32_t)atoi(a);          // A/B only
    if (const char *a = getenv("SYNCR_CDC_NT_OUT")) h->kp.nt_out = atoi(a) != 0;                 // A/B only
    if (const char *a = getenv("SYNCR_CDC_DENSE_BLOCKS")) h->kp.dense_blocks = (uint32_t)atoi(a);  // A/B only
    if (const char *a = getenv("SYNCR_CDC_TRACE"))                                              // timeline
        if (atoi(a)) CHECK_HIP(h->dbg.ensure(DBG_WORDS * sizeof(uint64_t)));
    if (const char *a = getenv("SYNCR_CDC_SPLIT_SEGC")) h->split_segc = std::max(256, atoi(a));        // A/B only
    if (const char *a = getenv("SYNCR_CDC_SPLIT_BLOCKS")) h->split_blocks = std::max(1, atoi(a));     // A/B only
    if (const char *a = getenv("SYNCR_B3_ABLATE")) h->b3_ablate = (uint32_t)atoi(a) % 3;   // timing-only
    if (const char *nt = getenv("SYNCR_B3_NT")) h->b3_nt = (uint32_t)atoi(nt) != 0;
    if (const char *sp = getenv("SYNCR_B3_SPLIT")) h->b3_nosplit = atoi(sp) == 0;          // A/B only
    if (const char *un = getenv("SYNCR_B3_UNI")) h->b3_nouni = atoi(un) == 0;              // A/B only
    if (const char *lp = getenv("SYNCR_B3_LPL")) h->b3_lpl = atoi(lp) == 1 ? 1u : (atoi(lp) == 4 ? 4u : 0u);  // A/B only
    if (const char *ld = getenv("SYNCR_B3_LOAD"))                                         // A/B only
        h->b3_coop = strcmp(ld, "plain") == 0  ? 0u
                     : strcmp(ld, "coop") == 0 ? 1u
                     : strcmp(ld, "pair") == 0 ? 2u : 3u;      // default / pairmq: + quad merges
    if (const char *k = getenv("SYNCR_CDC_SCAN")) {
        if (strcmp(k, "valu") == 0) h->geom = ScanGeom{SCAN_VALU, DEFAULT_RUN, 0};
        if (strcmp(k, "mfma") == 0) h->geom = ScanGeom{SCAN_MFMA, DEFAULT_NB, MFV_SINGLE | MFV_NOPIPE};
    }
    if (const char *r = getenv("SYNCR_CDC_RUN")) {      // implies the VALU scan
        const ScanGeom g{SCAN_VALU, atoi(r), 0};
        if (scan_supported(g)) h->geom = g;
    }
    if (const char *r = getenv("SYNCR_CDC_NB")) {       // implies the MFMA scan
        const ScanGeom g{SCAN_MFMA, atoi(r), h->geom.kind == SCAN_MFMA ? h->geom.var : MFV_SINGLE | MFV_NOPIPE};
        if (scan_supported(g)) h->geom = g;
    }
    if (const char *v = getenv("SYNCR_CDC_MFVAR")) {    // MFV_* bits of the MFMA scan
        if (h->geom.kind == SCAN_MFMA) h->geom.var = atoi(v) & 3;
    }
#endif
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0)
        cus = 256;
    h->scan_grid = (uint32_t)(cus * scan_blocks_per_cu(h->geom));
#ifdef SYNCR_CDC_DEV
    if (const char *g = getenv("SYNCR_CDC_SCAN_GRID")) {
        const int v = atoi(g);
        if (v > 0) h->scan_grid = (uint32_t)v;
    }
#endif
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
        delete h;
        return SYNCR_CDC_EIO;
    }
    // One blocking copy on the default stream (it zeroes the device-clock timing
    // sums).  Measured, not explained: once the default stream has been used the
    // scan's first ~20 launches after an idle gap -- the shader-clock dip of
    // DESIGN.md §4.2, where bench.py's timed window sits -- run 4-7 % faster,
    // while the sustained rate is unchanged (same box, tools/gpu.sh bench A/Bs,
    // profiles/r06at_default_stream/: 5602 vs 5967-6034 GiB/s; a copy on a
    // second, temporary stream gives 5876-5891).  Round 5's plan used the
    // default stream for every table upload; round 6's staged uploads stopped
    // using it and lost this.
    {
        const uint64_t zero[2] = {0, 0};
        if (h->tacc.ensure(16) != hipSuccess || hipMemcpy(h->tacc.p, zero, 16, hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipStreamDestroy(h->stream);
            delete h;
            return SYNCR_CDC_EIO;
        }
    }
    if (hipEventCreateWithFlags(&h->scan_done, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess) {
        (void)hipStreamDestroy(h->stream);
        delete h;
        return SYNCR_CDC_EIO;
    }
    scan_order(device).open++;
    *out = h;
    return SYNCR_CDC_OK;
}

void syncr_cdc_close(syncr_cdc *h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    (void)hipStreamSynchronize(h->stream);
    drain_timing(h);
    {
        ScanOrder &so = scan_order(h->device);
        std::lock_guard<std::mutex> g(so.mu);
        if (so.owner == h) {
            so.owner = nullptr;
            so.ev = nullptr;
        }
        so.open--;
        (void)hipEventDestroy(h->scan_done);
    }
    if (h->xstream_ev) (void)hipEventDestroy(h->xstream_ev);
    if (h->up_ev) (void)hipEventDestroy(h->up_ev);
    (void)hipStreamDestroy(h->stream);
    delete h;                   // every DevBuf member frees its memory (on this device, set above)
}

int32_t syncr_cdc_get_params(const syncr_cdc *h, syncr_cdc_params *p) {
    if (!h || !p) return SYNCR_CDC_EINVAL;
    *p = h->params;
    return SYNCR_CDC_OK;
}

int32_t syncr_cdc_plan(syncr_cdc *h, const uint64_t *file_off, const uint64_t *file_len,
                       uint32_t nfiles, uint64_t span) {
    if (!h) return SYNCR_CDC_EINVAL;
    if (nfiles && (!file_off || !file_len)) return SYNCR_CDC_EINVAL;
    try {
        CHECK_HIP(hipSetDevice(h->device));
        // the tables below are rewritten: a launch still running reads them, and
        // the previous plan's upload may still be writing them
        if (h->last_stream) CHECK_HIP(hipStreamSynchronize(h->last_stream));
        CHECK_HIP(stage_free(h));
        h->planned = false;
        h->launched = false;
        h->fc.valid = false;
        // validate: inside span, non-empty files must not overlap
        std::vector<uint32_t> ne;
        ne.reserve(nfiles);
        for (uint32_t i = 0; i < nfiles; i++) {
            if (file_len[i] > span || file_off[i] > span - file_len[i]) return SYNCR_CDC_EINVAL;
            if (file_len[i]) ne.push_back(i);
        }
        std::sort(ne.begin(), ne.end(), [&](uint32_t a, uint32_t b) { return file_off[a] < file_off[b]; });
        std::vector<uint64_t> starts(ne.size());
        for (size_t j = 0; j < ne.size(); j++) {
            starts[j] = file_off[ne[j]];
            if (j && file_off[ne[j - 1]] + file_len[ne[j - 1]] > starts[j]) return SYNCR_CDC_EINVAL;
        }
        const int TILE = scan_tile_bytes(h->geom);
        const uint64_t ntiles64 = (span + TILE - 1) / TILE;
        if (ntiles64 > 0x7fffffffull) return SYNCR_CDC_EINVAL;
        h->nfiles = nfiles;
        h->nstarts = (uint32_t)starts.size();
        h->span = span;
        h->ntiles = (uint32_t)ntiles64;
        h->nwords = (h->ntiles + 63) / 64;
        h->h_foff.assign(file_off, file_off + nfiles);
        h->h_flen.assign(file_len, file_len + nfiles);

        // resolve order: largest files first (longest serial chains start first)
        std::vector<uint32_t> order(nfiles);
        std::iota(order.begin(), order.end(), 0u);
        std::stable_sort(order.begin(), order.end(),
                         [&](uint32_t a, uint32_t b) { return file_len[a] > file_len[b]; });
        h->n_elig = 0;                  // files that may split their walk (a prefix of `order`)
        while (h->n_elig < nfiles && file_len[order[h->n_elig]] >= SPLIT_MIN_BYTES) h->n_elig++;
        h->h_cut_cap.resize(nfiles);
        for (uint32_t i = 0; i < nfiles; i++) h->h_cut_cap[i] = default_cut_cap(file_len[i], h->params.chunk_bits);

        CHECK_HIP(h->fstart.ensure(std::max<size_t>(starts.size(), 1) * 8));
        CHECK_HIP(h->foff.ensure(std::max<size_t>(nfiles, 1) * 8));
        CHECK_HIP(h->flen.ensure(std::max<size_t>(nfiles, 1) * 8));
        CHECK_HIP(h->order.ensure(std::max<size_t>(nfiles, 1) * 4));
        CHECK_HIP(h->ofile.ensure(std::max<size_t>(nfiles, 1) * 16));
        CHECK_HIP(h->counts.ensure(std::max<size_t>(nfiles, 1) * 8));
        CHECK_HIP(h->tile_meta.ensure(std::max<size_t>(h->ntiles, 1) * 4));
        CHECK_HIP(h->slots.ensure(std::max<size_t>(h->ntiles, 1) * LISTCAP * sizeof(uint2)));
        CHECK_HIP(h->zeroed.ensure(2 * zstride(h)));
        h->zclean[0] = h->zclean[1] = false;
        h->zpar = h->zlast = 0;
        CHECK_HIP(h->super_off.ensure(((size_t)h->nwords + 1) * 8));
        // dense tiles are rare (adversarial data); grow on demand in fetch()
        // (scan waves take their dense-list slots in batches of up to 64 pending
        // tiles, DensePend: the list has no holes, so ntiles slots always suffice)
        uint32_t dcap = std::max<uint32_t>(64u, h->ntiles / 256u);
        int32_t rc = ensure_dense(h, dcap);
        if (rc) return rc;
        rc = ensure_cand(h, std::max<uint64_t>(4096, 2ull * h->ntiles));
        if (rc) return rc;
        // every table of the plan goes up as one copy group (one wait)
        CopyGroup up;
        up.add(h->fstart.p, starts.data(), starts.size() * 8);
        std::vector<uint64_t> of(2ull * nfiles);
        for (uint32_t k = 0; k < nfiles; k++) {
            of[2 * k] = file_off[order[k]];
            of[2 * k + 1] = file_len[order[k]];
        }
        up.add(h->foff.p, file_off, nfiles * 8ull);
        up.add(h->flen.p, file_len, nfiles * 8ull);
        up.add(h->order.p, order.data(), nfiles * 4ull);
        up.add(h->ofile.p, of.data(), nfiles * 16ull);
        rc = upload_cut_tables(h, &up);
        if (rc) return rc;
        // read-boundary grid points k * read_cap of every file (production only)
        h->ngrid = 0;
        std::vector<uint64_t> gbase(nfiles), gpos, gend;
        if (h->params.read_cap && nfiles) {
            const uint64_t cap = h->params.read_cap;
            uint64_t acc = 0;
            for (uint32_t i = 0; i < nfiles; i++) {
                gbase[i] = acc;
                const uint64_t nk = (file_len[i] + cap - 1) / cap;
                for (uint64_t k = 0; k < nk; k++) {
                    gpos.push_back(file_off[i] + k * cap);
                    gend.push_back(file_off[i] + file_len[i]);
                }
                acc += nk;
            }
            if (acc > 0xffffffffull) return SYNCR_CDC_EINVAL;
            h->ngrid = (uint32_t)acc;
            CHECK_HIP(h->gbase.ensure(nfiles * 8ull));
            CHECK_HIP(h->gpos.ensure(std::max<uint64_t>(acc, 1) * 8));
            CHECK_HIP(h->gend.ensure(std::max<uint64_t>(acc, 1) * 8));
            CHECK_HIP(h->gfix.ensure(std::max<uint64_t>(acc, 1)));
            up.add(h->gbase.p, gbase.data(), nfiles * 8ull);
            up.add(h->gpos.p, gpos.data(), acc * 8);
            up.add(h->gend.p, gend.data(), acc * 8);
        }
        up.zero(zblock(h, 0), zeroed_bytes(h));      // the first launch's counter block, in the same dispatch
        CHECK_HIP(upload(h, up, false));
        h->zclean[0] = true;
        h->planned = true;
        return SYNCR_CDC_OK;
    } catch (const std::bad_alloc &) {
        return SYNCR_CDC_ENOMEM;
    } catch (...) {
        return SYNCR_CDC_EIO;
    }
}

int32_t syncr_cdc_launch(syncr_cdc *h, const uint8_t *d_bytes, void *stream) {
    if (!h) return SYNCR_CDC_EINVAL;
    if (!h->planned) return SYNCR_CDC_ESTATE;
    if (h->span && !d_bytes) return SYNCR_CDC_EINVAL;
    if (((uintptr_t)d_bytes & 15u) != 0) return SYNCR_CDC_EINVAL;
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    h->hash_on = false;
    h->reruns = 0;                         // re-runs are counted from the caller's launch on
    return do_launch(h, d_bytes, s);
}

int32_t syncr_cdc_launch_hashed(syncr_cdc *h, const uint8_t *d_bytes, void *stream) {
    if (!h) return SYNCR_CDC_EINVAL;
    if (!h->planned) return SYNCR_CDC_ESTATE;
    if (h->span && !d_bytes) return SYNCR_CDC_EINVAL;
    if (((uintptr_t)d_bytes & 15u) != 0) return SYNCR_CDC_EINVAL;
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    h->hash_on = true;
    h->reruns = 0;                         // re-runs are counted from the caller's launch on
    return do_launch(h, d_bytes, s);
}

namespace {
// the launch's cut slots (and, after a hashed launch, its hash counters and
// hashes) into the fetch cache by `dn`; with small_only, only when the group
// stays within one copy dispatch
bool add_results(syncr_cdc *h, CopyGroup &dn, bool small_only) {
    auto &fc = h->fc;
    const uint64_t bytes = h->total_cut_cap * (sizeof(DevCut) + (h->hash_on ? 32u : 0u)) + sizeof fc.hc;
    if (small_only && (dn.total + bytes > KCOPY_MAX || dn.items.size() + 3 > (size_t)COPY_MAX)) return false;
    fc.all.resize(h->total_cut_cap);
    dn.add(h->cuts.p, fc.all.data(), h->total_cut_cap * sizeof(DevCut));
    if (h->hash_on) {
        fc.hs.resize(h->total_cut_cap * 32);
        dn.add(h->hctr.p, fc.hc, sizeof fc.hc);
        dn.add(h->hashes.p, fc.hs.data(), fc.hs.size());
    }
    return true;
}

// fetch / fetch_hashed: exactly one of out / hout is used (the other may be null)
int32_t fetch_impl(syncr_cdc *h, syncr_cut *out, syncr_chunk_info *hout, bool hashed, uint64_t cap,
                   uint64_t *per_file_count, uint64_t *n_out) {
    if (!h) return SYNCR_CDC_EINVAL;
    if (!h->launched) return SYNCR_CDC_ESTATE;
    if (hashed && !h->hash_on) return SYNCR_CDC_ESTATE;
    try {
        CHECK_HIP(hipSetDevice(h->device));
        for (int attempt = 0; attempt < 8; attempt++) {
            if (h->last_stream) CHECK_HIP(hipStreamSynchronize(h->last_stream));
            auto &fc = h->fc;
            if (!fc.valid) {
                // the launch's counters, per-file counts and split counters in one
                // copy group (with a small launch's results)
                fc.counts.assign(h->nfiles, 0);
                CopyGroup dn;
                dn.add(zblock(h, h->zlast), fc.ctr, 16);
                dn.add(h->counts.p, fc.counts.data(), h->nfiles * 8ull);
                dn.add(zblock(h, h->zlast) + split_ctr_offset(h), fc.sp, sizeof fc.sp);
                fc.cuts = add_results(h, dn, true);
                CHECK_HIP(download(h, dn));
                fc.valid = true;
            }
            const uint32_t *ctr = fc.ctr;
            const std::vector<uint64_t> &counts = fc.counts;
            const uint32_t *sp = fc.sp;
            const uint64_t ncand = (uint64_t)ctr[CTR_CANDS_LO] | ((uint64_t)ctr[CTR_CANDS_HI] << 32);
            // for the next launch (also a re-run below): >= 64 Ki candidates at >= 1
            // per 16 KiB (random data: ~1 per MiB at chunk_bits 20)
            const bool hint = ncand >= std::max<uint64_t>(65536ull, h->span >> 14);
            if (hint != h->split_hint) {
                h->split_hint = hint;
                int32_t rc = ensure_split(h);
                if (rc) return rc;
            }
#ifdef SYNCR_CDC_DEV
            if (getenv("SYNCR_CDC_DEBUG_FETCH")) {
                fprintf(stderr, "fetch attempt %d: flags %u ncand %llu dense %u cand_cap %llu dense_cap %u seg_cap %u | "
                        "pub %u split %u reserved %u head %u done %u | counts",
                        attempt, ctr[CTR_FLAGS], (unsigned long long)ncand, ctr[CTR_DENSE],
                        (unsigned long long)h->cand_cap, h->dense_cap, h->seg_cap, sp[0], sp[1], sp[SPL_RESERVED],
                        sp[SPL_HEAD], sp[SPL_DONE]);
                for (uint32_t i = 0; i < h->nfiles && i < 8; i++)
                    fprintf(stderr, " %llu/%u", (unsigned long long)counts[i], h->h_cut_cap[i]);
                fprintf(stderr, "\n");
            }
#endif
            if (ctr[CTR_FLAGS] & FLAG_SCHED_STUCK) return SYNCR_CDC_EIO;   // (never: see cdc_internal.h)
            bool rerun = false;
            if (h->last_dense_off && ctr[CTR_DENSE]) {       // dense tiles the launch left unpassed
                h->dense_hint = true;
                rerun = true;
            }
            if (ctr[CTR_FLAGS] & FLAG_DENSE_OVERFLOW) {
                // the counter holds every dense tile of the launch: enough (the list has
                // at most one slot per tile; the dev library's DenseSlots scans pad
                // 8-slot chunks, up to 8 per scan wave)
                const uint64_t need = (uint64_t)ctr[CTR_DENSE] + ctr[CTR_DENSE] / 4 + 16;
#ifdef SYNCR_CDC_DEV
                const uint64_t lim = (uint64_t)h->ntiles + 8ull * h->scan_grid + 64;
#else
                const uint64_t lim = (uint64_t)h->ntiles + 64;
#endif
                const uint32_t want = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(need, 2ull * h->dense_cap), lim);
                int32_t rc = ensure_dense(h, want);
                if (rc) return rc;
                rerun = true;
            }
            if (ctr[CTR_FLAGS] & FLAG_CAND_OVERFLOW) {
                int32_t rc = ensure_cand(h, ncand + ncand / 8 + 1024);
                if (rc) return rc;
                rerun = true;
            }
            if (!rerun && (ctr[CTR_FLAGS] & FLAG_CUT_OVERFLOW)) {
                for (uint32_t i = 0; i < h->nfiles; i++)
                    if (counts[i] > h->h_cut_cap[i]) {
                        if (counts[i] > 0xffffffffull) return SYNCR_CDC_ERANGE;
                        h->h_cut_cap[i] = (uint32_t)counts[i];
                    }
                int32_t rc = upload_cut_tables(h);
                if (rc) return rc;
                rerun = true;
            }
            if (rerun) {
                int32_t rc = do_launch(h, h->last_bytes, h->last_stream ? h->last_stream : h->stream);
                if (rc) return rc;
                h->reruns++;
                continue;
            }
            // the launch is complete (synchronised above, nothing enqueued since): the
            // caller's stream is not touched again (the header lets the caller destroy it
            // after this fetch), so later plans / launches / fetches never use it
            h->last_stream = nullptr;
            h->stats[0] = ncand;
            h->stats[2] = h->ntiles;
            h->stats[3] = ctr[CTR_FLAGS];
            {
                // dense tiles the dense pass rolled (in the development library's
                // DenseSlots scans the list counter also counts unused 8-slot padding)
                h->stats[1] = ctr[CTR_DENSE] ? sp[SPL_DENSE_TILES] : 0u;
                // a batch with >= 1 % dense tiles: the next launch scans by tiles (stream tiles
                // branch on every dirty 16-byte group: 6 % slower on the dense workload)
                h->dense_heavy = (uint64_t)h->stats[1] * 100u >= (uint64_t)std::max<uint32_t>(h->ntiles, 1u);
                h->split_stats[0] = h->split_launched ? 4ull * h->split_blocks : 0ull;   // worker waves
                h->split_stats[1] = sp[SPL_PUB64 + 1];          // split files (high half of the 64-bit count)
                h->split_stats[2] = std::min<uint32_t>(sp[SPL_RESERVED], h->seg_cap);
                h->split_stats[3] = sp[SPL_WALKED];
                h->split_stats[4] = sp[SPL_ADOPTED];
                h->split_stats[5] = sp[SPL_GIVEUP];
            }
            uint64_t total = 0;
            for (uint32_t i = 0; i < h->nfiles; i++) total += counts[i];
            if (per_file_count)
                for (uint32_t i = 0; i < h->nfiles; i++) per_file_count[i] = counts[i];
            if (n_out) *n_out = total;
            if (total > cap || (total && !(hashed ? (void *)hout : (void *)out))) return SYNCR_CDC_ERANGE;
            if (total) {
                // the cut slots (and hash counters and hashes) in one copy group
                if (!fc.cuts) {
                    CopyGroup dn;
                    add_results(h, dn, false);
                    CHECK_HIP(download(h, dn));
                    fc.cuts = true;
                }
                const std::vector<DevCut> &all = fc.all;
                const std::vector<uint8_t> &hs = fc.hs;
                const uint64_t *hc = fc.hc;
                if (hashed && (hc[B3C_FLAGS] || hc[B3C_ITEMS] > h->items_cap || hc[B3C_TREES] > h->trees_cap ||
                               hc[B3C_PIECES] > h->pieces_cap))
                    return SYNCR_CDC_EIO;              // capacities are exact bounds: cannot happen
                uint64_t o = 0;
                for (uint32_t i = 0; i < h->nfiles; i++) {
                    const uint64_t b = h->h_cut_base[i];
                    for (uint64_t j = 0; j < counts[i]; j++, o++) {
                        const DevCut &c = all[b + j];
                        if (hashed) {
                            hout[o].offset = c.offset;
                            hout[o].len = c.len;
                            hout[o].file = c.file;
                            memcpy(hout[o].hash, hs.data() + (b + j) * 32, 32);
                        } else {
                            out[o].offset = c.offset;
                            out[o].len = c.len;
                            out[o].file = c.file;
                        }
                    }
                }
            }
            return SYNCR_CDC_OK;
        }
        return SYNCR_CDC_EIO;
    } catch (const std::bad_alloc &) {
        return SYNCR_CDC_ENOMEM;
    } catch (...) {
        return SYNCR_CDC_EIO;
    }
}
}  // namespace

int32_t syncr_cdc_fetch(syncr_cdc *h, syncr_cut *out, uint64_t cap, uint64_t *per_file_count,
                        uint64_t *n_out) {
    return fetch_impl(h, out, nullptr, false, cap, per_file_count, n_out);
}

int32_t syncr_cdc_fetch_hashed(syncr_cdc *h, syncr_chunk_info *out, uint64_t cap, uint64_t *per_file_count,
                               uint64_t *n_out) {
    return fetch_impl(h, nullptr, out, true, cap, per_file_count, n_out);
}

int32_t syncr_cdc_chunk_batch_device(syncr_cdc *h, const uint8_t *d_bytes, uint64_t span,
                                     const uint64_t *file_off, const uint64_t *file_len,
                                     uint32_t nfiles, syncr_cut *out, uint64_t cap,
                                     uint64_t *per_file_count, uint64_t *n_out, void *stream) {
    int32_t rc = syncr_cdc_plan(h, file_off, file_len, nfiles, span);
    if (rc) return rc;
    rc = syncr_cdc_launch(h, d_bytes, stream);
    if (rc) return rc;
    return syncr_cdc_fetch(h, out, cap, per_file_count, n_out);
}

int32_t syncr_cdc_chunk_batch_host(syncr_cdc *h, const uint8_t *data, uint64_t span,
                                   const uint64_t *file_off, const uint64_t *file_len,
                                   uint32_t nfiles, syncr_cut *out, uint64_t cap,
                                   uint64_t *per_file_count, uint64_t *n_out) {
    if (!h || (span && !data)) return SYNCR_CDC_EINVAL;
    CHECK_HIP(hipSetDevice(h->device));
    CHECK_HIP(h->stage.ensure(std::max<uint64_t>(span, 16)));
    if (span) CHECK_HIP(hipMemcpyAsync(h->stage.p, data, span, hipMemcpyHostToDevice, h->stream));
    return syncr_cdc_chunk_batch_device(h, h->stage.as<uint8_t>(), span, file_off, file_len, nfiles,
                                        out, cap, per_file_count, n_out, h->stream);
}

int32_t syncr_cdc_chunk_batch_host_hashed(syncr_cdc *h, const uint8_t *data, uint64_t span,
                                          const uint64_t *file_off, const uint64_t *file_len,
                                          uint32_t nfiles, syncr_chunk_info *out, uint64_t cap,
                                          uint64_t *per_file_count, uint64_t *n_out) {
    if (!h || (span && !data)) return SYNCR_CDC_EINVAL;
    CHECK_HIP(hipSetDevice(h->device));
    CHECK_HIP(h->stage.ensure(std::max<uint64_t>(span, 16)));
    if (span) CHECK_HIP(hipMemcpyAsync(h->stage.p, data, span, hipMemcpyHostToDevice, h->stream));
    int32_t rc = syncr_cdc_plan(h, file_off, file_len, nfiles, span);
    if (rc) return rc;
    rc = syncr_cdc_launch_hashed(h, h->stage.as<uint8_t>(), h->stream);
    if (rc) return rc;
    return syncr_cdc_fetch_hashed(h, out, cap, per_file_count, n_out);
}

int32_t syncr_cdc_chunk_host_hashed(syncr_cdc *h, const uint8_t *data, uint64_t len, syncr_chunk_info *out,
                                    uint64_t cap, uint64_t *n_out) {
    const uint64_t off = 0;
    uint64_t cnt = 0;
    return syncr_cdc_chunk_batch_host_hashed(h, data, len, &off, &len, 1, out, cap, &cnt, n_out);
}

int32_t syncr_cdc_chunk_host(syncr_cdc *h, const uint8_t *data, uint64_t len, syncr_cut *out,
                             uint64_t cap, uint64_t *n_out) {
    const uint64_t off = 0;
    uint64_t cnt = 0;
    int32_t rc = syncr_cdc_chunk_batch_host(h, data, len, &off, &len, 1, out, cap, &cnt, n_out);
    return rc;
}

int32_t syncr_cdc_device_alloc(syncr_cdc *h, uint64_t bytes, void **d_ptr) {
    if (!h || !d_ptr) return SYNCR_CDC_EINVAL;
    CHECK_HIP(hipSetDevice(h->device));
    CHECK_HIP(hipMalloc(d_ptr, std::max<uint64_t>(bytes, 16)));
    return SYNCR_CDC_OK;
}

int32_t syncr_cdc_device_free(syncr_cdc *h, void *d_ptr) {
    if (!h) return SYNCR_CDC_EINVAL;
    CHECK_HIP(hipSetDevice(h->device));
    CHECK_HIP(hipFree(d_ptr));
    return SYNCR_CDC_OK;
}

int32_t syncr_cdc_host_alloc_pinned(syncr_cdc *h, uint64_t bytes, void **ptr) {
    if (!h || !ptr) return SYNCR_CDC_EINVAL;
    CHECK_HIP(hipSetDevice(h->device));
    CHECK_HIP(hipHostMalloc(ptr, std::max<uint64_t>(bytes, 16), hipHostMallocDefault));
    return SYNCR_CDC_OK;
}

int32_t syncr_cdc_host_free_pinned(syncr_cdc *h, void *ptr) {
    if (!h) return SYNCR_CDC_EINVAL;
    CHECK_HIP(hipHostFree(ptr));
    return SYNCR_CDC_OK;
}

int32_t syncr_cdc_memcpy_h2d(syncr_cdc *h, void *d_dst, const void *src, uint64_t bytes, void *stream) {
    if (!h || (bytes && (!d_dst || !src))) return SYNCR_CDC_EINVAL;
    CHECK_HIP(hipSetDevice(h->device));
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    if (bytes) CHECK_HIP(hipMemcpyAsync(d_dst, src, bytes, hipMemcpyHostToDevice, s));
    return SYNCR_CDC_OK;
}

int32_t syncr_cdc_memcpy_d2h(syncr_cdc *h, void *dst, const void *d_src, uint64_t bytes, void *stream) {
    if (!h || (bytes && (!dst || !d_src))) return SYNCR_CDC_EINVAL;
    CHECK_HIP(hipSetDevice(h->device));
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    if (bytes) CHECK_HIP(hipMemcpyAsync(dst, d_src, bytes, hipMemcpyDeviceToHost, s));
    return SYNCR_CDC_OK;
}

int32_t syncr_cdc_memcpy_d2d(syncr_cdc *h, void *d_dst, const void *d_src, uint64_t bytes, void *stream) {
    if (!h || (bytes && (!d_dst || !d_src))) return SYNCR_CDC_EINVAL;
    CHECK_HIP(hipSetDevice(h->device));
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    if (bytes) CHECK_HIP(hipMemcpyAsync(d_dst, d_src, bytes, hipMemcpyDeviceToDevice, s));
    return SYNCR_CDC_OK;
}

namespace {
// Wait for this handle's work only (its own stream and the stream of its last
// launch): other handles and ingest pipelines on the device keep running.
hipError_t sync_handle(syncr_cdc *h) {
    hipError_t e = hipSuccess;
    if (h->last_stream && h->last_stream != h->stream) e = hipStreamSynchronize(h->last_stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    return e;
}
}  // namespace

int32_t syncr_cdc_synchronize(syncr_cdc *h) {
    if (!h) return SYNCR_CDC_EINVAL;
    CHECK_HIP(hipSetDevice(h->device));
    CHECK_HIP(sync_handle(h));
    return SYNCR_CDC_OK;
}

void *syncr_cdc_stream(syncr_cdc *h) { return h ? (void *)h->stream : nullptr; }

int32_t syncr_cdc_gen_corpus(syncr_cdc *h, uint8_t *d_bytes, const uint64_t *file_off,
                             const uint64_t *file_len, const uint64_t *file_index,
                             uint32_t nfiles, uint64_t first_index, void *stream) {
    if (!h || (nfiles && (!file_off || !file_len || !d_bytes))) return SYNCR_CDC_EINVAL;
    try {
        CHECK_HIP(hipSetDevice(h->device));
        hipStream_t s = stream ? (hipStream_t)stream : h->stream;
        // xorshift64 step as 64 GF(2) columns, squared GEN_JUMPS times
        std::vector<uint64_t> jump((size_t)GEN_JUMPS * 64);
        auto step = [](uint64_t x) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
        auto apply = [](const uint64_t *cols, uint64_t x) {
            uint64_t y = 0;
            for (int b = 0; b < 64; b++) if ((x >> b) & 1) y ^= cols[b];
            return y;
        };
        for (int b = 0; b < 64; b++) jump[b] = step(1ull << b);
        for (int k = 1; k < GEN_JUMPS; k++)
            for (int b = 0; b < 64; b++)
                jump[(size_t)k * 64 + b] = apply(&jump[(size_t)(k - 1) * 64], jump[(size_t)(k - 1) * 64 + b]);
        std::vector<uint64_t> seg(nfiles + 1, 0);
        for (uint32_t i = 0; i < nfiles; i++) {
            if (file_len[i] >> GEN_JUMPS) return SYNCR_CDC_EINVAL;
            seg[i + 1] = seg[i] + (file_len[i] + GEN_SEG - 1) / GEN_SEG;
        }
        const uint64_t nseg = seg[nfiles];
        if (!nseg) return SYNCR_CDC_OK;
        DevBuf dj, dfo, dfl, dsp, dfi;
        int32_t rc = SYNCR_CDC_OK;
        hipError_t e = hipSuccess;
        do {
            if ((e = dj.ensure(jump.size() * 8)) != hipSuccess) break;
            if ((e = dfo.ensure(nfiles * 8ull)) != hipSuccess) break;
            if ((e = dfl.ensure(nfiles * 8ull)) != hipSuccess) break;
            if ((e = dsp.ensure((nfiles + 1) * 8ull)) != hipSuccess) break;
            if (file_index) {
                if ((e = dfi.ensure(nfiles * 8ull)) != hipSuccess) break;
                if ((e = hipMemcpyAsync(dfi.p, file_index, nfiles * 8ull, hipMemcpyHostToDevice, s)) != hipSuccess) break;
            }
            if ((e = hipMemcpyAsync(dj.p, jump.data(), jump.size() * 8, hipMemcpyHostToDevice, s)) != hipSuccess) break;
            if ((e = hipMemcpyAsync(dfo.p, file_off, nfiles * 8ull, hipMemcpyHostToDevice, s)) != hipSuccess) break;
            if ((e = hipMemcpyAsync(dfl.p, file_len, nfiles * 8ull, hipMemcpyHostToDevice, s)) != hipSuccess) break;
            if ((e = hipMemcpyAsync(dsp.p, seg.data(), (nfiles + 1) * 8ull, hipMemcpyHostToDevice, s)) != hipSuccess) break;
            if ((e = launch_gen(d_bytes, dfo.as<uint64_t>(), dfl.as<uint64_t>(),
                                file_index ? dfi.as<uint64_t>() : nullptr, dsp.as<uint64_t>(), nfiles,
                                nseg, first_index, dj.as<uint64_t>(), s)) != hipSuccess) break;
            e = hipStreamSynchronize(s);
        } while (0);
        if (e != hipSuccess) rc = hip_err(e);
        dj.release(); dfo.release(); dfl.release(); dsp.release(); dfi.release();
        return rc;
    } catch (const std::bad_alloc &) {
        return SYNCR_CDC_ENOMEM;
    }
}

int32_t syncr_cdc_read_probe(syncr_cdc *h, const uint8_t *d_bytes, uint64_t bytes, uint32_t reps,
                             int32_t nt, double *ms2) {
    if (!h || !d_bytes || !ms2 || !reps || bytes < 16) return SYNCR_CDC_EINVAL;
    CHECK_HIP(hipSetDevice(h->device));
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess || cus <= 0)
        cus = 256;
    const uint64_t blocks_needed = (bytes / 16 + 4095) / 4096;     // 64 KiB per block step
    const uint32_t grid = (uint32_t)std::min<uint64_t>(blocks_needed, (uint64_t)cus * 8);
    DevBuf sink;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    hipError_t e = hipSuccess;
    double best = 1e30, sum = 0;
    do {
        if ((e = sink.ensure((size_t)grid * 4)) != hipSuccess) break;
        if ((e = hipEventCreateWithFlags(&e0, hipEventDisableSystemFence)) != hipSuccess) break;
        if ((e = hipEventCreateWithFlags(&e1, hipEventDisableSystemFence)) != hipSuccess) break;
        if ((e = launch_read_probe(d_bytes, bytes, nt != 0, grid, sink.as<uint32_t>(), h->stream)) != hipSuccess) break;
        for (uint32_t r = 0; r < reps && e == hipSuccess; ++r) {
            if ((e = hipEventRecord(e0, h->stream)) != hipSuccess) break;
            if ((e = launch_read_probe(d_bytes, bytes, nt != 0, grid, sink.as<uint32_t>(), h->stream)) != hipSuccess) break;
            if ((e = hipEventRecord(e1, h->stream)) != hipSuccess) break;
            if ((e = hipEventSynchronize(e1)) != hipSuccess) break;
            float f = 0;
            if ((e = hipEventElapsedTime(&f, e0, e1)) != hipSuccess) break;
            best = std::min(best, (double)f);
            sum += f;
        }
    } while (0);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    sink.release();
    if (e != hipSuccess) return hip_err(e);
    ms2[0] = best;
    ms2[1] = sum / reps;
    return SYNCR_CDC_OK;
}

int32_t syncr_cdc_set_timing(syncr_cdc *h, int32_t enable) {
    if (!h || enable < 0 || enable > 4) return SYNCR_CDC_EINVAL;
    CHECK_HIP(hipSetDevice(h->device));
    drain_timing(h);
    if (enable == 4) {
        CHECK_HIP(h->tacc.ensure(16));
        CHECK_HIP(sync_handle(h));                    // no earlier launch may still add to the sums
        CHECK_HIP(hipMemset(h->tacc.p, 0, 16));
    }
    h->timing = enable != 0;
    h->timing_scan_only = enable >= 2;
    h->timing_clock = enable == 4;
    for (double &m : h->ms) m = 0;
    h->timed_launches = 0;
    return SYNCR_CDC_OK;
}

namespace {
// the device-clock sums into ms[0] / timed_launches (timing mode 4)
int32_t read_clock_times(syncr_cdc *h) {
    if (!h->timing_clock || !h->tacc.p) return SYNCR_CDC_OK;
    CHECK_HIP(sync_handle(h));
    uint64_t v[2] = {0, 0};
    CHECK_HIP(hipMemcpy(v, h->tacc.p, 16, hipMemcpyDeviceToHost));
    h->ms[0] = (double)v[0] / (double)h->wall_khz;
    h->timed_launches = v[1];
    return SYNCR_CDC_OK;
}
}  // namespace

int32_t syncr_cdc_kernel_times(syncr_cdc *h, double *ms3, uint64_t *launches) {
    if (!h) return SYNCR_CDC_EINVAL;
    (void)hipSetDevice(h->device);
    drain_timing(h);
    int32_t rc = read_clock_times(h);
    if (rc) return rc;
    if (ms3) for (int k = 0; k < 3; k++) ms3[k] = h->ms[k];
    if (launches) *launches = h->timed_launches;
    return SYNCR_CDC_OK;
}

int32_t syncr_cdc_kernel_times_ex(syncr_cdc *h, double *ms, uint32_t n, uint64_t *launches) {
    if (!h || (n && !ms)) return SYNCR_CDC_EINVAL;
    (void)hipSetDevice(h->device);
    drain_timing(h);
    int32_t rc = read_clock_times(h);
    if (rc) return rc;
    for (uint32_t k = 0; k < n; k++) ms[k] = k < (uint32_t)NPHASE ? h->ms[k] : 0.0;
    if (launches) *launches = h->timed_launches;
    return SYNCR_CDC_OK;
}

int32_t syncr_cdc_split_stats(syncr_cdc *h, uint64_t *stats6) {
    if (!h || !stats6) return SYNCR_CDC_EINVAL;
    for (int k = 0; k < 6; k++) stats6[k] = h->split_stats[k];
    return SYNCR_CDC_OK;
}

int32_t syncr_cdc_fetch_reruns(syncr_cdc *h, uint64_t *reruns) {
    if (!h || !reruns) return SYNCR_CDC_EINVAL;
    *reruns = h->reruns;
    return SYNCR_CDC_OK;
}

int32_t syncr_cdc_last_scan(const syncr_cdc *h, uint64_t *info4, const char **name) {
    if (!h) return SYNCR_CDC_EINVAL;
    if (info4) for (int k = 0; k < 4; k++) info4[k] = h->scan_info[k];
    if (name) {
        switch ((int)h->scan_info[0]) {
            case SYNCR_CDC_SCAN_STREAM_TILES: *name = "cdc_scan_st_kernel"; break;
            case SYNCR_CDC_SCAN_CU:
            case SYNCR_CDC_SCAN_TILES: *name = "cdc_scan_kernel"; break;
            case SYNCR_CDC_SCAN_DEV: *name = "dev"; break;
            default: *name = ""; break;
        }
    }
    return SYNCR_CDC_OK;
}

int32_t syncr_cdc_last_stats(syncr_cdc *h, uint64_t *stats4) {
    if (!h || !stats4) return SYNCR_CDC_EINVAL;
    for (int k = 0; k < 4; k++) stats4[k] = h->stats[k];
    return SYNCR_CDC_OK;
}

}  // extern "C"

extern "C" int32_t syncr_cdc_get_info(const syncr_cdc *h, uint64_t *info8) {
    if (!h || !info8) return SYNCR_CDC_EINVAL;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess) cus = 0;
    info8[0] = (uint64_t)(h->geom.kind * 1000 + h->geom.param);
    info8[1] = (uint64_t)scan_tile_bytes(h->geom);
    info8[2] = h->scan_grid;
    info8[3] = (uint64_t)cus;
    info8[4] = (uint64_t)scan_blocks_per_cu(h->geom);
    info8[5] = (uint64_t)scan_lds_bytes(h->geom);
    info8[6] = (uint64_t)h->device;
    info8[7] = SYNCR_CDC_ABI_VERSION;
    return SYNCR_CDC_OK;
}

// ---------------------------------------------------------------------------
// Wire / on-disk text of chunk lists (include/syncr_cdc.h, SYNCR_FMT_*).
// ---------------------------------------------------------------------------
namespace {

// base64 URL_SAFE with padding (base64 0.22 general_purpose::URL_SAFE,
// util::hash_to_base64, src/util.rs:62-64): 32 bytes -> 44 chars
void b64url32(const uint8_t h[32], char out[44]) {
    static const char A[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";
    int o = 0;
    for (int i = 0; i < 30; i += 3) {
        const uint32_t v = (uint32_t)h[i] << 16 | (uint32_t)h[i + 1] << 8 | h[i + 2];
        out[o++] = A[v >> 18];
        out[o++] = A[(v >> 12) & 63];
        out[o++] = A[(v >> 6) & 63];
        out[o++] = A[v & 63];
    }
    const uint32_t v = (uint32_t)h[30] << 16 | (uint32_t)h[31] << 8;
    out[o++] = A[v >> 18];
    out[o++] = A[(v >> 12) & 63];
    out[o++] = A[(v >> 6) & 63];
    out[o++] = '=';
}

struct Sink {
    char *out;
    uint64_t cap, n = 0;
    void put(const char *s, size_t k) {
        if (n + k <= cap && out) memcpy(out + n, s, k);
        n += k;
    }
    void str(const char *s) { put(s, strlen(s)); }
    void u64(uint64_t v) {
        char b[24];
        int k = 0;
        do { b[k++] = (char)('0' + v % 10); v /= 10; } while (v);
        char r[24];
        for (int i = 0; i < k; i++) r[i] = b[k - 1 - i];
        put(r, (size_t)k);
    }
};

}  // namespace

extern "C" int32_t syncr_cdc_format_chunks(const syncr_chunk_info *c, uint64_t n, int32_t format, char *out,
                                           uint64_t cap, uint64_t *len_out) {
    if ((n && !c) || (format != SYNCR_FMT_LIST_LINES && format != SYNCR_FMT_HASHCHUNKS)) return SYNCR_CDC_EINVAL;
    Sink s{out, out ? cap : 0};
    char h[44];
    if (format == SYNCR_FMT_HASHCHUNKS) s.put("[", 1);
    for (uint64_t i = 0; i < n; i++) {
        b64url32(c[i].hash, h);
        if (format == SYNCR_FMT_LIST_LINES) {            // v3_server.rs:148-153, BTreeMap key order
            s.str("{\"hsh\":\"");
            s.put(h, 44);
            s.str("\",\"len\":");
            s.u64(c[i].len);
            s.str(",\"off\":");
            s.u64(c[i].offset);
            s.str(",\"typ\":\"C\"}\n");
        } else {                                         // types.rs:122-127, field order h, of, sz
            if (i) s.put(",", 1);
            s.str("{\"h\":\"");
            s.put(h, 44);
            s.str("\",\"of\":");
            s.u64(c[i].offset);
            s.str(",\"sz\":");
            s.u64(c[i].len);
            s.put("}", 1);
        }
    }
    if (format == SYNCR_FMT_HASHCHUNKS) s.put("]", 1);
    if (len_out) *len_out = s.n;
    return s.n > s.cap ? SYNCR_CDC_ERANGE : SYNCR_CDC_OK;
}

#ifdef SYNCR_CDC_DEV
// Development library only: the last launch's resolve timeline (SYNCR_CDC_TRACE=1).
extern "C" int32_t syncr_cdc_dev_trace(syncr_cdc *h, uint64_t *out, uint32_t n) {
    if (!h || !out || !h->dbg.p) return SYNCR_CDC_EINVAL;
    CHECK_HIP(hipSetDevice(h->device));
    CHECK_HIP(hipStreamSynchronize(h->last_stream ? h->last_stream : h->stream));
    CHECK_HIP(hipMemcpy(out, h->dbg.p, std::min<uint32_t>(n, DBG_WORDS) * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return SYNCR_CDC_OK;
}
#endif
