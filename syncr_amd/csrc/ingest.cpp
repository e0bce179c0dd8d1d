// ingest.cpp -- batched ingest pipeline over the CDC + BLAKE3 engine.
//
// Replaces the serial per-file loop of the reference's directory walk:
// traverse_and_stream (src/protocol/file_operations.rs:544-715) awaits
// compute_file_chunks (:721-788) for one file at a time (:599-605), each a
// 16 MiB buffer filled by <= 2 MiB tokio reads (:737-738, :776).  Here files are
// appended to pinned staging batches; a sealed batch is copied to the device
// (hipMemcpyAsync) and chunked + hashed on its own handle/stream while the next
// batch fills, so file reads (host), PCIe and the GPU kernels overlap.  Results
// go back per file, in submission order, through the caller's callback on the
// caller's thread.  An unreadable file yields status -errno and no chunks, like
// the reference's warn-and-return-empty (:727-744).
#include <errno.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/syncr_cdc.h"

namespace {

// A few worker threads for large copies/reads into pinned memory (one host
// thread moves ~5-10 GB/s; PCIe Gen5 takes ~55).
class Pool {
  public:
    explicit Pool(unsigned n) {
        for (unsigned i = 0; i < n; i++) th_.emplace_back([this] { run(); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    unsigned size() const { return (unsigned)th_.size(); }
    // run fn(0..n-1) on the pool plus the calling thread; returns when all done
    void parallel(unsigned n, const std::function<void(unsigned)> &fn) {
        if (n <= 1 || th_.empty()) {
            for (unsigned i = 0; i < n; i++) fn(i);
            return;
        }
        std::unique_lock<std::mutex> g(mu_);
        fn_ = &fn;
        next_ = 0;
        total_ = n;
        done_ = 0;
        ++gen_;
        g.unlock();
        cv_.notify_all();
        work();
        g.lock();
        done_cv_.wait(g, [&] { return done_ == total_; });
        fn_ = nullptr;
    }

  private:
    void work() {
        for (;;) {
            unsigned i;
            const std::function<void(unsigned)> *f;
            {
                std::lock_guard<std::mutex> g(mu_);
                if (!fn_ || next_ >= total_) return;
                i = next_++;
                f = fn_;
            }
            (*f)(i);
            std::lock_guard<std::mutex> g(mu_);
            if (++done_ == total_) done_cv_.notify_all();
        }
    }
    void run() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return stop_ || (gen_ != seen && fn_ && next_ < total_); });
                if (stop_) return;
                seen = gen_;
            }
            work();
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(unsigned)> *fn_ = nullptr;
    unsigned next_ = 0, total_ = 0, done_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

struct Slot {
    syncr_cdc *h = nullptr;           // own handle: own plan tables and stream
    uint8_t *host = nullptr;          // pinned staging
    uint8_t *dev = nullptr;
    uint64_t cap = 0, used = 0;
    std::vector<uint64_t> off, len, tag;
    std::vector<int32_t> status;
    // chunk cache: per file, the key to store the result under ("" = none) and
    // its (mtime, size); a cache hit carries its chunks in cbuf[cstart, +ccount)
    std::vector<std::string> key;
    std::vector<uint32_t> mtime;
    std::vector<uint64_t> fsize;
    std::vector<uint8_t> hit;
    std::vector<uint64_t> cstart, ccount;
    std::vector<syncr_chunk_info> cbuf;
    bool inflight = false;
    std::vector<syncr_chunk_info> out;
    std::vector<uint64_t> counts;
};

constexpr uint64_t PAR_COPY = 4ull << 20;   // copies above this are split over the pool
constexpr uint64_t PIECE = 2ull << 20;

}  // namespace

struct syncr_ingest {
    int32_t device = 0;
    syncr_cdc_params params{};
    uint64_t batch = 0;
    std::vector<Slot> slots;
    uint32_t cur = 0;
    syncr_ingest_cb cb = nullptr;
    void *ctx = nullptr;
    Pool *pool = nullptr;
    bool reserved = false;           // reserve() outstanding on slots[cur]
    uint64_t reserved_len = 0;
    uint64_t stats[4] = {0, 0, 0, 0};   // files, bytes, batches, chunks
    int32_t error = 0;                  // sticky engine error
    syncr_cache *cache = nullptr;       // optional (syncr_ingest_set_cache)
    uint64_t cache_hits = 0;
};

namespace {

int32_t hip_rc(hipError_t e) {
    if (e == hipSuccess) return SYNCR_CDC_OK;
    if (e == hipErrorOutOfMemory) return SYNCR_CDC_ENOMEM;
    return SYNCR_CDC_EIO;
}

void free_slot_buffers(syncr_ingest *g, Slot &s) {
    (void)hipSetDevice(g->device);
    if (s.host) (void)hipHostFree(s.host);
    if (s.dev) (void)hipFree(s.dev);
    s.host = s.dev = nullptr;
    s.cap = 0;
}

int32_t ensure_slot(syncr_ingest *g, Slot &s, uint64_t bytes) {
    if (bytes <= s.cap && s.host) return SYNCR_CDC_OK;
    free_slot_buffers(g, s);
    const uint64_t want = std::max<uint64_t>(bytes, 64);
    hipError_t e = hipHostMalloc((void **)&s.host, want, hipHostMallocDefault);
    if (e == hipSuccess) e = hipMalloc((void **)&s.dev, want);
    if (e != hipSuccess) {
        free_slot_buffers(g, s);
        return hip_rc(e);
    }
    s.cap = want;
    return SYNCR_CDC_OK;
}

void par_copy(syncr_ingest *g, uint8_t *dst, const uint8_t *src, uint64_t n) {
    if (n <= PAR_COPY || !g->pool) {
        memcpy(dst, src, n);
        return;
    }
    const unsigned pieces = (unsigned)((n + PIECE - 1) / PIECE);
    g->pool->parallel(pieces, [&](unsigned i) {
        const uint64_t a = (uint64_t)i * PIECE, b = std::min<uint64_t>(n, a + PIECE);
        memcpy(dst + a, src + a, b - a);
    });
}

// wait for a sealed batch, deliver its files in order, reset the slot
int32_t complete(syncr_ingest *g, Slot &s) {
    if (!s.inflight) return SYNCR_CDC_OK;
    s.inflight = false;
    const uint32_t nf = (uint32_t)s.off.size();
    s.counts.assign(std::max<uint32_t>(nf, 1), 0);
    uint64_t n = 0;
    int32_t rc = syncr_cdc_fetch_hashed(s.h, nullptr, 0, s.counts.data(), &n);
    if (rc == SYNCR_CDC_ERANGE || rc == SYNCR_CDC_OK) {
        s.out.resize(std::max<uint64_t>(n, 1));
        rc = syncr_cdc_fetch_hashed(s.h, s.out.data(), s.out.size(), s.counts.data(), &n);
    }
    if (rc) {
        g->error = rc;
        return rc;
    }
    uint64_t o = 0;
    for (uint32_t i = 0; i < nf; i++) {
        const syncr_chunk_info *ci;
        uint64_t c;
        if (s.hit[i]) {                                       // served by the chunk cache
            c = s.ccount[i];
            ci = c ? s.cbuf.data() + s.cstart[i] : nullptr;
        } else {
            c = s.status[i] ? 0 : s.counts[i];
            for (uint64_t k = 0; k < c; k++) s.out[o + k].file = 0;   // one file per callback
            ci = c ? s.out.data() + o : nullptr;
            if (g->cache && !s.status[i] && !s.key[i].empty())
                (void)syncr_cache_put(g->cache, s.key[i].c_str(), s.mtime[i], s.fsize[i], ci, c);
        }
        if (g->cb) g->cb(g->ctx, s.tag[i], s.status[i], ci, c);
        o += s.counts[i];
        g->stats[3] += c;
    }
    s.off.clear();
    s.len.clear();
    s.tag.clear();
    s.status.clear();
    s.key.clear();
    s.mtime.clear();
    s.fsize.clear();
    s.hit.clear();
    s.cstart.clear();
    s.ccount.clear();
    s.cbuf.clear();
    s.used = 0;
    return SYNCR_CDC_OK;
}

int32_t seal(syncr_ingest *g, Slot &s) {
    if (s.off.empty()) return SYNCR_CDC_OK;
    int32_t rc = syncr_cdc_plan(s.h, s.off.data(), s.len.data(), (uint32_t)s.off.size(), s.used);
    if (rc) return g->error = rc;
    void *stream = syncr_cdc_stream(s.h);
    rc = syncr_cdc_memcpy_h2d(s.h, s.dev, s.host, s.used, stream);
    if (rc) return g->error = rc;
    rc = syncr_cdc_launch_hashed(s.h, s.dev, stream);
    if (rc) return g->error = rc;
    s.inflight = true;
    g->stats[2]++;
    return SYNCR_CDC_OK;
}

// make slots[cur] ready to take `len` more bytes (sealing / completing as needed)
int32_t room(syncr_ingest *g, uint64_t len) {
    Slot *s = &g->slots[g->cur];
    if (s->used && s->used + len > s->cap) {
        int32_t rc = seal(g, *s);
        if (rc) return rc;
        g->cur = (g->cur + 1) % (uint32_t)g->slots.size();
        s = &g->slots[g->cur];
    }
    int32_t rc = complete(g, *s);
    if (rc) return rc;
    if (!s->used && len > s->cap) return ensure_slot(g, *s, len);   // a file bigger than a batch
    return SYNCR_CDC_OK;
}

void record(Slot &s, uint64_t len, uint64_t tag, int32_t status, const char *key = nullptr,
            uint32_t mtime = 0, uint64_t fsize = 0) {
    s.off.push_back(s.used);
    s.len.push_back(status ? 0 : len);
    s.tag.push_back(tag);
    s.status.push_back(status);
    s.key.emplace_back(key ? key : "");
    s.mtime.push_back(mtime);
    s.fsize.push_back(fsize);
    s.hit.push_back(0);
    s.cstart.push_back(0);
    s.ccount.push_back(0);
    if (!status) s.used += len;
}

}  // namespace

extern "C" {

int32_t syncr_ingest_open(int32_t device, const syncr_cdc_params *p, uint64_t batch_bytes, uint32_t depth,
                          uint32_t copy_threads, syncr_ingest_cb cb, void *ctx, syncr_ingest **out) {
    if (!out) return SYNCR_CDC_EINVAL;
    *out = nullptr;
    if (depth < 1 || depth > 8 || batch_bytes < 4096) return SYNCR_CDC_EINVAL;
    syncr_ingest *g = new (std::nothrow) syncr_ingest();
    if (!g) return SYNCR_CDC_ENOMEM;
    g->device = device;
    if (p) g->params = *p; else syncr_cdc_default_params(&g->params);
    g->batch = batch_bytes;
    g->cb = cb;
    g->ctx = ctx;
    try {
        g->slots.resize(depth);
        for (Slot &s : g->slots) {
            int32_t rc = syncr_cdc_open(device, &g->params, &s.h);
            if (rc == SYNCR_CDC_OK) rc = ensure_slot(g, s, batch_bytes);
            if (rc) {
                syncr_ingest_close(g);
                return rc;
            }
        }
        if (copy_threads > 1) g->pool = new Pool(std::min<uint32_t>(copy_threads, 64) - 1);
    } catch (...) {
        syncr_ingest_close(g);
        return SYNCR_CDC_ENOMEM;
    }
    *out = g;
    return SYNCR_CDC_OK;
}

int32_t syncr_ingest_reserve(syncr_ingest *g, uint64_t len, uint8_t **dst) {
    if (!g || !dst || g->reserved) return g ? (g->reserved ? SYNCR_CDC_ESTATE : SYNCR_CDC_EINVAL) : SYNCR_CDC_EINVAL;
    if (g->error) return g->error;
    int32_t rc = room(g, len);
    if (rc) return rc;
    Slot &s = g->slots[g->cur];
    *dst = s.host + s.used;
    g->reserved = true;
    g->reserved_len = len;
    return SYNCR_CDC_OK;
}

int32_t syncr_ingest_commit(syncr_ingest *g, uint64_t tag) {
    if (!g) return SYNCR_CDC_EINVAL;
    if (!g->reserved) return SYNCR_CDC_ESTATE;
    g->reserved = false;
    record(g->slots[g->cur], g->reserved_len, tag, 0);
    g->stats[0]++;
    g->stats[1] += g->reserved_len;
    return SYNCR_CDC_OK;
}

int32_t syncr_ingest_submit(syncr_ingest *g, const uint8_t *data, uint64_t len, uint64_t tag) {
    if (!g || (len && !data)) return SYNCR_CDC_EINVAL;
    uint8_t *dst = nullptr;
    int32_t rc = syncr_ingest_reserve(g, len, &dst);
    if (rc) return rc;
    par_copy(g, dst, data, len);
    return syncr_ingest_commit(g, tag);
}

int32_t syncr_ingest_submit_file(syncr_ingest *g, const char *path, uint64_t tag) {
    if (!g || !path) return SYNCR_CDC_EINVAL;
    if (g->reserved) return SYNCR_CDC_ESTATE;
    if (g->error) return g->error;
    const int fd = open(path, O_RDONLY | O_CLOEXEC);
    struct stat st;
    int32_t status = 0;
    if (fd < 0) status = -errno;
    else if (fstat(fd, &st) != 0) status = -errno;
    if (status) {                                    // file_operations.rs:727-733: empty list
        if (fd >= 0) close(fd);
        int32_t rc = room(g, 0);
        if (rc) return rc;
        record(g->slots[g->cur], 0, tag, status);
        g->stats[0]++;
        return SYNCR_CDC_OK;
    }
    const uint64_t len = (uint64_t)st.st_size;
    const uint32_t mt = (uint32_t)st.st_mtime;                // meta.mtime() as u32 (file_operations.rs:615)
    if (g->cache) {                                           // unchanged file: cached ChunkInfo list
        uint64_t n = 0;
        std::vector<syncr_chunk_info> tmp;
        int32_t rc = syncr_cache_get(g->cache, path, mt, len, nullptr, 0, &n);   // OK here: no chunks
        if (rc == SYNCR_CDC_ERANGE) {
            tmp.resize(n);
            rc = syncr_cache_get(g->cache, path, mt, len, tmp.data(), n, &n);
        }
        if (rc == SYNCR_CDC_OK) {
            close(fd);
            rc = room(g, 0);
            if (rc) return rc;
            Slot &s = g->slots[g->cur];
            record(s, 0, tag, 0);
            s.hit.back() = 1;
            s.cstart.back() = s.cbuf.size();
            s.ccount.back() = n;
            s.cbuf.insert(s.cbuf.end(), tmp.begin(), tmp.end());
            g->stats[0]++;
            g->cache_hits++;
            return SYNCR_CDC_OK;
        }
    }
    uint8_t *dst = nullptr;
    int32_t rc = syncr_ingest_reserve(g, len, &dst);
    if (rc) {
        close(fd);
        return rc;
    }
    // pread straight into pinned memory, split over the pool for big files
    int err = 0;
    uint64_t got_total = 0;
    std::mutex emu;
    auto read_range = [&](uint64_t a, uint64_t b) {
        uint64_t pos = a;
        while (pos < b) {
            const ssize_t r = pread(fd, dst + pos, (size_t)(b - pos), (off_t)pos);
            if (r < 0 && errno == EINTR) continue;
            if (r <= 0) {
                std::lock_guard<std::mutex> l(emu);
                if (!err) err = r < 0 ? errno : EIO;   // short file: changed under us
                return;
            }
            pos += (uint64_t)r;
        }
        std::lock_guard<std::mutex> l(emu);
        got_total += b - a;
    };
    if (len > PAR_COPY && g->pool) {
        const unsigned pieces = (unsigned)((len + PIECE - 1) / PIECE);
        g->pool->parallel(pieces, [&](unsigned i) {
            const uint64_t a = (uint64_t)i * PIECE;
            read_range(a, std::min<uint64_t>(len, a + PIECE));
        });
    } else {
        read_range(0, len);
    }
    close(fd);
    g->reserved = false;
    if (err) {                                       // file_operations.rs:740-743: empty list
        record(g->slots[g->cur], 0, tag, -err);
    } else {
        record(g->slots[g->cur], len, tag, 0, g->cache ? path : nullptr, mt, len);
        g->stats[1] += len;
    }
    g->stats[0]++;
    return SYNCR_CDC_OK;
}

int32_t syncr_ingest_set_cache(syncr_ingest *g, syncr_cache *c) {
    if (!g) return SYNCR_CDC_EINVAL;
    g->cache = c;
    return SYNCR_CDC_OK;
}

int32_t syncr_ingest_flush(syncr_ingest *g) {
    if (!g) return SYNCR_CDC_EINVAL;
    if (g->reserved) return SYNCR_CDC_ESTATE;
    if (g->error) return g->error;
    int32_t rc = seal(g, g->slots[g->cur]);
    if (rc) return rc;
    // complete every slot, oldest first (the one after cur is the oldest)
    const uint32_t n = (uint32_t)g->slots.size();
    for (uint32_t k = 1; k <= n; k++) {
        rc = complete(g, g->slots[(g->cur + k) % n]);
        if (rc) return rc;
    }
    g->cur = (g->cur + 1) % n;
    return SYNCR_CDC_OK;
}

int32_t syncr_ingest_stats(const syncr_ingest *g, uint64_t *stats4) {
    if (!g || !stats4) return SYNCR_CDC_EINVAL;
    for (int k = 0; k < 4; k++) stats4[k] = g->stats[k];
    return SYNCR_CDC_OK;
}

int32_t syncr_ingest_cache_hits(const syncr_ingest *g, uint64_t *hits) {
    if (!g || !hits) return SYNCR_CDC_EINVAL;
    *hits = g->cache_hits;
    return SYNCR_CDC_OK;
}

void syncr_ingest_close(syncr_ingest *g) {
    if (!g) return;
    for (Slot &s : g->slots) {
        if (s.h) {
            (void)syncr_cdc_synchronize(s.h);
            syncr_cdc_close(s.h);
        }
        free_slot_buffers(g, s);
    }
    delete g->pool;
    delete g;
}

}  // extern "C"
