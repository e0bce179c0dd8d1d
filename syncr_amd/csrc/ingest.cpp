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
// caller's thread.
//
// One `Pipe` is the pipeline of one device.  syncr_ingest_open drives one Pipe
// on the caller's thread.  syncr_ingest_open_multi drives one Pipe per listed
// device, each on its own worker thread (the reference's host is ONE process,
// src/protocol/factory.rs:116-125, so multi-GPU use needs this in-process
// fan-out): files are assigned whole to the least-loaded device (ingest_logic.h)
// and the results are put back into submission order before any callback.
//
// Read failures follow compute_file_chunks: a file that cannot be opened, or
// whose first read fails, yields -errno and no chunks (:727-744); a read that
// fails later breaks the loop and keeps the chunks cut so far (:776-782,
// ingest_logic.h read_error_keep); a file that shrank is chunked at the length
// actually read (reads stop at EOF).
#include <errno.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/syncr_cdc.h"
#include "ingest_logic.h"

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
    // Queue fn to run on a pool thread (inline when the pool has none).  Posted
    // tasks must not wait on anything the caller holds.
    void post(std::function<void()> fn) {
        if (th_.empty()) {
            fn();
            return;
        }
        {
            std::lock_guard<std::mutex> g(mu_);
            tasks_.push_back(std::move(fn));
        }
        cv_.notify_one();
    }
    // Run one posted task on the calling thread, if any is queued (a caller that
    // waits for its tasks helps instead of idling).
    bool run_one() {
        std::function<void()> f;
        {
            std::lock_guard<std::mutex> g(mu_);
            if (tasks_.empty()) return false;
            f = std::move(tasks_.front());
            tasks_.pop_front();
        }
        f();
        return true;
    }
    // run fn(0..n-1) on the pool plus the calling thread; returns when all done.
    // Callers on several threads (sub-pipelines sharing the pool) take turns.
    void parallel(unsigned n, const std::function<void(unsigned)> &fn) {
        if (n <= 1 || th_.empty()) {
            for (unsigned i = 0; i < n; i++) fn(i);
            return;
        }
        std::lock_guard<std::mutex> job(job_mu_);
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
            std::function<void()> task;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return stop_ || (gen_ != seen && fn_ && next_ < total_) || !tasks_.empty(); });
                if (stop_ && tasks_.empty()) return;
                if (gen_ != seen && fn_ && next_ < total_) {
                    seen = gen_;
                } else if (!tasks_.empty()) {
                    task = std::move(tasks_.front());
                    tasks_.pop_front();
                } else {
                    continue;
                }
            }
            if (task) task();
            else work();
        }
    }
    std::vector<std::thread> th_;
    std::mutex job_mu_;                       // one parallel() job at a time
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(unsigned)> *fn_ = nullptr;
    std::deque<std::function<void()>> tasks_;  // posted (asynchronous) tasks
    unsigned next_ = 0, total_ = 0, done_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

// One file read by the pool into a slot's staging, PIECE bytes per task.  Per
// piece: bytes read from its start and the errno that stopped it (0 = EOF: the
// file shrank under us).  In a deque: its address is stable while later files
// are queued.
struct PendingRead {
    int fd = -1;
    uint8_t *dst = nullptr;
    uint64_t len = 0;
    size_t entry = 0;                 // the file's index in the slot
    std::string path;                 // chunk cache key (when a cache is attached)
    uint32_t mtime = 0;
    uint64_t fault_off = UINT64_MAX;  // syncr_ingest_set_read_fault
    int fault_err = 0;
    std::vector<uint64_t> got;
    std::vector<int> perr;
    uint32_t left = 0;                // pieces of this file not yet read (guarded by Pipe::rmu)
};

struct Slot {
    syncr_cdc *h = nullptr;           // own handle: own plan tables and stream
    uint8_t *host = nullptr;          // pinned staging
    uint8_t *dev = nullptr;
    uint64_t cap = 0, used = 0;
    std::vector<uint64_t> off, len, tag;
    std::vector<int32_t> status;
    std::vector<uint8_t> trunc;       // read error after len > 0 bytes: keep the reference's prefix
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
    // files whose bytes the pool is reading into this slot (submit_file): their
    // entries above are provisional until seal() has waited for the reads
    std::deque<PendingRead> reads;
    uint32_t pending = 0;             // pieces not yet read (guarded by Pipe::rmu)
    uint32_t small_uses = 0;          // batch-sized batches since the slot was grown (shrink_slot)
};

constexpr uint64_t PAR_COPY = 4ull << 20;   // copies above this are split over the pool
constexpr uint64_t PIECE = 2ull << 20;
// Files whose reads are still queued or running keep their descriptor open.
// submit_file opens the next file only while fewer than this many are open
// (it helps with the queued reads, or waits, otherwise), so a walk of many
// small files on slow storage never runs the process out of descriptors --
// the reference limits itself the same way, 8 files at a time through its
// walk's semaphore (file_operations.rs:596-599, streaming.rs:91).
constexpr uint32_t MAX_OPEN_READS = 64;

typedef void (*deliver_fn)(void *owner, uint64_t tag, int32_t status, const syncr_chunk_info *chunks, uint64_t n);

// The pipeline of one device (all calls on one thread at a time).
struct Pipe {
    int32_t device = 0;
    syncr_cdc_params params{};
    uint64_t batch = 0;
    std::vector<Slot> slots;
    uint32_t cur = 0;
    deliver_fn deliver = nullptr;
    void *owner = nullptr;
    Pool *pool = nullptr;
    bool own_pool = true;            // false: the multi-device pipeline's shared pool
    bool reserved = false;           // reserve() outstanding on slots[cur]
    uint64_t reserved_len = 0;
    std::atomic<uint64_t> stats[4] = {{0}, {0}, {0}, {0}};   // files, bytes, batches, chunks
    int32_t error = 0;                  // sticky engine error
    syncr_cache *cache = nullptr;       // optional (syncr_ingest_set_cache)
    std::atomic<uint64_t> cache_hits{0};
    // syncr_ingest_set_read_fault: submit_file's reads stop at this file
    // offset with fault_err (0 = EOF there, as if the file shrank)
    std::atomic<uint64_t> fault_off{UINT64_MAX};
    std::atomic<int32_t> fault_err{0};
    // host time (ns) spent in each stage (syncr_ingest_timing): copies into
    // pinned staging, file reads into it, seal (plan + H2D and kernel enqueue),
    // waiting for a batch's results (fetch), per-file delivery
    std::atomic<uint64_t> tns[5] = {{0}, {0}, {0}, {0}, {0}};
    // completion of the pool's file reads (Slot::pending) and of open files
    std::mutex rmu;
    std::condition_variable rcv;
    uint32_t open_reads = 0;            // files with reads outstanding (guarded by rmu)
};

enum { T_COPY = 0, T_READ = 1, T_SEAL = 2, T_WAIT = 3, T_DELIVER = 4 };

uint64_t now_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

// adds the time from construction to destruction to one stage counter
struct StageTimer {
    std::atomic<uint64_t> &acc;
    uint64_t t0;
    explicit StageTimer(std::atomic<uint64_t> &a) : acc(a), t0(now_ns()) {}
    ~StageTimer() { acc += now_ns() - t0; }
};

int32_t hip_rc(hipError_t e) {
    if (e == hipSuccess) return SYNCR_CDC_OK;
    if (e == hipErrorOutOfMemory) return SYNCR_CDC_ENOMEM;
    return SYNCR_CDC_EIO;
}

void free_slot_buffers(Pipe *g, Slot &s) {
    (void)hipSetDevice(g->device);
    if (s.host) (void)hipHostFree(s.host);
    if (s.dev) (void)hipFree(s.dev);
    s.host = s.dev = nullptr;
    s.cap = 0;
}

// Grow a slot's buffers to `bytes`.  The new buffers are allocated before the
// old ones are freed (device memory first: a file too big for the GPU fails
// there without touching host memory), so a failed allocation for one
// oversized file leaves the slot as it was and only that file fails.  When
// old + new do not fit together, the old buffers are freed and the allocation
// is tried once more; if that fails too the slot is refilled at batch size
// (or left empty, which the next ensure_slot retries) and the error is that
// file's.
int32_t alloc_slot(Pipe *g, uint64_t want, uint8_t **dev, uint8_t **host) {
    *dev = *host = nullptr;
    hipError_t e = hipSetDevice(g->device);
    if (e == hipSuccess) e = hipMalloc((void **)dev, want);
    if (e == hipSuccess) e = hipHostMalloc((void **)host, want, hipHostMallocDefault);
    if (e != hipSuccess) {
        (void)hipGetLastError();                            // the failure is this call's, not sticky
        if (*dev) (void)hipFree(*dev);
        *dev = *host = nullptr;
    }
    return hip_rc(e);
}

int32_t ensure_slot(Pipe *g, Slot &s, uint64_t bytes) {
    if (bytes <= s.cap && s.host) return SYNCR_CDC_OK;
    const uint64_t want = std::max<uint64_t>(bytes, 64);
    uint8_t *dev = nullptr, *host = nullptr;
    int32_t rc = alloc_slot(g, want, &dev, &host);
    if (rc && s.host) {                                    // old + new at once did not fit
        free_slot_buffers(g, s);
        rc = alloc_slot(g, want, &dev, &host);
        if (rc) {
            const uint64_t back = std::max<uint64_t>(g->batch, 64);
            if (back < want && alloc_slot(g, back, &dev, &host) == SYNCR_CDC_OK) {
                s.host = host;
                s.dev = dev;
                s.cap = back;
            }
            return rc;
        }
    }
    if (rc) return rc;
    free_slot_buffers(g, s);
    s.host = host;
    s.dev = dev;
    s.cap = want;
    return SYNCR_CDC_OK;
}

// A slot grown for an oversized file goes back to batch size after SHRINK_AFTER
// batch-sized batches have been delivered from it, so the pipeline's pinned and
// device memory returns to depth x batch_bytes between runs of oversized files.
// (Shrinking right after each oversized file made a stream of them pay a
// device-synchronising free and a fresh pin per file: ADVICE r4.)
// A slot of up to KEEP_GROWN batches is kept as it is (the memory stays
// bounded, and a one-file-per-batch caller -- the per-file call site's depth-1
// pipelines -- met a file between 1 and 2 batches every ~100 files of zipf10k:
// a fresh pin and a device-synchronising free each time cost ~0.1 s per 10 000
// files); a bigger one shrinks after SHRINK_AFTER batch-sized batches, or at
// the next flush.
constexpr uint32_t SHRINK_AFTER = 4;
constexpr uint64_t KEEP_GROWN = 2;
void shrink_slot(Pipe *g, Slot &s, bool oversized) {
    if (s.cap <= KEEP_GROWN * std::max<uint64_t>(g->batch, 64) || s.inflight || s.used) return;
    s.small_uses = oversized ? 0u : s.small_uses + 1u;
    if (s.small_uses < SHRINK_AFTER) return;
    s.small_uses = 0;
    uint8_t *dev = nullptr, *host = nullptr;
    free_slot_buffers(g, s);
    if (alloc_slot(g, std::max<uint64_t>(g->batch, 64), &dev, &host) == SYNCR_CDC_OK) {
        s.host = host;
        s.dev = dev;
        s.cap = std::max<uint64_t>(g->batch, 64);
    }
}

void par_copy(Pipe *g, uint8_t *dst, const uint8_t *src, uint64_t n) {
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
int32_t complete(Pipe *g, Slot &s) {
    if (!s.inflight) return SYNCR_CDC_OK;
    s.inflight = false;
    const uint32_t nf = (uint32_t)s.off.size();
    s.counts.assign(std::max<uint32_t>(nf, 1), 0);
    uint64_t n = 0;
    int32_t rc;
    {
        StageTimer tw(g->tns[T_WAIT]);
        rc = syncr_cdc_fetch_hashed(s.h, nullptr, 0, s.counts.data(), &n);
        if (rc == SYNCR_CDC_ERANGE || rc == SYNCR_CDC_OK) {
            s.out.resize(std::max<uint64_t>(n, 1));
            rc = syncr_cdc_fetch_hashed(s.h, s.out.data(), s.out.size(), s.counts.data(), &n);
        }
    }
    if (rc) {
        g->error = rc;
        return rc;
    }
    StageTimer td(g->tns[T_DELIVER]);
    uint64_t o = 0;
    std::vector<uint64_t> ends;
    for (uint32_t i = 0; i < nf; i++) {
        const syncr_chunk_info *ci;
        uint64_t c;
        if (s.hit[i]) {                                       // served by the chunk cache
            c = s.ccount[i];
            ci = c ? s.cbuf.data() + s.cstart[i] : nullptr;
        } else {
            c = s.counts[i];
            for (uint64_t k = 0; k < c; k++) s.out[o + k].file = 0;   // one file per callback
            ci = c ? s.out.data() + o : nullptr;
            if (s.status[i]) {
                if (s.trunc[i]) {                              // read error after len bytes: the reference's prefix
                    ends.resize(c);
                    for (uint64_t k = 0; k < c; k++) ends[k] = ci[k].offset + ci[k].len;
                    c = ingest::read_error_keep(ends.data(), c, s.len[i], g->params.max_chunk,
                                                g->params.read_cap);
                } else {
                    c = 0;
                }
                if (!c) ci = nullptr;
            } else if (g->cache && !s.key[i].empty()) {
                (void)syncr_cache_put(g->cache, s.key[i].c_str(), s.mtime[i], s.fsize[i], ci, c);
            }
        }
        if (g->deliver) g->deliver(g->owner, s.tag[i], s.status[i], ci, c);
        o += s.counts[i];
        g->stats[3] += c;
    }
    s.off.clear();
    s.len.clear();
    s.tag.clear();
    s.status.clear();
    s.trunc.clear();
    s.key.clear();
    s.mtime.clear();
    s.fsize.clear();
    s.hit.clear();
    s.cstart.clear();
    s.ccount.clear();
    s.cbuf.clear();
    const bool oversized = s.used > g->batch;
    s.used = 0;
    shrink_slot(g, s, oversized);
    return SYNCR_CDC_OK;
}

// Wait for the pool's reads into slot s, then turn each file's provisional
// entry into its final one: the prefix read without a gap (the reference reads
// sequentially and stops at the first failure or EOF), its status, and its
// chunk-cache key when it was read whole.
void finish_reads(Pipe *g, Slot &s) {
    if (s.reads.empty()) return;
    {
        StageTimer tr(g->tns[T_READ]);
        for (;;) {
            {
                std::unique_lock<std::mutex> l(g->rmu);
                if (!s.pending) break;
            }
            if (g->pool && g->pool->run_one()) continue;          // help with queued reads
            std::unique_lock<std::mutex> l(g->rmu);
            g->rcv.wait_for(l, std::chrono::microseconds(200), [&] { return s.pending == 0; });
        }
    }
    for (PendingRead &pr : s.reads) {
        uint64_t P = 0;
        int err = 0;
        for (size_t i = 0; i < pr.got.size(); i++) {
            P += pr.got[i];
            const uint64_t want = std::min<uint64_t>(pr.len, (uint64_t)(i + 1) * PIECE) - (uint64_t)i * PIECE;
            if (pr.got[i] < want) { err = pr.perr[i]; break; }
        }
        const size_t e = pr.entry;
        s.len[e] = P;
        if (err) {                                   // file_operations.rs:738-743 (P = 0) / :776-782
            s.status[e] = -err;
            s.trunc[e] = P > 0 ? 1 : 0;
        } else if (g->cache && P == pr.len) {        // complete (or shrank to P bytes: EOF, not cached)
            s.key[e] = pr.path;
            s.mtime[e] = pr.mtime;
            s.fsize[e] = pr.len;
        }
        g->stats[1] += P;
    }
    s.reads.clear();
}

int32_t seal(Pipe *g, Slot &s) {
    finish_reads(g, s);
    if (s.off.empty()) return SYNCR_CDC_OK;
    StageTimer ts(g->tns[T_SEAL]);
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
int32_t room(Pipe *g, uint64_t len) {
    Slot *s = &g->slots[g->cur];
    if (s->used && s->used + len > s->cap) {
        int32_t rc = seal(g, *s);
        if (rc) return rc;
        g->cur = (g->cur + 1) % (uint32_t)g->slots.size();
        s = &g->slots[g->cur];
    }
    int32_t rc = complete(g, *s);
    if (rc) return rc;
    // a file bigger than a batch, or a slot left without buffers by a failed growth
    if (!s->used && (len > s->cap || !s->host)) return ensure_slot(g, *s, std::max<uint64_t>(len, g->batch));
    return SYNCR_CDC_OK;
}

// len bytes at s.used belong to this file (also for a truncated read); status
// != 0 with trunc = 0 means no chunks at all
void record(Slot &s, uint64_t len, uint64_t tag, int32_t status, bool trunc = false, const char *key = nullptr,
            uint32_t mtime = 0, uint64_t fsize = 0) {
    s.off.push_back(s.used);
    s.len.push_back(len);
    s.tag.push_back(tag);
    s.status.push_back(status);
    s.trunc.push_back(trunc ? 1 : 0);
    s.key.emplace_back(key ? key : "");
    s.mtime.push_back(mtime);
    s.fsize.push_back(fsize);
    s.hit.push_back(0);
    s.cstart.push_back(0);
    s.ccount.push_back(0);
    s.used += len;
}

void pipe_close(Pipe *g) {
    if (!g) return;
    for (Slot &s : g->slots) finish_reads(g, s);     // no read may outlive the buffers
    for (Slot &s : g->slots) {
        if (s.h) {
            (void)syncr_cdc_synchronize(s.h);
            syncr_cdc_close(s.h);
        }
        free_slot_buffers(g, s);
    }
    if (g->own_pool) delete g->pool;
    delete g;
}

int32_t pipe_open(int32_t device, const syncr_cdc_params &p, uint64_t batch_bytes, uint32_t depth,
                  uint32_t copy_threads, Pool *shared, deliver_fn deliver, void *owner, Pipe **out) {
    Pipe *g = new (std::nothrow) Pipe();
    if (!g) return SYNCR_CDC_ENOMEM;
    g->device = device;
    g->params = p;
    g->batch = batch_bytes;
    g->deliver = deliver;
    g->owner = owner;
    try {
        g->slots.resize(depth);
        for (Slot &s : g->slots) {
            int32_t rc = syncr_cdc_open(device, &g->params, &s.h);
            if (rc == SYNCR_CDC_OK) rc = ensure_slot(g, s, batch_bytes);
            if (rc) {
                pipe_close(g);
                return rc;
            }
        }
        if (shared) {
            g->pool = shared;
            g->own_pool = false;
        } else if (copy_threads > 1) {
            g->pool = new Pool(std::min<uint32_t>(copy_threads, 64) - 1);
        }
    } catch (...) {
        pipe_close(g);
        return SYNCR_CDC_ENOMEM;
    }
    *out = g;
    return SYNCR_CDC_OK;
}

int32_t pipe_reserve(Pipe *g, uint64_t len, uint8_t **dst) {
    if (g->reserved) return SYNCR_CDC_ESTATE;
    if (g->error) return g->error;
    int32_t rc = room(g, len);
    if (rc) return rc;
    Slot &s = g->slots[g->cur];
    *dst = s.host + s.used;
    g->reserved = true;
    g->reserved_len = len;
    return SYNCR_CDC_OK;
}

int32_t pipe_commit(Pipe *g, uint64_t tag) {
    if (!g->reserved) return SYNCR_CDC_ESTATE;
    g->reserved = false;
    record(g->slots[g->cur], g->reserved_len, tag, 0);
    g->stats[0]++;
    g->stats[1] += g->reserved_len;
    return SYNCR_CDC_OK;
}

int32_t pipe_submit(Pipe *g, const uint8_t *data, uint64_t len, uint64_t tag) {
    uint8_t *dst = nullptr;
    int32_t rc = pipe_reserve(g, len, &dst);
    if (rc) return rc;
    {
        StageTimer tc(g->tns[T_COPY]);
        par_copy(g, dst, data, len);
    }
    return pipe_commit(g, tag);
}

// Piece i of a file (bytes [i * PIECE, +PIECE) of it): pread until done, EOF
// (the file shrank) or an error; with an injected fault (the test hook), bytes
// at and past the fault offset are never read and the read that would cross it
// fails with fault_err (0: EOF there).
void read_piece(PendingRead &pr, unsigned i) {
    const uint64_t a = (uint64_t)i * PIECE, b = std::min<uint64_t>(pr.len, a + PIECE);
    const uint64_t e = std::min(b, std::max(a, pr.fault_off));
    uint64_t pos = a;
    const uint64_t stop = e < b ? e : b;
    while (pos < stop) {
        const ssize_t r = pread(pr.fd, pr.dst + pos, (size_t)(stop - pos), (off_t)pos);
        if (r < 0 && errno == EINTR) continue;
        if (r < 0) { pr.perr[i] = errno ? errno : EIO; break; }    // a real error (before any fault)
        if (r == 0) break;                                         // EOF before st_size / the fault
        pos += (uint64_t)r;
    }
    if (e < b && pos == e) pr.perr[i] = pr.fault_err;
    pr.got[i] = pos - a;
}

// Block until fewer than MAX_OPEN_READS files have reads outstanding, running
// queued reads on this thread meanwhile.
void wait_read_room(Pipe *g) {
    StageTimer tr(g->tns[T_READ]);
    for (;;) {
        {
            std::lock_guard<std::mutex> l(g->rmu);
            if (g->open_reads < MAX_OPEN_READS) return;
        }
        if (g->pool && g->pool->run_one()) continue;
        std::unique_lock<std::mutex> l(g->rmu);
        g->rcv.wait_for(l, std::chrono::microseconds(200), [&] { return g->open_reads < MAX_OPEN_READS; });
    }
}

int32_t pipe_submit_file(Pipe *g, const char *path, uint64_t tag) {
    if (g->reserved) return SYNCR_CDC_ESTATE;
    if (g->error) return g->error;
    wait_read_room(g);
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
    int32_t rc = pipe_reserve(g, len, &dst);
    if (rc) {
        close(fd);
        return rc;
    }
    g->reserved = false;
    Slot &s = g->slots[g->cur];
    g->stats[0]++;
    if (!len) {                                      // nothing to read: final now (and cacheable)
        close(fd);
        record(s, 0, tag, 0, false, g->cache ? path : nullptr, mt, 0);
        return SYNCR_CDC_OK;
    }
    record(s, len, tag, 0);                          // provisional: finish_reads() sets length and status
    // pread straight into pinned memory on the pool, PIECE bytes per task: the
    // caller goes on to the next file (many small files are read in parallel),
    // and seal() waits for the slot's reads before the batch's H2D
    PendingRead &pr = s.reads.emplace_back();
    pr.fd = fd;
    pr.dst = dst;
    pr.len = len;
    pr.entry = s.off.size() - 1;
    if (g->cache) pr.path = path;
    pr.mtime = mt;
    pr.fault_off = g->fault_off.load();
    pr.fault_err = g->fault_err.load();
    const unsigned pieces = (unsigned)((len + PIECE - 1) / PIECE);
    pr.got.assign(pieces, 0);
    pr.perr.assign(pieces, 0);
    {
        std::lock_guard<std::mutex> l(g->rmu);
        pr.left = pieces;
        s.pending += pieces;
        g->open_reads++;
    }
    for (unsigned i = 0; i < pieces; i++) {
        auto task = [g, &s, &pr, i] {
            read_piece(pr, i);
            std::lock_guard<std::mutex> l(g->rmu);            // (pr may be gone once pending drops)
            bool wake = false;
            if (--pr.left == 0) {
                close(pr.fd);
                wake = g->open_reads-- == MAX_OPEN_READS;     // a submit_file may be waiting for room
            }
            if (--s.pending == 0 || wake) g->rcv.notify_all();
        };
        if (g->pool) g->pool->post(task);
        else task();
    }
    return SYNCR_CDC_OK;
}

int32_t pipe_flush(Pipe *g) {
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
    // An idle pipeline keeps at most KEEP_GROWN x batch_bytes per slot: a slot
    // grown past that for one huge file is shrunk now, not after SHRINK_AFTER
    // more batches that may never come (a pooled per-file pipeline can sit idle
    // for the rest of the process).
    for (Slot &s : g->slots)
        if (s.cap > KEEP_GROWN * std::max<uint64_t>(g->batch, 64)) {
            s.small_uses = SHRINK_AFTER;
            shrink_slot(g, s, false);
        }
    return SYNCR_CDC_OK;
}

// ---- multi-device front end ------------------------------------------------

struct Result {
    int32_t status = 0;
    bool skip = false;                // a failed synchronous submit: no callback (as single-device)
    std::vector<syncr_chunk_info> chunks;
};

enum JobKind { J_FILE, J_COPY, J_RESERVE, J_COMMIT, J_FLUSH };

struct SyncSlot {                 // a job the caller waits for
    int32_t rc = 0;
    uint8_t *dst = nullptr;
    bool done = false;
};

struct Job {
    JobKind kind;
    std::string path;
    const uint8_t *data = nullptr;
    uint64_t len = 0;
    uint64_t seq = 0;
    SyncSlot *sync = nullptr;
};

struct Worker {
    Pipe *pipe = nullptr;
    std::thread th;
    std::mutex mu;
    std::condition_variable cv, done_cv;
    std::deque<Job> q;
    bool stop = false;
    int32_t err = 0;
};

constexpr size_t MAX_QUEUED = 256;   // jobs per worker before submit waits

}  // namespace

struct syncr_ingest {
    syncr_ingest_cb cb = nullptr;
    void *ctx = nullptr;
    std::vector<Pipe *> pipes;
    bool multi = false;
    // multi: workers, assignment, in-order delivery
    std::vector<Worker *> workers;
    ingest::Assigner *assign = nullptr;
    ingest::Reorder<Result> reorder;
    std::deque<uint64_t> tags;        // user tag of seq (next_deliver + k)
    uint64_t next_seq = 0;
    bool reserved = false;
    uint32_t reserve_dev = 0;
    int32_t error = 0;
    syncr_cache *cache = nullptr;
    Pool *pool = nullptr;             // multi: the copy pool the sub-pipelines share
};

namespace {

void deliver_single(void *owner, uint64_t tag, int32_t status, const syncr_chunk_info *c, uint64_t n) {
    syncr_ingest *g = (syncr_ingest *)owner;
    if (g->cb) g->cb(g->ctx, tag, status, c, n);
}

void deliver_multi(void *owner, uint64_t seq, int32_t status, const syncr_chunk_info *c, uint64_t n) {
    syncr_ingest *g = (syncr_ingest *)owner;
    Result r;
    r.status = status;
    if (n) r.chunks.assign(c, c + n);
    g->reorder.put(seq, std::move(r));
}

// A job that failed for its own file only (the pipe has no sticky engine
// error: e.g. ENOMEM for the pinned buffer of a file larger than a batch, which
// the single-device pipeline also reports for that call alone) still takes its
// place in the submission order, so later files keep being delivered: an
// asynchronous job (submit_file, commit) is delivered with its error status and
// no chunks; a synchronous submit, whose caller already got the error, is
// dropped without a callback, exactly as single-device mode does.
void fail_in_order(Pipe *p, const Job &j, int32_t rc) {
    syncr_ingest *g = (syncr_ingest *)p->owner;
    Result r;
    r.status = rc;
    r.skip = j.kind == J_COPY;
    g->reorder.put(j.seq, std::move(r));
}

void worker_main(Worker *w) {
    (void)hipSetDevice(w->pipe->device);
    for (;;) {
        Job j;
        {
            std::unique_lock<std::mutex> l(w->mu);
            w->cv.wait(l, [&] { return w->stop || !w->q.empty(); });
            if (w->q.empty()) return;                  // stop, queue drained
            j = std::move(w->q.front());
            w->q.pop_front();
        }
        int32_t rc = SYNCR_CDC_OK;
        uint8_t *dst = nullptr;
        Pipe *p = w->pipe;
        switch (j.kind) {
            case J_FILE: rc = pipe_submit_file(p, j.path.c_str(), j.seq); break;
            case J_COPY: rc = pipe_submit(p, j.data, j.len, j.seq); break;
            case J_RESERVE: rc = pipe_reserve(p, j.len, &dst); break;
            case J_COMMIT: rc = pipe_commit(p, j.seq); break;
            case J_FLUSH: rc = pipe_flush(p); break;
        }
        const bool per_file = rc && !p->error && (j.kind == J_FILE || j.kind == J_COPY || j.kind == J_COMMIT);
        if (per_file) fail_in_order(p, j, rc);
        {
            std::lock_guard<std::mutex> l(w->mu);
            if (rc && p->error && !w->err) w->err = p->error;      // only engine errors are sticky
            if (j.sync) {
                j.sync->rc = rc;
                j.sync->dst = dst;
                j.sync->done = true;
            }
        }
        w->done_cv.notify_all();
    }
}

void enqueue(Worker *w, Job j) {
    std::unique_lock<std::mutex> l(w->mu);
    w->done_cv.wait(l, [&] { return w->q.size() < MAX_QUEUED; });
    w->q.push_back(std::move(j));
    l.unlock();
    w->cv.notify_one();
}

int32_t run_sync(Worker *w, Job j) {
    SyncSlot ss;
    j.sync = &ss;
    enqueue(w, std::move(j));
    std::unique_lock<std::mutex> l(w->mu);
    w->done_cv.wait(l, [&] { return ss.done; });
    return ss.rc;
}

int32_t sticky(syncr_ingest *g) {
    if (g->error) return g->error;
    for (Worker *w : g->workers) {
        std::lock_guard<std::mutex> l(w->mu);
        if (w->err) return g->error = w->err;
    }
    return SYNCR_CDC_OK;
}

// deliver every result whose predecessors have all been delivered
void drain(syncr_ingest *g) {
    Result r;
    uint64_t seq;
    while (g->reorder.take(r, seq)) {
        const uint64_t tag = g->tags.front();
        g->tags.pop_front();
        if (r.skip) continue;
        if (g->cb) g->cb(g->ctx, tag, r.status, r.chunks.empty() ? nullptr : r.chunks.data(), r.chunks.size());
    }
}

uint64_t new_seq(syncr_ingest *g, uint64_t tag) {
    g->tags.push_back(tag);
    return g->next_seq++;
}

void close_multi(syncr_ingest *g) {
    for (Worker *w : g->workers) {
        {
            std::lock_guard<std::mutex> l(w->mu);
            w->stop = true;
        }
        w->cv.notify_all();
        if (w->th.joinable()) w->th.join();
    }
    for (Worker *w : g->workers) delete w;
    g->workers.clear();
}

}  // namespace

extern "C" {

int32_t syncr_ingest_open(int32_t device, const syncr_cdc_params *p, uint64_t batch_bytes, uint32_t depth,
                          uint32_t copy_threads, syncr_ingest_cb cb, void *ctx, syncr_ingest **out) {
    return syncr_ingest_open_multi(&device, 1, p, batch_bytes, depth, copy_threads, cb, ctx, out);
}

int32_t syncr_ingest_open_multi(const int32_t *devices, uint32_t ndevices, const syncr_cdc_params *p,
                                uint64_t batch_bytes, uint32_t depth, uint32_t copy_threads, syncr_ingest_cb cb,
                                void *ctx, syncr_ingest **out) {
    if (!out) return SYNCR_CDC_EINVAL;
    *out = nullptr;
    if (!devices || ndevices < 1 || ndevices > 64) return SYNCR_CDC_EINVAL;
    if (depth < 1 || depth > 8 || batch_bytes < 4096) return SYNCR_CDC_EINVAL;
    syncr_cdc_params prm;
    if (p) prm = *p; else syncr_cdc_default_params(&prm);
    syncr_ingest *g = new (std::nothrow) syncr_ingest();
    if (!g) return SYNCR_CDC_ENOMEM;
    g->cb = cb;
    g->ctx = ctx;
    g->multi = ndevices > 1;
    try {
        // one copy pool for the whole pipeline: the sub-pipelines take turns on it
        if (g->multi && copy_threads > 1) g->pool = new Pool(std::min<uint32_t>(copy_threads, 64) - 1);
        for (uint32_t k = 0; k < ndevices; k++) {
            Pipe *pp = nullptr;
            const int32_t rc = pipe_open(devices[k], prm, batch_bytes, depth, copy_threads, g->pool,
                                         g->multi ? deliver_multi : deliver_single, g, &pp);
            if (rc) {
                syncr_ingest_close(g);
                return rc;
            }
            g->pipes.push_back(pp);
        }
        if (g->multi) {
            g->assign = new ingest::Assigner(ndevices);
            for (Pipe *pp : g->pipes) {
                Worker *w = new Worker();
                w->pipe = pp;
                g->workers.push_back(w);
                w->th = std::thread(worker_main, w);
            }
        }
    } catch (...) {
        syncr_ingest_close(g);
        return SYNCR_CDC_ENOMEM;
    }
    *out = g;
    return SYNCR_CDC_OK;
}

int32_t syncr_ingest_reserve(syncr_ingest *g, uint64_t len, uint8_t **dst) {
    if (!g || !dst) return SYNCR_CDC_EINVAL;
    if (!g->multi) return pipe_reserve(g->pipes[0], len, dst);
    if (g->reserved) return SYNCR_CDC_ESTATE;
    int32_t rc = sticky(g);
    if (rc) return rc;
    const uint32_t d = g->assign->assign(len);
    Job j{J_RESERVE};
    j.len = len;
    SyncSlot ss;
    j.sync = &ss;
    Worker *w = g->workers[d];
    enqueue(w, std::move(j));
    {
        std::unique_lock<std::mutex> l(w->mu);
        w->done_cv.wait(l, [&] { return ss.done; });
    }
    drain(g);
    if (ss.rc) return ss.rc;
    *dst = ss.dst;
    g->reserved = true;
    g->reserve_dev = d;
    return SYNCR_CDC_OK;
}

int32_t syncr_ingest_commit(syncr_ingest *g, uint64_t tag) {
    if (!g) return SYNCR_CDC_EINVAL;
    if (!g->multi) return pipe_commit(g->pipes[0], tag);
    if (!g->reserved) return SYNCR_CDC_ESTATE;
    g->reserved = false;
    Job j{J_COMMIT};
    j.seq = new_seq(g, tag);
    enqueue(g->workers[g->reserve_dev], std::move(j));
    return SYNCR_CDC_OK;
}

int32_t syncr_ingest_submit(syncr_ingest *g, const uint8_t *data, uint64_t len, uint64_t tag) {
    if (!g || (len && !data)) return SYNCR_CDC_EINVAL;
    if (!g->multi) return pipe_submit(g->pipes[0], data, len, tag);
    if (g->reserved) return SYNCR_CDC_ESTATE;
    int32_t rc = sticky(g);
    if (rc) return rc;
    const uint32_t d = g->assign->assign(len);
    Job j{J_COPY};
    j.data = data;
    j.len = len;
    j.seq = new_seq(g, tag);
    rc = run_sync(g->workers[d], std::move(j));          // the bytes are copied before we return
    drain(g);
    return rc;
}

int32_t syncr_ingest_submit_file(syncr_ingest *g, const char *path, uint64_t tag) {
    if (!g || !path) return SYNCR_CDC_EINVAL;
    if (!g->multi) return pipe_submit_file(g->pipes[0], path, tag);
    if (g->reserved) return SYNCR_CDC_ESTATE;
    int32_t rc = sticky(g);
    if (rc) return rc;
    struct stat st;
    const uint64_t size = stat(path, &st) == 0 ? (uint64_t)st.st_size : 0;
    const uint32_t d = g->assign->assign(size);
    Job j{J_FILE};
    j.path = path;
    j.seq = new_seq(g, tag);
    enqueue(g->workers[d], std::move(j));                 // read + chunked on that device's thread
    drain(g);
    return SYNCR_CDC_OK;
}

int32_t syncr_ingest_set_cache(syncr_ingest *g, syncr_cache *c) {
    if (!g) return SYNCR_CDC_EINVAL;
    if (c) {
        syncr_cdc_params cp;
        int32_t rc = syncr_cache_get_params(c, &cp);
        if (rc) return rc;
        const syncr_cdc_params &ip = g->pipes[0]->params;
        // a chunk list cut under other parameters must never be served
        if (cp.chunk_bits != ip.chunk_bits || cp.max_chunk != ip.max_chunk || cp.read_cap != ip.read_cap)
            return SYNCR_CDC_EINVAL;
    }
    if (g->multi) {                                       // no job may be using the old cache
        int32_t rc = syncr_ingest_flush(g);
        if (rc) return rc;
    }
    g->cache = c;
    for (Pipe *p : g->pipes) p->cache = c;
    return SYNCR_CDC_OK;
}

int32_t syncr_ingest_flush(syncr_ingest *g) {
    if (!g) return SYNCR_CDC_EINVAL;
    if (!g->multi) return pipe_flush(g->pipes[0]);
    if (g->reserved) return SYNCR_CDC_ESTATE;
    int32_t rc = sticky(g);
    if (rc) return rc;
    std::vector<SyncSlot> ss(g->workers.size());
    for (size_t k = 0; k < g->workers.size(); k++) {
        Job j{J_FLUSH};
        j.sync = &ss[k];
        enqueue(g->workers[k], std::move(j));
    }
    for (size_t k = 0; k < g->workers.size(); k++) {
        Worker *w = g->workers[k];
        std::unique_lock<std::mutex> l(w->mu);
        w->done_cv.wait(l, [&] { return ss[k].done; });
    }
    drain(g);
    for (auto &s : ss)
        if (s.rc) return g->error = s.rc;
    rc = sticky(g);
    if (rc) return rc;
    return g->tags.empty() ? SYNCR_CDC_OK : (g->error = SYNCR_CDC_EIO);   // every file delivered
}

int32_t syncr_ingest_stats(const syncr_ingest *g, uint64_t *stats4) {
    if (!g || !stats4) return SYNCR_CDC_EINVAL;
    for (int k = 0; k < 4; k++) {
        stats4[k] = 0;
        for (const Pipe *p : g->pipes) stats4[k] += p->stats[k].load();
    }
    return SYNCR_CDC_OK;
}

int32_t syncr_ingest_device_stats(const syncr_ingest *g, uint64_t *stats, uint32_t n) {
    if (!g || (n && !stats)) return SYNCR_CDC_EINVAL;
    if (n < 4 * g->pipes.size()) return SYNCR_CDC_ERANGE;
    for (size_t k = 0; k < g->pipes.size(); k++) {
        const Pipe *p = g->pipes[k];
        stats[4 * k + 0] = (uint64_t)p->device;
        stats[4 * k + 1] = p->stats[0].load();           // files handled by this device
        stats[4 * k + 2] = p->stats[1].load();           // bytes
        stats[4 * k + 3] = p->stats[2].load();           // batches
    }
    return SYNCR_CDC_OK;
}

int32_t syncr_ingest_timing(const syncr_ingest *g, double *sec, uint32_t n) {
    if (!g || (n && !sec)) return SYNCR_CDC_EINVAL;
    for (uint32_t k = 0; k < n; k++) {
        uint64_t t = 0;
        if (k < 5)
            for (const Pipe *p : g->pipes) t += p->tns[k].load();
        sec[k] = (double)t * 1e-9;
    }
    return SYNCR_CDC_OK;
}

int32_t syncr_ingest_set_read_fault(syncr_ingest *g, uint64_t offset, int32_t err) {
    if (!g || err < 0) return SYNCR_CDC_EINVAL;
    for (Pipe *p : g->pipes) {
        p->fault_err.store(err);
        p->fault_off.store(offset);
    }
    return SYNCR_CDC_OK;
}

int32_t syncr_ingest_cache_hits(const syncr_ingest *g, uint64_t *hits) {
    if (!g || !hits) return SYNCR_CDC_EINVAL;
    *hits = 0;
    for (const Pipe *p : g->pipes) *hits += p->cache_hits.load();
    return SYNCR_CDC_OK;
}

void syncr_ingest_close(syncr_ingest *g) {
    if (!g) return;
    close_multi(g);
    for (Pipe *p : g->pipes) pipe_close(p);
    delete g->pool;
    delete g->assign;
    delete g;
}

}  // extern "C"
