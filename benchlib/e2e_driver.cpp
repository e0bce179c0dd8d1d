// e2e_driver.cpp -- the end-to-end legs of bench.py, driven from C++ the way
// syncr's Rust host would drive libsyncr_cdc.so: no Python per file.
//
//   e2e_driver MODE ROOT OUT [--reps R] [--device D]
//
// ROOT is a directory tree of files (bench.py writes the zipf10k corpus there);
// OUT receives every file's result (binary records, below) for the parity check
// against the golden digests; one JSON line with the timings goes to stdout.
//
// MODE
//   per_file   the integration of round 5 (rust/src/chunking_gpu.rs
//              compute_file_chunks_gpu): the reference's walk
//              (traverse_and_stream, src/protocol/file_operations.rs:544-715)
//              awaiting each file (:599-605) on a pooled depth-1 pipeline
//              (syncr_ingest_open: 64 MiB batch, depth 1, 4 threads):
//              submit_file -> flush -> one callback, per file.
//   walk       the batched walk (GpuWalk, integration/file_operations.diff):
//              every regular file submitted to one pipeline (256 MiB batches,
//              depth 3, 16 threads) as the walk meets it, entries sent in walk
//              order as their results come back.
//   files      the file list of ROOT (walked untimed) through submit_file and
//              one flush: the ingest pipeline on files without the walk.
//   mem        every file read into ordinary host memory first (untimed), then
//              syncr_ingest_submit per file (the library copies into pinned
//              staging on its pool) and one flush.
//   zero_copy  the same host bytes through syncr_ingest_reserve -> the caller
//              writes the bytes into the pinned staging itself (files above
//              4 MiB split over the caller's own 16 threads, as the library's
//              copy does) -> syncr_ingest_commit.
//   list       no device: print the walk's order (path, type, size, target)
//              per line (tests/test_cpp_mirror.py checks it against a Python
//              restatement of traverse_and_stream's order).
//
// Timed: each pass from its first call to the last delivered entry, best of
// --reps passes; the pipeline is opened once, before the passes (the Rust shim
// keeps its pipelines).  Latency of a file: from the call that submitted it to
// the moment its entry is sent / its result delivered.
//
// OUT records, in delivery order: u32 path length, path (relative to ROOT),
// i32 status, u32 n, n x syncr_chunk_info (48 bytes).
//
// Measurement tooling (benchlib/): links only the product library.
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <numeric>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include <fcntl.h>
#include <unistd.h>

#include "syncr_cdc.hpp"

namespace {

using Clock = std::chrono::steady_clock;

double secs(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }

struct Result {
    std::string path;
    int32_t status = 0;
    std::vector<syncr_chunk_info> chunks;
};

struct Pass {
    double seconds = 0;
    double fill_seconds = 0;          // zero_copy: the caller's own copies into staging
    std::vector<double> latency_us;
    std::vector<Result> results;
    double stage[5] = {0, 0, 0, 0, 0};
    uint64_t entries = 0;
};

// a few caller threads for zero_copy's fill (one parallel job at a time)
class Fill {
  public:
    explicit Fill(unsigned n) {
        for (unsigned i = 0; i < n; i++) th_.emplace_back([this] { run(); });
    }
    ~Fill() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    void parallel(unsigned n, const std::function<void(unsigned)> &fn) {
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
            {
                std::lock_guard<std::mutex> g(mu_);
                if (!fn_ || next_ >= total_) return;
                i = next_++;
            }
            (*fn_)(i);
            std::lock_guard<std::mutex> g(mu_);
            if (++done_ == total_) done_cv_.notify_all();
        }
    }
    void run() {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> g(mu_);
        for (;;) {
            cv_.wait(g, [&] { return stop_ || (gen_ != seen && fn_); });
            if (stop_) return;
            seen = gen_;
            g.unlock();
            work();
            g.lock();
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

struct Inbox {                       // the shim's deliver(): results in submission order
    std::vector<Result> *out = nullptr;
    const std::vector<std::string> *names = nullptr;
    std::vector<Clock::time_point> *t_submit = nullptr;
    std::vector<double> *lat = nullptr;
};

void on_file(void *ctx, uint64_t tag, int32_t status, const syncr_chunk_info *c, uint64_t n) {
    Inbox *in = static_cast<Inbox *>(ctx);
    const auto now = Clock::now();
    Result r;
    r.path = (*in->names)[tag];
    r.status = status;
    r.chunks.assign(c, c + n);
    in->out->push_back(std::move(r));
    in->lat->push_back(secs((*in->t_submit)[tag], now) * 1e6);
}

void stage_delta(syncr_ingest *g, double *acc, const double *before) {
    double now[5];
    syncr_ingest_timing(g, now, 5);
    for (int k = 0; k < 5; k++) acc[k] = now[k] - before[k];
}

syncr_cdc_params prod_params() {
    syncr_cdc_params p;
    syncr_cdc_default_params(&p);
    return p;
}

// ---- modes -----------------------------------------------------------------

Pass run_walk(const std::string &root, syncr::GpuWalk *w) {
    Pass p;
    double before[5];
    syncr_ingest_timing(w->handle(), before, 5);
    std::unordered_map<std::string, Clock::time_point> t_sub;
    auto send = [&](syncr::FileSystemEntry &&e) {   // sender.send(entry) (:707)
        p.entries++;
        if (e.entry_type != syncr::EntryType::File) return;
        p.latency_us.push_back(secs(t_sub[e.path], Clock::now()) * 1e6);
        Result r;
        r.path = e.path;
        r.status = e.status;
        r.chunks.resize(e.chunks.size());
        for (size_t k = 0; k < e.chunks.size(); k++) {
            r.chunks[k].offset = e.chunks[k].offset;
            r.chunks[k].len = e.chunks[k].size;
            r.chunks[k].file = 0;
            std::copy(e.chunks[k].hash.begin(), e.chunks[k].hash.end(), r.chunks[k].hash);
        }
        p.results.push_back(std::move(r));
    };
    const auto t0 = Clock::now();
    syncr::FileSystemEntry out;
    syncr::walk_tree(root, [&](const std::string &abs, syncr::FileSystemEntry &&e) {
        if (e.entry_type == syncr::EntryType::File) {
            t_sub[e.path] = Clock::now();
            w->push_file(abs, std::move(e));
        } else {
            w->push_entry(std::move(e));
        }
        while (w->pop_ready(out)) send(std::move(out));
    });
    w->finish();
    while (w->pop_ready(out)) send(std::move(out));
    p.seconds = secs(t0, Clock::now());
    stage_delta(w->handle(), p.stage, before);
    return p;
}

void on_result(void *ctx, uint64_t, int32_t st, const syncr_chunk_info *c, uint64_t n) {
    Result r;
    r.status = st;
    r.chunks.assign(c, c + n);
    static_cast<std::vector<Result> *>(ctx)->push_back(std::move(r));
}

// the pooled depth-1 pipeline of compute_file_chunks_gpu: `inbox` is its deliver() context
Pass run_per_file(const std::string &root, syncr_ingest *g, std::vector<Result> &inbox) {
    Pass p;
    double before[5];
    syncr_ingest_timing(g, before, 5);
    const auto t0 = Clock::now();
    syncr::walk_tree(root, [&](const std::string &abs, syncr::FileSystemEntry &&e) {
        p.entries++;
        if (e.entry_type != syncr::EntryType::File) return;
        const auto t1 = Clock::now();
        inbox.clear();                                     // GpuPipeline::chunk_file
        syncr::cdc_check(syncr_ingest_submit_file(g, abs.c_str(), 0), "submit_file");
        syncr::cdc_check(syncr_ingest_flush(g), "flush");
        p.latency_us.push_back(secs(t1, Clock::now()) * 1e6);
        if (inbox.size() != 1) throw std::runtime_error("per_file: not exactly one callback");
        inbox[0].path = e.path;
        p.results.push_back(std::move(inbox[0]));
    });
    p.seconds = secs(t0, Clock::now());
    stage_delta(g, p.stage, before);
    return p;
}

struct Corpus {
    std::vector<std::string> abs, rel;
    std::vector<uint64_t> off, len;
    uint8_t *host = nullptr;          // mem / zero_copy: every file in ordinary host memory
};

Corpus list_files(const std::string &root, bool load) {
    Corpus c;
    uint64_t tot = 0;
    syncr::walk_tree(root, [&](const std::string &abs, syncr::FileSystemEntry &&e) {
        if (e.entry_type != syncr::EntryType::File) return;
        c.abs.push_back(abs);
        c.rel.push_back(e.path);
        c.off.push_back(tot);
        c.len.push_back(e.size);
        tot += e.size;
    });
    if (load) {
        c.host = static_cast<uint8_t *>(aligned_alloc(4096, std::max<uint64_t>(4096, (tot + 4095) & ~4095ull)));
        if (!c.host) throw std::runtime_error("out of host memory");
        std::vector<std::thread> th;
        const unsigned nt = 16;
        for (unsigned t = 0; t < nt; t++)
            th.emplace_back([&, t] {
                for (size_t i = t; i < c.abs.size(); i += nt) {
                    const int fd = open(c.abs[i].c_str(), O_RDONLY);
                    uint64_t got = 0;
                    while (fd >= 0 && got < c.len[i]) {
                        const ssize_t r = pread(fd, c.host + c.off[i] + got, c.len[i] - got, (off_t)got);
                        if (r <= 0) break;
                        got += (uint64_t)r;
                    }
                    if (fd >= 0) close(fd);
                    if (got != c.len[i]) throw std::runtime_error("cannot read " + c.abs[i]);
                }
            });
        for (auto &t : th) t.join();
    }
    return c;
}

// one pipeline for the flat modes; `inbox` (its deliver() context) points at
// results / t_submit / lat
Pass run_ingest(const Corpus &c, const std::string &mode, syncr_ingest *g, Fill *fill, std::vector<Result> &results,
                std::vector<Clock::time_point> &t_submit, std::vector<double> &lat) {
    results.clear();
    lat.clear();
    t_submit.assign(c.abs.size(), Clock::time_point());
    Pass p;
    double before[5];
    syncr_ingest_timing(g, before, 5);
    const auto t0 = Clock::now();
    constexpr uint64_t PIECE = 2ull << 20, PAR = 4ull << 20;
    for (size_t i = 0; i < c.abs.size(); i++) {
        t_submit[i] = Clock::now();
        if (mode == "files") {
            syncr::cdc_check(syncr_ingest_submit_file(g, c.abs[i].c_str(), i), "submit_file");
        } else if (mode == "mem") {
            syncr::cdc_check(syncr_ingest_submit(g, c.host + c.off[i], c.len[i], i), "submit");
        } else {
            uint8_t *dst = nullptr;
            syncr::cdc_check(syncr_ingest_reserve(g, c.len[i], &dst), "reserve");
            const uint8_t *src = c.host + c.off[i];
            const uint64_t n = c.len[i];
            const auto f0 = Clock::now();
            if (n <= PAR) {
                memcpy(dst, src, n);
            } else {
                fill->parallel((unsigned)((n + PIECE - 1) / PIECE), [&](unsigned k) {
                    const uint64_t a = (uint64_t)k * PIECE, b = std::min<uint64_t>(n, a + PIECE);
                    memcpy(dst + a, src + a, b - a);
                });
            }
            p.fill_seconds += secs(f0, Clock::now());
            syncr::cdc_check(syncr_ingest_commit(g, i), "commit");
        }
    }
    syncr::cdc_check(syncr_ingest_flush(g), "flush");
    p.seconds = secs(t0, Clock::now());
    stage_delta(g, p.stage, before);
    p.results = results;
    p.latency_us = lat;
    p.entries = c.abs.size();
    return p;
}

double pct(std::vector<double> v, double q) {
    if (v.empty()) return 0;
    std::sort(v.begin(), v.end());
    return v[std::min(v.size() - 1, (size_t)(q * (double)(v.size() - 1) + 0.5))];
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s per_file|walk|files|mem|zero_copy ROOT OUT [--reps R] [--device D]\n", argv[0]);
        return 2;
    }
    const std::string mode = argv[1], root = argv[2], outp = argv[3];
    int reps = 2;
    int32_t device = 0;
    for (int i = 4; i + 1 < argc; i += 2) {
        if (!strcmp(argv[i], "--reps")) reps = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "--device")) device = atoi(argv[i + 1]);
    }
    try {
        if (mode == "list") {          // the walk's order only (no device): path, type, size per line
            syncr::walk_tree(root, [&](const std::string &, syncr::FileSystemEntry &&e) {
                printf("%s\t%s\t%llu\t%s\n", e.path.c_str(),
                       e.entry_type == syncr::EntryType::File ? "F" : e.entry_type == syncr::EntryType::Directory ? "D" : "S",
                       (unsigned long long)e.size, e.target.c_str());
            });
            return 0;
        }
        Corpus c;
        const bool flat = mode == "files" || mode == "mem" || mode == "zero_copy";
        if (flat) c = list_files(root, mode != "files");
        uint64_t bytes = 0, files = 0;
        syncr::walk_tree(root, [&](const std::string &, syncr::FileSystemEntry &&e) {
            if (e.entry_type == syncr::EntryType::File) {
                bytes += e.size;
                files++;
            }
        });
        // the pipelines are opened once, before the passes (the Rust shim keeps its pipelines)
        const syncr_cdc_params prm = prod_params();
        std::unique_ptr<syncr::GpuWalk> walk;
        syncr_ingest *g = nullptr;
        std::vector<Result> results;
        std::vector<Clock::time_point> t_submit;
        std::vector<double> lat;
        Inbox inbox{&results, &c.rel, &t_submit, &lat};
        std::unique_ptr<Fill> fill;
        if (mode == "walk") {
            syncr::GpuWalk::Options o;                           // GpuWalk::open in chunking_gpu.rs
            o.devices = {device};
            walk.reset(new syncr::GpuWalk(o));
        } else if (mode == "per_file") {                         // take_pipeline() in chunking_gpu.rs
            syncr::cdc_check(syncr_ingest_open(device, &prm, 64ull << 20, 1, 4, on_result, &results, &g),
                             "syncr_ingest_open");
        } else if (flat) {
            syncr::cdc_check(syncr_ingest_open(device, &prm, 256ull << 20, 3, 16, on_file, &inbox, &g),
                             "syncr_ingest_open");
            if (mode == "zero_copy") fill.reset(new Fill(15));
        } else {
            throw std::runtime_error("unknown mode " + mode);
        }
        Pass best;
        std::vector<double> all;
        for (int r = 0; r < reps; r++) {
            Pass p = mode == "walk" ? run_walk(root, walk.get())
                   : mode == "per_file" ? run_per_file(root, g, results)
                   : run_ingest(c, mode, g, fill.get(), results, t_submit, lat);
            all.push_back(p.seconds);
            if (r == 0 || p.seconds < best.seconds) best = std::move(p);
        }
        walk.reset();
        if (g) syncr_ingest_close(g);
        FILE *f = fopen(outp.c_str(), "wb");
        if (!f) throw std::runtime_error("cannot write " + outp);
        for (const Result &r : best.results) {
            const uint32_t pl = (uint32_t)r.path.size(), n = (uint32_t)r.chunks.size();
            fwrite(&pl, 4, 1, f);
            fwrite(r.path.data(), 1, pl, f);
            fwrite(&r.status, 4, 1, f);
            fwrite(&n, 4, 1, f);
            if (n) fwrite(r.chunks.data(), sizeof(syncr_chunk_info), n, f);
        }
        fclose(f);
        uint64_t nonzero = 0;
        for (const Result &r : best.results) nonzero += r.status != 0;
        // the files leave in the reference walk's order (per_file / walk) or in submission order
        std::vector<std::string> order;
        if (flat) order = c.rel;
        else
            syncr::walk_tree(root, [&](const std::string &, syncr::FileSystemEntry &&e) {
                if (e.entry_type == syncr::EntryType::File) order.push_back(e.path);
            });
        bool in_order = order.size() == best.results.size();
        for (size_t k = 0; in_order && k < order.size(); k++) in_order = order[k] == best.results[k].path;
        printf("{\"mode\": \"%s\", \"seconds\": %.6f, \"pass_seconds\": [", mode.c_str(), best.seconds);
        for (size_t k = 0; k < all.size(); k++) printf("%s%.6f", k ? ", " : "", all[k]);
        printf("], \"bytes\": %llu, \"files\": %llu, \"entries\": %llu, \"delivered\": %zu, \"status_nonzero\": %llu, "
               "\"in_walk_order\": %s, \"latency_us\": {\"p50\": %.1f, \"p90\": %.1f, \"p99\": %.1f, \"max\": %.1f, \"mean\": %.1f}, "
               "\"host_stage_seconds\": {\"copy\": %.4f, \"read\": %.4f, \"seal\": %.4f, \"wait\": %.4f, "
               "\"deliver\": %.4f}, \"caller_fill_seconds\": %.4f}\n",
               (unsigned long long)bytes, (unsigned long long)files, (unsigned long long)best.entries,
               best.results.size(), (unsigned long long)nonzero, in_order ? "true" : "false", pct(best.latency_us, 0.5),
               pct(best.latency_us, 0.9), pct(best.latency_us, 0.99), pct(best.latency_us, 1.0),
               best.latency_us.empty() ? 0.0
                                       : std::accumulate(best.latency_us.begin(), best.latency_us.end(), 0.0) /
                                             (double)best.latency_us.size(),
               best.stage[0], best.stage[1], best.stage[2], best.stage[3], best.stage[4], best.fill_seconds);
        free(c.host);
    } catch (const std::exception &e) {
        fprintf(stderr, "e2e_driver: %s\n", e.what());
        return 1;
    }
    return 0;
}
