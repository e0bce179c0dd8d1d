// syncr_cdc.hpp -- C++ host mirror of szilu/syncr's chunking interface over the
// C ABI in syncr_cdc.h.  Header-only; link with libsyncr_cdc.so.
//
//   syncr::chunking::{CHUNK_BITS, MAX_CHUNK_SIZE_FACTOR, MAX_CHUNK_SIZE}
//                                     src/chunking.rs:7,10,13
//   syncr::ChunkInfo                  src/protocol/types.rs:24-29 (hash = BLAKE3, util.rs:57-59,
//                                     computed on the GPU by chunk_hashed())
//   syncr::compute_file_chunks()      src/protocol/file_operations.rs:721-788
//   syncr::chunk_data()               tests/chunking_test.rs:170-192
//   syncr::FileSystemEntry            src/protocol/types.rs:37-51
//   syncr::walk_tree()                traverse_and_stream's walk order, file_operations.rs:544-715
//   syncr::GpuWalk                    the batched walk of rust/src/chunking_gpu.rs (GpuWalk)
//
// Error behaviour follows the reference: an unopenable/unreadable file yields
// an empty list (file_operations.rs:727-744).  Engine errors (no device, HIP
// failure) throw syncr::CdcError -- there is no silent CPU fallback.
#pragma once

#include <dirent.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <cstdint>
#include <cstring>
#include <deque>
#include <fstream>
#include <iterator>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "syncr_cdc.h"

namespace syncr {

namespace chunking {
constexpr uint32_t CHUNK_BITS = 20;                                   // src/chunking.rs:7
constexpr uint64_t MAX_CHUNK_SIZE_FACTOR = 16;                        // src/chunking.rs:10
constexpr uint64_t MAX_CHUNK_SIZE = (1ull << CHUNK_BITS) * MAX_CHUNK_SIZE_FACTOR;  // :13
constexpr uint64_t TOKIO_READ_CAP = 2ull * 1024 * 1024;               // tokio File::read cap
}  // namespace chunking

struct ChunkInfo {
    std::array<uint8_t, 32> hash{};  // BLAKE3 of the chunk (util::hash_binary, util.rs:57-59)
    uint64_t offset = 0;
    uint32_t size = 0;
};

class CdcError : public std::runtime_error {
  public:
    CdcError(int32_t code, const std::string &what)
        : std::runtime_error(what + ": " + syncr_cdc_strerror(code)), code_(code) {}
    int32_t code() const { return code_; }

  private:
    int32_t code_;
};

inline void cdc_check(int32_t rc, const char *what) {
    if (rc != SYNCR_CDC_OK) throw CdcError(rc, what);
}

// One engine handle (the role of Bup::new_with_chunk_bits, file_operations.rs:748).
class Chunker {
  public:
    explicit Chunker(uint32_t chunk_bits = chunking::CHUNK_BITS,
                     uint64_t max_chunk = chunking::MAX_CHUNK_SIZE,
                     uint64_t read_cap = chunking::TOKIO_READ_CAP, int32_t device = 0) {
        syncr_cdc_params p{chunk_bits, 0, max_chunk, read_cap};
        cdc_check(syncr_cdc_open(device, &p, &h_), "syncr_cdc_open");
    }
    ~Chunker() { syncr_cdc_close(h_); }
    Chunker(const Chunker &) = delete;
    Chunker &operator=(const Chunker &) = delete;
    Chunker(Chunker &&o) noexcept : h_(std::exchange(o.h_, nullptr)) {}

    syncr_cdc *handle() const { return h_; }

    // bytes -> chunk boundaries (one file, production or ideal per the handle)
    std::vector<ChunkInfo> chunk(const uint8_t *data, uint64_t len) {
        std::vector<syncr_cut> cuts(len / 4096 + 64);
        uint64_t n = 0;
        int32_t rc = syncr_cdc_chunk_host(h_, data, len, cuts.data(), cuts.size(), &n);
        if (rc == SYNCR_CDC_ERANGE) {
            cuts.resize(n);
            rc = syncr_cdc_chunk_host(h_, data, len, cuts.data(), cuts.size(), &n);
        }
        cdc_check(rc, "syncr_cdc_chunk_host");
        std::vector<ChunkInfo> out(n);
        for (uint64_t i = 0; i < n; i++) {
            out[i].offset = cuts[i].offset;
            out[i].size = cuts[i].len;
        }
        return out;
    }
    std::vector<ChunkInfo> chunk(const std::vector<uint8_t> &v) { return chunk(v.data(), v.size()); }

    // bytes -> complete ChunkInfo{hash, offset, size} (boundaries + BLAKE3 on the GPU)
    std::vector<ChunkInfo> chunk_hashed(const uint8_t *data, uint64_t len) {
        std::vector<syncr_chunk_info> cuts(len / 4096 + 64);
        uint64_t n = 0;
        int32_t rc = syncr_cdc_chunk_host_hashed(h_, data, len, cuts.data(), cuts.size(), &n);
        if (rc == SYNCR_CDC_ERANGE) {
            cuts.resize(n);
            rc = syncr_cdc_chunk_host_hashed(h_, data, len, cuts.data(), cuts.size(), &n);
        }
        cdc_check(rc, "syncr_cdc_chunk_host_hashed");
        std::vector<ChunkInfo> out(n);
        for (uint64_t i = 0; i < n; i++) {
            out[i].offset = cuts[i].offset;
            out[i].size = cuts[i].len;
            std::copy(cuts[i].hash, cuts[i].hash + 32, out[i].hash.begin());
        }
        return out;
    }
    std::vector<ChunkInfo> chunk_hashed(const std::vector<uint8_t> &v) { return chunk_hashed(v.data(), v.size()); }

  private:
    syncr_cdc *h_ = nullptr;
};

// compute_file_chunks (file_operations.rs:721-788, hashes as at :757) with the
// reference's error behaviour: open/read failure -> empty list.
inline std::vector<ChunkInfo> compute_file_chunks(const std::string &path, Chunker &c, bool hashed = true) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return {};
    std::vector<uint8_t> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    if (f.bad()) return {};
    return hashed ? c.chunk_hashed(buf) : c.chunk(buf);
}

// chunk_data (tests/chunking_test.rs:170-192): ideal in-memory semantics,
// (offset, size) pairs.
inline std::vector<std::pair<uint64_t, uint64_t>> chunk_data(const uint8_t *data, uint64_t len,
                                                              uint32_t chunk_bits,
                                                              uint64_t max_chunk) {
    Chunker c(chunk_bits, max_chunk, 0);
    std::vector<std::pair<uint64_t, uint64_t>> out;
    for (const ChunkInfo &ci : c.chunk(data, len)) out.emplace_back(ci.offset, ci.size);
    return out;
}

// ---- the directory walk ----------------------------------------------------

enum class EntryType { File, Directory, SymLink };

// FileSystemEntry (src/protocol/types.rs:37-51) as traverse_and_stream fills it
// (file_operations.rs:608-700), plus the engine's status of a file (0, or the
// -errno the reference only logs: :730, :741, :780).
struct FileSystemEntry {
    EntryType entry_type = EntryType::File;
    std::string path;                        // relative to the walk's base
    uint32_t mode = 0, user_id = 0, group_id = 0, created_time = 0, modified_time = 0;
    uint64_t size = 0;                       // files: st_size; directories and symlinks: 0
    std::string target;                      // symlinks: read_link (empty if it failed)
    std::vector<ChunkInfo> chunks;
    int32_t status = 0;
};

// traverse_and_stream's order (file_operations.rs:551-703): a stack of
// directories (last pushed, first read), each directory's entries in readdir
// order without "." and "..", lstat (symlink_metadata, :579) per entry;
// unreadable directories and entries that cannot be lstat'ed are skipped
// (:554-560, :579-585); a directory is visited (its entry emitted) when it is
// met and read later; only files, directories and symlinks are emitted
// (:701-703).  visit(absolute path, entry without chunks) is called per entry.
template <class Visit>
void walk_tree(const std::string &base, Visit &&visit) {
    std::vector<std::string> stack{base};
    while (!stack.empty()) {
        const std::string dir = stack.back();
        stack.pop_back();
        DIR *d = opendir(dir.c_str());
        if (!d) continue;
        std::vector<std::string> names;
        while (struct dirent *de = readdir(d))
            if (strcmp(de->d_name, ".") && strcmp(de->d_name, "..")) names.emplace_back(de->d_name);
        closedir(d);
        for (const std::string &name : names) {
            const std::string path = dir + "/" + name;
            struct stat st;
            if (lstat(path.c_str(), &st) != 0) continue;
            FileSystemEntry e;
            e.path = path.compare(0, base.size() + 1, base + "/") == 0 ? path.substr(base.size() + 1) : path;
            e.mode = st.st_mode;
            e.user_id = st.st_uid;
            e.group_id = st.st_gid;
            e.created_time = (uint32_t)st.st_ctime;
            e.modified_time = (uint32_t)st.st_mtime;
            if (S_ISREG(st.st_mode)) {
                e.entry_type = EntryType::File;
                e.size = (uint64_t)st.st_size;
            } else if (S_ISLNK(st.st_mode)) {
                e.entry_type = EntryType::SymLink;
                std::string t(4096, '\0');
                const ssize_t n = readlink(path.c_str(), &t[0], t.size());
                e.target = n > 0 ? t.substr(0, (size_t)n) : std::string();
            } else if (S_ISDIR(st.st_mode)) {
                e.entry_type = EntryType::Directory;
                stack.push_back(path);
            } else {
                continue;
            }
            visit(path, std::move(e));
        }
    }
}

// The batched walk (GpuWalk in rust/src/chunking_gpu.rs; the patched
// traverse_and_stream in integration/file_operations.diff): each regular file
// is submitted to one ingest pipeline (syncr_ingest_submit_file) instead of
// being awaited; entries leave in the walk's order, a file's once its
// ChunkInfo list is back, everything behind it waiting for it.  push_*() may
// run batches and deliver results; pop_ready() hands out the ready head of the
// queue; finish() flushes the pipeline so that every entry becomes ready.
class GpuWalk {
  public:
    struct Options {
        std::vector<int32_t> devices{0};
        uint64_t batch_bytes = 256ull << 20;
        uint32_t depth = 3;
        uint32_t copy_threads = 16;
        syncr_cdc_params params{chunking::CHUNK_BITS, 0, chunking::MAX_CHUNK_SIZE, chunking::TOKIO_READ_CAP};
    };
    GpuWalk() : GpuWalk(Options()) {}
    explicit GpuWalk(const Options &o) {
        cdc_check(syncr_ingest_open_multi(o.devices.data(), (uint32_t)o.devices.size(), &o.params, o.batch_bytes,
                                          o.depth, o.copy_threads, &GpuWalk::deliver, this, &g_),
                  "syncr_ingest_open_multi");
    }
    ~GpuWalk() { syncr_ingest_close(g_); }
    GpuWalk(const GpuWalk &) = delete;
    GpuWalk &operator=(const GpuWalk &) = delete;

    void push_file(const std::string &abs_path, FileSystemEntry e) {
        q_.push_back({std::move(e), false});
        waiting_.push_back(&q_.back());
        cdc_check(syncr_ingest_submit_file(g_, abs_path.c_str(), next_tag_++), "syncr_ingest_submit_file");
    }
    void push_entry(FileSystemEntry e) { q_.push_back({std::move(e), true}); }
    bool pop_ready(FileSystemEntry &out) {
        if (q_.empty() || !q_.front().ready) return false;
        out = std::move(q_.front().e);
        q_.pop_front();
        return true;
    }
    void finish() { cdc_check(syncr_ingest_flush(g_), "syncr_ingest_flush"); }
    size_t queued() const { return q_.size(); }
    syncr_ingest *handle() const { return g_; }

  private:
    struct Pending {
        FileSystemEntry e;
        bool ready;
    };
    // results arrive in submission order, on this thread, inside submit / flush
    static void deliver(void *ctx, uint64_t, int32_t status, const syncr_chunk_info *c, uint64_t n) {
        GpuWalk *w = static_cast<GpuWalk *>(ctx);
        Pending *p = w->waiting_.front();
        w->waiting_.pop_front();
        p->e.status = status;
        p->e.chunks.resize(n);
        for (uint64_t i = 0; i < n; i++) {
            p->e.chunks[i].offset = c[i].offset;
            p->e.chunks[i].size = c[i].len;
            std::copy(c[i].hash, c[i].hash + 32, p->e.chunks[i].hash.begin());
        }
        p->ready = true;
    }
    syncr_ingest *g_ = nullptr;
    std::deque<Pending> q_;             // the walk's order (references stay valid: push_back / pop_front)
    std::deque<Pending *> waiting_;     // files without their result, in submission order
    uint64_t next_tag_ = 0;
};

}  // namespace syncr
