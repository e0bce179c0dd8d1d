// cache.cpp -- persistent chunk cache (skip re-chunking unchanged files).
//
// Restates the reference's ChildCache (src/cache.rs:138-260): one entry per
// file path holding the file's metadata and its HashChunk list
// (CacheEntry{mt, uid, gid, ct, sz, md, ch}, :20-35); an entry is valid when its
// mtime equals the file's current mtime (is_valid, :167-179; get_chunks,
// :183-203; set, :207-218).  The reference keeps it in redb and never wires it
// into the scan; here it is consulted by the ingest pipeline's submit_file.
// Two deliberate strengthenings:
//   * the size must match too (a same-second rewrite of a different length can
//     never reuse the old chunk list);
//   * a cache is bound to one set of chunking parameters (chunk_bits,
//     max_chunk, read_cap -- compile-time constants in the reference,
//     src/chunking.rs:7-13, runtime syncr_cdc_params here), stored in the log
//     header: a log written under other parameters is refused, and so is
//     attaching the cache to an ingest pipeline with other parameters.
//
// Storage: an append-only log (32-byte header, then records), last record per
// key wins, each record guarded by an FNV-1a-64 checksum so a torn tail (crash
// mid-append) is dropped on load.  Each record is one pwrite at the known end
// of the log; a failed or short write is rolled back with ftruncate and the log
// is marked broken (no later append can land behind a torn record).  The log is
// flock'ed for the handle's lifetime (a second writer gets SYNCR_CDC_EBUSY),
// and rewritten (compacted) on close when it holds more than twice the live
// records.
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <sys/file.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdint>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/syncr_cdc.h"

namespace {

constexpr char MAGIC[8] = {'S', 'Y', 'N', 'C', 'R', 'C', 'C', '2'};
// the ABI-v2 log format: no parameter header, so its chunk lists cannot be
// trusted under any parameters; such a log is a stale cache, started afresh
constexpr char MAGIC_V1[8] = {'S', 'Y', 'N', 'C', 'R', 'C', 'C', '1'};
constexpr size_t HDR = 32;              // MAGIC | chunk_bits u32 | flags u32 | max_chunk u64 | read_cap u64

struct Entry {
    uint32_t mtime = 0;
    uint64_t size = 0;
    std::vector<syncr_chunk_info> chunks;
};

uint64_t fnv(const void *p, size_t n, uint64_t h = 0xcbf29ce484222325ull) {
    const uint8_t *b = (const uint8_t *)p;
    for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 0x100000001b3ull;
    return h;
}

void header(const syncr_cdc_params &p, uint8_t out[HDR]) {
    memcpy(out, MAGIC, 8);
    const uint32_t flags = 0;           // resolve variants are exact: not part of the key
    memcpy(out + 8, &p.chunk_bits, 4);
    memcpy(out + 12, &flags, 4);
    memcpy(out + 16, &p.max_chunk, 8);
    memcpy(out + 24, &p.read_cap, 8);
}

bool write_all(int fd, const uint8_t *b, size_t n, off_t at) {
    while (n) {
        const ssize_t r = pwrite(fd, b, n, at);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) return false;
        b += r;
        n -= (size_t)r;
        at += r;
    }
    return true;
}

}  // namespace

struct syncr_cache {
    std::string path;                  // empty: in memory only
    int fd = -1;
    uint64_t end = 0;                  // bytes of valid log (next record goes here)
    bool broken = false;               // a write failed: no more appends
    bool upgraded = false;             // an old-format (SYNCRCC1) log was started afresh
    syncr_cdc_params params{};
    std::unordered_map<std::string, Entry> map;
    uint64_t records = 0;              // records in the log (live + superseded)
    uint64_t stats[3] = {0, 0, 0};     // hits, misses, puts
    std::mutex mu;
};

namespace {

// record: u32 keylen | key | u32 mtime | u64 size | u64 n | n * 48 B | u64 fnv(all before)
std::vector<uint8_t> encode(const std::string &key, const Entry &e) {
    std::vector<uint8_t> buf;
    auto put = [&](const void *p, size_t n) { buf.insert(buf.end(), (const uint8_t *)p, (const uint8_t *)p + n); };
    const uint32_t kl = (uint32_t)key.size();
    const uint64_t n = e.chunks.size();
    put(&kl, 4);
    put(key.data(), kl);
    put(&e.mtime, 4);
    put(&e.size, 8);
    put(&n, 8);
    if (n) put(e.chunks.data(), n * sizeof(syncr_chunk_info));
    const uint64_t h = fnv(buf.data(), buf.size());
    put(&h, 8);
    return buf;
}

// Parse the log at c->fd.  Returns SYNCR_CDC_OK (c->end = valid length, torn
// tail truncated), SYNCR_CDC_EIO for a file that is not a cache log, or
// SYNCR_CDC_EINVAL for a log written under other parameters.
int32_t load(syncr_cache *c) {
    struct stat st;
    if (fstat(c->fd, &st) != 0) return SYNCR_CDC_EIO;
    std::vector<uint8_t> buf((size_t)st.st_size);
    size_t got = 0;
    while (got < buf.size()) {
        const ssize_t r = pread(c->fd, buf.data() + got, buf.size() - got, (off_t)got);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) break;
        got += (size_t)r;
    }
    buf.resize(got);
    uint8_t want[HDR];
    header(c->params, want);
    if (buf.size() >= 8 && memcmp(buf.data(), MAGIC_V1, 8) == 0) {        // stale format: a new cache
        if (ftruncate(c->fd, 0) != 0 || !write_all(c->fd, want, HDR, 0) || fsync(c->fd) != 0) return SYNCR_CDC_EIO;
        c->end = HDR;
        c->upgraded = true;
        return SYNCR_CDC_OK;
    }
    if (buf.size() < HDR) {
        // empty or torn while the header was being written (a prefix of the
        // magic, or of our own header): a new cache
        const size_t k = buf.size() < 8 ? buf.size() : 8;
        if (memcmp(buf.data(), MAGIC, k) != 0) return SYNCR_CDC_EIO;   // not ours: refuse to clobber
        if (memcmp(buf.data(), want, buf.size()) != 0) return SYNCR_CDC_EINVAL;
        if (ftruncate(c->fd, 0) != 0 || !write_all(c->fd, want, HDR, 0) || fsync(c->fd) != 0) return SYNCR_CDC_EIO;
        c->end = HDR;
        return SYNCR_CDC_OK;
    }
    if (memcmp(buf.data(), MAGIC, 8) != 0) return SYNCR_CDC_EIO;
    if (memcmp(buf.data(), want, HDR) != 0) return SYNCR_CDC_EINVAL;   // other chunking parameters
    size_t pos = HDR, good = HDR;
    auto take = [&](void *dst, size_t n) {
        if (buf.size() - pos < n) return false;
        memcpy(dst, buf.data() + pos, n);
        pos += n;
        return true;
    };
    for (;;) {
        uint32_t kl;
        if (!take(&kl, 4) || kl > (1u << 20)) break;
        std::string key(kl, '\0');
        Entry e;
        uint64_t n = 0, h = 0;
        if (!take(&key[0], kl) || !take(&e.mtime, 4) || !take(&e.size, 8) || !take(&n, 8) || n > e.size + 1 ||
            n > (buf.size() - pos) / sizeof(syncr_chunk_info))
            break;
        e.chunks.resize(n);
        if (n && !take(e.chunks.data(), n * sizeof(syncr_chunk_info))) break;
        const uint64_t x = fnv(buf.data() + good, pos - good);
        if (!take(&h, 8) || x != h) break;                   // torn / corrupt tail
        c->map[key] = std::move(e);
        c->records++;
        good = pos;
    }
    if (good < buf.size() && ftruncate(c->fd, (off_t)good) != 0) return SYNCR_CDC_EIO;   // drop a torn tail
    c->end = good;
    return SYNCR_CDC_OK;
}

bool rewrite(syncr_cache *c) {
    const std::string tmp = c->path + ".tmp";
    const int fd = open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    if (fd < 0) return false;
    uint8_t hdr[HDR];
    header(c->params, hdr);
    bool ok = write_all(fd, hdr, HDR, 0);
    off_t at = HDR;
    for (const auto &kv : c->map) {
        if (!ok) break;
        const std::vector<uint8_t> r = encode(kv.first, kv.second);
        ok = write_all(fd, r.data(), r.size(), at);
        at += (off_t)r.size();
    }
    ok = (fsync(fd) == 0) && ok;
    close(fd);
    if (!ok || rename(tmp.c_str(), c->path.c_str()) != 0) {
        unlink(tmp.c_str());
        return false;
    }
    c->records = c->map.size();
    return true;
}

}  // namespace

extern "C" {

int32_t syncr_cache_open(const char *path, const syncr_cdc_params *p, syncr_cache **out) {
    if (!out) return SYNCR_CDC_EINVAL;
    *out = nullptr;
    syncr_cdc_params prm;
    if (p) prm = *p; else syncr_cdc_default_params(&prm);
    if (prm.chunk_bits < 1 || prm.chunk_bits > 31 || prm.max_chunk < 1 || prm.max_chunk > 0xffffffffull)
        return SYNCR_CDC_EINVAL;
    syncr_cache *c = new (std::nothrow) syncr_cache();
    if (!c) return SYNCR_CDC_ENOMEM;
    c->params = prm;
    c->params.flags = 0;
    try {
        if (path && *path) {
            c->path = path;
            c->fd = open(path, O_RDWR | O_CREAT | O_CLOEXEC, 0644);
            if (c->fd < 0) {
                delete c;
                return SYNCR_CDC_EIO;
            }
            if (flock(c->fd, LOCK_EX | LOCK_NB) != 0) {     // one writer per log
                const int e = errno;
                close(c->fd);
                delete c;
                return e == EWOULDBLOCK ? SYNCR_CDC_EBUSY : SYNCR_CDC_EIO;
            }
            const int32_t rc = load(c);
            if (rc) {
                close(c->fd);
                delete c;
                return rc;
            }
        }
    } catch (...) {
        if (c->fd >= 0) close(c->fd);
        delete c;
        return SYNCR_CDC_ENOMEM;
    }
    *out = c;
    return SYNCR_CDC_OK;
}

int32_t syncr_cache_get_params(const syncr_cache *c, syncr_cdc_params *p) {
    if (!c || !p) return SYNCR_CDC_EINVAL;
    *p = c->params;
    return SYNCR_CDC_OK;
}

int32_t syncr_cache_get(syncr_cache *c, const char *key, uint32_t mtime, uint64_t size, syncr_chunk_info *out,
                        uint64_t cap, uint64_t *n_out) {
    if (!c || !key) return SYNCR_CDC_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    auto it = c->map.find(key);
    if (it == c->map.end() || it->second.mtime != mtime || it->second.size != size) {   // cache.rs:175
        c->stats[1]++;
        if (n_out) *n_out = 0;
        return SYNCR_CDC_ENOENT;
    }
    const uint64_t n = it->second.chunks.size();
    if (n_out) *n_out = n;
    if (n > cap || (n && !out)) return SYNCR_CDC_ERANGE;
    if (n) memcpy(out, it->second.chunks.data(), n * sizeof(syncr_chunk_info));
    c->stats[0]++;
    return SYNCR_CDC_OK;
}

int32_t syncr_cache_put(syncr_cache *c, const char *key, uint32_t mtime, uint64_t size,
                        const syncr_chunk_info *chunks, uint64_t n) {
    if (!c || !key || (n && !chunks)) return SYNCR_CDC_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    try {
        Entry e;
        e.mtime = mtime;
        e.size = size;
        e.chunks.assign(chunks, chunks + n);
        for (auto &ci : e.chunks) ci.file = 0;
        if (c->fd >= 0) {
            if (c->broken) return SYNCR_CDC_EIO;
            const std::vector<uint8_t> r = encode(key, e);
            if (!write_all(c->fd, r.data(), r.size(), (off_t)c->end)) {
                // roll back a partial record and never append again: a later
                // record behind a torn one would be dropped on the next load
                (void)ftruncate(c->fd, (off_t)c->end);
                c->broken = true;
                return SYNCR_CDC_EIO;
            }
            c->end += r.size();
            c->records++;
        }
        c->map[key] = std::move(e);
        c->stats[2]++;
    } catch (...) {
        return SYNCR_CDC_ENOMEM;
    }
    return SYNCR_CDC_OK;
}

int32_t syncr_cache_sync(syncr_cache *c) {
    if (!c) return SYNCR_CDC_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    if (c->fd >= 0 && fsync(c->fd) != 0) return SYNCR_CDC_EIO;
    return c->broken ? SYNCR_CDC_EIO : SYNCR_CDC_OK;
}

int32_t syncr_cache_stats(syncr_cache *c, uint64_t *stats4) {
    if (!c || !stats4) return SYNCR_CDC_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    stats4[0] = c->stats[0];
    stats4[1] = c->stats[1];
    stats4[2] = c->stats[2];
    stats4[3] = c->map.size();
    return SYNCR_CDC_OK;
}

void syncr_cache_close(syncr_cache *c) {
    if (!c) return;
    {
        std::lock_guard<std::mutex> g(c->mu);
        if (c->fd >= 0) {
            (void)fsync(c->fd);
            if (!c->broken && c->records > 2 * c->map.size() + 16) (void)rewrite(c);
            close(c->fd);                // releases the flock
            c->fd = -1;
        }
    }
    delete c;
}

}  // extern "C"
