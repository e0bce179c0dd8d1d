// cache.cpp -- persistent chunk cache (skip re-chunking unchanged files).
//
// Restates the reference's ChildCache (src/cache.rs:138-260): one entry per
// file path holding the file's metadata and its HashChunk list
// (CacheEntry{mt, uid, gid, ct, sz, md, ch}, :20-35); an entry is valid when its
// mtime equals the file's current mtime (is_valid, :167-179; get_chunks,
// :183-203; set, :207-218).  The reference keeps it in redb and never wires it
// into the scan; here it is consulted by the ingest pipeline's submit_file.
// One deliberate strengthening: the size must match too (a same-second
// rewrite of a different length can never reuse the old chunk list).
//
// Storage: an append-only log, last record per key wins, each record guarded
// by an FNV-1a-64 checksum so a torn tail (crash mid-append) is dropped on
// load.  The log is rewritten (compacted) on close when it holds more than
// twice the live records.
#include <stdio.h>
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

constexpr char MAGIC[8] = {'S', 'Y', 'N', 'C', 'R', 'C', 'C', '1'};

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

}  // namespace

struct syncr_cache {
    std::string path;                  // empty: in memory only
    FILE *log = nullptr;
    std::unordered_map<std::string, Entry> map;
    uint64_t records = 0;              // records in the log (live + superseded)
    uint64_t stats[3] = {0, 0, 0};     // hits, misses, puts
    std::mutex mu;
};

namespace {

// record: u32 keylen | key | u32 mtime | u64 size | u64 n | n * 48 B | u64 fnv(all before)
bool write_record(FILE *f, const std::string &key, const Entry &e) {
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
    return fwrite(buf.data(), 1, buf.size(), f) == buf.size();
}

bool load(syncr_cache *c) {
    FILE *f = fopen(c->path.c_str(), "rb");
    if (!f) return true;                               // a new cache
    char m[8];
    if (fread(m, 1, 8, f) != 8 || memcmp(m, MAGIC, 8) != 0) {
        fclose(f);
        return false;                                  // not a cache file: refuse to clobber it
    }
    long good = 8;
    for (;;) {
        uint32_t kl;
        if (fread(&kl, 1, 4, f) != 4 || kl > (1u << 20)) break;
        std::string key(kl, '\0');
        Entry e;
        uint64_t n = 0, h = 0;
        if (fread(&key[0], 1, kl, f) != kl || fread(&e.mtime, 1, 4, f) != 4 || fread(&e.size, 1, 8, f) != 8 ||
            fread(&n, 1, 8, f) != 8 || n > (e.size + 1))
            break;
        e.chunks.resize(n);
        if (n && fread(e.chunks.data(), sizeof(syncr_chunk_info), n, f) != n) break;
        if (fread(&h, 1, 8, f) != 8) break;
        uint64_t x = fnv(&kl, 4);
        x = fnv(key.data(), kl, x);
        x = fnv(&e.mtime, 4, x);
        x = fnv(&e.size, 8, x);
        x = fnv(&n, 8, x);
        if (n) x = fnv(e.chunks.data(), n * sizeof(syncr_chunk_info), x);
        if (x != h) break;                             // torn / corrupt tail
        c->map[key] = std::move(e);
        c->records++;
        good = ftell(f);
    }
    fclose(f);
    if (truncate(c->path.c_str(), good) != 0) return false;   // drop a torn tail before appending
    return true;
}

bool rewrite(syncr_cache *c) {
    const std::string tmp = c->path + ".tmp";
    FILE *f = fopen(tmp.c_str(), "wb");
    if (!f) return false;
    bool ok = fwrite(MAGIC, 1, 8, f) == 8;
    for (const auto &kv : c->map) ok = ok && write_record(f, kv.first, kv.second);
    ok = (fflush(f) == 0) && ok;
    ok = (fsync(fileno(f)) == 0) && ok;
    fclose(f);
    if (!ok || rename(tmp.c_str(), c->path.c_str()) != 0) {
        unlink(tmp.c_str());
        return false;
    }
    c->records = c->map.size();
    return true;
}

}  // namespace

extern "C" {

int32_t syncr_cache_open(const char *path, syncr_cache **out) {
    if (!out) return SYNCR_CDC_EINVAL;
    *out = nullptr;
    syncr_cache *c = new (std::nothrow) syncr_cache();
    if (!c) return SYNCR_CDC_ENOMEM;
    try {
        if (path && *path) {
            c->path = path;
            if (!load(c)) {
                delete c;
                return SYNCR_CDC_EIO;
            }
            struct stat st;
            const bool fresh = stat(path, &st) != 0 || st.st_size == 0;
            c->log = fopen(path, "ab");
            if (!c->log || (fresh && fwrite(MAGIC, 1, 8, c->log) != 8)) {
                if (c->log) fclose(c->log);
                delete c;
                return SYNCR_CDC_EIO;
            }
        }
    } catch (...) {
        delete c;
        return SYNCR_CDC_ENOMEM;
    }
    *out = c;
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
        if (c->log) {
            if (!write_record(c->log, key, e)) return SYNCR_CDC_EIO;
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
    if (c->log && (fflush(c->log) != 0 || fsync(fileno(c->log)) != 0)) return SYNCR_CDC_EIO;
    return SYNCR_CDC_OK;
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
        if (c->log) {
            fflush(c->log);
            fclose(c->log);
            c->log = nullptr;
            if (c->records > 2 * c->map.size() + 16) (void)rewrite(c);
        }
    }
    delete c;
}

}  // extern "C"
