// walk_sequence_test.cpp -- the batched walk's exact call order through the C ABI.
//
// The traverse_and_stream patch (integration/file_operations.diff, GpuWalk in
// rust/src/chunking_gpu.rs) walks the tree in the reference's order
// (src/protocol/file_operations.rs:551-703), submits every regular file to one
// ingest pipeline (syncr_ingest_submit_file), and sends the entries (:707) in
// walk order as the results come back (flush at the walk's end).  This test
// replays that order with syncr::walk_tree + syncr::GpuWalk (include/
// syncr_cdc.hpp, the same calls) over a nested tree and checks
//   - the sequence of entries (path, type, size, symlink target) equals the
//     reference walk's, for every pipeline shape below;
//   - every file's status and ChunkInfo list (boundaries and BLAKE3) equals the
//     oracle's (oracle/liborc_bup.so: the literal compute_file_chunks loop) on
//     its bytes: random, empty, b"small", periodic, constant, larger than a
//     batch, many small files, a file that vanishes between the directory read
//     and its open (-ENOENT, no chunks: :727-733), an unreadable file (-EACCES,
//     no chunks, when the test does not run as root), a directory symlink and an
//     empty directory.
// Pipelines: one device with small batches (many seals, an oversized file in
// its own batch, depth 2), the same pipeline walked again, and devices {0, 0}.
//
// Test infrastructure (links the oracle); run by tests/test_cpp_mirror.py.
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include "syncr_cdc.hpp"

extern "C" {
uint64_t orc_chunk_production(const uint8_t *file, uint64_t F, uint32_t bits, uint64_t max_chunk, uint64_t read_cap,
                              uint64_t *ends, uint64_t ends_cap);
uint64_t orc_chunk_production_window(const uint8_t *file, uint64_t F, uint32_t bits, uint64_t max_chunk,
                                     uint64_t read_cap, uint64_t *ends, uint64_t ends_cap);
void orc_blake3(const uint8_t *in, uint64_t len, uint8_t out[32]);
void orc_xorshift_fill(uint64_t seed, uint64_t discard, uint8_t *out, uint64_t n);
}

namespace {

int failures = 0;
#define CHECK(cond, ...)                                                  \
    do {                                                                  \
        if (!(cond)) {                                                    \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);          \
            fprintf(stderr, __VA_ARGS__);                                 \
            fprintf(stderr, "\n");                                        \
            ++failures;                                                   \
        }                                                                 \
    } while (0)

std::vector<uint8_t> random_bytes(uint64_t seed, size_t n) {
    std::vector<uint8_t> v(n);
    if (n) orc_xorshift_fill(seed, 64, v.data(), n);
    return v;
}

// a 64-byte period that hits at chunk_bits 20 once per period (as shim_sequence_test.cpp)
std::vector<uint8_t> periodic(size_t n) {
    std::vector<uint8_t> pat(64);
    for (uint64_t seed = 1;; seed++) {
        orc_xorshift_fill(seed * 0x9E3779B97F4A7C15ull, 64, pat.data(), 62);
        int64_t rest = 0;
        for (int k = 0; k < 62; k++) rest += (int64_t)(64 - k) * pat[k];
        const int64_t t = ((0x17BF - rest) % 65536 + 65536) % 65536;
        for (int x1 = 0; x1 < 256; x1++) {
            const int64_t x0 = t - 2 * x1;
            if (x0 < 0 || x0 > 255) continue;
            pat[62] = (uint8_t)x1;
            pat[63] = (uint8_t)x0;
            int64_t S = 0;
            for (int k = 0; k < 64; k++) S += pat[k];
            if ((1984 + S) % 16 == 15) {
                std::vector<uint8_t> v(n);
                for (size_t i = 0; i < n; i++) v[i] = pat[i % 64];
                return v;
            }
        }
    }
}

std::vector<syncr::ChunkInfo> oracle_chunks(const std::vector<uint8_t> &f, bool periodic_file) {
    std::vector<uint64_t> ends(f.size() + 1);
    const uint64_t n = periodic_file
        ? orc_chunk_production_window(f.data(), f.size(), 20, 16ull << 20, 2ull << 20, ends.data(), ends.size())
        : orc_chunk_production(f.data(), f.size(), 20, 16ull << 20, 2ull << 20, ends.data(), ends.size());
    std::vector<syncr::ChunkInfo> out(n);
    uint64_t s = 0;
    for (uint64_t k = 0; k < n; k++) {
        out[k].offset = s;
        out[k].size = (uint32_t)(ends[k] - s);
        orc_blake3(f.data() + s, ends[k] - s, out[k].hash.data());
        s = ends[k];
    }
    return out;
}

bool write_file(const std::string &path, const std::vector<uint8_t> &v) {
    FILE *f = fopen(path.c_str(), "wb");
    if (!f) return false;
    const bool ok = v.empty() || fwrite(v.data(), 1, v.size(), f) == v.size();
    return fclose(f) == 0 && ok;
}

struct Want {
    std::vector<uint8_t> bytes;
    bool periodic = false;
    int32_t status = 0;              // 0, or the -errno the engine reports (no chunks then)
};

const char *type_name(syncr::EntryType t) {
    return t == syncr::EntryType::File ? "file" : t == syncr::EntryType::Directory ? "dir" : "symlink";
}

// one walk through `w`, entries in the order they are sent
std::vector<syncr::FileSystemEntry> gpu_walk(const std::string &root, syncr::GpuWalk &w, const std::string &vanish,
                                             const std::vector<uint8_t> &vanish_bytes) {
    std::vector<syncr::FileSystemEntry> sent;
    syncr::FileSystemEntry out;
    syncr::walk_tree(root, [&](const std::string &abs, syncr::FileSystemEntry &&e) {
        if (e.entry_type == syncr::EntryType::File) {
            if (e.path == vanish) unlink(abs.c_str());        // gone between read_dir and open
            w.push_file(abs, std::move(e));
        } else {
            w.push_entry(std::move(e));
        }
        while (w.pop_ready(out)) sent.push_back(std::move(out));
    });
    w.finish();
    while (w.pop_ready(out)) sent.push_back(std::move(out));
    CHECK(w.queued() == 0, "%zu entries still queued after finish", w.queued());
    write_file(root + "/" + vanish, vanish_bytes);             // back for the next walk
    return sent;
}

}  // namespace

int main() {
    int32_t ndev = 0;
    if (syncr_cdc_device_count(&ndev) != SYNCR_CDC_OK || ndev < 1) {
        fprintf(stderr, "no HIP device\n");
        return 2;
    }
    char tmpl[] = "/tmp/syncr_walk_XXXXXX";
    const char *dir = mkdtemp(tmpl);
    if (!dir) {
        perror("mkdtemp");
        return 2;
    }
    const std::string root(dir);
    std::map<std::string, Want> files;                       // relative path -> expectation
    auto add = [&](const std::string &rel, std::vector<uint8_t> bytes, bool per = false) {
        if (!write_file(root + "/" + rel, bytes)) {
            fprintf(stderr, "cannot write %s\n", rel.c_str());
            exit(2);
        }
        files[rel] = Want{std::move(bytes), per, 0};
    };
    mkdir((root + "/sub1").c_str(), 0755);
    mkdir((root + "/sub1/sub2").c_str(), 0755);
    mkdir((root + "/emptydir").c_str(), 0755);
    mkdir((root + "/many").c_str(), 0755);
    add("a.bin", random_bytes(0xA1, 3u << 20));
    add("empty", {});
    add("small", {'s', 'm', 'a', 'l', 'l'});                   // protocol_list_test.rs:305-322
    add("sub1/r1", random_bytes(0x51, 9u << 20 | 13));
    add("sub1/big", random_bytes(0xB16, 40u << 20 | 7));       // larger than the 16 MiB test batch
    add("sub1/periodic", periodic(5u << 20 | 3), true);
    add("sub1/sub2/const", std::vector<uint8_t>(20u << 20, 0xAB));
    add("sub1/sub2/unreadable", random_bytes(0x0E, 1u << 20));
    add("sub1/sub2/vanishing", random_bytes(0x7A, 300000));
    for (int i = 0; i < 300; i++)
        add("many/f" + std::to_string(i), random_bytes(0x1000 + i, 1024 + (size_t)i * 61));
    if (symlink("../sub1", (root + "/sub1/sub2/link").c_str()) != 0) perror("symlink");
    chmod((root + "/sub1/sub2/unreadable").c_str(), 0);
    {
        const int fd = open((root + "/sub1/sub2/unreadable").c_str(), O_RDONLY);
        if (fd < 0) files["sub1/sub2/unreadable"].status = -errno;     // not root: EACCES, no chunks
        else close(fd);                                               // root reads it: chunks as usual
    }
    const std::string vanish = "sub1/sub2/vanishing";
    const std::vector<uint8_t> vanish_bytes = files[vanish].bytes;
    files[vanish].status = -ENOENT;

    // the reference walk's sequence (no chunking)
    std::vector<syncr::FileSystemEntry> ref;
    syncr::walk_tree(root, [&](const std::string &, syncr::FileSystemEntry &&e) { ref.push_back(std::move(e)); });
    CHECK(ref.size() == files.size() + 5, "reference walk: %zu entries", ref.size());

    std::map<std::string, std::vector<syncr::ChunkInfo>> want_chunks;
    for (auto &kv : files)
        if (!kv.second.status) want_chunks[kv.first] = oracle_chunks(kv.second.bytes, kv.second.periodic);

    auto check_walk = [&](const std::vector<syncr::FileSystemEntry> &sent, const char *what) {
        CHECK(sent.size() == ref.size(), "%s: %zu entries sent, the walk has %zu", what, sent.size(), ref.size());
        for (size_t k = 0; k < std::min(sent.size(), ref.size()); k++) {
            const auto &a = sent[k], &b = ref[k];
            if (a.path != b.path || a.entry_type != b.entry_type || a.size != b.size || a.target != b.target) {
                CHECK(false, "%s: entry %zu is %s %s, the walk has %s %s", what, k, type_name(a.entry_type),
                      a.path.c_str(), type_name(b.entry_type), b.path.c_str());
                return;
            }
            if (a.entry_type != syncr::EntryType::File) {
                CHECK(a.chunks.empty() && a.status == 0, "%s: %s has chunks", what, a.path.c_str());
                continue;
            }
            const Want &w = files[a.path];
            CHECK(a.status == w.status, "%s: %s status %d, want %d", what, a.path.c_str(), a.status, w.status);
            const std::vector<syncr::ChunkInfo> none;
            const auto &wc = w.status ? none : want_chunks[a.path];
            bool same = a.chunks.size() == wc.size();
            for (size_t i = 0; same && i < wc.size(); i++)
                same = a.chunks[i].offset == wc[i].offset && a.chunks[i].size == wc[i].size &&
                       a.chunks[i].hash == wc[i].hash;
            CHECK(same, "%s: %s: %zu chunks differ from the oracle's %zu", what, a.path.c_str(), a.chunks.size(),
                  wc.size());
        }
    };

    try {
        syncr::GpuWalk::Options o;
        o.batch_bytes = 16ull << 20;                           // many seals; sub1/big gets its own batch
        o.depth = 2;
        o.copy_threads = 4;
        {
            syncr::GpuWalk w(o);
            check_walk(gpu_walk(root, w, vanish, vanish_bytes), "one device");
            check_walk(gpu_walk(root, w, vanish, vanish_bytes), "one device, walked again");
            uint64_t st[4];
            CHECK(syncr_ingest_stats(w.handle(), st) == SYNCR_CDC_OK && st[2] >= 6, "batches: %llu",
                  (unsigned long long)st[2]);
        }
        o.devices = {0, 0};
        {
            syncr::GpuWalk w(o);
            check_walk(gpu_walk(root, w, vanish, vanish_bytes), "devices {0,0}");
        }
        {
            syncr::GpuWalk w;                                  // the shim's defaults (256 MiB, depth 3)
            check_walk(gpu_walk(root, w, vanish, vanish_bytes), "defaults");
        }
    } catch (const std::exception &e) {
        CHECK(false, "engine error: %s", e.what());
    }

    chmod((root + "/sub1/sub2/unreadable").c_str(), 0644);
    const std::string rm = "rm -rf '" + root + "'";
    if (system(rm.c_str()) != 0) fprintf(stderr, "could not remove %s\n", root.c_str());
    if (failures) {
        fprintf(stderr, "%d failures\n", failures);
        return 1;
    }
    printf("walk sequence: all checks passed\n");
    return 0;
}
