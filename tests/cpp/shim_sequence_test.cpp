// shim_sequence_test.cpp -- the Rust shim's exact call sequence through the C ABI.
//
// rust/src/chunking_gpu.rs drives libsyncr_cdc.so in two ways; this test makes
// the same calls in the same order, from C++, and checks every result against
// the CPU oracle (oracle/liborc_bup.so: the literal compute_file_chunks loop,
// src/protocol/file_operations.rs:721-788, and the BLAKE3 restatement):
//
//  1. GpuPipeline::chunk_file (the call site in compute_file_chunks):
//     syncr_ingest_open(device 0, params(), 64 MiB, depth 1, 4 threads, deliver)
//     then per file submit_file(path, 0) -> flush -> exactly one callback ->
//     next file, and syncr_ingest_close at the end.  Files: random of several
//     sizes, larger than the batch (its own batch), empty, the reference's
//     b"small", periodic-64, constant bytes, a missing path (status -ENOENT, no
//     chunks: file_operations.rs:727-733), a directory (-EISDIR).
//  2. GpuChunker::chunk: syncr_cdc_chunk_host_hashed with a capacity guess that
//     is too small -> SYNCR_CDC_ERANGE with the exact count -> the retry.
//
// Test infrastructure (links the oracle); run by tests/test_cpp_mirror.py.
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include <sys/stat.h>
#include <unistd.h>

#include "syncr_cdc.h"

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

struct Delivered {
    uint64_t tag;
    int32_t status;
    std::vector<syncr_chunk_info> chunks;
};

// the shim's `deliver` callback: results appended in submission order
void deliver(void *ctx, uint64_t tag, int32_t status, const syncr_chunk_info *chunks, uint64_t n) {
    auto *inbox = static_cast<std::vector<Delivered> *>(ctx);
    inbox->push_back({tag, status, std::vector<syncr_chunk_info>(chunks, chunks + n)});
}

syncr_cdc_params shim_params() {      // chunking_gpu.rs params(): src/chunking.rs:7-13 + the 2 MiB read cap
    syncr_cdc_params p;
    p.chunk_bits = 20;
    p.flags = 0;
    p.max_chunk = 16ull << 20;
    p.read_cap = 2ull << 20;
    return p;
}

// the oracle's ChunkInfo list for one file's bytes (production semantics)
std::vector<syncr_chunk_info> oracle_chunks(const std::vector<uint8_t> &f, bool periodic) {
    std::vector<uint64_t> ends(f.size() + 1);
    const uint64_t n = periodic
        ? orc_chunk_production_window(f.data(), f.size(), 20, 16ull << 20, 2ull << 20, ends.data(), ends.size())
        : orc_chunk_production(f.data(), f.size(), 20, 16ull << 20, 2ull << 20, ends.data(), ends.size());
    std::vector<syncr_chunk_info> out(n);
    uint64_t s = 0;
    for (uint64_t k = 0; k < n; k++) {
        out[k].offset = s;
        out[k].len = (uint32_t)(ends[k] - s);
        out[k].file = 0;
        orc_blake3(f.data() + s, ends[k] - s, out[k].hash);
        s = ends[k];
    }
    return out;
}

bool same(const std::vector<syncr_chunk_info> &a, const std::vector<syncr_chunk_info> &b, const char *what) {
    if (a.size() != b.size()) {
        fprintf(stderr, "%s: %zu chunks vs %zu from the oracle\n", what, a.size(), b.size());
        return false;
    }
    for (size_t k = 0; k < a.size(); k++)
        if (a[k].offset != b[k].offset || a[k].len != b[k].len || memcmp(a[k].hash, b[k].hash, 32) != 0) {
            fprintf(stderr, "%s: chunk %zu differs (%llu+%u vs %llu+%u)\n", what, k,
                    (unsigned long long)a[k].offset, a[k].len, (unsigned long long)b[k].offset, b[k].len);
            return false;
        }
    return true;
}

std::vector<uint8_t> random_bytes(uint64_t seed, size_t n) {
    std::vector<uint8_t> v(n);
    if (n) orc_xorshift_fill(seed, 64, v.data(), n);
    return v;
}

// a 64-byte period whose extension hits the edge test at chunk_bits 20 once per
// period (as benchlib.workloads.periodic_pattern): 62 random bytes, the last two
// (weights 2 and 1) solved for W = 0x17BF mod 2^16, kept when S = 15 mod 16
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

bool write_file(const std::string &path, const std::vector<uint8_t> &v) {
    FILE *f = fopen(path.c_str(), "wb");
    if (!f) return false;
    const bool ok = v.empty() || fwrite(v.data(), 1, v.size(), f) == v.size();
    return fclose(f) == 0 && ok;
}

}  // namespace

int main() {
    int32_t ndev = 0;
    if (syncr_cdc_device_count(&ndev) != SYNCR_CDC_OK || ndev < 1) {
        fprintf(stderr, "no HIP device\n");
        return 2;
    }
    char tmpl[] = "/tmp/syncr_shim_XXXXXX";
    const char *dir = mkdtemp(tmpl);
    if (!dir) {
        perror("mkdtemp");
        return 2;
    }
    const std::string d(dir);

    // ---- 1. the per-file pipeline of compute_file_chunks_gpu ----------------
    struct Case {
        std::string name;
        std::vector<uint8_t> bytes;
        bool exists, periodic;
        int32_t status;                // expected
    };
    std::vector<Case> cases;
    cases.push_back({"random_9MiB", random_bytes(0x5151, 9u << 20 | 13), true, false, 0});
    cases.push_back({"random_70MiB_own_batch", random_bytes(0x7070, 70u << 20 | 5), true, false, 0});
    cases.push_back({"empty", {}, true, false, 0});
    cases.push_back({"small", {'s', 'm', 'a', 'l', 'l'}, true, false, 0});     // protocol_list_test.rs:305-322
    cases.push_back({"periodic_5MiB", periodic(5u << 20 | 3), true, true, 0});
    cases.push_back({"constant_20MiB", std::vector<uint8_t>(20u << 20, 0xAB), true, false, 0});
    cases.push_back({"missing", {}, false, false, -ENOENT});
    cases.push_back({"random_1MiB", random_bytes(0x1111, 1u << 20), true, false, 0});
    for (auto &c : cases)
        if (c.exists && !write_file(d + "/" + c.name, c.bytes)) {
            fprintf(stderr, "cannot write %s\n", c.name.c_str());
            return 2;
        }
    mkdir((d + "/a_directory").c_str(), 0755);

    std::vector<Delivered> inbox;
    syncr_ingest *g = nullptr;
    const syncr_cdc_params p = shim_params();
    int32_t rc = syncr_ingest_open(0, &p, 64ull << 20, 1, 4, deliver, &inbox, &g);
    CHECK(rc == SYNCR_CDC_OK && g, "syncr_ingest_open rc=%d", rc);
    if (!g) return 1;
    for (int round = 0; round < 2; round++) {           // the pool reuses a pipeline across files
        for (const auto &c : cases) {
            inbox.clear();
            const std::string path = d + "/" + c.name;
            rc = syncr_ingest_submit_file(g, path.c_str(), 0);
            CHECK(rc == SYNCR_CDC_OK, "%s: submit_file rc=%d", c.name.c_str(), rc);
            rc = syncr_ingest_flush(g);
            CHECK(rc == SYNCR_CDC_OK, "%s: flush rc=%d", c.name.c_str(), rc);
            CHECK(inbox.size() == 1, "%s: %zu callbacks after flush", c.name.c_str(), inbox.size());
            if (inbox.size() != 1) continue;
            CHECK(inbox[0].status == c.status, "%s: status %d, want %d", c.name.c_str(), inbox[0].status, c.status);
            const auto want = c.exists ? oracle_chunks(c.bytes, c.periodic) : std::vector<syncr_chunk_info>{};
            CHECK(same(inbox[0].chunks, want, c.name.c_str()), "%s: ChunkInfo list differs from the oracle",
                  c.name.c_str());
        }
        inbox.clear();                                   // a directory: the reference's open/read fails
        rc = syncr_ingest_submit_file(g, (d + "/a_directory").c_str(), 0);
        if (rc == SYNCR_CDC_OK) rc = syncr_ingest_flush(g);
        CHECK(rc == SYNCR_CDC_OK && inbox.size() == 1 && inbox[0].status == -EISDIR && inbox[0].chunks.empty(),
              "directory: rc=%d callbacks=%zu", rc, inbox.size());
    }
    uint64_t st[4] = {0, 0, 0, 0};
    CHECK(syncr_ingest_stats(g, st) == SYNCR_CDC_OK && st[0] >= 2 * 7, "ingest stats: %llu files",
          (unsigned long long)st[0]);
    syncr_ingest_close(g);

    // ---- 2. GpuChunker::chunk: a capacity guess that is too small ------------
    syncr_cdc *h = nullptr;
    rc = syncr_cdc_open(0, &p, &h);
    CHECK(rc == SYNCR_CDC_OK && h, "syncr_cdc_open rc=%d", rc);
    if (h) {
        for (const auto &c : cases) {
            if (!c.exists) continue;
            std::vector<syncr_chunk_info> out(1);       // forces ERANGE whenever there are 2+ chunks
            uint64_t n = 0;
            rc = syncr_cdc_chunk_host_hashed(h, c.bytes.data(), c.bytes.size(), out.data(), out.size(), &n);
            const auto want = oracle_chunks(c.bytes, c.periodic);
            if (want.size() > 1) {
                CHECK(rc == SYNCR_CDC_ERANGE && n == want.size(), "%s: first call rc=%d n=%llu (want ERANGE, %zu)",
                      c.name.c_str(), rc, (unsigned long long)n, want.size());
                out.resize(n);
                rc = syncr_cdc_chunk_host_hashed(h, c.bytes.data(), c.bytes.size(), out.data(), out.size(), &n);
            }
            CHECK(rc == SYNCR_CDC_OK, "%s: rc=%d", c.name.c_str(), rc);
            out.resize(rc == SYNCR_CDC_OK ? n : 0);
            CHECK(same(out, want, c.name.c_str()), "%s: chunk_host_hashed differs from the oracle", c.name.c_str());
        }
        syncr_cdc_close(h);
    }

    for (const auto &c : cases)
        if (c.exists) unlink((d + "/" + c.name).c_str());
    rmdir((d + "/a_directory").c_str());
    rmdir(dir);
    if (failures) {
        fprintf(stderr, "%d failures\n", failures);
        return 1;
    }
    printf("shim sequence: all checks passed\n");
    return 0;
}
