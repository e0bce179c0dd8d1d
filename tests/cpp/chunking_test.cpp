// C++ mirror of the reference's chunker tests, run against the MI355X engine
// through include/syncr_cdc.hpp.  Each TEST names the reference test it follows
// (tests/chunking_test.rs, tests/protocol_list_test.rs).  Exit code 0 = pass.
//
// Build (tests/test_cpp_mirror.py does this):
//   g++ -O2 -std=c++17 -I include tests/cpp/chunking_test.cpp -L syncr_amd -lsyncr_cdc \
//       -Wl,-rpath,<repo>/syncr_amd -o build/chunking_test
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "syncr_cdc.hpp"

static int failures = 0;
#define CHECK(cond)                                                              \
    do {                                                                         \
        if (!(cond)) {                                                           \
            std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #cond); \
            failures++;                                                          \
        }                                                                        \
    } while (0)

// tests/chunking_test.rs:7-8
constexpr uint32_t CHUNK_BITS = 13;
constexpr uint64_t MAX_CHUNK_SIZE = (1ull << CHUNK_BITS) * 16;

using Cuts = std::vector<std::pair<uint64_t, uint64_t>>;

static std::vector<uint8_t> rep(const std::string &s, size_t n) {
    std::vector<uint8_t> v;
    for (size_t i = 0; i < n; i++) v.insert(v.end(), s.begin(), s.end());
    return v;
}

static Cuts chunk_data(const std::vector<uint8_t> &d) {
    return syncr::chunk_data(d.data(), d.size(), CHUNK_BITS, MAX_CHUNK_SIZE);
}

static bool contiguous_cover(const Cuts &c, uint64_t len) {
    uint64_t off = 0;
    for (auto &p : c) {
        if (p.first != off) return false;
        off += p.second;
    }
    return off == len;
}

int main() {
    {   // test_chunking_deterministic (chunking_test.rs:10-23)
        auto content = rep("This is test content that will be chunked. ", 100);
        CHECK(chunk_data(content) == chunk_data(content));
    }
    {   // test_chunking_small_file (:25-34)
        std::string s = "Small file";
        auto c = chunk_data(std::vector<uint8_t>(s.begin(), s.end()));
        CHECK(c.size() == 1 && c[0].first == 0 && c[0].second == s.size());
    }
    {   // test_chunking_empty_file (:36-43)
        CHECK(chunk_data({}).empty());
    }
    {   // test_chunking_large_file (:45-73)
        std::vector<uint8_t> content;
        for (int i = 0; i < 1000; i++) {
            std::string l = "Line " + std::to_string(i) + " with some varied content\n";
            content.insert(content.end(), l.begin(), l.end());
        }
        std::string pad = "Additional padding content to reach size. ";
        while (content.size() < 100 * 1024) content.insert(content.end(), pad.begin(), pad.end());
        auto c = chunk_data(content);
        CHECK(!c.empty());
        CHECK(contiguous_cover(c, content.size()));
    }
    {   // test_chunking_content_shifting (:75-92)
        auto base = rep("AAAAA", 1000);
        std::vector<uint8_t> c2 = rep("PREFIX", 1);
        c2.insert(c2.end(), base.begin(), base.end());
        CHECK(chunk_data(c2).size() >= chunk_data(base).size());
    }
    {   // test_chunk_boundaries (:94-108)
        auto c = chunk_data(std::vector<uint8_t>(MAX_CHUNK_SIZE * 2, 'A'));
        for (auto &p : c) CHECK(p.second <= MAX_CHUNK_SIZE);
    }
    {   // test_chunking_binary_data (:110-120)
        std::vector<uint8_t> content(50000);
        for (size_t i = 0; i < content.size(); i++) content[i] = (uint8_t)(i % 256);
        auto c = chunk_data(content);
        CHECK(!c.empty() && contiguous_cover(c, content.size()));
    }
    {   // test_chunking_identical_blocks (:122-134)
        auto content = rep("IDENTICAL_BLOCK_CONTENT", 500);
        auto c = chunk_data(content);
        CHECK(!c.empty() && contiguous_cover(c, content.size()));
    }
    {   // test_chunking_from_file (:136-154) via compute_file_chunks
        auto content = rep("Test data for chunking ", 1000);
        std::string path = "chunking_test_from_file.dat";
        { std::ofstream f(path, std::ios::binary); f.write((const char *)content.data(), content.size()); }
        syncr::Chunker ch(CHUNK_BITS, MAX_CHUNK_SIZE, 0);
        auto c = syncr::compute_file_chunks(path, ch);
        std::remove(path.c_str());
        uint64_t total = 0;
        for (auto &ci : c) total += ci.size;
        CHECK(!c.empty() && total == content.size());
        CHECK(syncr::compute_file_chunks("/nonexistent/file", ch).empty());   // file_operations.rs:727-733
    }
    {   // test_chunk_offset_progression (:156-167)
        auto c = chunk_data(std::vector<uint8_t>(100000, 'X'));
        CHECK(contiguous_cover(c, 100000));
    }
    {   // test_chunking_reproduces_after_modification (:194-233)
        auto c1 = rep("STABLE_PREFIX_", 1000), c2 = c1;
        std::string e1 = "_ENDING_1", e2 = "_ENDING_2";
        c1.insert(c1.end(), e1.begin(), e1.end());
        c2.insert(c2.end(), e2.begin(), e2.end());
        auto a = chunk_data(c1), b = chunk_data(c2);
        CHECK(!a.empty() && !b.empty());
        CHECK(contiguous_cover(a, c1.size()) && contiguous_cover(b, c2.size()));
    }
    {   // protocol_list_test.rs:305-400 on production semantics (defaults)
        syncr::Chunker prod;
        std::string s = "small";
        auto c = prod.chunk((const uint8_t *)s.data(), s.size());
        CHECK(c.size() == 1 && c[0].offset == 0 && c[0].size == 5);
        std::vector<uint8_t> big(50ull << 20, 'A');
        auto cb = prod.chunk(big);
        uint64_t total = 0;
        for (auto &ci : cb) total += ci.size;
        CHECK(cb.size() == 25 && total == big.size());   // 25 x 2 MiB read-boundary cuts
        std::vector<uint8_t> xs(100000, 'X');
        auto cx = prod.chunk(xs);
        uint64_t off = 0;
        for (auto &ci : cx) { CHECK(ci.offset == off); off += ci.size; }
        CHECK(off == xs.size());
    }
    if (failures) {
        std::fprintf(stderr, "%d check(s) failed\n", failures);
        return 1;
    }
    std::printf("chunking_test (C++ mirror): all checks passed\n");
    return 0;
}
