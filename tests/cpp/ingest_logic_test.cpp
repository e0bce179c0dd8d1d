// CPU test of the multi-device ingest's host logic (syncr_amd/csrc/ingest_logic.h):
// device assignment (online LPT), in-order delivery across worker threads, and
// the read-error prefix rule checked against the oracle's literal
// compute_file_chunks loop with a failing reader (oracle/bup_oracle.c).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <numeric>
#include <random>
#include <thread>
#include <vector>

#include "ingest_logic.h"

extern "C" {
uint64_t orc_chunk_production(const uint8_t *file, uint64_t F, uint32_t bits, uint64_t max_chunk,
                              uint64_t read_cap, uint64_t *ends, uint64_t ends_cap);
uint64_t orc_chunk_production_read_error(const uint8_t *file, uint64_t P, uint32_t bits, uint64_t max_chunk,
                                         uint64_t read_cap, uint64_t *ends, uint64_t ends_cap);
void orc_xorshift_fill(uint64_t seed, uint64_t discard, uint8_t *out, uint64_t n);
}

static int fails = 0;
#define CHECK(c)                                                             \
    do {                                                                     \
        if (!(c)) {                                                          \
            fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
            fails++;                                                         \
        }                                                                    \
    } while (0)

static void test_assigner() {
    // a size-descending stream: greedy least-loaded == LPT; every file assigned once
    std::mt19937_64 rng(7);
    std::vector<uint64_t> sizes(5000);
    for (auto &s : sizes) s = 4096ull << (rng() % 15);
    std::sort(sizes.rbegin(), sizes.rend());
    for (uint32_t nd : {1u, 2u, 3u, 8u}) {
        ingest::Assigner a(nd);
        std::vector<uint64_t> load(nd, 0);
        for (uint64_t s : sizes) {
            const uint32_t d = a.assign(s);
            CHECK(d < nd);
            // it picked a least-loaded device (lowest index on ties)
            const uint64_t mn = *std::min_element(load.begin(), load.end());
            CHECK(load[d] == mn);
            for (uint32_t k = 0; k < d; k++) CHECK(load[k] > mn);
            load[d] += s;
        }
        uint64_t tot = 0, files = 0;
        for (uint32_t d = 0; d < nd; d++) {
            CHECK(a.load(d) == load[d]);
            tot += a.load(d);
            files += a.files(d);
        }
        CHECK(tot == std::accumulate(sizes.begin(), sizes.end(), 0ull));
        CHECK(files == sizes.size());
        const uint64_t mx = *std::max_element(load.begin(), load.end());
        CHECK((double)mx <= (double)tot / nd + (double)sizes.front());      // LPT bound
    }
    // two devices, the same list in an adversarial order (small first): still
    // within one largest file of the mean
    ingest::Assigner b(2);
    std::vector<uint64_t> asc(sizes.rbegin(), sizes.rend());
    for (uint64_t s : asc) b.assign(s);
    const uint64_t tot = b.load(0) + b.load(1);
    CHECK(std::max(b.load(0), b.load(1)) <= tot / 2 + sizes.front());
}

static void test_reorder() {
    // 4 worker threads put results of interleaved sequence numbers in scrambled
    // order; the consumer sees exactly 0, 1, 2, ... with the right payloads
    const uint64_t N = 20000;
    ingest::Reorder<uint64_t> r;
    std::vector<std::thread> th;
    for (int w = 0; w < 4; w++) {
        th.emplace_back([&, w] {
            std::vector<uint64_t> mine;
            for (uint64_t s = (uint64_t)w; s < N; s += 4) mine.push_back(s);
            std::shuffle(mine.begin(), mine.end(), std::mt19937_64(w));
            for (uint64_t s : mine) r.put(s, s * 3 + 1);
        });
    }
    uint64_t expect = 0;
    while (expect < N) {
        uint64_t v, seq;
        if (r.take(v, seq)) {
            CHECK(seq == expect);
            CHECK(v == seq * 3 + 1);
            expect++;
        } else {
            std::this_thread::yield();
        }
    }
    for (auto &t : th) t.join();
    uint64_t v, seq;
    CHECK(!r.take(v, seq));
    CHECK(r.pending() == 0 && r.next() == N);
}

static void test_read_error_keep() {
    // random bytes (cuts every ~2^bits) and long runs of zeros (forced MAX /
    // read-cap cuts), bad offset P anywhere: keep(walk of the P-byte file) ==
    // the literal loop with a reader that fails at P
    struct Case { uint32_t bits; uint64_t max, cap; };
    const Case cases[] = {{13, 128 << 10, 0}, {13, 128 << 10, 3000}, {12, 64 << 10, 16 << 10},
                          {10, 8 << 10, 8 << 10}, {20, 16 << 20, 2 << 20}};
    const uint64_t F = 6 << 20;
    std::vector<uint8_t> data(F);
    orc_xorshift_fill(88172645463325252ull, 0, data.data(), F);
    std::fill(data.begin() + (1 << 20), data.begin() + (3 << 20), 0);    // a low-entropy stretch
    std::vector<uint64_t> ends(F + 1), ref(F + 1);
    std::mt19937_64 rng(11);
    int checked = 0;
    for (const Case &c : cases) {
        for (int t = 0; t < 40; t++) {
            uint64_t P = t == 0 ? 1 : (t == 1 ? F : rng() % F + 1);
            if (t == 2) P = c.cap ? c.cap : c.max;                       // exactly at a read boundary
            const uint64_t n = orc_chunk_production(data.data(), P, c.bits, c.max, c.cap, ends.data(), ends.size());
            const uint64_t want =
                orc_chunk_production_read_error(data.data(), P, c.bits, c.max, c.cap, ref.data(), ref.size());
            const uint64_t keep = ingest::read_error_keep(ends.data(), n, P, c.max, c.cap);
            CHECK(keep == want);
            CHECK(keep <= n);
            for (uint64_t k = 0; k < std::min(keep, want); k++) CHECK(ends[k] == ref[k]);
            checked++;
        }
    }
    printf("read_error_keep: %d cases\n", checked);
}

int main() {
    test_assigner();
    test_reorder();
    test_read_error_keep();
    if (fails) {
        printf("%d checks failed\n", fails);
        return 1;
    }
    printf("all checks passed\n");
    return 0;
}
