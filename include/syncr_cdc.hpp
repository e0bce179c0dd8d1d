// syncr_cdc.hpp -- C++ host mirror of szilu/syncr's chunking interface over the
// C ABI in syncr_cdc.h.  Header-only; link with libsyncr_cdc.so.
//
//   syncr::chunking::{CHUNK_BITS, MAX_CHUNK_SIZE_FACTOR, MAX_CHUNK_SIZE}
//                                     src/chunking.rs:7,10,13
//   syncr::ChunkInfo                  src/protocol/types.rs:24-29 (hash = BLAKE3, util.rs:57-59,
//                                     computed on the GPU by chunk_hashed())
//   syncr::compute_file_chunks()      src/protocol/file_operations.rs:721-788
//   syncr::chunk_data()               tests/chunking_test.rs:170-192
//
// Error behaviour follows the reference: an unopenable/unreadable file yields
// an empty list (file_operations.rs:727-744).  Engine errors (no device, HIP
// failure) throw syncr::CdcError -- there is no silent CPU fallback.
#pragma once

#include <algorithm>
#include <array>
#include <cstdint>
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

}  // namespace syncr
