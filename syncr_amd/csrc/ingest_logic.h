// ingest_logic.h -- host-only logic of the ingest pipeline (no HIP): device
// assignment, in-order delivery, and the read-error prefix rule.  Kept free of
// HIP so tests/cpp/ingest_logic_test.cpp checks it with plain g++ on the CPU.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <vector>

namespace ingest {

// Files are independent (file_operations.rs:721-788: a fresh Bup at offset 0,
// no cross-file state), so a multi-device pipeline assigns each file whole to
// one device.  The stream of submissions is not known in advance, so this is
// the online form of LPT: each file goes to the device with the fewest bytes
// assigned so far (ties: lowest index).  For a size-descending stream it is
// exactly LPT.
class Assigner {
  public:
    explicit Assigner(uint32_t n) : load_(n, 0), files_(n, 0) {}
    uint32_t assign(uint64_t bytes) {
        uint32_t best = 0;
        for (uint32_t d = 1; d < load_.size(); d++)
            if (load_[d] < load_[best]) best = d;
        load_[best] += bytes;
        files_[best] += 1;
        return best;
    }
    uint64_t load(uint32_t d) const { return load_[d]; }
    uint64_t files(uint32_t d) const { return files_[d]; }
    uint32_t size() const { return (uint32_t)load_.size(); }

  private:
    std::vector<uint64_t> load_, files_;
};

// Results of files that finished on any device, released strictly in
// submission order (seq 0, 1, 2, ...): the reference's walk emits entries in
// traversal order (file_operations.rs:599-605, :707), and so does the
// single-device pipeline.  put() may be called from worker threads; take()
// from the thread that delivers callbacks.
template <class Result>
class Reorder {
  public:
    void put(uint64_t seq, Result r) {
        std::lock_guard<std::mutex> g(mu_);
        ready_.emplace(seq, std::move(r));
    }
    // the next result in order, if it has arrived
    bool take(Result &out, uint64_t &seq) {
        std::lock_guard<std::mutex> g(mu_);
        auto it = ready_.find(next_);
        if (it == ready_.end()) return false;
        out = std::move(it->second);
        ready_.erase(it);
        seq = next_++;
        return true;
    }
    uint64_t next() const {
        std::lock_guard<std::mutex> g(mu_);
        return next_;
    }
    size_t pending() const {
        std::lock_guard<std::mutex> g(mu_);
        return ready_.size();
    }

  private:
    mutable std::mutex mu_;
    std::map<uint64_t, Result> ready_;
    uint64_t next_ = 0;
};

// A read error partway through a file.  compute_file_chunks reads at most
// read_cap bytes per tokio read (file_operations.rs:738,776); assuming the
// reads return every byte before the bad offset P, they are exactly the reads
// of a P-byte file until the first read that STARTS at P with a non-empty
// request: that one fails and the loop breaks (:779-782), dropping the bytes it
// had buffered but not yet cut.  Given the cut ends of the P-byte file's walk
// (production semantics, the GPU resolve), returns how many of them the
// reference keeps.  A zero-length request (16 MiB buffer full) does not touch
// the file and cannot fail.  read_cap 0 = no cap.
inline uint64_t read_error_keep(const uint64_t *ends, uint64_t n, uint64_t P, uint64_t max_chunk,
                                uint64_t read_cap) {
    const uint64_t cap = read_cap ? read_cap : ~0ull;
    uint64_t R = std::min(std::min(P, max_chunk), cap);   // first read (:738)
    uint64_t s = 0;
    for (uint64_t j = 0; j < n; j++) {
        s = ends[j];                                       // cut, copy_within (:771)
        const uint64_t want = max_chunk - (R - s);         // f.read(&mut buf[n..]) (:776)
        if (want == 0) continue;
        if (R >= P) return j + 1;                          // the read at P fails: break (:781)
        R += std::min(std::min(want, cap), P - R);
    }
    return n;
}

}  // namespace ingest
