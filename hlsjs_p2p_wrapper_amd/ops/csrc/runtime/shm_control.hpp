// Intra-node control plane of the swarm: a shared-memory all-gather for the per-round
// control messages (wants, cache deltas, flags) of the ranks that share one host.
//
// Each exchange round every rank all-gathers a few KB of int64 words.  Over gloo (TCP
// loopback, a ring of world-1 steps) that costs 0.25 ms at 2 ranks and grows with the
// rank count; here a rank writes its message into its slot of a shared mapping and meets
// the others at a monotonic arrival counter, so a round costs a few cache-line transfers.
//
// Layout (one mapping, created by rank 0, unlinked as soon as every rank has attached):
//   Header { magic, world, slot_words, arrive (atomic, monotonic) }
//   slots[2 parities][world][1 + slot_words]  (int64: length, then payload)
// Generation g uses parity g & 1; a rank only rewrites parity p at g + 2, after the barrier
// of g + 1, which nobody passes before every rank has finished reading generation g.
#pragma once
#include <atomic>
#include <cstdint>
#include <string>
#include <vector>

namespace hlsp2p {

class ShmControl {
 public:
  // create=true on exactly one rank (it sizes and initialises the mapping)
  ShmControl(const std::string& name, int rank, int world, int64_t slot_words, bool create);
  ~ShmControl();
  ShmControl(const ShmControl&) = delete;
  ShmControl& operator=(const ShmControl&) = delete;

  // remove the name from the filesystem (mappings stay valid); call once all ranks attached
  void unlink();

  // Write `n` words (n <= slot_words, else only the length is published and the caller
  // must fall back to another transport: every rank sees the same lengths).  Blocks until
  // all ranks have written this generation; then `out_len[r]` holds rank r's length and
  // `read(r, dst)` copies its payload.  Throws after `timeout_s` without all arrivals.
  void exchange(const int64_t* msg, int64_t n, double timeout_s);
  int64_t length(int r) const;
  void read(int r, int64_t* dst) const;  // copies min(length, slot_words) words
  void barrier(double timeout_s);

  int64_t slot_words() const { return slot_words_; }
  int rank() const { return rank_; }
  int world() const { return world_; }
  uint64_t generation() const { return gen_; }

 private:
  struct Header {
    uint64_t magic;
    int64_t world;
    int64_t slot_words;
    alignas(64) std::atomic<uint64_t> arrive;
  };
  int64_t* slot(int parity, int r) const;
  void arrive_and_wait(double timeout_s);

  std::string name_;
  int rank_, world_;
  int64_t slot_words_;
  size_t bytes_ = 0;
  void* base_ = nullptr;
  Header* hdr_ = nullptr;
  int64_t* slots_ = nullptr;
  uint64_t gen_ = 0;  // generations completed by this rank
  bool linked_ = false;
};

}  // namespace hlsp2p
