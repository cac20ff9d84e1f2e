// Want table of one swarm node: every segment this rank has asked the swarm for and not
// received yet, and who is waiting for it.
//
// The reference hands each fragment request to the peer agent one `getSegment` call at a
// time (lib/integration/p2p-loader-generator.js:164).  A GPU node serves hundreds of
// thousands of them per second, so the per-request state lives here, natively, as rows:
// a request is a 64-bit *token* (the caller's id: a fleet player's request, or an
// in-process loader handle) joined to the want of its segment key.  One call per round
// picks the wants to announce (FIFO, player requests before prefetch, bounded by what the
// HBM ring can place: backpressure), encodes their control rows, and, once the round has
// delivered, turns served wants back into the token columns the caller answers.  No
// per-request object exists on the node's hot path.
#pragma once
#include <cstdint>
#include <deque>
#include <string>
#include <unordered_map>
#include <vector>

#include "planner.hpp"
#include "store.hpp"

namespace hlsp2p {

// want state bits (bits 0-2 are the planner's WantFlag: force_cdn, not_staged, staging)
enum WantBits : int32_t {
  kWForceCdn = 1,   // a previous peer copy failed its CRC, or a requester has P2P download off
  kWNotStaged = 2,  // network origin: the body is not in host memory yet (size may be unknown)
  kWStaging = 4,    // network origin: this rank is downloading the body now
  kWPrefetch = 8,   // issued by an agent's prefetch planner (may have no waiter)
  kWPy = 16,        // the node keeps Python-side state for it (network / live origin)
  kWCorrupt = 32,   // fault injection: corrupt the CDN copy on ingest
  kWHeld = 64,      // announced before and not served (the planner holds a want back at most once)
  kWOnDev = 128,    // the node's: the origin bytes live in device memory (D2D ingest copies)
};

constexpr int64_t kNoToken = -1;

struct WantRec {
  SegKey key{};
  int64_t id = 0;
  int64_t size = 0;      // bytes this rank reserves and announces
  int64_t src_ptr = 0;   // address of the (ranged) origin bytes; 0 = resolved by the caller at fetch
  int64_t src_base = 0;  // base address of that origin allocation (merging of contiguous DMAs)
  int32_t flags = 0;
  int32_t round = -1;    // round it is in flight in, -1 = waiting
  int32_t attempts = 0;
  std::vector<int64_t> waiters;  // live tokens
};

class WantTable {
 public:
  // Join `token` (kNoToken: none) to the want of `key`, creating it when absent.  A requester
  // with kWForceCdn forces a waiting want to the CDN; a real token clears kWPrefetch's
  // "no waiter" status.  Returns the want id; *created tells whether it is new.
  int64_t add(const SegKey& key, int64_t size, int64_t src_ptr, int64_t src_base, int32_t flags, int64_t token,
              bool* created);
  // Forget a token (aborted request); false when unknown.
  bool abort(int64_t token);
  int64_t lookup(const SegKey& key) const;
  WantRec* get(int64_t id);
  const WantRec* get(int64_t id) const;

  // One round's announcement.  Walks the waiting wants in creation order: requested ones
  // first (up to `cap`, -1 = unbounded), then prefetch-only ones in the room left; a want
  // whose waiters all aborted is removed (`dropped`).  A not-staged want of unknown size
  // takes the length the directory knows for its key (a holder announced it), so the ring
  // reserves what a peer will send.  Backpressure: the largest prefix whose aligned sizes
  // fit the ring now is admitted (marked in flight in `round`); of the rest, wants larger
  // than the whole cache go to `too_big` (removed), the others wait (`deferred`).
  void select(const SegmentStore& store, const Directory* dir, int64_t cap, int32_t round,
              std::vector<int64_t>* admitted, std::vector<int64_t>* dropped, std::vector<int64_t>* too_big,
              int64_t* deferred);
  // Control rows of wants: [key x4, size, id | force_cdn << 62 | not_staged << 61 | staging << 60 |
  // held << 59].
  void encode(const int64_t* ids, int64_t n, int64_t* rows) const;
  // Remove served (or failed) wants; appends their live tokens, the index of each token's
  // want in `ids`, and per want whether it was a prefetch with nobody waiting.
  void finish(const int64_t* ids, int64_t n, std::vector<int64_t>* tokens, std::vector<int64_t>* index,
              std::vector<uint8_t>* prefetch_only);
  // Back to waiting (announced but not served: kWHeld from now on); `force_cdn`: next time
  // from the CDN (+1 attempt).
  void requeue(const int64_t* ids, int64_t n, bool force_cdn);

  // Replicated-state audit (agent/audit.py): index <-> records, token map <-> waiter lists,
  // creation order covers every record; messages appended (empty: consistent).
  void audit(std::vector<std::string>* errors) const;
  // Every want id; every live token with its want id.
  void ids(std::vector<int64_t>* out) const;
  void token_map(std::vector<int64_t>* tokens, std::vector<int64_t>* wants) const;

  int64_t size() const { return static_cast<int64_t>(recs_.size()); }
  int64_t waiting() const;  // wants not in flight and not being downloaded
  int64_t tokens() const { return static_cast<int64_t>(token_.size()); }

 private:
  void erase(std::unordered_map<int64_t, WantRec>::iterator it);
  void compact();

  std::unordered_map<SegKey, int64_t, SegKeyHash> index_;
  std::unordered_map<int64_t, WantRec> recs_;
  std::unordered_map<int64_t, int64_t> token_;  // token -> want id
  std::deque<int64_t> order_;                   // want ids in creation order (lazily pruned)
  int64_t next_id_ = 1;
};

}  // namespace hlsp2p
