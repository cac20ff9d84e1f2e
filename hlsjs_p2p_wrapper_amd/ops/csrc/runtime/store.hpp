// Segment cache bookkeeping for one swarm node (one MI355X = one peer).
//
// The bytes live in a single device uint8 arena (a torch tensor in HBM, up to the 288 GB
// of the part); this class owns only the *layout*: a ring allocator over arena offsets, a
// key -> entry index, pin counts, and the add/remove delta log that the node gossips to the
// swarm every exchange round (the tracker "have" analog).
//
// Why a ring: segment traffic is a stream (live windows slide, VOD is watched forward), so
// FIFO eviction is the natural policy, allocation is O(1), and a batch of segments received
// in one round lands *contiguously* — one RCCL recv per peer per round instead of one per
// segment (fewer, larger transfers over the 7 xGMI links).
#pragma once
#include <cstdint>
#include <cstddef>
#include <deque>
#include <string>
#include <utility>
#include <unordered_map>
#include <vector>

namespace hlsp2p {

struct SegKey {
  uint32_t swarm, level, url_id, sn;
  bool operator==(const SegKey& o) const {
    return swarm == o.swarm && level == o.level && url_id == o.url_id && sn == o.sn;
  }
  bool operator<(const SegKey& o) const {
    if (swarm != o.swarm) return swarm < o.swarm;
    if (level != o.level) return level < o.level;
    if (url_id != o.url_id) return url_id < o.url_id;
    return sn < o.sn;
  }
};

inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// 32-bit digest of a segment key that binds a CRC to it (crc ^ key_digest): the 12-byte wire
// key [level, urlId, sn] plus the swarm id.  Device twin: kernels/crc32_mfma.hip key_digest
// (the CRC combine kernel's keyed mode); the two must agree bit for bit (tests).
inline uint32_t key_digest(const SegKey& k) {
  const uint64_t a = uint64_t(k.level) | (uint64_t(k.url_id) << 32);
  const uint64_t b = uint64_t(k.sn) | (uint64_t(k.swarm) << 32);
  const uint64_t z = mix64(a ^ mix64(b + 0x9E3779B97F4A7C15ull));
  return static_cast<uint32_t>(z ^ (z >> 32));
}

struct SegKeyHash {
  size_t operator()(const SegKey& k) const {
    uint64_t a = (uint64_t(k.swarm) << 32) | k.level;
    uint64_t b = (uint64_t(k.url_id) << 32) | k.sn;
    return static_cast<size_t>(mix64(a ^ mix64(b + 0x9E3779B97F4A7C15ull)));
  }
};

enum EntryState : int32_t { kFree = 0, kPending = 1, kResident = 2 };

struct Entry {
  SegKey key{};
  int64_t offset = 0;
  int64_t length = 0;
  int64_t alloc_bytes = 0;
  int32_t state = kFree;
  int32_t pins = 0;
  int64_t tick = 0;
  uint64_t gen = 0;  // bumped on release: FIFO records carry it to detect reuse
};

class SegmentStore {
 public:
  SegmentStore(int64_t capacity, int64_t align);

  int64_t capacity() const { return capacity_; }
  int64_t used_bytes() const { return used_; }
  int64_t num_entries() const { return static_cast<int64_t>(index_.size()); }
  int64_t evictions() const { return evictions_; }
  int64_t max_entries() const { return static_cast<int64_t>(entries_.size()); }

  // -1 if absent (pending entries are reported only when `include_pending`).
  int64_t lookup(const SegKey& k, bool include_pending) const;
  const Entry& entry(int64_t id) const { return entries_[id]; }

  // Reserve one contiguous run for `n` segments (in order).  On success returns the run's
  // base offset and writes entry ids / offsets; returns -1 if the ring cannot make room
  // (a pinned entry blocks eviction, or the run exceeds capacity).  Keys already present
  // are replaced.
  int64_t reserve_run(const SegKey* keys, const int64_t* lens, int64_t n, int64_t tick, int64_t* ids,
                      int64_t* offsets);
  // Would a run of `total` aligned bytes fit at the head now (no pinned entry in its way)?
  // Non-mutating; consecutive smaller runs of the same total then fit too (backpressure).
  bool fits(int64_t total) const;
  // A round about to reserve several runs totalling `total` (a CDN run, one run per source
  // peer): when they would cross the ring's end, wrap NOW -- evict the tail past the head and
  // continue at 0 -- so every run of the round lands in [0, total), the region fits(total)
  // checked.  (Runs wrapping one by one skip the tail in the middle of the round, and the
  // runs after the wrap can reach the round's own earlier, pinned, runs.)  False if a pinned
  // entry is in the tail (admission rules that out).
  bool wrap_for(int64_t total);
  // Detach (and announce the removal of) every entry a reservation of `total` bytes at the
  // head would overwrite -- the entries `fits(total)` walks.  A round calls it for the bytes
  // it admitted, before its control message goes out: no peer then plans a transfer from an
  // entry this rank overwrites in the same round (the send would pin it after admission and
  // the reservation would find it pinned).  Returns the number detached.
  int64_t retire_region(int64_t total);
  int64_t aligned(int64_t len) const {
    const int64_t a = (len + align_ - 1) & ~(align_ - 1);
    return a == 0 ? align_ : a;
  }
  void commit(int64_t id);  // pending -> resident (+ "add" delta)
  void drop(int64_t id);    // remove now (+ "remove" delta if it was resident)
  // Take the entry out of the index (+ "remove" delta if it was resident) but keep its bytes
  // until its pins drop and the ring reaches it -- for a copy that readers still hold pins on
  // and must not be found again (a received segment that failed its deferred CRC check).
  void detach(int64_t id);
  void pin(int64_t id) { entries_[id].pins += 1; }
  void unpin(int64_t id) {
    Entry& e = entries_[id];
    if (e.pins > 0) {
      e.pins -= 1;
    } else if (e.state != kFree) {
      // a live entry unpinned more often than pinned: some holder gave up a pin it did not
      // own (the entry may already have been overwritten under another holder).  Clamped as
      // before, but counted: the audit reports any (a free entry's unpin is the normal end of
      // a pin on an entry dropped meanwhile, e.g. a received copy that failed its CRC)
      unpin_underflows_ += 1;
    }
  }
  int64_t unpin_underflows() const { return unpin_underflows_; }
  // Replicated-state audit (HLSP2P_AUDIT, agent/audit.py): the layout invariants of the ring,
  // index and FIFO, appended as messages (empty: consistent).  O(entries); diagnostics only.
  void audit(std::vector<std::string>* errors) const;
  // The delta log not taken yet (what the next control message will announce).
  void peek_delta(std::vector<SegKey>* added, std::vector<SegKey>* removed) const {
    *added = delta_add_;
    *removed = delta_rm_;
  }
  // Ring region a reservation of `total` bytes at the head would occupy now (the region
  // fits() walks): [start, start + total).
  int64_t region_start(int64_t total) const { return head_ + total > capacity_ ? 0 : head_; }
  // Drop resident, unpinned entries of `swarm` (all tracks) with sn < min_sn.
  int64_t evict_below(uint32_t swarm, uint32_t min_sn);

  // Delta log since the last call.
  void take_delta(std::vector<SegKey>* added, std::vector<int64_t>* added_len, std::vector<SegKey>* removed);
  void all_resident(std::vector<SegKey>* keys, std::vector<int64_t>* lens) const;
  // Resident entry ids, oldest first (allocation order: restoring them in this order keeps
  // the eviction order of a checkpointed cache).
  void resident_ids(std::vector<int64_t>* ids) const;

 private:
  int64_t new_entry();
  void release(int64_t id, bool log_remove);
  bool make_room(int64_t start, int64_t len, bool wrapped);

  int64_t capacity_, align_;
  int64_t head_ = 0;
  int64_t used_ = 0;
  int64_t evictions_ = 0;
  int64_t unpin_underflows_ = 0;
  std::vector<Entry> entries_;
  std::vector<int64_t> free_ids_;
  std::deque<std::pair<int64_t, uint64_t>> fifo_;  // (entry id, gen) in allocation order
  std::unordered_map<SegKey, int64_t, SegKeyHash> index_;
  std::vector<SegKey> delta_add_;
  std::vector<int64_t> delta_add_len_;
  std::vector<SegKey> delta_rm_;
};

}  // namespace hlsp2p
