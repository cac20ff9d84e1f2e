#include "store.hpp"

#include <algorithm>
#include <sstream>
#include <stdexcept>

namespace hlsp2p {

SegmentStore::SegmentStore(int64_t capacity, int64_t align) : capacity_(capacity), align_(align) {
  if (capacity <= 0) throw std::invalid_argument("capacity must be > 0");
  if (align <= 0 || (align & (align - 1))) throw std::invalid_argument("align must be a power of two");
}

int64_t SegmentStore::lookup(const SegKey& k, bool include_pending) const {
  auto it = index_.find(k);
  if (it == index_.end()) return -1;
  const Entry& e = entries_[it->second];
  if (e.state == kResident || (include_pending && e.state == kPending)) return it->second;
  return -1;
}

int64_t SegmentStore::new_entry() {
  if (!free_ids_.empty()) {
    int64_t id = free_ids_.back();
    free_ids_.pop_back();
    return id;
  }
  entries_.emplace_back();
  return static_cast<int64_t>(entries_.size()) - 1;
}

void SegmentStore::release(int64_t id, bool log_remove) {
  Entry& e = entries_[id];
  if (e.state == kFree) return;
  auto it = index_.find(e.key);
  const bool owned = it != index_.end() && it->second == id;
  if (owned) index_.erase(it);
  // Only announce a removal when the node actually stops holding the key (a detached,
  // replaced copy going away is not news to the swarm).
  if (log_remove && owned && e.state == kResident) delta_rm_.push_back(e.key);
  used_ -= e.alloc_bytes;
  e.gen += 1;
  e.state = kFree;
  e.pins = 0;
  free_ids_.push_back(id);
}

// Pop FIFO entries living inside the region we are about to overwrite.  Live entries
// occupy one cyclic interval [tail, head) in allocation order, so the region starting at
// `head` (plus [head, capacity) when wrapping) is always at the FIFO front.
bool SegmentStore::make_room(int64_t start, int64_t len, bool wrapped) {
  const int64_t end = start + len;
  while (!fifo_.empty()) {
    const int64_t id = fifo_.front().first;
    const Entry& e = entries_[id];
    if (e.state == kFree || e.gen != fifo_.front().second) {  // stale (dropped, maybe reused)
      fifo_.pop_front();
      continue;
    }
    bool in_skip = wrapped && e.offset >= head_;
    bool overlaps = e.offset < end && e.offset + e.alloc_bytes > start;
    if (!in_skip && !overlaps) break;
    if (e.pins > 0) return false;
    fifo_.pop_front();
    release(id, true);
    evictions_ += 1;
  }
  return true;
}

void SegmentStore::resident_ids(std::vector<int64_t>* ids) const {
  ids->clear();
  for (const auto& fe : fifo_) {
    const Entry& e = entries_[fe.first];
    if (e.state != kResident || e.gen != fe.second) continue;
    auto it = index_.find(e.key);
    if (it == index_.end() || it->second != fe.first) continue;  // detached, replaced copy
    ids->push_back(fe.first);
  }
}

bool SegmentStore::fits(int64_t total) const {
  if (total <= 0) return true;
  if (total > capacity_) return false;
  int64_t start = head_;
  bool wrapped = false;
  if (start + total > capacity_) {
    start = 0;
    wrapped = true;
  }
  const int64_t end = start + total;
  // same walk as make_room, without evicting: every FIFO entry it would have to evict
  // must be unpinned
  for (const auto& fe : fifo_) {
    const Entry& e = entries_[fe.first];
    if (e.state == kFree || e.gen != fe.second) continue;
    const bool in_skip = wrapped && e.offset >= head_;
    const bool overlaps = e.offset < end && e.offset + e.alloc_bytes > start;
    if (!in_skip && !overlaps) break;
    if (e.pins > 0) return false;
  }
  return true;
}

bool SegmentStore::wrap_for(int64_t total) {
  if (total <= 0 || head_ + total <= capacity_) return true;
  if (!make_room(0, 0, true)) return false;  // len 0: only the tail entries (offset >= head) go
  head_ = 0;
  return true;
}

int64_t SegmentStore::retire_region(int64_t total) {
  if (total <= 0) return 0;
  if (total > capacity_) total = capacity_;
  int64_t start = head_;
  bool wrapped = false;
  if (start + total > capacity_) {
    start = 0;
    wrapped = true;
  }
  const int64_t end = start + total;
  std::vector<int64_t> victims;
  for (const auto& fe : fifo_) {  // the walk of fits() / make_room()
    const Entry& e = entries_[fe.first];
    if (e.state == kFree || e.gen != fe.second) continue;
    const bool in_skip = wrapped && e.offset >= head_;
    const bool overlaps = e.offset < end && e.offset + e.alloc_bytes > start;
    if (!in_skip && !overlaps) break;
    victims.push_back(fe.first);
  }
  int64_t n = 0;
  for (int64_t id : victims) {
    const Entry& e = entries_[id];
    auto it = index_.find(e.key);
    if (it == index_.end() || it->second != id) continue;  // already detached / replaced
    detach(id);
    ++n;
  }
  return n;
}

int64_t SegmentStore::reserve_run(const SegKey* keys, const int64_t* lens, int64_t n, int64_t tick, int64_t* ids,
                                  int64_t* offsets) {
  int64_t total = 0;
  std::vector<int64_t> rel(n);
  for (int64_t i = 0; i < n; ++i) {
    rel[i] = total;
    int64_t a = (lens[i] + align_ - 1) & ~(align_ - 1);
    if (a == 0) a = align_;
    total += a;
  }
  if (n == 0) return head_;
  if (total > capacity_) return -1;
  int64_t start = head_;
  bool wrapped = false;
  if (start + total > capacity_) {
    start = 0;
    wrapped = true;
  }
  if (!make_room(start, total, wrapped)) return -1;
  // Replace existing keys (their old copies become stale).
  for (int64_t i = 0; i < n; ++i) {
    auto it = index_.find(keys[i]);
    if (it != index_.end()) {
      Entry& old = entries_[it->second];
      if (old.pins > 0) {
        if (old.state == kResident) delta_rm_.push_back(old.key);
        index_.erase(it);  // detach; bytes freed when the FIFO reaches it and pins drop
      } else {
        release(it->second, true);
      }
    }
  }
  for (int64_t i = 0; i < n; ++i) {
    int64_t id = new_entry();
    Entry& e = entries_[id];
    e.key = keys[i];
    e.offset = start + rel[i];
    e.length = lens[i];
    e.alloc_bytes = (i + 1 < n ? rel[i + 1] : total) - rel[i];
    e.state = kPending;
    e.pins = 0;
    e.tick = tick;
    used_ += e.alloc_bytes;
    index_[keys[i]] = id;
    fifo_.emplace_back(id, e.gen);
    ids[i] = id;
    offsets[i] = e.offset;
  }
  head_ = start + total;
  if (head_ >= capacity_) head_ = 0;
  return start;
}

void SegmentStore::commit(int64_t id) {
  Entry& e = entries_[id];
  if (e.state != kPending) return;
  e.state = kResident;
  // a copy detached meanwhile (a newer copy of the key took its index slot) serves only the
  // readers holding it: announcing it would let peers plan transfers this rank cannot look up
  auto it = index_.find(e.key);
  if (it == index_.end() || it->second != id) return;
  delta_add_.push_back(e.key);
  delta_add_len_.push_back(e.length);
}

void SegmentStore::drop(int64_t id) {
  if (id < 0 || id >= static_cast<int64_t>(entries_.size())) return;
  release(id, true);
}

void SegmentStore::detach(int64_t id) {
  if (id < 0 || id >= static_cast<int64_t>(entries_.size())) return;
  Entry& e = entries_[id];
  if (e.state == kFree) return;
  auto it = index_.find(e.key);
  if (it == index_.end() || it->second != id) return;  // already replaced / detached
  if (e.state == kResident) delta_rm_.push_back(e.key);
  index_.erase(it);
}

int64_t SegmentStore::evict_below(uint32_t swarm, uint32_t min_sn) {
  std::vector<int64_t> victims;
  for (const auto& kv : index_) {
    const Entry& e = entries_[kv.second];
    if (kv.first.swarm == swarm && kv.first.sn < min_sn && e.state == kResident && e.pins == 0)
      victims.push_back(kv.second);
  }
  for (int64_t id : victims) release(id, true);
  evictions_ += static_cast<int64_t>(victims.size());
  return static_cast<int64_t>(victims.size());
}

void SegmentStore::take_delta(std::vector<SegKey>* added, std::vector<int64_t>* added_len,
                              std::vector<SegKey>* removed) {
  added->swap(delta_add_);
  added_len->swap(delta_add_len_);
  removed->swap(delta_rm_);
  delta_add_.clear();
  delta_add_len_.clear();
  delta_rm_.clear();
}

void SegmentStore::all_resident(std::vector<SegKey>* keys, std::vector<int64_t>* lens) const {
  for (const auto& kv : index_) {
    const Entry& e = entries_[kv.second];
    if (e.state == kResident) {
      keys->push_back(kv.first);
      lens->push_back(e.length);
    }
  }
}

void SegmentStore::audit(std::vector<std::string>* errors) const {
  auto err = [&](const std::string& m) {
    if (errors->size() < 64) errors->push_back(m);
  };
  const int64_t n = static_cast<int64_t>(entries_.size());
  int64_t used = 0, live = 0;
  for (int64_t id = 0; id < n; ++id) {
    const Entry& e = entries_[id];
    if (e.state == kFree) continue;
    ++live;
    used += e.alloc_bytes;
    if (e.state != kPending && e.state != kResident) err("entry " + std::to_string(id) + " in state " + std::to_string(e.state));
    if (e.pins < 0) err("entry " + std::to_string(id) + " has " + std::to_string(e.pins) + " pins");
    if (e.offset < 0 || e.alloc_bytes < aligned(e.length) || e.offset + e.alloc_bytes > capacity_) {
      std::ostringstream o;
      o << "entry " << id << " out of the ring: offset " << e.offset << " alloc " << e.alloc_bytes << " length "
        << e.length << " capacity " << capacity_;
      err(o.str());
    }
  }
  if (used != used_) err("used bytes " + std::to_string(used_) + " != sum of live allocations " + std::to_string(used));
  if (unpin_underflows_) err(std::to_string(unpin_underflows_) + " unpins of live entries that held no pin");
  // the index names live entries under their own keys
  for (const auto& kv : index_) {
    const int64_t id = kv.second;
    if (id < 0 || id >= n) {
      err("index names entry id " + std::to_string(id) + " out of range");
      continue;
    }
    const Entry& e = entries_[id];
    if (e.state == kFree) err("index names free entry " + std::to_string(id));
    if (!(e.key == kv.first)) err("index key of entry " + std::to_string(id) + " differs from the entry's key");
  }
  // every live entry is in the FIFO exactly once (current generation), and the FIFO's live
  // records lie in allocation order around the ring: at most one wrap, no overlap
  std::vector<int> seen(static_cast<size_t>(n), 0);
  int64_t prev_end = -1, first_off = -1, wraps = 0;
  for (const auto& fe : fifo_) {
    const int64_t id = fe.first;
    if (id < 0 || id >= n) {
      err("FIFO names entry id " + std::to_string(id) + " out of range");
      continue;
    }
    const Entry& e = entries_[id];
    if (e.state == kFree || e.gen != fe.second) continue;  // stale record
    seen[static_cast<size_t>(id)] += 1;
    if (first_off < 0) first_off = e.offset;
    if (prev_end >= 0 && e.offset < prev_end) {  // the allocation wrapped to the ring's start
      wraps += 1;
      if (wraps > 1) err("FIFO wraps the ring more than once (entry " + std::to_string(id) + ")");
    }
    if (wraps == 1 && e.offset + e.alloc_bytes > first_off) {  // after the wrap: below the oldest
      std::ostringstream o;
      o << "FIFO: entry " << id << " ends at " << e.offset + e.alloc_bytes << " past the oldest live entry at "
        << first_off;
      err(o.str());
    }
    prev_end = e.offset + e.alloc_bytes;
  }
  int64_t in_fifo = 0;
  for (int64_t id = 0; id < n; ++id) {
    if (entries_[id].state == kFree) continue;
    if (seen[static_cast<size_t>(id)] != 1)
      err("live entry " + std::to_string(id) + " appears " + std::to_string(seen[static_cast<size_t>(id)]) +
          " times in the FIFO");
    in_fifo += seen[static_cast<size_t>(id)];
  }
  (void)live;
  (void)in_fifo;
}

}  // namespace hlsp2p
