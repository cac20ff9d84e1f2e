#include "wants.hpp"

#include <algorithm>
#include <stdexcept>
#include <unordered_set>

namespace hlsp2p {

int64_t WantTable::add(const SegKey& key, int64_t size, int64_t src_ptr, int64_t src_base, int32_t flags,
                       int64_t token, bool* created) {
  auto it = index_.find(key);
  int64_t id;
  if (it == index_.end()) {
    id = next_id_++;
    WantRec& r = recs_[id];
    r.key = key;
    r.id = id;
    r.size = size;
    r.src_ptr = src_ptr;
    r.src_base = src_base;
    r.flags = flags;
    index_.emplace(key, id);
    order_.push_back(id);
    *created = true;
  } else {
    id = it->second;
    WantRec& r = recs_[id];
    // a requester that may not download from peers makes a waiting want a CDN fetch (one in
    // flight already keeps its plan)
    if ((flags & kWForceCdn) && r.round < 0) r.flags |= kWForceCdn;
    if (token != kNoToken) r.flags &= ~kWPrefetch;
    *created = false;
  }
  if (token != kNoToken) {
    recs_[id].waiters.push_back(token);
    token_[token] = id;
  }
  return id;
}

bool WantTable::abort(int64_t token) {
  auto t = token_.find(token);
  if (t == token_.end()) return false;
  auto it = recs_.find(t->second);
  token_.erase(t);
  if (it == recs_.end()) return false;
  auto& w = it->second.waiters;
  auto p = std::find(w.begin(), w.end(), token);
  if (p != w.end()) {
    *p = w.back();
    w.pop_back();
  }
  return true;
}

int64_t WantTable::lookup(const SegKey& key) const {
  auto it = index_.find(key);
  return it == index_.end() ? -1 : it->second;
}

WantRec* WantTable::get(int64_t id) {
  auto it = recs_.find(id);
  return it == recs_.end() ? nullptr : &it->second;
}

const WantRec* WantTable::get(int64_t id) const {
  auto it = recs_.find(id);
  return it == recs_.end() ? nullptr : &it->second;
}

void WantTable::erase(std::unordered_map<int64_t, WantRec>::iterator it) {
  for (int64_t t : it->second.waiters) token_.erase(t);
  index_.erase(it->second.key);
  recs_.erase(it);
}

void WantTable::compact() {
  std::deque<int64_t> keep;
  for (int64_t id : order_)
    if (recs_.count(id)) keep.push_back(id);
  order_.swap(keep);
}

void WantTable::select(const SegmentStore& store, const Directory* dir, int64_t cap, int32_t round,
                       std::vector<int64_t>* admitted, std::vector<int64_t>* dropped,
                       std::vector<int64_t>* too_big, int64_t* deferred) {
  if (order_.size() > 64 && order_.size() > 2 * recs_.size()) compact();
  std::vector<int64_t> pick, spec;
  const size_t limit = cap < 0 ? SIZE_MAX : static_cast<size_t>(cap);
  for (size_t i = 0; i < order_.size(); ++i) {
    auto it = recs_.find(order_[i]);
    if (it == recs_.end()) {  // finished: prune the front eagerly
      if (i == 0) {
        order_.pop_front();
        --i;
      }
      continue;
    }
    WantRec& r = it->second;
    if (r.round >= 0) continue;
    if (r.waiters.empty()) {
      if (r.flags & kWPrefetch) {
        if (spec.size() < limit) spec.push_back(r.id);
        continue;
      }
      dropped->push_back(r.id);
      erase(it);
      if (i == 0) {
        order_.pop_front();
        --i;
      }
      continue;
    }
    if (pick.size() >= limit) break;  // (cap 0 admits nothing: checked before the push)
    pick.push_back(r.id);
  }
  for (int64_t id : spec) {
    if (pick.size() >= limit) break;
    pick.push_back(id);
  }
  // sizes (a not-staged network want of unknown size takes a holder's announced length)
  std::vector<int64_t> need(pick.size());
  int64_t total = 0;
  for (size_t i = 0; i < pick.size(); ++i) {
    WantRec& r = recs_[pick[i]];
    if ((r.flags & kWNotStaged) && r.size == 0 && dir != nullptr) {
      const DirEntry* e = dir->find(r.key);
      if (e != nullptr) r.size = e->length;
    }
    need[i] = store.aligned(r.size);
    total += need[i];
  }
  size_t keep = pick.size();
  if (!store.fits(total)) {  // largest prefix that fits the ring now
    size_t lo = 0, hi = pick.size();
    std::vector<int64_t> prefix(pick.size() + 1, 0);
    for (size_t i = 0; i < pick.size(); ++i) prefix[i + 1] = prefix[i] + need[i];
    while (lo < hi) {
      const size_t mid = (lo + hi + 1) / 2;
      if (store.fits(prefix[mid]))
        lo = mid;
      else
        hi = mid - 1;
    }
    keep = lo;
  }
  for (size_t i = 0; i < keep; ++i) {
    recs_[pick[i]].round = round;
    admitted->push_back(pick[i]);
  }
  int64_t d = 0;
  for (size_t i = keep; i < pick.size(); ++i) {
    if (need[i] > store.capacity()) {
      too_big->push_back(pick[i]);  // the caller fails its waiters (and then finishes it)
    } else {
      ++d;
    }
  }
  *deferred = d;
}

void WantTable::encode(const int64_t* ids, int64_t n, int64_t* rows) const {
  for (int64_t i = 0; i < n; ++i) {
    int64_t* o = rows + 6 * i;
    auto it = recs_.find(ids[i]);
    if (it == recs_.end()) throw std::out_of_range("encode: unknown want id");
    const WantRec& r = it->second;
    o[0] = r.key.swarm;
    o[1] = r.key.level;
    o[2] = r.key.url_id;
    o[3] = r.key.sn;
    o[4] = r.size;
    o[5] = r.id | (int64_t(r.flags & kWForceCdn ? 1 : 0) << 62) | (int64_t(r.flags & kWNotStaged ? 1 : 0) << 61) |
           (int64_t(r.flags & kWStaging ? 1 : 0) << 60) | (int64_t(r.flags & kWHeld ? 1 : 0) << 59);
  }
}

void WantTable::finish(const int64_t* ids, int64_t n, std::vector<int64_t>* tokens, std::vector<int64_t>* index,
                       std::vector<uint8_t>* prefetch_only) {
  for (int64_t i = 0; i < n; ++i) {
    auto it = recs_.find(ids[i]);
    if (it == recs_.end()) {
      prefetch_only->push_back(0);
      continue;
    }
    WantRec& r = it->second;
    prefetch_only->push_back((r.flags & kWPrefetch) && r.waiters.empty() ? 1 : 0);
    for (int64_t t : r.waiters) {
      tokens->push_back(t);
      index->push_back(i);
    }
    erase(it);
  }
}

void WantTable::requeue(const int64_t* ids, int64_t n, bool force_cdn) {
  for (int64_t i = 0; i < n; ++i) {
    auto it = recs_.find(ids[i]);
    if (it == recs_.end()) continue;
    it->second.round = -1;
    it->second.flags |= kWHeld;
    if (force_cdn) {
      it->second.flags |= kWForceCdn;
      it->second.attempts += 1;
    }
  }
}

int64_t WantTable::waiting() const {
  int64_t n = 0;
  for (const auto& kv : recs_)
    if (kv.second.round < 0 && !(kv.second.flags & kWStaging)) ++n;
  return n;
}

void WantTable::audit(std::vector<std::string>* errors) const {
  auto err = [&](const std::string& m) {
    if (errors->size() < 64) errors->push_back(m);
  };
  for (const auto& kv : index_) {
    auto it = recs_.find(kv.second);
    if (it == recs_.end()) {
      err("index names unknown want " + std::to_string(kv.second));
    } else if (!(it->second.key == kv.first)) {
      err("index key of want " + std::to_string(kv.second) + " differs from the want's key");
    }
  }
  std::unordered_set<int64_t> in_order(order_.begin(), order_.end());
  for (const auto& kv : recs_) {
    const WantRec& r = kv.second;
    if (r.id != kv.first) err("want " + std::to_string(kv.first) + " records id " + std::to_string(r.id));
    auto ix = index_.find(r.key);
    if (ix == index_.end() || ix->second != kv.first) err("want " + std::to_string(kv.first) + " is not indexed by its key");
    if (!in_order.count(kv.first)) err("want " + std::to_string(kv.first) + " is missing from the creation order");
    if (kv.first >= next_id_) err("want id " + std::to_string(kv.first) + " >= next id");
    std::unordered_set<int64_t> w;
    for (int64_t t : r.waiters) {
      if (!w.insert(t).second) err("token " + std::to_string(t) + " waits twice on want " + std::to_string(kv.first));
      auto tt = token_.find(t);
      if (tt == token_.end()) {
        err("waiter " + std::to_string(t) + " of want " + std::to_string(kv.first) + " is not in the token map");
      } else if (tt->second != kv.first) {
        err("waiter " + std::to_string(t) + " of want " + std::to_string(kv.first) + " maps to want " +
            std::to_string(tt->second));
      }
    }
  }
  for (const auto& kv : token_) {
    auto it = recs_.find(kv.second);
    if (it == recs_.end()) {
      err("token " + std::to_string(kv.first) + " maps to unknown want " + std::to_string(kv.second));
      continue;
    }
    const auto& w = it->second.waiters;
    if (std::count(w.begin(), w.end(), kv.first) != 1)
      err("token " + std::to_string(kv.first) + " is not a waiter of its want " + std::to_string(kv.second));
  }
}

void WantTable::ids(std::vector<int64_t>* out) const {
  out->clear();
  out->reserve(recs_.size());
  for (const auto& kv : recs_) out->push_back(kv.first);
  std::sort(out->begin(), out->end());
}

void WantTable::token_map(std::vector<int64_t>* tokens, std::vector<int64_t>* wants) const {
  tokens->clear();
  wants->clear();
  for (const auto& kv : token_) {
    tokens->push_back(kv.first);
    wants->push_back(kv.second);
  }
}

}  // namespace hlsp2p
