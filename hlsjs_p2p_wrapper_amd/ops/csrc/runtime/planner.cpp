#include "planner.hpp"

#include <algorithm>
#include <stdexcept>

namespace hlsp2p {

void Directory::apply_add(int rank, const SegKey& k, int64_t length) {
  DirEntry& e = map_[k];
  e.holders |= (uint64_t(1) << rank);
  e.length = length;
}

void Directory::apply_remove(int rank, const SegKey& k) {
  auto it = map_.find(k);
  if (it == map_.end()) return;
  it->second.holders &= ~(uint64_t(1) << rank);
  if (it->second.holders == 0) map_.erase(it);
}

void Directory::drop_rank(int rank) {
  const uint64_t mask = ~(uint64_t(1) << rank);
  for (auto it = map_.begin(); it != map_.end();) {
    it->second.holders &= mask;
    if (it->second.holders == 0)
      it = map_.erase(it);
    else
      ++it;
  }
}

const DirEntry* Directory::find(const SegKey& k) const {
  auto it = map_.find(k);
  return it == map_.end() ? nullptr : &it->second;
}

std::vector<Transfer> plan_round(const Directory& dir, const std::vector<Want>& wants_in,
                                 const std::vector<int64_t>& flags, int world) {
  if (world <= 0 || world > kMaxRanks) throw std::invalid_argument("world size out of range");
  std::vector<Want> wants(wants_in);
  std::stable_sort(wants.begin(), wants.end(), [](const Want& a, const Want& b) {
    if (!(a.key == b.key)) return a.key < b.key;
    if (a.rank != b.rank) return a.rank < b.rank;
    return a.want_id < b.want_id;
  });
  auto flag = [&](int r, int64_t f) { return (flags[r] & f) != 0; };
  // may want `wt` receive a peer copy of `size` bytes?  Staged (or in-process) wants always
  // announce the size they reserved; a not-staged one only once it reserved at least that
  auto fits_recv = [](const Want& wt, int64_t size) { return !(wt.flags & kNotStaged) || wt.size >= size; };

  std::vector<int64_t> link(size_t(world) * world, 0);  // bytes src->dst this round
  std::vector<int64_t> send_total(world, 0), cdn_total(world, 0);
  std::vector<Transfer> cdn, p2p;
  // a CDN fetch for want w, or its STAGE row when w's body is not in host memory yet
  auto cdn_or_stage = [&](const Want& wt, const SegKey& key) {
    if (wt.flags & kStaging) return;  // its download is running: nothing to plan yet
    const bool staged = !(wt.flags & kNotStaged);
    cdn.push_back({key, wt.size, staged ? kCdn : kStage, wt.rank, wt.want_id, 0});
    if (staged) cdn_total[wt.rank] += wt.size;
  };
  // keys no peer holds yet but several ranks want: ONE rank fetches from the CDN and
  // forwards in the same round ("seeding"); assigned after the pass (run-affine, below)
  struct SeedGroup {
    SegKey key;
    size_t i, j;
    std::vector<size_t> unserved;
    uint64_t cands;  // wanting ranks that may upload (staged ones only, when any is)
    bool staged;     // the seeder has the body in host memory (else it only stages it)
  };
  std::vector<SeedGroup> seeds;

  size_t i = 0;
  while (i < wants.size()) {
    size_t j = i;
    while (j < wants.size() && wants[j].key == wants[i].key) ++j;
    const SegKey key = wants[i].key;
    const DirEntry* de = dir.find(key);
    uint64_t holders = 0;
    if (de) {
      for (int r = 0; r < world; ++r)
        if (((de->holders >> r) & 1u) && flag(r, kOnline) && flag(r, kUploadOn)) holders |= uint64_t(1) << r;
    }
    std::vector<size_t> unserved;
    for (size_t w = i; w < j; ++w) {
      const Want& wt = wants[w];
      const int d = wt.rank;
      if (!flag(d, kOnline) || !flag(d, kDownloadOn) || (wt.flags & kForceCdn)) {
        cdn_or_stage(wt, key);
        continue;
      }
      uint64_t cand = holders & ~(uint64_t(1) << d);
      if (!cand) {
        unserved.push_back(w);
        continue;
      }
      // a wanter only receives what its admission reserved: a not-staged network want that
      // does not know the holder's length yet waits a round (its node reads the length from
      // the directory and reserves it before announcing the want again)
      if (!fits_recv(wt, de ? de->length : wt.size)) continue;
      int best = -1;
      for (int k = 1; k <= world; ++k) {  // rotation start: the rank after d
        int h = (d + k) % world;
        if (!((cand >> h) & 1u)) continue;
        if (best < 0) { best = h; continue; }
        int64_t lh = link[size_t(h) * world + d], lb = link[size_t(best) * world + d];
        if (lh < lb || (lh == lb && send_total[h] < send_total[best])) best = h;
      }
      const int64_t size = de ? de->length : wt.size;
      p2p.push_back({key, size, best, d, wt.want_id, 0});
      link[size_t(best) * world + d] += size;
      send_total[best] += size;
    }
    if (!unserved.empty()) {
      bool dedup = unserved.size() > 1;
      for (size_t w : unserved) dedup = dedup && flag(wants[w].rank, kCdnDedup);
      uint64_t cands = 0;
      if (dedup)
        for (size_t w : unserved)
          if (flag(wants[w].rank, kUploadOn)) cands |= uint64_t(1) << wants[w].rank;
      if (cands) {
        // staged wanters seed; with none staged yet, one wanter is chosen to stage it
        uint64_t ready = 0;
        bool staging = false;
        for (size_t w : unserved) {
          if (!(wants[w].flags & kNotStaged)) ready |= uint64_t(1) << wants[w].rank;
          staging = staging || (wants[w].flags & kStaging);
        }
        if ((cands & ready) || !staging)  // else a wanter is downloading it: all wait this round
          seeds.push_back({key, i, j, std::move(unserved), (cands & ready) ? (cands & ready) : cands,
                           (cands & ready) != 0});  // seeder chosen below
      } else {
        for (size_t w : unserved) cdn_or_stage(wants[w], key);
      }
    }
    i = j;
  }
  // Seeder assignment, run-affine: consecutive keys (sorted: same track, ascending sn) go
  // to the same rank until it holds its share of the round's seed bytes.  Load stays
  // balanced, and each rank's CDN fetches form ONE contiguous sn run, i.e. one merged
  // pinned-host -> HBM DMA instead of every world-th segment.
  if (!seeds.empty()) {
    int64_t seed_bytes = 0;
    uint64_t all = 0;
    for (const auto& g : seeds) {
      int64_t sz = 0;  // a not-yet-staged network want does not know its size (0)
      for (size_t w : g.unserved) sz = std::max(sz, wants[w].size);
      seed_bytes += sz;
      all |= g.cands;
    }
    int nseed = 0;
    for (int r = 0; r < world; ++r) nseed += int((all >> r) & 1u);
    const int64_t quota = (seed_bytes + nseed - 1) / std::max(nseed, 1);
    std::vector<int64_t> seeded(world, 0);
    int cur = -1;
    for (const auto& g : seeds) {
      int seeder = -1;
      if (cur >= 0 && ((g.cands >> cur) & 1u) && seeded[cur] < quota) seeder = cur;
      if (seeder < 0) {  // next rank (in rank order) with room, else the least loaded
        for (int k = 1; k <= world && seeder < 0; ++k) {
          const int r = ((cur < 0 ? -1 : cur) + k + world) % world;
          if (((g.cands >> r) & 1u) && seeded[r] < quota) seeder = r;
        }
        for (int r = 0; r < world && seeder < 0; ++r) {
          if (!((g.cands >> r) & 1u)) continue;
          int best = r;
          for (int q = r + 1; q < world; ++q)
            if (((g.cands >> q) & 1u) && seeded[q] < seeded[best]) best = q;
          seeder = best;
        }
      }
      cur = seeder;
      // the seeder's want carries the size every forwarded copy has (a wanter that has not
      // staged the body itself may not know it)
      const Want* own = nullptr;
      for (size_t w : g.unserved)
        if (wants[w].rank == seeder && own == nullptr) own = &wants[w];
      const int64_t sz = own->size;
      seeded[seeder] += sz;
      if (!g.staged) {  // nobody has the body yet: the seeder stages it, the rest wait
        cdn.push_back({g.key, sz, kStage, seeder, own->want_id, 0});
        continue;
      }
      for (size_t w : g.unserved) {
        const Want& wt = wants[w];
        if (wt.rank == seeder) {
          cdn.push_back({g.key, wt.size, kCdn, seeder, wt.want_id, 0});
          cdn_total[seeder] += wt.size;
        }
      }
      for (size_t w : g.unserved) {
        const Want& wt = wants[w];
        if (wt.rank == seeder) continue;
        if (!fits_recv(wt, sz)) continue;  // (see above) it gets the seeder's copy next round
        p2p.push_back({g.key, sz, seeder, wt.rank, wt.want_id, 1});
        link[size_t(seeder) * world + wt.rank] += sz;
        send_total[seeder] += sz;
      }
    }
  }
  std::stable_sort(p2p.begin(), p2p.end(), [](const Transfer& a, const Transfer& b) {
    if (a.src != b.src) return a.src < b.src;
    if (a.dst != b.dst) return a.dst < b.dst;
    return a.key < b.key;
  });
  std::vector<Transfer> out;
  out.reserve(cdn.size() + p2p.size());
  out.insert(out.end(), cdn.begin(), cdn.end());
  out.insert(out.end(), p2p.begin(), p2p.end());
  return out;
}

}  // namespace hlsp2p
