#include "planner.hpp"

#include <algorithm>
#include <mutex>
#include <stdexcept>

namespace hlsp2p {

Directory::Directory() { rehash(1024); }

namespace {
inline uint64_t fmix64(uint64_t x) {  // murmur3 finalizer: full avalanche of every input bit
  x ^= x >> 33;
  x *= 0xFF51AFD7ED558CCDull;
  x ^= x >> 33;
  x *= 0xC4CEB9FE1A85EC53ull;
  return x ^ (x >> 33);
}
// a well-mixed 64-bit draw from a segment key (planner tie-breaks that must agree on every
// replica but not favour low ranks)
inline uint64_t key_draw(const SegKey& k) {
  return fmix64((uint64_t(k.swarm) << 32) ^ (uint64_t(k.level) << 48) ^ (uint64_t(k.url_id) << 16) ^
                uint64_t(k.sn));
}
}  // namespace

uint64_t Directory::entry_terms(const Slot& s) {
  const uint64_t hk = DirKeyHash{}(s.key);
  uint64_t d = length_term(hk, s.e.length);
  for (uint64_t m = s.e.holders; m; m &= m - 1) d += holder_term(hk, __builtin_ctzll(m));
  return d;
}

void Directory::rehash(size_t cap) {
  std::vector<Slot> old;
  old.swap(slots_);
  slots_.assign(cap, Slot{});
  mask_ = cap - 1;
  size_ = 0;
  digest_ = 0;  // recomputed: drop_rank edits holder masks in place before re-packing
  for (const Slot& s : old) {
    if (s.e.holders == 0) continue;
    digest_ += entry_terms(s);
    size_t i = home(s.key);
    while (slots_[i].e.holders != 0) i = (i + 1) & mask_;
    slots_[i] = s;
    ++size_;
  }
}

void Directory::apply_add(int rank, const SegKey& k, int64_t length) {
  if (size_t(size_ + 1) * 2 > slots_.size()) rehash(slots_.size() * 2);
  const uint64_t hk = DirKeyHash{}(k);
  size_t i = hk & mask_;
  while (slots_[i].e.holders != 0 && !(slots_[i].key == k)) i = (i + 1) & mask_;
  Slot& s = slots_[i];
  const uint64_t bit = uint64_t(1) << rank;
  if (s.e.holders == 0) {
    s.key = k;
    ++size_;
    digest_ += length_term(hk, length);
  } else if (s.e.length != length) {
    digest_ += length_term(hk, length) - length_term(hk, s.e.length);
  }
  if (!(s.e.holders & bit)) digest_ += holder_term(hk, rank);
  s.e.holders |= bit;
  s.e.length = length;
}

// backward-shift deletion: pull later members of the probe run into the hole so every key
// stays reachable from its home slot without tombstones
void Directory::erase_at(size_t i) {
  size_t j = i;
  for (;;) {
    j = (j + 1) & mask_;
    if (slots_[j].e.holders == 0) break;
    const size_t k = home(slots_[j].key);
    // slot j may move to i iff its home k is not cyclically inside (i, j]
    const bool stays = (i <= j) ? (i < k && k <= j) : (i < k || k <= j);
    if (stays) continue;
    slots_[i] = slots_[j];
    i = j;
  }
  slots_[i] = Slot{};
  --size_;
}

void Directory::apply_remove(int rank, const SegKey& k) {
  const uint64_t hk = DirKeyHash{}(k);
  size_t i = hk & mask_;
  while (slots_[i].e.holders != 0) {
    if (slots_[i].key == k) {
      const uint64_t bit = uint64_t(1) << rank;
      if (slots_[i].e.holders & bit) digest_ -= holder_term(hk, rank);
      slots_[i].e.holders &= ~bit;
      if (slots_[i].e.holders == 0) {
        digest_ -= length_term(hk, slots_[i].e.length);
        slots_[i].e.holders = 1;  // still occupied while erase_at shifts the run
        erase_at(i);
      }
      return;
    }
    i = (i + 1) & mask_;
  }
}

void Directory::drop_rank(int rank) {
  const uint64_t mask = ~(uint64_t(1) << rank);
  for (Slot& s : slots_) s.e.holders &= mask;
  rehash(slots_.size());  // drops the emptied entries, re-packs the probe runs
}

const DirEntry* Directory::find(const SegKey& k) const {
  size_t i = home(k);
  while (slots_[i].e.holders != 0) {
    if (slots_[i].key == k) return &slots_[i].e;
    i = (i + 1) & mask_;
  }
  return nullptr;
}

namespace {
// Working storage of plan_round: every vector keeps its capacity from round to round, so a
// warm round allocates (and page-faults) nothing -- at 8 ranks x 512 wants a fresh ~1 MB of
// vectors per call cost ~40 % of the planner's time.  One process-wide instance behind a
// mutex (in-process swarms plan from several threads): a thread_local one measured ~35 %
// slower inside the dlopen-ed module (every access through the TLS wrapper).
struct PlanScratch {
  std::vector<Want> wants;
  std::vector<uint32_t> cnt;
  std::vector<int32_t> tab;
  std::vector<SegKey> gkey;
  std::vector<uint32_t> gcount, gid, gord, gpos;
  std::vector<int64_t> link, send_total, cdn_total, seeded;
  std::vector<Transfer> cdn, p2p, sorted;
  std::vector<size_t> members, unserved;
  std::vector<uint32_t> start, split, fill;
};
PlanScratch g_scratch;
std::mutex g_scratch_mu;

// Grouping fast path.  A round's wants are, in the common case, a few tracks over a narrow sn
// window (players ask for consecutive segments), concatenated rank by rank (ingest_control),
// each rank wanting a key at most once.  A stable counting sort by (track, sn) then yields the
// (key, rank, want id) order directly: O(n + window) with no hashing (~3x cheaper than the
// general path at 8 ranks x 256 wants).  Returns false -- nothing written -- when the input is
// not of that shape; the caller then takes the general path.
bool group_by_window(const Want* in, size_t n, std::vector<uint32_t>* cnt_buf, Want* out) {
  constexpr int kTracks = 8;
  if (n < 16) return false;
  SegKey tk[kTracks]{};
  uint32_t lo[kTracks]{}, hi[kTracks]{};
  int nt = 0, last = 0, prev_rank = -1;
  for (size_t i = 0; i < n; ++i) {
    const Want& w = in[i];
    if (w.rank < prev_rank) return false;  // not rank-major
    prev_rank = w.rank;
    const SegKey& k = w.key;
    int t = last;
    if (t >= nt || !(tk[t].swarm == k.swarm && tk[t].level == k.level && tk[t].url_id == k.url_id)) {
      for (t = 0; t < nt; ++t)
        if (tk[t].swarm == k.swarm && tk[t].level == k.level && tk[t].url_id == k.url_id) break;
      if (t == nt) {
        if (nt == kTracks) return false;
        tk[nt] = k;
        lo[nt] = hi[nt] = k.sn;
        ++nt;
      }
      last = t;
    }
    lo[t] = std::min(lo[t], k.sn);
    hi[t] = std::max(hi[t], k.sn);
  }
  // tracks in key order, each one's sn window placed after the previous ones
  int ord[kTracks];
  for (int t = 0; t < nt; ++t) ord[t] = t;
  std::sort(ord, ord + nt, [&](int a, int b) { return tk[a] < tk[b]; });
  uint64_t base[kTracks], range = 0;
  for (int q = 0; q < nt; ++q) {
    base[ord[q]] = range;
    range += uint64_t(hi[ord[q]]) - lo[ord[q]] + 1;
  }
  if (range > 4 * n + 1024) return false;  // too sparse: hashing is cheaper
  std::vector<uint32_t>& cnt = *cnt_buf;
  cnt.assign(range + 1, 0);
  auto slot_of = [&](const SegKey& k) -> size_t {
    int t = 0;
    while (!(tk[t].swarm == k.swarm && tk[t].level == k.level && tk[t].url_id == k.url_id)) ++t;
    return size_t(base[t] + (k.sn - lo[t]));
  };
  if (nt == 1) {
    for (size_t i = 0; i < n; ++i) ++cnt[size_t(in[i].key.sn - lo[0]) + 1];
  } else {
    for (size_t i = 0; i < n; ++i) ++cnt[slot_of(in[i].key) + 1];
  }
  for (size_t x = 0; x < range; ++x) cnt[x + 1] += cnt[x];
  if (nt == 1) {
    for (size_t i = 0; i < n; ++i) out[cnt[size_t(in[i].key.sn - lo[0])]++] = in[i];
  } else {
    for (size_t i = 0; i < n; ++i) out[cnt[slot_of(in[i].key)]++] = in[i];
  }
  // equal keys keep the input's rank order; a rank listing a key twice (not produced by the
  // want table) is ordered by want id here
  for (size_t x = 1; x < n; ++x)
    for (size_t y = x; y > 0 && out[y].key == out[y - 1].key && out[y].rank == out[y - 1].rank &&
                       out[y].want_id < out[y - 1].want_id; --y)
      std::swap(out[y], out[y - 1]);
  return true;
}
}  // namespace

void plan_round_into(const Directory& dir, const Want* wants_in, size_t n_in, const std::vector<int64_t>& flags,
                     int world, std::vector<Transfer>* out_rows, const int64_t* cdn_bytes) {
  if (world <= 0 || world > kMaxRanks) throw std::invalid_argument("world size out of range");
  if (flags.size() < size_t(world)) throw std::invalid_argument("flags must have world entries");
  std::lock_guard<std::mutex> lock(g_scratch_mu);
  PlanScratch& S = g_scratch;
  // Wants in (key, rank, want id) order -- a total order, so every rank gets the same plan
  // -- without a comparison sort of all n wants (8 ranks x 512 wants: ~0.4 ms): group by key
  // with a hash table (n is 8x the distinct keys when every rank wants the same segments),
  // sort only the distinct keys (already ascending in the common case: players ask for
  // consecutive sns), place each want in its group's slot range, and order each group by
  // (rank, want id) with an insertion sort (a group holds at most one want per rank).
  const size_t n = n_in;
  std::vector<Want>& wants = S.wants;
  wants.resize(n);
  if (!group_by_window(wants_in, n, &S.cnt, wants.data())) {
    size_t cap = 16;
    while (cap < 2 * n) cap <<= 1;
    const size_t mask = cap - 1;
    std::vector<int32_t>& tab = S.tab;
    tab.assign(cap, -1);
    std::vector<SegKey>& gkey = S.gkey;
    std::vector<uint32_t>& gcount = S.gcount;
    std::vector<uint32_t>& gid = S.gid;
    gkey.clear();
    gcount.clear();
    gid.resize(n);
    for (size_t i = 0; i < n; ++i) {
      const SegKey& k = wants_in[i].key;
      size_t h = DirKeyHash{}(k) & mask;
      while (tab[h] >= 0 && !(gkey[size_t(tab[h])] == k)) h = (h + 1) & mask;
      if (tab[h] < 0) {
        tab[h] = static_cast<int32_t>(gkey.size());
        gkey.push_back(k);
        gcount.push_back(0);
      }
      gid[i] = static_cast<uint32_t>(tab[h]);
      ++gcount[gid[i]];
    }
    const size_t G = gkey.size();
    std::vector<uint32_t>& gord = S.gord;
    gord.resize(G);
    for (size_t g = 0; g < G; ++g) gord[g] = static_cast<uint32_t>(g);
    auto key_less = [&](uint32_t a, uint32_t b) { return gkey[a] < gkey[b]; };
    if (!std::is_sorted(gord.begin(), gord.end(), key_less)) std::sort(gord.begin(), gord.end(), key_less);
    std::vector<uint32_t>& gpos = S.gpos;
    gpos.resize(G);
    uint32_t pos = 0;
    for (uint32_t g : gord) {
      gpos[g] = pos;
      pos += gcount[g];
    }
    for (size_t i = 0; i < n; ++i) wants[gpos[gid[i]]++] = wants_in[i];
    auto within = [](const Want& a, const Want& b) {
      return a.rank != b.rank ? a.rank < b.rank : a.want_id < b.want_id;
    };
    size_t a = 0;
    for (uint32_t g : gord) {
      const size_t b = a + gcount[g];
      for (size_t x = a + 1; x < b; ++x)  // insertion sort: already ordered for rank-major input
        for (size_t y = x; y > a && within(wants[y], wants[y - 1]); --y) std::swap(wants[y], wants[y - 1]);
      a = b;
    }
  }
  auto flag = [&](int r, int64_t f) { return (flags[r] & f) != 0; };
  // may want `wt` receive a peer copy of `size` bytes?  Only within what its admission
  // reserved: the wanter's node retired exactly that much of its ring before announcing the
  // want (node.py: retire_region), so a larger copy could land on entries a peer is sending
  // from.  A not-staged network want that does not know the holder's length yet waits a round
  // (its node reads the length from the directory and reserves it before announcing again); a
  // staged want whose own size is smaller than the holder's copy fetches from the CDN.
  auto fits_recv = [](const Want& wt, int64_t size) { return wt.size >= size; };

  std::vector<int64_t>& link = S.link;  // bytes src->dst this round
  link.assign(size_t(world) * world, 0);
  std::vector<int64_t>& send_total = S.send_total;
  std::vector<int64_t>& cdn_total = S.cdn_total;
  send_total.assign(world, 0);
  cdn_total.assign(world, 0);
  std::vector<Transfer>& cdn = S.cdn;
  std::vector<Transfer>& p2p = S.p2p;
  cdn.clear();
  p2p.clear();
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
    size_t a, b;     // its unserved wants: members[a, b)
    uint64_t cands;  // wanting ranks that may upload (staged ones only, when any is)
    bool staged;     // the seeder has the body in host memory (else it only stages it)
  };
  std::vector<SeedGroup> seeds;
  seeds.reserve(64);
  std::vector<size_t>& members = S.members;  // every seed group's unserved want indices, back to back
  std::vector<size_t>& unserved = S.unserved;  // reused per key
  members.clear();

  // CDN balance (see planner.hpp): is rank d over its share of the swarm's CDN bytes?
  constexpr int64_t kBalanceMinBytes = int64_t(256) << 20;  // no decisions on start-up noise
  constexpr uint32_t kFollowSns = 4096;                      // "about to want": within this many sns
  uint64_t over_share = 0;
  if (cdn_bytes != nullptr && world > 1) {
    int64_t total = 0;
    int active = 0;
    for (int r = 0; r < world; ++r)
      if (flag(r, kOnline) && flag(r, kCdnDedup)) {
        total += cdn_bytes[r];
        ++active;
      }
    if (active > 1 && total >= kBalanceMinBytes)
      for (int r = 0; r < world; ++r)  // share > 1.1 / active, and the rank's link is its bound
        if (flag(r, kOnline) && flag(r, kCdnBound) && cdn_bytes[r] * 10 * active > total * 11)
          over_share |= uint64_t(1) << r;
  }
  // per track (swarm, level, url_id): each rank's first wanted sn this round (wants are in key
  // order, so the first want of a rank inside a track run has its smallest sn)
  uint32_t track_first[kMaxRanks];
  uint64_t track_ranks = 0;
  size_t track_end = 0;
  auto same_track = [](const SegKey& a, const SegKey& b) {
    return a.swarm == b.swarm && a.level == b.level && a.url_id == b.url_id;
  };

  size_t i = 0;
  while (i < wants.size()) {
    size_t j = i;
    while (j < wants.size() && wants[j].key == wants[i].key) ++j;
    const SegKey key = wants[i].key;
    if (over_share && i >= track_end) {  // entering a new track: scan its wants once
      track_ranks = 0;
      track_end = i;
      while (track_end < wants.size() && same_track(wants[track_end].key, key)) {
        const int r = wants[track_end].rank;
        if (!((track_ranks >> r) & 1u)) {
          track_ranks |= uint64_t(1) << r;
          track_first[r] = wants[track_end].key.sn;
        }
        ++track_end;
      }
    }
    const DirEntry* de = dir.find(key);
    uint64_t holders = 0;
    if (de) {
      for (int r = 0; r < world; ++r)
        if (((de->holders >> r) & 1u) && flag(r, kOnline) && flag(r, kUploadOn)) holders |= uint64_t(1) << r;
    }
    unserved.clear();
    // holder rotation offset drawn from the key (same on every replica): a lone wanter's
    // equal-load holders take turns across rounds instead of the rank after it every time
    const int koff = world > 1 ? int(key_draw(key) % uint64_t(world)) : 0;
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
      // a wanter only receives what its admission reserved (fits_recv)
      if (!fits_recv(wt, de ? de->length : wt.size)) {
        if (!(wt.flags & kNotStaged)) cdn_or_stage(wt, key);
        continue;
      }
      int best = -1;
      for (int k = 1; k <= world; ++k) {  // rotation start: the rank after d, shifted by the key
        int h = (d + koff + k) % world;
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
        if ((cands & ready) || !staging) {  // else a wanter is downloading it: all wait this round
          const size_t a = members.size();
          members.insert(members.end(), unserved.begin(), unserved.end());
          seeds.push_back({key, a, members.size(), (cands & ready) ? (cands & ready) : cands,
                           (cands & ready) != 0});  // seeder chosen below
        }
      } else {
        for (size_t w : unserved) {
          const Want& wt = wants[w];
          if (unserved.size() == 1 && ((over_share >> wt.rank) & 1u) && !(wt.flags & (kHeld | kForceCdn)) &&
              flag(wt.rank, kCdnDedup)) {
            bool follower = false;  // another rank that will want it: online, in the swarm, behind
            for (int r = 0; r < world && !follower; ++r)
              follower = r != wt.rank && ((track_ranks >> r) & 1u) && flag(r, kOnline) && flag(r, kCdnDedup) &&
                         flag(r, kDownloadOn) && track_first[r] <= key.sn && key.sn - track_first[r] <= kFollowSns;
            if (follower) continue;  // held back one announcement (kHeld next time)
          }
          cdn_or_stage(wt, key);
        }
      }
    }
    i = j;
  }
  const size_t p2p_main = p2p.size();  // holder transfers, generated in key order
  // Seeder assignment, run-affine: consecutive keys (sorted: same track, ascending sn) go
  // to the same rank until it holds its share of the round's seed bytes.  Load stays
  // balanced, and each rank's CDN fetches form ONE contiguous sn run, i.e. one merged
  // pinned-host -> HBM DMA instead of every world-th segment.  The rotation starts at a rank
  // drawn from the round's first seed key (the same on every replica): a round with fewer
  // seeds than wanters -- the live edge, one new segment per round -- would otherwise give
  // every seed to the lowest wanting rank, whose CDN link then fetches for the whole swarm.
  if (!seeds.empty()) {
    int64_t seed_bytes = 0;
    uint64_t all = 0;
    for (const auto& g : seeds) {
      int64_t sz = 0;  // a not-yet-staged network want does not know its size (0)
      for (size_t m = g.a; m < g.b; ++m) sz = std::max(sz, wants[members[m]].size);
      seed_bytes += sz;
      all |= g.cands;
    }
    int nseed = 0;
    for (int r = 0; r < world; ++r) nseed += int((all >> r) & 1u);
    const int64_t quota = (seed_bytes + nseed - 1) / std::max(nseed, 1);
    std::vector<int64_t>& seeded = S.seeded;
    seeded.assign(world, 0);
    const int start = int(key_draw(seeds.front().key) % uint64_t(world));
    int cur = -1;
    for (const auto& g : seeds) {
      int seeder = -1;
      if (cur >= 0 && ((g.cands >> cur) & 1u) && seeded[cur] < quota) seeder = cur;
      if (seeder < 0) {  // next rank (in rank order) with room, else the least loaded
        for (int k = 1; k <= world && seeder < 0; ++k) {
          const int r = ((cur < 0 ? start - 1 : cur) + k + world) % world;
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
      for (size_t m = g.a; m < g.b; ++m)
        if (wants[members[m]].rank == seeder && own == nullptr) own = &wants[members[m]];
      const int64_t sz = own->size;
      seeded[seeder] += sz;
      if (!g.staged) {  // nobody has the body yet: the seeder stages it, the rest wait
        cdn.push_back({g.key, sz, kStage, seeder, own->want_id, 0});
        continue;
      }
      for (size_t m = g.a; m < g.b; ++m) {
        const Want& wt = wants[members[m]];
        if (wt.rank == seeder) {
          cdn.push_back({g.key, wt.size, kCdn, seeder, wt.want_id, 0});
          cdn_total[seeder] += wt.size;
        }
      }
      for (size_t m = g.a; m < g.b; ++m) {
        const Want& wt = wants[members[m]];
        if (wt.rank == seeder) continue;
        if (!fits_recv(wt, sz)) {  // (fits_recv) a not-staged one gets the seeder's copy next round
          if (!(wt.flags & kNotStaged)) cdn_or_stage(wt, g.key);
          continue;
        }
        p2p.push_back({g.key, sz, seeder, wt.rank, wt.want_id, 1});
        link[size_t(seeder) * world + wt.rank] += sz;
        send_total[seeder] += sz;
      }
    }
  }
  // P2P rows grouped by (src, dst), key order inside a pair.  Both parts of `p2p` (holder
  // transfers, then seeded forwards) were generated in ascending key order and a pair sees a
  // key at most once, so a stable counting sort by pair plus one merge of the two runs
  // inside each pair gives exactly the (src, dst, key) order, in O(n).
  {
    const size_t P = size_t(world) * world;
    std::vector<uint32_t>& start = S.start;
    std::vector<uint32_t>& split = S.split;
    start.assign(P + 1, 0);
    split.assign(P, 0);
    for (const Transfer& t : p2p) ++start[size_t(t.src) * world + t.dst + 1];
    for (size_t b = 0; b < P; ++b) start[b + 1] += start[b];
    std::vector<uint32_t>& fill = S.fill;
    fill.assign(start.begin(), start.end() - 1);
    std::vector<Transfer>& sorted = S.sorted;
    sorted.resize(p2p.size());
    for (size_t x = 0; x < p2p.size(); ++x) {
      const size_t b = size_t(p2p[x].src) * world + p2p[x].dst;
      if (x < p2p_main) ++split[b];
      sorted[fill[b]++] = p2p[x];
    }
    auto by_key = [](const Transfer& a, const Transfer& b) {
      return !(a.key == b.key) ? a.key < b.key : a.want_id < b.want_id;
    };
    for (size_t b = 0; b < P; ++b) {
      const size_t lo = start[b], mid = lo + split[b], hi = start[b + 1];
      if (mid > lo && mid < hi)
        std::inplace_merge(sorted.begin() + lo, sorted.begin() + mid, sorted.begin() + hi, by_key);
    }
    p2p.swap(sorted);
  }
  std::vector<Transfer>& out = *out_rows;
  out.clear();
  out.reserve(cdn.size() + p2p.size());
  out.insert(out.end(), cdn.begin(), cdn.end());
  out.insert(out.end(), p2p.begin(), p2p.end());
}

uint64_t plan_digest(const std::vector<Transfer>& plan) {
  // per row: the fields' independent multiplies folded into one word, then one multiply on
  // the running (order-sensitive) chain -- ~6 cycles a row, so the digest stays a few us at
  // 8 ranks x 256 wants; the final fmix spreads every bit
  uint64_t h = 0x243F6A8885A308D3ull ^ plan.size();
  for (const Transfer& t : plan) {
    const uint64_t x = ((uint64_t(t.key.swarm) << 32 | t.key.level) * 0x9E3779B97F4A7C15ull) ^
                       ((uint64_t(t.key.url_id) << 32 | t.key.sn) * 0xC2B2AE3D27D4EB4Full) ^
                       (uint64_t(t.size) * 0x165667B19E3779F9ull) ^
                       ((uint64_t(uint32_t(t.src)) << 32 | uint32_t(t.dst)) * 0xD6E8FEB86659FD93ull) ^
                       ((uint64_t(t.want_id) ^ (uint64_t(t.seeded) << 63)) * 0xA0761D6478BD642Full);
    h = (h ^ x ^ (x >> 29)) * 0xFF51AFD7ED558CCDull;
  }
  return fmix64(h);
}

std::vector<Transfer> plan_round(const Directory& dir, const std::vector<Want>& wants_in,
                                 const std::vector<int64_t>& flags, int world) {
  std::vector<Transfer> out;
  plan_round_into(dir, wants_in.data(), wants_in.size(), flags, world, &out);
  return out;
}

}  // namespace hlsp2p
