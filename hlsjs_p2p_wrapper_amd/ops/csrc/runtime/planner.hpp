// Swarm directory + deterministic exchange planner.
//
// The reference hands segment exchange to the closed-source peer agent over WebRTC
// DataChannels with a tracker.  RCCL point-to-point is two-sided and
// ordered, so on the MI355X node on-demand request/response becomes *exchange rounds*:
// every rank all-gathers a small control message (its wants and its cache delta), applies
// the deltas to an identical replicated directory, and runs this planner — pure,
// deterministic, same inputs on every rank — so all ranks agree on who sends what to whom
// without any further negotiation.  Each rank then posts exactly the matching RCCL
// send/recv batch.
//
// Planning policy per wanted key (keys processed in sorted order, wanters in rank order):
//   1. wanter offline or P2P download off              -> CDN fetch by the wanter;
//   2. some other online, upload-enabled rank holds it -> P2P from the holder whose link
//      to the wanter is least loaded this round (then least total send bytes, then a
//      rotation), spreading traffic over the 7 point-to-point xGMI links;
//   3. nobody holds it: with CDN de-duplication one wanter (least CDN bytes this round,
//      hash rotation on ties) "seeds" it from the CDN and forwards it to the other wanters
//      in the same round; without it every wanter goes to the CDN.
// A CDN fetch needs the body in host memory.  In-process origins always have it; a network
// origin (net/network.py) first downloads it ("stages" it).  A want flagged kNotStaged is
// never given a CDN row: where it would be, the planner emits a STAGE row (src = kStage) for
// that rank instead — for a seed group only for the rank chosen as seeder, the others wait —
// and the want is planned again once its rank reports it staged.  While some wanter is
// still downloading (kStaging) nobody else is told to: the key's other wanters wait.  So a segment crosses the
// network once per swarm, and the same round protocol serves both origin kinds.
#pragma once
#include <cstdint>
#include <unordered_map>
#include <vector>

#include "store.hpp"

namespace hlsp2p {

constexpr int kMaxRanks = 64;

// kCdnBound: the rank's CDN copies keep its ingest link busy most of the time (its link is the
// bottleneck); only such a rank is relieved by the CDN balance (plan_round_into)
enum RankFlag : int64_t { kOnline = 1, kUploadOn = 2, kDownloadOn = 4, kCdnDedup = 8, kCdnBound = 16 };

struct DirEntry {
  uint64_t holders = 0;
  int64_t length = 0;
};

// kNotStaged: the body is not in host memory yet; kStaging: this rank is downloading it now;
// kHeld: announced before without being served (a want is held back at most once, see
// plan_round_into's CDN balance)
enum WantFlag : int64_t { kForceCdn = 1, kNotStaged = 2, kStaging = 4, kHeld = 8 };

constexpr int32_t kCdn = -1;    // Transfer.src: CDN fetch (body in host memory) by dst
constexpr int32_t kStage = -2;  // Transfer.src: dst downloads the body from its network origin

struct Want {
  SegKey key;
  int64_t size;
  int64_t want_id;
  int32_t rank;
  int64_t flags = 0;  // WantFlag bits (kForceCdn: a previous peer copy failed its CRC)
};

struct Transfer {  // one segment moving src -> dst
  SegKey key;
  int64_t size;
  int32_t src;      // kCdn (-1) = CDN fetch, kStage (-2) = stage, else the sending rank
  int32_t dst;
  int64_t want_id;  // want id at dst
  int32_t seeded;   // 1: src fetched it from the CDN this round (forwarding)
};

// The replicated "who holds what" map.  Every rank applies every rank's adds and removes each
// round (8 ranks x hundreds of deltas), so this is an open-addressing table (linear probing,
// backward-shift deletion, load <= 1/2) of 32-byte slots in one array: no node allocation
// per insert or free per erase, one or two cache lines per probe.  A slot is empty iff its
// holder mask is 0 (an entry is erased the moment its last holder drops it).
// One multiply-xorshift: the directory and the planner's key grouping hash a key per
// delta / want (~10^4 a round at 8 ranks), so the two-round mix of SegKeyHash is not paid
// here.  Consecutive sns (the common key stream) land in distinct slots.
struct DirKeyHash {
  size_t operator()(const SegKey& k) const {
    uint64_t x = ((uint64_t(k.swarm) << 32) | k.level) * 0x9E3779B97F4A7C15ull;
    x ^= ((uint64_t(k.url_id) << 32) | k.sn);
    x *= 0xD6E8FEB86659FD93ull;
    return static_cast<size_t>(x ^ (x >> 32));
  }
};

class Directory {
 public:
  Directory();
  void apply_add(int rank, const SegKey& k, int64_t length);
  void apply_remove(int rank, const SegKey& k);
  void drop_rank(int rank);  // a rank left: forget everything it held
  const DirEntry* find(const SegKey& k) const;
  int64_t size() const { return size_; }
  // Keys (and lengths) `rank` is a holder of (the audit's view of what peers believe it holds).
  void holder_keys(int rank, std::vector<SegKey>* keys, std::vector<int64_t>* lens) const {
    for (const Slot& s : slots_)
      if ((s.e.holders >> rank) & 1u) {
        keys->push_back(s.key);
        lens->push_back(s.e.length);
      }
  }
  // Order-independent 64-bit digest of the whole content (every key with its holder mask
  // and length), kept up to date by every add / remove in O(1).  Every rank replays the same
  // deltas into its replica, so the replicas' digests must agree at every round; ranks
  // compare them in the control all-gather and stop before planning on a divergent state
  // (a two-sided transport would otherwise hang in a send/recv group nobody matches).
  uint64_t digest() const { return digest_; }

 private:
  struct Slot {
    SegKey key;
    DirEntry e;
  };
  size_t home(const SegKey& k) const { return DirKeyHash{}(k) & mask_; }
  void rehash(size_t cap);
  void erase_at(size_t i);
  // digest terms: one per (key, holder rank) and one per (key, length), summed mod 2^64 --
  // an add or remove changes one or two terms (one multiply each), so the digest costs
  // ~1 ns per delta on the control path instead of re-hashing the entry
  static uint64_t holder_term(uint64_t hk, int rank) {
    return (hk + uint64_t(rank + 1) * 0x9E3779B97F4A7C15ull) * 0xD6E8FEB86659FD93ull;
  }
  static uint64_t length_term(uint64_t hk, int64_t length) {
    return (hk ^ (uint64_t(length) * 0xA0761D6478BD642Full)) * 0xE7037ED1A0B428DBull;
  }
  static uint64_t entry_terms(const Slot& s);
  std::vector<Slot> slots_;
  uint64_t digest_ = 0;
  size_t mask_ = 0;
  int64_t size_ = 0;
};

// Returns every transfer of the round (CDN fetches have src = -1), in a canonical order:
// all CDN fetches first, then P2P transfers grouped by (src, dst) in key order — the order
// in which both sides pack / unpack their per-pair buffers.
// Order-sensitive 64-bit digest of a plan (every row's key, size, src, dst, want id,
// seeded): identical inputs give identical plans, so every rank's digest of a round's FULL
// plan must agree; a rank that planned differently would post sends or receives nobody matches.
uint64_t plan_digest(const std::vector<Transfer>& plan);

std::vector<Transfer> plan_round(const Directory& dir, const std::vector<Want>& wants,
                                 const std::vector<int64_t>& rank_flags, int world);
// The same plan written into `out` (cleared first; its capacity is reused round to round).
// `cdn_bytes` (optional, one entry per rank: each rank's cumulative CDN bytes, from the
// round's control headers): CDN balance -- a segment only one rank wants, no peer holds and
// another rank is about to want (it already asks for an earlier segment of the same track),
// is held back one announcement when its wanter has fetched more than its share from the
// CDN; the follower then fetches it alone and the leader takes the copy.  Ranks whose players
// run a round apart never co-want a segment, so without this the rank ahead seeds the whole
// swarm.  Only a rank flagged kCdnBound is relieved: a held want arrives a round later, which
// measured -18.5 % on the rehearsal plane when the leader's ingest was cheap (HBM origin).  The
// node keeps the balance opt-in (HLSP2P_CDN_BALANCE=1): with the gate, the one-GPU rehearsals
// still lost 7-13 % with a PCIe origin, where all ranks share one link and spreading the
// fetches cannot add bandwidth (profiles/r4_balance/NOTES.md).
void plan_round_into(const Directory& dir, const Want* wants, size_t n, const std::vector<int64_t>& rank_flags,
                     int world, std::vector<Transfer>* out, const int64_t* cdn_bytes = nullptr);

}  // namespace hlsp2p
