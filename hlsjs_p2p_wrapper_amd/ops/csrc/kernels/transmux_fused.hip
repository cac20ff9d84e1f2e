// Fused AES-128-CBC decrypt + MPEG-TS demux of a batch of HLS segments (SURVEY §2.2 K10 +
// K11) — CDNA4 / gfx950.  One pass over the ciphertext: the plaintext never exists in HBM.
// OPT-IN (HLSP2P_TRANSMUX=fused): the split sequence (aes_cbc.hip + ts_demux.hip) is the
// default because it measured faster — profiles/r3_transmux_fused_vs_split.md records the
// design iterations, their per-role timers and why.
//
// The split pipeline moves each segment through HBM ~5 times: decrypt reads the ciphertext
// and writes plaintext, the scan re-reads packet headers, the gather re-reads the plaintext
// and writes the elementary streams.  Here a persistent workgroup (one per CU) decrypts a
// TILE of a segment (128 TS packets = 32 x 47 AES blocks = 24,064 bytes; 4 packets = 47
// blocks is the smallest unit on which the 16-byte block grid and the 188-byte packet grid
// align) straight into LDS, parses the packet headers there, learns where its payload bytes
// go from the tiles before it, and writes them to the elementary-stream buffer: ciphertext
// read once, ES written once.
//
// Three kernels per batch:
//   transmux_psi_kernel    one wave per segment: decrypts the segment's first packets
//                          (4 at a time, until PAT and PMT are found, at most 64) and
//                          publishes the elementary PIDs — so no tile ever waits for the
//                          workgroup that happens to hold its segment's first tile.
//   transmux_fused_kernel  the persistent pipeline below.
//   transmux_tail_kernel   what only the whole segment knows (first / last PTS, padding).
//
// Wave specialisation inside the fused kernel (the 16 waves never meet at an s_barrier after
// setup; hand-offs are monotonic LDS counters and tags — release: the writer's LDS traffic
// drains (lgkmcnt only); acquire: the poller reads the flag before the data):
//   waves 0..7    DECRYPT (two per SIMD): the AES rounds are LDS bound (160 ds_read_b32 per
//                 block); three independent CBC blocks per lane, the next tile's ciphertext
//                 and geometry fetched during this tile, round keys by scalar loads.
//   waves 8..9    CONTROL, alternate tiles: packet parse (two packets per lane, two LDS
//                 round trips), DPP scans, the tile's aggregate, the inter-tile look-back,
//                 PES entries, the copy plan.
//   waves 10..14  COPY-OUT: read a parsed tile's payload words into registers at once —
//                 releasing its stage to the decrypt waves before the look-back is known —
//                 and store them once the plan (class bases) arrives.
//   wave 15       SCHEDULER: tickets from the global counter, segment geometry, PIDs.
// The latency-bound roles run at s_setprio 3 so their dependent LDS accesses are not queued
// behind the AES table reads.
//
// LDS (~139 KiB, one 1024-thread workgroup per CU):
//   [0, 64K)     row x (256 B) = [32 lane copies of Td0[x] | 32 copies of Td2[x]]; lane l
//                reads dword l % 32 of a half-row: every ds_read_b32 of the rounds is bank
//                conflict free.  Td2 = Td0 rotated by 16, so a column needs ONE rotation:
//                  Td0[a] ^ Td1[b] ^ Td2[c] ^ Td3[d] ^ k = Td0[a] ^ Td2[c] ^ rot8(Td0[b] ^ Td2[d] ^ rot24(k))
//                (the host passes the rounds' keys pre-rotated by 24).  No InvSbox
//                table: the byte-XOR of Td0[x] = (0e ^ 09 ^ 0d ^ 0b) . InvSbox[x] = InvSbox[x],
//                so the last round reads Td0 too and folds bytes on the VALU.
//   [64K, ...)   three plaintext stages, job ring, copy plans, hand-off words.
//
// Inter-tile prefix (decoupled look-back).  A tile's payload bytes land at the running sum
// of the payload bytes of the tiles before it (per class: video, audio, id3), and its PES
// entries at the running PES count.  Tiles are taken from a global ticket counter in order,
// and a workgroup processes its tickets in order, so every lower ticket belongs to a
// workgroup that will finish it without waiting on a higher one: a tile publishes its
// aggregate (three 8-byte {status, PES count, bytes} granules, one per class, written by
// single agent-scope stores and read back by agent-scope loads — the data is its own flag,
// no fence), looks back over its predecessors (all three classes per load, 256 tiles per
// round trip) until each class meets an inclusive prefix, then publishes its own inclusive
// prefix.  Every spin is bounded: a hand-off that never arrives sets the launch's timeout
// word and the tile proceeds (wrong output, no hang).
//
// ES layout per segment at es_off[seg]: three regions of es_cap[seg] bytes, video / audio /
// id3, each class written at its running offset in its own region; the info row says where
// each class starts (slots 22, 23).  PES tables and info rows are the split pipeline's and
// the host oracle's (runtime/ts.cpp).
#include "common.h"
#include "demux_dev.h"
#include "transmux_args.h"

namespace hlsp2p {
namespace dev {

namespace {

constexpr int kFThreads = 1024;
constexpr int kDWaves = 8;                        // decrypt waves 0..7 (two per SIMD)
constexpr int kCWave0 = kDWaves;                  // control waves 8..9
constexpr int kCWaves = 2;
constexpr int kXWave0 = kCWave0 + kCWaves;        // copy-out waves 10..14
constexpr int kXWaves = 5;
constexpr int kSWave = kXWave0 + kXWaves;         // scheduler wave 15
static_assert(kSWave == kFThreads / 64 - 1, "wave roles");
constexpr int kPktF = 188;
constexpr int kTilePkts = 128;                    // 32 x 4 packets
constexpr int kTileBytes = kTilePkts * kPktF;     // 24,064 = 16 x 1,504
constexpr int kTileBlocks = kTileBytes / 16;      // 1,504 AES blocks
constexpr int kFBlk = 3;                          // blocks per lane (independent chains)
constexpr int kWaveBlk = 64 * kFBlk;              // blocks per decrypt wave and tile
static_assert(kDWaves * kWaveBlk >= kTileBlocks && kTileBytes % 16 == 0 && kTilePkts % 4 == 0, "tile shape");
constexpr int kLanePk = 2;                        // packets per control lane (consecutive)
static_assert(64 * kLanePk >= kTilePkts, "a control wave covers the tile");
constexpr int kXIters = 6;                        // copy-out: 5 waves x 5 packets x 6 >= 128
static_assert(kXWaves * 5 * kXIters >= kTilePkts, "copy-out covers the tile");
constexpr int kTabDwords = 256 * 64;              // 64 KiB: [Td0 | Td2] rows
constexpr int kStages = 3;                        // plaintext stages
constexpr int kStageDwords = kTileBytes / 4 + 8;  // + slack for the funnel reads past a packet
constexpr int kRing = 8;                          // scheduled jobs in flight
constexpr int kPlanRing = 4;                      // copy plans in flight (see the copy-out role)
constexpr int kPsiPkts = 64;                      // PAT / PMT window (runtime/ts.cpp)
constexpr int kClassesF = 3;
constexpr int kInfoF = 24;
// info slots / status bits (runtime/ts.hpp, ts_demux.hip)
constexpr int kStatusF = 0, kPmtPidF = 1, kVideoPidF = 2, kNumPacketsF = 5, kBytes0F = 6, kPes0F = 9,
              kVideoTypeF = 12, kAudioTypeF = 13, kPayloadBytesF = 14, kFirstPtsF = 16, kLastPtsF = 19,
              kAudioEsOffsetF = 22, kId3EsOffsetF = 23;
constexpr uint32_t kBadSyncF = 1, kNoPatF = 2, kNoPmtF = 4, kPesOverflowF = 8, kPesHeaderErrorF = 16,
                   kBadLengthF = 32;
constexpr uint64_t kAgg = 1ull << 62, kIncl = 2ull << 62;
constexpr uint32_t kSpinLimit = 1u << 22;  // ~0.1 s of polling: only a broken hand-off gets here

// One scheduled tile.  Written by the scheduler wave, read by the decrypt and control
// waves; `plen` is filled in by the decrypt lane that holds the segment's last block.
struct Job {
  int64_t t;         // ticket (global tile index); -1 = no more work
  int64_t tile0;     // ticket of the segment's first tile
  int64_t blk0;      // the tile's first 16-byte source block, absolute in a.src
  int64_t seg_blk0;  // the segment's first source block (its CBC input is the IV)
  int64_t last_blk;  // the segment's last block (encrypted), else -1
  int64_t plen;      // -2: not the segment's last tile; -1: bad padding; else plaintext length
  int64_t es_off, es_cap;  // the segment's ES regions
  int32_t seg, tile, ntile, enc, nb;  // nb: source blocks in the tile (clear: rounded up)
  int32_t pid[3];    // video / audio / id3 PID of the segment, -1 = absent
};

// Per stage, control -> copy-out: where the tile's payloads go (the per-packet in-tile
// offsets are written at parse time; the look-back adds the class bases here).
struct CopyPlan {
  int64_t es_off, cap;
  int64_t base[3];  // per class: ES bytes of the segment's tiles before this one
  int32_t live;     // 0: no more tiles
  uint32_t tag;     // tile + 1 once the plan is in place
};

#define SELF(k) (0x0c020000u | ((4u + (k)) << 8))
#define LDSW(addr) (*reinterpret_cast<const uint32_t*>(s_bytes + (addr)))
#define XOR3F(a, b, c) __builtin_amdgcn_bitop3_b32((a), (b), (c), 0x96)
#define ROT(v, r) __builtin_amdgcn_alignbit((v), (v), 32u - (r))
// T-table address of byte k of w in the Td0 (td0_base) or Td2 (td2_base) half-row
#define TDA(w, base, k) __builtin_amdgcn_perm((w), (base), SELF(k))

using demux::dpp_scan;
using demux::dpp_sum;
using demux::gload;
using demux::gstore;
using demux::parse_pkt;
using demux::Pkt;

__device__ __forceinline__ int64_t pkcs7_len_f(uint4 p, int64_t nbytes) {
  const uint32_t pad = p.w >> 24;
  if (pad < 1 || pad > 16) return -1;
  const uint32_t w[4] = {p.x, p.y, p.z, p.w};
  bool ok = true;
#pragma unroll
  for (int b = 0; b < 16; ++b) {
    const uint32_t byte = (w[b >> 2] >> (8 * (b & 3))) & 0xff;
    if (b >= 16 - static_cast<int>(pad) && byte != pad) ok = false;
  }
  return ok ? nbytes - static_cast<int64_t>(pad) : -1;
}

__device__ __forceinline__ int64_t uniform64f(int64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(static_cast<uint64_t>(v) >> 32));
  return static_cast<int64_t>((static_cast<uint64_t>(hi) << 32) | lo);
}
__device__ __forceinline__ int uniform32f(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Intra-workgroup hand-off on a monotonic LDS counter.  signal / publish: the wave's LDS
// writes land first (lgkmcnt(0) only: a workgroup-scope release fence would also wait for
// vmcnt(0) — the decrypt waves' next-tile prefetch, the control and copy-out waves' global
// stores — none of which the consumer reads); wait: the whole wave polls (a broadcast read)
// until the count reaches `v`.  LDS serves a workgroup's waves from one in-order pipeline.
__device__ __forceinline__ void lds_release() {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_s_waitcnt(0xC07F);  // gfx9 encoding: vmcnt 63, expcnt 7, lgkmcnt 0
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}
__device__ __forceinline__ void lds_signal(uint32_t* c, int lane) {
  lds_release();
  if (lane == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_publish(uint32_t* c, uint32_t v, int lane) {
  lds_release();
  if (lane == 0) __hip_atomic_store(c, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// The poll is one lane's read: a full-wave broadcast read costs the LDS the cycles of a
// 64-lane instruction, and six waves polling every ~100 cycles would take a tenth of the
// bandwidth the decrypt waves live on.
__device__ __forceinline__ void lds_wait(uint32_t* c, uint32_t v, unsigned int* timeout, int lane) {
  uint32_t spins = 0;
  for (;;) {
    uint32_t x = 0;
    if (lane == 0) x = __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(x)) >= v) break;
    if (++spins > kSpinLimit) {
      if (lane == 0) atomicOr(timeout, 2u);
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// diagnostics: the kProf instance of the fused kernel (launched when a.prof != null) keeps
// shader-clock per-role timers; the production instance compiles them out
template <bool kProf>
__device__ __forceinline__ uint64_t pclk() {
  return kProf ? __builtin_readcyclecounter() : 0;
}
template <bool kProf>
__device__ __forceinline__ void pflush(const TransmuxArgs& a, int slot0, const uint64_t* v, int n, int lane) {
  if (kProf && lane == 0)
    for (int k = 0; k < n; ++k) a.prof[blockIdx.x * 16 + slot0 + k] = v[k];
}

// PAT / PMT over the first `scan` packets of `s` (the host oracle's rules, runtime/ts.cpp):
// the first PAT's first program, then the first PMT section of that PID.  `pmt_found`:
// both found, so more packets cannot change the answer.
struct Psi {
  int pmt_pid, vpid, apid, ipid, vtype, atype;
  bool pmt_found;
};
__device__ Psi psi_scan(const uint8_t* s, int scan) {
  Psi r{-1, -1, -1, -1, 0, 0, false};
  for (int q0 = 0; q0 < scan && r.pmt_pid < 0; ++q0) {
    const uint8_t* p = s + q0 * kPktF;
    if (p[0] != 0x47) continue;
    const int pid = ((p[1] & 0x1f) << 8) | p[2];
    if (pid != 0 || !(p[1] & 0x40)) continue;
    const int afc = (p[3] >> 4) & 3;
    int ps = 4 + ((afc & 2) ? 1 + p[4] : 0);
    if (!(afc & 1) || ps >= kPktF) continue;
    ps += 1 + p[ps];
    if (ps + 8 > kPktF || p[ps] != 0x00) continue;
    const int sl = ((p[ps + 1] & 0x0f) << 8) | p[ps + 2];
    const int end = ps + 3 + sl - 4 < kPktF ? ps + 3 + sl - 4 : kPktF;
    for (int q = ps + 8; q + 4 <= end; q += 4) {
      const int prog = (p[q] << 8) | p[q + 1];
      if (prog != 0) {
        r.pmt_pid = ((p[q + 2] & 0x1f) << 8) | p[q + 3];
        break;
      }
    }
  }
  for (int q0 = 0; q0 < scan && r.pmt_pid >= 0 && !r.pmt_found; ++q0) {
    const uint8_t* p = s + q0 * kPktF;
    if (p[0] != 0x47) continue;
    const int pid = ((p[1] & 0x1f) << 8) | p[2];
    if (pid != r.pmt_pid || !(p[1] & 0x40)) continue;
    const int afc = (p[3] >> 4) & 3;
    int ps = 4 + ((afc & 2) ? 1 + p[4] : 0);
    if (!(afc & 1) || ps >= kPktF) continue;
    ps += 1 + p[ps];
    if (ps + 12 > kPktF || p[ps] != 0x02) continue;
    r.pmt_found = true;
    const int sl = ((p[ps + 1] & 0x0f) << 8) | p[ps + 2];
    const int end = ps + 3 + sl - 4 < kPktF ? ps + 3 + sl - 4 : kPktF;
    const int pil = ((p[ps + 10] & 0x0f) << 8) | p[ps + 11];
    for (int q = ps + 12 + pil; q + 5 <= end;) {
      const int type = p[q];
      const int epid = ((p[q + 1] & 0x1f) << 8) | p[q + 2];
      const int eil = ((p[q + 3] & 0x0f) << 8) | p[q + 4];
      if ((type == 0x1B || type == 0x24) && r.vpid < 0) {
        r.vpid = epid;
        r.vtype = type;
      } else if ((type == 0x0F || type == 0x03 || type == 0x04) && r.apid < 0) {
        r.apid = epid;
        r.atype = type;
      } else if (type == 0x15 && r.ipid < 0) {
        r.ipid = epid;
      }
      q += 5 + eil;
    }
  }
  return r;
}

}  // namespace

// One wave per segment: the elementary PIDs (and the PAT / PMT status bits) before the
// fused kernel starts.  Decrypts the segment's first packets four at a time (47 blocks, one
// per lane, T-tables in LDS) until PAT and PMT are both found or the 64-packet window is
// exhausted — usually after the first four packets.
__global__ __launch_bounds__(64) void transmux_psi_kernel(TransmuxArgs a) {
  __shared__ uint32_t s_td[256];
  __shared__ uint8_t s_is[256];
  __shared__ __attribute__((aligned(16))) uint32_t s_p[kPsiPkts * kPktF / 4 + 4];
  __shared__ int s_done;
  __shared__ int64_t s_plen;
  const int seg = blockIdx.x, lane = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    s_td[lane + 64 * k] = a.tdl[lane + 64 * k];
    s_is[lane + 64 * k] = a.isb[lane + 64 * k];
  }
  const int64_t slen = a.src_len[seg];
  const bool enc = a.enc[seg] != 0;
  const uint4* cs = reinterpret_cast<const uint4*>(a.src + a.src_off[seg]);
  const uint32_t* rk = a.drk + static_cast<int64_t>(seg) * 44;
  const uint4 iv = reinterpret_cast<const uint4*>(a.ivw)[seg];
  __syncthreads();
  auto decrypt = [&](int64_t b) -> uint4 {  // plaintext of block b (CBC)
    const uint4 c = cs[b];
    uint32_t s0 = c.x ^ rk[0], s1 = c.y ^ rk[1], s2 = c.z ^ rk[2], s3 = c.w ^ rk[3];
    for (int r = 1; r < 10; ++r) {
      const uint32_t* k = rk + 4 * r;
      const uint32_t n0 = s_td[s0 & 0xff] ^ ROT(s_td[(s3 >> 8) & 0xff], 8) ^ ROT(s_td[(s2 >> 16) & 0xff], 16) ^
                          ROT(s_td[s1 >> 24], 24) ^ k[0];
      const uint32_t n1 = s_td[s1 & 0xff] ^ ROT(s_td[(s0 >> 8) & 0xff], 8) ^ ROT(s_td[(s3 >> 16) & 0xff], 16) ^
                          ROT(s_td[s2 >> 24], 24) ^ k[1];
      const uint32_t n2 = s_td[s2 & 0xff] ^ ROT(s_td[(s1 >> 8) & 0xff], 8) ^ ROT(s_td[(s0 >> 16) & 0xff], 16) ^
                          ROT(s_td[s3 >> 24], 24) ^ k[2];
      const uint32_t n3 = s_td[s3 & 0xff] ^ ROT(s_td[(s2 >> 8) & 0xff], 8) ^ ROT(s_td[(s1 >> 16) & 0xff], 16) ^
                          ROT(s_td[s0 >> 24], 24) ^ k[3];
      s0 = n0; s1 = n1; s2 = n2; s3 = n3;
    }
    const uint4 pv = b == 0 ? iv : cs[b - 1];
    auto fin = [&](uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3) {
      return static_cast<uint32_t>(s_is[x0 & 0xff]) | (static_cast<uint32_t>(s_is[(x1 >> 8) & 0xff]) << 8) |
             (static_cast<uint32_t>(s_is[(x2 >> 16) & 0xff]) << 16) | (static_cast<uint32_t>(s_is[x3 >> 24]) << 24);
    };
    return make_uint4(fin(s0, s3, s2, s1) ^ rk[40] ^ pv.x, fin(s1, s0, s3, s2) ^ rk[41] ^ pv.y,
                      fin(s2, s1, s0, s3) ^ rk[42] ^ pv.z, fin(s3, s2, s1, s0) ^ rk[43] ^ pv.w);
  };
  // plaintext length: only a segment shorter than the window needs its padding checked here
  if (lane == 0) {
    int64_t n = slen;
    if (enc && slen < (kPsiPkts + 1) * kPktF) n = slen >= 16 ? pkcs7_len_f(decrypt(slen / 16 - 1), slen) : -1;
    s_plen = n;
    s_done = 0;
  }
  __syncthreads();
  const int64_t plen = s_plen;
  const int64_t npk = plen < 0 ? 0 : plen / kPktF;
  const int scan = static_cast<int>(npk < kPsiPkts ? npk : kPsiPkts);
  const uint8_t* sb = reinterpret_cast<const uint8_t*>(s_p);
  Psi r{-1, -1, -1, -1, 0, 0, false};
  const int64_t nblk_src = (slen + 15) / 16;
  for (int c = 0; 4 * c < scan; ++c) {
    const int64_t b = 47 * static_cast<int64_t>(c) + lane;
    if (lane < 47 && b < nblk_src) reinterpret_cast<uint4*>(s_p)[b] = enc ? decrypt(b) : cs[b];
    __syncthreads();
    if (lane == 0) {
      const int have = 4 * (c + 1) < scan ? 4 * (c + 1) : scan;
      r = psi_scan(sb, have);
      s_done = r.pmt_found ? 1 : 0;
    }
    __syncthreads();
    if (s_done) break;
  }
  if (lane == 0) {
    int64_t* inf = a.info + static_cast<int64_t>(seg) * kInfoF;
    uint32_t status = 0;
    if (r.pmt_pid < 0) status |= kNoPatF;
    if (r.pmt_pid >= 0 && !r.pmt_found) status |= kNoPmtF;
    inf[kStatusF] = status;
    inf[kPmtPidF] = r.pmt_pid;
    inf[kVideoPidF] = r.vpid;
    inf[kVideoPidF + 1] = r.apid;
    inf[kVideoPidF + 2] = r.ipid;
    inf[kVideoTypeF] = r.vtype;
    inf[kAudioTypeF] = r.atype;
    // PIDs are 13-bit: 16-bit fields, 0xffff = absent, bit 63 = ready
    auto f = [](int v) { return static_cast<uint64_t>(v < 0 ? 0xffff : v); };
    a.psi[2 * static_cast<int64_t>(seg)] = (1ull << 63) | f(r.vpid) | (f(r.apid) << 16) | (f(r.ipid) << 32);
  }
}

// The fused kernel's LDS as ONE object, so the table image sits at LDS address 0: the
// v_perm that extracts a state byte then IS the ds_read address (no add per lookup).
struct FusedLds {
  uint32_t tab[kTabDwords];                 // [Td0 | Td2] rows
  uint32_t pk[kStages][kStageDwords];       // plaintext stages
  Job job[kRing];
  CopyPlan plan[kPlanRing];                 // control -> copy-out (tag = tile + 1): class bases
  uint32_t meta[kStages][kTilePkts];        // per packet: class | ps << 2 | len << 10
  int32_t dst[kStages][kTilePkts];          // per packet: in-tile offset in its class
  uint32_t ptag[kStages];                   // ptag[i % kStages] == i + 1: tile i is parsed
  uint32_t plive[kStages];                  // 0 with the tag: no more tiles
  uint32_t seq[kRing];                      // seq[j % kRing] == j + 1: job j is staged
  uint32_t jdone[kRing];                    // jdone[j % kRing] == j + 1: its control wave is done
  uint32_t ddone[kStages];                  // decrypt waves' completions per stage (not in step)
  uint32_t xread[kStages];                  // copy-out waves that have read the stage's payloads
};
static_assert(sizeof(FusedLds) <= 160 * 1024, "fused kernel LDS");

template <bool kProf>
__global__ __launch_bounds__(kFThreads, 1) void transmux_fused_kernel(TransmuxArgs a) {
  __shared__ __attribute__((aligned(16))) FusedLds L;
  const int tid = threadIdx.x;
  // wave-uniform role index (readfirstlane: the compiler then keeps per-wave values in SGPRs
  // and branches on roles without exec masking)
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  {  // table image; thread t fills dwords t + 1024 k: row d >> 6 = [Td0 | Td2]
    uint32_t v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int d = tid + k * kFThreads;
      const uint32_t td = a.tdl[d >> 6];
      v[k] = (d & 32) ? ROT(td, 16) : td;
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) L.tab[tid + k * kFThreads] = v[k];
    if (tid < kRing) {
      L.seq[tid] = 0;
      L.jdone[tid] = 0;
    }
    if (tid < kStages) {
      L.ddone[tid] = 0;
      L.xread[tid] = 0;
      L.ptag[tid] = 0;
    }
    if (tid < kPlanRing) L.plan[tid].tag = 0;
  }
  __syncthreads();  // the only workgroup barrier: from here on the roles run free
  const uint8_t* s_bytes = reinterpret_cast<const uint8_t*>(L.tab);
  // the latency-bound roles issue ahead of the decrypt waves: their dependent LDS accesses
  // would otherwise wait behind a saturated stream of AES table reads
  if (wave >= kCWave0 && !(a.flags & 1)) __builtin_amdgcn_s_setprio(3);

  if (wave == kSWave) {
    // ================================================================ SCHEDULER
    uint64_t ps[2] = {0, 0};  // diagnostics: waiting for a free ring entry, staging a job
    for (uint32_t j = 0;; ++j) {
      const uint64_t c0 = pclk<kProf>();
      if (j >= kRing) lds_wait(&L.jdone[j % kRing], j - kRing + 1, a.timeout, lane);  // entry free
      const uint64_t c1 = pclk<kProf>();
      ps[0] += c1 - c0;
      unsigned int tk = 0;
      if (lane == 0) tk = atomicAdd(a.ticket, 1u);
      const int64_t t = static_cast<int64_t>(__builtin_amdgcn_readfirstlane(tk));
      if (t >= a.total_tiles) {
        // one end marker per control wave (each walks its own residue of job indices); the
        // first (-1) also releases the copy-out waves
        for (uint32_t e = 0; e < static_cast<uint32_t>(kCWaves); ++e) {
          const uint32_t jj = j + e;
          if (jj >= kRing) lds_wait(&L.jdone[jj % kRing], jj - kRing + 1, a.timeout, lane);
          if (lane == 0) L.job[jj % kRing].t = e == 0 ? -1 : -2;
          lds_publish(&L.seq[jj % kRing], jj + 1, lane);
        }
        break;
      }
      Job& J = L.job[j % kRing];
      const int seg = find_seg_wave(a.tile_prefix, a.nseg, t);
      const int64_t tile0 = a.tile_prefix[seg];
      const int tile = static_cast<int>(t - tile0);
      const int ntile = static_cast<int>(a.tile_prefix[seg + 1] - tile0);
      const int64_t slen = a.src_len[seg];
      const int enc = a.enc[seg] != 0;
      const int64_t tbyte0 = static_cast<int64_t>(tile) * kTileBytes;
      const int64_t tbytes = slen - tbyte0 < kTileBytes ? slen - tbyte0 : kTileBytes;
      const int64_t sb0 = a.src_off[seg] / 16;  // segments are 16-byte aligned in the batch
      const uint64_t g = a.psi[2 * static_cast<int64_t>(seg)];  // transmux_psi_kernel's PIDs
      if (lane < 3) {
        const uint32_t f = static_cast<uint32_t>(g >> (16 * lane)) & 0xffff;
        J.pid[lane] = f == 0xffff ? -1 : static_cast<int32_t>(f);
      }
      if (lane == 0) {
        J.t = t;
        J.tile0 = tile0;
        J.blk0 = sb0 + tbyte0 / 16;
        J.seg_blk0 = sb0;
        J.last_blk = enc ? sb0 + slen / 16 - 1 : -1;
        J.plen = (!enc && tile == ntile - 1) ? slen : -2;
        J.seg = seg;
        J.tile = tile;
        J.ntile = ntile;
        J.enc = enc;
        J.nb = static_cast<int>(enc ? tbytes / 16 : (tbytes + 15) / 16);
        J.es_off = a.es_off[seg];
        J.es_cap = a.es_cap[seg];
      }
      lds_publish(&L.seq[j % kRing], j + 1, lane);
      ps[1] += pclk<kProf>() - c1;
    }
    pflush<kProf>(a, 12, ps, 2, lane);
    return;
  }

  if (wave < kDWaves) {
    // ================================================================ DECRYPT
    // Everything a tile needs is in registers before its first round: the ciphertext and the
    // job's geometry were fetched during the previous tile, the round keys come by scalar
    // loads, and the CBC chaining input is the ciphertext of the lane below (DPP wave_shr:1;
    // one prefetched block per wave for its first lane) — no memory round trip at a tile
    // boundary, where all decrypt waves would otherwise stall together and idle the LDS.
    const uint32_t l4 = static_cast<uint32_t>(tid & 31) << 2;
    const uint32_t td0_base = l4, td2_base = 128u | l4;
    const uint4* src4 = reinterpret_cast<const uint4*>(a.src);
    const int wb0 = wave * kWaveBlk;  // the wave's first block in a tile
    lds_wait(&L.seq[0], 1, a.timeout, lane);
    if (uniform64f(L.job[0].t) < 0) return;
    // the current job's geometry (uniform)
    int64_t b0 = uniform64f(L.job[0].blk0), sb0 = uniform64f(L.job[0].seg_blk0), lastb = uniform64f(L.job[0].last_blk);
    int nb = uniform32f(L.job[0].nb), seg = uniform32f(L.job[0].seg);
    bool enc = uniform32f(L.job[0].enc) != 0;
    uint4 cc[kFBlk];  // this tile's source blocks
    uint4 cf;         // the block before the wave's first block (CBC input of its lane 0)
    {
#pragma unroll
      for (int j = 0; j < kFBlk; ++j) {
        const int lb = wb0 + 64 * j + lane;
        cc[j] = lb < nb ? src4[b0 + lb] : make_uint4(0, 0, 0, 0);
      }
      cf = (wb0 < nb && b0 + wb0 > sb0) ? src4[b0 + wb0 - 1] : make_uint4(0, 0, 0, 0);
    }
    uint64_t pd[4] = {0, 0, 0, 0};  // diagnostics: next-job wait, stage wait, decrypt, tiles
    for (uint32_t i = 0;; ++i) {
      const uint64_t c0 = pclk<kProf>();
      // the next job: geometry now, source blocks streaming in under this tile's rounds
      lds_wait(&L.seq[(i + 1) % kRing], i + 2, a.timeout, lane);
      const Job& N = L.job[(i + 1) % kRing];
      const bool has_next = uniform64f(N.t) >= 0;
      int64_t nb0 = 0, nsb0 = 0, nlastb = -1;
      int nnb = 0, nseg = 0;
      bool nenc = false;
      if (has_next) {
        nb0 = uniform64f(N.blk0);
        nsb0 = uniform64f(N.seg_blk0);
        nlastb = uniform64f(N.last_blk);
        nnb = uniform32f(N.nb);
        nseg = uniform32f(N.seg);
        nenc = uniform32f(N.enc) != 0;
      }
      uint4 cn[kFBlk], cnf;
#pragma unroll
      for (int j = 0; j < kFBlk; ++j) {
        const int lb = wb0 + 64 * j + lane;
        cn[j] = lb < nnb ? src4[nb0 + lb] : make_uint4(0, 0, 0, 0);
      }
      cnf = (wb0 < nnb && nb0 + wb0 > nsb0) ? src4[nb0 + wb0 - 1] : make_uint4(0, 0, 0, 0);
      const uint64_t c1 = pclk<kProf>();
      // stage i % kStages is free once every copy-out wave has read tile i - kStages
      if (i >= kStages) lds_wait(&L.xread[i % kStages], kXWaves * (i / kStages), a.timeout, lane);
      const uint64_t c2 = pclk<kProf>();
      pd[0] += c1 - c0;
      pd[1] += c2 - c1;
      uint4* stg = reinterpret_cast<uint4*>(L.pk[i % kStages]);
      if (enc) {
        const uint32_t* rk = a.drk_rot + static_cast<int64_t>(seg) * 44;  // uniform: scalar loads
        {  // CBC chaining input: the ciphertext block below, i.e. lane - 1's (wave_shr:1); lane 0
           // takes lane 63 of the chain before (readlane) or, in chain 0, the prefetched block.
           // Parked in the block's own stage slot until the last round (fewer VGPRs across
           // the rounds; each lane reads back only what it wrote).
          const uint4 iv = reinterpret_cast<const uint4*>(a.ivw)[seg];
#pragma unroll
          for (int j = 0; j < kFBlk; ++j) {
            uint32_t bx = cf.x, by = cf.y, bz = cf.z, bw = cf.w;
            if (j > 0) {
              bx = __builtin_amdgcn_readlane(cc[j - 1].x, 63);
              by = __builtin_amdgcn_readlane(cc[j - 1].y, 63);
              bz = __builtin_amdgcn_readlane(cc[j - 1].z, 63);
              bw = __builtin_amdgcn_readlane(cc[j - 1].w, 63);
            }
            uint4 pv;
            pv.x = __builtin_amdgcn_update_dpp(bx, cc[j].x, 0x138, 0xf, 0xf, false);  // wave_shr:1
            pv.y = __builtin_amdgcn_update_dpp(by, cc[j].y, 0x138, 0xf, 0xf, false);
            pv.z = __builtin_amdgcn_update_dpp(bz, cc[j].z, 0x138, 0xf, 0xf, false);
            pv.w = __builtin_amdgcn_update_dpp(bw, cc[j].w, 0x138, 0xf, 0xf, false);
            const int lb = wb0 + 64 * j + lane;
            if (b0 + lb == sb0) pv = iv;  // the segment's first block
            if (lb < nb) stg[lb] = pv;
          }
        }
        uint32_t st[kFBlk][4];
#pragma unroll
        for (int j = 0; j < kFBlk; ++j) {
          st[j][0] = cc[j].x ^ rk[0]; st[j][1] = cc[j].y ^ rk[1];
          st[j][2] = cc[j].z ^ rk[2]; st[j][3] = cc[j].w ^ rk[3];
        }
        // rounds 1..9: chain j's 16 LDS reads are issued before chain j-1's XORs consume theirs
#pragma unroll
        for (int r = 1; r < 10; ++r) {
          const uint32_t* k = rk + 4 * r;  // pre-rotated by 24
          uint32_t v[2][16];
#pragma unroll
          for (int j = 0; j <= kFBlk; ++j) {
            if (j < kFBlk) {
              const uint32_t* sj = st[j];
              uint32_t* o = v[j & 1];
              // column c: Td0[s[c].b0], Td2[s[c+2].b2] | Td0[s[c+3].b1], Td2[s[c+1].b3] (rotated)
              const uint32_t ad[16] = {
                  TDA(sj[0], td0_base, 0), TDA(sj[2], td2_base, 2), TDA(sj[3], td0_base, 1), TDA(sj[1], td2_base, 3),
                  TDA(sj[1], td0_base, 0), TDA(sj[3], td2_base, 2), TDA(sj[0], td0_base, 1), TDA(sj[2], td2_base, 3),
                  TDA(sj[2], td0_base, 0), TDA(sj[0], td2_base, 2), TDA(sj[1], td0_base, 1), TDA(sj[3], td2_base, 3),
                  TDA(sj[3], td0_base, 0), TDA(sj[1], td2_base, 2), TDA(sj[2], td0_base, 1), TDA(sj[0], td2_base, 3)};
#pragma unroll
              for (int q = 0; q < 16; ++q) o[q] = LDSW(ad[q]);
            }
            if (j > 0) {
              uint32_t* sj = st[j - 1];
              const uint32_t* x = v[(j - 1) & 1];
#pragma unroll
              for (int c = 0; c < 4; ++c)
                sj[c] = XOR3F(x[4 * c], x[4 * c + 1], ROT(XOR3F(x[4 * c + 2], x[4 * c + 3], k[c]), 8));
            }
          }
        }
        const uint32_t* kf = rk + 40;
        uint4 pvs[kFBlk];
#pragma unroll
        for (int j = 0; j < kFBlk; ++j) {
          const int lb = wb0 + 64 * j + lane;
          pvs[j] = stg[lb < nb ? lb : 0];
        }
        // last round: InvSbox[x] = byte-XOR of Td0[x].  For output word c, byte j comes from
        // T_j = Td0[x_j]; with U_j = T_j ^ rot16(T_j), byte j of the result is
        // U_j.b[j] ^ U_j.b[j-1]: four v_perm gather those, three XORs fold them.
#pragma unroll
        for (int j = 0; j < kFBlk; ++j) {
          const uint32_t* sj = st[j];
          uint32_t T[16];
          const uint32_t ad[16] = {TDA(sj[0], td0_base, 0), TDA(sj[3], td0_base, 1), TDA(sj[2], td0_base, 2), TDA(sj[1], td0_base, 3),
                                   TDA(sj[1], td0_base, 0), TDA(sj[0], td0_base, 1), TDA(sj[3], td0_base, 2), TDA(sj[2], td0_base, 3),
                                   TDA(sj[2], td0_base, 0), TDA(sj[1], td0_base, 1), TDA(sj[0], td0_base, 2), TDA(sj[3], td0_base, 3),
                                   TDA(sj[3], td0_base, 0), TDA(sj[2], td0_base, 1), TDA(sj[1], td0_base, 2), TDA(sj[0], td0_base, 3)};
#pragma unroll
          for (int q = 0; q < 16; ++q) T[q] = LDSW(ad[q]);
          uint32_t o[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const uint32_t u0 = T[4 * c] ^ ROT(T[4 * c], 16), u1 = T[4 * c + 1] ^ ROT(T[4 * c + 1], 16),
                           u2 = T[4 * c + 2] ^ ROT(T[4 * c + 2], 16), u3 = T[4 * c + 3] ^ ROT(T[4 * c + 3], 16);
            const uint32_t p01 = __builtin_amdgcn_perm(u1, u0, 0x0c0c0500u);  // [u0.b0, u1.b1, 0, 0]
            const uint32_t p23 = __builtin_amdgcn_perm(u3, u2, 0x07020c0cu);  // [0, 0, u2.b2, u3.b3]
            const uint32_t q01 = __builtin_amdgcn_perm(u1, u0, 0x0c0c0403u);  // [u0.b3, u1.b0, 0, 0]
            const uint32_t q23 = __builtin_amdgcn_perm(u3, u2, 0x06010c0cu);  // [0, 0, u2.b1, u3.b2]
            o[c] = XOR3F(XOR3F(p01, p23, q01), q23, kf[c]);
          }
          const uint4 pv = pvs[j];
          const int lb = wb0 + 64 * j + lane;
          const int64_t b = b0 + lb;
          const uint4 out = make_uint4(o[0] ^ pv.x, o[1] ^ pv.y, o[2] ^ pv.z, o[3] ^ pv.w);
          if (lb < nb) {
            stg[lb] = out;
            if (b == lastb) L.job[i % kRing].plen = pkcs7_len_f(out, (lastb - sb0 + 1) * 16);  // PKCS#7
          }
        }
      } else {  // clear segment: the tile's bytes into LDS (16 B per lane; the source has slack)
#pragma unroll
        for (int j = 0; j < kFBlk; ++j) {
          const int lb = wb0 + 64 * j + lane;
          if (lb < nb) stg[lb] = cc[j];
        }
      }
      lds_signal(&L.ddone[i % kStages], lane);
      pd[2] += pclk<kProf>() - c2;
      pd[3] += 1;
      if (!has_next) {
        if (wave == 0) pflush<kProf>(a, 8, pd, 4, lane);
        return;
      }
#pragma unroll
      for (int j = 0; j < kFBlk; ++j) cc[j] = cn[j];
      cf = cnf;
      b0 = nb0;
      sb0 = nsb0;
      lastb = nlastb;
      nb = nnb;
      seg = nseg;
      enc = nenc;
    }
  }

  if (wave >= kXWave0) {
    // ================================================================ COPY-OUT
    // Read early, store late: as soon as the control wave has parsed tile i, every payload
    // word this wave will write is read into registers and the stage is released to the
    // decrypt waves; the stores wait for the tile's class bases (the look-back) — so the
    // look-back latency is never on the path that recycles a stage.
    // Five packets per wave iteration: a 12-lane group moves one payload (<= 184 B = 46
    // dwords); lane `sub` writes destination dwords 4sub..4sub+3 with ONE dwordx4 buffer
    // store, funnelled (v_alignbyte) out of a 6-dword source window that covers every
    // destination alignment; byte stores for the <= 3 + 3 unaligned head / tail bytes.
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    const int xw = wave - kXWave0;
    const int grp = lane / 12, sub = lane - 12 * grp;  // groups 0..4; lanes 60..63 idle
    const int k0s = 4 * sub;
    uint64_t px[2] = {0, 0};  // diagnostics: parse wait, plan wait + copy
    for (uint32_t i = 0;; ++i) {
      const uint64_t c0 = pclk<kProf>();
      const int st = i % kStages;
      lds_wait(&L.ptag[st], i + 1, a.timeout, lane);
      if (!uniform32f(L.plive[st])) break;
      const uint64_t c1 = pclk<kProf>();
      px[0] += c1 - c0;
      const uint8_t* stage = reinterpret_cast<const uint8_t*>(L.pk[st]);
      const uint32_t* stagew = L.pk[st];
      uint32_t win[kXIters][6], mt[kXIters], hw[kXIters], tw[kXIters];
      int32_t dd[kXIters];
      if (a.diag == 0) {
#pragma unroll
        for (int it = 0; it < kXIters; ++it) {
          const int j = it * (kXWaves * 5) + xw * 5 + grp;
          const bool ok = grp < 5 && j < kTilePkts;
          mt[it] = ok ? L.meta[st][j] : 3u;
          dd[it] = ok ? L.dst[st][j] : 0;
        }
#pragma unroll
        for (int it = 0; it < kXIters; ++it) {
          const int j = it * (kXWaves * 5) + xw * 5 + grp;
          const bool ok = grp < 5 && j < kTilePkts;
          const uint32_t mm = mt[it];
          const int jc = mm & 3, jps = (mm >> 2) & 0xff, jlen = jc < 3 ? static_cast<int>((mm >> 10) & 0xff) : 0;
          const int s0 = (ok ? j : 0) * kPktF;
          const int s = s0 + (jlen ? jps : 0);  // LDS byte offset of the payload
          int aa = s + 4 * k0s;                 // the window: source bytes [4 k0s, 4 k0s + 20) of the payload
          aa = aa < s0 + kPktF - 4 ? aa : s0 + kPktF - 4;  // clamped: the lane may have no body
          const uint32_t* w = stagew + (aa >> 2);
#pragma unroll
          for (int m = 0; m < 6; ++m) win[it][m] = w[m];
          // payload bytes 0..3 and the last three (+1), each as one funnelled dword
          const int te = s + jlen - 3;  // may start in the packet header: jlen < 3 keeps the same indexing
          const uint32_t* h = stagew + (s >> 2);
          const uint32_t* e = stagew + (te >> 2);
          hw[it] = __builtin_amdgcn_alignbyte(h[1], h[0], static_cast<uint32_t>(s & 3));
          tw[it] = __builtin_amdgcn_alignbyte(e[1], e[0], static_cast<uint32_t>(te & 3));
        }
      }
      lds_signal(&L.xread[st], lane);  // registers hold the tile: the stage goes back to decrypt
      // the tile's class bases (plan ring: the slot is rewritten only after this wave has
      // stored this tile — planning tile i + kPlanRing needs the stage this wave frees next)
      CopyPlan& P = L.plan[i % kPlanRing];
      lds_wait(&P.tag, i + 1, a.timeout, lane);
      if (a.diag == 0) {
        const int64_t es_off = uniform64f(P.es_off), cap = uniform64f(P.cap);
        const int64_t base0 = uniform64f(P.base[0]), base1 = uniform64f(P.base[1]), base2 = uniform64f(P.base[2]);
        uint8_t* ebase = a.es + es_off;
        const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(ebase, 0, 0x7fffffff, 0x00020000);
#pragma unroll
        for (int it = 0; it < kXIters; ++it) {
          const uint32_t mm = mt[it];
          const int jc = mm & 3, jps = (mm >> 2) & 0xff, jlen = jc < 3 ? static_cast<int>((mm >> 10) & 0xff) : 0;
          if (grp >= 5 || jlen == 0) continue;
          const int64_t cb = jc == 0 ? base0 : jc == 1 ? base1 : base2;
          const int64_t dst64 = jc * cap + cb + dd[it];  // the class's region
          uint8_t* d = ebase + dst64;
          const int head0 = static_cast<int>((4 - (reinterpret_cast<uintptr_t>(d) & 3)) & 3);
          const int head = head0 < jlen ? head0 : jlen;
          const int body = (jlen - head) >> 2;
          const int tail = jlen - head - 4 * body;
          if (sub < head) d[sub] = static_cast<uint8_t>(hw[it] >> (8 * sub));
          if (k0s < body) {
            // destination dword 4sub + m = payload bytes head + 16 sub + 4m: in the window at
            // delta = (window start misalignment) + head
            const int sa = jps & 3;  // the payload start's misalignment in the stage (packets are dword aligned)
            const int delta = sa + head;          // 0..6
            const uint32_t sh = static_cast<uint32_t>(delta & 3);
            const bool hi = delta >= 4;
            const uint32_t y0 = hi ? win[it][1] : win[it][0], y1 = hi ? win[it][2] : win[it][1],
                           y2 = hi ? win[it][3] : win[it][2], y3 = hi ? win[it][4] : win[it][3],
                           y4 = hi ? win[it][5] : win[it][4];
            const uint32_t o0 = __builtin_amdgcn_alignbyte(y1, y0, sh), o1 = __builtin_amdgcn_alignbyte(y2, y1, sh),
                           o2 = __builtin_amdgcn_alignbyte(y3, y2, sh), o3 = __builtin_amdgcn_alignbyte(y4, y3, sh);
            if (k0s + 4 <= body) {
              const v4u q = {o0, o1, o2, o3};
              __builtin_amdgcn_raw_buffer_store_b128(q, rsrc, static_cast<int>(dst64) + head + 4 * k0s, 0, 0);
            } else {
              uint32_t* dw = reinterpret_cast<uint32_t*>(d + head) + k0s;
              dw[0] = o0;
              if (k0s + 1 < body) dw[1] = o1;
              if (k0s + 2 < body) dw[2] = o2;
            }
          }
          // tail bytes: payload byte jlen - tail + sub is byte 3 - tail + sub of the last-three word
          if (sub < tail) d[head + 4 * body + sub] = static_cast<uint8_t>(tw[it] >> (8 * (3 - tail + sub)));
        }
      }
      px[1] += pclk<kProf>() - c1;
    }
    if (xw == 0) pflush<kProf>(a, 14, px, 2, lane);
    return;
  }

  // ================================================================== CONTROL (waves 8..10)
  // Control wave c takes tiles c, c + 3, c + 6, ...: parse, publish the tile's aggregate,
  // look back, PES entries, copy plan.  Three of them, so one tile's look-back latency
  // (agent-scope loads across XCDs) overlaps the others' work.
  const int cw = wave - kCWave0;
  uint64_t pm[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // diagnostics: job, plaintext, parse, look-back, plan
  for (uint32_t i = cw;; i += kCWaves) {
    uint64_t c0 = pclk<kProf>(), c1;
#define PSTAMP(k) c1 = pclk<kProf>(); pm[k] += c1 - c0; c0 = c1
    const int st = i % kStages;
    lds_wait(&L.seq[i % kRing], i + 1, a.timeout, lane);
    Job& J = L.job[i % kRing];
    const int64_t t = uniform64f(J.t);
    if (t < 0) {
      if (t == -1) {  // the first index past the last tile: release the copy-out waves
        if (i >= kStages) lds_wait(&L.xread[st], kXWaves * (i / kStages), a.timeout, lane);
        if (lane == 0) L.plive[st] = 0;
        lds_publish(&L.ptag[st], i + 1, lane);
      }
      if (cw == 0) pflush<kProf>(a, 0, pm, 8, lane);
      return;
    }
    PSTAMP(0);
    lds_wait(&L.ddone[st], kDWaves * (i / kStages + 1), a.timeout, lane);  // tile i's plaintext
    PSTAMP(1);
    pm[7] += 1;
    if (a.diag == 1) {  // diagnostics: the decrypt alone
      if (lane == 0) L.plive[st] = 1;
      lds_publish(&L.ptag[st], i + 1, lane);
      lds_publish(&L.plan[i % kPlanRing].tag, i + 1, lane);
      lds_publish(&L.jdone[i % kRing], i + 1, lane);
      continue;
    }
    const uint32_t* stagew = L.pk[st];
    const int seg = uniform32f(J.seg);
    const int tile = uniform32f(J.tile);
    const int ntile = uniform32f(J.ntile);
    const int64_t tile0 = uniform64f(J.tile0);
    const int64_t plen = uniform64f(J.plen);
    const int64_t es_off = uniform64f(J.es_off), cap = uniform64f(J.es_cap);
    const int pid0 = uniform32f(J.pid[0]), pid1 = uniform32f(J.pid[1]), pid2 = uniform32f(J.pid[2]);
    int npk;  // valid packets of this tile: all of them unless it holds the segment's end
    if (plen == -2) {
      npk = kTilePkts;
    } else {
      const int64_t n = plen < 0 ? 0 : plen;
      const int64_t np = n / kPktF - static_cast<int64_t>(tile) * kTilePkts;
      npk = np < 0 ? 0 : (np > kTilePkts ? kTilePkts : static_cast<int>(np));
    }
    // ---------------------------------------------------------------- parse (2 LDS round trips)
    // lane l holds packets kLanePk l .. kLanePk l + kLanePk - 1 (consecutive: the in-lane
    // running sum is in packet order)
    uint32_t w0[kLanePk], w1[kLanePk];
#pragma unroll
    for (int q = 0; q < kLanePk; ++q) {
      const int k = kLanePk * lane + q;
      const uint32_t* w = stagew + (k < kTilePkts ? k : 0) * (kPktF / 4);
      w0[q] = w[0];
      w1[q] = w[1];
    }
    int sps[kLanePk], at[kLanePk];
    uint32_t hw[kLanePk][6];
#pragma unroll
    for (int q = 0; q < kLanePk; ++q) {
      const int k = kLanePk * lane + q;
      const int afc = (w0[q] >> 28) & 3;
      const int s = 4 + ((afc & 2) ? 1 + static_cast<int>(w1[q] & 0xff) : 0);
      sps[q] = s;
      at[q] = (k < kTilePkts ? k : 0) * kPktF + (s <= kPktF ? s : 0);
      const uint32_t* w = stagew + (at[q] >> 2);
#pragma unroll
      for (int m = 0; m < 6; ++m) hw[q][m] = w[m];
    }
    Pkt pk[kLanePk];
#pragma unroll
    for (int q = 0; q < kLanePk; ++q) {
      const int k = kLanePk * lane + q;
      const uint32_t sh = static_cast<uint32_t>(at[q] & 3);
      uint32_t h[5];
#pragma unroll
      for (int m = 0; m < 5; ++m) h[m] = __builtin_amdgcn_alignbyte(hw[q][m + 1], hw[q][m], sh);
      pk[q] = parse_pkt(k < npk, w0[q], h, sps[q], pid0, pid1, pid2);
    }
    // packed per-lane totals: bytes <= kLanePk x 184 per lane, < 2^16 per tile; PES < 2^8
    uint32_t lA = 0, lB = 0, lC = 0, err = 0;
#pragma unroll
    for (int q = 0; q < kLanePk; ++q) {
      const uint32_t lb = static_cast<uint32_t>(pk[q].len), pf = static_cast<uint32_t>(pk[q].pesf);
      const int c = pk[q].c;
      lA += (c == 0 ? lb : 0u) | ((c == 1 ? lb : 0u) << 16);
      lB += (c == 2 ? lb : 0u) | ((c == 0 ? pf : 0u) << 16) | ((c == 1 ? pf : 0u) << 24);
      lC += c == 2 ? pf : 0u;
      err |= pk[q].err;
    }
    const uint32_t iA = dpp_scan(lA), iB = dpp_scan(lB), iC = dpp_scan(lC);
    const uint32_t tA = __builtin_amdgcn_readlane(static_cast<int>(iA), 63),
                   tB = __builtin_amdgcn_readlane(static_cast<int>(iB), 63),
                   tC = __builtin_amdgcn_readlane(static_cast<int>(iC), 63);
    const int32_t agb[3] = {static_cast<int32_t>(tA & 0xffff), static_cast<int32_t>(tA >> 16),
                            static_cast<int32_t>(tB & 0xffff)};
    const int32_t agp[3] = {static_cast<int32_t>((tB >> 16) & 0xff), static_cast<int32_t>(tB >> 24),
                            static_cast<int32_t>(tC)};
    uint64_t* look = a.look + 3 * t;
    {  // publish the aggregate first (a segment's first tile: its inclusive prefix)
      const uint64_t tag = tile == 0 ? kIncl : kAgg;
#pragma unroll
      for (int k = 0; k < 3; ++k)
        if (lane == k) gstore(look + k, tag | (static_cast<uint64_t>(agp[k]) << 32) | static_cast<uint32_t>(agb[k]));
    }
    {  // copy plans, in-tile part: class, payload start, length, offset among the tile's class bytes
      uint32_t rA = iA - lA, rB = iB - lB;
#pragma unroll
      for (int q = 0; q < kLanePk; ++q) {
        const int k = kLanePk * lane + q;
        const int c = pk[q].c;
        const uint32_t before_b = c == 0 ? (rA & 0xffff) : c == 1 ? (rA >> 16) : (rB & 0xffff);
        const uint32_t lb = static_cast<uint32_t>(pk[q].len), pf = static_cast<uint32_t>(pk[q].pesf);
        rA += (c == 0 ? lb : 0u) | ((c == 1 ? lb : 0u) << 16);
        rB += (c == 2 ? lb : 0u) | ((c == 0 ? pf : 0u) << 16) | ((c == 1 ? pf : 0u) << 24);
        if (k < kTilePkts) {
          L.meta[st][k] = static_cast<uint32_t>(c & 3) | (static_cast<uint32_t>(pk[q].ps) << 2) |
                          (static_cast<uint32_t>(pk[q].len) << 10);
          L.dst[st][k] = c < 3 ? static_cast<int32_t>(before_b) : 0;
        }
      }
    }
    if (lane == 0) L.plive[st] = 1;
    lds_publish(&L.ptag[st], i + 1, lane);  // the copy-out waves may read the tile now
    PSTAMP(2);

    // ---------------------------------------------------------------- look-back
    int64_t exb[3] = {0, 0, 0}, exq[3] = {0, 0, 0};
    if (tile > 0) {
      // four windows of 64 predecessors per round trip (lane q, window w: tile win - 64 w - q)
      constexpr int kW = 4;
      uint32_t open = 7;  // classes still summing back
      int64_t win = t - 1;
      uint32_t spins = 0;
      while (open) {
        uint64_t g[kW][3];
#pragma unroll
        for (int w = 0; w < kW; ++w) {
          const int64_t pt = win - 64 * w - lane;
#pragma unroll
          for (int k = 0; k < 3; ++k) g[w][k] = pt < tile0 ? kIncl : gload(a.look + 3 * pt + k);  // before the segment: 0
        }
        int stop[3], upto[3];  // per class: the window and lane of the nearest inclusive prefix
        bool wait = false;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          stop[k] = 64;
          upto[k] = kW - 1;
          if (!((open >> k) & 1)) continue;
#pragma unroll
          for (int w = 0; w < kW; ++w) {
            const uint64_t incl = __ballot((g[w][k] >> 62) == 2);
            const uint64_t none = __ballot((g[w][k] >> 62) == 0);
            const int sp = incl ? __builtin_ctzll(incl) : 64;
            const uint64_t need = sp >= 63 ? ~0ull : ((2ull << sp) - 1);
            if (none & need) wait = true;
            if (incl || (none & need)) {
              stop[k] = sp;
              upto[k] = w;
              break;
            }
          }
        }
        if (wait) {
          if (++spins > kSpinLimit) {
            if (lane == 0) atomicOr(a.timeout, 1u);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          if (!((open >> k) & 1)) continue;
          uint32_t vb = 0, vq = 0;
#pragma unroll
          for (int w = 0; w < kW; ++w) {
            const bool in = w < upto[k] || (w == upto[k] && lane <= stop[k]);
            vb += in ? static_cast<uint32_t>(g[w][k]) : 0u;
            vq += in ? static_cast<uint32_t>((g[w][k] >> 32) & 0x3fffffffu) : 0u;
          }
          exb[k] += dpp_sum(vb);
          exq[k] += dpp_sum(vq);
          if (stop[k] < 64) open &= ~(1u << k);
        }
        win -= 64 * kW;
      }
#pragma unroll
      for (int k = 0; k < 3; ++k)
        if (lane == k)
          gstore(look + k, kIncl | (static_cast<uint64_t>(exq[k] + agp[k]) << 32) | static_cast<uint32_t>(exb[k] + agb[k]));
    }
    PSTAMP(3);

    // ---------------------------------------------------------------- PES entries + copy plan
    {
      int64_t* inf = a.info + static_cast<int64_t>(seg) * kInfoF;
      const int64_t seg64 = seg;
      uint32_t rA = iA - lA, rB = iB - lB, rC = iC - lC;  // lane-exclusive running totals
#pragma unroll
      for (int q = 0; q < kLanePk; ++q) {
        const Pkt& p = pk[q];
        const int c = p.c;
        if (c < 3 && p.pesf) {
          const uint32_t before_b = c == 0 ? (rA & 0xffff) : c == 1 ? (rA >> 16) : (rB & 0xffff);
          const uint32_t before_p = c == 0 ? ((rB >> 16) & 0xff) : c == 1 ? (rB >> 24) : rC;
          const int64_t es_in_class = exb[c] + before_b;
          const int64_t pidx = exq[c] + before_p;
          if (pidx < a.max_pes) {
            int64_t* r = a.pes + ((seg64 * kClassesF + c) * a.max_pes + pidx) * 3;
            r[0] = es_in_class;
            r[1] = p.pts;
            r[2] = p.dts;
          }
          if (static_cast<int32_t>(before_p) + 1 == agp[c]) {  // the tile's last PES start of its class
            int64_t* lp = a.lastpes + (t * kClassesF + c) * 2;
            lp[0] = pidx;
            lp[1] = p.pts;
          }
        }
        const uint32_t lb = static_cast<uint32_t>(p.len), pf = static_cast<uint32_t>(p.pesf);
        rA += (c == 0 ? lb : 0u) | ((c == 1 ? lb : 0u) << 16);
        rB += (c == 2 ? lb : 0u) | ((c == 0 ? pf : 0u) << 16) | ((c == 1 ? pf : 0u) << 24);
        rC += c == 2 ? pf : 0u;
      }
      uint32_t status = 0;
#pragma unroll
      for (int b = 0; b < 6; ++b)
        if (__ballot((err >> b) & 1)) status |= 1u << b;
      if (tile == ntile - 1) {  // the last tile's inclusive prefix = segment totals
        const int64_t n = plen < 0 ? 0 : plen;
        if (plen < 0 || n % kPktF) status |= kBadLengthF;
        int64_t total_b = 0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const int64_t tb = exb[k] + agb[k], tp = exq[k] + agp[k];
          total_b += tb;
          if (tp > a.max_pes) status |= kPesOverflowF;
          if (lane == 0) {
            inf[kBytes0F + k] = tb;
            inf[kPes0F + k] = tp;
          }
        }
        if (lane == 0) {
          a.out_len[seg] = plen;
          inf[kPayloadBytesF] = total_b;
          inf[kNumPacketsF] = n / kPktF;
          inf[kAudioEsOffsetF] = cap;  // per-class regions (no compaction pass)
          inf[kId3EsOffsetF] = 2 * cap;
        }
      }
      if (status && lane == 0)
        atomicOr(reinterpret_cast<unsigned long long*>(inf + kStatusF), static_cast<unsigned long long>(status));
      CopyPlan& P = L.plan[i % kPlanRing];
      if (lane == 0) {
        P.es_off = es_off;
        P.cap = cap;
        P.live = 1;
      }
#pragma unroll
      for (int k = 0; k < 3; ++k)
        if (lane == k) P.base[k] = exb[k];
      lds_publish(&P.tag, i + 1, lane);  // tile i's class bases are in LDS
    }
    lds_publish(&L.jdone[i % kRing], i + 1, lane);
    PSTAMP(4);
#undef PSTAMP
  }
}

// One wave per segment, after the fused kernel: first / last PTS per class, and a segment
// whose padding failed reports no media (its tiles could not know before they wrote).
__global__ __launch_bounds__(64) void transmux_tail_kernel(TransmuxArgs a) {
  const int seg = blockIdx.x;
  const int tid = threadIdx.x;
  int64_t* inf = a.info + static_cast<int64_t>(seg) * kInfoF;
  const int64_t t0 = a.tile_prefix[seg], t1 = a.tile_prefix[seg + 1];
  const int64_t plen = t1 > t0 ? a.out_len[seg] : (a.enc[seg] ? -1 : a.src_len[seg]);
  if (plen < 0 || t1 == t0) {
    // bad PKCS#7 padding (or an empty segment): nothing is demuxed, as the split pipeline
    // reports it -- its tiles could not know before they wrote
    if (tid == 0) {
      if (t1 == t0) a.out_len[seg] = plen;
      for (int k = 0; k < 3; ++k) {
        inf[kBytes0F + k] = 0;
        inf[kPes0F + k] = 0;
        inf[kFirstPtsF + k] = -1;
        inf[kLastPtsF + k] = -1;
        inf[kVideoPidF + k] = -1;
      }
      inf[kPmtPidF] = -1;
      inf[kVideoTypeF] = 0;
      inf[kAudioTypeF] = 0;
      inf[kPayloadBytesF] = 0;
      inf[kNumPacketsF] = 0;
      inf[kAudioEsOffsetF] = 0;
      inf[kId3EsOffsetF] = 0;
      inf[kStatusF] = kNoPatF | (plen < 0 || plen % kPktF ? kBadLengthF : 0);
    }
    return;
  }
  if (tid < 3) {
    const int k = tid;
    const int64_t np = inf[kPes0F + k];
    const int64_t* pe = a.pes + (static_cast<int64_t>(seg) * kClassesF + k) * a.max_pes * 3;
    inf[kFirstPtsF + k] = (np > 0 && a.max_pes > 0) ? pe[1] : -1;
    int64_t last = -1;
    for (int64_t t = t1 - 1; t >= t0; --t) {
      const int64_t* lp = a.lastpes + (t * kClassesF + k) * 2;
      if (lp[0] >= 0) {
        last = lp[1];
        break;
      }
    }
    inf[kLastPtsF + k] = np > 0 ? last : -1;
  }
}

int transmux_tile_bytes() { return kTileBytes; }

hipError_t launch_transmux_fused(const TransmuxArgs& args, int num_cu, hipStream_t stream) {
  if (args.nseg <= 0) return hipSuccess;
  hipLaunchKernelGGL(transmux_psi_kernel, dim3(static_cast<unsigned>(args.nseg)), dim3(64), 0, stream, args);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (args.total_tiles > 0) {
    int64_t grid = args.total_tiles < num_cu ? args.total_tiles : num_cu;
    if (grid < 1) grid = 1;
    if (args.prof != nullptr)
      hipLaunchKernelGGL(transmux_fused_kernel<true>, dim3(static_cast<unsigned>(grid)), dim3(kFThreads), 0, stream, args);
    else
      hipLaunchKernelGGL(transmux_fused_kernel<false>, dim3(static_cast<unsigned>(grid)), dim3(kFThreads), 0, stream, args);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(transmux_tail_kernel, dim3(static_cast<unsigned>(args.nseg)), dim3(64), 0, stream, args);
  return hipGetLastError();
}

#undef SELF
#undef LDSW
#undef XOR3F
#undef ROT
#undef TDA

}  // namespace dev
}  // namespace hlsp2p
