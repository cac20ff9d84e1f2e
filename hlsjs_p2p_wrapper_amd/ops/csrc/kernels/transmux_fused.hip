// Fused AES-128-CBC decrypt + MPEG-TS demux of a batch of HLS segments (SURVEY §2.2 K10 +
// K11) — CDNA4 / gfx950.  One pass over the ciphertext: the plaintext never exists in HBM.
//
// The split pipeline (aes_cbc.hip + ts_demux.hip) moves each segment through HBM ~5 times:
// decrypt reads the ciphertext and writes plaintext, the scan re-reads packet headers, the
// gather re-reads the plaintext and writes the elementary streams.  Here a workgroup
// decrypts one TILE of a segment (260 TS packets = 65 x 47 AES blocks = 48,880 bytes; 4
// packets = 47 blocks is the smallest unit on which the 16-byte block grid and the 188-byte
// packet grid align) straight into LDS, parses the packet headers there, learns where its payload
// bytes go from the tiles before it, and writes them to the elementary-stream buffer:
// ciphertext read once, ES written once.
//
// LDS (one 1024-thread workgroup per CU):
//   [0, 64K)       table image, row x (256 B) = [32 lane copies of TdL[x] | 32 lane copies of
//                  InvSbox[x]]; lane l reads dword l % 32 of a half-row: every ds_read_b32 of
//                  the rounds is bank-conflict free.  Td1..Td3 are byte rotations of TdL
//                  (one v_alignbit each: VALU has room, the rounds are LDS bound), which is
//                  what frees the 64 KiB the split kernel spent on pre-rotated copies.
//   [64K, +48K)    the tile's plaintext (decrypted by ds_write_b128, one per block)
//   + small scan / hand-off scratch.
//
// Inter-tile prefix (decoupled look-back).  A tile's payload bytes land at the running sum
// of the payload bytes of the tiles before it (per class: video, audio, id3), and its PES
// entries at the running PES count.  Tiles are taken from a global ticket counter, so
// every lower ticket belongs to a workgroup that is running or done: a tile publishes its
// aggregate (three 8-byte {status, PES count, bytes} granules, one per class, written by
// single agent-scope stores and read back by agent-scope loads — the data is its own flag,
// no fence), looks back over its predecessors (one wave, 64 at a time) until it meets an
// inclusive prefix, then publishes its own inclusive prefix.  Tile 0 of a segment parses
// PAT/PMT and publishes the PIDs the same way; the other tiles of the segment wait for them
// (by then tile 0 is long past its decrypt).  Every spin is bounded: a hand-off that never
// arrives sets the launch's timeout word and the tile proceeds (wrong output, no hang).
//
// ES layout per segment at es_off[seg]: three regions of es_cap[seg] bytes, video / audio /
// id3, each class written at its running offset in its own region (packing the classes back
// to back would need the segment's video total before the first audio byte is written, i.e.
// another pass); the info row says where each class starts (slots 22, 23).  PES tables and
// info rows are the split pipeline's and the host oracle's (runtime/ts.cpp);
// transmux_tail_kernel finishes what only the whole segment knows (first / last PTS, a
// failed padding check).
#include "common.h"
#include "transmux_args.h"

namespace hlsp2p {
namespace dev {

namespace {

constexpr int kFThreads = 1024;
constexpr int kFWaves = kFThreads / 64;
constexpr int kPktF = 188;
constexpr int kTilePkts = 260;                    // 65 x 4 packets
constexpr int kTileBytes = kTilePkts * kPktF;     // 48,880 = 16 x 3,055
constexpr int kTileBlocks = kTileBytes / 16;      // 3,055 AES blocks
constexpr int kFBlk = 3;                          // blocks per lane (independent chains): 16 x 64 x 3 >= 3,055
constexpr int kWaveBlk = 64 * kFBlk;              // blocks per wave and tile
static_assert(kFWaves * kWaveBlk >= kTileBlocks && kTileBytes % 16 == 0 && kTilePkts % 4 == 0, "tile shape");
constexpr int kTabDwords = 256 * 64;              // 64 KiB
constexpr int kStageDwords = kTileBytes / 4 + 8;  // + slack for the copy-out funnel reads
constexpr int kClassesF = 3;
constexpr int kInfoF = 24;
constexpr int kScanWaves = (kTilePkts + 63) / 64;  // 6 waves hold one packet per lane
// info slots / status bits (runtime/ts.hpp, ts_demux.hip)
constexpr int kStatusF = 0, kPmtPidF = 1, kVideoPidF = 2, kNumPacketsF = 5, kBytes0F = 6, kPes0F = 9,
              kVideoTypeF = 12, kAudioTypeF = 13, kPayloadBytesF = 14, kFirstPtsF = 16, kLastPtsF = 19,
              kAudioEsOffsetF = 22, kId3EsOffsetF = 23;
constexpr uint32_t kBadSyncF = 1, kNoPatF = 2, kNoPmtF = 4, kPesOverflowF = 8, kPesHeaderErrorF = 16,
                   kBadLengthF = 32;
constexpr uint64_t kAgg = 1ull << 62, kIncl = 2ull << 62;
constexpr uint32_t kSpinLimit = 1u << 22;  // ~seconds of polling: only a broken hand-off gets here

#define SELF(k) (0x0c020000u | ((4u + (k)) << 8))
#define LDSW(addr) (*reinterpret_cast<const uint32_t*>(s_bytes + (addr)))
#define XOR3F(a, b, c) __builtin_amdgcn_bitop3_b32((a), (b), (c), 0x96)
#define ROT(v, r) __builtin_amdgcn_alignbit((v), (v), 32u - (r))
// TdL lookup of byte k of w (the t-rotation is applied by the caller)
#define TDA_F(w, k) __builtin_amdgcn_perm((w), td_base, SELF(k))
#define IS_F(w, k) (LDSW(__builtin_amdgcn_perm((w), is_base, SELF(k))) & 0xffu)

__device__ __forceinline__ int64_t read_pts_f(const uint8_t* p) {
  return (int64_t((p[0] >> 1) & 0x07) << 30) | (int64_t(p[1]) << 22) | (int64_t(p[2] >> 1) << 15) |
         (int64_t(p[3]) << 7) | int64_t(p[4] >> 1);
}

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

// agent-scope 8-byte granules (stores and loads bypass the non-coherent L1; the value is
// its own ready flag)
__device__ __forceinline__ void gstore(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t gload(uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int wave_incl_scan_f(int v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(v, o);
    if (lane >= o) v += t;
  }
  return v;
}

}  // namespace


__global__ __launch_bounds__(kFThreads, 1) void transmux_fused_kernel(TransmuxArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t s_tab[kTabDwords];
  __shared__ __attribute__((aligned(16))) uint32_t s_pk[kStageDwords];
  __shared__ uint32_t s_wave[kScanWaves][3];  // per-wave packed scan totals
  __shared__ int32_t s_ex[2 * kClassesF];     // tile's exclusive prefix (bytes, PES) per class
  __shared__ int32_t s_agg[2 * kClassesF];    // tile's aggregate
  __shared__ int32_t s_psi[8];                // pmt, vpid, apid, ipid, vtype, atype, valid
  __shared__ int64_t s_len;                   // plaintext length when this tile holds the last block
  __shared__ unsigned int s_ticket;
  __shared__ uint32_t s_err;
  __shared__ uint32_t s_meta[kTilePkts];      // per packet: class | ps << 2 | len << 10 | pes << 18
  __shared__ int32_t s_dst[kTilePkts];        // per packet: destination offset in its class (tile-local)
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  {  // table image: row x = [32 x TdL[x] | 32 x InvSbox[x]]; thread t fills dwords t + 1024 k
    uint32_t v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int d = tid + k * kFThreads;  // dword index: row d >> 6, column d & 63
      const int x = d >> 6;
      v[k] = (d & 32) ? static_cast<uint32_t>(a.isb[x]) : a.tdl[x];
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) s_tab[tid + k * kFThreads] = v[k];
  }
  const uint8_t* s_bytes = reinterpret_cast<const uint8_t*>(s_tab);
  uint8_t* s_stage = reinterpret_cast<uint8_t*>(s_pk);
  const uint32_t l4 = static_cast<uint32_t>(tid & 31) << 2;
  const uint32_t td_base = l4, is_base = 128u | l4;

  for (;;) {
    __syncthreads();  // previous tile's LDS use is over (and, first time, the table image is in)
    if (tid == 0) {
      s_ticket = atomicAdd(a.ticket, 1u);
      s_len = -2;
      s_err = 0;
    }
    __syncthreads();
    const int64_t t = s_ticket;
    if (t >= a.total_tiles) break;
    const int seg = find_seg_wave(a.tile_prefix, a.nseg, t);
    const int64_t tile0 = a.tile_prefix[seg];
    const int tile = static_cast<int>(t - tile0);
    const int ntile = static_cast<int>(a.tile_prefix[seg + 1] - tile0);
    const int64_t slen = a.src_len[seg];
    const bool encrypted = a.enc[seg] != 0;
    const int64_t tbyte0 = static_cast<int64_t>(tile) * kTileBytes;  // tile start in the segment
    const int64_t tbytes = slen - tbyte0 < kTileBytes ? slen - tbyte0 : kTileBytes;  // source bytes in the tile
    const uint8_t* src = a.src + a.src_off[seg];

    // ---------------------------------------------------------------- A. decrypt into LDS
    if (encrypted) {
      uint32_t rk[44];
#pragma unroll
      for (int k = 0; k < 44; ++k) rk[k] = a.drk[seg * 44 + k];
      const int64_t nblk = slen / 16;
      const int64_t bt0 = tbyte0 / 16;  // first block of the tile
      const int tb = static_cast<int>(tbytes / 16);  // blocks in the tile
      const uint4* cs = reinterpret_cast<const uint4*>(src);
      uint32_t st[kFBlk][4];
#pragma unroll
      for (int j = 0; j < kFBlk; ++j) {
        const int lb = wave * kWaveBlk + 64 * j + lane;  // block within the tile
        const uint4 c = lb < tb ? cs[bt0 + lb] : make_uint4(0, 0, 0, 0);
        st[j][0] = c.x ^ rk[0]; st[j][1] = c.y ^ rk[1]; st[j][2] = c.z ^ rk[2]; st[j][3] = c.w ^ rk[3];
      }
      // rounds 1..9: chain j's 16 LDS reads are issued before chain j-1's XORs consume theirs
#pragma unroll
      for (int r = 1; r < 10; ++r) {
        const uint32_t* k = rk + 4 * r;
        uint32_t v[2][16];
#pragma unroll
        for (int j = 0; j <= kFBlk; ++j) {
          if (j < kFBlk) {
            const uint32_t* s = st[j];
            uint32_t* o = v[j & 1];
            const uint32_t ad[16] = {TDA_F(s[0], 0), TDA_F(s[3], 1), TDA_F(s[2], 2), TDA_F(s[1], 3),
                                     TDA_F(s[1], 0), TDA_F(s[0], 1), TDA_F(s[3], 2), TDA_F(s[2], 3),
                                     TDA_F(s[2], 0), TDA_F(s[1], 1), TDA_F(s[0], 2), TDA_F(s[3], 3),
                                     TDA_F(s[3], 0), TDA_F(s[2], 1), TDA_F(s[1], 2), TDA_F(s[0], 3)};
#pragma unroll
            for (int q = 0; q < 16; ++q) o[q] = LDSW(ad[q]);
          }
          if (j > 0) {
            uint32_t* s = st[j - 1];
            const uint32_t* x = v[(j - 1) & 1];
            s[0] = XOR3F(XOR3F(x[0], ROT(x[1], 8), ROT(x[2], 16)), ROT(x[3], 24), k[0]);
            s[1] = XOR3F(XOR3F(x[4], ROT(x[5], 8), ROT(x[6], 16)), ROT(x[7], 24), k[1]);
            s[2] = XOR3F(XOR3F(x[8], ROT(x[9], 8), ROT(x[10], 16)), ROT(x[11], 24), k[2]);
            s[3] = XOR3F(XOR3F(x[12], ROT(x[13], 8), ROT(x[14], 16)), ROT(x[15], 24), k[3]);
          }
        }
      }
      const uint32_t* kf = rk + 40;
      // CBC chaining input, loaded after the rounds (an L2 hit: the wave read these lines
      // for its own blocks) instead of held in 16 VGPRs across them
      uint4 pv[kFBlk];
#pragma unroll
      for (int j = 0; j < kFBlk; ++j) {
        const int lb = wave * kWaveBlk + 64 * j + lane;
        const int64_t b = bt0 + lb;
        pv[j] = (lb < tb && b == 0) ? reinterpret_cast<const uint4*>(a.ivw)[seg]
                                    : (lb < tb ? cs[b - 1] : make_uint4(0, 0, 0, 0));
      }
#pragma unroll
      for (int j = 0; j < kFBlk; ++j) {
        const uint32_t* s = st[j];
        const uint32_t o0 = XOR3F(IS_F(s[0], 0) | (IS_F(s[3], 1) << 8) | (IS_F(s[2], 2) << 16) | (IS_F(s[1], 3) << 24),
                                  kf[0], pv[j].x);
        const uint32_t o1 = XOR3F(IS_F(s[1], 0) | (IS_F(s[0], 1) << 8) | (IS_F(s[3], 2) << 16) | (IS_F(s[2], 3) << 24),
                                  kf[1], pv[j].y);
        const uint32_t o2 = XOR3F(IS_F(s[2], 0) | (IS_F(s[1], 1) << 8) | (IS_F(s[0], 2) << 16) | (IS_F(s[3], 3) << 24),
                                  kf[2], pv[j].z);
        const uint32_t o3 = XOR3F(IS_F(s[3], 0) | (IS_F(s[2], 1) << 8) | (IS_F(s[1], 2) << 16) | (IS_F(s[0], 3) << 24),
                                  kf[3], pv[j].w);
        const int lb = wave * kWaveBlk + 64 * j + lane;
        if (lb < tb) {
          reinterpret_cast<uint4*>(s_stage)[lb] = make_uint4(o0, o1, o2, o3);
          if (bt0 + lb == nblk - 1) {  // the segment's last block: PKCS#7
            const int64_t n = pkcs7_len_f(make_uint4(o0, o1, o2, o3), nblk * 16);
            s_len = n;
            a.out_len[seg] = n;
          }
        }
      }
    } else {  // clear segment: the tile's bytes into LDS (16 B per lane; the source has slack)
      const uint4* cs = reinterpret_cast<const uint4*>(src + tbyte0);
      const int nv = static_cast<int>((tbytes + 15) / 16);
#pragma unroll
      for (int j = 0; j < kFBlk; ++j) {
        const int lv = wave * kWaveBlk + 64 * j + lane;
        if (lv < nv) reinterpret_cast<uint4*>(s_stage)[lv] = cs[lv];
      }
      if (tile == ntile - 1 && tid == 0) {
        s_len = slen;
        a.out_len[seg] = slen;
      }
    }
    __syncthreads();
    if (a.diag == 1) continue;  // diagnostics: the decrypt alone

    // valid packets of this tile: all of them unless it holds the segment's end
    const int64_t plen = s_len;  // -2: not the last tile; -1: bad padding; else the plaintext length
    int npk;
    if (plen == -2) {
      npk = kTilePkts;
    } else {
      const int64_t n = plen < 0 ? 0 : plen;
      const int64_t np = n / kPktF - static_cast<int64_t>(tile) * kTilePkts;
      npk = np < 0 ? 0 : (np > kTilePkts ? kTilePkts : static_cast<int>(np));
    }

    // ---------------------------------------------------------------- B. PSI (tile 0)
    int64_t* inf = a.info + static_cast<int64_t>(seg) * kInfoF;
    uint64_t* psi = a.psi + 2 * static_cast<int64_t>(seg);
    if (tile == 0) {
      if (tid == 0) {
        const int scan = npk < 64 ? npk : 64;
        int pmt_pid = -1, vpid = -1, apid = -1, ipid = -1, vtype = 0, atype = 0;
        uint32_t status = 0;
        for (int i = 0; i < scan && pmt_pid < 0; ++i) {
          const uint8_t* p = s_stage + i * kPktF;
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
              pmt_pid = ((p[q + 2] & 0x1f) << 8) | p[q + 3];
              break;
            }
          }
        }
        if (pmt_pid < 0) status |= kNoPatF;
        bool pmt_found = false;
        for (int i = 0; i < scan && pmt_pid >= 0 && !pmt_found; ++i) {
          const uint8_t* p = s_stage + i * kPktF;
          if (p[0] != 0x47) continue;
          const int pid = ((p[1] & 0x1f) << 8) | p[2];
          if (pid != pmt_pid || !(p[1] & 0x40)) continue;
          const int afc = (p[3] >> 4) & 3;
          int ps = 4 + ((afc & 2) ? 1 + p[4] : 0);
          if (!(afc & 1) || ps >= kPktF) continue;
          ps += 1 + p[ps];
          if (ps + 12 > kPktF || p[ps] != 0x02) continue;
          pmt_found = true;
          const int sl = ((p[ps + 1] & 0x0f) << 8) | p[ps + 2];
          const int end = ps + 3 + sl - 4 < kPktF ? ps + 3 + sl - 4 : kPktF;
          const int pil = ((p[ps + 10] & 0x0f) << 8) | p[ps + 11];
          for (int q = ps + 12 + pil; q + 5 <= end;) {
            const int type = p[q];
            const int epid = ((p[q + 1] & 0x1f) << 8) | p[q + 2];
            const int eil = ((p[q + 3] & 0x0f) << 8) | p[q + 4];
            if ((type == 0x1B || type == 0x24) && vpid < 0) {
              vpid = epid;
              vtype = type;
            } else if ((type == 0x0F || type == 0x03 || type == 0x04) && apid < 0) {
              apid = epid;
              atype = type;
            } else if (type == 0x15 && ipid < 0) {
              ipid = epid;
            }
            q += 5 + eil;
          }
        }
        if (pmt_pid >= 0 && !pmt_found) status |= kNoPmtF;
        inf[kPmtPidF] = pmt_pid;
        inf[kVideoPidF] = vpid;
        inf[kVideoPidF + 1] = apid;
        inf[kVideoPidF + 2] = ipid;
        inf[kVideoTypeF] = vtype;
        inf[kAudioTypeF] = atype;
        if (status) atomicOr(reinterpret_cast<unsigned long long*>(inf + kStatusF), static_cast<unsigned long long>(status));
        s_psi[0] = pmt_pid; s_psi[1] = vpid; s_psi[2] = apid; s_psi[3] = ipid; s_psi[6] = 1;
        // PIDs are 13-bit: 16-bit fields, 0xffff = absent, bit 63 = ready
        auto f = [](int v) { return static_cast<uint64_t>(v < 0 ? 0xffff : v); };
        gstore(psi, (1ull << 63) | f(vpid) | (f(apid) << 16) | (f(ipid) << 32));
      }
    } else if (wave == 0) {  // wait for tile 0's PIDs (bounded)
      uint64_t g = 0;
      uint32_t spins = 0;
      for (;;) {
        g = gload(psi);
        if (g >> 63) break;
        if (++spins > kSpinLimit) {
          if (lane == 0) atomicOr(a.timeout, 1u);
          g = (1ull << 63) | 0xffffffffffffull;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (lane == 0) {
        auto u = [](uint64_t v) { return v == 0xffff ? -1 : static_cast<int>(v); };
        s_psi[1] = u(g & 0xffff);
        s_psi[2] = u((g >> 16) & 0xffff);
        s_psi[3] = u((g >> 32) & 0xffff);
      }
    }
    __syncthreads();

    // ---------------------------------------------------------------- C. packet headers
    const int cpid0 = s_psi[1], cpid1 = s_psi[2], cpid2 = s_psi[3];
    int c = 3, ps = 0, len = 0, pesf = 0;
    int64_t pts = -1, dts = -1;
    if (tid < kTilePkts) {
      uint32_t err = 0;
      if (tid < npk) {
        const uint8_t* p = s_stage + tid * kPktF;
        const uint32_t hdr = *reinterpret_cast<const uint32_t*>(p);  // packets are 4-byte aligned
        const int sync = hdr & 0xff;
        const int b1 = (hdr >> 8) & 0xff, b2 = (hdr >> 16) & 0xff, b3 = hdr >> 24;
        if (sync != 0x47) {
          err |= kBadSyncF;
        } else {
          const int pid = ((b1 & 0x1f) << 8) | b2;
          const int cls = (cpid0 >= 0 && pid == cpid0) ? 0 : (cpid1 >= 0 && pid == cpid1) ? 1
                        : (cpid2 >= 0 && pid == cpid2) ? 2 : 3;
          const int afc = (b3 >> 4) & 3;
          if (cls < 3 && (afc & 1)) {
            int s = 4 + ((afc & 2) ? 1 + p[4] : 0);
            if (s > kPktF) {
              err |= kBadLengthF;
            } else {
              int l = kPktF - s;
              bool ok = true;
              if (b1 & 0x40) {
                const uint8_t* h = p + s;
                if (l < 9 || h[0] != 0 || h[1] != 0 || h[2] != 1 || 9 + h[8] > l) {
                  err |= kPesHeaderErrorF;
                  ok = false;
                } else {
                  pts = ((h[7] & 0x80) && l >= 14) ? read_pts_f(h + 9) : -1;
                  dts = ((h[7] & 0xC0) == 0xC0 && l >= 19) ? read_pts_f(h + 14) : -1;
                  pesf = 1;
                  s += 9 + h[8];
                  l -= 9 + h[8];
                }
              }
              if (ok) {
                c = cls;
                ps = s;
                len = l;
              }
            }
          }
        }
      }
      if (err) atomicOr(&s_err, err);
    }
    // ---------------------------------------------------------------- D. tile scan
    // packed in-wave inclusive scans (bytes <= 64 x 184 < 2^16, PES starts <= 64 < 2^8)
    const uint32_t lb = static_cast<uint32_t>(len), pf = static_cast<uint32_t>(pesf);
    uint32_t sA = (c == 0 ? lb : 0u) | ((c == 1 ? lb : 0u) << 16);
    uint32_t sB = (c == 2 ? lb : 0u) | ((c == 0 ? pf : 0u) << 16) | ((c == 1 ? pf : 0u) << 24);
    uint32_t sC = c == 2 ? pf : 0u;
    if (wave < kScanWaves) {
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t tA = __shfl_up(sA, o), tB = __shfl_up(sB, o), tC = __shfl_up(sC, o);
        if (lane >= o) {
          sA += tA;
          sB += tB;
          sC += tC;
        }
      }
      if (lane == 63) {
        s_wave[wave][0] = sA;
        s_wave[wave][1] = sB;
        s_wave[wave][2] = sC;
      }
    }
    __syncthreads();
    if (tid == 0) {  // tile aggregate (sums over 6 waves of up to 64 x 184 bytes: fits int32)
      int32_t ag[6] = {0, 0, 0, 0, 0, 0};
      for (int w = 0; w < kScanWaves; ++w) {
        const uint32_t A = s_wave[w][0], B = s_wave[w][1], C = s_wave[w][2];
        ag[0] += A & 0xffff; ag[2] += A >> 16; ag[4] += B & 0xffff;     // bytes v, a, i
        ag[1] += (B >> 16) & 0xff; ag[3] += B >> 24; ag[5] += C;          // PES v, a, i
      }
      for (int k = 0; k < 6; ++k) s_agg[k] = ag[k];
    }
    __syncthreads();
    // ---------------------------------------------------------------- E. look-back
    if (wave == 0) {
      uint64_t* look = a.look + 3 * t;
      const int32_t ag_b[3] = {s_agg[0], s_agg[2], s_agg[4]}, ag_p[3] = {s_agg[1], s_agg[3], s_agg[5]};
      if (tile == 0) {  // first tile of its segment: inclusive = aggregate
        if (lane < 3)
          gstore(look + lane, kIncl | (static_cast<uint64_t>(ag_p[lane]) << 32) | static_cast<uint32_t>(ag_b[lane]));
        if (lane < 6) s_ex[lane] = 0;
      } else {
        if (lane < 3)
          gstore(look + lane, kAgg | (static_cast<uint64_t>(ag_p[lane]) << 32) | static_cast<uint32_t>(ag_b[lane]));
        int64_t exb[3] = {0, 0, 0}, exp_[3] = {0, 0, 0};
#pragma unroll
        for (int k = 0; k < 3; ++k) {  // per class: sum back to the nearest inclusive prefix
          int64_t win = t - 1;          // lane i looks at tile win - i
          uint32_t spins = 0;
          for (;;) {
            const int64_t pt = win - lane;
            uint64_t g;
            if (pt < tile0) {
              g = kIncl;  // before the segment: inclusive zero
            } else {
              g = gload(a.look + 3 * pt + k);
            }
            const uint64_t st = g >> 62;
            const uint64_t incl = __ballot(st == 2);
            const uint64_t none = __ballot(st == 0);
            const int stop = incl ? __builtin_ctzll(incl) : 64;  // nearest inclusive lane
            const uint64_t need = stop == 64 ? ~0ull : ((stop == 63 ? ~0ull : ((2ull << stop) - 1)));
            if (none & need) {
              if (++spins > kSpinLimit) {
                if (lane == 0) atomicOr(a.timeout, 1u);
                break;
              }
              __builtin_amdgcn_s_sleep(1);
              continue;
            }
            int64_t vb = (lane <= stop) ? static_cast<int64_t>(g & 0xffffffffu) : 0;
            int64_t vp = (lane <= stop) ? static_cast<int64_t>((g >> 32) & 0x3fffffffu) : 0;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
              vb += __shfl_xor(vb, o);
              vp += __shfl_xor(vp, o);
            }
            exb[k] += vb;
            exp_[k] += vp;
            if (stop < 64) break;
            win -= 64;
          }
        }
        if (lane < 3)
          gstore(look + lane, kIncl | (static_cast<uint64_t>(exp_[lane] + ag_p[lane]) << 32) |
                                  static_cast<uint32_t>(exb[lane] + ag_b[lane]));
        if (lane == 0) {
          for (int k = 0; k < 3; ++k) {
            s_ex[2 * k] = static_cast<int32_t>(exb[k]);
            s_ex[2 * k + 1] = static_cast<int32_t>(exp_[k]);
          }
        }
      }
    }
    __syncthreads();
    // ---------------------------------------------------------------- F. PES entries
    const int64_t seg64 = seg;
    if (tid < kTilePkts) {
      uint32_t wA = 0, wB = 0, wC = 0;  // earlier waves' packed totals
      for (int w = 0; w < wave; ++w) {
        wA += s_wave[w][0];
        wB += s_wave[w][1];
        wC += s_wave[w][2];
      }
      const uint32_t iA = sA + wA, iB = sB + wB, iC = sC + wC;  // tile-inclusive (no field overflow)
      int32_t dst = 0;
      if (c < 3) {
        const uint32_t inc_b = c == 0 ? (iA & 0xffff) : c == 1 ? (iA >> 16) : (iB & 0xffff);
        const uint32_t inc_p = c == 0 ? ((iB >> 16) & 0xff) : c == 1 ? (iB >> 24) : iC;
        const int64_t es_in_class = static_cast<int64_t>(s_ex[2 * c]) + inc_b - len;
        dst = static_cast<int32_t>(es_in_class);
        if (pesf) {
          const int64_t pidx = static_cast<int64_t>(s_ex[2 * c + 1]) + inc_p - 1;
          if (pidx < a.max_pes) {
            int64_t* r = a.pes + ((seg64 * kClassesF + c) * a.max_pes + pidx) * 3;
            r[0] = es_in_class;
            r[1] = pts;
            r[2] = dts;
          }
          if (static_cast<int32_t>(inc_p) == s_agg[2 * c + 1]) {  // the tile's last PES start of its class
            int64_t* lp = a.lastpes + (t * kClassesF + c) * 2;
            lp[0] = pidx;
            lp[1] = pts;
          }
        }
      }
      s_meta[tid] = static_cast<uint32_t>(c & 3) | (static_cast<uint32_t>(ps) << 2) |
                    (static_cast<uint32_t>(len) << 10);
      s_dst[tid] = dst;
    }
    if (tid == 0) {
      const uint32_t e = s_err;
      if (e) atomicOr(reinterpret_cast<unsigned long long*>(inf + kStatusF), static_cast<unsigned long long>(e));
    }
    __syncthreads();
    // ---------------------------------------------------------------- G. payloads out
    // Five packets per wave iteration: a 12-lane group moves one payload (<= 184 B = 46
    // dwords): lane `sub` funnels body dwords 4sub..4sub+3 out of 5 LDS dwords (v_alignbyte)
    // and writes them with ONE dwordx4 buffer store to a dword-aligned address; byte stores
    // for the <= 3 + 3 unaligned head / tail bytes.  Each class goes to its own region (one
    // buffer resource per segment covers all three).
    if (a.diag != 2) {
      typedef unsigned int v4u __attribute__((ext_vector_type(4)));
      uint8_t* ebase = a.es + a.es_off[seg];
      const int64_t cap = a.es_cap[seg];
      const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(ebase, 0, 0x7fffffff, 0x00020000);
      const int grp = lane / 12, sub = lane - 12 * grp;  // groups 0..4; lanes 60..63 idle
      // wave w takes packets w*5 + g, then + 80, ...: every wave moves its share
      for (int base = wave * 5; base < kTilePkts; base += kFWaves * 5) {
        const int j = base + grp;
        const bool valid = grp < 5 && j < kTilePkts;
        const uint32_t m = valid ? s_meta[j] : 3u;
        const int jc = m & 3, jps = (m >> 2) & 0xff;
        const int jlen = (jc < 3) ? static_cast<int>((m >> 10) & 0xff) : 0;
        if (jlen == 0) continue;
        const int64_t dst64 = jc * cap + s_dst[j];  // the class's region
        const int jdst = static_cast<int>(dst64);
        const int s = j * kPktF + jps;  // LDS byte offset of the payload
        uint8_t* d = ebase + dst64;
        const int mis = static_cast<int>((4 - (reinterpret_cast<uintptr_t>(d) & 3)) & 3);
        const int head = mis < jlen ? mis : jlen;
        const int body = (jlen - head) >> 2;
        const int tail = jlen - head - 4 * body;
        if (sub < head) d[sub] = s_stage[s + sub];
        const int k0 = 4 * sub;
        if (k0 < body) {
          const int aa = s + head + 4 * k0;
          const uint32_t sh = static_cast<uint32_t>(aa & 3);
          const uint32_t* w = s_pk + (aa >> 2);
          const uint32_t x0 = w[0], x1 = w[1], x2 = w[2], x3 = w[3], x4 = w[4];
          const uint32_t o0 = __builtin_amdgcn_alignbyte(x1, x0, sh), o1 = __builtin_amdgcn_alignbyte(x2, x1, sh),
                         o2 = __builtin_amdgcn_alignbyte(x3, x2, sh), o3 = __builtin_amdgcn_alignbyte(x4, x3, sh);
          uint32_t* dw = reinterpret_cast<uint32_t*>(d + head) + k0;
          if (k0 + 4 <= body) {
            const v4u q = {o0, o1, o2, o3};
            __builtin_amdgcn_raw_buffer_store_b128(q, rsrc, jdst + head + 4 * k0, 0, 0);
          } else {
            dw[0] = o0;
            if (k0 + 1 < body) dw[1] = o1;
            if (k0 + 2 < body) dw[2] = o2;
          }
        }
        if (sub < tail) d[head + 4 * body + sub] = s_stage[s + head + 4 * body + sub];
      }
    }
    // ---------------------------------------------------------------- H. segment totals
    if (tile == ntile - 1 && tid == 0) {  // the last tile's inclusive prefix = segment totals
      const int64_t n = plen < 0 ? 0 : plen;
      uint32_t status = 0;
      if (plen < 0 || n % kPktF) status |= kBadLengthF;
      int64_t over = 0;
      int64_t total_b = 0;
      for (int k = 0; k < 3; ++k) {
        const int64_t tb = static_cast<int64_t>(s_ex[2 * k]) + s_agg[2 * k];
        const int64_t tp = static_cast<int64_t>(s_ex[2 * k + 1]) + s_agg[2 * k + 1];
        inf[kBytes0F + k] = tb;
        inf[kPes0F + k] = tp;
        total_b += tb;
        if (tp > a.max_pes) over = kPesOverflowF;
      }
      inf[kPayloadBytesF] = total_b;
      inf[kNumPacketsF] = n / kPktF;
      inf[kAudioEsOffsetF] = a.es_cap[seg];  // per-class regions (no compaction pass)
      inf[kId3EsOffsetF] = 2 * a.es_cap[seg];
      status |= static_cast<uint32_t>(over);
      if (status) atomicOr(reinterpret_cast<unsigned long long*>(inf + kStatusF), static_cast<unsigned long long>(status));
    }
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
  if (args.total_tiles > 0) {
    int64_t grid = args.total_tiles < num_cu ? args.total_tiles : num_cu;
    if (grid < 1) grid = 1;
    hipLaunchKernelGGL(transmux_fused_kernel, dim3(static_cast<unsigned>(grid)), dim3(kFThreads), 0, stream, args);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(transmux_tail_kernel, dim3(static_cast<unsigned>(args.nseg)), dim3(64), 0, stream, args);
  return hipGetLastError();
}

#undef SELF
#undef LDSW
#undef XOR3F
#undef ROT
#undef TDA_F
#undef IS_F

}  // namespace dev
}  // namespace hlsp2p
