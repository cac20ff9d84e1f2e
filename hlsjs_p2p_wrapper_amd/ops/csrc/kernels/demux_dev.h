// Device helpers shared by the TS demux kernels (ts_demux.hip's one-pass kernel and the
// fused decrypt + demux kernel, transmux_fused.hip): the oracle's packet-header rules on
// LDS-staged packets, VALU-only wave scans, agent-scope look-back granules.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hlsp2p {
namespace dev {
namespace demux {

constexpr int kPkt = 188;
// status bits (runtime/ts.hpp)
constexpr uint32_t kBadSync = 1, kNoPat = 2, kNoPmt = 4, kPesOverflow = 8, kPesHeaderError = 16, kBadLength = 32;
// look-back granule states: {state:2 | PES count:30 | bytes:32}; 0 = not yet published
constexpr uint64_t kAgg = 1ull << 62, kIncl = 2ull << 62;

// per-packet meta word of the split demux (scan -> gather / place): class (2b, 3 = none) |
// payload start (8b) << 2 | payload len (8b) << 10 | PES start (1b) << 18
__device__ __forceinline__ uint32_t pack_meta(int c, int ps, int len, int pes) {
  return static_cast<uint32_t>(c & 3) | (static_cast<uint32_t>(ps) << 2) | (static_cast<uint32_t>(len) << 10) |
         (static_cast<uint32_t>(pes) << 18);
}

__device__ __forceinline__ int64_t pts5(uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3, uint32_t b4) {
  return (int64_t((b0 >> 1) & 0x07) << 30) | (int64_t(b1) << 22) | (int64_t(b2 >> 1) << 15) | (int64_t(b3) << 7) |
         int64_t(b4 >> 1);
}

// Wave64 inclusive prefix sum on the DPP paths (row shifts, then the row broadcasts): VALU
// only — a __shfl_up scan is ds_bpermute traffic through the LDS pipeline.
__device__ __forceinline__ uint32_t dpp_scan(uint32_t v) {
  int x = static_cast<int>(v);
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return static_cast<uint32_t>(x);
}
__device__ __forceinline__ uint32_t dpp_sum(uint32_t v) {
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(dpp_scan(v)), 63));
}

// agent-scope 8-byte granules (stores and loads bypass the non-coherent L1; the value is
// its own ready flag)
__device__ __forceinline__ void gstore(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t gload(uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One TS packet's header as the oracle reads it (runtime/ts.cpp demux_segment), from the
// packet's first dword and the 20 bytes at its payload start `s` (h: five funnel-aligned
// dwords).  c: 0 video, 1 audio, 2 id3, 3 none; ps / len: payload start / length after any
// PES header; pesf: a PES starts here.
struct Pkt {
  int c, ps, len, pesf;
  int64_t pts, dts;
  uint32_t err;
};
__device__ __forceinline__ Pkt parse_pkt(bool valid, uint32_t w0, const uint32_t* h, int s, int p0, int p1, int p2) {
  Pkt r{3, 0, 0, 0, -1, -1, 0};
  if (!valid) return r;
  if ((w0 & 0xff) != 0x47) {
    r.err = kBadSync;
    return r;
  }
  const int b1 = (w0 >> 8) & 0xff, b2 = (w0 >> 16) & 0xff, b3 = w0 >> 24;
  const int pid = ((b1 & 0x1f) << 8) | b2;
  const int cls = (p0 >= 0 && pid == p0) ? 0 : (p1 >= 0 && pid == p1) ? 1 : (p2 >= 0 && pid == p2) ? 2 : 3;
  const int afc = (b3 >> 4) & 3;
  if (cls == 3 || !(afc & 1)) return r;
  if (s > kPkt) {
    r.err = kBadLength;
    return r;
  }
  int l = kPkt - s;
  if (b1 & 0x40) {
    const uint32_t h0 = h[0], h1 = h[1], h2 = h[2], h3 = h[3], h4 = h[4];
    const uint32_t h7 = h1 >> 24, h8 = h2 & 0xff;
    if (l < 9 || (h0 & 0xffffff) != 0x010000 || 9 + static_cast<int>(h8) > l) {
      r.err = kPesHeaderError;
      return r;
    }
    r.pts = ((h7 & 0x80) && l >= 14) ? pts5((h2 >> 8) & 0xff, (h2 >> 16) & 0xff, h2 >> 24, h3 & 0xff, (h3 >> 8) & 0xff)
                                     : -1;
    r.dts = ((h7 & 0xC0) == 0xC0 && l >= 19)
                ? pts5((h3 >> 16) & 0xff, h3 >> 24, h4 & 0xff, (h4 >> 8) & 0xff, (h4 >> 16) & 0xff)
                : -1;
    r.pesf = 1;
    s += 9 + static_cast<int>(h8);
    l -= 9 + static_cast<int>(h8);
  }
  r.c = cls;
  r.ps = s;
  r.len = l;
  return r;
}

// Parse the packet at LDS dword `pw` (packet start, dword aligned): two LDS round trips —
// the header dwords, then five funnelled dwords at the payload start.
__device__ __forceinline__ Pkt parse_lds(bool valid, const uint32_t* pw, int p0, int p1, int p2) {
  const uint32_t w0 = pw[0], w1 = pw[1];
  const int afc = (w0 >> 28) & 3;
  const int s = 4 + ((afc & 2) ? 1 + static_cast<int>(w1 & 0xff) : 0);
  const int at = s <= kPkt ? s : 0;
  const uint32_t* w = pw + (at >> 2);
  uint32_t hw[6];
#pragma unroll
  for (int m = 0; m < 6; ++m) hw[m] = w[m];
  uint32_t h[5];
#pragma unroll
  for (int m = 0; m < 5; ++m) h[m] = __builtin_amdgcn_alignbyte(hw[m + 1], hw[m], static_cast<uint32_t>(at & 3));
  return parse_pkt(valid, w0, h, s, p0, p1, p2);
}

// Decoupled look-back over `look` (three class granules per tile): the exclusive prefix
// (bytes, PES) per class of tile `t`, summing predecessors back to each class's nearest
// inclusive prefix; tiles before `tile0` (the segment's first) count as an inclusive zero.
// One wave, four windows of 64 predecessors per round trip.  Bounded: a predecessor that
// never publishes sets *timeout and returns what it has.
__device__ __forceinline__ void look_back(uint64_t* look, int64_t t, int64_t tile0, int lane, unsigned int* timeout,
                                          uint32_t spin_limit, int64_t exb[3], int64_t exq[3]) {
  constexpr int kW = 4;
  exb[0] = exb[1] = exb[2] = 0;
  exq[0] = exq[1] = exq[2] = 0;
  uint32_t open = 7;  // classes still summing back
  int64_t win = t - 1;
  uint32_t spins = 0;
  while (open) {
    uint64_t g[kW][3];
#pragma unroll
    for (int w = 0; w < kW; ++w) {
      const int64_t pt = win - 64 * w - lane;
#pragma unroll
      for (int k = 0; k < 3; ++k) g[w][k] = pt < tile0 ? kIncl : gload(look + 3 * pt + k);
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
      if (++spins > spin_limit) {
        if (lane == 0) atomicOr(timeout, 1u);
        return;
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
}

}  // namespace demux
}  // namespace dev
}  // namespace hlsp2p
