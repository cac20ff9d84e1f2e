// MPEG-TS demux of a batch of decrypted segments — CDNA4 / gfx950.
//
// Output contract (identical to the CPU oracle runtime/ts.cpp demux_segment):
//   es:   per segment, [video ES | audio ES | id3 ES] written at es_off[seg]
//   pes:  int64[seg][3 classes][max_pes][3] = (ES byte offset, PTS, DTS)  (-1 = absent)
//   info: int64[seg][16] (status bits, PIDs, packet count, per-class bytes / PES counts)
//
// Four launches, no host round trip (segment lengths come from the decrypt kernel's
// on-device out_len):
//   1. ts_psi_kernel     — one wave per segment: PAT -> PMT PID, PMT -> ES PIDs/types
//                          (first 64 packets), zero-inits info / PES tables.
//   2. ts_scan_kernel    — one lane per 188-byte packet: sync check, PID class, payload
//                          start/len, PES header (PTS/DTS, header skip); per-256-packet
//                          block sums of (payload bytes, PES starts) per class.
//   3. ts_prefix_kernel  — one wave per segment: exclusive block prefixes + segment totals.
//   4. ts_gather_kernel  — same grid as the scan: the block's packets are staged in LDS by
//                          LDS-DMA, packed in-wave scans + the block prefix give every packet
//                          its ES destination, and 16-lane groups copy four payloads per wave
//                          iteration with dword-aligned stores (v_alignbyte funnel for the
//                          unaligned LDS source).
#include "common.h"

namespace hlsp2p {
namespace dev {

constexpr int kPkt = 188;
constexpr int kTsThreads = 256;
constexpr int kClasses = 3;
constexpr int kInfo = 24;
constexpr int kPsiScan = 64;
// info slots / status bits (must match runtime/ts.hpp)
constexpr int kStatus = 0, kPmtPid = 1, kVideoPid = 2, kNumPackets = 5, kBytes0 = 6, kPes0 = 9, kVideoType = 12,
              kAudioType = 13, kPayloadBytes = 14, kFirstPts = 16, kLastPts = 19, kAudioEsOffset = 22,
              kId3EsOffset = 23;
constexpr int64_t kBadSync = 1, kNoPat = 2, kNoPmt = 4, kPesOverflow = 8, kPesHeaderError = 16, kBadLength = 32;

__device__ __forceinline__ int64_t read_pts(const uint8_t* p) {
  return (int64_t((p[0] >> 1) & 0x07) << 30) | (int64_t(p[1]) << 22) | (int64_t(p[2] >> 1) << 15) |
         (int64_t(p[3]) << 7) | int64_t(p[4] >> 1);
}

__device__ __forceinline__ int64_t seg_length(const int64_t* len_dev, int seg) {
  const int64_t n = len_dev[seg];
  return n < 0 ? 0 : n;
}

// ---------------------------------------------------------------- 1. PSI
__global__ __launch_bounds__(64) void ts_psi_kernel(const uint8_t* __restrict__ buf, const int64_t* __restrict__ seg_off,
                                                    const int64_t* __restrict__ seg_len, int64_t* __restrict__ info,
                                                    int64_t* __restrict__ pes, int64_t max_pes) {
  const int seg = blockIdx.x;
  const int lane = threadIdx.x;
  int64_t* inf = info + static_cast<int64_t>(seg) * kInfo;
  int64_t* pe = pes + static_cast<int64_t>(seg) * kClasses * max_pes * 3;
  for (int64_t i = lane; i < static_cast<int64_t>(kClasses) * max_pes * 3; i += 64) pe[i] = -1;
  if (lane != 0) return;
  const int64_t raw_len = seg_len[seg];
  const int64_t n = raw_len < 0 ? 0 : raw_len;
  const uint8_t* d = buf + seg_off[seg];
  const int64_t np = n / kPkt;
  int64_t status = (raw_len < 0 || n % kPkt) ? kBadLength : 0;
  int pmt_pid = -1, vpid = -1, apid = -1, ipid = -1, vtype = 0, atype = 0;
  const int64_t scan = np < kPsiScan ? np : kPsiScan;
  for (int64_t i = 0; i < scan && pmt_pid < 0; ++i) {
    const uint8_t* p = d + i * kPkt;
    if (p[0] != 0x47) continue;
    const int pid = ((p[1] & 0x1f) << 8) | p[2];
    if (pid != 0 || !(p[1] & 0x40)) continue;
    const int afc = (p[3] >> 4) & 3;
    int ps = 4 + ((afc & 2) ? 1 + p[4] : 0);
    if (!(afc & 1) || ps >= kPkt) continue;
    ps += 1 + p[ps];
    if (ps + 8 > kPkt || p[ps] != 0x00) continue;
    const int slen = ((p[ps + 1] & 0x0f) << 8) | p[ps + 2];
    const int end = ps + 3 + slen - 4 < kPkt ? ps + 3 + slen - 4 : kPkt;
    for (int q = ps + 8; q + 4 <= end; q += 4) {
      const int prog = (p[q] << 8) | p[q + 1];
      if (prog != 0) {
        pmt_pid = ((p[q + 2] & 0x1f) << 8) | p[q + 3];
        break;
      }
    }
  }
  if (pmt_pid < 0) status |= kNoPat;
  bool pmt_found = false;
  for (int64_t i = 0; i < scan && pmt_pid >= 0 && !pmt_found; ++i) {
    const uint8_t* p = d + i * kPkt;
    if (p[0] != 0x47) continue;
    const int pid = ((p[1] & 0x1f) << 8) | p[2];
    if (pid != pmt_pid || !(p[1] & 0x40)) continue;
    const int afc = (p[3] >> 4) & 3;
    int ps = 4 + ((afc & 2) ? 1 + p[4] : 0);
    if (!(afc & 1) || ps >= kPkt) continue;
    ps += 1 + p[ps];
    if (ps + 12 > kPkt || p[ps] != 0x02) continue;
    pmt_found = true;
    const int slen = ((p[ps + 1] & 0x0f) << 8) | p[ps + 2];
    const int end = ps + 3 + slen - 4 < kPkt ? ps + 3 + slen - 4 : kPkt;
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
  if (pmt_pid >= 0 && !pmt_found) status |= kNoPmt;
  for (int k = 0; k < kInfo; ++k) inf[k] = 0;
  inf[kStatus] = status;
  inf[kPmtPid] = pmt_pid;
  inf[kVideoPid] = vpid;
  inf[kVideoPid + 1] = apid;
  inf[kVideoPid + 2] = ipid;
  inf[kNumPackets] = np;
  inf[kVideoType] = vtype;
  inf[kAudioType] = atype;
  for (int c = 0; c < kClasses; ++c) {
    inf[kFirstPts + c] = -1;
    inf[kLastPts + c] = -1;
  }
}

// per-packet meta word (scan -> gather): class (2b, 3 = none) | payload start (8b) << 2 |
// payload len (8b) << 10 | PES start (1b) << 18
__device__ __forceinline__ uint32_t pack_meta(int c, int ps, int len, int pes) {
  return static_cast<uint32_t>(c & 3) | (static_cast<uint32_t>(ps) << 2) | (static_cast<uint32_t>(len) << 10) |
         (static_cast<uint32_t>(pes) << 18);
}

// ---------------------------------------------------------------- 2. scan
// Inclusive prefix sum over the wave64 in six DPP-modified moves and adds, no LDS traffic
// (a __shfl_up ladder is six ds_bpermute round trips): row_shr:1/2/4/8 scan each 16-lane row
// (bound_ctrl fills 0 past the row start), row_bcast:15 adds row 0's / row 2's total to rows 1
// and 3, row_bcast:31 adds rows 0-1's total to rows 2 and 3.
__device__ __forceinline__ uint32_t wave_scan_dpp(uint32_t v) {
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x111, 0xf, 0xf, true));
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x112, 0xf, 0xf, true));
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x114, 0xf, 0xf, true));
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x118, 0xf, 0xf, true));
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x142, 0xa, 0xf, false));
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x143, 0xc, 0xf, false));
  return v;
}
// the wave's total (lane 63 of the inclusive scan), wave-uniform
__device__ __forceinline__ uint32_t wave_sum_dpp(uint32_t v) {
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(wave_scan_dpp(v)), 63));
}
__device__ __forceinline__ int wave_incl_scan(int v, int /*lane*/) {
  return static_cast<int>(wave_scan_dpp(static_cast<uint32_t>(v)));
}

// hdr_rec / hdr_off (optional, from the decrypt: aes_cbc.hip AesHdr): record p of a segment is
// the 16-byte block holding packet p's header at byte (188 p) mod 16 -- read densely instead of
// one plaintext line per packet; byte 4 (adaptation-field length) comes from it too unless the
// header sits at byte 12, and PES headers still come from the plaintext (a few % of packets).
//
// One workgroup scans kScanBlocks consecutive 256-packet blocks (the unit of blk_sums): the
// segment lookup and PID loads are paid once, and every block's header loads are issued before
// the first block is parsed (a workgroup per block was a chain of dependent loads per 256
// packets: latency, not bandwidth, set the scan's time).
constexpr int kScanBlocks = 4;

struct ScanPkt {
  uint32_t hdr;
  int b4;  // byte 4 when known (-1: read it from the plaintext)
};

__device__ __forceinline__ ScanPkt scan_load(const uint8_t* __restrict__ p, const uint4* __restrict__ rec, int64_t pk) {
  ScanPkt r;
  r.b4 = -1;
  if (rec != nullptr) {
    const uint4 v = *rec;
    const int o = static_cast<int>((pk * kPkt) & 15);  // 0, 4, 8 or 12
    r.hdr = o == 0 ? v.x : o == 4 ? v.y : o == 8 ? v.z : v.w;
    if (o < 12) r.b4 = static_cast<int>((o == 0 ? v.y : o == 4 ? v.z : v.w) & 0xff);
  } else {
    r.hdr = *reinterpret_cast<const uint32_t*>(p);  // packets are 4-byte aligned
  }
  return r;
}

__global__ __launch_bounds__(kTsThreads) void ts_scan_kernel(
    const uint8_t* __restrict__ buf, const int64_t* __restrict__ seg_off, const int64_t* __restrict__ seg_len,
    const int64_t* __restrict__ blk_prefix, int nseg, int64_t total_blocks, int64_t* __restrict__ info,
    uint32_t* __restrict__ meta, int64_t* __restrict__ pts_dts, int32_t* __restrict__ blk_sums,
    const uint4* __restrict__ hdr_rec, const int64_t* __restrict__ hdr_off) {
  __shared__ int32_t s_sum[kScanBlocks][2 * kClasses];
  __shared__ int32_t s_err[kScanBlocks];
  const int tid = threadIdx.x;
  const int64_t gb0 = static_cast<int64_t>(blockIdx.x) * kScanBlocks;
  const int nb = static_cast<int>(total_blocks - gb0 < kScanBlocks ? total_blocks - gb0 : kScanBlocks);
  if (tid < kScanBlocks * 2 * kClasses) (&s_sum[0][0])[tid] = 0;
  if (tid < kScanBlocks) s_err[tid] = 0;
  // the segment of each block (uniform), then every block's header load in flight at once
  int segs[kScanBlocks];
  int seg = find_seg_wave(blk_prefix, nseg, gb0);
  ScanPkt pkt[kScanBlocks];
  int64_t pks[kScanBlocks];
  const uint8_t* pp[kScanBlocks];
#pragma unroll
  for (int u = 0; u < kScanBlocks; ++u) {
    segs[u] = seg;
    pks[u] = -1;
    if (u < nb) {
      if (u > 0) {
        seg = __builtin_amdgcn_readfirstlane(advance_seg(blk_prefix, seg, gb0 + u));
        segs[u] = seg;
      }
      const int64_t np = seg_length(seg_len, seg) / kPkt;
      const int64_t pk = (gb0 + u - blk_prefix[seg]) * kTsThreads + tid;
      if (pk < np) {
        pks[u] = pk;
        pp[u] = buf + seg_off[seg] + pk * kPkt;
        pkt[u] = scan_load(pp[u], hdr_rec != nullptr ? hdr_rec + hdr_off[seg] + pk : nullptr, pk);
      }
    }
  }
  // The bytes a packet's parse needs beyond its header record, loaded for every block before the
  // first block is parsed (issued per block inside the parse they were 2-3 dependent round trips
  // per block): byte 4 when the record does not hold it and an adaptation field is present,
  // then, for a payload-unit start, the PES header's first 20 bytes as 6 dwords realigned in
  // registers (dwords past the packet read as 0; the parse never uses bytes past its length).
  int b4v[kScanBlocks];
#pragma unroll
  for (int u = 0; u < kScanBlocks; ++u) {
    b4v[u] = 0;
    if (pks[u] >= 0) {
      const uint32_t hdr = pkt[u].hdr;
      const int afc = (hdr >> 28) & 3;
      b4v[u] = pkt[u].b4 >= 0 ? pkt[u].b4 : ((afc & 2) ? static_cast<int>(pp[u][4]) : 0);
    }
  }
  uint32_t hw[kScanBlocks][5];
#pragma unroll
  for (int u = 0; u < kScanBlocks; ++u) {
#pragma unroll
    for (int k = 0; k < 5; ++k) hw[u][k] = 0;
    if (pks[u] >= 0) {
      const uint32_t hdr = pkt[u].hdr;
      const int afc = (hdr >> 28) & 3, b1 = (hdr >> 8) & 0xff;
      const int s0 = 4 + ((afc & 2) ? 1 + b4v[u] : 0);
      if ((hdr & 0xff) == 0x47 && (b1 & 0x40) && (afc & 1) && s0 + 9 <= kPkt) {
        const uint8_t* h = pp[u] + s0;
        const uint32_t* w = reinterpret_cast<const uint32_t*>(reinterpret_cast<uintptr_t>(h) & ~uintptr_t(3));
        const uint32_t* wend = reinterpret_cast<const uint32_t*>(pp[u] + kPkt);  // packets are 4-byte aligned
        uint32_t d[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) d[k] = w + k < wend ? w[k] : 0u;
        const uint32_t mis = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(h) & 3);
#pragma unroll
        for (int k = 0; k < 5; ++k) hw[u][k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], mis);
      }
    }
  }
  __syncthreads();
  int cur = -1, cpid0 = -1, cpid1 = -1, cpid2 = -1;
#pragma unroll
  for (int u = 0; u < kScanBlocks; ++u) {
    if (u >= nb) break;
    if (segs[u] != cur) {
      cur = segs[u];
      const int64_t* inf = info + static_cast<int64_t>(cur) * kInfo;
      cpid0 = static_cast<int>(inf[kVideoPid]);
      cpid1 = static_cast<int>(inf[kVideoPid + 1]);
      cpid2 = static_cast<int>(inf[kVideoPid + 2]);
    }
    const int64_t gpk = (gb0 + u) * kTsThreads + tid;  // global packet slot (meta index)
    int c = 3, ps = 0, len = 0, pes = 0;
    int err = 0;
    if (pks[u] >= 0) {
      const uint32_t hdr = pkt[u].hdr;
      const int sync = hdr & 0xff;
      const int b1 = (hdr >> 8) & 0xff, b2 = (hdr >> 16) & 0xff, b3 = hdr >> 24;
      if (sync != 0x47) {
        err |= static_cast<int>(kBadSync);
      } else {
        const int pid = ((b1 & 0x1f) << 8) | b2;
        const int cls = (cpid0 >= 0 && pid == cpid0) ? 0 : (cpid1 >= 0 && pid == cpid1) ? 1 : (cpid2 >= 0 && pid == cpid2) ? 2 : 3;
        const int afc = (b3 >> 4) & 3;
        if (cls < 3 && (afc & 1)) {
          int s = 4 + ((afc & 2) ? 1 + b4v[u] : 0);
          if (s > kPkt) {
            err |= static_cast<int>(kBadLength);
          } else {
            int l = kPkt - s;
            bool ok = true;
            if (b1 & 0x40) {
#define HB(i) static_cast<int>((hw[u][(i) >> 2] >> (8 * ((i) & 3))) & 0xffu)
              if (l < 9 || HB(0) != 0 || HB(1) != 0 || HB(2) != 1 || 9 + HB(8) > l) {
                err |= static_cast<int>(kPesHeaderError);
                ok = false;
              } else {
                const int f7 = HB(7);
                const int64_t pts = ((f7 & 0x80) && l >= 14)
                                        ? (int64_t((HB(9) >> 1) & 0x07) << 30) | (int64_t(HB(10)) << 22) |
                                              (int64_t(HB(11) >> 1) << 15) | (int64_t(HB(12)) << 7) | int64_t(HB(13) >> 1)
                                        : -1;
                const int64_t dts = ((f7 & 0xC0) == 0xC0 && l >= 19)
                                        ? (int64_t((HB(14) >> 1) & 0x07) << 30) | (int64_t(HB(15)) << 22) |
                                              (int64_t(HB(16) >> 1) << 15) | (int64_t(HB(17)) << 7) | int64_t(HB(18) >> 1)
                                        : -1;
                pts_dts[2 * gpk] = pts;
                pts_dts[2 * gpk + 1] = dts;
                pes = 1;
                s += 9 + HB(8);
                l -= 9 + HB(8);
              }
#undef HB
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
    meta[gpk] = pack_meta(c, ps, len, pes);
    // wave-level sums per class (bytes < 2^16 and PES starts packed in one word), then one
    // LDS atomic per wave per class
#pragma unroll
    for (int k = 0; k < kClasses; ++k) {
      const uint32_t v = wave_sum_dpp((c == k) ? static_cast<uint32_t>(len | (pes << 16)) : 0u);
      if ((tid & 63) == 0 && v) {
        atomicAdd(&s_sum[u][2 * k], static_cast<int>(v & 0xffff));
        atomicAdd(&s_sum[u][2 * k + 1], static_cast<int>(v >> 16));
      }
    }
    if (err) atomicOr(&s_err[u], err);
  }
  __syncthreads();
  if (tid < nb * 2 * kClasses) {
    const int u = tid / (2 * kClasses), k = tid % (2 * kClasses);
    blk_sums[(gb0 + u) * 2 * kClasses + k] = s_sum[u][k];
  }
  if (tid == 0) {
    for (int u = 0; u < nb; ++u)
      if (s_err[u])
        atomicOr(reinterpret_cast<unsigned long long*>(info + static_cast<int64_t>(segs[u]) * kInfo + kStatus),
                 static_cast<unsigned long long>(s_err[u]));
  }
}

// ---------------------------------------------------------------- 2b. block prefix
// One wave per segment turns the scan's block sums into exclusive per-block prefixes
// (blk_pre) and segment totals (seg_tot, info), so a gather block reads its 12 numbers
// instead of re-reducing all of its segment's block sums.  (A last-arriving-block variant
// inside the scan kernel needed an agent-scope release per block: on gfx950 that writes
// back the XCD's L2, and the scan took 5x longer.)
__global__ __launch_bounds__(64) void ts_prefix_kernel(const int64_t* __restrict__ blk_prefix,
                                                       const int32_t* __restrict__ blk_sums,
                                                       int32_t* __restrict__ blk_pre, int32_t* __restrict__ seg_tot,
                                                       int64_t* __restrict__ info, int64_t max_pes) {
  const int seg = blockIdx.x;
  const int lane = threadIdx.x;
  const int64_t b0 = blk_prefix[seg];
  const int64_t nblk = blk_prefix[seg + 1] - b0;
  int carry[2 * kClasses] = {0, 0, 0, 0, 0, 0};
  for (int64_t bb = 0; bb < nblk; bb += 64) {
    const int64_t b = bb + lane;
    int v[2 * kClasses];
#pragma unroll
    for (int k = 0; k < 2 * kClasses; ++k) v[k] = b < nblk ? blk_sums[(b0 + b) * 2 * kClasses + k] : 0;
#pragma unroll
    for (int k = 0; k < 2 * kClasses; ++k) {
      const int inc = wave_incl_scan(v[k], lane);
      if (b < nblk) blk_pre[(b0 + b) * 2 * kClasses + k] = carry[k] + inc - v[k];
      carry[k] += __shfl(inc, 63);
    }
  }
  if (lane == 0) {  // carry[] is wave-uniform
#pragma unroll
    for (int k = 0; k < 2 * kClasses; ++k) seg_tot[seg * 2 * kClasses + k] = carry[k];
    int64_t* inf = info + static_cast<int64_t>(seg) * kInfo;
    int64_t over = 0;
    for (int k = 0; k < kClasses; ++k) {
      inf[kBytes0 + k] = carry[2 * k];
      inf[kPes0 + k] = carry[2 * k + 1];
      if (carry[2 * k + 1] > max_pes) over = kPesOverflow;
    }
    inf[kPayloadBytes] = static_cast<int64_t>(carry[0]) + carry[2] + carry[4];
    inf[kAudioEsOffset] = carry[0];  // [video | audio | id3] packed
    inf[kId3EsOffset] = static_cast<int64_t>(carry[0]) + carry[2];
    if (over) atomicOr(reinterpret_cast<unsigned long long*>(inf + kStatus), static_cast<unsigned long long>(over));
  }
}

// ---------------------------------------------------------------- 3. gather
__global__ __launch_bounds__(kTsThreads) void ts_gather_kernel(
    const uint8_t* __restrict__ buf, const int64_t* __restrict__ seg_off, const int64_t* __restrict__ seg_len,
    const int64_t* __restrict__ blk_prefix, int nseg, const uint32_t* __restrict__ meta,
    const int64_t* __restrict__ pts_dts, const int32_t* __restrict__ blk_pre, const int32_t* __restrict__ seg_tot,
    uint8_t* __restrict__ es, const int64_t* __restrict__ es_off, int64_t* __restrict__ pes, int64_t max_pes,
    int64_t* __restrict__ info) {
  // this block's 256 packets (47 KiB), rounded up to whole 16-byte-per-lane LDS-DMA waves
  constexpr int kStageVec = (kTsThreads * kPkt + 16 * kTsThreads - 1) / (16 * kTsThreads);  // 12
  __shared__ __attribute__((aligned(16))) uint32_t s_pk[kStageVec * kTsThreads * 4];
  __shared__ uint32_t s_wave[4][3];      // per-wave packed scan totals
  __shared__ uint8_t s_order[4][64];      // per wave: active-packet rank -> lane
  const int64_t gblk = blockIdx.x;
  const int seg = find_seg_wave(blk_prefix, nseg, gblk);
  const int64_t blk = gblk - blk_prefix[seg];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // Stage the block's packets (<= 47 KiB) into LDS by LDS-DMA: 12 global_load_lds_dwordx4 per
  // wave (1 KiB each, lane-linear image), all in flight at once and drained by the barrier.
  // (A register-staged loop compiled to load / vmcnt(0) / ds_write per 16 B: ~12 serialised
  // HBM round trips per block.)
  {
    const int64_t np = seg_length(seg_len, seg) / kPkt;
    const int64_t first = blk * kTsThreads;
    const int64_t npk = np - first < kTsThreads ? (np - first > 0 ? np - first : 0) : kTsThreads;
    const int nvec = static_cast<int>((npk * kPkt + 15) / 16);
    const uint8_t* g = buf + seg_off[seg] + first * kPkt;
    const int last = nvec - 1;
#pragma unroll
    for (int k = 0; k < kStageVec; ++k) {
      const int wbase = k * kTsThreads + wave * 64;  // wave-uniform
      if (wbase < nvec) {
        const int i = wbase + lane < last ? wbase + lane : last;  // tail lanes re-read the last vector
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(g + 16 * static_cast<int64_t>(i)),
                                         (__attribute__((address_space(3))) void*)(
                                             reinterpret_cast<uint8_t*>(s_pk) + 16 * wbase),
                                         16, 0, 0);
      }
    }
  }
  const int64_t gpk = gblk * kTsThreads + tid;
  const uint32_t m = meta[gpk];
  // block prefix and segment totals: computed once per segment by the scan kernel's last
  // block; uniform addresses, so these are scalar loads in flight with the stage
  int32_t pre[2 * kClasses], tot[2 * kClasses];
#pragma unroll
  for (int k = 0; k < 2 * kClasses; ++k) {
    pre[k] = blk_pre[gblk * 2 * kClasses + k];
    tot[k] = seg_tot[seg * 2 * kClasses + k];
  }
  const int c = m & 3, ps = (m >> 2) & 0xff, len = (m >> 10) & 0xff, pes_flag = (m >> 18) & 1;
  // In-wave inclusive scans of (bytes, PES starts) per class, packed three to a word (wave
  // totals: bytes <= 64 x 184 < 2^16, PES starts <= 64 < 2^8): 3 scans instead of 6.
  const uint32_t lb = static_cast<uint32_t>(len), pf = static_cast<uint32_t>(pes_flag);
  uint32_t sA = (c == 0 ? lb : 0u) | ((c == 1 ? lb : 0u) << 16);
  uint32_t sB = (c == 2 ? lb : 0u) | ((c == 0 ? pf : 0u) << 16) | ((c == 1 ? pf : 0u) << 24);
  uint32_t sC = c == 2 ? pf : 0u;
  sA = wave_scan_dpp(sA);
  sB = wave_scan_dpp(sB);
  sC = wave_scan_dpp(sC);
  if (lane == 63) {
    s_wave[wave][0] = sA;
    s_wave[wave][1] = sB;
    s_wave[wave][2] = sC;
  }
  __syncthreads();
  int64_t dst_b = 0, pes_idx = 0;
  if (c < 3) {
    uint32_t wA = 0, wB = 0, wC = 0;  // earlier waves' packed totals (no field overflows: <= 256 packets)
    for (int w = 0; w < wave; ++w) {
      wA += s_wave[w][0];
      wB += s_wave[w][1];
      wC += s_wave[w][2];
    }
    sA += wA;
    sB += wB;
    sC += wC;
    const uint32_t inc_b = c == 0 ? (sA & 0xffff) : c == 1 ? (sA >> 16) : (sB & 0xffff);
    const uint32_t inc_p = c == 0 ? ((sB >> 16) & 0xff) : c == 1 ? (sB >> 24) : sC;
    const int64_t class_base = (c >= 1 ? tot[0] : 0) + (c >= 2 ? tot[2] : 0);
    const int64_t es_in_class = static_cast<int64_t>(pre[2 * c]) + inc_b - len;  // exclusive
    dst_b = class_base + es_in_class;
    pes_idx = static_cast<int64_t>(pre[2 * c + 1]) + inc_p - pes_flag;
    if (pes_flag) {
      const int64_t tot_pes = tot[2 * c + 1];
      int64_t* infc = info + static_cast<int64_t>(seg) * kInfo;
      if (pes_idx == 0) infc[kFirstPts + c] = pts_dts[2 * gpk];
      if (pes_idx == tot_pes - 1) infc[kLastPts + c] = pts_dts[2 * gpk];
      if (pes_idx < max_pes) {
        int64_t* r = pes + ((static_cast<int64_t>(seg) * kClasses + c) * max_pes + pes_idx) * 3;
        r[0] = es_in_class;
        r[1] = pts_dts[2 * gpk];
        r[2] = pts_dts[2 * gpk + 1];
      }
    }
  }
  // Copy out of the LDS-staged block, FIVE packets per wave iteration: each 12-lane group
  // moves one payload (<= 184 B = 46 dwords): lane `sub` funnels body dwords 4sub..4sub+3 out
  // of 5 LDS dwords (v_alignbyte, shift 0 passes the low word) and writes them with ONE
  // dwordx4 store to a dword-aligned address; byte stores only for the <= 3 + 3 unaligned
  // head/tail bytes and a short last quad.  Active packets are ranked with mbcnt; s_order
  // maps rank -> lane so group g of iteration i takes rank 5i+g.  (Four 16-lane groups with
  // three dword stores per lane: 20 % slower.)
  const uint8_t* s_bytes = reinterpret_cast<const uint8_t*>(s_pk);
  uint8_t* ebase = es + es_off[seg];
  const bool act = c < 3 && len > 0;
  const uint64_t amask = __ballot(act);
  const int nact = __popcll(amask);
  if (act) {
    const int rank = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(amask >> 32),
                                               __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(amask), 0));
    s_order[wave][rank] = static_cast<uint8_t>(lane);
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  // ES stores go through a buffer resource: buffer_store_dwordx4 at a dword-aligned offset
  // (a plain 16-byte store at 4-byte alignment is split by the compiler into dwordx3 + dword)
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t es_rsrc = __builtin_amdgcn_make_buffer_rsrc(ebase, 0, 0x7fffffff, 0x00020000);
  const int dst32 = static_cast<int>(dst_b);  // within one segment's ES (< 2 GiB)
  const int grp = lane / 12, sub = lane - 12 * grp;  // groups 0..4; lanes 60..63 idle
  for (int base = 0; base < nact; base += 5) {
    const int r = base + grp;
    const bool valid = grp < 5 && r < nact;
    const int j = valid ? s_order[wave][r] : 0;
    const int jlen_all = __shfl(len, j);
    const int jps = __shfl(ps, j);
    const int jdst = __shfl(dst32, j);
    const int jlen = valid ? jlen_all : 0;
    const int s = (wave * 64 + j) * kPkt + jps;  // LDS byte offset of the payload
    uint8_t* d = ebase + jdst;
    const int mis = static_cast<int>((4 - (reinterpret_cast<uintptr_t>(d) & 3)) & 3);
    const int head = mis < jlen ? mis : jlen;
    const int body = (jlen - head) >> 2;
    const int tail = jlen - head - 4 * body;
    if (sub < head) d[sub] = s_bytes[s + sub];
    const int k0 = 4 * sub;
    if (k0 < body) {
      const int a = s + head + 4 * k0;
      const uint32_t sh = static_cast<uint32_t>(a & 3);
      const uint32_t* w = s_pk + (a >> 2);
      const uint32_t x0 = w[0], x1 = w[1], x2 = w[2], x3 = w[3], x4 = w[4];
      const uint32_t o0 = __builtin_amdgcn_alignbyte(x1, x0, sh), o1 = __builtin_amdgcn_alignbyte(x2, x1, sh),
                     o2 = __builtin_amdgcn_alignbyte(x3, x2, sh), o3 = __builtin_amdgcn_alignbyte(x4, x3, sh);
      uint32_t* dw = reinterpret_cast<uint32_t*>(d + head) + k0;
      if (k0 + 4 <= body) {
        const v4u q = {o0, o1, o2, o3};
        __builtin_amdgcn_raw_buffer_store_b128(q, es_rsrc, jdst + head + 4 * k0, 0, 0);
      } else {
        dw[0] = o0;
        if (k0 + 1 < body) dw[1] = o1;
        if (k0 + 2 < body) dw[2] = o2;
      }
    }
    if (sub < tail) d[head + 4 * body + sub] = s_bytes[s + head + 4 * body + sub];
  }
}


hipError_t launch_ts_demux(const uint8_t* buf, const int64_t* seg_off, const int64_t* seg_len,
                           const int64_t* blk_prefix, int nseg, int64_t total_blocks, uint32_t* meta,
                           int64_t* pts_dts, int32_t* aux, uint8_t* es, const int64_t* es_off, int64_t* pes,
                           int64_t max_pes, int64_t* info, hipStream_t stream, const void* hdr_rec,
                           const int64_t* hdr_off) {
  if (nseg <= 0) return hipSuccess;
  // aux (int32): [blk_sums: blocks x 6 | blk_pre: blocks x 6 | seg_tot: nseg x 6 | spare: nseg]
  int32_t* blk_sums = aux;
  int32_t* blk_pre = blk_sums + total_blocks * 2 * kClasses;
  int32_t* seg_tot = blk_pre + total_blocks * 2 * kClasses;
  hipLaunchKernelGGL(ts_psi_kernel, dim3(nseg), dim3(64), 0, stream, buf, seg_off, seg_len, info, pes, max_pes);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || total_blocks <= 0) return e;
  hipLaunchKernelGGL(ts_scan_kernel, dim3(static_cast<unsigned>((total_blocks + kScanBlocks - 1) / kScanBlocks)),
                     dim3(kTsThreads), 0, stream, buf, seg_off, seg_len, blk_prefix, nseg, total_blocks, info, meta,
                     pts_dts, blk_sums,
                     reinterpret_cast<const uint4*>(hdr_rec), hdr_rec != nullptr ? hdr_off : nullptr);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(ts_prefix_kernel, dim3(nseg), dim3(64), 0, stream, blk_prefix, blk_sums, blk_pre, seg_tot, info,
                     max_pes);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(ts_gather_kernel, dim3(static_cast<unsigned>(total_blocks)), dim3(kTsThreads), 0, stream, buf,
                     seg_off, seg_len, blk_prefix, nseg, meta, pts_dts, blk_pre, seg_tot, es, es_off, pes, max_pes,
                     info);
  return hipGetLastError();
}

}  // namespace dev
}  // namespace hlsp2p
