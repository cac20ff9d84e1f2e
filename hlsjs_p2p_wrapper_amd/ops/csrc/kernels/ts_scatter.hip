// Scatter demux of AES-128-CBC MPEG-TS segments (SURVEY §2.2 K10 + K11) — CDNA4 / gfx950.
//
// The split sequence decrypts every byte to a plaintext buffer in HBM and then re-reads it
// twice (header scan, payload gather).  Here the plaintext never exists in HBM: CBC
// decryption is random-access (P_i = D_K(C_i) ^ C_{i-1}), so the demux first learns where
// every payload byte goes from a sparse decrypt of the packet headers only, and the bulk
// decrypt then writes each payload byte straight to its elementary-stream position.
//
//   1. tsx_hdr_kernel   — one lane per group of 4 packets (752 B = 47 AES blocks): decrypt the
//                         5 blocks holding the 4 packet headers (bytes 0..4 of each packet:
//                         blocks 0, 11, 12, 23, 35 of the group) with the 160 KiB LDS table
//                         image, five independent chains per lane; one header word per packet.
//   2. tsx_psi_kernel   — one wave per segment: the plaintext length from the last block's
//                         PKCS#7 padding; PAT / PMT from the first packets whose headers say
//                         PID 0 / PMT PID (those packets decrypted whole, parsed as the oracle).
//   3. tsx_scan_kernel  — one lane per packet, from the header words: class, payload start and
//                         length; PES-starting packets decrypt the 2-3 blocks of their PES
//                         header (small LDS tables) for PTS / DTS / header length; per-block
//                         class sums (the split scan's output, without reading the plaintext).
//   4. ts_prefix_kernel — (ts_demux.hip) block prefixes and segment totals.
//   5. tsx_place_kernel — per packet: ES destination (in-wave scans + block prefix, as the
//                         split gather), PES table rows, first / last PTS; the packet's
//                         (ES bias, payload range) entry.
//   6. aes128_cbc_decrypt_kernel<true> — (aes_cbc.hip) the bulk decrypt at full rate; its
//                         epilogue stores every whole aligned ES dword of payload (dwordx4 for
//                         a block inside a payload) and leaves each run's <= 3 + 3 seam bytes.
//   7. tsx_seam_kernel  — one lane per packet: the seam bytes (shared ES dwords) as bytes.
//
// HBM traffic per segment: the header pass touches one 128 B line per packet (~0.7 of the
// segment), the bulk decrypt reads the ciphertext once and writes the ES once — against
// decrypt (read + write) + scan (~0.7) + gather (read + write) for the split sequence.
// Output contract: identical to the split sequence and the CPU oracle (runtime/ts.cpp).
#include "aes_dev.h"
#include "common.h"
#include "demux_dev.h"
#include "ts_scatter.h"

namespace hlsp2p {
namespace dev {

hipError_t launch_ts_prefix(const int64_t* blk_prefix, const int32_t* blk_sums, int32_t* blk_pre, int32_t* seg_tot,
                            int64_t* info, int64_t max_pes, int nseg, hipStream_t stream);
hipError_t launch_aes128_cbc_scatter(const uint8_t* src, const int64_t* src_off, const int64_t* blk_prefix,
                                     const int64_t* chunk_prefix, const uint32_t* drk, const uint32_t* ivw,
                                     const uint32_t* tdl, const uint8_t* isb, const uint2* place,
                                     const int64_t* pkt_base, const int64_t* pkt_slots, uint8_t* es,
                                     const int64_t* es_off, uint32_t* seam, int nseg, int64_t total_chunks,
                                     int num_cu, hipStream_t stream);

namespace {

constexpr int kPkt = 188;
constexpr int kClasses = 3;
constexpr int kInfo = 24;
constexpr int kPsiScan = 64;
using demux::kBadLength;
using demux::kNoPat;
using demux::kNoPmt;
constexpr int kThreads = 256;  // scan / place blocks: one lane per packet
// info slots (runtime/ts.hpp)
constexpr int kStatus = 0, kPmtPid = 1, kVideoPid = 2, kNumPackets = 5, kVideoType = 12, kAudioType = 13,
              kFirstPts = 16, kLastPts = 19;

// header word: b1 | b2 << 8 | bad sync << 16 | (b3 & 0xf0) << 16 | b4 << 24 (the continuity
// counter's bits carry the sync flag; the demux never reads them)
__device__ __forceinline__ uint32_t hdr_word(uint32_t w0, uint32_t b4) {
  const uint32_t bad = (w0 & 0xffu) != 0x47u ? 1u : 0u;
  return ((w0 >> 8) & 0xffffu) | (bad << 16) | (((w0 >> 24) & 0xf0u) << 16) | ((b4 & 0xffu) << 24);
}
// the packet's first dword as demux::parse_pkt reads it
__device__ __forceinline__ uint32_t hdr_w0(uint32_t h) {
  return (((h >> 16) & 1u) ? 0u : 0x47u) | ((h & 0xffffu) << 8) | ((h & 0x00f00000u) << 8);
}
__device__ __forceinline__ int hdr_pid(uint32_t h) { return static_cast<int>(((h & 0x1fu) << 8) | ((h >> 8) & 0xffu)); }
__device__ __forceinline__ int hdr_afc(uint32_t h) { return static_cast<int>((h >> 20) & 3u); }
__device__ __forceinline__ int hdr_payload_start(uint32_t h) {
  return 4 + ((hdr_afc(h) & 2) ? 1 + static_cast<int>(h >> 24) : 0);
}

// AES block offsets (within a 4-packet group) of the blocks holding packet k's bytes 0..4
__device__ __forceinline__ constexpr int group_block(int k) {
  return k == 0 ? 0 : k == 1 ? 11 : k == 2 ? 12 : k == 3 ? 23 : 35;
}

// ---------------------------------------------------------------- 1. headers
__global__ __launch_bounds__(kAesImageThreads, 1) void tsx_hdr_kernel(ScatterArgs a, int64_t per_wg) {
  __shared__ uint32_t s_tab[kTdDwords + kIsDwords];
  const int tid = threadIdx.x;
  aes_image_fill(s_tab, a.tdl, a.isb, tid);
  __syncthreads();
  const uint8_t* s_bytes = reinterpret_cast<const uint8_t*>(s_tab);
  uint32_t td_base[4], is_base;
  aes_image_bases(tid, td_base, is_base);
  const int lane = tid & 63;
  constexpr int kWaves = kAesImageThreads / 64;
  constexpr int kChains = 5;

  const int64_t begin = static_cast<int64_t>(blockIdx.x) * per_wg;
  const int64_t end = begin + per_wg < a.hdr_total_chunks ? begin + per_wg : a.hdr_total_chunks;
  int cur = -1;
  uint32_t rk[44];
  int64_t so = 0, cstart = 0, cend = 0, nb = 0, pbase = 0;
  for (int64_t ch = uniform64(begin + (tid >> 6)); ch < end; ch += kWaves) {
    if (cur < 0 || ch >= cend) {
      cur = cur < 0 ? find_seg_wave(a.hdr_chunks, a.nseg, ch)
                    : __builtin_amdgcn_readfirstlane(advance_seg(a.hdr_chunks, cur, ch));
#pragma unroll
      for (int k = 0; k < 44; ++k) rk[k] = a.drk[cur * 44 + k];
      so = a.src_off[cur];
      cstart = a.hdr_chunks[cur];
      cend = a.hdr_chunks[cur + 1];
      nb = a.aes_blk[cur + 1] - a.aes_blk[cur];
      pbase = a.pkt_base[cur];
    }
    const int64_t g = (ch - cstart) * kScatterChunkGroups + lane;  // this lane's group
    const int64_t npk = nb * 16 / kPkt;  // packets entirely inside the ciphertext
    const int64_t gb = 47 * g;
    const uint4* cs = reinterpret_cast<const uint4*>(a.src + so);
    uint4 c[kChains], pv[kChains];
#pragma unroll
    for (int k = 0; k < kChains; ++k) {
      const int64_t b = gb + group_block(k);
      c[k] = b < nb ? cs[b] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < kChains; ++k) {
      const int64_t b = gb + group_block(k);
      pv[k] = b == 0 ? reinterpret_cast<const uint4*>(a.ivw)[cur] : (b < nb ? cs[b - 1] : make_uint4(0, 0, 0, 0));
    }
    uint32_t st[kChains][4];
#pragma unroll
    for (int k = 0; k < kChains; ++k) {
      st[k][0] = c[k].x ^ rk[0]; st[k][1] = c[k].y ^ rk[1]; st[k][2] = c[k].z ^ rk[2]; st[k][3] = c[k].w ^ rk[3];
    }
    AES_ROUNDS_PIPELINED(kChains, st, rk)
    uint32_t o[kChains][4];
#pragma unroll
    for (int k = 0; k < kChains; ++k) {
      AES_FINAL(st[k][0], st[k][1], st[k][2], st[k][3], o[k][0], o[k][1], o[k][2], o[k][3], rk + 40, pv[k])
    }
    if (4 * g < npk) {
      // packet 4g + k starts at byte 188k of the group: offsets 0, 12, 8, 4 in blocks 0, 11, 23, 35
      const uint4 h = make_uint4(hdr_word(o[0][0], o[0][1]), hdr_word(o[1][3], o[2][0]), hdr_word(o[3][2], o[3][3]),
                                 hdr_word(o[4][1], o[4][2]));
      *reinterpret_cast<uint4*>(a.hdr + pbase + 4 * g) = h;
    }
  }
}

// ---------------------------------------------------------------- 2. PSI + length
// Decrypt packet i of the segment whole into s_pk (lanes 0..12 one block each); returns the
// packet's byte offset in s_pk.  Collective over the wave.
__device__ __forceinline__ int psi_decrypt_packet(int i, const uint4* cs, int64_t nb, uint4 iv, const uint32_t* rk,
                                                  const uint32_t* s_td, const uint8_t* s_is, uint32_t* s_pk,
                                                  int lane) {
  const int x = kPkt * i, fb = x / 16, lb = (x + kPkt - 1) / 16;
  const int b = fb + lane;
  if (b <= lb && b < nb) {
    const uint4 p = aes_dec_small(s_td, s_is, rk, cs[b], b == 0 ? iv : cs[b - 1]);
    s_pk[4 * lane] = p.x;
    s_pk[4 * lane + 1] = p.y;
    s_pk[4 * lane + 2] = p.z;
    s_pk[4 * lane + 3] = p.w;
  }
  __syncthreads();
  return x - 16 * fb;
}

__global__ __launch_bounds__(64) void tsx_psi_kernel(ScatterArgs a) {
  __shared__ uint32_t s_td[256];
  __shared__ uint8_t s_is[256];
  __shared__ uint32_t s_pk[4 * 13];
  __shared__ int s_res[8];
  const int seg = blockIdx.x;
  const int lane = threadIdx.x;
  aes_small_fill(s_td, s_is, a.tdl, a.isb, lane, 64);
  int64_t* inf = a.info + static_cast<int64_t>(seg) * kInfo;
  int64_t* pe = a.pes + static_cast<int64_t>(seg) * kClasses * a.max_pes * 3;
  for (int64_t i = lane; i < static_cast<int64_t>(kClasses) * a.max_pes * 3; i += 64) pe[i] = -1;
  __syncthreads();
  const uint4* cs = reinterpret_cast<const uint4*>(a.src + a.src_off[seg]);
  const int64_t nb = a.aes_blk[seg + 1] - a.aes_blk[seg];
  const uint32_t* rk = a.drk + seg * 44;
  const uint4 iv = reinterpret_cast<const uint4*>(a.ivw)[seg];
  int64_t n = -1;
  if (lane == 0) {  // the plaintext length: the last block's PKCS#7 padding
    n = nb >= 1 ? pkcs7_len(aes_dec_small(s_td, s_is, rk, cs[nb - 1], nb >= 2 ? cs[nb - 2] : iv), nb * 16) : -1;
    a.out_len[seg] = n;
  }
  n = uniform64(n);
  const int64_t nn = n < 0 ? 0 : n;
  const int64_t np = nn / kPkt;
  int64_t status = (n < 0 || nn % kPkt) ? kBadLength : 0;
  const int scan = static_cast<int>(np < kPsiScan ? np : kPsiScan);
  const uint32_t h = lane < scan ? a.hdr[a.pkt_base[seg] + lane] : 0u;
  const bool hok = lane < scan && !((h >> 16) & 1u) && (h & 0x40u) && (hdr_afc(h) & 1) && hdr_payload_start(h) < kPkt;
  const int pid = hdr_pid(h);
  const uint8_t* bytes = reinterpret_cast<const uint8_t*>(s_pk);
  int pmt_pid = -1, vpid = -1, apid = -1, ipid = -1, vtype = 0, atype = 0;
  // PAT: the first candidate (PID 0, payload unit start) that parses, as the oracle scans
  uint64_t m = __ballot(hok && pid == 0);
  while (m && pmt_pid < 0) {
    const int i = __builtin_ctzll(m);
    m &= m - 1;
    const int off = psi_decrypt_packet(i, cs, nb, iv, rk, s_td, s_is, s_pk, lane);
    if (lane == 0) {
      const uint8_t* p = bytes + off;
      int ps = 4 + ((((p[3] >> 4) & 3) & 2) ? 1 + p[4] : 0);
      int found = -1;
      ps += 1 + p[ps];  // pointer field
      if (!(ps + 8 > kPkt || p[ps] != 0x00)) {
        const int slen = ((p[ps + 1] & 0x0f) << 8) | p[ps + 2];
        const int end = ps + 3 + slen - 4 < kPkt ? ps + 3 + slen - 4 : kPkt;
        for (int q = ps + 8; q + 4 <= end; q += 4) {
          const int prog = (p[q] << 8) | p[q + 1];
          if (prog != 0) {
            found = ((p[q + 2] & 0x1f) << 8) | p[q + 3];
            break;
          }
        }
      }
      s_res[0] = found;
    }
    __syncthreads();
    pmt_pid = s_res[0];
    __syncthreads();
  }
  if (pmt_pid < 0) status |= kNoPat;
  bool pmt_found = false;
  m = pmt_pid >= 0 ? __ballot(hok && pid == pmt_pid) : 0ull;
  while (m && !pmt_found) {
    const int i = __builtin_ctzll(m);
    m &= m - 1;
    const int off = psi_decrypt_packet(i, cs, nb, iv, rk, s_td, s_is, s_pk, lane);
    if (lane == 0) {
      const uint8_t* p = bytes + off;
      int ps = 4 + ((((p[3] >> 4) & 3) & 2) ? 1 + p[4] : 0);
      int r[6] = {0, -1, -1, -1, 0, 0};  // found, vpid, apid, ipid, vtype, atype
      ps += 1 + p[ps];
      if (!(ps + 12 > kPkt || p[ps] != 0x02)) {
        r[0] = 1;
        const int slen = ((p[ps + 1] & 0x0f) << 8) | p[ps + 2];
        const int end = ps + 3 + slen - 4 < kPkt ? ps + 3 + slen - 4 : kPkt;
        const int pil = ((p[ps + 10] & 0x0f) << 8) | p[ps + 11];
        for (int q = ps + 12 + pil; q + 5 <= end;) {
          const int type = p[q];
          const int epid = ((p[q + 1] & 0x1f) << 8) | p[q + 2];
          const int eil = ((p[q + 3] & 0x0f) << 8) | p[q + 4];
          if ((type == 0x1B || type == 0x24) && r[1] < 0) {
            r[1] = epid;
            r[4] = type;
          } else if ((type == 0x0F || type == 0x03 || type == 0x04) && r[2] < 0) {
            r[2] = epid;
            r[5] = type;
          } else if (type == 0x15 && r[3] < 0) {
            r[3] = epid;
          }
          q += 5 + eil;
        }
      }
      for (int k = 0; k < 6; ++k) s_res[k] = r[k];
    }
    __syncthreads();
    pmt_found = s_res[0] != 0;
    if (pmt_found) {
      vpid = s_res[1];
      apid = s_res[2];
      ipid = s_res[3];
      vtype = s_res[4];
      atype = s_res[5];
    }
    __syncthreads();
  }
  if (pmt_pid >= 0 && !pmt_found) status |= kNoPmt;
  if (lane == 0) {
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
}

// ---------------------------------------------------------------- 3. scan
__global__ __launch_bounds__(kThreads) void tsx_scan_kernel(ScatterArgs a) {
  __shared__ uint32_t s_td[256];
  __shared__ uint8_t s_is[256];
  __shared__ uint32_t s_buf[kThreads * 12];  // per lane: up to 3 decrypted PES-header blocks
  __shared__ int32_t s_sum[2 * kClasses];
  __shared__ int32_t s_err, s_nq;
  __shared__ int16_t s_q[kThreads];
  const int64_t gblk = blockIdx.x;
  const int seg = find_seg_wave(a.blk_prefix, a.nseg, gblk);
  const int64_t blk = gblk - a.blk_prefix[seg];
  const int tid = threadIdx.x;
  if (tid < 2 * kClasses) s_sum[tid] = 0;
  if (tid == 0) s_err = s_nq = 0;
  aes_small_fill(s_td, s_is, a.tdl, a.isb, tid, kThreads);
  __syncthreads();
  const int64_t* inf = a.info + static_cast<int64_t>(seg) * kInfo;
  const int p0 = static_cast<int>(inf[kVideoPid]), p1 = static_cast<int>(inf[kVideoPid + 1]),
            p2 = static_cast<int>(inf[kVideoPid + 2]);
  const int64_t n = a.out_len[seg];
  const int64_t np = (n < 0 ? 0 : n) / kPkt;
  const int64_t pk = blk * kThreads + tid;
  const int64_t gpk = gblk * kThreads + tid;
  // PES-starting packets need their PES header (bytes [s, s + 20)): those lanes queue up, and
  // the block's first lanes decrypt the 2-3 blocks of each into the owner's s_buf row
  // (~2 % of packets: compacted, one wave does the AES work instead of every wave diverging)
  uint32_t h = 0;
  int s = 0;
  if (pk < np) {
    h = a.hdr[gpk];
    s = hdr_payload_start(h);
    const int pid = hdr_pid(h);
    const bool cls = (p0 >= 0 && pid == p0) || (p1 >= 0 && pid == p1) || (p2 >= 0 && pid == p2);
    if (!((h >> 16) & 1u) && (h & 0x40u) && cls && (hdr_afc(h) & 1) && s + 9 <= kPkt) s_q[atomicAdd(&s_nq, 1)] = tid;
  }
  __syncthreads();
  const int nq = s_nq;
  if (tid < nq) {  // <= 256 queued per block, one per lane
    const int q = s_q[tid];
    const uint4* cs = reinterpret_cast<const uint4*>(a.src + a.src_off[seg]);
    const int64_t nb = a.aes_blk[seg + 1] - a.aes_blk[seg];
    const uint32_t* rk = a.drk + seg * 44;
    const int64_t x = kPkt * (blk * kThreads + q) + hdr_payload_start(a.hdr[gblk * kThreads + q]);
    const int64_t fb = x / 16;
    uint32_t* row = s_buf + q * 12;
    for (int k = 0; k < 3; ++k) {
      const int64_t b = fb + k;
      if (b < nb && b * 16 < x + 20) {
        const uint4 p = aes_dec_small(s_td, s_is, rk, cs[b],
                                      b == 0 ? reinterpret_cast<const uint4*>(a.ivw)[seg] : cs[b - 1]);
        row[4 * k] = p.x;
        row[4 * k + 1] = p.y;
        row[4 * k + 2] = p.z;
        row[4 * k + 3] = p.w;
      }
    }
  }
  __syncthreads();
  demux::Pkt r{3, 0, 0, 0, -1, -1, 0};
  if (pk < np) {
    uint32_t hh[5] = {0, 0, 0, 0, 0};
    const int at = static_cast<int>((kPkt * pk + s) & 15);
    const uint32_t* w = s_buf + tid * 12 + (at >> 2);
    uint32_t hw[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) hw[q] = w[q];  // meaningful for the queued lanes only
#pragma unroll
    for (int q = 0; q < 5; ++q) hh[q] = __builtin_amdgcn_alignbyte(hw[q + 1], hw[q], static_cast<uint32_t>(at & 3));
    r = demux::parse_pkt(true, hdr_w0(h), hh, s, p0, p1, p2);
  }
  a.meta[gpk] = demux::pack_meta(r.c, r.ps, r.len, r.pesf);
  if (r.pesf) {
    a.pts_dts[2 * gpk] = r.pts;
    a.pts_dts[2 * gpk + 1] = r.dts;
  }
#pragma unroll
  for (int k = 0; k < kClasses; ++k) {
    int vb = (r.c == k) ? r.len : 0;
    int vp = (r.c == k) ? r.pesf : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      vb += __shfl_xor(vb, o);
      vp += __shfl_xor(vp, o);
    }
    if ((tid & 63) == 0) {
      if (vb) atomicAdd(&s_sum[2 * k], vb);
      if (vp) atomicAdd(&s_sum[2 * k + 1], vp);
    }
  }
  if (r.err) atomicOr(&s_err, static_cast<int32_t>(r.err));
  __syncthreads();
  if (tid < 2 * kClasses) a.aux[gblk * 2 * kClasses + tid] = s_sum[tid];
  if (tid == 0 && s_err)
    atomicOr(reinterpret_cast<unsigned long long*>(a.info + static_cast<int64_t>(seg) * kInfo + kStatus),
             static_cast<unsigned long long>(s_err));
}

// ---------------------------------------------------------------- 5. place
__global__ __launch_bounds__(kThreads) void tsx_place_kernel(ScatterArgs a) {
  __shared__ uint32_t s_wave[4][3];  // per-wave packed scan totals
  const int64_t gblk = blockIdx.x;
  const int seg = find_seg_wave(a.blk_prefix, a.nseg, gblk);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int32_t* blk_pre = a.aux + a.total_blocks * 2 * kClasses;
  const int32_t* seg_tot = blk_pre + a.total_blocks * 2 * kClasses;
  const int64_t gpk = gblk * kThreads + tid;
  const uint32_t m = a.meta[gpk];
  int32_t pre[2 * kClasses], tot[2 * kClasses];
#pragma unroll
  for (int k = 0; k < 2 * kClasses; ++k) {
    pre[k] = blk_pre[gblk * 2 * kClasses + k];
    tot[k] = seg_tot[seg * 2 * kClasses + k];
  }
  const int c = m & 3, ps = (m >> 2) & 0xff, len = (m >> 10) & 0xff, pes_flag = (m >> 18) & 1;
  // in-wave inclusive scans of (bytes, PES starts) per class, packed three to a word (as the
  // split gather: wave totals fit their fields)
  const uint32_t lb = static_cast<uint32_t>(len), pf = static_cast<uint32_t>(pes_flag);
  uint32_t sA = (c == 0 ? lb : 0u) | ((c == 1 ? lb : 0u) << 16);
  uint32_t sB = (c == 2 ? lb : 0u) | ((c == 0 ? pf : 0u) << 16) | ((c == 1 ? pf : 0u) << 24);
  uint32_t sC = c == 2 ? pf : 0u;
  sA = demux::dpp_scan(sA);
  sB = demux::dpp_scan(sB);
  sC = demux::dpp_scan(sC);
  if (lane == 63) {
    s_wave[wave][0] = sA;
    s_wave[wave][1] = sB;
    s_wave[wave][2] = sC;
  }
  __syncthreads();
  uint2 out = make_uint2(0, 0);
  if (c < 3) {
    uint32_t wA = 0, wB = 0, wC = 0;
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
    const int64_t dst_b = class_base + es_in_class;
    const int64_t pes_idx = static_cast<int64_t>(pre[2 * c + 1]) + inc_p - pes_flag;
    if (pes_flag) {
      const int64_t tot_pes = tot[2 * c + 1];
      int64_t* infc = a.info + static_cast<int64_t>(seg) * kInfo;
      if (pes_idx == 0) infc[kFirstPts + c] = a.pts_dts[2 * gpk];
      if (pes_idx == tot_pes - 1) infc[kLastPts + c] = a.pts_dts[2 * gpk];
      if (pes_idx < a.max_pes) {
        int64_t* r = a.pes + ((static_cast<int64_t>(seg) * kClasses + c) * a.max_pes + pes_idx) * 3;
        r[0] = es_in_class;
        r[1] = a.pts_dts[2 * gpk];
        r[2] = a.pts_dts[2 * gpk + 1];
      }
    }
    if (len > 0)
      out = make_uint2(static_cast<uint32_t>(static_cast<int32_t>(dst_b - ps)),
                       static_cast<uint32_t>(ps) | (static_cast<uint32_t>(ps + len) << 16));
  }
  a.place[gpk] = out;
}

// ---------------------------------------------------------------- 7. seams
// One lane per packet: its payload run's head bytes (until its first aligned ES dword) and
// tail bytes (after its last full dword), <= 3 each, share an ES dword with the neighbouring
// same-class runs; the bulk decrypt left them in seam[2 * pkt + {0, 1}] (low bytes first).
__global__ __launch_bounds__(kThreads) void tsx_seam_kernel(ScatterArgs a) {
  const int64_t gblk = blockIdx.x;
  const int seg = find_seg_wave(a.blk_prefix, a.nseg, gblk);
  const int64_t gpk = gblk * kThreads + threadIdx.x;
  const uint2 pl = a.place[gpk];
  const int lo = static_cast<int>(pl.y & 0xffff), hi = static_cast<int>(pl.y >> 16);
  if (hi <= lo) return;
  uint8_t* es = a.es + a.es_off[seg];
  const int d = static_cast<int>(pl.x) + lo;  // ES offset of the run's first byte
  const int hh = (-d) & 3, h = hh < hi - lo ? hh : hi - lo;
  const int t = h + ((hi - lo - h) & ~3);  // run offset of the tail
  const uint32_t head = h ? a.seam[2 * gpk] : 0u, tail = t < hi - lo ? a.seam[2 * gpk + 1] : 0u;
  for (int i = 0; i < h; ++i) es[d + i] = static_cast<uint8_t>(head >> (8 * i));
  for (int i = 0; i < hi - lo - t; ++i) es[d + t + i] = static_cast<uint8_t>(tail >> (8 * i));
}

}  // namespace

hipError_t launch_ts_scatter(const ScatterArgs& a, int num_cu, hipStream_t stream) {
  if (a.nseg <= 0) return hipSuccess;
  if (a.hdr_total_chunks > 0) {
    constexpr int64_t kWaves = kAesImageThreads / 64;
    int64_t grid = (a.hdr_total_chunks + kWaves * 2 - 1) / (kWaves * 2);
    if (grid > num_cu) grid = num_cu;
    if (grid < 1) grid = 1;
    int64_t per_wg = (a.hdr_total_chunks + grid - 1) / grid;
    grid = (a.hdr_total_chunks + per_wg - 1) / per_wg;
    hipLaunchKernelGGL(tsx_hdr_kernel, dim3(static_cast<unsigned>(grid)), dim3(kAesImageThreads), 0, stream, a, per_wg);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(tsx_psi_kernel, dim3(a.nseg), dim3(64), 0, stream, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || a.total_blocks <= 0) return e;
  hipLaunchKernelGGL(tsx_scan_kernel, dim3(static_cast<unsigned>(a.total_blocks)), dim3(kThreads), 0, stream, a);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  int32_t* blk_sums = a.aux;
  int32_t* blk_pre = blk_sums + a.total_blocks * 2 * kClasses;
  int32_t* seg_tot = blk_pre + a.total_blocks * 2 * kClasses;
  e = launch_ts_prefix(a.blk_prefix, blk_sums, blk_pre, seg_tot, a.info, a.max_pes, a.nseg, stream);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(tsx_place_kernel, dim3(static_cast<unsigned>(a.total_blocks)), dim3(kThreads), 0, stream, a);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = launch_aes128_cbc_scatter(a.src, a.src_off, a.aes_blk, a.aes_chunks, a.drk, a.ivw, a.tdl, a.isb, a.place,
                                   a.pkt_base, a.pkt_slots, a.es, a.es_off, a.seam, a.nseg, a.aes_total_chunks,
                                   num_cu, stream);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(tsx_seam_kernel, dim3(static_cast<unsigned>(a.total_blocks)), dim3(kThreads), 0, stream, a);
  return hipGetLastError();
}

}  // namespace dev
}  // namespace hlsp2p
