// AES-128-CBC decryption of a batch of HLS segments — CDNA4 / gfx950.
//
// CBC *decryption* is block-parallel: P_i = D_K(C_i) xor C_{i-1}.  Work unit = a CHUNK of
// 256 consecutive 16-byte blocks of one segment per wave: lane l runs four independent AES
// chains (blocks 64j + l, interleaved for ILP against LDS latency), so each of the wave's
// global load/store instructions moves 1 KB contiguous (TA/TD-friendly); C_{i-1} is a
// second coalesced load that hits L1.  A wave never straddles segments: the segment's 44
// round keys are wave-uniform and live in SGPRs (scalar loads).
//
// AES is table bound, not matmul shaped (no MFMA).  Design for the CDNA4 LDS + VALU:
//  * Tables in LITTLE-ENDIAN column form (TdL = bswap(Td0), round keys pre-swapped on the
//    host), so state words are used exactly as loaded — no byte swaps in the kernel.
//  * The whole 160 KiB of the CU's LDS holds one image shared by a 1024-thread workgroup:
//      [0, 64K)     row x (256 B) = [32 lane copies of Td0L[x] | 32 copies of Td1L[x]]
//      [64K, 128K)  row x (256 B) = [32 lane copies of Td2L[x] | 32 copies of Td3L[x]]
//      [128K,160K)  row x (128 B) =  32 lane copies of InvSbox[x]
//    Td1..Td3 are the byte rotations of Td0, stored pre-rotated so a round needs NO
//    v_alignbit.  Lane l reads dword l of a 32-dword half-row: for ds_read_b32 (bank =
//    dword % 32) every lane of a 32-lane group owns a bank -> all 160 lookups per block are
//    conflict-free.
//  * Td address of entry x for lane l = (region << 16) | (x << 8) | (half << 7) | (l << 2):
//    ONE v_perm_b32 builds it from the state word (byte k -> bits 8..15; bits 0..7 and
//    16..23 come from a per-lane per-table base) — no extract + shift-or.
//    Per round: 16 v_perm + 16 ds_read_b32 + 8 v_bitop3 (3-input XOR, round key as SGPR).
//  * One workgroup per CU: 16 waves = 4 per SIMD (109 VGPRs).
//
// Persistent grid (1 workgroup per CU), each streaming one contiguous range of the batch's
// chunk index space; the segment table is walked monotonically so per-segment state (44
// round keys, IV, offsets) reloads only at boundaries.  PKCS#7: the lane holding a
// segment's last block validates the padding and writes the plaintext length (or -1) to
// out_len[seg] on device — the demux kernels read it directly (no host round trip).
#include "common.h"

#include "aes_dev.h"
#include "demux_dev.h"
#include "ts_scatter.h"

namespace hlsp2p {
namespace dev {

constexpr int kAesThreads = kAesImageThreads;
constexpr int kAesWgPerCu = 1;
constexpr int kBlk = 4;  // blocks per lane per chunk (chunk = 64 * kBlk blocks): independent chains
static_assert(64 * kBlk == kScatterChunkBlocks + 1, "scatter chunks: one lookahead block per iteration");

// Scatter epilogue (the scatter demux, ts_scatter.hip): instead of writing the plaintext,
// every block writes the bytes of it that are TS payload straight to their elementary-stream
// position.  place[pkt] = (bias, lo | hi << 16): payload bytes y in [lo, hi) of packet pkt go
// to es + es_off[seg] + bias + y.
struct AesScatter {
  const uint2* place;        // per packet slot (the demux's 256-packet block grid)
  const int64_t* pkt_base;   // [nseg] first packet slot of the segment
  const int64_t* pkt_slots;  // [nseg] packet slots of the segment
  uint8_t* es;
  const int64_t* es_off;     // [nseg]
  uint32_t* seam;            // [packet slots][2] head / tail seam bytes
};

// Scatter epilogue of one wave iteration.  The scatter decrypt walks a segment in chunks of
// kScatterChunkBlocks = 255 blocks but decrypts 256: chain j, lane l holds block b0 + 64j + l,
// and the last (chain N-1, lane 63) is a LOOKAHEAD: the next chunk owns it, it only lends its
// first bytes.  Every owned block writes the payload bytes of the (at most two) packets it
// overlaps: per packet run [s, e) in the block,
//  * the aligned ES dwords whose first byte is in [s, e) and whose four bytes are all payload
//    of the run -- one buffer_store_dwordx4 for a block inside a payload, else up to three
//    dword stores; up to 3 bytes may come from the next block (lane l + 1 by DPP, or the next
//    chain's lane 0);
//  * the run's SEAM bytes, which share an ES dword with the previous / next same-class
//    packet: the head (until the run's first aligned dword) and the tail (after its last
//    full dword), each <= 3 bytes, as one word into seam[2 * pkt + {0, 1}]; tsx_seam_kernel
//    (ts_scatter.hip) stores them as bytes.
// No byte stores and no divergent loops here: the bulk decrypt is VALU/LDS bound.
__device__ __forceinline__ uint32_t sel4(uint32_t a, uint32_t b, uint32_t c, uint32_t d, int i) {
  return i == 0 ? a : i == 1 ? b : i == 2 ? c : d;
}
// the 4 bytes at offset u (0..15) of the 20 bytes w0..w3, nx
__device__ __forceinline__ uint32_t funnel(const uint32_t* w, uint32_t nx, int u) {
  const int i = u >> 2;
  return __builtin_amdgcn_alignbyte(sel4(w[1], w[2], w[3], nx, i), sel4(w[0], w[1], w[2], w[3], i),
                                    static_cast<uint32_t>(u & 3));
}

template <int N>
__device__ __forceinline__ void scatter_epilogue(const uint32_t (&w)[N][4], int64_t b0, int64_t nblk, int lane,
                                                 const uint2* __restrict__ place, int64_t pbase, int64_t slots,
                                                 __amdgpu_buffer_rsrc_t es_rsrc, uint32_t* __restrict__ seam) {
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const int64_t b = b0 + 64 * j;
    // next block's first word: lane l + 1 (wave_shl:1), or the next chain's lane 0 -- read with
    // every lane active (a DPP source lane outside EXEC would read as 0)
    uint32_t nx = static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(w[j][0]), 0x130, 0xf, 0xf, false));
    if (j + 1 < N) {
      const uint32_t first = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(w[j + 1][0]), 0));
      nx = lane == 63 ? first : nx;
    }
    const bool own = b < nblk && !(j == N - 1 && lane == 63);
    const int x0 = static_cast<int>(16 * b);
    const int p = x0 / demux::kPkt;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int pk = p + r, P = demux::kPkt * pk;
      const bool any = own && pk < slots && P < x0 + 16;
      const uint2 pl = any ? place[pbase + pk] : make_uint2(0, 0);
      const int lo = static_cast<int>(pl.y & 0xffff), hi = static_cast<int>(pl.y >> 16);
      const int RS = P + lo, RE = P + hi;
      const int s = x0 > RS ? x0 : RS, e = x0 + 16 < RE ? x0 + 16 : RE;
      if (!(any && s < e)) continue;
      const int dbias = static_cast<int>(pl.x) - P;  // ES offset of segment byte x = dbias + x
      const int xf = s + ((-(dbias + s)) & 3);       // first owned aligned dword's source byte
      const int lim = e < RE - 3 ? e : RE - 3;       // owned: x < e and x + 4 <= RE
      const int n = xf < lim ? (lim - xf + 3) >> 2 : 0;
      const int u0 = xf - x0;
      const uint32_t sh = static_cast<uint32_t>(u0 & 3);
      const uint32_t g0 = __builtin_amdgcn_alignbyte(w[j][1], w[j][0], sh),
                     g1 = __builtin_amdgcn_alignbyte(w[j][2], w[j][1], sh),
                     g2 = __builtin_amdgcn_alignbyte(w[j][3], w[j][2], sh),
                     g3 = __builtin_amdgcn_alignbyte(nx, w[j][3], sh);
      if (n == 4) {  // u0 < 4: the whole dword window of the block
        const v4u q = {g0, g1, g2, g3};
        __builtin_amdgcn_raw_buffer_store_b128(q, es_rsrc, dbias + xf, 0, 0);
      } else {
        const int i0 = u0 >> 2;
#pragma unroll
        for (int k = 0; k < 3; ++k)
          if (k < n) __builtin_amdgcn_raw_buffer_store_b32(sel4(g0, g1, g2, g3, i0 + k), es_rsrc, dbias + xf + 4 * k, 0, 0);
      }
      const int hh = (-(dbias + RS)) & 3, h = hh < RE - RS ? hh : RE - RS;
      if (s == RS && h > 0) seam[2 * (pbase + pk)] = funnel(w[j], nx, RS - x0);
      const int T = RS + h + ((RE - RS - h) & ~3);
      if (T < RE && T >= s && T < e) seam[2 * (pbase + pk) + 1] = funnel(w[j], nx, T - x0);
    }
  }
}

// tdl: little-endian Td0 (256 words); isb: inverse S-box (256 bytes)
// drk: per-segment little-endian equivalent-inverse-cipher round keys (44 words)
// chunk_prefix: exclusive prefix of per-segment 256-block chunks (one chunk = one wave
//   iteration: lane l decrypts blocks 64j + l, j < kBlk, so every load/store instruction
//   moves 1 KB contiguous); waves never straddle segments
// kScatter: the payload bytes go to their ES positions (AesScatter); dst / out_len are unused
//   (out_len is the scatter demux's, computed before this launch)
template <bool kScatter>
__global__ __launch_bounds__(kAesThreads, 1) void aes128_cbc_decrypt_kernel(
    const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, const int64_t* __restrict__ src_off,
    const int64_t* __restrict__ dst_off, const int64_t* __restrict__ blk_prefix,
    const int64_t* __restrict__ chunk_prefix, const uint32_t* __restrict__ drk, const uint32_t* __restrict__ ivw,
    const uint32_t* __restrict__ tdl_g, const uint8_t* __restrict__ isb_g, int64_t* __restrict__ out_len, int nseg,
    int64_t total_chunks, int64_t per_wg, AesScatter sc) {
  __shared__ uint32_t s_tab[kTdDwords + kIsDwords];  // 160 KiB (layout above)
  const int tid = threadIdx.x;
  aes_image_fill(s_tab, tdl_g, isb_g, tid);
  __syncthreads();
  const uint8_t* s_bytes = reinterpret_cast<const uint8_t*>(s_tab);
  uint32_t td_base[4], is_base;
  aes_image_bases(tid, td_base, is_base);
  const int lane = tid & 63;
  constexpr int kWaves = kAesThreads / 64;

  // per_wg chunks per workgroup; wave w of the group takes chunks begin + w, + kWaves, ...
  const int64_t begin = static_cast<int64_t>(blockIdx.x) * per_wg;
  const int64_t end = begin + per_wg < total_chunks ? begin + per_wg : total_chunks;
  // segment state is wave-uniform (SGPRs): round keys come in by scalar loads
  int cur = -1;
  uint32_t rk[44];
  int64_t so = 0, dof = 0, cstart = 0, cend = 0, nblk = 0, pbase = 0, slots = 0;
  uint8_t* esb = nullptr;
  for (int64_t ch = uniform64(begin + (tid >> 6)); ch < end; ch += kWaves) {
    if (cur < 0 || ch >= cend) {
      cur = cur < 0 ? find_seg_wave(chunk_prefix, nseg, ch)  // whole wave active: ch is uniform
                    : __builtin_amdgcn_readfirstlane(advance_seg(chunk_prefix, cur, ch));
#pragma unroll
      for (int k = 0; k < 44; ++k) rk[k] = drk[cur * 44 + k];
      so = src_off[cur];
      dof = dst_off[cur];
      cstart = chunk_prefix[cur];
      cend = chunk_prefix[cur + 1];
      nblk = blk_prefix[cur + 1] - blk_prefix[cur];
      if (kScatter) {
        pbase = sc.pkt_base[cur];
        slots = sc.pkt_slots[cur];
        esb = sc.es + sc.es_off[cur];
      }
    }
    // this lane's first block (scatter: chunks of kScatterChunkBlocks, the last lane a lookahead)
    const int64_t b0 = (ch - cstart) * (kScatter ? kScatterChunkBlocks : 64 * kBlk) + lane;
    const uint4* cs = reinterpret_cast<const uint4*>(src + so);
    uint4 c[kBlk], pv[kBlk];
#pragma unroll
    for (int j = 0; j < kBlk; ++j) {
      const int64_t b = b0 + 64 * j;
      c[j] = b < nblk ? cs[b] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < kBlk; ++j) {  // CBC chaining input: the previous block (an L1 hit)
      const int64_t b = b0 + 64 * j;
      pv[j] = b == 0 ? reinterpret_cast<const uint4*>(ivw)[cur] : (b < nblk ? cs[b - 1] : make_uint4(0, 0, 0, 0));
    }
    uint32_t st[kBlk][4];
#pragma unroll
    for (int j = 0; j < kBlk; ++j) {
      st[j][0] = c[j].x ^ rk[0]; st[j][1] = c[j].y ^ rk[1]; st[j][2] = c[j].z ^ rk[2]; st[j][3] = c[j].w ^ rk[3];
    }
    AES_ROUNDS_PIPELINED(kBlk, st, rk)
    if (kScatter) {
      uint32_t w[kBlk][4];
#pragma unroll
      for (int j = 0; j < kBlk; ++j) {
        AES_FINAL(st[j][0], st[j][1], st[j][2], st[j][3], w[j][0], w[j][1], w[j][2], w[j][3], rk + 40, pv[j])
      }
      scatter_epilogue<kBlk>(w, b0, nblk, lane, sc.place, pbase, slots,
                             __builtin_amdgcn_make_buffer_rsrc(esb, 0, 0x7fffffff, 0x00020000), sc.seam);
    } else {
      uint4* ds = reinterpret_cast<uint4*>(dst + dof);
#pragma unroll
      for (int j = 0; j < kBlk; ++j) {
        uint32_t o0, o1, o2, o3;
        AES_FINAL(st[j][0], st[j][1], st[j][2], st[j][3], o0, o1, o2, o3, rk + 40, pv[j])
        const uint4 p = make_uint4(o0, o1, o2, o3);
        const int64_t b = b0 + 64 * j;
        if (b < nblk) ds[b] = p;
        if (b == nblk - 1) out_len[cur] = pkcs7_len(p, nblk * 16);
      }
    }
  }
}

// 16-byte blocks per wave iteration (the host sizes its chunk index space with this)
int aes_chunk_blocks() { return 64 * kBlk; }

namespace {
void aes_grid(int64_t total_chunks, int num_cu, int64_t& grid, int64_t& per_wg) {
  constexpr int64_t kWaves = kAesThreads / 64;
  const int64_t max_wg = static_cast<int64_t>(num_cu) * kAesWgPerCu;
  grid = (total_chunks + kWaves * 2 - 1) / (kWaves * 2);
  if (grid > max_wg) grid = max_wg;
  if (grid < 1) grid = 1;
  per_wg = (total_chunks + grid - 1) / grid;
  grid = (total_chunks + per_wg - 1) / per_wg;
}
}  // namespace

hipError_t launch_aes128_cbc_decrypt(const uint8_t* src, uint8_t* dst, const int64_t* src_off, const int64_t* dst_off,
                                     const int64_t* blk_prefix, const int64_t* chunk_prefix, const uint32_t* drk,
                                     const uint32_t* ivw, const uint32_t* tdl, const uint8_t* isb, int64_t* out_len,
                                     int nseg, int64_t total_chunks, int num_cu, hipStream_t stream) {
  if (total_chunks <= 0) return hipSuccess;
  int64_t grid, per_wg;
  aes_grid(total_chunks, num_cu, grid, per_wg);
  hipLaunchKernelGGL(aes128_cbc_decrypt_kernel<false>, dim3(static_cast<unsigned>(grid)), dim3(kAesThreads), 0, stream,
                     src, dst, src_off, dst_off, blk_prefix, chunk_prefix, drk, ivw, tdl, isb, out_len, nseg,
                     total_chunks, per_wg, AesScatter{});
  return hipGetLastError();
}

// The scatter demux's decrypt (ts_scatter.hip): payload dwords straight to the ES buffer, seam
// bytes to `seam` for tsx_seam_kernel.  chunk_prefix counts kScatterChunkBlocks-block chunks.
hipError_t launch_aes128_cbc_scatter(const uint8_t* src, const int64_t* src_off, const int64_t* blk_prefix,
                                     const int64_t* chunk_prefix, const uint32_t* drk, const uint32_t* ivw,
                                     const uint32_t* tdl, const uint8_t* isb, const uint2* place,
                                     const int64_t* pkt_base, const int64_t* pkt_slots, uint8_t* es,
                                     const int64_t* es_off, uint32_t* seam, int nseg, int64_t total_chunks,
                                     int num_cu, hipStream_t stream) {
  if (total_chunks <= 0) return hipSuccess;
  int64_t grid, per_wg;
  aes_grid(total_chunks, num_cu, grid, per_wg);
  hipLaunchKernelGGL(aes128_cbc_decrypt_kernel<true>, dim3(static_cast<unsigned>(grid)), dim3(kAesThreads), 0, stream,
                     src, nullptr, src_off, src_off, blk_prefix, chunk_prefix, drk, ivw, tdl, isb, nullptr, nseg,
                     total_chunks, per_wg, AesScatter{place, pkt_base, pkt_slots, es, es_off, seam});
  return hipGetLastError();
}

}  // namespace dev
}  // namespace hlsp2p
