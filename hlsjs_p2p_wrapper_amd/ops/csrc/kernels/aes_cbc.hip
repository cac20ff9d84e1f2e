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

namespace hlsp2p {
namespace dev {

constexpr int kAesThreads = kAesImageThreads;
constexpr int kAesWgPerCu = 1;
constexpr int kBlk = 4;  // blocks per lane per chunk (chunk = 64 * kBlk blocks): independent chains

typedef int v4i __attribute__((ext_vector_type(4)));
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
constexpr uint32_t kOutOfRange = 0x80000000u;  // a buffer offset past every segment (reads 0)
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

// Optional CRC-32 of the CIPHERTEXT, fused into the decrypt (SURVEY K12 on the receive path:
// a segment that arrived from a peer is verified by the batch that decrypts it, instead of by a
// separate read pass).  The ciphertext is already in VGPRs and the matrix cores sit idle
// while the decrypt is VALU / LDS bound, so each flagged chunk adds 16 FP4 MFMAs
// (v_mfma_scale_f32_32x32x64_f8f6f4, the operand scheme of crc32_mfma.hip): chains 2p and 2p + 1
// share accumulator set p; step (j & 1, d) feeds dword d of the lane's block 64j + l, row
// rho = l & 31 collecting blocks 64j + rho and 64j + rho + 32 (k half l >> 5).  The 8 weight
// steps are the same for both pairs (crc_host.cpp: mfma_chunk_weights_fp4), so they are loaded
// once per wave and stay in 32 VGPRs; the pair's position moves to the fold.  The parities of
// the 2 x 16 accumulators go out as one dword per lane (`masks`: 64 per chunk, bit 16 p + i =
// row (i & 3) + 8 (i >> 2) + 4 (lane >> 5), column lane & 31); crc32_fold_combine_kernel
// (crc32_mfma.hip) turns them into the chunk residue with a second FP4 GEMM.
//
// (Round 4 measured a one-level form first -- 16 chain-specific weight steps re-read from L1
// per chunk, one parity word per lane: +50 us per 256-segment batch in this kernel; then one
// accumulator set per chain (4 steps in VGPRs): +76 us at +15.7 % VALU instructions and the
// same clock -- the kernel is VALU + LDS co-bound, so every operand or parity instruction
// costs time.  profiles/r4_fused.)
struct AesCrc {
  const int64_t* mask_off;  // [nseg] the segment's first mask dword (64 per 4096-byte chunk), -1:
                            // no CRC for it (nullptr: for no segment)
  const v4i* wfrag;         // [8 steps][64 lanes] B fragments
  uint32_t* masks;
};
constexpr int kCrcSteps = 8;  // [chain parity jj][data dword d]

__device__ __forceinline__ void crc_chunk_masks(const uint4 (&c)[kBlk], const v4i (&w)[kCrcSteps], int lane,
                                                uint32_t* __restrict__ out) {
  // accumulators start at 2^23: the counts stay exact and the float's mantissa LSB is the parity,
  // so one v_alignbit per accumulator moves it into the mask word (no float -> int conversion)
  const v16f init = {8388608.f, 8388608.f, 8388608.f, 8388608.f, 8388608.f, 8388608.f, 8388608.f, 8388608.f,
                     8388608.f, 8388608.f, 8388608.f, 8388608.f, 8388608.f, 8388608.f, 8388608.f, 8388608.f};
  uint32_t m = 0;
  v16f acc = init;
#pragma unroll
  for (int j = 0; j < kBlk; ++j) {  // chains 2p and 2p + 1 share accumulator set p
    const uint32_t dw[4] = {c[j].x, c[j].y, c[j].z, c[j].w};
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const uint32_t x = dw[d];
      const v8i a = {static_cast<int>(x & 0x11111111u), static_cast<int>(x & 0x22222222u),
                     static_cast<int>(x & 0x44444444u), static_cast<int>((x >> 1) & 0x44444444u), 0, 0, 0, 0};
      const v4i& wv = w[4 * (j & 1) + d];
      const v8i b = {wv.x, wv.y, wv.z, wv.w, 0, 0, 0, 0};
      acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc, 4, 4, 0, 0, 0, 0);
    }
    if (j & 1) {
#pragma unroll
      for (int i = 0; i < 16; ++i) m = __builtin_amdgcn_alignbit(__float_as_uint(acc[i]), m, 1);
      acc = init;
    }
  }
  out[lane] = m;  // bits 16 p + i
}

// Optional packet-header records for the demux scan (ts_demux.hip: ts_scan_kernel): the block
// holding packet q's 4-byte TS header (byte 188 q; 188 q mod 16 is 0, 4, 8 or 12, so the header
// never straddles blocks) is also stored, whole, as record q of the segment.  The scan then
// reads 16 dense bytes per packet instead of one 128-byte line of plaintext per packet (0.68 of
// a pass).  Per block: one multiply-high division by 188 and a compare; one masked 16-byte
// store in ~1 of 12 lanes.
struct AesHdr {
  const int64_t* off;  // [nseg] the segment's first record (nullptr: no records)
  uint4* rec;
};
constexpr uint32_t kDiv188Magic = 2924233053u;  // floor(x / 188) = umulhi(x, M) >> 7 for all 32-bit x

// tdl: little-endian Td0 (256 words); isb: inverse S-box (256 bytes)
// drk: per-segment little-endian equivalent-inverse-cipher round keys (44 words)
// chunk_prefix: exclusive prefix of per-segment 256-block chunks (one chunk = one wave
//   iteration: lane l decrypts blocks 64j + l, j < kBlk, so every load/store instruction
//   moves 1 KB contiguous); waves never straddle segments
// kCrc: 0 without the fused CRC code (its registers), 1 with it; kHdr: packet-header records
template <int kCrc, int kHdr>
__global__ __launch_bounds__(kAesThreads, 1) void aes128_cbc_decrypt_kernel(
    const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, const int64_t* __restrict__ src_off,
    const int64_t* __restrict__ dst_off, const int64_t* __restrict__ blk_prefix,
    const int64_t* __restrict__ chunk_prefix, const uint32_t* __restrict__ drk, const uint32_t* __restrict__ ivw,
    const uint32_t* __restrict__ tdl_g, const uint8_t* __restrict__ isb_g, int64_t* __restrict__ out_len, int nseg,
    int64_t total_chunks, int64_t per_wg, AesCrc crc, AesHdr hdr) {
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
  int64_t so = 0, dof = 0, cstart = 0, cend = 0, nblk = 0, maskb = -1, hdrb = 0;
  // the current segment's ciphertext / plaintext as buffer ranges (empty until the first segment)
  __amdgpu_buffer_rsrc_t s_rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(src), 0, 0, 0x00020000);
  __amdgpu_buffer_rsrc_t d_rsrc = __builtin_amdgcn_make_buffer_rsrc(dst, 0, 0, 0x00020000);
  v4i crc_w[kCrcSteps];
  if constexpr (kCrc == 1) {
#pragma unroll
    for (int d = 0; d < kCrcSteps; ++d) crc_w[d] = crc.wfrag[d * 64 + lane];
  }
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
      maskb = crc.mask_off != nullptr ? crc.mask_off[cur] : -1;
      if constexpr (kHdr == 1) hdrb = hdr.off[cur];
      s_rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(src + so), 0, static_cast<int>(nblk * 16),
                                                 0x00020000);
      d_rsrc = __builtin_amdgcn_make_buffer_rsrc(dst + dof, 0, static_cast<int>(nblk * 16), 0x00020000);
    }
    const int64_t b0 = (ch - cstart) * (64 * kBlk) + lane;  // this lane's first block
    // buffer loads over the segment: blocks past its end read as 0 (no per-block predicate, no
    // zero fill); the chaining input of block 0 is the IV
    uint4 c[kBlk], pv[kBlk];
    const uint32_t boff = static_cast<uint32_t>(b0) << 4;  // segments are < 2 GiB (host-checked)
#pragma unroll
    for (int j = 0; j < kBlk; ++j) {
      const v4u q = __builtin_amdgcn_raw_buffer_load_b128(s_rsrc, boff + 1024u * j, 0, 0);
      c[j] = make_uint4(q[0], q[1], q[2], q[3]);
    }
#pragma unroll
    for (int j = 0; j < kBlk; ++j) {  // CBC chaining input: the previous block (an L1 hit)
      const uint32_t o = boff + 1024u * j;
      const v4u q = __builtin_amdgcn_raw_buffer_load_b128(s_rsrc, j == 0 && o == 0 ? kOutOfRange : o - 16u, 0, 0);
      pv[j] = make_uint4(q[0], q[1], q[2], q[3]);
    }
    if (ch == cstart && lane == 0) pv[0] = reinterpret_cast<const uint4*>(ivw)[cur];
    if constexpr (kCrc == 1) {
      if (maskb >= 0)  // wave-uniform
        crc_chunk_masks(c, crc_w, lane, crc.masks + maskb + (ch - cstart) * 64);
    }
    uint32_t st[kBlk][4];
#pragma unroll
    for (int j = 0; j < kBlk; ++j) {
      st[j][0] = c[j].x ^ rk[0]; st[j][1] = c[j].y ^ rk[1]; st[j][2] = c[j].z ^ rk[2]; st[j][3] = c[j].w ^ rk[3];
    }
    AES_ROUNDS_PIPELINED(kBlk, st, rk)
#pragma unroll
    for (int j = 0; j < kBlk; ++j) {
      uint32_t o0, o1, o2, o3;
      AES_FINAL(st[j][0], st[j][1], st[j][2], st[j][3], o0, o1, o2, o3, rk + 40, pv[j])
      const uint4 p = make_uint4(o0, o1, o2, o3);
      const int64_t b = b0 + 64 * j;
      const v4u pw = {o0, o1, o2, o3};  // a store past the segment's end is dropped by the range check
      __builtin_amdgcn_raw_buffer_store_b128(pw, d_rsrc, static_cast<uint32_t>(b) << 4, 0, 0);
      if constexpr (kHdr == 1) {  // does packet q = ceil(16 b / 188) start in this block?
        const uint32_t b16 = static_cast<uint32_t>(b) << 4;
        const uint32_t q = __umulhi(b16 + 187u, kDiv188Magic) >> 7;
        if (q * 188u - b16 < 16u && b < nblk) hdr.rec[hdrb + q] = p;
      }
      if (b == nblk - 1) out_len[cur] = pkcs7_len(p, nblk * 16);
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

// crc_mask_off / crc_wfrag / crc_masks: the fused ciphertext CRC (nullptr: off);
// hdr_off / hdr_rec: packet-header records for the demux scan (nullptr: off)
hipError_t launch_aes128_cbc_decrypt(const uint8_t* src, uint8_t* dst, const int64_t* src_off, const int64_t* dst_off,
                                     const int64_t* blk_prefix, const int64_t* chunk_prefix, const uint32_t* drk,
                                     const uint32_t* ivw, const uint32_t* tdl, const uint8_t* isb, int64_t* out_len,
                                     int nseg, int64_t total_chunks, int num_cu, hipStream_t stream,
                                     const int64_t* crc_mask_off, const void* crc_wfrag, uint32_t* crc_masks,
                                     const int64_t* hdr_off, void* hdr_rec) {
  if (total_chunks <= 0) return hipSuccess;
  int64_t grid, per_wg;
  aes_grid(total_chunks, num_cu, grid, per_wg);
  const AesCrc crc{crc_mask_off, reinterpret_cast<const v4i*>(crc_wfrag), crc_masks};
#define AES_LAUNCH(M, H)                                                                                          \
  hipLaunchKernelGGL((aes128_cbc_decrypt_kernel<M, H>), dim3(static_cast<unsigned>(grid)), dim3(kAesThreads), 0,     \
                     stream, src, dst, src_off, dst_off, blk_prefix, chunk_prefix, drk, ivw, tdl, isb, out_len, nseg, \
                     total_chunks, per_wg, crc, hdr)
  const AesHdr hdr{hdr_off, reinterpret_cast<uint4*>(hdr_rec)};
  const bool with_hdr = hdr_off != nullptr && hdr_rec != nullptr;
  if (crc_mask_off == nullptr) {
    if (with_hdr) AES_LAUNCH(0, 1); else AES_LAUNCH(0, 0);
  } else {
    if (with_hdr) AES_LAUNCH(1, 1); else AES_LAUNCH(1, 0);
  }
#undef AES_LAUNCH
  return hipGetLastError();
}

}  // namespace dev
}  // namespace hlsp2p
