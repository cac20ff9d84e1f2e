// AES-128-CBC decryption of a batch of HLS segments — CDNA4 / gfx950.
//
// CBC *decryption* is block-parallel: P_i = D_K(C_i) xor C_{i-1}.  One lane decrypts one
// 16-byte block per iteration; consecutive lanes take consecutive blocks, so every wave
// moves 1 KiB with fully coalesced dwordx4 loads/stores (the C_{i-1} re-load hits L1).
//
// AES is table/bit bound, not matmul shaped (no MFMA).  The limiter is LDS: each block
// does 144 T-table lookups + 16 inverse-S-box lookups.  Random 32-bit lookups into a
// 1 KiB table from 32 lanes hit the 32 banks of ds_read_b32 with ~3-4-way conflicts, so
// the tables are REPLICATED 32x with entry e of copy c at word e*32 + c and lane l reads
// copy (l & 31): every lane of a 32-lane group owns a bank -> conflict-free, 2 LDS
// cycles per wave lookup.  Td1..Td3 are byte rotations of Td0 (v_alignbit), so the
// whole working set is Td0 x32 (32 KiB) + InvSbox x32 (32 KiB) = 64 KiB -> 2
// workgroups (8 waves) per CU; the VALU work (~700 ops/block) and LDS work balance at
// roughly 5 CU-cycles per block.
//
// Persistent grid: 2 workgroups per CU, each streams one contiguous range of the batch's
// global block index space (good DRAM locality), walking the segment table monotonically
// so the per-segment state (44 round keys, IV, offsets) is reloaded only at boundaries.
// PKCS#7: the lane that decrypts a segment's last block validates the padding and writes
// the plaintext length (or -1) to out_len[seg] — the demux kernels read it on device, so
// no host round trip sits between decrypt and demux.
#include "common.h"

namespace hlsp2p {
namespace dev {

constexpr int kAesThreads = 256;
constexpr int kRep = 32;

__global__ __launch_bounds__(kAesThreads, 2) void aes128_cbc_decrypt_kernel(
    const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, const int64_t* __restrict__ src_off,
    const int64_t* __restrict__ dst_off, const int64_t* __restrict__ blk_prefix, const uint32_t* __restrict__ drk,
    const uint32_t* __restrict__ ivw, const uint32_t* __restrict__ td0_g, const uint8_t* __restrict__ isb_g,
    int64_t* __restrict__ out_len, int nseg, int64_t total, int64_t per_wg) {
  __shared__ uint32_t s_td[256 * kRep];
  __shared__ uint32_t s_is[256 * kRep];
  const int tid = threadIdx.x;
  const uint32_t l32 = tid & 31;
  for (int i = tid; i < 256 * kRep; i += kAesThreads) {
    s_td[i] = td0_g[i >> 5];
    s_is[i] = isb_g[i >> 5];
  }
  __syncthreads();

  const int64_t begin = static_cast<int64_t>(blockIdx.x) * per_wg;
  const int64_t end = begin + per_wg < total ? begin + per_wg : total;

#define TD(x) s_td[((x) << 5) | l32]
#define IS(x) s_is[((x) << 5) | l32]

  int cur = -1;
  uint32_t rk[44];
  uint32_t iv0 = 0, iv1 = 0, iv2 = 0, iv3 = 0;
  int64_t so = 0, dof = 0, bstart = 0, bend = 0;
  for (int64_t gb = begin + tid; gb < end; gb += kAesThreads) {
    if (cur < 0 || gb >= bend) {
      cur = cur < 0 ? find_seg(blk_prefix, nseg, gb) : advance_seg(blk_prefix, cur, gb);
#pragma unroll
      for (int k = 0; k < 44; ++k) rk[k] = drk[cur * 44 + k];
      iv0 = ivw[cur * 4 + 0]; iv1 = ivw[cur * 4 + 1]; iv2 = ivw[cur * 4 + 2]; iv3 = ivw[cur * 4 + 3];
      so = src_off[cur];
      dof = dst_off[cur];
      bstart = blk_prefix[cur];
      bend = blk_prefix[cur + 1];
    }
    const int64_t i = gb - bstart;
    const uint4* cp = reinterpret_cast<const uint4*>(src + so) + i;
    const uint4 c = *cp;
    uint4 pv;
    if (i == 0) {
      pv.x = iv0; pv.y = iv1; pv.z = iv2; pv.w = iv3;
    } else {
      pv = cp[-1];
    }
    uint32_t s0 = bswap32(c.x) ^ rk[0], s1 = bswap32(c.y) ^ rk[1], s2 = bswap32(c.z) ^ rk[2],
             s3 = bswap32(c.w) ^ rk[3];
#pragma unroll
    for (int r = 1; r < 10; ++r) {
      const uint32_t t0 = TD(s0 >> 24) ^ rotr(TD((s3 >> 16) & 0xff), 8) ^ rotr(TD((s2 >> 8) & 0xff), 16) ^
                          rotr(TD(s1 & 0xff), 24) ^ rk[4 * r + 0];
      const uint32_t t1 = TD(s1 >> 24) ^ rotr(TD((s0 >> 16) & 0xff), 8) ^ rotr(TD((s3 >> 8) & 0xff), 16) ^
                          rotr(TD(s2 & 0xff), 24) ^ rk[4 * r + 1];
      const uint32_t t2 = TD(s2 >> 24) ^ rotr(TD((s1 >> 16) & 0xff), 8) ^ rotr(TD((s0 >> 8) & 0xff), 16) ^
                          rotr(TD(s3 & 0xff), 24) ^ rk[4 * r + 2];
      const uint32_t t3 = TD(s3 >> 24) ^ rotr(TD((s2 >> 16) & 0xff), 8) ^ rotr(TD((s1 >> 8) & 0xff), 16) ^
                          rotr(TD(s0 & 0xff), 24) ^ rk[4 * r + 3];
      s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    const uint32_t o0 = ((IS(s0 >> 24) << 24) | (IS((s3 >> 16) & 0xff) << 16) | (IS((s2 >> 8) & 0xff) << 8) |
                         IS(s1 & 0xff)) ^ rk[40];
    const uint32_t o1 = ((IS(s1 >> 24) << 24) | (IS((s0 >> 16) & 0xff) << 16) | (IS((s3 >> 8) & 0xff) << 8) |
                         IS(s2 & 0xff)) ^ rk[41];
    const uint32_t o2 = ((IS(s2 >> 24) << 24) | (IS((s1 >> 16) & 0xff) << 16) | (IS((s0 >> 8) & 0xff) << 8) |
                         IS(s3 & 0xff)) ^ rk[42];
    const uint32_t o3 = ((IS(s3 >> 24) << 24) | (IS((s2 >> 16) & 0xff) << 16) | (IS((s1 >> 8) & 0xff) << 8) |
                         IS(s0 & 0xff)) ^ rk[43];
    uint4 p;
    p.x = bswap32(o0) ^ pv.x;
    p.y = bswap32(o1) ^ pv.y;
    p.z = bswap32(o2) ^ pv.z;
    p.w = bswap32(o3) ^ pv.w;
    reinterpret_cast<uint4*>(dst + dof)[i] = p;
    if (gb == bend - 1) {  // last block of the segment: PKCS#7 check
      const uint32_t pad = p.w >> 24;
      int64_t len = -1;
      if (pad >= 1 && pad <= 16) {
        bool ok = true;
        const uint32_t w[4] = {p.x, p.y, p.z, p.w};
#pragma unroll
        for (int b = 0; b < 16; ++b) {
          const uint32_t byte = (w[b >> 2] >> (8 * (b & 3))) & 0xff;
          if (b >= 16 - static_cast<int>(pad) && byte != pad) ok = false;
        }
        if (ok) len = (bend - bstart) * 16 - static_cast<int64_t>(pad);
      }
      out_len[cur] = len;
    }
  }
#undef TD
#undef IS
}

hipError_t launch_aes128_cbc_decrypt(const uint8_t* src, uint8_t* dst, const int64_t* src_off, const int64_t* dst_off,
                                     const int64_t* blk_prefix, const uint32_t* drk, const uint32_t* ivw,
                                     const uint32_t* td0, const uint8_t* isb, int64_t* out_len, int nseg,
                                     int64_t total_blocks, int num_cu, hipStream_t stream) {
  if (total_blocks <= 0) return hipSuccess;
  const int64_t max_wg = static_cast<int64_t>(num_cu) * 2;
  int64_t grid = (total_blocks + kAesThreads * 4 - 1) / (kAesThreads * 4);
  if (grid > max_wg) grid = max_wg;
  if (grid < 1) grid = 1;
  int64_t per_wg = (total_blocks + grid - 1) / grid;
  per_wg = (per_wg + kAesThreads - 1) / kAesThreads * kAesThreads;
  grid = (total_blocks + per_wg - 1) / per_wg;
  hipLaunchKernelGGL(aes128_cbc_decrypt_kernel, dim3(static_cast<unsigned>(grid)), dim3(kAesThreads), 0, stream, src,
                     dst, src_off, dst_off, blk_prefix, drk, ivw, td0, isb, out_len, nseg, total_blocks, per_wg);
  return hipGetLastError();
}

}  // namespace dev
}  // namespace hlsp2p
