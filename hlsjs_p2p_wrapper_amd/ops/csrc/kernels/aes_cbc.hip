// AES-128-CBC decryption of a batch of HLS segments — CDNA4 / gfx950.
//
// CBC *decryption* is block-parallel: P_i = D_K(C_i) xor C_{i-1}.  Work unit = a PAIR of
// consecutive 16-byte blocks of one segment: each lane runs two independent AES chains
// interleaved (ILP hides the LDS latency of a round's dependent lookups) and moves 32
// contiguous bytes; C_{i-1} for the pair's first block is an L1 hit (neighbour lane).
//
// AES is table bound, not matmul shaped (no MFMA).  Design for the CDNA4 LDS + VALU:
//  * Tables in LITTLE-ENDIAN column form (TdL = bswap(Td0), round keys pre-swapped on the
//    host), so state words are used exactly as loaded — no byte swaps in the kernel.
//  * One 64 KiB LDS image of 256 rows x 256 B: row x = [32 lane copies of TdL[x] | 32 lane
//    copies of InvSbox[x]].  Lane l reads word l (Td) or word 32+l (S-box) of the row, so
//    for ds_read_b32 (bank = dword % 32) every lane of a 32-lane half owns a bank: both the
//    144 Td lookups and the 16 final-round S-box lookups per block are conflict-free.
//  * With 256-byte rows the LDS byte address of entry x for lane l is  (x << 8) | (l << 2)
//    [| 128 for the S-box] — ONE v_perm_b32 builds it from the state word (selects byte k
//    into bits 8..15, the lane offset into bits 0..7), instead of extract + shift-or.
//    Per round: 16 v_perm + 16 ds_read_b32 + 12 v_alignbit (Td1..Td3 are rotations of Td0)
//    + 16 v_xor.
//  * 512-thread workgroups (8 waves) share the 64 KiB image: 2 per CU = 4 waves per SIMD.
//
// Persistent grid (2 workgroups per CU), each streaming one contiguous range of the batch's
// pair index space; the segment table is walked monotonically so per-segment state (44
// round keys, IV, offsets) reloads only at boundaries.  PKCS#7: the lane holding a
// segment's last block validates the padding and writes the plaintext length (or -1) to
// out_len[seg] on device — the demux kernels read it directly (no host round trip).
#include "common.h"

namespace hlsp2p {
namespace dev {

constexpr int kAesThreads = 512;
constexpr int kAesWgPerCu = 2;

// v_perm_b32 selectors: byte k of the state word -> bits 8..15, lane offset byte -> 0..7
#define SEL(k) (0x0c0c0000u | ((4u + (k)) << 8))
#define LDS32(addr) (*reinterpret_cast<const uint32_t*>(s_bytes + (addr)))
#define TD(w, k) LDS32(__builtin_amdgcn_perm((w), td_base, SEL(k)))
#define IS(w, k) LDS32(__builtin_amdgcn_perm((w), is_base, SEL(k)))
#define ROTL(x, s) __builtin_amdgcn_alignbit((x), (x), 32 - (s))

// little-endian column form of the equivalent inverse cipher round
#define AES_ROUND(s0, s1, s2, s3, t0, t1, t2, t3, k)                                            \
  t0 = TD(s0, 0) ^ ROTL(TD(s3, 1), 8) ^ ROTL(TD(s2, 2), 16) ^ ROTL(TD(s1, 3), 24) ^ (k)[0];     \
  t1 = TD(s1, 0) ^ ROTL(TD(s0, 1), 8) ^ ROTL(TD(s3, 2), 16) ^ ROTL(TD(s2, 3), 24) ^ (k)[1];     \
  t2 = TD(s2, 0) ^ ROTL(TD(s1, 1), 8) ^ ROTL(TD(s0, 2), 16) ^ ROTL(TD(s3, 3), 24) ^ (k)[2];     \
  t3 = TD(s3, 0) ^ ROTL(TD(s2, 1), 8) ^ ROTL(TD(s1, 2), 16) ^ ROTL(TD(s0, 3), 24) ^ (k)[3];

#define AES_FINAL(s0, s1, s2, s3, o0, o1, o2, o3, k)                                               \
  o0 = (IS(s0, 0) | (IS(s3, 1) << 8) | (IS(s2, 2) << 16) | (IS(s1, 3) << 24)) ^ (k)[0];           \
  o1 = (IS(s1, 0) | (IS(s0, 1) << 8) | (IS(s3, 2) << 16) | (IS(s2, 3) << 24)) ^ (k)[1];           \
  o2 = (IS(s2, 0) | (IS(s1, 1) << 8) | (IS(s0, 2) << 16) | (IS(s3, 3) << 24)) ^ (k)[2];           \
  o3 = (IS(s3, 0) | (IS(s2, 1) << 8) | (IS(s1, 2) << 16) | (IS(s0, 3) << 24)) ^ (k)[3];

__device__ __forceinline__ int64_t pkcs7_len(uint4 p, int64_t nbytes) {
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

// tdl: little-endian Td0 (256 words); isb: inverse S-box (256 bytes)
// drk: per-segment little-endian equivalent-inverse-cipher round keys (44 words)
__global__ __launch_bounds__(kAesThreads, 1) void aes128_cbc_decrypt_kernel(
    const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, const int64_t* __restrict__ src_off,
    const int64_t* __restrict__ dst_off, const int64_t* __restrict__ blk_prefix,
    const int64_t* __restrict__ pair_prefix, const uint32_t* __restrict__ drk, const uint32_t* __restrict__ ivw,
    const uint32_t* __restrict__ tdl_g, const uint8_t* __restrict__ isb_g, int64_t* __restrict__ out_len, int nseg,
    int64_t total_pairs, int64_t per_wg) {
  __shared__ uint32_t s_tab[256 * 64];  // 64 KiB: [row x][32 TdL copies | 32 InvSbox copies]
  const int tid = threadIdx.x;
  for (int i = tid; i < 256 * 64; i += kAesThreads) {
    const int row = i >> 6, col = i & 63;
    s_tab[i] = col < 32 ? tdl_g[row] : static_cast<uint32_t>(isb_g[row]);
  }
  __syncthreads();
  const uint8_t* s_bytes = reinterpret_cast<const uint8_t*>(s_tab);
  const uint32_t l32 = tid & 31;
  const uint32_t td_base = l32 << 2;          // byte offset of this lane's Td copy in a row
  const uint32_t is_base = 128u | (l32 << 2);  // ... and of its S-box copy

  const int64_t begin = static_cast<int64_t>(blockIdx.x) * per_wg;
  const int64_t end = begin + per_wg < total_pairs ? begin + per_wg : total_pairs;
  int cur = -1;
  uint32_t rk[44];
  uint32_t iv0 = 0, iv1 = 0, iv2 = 0, iv3 = 0;
  int64_t so = 0, dof = 0, pstart = 0, pend = 0, nblk = 0;
  for (int64_t gp = begin + tid; gp < end; gp += kAesThreads) {
    if (cur < 0 || gp >= pend) {
      cur = cur < 0 ? find_seg(pair_prefix, nseg, gp) : advance_seg(pair_prefix, cur, gp);
#pragma unroll
      for (int k = 0; k < 44; ++k) rk[k] = drk[cur * 44 + k];
      iv0 = ivw[cur * 4 + 0]; iv1 = ivw[cur * 4 + 1]; iv2 = ivw[cur * 4 + 2]; iv3 = ivw[cur * 4 + 3];
      so = src_off[cur];
      dof = dst_off[cur];
      pstart = pair_prefix[cur];
      pend = pair_prefix[cur + 1];
      nblk = blk_prefix[cur + 1] - blk_prefix[cur];
    }
    const int64_t i0 = 2 * (gp - pstart);
    const bool has2 = i0 + 1 < nblk;
    const uint4* cp = reinterpret_cast<const uint4*>(src + so) + i0;
    const uint4 c0 = cp[0];
    const uint4 c1 = has2 ? cp[1] : c0;
    uint4 pv;
    if (i0 == 0) {
      pv = make_uint4(iv0, iv1, iv2, iv3);
    } else {
      pv = cp[-1];
    }
    uint32_t a0 = c0.x ^ rk[0], a1 = c0.y ^ rk[1], a2 = c0.z ^ rk[2], a3 = c0.w ^ rk[3];
    uint32_t b0 = c1.x ^ rk[0], b1 = c1.y ^ rk[1], b2 = c1.z ^ rk[2], b3 = c1.w ^ rk[3];
#pragma unroll
    for (int r = 1; r < 10; ++r) {
      uint32_t t0, t1, t2, t3, u0, u1, u2, u3;
      AES_ROUND(a0, a1, a2, a3, t0, t1, t2, t3, rk + 4 * r)
      AES_ROUND(b0, b1, b2, b3, u0, u1, u2, u3, rk + 4 * r)
      a0 = t0; a1 = t1; a2 = t2; a3 = t3;
      b0 = u0; b1 = u1; b2 = u2; b3 = u3;
    }
    uint32_t o0, o1, o2, o3, q0, q1, q2, q3;
    AES_FINAL(a0, a1, a2, a3, o0, o1, o2, o3, rk + 40)
    AES_FINAL(b0, b1, b2, b3, q0, q1, q2, q3, rk + 40)
    const uint4 p0 = make_uint4(o0 ^ pv.x, o1 ^ pv.y, o2 ^ pv.z, o3 ^ pv.w);
    const uint4 p1 = make_uint4(q0 ^ c0.x, q1 ^ c0.y, q2 ^ c0.z, q3 ^ c0.w);
    uint4* dp = reinterpret_cast<uint4*>(dst + dof) + i0;
    dp[0] = p0;
    if (has2) dp[1] = p1;
    if (i0 == nblk - 1) out_len[cur] = pkcs7_len(p0, nblk * 16);
    if (has2 && i0 + 1 == nblk - 1) out_len[cur] = pkcs7_len(p1, nblk * 16);
  }
}
#undef TD
#undef IS
#undef LDS32
#undef SEL
#undef ROTL

hipError_t launch_aes128_cbc_decrypt(const uint8_t* src, uint8_t* dst, const int64_t* src_off, const int64_t* dst_off,
                                     const int64_t* blk_prefix, const int64_t* pair_prefix, const uint32_t* drk,
                                     const uint32_t* ivw, const uint32_t* tdl, const uint8_t* isb, int64_t* out_len,
                                     int nseg, int64_t total_pairs, int num_cu, hipStream_t stream) {
  if (total_pairs <= 0) return hipSuccess;
  const int64_t max_wg = static_cast<int64_t>(num_cu) * kAesWgPerCu;
  int64_t grid = (total_pairs + kAesThreads * 4 - 1) / (kAesThreads * 4);
  if (grid > max_wg) grid = max_wg;
  if (grid < 1) grid = 1;
  int64_t per_wg = (total_pairs + grid - 1) / grid;
  per_wg = (per_wg + kAesThreads - 1) / kAesThreads * kAesThreads;
  grid = (total_pairs + per_wg - 1) / per_wg;
  hipLaunchKernelGGL(aes128_cbc_decrypt_kernel, dim3(static_cast<unsigned>(grid)), dim3(kAesThreads), 0, stream, src,
                     dst, src_off, dst_off, blk_prefix, pair_prefix, drk, ivw, tdl, isb, out_len, nseg, total_pairs,
                     per_wg);
  return hipGetLastError();
}

}  // namespace dev
}  // namespace hlsp2p
