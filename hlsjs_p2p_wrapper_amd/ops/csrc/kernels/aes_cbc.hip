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

namespace hlsp2p {
namespace dev {

constexpr int kAesThreads = 1024;
constexpr int kAesWgPerCu = 1;
constexpr int kBlk = 4;  // blocks per lane per chunk (chunk = 64 * kBlk blocks): independent chains
constexpr int kTdDwords = 2 * 256 * 64;  // regions A + B
constexpr int kIsDwords = 256 * 32;      // region C
constexpr uint32_t kIsRegion = 0x20000u;

// v_perm_b32 selector: byte k of the state word -> bits 8..15; bits 0..7 and 16..23 from
// the per-lane table base (S1 bytes 0 and 2); bits 24..31 = 0
#define SEL(k) (0x0c020000u | ((4u + (k)) << 8))
#define LDS32(addr) (*reinterpret_cast<const uint32_t*>(s_bytes + (addr)))
#define TD(t, w, k) LDS32(__builtin_amdgcn_perm((w), td_base[t], SEL(k)))
#define IS(w, k) LDS32(((((w) >> (8 * (k))) & 0xffu) << 7) + is_base)

// CDNA4 3-input bitwise op (truth table 0x96 = a ^ b ^ c); the round key is an SGPR operand
#define XOR3(a, b, c) __builtin_amdgcn_bitop3_b32((a), (b), (c), 0x96)

// little-endian column form of the equivalent inverse cipher round: TdtL = rotl(Td0L, 8t);
// per column 4 v_perm + 4 ds_read_b32 + 2 v_bitop3
#define AES_ROUND(s0, s1, s2, s3, t0, t1, t2, t3, k)                                     \
  t0 = XOR3(XOR3(TD(0, s0, 0), TD(1, s3, 1), TD(2, s2, 2)), TD(3, s1, 3), (k)[0]);      \
  t1 = XOR3(XOR3(TD(0, s1, 0), TD(1, s0, 1), TD(2, s3, 2)), TD(3, s2, 3), (k)[1]);      \
  t2 = XOR3(XOR3(TD(0, s2, 0), TD(1, s1, 1), TD(2, s0, 2)), TD(3, s3, 3), (k)[2]);      \
  t3 = XOR3(XOR3(TD(0, s3, 0), TD(1, s2, 1), TD(2, s1, 2)), TD(3, s0, 3), (k)[3]);

// The same round split in two phases (used by the kernel for explicit pipelining):
// 16 table addresses + 16 LDS reads of one state, then the 8 v_bitop3 that fold them.
#define TDA(t, w, k) __builtin_amdgcn_perm((w), td_base[t], SEL(k))
#define ROUND_READS(v, s)                                                                   \
  do {                                                                                      \
    uint32_t a_[16];                                                                        \
    a_[0] = TDA(0, s[0], 0); a_[1] = TDA(1, s[3], 1); a_[2] = TDA(2, s[2], 2); a_[3] = TDA(3, s[1], 3);     \
    a_[4] = TDA(0, s[1], 0); a_[5] = TDA(1, s[0], 1); a_[6] = TDA(2, s[3], 2); a_[7] = TDA(3, s[2], 3);     \
    a_[8] = TDA(0, s[2], 0); a_[9] = TDA(1, s[1], 1); a_[10] = TDA(2, s[0], 2); a_[11] = TDA(3, s[3], 3);   \
    a_[12] = TDA(0, s[3], 0); a_[13] = TDA(1, s[2], 1); a_[14] = TDA(2, s[1], 2); a_[15] = TDA(3, s[0], 3); \
    _Pragma("unroll") for (int q_ = 0; q_ < 16; ++q_) v[q_] = LDS32(a_[q_]);                \
  } while (0)
#define ROUND_XORS(s, v, k)                                                                 \
  do {                                                                                      \
    s[0] = XOR3(XOR3(v[0], v[1], v[2]), v[3], (k)[0]);                                      \
    s[1] = XOR3(XOR3(v[4], v[5], v[6]), v[7], (k)[1]);                                      \
    s[2] = XOR3(XOR3(v[8], v[9], v[10]), v[11], (k)[2]);                                    \
    s[3] = XOR3(XOR3(v[12], v[13], v[14]), v[15], (k)[3]);                                  \
  } while (0)

// final round fused with the CBC chaining: o = InvShiftRows/InvSubBytes(s) ^ k ^ px
#define AES_FINAL(s0, s1, s2, s3, o0, o1, o2, o3, k, px)                                                  \
  o0 = XOR3(IS(s0, 0) | (IS(s3, 1) << 8) | (IS(s2, 2) << 16) | (IS(s1, 3) << 24), (k)[0], (px).x);        \
  o1 = XOR3(IS(s1, 0) | (IS(s0, 1) << 8) | (IS(s3, 2) << 16) | (IS(s2, 3) << 24), (k)[1], (px).y);        \
  o2 = XOR3(IS(s2, 0) | (IS(s1, 1) << 8) | (IS(s0, 2) << 16) | (IS(s3, 3) << 24), (k)[2], (px).z);        \
  o3 = XOR3(IS(s3, 0) | (IS(s2, 1) << 8) | (IS(s1, 2) << 16) | (IS(s0, 3) << 24), (k)[3], (px).w);

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

// 64-bit wave-uniform value (lane 0's) -> SGPRs
__device__ __forceinline__ int64_t uniform64(int64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(static_cast<uint64_t>(v) >> 32));
  return static_cast<int64_t>((static_cast<uint64_t>(hi) << 32) | lo);
}

// tdl: little-endian Td0 (256 words); isb: inverse S-box (256 bytes)
// drk: per-segment little-endian equivalent-inverse-cipher round keys (44 words)
// chunk_prefix: exclusive prefix of per-segment 256-block chunks (one chunk = one wave
//   iteration: lane l decrypts blocks 64j + l, j < kBlk, so every load/store instruction
//   moves 1 KB contiguous); waves never straddle segments
__global__ __launch_bounds__(kAesThreads, 1) void aes128_cbc_decrypt_kernel(
    const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, const int64_t* __restrict__ src_off,
    const int64_t* __restrict__ dst_off, const int64_t* __restrict__ blk_prefix,
    const int64_t* __restrict__ chunk_prefix, const uint32_t* __restrict__ drk, const uint32_t* __restrict__ ivw,
    const uint32_t* __restrict__ tdl_g, const uint8_t* __restrict__ isb_g, int64_t* __restrict__ out_len, int nseg,
    int64_t total_chunks, int64_t per_wg) {
  __shared__ uint32_t s_tab[kTdDwords + kIsDwords];  // 160 KiB (layout above)
  const int tid = threadIdx.x;
  {  // image fill: thread tid writes dwords tid + 1024k, i.e. Td rows (tid >> 6) + 16(k & 15) in region
     // k >> 4 and InvSbox rows (tid >> 5) + 32k; all 24 source loads are issued before the
     // first LDS store (a strided load/store loop paid ~40 serialised L2 round trips)
    static_assert(kAesThreads == 1024 && kTdDwords == 32 * kAesThreads && kIsDwords == 8 * kAesThreads, "fill map");
    uint32_t td[16], is[8];
#pragma unroll
    for (int k = 0; k < 16; ++k) td[k] = tdl_g[(tid >> 6) + 16 * k];
#pragma unroll
    for (int k = 0; k < 8; ++k) is[k] = isb_g[(tid >> 5) + 32 * k];
    const int half = (tid >> 5) & 1;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      const uint32_t v = td[k & 15];
      const int rot = 8 * (2 * (k >> 4) + half);
      s_tab[tid + k * kAesThreads] = rot ? __builtin_amdgcn_alignbit(v, v, 32 - rot) : v;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) s_tab[kTdDwords + tid + k * kAesThreads] = is[k];
  }
  __syncthreads();
  const uint8_t* s_bytes = reinterpret_cast<const uint8_t*>(s_tab);
  const uint32_t l4 = static_cast<uint32_t>(tid & 31) << 2;
  const uint32_t td_base[4] = {l4, 128u | l4, 0x10000u | l4, 0x10000u | 128u | l4};  // Td0..Td3
  const uint32_t is_base = kIsRegion + l4;
  const int lane = tid & 63;
  constexpr int kWaves = kAesThreads / 64;

  // per_wg chunks per workgroup; wave w of the group takes chunks begin + w, + kWaves, ...
  const int64_t begin = static_cast<int64_t>(blockIdx.x) * per_wg;
  const int64_t end = begin + per_wg < total_chunks ? begin + per_wg : total_chunks;
  // segment state is wave-uniform (SGPRs): round keys come in by scalar loads
  int cur = -1;
  uint32_t rk[44];
  int64_t so = 0, dof = 0, cstart = 0, cend = 0, nblk = 0;
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
    }
    const int64_t b0 = (ch - cstart) * (64 * kBlk) + lane;  // this lane's first block
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
    // Rounds 1..9, software-pipelined across the chains IN SOURCE ORDER (the backend keeps
    // this huge unrolled block in emission order): chain j's 16 LDS reads are issued before
    // chain j-1's XORs consume theirs, so each wave keeps ~16 reads in flight instead of 2-3.
#pragma unroll
    for (int r = 1; r < 10; ++r) {
      const uint32_t* k = rk + 4 * r;
      uint32_t v[2][16];
      ROUND_READS(v[0], st[0]);
#pragma unroll
      for (int j = 1; j < kBlk; ++j) {
        ROUND_READS(v[j & 1], st[j]);
        ROUND_XORS(st[j - 1], v[(j - 1) & 1], k);
      }
      ROUND_XORS(st[kBlk - 1], v[(kBlk - 1) & 1], k);
    }
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
#undef TD
#undef IS
#undef LDS32
#undef SEL
#undef XOR3
#undef TDA
#undef ROUND_READS
#undef ROUND_XORS

// 16-byte blocks per wave iteration (the host sizes its chunk index space with this)
int aes_chunk_blocks() { return 64 * kBlk; }

hipError_t launch_aes128_cbc_decrypt(const uint8_t* src, uint8_t* dst, const int64_t* src_off, const int64_t* dst_off,
                                     const int64_t* blk_prefix, const int64_t* chunk_prefix, const uint32_t* drk,
                                     const uint32_t* ivw, const uint32_t* tdl, const uint8_t* isb, int64_t* out_len,
                                     int nseg, int64_t total_chunks, int num_cu, hipStream_t stream) {
  if (total_chunks <= 0) return hipSuccess;
  constexpr int64_t kWaves = kAesThreads / 64;
  const int64_t max_wg = static_cast<int64_t>(num_cu) * kAesWgPerCu;
  int64_t grid = (total_chunks + kWaves * 2 - 1) / (kWaves * 2);
  if (grid > max_wg) grid = max_wg;
  if (grid < 1) grid = 1;
  const int64_t per_wg = (total_chunks + grid - 1) / grid;
  grid = (total_chunks + per_wg - 1) / per_wg;
  hipLaunchKernelGGL(aes128_cbc_decrypt_kernel, dim3(static_cast<unsigned>(grid)), dim3(kAesThreads), 0, stream, src,
                     dst, src_off, dst_off, blk_prefix, chunk_prefix, drk, ivw, tdl, isb, out_len, nseg, total_chunks,
                     per_wg);
  return hipGetLastError();
}

}  // namespace dev
}  // namespace hlsp2p
