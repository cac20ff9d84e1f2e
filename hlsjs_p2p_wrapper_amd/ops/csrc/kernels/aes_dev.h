// AES-128 decryption building blocks of the CDNA4 bulk CBC decrypt (aes_cbc.hip).
//
// The per-CU 160 KiB LDS IMAGE (1024-thread workgroups): Td0..Td3 in little-endian column
// form, 32 lane copies per row, plus 32 copies of InvSbox — every lookup of a 32-lane group
// is bank-conflict free (layout in aes_cbc.hip's header).  Used through the macros below,
// which expect `s_bytes`, `td_base[4]` and `is_base` in scope (aes_image_fill +
// aes_image_bases set them up).
//
// Round keys: per segment 44 little-endian words of the equivalent inverse cipher (host
// pre-swapped): [0..3] initial whitening, [4r..4r+3] round r (1..9), [40..43] last round.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hlsp2p {
namespace dev {

constexpr int kAesImageThreads = 1024;
constexpr int kTdDwords = 2 * 256 * 64;  // image regions A + B
constexpr int kIsDwords = 256 * 32;      // image region C
constexpr uint32_t kIsRegion = 0x20000u;

// v_perm_b32 selector: byte k of the state word -> bits 8..15; bits 0..7 and 16..23 from
// the per-lane table base (S1 bytes 0 and 2); bits 24..31 = 0
#define AES_SEL(k) (0x0c020000u | ((4u + (k)) << 8))
#define AES_LDS32(addr) (*reinterpret_cast<const uint32_t*>(s_bytes + (addr)))
#define AES_TD(t, w, k) AES_LDS32(__builtin_amdgcn_perm((w), td_base[t], AES_SEL(k)))
#define AES_IS(w, k) AES_LDS32(((((w) >> (8 * (k))) & 0xffu) << 7) + is_base)

// CDNA4 3-input bitwise op (truth table 0x96 = a ^ b ^ c); the round key is an SGPR operand
#define AES_XOR3(a, b, c) __builtin_amdgcn_bitop3_b32((a), (b), (c), 0x96)

// One round split in two phases (explicit software pipelining across chains): 16 table
// addresses + 16 LDS reads of one state, then the 8 v_bitop3 that fold them.
#define AES_TDA(t, w, k) __builtin_amdgcn_perm((w), td_base[t], AES_SEL(k))
#define AES_ROUND_READS(v, s)                                                                                     \
  do {                                                                                                            \
    uint32_t a_[16];                                                                                              \
    a_[0] = AES_TDA(0, s[0], 0); a_[1] = AES_TDA(1, s[3], 1); a_[2] = AES_TDA(2, s[2], 2); a_[3] = AES_TDA(3, s[1], 3);     \
    a_[4] = AES_TDA(0, s[1], 0); a_[5] = AES_TDA(1, s[0], 1); a_[6] = AES_TDA(2, s[3], 2); a_[7] = AES_TDA(3, s[2], 3);     \
    a_[8] = AES_TDA(0, s[2], 0); a_[9] = AES_TDA(1, s[1], 1); a_[10] = AES_TDA(2, s[0], 2); a_[11] = AES_TDA(3, s[3], 3);   \
    a_[12] = AES_TDA(0, s[3], 0); a_[13] = AES_TDA(1, s[2], 1); a_[14] = AES_TDA(2, s[1], 2); a_[15] = AES_TDA(3, s[0], 3); \
    _Pragma("unroll") for (int q_ = 0; q_ < 16; ++q_) v[q_] = AES_LDS32(a_[q_]);                                  \
  } while (0)
#define AES_ROUND_XORS(s, v, k)                                                                                   \
  do {                                                                                                            \
    s[0] = AES_XOR3(AES_XOR3(v[0], v[1], v[2]), v[3], (k)[0]);                                                    \
    s[1] = AES_XOR3(AES_XOR3(v[4], v[5], v[6]), v[7], (k)[1]);                                                    \
    s[2] = AES_XOR3(AES_XOR3(v[8], v[9], v[10]), v[11], (k)[2]);                                                  \
    s[3] = AES_XOR3(AES_XOR3(v[12], v[13], v[14]), v[15], (k)[3]);                                                \
  } while (0)

// final round fused with the CBC chaining: o = InvShiftRows/InvSubBytes(s) ^ k ^ px.  The
// InvSbox image is replicated (every byte of a row's dwords holds InvSbox[x]): two v_perm pick the four output bytes into disjoint byte lanes, one
// 3-input XOR merges them with the round key, one XOR applies the CBC chaining input
#define AES_FINAL(s0, s1, s2, s3, o0, o1, o2, o3, k, px)                                                      \
  o0 = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_perm(AES_IS(s3, 1), AES_IS(s0, 0), 0x0c0c0500u),               \
                                   __builtin_amdgcn_perm(AES_IS(s1, 3), AES_IS(s2, 2), 0x07020c0cu), (k)[0], 0x96) ^ \
       (px).x;                                                                                                    \
  o1 = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_perm(AES_IS(s0, 1), AES_IS(s1, 0), 0x0c0c0500u),               \
                                   __builtin_amdgcn_perm(AES_IS(s2, 3), AES_IS(s3, 2), 0x07020c0cu), (k)[1], 0x96) ^ \
       (px).y;                                                                                                    \
  o2 = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_perm(AES_IS(s1, 1), AES_IS(s2, 0), 0x0c0c0500u),               \
                                   __builtin_amdgcn_perm(AES_IS(s3, 3), AES_IS(s0, 2), 0x07020c0cu), (k)[2], 0x96) ^ \
       (px).z;                                                                                                    \
  o3 = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_perm(AES_IS(s2, 1), AES_IS(s3, 0), 0x0c0c0500u),               \
                                   __builtin_amdgcn_perm(AES_IS(s0, 3), AES_IS(s1, 2), 0x07020c0cu), (k)[3], 0x96) ^ \
       (px).w;

// Rounds 1..9 of N independent chains, software-pipelined IN SOURCE ORDER (the backend keeps
// the unrolled block in emission order): chain j's 16 LDS reads are issued before chain
// j-1's XORs consume theirs, so a wave keeps ~16 reads in flight instead of 2-3.
#define AES_ROUNDS_PIPELINED(N, st, rk)                                                                           \
  _Pragma("unroll") for (int r_ = 1; r_ < 10; ++r_) {                                                             \
    const uint32_t* k_ = (rk) + 4 * r_;                                                                           \
    uint32_t v_[2][16];                                                                                           \
    AES_ROUND_READS(v_[0], st[0]);                                                                                \
    _Pragma("unroll") for (int j_ = 1; j_ < (N); ++j_) {                                                          \
      AES_ROUND_READS(v_[j_ & 1], st[j_]);                                                                        \
      AES_ROUND_XORS(st[j_ - 1], v_[(j_ - 1) & 1], k_);                                                           \
    }                                                                                                             \
    AES_ROUND_XORS(st[(N) - 1], v_[((N) - 1) & 1], k_);                                                           \
  }

// Fill the 160 KiB image (1024 threads): thread tid writes dwords tid + 1024k, i.e. Td rows
// (tid >> 6) + 16(k & 15) in region k >> 4 and InvSbox rows (tid >> 5) + 32k; all 24 source
// loads are issued before the first LDS store (a strided load/store loop paid ~40
// serialised L2 round trips).  The caller synchronises.
__device__ __forceinline__ void aes_image_fill(uint32_t* s_tab, const uint32_t* __restrict__ tdl_g,
                                               const uint8_t* __restrict__ isb_g, int tid) {
  static_assert(kTdDwords == 32 * kAesImageThreads && kIsDwords == 8 * kAesImageThreads, "fill map");
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
    s_tab[tid + k * kAesImageThreads] = rot ? __builtin_amdgcn_alignbit(v, v, 32 - rot) : v;
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) s_tab[kTdDwords + tid + k * kAesImageThreads] = is[k] * 0x01010101u;
}

// Per-lane image bases: Td address of entry x for lane l = (region << 16) | (x << 8) |
// (half << 7) | (l << 2) (ONE v_perm builds it from a state word).
__device__ __forceinline__ void aes_image_bases(int tid, uint32_t td_base[4], uint32_t& is_base) {
  const uint32_t l4 = static_cast<uint32_t>(tid & 31) << 2;
  td_base[0] = l4;
  td_base[1] = 128u | l4;
  td_base[2] = 0x10000u | l4;
  td_base[3] = 0x10000u | 128u | l4;
  is_base = kIsRegion + l4;
}

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

}  // namespace dev
}  // namespace hlsp2p
