#include "aes_host.hpp"

#include <cstring>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

namespace hlsp2p {
namespace aes {
namespace {

inline uint8_t xtime(uint8_t x) { return static_cast<uint8_t>((x << 1) ^ ((x & 0x80) ? 0x1b : 0x00)); }

uint8_t gmul(uint8_t a, uint8_t b) {
  uint8_t p = 0;
  while (b) {
    if (b & 1) p ^= a;
    a = xtime(a);
    b >>= 1;
  }
  return p;
}

inline uint32_t rotr8(uint32_t x) { return (x >> 8) | (x << 24); }
inline uint32_t rotr16(uint32_t x) { return (x >> 16) | (x << 16); }
inline uint32_t rotr24(uint32_t x) { return (x >> 24) | (x << 8); }

// Build S-box from the field inverse + affine map (FIPS-197 §5.1.1) — no literal tables.
Tables build_tables() {
  Tables t{};
  uint8_t inv[256];
  inv[0] = 0;
  for (int a = 1; a < 256; ++a) {
    for (int b = 1; b < 256; ++b) {
      if (gmul(static_cast<uint8_t>(a), static_cast<uint8_t>(b)) == 1) {
        inv[a] = static_cast<uint8_t>(b);
        break;
      }
    }
  }
  for (int x = 0; x < 256; ++x) {
    uint8_t b = inv[x];
    uint8_t s = b;
    for (int i = 1; i <= 4; ++i) s ^= static_cast<uint8_t>((b << i) | (b >> (8 - i)));
    s ^= 0x63;
    t.sbox[x] = s;
    t.inv_sbox[s] = static_cast<uint8_t>(x);
  }
  for (int x = 0; x < 256; ++x) {
    uint8_t s = t.sbox[x];
    t.te0[x] = (uint32_t(gmul(s, 2)) << 24) | (uint32_t(s) << 16) | (uint32_t(s) << 8) | uint32_t(gmul(s, 3));
    uint8_t si = t.inv_sbox[x];
    t.td0[x] = (uint32_t(gmul(si, 14)) << 24) | (uint32_t(gmul(si, 9)) << 16) | (uint32_t(gmul(si, 13)) << 8) |
               uint32_t(gmul(si, 11));
  }
  return t;
}

inline uint32_t load_be(const uint8_t* p) {
  return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | uint32_t(p[3]);
}
inline void store_be(uint8_t* p, uint32_t v) {
  p[0] = uint8_t(v >> 24);
  p[1] = uint8_t(v >> 16);
  p[2] = uint8_t(v >> 8);
  p[3] = uint8_t(v);
}

}  // namespace

const Tables& tables() {
  static const Tables t = build_tables();
  return t;
}

void expand_key_enc(const uint8_t key[16], uint32_t rk[44]) {
  const Tables& T = tables();
  for (int i = 0; i < 4; ++i) rk[i] = load_be(key + 4 * i);
  uint8_t rcon = 1;
  for (int i = 4; i < 44; ++i) {
    uint32_t tmp = rk[i - 1];
    if (i % 4 == 0) {
      tmp = (uint32_t(T.sbox[(tmp >> 16) & 0xff]) << 24) | (uint32_t(T.sbox[(tmp >> 8) & 0xff]) << 16) |
            (uint32_t(T.sbox[tmp & 0xff]) << 8) | uint32_t(T.sbox[tmp >> 24]);
      tmp ^= uint32_t(rcon) << 24;
      rcon = xtime(rcon);
    }
    rk[i] = rk[i - 4] ^ tmp;
  }
}

void expand_key_dec(const uint8_t key[16], uint32_t drk[44]) {
  const Tables& T = tables();
  uint32_t rk[44];
  expand_key_enc(key, rk);
  for (int r = 0; r <= 10; ++r)
    for (int c = 0; c < 4; ++c) drk[4 * r + c] = rk[4 * (10 - r) + c];
  for (int r = 1; r < 10; ++r) {
    for (int c = 0; c < 4; ++c) {
      uint32_t w = drk[4 * r + c];
      drk[4 * r + c] = T.td0[T.sbox[w >> 24]] ^ rotr8(T.td0[T.sbox[(w >> 16) & 0xff]]) ^
                       rotr16(T.td0[T.sbox[(w >> 8) & 0xff]]) ^ rotr24(T.td0[T.sbox[w & 0xff]]);
    }
  }
}

void encrypt_block(const uint32_t rk[44], const uint8_t in[16], uint8_t out[16]) {
  const Tables& T = tables();
  uint32_t s0 = load_be(in) ^ rk[0], s1 = load_be(in + 4) ^ rk[1], s2 = load_be(in + 8) ^ rk[2],
           s3 = load_be(in + 12) ^ rk[3];
  for (int r = 1; r < 10; ++r) {
    const uint32_t* k = rk + 4 * r;
    uint32_t t0 = T.te0[s0 >> 24] ^ rotr8(T.te0[(s1 >> 16) & 0xff]) ^ rotr16(T.te0[(s2 >> 8) & 0xff]) ^
                  rotr24(T.te0[s3 & 0xff]) ^ k[0];
    uint32_t t1 = T.te0[s1 >> 24] ^ rotr8(T.te0[(s2 >> 16) & 0xff]) ^ rotr16(T.te0[(s3 >> 8) & 0xff]) ^
                  rotr24(T.te0[s0 & 0xff]) ^ k[1];
    uint32_t t2 = T.te0[s2 >> 24] ^ rotr8(T.te0[(s3 >> 16) & 0xff]) ^ rotr16(T.te0[(s0 >> 8) & 0xff]) ^
                  rotr24(T.te0[s1 & 0xff]) ^ k[2];
    uint32_t t3 = T.te0[s3 >> 24] ^ rotr8(T.te0[(s0 >> 16) & 0xff]) ^ rotr16(T.te0[(s1 >> 8) & 0xff]) ^
                  rotr24(T.te0[s2 & 0xff]) ^ k[3];
    s0 = t0; s1 = t1; s2 = t2; s3 = t3;
  }
  const uint32_t* k = rk + 40;
  auto S = [&](uint32_t v, int sh) { return uint32_t(T.sbox[(v >> sh) & 0xff]); };
  store_be(out, (S(s0, 24) << 24 | S(s1, 16) << 16 | S(s2, 8) << 8 | S(s3, 0)) ^ k[0]);
  store_be(out + 4, (S(s1, 24) << 24 | S(s2, 16) << 16 | S(s3, 8) << 8 | S(s0, 0)) ^ k[1]);
  store_be(out + 8, (S(s2, 24) << 24 | S(s3, 16) << 16 | S(s0, 8) << 8 | S(s1, 0)) ^ k[2]);
  store_be(out + 12, (S(s3, 24) << 24 | S(s0, 16) << 16 | S(s1, 8) << 8 | S(s2, 0)) ^ k[3]);
}

void decrypt_block(const uint32_t drk[44], const uint8_t in[16], uint8_t out[16]) {
  const Tables& T = tables();
  uint32_t s0 = load_be(in) ^ drk[0], s1 = load_be(in + 4) ^ drk[1], s2 = load_be(in + 8) ^ drk[2],
           s3 = load_be(in + 12) ^ drk[3];
  for (int r = 1; r < 10; ++r) {
    const uint32_t* k = drk + 4 * r;
    uint32_t t0 = T.td0[s0 >> 24] ^ rotr8(T.td0[(s3 >> 16) & 0xff]) ^ rotr16(T.td0[(s2 >> 8) & 0xff]) ^
                  rotr24(T.td0[s1 & 0xff]) ^ k[0];
    uint32_t t1 = T.td0[s1 >> 24] ^ rotr8(T.td0[(s0 >> 16) & 0xff]) ^ rotr16(T.td0[(s3 >> 8) & 0xff]) ^
                  rotr24(T.td0[s2 & 0xff]) ^ k[1];
    uint32_t t2 = T.td0[s2 >> 24] ^ rotr8(T.td0[(s1 >> 16) & 0xff]) ^ rotr16(T.td0[(s0 >> 8) & 0xff]) ^
                  rotr24(T.td0[s3 & 0xff]) ^ k[2];
    uint32_t t3 = T.td0[s3 >> 24] ^ rotr8(T.td0[(s2 >> 16) & 0xff]) ^ rotr16(T.td0[(s1 >> 8) & 0xff]) ^
                  rotr24(T.td0[s0 & 0xff]) ^ k[3];
    s0 = t0; s1 = t1; s2 = t2; s3 = t3;
  }
  const uint32_t* k = drk + 40;
  auto S = [&](uint32_t v, int sh) { return uint32_t(T.inv_sbox[(v >> sh) & 0xff]); };
  store_be(out, (S(s0, 24) << 24 | S(s3, 16) << 16 | S(s2, 8) << 8 | S(s1, 0)) ^ k[0]);
  store_be(out + 4, (S(s1, 24) << 24 | S(s0, 16) << 16 | S(s3, 8) << 8 | S(s2, 0)) ^ k[1]);
  store_be(out + 8, (S(s2, 24) << 24 | S(s1, 16) << 16 | S(s0, 8) << 8 | S(s3, 0)) ^ k[2]);
  store_be(out + 12, (S(s3, 24) << 24 | S(s2, 16) << 16 | S(s1, 8) << 8 | S(s0, 0)) ^ k[3]);
}

size_t cbc_encrypt_pkcs7(const uint8_t key[16], const uint8_t iv[16], const uint8_t* in, size_t n, uint8_t* out) {
  uint32_t rk[44];
  expand_key_enc(key, rk);
  const size_t pad = 16 - (n % 16);
  const size_t total = n + pad;
  uint8_t prev[16];
  std::memcpy(prev, iv, 16);
  uint8_t blk[16];
  for (size_t off = 0; off < total; off += 16) {
    for (int i = 0; i < 16; ++i) {
      size_t idx = off + i;
      uint8_t p = idx < n ? in[idx] : static_cast<uint8_t>(pad);
      blk[i] = p ^ prev[i];
    }
    encrypt_block(rk, blk, out + off);
    std::memcpy(prev, out + off, 16);
  }
  return total;
}

bool have_aesni() {
#if defined(__x86_64__)
  static const bool ok = __builtin_cpu_supports("aes") && __builtin_cpu_supports("sse4.1");
  return ok;
#else
  return false;
#endif
}

#if defined(__x86_64__)
namespace {
// AESDEC is one round of the equivalent inverse cipher, so the drk schedule (four
// big-endian column words per round) maps onto it byte for byte.
__attribute__((target("aes,sse4.1"))) void cbc_decrypt_aesni(const uint32_t drk[44], const uint8_t iv[16],
                                                              const uint8_t* in, size_t n, uint8_t* out) {
  __m128i k[11];
  for (int r = 0; r < 11; ++r) {
    uint8_t b[16];
    for (int c = 0; c < 4; ++c) store_be(b + 4 * c, drk[4 * r + c]);
    k[r] = _mm_loadu_si128(reinterpret_cast<const __m128i*>(b));
  }
  __m128i prev = _mm_loadu_si128(reinterpret_cast<const __m128i*>(iv));
  const size_t nb = n / 16;
  size_t i = 0;
  for (; i + 8 <= nb; i += 8) {  // eight independent blocks in flight
    __m128i c[8], s[8];
    for (int j = 0; j < 8; ++j) {
      c[j] = _mm_loadu_si128(reinterpret_cast<const __m128i*>(in + 16 * (i + j)));
      s[j] = _mm_xor_si128(c[j], k[0]);
    }
    for (int r = 1; r < 10; ++r)
      for (int j = 0; j < 8; ++j) s[j] = _mm_aesdec_si128(s[j], k[r]);
    for (int j = 0; j < 8; ++j) s[j] = _mm_aesdeclast_si128(s[j], k[10]);
    _mm_storeu_si128(reinterpret_cast<__m128i*>(out + 16 * i), _mm_xor_si128(s[0], prev));
    for (int j = 1; j < 8; ++j)
      _mm_storeu_si128(reinterpret_cast<__m128i*>(out + 16 * (i + j)), _mm_xor_si128(s[j], c[j - 1]));
    prev = c[7];
  }
  for (; i < nb; ++i) {
    __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(in + 16 * i));
    __m128i s = _mm_xor_si128(c, k[0]);
    for (int r = 1; r < 10; ++r) s = _mm_aesdec_si128(s, k[r]);
    s = _mm_aesdeclast_si128(s, k[10]);
    _mm_storeu_si128(reinterpret_cast<__m128i*>(out + 16 * i), _mm_xor_si128(s, prev));
    prev = c;
  }
}
}  // namespace
#endif

void cbc_decrypt_raw(const uint32_t drk[44], const uint8_t iv[16], const uint8_t* in, size_t n, uint8_t* out) {
#if defined(__x86_64__)
  if (have_aesni()) {
    cbc_decrypt_aesni(drk, iv, in, n, out);
    return;
  }
#endif
  uint8_t prev[16], cur[16], tmp[16];
  std::memcpy(prev, iv, 16);
  for (size_t off = 0; off + 16 <= n; off += 16) {
    std::memcpy(cur, in + off, 16);  // in-place safe
    decrypt_block(drk, cur, tmp);
    for (int i = 0; i < 16; ++i) out[off + i] = tmp[i] ^ prev[i];
    std::memcpy(prev, cur, 16);
  }
}

int64_t cbc_decrypt_pkcs7(const uint8_t key[16], const uint8_t iv[16], const uint8_t* in, size_t n, uint8_t* out) {
  if (n == 0 || n % 16 != 0) return -1;
  uint32_t drk[44];
  expand_key_dec(key, drk);
  cbc_decrypt_raw(drk, iv, in, n, out);
  uint8_t pad = out[n - 1];
  if (pad == 0 || pad > 16) return -1;
  for (size_t i = n - pad; i < n; ++i)
    if (out[i] != pad) return -1;
  return static_cast<int64_t>(n - pad);
}

}  // namespace aes
}  // namespace hlsp2p
