#include "crc_host.hpp"

#include <cstring>

namespace hlsp2p {
namespace crc {
namespace {

struct ByteTable {
  uint32_t t[8][256];
  ByteTable() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t r = i;
      for (int k = 0; k < 8; ++k) r = (r >> 1) ^ (kPoly & (0u - (r & 1u)));
      t[0][i] = r;
    }
    for (int s = 1; s < 8; ++s)
      for (uint32_t i = 0; i < 256; ++i) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xff];
  }
};

const ByteTable& table() {
  static const ByteTable tb;
  return tb;
}

}  // namespace

uint32_t crc32(const uint8_t* p, size_t n, uint32_t crc) {
  const ByteTable& T = table();
  uint32_t r = ~crc;
  while (n >= 8) {  // slice-by-8
    uint32_t lo, hi;
    std::memcpy(&lo, p, 4);
    std::memcpy(&hi, p + 4, 4);
    lo ^= r;
    r = T.t[7][lo & 0xff] ^ T.t[6][(lo >> 8) & 0xff] ^ T.t[5][(lo >> 16) & 0xff] ^ T.t[4][lo >> 24] ^
        T.t[3][hi & 0xff] ^ T.t[2][(hi >> 8) & 0xff] ^ T.t[1][(hi >> 16) & 0xff] ^ T.t[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) r = (r >> 8) ^ T.t[0][(r ^ *p++) & 0xff];
  return ~r;
}

uint32_t apply(const Mat& m, uint32_t v) {
  uint32_t out = 0;
  for (int i = 0; v; ++i, v >>= 1)
    if (v & 1u) out ^= m.col[i];
  return out;
}

Mat mul(const Mat& a, const Mat& b) {
  Mat c;
  for (int i = 0; i < 32; ++i) c.col[i] = apply(a, b.col[i]);
  return c;
}

Mat zero_byte_op() {
  const ByteTable& T = table();
  Mat m;
  for (int i = 0; i < 32; ++i) {
    uint32_t r = 1u << i;
    m.col[i] = (r >> 8) ^ T.t[0][r & 0xff];
  }
  return m;
}

Mat power(const Mat& m, uint64_t e) {
  Mat result;
  for (int i = 0; i < 32; ++i) result.col[i] = 1u << i;
  Mat base = m;
  while (e) {
    if (e & 1) result = mul(base, result);
    base = mul(base, base);
    e >>= 1;
  }
  return result;
}

bool inverse(const Mat& m, Mat* out) {
  // Gauss-Jordan on rows: build row-major bit matrix [M | I].
  uint64_t rows[32];
  for (int r = 0; r < 32; ++r) {
    uint32_t row = 0;
    for (int c = 0; c < 32; ++c)
      if ((m.col[c] >> r) & 1u) row |= 1u << c;
    rows[r] = uint64_t(row) | (uint64_t(1u << r) << 32);
  }
  for (int c = 0; c < 32; ++c) {
    int piv = -1;
    for (int r = c; r < 32; ++r)
      if ((rows[r] >> c) & 1u) { piv = r; break; }
    if (piv < 0) return false;
    std::swap(rows[c], rows[piv]);
    for (int r = 0; r < 32; ++r)
      if (r != c && ((rows[r] >> c) & 1u)) rows[r] ^= rows[c];
  }
  for (int c = 0; c < 32; ++c) {
    uint32_t col = 0;
    for (int r = 0; r < 32; ++r)
      if ((rows[r] >> (32 + c)) & 1u) col |= 1u << r;
    out->col[c] = col;
  }
  return true;
}

void slice_table(const Mat& m, uint32_t* out) {
  for (int b = 0; b < 4; ++b)
    for (uint32_t x = 0; x < 256; ++x) out[b * 256 + x] = apply(m, x << (8 * b));
}

std::vector<int8_t> mfma_group_weights() {
  const ByteTable& T = table();
  // v[byte][bit]: raw CRC (zero init) of a 256-byte group with only that bit set.
  static uint32_t v[kGroupBytes][8];
  for (int bit = 0; bit < 8; ++bit) {
    uint32_t r = T.t[0][1u << bit];  // one byte (1<<bit) from a zero register
    for (int b = kGroupBytes - 1; b >= 0; --b) {
      v[b][bit] = r;
      r = (r >> 8) ^ T.t[0][r & 0xff];  // one more zero byte after it
    }
  }
  // Fragment order: lane l (col = l & 31 = CRC bit column, h = l >> 5) at step s = 8q + jb
  // holds B[k][col] for its 16 k's; k(s, h, e) <-> group byte 32q + 16h + e, bit jb.
  // The kernel feeds RAW data bytes masked to bit jb (value 2^jb; -128 as i8 for jb = 7),
  // so B is scaled by 2^(7-jb) (-128 for jb = 0): every nonzero product is +-128 and the
  // accumulator is 128 x (the GF(2) sum) -> the residue bit is bit 7 of the accumulator.
  std::vector<int8_t> w(64 * 64 * 16);
  for (int s = 0; s < 64; ++s) {
    const int q = s >> 3, jb = s & 7;
    const int scale = jb == 0 ? -128 : (1 << (7 - jb));
    for (int lane = 0; lane < 64; ++lane) {
      int col = lane & 31, h = lane >> 5;
      for (int e = 0; e < 16; ++e) {
        int byte = 32 * q + 16 * h + e;
        w[(s * 64 + lane) * 16 + e] = static_cast<int8_t>(((v[byte][jb] >> col) & 1u) ? scale : 0);
      }
    }
  }
  return w;
}

namespace {
// v[byte][bit]: raw CRC (zero init) of a 256-byte group with only that bit set
struct GroupBitCrc {
  uint32_t v[kGroupBytes][8];
  GroupBitCrc() {
    const ByteTable& T = table();
    for (int bit = 0; bit < 8; ++bit) {
      uint32_t r = T.t[0][1u << bit];
      for (int b = kGroupBytes - 1; b >= 0; --b) {
        v[b][bit] = r;
        r = (r >> 8) ^ T.t[0][r & 0xff];
      }
    }
  }
};
}  // namespace

std::vector<uint8_t> mfma_group_weights_fp4() {
  static const GroupBitCrc g;
  // Step s = 4q + w consumes data dword w of the lane's 16-byte chunk q, i.e. group bytes
  // [32q + 16h + 4w, +4) for lane half h.  The kernel feeds that dword d as 4 fp4 operand
  // dwords: A_v = d & 0x11111111 (bit 0 of each nibble = e2m1 0.5), d & 0x22222222 (bit 1 =
  // 1.0), d & 0x44444444 (bit 2 = 2.0) and (d >> 1) & 0x44444444 (bit 3 = 2.0): element
  // j = 8v + e (nibble e of operand dword v) carries data bit 4e + v of d.  B holds the
  // weight bit of the same k scaled by the inverse (2.0, 1.0, 0.5, 0.5), so every nonzero
  // product is exactly 1.0 and the f32 accumulator counts set terms: its parity is the
  // GF(2) sum.  A and B share the element -> k assignment, so the MFMA's internal k order
  // does not matter.
  static const uint8_t kOne[4] = {0x4, 0x2, 0x1, 0x1};  // e2m1: 2.0, 1.0, 0.5, 0.5
  std::vector<uint8_t> w(32 * 64 * 16, 0);
  for (int s = 0; s < 32; ++s) {
    const int q = s >> 2, wd = s & 3;
    for (int lane = 0; lane < 64; ++lane) {
      const int col = lane & 31, h = lane >> 5;
      uint8_t* frag = &w[(size_t(s) * 64 + lane) * 16];
      for (int v = 0; v < 4; ++v)
        for (int e = 0; e < 8; ++e) {
          const int bit = 4 * e + v;  // bit of the data dword
          const int byte = 32 * q + 16 * h + 4 * wd + (bit >> 3);
          if (!((g.v[byte][bit & 7] >> col) & 1u)) continue;
          frag[4 * v + (e >> 1)] |= static_cast<uint8_t>(kOne[v] << (4 * (e & 1)));
        }
    }
  }
  return w;
}

std::vector<uint8_t> mfma_chunk_weights_fp4() {
  const ByteTable& T = table();
  const Mat a8 = zero_byte_op();
  static const uint8_t kOne[4] = {0x4, 0x2, 0x1, 0x1};  // e2m1: 2.0, 1.0, 0.5, 0.5 (as the group form)
  std::vector<uint8_t> w(size_t(kFusedAesSteps + kFusedFoldSteps) * 64 * 16, 0);
  auto put = [&](uint8_t* frag, int v, int e) { frag[4 * v + (e >> 1)] |= static_cast<uint8_t>(kOne[v] << (4 * (e & 1))); };
  // decrypt side: vec[jj][h][y][bit] = A^(8 (1024 (1 - jj) + 512 (1 - h) + 15 - y)) t(bit)
  static uint32_t vec[2][2][16][8];
  for (int jj = 0; jj < 2; ++jj)
    for (int h = 0; h < 2; ++h) {
      const Mat u = power(a8, uint64_t(1024) * (1 - jj) + uint64_t(512) * (1 - h));
      for (int bit = 0; bit < 8; ++bit) {
        uint32_t r = apply(u, T.t[0][1u << bit]);
        for (int y = 15; y >= 0; --y) {
          vec[jj][h][y][bit] = r;
          r = (r >> 8) ^ T.t[0][r & 0xff];  // one more zero byte after it
        }
      }
    }
  for (int st = 0; st < kFusedAesSteps; ++st) {
    const int jj = st >> 2, d = st & 3;
    for (int lane = 0; lane < 64; ++lane) {
      const int col = lane & 31, h = lane >> 5;
      uint8_t* frag = &w[(size_t(st) * 64 + lane) * 16];
      for (int v = 0; v < 4; ++v)
        for (int e = 0; e < 8; ++e) {
          const int bit = 4 * e + v;  // bit of the data dword (element 8v + e)
          if ((vec[jj][h][4 * d + (bit >> 3)][bit & 7] >> col) & 1u) put(frag, v, e);
        }
    }
  }
  // fold side: S[p][rho] = A^(8 * 16 (159 - 128 p - rho)) moves row rho of chain pair p to the chunk end
  static Mat S[2][32];
  const Mat m16 = power(a8, 16);
  for (int p = 0; p < 2; ++p)
    for (int rho = 0; rho < 32; ++rho) S[p][rho] = power(m16, uint64_t(159 - 128 * p - rho));
  for (int s = 0; s < kFusedFoldSteps; ++s)
    for (int lane = 0; lane < 64; ++lane) {
      const int row = lane & 31, hh = lane >> 5;  // A row = output CRC bit; k half
      const int lp = s + 32 * hh;                 // the chunk's mask dword this k half reads = its decrypt lane
      uint8_t* frag = &w[(size_t(kFusedAesSteps + s) * 64 + lane) * 16];
      for (int v = 0; v < 4; ++v)
        for (int e = 0; e < 8; ++e) {
          const int b = 4 * e + v;  // bit of the mask dword
          const int p = b >> 4, i = b & 15;
          const int rho = (i & 3) + 8 * (i >> 2) + 4 * (lp >> 5), n = lp & 31;
          if ((S[p][rho].col[n] >> row) & 1u) put(frag, v, e);
        }
    }
  return w;
}

uint32_t init_fold(int64_t nbytes) {
  if (nbytes < 4) return 0;
  const ByteTable& T = table();
  uint32_t r = 0;
  for (int i = 0; i < 4; ++i) r = (r >> 8) ^ T.t[0][(r ^ 0xffu) & 0xff];
  return apply(power(zero_byte_op(), static_cast<uint64_t>(nbytes - 4)), r);
}

std::vector<uint32_t> shift_tables() {
  std::vector<uint32_t> out(size_t(kNumP + kNumQ) * kSliceWords);
  Mat a8 = zero_byte_op();
  Mat p = a8;  // A^(8 * 2^0)
  for (int b = 0; b < kNumP; ++b) {
    slice_table(p, out.data() + size_t(b) * kSliceWords);
    p = mul(p, p);
  }
  Mat inv;
  inverse(a8, &inv);
  Mat q = inv;
  for (int b = 0; b < kNumQ; ++b) {
    slice_table(q, out.data() + size_t(kNumP + b) * kSliceWords);
    q = mul(q, q);
  }
  return out;
}

}  // namespace crc
}  // namespace hlsp2p
