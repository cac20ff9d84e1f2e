// CRC-32 (zlib) of a batch of segments on the MFMA matrix cores.
//
// CRC is linear over GF(2).  For a 256-byte group g, its zero-init register contribution
// is a 32-bit vector r_g = W^T bits(g) (mod 2) with W a fixed 2048 x 32 binary matrix.
// Integer accumulation followed by "& 1" equals the GF(2) sum, so the 8-bit integer MFMA
// computes 32 groups x 32 CRC bits per wave tile:
//
//     D[32 groups][32 bits] += A[32 groups][32 k] * B[32 k][32 bits]   (i8 -> i32)
//     v_mfma_i32_32x32x32_i8, 64 k-steps per 256-byte group (k = 2048 data bits)
//
// Layout choice (so no LDS transpose of the data is needed): lane l = (row r = l & 31,
// half h = l >> 5) owns the 16-byte chunks [32q + 16h, +16), q < 8, of group r, loaded as 8
// dwordx4 (the row's two lanes read 32 contiguous bytes per instruction; a 128h-split
// layout read two 16-byte pieces 128 B apart: 64 line pieces per wave-load instead of 32).
// k-step s = 8q + jb feeds chunk q's 16 RAW bytes masked to bit jb
// (one v_and per dword: values 2^jb, -128 as i8 for jb = 7) — no bit expansion.  The B
// fragment of the same 16 k's is W scaled by 2^(7-jb) (-128 for jb = 0), so every nonzero
// product is +-128 and the accumulator is 128 x (the GF(2) sum): the residue bit is bit 7.
// Fragments are precomputed on the host (runtime/crc_host.cpp) in MFMA order, 64 KiB,
// staged once per workgroup in LDS and read with one ds_read_b128 per lane per step.
// Because A and B use the same k permutation the product is independent of the MFMA's
// internal k ordering.
//
// The 16 accumulator registers hold rows (i&3)+8(i>>2)+4h, column = lane&31 (gfx950 C/D
// map); a wave ballot of the parity bits yields two 32-bit group residues per register.
// A second kernel (one workgroup per segment) folds the residues with GF(2) shift
// operators (byte-slice tables in LDS): Horner over runs of groups, then a log tree, then
// it undoes the zero padding of the last group (A^-8p) and adds the init/xor-out terms.
// Result is bit-identical to zlib.crc32.
#include "common.h"

namespace hlsp2p {
namespace dev {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// 8 waves share one 64 KiB LDS copy of W: 2 workgroups per CU = 4 waves per SIMD, so one
// wave's global loads / nibble expansion overlap other waves' MFMAs.
constexpr int kCrcThreads = 512;
constexpr int kTileBytes = 32 * 256;
constexpr int kNumP = 40;
constexpr int kSlice = 1024;  // u32 per byte-slice table set

// 16 bytes at byte offset `o` of a segment of `len` > 0 bytes, zero beyond the end (last
// tile).  Segment starts are 16-byte aligned, so the aligned 16-byte chunk holding a
// segment's last byte never crosses a page: load it whole and mask; chunks entirely past
// the end re-read the segment's first chunk and mask it to zero (no branches, no scratch).
__device__ __forceinline__ uint32_t keep_mask(int64_t rem) {
  return rem >= 4 ? 0xFFFFFFFFu : rem <= 0 ? 0u : (1u << (8 * rem)) - 1u;
}
__device__ __forceinline__ uint4 load_tail(const uint8_t* __restrict__ buf, int64_t base, int64_t o, int64_t len) {
  const int64_t rem = len - o;
  uint4 v = *reinterpret_cast<const uint4*>(buf + base + (rem > 0 ? o : 0));
  v.x &= keep_mask(rem);
  v.y &= keep_mask(rem - 4);
  v.z &= keep_mask(rem - 8);
  v.w &= keep_mask(rem - 12);
  return v;
}

__global__ __launch_bounds__(kCrcThreads) void crc32_group_residue_kernel(
    const uint8_t* __restrict__ buf, const int64_t* __restrict__ seg_off, const int64_t* __restrict__ seg_len,
    const int64_t* __restrict__ tile_prefix, const int64_t* __restrict__ res_off, const v4i* __restrict__ wfrag,
    uint32_t* __restrict__ residues, int nseg, int64_t total_tiles, int64_t tiles_per_wave) {
  __shared__ v4i s_w[64 * 64];  // 64 KiB: [step][lane] fragments
  const int tid = threadIdx.x;
  lds_fill<64 * 64 / kCrcThreads>(s_w, wfrag, 64 * 64, tid, kCrcThreads);
  __syncthreads();

  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int64_t gwave = static_cast<int64_t>(blockIdx.x) * (kCrcThreads / 64) + wave;
  const int64_t t_begin = gwave * tiles_per_wave;
  const int64_t t_end = t_begin + tiles_per_wave < total_tiles ? t_begin + tiles_per_wave : total_tiles;
  if (t_begin >= t_end) return;
  // Software pipeline over the wave's tiles: the lane's 128 bytes of tile t+1 (8 x dwordx4,
  // 8 KB per wave) are in flight while tile t's 64 MFMAs run.  Without it every tile paid a
  // full HBM round trip before its MFMAs (~2.5 TB/s chip-wide).
  int seg = find_seg_wave(tile_prefix, nseg, t_begin);
  int64_t base = seg_off[seg], len = seg_len[seg], tstart = tile_prefix[seg], tend = tile_prefix[seg + 1];
  int64_t roff = res_off[seg];
  uint4 n0, n1, n2, n3, n4, n5, n6, n7;  // the next tile's chunks
  auto load_tile = [&](int64_t tile) {
    // chunk q of lane (r, h) = bytes [32q + 16h, +16) of group r: the two lanes of a row read
    // 32 contiguous bytes per instruction (32 line pieces per wave-load instead of 64)
    const int64_t my = tile * kTileBytes + r * 256 + h * 16;
    if ((tile + 1) * kTileBytes <= len) {  // wave-uniform: only a segment's last tile is partial
      const uint4* p = reinterpret_cast<const uint4*>(buf + base + my);
      n0 = p[0]; n1 = p[2]; n2 = p[4]; n3 = p[6]; n4 = p[8]; n5 = p[10]; n6 = p[12]; n7 = p[14];
    } else {
      n0 = load_tail(buf, base, my, len);        n1 = load_tail(buf, base, my + 32, len);
      n2 = load_tail(buf, base, my + 64, len);   n3 = load_tail(buf, base, my + 96, len);
      n4 = load_tail(buf, base, my + 128, len);  n5 = load_tail(buf, base, my + 160, len);
      n6 = load_tail(buf, base, my + 192, len);  n7 = load_tail(buf, base, my + 224, len);
    }
  };
  load_tile(t_begin - tstart);
  for (int64_t t = t_begin; t < t_end; ++t) {
    uint4 c0 = n0, c1 = n1, c2 = n2, c3 = n3, c4 = n4, c5 = n5, c6 = n6, c7 = n7;
    const int64_t tile = t - tstart;
    const int64_t c_len = len, c_roff = roff;
    if (t + 1 < t_end) {
      if (t + 1 >= tend) {
        seg = advance_seg(tile_prefix, seg, t + 1);
        base = seg_off[seg];
        len = seg_len[seg];
        tstart = tile_prefix[seg];
        tend = tile_prefix[seg + 1];
        roff = res_off[seg];
      }
      load_tile(t + 1 - tstart);
    }
    v16i acc = {};
    // not unrolled (an unrolled q loop hoists all 64 B fragments into registers); the chunk
    // registers rotate instead of being indexed, so nothing goes to scratch
#pragma unroll 1
    for (int q = 0; q < 8; ++q) {
      // 8 MFMAs per 16-byte chunk, one per bit position jb: A = the raw bytes masked to
      // bit jb (4 v_and), B pre-scaled by 2^(7-jb) on the host, so each nonzero product is
      // +-128 and the GF(2) sum lands in bit 7 of the accumulator
#pragma unroll
      for (int jb = 0; jb < 8; ++jb) {
        const uint32_t m = 0x01010101u << jb;
        v4i a;
        a.x = static_cast<int>(c0.x & m);
        a.y = static_cast<int>(c0.y & m);
        a.z = static_cast<int>(c0.z & m);
        a.w = static_cast<int>(c0.w & m);
        const v4i b = s_w[(8 * q + jb) * 64 + lane];
        acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc, 0, 0, 0);
      }
      c0 = c1; c1 = c2; c2 = c3; c3 = c4; c4 = c5; c5 = c6; c6 = c7;
    }
    // lane `row` takes its group's residue from the 16 ballots; one masked store (see the
    // fp4 kernel)
    uint32_t res = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint64_t m = __ballot(acc[i] & 0x80);  // 128 x GF(2) sum: parity is bit 7
      const int row = (i & 3) + 8 * (i >> 2);
      res = lane == row ? static_cast<uint32_t>(m) : res;
      res = lane == row + 4 ? static_cast<uint32_t>(m >> 32) : res;
    }
    const int64_t groups = (c_len + 255) >> 8;
    const int64_t g = tile * 32 + lane;
    if (lane < 32 && g < groups) residues[c_roff + g] = res;
  }
}

// FP4 variant on the block-scaled f8f6f4 matrix cores (v_mfma_scale_f32_32x32x64_f8f6f4,
// e2m1 A and B, unit scales).  An FP4 MFMA takes the cycles of the i8 32x32x32 one but
// covers 64 k, so a tile needs 32 MFMAs instead of 64; each consumes ONE data dword per lane
// (vs 16 bytes masked to one bit), fed as 4 operand dwords -- bits 0/1/2/3 of every nibble:
// d & 0x11111111 (= 0.5), d & 0x22222222 (= 1.0), d & 0x44444444 (= 2.0),
// (d >> 1) & 0x44444444 (= 2.0) -- with B pre-scaled by the inverse on the host
// (crc_host.cpp: mfma_group_weights_fp4), so every nonzero product is exactly 1.0 and the
// f32 accumulator is an exact count (<= 2048): its parity is the GF(2) residue bit.
// Step s = 4q + w uses dword w of the lane's 16-byte chunk q (same loads as the i8 path).
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(kCrcThreads) void crc32_group_residue_fp4_kernel(
    const uint8_t* __restrict__ buf, const int64_t* __restrict__ seg_off, const int64_t* __restrict__ seg_len,
    const int64_t* __restrict__ tile_prefix, const int64_t* __restrict__ res_off, const v4i* __restrict__ wfrag,
    uint32_t* __restrict__ residues, int nseg, int64_t total_tiles, int64_t tiles_per_wave) {
  __shared__ v4i s_w[32 * 64];  // 32 KiB: [step][lane] fragments
  const int tid = threadIdx.x;
  lds_fill<32 * 64 / kCrcThreads>(s_w, wfrag, 32 * 64, tid, kCrcThreads);
  __syncthreads();

  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int64_t gwave = static_cast<int64_t>(blockIdx.x) * (kCrcThreads / 64) + wave;
  const int64_t t_begin = gwave * tiles_per_wave;
  const int64_t t_end = t_begin + tiles_per_wave < total_tiles ? t_begin + tiles_per_wave : total_tiles;
  if (t_begin >= t_end) return;
  int seg = find_seg_wave(tile_prefix, nseg, t_begin);
  int64_t base = seg_off[seg], len = seg_len[seg], tstart = tile_prefix[seg], tend = tile_prefix[seg + 1];
  int64_t roff = res_off[seg];
  uint4 n0, n1, n2, n3, n4, n5, n6, n7;  // the next tile's chunks
  auto load_tile = [&](int64_t tile) {
    const int64_t my = tile * kTileBytes + r * 256 + h * 16;
    if ((tile + 1) * kTileBytes <= len) {
      const uint4* p = reinterpret_cast<const uint4*>(buf + base + my);
      n0 = p[0]; n1 = p[2]; n2 = p[4]; n3 = p[6]; n4 = p[8]; n5 = p[10]; n6 = p[12]; n7 = p[14];
    } else {
      n0 = load_tail(buf, base, my, len);        n1 = load_tail(buf, base, my + 32, len);
      n2 = load_tail(buf, base, my + 64, len);   n3 = load_tail(buf, base, my + 96, len);
      n4 = load_tail(buf, base, my + 128, len);  n5 = load_tail(buf, base, my + 160, len);
      n6 = load_tail(buf, base, my + 192, len);  n7 = load_tail(buf, base, my + 224, len);
    }
  };
  load_tile(t_begin - tstart);
  for (int64_t t = t_begin; t < t_end; ++t) {
    uint4 c0 = n0, c1 = n1, c2 = n2, c3 = n3, c4 = n4, c5 = n5, c6 = n6, c7 = n7;
    const int64_t tile = t - tstart;
    const int64_t c_len = len, c_roff = roff;
    if (t + 1 < t_end) {
      if (t + 1 >= tend) {
        seg = advance_seg(tile_prefix, seg, t + 1);
        base = seg_off[seg];
        len = seg_len[seg];
        tstart = tile_prefix[seg];
        tend = tile_prefix[seg + 1];
        roff = res_off[seg];
      }
      load_tile(t + 1 - tstart);
    }
    v16f acc = {};
#pragma unroll 1
    for (int q = 0; q < 8; ++q) {
      const uint32_t dw[4] = {c0.x, c0.y, c0.z, c0.w};
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const uint32_t d = dw[w];
        const v8i a = {static_cast<int>(d & 0x11111111u), static_cast<int>(d & 0x22222222u),
                       static_cast<int>(d & 0x44444444u), static_cast<int>((d >> 1) & 0x44444444u), 0, 0, 0, 0};
        const v4i b4 = s_w[(4 * q + w) * 64 + lane];
        const v8i b = {b4.x, b4.y, b4.z, b4.w, 0, 0, 0, 0};
        // cbsz = blgp = 4: e2m1 A and B; scale exponents 0 select the unscaled form
        acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc, 4, 4, 0, 0, 0, 0);
      }
      c0 = c1; c1 = c2; c2 = c3; c3 = c4; c4 = c5; c5 = c6; c6 = c7;
    }
    // 16 ballots (wave-uniform, SGPRs) hold the tile's 32 group residues: lane `row` selects
    // its group's word, then ONE masked store writes all 32 (instead of 32 single-lane
    // stores behind branches)
    uint32_t res = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint64_t m = __ballot(static_cast<int>(acc[i]) & 1);  // exact count: parity = GF(2) sum
      const int row = (i & 3) + 8 * (i >> 2);
      res = lane == row ? static_cast<uint32_t>(m) : res;
      res = lane == row + 4 ? static_cast<uint32_t>(m >> 32) : res;
    }
    const int64_t groups = (c_len + 255) >> 8;
    const int64_t g = tile * 32 + lane;
    if (lane < 32 && g < groups) residues[c_roff + g] = res;
  }
}

__device__ __forceinline__ uint32_t apply_tab(const uint32_t* __restrict__ t, uint32_t v) {
  return t[v & 0xff] ^ t[256 + ((v >> 8) & 0xff)] ^ t[512 + ((v >> 16) & 0xff)] ^ t[768 + (v >> 24)];
}

constexpr int kCombineThreads = 1024;
constexpr int kCombineLdsTables = 15;  // P_8 .. P_22
constexpr int kNumQ = 12;              // Q_b = A^(-8 * 2^b): pad removal (pad < 4096 bytes)
// Residue of the group [FF FF FF FF 00 .. 00]: for n >= 4 the zlib init value 0xFFFFFFFF
// equals XOR-ing FF into the message's first 4 bytes, so it folds into group 0's residue
// (= zlib(FF^4 0^(G-4)) ^ zlib(0^G)) instead of a 20-step chain of dependent global table
// lookups on one thread after the tree (that tail was most of the kernel).
constexpr uint32_t kInitFold256 = 0xf2697aa7u;   // 256-byte groups (crc_host.cpp: init_fold)
constexpr uint32_t kInitFold4096 = 0x38e3ffeeu;  // 4096-byte chunks of the fused decrypt CRC

// Digest of a segment key (segment-view.js:9-17,59-61): the 12-byte wire key
// [level, urlId, sn] plus the swarm id, mixed to 32 bits (splitmix64 finalizer, the store's
// mix64).  The combine below binds a CRC to the key it was computed for (crc ^ digest), so a
// segment that reaches a peer under another key -- an entry the sender overwrote with another
// segment, whose table CRC is then consistent with the wrong bytes -- fails the receiver's
// check.  Host twin: runtime key_digest (store.hpp); tests compare the two.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint32_t key_digest(const int64_t* __restrict__ k) {
  const uint64_t a = uint64_t(uint32_t(k[1])) | (uint64_t(uint32_t(k[2])) << 32);  // level | urlId
  const uint64_t b = uint64_t(uint32_t(k[3])) | (uint64_t(uint32_t(k[0])) << 32);  // sn | swarm
  const uint64_t z = mix64(a ^ mix64(b + 0x9E3779B97F4A7C15ull));
  return uint32_t(z ^ (z >> 32));
}

// One workgroup per segment.  tables: P_0..P_39 then Q_0..Q_11 (each kSlice u32).  Group
// residues of 2^kLg bytes: 256-byte groups (the residue kernels above) or 4096-byte chunks
// (the CRC fused into the decrypt, folded by crc32_fold_combine_kernel).
template <int kLg>
__device__ __forceinline__ void combine_segment(
    int seg, int tid, uint32_t* __restrict__ s_tab, uint32_t* __restrict__ s_q, uint32_t* __restrict__ s_acc,
    const uint32_t* __restrict__ residues, const int64_t* __restrict__ res_off, const int64_t* __restrict__ seg_len,
    const uint32_t* __restrict__ tables, uint32_t* __restrict__ crc_out, const uint32_t* __restrict__ expect,
    uint8_t* __restrict__ ok_out, const int64_t* __restrict__ scatter_idx, uint32_t* __restrict__ scatter_out,
    int64_t scatter_n, const int64_t* __restrict__ keys) {
  const int64_t n = seg_len[seg];
  const int64_t G = (n + (int64_t(1) << kLg) - 1) >> kLg;
  // run length L = next pow2 of ceil(G / threads)
  int lgL = 0;
  while ((static_cast<int64_t>(kCombineThreads) << lgL) < G) ++lgL;
  const int need = kLg - 8 + 1 + lgL + 10;  // P_8 .. P_(kLg + lgL + 10) from LDS
  const int lds_tables = need <= kCombineLdsTables ? need : kCombineLdsTables;
  lds_fill<kCombineLdsTables * kSlice / 4 / kCombineThreads + 1>(
      reinterpret_cast<uint4*>(s_tab), reinterpret_cast<const uint4*>(tables + 8 * kSlice), lds_tables * kSlice / 4,
      tid, kCombineThreads);
  lds_fill<kLg * kSlice / 4 / kCombineThreads>(reinterpret_cast<uint4*>(s_q),
                                                reinterpret_cast<const uint4*>(tables + kNumP * kSlice),
                                                kLg * kSlice / 4, tid, kCombineThreads);
  __syncthreads();
  const int64_t L = int64_t(1) << lgL;
  const int64_t span = L * kCombineThreads;
  const int64_t front = span - G;  // virtual zero groups in front
  const uint32_t* __restrict__ res = residues + res_off[seg];
  const uint32_t fold0 = n >= 4 ? (kLg == 8 ? kInitFold256 : kInitFold4096) : 0u;
  uint32_t acc = 0;
  const uint32_t* pg = s_tab + (kLg - 8) * kSlice;  // A^(8 * 2^kLg): one group
  // Horner over this thread's run of L groups, 8 residues loaded ahead per step (a
  // load-per-iteration loop paid one global round trip per group: L of them in series)
  constexpr int kAhead = 8;
  for (int64_t k0 = 0; k0 < L; k0 += kAhead) {
    uint32_t rv[kAhead];
#pragma unroll
    for (int j = 0; j < kAhead; ++j) {
      const int64_t g = static_cast<int64_t>(tid) * L + k0 + j - front;
      rv[j] = (k0 + j < L && g >= 0) ? res[g] : 0u;
    }
#pragma unroll
    for (int j = 0; j < kAhead; ++j) {
      if (k0 + j < L) {
        const int64_t g = static_cast<int64_t>(tid) * L + k0 + j - front;
        acc = apply_tab(pg, acc) ^ rv[j] ^ (g == 0 ? fold0 : 0u);
      }
    }
  }
  s_acc[tid] = acc;
  __syncthreads();
  // tree: level m merges runs of L*2^m groups: left = A^(8*2^kLg*L*2^m) left ^ right
  for (int m = 0; (1 << m) < kCombineThreads; ++m) {
    const int stride = 1 << m;
    const int b = kLg + lgL + m;  // shift of 2^b bytes
    if ((tid & (2 * stride - 1)) == 0) {
      const uint32_t* tab = (b - 8) < lds_tables ? s_tab + (b - 8) * kSlice : tables + static_cast<int64_t>(b) * kSlice;
      s_acc[tid] = apply_tab(tab, s_acc[tid]) ^ s_acc[tid + stride];
    }
    __syncthreads();
  }
  if (tid == 0) {
    uint32_t raw = s_acc[0];
    const int64_t pad = (G << kLg) - n;
    for (int b = 0; b < kLg; ++b)
      if ((pad >> b) & 1) raw = apply_tab(s_q + b * kSlice, raw);
    uint32_t init = 0;  // folded into group 0 (n >= 4)
    if (n < 4) {
      init = 0xFFFFFFFFu;
      for (int b = 0; b < 2; ++b)
        if ((n >> b) & 1) init = apply_tab(tables + static_cast<int64_t>(b) * kSlice, init);
    }
    const uint32_t crc = raw ^ init ^ 0xFFFFFFFFu;
    crc_out[seg] = crc;
    // keyed (keys given): the expected value and the table entry are the CRC bound to the
    // segment's key (a peer's trailer is its table entry)
    const uint32_t digest = keys ? crc ^ key_digest(keys + 4 * seg) : crc;
    if (ok_out) ok_out[seg] = (expect && expect[seg] == digest) ? 1 : 0;
    // optional scatter into a per-entry CRC table (the cache's ingest CRCs): saves the
    // caller an index H2D plus an index_put launch per round; out-of-range ids are dropped
    if (scatter_out) {
      const int64_t d = scatter_idx[seg];
      if (d >= 0 && d < scatter_n) scatter_out[d] = digest;
    }
  }
}

template <int kLg>
__global__ __launch_bounds__(kCombineThreads) void crc32_combine_kernel(
    const uint32_t* __restrict__ residues, const int64_t* __restrict__ res_off, const int64_t* __restrict__ seg_len,
    const uint32_t* __restrict__ tables, uint32_t* __restrict__ crc_out, const uint32_t* __restrict__ expect,
    uint8_t* __restrict__ ok_out, const int64_t* __restrict__ scatter_idx, uint32_t* __restrict__ scatter_out,
    int64_t scatter_n, const int64_t* __restrict__ keys) {
  __shared__ __attribute__((aligned(16))) uint32_t s_tab[kCombineLdsTables * kSlice];  // 60 KiB
  __shared__ __attribute__((aligned(16))) uint32_t s_q[kLg * kSlice];                  // 32 / 48 KiB
  __shared__ uint32_t s_acc[kCombineThreads];
  combine_segment<kLg>(blockIdx.x, threadIdx.x, s_tab, s_q, s_acc, residues, res_off, seg_len, tables, crc_out, expect,
                       ok_out, scatter_idx, scatter_out, scatter_n, keys);
}

// The fused decrypt CRC's second level (aes_cbc.hip: crc_chunk_masks writes 64 mask dwords per
// 4096-byte chunk, the accumulator parities of chain pairs p = 0, 1 in bits 16 p + i).  The
// chunk residue is XOR_{p,rho} S[p][rho] D_p[rho] -- over GF(2) a [32 CRC bits x 2048] x
// [2048 x chunks] GEMM, on the same FP4 MFMA: A = the host's S fragments (crc_host.cpp:
// mfma_chunk_weights_fp4 after the 8 decrypt steps; 32 KiB, one ds_read_b128 per lane per step
// from LDS), B = the chunk's mask dwords fed as e2m1 bit planes (k half hh of step s = mask
// dword s + 32 hh), 32 chunks per wave tile, 32 MFMAs per tile.  Lane l ends with 16 residue
// bits of chunk l & 31 (rows (i & 3) + 8 (i >> 2) + 4 (l >> 5)); one cross-half swap completes
// the word.  (Round 4's first fold transposed one-level masks with 16 ballots per chunk and a
// 5-level table tree: 45-50 us per 256-segment batch.)
constexpr int kFoldSteps = 32;
constexpr int kMaskDwords = 64;  // per chunk
// One 32-chunk tile of the fold: chunks [cbase, cbase + 32) below cend, one wave.
__device__ __forceinline__ void fold_tile(const uint32_t* __restrict__ masks, const v4i* __restrict__ s_w,
                                          uint32_t* __restrict__ chunk_res, int64_t cbase, int64_t cend, int lane) {
  // the weight reads below are the same for every tile: without this barrier the compiler
  // hoists all 32 of them out of the caller's tile loop (128 VGPRs held live, spills)
  __asm__ volatile("" ::: "memory");
  const int hh = lane >> 5;
  const int64_t c = cbase + (lane & 31);
  const bool valid = c < cend;
  const uint4* src = reinterpret_cast<const uint4*>(masks + (valid ? c : 0) * kMaskDwords + 32 * hh);
  uint4 x[kFoldSteps / 4];  // this lane's 32 mask dwords (128 contiguous bytes), all loads in flight
#pragma unroll
  for (int k = 0; k < kFoldSteps / 4; ++k) x[k] = valid ? src[k] : make_uint4(0, 0, 0, 0);
  v16f acc = {};
#pragma unroll
  for (int k = 0; k < kFoldSteps / 4; ++k) {
    const uint32_t dw[4] = {x[k].x, x[k].y, x[k].z, x[k].w};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t d = dw[u];
      const v8i b = {static_cast<int>(d & 0x11111111u), static_cast<int>(d & 0x22222222u),
                     static_cast<int>(d & 0x44444444u), static_cast<int>((d >> 1) & 0x44444444u), 0, 0, 0, 0};
      const v4i a4 = s_w[(4 * k + u) * 64 + lane];
      const v8i a = {a4.x, a4.y, a4.z, a4.w, 0, 0, 0, 0};
      acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc, 4, 4, 0, 0, 0, 0);
    }
    // keep the next group's LDS reads below this one (hoisting them all spills)
    __builtin_amdgcn_sched_barrier(0);
  }
  uint32_t part = 0;  // CRC bits (i & 3) + 8 (i >> 2) + 4 hh of chunk lane & 31
#pragma unroll
  for (int i = 0; i < 16; ++i)
    part |= (static_cast<uint32_t>(static_cast<int>(acc[i])) & 1u) << ((i & 3) + 8 * (i >> 2) + 4 * hh);
  const uint32_t res = part | static_cast<uint32_t>(__shfl_xor(static_cast<int>(part), 32, 64));
  if (lane < 32 && valid) chunk_res[c] = res;
}

// Fold + combine in one workgroup per segment: the segment's chunk tiles over its 16 waves,
// then the combine over the residues it just wrote (L2-resident).  144 KiB of LDS: the fold's
// A fragments beside the combine's tables.  (A separate fold kernel over all chunks followed by
// the combine kernel took 19.1 + 8.4 us per 256-segment batch and two launches; this one takes
// 25.9 us, profiles/r4_dpp/NOTES.md.)
__global__ __launch_bounds__(kCombineThreads) void crc32_fold_combine_kernel(
    const uint32_t* __restrict__ masks, const v4i* __restrict__ wfold, const int64_t* __restrict__ chunk_off,
    const int64_t* __restrict__ seg_len, const uint32_t* __restrict__ tables, uint32_t* __restrict__ chunk_res,
    uint32_t* __restrict__ crc_out, const uint32_t* __restrict__ expect, uint8_t* __restrict__ ok_out,
    const int64_t* __restrict__ scatter_idx, uint32_t* __restrict__ scatter_out, int64_t scatter_n) {
  __shared__ v4i s_w[kFoldSteps * 64];                                                  // 32 KiB
  __shared__ __attribute__((aligned(16))) uint32_t s_tab[kCombineLdsTables * kSlice];  // 60 KiB
  __shared__ __attribute__((aligned(16))) uint32_t s_q[12 * kSlice];                   // 48 KiB
  __shared__ uint32_t s_acc[kCombineThreads];
  const int seg = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  lds_fill<kFoldSteps * 64 / kCombineThreads>(s_w, wfold, kFoldSteps * 64, tid, kCombineThreads);
  __syncthreads();
  const int64_t n = seg_len[seg] < 0 ? 0 : seg_len[seg];
  const int64_t c0 = chunk_off[seg], cend = c0 + ((n + 4095) >> 12);
  const int64_t tiles = (cend - c0 + 31) >> 5;
  for (int64_t t = tid >> 6; t < tiles; t += kCombineThreads / 64) fold_tile(masks, s_w, chunk_res, c0 + 32 * t, cend, lane);
  __syncthreads();  // the segment's chunk residues, written by its own waves, before the combine reads them
  combine_segment<12>(seg, tid, s_tab, s_q, s_acc, chunk_res, chunk_off, seg_len, tables, crc_out, expect, ok_out,
                      scatter_idx, scatter_out, scatter_n, nullptr);
}

// masks: 64 dwords per 4096-byte chunk for each segment, the segment's chunks starting at
// dword 64 * chunk_off[seg]; wfold: the fold's A fragments; chunk_res: scratch of total_chunks
// words.  Same outputs as launch_crc32_batch.
hipError_t launch_crc32_from_masks(const uint32_t* masks, const void* wfold, const int64_t* chunk_off,
                                   const int64_t* seg_len, const uint32_t* tables, uint32_t* chunk_res,
                                   uint32_t* crc_out, const uint32_t* expect, uint8_t* ok_out,
                                   const int64_t* scatter_idx, uint32_t* scatter_out, int64_t scatter_n, int nseg,
                                   int64_t /*total_chunks*/, int /*num_cu*/, hipStream_t stream) {
  if (nseg <= 0) return hipSuccess;
  hipLaunchKernelGGL(crc32_fold_combine_kernel, dim3(static_cast<unsigned>(nseg)), dim3(kCombineThreads), 0, stream,
                     masks, reinterpret_cast<const v4i*>(wfold), chunk_off, seg_len, tables, chunk_res, crc_out, expect,
                     ok_out, scatter_idx, scatter_out, scatter_n);
  return hipGetLastError();
}

hipError_t launch_crc32_batch(const uint8_t* buf, const int64_t* seg_off, const int64_t* seg_len,
                              const int64_t* tile_prefix, const int64_t* res_off, const void* wfrag,
                              const uint32_t* tables, uint32_t* residues, uint32_t* crc_out, const uint32_t* expect,
                              uint8_t* ok_out, const int64_t* scatter_idx, uint32_t* scatter_out, int64_t scatter_n,
                              int nseg, int64_t total_tiles, int num_cu, bool fp4, hipStream_t stream,
                              const int64_t* keys) {
  if (nseg <= 0) return hipSuccess;
  if (total_tiles > 0) {
    const int64_t waves_max = static_cast<int64_t>(num_cu) * 2 * (kCrcThreads / 64);
    int64_t tiles_per_wave = (total_tiles + waves_max - 1) / waves_max;
    if (tiles_per_wave < 1) tiles_per_wave = 1;
    const int64_t waves = (total_tiles + tiles_per_wave - 1) / tiles_per_wave;
    const int64_t grid = (waves + (kCrcThreads / 64) - 1) / (kCrcThreads / 64);
    if (fp4)
      hipLaunchKernelGGL(crc32_group_residue_fp4_kernel, dim3(static_cast<unsigned>(grid)), dim3(kCrcThreads), 0,
                         stream, buf, seg_off, seg_len, tile_prefix, res_off, reinterpret_cast<const v4i*>(wfrag),
                         residues, nseg, total_tiles, tiles_per_wave);
    else
      hipLaunchKernelGGL(crc32_group_residue_kernel, dim3(static_cast<unsigned>(grid)), dim3(kCrcThreads), 0, stream,
                         buf, seg_off, seg_len, tile_prefix, res_off, reinterpret_cast<const v4i*>(wfrag), residues,
                         nseg, total_tiles, tiles_per_wave);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(crc32_combine_kernel<8>, dim3(static_cast<unsigned>(nseg)), dim3(kCombineThreads), 0, stream,
                     residues, res_off, seg_len, tables, crc_out, expect, ok_out, scatter_idx, scatter_out, scatter_n,
                     keys);
  return hipGetLastError();
}

}  // namespace dev
}  // namespace hlsp2p
