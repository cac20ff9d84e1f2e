// CRC-32 (IEEE 802.3 / zlib, reflected polynomial 0xEDB88320) host side.
//
// * crc32(): oracle (bit-identical to zlib.crc32) for tests and CPU mode;
// * GF(2) operator algebra used to build the constant tables the MFMA CRC kernel consumes
//   (kernels/crc32_mfma.hip):
//     - the 256-byte "group" weight matrix W (2048 data bits x 32 CRC bits), emitted in the
//       exact MFMA B-fragment order the kernel loads with one ds_read_b128 per step;
//     - byte-slice tables of the zero-byte shift operators P_b = A^(8*2^b) (b = 0..39) and
//       their inverses Q_b = A^(-8*2^b) (b = 0..7) that combine group residues and undo the
//       zero padding of the last group.
//
// CRC algebra: with raw(M, r0) the register after processing M from r0 (no final xor),
//   raw(M1||M2, 0) = A^(8|M2|) raw(M1, 0) xor raw(M2, 0),
//   crc(M)         = raw(M, 0) xor A^(8|M|)(0xFFFFFFFF) xor 0xFFFFFFFF.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace hlsp2p {
namespace crc {

constexpr uint32_t kPoly = 0xEDB88320u;
constexpr int kGroupBytes = 256;      // data bytes per MFMA output row
constexpr int kNumP = 40;             // P_b tables, b = 0..39  (shift up to 2^39 bytes)
constexpr int kNumQ = 12;             // Q_b tables, b = 0..11  (undo pad < 4096 bytes)
constexpr int kChunkBytes = 4096;     // data bytes per fused decrypt + CRC chunk (aes_cbc.hip)
constexpr int kSliceWords = 4 * 256;  // one byte-slice table set (4 KiB)

uint32_t crc32(const uint8_t* data, size_t n, uint32_t crc = 0);  // zlib-compatible update

// 32x32 GF(2) matrix as 32 column vectors.
struct Mat {
  uint32_t col[32];
};
uint32_t apply(const Mat& m, uint32_t v);
Mat mul(const Mat& a, const Mat& b);
Mat zero_byte_op();              // A^8
Mat power(const Mat& m, uint64_t e);
bool inverse(const Mat& m, Mat* out);
void slice_table(const Mat& m, uint32_t* out /* kSliceWords */);

// MFMA B-fragment weight table: [step s=0..63][lane=0..63][16 int8] = 65536 bytes.
std::vector<int8_t> mfma_group_weights();
// FP4 (e2m1) variant for v_mfma_scale_f32_32x32x64_f8f6f4: [step s=0..31][lane][16 bytes of
// packed nibbles] = 32768 bytes (see crc32_mfma.hip for the operand scheme).
std::vector<uint8_t> mfma_group_weights_fp4();
// Byte-slice tables: P_0..P_39 then Q_0..Q_11, each kSliceWords u32.
std::vector<uint32_t> shift_tables();
// The CRC fused into the AES-CBC decrypt (aes_cbc.hip), two FP4 MFMA levels:
//  * decrypt side: a wave's 4096-byte chunk holds block 64j + l in lane l (chain j).  Chains 2p
//    and 2p + 1 share accumulator set p: step (jj = j & 1, d = data dword) feeds dword d of the
//    lane's chain-j block; row rho (= lane & 31) collects blocks 64j + rho and 64j + rho + 32
//    (k half h = lane >> 5).  The B fragments [st = 4 jj + d][lane][16 bytes] weigh data bit
//    (byte y, bit b) by A^(8 (1024 (1 - jj) + 512 (1 - h) + 15 - y)) t(b) -- the same for both
//    pairs, so the 8 steps stay in VGPRs.  The accumulator parities go out as one dword per
//    lane per chunk (bit 16 p + i = row (i & 3) + 8 (i >> 2) + 4 (lane >> 5), column lane & 31).
//  * fold side (crc32_mfma.hip): chunk residue = XOR_{p,rho} S[p][rho] D_p[rho] with
//    S[p][rho] = A^(8 * 16 (159 - 128 p - rho)) -- a [32 x 2048] x [2048 x chunks] GF(2) GEMM;
//    A fragments [s = 0..31][lane][16 bytes] (row = CRC bit, k half hh reads mask dword
//    s + 32 hh of the chunk).
// Returns the decrypt fragments followed by the fold fragments.
constexpr int kFusedAesSteps = 8;
constexpr int kFusedFoldSteps = 32;
constexpr int kFusedMaskDwords = 64;  // mask dwords per 4096-byte chunk
std::vector<uint8_t> mfma_chunk_weights_fp4();
// Raw (zero-init) CRC of [FF FF FF FF 00 ...] of `nbytes` bytes: zlib's init value folded into
// the first group's residue.
uint32_t init_fold(int64_t nbytes);

}  // namespace crc
}  // namespace hlsp2p
