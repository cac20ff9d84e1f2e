// AES-128 host implementation: key schedules, block cipher, CBC + PKCS#7.
//
// Roles:
//   * packager: the synthetic origin encrypts segments exactly as an HLS packager does
//     (METHOD=AES-128, CBC, PKCS#7; RFC 8216 §5.2) — CBC *encryption* is sequential per
//     segment so it lives on the host;
//   * oracle: CPU reference for the CDNA4 decrypt kernel (kernels/aes_cbc.hip) and the
//     CPU-mode decrypt path used by the no-GPU test tier;
//   * table source: the device kernel's Td0 / inverse S-box tables and the
//     equivalent-inverse-cipher round keys are produced here, so host and device agree
//     bit-for-bit by construction.
//
// Word convention: a 128-bit state is four big-endian 32-bit column words.
#pragma once
#include <cstddef>
#include <cstdint>

namespace hlsp2p {
namespace aes {

struct Tables {
  uint8_t sbox[256];
  uint8_t inv_sbox[256];
  uint32_t te0[256];  // (2s, s, s, 3s)
  uint32_t td0[256];  // (14si, 9si, 13si, 11si)
};

const Tables& tables();

// 44 words: encryption round keys.
void expand_key_enc(const uint8_t key[16], uint32_t rk[44]);
// 44 words: equivalent-inverse-cipher round keys (round order reversed, InvMixColumns
// applied to rounds 1..9).  This is the layout the device kernel consumes.
void expand_key_dec(const uint8_t key[16], uint32_t drk[44]);

void encrypt_block(const uint32_t rk[44], const uint8_t in[16], uint8_t out[16]);
void decrypt_block(const uint32_t drk[44], const uint8_t in[16], uint8_t out[16]);

// CBC encrypt with PKCS#7 padding.  `out` must hold n + 16 bytes.  Returns output size.
size_t cbc_encrypt_pkcs7(const uint8_t key[16], const uint8_t iv[16], const uint8_t* in, size_t n,
                         uint8_t* out);
// CBC decrypt of n bytes (multiple of 16, no unpadding) with equivalent-inverse-cipher
// round keys.  Uses the x86 AES instructions when the CPU has them (CBC decryption is
// block-parallel: eight blocks in flight), the T-table cipher otherwise.
void cbc_decrypt_raw(const uint32_t drk[44], const uint8_t iv[16], const uint8_t* in, size_t n, uint8_t* out);
bool have_aesni();

// CBC decrypt + PKCS#7 unpad.  `n` must be a multiple of 16.  Returns plaintext size, or
// -1 on a bad size / padding.
int64_t cbc_decrypt_pkcs7(const uint8_t key[16], const uint8_t iv[16], const uint8_t* in, size_t n,
                          uint8_t* out);

}  // namespace aes
}  // namespace hlsp2p
