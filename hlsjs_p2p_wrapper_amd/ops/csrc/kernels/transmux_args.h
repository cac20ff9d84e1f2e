// Argument block of the fused decrypt + demux launch (transmux_fused.hip), shared by the
// kernel and its host launcher (transmux.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hlsp2p {
namespace dev {

struct TransmuxArgs {
  const uint8_t* src;        // batch source (ciphertext or clear segments), 16-byte aligned per segment
  const int64_t* src_off;    // [nseg]
  const int64_t* src_len;    // [nseg] source bytes (encrypted: a positive multiple of 16)
  const uint8_t* enc;        // [nseg] 1 = AES-128-CBC
  const uint32_t* drk;       // [nseg][44] little-endian equivalent-inverse-cipher round keys
  const uint32_t* drk_rot;   // [nseg][44] the same, rounds 1..9 rotated left by 24 (the fused rounds' form)
  const uint32_t* ivw;       // [nseg][4]
  const uint32_t* tdl;       // TdL[256]
  const uint8_t* isb;        // InvSbox[256]
  const int64_t* tile_prefix;  // [nseg + 1] tiles per segment, exclusive prefix
  uint8_t* es;               // ES buffer: per segment three class regions (video, audio, id3)
  const int64_t* es_off;     // [nseg] (3 x es_cap bytes from here belong to the segment)
  const int64_t* es_cap;     // [nseg] region size: audio at + es_cap, id3 at + 2 es_cap
  int64_t* pes;              // [nseg][3][max_pes][3], pre-filled with -1
  int64_t* info;             // [nseg][24], pre-zeroed
  int64_t* out_len;          // [nseg] plaintext length (-1: bad padding)
  uint64_t* look;            // [tiles][3] granules, pre-zeroed
  uint64_t* psi;             // [nseg][2] granules, pre-zeroed
  int64_t* lastpes;          // [tiles][3][2] (last PES index in the tile, its PTS), pre-filled with -1
  unsigned int* ticket;      // pre-zeroed
  unsigned int* timeout;     // pre-zeroed; nonzero = a hand-off spin gave up
  uint64_t* prof;            // diagnostics only: [grid][16] per-role cycle counters, or null
  int64_t max_pes;
  int diag;                  // diagnostics only: 1 = decrypt alone, 2 = skip the payload copy-out
  int flags;                 // experiments only: bit 0 = no s_setprio for the latency-bound roles
  int nseg;
  int64_t total_tiles;
};

int transmux_tile_bytes();
hipError_t launch_transmux_fused(const TransmuxArgs& args, int num_cu, hipStream_t stream);

}  // namespace dev
}  // namespace hlsp2p
