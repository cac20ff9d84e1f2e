// Argument block of the scatter demux (ts_scatter.hip): AES-128-CBC segments demuxed without
// a plaintext buffer.  Shared by the kernels' launcher and the host (transmux.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hlsp2p {
namespace dev {

struct ScatterArgs {
  const uint8_t* src;           // ciphertext segments (16-byte aligned)
  const int64_t* src_off;       // [nseg]
  const int64_t* aes_blk;       // [nseg + 1] 16-byte blocks per segment, exclusive prefix
  const int64_t* aes_chunks;    // [nseg + 1] scatter-decrypt chunks (kScatterChunkBlocks blocks), prefix
  const int64_t* hdr_chunks;    // [nseg + 1] header chunks (64 groups of 4 packets), prefix
  const uint32_t* drk;          // [nseg][44] little-endian equivalent-inverse-cipher round keys
  const uint32_t* ivw;          // [nseg][4]
  const uint32_t* tdl;          // TdL[256]
  const uint8_t* isb;           // InvSbox[256]
  const int64_t* blk_prefix;    // [nseg + 1] 256-packet demux blocks, exclusive prefix
  const int64_t* pkt_base;      // [nseg] blk_prefix * 256: the segment's first packet slot
  const int64_t* pkt_slots;     // [nseg] its packet slots
  uint32_t* hdr;                // [blocks * 256] packet header words
  uint32_t* meta;               // [blocks * 256]
  int64_t* pts_dts;             // [blocks * 256 * 2]
  int32_t* aux;                 // [blocks * 12 + nseg * 7]: block sums | block prefixes | segment totals
  uint2* place;                 // [blocks * 256] (ES bias, payload range) per packet
  uint32_t* seam;               // [blocks * 256][2] head / tail seam bytes per packet
  uint8_t* es;                  // ES buffer, [video | audio | id3] packed per segment at es_off
  const int64_t* es_off;        // [nseg]
  int64_t* pes;                 // [nseg][3][max_pes][3]
  int64_t* info;                // [nseg][24]
  int64_t* out_len;             // [nseg] plaintext length (-1: bad padding)
  int64_t max_pes;
  int nseg;
  int64_t total_blocks;         // demux blocks
  int64_t aes_total_chunks;
  int64_t hdr_total_chunks;
};

// blocks one wave of the scatter decrypt owns per iteration (aes_cbc.hip: 64 lanes x kBlk
// chains decrypt 256; the last is a lookahead lending its first bytes to the 255th)
constexpr int kScatterChunkBlocks = 255;
// header chunk = 64 lanes x one 4-packet group (752 bytes = 47 AES blocks) each
constexpr int kScatterGroupPackets = 4;
constexpr int kScatterChunkGroups = 64;

hipError_t launch_ts_scatter(const ScatterArgs& a, int num_cu, hipStream_t stream);

}  // namespace dev
}  // namespace hlsp2p
