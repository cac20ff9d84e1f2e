// Argument block of the one-pass TS demux (ts_demux.hip ts_onepass_kernel), shared by the
// kernel and its host launchers (transmux.cpp, bindings.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hlsp2p {
namespace dev {

struct OnepassArgs {
  const uint8_t* buf;          // plaintext segments
  const int64_t* seg_off;      // [nseg] byte offset in buf (4-byte aligned)
  const int64_t* seg_len;      // [nseg] plaintext length (device; < 0 = failed padding: no packets)
  const int64_t* blk_prefix;   // [nseg + 1] onepass_block_packets()-packet blocks per segment, exclusive prefix
  int nseg;
  int64_t total_blocks;
  uint8_t* es;                 // per segment three class regions at es_off: video | audio | id3
  const int64_t* es_off;       // [nseg]
  const int64_t* es_cap;       // [nseg] class region size (audio at + es_cap, id3 at + 2 es_cap)
  int64_t* pes;                // [nseg][3][max_pes][3]
  int64_t max_pes;
  int64_t* info;               // [nseg][24]
  uint64_t* look;              // [blocks][3] look-back granules, pre-zeroed
  int64_t* lastpes;            // [blocks][3][2] (last PES index of the block, its PTS), pre-filled -1
  unsigned int* ticket;        // [2] pre-zeroed: block ticket, timeout word
};

hipError_t launch_ts_onepass(const OnepassArgs& a, hipStream_t stream);
int onepass_block_packets();

}  // namespace dev
}  // namespace hlsp2p
