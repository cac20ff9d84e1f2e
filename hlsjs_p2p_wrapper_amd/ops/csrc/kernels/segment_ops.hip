// Segment data-movement kernel.
//
//  * segment_copy_kernel  (K4) — batched byte-range copy (pack a peer's non-contiguous
//    segments into one send buffer, byte-range slicing of cached segments, the fleet's
//    payload copies); dwordx4 when both sides are 16-byte aligned, byte tail otherwise.
//
// The segment index (K2 key hash, K3 cache table) and the time-range select (K1) are
// host-native by design: every round is planned on the host (runtime/store.cpp SegmentStore,
// runtime/wants.cpp WantTable, both keyed by SegKeyHash) and every MediaMap query has its
// answer consumed on the host, so device copies of the index and a range-select kernel had
// no consumer (a launch + D2H sync costs more than the host bisects it would replace) and
// were removed.
#include "common.h"

namespace hlsp2p {
namespace dev {

// ------------------------------------------------------------------ K4
constexpr int kCopyThreads = 256;
constexpr int64_t kCopyChunk = 64 * 1024;

// chunk_prefix: per copy, number of 64 KiB chunks (exclusive prefix, ncopy + 1 entries)
__global__ __launch_bounds__(kCopyThreads) void segment_copy_kernel(
    const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, const int64_t* __restrict__ src_off,
    const int64_t* __restrict__ dst_off, const int64_t* __restrict__ len, const int64_t* __restrict__ chunk_prefix,
    int ncopy) {
  const int64_t gchunk = blockIdx.x;
  const int c = find_seg_wave(chunk_prefix, ncopy, gchunk);
  const int64_t chunk = gchunk - chunk_prefix[c];
  const int64_t n = len[c];
  const int64_t beg = chunk * kCopyChunk;
  const int64_t end = beg + kCopyChunk < n ? beg + kCopyChunk : n;
  const uint8_t* s = src + src_off[c];
  uint8_t* d = dst + dst_off[c];
  const bool vec = ((reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d)) & 15) == 0;
  int64_t i = beg;
  if (vec) {
    const int64_t vend = beg + ((end - beg) & ~int64_t(15));
    // 8 x 16 B per lane in flight per step (a load/store-per-iteration loop waited one HBM
    // round trip per 16 B); tail lanes re-copy the last vector (unconditional stores keep
    // the loads from being sunk next to guarded stores)
    constexpr int kUnroll = 8;
    const int64_t last = vend - 16;
    for (int64_t o0 = beg + 16 * threadIdx.x; o0 < vend; o0 += 16 * kCopyThreads * kUnroll) {
      uint4 v[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int64_t o = o0 + 16 * kCopyThreads * u;
        v[u] = *reinterpret_cast<const uint4*>(s + (o < last ? o : last));
      }
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int64_t o = o0 + 16 * kCopyThreads * u;
        *reinterpret_cast<uint4*>(d + (o < last ? o : last)) = v[u];  // tail: same bytes again
      }
    }
    i = vend;
  }
  for (int64_t o = i + threadIdx.x; o < end; o += kCopyThreads) d[o] = s[o];
}

// ------------------------------------------------------------------ launchers
hipError_t launch_segment_copy(const uint8_t* src, uint8_t* dst, const int64_t* src_off, const int64_t* dst_off,
                               const int64_t* len, const int64_t* chunk_prefix, int ncopy, int64_t total_chunks,
                               hipStream_t stream) {
  if (ncopy <= 0 || total_chunks <= 0) return hipSuccess;
  hipLaunchKernelGGL(segment_copy_kernel, dim3(static_cast<unsigned>(total_chunks)), dim3(kCopyThreads), 0, stream,
                     src, dst, src_off, dst_off, len, chunk_prefix, ncopy);
  return hipGetLastError();
}

}  // namespace dev
}  // namespace hlsp2p
