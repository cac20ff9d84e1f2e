// Segment data-movement kernels.
//
//  * range_select_kernel  (K1) — batched MediaMap.getSegmentList: for (track, t0, dur)
//    queries over per-track sorted fragment start times (f64), two binary searches give
//    the contiguous index range with t0 <= start <= t0 + dur (closed, as the reference's
//    linear scan at media-map.js:41-51).
//  * segment_copy_kernel  (K4) — batched byte-range copy (pack a peer's non-contiguous
//    segments into one send buffer, byte-range slicing of cached segments, the fleet's
//    payload copies); dwordx4 when both sides are 16-byte aligned, byte tail otherwise.
//
// The segment index (K2 key hash, K3 cache table) is host-native by design: every round is
// planned on the host (runtime/store.cpp SegmentStore, runtime/wants.cpp WantTable, both
// keyed by SegKeyHash), so a device-side copy of the index had no consumer and was removed.
#include "common.h"

namespace hlsp2p {
namespace dev {

// ------------------------------------------------------------------ K1
__global__ void range_select_kernel(const double* __restrict__ starts, const int64_t* __restrict__ track_off,
                                    const int64_t* __restrict__ q_track, const double* __restrict__ q_begin,
                                    const double* __restrict__ q_dur, int64_t* __restrict__ out_lo,
                                    int64_t* __restrict__ out_hi, int64_t nq, int64_t ntracks) {
  const int64_t q = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (q >= nq) return;
  const int64_t t = q_track[q];
  if (t < 0 || t >= ntracks) {
    out_lo[q] = -1;
    out_hi[q] = -1;
    return;
  }
  const double* s = starts + track_off[t];
  const int64_t n = track_off[t + 1] - track_off[t];
  const double b = q_begin[q], e = q_begin[q] + q_dur[q];
  int64_t lo = 0, hi = n;  // first index with s >= b
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (s[mid] < b) lo = mid + 1; else hi = mid;
  }
  const int64_t first = lo;
  hi = n;  // first index with s > e
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (s[mid] <= e) lo = mid + 1; else hi = mid;
  }
  out_lo[q] = first;
  out_hi[q] = lo;
}

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
hipError_t launch_range_select(const double* starts, const int64_t* track_off, const int64_t* q_track,
                               const double* q_begin, const double* q_dur, int64_t* out_lo, int64_t* out_hi,
                               int64_t nq, int64_t ntracks, hipStream_t stream) {
  if (nq <= 0) return hipSuccess;
  hipLaunchKernelGGL(range_select_kernel, dim3(ceil_div(nq, 256)), dim3(256), 0, stream, starts, track_off, q_track,
                     q_begin, q_dur, out_lo, out_hi, nq, ntracks);
  return hipGetLastError();
}

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
