// Segment-identity and data-movement kernels.
//
//  * range_select_kernel  (K1) — batched MediaMap.getSegmentList: for (track, t0, dur)
//    queries over per-track sorted fragment start times (f64), two binary searches give
//    the contiguous index range with t0 <= start <= t0 + dur (closed, as the reference's
//    linear scan at media-map.js:41-51).
//  * key_hash_kernel      (K2) — 64-bit hash of [swarm, level, urlId, sn] keys (the same
//    mix as the host SegKeyHash, so host and device agree).
//  * device hash table    (K3) — open addressing, linear probing, 32-byte slots
//    {u64 tag, u32 key[4], i64 value}; insert claims a slot with a 64-bit CAS on the tag,
//    lookup / erase are read-mostly.  This is the HBM-resident cache index used for
//    on-device residency queries (batched lookups of wanted keys without a host trip).
//  * segment_copy_kernel  (K4) — batched byte-range copy (pack a peer's non-contiguous
//    segments into one send buffer, byte-range slicing of cached segments); dwordx4
//    when both sides are 16-byte aligned, byte tail otherwise.
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

// ------------------------------------------------------------------ K2
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t key_hash(uint32_t s, uint32_t l, uint32_t u, uint32_t n) {
  const uint64_t a = (uint64_t(s) << 32) | l;
  const uint64_t b = (uint64_t(u) << 32) | n;
  return mix64(a ^ mix64(b + 0x9E3779B97F4A7C15ull));
}

__global__ void key_hash_kernel(const int32_t* __restrict__ keys, uint64_t* __restrict__ out, int64_t n) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4 k = reinterpret_cast<const uint4*>(keys)[i];
  out[i] = key_hash(k.x, k.y, k.z, k.w);
}

// ------------------------------------------------------------------ K3
struct alignas(32) Slot {
  unsigned long long tag;  // 0 empty, 1 tombstone, else hash | 2
  uint32_t key[4];
  long long value;
};

__device__ __forceinline__ unsigned long long make_tag(uint64_t h) { return (h | 2ull); }

__global__ void table_insert_kernel(Slot* __restrict__ slots, uint64_t mask, const int32_t* __restrict__ keys,
                                    const int64_t* __restrict__ values, int64_t n, int32_t* __restrict__ ok) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4 k = reinterpret_cast<const uint4*>(keys)[i];
  const uint64_t h = key_hash(k.x, k.y, k.z, k.w);
  const unsigned long long tag = make_tag(h);
  uint64_t pos = h & mask;
  for (uint64_t probe = 0; probe <= mask; ++probe, pos = (pos + 1) & mask) {
    Slot* s = slots + pos;
    unsigned long long cur = __hip_atomic_load(&s->tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == tag && s->key[0] == k.x && s->key[1] == k.y && s->key[2] == k.z && s->key[3] == k.w) {
      s->value = values[i];  // update in place
      ok[i] = 1;
      return;
    }
    if (cur == 0 || cur == 1) {
      const unsigned long long prev = atomicCAS(&s->tag, cur, tag);
      if (prev == cur) {
        s->key[0] = k.x; s->key[1] = k.y; s->key[2] = k.z; s->key[3] = k.w;
        s->value = values[i];
        ok[i] = 1;
        return;
      }
      // lost the race: re-examine this slot
      --probe;
      pos = (pos - 1) & mask;
    }
  }
  ok[i] = 0;  // table full
}

__global__ void table_lookup_kernel(const Slot* __restrict__ slots, uint64_t mask, const int32_t* __restrict__ keys,
                                    int64_t* __restrict__ out, int64_t n, int erase) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4 k = reinterpret_cast<const uint4*>(keys)[i];
  const uint64_t h = key_hash(k.x, k.y, k.z, k.w);
  const unsigned long long tag = make_tag(h);
  uint64_t pos = h & mask;
  for (uint64_t probe = 0; probe <= mask; ++probe, pos = (pos + 1) & mask) {
    const Slot* s = slots + pos;
    const unsigned long long cur = s->tag;
    if (cur == 0) break;
    if (cur == tag && s->key[0] == k.x && s->key[1] == k.y && s->key[2] == k.z && s->key[3] == k.w) {
      out[i] = s->value;
      if (erase) const_cast<Slot*>(s)->tag = 1ull;
      return;
    }
  }
  out[i] = -1;
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

hipError_t launch_key_hash(const int32_t* keys, uint64_t* out, int64_t n, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(key_hash_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, stream, keys, out, n);
  return hipGetLastError();
}

hipError_t launch_table_insert(void* slots, uint64_t mask, const int32_t* keys, const int64_t* values, int64_t n,
                               int32_t* ok, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(table_insert_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, stream, static_cast<Slot*>(slots),
                     mask, keys, values, n, ok);
  return hipGetLastError();
}

hipError_t launch_table_lookup(const void* slots, uint64_t mask, const int32_t* keys, int64_t* out, int64_t n,
                               int erase, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(table_lookup_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, stream,
                     static_cast<const Slot*>(slots), mask, keys, out, n, erase);
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
