// Shared device helpers for the CDNA4 (gfx950) kernels.  Wave64 everywhere.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hlsp2p {
namespace dev {

constexpr int kWave = 64;

// Host-side launch status (filled by launchers, returned to the binding).
struct LaunchStatus {
  hipError_t err;
};

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

__device__ __forceinline__ uint32_t rotr(uint32_t x, int s) { return (x >> s) | (x << (32 - s)); }

// Monotone segment walk: first index s with prefix[s + 1] > v, starting from `s`.
__device__ __forceinline__ int advance_seg(const int64_t* __restrict__ prefix, int s, int64_t v) {
  while (prefix[s + 1] <= v) ++s;
  return s;
}

// Binary search: largest s in [0, n) with prefix[s] <= v  (prefix has n+1 entries).
__device__ __forceinline__ int find_seg(const int64_t* __restrict__ prefix, int n, int64_t v) {
  int lo = 0, hi = n;  // invariant: prefix[lo] <= v < prefix[hi]
  while (hi - lo > 1) {
    int mid = (lo + hi) >> 1;
    if (prefix[mid] <= v) lo = mid; else hi = mid;
  }
  return lo;
}

// Same result as find_seg for a wave-uniform v, with all 64 lanes active: each lane tests
// one prefix entry and a ballot counts the entries <= v, so segment lookup costs ONE
// global round trip per 64-way level (n <= 64: one) instead of log2(n) dependent loads
// at the head of every workgroup.
__device__ __forceinline__ int find_seg_wave(const int64_t* __restrict__ prefix, int n, int64_t v) {
  const int lane = static_cast<int>(threadIdx.x & 63);
  int lo = 0, cnt = n;  // answer in [lo, lo + cnt)
  while (cnt > 64) {
    const int stride = (cnt + 63) >> 6;
    const int idx = lo + lane * stride;
    const bool le = idx < lo + cnt && prefix[idx] <= v;
    lo += (__popcll(__ballot(le)) - 1) * stride;
    cnt = stride < n - lo ? stride : n - lo;
  }
  const bool le = lane < cnt && prefix[lo + lane] <= v;
  return __builtin_amdgcn_readfirstlane(lo + __popcll(__ballot(le)) - 1);
}

// Workgroup copy of `count` elements global -> LDS with every load of the thread issued
// before its first LDS store (kIters >= ceil(count / nthreads)).  The plain strided loop
// compiles to load / s_waitcnt vmcnt(0) / ds_write per element: one L2 round trip per
// iteration, serialised — 8-40 of them at the head of a kernel.
template <int kIters, typename T>
__device__ __forceinline__ void lds_fill(T* __restrict__ dst, const T* __restrict__ src, int count, int tid,
                                         int nthreads) {
  T v[kIters];
  const int last = count - 1;
#pragma unroll
  for (int k = 0; k < kIters; ++k) {
    const int i = tid + k * nthreads;
    v[k] = src[i < last ? i : last];
  }
  // out-of-range lanes store src[last] to dst[last] again (same value): an unconditional
  // store keeps the compiler from sinking each load into a guarded block next to its store
#pragma unroll
  for (int k = 0; k < kIters; ++k) {
    const int i = tid + k * nthreads;
    dst[i < last ? i : last] = v[k];
  }
}

// Host helpers
inline int ceil_div(int64_t a, int64_t b) { return static_cast<int>((a + b - 1) / b); }

}  // namespace dev
}  // namespace hlsp2p
