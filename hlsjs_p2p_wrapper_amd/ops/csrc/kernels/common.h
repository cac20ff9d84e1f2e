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

// Host helpers
inline int ceil_div(int64_t a, int64_t b) { return static_cast<int>((a + b - 1) / b); }

}  // namespace dev
}  // namespace hlsp2p
