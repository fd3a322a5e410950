// Common device helpers for the wormhole_amd CDNA4 (gfx950) kernels.
// Wave64 everywhere: lane = threadIdx.x & 63, ballots are 64-bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wh {

constexpr int kWave = 64;
constexpr uint64_t kEmptyKey = ~0ull;  // reserved: never a valid feature id

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t x) {
  // splitmix64 finaliser: table-probe hash
  x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27; x *= 0x94d049bb133111ebull;
  x ^= x >> 31;
  return x;
}

__host__ __device__ __forceinline__ uint64_t mix64b(uint64_t x) {
  // a second, independent mixer (murmur3 fmix64) used for shard ownership so
  // the owner choice is uncorrelated with the in-table probe position
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

__host__ __device__ __forceinline__ int owner_of(uint64_t key, int nshard) {
  return nshard <= 1 ? 0 : (int)(mix64b(key) % (uint64_t)nshard);
}

// XCD-aware block remap (bijective for any n): blocks b, b + 8, ... share an
// XCD's L2 under round-robin dispatch, so group b % 8 gets a CONTIGUOUS
// range of the logical blocks -- neighbouring tiles whose reads or partial
// line writes overlap then meet in one L2 (MI355X: 8 XCDs, 4 MB L2 each)
__device__ __forceinline__ int64_t xcd_swizzle(int64_t b, int64_t n) {
  const int64_t g = b & 7, q = n >> 3, r = n & 7;
  return (g < r ? g * (q + 1) : r * (q + 1) + (g - r) * q) + (b >> 3);
}

// counter-based uniform in [0,1): stateless, reproducible per (seed, a, b)
__host__ __device__ __forceinline__ float uhash01(uint64_t seed, uint64_t a, uint64_t b = 0) {
  uint64_t h = mix64(seed ^ mix64(a * 0x9e3779b97f4a7c15ull + b));
  return (float)(h >> 40) * (1.0f / 16777216.0f);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// sum over aligned groups of G lanes (G power of two <= 64)
template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block-wide double sum, result valid in thread 0; `sh` needs >= nwaves doubles
__device__ __forceinline__ double block_sum_d(double v, double* sh) {
  v = wave_sum_d(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) sh[wid] = v;
  __syncthreads();
  double r = 0;
  if (threadIdx.x == 0) {
    const int nw = (blockDim.x + 63) >> 6;
    for (int i = 0; i < nw; ++i) r += sh[i];
  }
  return r;
}

__device__ __forceinline__ long long wave_sum_ll(long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Runs job(src, gl) for every lane `src` whose `has` is set, G lanes per job.
// job() is called by ALL lanes (src < 0: this group is idle this round) so it
// may shuffle; it must read per-job data with __shfl(v, src >= 0 ? src : lane).
template <int G, typename F>
__device__ __forceinline__ void for_each_row_job(bool has, F&& job) {
  const int lane = threadIdx.x & 63, grp = lane / G, gl = lane & (G - 1);
  uint64_t m = __ballot(has);
  while (m) {
    int src = -1;
#pragma unroll
    for (int t = 0; t < 64 / G; ++t) {
      if (m) {
        const int b = __ffsll((unsigned long long)m) - 1;
        if (t == grp) src = b;
        m &= m - 1;
      }
    }
    job(src, gl);
  }
}

inline int grid_for(int64_t n, int threads, int max_blocks = 0x7fffffff) {
  int64_t b = (n + threads - 1) / threads;
  if (b < 1) b = 1;
  if (b > max_blocks) b = max_blocks;
  return (int)b;
}

}  // namespace wh

#define WH_HIP_CHECK(expr)                                                   \
  do {                                                                       \
    hipError_t _e = (expr);                                                  \
    if (_e != hipSuccess) {                                                  \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(_e),      \
              __FILE__, __LINE__);                                           \
      abort();                                                               \
    }                                                                        \
  } while (0)
