// Device-wide exclusive prefix sum (reduce-then-scan, 3 launches).
// Used for localize owner buckets, CSC offsets and backward chunk offsets.
#include "wh_common.h"
#include "wh_kernels.h"

namespace wh {
namespace {

constexpr int kThreads = 256;
constexpr int kItems = 8;
constexpr int kTile = kThreads * kItems;

__device__ __forceinline__ int64_t wave_incl_scan(int64_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int64_t t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

// exclusive block scan of one value per thread; returns exclusive prefix and
// writes the block total to *total
__device__ __forceinline__ int64_t block_excl_scan(int64_t v, int64_t* sh, int64_t* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int64_t inc = wave_incl_scan(v);
  if (lane == 63) sh[wid] = inc;
  __syncthreads();
  int64_t wbase = 0, tot = 0;
  const int nw = blockDim.x >> 6;
  for (int i = 0; i < nw; ++i) {
    if (i < wid) wbase += sh[i];
    tot += sh[i];
  }
  *total = tot;
  __syncthreads();
  return wbase + inc - v;
}

template <typename T>
__global__ __launch_bounds__(kThreads) void k_tile_sum(const T* in, int64_t n, int64_t* tmp) {
  __shared__ int64_t sh[kThreads / 64];
  const int64_t base = (int64_t)blockIdx.x * kTile + (int64_t)threadIdx.x * kItems;
  int64_t s = 0;
#pragma unroll
  for (int i = 0; i < kItems; ++i) {
    int64_t j = base + i;
    if (j < n) s += (int64_t)in[j];
  }
  int64_t tot;
  block_excl_scan(s, sh, &tot);
  if (threadIdx.x == 0) tmp[blockIdx.x] = tot;
}

__global__ __launch_bounds__(1024) void k_scan_partials(int64_t* tmp, int64_t nb) {
  __shared__ int64_t sh[16];
  int64_t carry = 0;
  for (int64_t b0 = 0; b0 < nb; b0 += blockDim.x) {
    int64_t j = b0 + threadIdx.x;
    int64_t v = j < nb ? tmp[j] : 0;
    int64_t tot;
    int64_t ex = block_excl_scan(v, sh, &tot);
    if (j < nb) tmp[j] = carry + ex;
    carry += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) tmp[nb] = carry;
}

template <typename T>
__global__ __launch_bounds__(kThreads) void k_tile_scan(const T* in, int64_t n, const int64_t* tmp,
                                                        int64_t* out, int64_t nb) {
  __shared__ int64_t sh[kThreads / 64];
  const int64_t base = (int64_t)blockIdx.x * kTile + (int64_t)threadIdx.x * kItems;
  int64_t v[kItems];
  int64_t s = 0;
#pragma unroll
  for (int i = 0; i < kItems; ++i) {
    int64_t j = base + i;
    v[i] = j < n ? (int64_t)in[j] : 0;
    s += v[i];
  }
  int64_t tot;
  int64_t run = block_excl_scan(s, sh, &tot) + tmp[blockIdx.x];
#pragma unroll
  for (int i = 0; i < kItems; ++i) {
    int64_t j = base + i;
    if (j < n) out[j] = run;
    run += v[i];
  }
  if (blockIdx.x == nb - 1 && threadIdx.x == 0) out[n] = tmp[nb];
}

template <typename T>
void scan_impl(const T* in, int64_t* out, int64_t n, int64_t* tmp, hipStream_t s) {
  if (n <= 0) {
    WH_HIP_CHECK(hipMemsetAsync(out, 0, sizeof(int64_t), s));
    return;
  }
  const int64_t nb = (n + kTile - 1) / kTile;
  hipLaunchKernelGGL(k_tile_sum<T>, dim3((unsigned)nb), dim3(kThreads), 0, s, in, n, tmp);
  hipLaunchKernelGGL(k_scan_partials, dim3(1), dim3(1024), 0, s, tmp, nb);
  hipLaunchKernelGGL(k_tile_scan<T>, dim3((unsigned)nb), dim3(kThreads), 0, s, in, n, tmp, out,
                     nb);
}

}  // namespace

int64_t lookback_ws_words() { return (int64_t)kLbChannels * kLbMaxTiles + 2; }

Lookback lookback_bind(void* ws) {
  static unsigned int epoch = 0;  // 30-bit, never 0
  epoch = (epoch + 1) & ((1u << 30) - 1);
  if (epoch == 0) epoch = 1;
  Lookback lb;
  lb.gran = static_cast<unsigned long long*>(ws);
  unsigned int* tail = reinterpret_cast<unsigned int*>(lb.gran + (size_t)kLbChannels * kLbMaxTiles);
  lb.ticket = tail;
  lb.err = tail + 1;
  lb.epoch = epoch;
  return lb;
}

int64_t scan_tmp_elems(int64_t n) { return (n + kTile - 1) / kTile + 1; }

void scan_i32(const int32_t* in, int64_t* out, int64_t n, int64_t* tmp, hipStream_t s) {
  scan_impl<int32_t>(in, out, n, tmp, s);
}
void scan_i64(const int64_t* in, int64_t* out, int64_t n, int64_t* tmp, hipStream_t s) {
  scan_impl<int64_t>(in, out, n, tmp, s);
}

}  // namespace wh
