// OWL-QN L-BFGS vector kernels (reference learn/solver/lbfgs.h:358-407 SetL1Dir
// / FixDirL1Sign / FixWeightL1Sign and the dot-product batch of
// FindChangeDirection :216-318). Memory-bound elementwise passes with their
// reductions fused: each kernel reads its operands once and finishes its fp64
// sum with one atomic per block.
#include <hip/hip_runtime.h>

#include "wh_common.h"
#include "wh_kernels.h"

namespace wh {
namespace {

constexpr int kT = 256;

__device__ __forceinline__ double block_sum_d(double v, double* sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) sh[w] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0)
    for (int i = 0; i < kT / 64; ++i) s += sh[i];
  return s;  // valid in thread 0
}

// d = pseudo-gradient steepest-descent direction (SetL1Dir)
__global__ __launch_bounds__(kT) void k_owlqn_dir(const float* __restrict__ g,
                                                  const float* __restrict__ w, int64_t n, float l1,
                                                  float* __restrict__ d) {
  const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  const float gi = g[i], wi = w[i];
  float r;
  if (l1 == 0.f) {
    r = -gi;
  } else if (wi > 0.f) {
    r = -gi - l1;
  } else if (wi < 0.f) {
    r = -gi + l1;
  } else {
    r = gi < -l1 ? -gi - l1 : (gi > l1 ? -gi + l1 : 0.f);
  }
  d[i] = r;
}

// d[i] = 0 where d * steep <= 0 (FixDirL1Sign, l1 != 0); vdot += d * steep
__global__ __launch_bounds__(kT) void k_owlqn_fix_dot(float* __restrict__ d,
                                                      const float* __restrict__ steep, int64_t n,
                                                      int fix, double* __restrict__ vdot) {
  __shared__ double sh[kT / 64];
  const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
  double acc = 0.0;
  if (i < n) {
    float di = d[i];
    const float si = steep[i];
    if (fix && di * si <= 0.f) {
      di = 0.f;
      d[i] = 0.f;
    }
    acc = (double)di * (double)si;
  }
  const double s = block_sum_d(acc, sh);
  if (threadIdx.x == 0) atomicAdd(vdot, s);
}

// nw = w + alpha d, zeroed where its sign flips (FixWeightL1Sign, l1 != 0);
// l1sum += |nw|
__global__ __launch_bounds__(kT) void k_owlqn_step(const float* __restrict__ w,
                                                   const float* __restrict__ d, int64_t n,
                                                   float alpha, int fix, float* __restrict__ nw,
                                                   double* __restrict__ l1sum) {
  __shared__ double sh[kT / 64];
  const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
  double acc = 0.0;
  if (i < n) {
    const float wi = w[i];
    float v = wi + d[i] * alpha;
    if (fix && v * wi < 0.f) v = 0.f;
    nw[i] = v;
    acc = fabs((double)v);
  }
  const double s = block_sum_d(acc, sh);
  if (threadIdx.x == 0) atomicAdd(l1sum, s);
}

// out[p] += sum_j H[ia[p]][j] * H[ib[p]][j] for up to kMaxPairs pairs over
// rows of H [R, n]: one pass over the history (each column's R values are
// loaded once per thread), fp64 per-thread partials, one atomic per block
// and pair.
constexpr int kMaxRows = 64, kMaxPairs = 64;

__global__ __launch_bounds__(kT) void k_multi_dot(const float* __restrict__ H, int R, int64_t n,
                                                  const int32_t* __restrict__ ia,
                                                  const int32_t* __restrict__ ib, int np,
                                                  double* __restrict__ out) {
  __shared__ float col[kMaxRows][kT];
  __shared__ double red[kMaxPairs][kT / 64];
  __shared__ int pa[kMaxPairs], pb[kMaxPairs];
  if (threadIdx.x < np) {
    pa[threadIdx.x] = ia[threadIdx.x];
    pb[threadIdx.x] = ib[threadIdx.x];
  }
  double acc[kMaxPairs];
#pragma unroll
  for (int p = 0; p < kMaxPairs; ++p) acc[p] = 0.0;
  __syncthreads();
  for (int64_t j = (int64_t)blockIdx.x * kT + threadIdx.x; j - threadIdx.x < n;
       j += (int64_t)gridDim.x * kT) {
    for (int r = 0; r < R; ++r) col[r][threadIdx.x] = j < n ? H[(int64_t)r * n + j] : 0.f;
#pragma unroll
    for (int p = 0; p < kMaxPairs; ++p)
      if (p < np) acc[p] += (double)col[pa[p]][threadIdx.x] * (double)col[pb[p]][threadIdx.x];
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int p = 0; p < kMaxPairs; ++p) {
    if (p >= np) break;
    double v = acc[p];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) red[p][w] = v;
  }
  __syncthreads();
  if (threadIdx.x < np) {
    double s = 0.0;
    for (int i = 0; i < kT / 64; ++i) s += red[threadIdx.x][i];
    atomicAdd(out + threadIdx.x, s);
  }
}

inline unsigned blocks(int64_t n) { return (unsigned)((n + kT - 1) / kT); }

}  // namespace

void owlqn_dir(const float* g, const float* w, int64_t n, float l1, float* d, hipStream_t s) {
  if (n > 0) hipLaunchKernelGGL(k_owlqn_dir, dim3(blocks(n)), dim3(kT), 0, s, g, w, n, l1, d);
}

void owlqn_fix_dot(float* d, const float* steep, int64_t n, int fix, double* vdot,
                   hipStream_t s) {
  if (n > 0)
    hipLaunchKernelGGL(k_owlqn_fix_dot, dim3(blocks(n)), dim3(kT), 0, s, d, steep, n, fix, vdot);
}

void owlqn_step(const float* w, const float* d, int64_t n, float alpha, int fix, float* nw,
                double* l1sum, hipStream_t s) {
  if (n > 0)
    hipLaunchKernelGGL(k_owlqn_step, dim3(blocks(n)), dim3(kT), 0, s, w, d, n, alpha, fix, nw,
                       l1sum);
}

bool multi_dot(const float* H, int R, int64_t n, const int32_t* ia, const int32_t* ib, int np,
               double* out, hipStream_t s) {
  if (R > kMaxRows || np > kMaxPairs || np > kT) return false;
  if (n <= 0 || np <= 0) return true;
  const int64_t b = (n + kT - 1) / kT;
  const unsigned grid = (unsigned)(b < 2048 ? b : 2048);
  hipLaunchKernelGGL(k_multi_dot, dim3(grid), dim3(kT), 0, s, H, R, n, ia, ib, np, out);
  return true;
}

}  // namespace wh
