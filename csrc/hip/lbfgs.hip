// OWL-QN L-BFGS vector kernels (reference learn/solver/lbfgs.h:358-407 SetL1Dir
// / FixDirL1Sign / FixWeightL1Sign, the dot-product batch of
// FindChangeDirection :216-318 and its direction build :288-299).
// Memory-bound passes over 2^24-element vectors with their reductions fused:
// each kernel reads its operands once and leaves one fp64 partial per block
// (summed in block order by sum_parts: deterministic).
#include <hip/hip_runtime.h>

#include "wh_common.h"
#include "wh_kernels.h"

namespace wh {
namespace {

constexpr int kT = 256;

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

// Reductions: a bounded grid (kRedBlocks) grid-strides over the vectors
// and every block leaves one fp64 partial per value; sum_parts (glm.hip)
// adds them in block order. (One fp64 atomic per 256-element block on ONE
// word serialised 65k atomics at 2^24 weights: 0.8 ms per pass.)
constexpr int kRedBlocks = 1024;

template <int NV>
__device__ __forceinline__ void block_partials(double (&v)[NV], double* __restrict__ part) {
  __shared__ double sh[NV][kT / 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const double s = wave_sum_d(v[k]);
    if (lane == 0) sh[k][wv] = s;
  }
  __syncthreads();
  if (threadIdx.x < NV) {
    double s = 0.0;
    for (int i = 0; i < kT / 64; ++i) s += sh[threadIdx.x][i];
    part[(int64_t)blockIdx.x * NV + threadIdx.x] = s;
  }
}

// d[i] = 0 where d * steep <= 0 (FixDirL1Sign, l1 != 0); partial sums of
// d * steep (float product, fp64 sum: the reference Dot)
__global__ __launch_bounds__(kT) void k_owlqn_fix_dot(float* __restrict__ d,
                                                      const float* __restrict__ steep, int64_t n,
                                                      int fix, double* __restrict__ part) {
  double acc[1] = {0.0};
  for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kT) {
    float di = d[i];
    const float si = steep[i];
    if (fix && di * si <= 0.f) {
      di = 0.f;
      d[i] = 0.f;
    }
    acc[0] += (double)(di * si);
  }
  block_partials<1>(acc, part);
}

// nw = w + alpha d, zeroed where its sign flips (FixWeightL1Sign, l1 != 0);
// partial sums of |nw|
__global__ __launch_bounds__(kT) void k_owlqn_step(const float* __restrict__ w,
                                                   const float* __restrict__ d, int64_t n,
                                                   float alpha, int fix, float* __restrict__ nw,
                                                   double* __restrict__ part) {
  double acc[1] = {0.0};
  for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kT) {
    const float wi = w[i];
    float v = wi + d[i] * alpha;
    if (fix && v * wi < 0.f) v = 0.f;
    nw[i] = v;
    acc[0] += fabs((double)v);
  }
  block_partials<1>(acc, part);
}

// The history dots of one L-BFGS iteration against its probe rows (the new
// steepest direction and the newest s / y: every dot FindChangeDirection
// needs, lbfgs.h:237-256, is <H_r, H_probe>): out[r][k] = <H[r0 + r],
// H[probe k]> for nr <= RM rows, one pass over the rows (float4 columns,
// RM rows' loads in flight per thread, exact fp64 products and sums), one
// partial per block and value.
template <int RM, int KP>
__global__ __launch_bounds__(kT) void k_hist_dots(const float* __restrict__ H, int64_t n4,
                                                  int64_t ld, int r0, int nr, int4 probes,
                                                  double* __restrict__ part) {
  double acc[RM * KP];
#pragma unroll
  for (int i = 0; i < RM * KP; ++i) acc[i] = 0.0;
  const int pr[4] = {probes.x, probes.y, probes.z, probes.w};
  for (int64_t j = (int64_t)blockIdx.x * kT + threadIdx.x; j < n4; j += (int64_t)gridDim.x * kT) {
    float4 p[KP];
#pragma unroll
    for (int k = 0; k < KP; ++k)
      p[k] = reinterpret_cast<const float4*>(H + (int64_t)pr[k] * ld)[j];
    float4 h[RM];
#pragma unroll
    for (int r = 0; r < RM; ++r)
      h[r] = r < nr ? reinterpret_cast<const float4*>(H + (int64_t)(r0 + r) * ld)[j]
                    : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int r = 0; r < RM; ++r)
#pragma unroll
      for (int k = 0; k < KP; ++k) {
        double a = acc[r * KP + k];
        a = fma((double)h[r].x, (double)p[k].x, a);
        a = fma((double)h[r].y, (double)p[k].y, a);
        a = fma((double)h[r].z, (double)p[k].z, a);
        a = fma((double)h[r].w, (double)p[k].w, a);
        acc[r * KP + k] = a;
      }
  }
  block_partials<RM * KP>(acc, part);
}

// The direction slice and its sign fix + dot in one pass (lbfgs.h:288-299):
// d = sum over the listed rows (in the reference's AddScale order) of
// coef * H[row], accumulated in fp32; then FixDirL1Sign against the steepest
// direction row and partials of d * steep.
struct DirRows {
  int32_t row[64];
  float coef[64];
};

__global__ __launch_bounds__(kT) void k_dir_fix_dot(const float* __restrict__ H, int64_t n,
                                                    int64_t ld, DirRows rows, int nrow,
                                                    int steep_row, int fix,
                                                    float* __restrict__ d,
                                                    double* __restrict__ part) {
  double acc[1] = {0.0};
  const float* st = H + (int64_t)steep_row * ld;
  for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kT) {
    float v = 0.f;
#pragma unroll 8
    for (int r = 0; r < nrow; ++r) v += H[(int64_t)rows.row[r] * ld + i] * rows.coef[r];
    const float si = st[i];
    if (fix && v * si <= 0.f) v = 0.f;
    d[i] = v;
    acc[0] += (double)(v * si);
  }
  block_partials<1>(acc, part);
}

// out[p] += sum_j H[ia[p]][j] * H[ib[p]][j] for up to kMaxPairs pairs over
// rows of H [R, n] (the general form; the solver uses k_hist_dots)
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

inline unsigned red_blocks(int64_t n) {
  const int64_t b = (n + kT - 1) / kT;
  return (unsigned)(b < kRedBlocks ? (b < 1 ? 1 : b) : kRedBlocks);
}

int64_t owlqn_part_doubles() { return kRedBlocks * 64; }

void owlqn_fix_dot(float* d, const float* steep, int64_t n, int fix, double* part,
                   double* vdot, hipStream_t s) {
  const unsigned nb = red_blocks(n);
  hipLaunchKernelGGL(k_owlqn_fix_dot, dim3(nb), dim3(kT), 0, s, d, steep, n, fix, part);
  sum_parts(part, (int)nb, 1, vdot, s);
}

void owlqn_step(const float* w, const float* d, int64_t n, float alpha, int fix, float* nw,
                double* part, double* l1sum, hipStream_t s) {
  const unsigned nb = red_blocks(n);
  hipLaunchKernelGGL(k_owlqn_step, dim3(nb), dim3(kT), 0, s, w, d, n, alpha, fix, nw, part);
  sum_parts(part, (int)nb, 1, l1sum, s);
}

// rows [0, R) of H (row stride ld floats, n columns, n % 4 == 0 and H
// 16-byte aligned) against up to 4 probe rows: out [R][K] (fp64)
bool hist_dots(const float* H, int R, int64_t n, int64_t ld, const int32_t* probe, int K,
               double* part, double* out, hipStream_t s) {
  if (K < 1 || K > 4 || R < 1 || (n & 3) || (ld & 3) ||
      (reinterpret_cast<uintptr_t>(H) & 15))
    return false;
  constexpr int RM = 11;
  const int4 pr = make_int4(probe[0], K > 1 ? probe[1] : 0, K > 2 ? probe[2] : 0,
                            K > 3 ? probe[3] : 0);
  const unsigned nb = red_blocks(n / 4);
  for (int r0 = 0; r0 < R; r0 += RM) {
    const int nr = R - r0 < RM ? R - r0 : RM;
    switch (K) {
      case 1: hipLaunchKernelGGL((k_hist_dots<RM, 1>), dim3(nb), dim3(kT), 0, s, H, n / 4, ld, r0, nr, pr, part); break;
      case 2: hipLaunchKernelGGL((k_hist_dots<RM, 2>), dim3(nb), dim3(kT), 0, s, H, n / 4, ld, r0, nr, pr, part); break;
      case 3: hipLaunchKernelGGL((k_hist_dots<RM, 3>), dim3(nb), dim3(kT), 0, s, H, n / 4, ld, r0, nr, pr, part); break;
      default: hipLaunchKernelGGL((k_hist_dots<RM, 4>), dim3(nb), dim3(kT), 0, s, H, n / 4, ld, r0, nr, pr, part); break;
    }
    sum_parts(part, (int)nb, nr * K, out + (int64_t)r0 * K, s, RM * K);
  }
  return true;
}

bool dir_fix_dot(const float* H, int64_t n, int64_t ld, const int32_t* rows, const float* coef,
                 int nrow, int steep_row, int fix, float* d, double* part, double* vdot,
                 hipStream_t s) {
  if (nrow < 0 || nrow > 64) return false;
  DirRows dr;
  for (int r = 0; r < 64; ++r) {
    dr.row[r] = r < nrow ? rows[r] : 0;
    dr.coef[r] = r < nrow ? coef[r] : 0.f;
  }
  const unsigned nb = red_blocks(n);
  hipLaunchKernelGGL(k_dir_fix_dot, dim3(nb), dim3(kT), 0, s, H, n, ld, dr, nrow, steep_row, fix,
                     d, part);
  sum_parts(part, (int)nb, 1, vdot, s);
  return true;
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
