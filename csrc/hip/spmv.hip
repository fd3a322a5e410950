// Sparse matrix-vector products on device-resident CSR/CSC (K4/K5 in
// SURVEY §2.5; reference learn/base/spmv.h:72-119 partitions rows / output
// ranges over OpenMP threads).
//   spmv   : y = X x           G lanes stride over one CSR row, group reduce
//   spmv_t : y = X^T p         one lane per CSC column (segmented sum over the
//                              column's occurrence list: no atomics)
// Columns are the dense local ids produced by `localize`, so the same
// kernels serve L-BFGS (whole split resident in HBM) and minibatch apps.
#include "wh_common.h"
#include "wh_kernels.h"

namespace wh {
namespace {

constexpr int kThreads = 256;

template <int G>
__global__ __launch_bounds__(kThreads) void k_spmv(int64_t nrows, const int64_t* __restrict__ off,
                                                   const int32_t* __restrict__ col,
                                                   const float* __restrict__ val,
                                                   const float* __restrict__ x, float* __restrict__ y) {
  const int lane = threadIdx.x & 63, gl = lane & (G - 1);
  const int64_t row = ((int64_t)blockIdx.x * kThreads + threadIdx.x) / G;
  float acc = 0.f;
  if (row < nrows) {
    const int64_t b = off[row], e = off[row + 1];
    for (int64_t j = b + gl; j < e; j += G) {
      const int c = col[j];
      if (c >= 0) acc += (val ? val[j] : 1.f) * x[c];
    }
  }
  acc = group_sum<G>(acc);
  if (row < nrows && gl == 0) y[row] = acc;
}

__global__ __launch_bounds__(kThreads) void k_spmv_t(int64_t ncol, const int64_t* __restrict__ csc_off,
                                                     const int32_t* __restrict__ csc_row,
                                                     const float* __restrict__ csc_val,
                                                     const float* __restrict__ p, float* __restrict__ y) {
  const int64_t c = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (c >= ncol) return;
  const int64_t b = csc_off[c], e = csc_off[c + 1];
  float acc0 = 0.f, acc1 = 0.f;
  int64_t j = b;
  for (; j + 1 < e; j += 2) {
    acc0 += p[csc_row[j]] * (csc_val ? csc_val[j] : 1.f);
    acc1 += p[csc_row[j + 1]] * (csc_val ? csc_val[j + 1] : 1.f);
  }
  if (j < e) acc0 += p[csc_row[j]] * (csc_val ? csc_val[j] : 1.f);
  y[c] = acc0 + acc1;
}

}  // namespace

void spmv(int64_t nrows, const int64_t* off, const int32_t* col, const float* val, const float* x,
          float* y, hipStream_t s) {
  if (nrows <= 0) return;
  constexpr int G = 8;
  hipLaunchKernelGGL(k_spmv<G>, dim3(grid_for(nrows * G, kThreads)), dim3(kThreads), 0, s, nrows,
                     off, col, val, x, y);
}

void spmv_t(int64_t ncol, const int64_t* csc_off, const int32_t* csc_row, const float* csc_val,
            const float* p, float* y, hipStream_t s) {
  if (ncol <= 0) return;
  hipLaunchKernelGGL(k_spmv_t, dim3(grid_for(ncol, kThreads)), dim3(kThreads), 0, s, ncol,
                     csc_off, csc_row, csc_val, p, y);
}

}  // namespace wh
