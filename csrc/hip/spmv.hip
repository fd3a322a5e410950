// Sparse matrix-vector products on device-resident CSR/CSC (K4/K5 in
// SURVEY §2.5; reference learn/base/spmv.h:72-119 partitions rows / output
// ranges over OpenMP threads).
//   spmv   : y = X x           G lanes stride over one CSR row, group reduce
//   spmv_t : y = X^T p         runs on the linear backward's chunked
//                              segmented sums (fm.hip; csrc/bind/hip_ops.cc
//                              spmv_t): skew-robust over power-law columns
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

}  // namespace

void spmv(int64_t nrows, const int64_t* off, const int32_t* col, const float* val, const float* x,
          float* y, hipStream_t s) {
  if (nrows <= 0) return;
  constexpr int G = 8;
  hipLaunchKernelGGL(k_spmv<G>, dim3(grid_for(nrows * G, kThreads)), dim3(kThreads), 0, s, nrows,
                     off, col, val, x, y);
}


}  // namespace wh
