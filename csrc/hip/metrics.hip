// Per-minibatch evaluation metrics (reference learn/base/binary_class_evaluation.h).
// Loss / objective / accuracy sums are fused into the forward kernel (fm.hip);
// this file holds the exact AUC rank-sum over predictions sorted ascending.
#include <rocprim/device/device_radix_sort.hpp>

#include "wh_common.h"
#include "wh_kernels.h"

#include <algorithm>

namespace wh {
namespace {

constexpr int kThreads = 256;

__global__ void k_pos_flags(const float* lab, int64_t n, int32_t* flags) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i < n) flags[i] = lab[i] > 0.f ? 1 : 0;
}

// area = sum over negatives of #positives ranked strictly before them
__global__ __launch_bounds__(kThreads) void k_auc_area(const float* lab, const int64_t* excl,
                                                       int64_t n, double* out) {
  __shared__ double sh[kThreads / 64];
  double a = 0;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kThreads)
    if (!(lab[i] > 0.f)) a += (double)excl[i];
  const double r = block_sum_d(a, sh);
  if (threadIdx.x == 0) atomicAdd(out + 1, r);
}

__global__ void k_auc_final(const int64_t* excl, int64_t n, double* out) {
  const double tp = (double)excl[n];
  double auc;
  if (tp == 0 || tp == (double)n) {
    auc = 1.0;
  } else {
    double area = out[1] / (tp * ((double)n - tp));
    auc = area < 0.5 ? 1 - area : area;
  }
  out[0] = auc;
}

}  // namespace

size_t auc_sort_tmp_bytes(int64_t n) {
  size_t bytes = 0;
  WH_HIP_CHECK(rocprim::radix_sort_pairs(nullptr, bytes, (float*)nullptr, (float*)nullptr,
                                         (float*)nullptr, (float*)nullptr,
                                         (size_t)std::max<int64_t>(n, 1), 0, 32, (hipStream_t)0));
  return bytes;
}

void sort_by_score(const float* py, const float* label, int64_t n, float* py_sorted,
                   float* label_sorted, void* tmp, size_t tmp_bytes, hipStream_t s) {
  if (n <= 0) return;
  size_t bytes = tmp_bytes;
  WH_HIP_CHECK(rocprim::radix_sort_pairs(tmp, bytes, py, py_sorted, label, label_sorted,
                                         (size_t)n, 0, 32, s));
}

void auc_from_sorted(const float* label_sorted, int64_t n, double* out, int64_t* tmp_i64,
                     hipStream_t s) {
  // tmp layout: [n int32 flags (as n/2+1 int64)] [n+1 excl] [scan tmp]
  int32_t* flags = reinterpret_cast<int32_t*>(tmp_i64);
  int64_t* excl = tmp_i64 + (n / 2 + 1);
  int64_t* stmp = excl + (n + 1);
  WH_HIP_CHECK(hipMemsetAsync(out, 0, 2 * sizeof(double), s));
  if (n <= 0) {
    hipLaunchKernelGGL(k_auc_final, dim3(1), dim3(1), 0, s, excl, (int64_t)0, out);
    return;
  }
  hipLaunchKernelGGL(k_pos_flags, dim3(grid_for(n, kThreads)), dim3(kThreads), 0, s, label_sorted,
                     n, flags);
  scan_i32(flags, excl, n, stmp, s);
  hipLaunchKernelGGL(k_auc_area, dim3(grid_for(n, kThreads, 1024)), dim3(kThreads), 0, s,
                     label_sorted, excl, n, out);
  hipLaunchKernelGGL(k_auc_final, dim3(1), dim3(1), 0, s, excl, n, out);
}

}  // namespace wh
