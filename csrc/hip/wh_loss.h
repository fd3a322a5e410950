// Per-example losses and the per-launch metric sums shared by the forward
// kernels (fm.hip: localized minibatches; linear_direct.hip: the fused
// localize-free linear step).
#pragma once
#include "wh_common.h"
#include "wh_lookback.h"

namespace wh {
namespace {

// The four metric sums leave each block as stores into part[block][4]
// (summed by the last block): one same-address float64 atomic per block costs
// ~12 ns at the memory side, which at 25k blocks was a millisecond.
// The LAST block to finish (arrival ticket) sums the partials into met, so
// the forward is one launch: partials are stored write-through (agent-scope
// atomic stores) and drained before the ticket add, and read back with
// agent-scope loads (wh_lookback.h: no fences needed in this form).
// acc5: met[4] += this launch's accuracy, flipped below 0.5 (the reference
// sums per-minibatch accuracies: learn/base/binary_class_evaluation.h:40-51,
// learn/linear/loss.h:85)
__device__ __forceinline__ void block_partials(double* part, double* sh, double a, double b,
                                               double c, double d, double* met,
                                               unsigned int* ticket, int acc5 = 0) {
  __shared__ int last;
  double v[4] = {a, b, c, d};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const double r = block_sum_d(v[i], sh);
    if (threadIdx.x == 0)
      lb_store(reinterpret_cast<unsigned long long*>(part) + blockIdx.x * 4 + i,
               (unsigned long long)__double_as_longlong(r));
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = arrive_last(ticket, blockIdx.x, gridDim.x);
  }
  __syncthreads();
  if (!last) return;
  const unsigned long long* pp = reinterpret_cast<const unsigned long long*>(part);
  double tot[4];
  for (int i = 0; i < 4; ++i) {
    double s = 0;
    for (int bidx = threadIdx.x; bidx < (int)gridDim.x; bidx += blockDim.x)
      s += __longlong_as_double((long long)lb_load(pp + bidx * 4 + i));
    tot[i] = block_sum_d(s, sh);
    if (threadIdx.x == 0) met[i] += tot[i];
    __syncthreads();
  }
  if (acc5 && threadIdx.x == 0 && tot[3] > 0) {
    const double acc = tot[2] / tot[3];
    met[4] += acc > 0.5 ? acc : 1.0 - acc;
  }
}

struct LossOut {
  float objv, dual;
};

__device__ __forceinline__ float softplus(float x) {  // log(1 + exp(x)), stable
  return x > 0.f ? x + log1pf(__expf(-x)) : log1pf(__expf(x));
}

__device__ __forceinline__ LossOut eval_loss(int loss, float label, float py) {
  LossOut o;
  if (loss == 1) {  // square: 0.5 (p - y)^2
    const float d = py - label;
    o.objv = 0.5f * d * d;
    o.dual = d;
  } else if (loss == 4) {  // squared hinge: max(0, 1 - y p)^2
    const float y = label > 0.f ? 1.f : -1.f;
    const float t = fmaxf(1.f - y * py, 0.f);
    o.objv = t * t;
    o.dual = -2.f * y * t;
  } else {  // logit
    const float y = label > 0.f ? 1.f : -1.f;
    o.objv = softplus(-y * py);
    o.dual = -y / (1.f + __expf(y * py));
  }
  return o;
}

}  // namespace
}  // namespace wh
