// Generalised linear model passes over a device-resident data split: the
// objective and gradient of the L-BFGS linear learner (reference
// learn/lbfgs-linear/linear.h:74-121 Eval / CalcGrad: margin by a sparse dot
// per row, loss or pred - label, then X^T (pred - label)).
//
// The split is static for the whole run, so it is prepared ONCE for these
// passes (wormhole_amd/models/lbfgs_models.py _GLMData):
//   gcol [nnz]  int32  CSR entries' GLOBAL weight index (-1: outside the model)
//   CSC  rows   int32  the per-column occurrence lists of localize, columns
//                      in local-id order, plus
//        hb     u64    one bit per entry: set where a column starts
//        col0   int32  per 1024-entry wave: the column of its first entry
//        ucol   int32  per column: its global weight index (-1: outside)
//
// Forward (k_glm_fwd): G = 8 lanes per row, eight entries per lane issued
// together (index loads, then the weight gathers), rows grid-strided over a
// bounded grid whose blocks leave ONE fp64 partial each (loss; and the sum
// of pred - label for the bias gradient): no atomics on a single word.
//
// X^T g (k_glm_xtg): a segmented sum over a stream of entries grouped in
// RUNS (one output index per run), not one thread per column: each wave
// takes 1024 consecutive entries, gathers g at their rows (in wave order,
// transposed through LDS to 16 consecutive entries per lane), sums the runs
// inside each lane serially and joins runs that cross lanes with one
// segmented wave scan.
// Over a plain CSC (run = column) a column inside one wave is written with a
// plain store and only the (at most two) runs cut by a wave boundary are
// added atomically, so a heavy power-law column costs its entries, not a
// serial loop of one thread (the per-column chunk walk before this ran at
// ~0.3 TB/s on 156M entries). The L-BFGS plan streams the entries ROW-BLOCK
// major instead (runs = (block of 2^19 rows, column)): the g slice a block
// gathers from (2 MB) stays in L2, where the plain CSC's uniformly random row
// gathers fetched a 128-byte line per 4-byte value from the 16 MB g (1.8 ms
// per 156M entries, MALL-bound). The run sums land in stream order in S
// (coalesced), and k_glm_runs_reduce adds each column's <= 8 runs into the
// gradient (adding the runs atomically into the 64 MB gradient instead
// re-fetched its lines once per block: 1.07 ms, 13M atomics).
#include "wh_common.h"
#include "wh_kernels.h"

namespace wh {
namespace {

constexpr int kT = 256;
constexpr int kFwdG = 8, kFwdU = 8;  // lanes per row, entries per lane per pass
constexpr int kXE = 16;              // CSC entries per lane
constexpr int kXW = 64 * kXE;        // CSC entries per wave

__device__ __forceinline__ float logistic_loss(float y, float m) {
  // margin_to_loss (models/lbfgs_models.py): -log p(y | m), stable form
  const float nlp = m > 0.f ? log1pf(expf(-m)) : -m + log1pf(expf(m));
  return y * nlp + (1.f - y) * (m + nlp);
}

// MODE 0: loss partials; 1: g = pred - label into out + {loss, sum g}
// partials; 2: margins into out; 3: margins into out + loss partials (an
// objective evaluation whose margins the next gradient at the same weights
// reuses)
template <int MODE>
__global__ __launch_bounds__(kT) void k_glm_fwd(int64_t nrows, const int64_t* __restrict__ off,
                                                const int32_t* __restrict__ gcol,
                                                const float* __restrict__ val,
                                                const float* __restrict__ w,
                                                const float* __restrict__ bias, float base,
                                                const float* __restrict__ label, int loss,
                                                float* __restrict__ out,
                                                double* __restrict__ part) {
  const int lane = threadIdx.x & 63, gl = lane & (kFwdG - 1);
  const float b0 = base + (bias ? *bias : 0.f);
  const int64_t groups = (int64_t)gridDim.x * (kT / kFwdG);
  double sl = 0.0, sg = 0.0;
  for (int64_t row = ((int64_t)blockIdx.x * kT + threadIdx.x) / kFwdG; row < nrows;
       row += groups) {
    const int64_t b = off[row], e = off[row + 1];
    float acc = 0.f;
    for (int64_t j0 = b; j0 < e; j0 += kFwdG * kFwdU) {
      int32_t c[kFwdU];
#pragma unroll
      for (int u = 0; u < kFwdU; ++u) {
        const int64_t j = j0 + u * kFwdG + gl;
        c[u] = j < e ? gcol[j] : -1;
      }
      float x[kFwdU];
#pragma unroll
      for (int u = 0; u < kFwdU; ++u) x[u] = c[u] >= 0 ? w[c[u]] : 0.f;
      if (val) {
#pragma unroll
        for (int u = 0; u < kFwdU; ++u) {
          const int64_t j = j0 + u * kFwdG + gl;
          if (c[u] >= 0) x[u] *= val[j];
        }
      }
#pragma unroll
      for (int u = 0; u < kFwdU; ++u) acc += x[u];
    }
    const float m = group_sum<kFwdG>(acc) + b0;
    if (gl == 0) {
      if (MODE == 2 || MODE == 3) out[row] = m;
      if (MODE != 2) {
        const float y = label[row];
        float l;
        if (loss == 1) {
          l = logistic_loss(y, m);
        } else {
          const float d = m - y;
          l = 0.5f * d * d;
        }
        sl += (double)l;
        if (MODE == 1) {
          const float p = loss == 1 ? 1.f / (1.f + expf(-m)) : m;
          const float g = p - y;
          out[row] = g;
          sg += (double)g;
        }
      }
    }
  }
  if (MODE == 2) return;
  __shared__ double sh[2][kT / 64];
  sl = wave_sum_d(sl);
  sg = wave_sum_d(sg);
  if (lane == 0) {
    sh[0][threadIdx.x >> 6] = sl;
    sh[1][threadIdx.x >> 6] = sg;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    double s = 0.0;
    for (int i = 0; i < kT / 64; ++i) s += sh[threadIdx.x][i];
    part[2 * (int64_t)blockIdx.x + threadIdx.x] = s;
  }
}

// g = pred - label from stored margins + {loss, sum g} partials (the
// gradient pass at weights whose margins an evaluation just computed)
__global__ __launch_bounds__(kT) void k_glm_from_margin(int64_t nrows,
                                                        const float* __restrict__ margin,
                                                        const float* __restrict__ label, int loss,
                                                        float* __restrict__ g_out,
                                                        double* __restrict__ part) {
  double sl = 0.0, sg = 0.0;
  for (int64_t row = (int64_t)blockIdx.x * kT + threadIdx.x; row < nrows;
       row += (int64_t)gridDim.x * kT) {
    const float m = margin[row], y = label[row];
    float l, p;
    if (loss == 1) {
      l = logistic_loss(y, m);
      p = 1.f / (1.f + expf(-m));
    } else {
      const float d = m - y;
      l = 0.5f * d * d;
      p = m;
    }
    const float g = p - y;
    g_out[row] = g;
    sl += (double)l;
    sg += (double)g;
  }
  __shared__ double sh[2][kT / 64];
  sl = wave_sum_d(sl);
  sg = wave_sum_d(sg);
  if ((threadIdx.x & 63) == 0) {
    sh[0][threadIdx.x >> 6] = sl;
    sh[1][threadIdx.x >> 6] = sg;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    double s = 0.0;
    for (int i = 0; i < kT / 64; ++i) s += sh[threadIdx.x][i];
    part[2 * (int64_t)blockIdx.x + threadIdx.x] = s;
  }
}

// out[v] = sum over blocks of part[b * stride + v], v < nv (one block per
// value, fixed order: deterministic)
__global__ __launch_bounds__(kT) void k_sum_parts(const double* __restrict__ part, int nblk,
                                                  int stride, double* __restrict__ out) {
  __shared__ double sh[kT / 64];
  const int v = blockIdx.x;
  double s = 0.0;
  for (int b = threadIdx.x; b < nblk; b += kT) s += part[(int64_t)b * stride + v];
  s = block_sum_d(s, sh);
  if (threadIdx.x == 0) out[v] = s;
}

__device__ __forceinline__ void xtg_emit(const int32_t* ucol, int col, float v, bool atomic,
                                         float* grad) {
  const int32_t gi = ucol ? ucol[col] : col;
  if (gi < 0) return;
  if (atomic) atomicAdd(grad + gi, v);
  else grad[gi] = v;
}

__global__ __launch_bounds__(kT) void k_glm_xtg(int64_t nnz, const int32_t* __restrict__ crow,
                                                const float* __restrict__ cval,
                                                const uint64_t* __restrict__ hb,
                                                const int32_t* __restrict__ col0w,
                                                const int32_t* __restrict__ ucol,
                                                const float* __restrict__ g,
                                                float* __restrict__ grad, int all_atomic) {
  const int lane = threadIdx.x & 63;
  const int64_t wv = ((int64_t)blockIdx.x * kT + threadIdx.x) >> 6;
  const int64_t wbase = wv * kXW;
  if (wbase >= nnz) return;  // (uniform per wave)
  const bool full = wbase + kXW <= nnz;
  // Gathers in WAVE order (instruction k reads entries wbase + 64 k + lane):
  // a hot column's consecutive entries are rows a few apart, so the lanes of
  // one gather share g's cache lines (each distinct line is one L2 request;
  // lane-contiguous gathers put every lane on its own line). The values are
  // then transposed through LDS to 16 consecutive entries per lane.
  __shared__ float xs[kT / 64][kXW + kXW / 16];
  float* xw = xs[threadIdx.x >> 6];
  {
    int32_t r[kXE];
#pragma unroll
    for (int k = 0; k < kXE; ++k) {
      const int64_t p = wbase + k * 64 + lane;
      r[k] = (full || p < nnz) ? crow[p] : -1;
    }
    float v[kXE];
#pragma unroll
    for (int k = 0; k < kXE; ++k) v[k] = r[k] >= 0 ? g[r[k]] : 0.f;
    if (cval) {
#pragma unroll
      for (int k = 0; k < kXE; ++k)
        if (r[k] >= 0) v[k] *= cval[wbase + k * 64 + lane];
    }
#pragma unroll
    for (int k = 0; k < kXE; ++k) {
      const int i = k * 64 + lane;
      xw[i + (i >> 4)] = v[k];  // (one pad word per 16: conflict-free reads below)
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  float x[kXE];
#pragma unroll
  for (int k = 0; k < kXE; ++k) x[k] = xw[lane * (kXE + 1) + k];
  // this lane's 16 column-start bits (entries past nnz carry none)
  const uint32_t bits =
      (uint32_t)(hb[(wbase >> 6) + (lane >> 2)] >> ((lane & 3) * kXE)) & 0xffffu;
  // column starts after the wave's first entry advance the column index
  const uint32_t cbits = lane == 0 ? (bits & ~1u) : bits;
  int ex_c = __popc(cbits), ex_a = __popc(bits);
  const int own_c = ex_c, own_a = ex_a;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {  // inclusive scans, then exclusive
    const int tc = __shfl_up(ex_c, o, 64), ta = __shfl_up(ex_a, o, 64);
    if (lane >= o) {
      ex_c += tc;
      ex_a += ta;
    }
  }
  const int tot_c = __shfl(ex_c, 63, 64), tot_a = __shfl(ex_a, 63, 64);
  ex_c -= own_c;
  ex_a -= own_a;
  const int c0 = col0w[wv];
  // runs inside the lane: lead (before the first start) / complete runs
  // (stored) / tail (open at the lane's end)
  int cur = c0 + ex_c;
  const int lead_col = cur;
  float acc = 0.f, lead = 0.f;
  bool has = false;
#pragma unroll
  for (int k = 0; k < kXE; ++k) {
    if ((bits >> k) & 1u) {
      if (has) xtg_emit(ucol, cur, acc, all_atomic, grad);
      else lead = acc;
      has = true;
      acc = 0.f;
      if ((cbits >> k) & 1u) ++cur;
    }
    acc += x[k];
  }
  if (!has) lead = acc;  // no start in this lane: all of it continues a run
  // segmented inclusive scan over lanes of (has, has ? tail : lead)
  float s = has ? acc : lead;
  bool f = has;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float ts = __shfl_up(s, o, 64);
    const int tf = __shfl_up((int)f, o, 64);
    if (lane >= o) {
      if (!f) s += ts;
      f = f || tf;
    }
  }
  const float prev = __shfl_up(s, 1, 64);
  // the run that ends at this lane's first start (lane 0 starting the wave
  // with a column start: nothing before it here)
  if (has && !(lane == 0 && (bits & 1u))) {
    const float v = (lane > 0 ? prev : 0.f) + lead;
    xtg_emit(ucol, lead_col, v, all_atomic || ex_a == 0, grad);  // started before this wave
  }
  if (lane == 63) {  // the run open at the wave's end
    const int64_t nb = (wbase >> 6) + 16;
    const bool ends = !full || wbase + kXW >= nnz || (hb[nb] & 1ull);
    xtg_emit(ucol, c0 + tot_c, s, all_atomic || !(ends && tot_a > 0), grad);
  }
}

// column starts: hb bit csc_off[u] for every column u
__global__ __launch_bounds__(kT) void k_glm_heads(const int64_t* __restrict__ csc_off, int64_t U,
                                                  unsigned long long* __restrict__ hb) {
  const int64_t u = (int64_t)blockIdx.x * kT + threadIdx.x;
  if (u >= U) return;
  const int64_t p = csc_off[u];
  if (csc_off[u + 1] > p) atomicOr(hb + (p >> 6), 1ull << (p & 63));
}

// grad[cgid[c]] = sum of the run sums S over column c's runs (rlist
// [coff[c], coff[c + 1]), in block order: deterministic)
__global__ __launch_bounds__(kT) void k_glm_runs_reduce(int64_t ncol,
                                                        const int64_t* __restrict__ coff,
                                                        const int32_t* __restrict__ rlist,
                                                        const float* __restrict__ S,
                                                        const int32_t* __restrict__ cgid,
                                                        float* __restrict__ grad) {
  const int64_t c = (int64_t)blockIdx.x * kT + threadIdx.x;
  if (c >= ncol) return;
  const int64_t b = coff[c], e = coff[c + 1];
  float v = 0.f;
  for (int64_t k = b; k < e; ++k) v += S[rlist[k]];
  grad[cgid[c]] = v;
}

}  // namespace

void sum_parts(const double* part, int nblk, int nv, double* out, hipStream_t s, int stride) {
  if (nv > 0)
    hipLaunchKernelGGL(k_sum_parts, dim3(nv), dim3(kT), 0, s, part, nblk, stride > 0 ? stride : nv,
                       out);
}

int64_t glm_fwd_blocks(int64_t nrows) {
  return grid_for(nrows * kFwdG, kT, 2048);
}

void glm_fwd(int mode, int64_t nrows, const int64_t* off, const int32_t* gcol, const float* val,
             const float* w, const float* bias, float base, const float* label, int loss,
             float* out, double* part, double* sums, hipStream_t s) {
  if (nrows <= 0) {
    if (mode != 2) WH_HIP_CHECK(hipMemsetAsync(sums, 0, 2 * sizeof(double), s));
    return;
  }
  const int nb = (int)glm_fwd_blocks(nrows);
  if (mode == 0)
    hipLaunchKernelGGL(k_glm_fwd<0>, dim3(nb), dim3(kT), 0, s, nrows, off, gcol, val, w, bias,
                       base, label, loss, out, part);
  else if (mode == 1)
    hipLaunchKernelGGL(k_glm_fwd<1>, dim3(nb), dim3(kT), 0, s, nrows, off, gcol, val, w, bias,
                       base, label, loss, out, part);
  else if (mode == 2)
    hipLaunchKernelGGL(k_glm_fwd<2>, dim3(nb), dim3(kT), 0, s, nrows, off, gcol, val, w, bias,
                       base, label, loss, out, part);
  else
    hipLaunchKernelGGL(k_glm_fwd<3>, dim3(nb), dim3(kT), 0, s, nrows, off, gcol, val, w, bias,
                       base, label, loss, out, part);
  if (mode != 2) sum_parts(part, nb, 2, sums, s);
}

void glm_runs_reduce(int64_t ncol, const int64_t* coff, const int32_t* rlist, const float* S,
                     const int32_t* cgid, float* grad, hipStream_t s) {
  if (ncol > 0)
    hipLaunchKernelGGL(k_glm_runs_reduce, dim3(grid_for(ncol, kT)), dim3(kT), 0, s, ncol, coff,
                       rlist, S, cgid, grad);
}

void glm_grad_from_margin(int64_t nrows, const float* margin, const float* label, int loss,
                          float* g, double* part, double* sums, hipStream_t s) {
  if (nrows <= 0) {
    WH_HIP_CHECK(hipMemsetAsync(sums, 0, 2 * sizeof(double), s));
    return;
  }
  const int nb = (int)glm_fwd_blocks(nrows);
  hipLaunchKernelGGL(k_glm_from_margin, dim3(nb), dim3(kT), 0, s, nrows, margin, label, loss, g,
                     part);
  sum_parts(part, nb, 2, sums, s);
}

int64_t glm_xtg_waves(int64_t nnz) { return (nnz + kXW - 1) / kXW; }
int64_t glm_heads_words(int64_t nnz) { return glm_xtg_waves(nnz) * 16 + 16; }

void glm_heads(const int64_t* csc_off, int64_t U, uint64_t* hb, int64_t words, hipStream_t s) {
  WH_HIP_CHECK(hipMemsetAsync(hb, 0, words * sizeof(uint64_t), s));
  if (U > 0)
    hipLaunchKernelGGL(k_glm_heads, dim3(grid_for(U, kT)), dim3(kT), 0, s, csc_off, U,
                       reinterpret_cast<unsigned long long*>(hb));
}

void glm_xtg(int64_t nnz, const int32_t* crow, const float* cval, const uint64_t* hb,
             const int32_t* col0w, const int32_t* ucol, const float* g, float* grad,
             int all_atomic, hipStream_t s) {
  if (nnz <= 0) return;
  const int64_t waves = glm_xtg_waves(nnz);
  hipLaunchKernelGGL(k_glm_xtg, dim3((unsigned)((waves + 3) / 4)), dim3(kT), 0, s, nnz, crow,
                     cval, hb, col0w, ucol, g, grad, all_atomic);
}

}  // namespace wh
