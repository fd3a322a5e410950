// Histogram GBDT kernels (K21 in SURVEY §2.5; replaces the external xgboost
// learner's hist tree builder):
//   gbdt_bin       value -> quantile bin (uint8, 255 = missing) by binary
//                  search in the feature's cut points
//   gbdt_hist      per (node, feature-group, row-chunk) block: LDS-privatised
//                  fp32 (g, h) histograms (ds_add_f32), flushed once per block
//                  into the node's fp64 histogram with device-scope atomics
//   gbdt_goleft / gbdt_scatter   stable per-node row partition after a split
//   gbdt_leaf_add  margin += leaf value for the rows of every leaf segment
//   gbdt_predict   one lane per row walks a tree on raw values (NaN = missing)
#include "wh_common.h"
#include "wh_kernels.h"

namespace wh {
namespace {

constexpr int kMissing = 255;

__global__ void k_bin(const float* __restrict__ X, int64_t n, int f, const float* __restrict__ cuts,
                      const int32_t* __restrict__ cut_off, uint8_t* __restrict__ B) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * f) return;
  const int j = (int)(t % f);
  const float v = X[t];
  uint8_t b = kMissing;
  if (!isnan(v)) {
    // bin = #cuts <= v  (so v < cuts[b] <=> bin <= b); the last cut is +inf-like
    int lo = cut_off[j], hi = cut_off[j + 1];
    const int base = lo;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (cuts[mid] <= v) lo = mid + 1;
      else hi = mid;
    }
    int bin = lo - base;
    const int nb = cut_off[j + 1] - base;
    if (bin >= nb) bin = nb - 1;
    b = (uint8_t)bin;
  }
  B[t] = b;
}

// Task = (node slot, feature group, row chunk). LDS holds fg x nbin (g, h) fp32.
struct HistTask {
  int32_t node;   // output histogram slot
  int32_t fbeg;   // first feature of the group
  int32_t fcnt;   // features in the group
  int32_t rbeg;   // [rbeg, rend) into ridx
  int32_t rend;
};

__global__ __launch_bounds__(256) void k_hist(const uint8_t* __restrict__ B, int f, int nbin,
                                              const int32_t* __restrict__ ridx,
                                              const float2* __restrict__ gpair,
                                              const HistTask* __restrict__ tasks,
                                              double* __restrict__ hist) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const HistTask tk = tasks[blockIdx.x];
  const int nl = tk.fcnt * nbin;
  for (int i = threadIdx.x; i < 2 * nl; i += blockDim.x) lds[i] = 0.f;
  __syncthreads();
  // threads sweep (row, feature) pairs of the chunk: consecutive lanes read
  // consecutive feature bytes of a row
  const int64_t pairs = (int64_t)(tk.rend - tk.rbeg) * tk.fcnt;
  for (int64_t p = threadIdx.x; p < pairs; p += blockDim.x) {
    const int r = tk.rbeg + (int)(p / tk.fcnt);
    const int fj = (int)(p % tk.fcnt);
    const int row = ridx[r];
    const int b = B[(int64_t)row * f + tk.fbeg + fj];
    if (b != kMissing) {
      const float2 gh = gpair[row];
      atomicAdd(&lds[2 * (fj * nbin + b)], gh.x);
      atomicAdd(&lds[2 * (fj * nbin + b) + 1], gh.y);
    }
  }
  __syncthreads();
  double* out = hist + ((int64_t)tk.node * f + tk.fbeg) * nbin * 2;
  for (int i = threadIdx.x; i < 2 * nl; i += blockDim.x) {
    const float v = lds[i];
    if (v != 0.f) atomicAdd(out + i, (double)v);
  }
}

__global__ void k_goleft(const uint8_t* __restrict__ B, int f, const int32_t* __restrict__ ridx,
                         int64_t nrows_seg, const int32_t* __restrict__ pos_node,
                         const int32_t* __restrict__ node_feat, const int32_t* __restrict__ node_bin,
                         const uint8_t* __restrict__ node_defl, int32_t* __restrict__ left) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nrows_seg) return;
  const int nd = pos_node[i];
  int l = 0;
  const int feat = nd >= 0 ? node_feat[nd] : -1;
  if (feat >= 0) {
    const int b = B[(int64_t)ridx[i] * f + feat];
    l = (b == kMissing) ? (int)node_defl[nd] : (b <= node_bin[nd] ? 1 : 0);
  }
  left[i] = l;
}

__global__ void k_scatter(const int32_t* __restrict__ ridx, int64_t n,
                          const int32_t* __restrict__ pos_node, const int32_t* __restrict__ node_feat,
                          const int32_t* __restrict__ seg_beg, const int32_t* __restrict__ nleft,
                          const int32_t* __restrict__ left, const int64_t* __restrict__ lscan,
                          int32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int nd = pos_node[i];
  if (nd < 0 || node_feat[nd] < 0) {
    out[i] = ridx[i];
    return;
  }
  const int64_t b = seg_beg[nd];
  const int64_t lbefore = lscan[i] - lscan[b];
  const int64_t dst = left[i] ? b + lbefore : b + nleft[nd] + ((i - b) - lbefore);
  out[dst] = ridx[i];
}

__global__ void k_leaf_add(const int32_t* __restrict__ ridx, int64_t n,
                           const int32_t* __restrict__ pos_node, const float* __restrict__ leaf,
                           float* __restrict__ margin) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int nd = pos_node[i];
  if (nd >= 0) margin[ridx[i]] += leaf[nd];
}

__global__ void k_predict(const float* __restrict__ X, int64_t n, int f,
                          const int32_t* __restrict__ feat, const float* __restrict__ thr,
                          const int32_t* __restrict__ left, const int32_t* __restrict__ right,
                          const uint8_t* __restrict__ defl, const float* __restrict__ leaf,
                          float* __restrict__ margin) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int nd = 0;
  while (feat[nd] >= 0) {
    const float v = X[i * f + feat[nd]];
    const bool go_left = isnan(v) ? (defl[nd] != 0) : (v < thr[nd]);
    nd = go_left ? left[nd] : right[nd];
  }
  margin[i] += leaf[nd];
}

}  // namespace

void gbdt_bin(const float* X, int64_t n, int f, const float* cuts, const int32_t* cut_off,
              uint8_t* B, hipStream_t s) {
  if (n * f <= 0) return;
  hipLaunchKernelGGL(k_bin, dim3(grid_for(n * f, 256)), dim3(256), 0, s, X, n, f, cuts, cut_off, B);
}

size_t gbdt_hist_lds(int fcnt, int nbin) { return (size_t)fcnt * nbin * 2 * sizeof(float); }

void gbdt_hist(const uint8_t* B, int f, int nbin, const int32_t* ridx, const float* gpair,
               const int32_t* tasks, int ntask, int max_fcnt, double* hist, hipStream_t s) {
  if (ntask <= 0) return;
  hipLaunchKernelGGL(k_hist, dim3(ntask), dim3(256), gbdt_hist_lds(max_fcnt, nbin), s, B, f, nbin,
                     ridx, reinterpret_cast<const float2*>(gpair),
                     reinterpret_cast<const HistTask*>(tasks), hist);
}

void gbdt_goleft(const uint8_t* B, int f, const int32_t* ridx, int64_t n, const int32_t* pos_node,
                 const int32_t* node_feat, const int32_t* node_bin, const uint8_t* node_defl,
                 int32_t* left, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_goleft, dim3(grid_for(n, 256)), dim3(256), 0, s, B, f, ridx, n, pos_node,
                     node_feat, node_bin, node_defl, left);
}

void gbdt_scatter(const int32_t* ridx, int64_t n, const int32_t* pos_node, const int32_t* node_feat,
                  const int32_t* seg_beg, const int32_t* nleft, const int32_t* left,
                  const int64_t* lscan, int32_t* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_scatter, dim3(grid_for(n, 256)), dim3(256), 0, s, ridx, n, pos_node,
                     node_feat, seg_beg, nleft, left, lscan, out);
}

void gbdt_leaf_add(const int32_t* ridx, int64_t n, const int32_t* pos_node, const float* leaf,
                   float* margin, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_leaf_add, dim3(grid_for(n, 256)), dim3(256), 0, s, ridx, n, pos_node, leaf,
                     margin);
}

void gbdt_predict(const float* X, int64_t n, int f, const int32_t* feat, const float* thr,
                  const int32_t* left, const int32_t* right, const uint8_t* defl,
                  const float* leaf, float* margin, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_predict, dim3(grid_for(n, 256)), dim3(256), 0, s, X, n, f, feat, thr, left,
                     right, defl, leaf, margin);
}

}  // namespace wh
