// Histogram GBDT kernels (K21 in SURVEY §2.5; replaces the external xgboost
// learner's hist tree builder):
//   gbdt_bin       value -> quantile bin (uint8, 255 = missing) by binary
//                  search in the feature's cut points
//   gbdt_hist      per (node, feature-group, row-chunk) block: LDS-privatised
//                  fp32 (g, h) histograms (ds_add_f32) stored as per-block
//                  partials, then summed per (node, group) in fp64
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

// Partial-sum reduction of the tasks of one (slot, feature group):
// tasks t0, t0 + tstride, ... (nt of them).
struct HistReduce {
  int32_t node;
  int32_t fbeg;
  int32_t fcnt;
  int32_t t0;
  int32_t nt;
  int32_t tstride;
};

constexpr int kHistThreads = 1024;  // 2 blocks (2 x <= 64 KB LDS) fill a CU's 32 wave slots

__device__ __forceinline__ void hist_add(float* lds, int nbin, int fj, int b, float2 gh) {
  if (b != kMissing) {
    atomicAdd(&lds[2 * (fj * nbin + b)], gh.x);
    atomicAdd(&lds[2 * (fj * nbin + b) + 1], gh.y);
  }
}

// LDS-privatised histogram of one task, written (not atomically added) to the
// task's fp32 partial slice; k_hist_reduce sums the slices in fp64.  Replacing
// the per-block fp64 atomic flush (14 K memory-side atomics per block) by
// plain coalesced stores is what makes small row chunks -- and so a full grid
// at every tree level -- affordable.
//
// DW: the group's bytes of a row are 4-aligned (f % 4 == 0, fbeg % 4 == 0,
// fcnt % 4 == 0): D = fcnt / 4 lanes share a row and each loads one dword
// (4 bins), so a wave fetches floor(64 / D) rows with one load instruction
// instead of one byte per lane per feature.  Four row batches are loaded
// before any LDS atomic is issued, keeping 4 dependent gathers in flight per
// wave.  Otherwise one thread per row walks the group's bytes.
template <bool DW>
__global__ __launch_bounds__(kHistThreads) void k_hist(const uint8_t* __restrict__ B, int f,
                                                       int nbin, const int32_t* __restrict__ ridx,
                                                       const float2* __restrict__ gpair,
                                                       const HistTask* __restrict__ tasks,
                                                       float* __restrict__ part, int64_t pstride) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const HistTask tk = tasks[blockIdx.x];
  const int nl2 = 2 * tk.fcnt * nbin;
  for (int i = threadIdx.x; i < nl2; i += blockDim.x) lds[i] = 0.f;
  __syncthreads();
  const int nrow = tk.rend - tk.rbeg;
  const int32_t* rid = ridx + tk.rbeg;
  if (DW) {
    constexpr int U = 4;
    const int D = tk.fcnt >> 2;
    const int R = 64 / D;  // rows per wave batch
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int ri = lane / D, dj = lane - ri * D;
    const bool act = ri < R;
    const uint8_t* Bg = B + tk.fbeg + 4 * dj;
    for (int base = wave * R; base < nrow; base += nw * R * U) {
      uint32_t word[U];
      float2 g[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int r = base + u * nw * R + ri;
        const bool ok = act && r < nrow;
        const int row = ok ? rid[r] : 0;
        word[u] = ok ? *reinterpret_cast<const uint32_t*>(Bg + (int64_t)row * f) : 0xffffffffu;
        g[u] = ok ? gpair[row] : make_float2(0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int c = 0; c < 4; ++c) hist_add(lds, nbin, 4 * dj + c, (word[u] >> (8 * c)) & 255, g[u]);
    }
  } else {
    const int lane = threadIdx.x & 63;
    for (int r = threadIdx.x; r < nrow; r += blockDim.x) {
      const int row = rid[r];
      const float2 gh = gpair[row];
      const uint8_t* brow = B + (int64_t)row * f + tk.fbeg;
      int fj = lane % tk.fcnt;  // lane-rotated feature order spreads the atomics
      for (int q = 0; q < tk.fcnt; ++q) {
        hist_add(lds, nbin, fj, brow[fj], gh);
        fj = fj + 1 == tk.fcnt ? 0 : fj + 1;
      }
    }
  }
  __syncthreads();
  float* out = part + (int64_t)blockIdx.x * pstride;
  for (int i = threadIdx.x; i < nl2; i += blockDim.x) out[i] = lds[i];
}

__global__ __launch_bounds__(256) void k_hist_reduce(const float* __restrict__ part,
                                                     int64_t pstride,
                                                     const HistReduce* __restrict__ red, int f,
                                                     int nbin, double* __restrict__ hist) {
  const HistReduce rd = red[blockIdx.y];
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= 2 * rd.fcnt * nbin) return;
  const float* p = part + (int64_t)rd.t0 * pstride + e;
  double acc = 0.0;
  for (int k = 0; k < rd.nt; ++k) acc += (double)p[(int64_t)k * rd.tstride * pstride];
  hist[((int64_t)rd.node * f + rd.fbeg) * nbin * 2 + e] = acc;
}

// out[i] = node of the segment containing position i; segments sorted by
// begin and tiling [0, n) (finished-leaf gaps carry node -1)
__global__ __launch_bounds__(256) void k_seg_fill(const int32_t* __restrict__ beg,
                                                  const int32_t* __restrict__ node, int nseg,
                                                  int64_t n, int32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int lo = 0, hi = nseg - 1;  // last segment with beg <= i
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (beg[mid] <= i) lo = mid;
    else hi = mid - 1;
  }
  out[i] = node[lo];
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

int64_t gbdt_hist_pstride(int max_fcnt, int nbin) { return ((int64_t)2 * max_fcnt * nbin + 63) & ~63; }

void gbdt_hist(const uint8_t* B, int f, int nbin, const int32_t* ridx, const float* gpair,
               const int32_t* tasks, int ntask, const int32_t* red, int nred, int max_fcnt,
               bool dword_rows, float* part, double* hist, hipStream_t s) {
  if (ntask <= 0) return;
  const int64_t ps = gbdt_hist_pstride(max_fcnt, nbin);
  const size_t lds = gbdt_hist_lds(max_fcnt, nbin);
  const auto* tk = reinterpret_cast<const HistTask*>(tasks);
  const auto* gp = reinterpret_cast<const float2*>(gpair);
  if (dword_rows)
    hipLaunchKernelGGL(k_hist<true>, dim3(ntask), dim3(kHistThreads), lds, s, B, f, nbin, ridx, gp,
                       tk, part, ps);
  else
    hipLaunchKernelGGL(k_hist<false>, dim3(ntask), dim3(kHistThreads), lds, s, B, f, nbin, ridx,
                       gp, tk, part, ps);
  if (nred > 0)
    hipLaunchKernelGGL(k_hist_reduce, dim3((unsigned)((2 * max_fcnt * nbin + 255) / 256), nred),
                       dim3(256), 0, s, part, ps, reinterpret_cast<const HistReduce*>(red), f,
                       nbin, hist);
}

void gbdt_seg_fill(const int32_t* beg, const int32_t* node, int nseg, int64_t n, int32_t* out,
                   hipStream_t s) {
  if (n <= 0 || nseg <= 0) return;
  hipLaunchKernelGGL(k_seg_fill, dim3(grid_for(n, 256)), dim3(256), 0, s, beg, node, nseg, n, out);
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
