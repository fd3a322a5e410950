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
#include <algorithm>
#include <cstdlib>

#include "wh_common.h"
#include "wh_kernels.h"
#include "wh_lookback.h"

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
    b = nb > 0 ? (uint8_t)bin : (uint8_t)kMissing;  // (a feature without cuts)
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

constexpr int kHistThreads = 1024;
constexpr int kHistLdsMax = 160 * 1024;  // one block per CU (<= 160 KB LDS) = 16 waves

// Histograms accumulate in 64-bit fixed point: ds_add_f32 on gfx950 runs ~20x
// slower than ds_add_u32 / ~8x slower than ds_add_u64 (tools/microbench/
// hist_bench.hip: 11M x 28 rows in 3.04 ms with f32 LDS atomics, 0.43 ms with
// u64), and integer sums are exact, so a node's histogram no longer depends
// on block scheduling.  qscale = {2^eg, 2^eh} is chosen by the caller so that
// |sum of a node| * scale < 2^62 for every node (power-of-two: the scaling of
// the fp32 gradient is exact; only its bits below 2^-e are rounded away).
__device__ __forceinline__ void hist_add(unsigned long long* lds, int nbin, int fj, int b,
                                         long long qg, long long qh) {
  if (b != kMissing) {
    atomicAdd(&lds[2 * (fj * nbin + b)], (unsigned long long)qg);
    atomicAdd(&lds[2 * (fj * nbin + b) + 1], (unsigned long long)qh);
  }
}

// 32-bit variant (W32): the caller picks the scale so that |q| <= 2^31 / R
// for every row (R = qscale[2] rows); a block sums at most R rows in int32
// LDS, adds them into its int64 partial and starts again.  ds_add_u32 issues
// ~2x the rate of ds_add_u64 and the histogram takes half the LDS.  Rows are
// rounded with the same scale in every block, so the sums stay exact integers:
// any chunking, grower or the CSR kernel gives bit-identical histograms.
__device__ __forceinline__ void hist_add32(unsigned* lds, int nbin, int fj, int b, int qg,
                                           int qh) {
  if (b != kMissing) {
    atomicAdd(&lds[2 * (fj * nbin + b)], (unsigned)qg);
    atomicAdd(&lds[2 * (fj * nbin + b) + 1], (unsigned)qh);
  }
}

// LDS-privatised histogram of one task, written (not atomically added) to the
// task's int64 partial slice; k_hist_reduce sums the slices per (node, group).
// Plain coalesced stores instead of a per-block atomic flush make small row
// chunks -- and so a full grid at every tree level -- affordable.
//
// DW: the group's bytes of a row are 4-aligned (f % 4 == 0, fbeg % 4 == 0,
// fcnt % 4 == 0): D = fcnt / 4 lanes share a row and each loads one dword
// (4 bins), so a wave fetches floor(64 / D) rows with one load instruction
// instead of one byte per lane per feature.  Four row batches are loaded
// before any LDS atomic is issued, keeping 4 dependent gathers in flight per
// wave.  Otherwise one thread per row walks the group's bytes.
//
// W32: qscale = {2^eg, 2^eh, R}: int32 LDS sums over sub-batches of <= R rows.
template <bool DW, bool W32>
__global__ __launch_bounds__(kHistThreads) void k_hist(const uint8_t* __restrict__ B, int f,
                                                       int nbin, const int32_t* __restrict__ ridx,
                                                       const float2* __restrict__ gpair,
                                                       const float* __restrict__ qscale,
                                                       const HistTask* __restrict__ tasks,
                                                       long long* __restrict__ part,
                                                       int64_t pstride,
                                                       const int32_t* __restrict__ dseg,
                                                       const int32_t* __restrict__ ntask_dev) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long lds64[];
  // (a device-built task list: the grid is its upper bound)
  if (ntask_dev && (int)blockIdx.x >= *ntask_dev) return;
  HistTask tk = tasks[blockIdx.x];
  if (dseg) {  // dynamic rows: {chunk index, chunk rows} of the slot's device segment
    const int32_t sb = dseg[2 * tk.node], se = dseg[2 * tk.node + 1];
    const int32_t rb = sb + tk.rbeg * tk.rend;
    if (rb >= se) return;  // past the segment: the reduce skips this task
    tk.rend = rb + tk.rend < se ? rb + tk.rend : se;
    tk.rbeg = rb;
  }
  const float sg = qscale[0], sh = qscale[1];
  const int nl2 = 2 * tk.fcnt * nbin;
  const int nall = tk.rend - tk.rbeg;
  unsigned* lds32 = reinterpret_cast<unsigned*>(lds64);
  const int R = W32 ? max(1, (int)qscale[2]) : max(1, nall);
  long long* out = part + (int64_t)blockIdx.x * pstride;
  int r0 = 0;
  do {  // (one pass unless W32 and the task holds more than R rows)
    if (W32)
      for (int i = threadIdx.x; i < nl2; i += blockDim.x) lds32[i] = 0u;
    else
      for (int i = threadIdx.x; i < nl2; i += blockDim.x) lds64[i] = 0ull;
    __syncthreads();
    const int nrow = min(R, nall - r0);
    const int32_t* rid = ridx + tk.rbeg + r0;
    if (DW) {
      constexpr int U = 4;
      const int D = tk.fcnt >> 2;
      const int RW = 64 / D;  // rows per wave batch
      const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
      const int ri = lane / D, dj = lane - ri * D;
      const bool act = ri < RW;
      const uint8_t* Bg = B + tk.fbeg + 4 * dj;
      for (int base = wave * RW; base < nrow; base += nw * RW * U) {
        uint32_t word[U];
        float2 g[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int r = base + u * nw * RW + ri;
          const bool ok = act && r < nrow;
          const int row = ok ? rid[r] : 0;
          word[u] = ok ? *reinterpret_cast<const uint32_t*>(Bg + (int64_t)row * f) : 0xffffffffu;
          g[u] = ok ? gpair[row] : make_float2(0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (W32) {
            const int qg = __float2int_rn(g[u].x * sg), qh = __float2int_rn(g[u].y * sh);
#pragma unroll
            for (int c = 0; c < 4; ++c)
              hist_add32(lds32, nbin, 4 * dj + c, (word[u] >> (8 * c)) & 255, qg, qh);
          } else {
            const long long qg = __float2ll_rn(g[u].x * sg), qh = __float2ll_rn(g[u].y * sh);
#pragma unroll
            for (int c = 0; c < 4; ++c)
              hist_add(lds64, nbin, 4 * dj + c, (word[u] >> (8 * c)) & 255, qg, qh);
          }
        }
      }
    } else {
      const int lane = threadIdx.x & 63;
      for (int r = threadIdx.x; r < nrow; r += blockDim.x) {
        const int row = rid[r];
        const float2 gh = gpair[row];
        const uint8_t* brow = B + (int64_t)row * f + tk.fbeg;
        int fj = lane % tk.fcnt;  // lane-rotated feature order spreads the atomics
        if (W32) {
          const int qg = __float2int_rn(gh.x * sg), qh = __float2int_rn(gh.y * sh);
          for (int q = 0; q < tk.fcnt; ++q) {
            hist_add32(lds32, nbin, fj, brow[fj], qg, qh);
            fj = fj + 1 == tk.fcnt ? 0 : fj + 1;
          }
        } else {
          const long long qg = __float2ll_rn(gh.x * sg), qh = __float2ll_rn(gh.y * sh);
          for (int q = 0; q < tk.fcnt; ++q) {
            hist_add(lds64, nbin, fj, brow[fj], qg, qh);
            fj = fj + 1 == tk.fcnt ? 0 : fj + 1;
          }
        }
      }
    }
    __syncthreads();
    // each thread owns the same elements in every pass: no race on out
    for (int i = threadIdx.x; i < nl2; i += blockDim.x) {
      const long long v = W32 ? (long long)(int)lds32[i] : (long long)lds64[i];
      out[i] = r0 == 0 ? v : out[i] + v;
    }
    __syncthreads();  // before the next pass clears the LDS
    r0 += R;
  } while (r0 < nall);
}

// One block = 64 consecutive elements x 16 task slices: thread (e, k) sums
// tasks k, k + 16, ... of its element (each 64-element row read is 512 B
// contiguous), then the 16 slices are combined in LDS.
constexpr int kRedE = 64, kRedK = 16;
__global__ __launch_bounds__(kRedE * kRedK) void k_hist_reduce(
    const long long* __restrict__ part, int64_t pstride, const HistReduce* __restrict__ red, int f,
    int nbin, const float* __restrict__ qscale, double* __restrict__ hist,
    const int32_t* __restrict__ dseg, int chunk, const double* __restrict__ sib_hf,
    const int32_t* __restrict__ sib_sp, const int32_t* __restrict__ sib_par) {
  __shared__ unsigned long long acc_s[kRedK][kRedE];
  HistReduce rd = red[blockIdx.y];
  if (dseg) {  // only the chunks that cover the slot's device segment wrote
    const int64_t len = (int64_t)dseg[2 * rd.node + 1] - dseg[2 * rd.node];
    const int64_t live = len > 0 ? (len + chunk - 1) / chunk : 0;
    rd.nt = live < rd.nt ? (int32_t)live : rd.nt;
  }
  const int ei = threadIdx.x % kRedE, kj = threadIdx.x / kRedE;
  const int e = blockIdx.x * kRedE + ei;
  const int nl2 = 2 * rd.fcnt * nbin;
  unsigned long long acc = 0;  // two's-complement sum: exact while |sum| < 2^63
  if (e < nl2) {
    const long long* p = part + (int64_t)rd.t0 * pstride + e;
    for (int k = kj; k < rd.nt; k += kRedK) acc += (unsigned long long)p[(int64_t)k * rd.tstride * pstride];
  }
  acc_s[kj][ei] = acc;
  __syncthreads();
  if (kj == 0 && e < nl2) {
#pragma unroll
    for (int k = 1; k < kRedK; ++k) acc += acc_s[k][ei];
    const double v = (double)(long long)acc / (double)qscale[e & 1];
    if (sib_hf) {  // fused sibling step: both children of split rd.node
      const int64_t per = (int64_t)f * nbin * 2, ge = (int64_t)rd.fbeg * nbin * 2 + e;
      const int k = rd.node;
      const double other = sib_hf[(int64_t)sib_par[k] * per + ge] - v;
      const bool bl = sib_sp[4 * k + 3] != 0;
      hist[(int64_t)(2 * k) * per + ge] = bl ? v : other;
      hist[(int64_t)(2 * k + 1) * per + ge] = bl ? other : v;
    } else {
      hist[((int64_t)rd.node * f + rd.fbeg) * nbin * 2 + e] = v;
    }
  }
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

// Bc (optional): the bin matrix feature-major [f][nrows]. Rows of a segment
// are ascending, so one feature's bytes of consecutive rows share cache lines
// (row-major, each row's byte costs a line of its own on deep levels).
__global__ void k_goleft(const uint8_t* __restrict__ B, const uint8_t* __restrict__ Bc,
                         int64_t nrows, int f, const int32_t* __restrict__ ridx,
                         int64_t nrows_seg, const int32_t* __restrict__ pos_node,
                         const int32_t* __restrict__ node_feat, const int32_t* __restrict__ node_bin,
                         const uint8_t* __restrict__ node_defl, int32_t* __restrict__ left) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nrows_seg) return;
  const int nd = pos_node[i];
  int l = 0;
  const int feat = nd >= 0 ? node_feat[nd] : -1;
  if (feat >= 0) {
    const int b = Bc ? Bc[(int64_t)feat * nrows + ridx[i]] : B[(int64_t)ridx[i] * f + feat];
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

// Training margins after a tree: one lane per row walks the (pruned) tree on
// the row's bins, in row order. Replaces the leaf-segment scatter
// margin[ridx[i]] += leaf[node(i)] (a random 4-byte read-modify-write per
// row, 336 us per tree at 11M rows) with one coalesced pass over the bin
// matrix (28 bytes per row) and a coalesced margin update. Same decisions
// as the partition (bin <= split bin; missing -> default direction).
__global__ __launch_bounds__(256) void k_leaf_walk(
    const uint8_t* __restrict__ B, int64_t n, int f, const int32_t* __restrict__ feat,
    const int32_t* __restrict__ bin, const uint8_t* __restrict__ defl,
    const int32_t* __restrict__ left, const int32_t* __restrict__ right,
    const float* __restrict__ val, float* __restrict__ margin) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* row = B + i * f;
  int nd = 0;
  for (int d = 0; d < 64; ++d) {  // (depth bound: a malformed tree cannot spin)
    const int ft = feat[nd];
    if (ft < 0) break;
    const int b = row[ft];
    const bool l = b == kMissing ? defl[nd] != 0 : b <= bin[nd];
    nd = l ? left[nd] : right[nd];
  }
  margin[i] += val[nd];
}

// LDS variant: the block's rows are read ONCE, coalesced, into LDS (the
// per-level byte gathers of k_leaf_walk re-fetch a 28-row x 64 B footprint
// per wave at every level, ~8x the bytes of B through L2), and the tree is
// packed into LDS as {feat:16 | bin:8 | defl:8, left:16 | right:16}; the walk
// then touches no global memory until the margin update. Host guarantees:
// f <= kWalkMaxF, nn <= 65535, bins < 256 (see gbdt_leaf_walk below).
constexpr int kWalkRows = 256, kWalkMaxF = 96;
__global__ __launch_bounds__(kWalkRows) void k_leaf_walk_lds(
    const uint8_t* __restrict__ B, int64_t n, int f, int nn, const int32_t* __restrict__ feat,
    const int32_t* __restrict__ bin, const uint8_t* __restrict__ defl,
    const int32_t* __restrict__ left, const int32_t* __restrict__ right,
    const float* __restrict__ val, float* __restrict__ margin) {
  extern __shared__ __attribute__((aligned(16))) uint32_t walk_lds[];
  uint2* tree = reinterpret_cast<uint2*>(walk_lds);
  uint8_t* rows = reinterpret_cast<uint8_t*>(walk_lds + 2 * nn);
  for (int j = threadIdx.x; j < nn; j += blockDim.x) {
    const int ft = feat[j];
    const uint32_t w0 = ft < 0 ? 0xffffu : ((uint32_t)ft | ((uint32_t)bin[j] & 255u) << 16 |
                                           (uint32_t)(defl[j] != 0) << 24);
    tree[j] = make_uint2(w0, ((uint32_t)left[j] & 0xffffu) | ((uint32_t)right[j] << 16));
  }
  // persistent over row tiles: the tree is packed into LDS ONCE per block
  // (one block per 256-row tile re-read the whole node table from L2 per
  // tile: 511 nodes x 17 B for every 256 rows, more bytes than the rows)
  for (int64_t tile = blockIdx.x; tile * kWalkRows < n; tile += gridDim.x) {
    const int64_t i0 = tile * kWalkRows;
    const int nr = (int)min<int64_t>(kWalkRows, n - i0);
    const int nbytes = nr * f;
    const uint8_t* src = B + i0 * f;  // 4-aligned: i0 * f is a multiple of 4 (kWalkRows % 4 == 0)
    const int nw = nbytes >> 2;
    __syncthreads();  // (the tree on the first tile; the previous tile's rows after)
    for (int k = threadIdx.x; k < nw; k += blockDim.x)
      reinterpret_cast<uint32_t*>(rows)[k] = reinterpret_cast<const uint32_t*>(src)[k];
    for (int k = 4 * nw + threadIdx.x; k < nbytes; k += blockDim.x) rows[k] = src[k];
    __syncthreads();
    if ((int)threadIdx.x < nr) {
      const uint8_t* row = rows + threadIdx.x * f;
      int nd = 0;
      for (int d = 0; d < 64; ++d) {
        const uint2 t = tree[nd];
        const uint32_t ft = t.x & 0xffffu;
        if (ft == 0xffffu) break;
        const int b = row[ft];
        const bool l = b == kMissing ? (t.x >> 24) != 0 : b <= (int)((t.x >> 16) & 255u);
        const int nx = (int)(l ? (t.y & 0xffffu) : (t.y >> 16));
        if (nx >= nn) break;  // (a malformed child id cannot read past the tree)
        nd = nx;
      }
      margin[i0 + threadIdx.x] += val[nd];
    }
  }
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

size_t gbdt_hist_lds(int fcnt, int nbin) { return (size_t)fcnt * nbin * 2 * sizeof(int64_t); }

int64_t gbdt_hist_pstride(int max_fcnt, int nbin) { return ((int64_t)2 * max_fcnt * nbin + 31) & ~31; }

void gbdt_hist(const uint8_t* B, int f, int nbin, const int32_t* ridx, const float* gpair,
               const float* qscale, const int32_t* tasks, int ntask, const int32_t* red, int nred,
               int max_fcnt, bool dword_rows, int64_t* part, double* hist, hipStream_t s,
               const int32_t* dseg, int chunk, const int32_t* ntask_dev, bool w32,
               const double* sib_hf, const int32_t* sib_sp, const int32_t* sib_par) {
  if (ntask <= 0) return;
  static bool attr = false;
  if (!attr) {  // dynamic LDS above 64 KB must be opted into per kernel
    const void* ks[4] = {(const void*)k_hist<true, false>, (const void*)k_hist<false, false>,
                         (const void*)k_hist<true, true>, (const void*)k_hist<false, true>};
    for (const void* k : ks)
      WH_HIP_CHECK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kHistLdsMax));
    attr = true;
  }
  const int64_t ps = gbdt_hist_pstride(max_fcnt, nbin);
  const size_t lds = gbdt_hist_lds(max_fcnt, nbin) / (w32 ? 2 : 1);
  const auto* tk = reinterpret_cast<const HistTask*>(tasks);
  const auto* gp = reinterpret_cast<const float2*>(gpair);
  auto* pt = reinterpret_cast<long long*>(part);
  auto kern = dword_rows ? (w32 ? k_hist<true, true> : k_hist<true, false>)
                         : (w32 ? k_hist<false, true> : k_hist<false, false>);
  hipLaunchKernelGGL(kern, dim3(ntask), dim3(kHistThreads), lds, s, B, f, nbin, ridx, gp, qscale, tk,
                     pt, ps, dseg, ntask_dev);
  if (nred > 0)
    hipLaunchKernelGGL(k_hist_reduce, dim3((unsigned)((2 * max_fcnt * nbin + kRedE - 1) / kRedE), nred),
                       dim3(kRedE * kRedK), 0, s, pt, ps, reinterpret_cast<const HistReduce*>(red), f, nbin,
                       qscale, hist, ntask_dev ? nullptr : dseg, chunk, sib_hf, sib_sp, sib_par);
}

// Level bookkeeping on the device (the host tree grower, csrc/bind/gbdt_grow.cc):
// sp[k] = {parent node, parent begin, parent end, build_left} of split k ->
// dseg[k] = rows of the child whose histogram is built (nleft from the
// partition, never read by the host before the next level).
__global__ void k_child_segs(const int32_t* __restrict__ sp, int nsplit,
                             const int32_t* __restrict__ nleft, int32_t* __restrict__ dseg) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nsplit) return;
  const int nd = sp[4 * k], b = sp[4 * k + 1], e = sp[4 * k + 2], bl = sp[4 * k + 3];
  const int m = b + nleft[nd];
  dseg[2 * k] = bl ? b : m;
  dseg[2 * k + 1] = bl ? m : e;
}

// next frontier histograms: for split k (parent slot par[k]) with built child
// histogram hs[k], out[2k] = left child, out[2k+1] = right child, the other
// one being parent - built
__global__ void k_sibling(const double* __restrict__ hf, const double* __restrict__ hs,
                          const int32_t* __restrict__ sp, const int32_t* __restrict__ par,
                          int nsplit, int64_t per, double* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)nsplit * per) return;
  const int k = (int)(t / per);
  const int64_t e = t - (int64_t)k * per;
  const double built = hs[t];
  const double other = hf[(int64_t)par[k] * per + e] - built;
  const bool bl = sp[4 * k + 3] != 0;
  out[(int64_t)(2 * k) * per + e] = bl ? built : other;
  out[(int64_t)(2 * k + 1) * per + e] = bl ? other : built;
}

// One-pass partition of the split nodes' rows (the grower's default): a block
// takes 4096 positions, finds each one's segment by a binary search over the
// segment table in LDS, counts its left / right rows per segment in LDS, then
// reserves room with ONE global atomic per (block, segment, side) on the
// node's cursors (left rows fill the segment from its start, right rows from
// its end down) and scatters. Replaces position->node fill + flags + a
// 3-kernel scan + scatter (5 passes over n per level). Row order inside a
// child is not preserved -- the histograms are exact fixed-point sums, so
// every tree is unchanged.
constexpr int kPcThreads = 256, kPcPer = 16, kPcTile = kPcThreads * kPcPer;
constexpr int kPcMaxTiles = 2048, kPcMaxLocal = 512;

__global__ __launch_bounds__(kPcThreads) void k_part_cursor(
    const uint8_t* __restrict__ B, const uint8_t* __restrict__ Bc, int64_t nrows, int f,
    const int32_t* __restrict__ ridx, int64_t n, const int32_t* __restrict__ tb, int tbs,
    const int32_t* __restrict__ tn, int nt, const int32_t* __restrict__ node_feat,
    const int32_t* __restrict__ node_bin, const uint8_t* __restrict__ node_defl,
    int32_t* __restrict__ lcur, int32_t* __restrict__ rcur, int32_t* __restrict__ out) {
  __shared__ int32_t s_tb[kPcMaxTiles];
  __shared__ uint32_t cnt[2][kPcMaxLocal];
  __shared__ int32_t base[2][kPcMaxLocal];
  __shared__ int32_t s_feat[kPcMaxLocal], s_bin[kPcMaxLocal], s_defl[kPcMaxLocal];
  for (int i = threadIdx.x; i < nt; i += kPcThreads) s_tb[i] = tb[(int64_t)i * tbs];
  for (int i = threadIdx.x; i < kPcMaxLocal; i += kPcThreads) cnt[0][i] = cnt[1][i] = 0;
  __syncthreads();
  const int64_t p0 = (int64_t)blockIdx.x * kPcTile;
  auto seg_of = [&](int64_t i) {  // last segment with begin <= i
    int lo = 0, hi = nt - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_tb[mid] <= i) lo = mid;
      else hi = mid - 1;
    }
    return lo;
  };
  const int sg0 = seg_of(p0);
  const int sgl = seg_of(min(p0 + kPcTile, n) - 1);
#if !defined(WH_PC_OLD)
  if (sg0 == sgl) {
    // Stable split of a tile inside ONE segment (every tile above the deep
    // levels): thread t owns the 16 consecutive positions p0 + 16 t + u, and a
    // block scan of the per-thread left counts ranks each row in position
    // order, so a child receives each block's rows in the order they had --
    // ascending row ids, as the level-0 identity order is. The next level's
    // feature-byte gathers (Bc, one byte of feature-major bins per row) then
    // walk each block's rows upwards through shared cache lines instead of
    // jumping at random (the LDS-atomic ranks of the general path scramble
    // a block's rows). The histograms are exact sums: trees are unchanged.
    __shared__ int32_t s_base[2];
    __shared__ uint32_t s_wl[kPcThreads / 64];
    const int nd = tn[sg0];
    const int feat = nd >= 0 ? node_feat[nd] : -1;
    const int64_t ib = p0 + (int64_t)threadIdx.x * kPcPer;
    int32_t rw[kPcPer];
    if (ib + kPcPer <= n && (reinterpret_cast<uintptr_t>(ridx) & 15) == 0) {
      const int4* r4 = reinterpret_cast<const int4*>(ridx + ib);
#pragma unroll
      for (int v = 0; v < kPcPer / 4; ++v) {
        const int4 x = r4[v];
        rw[4 * v] = x.x; rw[4 * v + 1] = x.y; rw[4 * v + 2] = x.z; rw[4 * v + 3] = x.w;
      }
    } else {
#pragma unroll
      for (int u = 0; u < kPcPer; ++u) rw[u] = ib + u < n ? ridx[ib + u] : 0;
    }
    const int nv = (int)max((int64_t)0, min((int64_t)kPcPer, n - ib));  // valid positions
    if (feat < 0) {  // finished leaf / unsplit node: the rows stay put
      for (int u = 0; u < nv; ++u) out[ib + u] = rw[u];
      return;
    }
    const int bin = node_bin[nd], defl = (int)node_defl[nd];
    int bv[kPcPer];
#pragma unroll
    for (int u = 0; u < kPcPer; ++u)  // every gather in flight before the first is used
      bv[u] = u < nv ? (Bc ? Bc[(int64_t)feat * nrows + rw[u]] : B[(int64_t)rw[u] * f + feat]) : 0;
    uint32_t lm = 0;  // left flags of the thread's positions
#pragma unroll
    for (int u = 0; u < kPcPer; ++u) {
      const int l = bv[u] == kMissing ? defl : (bv[u] <= bin ? 1 : 0);
      lm |= (u < nv && l) ? 1u << u : 0u;
    }
    const uint32_t nl = (uint32_t)__popc(lm);
    uint32_t inc = nl;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o, 64);
      if (lane >= o) inc += y;
    }
    if (lane == 63) s_wl[wid] = inc;
    __syncthreads();
    uint32_t lbefore = inc - nl, ltot = 0;
#pragma unroll
    for (int w = 0; w < kPcThreads / 64; ++w) {
      if (w < wid) lbefore += s_wl[w];
      ltot += s_wl[w];
    }
    const int64_t vtot = min((int64_t)kPcTile, n - p0);
    if (threadIdx.x == 0) {
      const int rtot = (int)(vtot - ltot);
      s_base[0] = ltot ? atomicAdd(&lcur[nd], (int)ltot) : 0;
      s_base[1] = rtot ? atomicSub(&rcur[nd], rtot) - rtot : 0;
    }
    __syncthreads();
#if defined(WH_PC_DIRECT)
    int lo = s_base[0] + (int)lbefore;
    int ro = s_base[1] + (int)(min((int64_t)threadIdx.x * kPcPer, vtot) - lbefore);
#pragma unroll
    for (int u = 0; u < kPcPer; ++u) {
      if (u >= nv) continue;
      if ((lm >> u) & 1u) out[lo++] = rw[u];
      else out[ro++] = rw[u];
    }
#else
    // staged through LDS in child order (left rows, then right rows), then
    // stored as two contiguous runs: every store instruction writes whole
    // lines (the per-thread runs of the direct stores were ~8 rows each)
    __shared__ int32_t s_rows[kPcTile];
    int lo = (int)lbefore;
    int ro = (int)ltot + (int)(min((int64_t)threadIdx.x * kPcPer, vtot) - lbefore);
#pragma unroll
    for (int u = 0; u < kPcPer; ++u) {
      if (u >= nv) continue;
      if ((lm >> u) & 1u) s_rows[lo++] = rw[u];
      else s_rows[ro++] = rw[u];
    }
    __syncthreads();
    const int bl = s_base[0], br = s_base[1] - (int)ltot;
    for (int i = threadIdx.x; i < (int)vtot; i += kPcThreads)
      out[(i < (int)ltot ? bl : br) + i] = s_rows[i];
#endif
    return;
  }
#endif
  // the tile's segments' split rules, read once per block into LDS
  for (int l = threadIdx.x; l < min(sgl - sg0 + 1, kPcMaxLocal); l += kPcThreads) {
    const int nd = tn[sg0 + l];
    const int feat = nd >= 0 ? node_feat[nd] : -1;
    s_feat[l] = feat;
    s_bin[l] = feat >= 0 ? node_bin[nd] : 0;
    s_defl[l] = feat >= 0 ? (int)node_defl[nd] : 0;
  }
  __syncthreads();
  auto seg_in = [&](int64_t i) {  // seg_of over [sg0, sgl] only
    int lo = sg0, hi = sgl;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_tb[mid] <= i) lo = mid;
      else hi = mid - 1;
    }
    return lo;
  };
  int ls[kPcPer], side[kPcPer];
  uint32_t rk[kPcPer];
  int32_t rw[kPcPer];
#pragma unroll
  for (int u = 0; u < kPcPer; ++u) {
    const int64_t i = p0 + u * kPcThreads + threadIdx.x;
    ls[u] = -1;
    side[u] = 0;
    rk[u] = 0;
    rw[u] = i < n ? ridx[i] : 0;
  }
  // every bin gather of the thread issued before the first is used
  int bv[kPcPer];
#pragma unroll
  for (int u = 0; u < kPcPer; ++u) {
    const int64_t i = p0 + u * kPcThreads + threadIdx.x;
    bv[u] = -2;  // -2: no row / finished leaf
    if (i >= n) continue;
    const int l = seg_in(i) - sg0;
    ls[u] = l;
    int feat;
    if (l < kPcMaxLocal) {
      feat = s_feat[l];
    } else {
      const int nd = tn[sg0 + l];
      feat = nd >= 0 ? node_feat[nd] : -1;
    }
    if (feat >= 0)
      bv[u] = Bc ? Bc[(int64_t)feat * nrows + rw[u]] : B[(int64_t)rw[u] * f + feat];
  }
#pragma unroll
  for (int u = 0; u < kPcPer; ++u) {
    const int64_t i = p0 + u * kPcThreads + threadIdx.x;
    if (i >= n) continue;
    if (bv[u] == -2) {
      out[i] = rw[u];  // finished leaf / unsplit node: the row stays put
      ls[u] = -1;
      continue;
    }
    const int b = bv[u];
    if (ls[u] < kPcMaxLocal) {
      const int l = (b == kMissing) ? s_defl[ls[u]] : (b <= s_bin[ls[u]] ? 1 : 0);
      side[u] = l ? 0 : 1;
      rk[u] = atomicAdd(&cnt[side[u]][ls[u]], 1u);
    } else {  // (a tile crossing > kPcMaxLocal segments: a global cursor each)
      const int nd = tn[sg0 + ls[u]];
      const int l = (b == kMissing) ? (int)node_defl[nd] : (b <= node_bin[nd] ? 1 : 0);
      rk[u] = 0;
      out[l ? atomicAdd(&lcur[nd], 1) : atomicSub(&rcur[nd], 1) - 1] = rw[u];
      ls[u] = -1;
    }
  }
  __syncthreads();
  const int nloc = min(sgl - sg0 + 1, kPcMaxLocal);
  for (int q = threadIdx.x; q < 2 * nloc; q += kPcThreads) {
    const int sd = q / nloc, l = q - sd * nloc;
    const uint32_t c = cnt[sd][l];
    if (c == 0) continue;
    const int nd = tn[sg0 + l];
    base[sd][l] = sd == 0 ? atomicAdd(&lcur[nd], (int)c) : atomicSub(&rcur[nd], (int)c) - (int)c;
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kPcPer; ++u)
    if (ls[u] >= 0) out[base[side[u]][ls[u]] + (int)rk[u]] = rw[u];
}

__global__ void k_nleft(const int32_t* __restrict__ lcur, const int32_t* __restrict__ sb, int nnode,
                        int32_t* __restrict__ nleft) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nnode) nleft[i] = lcur[i] - sb[i];
}

bool gbdt_partition_cursor(const uint8_t* B, const uint8_t* Bc, int64_t nrows, int f,
                           const int32_t* ridx, int64_t n, const int32_t* tb, int tbs,
                           const int32_t* tn, int nt, const int32_t* node_feat,
                           const int32_t* node_bin, const uint8_t* node_defl, int32_t* lcur,
                           int32_t* rcur, const int32_t* seg_beg, int nnode, int32_t* nleft,
                           int32_t* out, hipStream_t s) {
  if (nt > kPcMaxTiles || n <= 0) return false;
  hipLaunchKernelGGL(k_part_cursor, dim3((unsigned)((n + kPcTile - 1) / kPcTile)),
                     dim3(kPcThreads), 0, s, B, Bc, nrows, f, ridx, n, tb, tbs, tn, nt, node_feat,
                     node_bin, node_defl, lcur, rcur, out);
  if (nleft)  // (the device grower reads the left cursors themselves)
    hipLaunchKernelGGL(k_nleft, dim3((nnode + 255) / 256), dim3(256), 0, s, lcur, seg_beg, nnode,
                       nleft);
  return true;
}

void gbdt_child_segs(const int32_t* sp, int nsplit, const int32_t* nleft, int32_t* dseg,
                     hipStream_t s) {
  if (nsplit <= 0) return;
  hipLaunchKernelGGL(k_child_segs, dim3((nsplit + 255) / 256), dim3(256), 0, s, sp, nsplit, nleft,
                     dseg);
}

void gbdt_sibling(const double* hf, const double* hs, const int32_t* sp, const int32_t* par,
                  int nsplit, int64_t per, double* out, hipStream_t s) {
  const int64_t n = (int64_t)nsplit * per;
  if (n <= 0) return;
  hipLaunchKernelGGL(k_sibling, dim3(grid_for(n, 256)), dim3(256), 0, s, hf, hs, sp, par, nsplit,
                     per, out);
}

void gbdt_seg_fill(const int32_t* beg, const int32_t* node, int nseg, int64_t n, int32_t* out,
                   hipStream_t s) {
  if (n <= 0 || nseg <= 0) return;
  hipLaunchKernelGGL(k_seg_fill, dim3(grid_for(n, 256)), dim3(256), 0, s, beg, node, nseg, n, out);
}

void gbdt_goleft(const uint8_t* B, const uint8_t* Bc, int64_t nrows, int f, const int32_t* ridx,
                 int64_t n, const int32_t* pos_node, const int32_t* node_feat,
                 const int32_t* node_bin, const uint8_t* node_defl, int32_t* left, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_goleft, dim3(grid_for(n, 256)), dim3(256), 0, s, B, Bc, nrows, f, ridx, n,
                     pos_node, node_feat, node_bin, node_defl, left);
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

namespace {
// Gradient pairs of one boosting round in one launch, with the tree's root
// statistics (reference: xgboost's ObjFunction::GetGradient, then the
// GPU hist updater's root sum): gpair[i] = {g, h} for binary:logistic
// (p = sigmoid(margin), g = p - y, h = max(p (1 - p), 1e-16)) or squared
// error (g = margin - y, h = 1), times the row weight; stats = {sum g,
// sum h (fp64), max |g|, max |h|} by per-block partials + arrival ticket.
// Replaced ~12 torch launches (~0.45 ms per tree at 11M rows).
constexpr int kGpThreads = 256, kGpBlocks = 1024;
__global__ __launch_bounds__(kGpThreads) void k_gpair(int64_t n, const float* __restrict__ margin,
                                                      const float* __restrict__ label,
                                                      const float* __restrict__ weight,
                                                      int logistic, float2* __restrict__ out,
                                                      double* __restrict__ part,
                                                      unsigned int* ticket, double* stats) {
  __shared__ double sh[4][kGpThreads / 64];
  __shared__ int last;
  double sg = 0, shh = 0, mg = 0, mh = 0;
  for (int64_t i = (int64_t)blockIdx.x * kGpThreads + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kGpThreads) {
    const float m = margin[i], y = label[i];
    float g, h;
    if (logistic) {
      const float p = 1.f / (1.f + expf(-m));
      g = p - y;
      h = fmaxf(p * (1.f - p), 1e-16f);
    } else {
      g = m - y;
      h = 1.f;
    }
    if (weight) {
      const float w = weight[i];
      g *= w;
      h *= w;
    }
    out[i] = make_float2(g, h);
    sg += g;
    shh += h;
    mg = fmax(mg, (double)fabsf(g));
    mh = fmax(mh, (double)fabsf(h));
  }
  sg = wave_sum_d(sg);
  shh = wave_sum_d(shh);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mg = fmax(mg, __shfl_xor(mg, o, 64));
    mh = fmax(mh, __shfl_xor(mh, o, 64));
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    sh[0][wid] = sg; sh[1][wid] = shh; sh[2][wid] = mg; sh[3][wid] = mh;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double v[4] = {0, 0, 0, 0};
    for (int w = 0; w < kGpThreads / 64; ++w) {
      v[0] += sh[0][w]; v[1] += sh[1][w];
      v[2] = fmax(v[2], sh[2][w]); v[3] = fmax(v[3], sh[3][w]);
    }
    for (int q = 0; q < 4; ++q)
      lb_store(reinterpret_cast<unsigned long long*>(part) + blockIdx.x * 4 + q,
               (unsigned long long)__double_as_longlong(v[q]));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = arrive_last(ticket, blockIdx.x, gridDim.x);
  }
  __syncthreads();
  if (!last) return;
  // the last block sums the partials: thread t takes blocks t, t + 256, ...
  // (all loads in flight; one serial walk cost ~200 us of load latency), then
  // a fixed-order tree -- the same sums every run
  double v[4] = {0, 0, 0, 0};
  const unsigned long long* pp = reinterpret_cast<const unsigned long long*>(part);
  for (unsigned b = threadIdx.x; b < gridDim.x; b += kGpThreads) {
    v[0] += __longlong_as_double((long long)lb_load(pp + b * 4));
    v[1] += __longlong_as_double((long long)lb_load(pp + b * 4 + 1));
    v[2] = fmax(v[2], __longlong_as_double((long long)lb_load(pp + b * 4 + 2)));
    v[3] = fmax(v[3], __longlong_as_double((long long)lb_load(pp + b * 4 + 3)));
  }
  v[0] = wave_sum_d(v[0]);
  v[1] = wave_sum_d(v[1]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    v[2] = fmax(v[2], __shfl_xor(v[2], o, 64));
    v[3] = fmax(v[3], __shfl_xor(v[3], o, 64));
  }
  __syncthreads();
  if (lane == 0) {
    sh[0][wid] = v[0]; sh[1][wid] = v[1]; sh[2][wid] = v[2]; sh[3][wid] = v[3];
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  double r[4] = {0, 0, 0, 0};
  for (int w = 0; w < kGpThreads / 64; ++w) {
    r[0] += sh[0][w]; r[1] += sh[1][w];
    r[2] = fmax(r[2], sh[2][w]); r[3] = fmax(r[3], sh[3][w]);
  }
  for (int q = 0; q < 4; ++q) stats[q] = r[q];
}
}  // namespace

namespace {
// Histogram fixed-point scales from the (allreduced) max |g|, max |h| in one
// launch instead of ~12 torch ops per tree (models/gbdt.py GBTree._qscale):
// out = {2^eg, 2^eh[, R]}, e = floor(log2(2^61 / (N m))), with R > 0 also
// <= floor(log2(2^30 / (R m))), clamped to [-60, 100].
__global__ void k_qscale(const float* __restrict__ m, double nglobal, int R,
                         float* __restrict__ out) {
  const int t = threadIdx.x;
  if (t < 2) {
    const double mm = fmax((double)m[t], 1e-30);
    double e = floor(log2(0x1p61 / (nglobal * mm)));
    if (R > 0) e = fmin(e, floor(log2(0x1p30 / ((double)R * mm))));
    e = fmin(fmax(e, -60.0), 100.0);
    out[t] = (float)exp2(e);
  } else if (t == 2 && R > 0) {
    out[2] = (float)R;
  }
}
}  // namespace

void gbdt_qscale(const float* m, double nglobal, int R, float* out, hipStream_t s) {
  hipLaunchKernelGGL(k_qscale, dim3(1), dim3(64), 0, s, m, nglobal, R, out);
}

int64_t gbdt_gpair_scratch() { return 4 * (int64_t)kGpBlocks + kArriveWords / 2 + 1; }

void gbdt_gpair(int64_t n, const float* margin, const float* label, const float* weight,
                bool logistic, float* gpair, double* scratch, double* stats, hipStream_t s) {
  // scratch: per-block partials, then the (zeroed) arrival ticket words
  unsigned int* ticket = reinterpret_cast<unsigned int*>(scratch + 4 * kGpBlocks);
  const int nb = std::max(1, std::min<int>(kGpBlocks, grid_for(n, kGpThreads)));
  hipLaunchKernelGGL(k_gpair, dim3(nb), dim3(kGpThreads), 0, s, n, margin, label, weight,
                     logistic ? 1 : 0, reinterpret_cast<float2*>(gpair), scratch, ticket, stats);
}

void gbdt_leaf_walk(const uint8_t* B, int64_t n, int f, int nn, const int32_t* feat, const int32_t* bin,
                    const uint8_t* defl, const int32_t* left, const int32_t* right,
                    const float* val, float* margin, hipStream_t s, bool lds) {
  if (n <= 0) return;
  const size_t lbytes = (size_t)nn * 8 + (size_t)kWalkRows * f;
  if (nn > 0 && nn <= 65535 && f <= kWalkMaxF && lbytes <= 48 * 1024 &&
      (reinterpret_cast<uintptr_t>(B) & 3) == 0 && lds) {
    // persistent: ~8 blocks per CU, each walking many tiles
    const int64_t tiles = (n + kWalkRows - 1) / kWalkRows;
    static int cus = 0;
    if (cus == 0) {
      int dev = 0;
      WH_HIP_CHECK(hipGetDevice(&dev));
      WH_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    }
    const unsigned grid = (unsigned)std::min<int64_t>(tiles, (int64_t)8 * std::max(cus, 1));
    hipLaunchKernelGGL(k_leaf_walk_lds, dim3(grid), dim3(kWalkRows), lbytes, s, B, n, f, nn, feat,
                       bin, defl, left, right, val, margin);
    return;
  }
  hipLaunchKernelGGL(k_leaf_walk, dim3(grid_for(n, 256)), dim3(256), 0, s, B, n, f, feat, bin, defl,
                     left, right, val, margin);
}

void gbdt_predict(const float* X, int64_t n, int f, const int32_t* feat, const float* thr,
                  const int32_t* left, const int32_t* right, const uint8_t* defl,
                  const float* leaf, float* margin, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_predict, dim3(grid_for(n, 256)), dim3(256), 0, s, X, n, f, feat, thr, left,
                     right, defl, leaf, margin);
}

}  // namespace wh

namespace wh {
namespace {

// ---- the level loop on the device (gbdt_grow_dev) --------------------------
// Heap-numbered nodes: depth d holds slots s = 0..2^d - 1, node id 2^d - 1 + s,
// children 2s / 2s + 1 at depth d + 1. Every slot owns a segment of ridx;
// the segments of a depth tile [0, n) in slot order (a dead slot -- the
// child of a leaf -- is empty, or carries its leaf parent's rows as one
// "stay put" segment), so the one-pass cursor partition (k_part_cursor) runs
// on the device's segment table. Node record (doubles): {alive, feat, bin,
// defl, gain, cover, base weight, leaf, begin, end}.
constexpr int kNodeRec = 10;

// heap node records -> the row walk's arrays: node h splits on feat / bin
// (children 2h + 1, 2h + 2) when alive and split, else is a leaf of value
// rec[7] (dead nodes are never reached)
__global__ __launch_bounds__(256) void k_heap_tree(const double* __restrict__ nodes, int nn,
                                                   int32_t* __restrict__ feat,
                                                   int32_t* __restrict__ bin,
                                                   uint8_t* __restrict__ defl,
                                                   int32_t* __restrict__ left,
                                                   int32_t* __restrict__ right,
                                                   float* __restrict__ leaf) {
  for (int h = blockIdx.x * blockDim.x + threadIdx.x; h < nn; h += gridDim.x * blockDim.x) {
    const double* q = nodes + (int64_t)h * kNodeRec;
    const bool split = q[0] != 0.0 && q[1] >= 0.0 && 2 * h + 2 < nn;
    feat[h] = split ? (int32_t)q[1] : -1;
    bin[h] = split ? (int32_t)q[2] : 0;
    defl[h] = split ? (uint8_t)q[3] : 0;
    left[h] = split ? 2 * h + 1 : -1;
    right[h] = split ? 2 * h + 2 : -1;
    leaf[h] = (float)q[7];
  }
}



// One block: for slot s of depth d (S slots), decide its split from the
// split search's result, record the node, and set up the partition and the
// next level's totals (the host grower's level bookkeeping).
__global__ __launch_bounds__(256) void k_gd_apply(
    int S, int node0, int last, const double* __restrict__ so, const double* __restrict__ tot,
    const int32_t* __restrict__ seg, const uint8_t* __restrict__ alive, double eta, double alpha,
    double lambda, double mcw, double rt_eps, double* __restrict__ nodes,
    int32_t* __restrict__ pfeat, int32_t* __restrict__ pbin, uint8_t* __restrict__ pdefl,
    int32_t* __restrict__ lcur, int32_t* __restrict__ rcur, uint8_t* __restrict__ split,
    uint8_t* __restrict__ build_left, double* __restrict__ tot_next, int32_t* __restrict__ nleft) {
  for (int sl = threadIdx.x; sl < S; sl += blockDim.x) {
    if (nleft) nleft[sl] = 0;  // the partition's left counts (no memset launch)
    const double G = tot[2 * sl], H = tot[2 * sl + 1];
    const int b = seg[2 * sl], e = seg[2 * sl + 1];
    double* nd = nodes + (int64_t)(node0 + sl) * kNodeRec;
    const bool al = alive[sl] != 0;
    const double* o = so + (int64_t)sl * 6;
    const bool sp = al && !last && o[0] > rt_eps;
    double bw = 0.0;
    if (H >= mcw) {
      const double g = alpha <= 0 ? G : (G > alpha ? G - alpha : (G < -alpha ? G + alpha : 0.0));
      bw = -g / (H + lambda);
    }
    nd[0] = al ? 1.0 : 0.0;
    nd[1] = sp ? o[1] : -1.0;
    nd[2] = sp ? o[2] : 0.0;
    nd[3] = sp ? o[3] : 0.0;
    nd[4] = sp ? o[0] : 0.0;
    nd[5] = H;
    nd[6] = bw;
    nd[7] = eta * bw;
    nd[8] = b;
    nd[9] = e;
    pfeat[sl] = sp ? (int32_t)o[1] : -1;
    pbin[sl] = sp ? (int32_t)o[2] : 0;
    pdefl[sl] = sp ? (uint8_t)o[3] : 0;
    lcur[sl] = b;
    rcur[sl] = e;
    split[sl] = sp ? 1 : 0;
    const double GL = sp ? o[4] : 0.0, HL = sp ? o[5] : 0.0;
    const double GR = sp ? G - GL : 0.0, HR = sp ? H - HL : 0.0;
    build_left[sl] = HL <= HR ? 1 : 0;  // build the child with the smaller global hessian
    if (tot_next) {
      tot_next[4 * sl] = GL;
      tot_next[4 * sl + 1] = HL;
      tot_next[4 * sl + 2] = GR;
      tot_next[4 * sl + 3] = HR;
    }
  }
}

// One block (S <= 1024 slots): the next level's segments / alive flags, the
// built children's rows (dseg), the sibling table, and the histogram task
// list of the built children: per slot ceil(rows / chunk) chunks x G feature
// groups (offsets by a block scan), its count, and the reduce entries.
__global__ __launch_bounds__(1024) void k_gd_children(
    int S, const int32_t* __restrict__ seg, const uint8_t* __restrict__ split,
    const uint8_t* __restrict__ build_left, const int32_t* __restrict__ lcur,
    const int32_t* __restrict__ fg, int G, int chunk, int32_t* __restrict__ seg_next,
    uint8_t* __restrict__ alive_next, int32_t* __restrict__ dseg, int32_t* __restrict__ sp,
    int32_t* __restrict__ par, HistTask* __restrict__ tasks, int32_t* __restrict__ ntask,
    HistReduce* __restrict__ red) {
  __shared__ int32_t ws[16];
  const int sl = threadIdx.x, lane = sl & 63, w = sl >> 6;
  int32_t nch = 0, b = 0, e = 0, m = 0;
  bool s_ = false;
  if (sl < S) {
    b = seg[2 * sl];
    e = seg[2 * sl + 1];
    s_ = split[sl] != 0;
    m = s_ ? lcur[sl] : e;  // the left cursor after the partition (= b when none ran)
    seg_next[4 * sl] = b;
    seg_next[4 * sl + 1] = m;
    seg_next[4 * sl + 2] = m;
    seg_next[4 * sl + 3] = e;
    alive_next[2 * sl] = alive_next[2 * sl + 1] = s_ ? 1 : 0;
    const bool bl = build_left[sl] != 0;
    const int32_t db = s_ ? (bl ? b : m) : 0, de = s_ ? (bl ? m : e) : 0;
    dseg[2 * sl] = db;
    dseg[2 * sl + 1] = de;
    sp[4 * sl] = sl;
    sp[4 * sl + 1] = b;
    sp[4 * sl + 2] = e;
    sp[4 * sl + 3] = bl ? 1 : 0;
    par[sl] = sl;
    nch = s_ ? (de - db + chunk - 1) / chunk : 0;
  }
  // exclusive scan of the chunk counts
  int32_t x = nch;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) ws[w] = x;
  __syncthreads();
  int32_t base = x - nch, tot = 0;
  for (int q = 0; q < (int)(blockDim.x >> 6); ++q) {
    if (q < w) base += ws[q];
    tot += ws[q];
  }
  __shared__ int32_t soff[1025];
  if (sl < S) soff[sl] = base;
  if (sl == 0) soff[S] = tot;
  __syncthreads();
  // the tasks, spread over the block: chunk q of the level belongs to the
  // last slot whose offset is <= q (one slot's thread writing all its chunks
  // serialised ~500 task stores at the root's children)
  for (int q = sl; q < tot; q += blockDim.x) {
    int lo = 0, hi = S - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (soff[mid] <= q) lo = mid;
      else hi = mid - 1;
    }
    for (int gi = 0; gi < G; ++gi) {
      HistTask t;
      t.node = lo;
      t.fbeg = fg[2 * gi];
      t.fcnt = fg[2 * gi + 1];
      t.rbeg = q - soff[lo];
      t.rend = chunk;
      tasks[(int64_t)q * G + gi] = t;
    }
  }
  if (sl < S) {
    for (int gi = 0; gi < G; ++gi) {
      HistReduce r;
      r.node = sl;
      r.fbeg = fg[2 * gi];
      r.fcnt = fg[2 * gi + 1];
      r.t0 = base * G + gi;
      r.nt = nch;
      r.tstride = G;
      red[(int64_t)sl * G + gi] = r;
    }
  }
  if (sl == 0) *ntask = tot * G;
}

}  // namespace

void gbdt_heap_tree(const double* nodes, int nn, int32_t* feat, int32_t* bin, uint8_t* defl,
                    int32_t* left, int32_t* right, float* leaf, hipStream_t s) {
  if (nn <= 0) return;
  hipLaunchKernelGGL(k_heap_tree, dim3((unsigned)((nn + 255) / 256)), dim3(256), 0, s, nodes, nn,
                     feat, bin, defl, left, right, leaf);
}

int gbdt_node_rec() { return kNodeRec; }

void gbdt_dev_apply(int S, int node0, bool last, const double* so, const double* tot,
                    const int32_t* seg, const uint8_t* alive, double eta, double alpha,
                    double lambda, double mcw, double rt_eps, double* nodes, int32_t* pfeat,
                    int32_t* pbin, uint8_t* pdefl, int32_t* lcur, int32_t* rcur, uint8_t* split,
                    uint8_t* build_left, double* tot_next, int32_t* nleft, hipStream_t s) {
  hipLaunchKernelGGL(k_gd_apply, dim3(1), dim3(256), 0, s, S, node0, last ? 1 : 0, so, tot, seg,
                     alive, eta, alpha, lambda, mcw, rt_eps, nodes, pfeat, pbin, pdefl, lcur, rcur,
                     split, build_left, tot_next, nleft);
}

bool gbdt_dev_children(int S, const int32_t* seg, const uint8_t* split, const uint8_t* build_left,
                       const int32_t* lcur, const int32_t* fg, int G, int chunk,
                       int32_t* seg_next, uint8_t* alive_next, int32_t* dseg, int32_t* sp,
                       int32_t* par, int32_t* tasks, int32_t* ntask, int32_t* red,
                       hipStream_t s) {
  if (S > 1024) return false;
  hipLaunchKernelGGL(k_gd_children, dim3(1), dim3(1024), 0, s, S, seg, split, build_left, lcur,
                     fg, G, chunk, seg_next, alive_next, dseg, sp, par,
                     reinterpret_cast<HistTask*>(tasks), ntask, reinterpret_cast<HistReduce*>(red));
  return true;
}

}  // namespace wh

// ---- split search -----------------------------------------------------
// One block per (node, feature): inclusive scan of the feature's (g, h) bins
// in double, both default directions for the rows missing the feature, the
// regularised gain of every threshold, and the block's best candidate; then
// one wave per node picks the best feature. Ties resolve to the smallest
// flat index ((f * nbin + b) * 2 + dir), like a row-major argmax.
namespace {

constexpr int kSplitThreads = 256;
constexpr int kSplitMaxPer = 4;  // bins per thread (nbin <= 1024)

struct SplitParam {
  double alpha, lambda, mcw;
};

__device__ __forceinline__ double split_gain(double G, double H, const SplitParam& p) {
  if (H < p.mcw) return 0.0;
  double g = G;
  if (p.alpha != 0.0) g = G > p.alpha ? G - p.alpha : (G < -p.alpha ? G + p.alpha : 0.0);
  return g * g / (H + p.lambda);
}

__device__ __forceinline__ double shfl_up_d(double v, int o) {
  return __shfl_up(v, o, 64);
}

__device__ __forceinline__ bool better(double g, long long i, double bg, long long bi) {
  return g > bg || (g == bg && i < bi);
}

__global__ __launch_bounds__(kSplitThreads) void k_split_feat(
    const double* __restrict__ hist, const double* __restrict__ totals,
    const uint8_t* __restrict__ valid, int F, int nbin, SplitParam p, double* __restrict__ cand) {
  const int s = blockIdx.x / F, f = blockIdx.x % F;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const double* hb = hist + ((int64_t)s * F + f) * nbin * 2;
  const int per = (nbin + kSplitThreads - 1) / kSplitThreads;
  double lg[kSplitMaxPer], lh[kSplitMaxPer];
  double sg = 0.0, sh = 0.0;
#pragma unroll
  for (int u = 0; u < kSplitMaxPer; ++u) {
    const int b = t * per + u;
    const bool ok = u < per && b < nbin;
    sg += ok ? hb[2 * b] : 0.0;
    sh += ok ? hb[2 * b + 1] : 0.0;
    lg[u] = sg;
    lh[u] = sh;
  }
  // exclusive prefix of the thread totals: wave scans + wave totals in LDS
  __shared__ double wg[kSplitThreads / 64], wh[kSplitThreads / 64];
  double xg = sg, xh = sh;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double yg = shfl_up_d(xg, o), yh = shfl_up_d(xh, o);
    if (lane >= o) {
      xg += yg;
      xh += yh;
    }
  }
  if (lane == 63) {
    wg[w] = xg;
    wh[w] = xh;
  }
  __syncthreads();
  double og = xg - sg, oh = xh - sh, pg = 0.0, ph = 0.0;
  for (int i = 0; i < kSplitThreads / 64; ++i) {
    if (i < w) {
      og += wg[i];
      oh += wh[i];
    }
    pg += wg[i];
    ph += wh[i];
  }
  const double TG = totals[2 * s], TH = totals[2 * s + 1];
  const double mg = TG - pg, mh = TH - ph;  // rows missing this feature
  const double parent = split_gain(TG, TH, p);
  double best = -INFINITY;
  long long bidx = 0x7fffffffffffffffll;
  double bgl = 0.0, bhl = 0.0;
#pragma unroll
  for (int u = 0; u < kSplitMaxPer; ++u) {
    const int b = t * per + u;
    if (u >= per || b >= nbin) break;
    if (!valid[(int64_t)f * nbin + b]) continue;
#pragma unroll
    for (int d = 0; d < 2; ++d) {
      const double GL = og + lg[u] + (d ? mg : 0.0), HL = oh + lh[u] + (d ? mh : 0.0);
      const double GR = TG - GL, HR = TH - HL;
      if (!(HL >= p.mcw && HR >= p.mcw)) continue;
      const double g = split_gain(GL, HL, p) + split_gain(GR, HR, p) - parent;
      const long long idx = ((long long)f * nbin + b) * 2 + d;
      if (better(g, idx, best, bidx)) {
        best = g;
        bidx = idx;
        bgl = GL;
        bhl = HL;
      }
    }
  }
  // block argmax (gain desc, index asc)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double g2 = __shfl_xor(best, o, 64);
    const long long i2 = __shfl_xor(bidx, o, 64);
    const double l2 = __shfl_xor(bgl, o, 64), h2 = __shfl_xor(bhl, o, 64);
    if (better(g2, i2, best, bidx)) {
      best = g2;
      bidx = i2;
      bgl = l2;
      bhl = h2;
    }
  }
  __shared__ double rg[kSplitThreads / 64], rl[kSplitThreads / 64], rh[kSplitThreads / 64];
  __shared__ long long ri[kSplitThreads / 64];
  if (lane == 0) {
    rg[w] = best;
    ri[w] = bidx;
    rl[w] = bgl;
    rh[w] = bhl;
  }
  __syncthreads();
  if (t == 0) {
    for (int i = 1; i < kSplitThreads / 64; ++i)
      if (better(rg[i], ri[i], best, bidx)) {
        best = rg[i];
        bidx = ri[i];
        bgl = rl[i];
        bhl = rh[i];
      }
    double* c = cand + ((int64_t)s * F + f) * 4;
    c[0] = best;
    c[1] = (double)bidx;
    c[2] = bgl;
    c[3] = bhl;
  }
}

__global__ __launch_bounds__(64) void k_split_node(const double* __restrict__ cand, int F,
                                                   int nbin, double* __restrict__ out) {
  const int s = blockIdx.x, lane = threadIdx.x;
  double best = -INFINITY, bgl = 0.0, bhl = 0.0;
  long long bidx = 0x7fffffffffffffffll;
  for (int f = lane; f < F; f += 64) {
    const double* c = cand + ((int64_t)s * F + f) * 4;
    const long long i = c[0] == -INFINITY ? (long long)f * nbin * 2 : (long long)c[1];
    if (better(c[0], i, best, bidx)) {
      best = c[0];
      bidx = i;
      bgl = c[2];
      bhl = c[3];
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double g2 = __shfl_xor(best, o, 64);
    const long long i2 = __shfl_xor(bidx, o, 64);
    const double l2 = __shfl_xor(bgl, o, 64), h2 = __shfl_xor(bhl, o, 64);
    if (better(g2, i2, best, bidx)) {
      best = g2;
      bidx = i2;
      bgl = l2;
      bhl = h2;
    }
  }
  if (lane == 0) {
    if (best == -INFINITY) bidx = 0;  // all candidates invalid: argmax of -inf is index 0
    double* o = out + (int64_t)s * 6;
    o[0] = best;
    o[1] = (double)(bidx / 2 / nbin);
    o[2] = (double)((bidx / 2) % nbin);
    o[3] = (double)(bidx % 2);
    o[4] = bgl;
    o[5] = bhl;
  }
}

}  // namespace

namespace wh {

bool gbdt_split(const double* hist, const double* totals, const uint8_t* valid, int S, int F,
                int nbin, double alpha, double lambda, double mcw, double* cand, double* out,
                hipStream_t s) {
  if (nbin > kSplitThreads * kSplitMaxPer || S <= 0 || F <= 0) return false;
  const SplitParam p{alpha, lambda, mcw};
  hipLaunchKernelGGL(k_split_feat, dim3((unsigned)(S * F)), dim3(kSplitThreads), 0, s, hist,
                     totals, valid, F, nbin, p, cand);
  hipLaunchKernelGGL(k_split_node, dim3((unsigned)S), dim3(64), 0, s, cand, F, nbin, out);
  return true;
}

}  // namespace wh

// ---- sparse (CSR) input -------------------------------------------------
// A libsvm-style matrix stays CSR: each stored value gets a GLOBAL bin id
// cut_off[feature] + bin (features own cut_off[f+1] - cut_off[f] bins, 0 for
// a feature that never occurs), histograms are [slots][total bins][2] in that
// compact layout (no F x max_bin padding, no dense n x F matrix), and a row
// missing a feature takes the split's default direction (the split search
// derives the missing mass as node total - the feature's stored mass, as in
// the dense path). Row feature ids are ascending within a row.
namespace wh {
namespace {

__global__ void k_bin_csr(const int32_t* __restrict__ fid, const float* __restrict__ val,
                          int64_t nnz, int ncol, const float* __restrict__ cuts,
                          const int32_t* __restrict__ cut_off, int32_t* __restrict__ gbin) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nnz) return;
  const int f = fid[i];
  if (f < 0 || f >= ncol) {
    gbin[i] = -1;
    return;
  }
  const int lo0 = cut_off[f], hi0 = cut_off[f + 1];
  if (hi0 <= lo0) {
    gbin[i] = -1;
    return;
  }
  const float v = val ? val[i] : 1.f;
  int lo = lo0, hi = hi0 - 1;  // first cut > v (upper_bound), capped at the last bin
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (cuts[mid] > v) hi = mid;
    else lo = mid + 1;
  }
  gbin[i] = lo;
}

// one thread per row of the task: adds its stored values' (g, h) into the
// slot's compact histogram (fixed-point int64 global atomics: exact and
// order-free; total bins can be far beyond an LDS tile)
__global__ void k_hist_csr(const int64_t* __restrict__ row_off, const int32_t* __restrict__ gbin,
                           const int32_t* __restrict__ ridx, const float2* __restrict__ gpair,
                           const float* __restrict__ qscale, const int32_t* __restrict__ tasks,
                           int64_t tb, unsigned long long* __restrict__ hist) {
  const int32_t* tk = tasks + 3 * blockIdx.y;  // {slot, rbeg, rend}
  const int r = tk[1] + blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= tk[2]) return;
  const int row = ridx[r];
  const float2 gh = gpair[row];
  const long long qg = __float2ll_rn(gh.x * qscale[0]), qh = __float2ll_rn(gh.y * qscale[1]);
  unsigned long long* h = hist + (int64_t)tk[0] * tb * 2;
  for (int64_t j = row_off[row]; j < row_off[row + 1]; ++j) {
    const int b = gbin[j];
    if (b < 0) continue;
    atomicAdd(h + 2 * (int64_t)b, (unsigned long long)qg);
    atomicAdd(h + 2 * (int64_t)b + 1, (unsigned long long)qh);
  }
}

__global__ void k_hist_csr_fin(const unsigned long long* __restrict__ q, int64_t n,
                               const float* __restrict__ qscale, double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (double)(long long)q[i] / (double)qscale[i & 1];
}

// best split per (node, feature): one thread walks the feature's bins; then
// per node the best feature (ties: smallest (feature, bin, dir) as dense).
// cand [S][F] = {gain, bin, dir, GL, HL}
__global__ void k_split_csr_feat(const double* __restrict__ hist, int64_t tb,
                                 const double* __restrict__ totals,
                                 const int32_t* __restrict__ cut_off,
                                 const uint8_t* __restrict__ fvalid, int F, SplitParam p,
                                 double* __restrict__ cand) {
  const int s = blockIdx.y;
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= F) return;
  double* c = cand + ((int64_t)s * F + f) * 5;
  c[0] = -INFINITY;
  const int b0 = cut_off[f], b1 = cut_off[f + 1];
  if (b1 <= b0 || (fvalid && !fvalid[f])) return;
  const double* hb = hist + (int64_t)s * tb * 2;
  const double TG = totals[2 * s], TH = totals[2 * s + 1];
  double pg = 0.0, ph = 0.0;
  for (int b = b0; b < b1; ++b) pg += hb[2 * b], ph += hb[2 * b + 1];
  const double mg = TG - pg, mh = TH - ph, parent = split_gain(TG, TH, p);
  double best = -INFINITY, gl = 0.0, hl = 0.0, sg = 0.0, sh = 0.0;
  int bb = 0, bd = 0;
  for (int b = b0; b < b1; ++b) {
    sg += hb[2 * b];
    sh += hb[2 * b + 1];
    for (int d = 0; d < 2; ++d) {
      const double GL = sg + (d ? mg : 0.0), HL = sh + (d ? mh : 0.0);
      const double GR = TG - GL, HR = TH - HL;
      if (!(HL >= p.mcw && HR >= p.mcw)) continue;
      const double g = split_gain(GL, HL, p) + split_gain(GR, HR, p) - parent;
      if (g > best) {
        best = g, bb = b - b0, bd = d, gl = GL, hl = HL;
      }
    }
  }
  c[0] = best, c[1] = bb, c[2] = bd, c[3] = gl, c[4] = hl;
}

__global__ __launch_bounds__(256) void k_split_csr_node(const double* __restrict__ cand, int F,
                                                        double* __restrict__ out) {
  const int s = blockIdx.x;
  double best = -INFINITY;
  long long bi = 0x7fffffffffffffffll;
  for (int f = threadIdx.x; f < F; f += 256) {
    const double* c = cand + ((int64_t)s * F + f) * 5;
    const long long idx = (long long)f * 2048 + (long long)c[1] * 2 + (long long)c[2];
    if (better(c[0], idx, best, bi)) best = c[0], bi = idx;
  }
  __shared__ double sb[256];
  __shared__ long long si[256];
  sb[threadIdx.x] = best;
  si[threadIdx.x] = bi;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o && better(sb[threadIdx.x + o], si[threadIdx.x + o], sb[threadIdx.x],
                                  si[threadIdx.x])) {
      sb[threadIdx.x] = sb[threadIdx.x + o];
      si[threadIdx.x] = si[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    double* o = out + 6 * s;
    if (!(sb[0] > -INFINITY)) {
      o[0] = -INFINITY, o[1] = o[2] = o[3] = o[4] = o[5] = 0.0;
      return;
    }
    const int f = (int)(si[0] / 2048);
    const double* c = cand + ((int64_t)s * F + f) * 5;
    o[0] = c[0], o[1] = f, o[2] = c[1], o[3] = c[2], o[4] = c[3], o[5] = c[4];
  }
}

// go-left flag of every position: the row's stored value of the node's
// feature (binary search in the row's ascending ids), else the default
__global__ void k_goleft_csr(const int64_t* __restrict__ row_off, const int32_t* __restrict__ fid,
                             const int32_t* __restrict__ gbin, const int32_t* __restrict__ cut_off,
                             const int32_t* __restrict__ ridx, int64_t n,
                             const int32_t* __restrict__ pos_node,
                             const int32_t* __restrict__ node_feat,
                             const int32_t* __restrict__ node_bin,
                             const uint8_t* __restrict__ node_defl, int32_t* __restrict__ left) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int nd = pos_node[i];
  const int f = nd >= 0 ? node_feat[nd] : -1;
  int l = 0;
  if (f >= 0) {
    const int row = ridx[i];
    int64_t lo = row_off[row], hi = row_off[row + 1];
    int b = -1;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      const int v = fid[mid];
      if (v == f) {
        b = gbin[mid];
        break;
      }
      if (v < f) lo = mid + 1;
      else hi = mid;
    }
    l = b < 0 ? (int)node_defl[nd] : (b - cut_off[f] <= node_bin[nd] ? 1 : 0);
  }
  left[i] = l;
}

// tree walk on CSR rows (raw values; missing -> default direction)
__global__ void k_predict_csr(const int64_t* __restrict__ row_off, const int32_t* __restrict__ fid,
                              const float* __restrict__ val, int64_t n,
                              const int32_t* __restrict__ feat, const float* __restrict__ thr,
                              const int32_t* __restrict__ left, const int32_t* __restrict__ right,
                              const uint8_t* __restrict__ defl, const float* __restrict__ leaf,
                              float* __restrict__ margin) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  int nd = 0;
  for (int depth = 0; depth < 64 && feat[nd] >= 0; ++depth) {
    const int f = feat[nd];
    int64_t lo = row_off[r], hi = row_off[r + 1];
    bool found = false;
    float v = 0.f;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      const int x = fid[mid];
      if (x == f) {
        found = true;
        v = val ? val[mid] : 1.f;
        break;
      }
      if (x < f) lo = mid + 1;
      else hi = mid;
    }
    const bool goleft = found ? (v < thr[nd]) : (defl[nd] != 0);
    nd = goleft ? left[nd] : right[nd];
  }
  margin[r] += leaf[nd];
}

}  // namespace

void gbdt_bin_csr(const int32_t* fid, const float* val, int64_t nnz, int ncol, const float* cuts,
                  const int32_t* cut_off, int32_t* gbin, hipStream_t s) {
  if (nnz <= 0) return;
  hipLaunchKernelGGL(k_bin_csr, dim3(grid_for(nnz, 256)), dim3(256), 0, s, fid, val, nnz, ncol,
                     cuts, cut_off, gbin);
}

void gbdt_hist_csr(const int64_t* row_off, const int32_t* gbin, const int32_t* ridx,
                   const float* gpair, const float* qscale, const int32_t* tasks, int ntask,
                   int max_rows, int64_t tb, int nslot, int64_t* hq, double* hist, hipStream_t s) {
  const int64_t ne = (int64_t)nslot * tb * 2;
  if (ne <= 0) return;
  WH_HIP_CHECK(hipMemsetAsync(hq, 0, ne * 8, s));
  if (ntask > 0 && max_rows > 0)
    hipLaunchKernelGGL(k_hist_csr, dim3((unsigned)((max_rows + 255) / 256), ntask), dim3(256), 0,
                       s, row_off, gbin, ridx, reinterpret_cast<const float2*>(gpair), qscale,
                       tasks, tb, reinterpret_cast<unsigned long long*>(hq));
  hipLaunchKernelGGL(k_hist_csr_fin, dim3(grid_for(ne, 256)), dim3(256), 0, s,
                     reinterpret_cast<const unsigned long long*>(hq), ne, qscale, hist);
}

void gbdt_split_csr(const double* hist, int64_t tb, const double* totals,
                    const int32_t* cut_off, const uint8_t* fvalid, int S, int F, double alpha,
                    double lambda, double mcw, double* cand, double* out, hipStream_t s) {
  if (S <= 0 || F <= 0) return;
  const SplitParam p{alpha, lambda, mcw};
  hipLaunchKernelGGL(k_split_csr_feat, dim3((unsigned)((F + 255) / 256), S), dim3(256), 0, s,
                     hist, tb, totals, cut_off, fvalid, F, p, cand);
  hipLaunchKernelGGL(k_split_csr_node, dim3((unsigned)S), dim3(256), 0, s, cand, F, out);
}

void gbdt_goleft_csr(const int64_t* row_off, const int32_t* fid, const int32_t* gbin,
                     const int32_t* cut_off, const int32_t* ridx, int64_t n,
                     const int32_t* pos_node, const int32_t* node_feat, const int32_t* node_bin,
                     const uint8_t* node_defl, int32_t* left, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_goleft_csr, dim3(grid_for(n, 256)), dim3(256), 0, s, row_off, fid, gbin,
                     cut_off, ridx, n, pos_node, node_feat, node_bin, node_defl, left);
}

void gbdt_predict_csr(const int64_t* row_off, const int32_t* fid, const float* val, int64_t n,
                      const int32_t* feat, const float* thr, const int32_t* left,
                      const int32_t* right, const uint8_t* defl, const float* leaf, float* margin,
                      hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_predict_csr, dim3(grid_for(n, 256)), dim3(256), 0, s, row_off, fid, val, n,
                     feat, thr, left, right, defl, leaf, margin);
}

}  // namespace wh
