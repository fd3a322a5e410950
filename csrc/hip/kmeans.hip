// Spherical k-means on MFMA (K17/K18 in SURVEY §2.5; reference
// learn/kmeans/kmeans.cc:108-130,171-190: for every row, argmax_k <c_k, x>
// over L2-normalised centroids, then per-cluster sums + counts).
//
// Assignment = X C^T with a fused row-argmax epilogue, never materialising
// the N x K score matrix:
//   * X is packed ONCE (it is static across iterations) into MFMA fragment
//     order for v_mfma_f32_32x32x2_f32 (exact fp32, lane l holds
//     X[row = l&31][k = 2s + (l>>5)] of k-step s), so every A-operand load is
//     one coalesced 256-byte wave access; a wave keeps its 32-row tile's
//     fragments in VGPRs for the whole sweep over the centroids.
//   * C is re-packed every iteration (K x F is tiny) into the same B-operand
//     order, 32 clusters per chunk, and streams through L2.
//   * per chunk each lane keeps a running (max, argmax) for its 16 output
//     rows; one cross-lane reduction per tile at the end (ties -> lowest k,
//     the reference's strict '>' scan order).
// Accumulation: one wave per row adds the row into its cluster's sum with
// 256-byte-contiguous float atomics (the chip-wide atomic rate shape).
#include <algorithm>
#include <cstdlib>

#include "wh_common.h"
#include "wh_kernels.h"

#include <cstdlib>

namespace wh {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void k_pack_x(const float* __restrict__ X, int64_t n, int f, int ks,
                         float* __restrict__ Xp) {
  // Xp[(tile*ks + s)*64 + lane] = X[tile*32 + (lane&31)][2s + (lane>>5)]
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t ntiles = (n + 31) / 32;
  if (t >= ntiles * ks * 64) return;
  const int lane = (int)(t & 63);
  const int64_t ts = t >> 6;
  const int s = (int)(ts % ks);
  const int64_t tile = ts / ks;
  const int64_t row = tile * 32 + (lane & 31);
  const int col = 2 * s + (lane >> 5);
  Xp[t] = (row < n && col < f) ? X[row * f + col] : 0.f;
}

__global__ void k_pack_c(const float* __restrict__ C, int k, int f, int ks, int nchunk,
                         float* __restrict__ Cp) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)nchunk * ks * 64) return;
  const int lane = (int)(t & 63);
  const int64_t ts = t >> 6;
  const int s = (int)(ts % ks);
  const int chunk = (int)(ts / ks);
  const int cl = chunk * 32 + (lane & 31);
  const int col = 2 * s + (lane >> 5);
  Cp[t] = (cl < k && col < f) ? C[(int64_t)cl * f + col] : 0.f;
}

// Block-tiled assignment for F <= 128 (KS <= 64 k-steps). A workgroup of 4
// waves owns 128 rows (each wave a 32-row tile, A fragments in VGPRs) and
// sweeps the centroids in chunks of 128 (4 subtiles of 32) staged in LDS,
// double-buffered: while the MFMAs consume chunk c from LDS, chunk c+1's
// global loads are in flight in registers. One B read per k-step is a
// ds_read_b128 holding the 4 subtiles' operands (LDS layout [s][lane][j]),
// so each A fragment feeds 4 independent accumulators (4 x 32x32 outputs);
// chunks arrive by LDS-DMA (no staging registers).
// Replaces a per-wave kernel that streamed every B operand from L2 (rocprof:
// 34 TF of the 157 TF fp32 MFMA peak at 10M x 128, k = 1000).
__global__ void k_pack_cn(const float* __restrict__ C, int k, int f, int ks, int nchunk, int nsub,
                          float* __restrict__ Cp) {
  // Cp[((chunk*ks + s)*64 + lane)*nsub + j] = C[chunk*32nsub + j*32 + (lane&31)][2s + (lane>>5)]
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)nchunk * ks * 64 * nsub) return;
  const int j = (int)(t % nsub);
  const int lane = (int)((t / nsub) & 63);
  const int64_t cs = t / nsub / 64;
  const int s = (int)(cs % ks);
  const int chunk = (int)(cs / ks);
  const int cl = chunk * 32 * nsub + j * 32 + (lane & 31);
  const int col = 2 * s + (lane >> 5);
  Cp[t] = (cl < k && col < f) ? C[(int64_t)cl * f + col] : 0.f;
}

template <int NSUB>
struct BVec;
template <>
struct BVec<4> { typedef float4 T; };
template <>
struct BVec<2> { typedef float2 T; };

template <int KS, int NSUB>
__global__ __launch_bounds__(256, 1) void k_assign_blk(const float* __restrict__ Xp, int64_t n,
                                                       const float* __restrict__ Cp, int nchunk,
                                                       int k, int32_t* __restrict__ assign,
                                                       float* __restrict__ score) {
  typedef typename BVec<NSUB>::T BT;
  constexpr int CH = 32 * NSUB;               // centroids per chunk
  constexpr int CF = KS * 64 * NSUB;          // floats per LDS chunk
  constexpr int PER = CF / 4 / 256;           // 16-byte DMA pieces per thread per chunk
  __shared__ float4 lds4[2 * CF / 4];         // 2 x KS*NSUB/4 KiB (128 KiB at KS 64, NSUB 4)
  float4* buf0 = lds4;
  float4* buf1 = lds4 + CF / 4;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t ntiles = (n + 31) / 32;
  const int64_t tile = (int64_t)blockIdx.x * 4 + wid;
  const bool live = tile < ntiles;
  float a[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) a[s] = live ? Xp[(tile * KS + s) * 64 + lane] : 0.f;
  float bv[16];
  int bk[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    bv[r] = -INFINITY;
    bk[r] = 0x7fffffff;
  }
  const float4* cp4 = reinterpret_cast<const float4*>(Cp);
  // chunk -> LDS with LDS-DMA (global_load_lds_dwordx4): the image is
  // lane-linear ([s][lane][j] in both), so each wave-instruction writes 1 KiB
  // at a wave-uniform base + lane * 16 B, with no staging registers
  auto stage = [&](float4* dst, const float4* src) {
#pragma unroll
    for (int i = 0; i < PER; ++i)
      __builtin_amdgcn_global_load_lds(
          src + i * 256 + threadIdx.x,
          (__attribute__((address_space(3))) void*)(dst + i * 256 + wid * 64), 16, 0, 0);
  };
  stage(buf0, cp4);
  __syncthreads();  // drains the DMA (vmcnt(0)) and publishes the chunk
  for (int c = 0; c < nchunk; ++c) {
    const float4* cur = (c & 1) ? buf1 : buf0;
    float4* nxt = (c & 1) ? buf0 : buf1;
    if (c + 1 < nchunk) stage(nxt, cp4 + (int64_t)(c + 1) * (CF / 4));
    f32x16 acc[NSUB];
#pragma unroll
    for (int j = 0; j < NSUB; ++j) acc[j] = f32x16{0.f};
    const BT* curb = reinterpret_cast<const BT*>(cur);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const BT b = curb[s * 64 + lane];
      const float* bf = reinterpret_cast<const float*>(&b);
#pragma unroll
      for (int j = 0; j < NSUB; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], bf[j], acc[j], 0, 0, 0);
    }
    const int col0 = c * CH + (lane & 31);
    // subtiles in increasing column order; strict '>' keeps the lowest k on ties
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int j = 0; j < NSUB; ++j)
        if (col0 + 32 * j < k && acc[j][r] > bv[r]) {
          bv[r] = acc[j][r];
          bk[r] = col0 + 32 * j;
        }
    }
    __syncthreads();  // next chunk landed; everyone is done with this one
  }
  if (!live) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float v = bv[r];
    int kk = bk[r];
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) {
      const float ov = __shfl_xor(v, o, 64);
      const int ok = __shfl_xor(kk, o, 64);
      if (ov > v || (ov == v && ok < kk)) {
        v = ov;
        kk = ok;
      }
    }
    if ((lane & 31) == 0) {
      const int64_t row = tile * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (row < n) {
        assign[row] = kk == 0x7fffffff ? 0 : kk;
        if (score) score[row] = v;
      }
    }
  }
}

template <int KS>
__global__ __launch_bounds__(256) void k_assign(const float* __restrict__ Xp, int64_t n,
                                                int ks_rt, const float* __restrict__ Cp,
                                                int nchunk, int k, int32_t* __restrict__ assign,
                                                float* __restrict__ score) {
  const int lane = threadIdx.x & 63;
  const int64_t tile = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t ntiles = (n + 31) / 32;
  if (tile >= ntiles) return;
  const int ks = KS > 0 ? KS : ks_rt;
  // A fragments resident in registers for the whole centroid sweep
  float a[KS > 0 ? KS : 1];
  if (KS > 0) {
#pragma unroll
    for (int s = 0; s < KS; ++s) a[s] = Xp[(tile * ks + s) * 64 + lane];
  }
  float bv[16];
  int bk[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    bv[r] = -INFINITY;
    bk[r] = 0x7fffffff;
  }
  for (int c = 0; c < nchunk; ++c) {
    f32x16 acc = {0.f};
    const float* bp = Cp + (int64_t)c * ks * 64 + lane;
    if (KS > 0) {
#pragma unroll
      for (int s = 0; s < KS; ++s)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s], bp[s * 64], acc, 0, 0, 0);
    } else {
      const float* ap = Xp + tile * ks * 64 + lane;
      for (int s = 0; s < ks; ++s)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ap[s * 64], bp[s * 64], acc, 0, 0, 0);
    }
    const int col = c * 32 + (lane & 31);
    if (col < k) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (acc[r] > bv[r]) {
          bv[r] = acc[r];
          bk[r] = col;
        }
      }
    }
  }
  // reduce over the 32 lanes that share each output row (lanes l, l^1 .. l^16)
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float v = bv[r];
    int kk = bk[r];
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) {
      const float ov = __shfl_xor(v, o, 64);
      const int ok = __shfl_xor(kk, o, 64);
      if (ov > v || (ov == v && ok < kk)) {
        v = ov;
        kk = ok;
      }
    }
    if ((lane & 31) == 0) {
      const int64_t row = tile * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (row < n) {
        assign[row] = kk == 0x7fffffff ? 0 : kk;
        if (score) score[row] = v;
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_accum(const float* __restrict__ X, int64_t n, int f,
                                               const int32_t* __restrict__ assign,
                                               float* __restrict__ sums) {
  // one wave per row: 256-byte contiguous float atomics into the cluster row
  const int lane = threadIdx.x & 63;
  const int64_t row = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (row >= n) return;
  const int kk = assign[row];
  float* dst = sums + (int64_t)kk * (f + 1);
  const float* src = X + row * f;
  for (int j = lane; j < f; j += 64) atomicAdd(dst + j, src[j]);
  if (lane == 0) atomicAdd(dst + f, 1.f);
}

// ---- sort-based accumulation ------------------------------------------
// sums[c] = sum of the rows assigned to c (+ count). One float atomic per
// row element (k_accum) is 1.28 G atomics for 10M x 128: 7 ms of atomic
// traffic per iteration, a quarter of the step. Instead the rows are bucketed
// by cluster (a counting sort: per-block LDS histograms -> one scan -> LDS
// cursors) and summed segment by segment in registers, flushing one row of
// atomics per (wave, cluster) boundary.
constexpr int kKmRows = 8192;     // rows per histogram / scatter block
constexpr int kKmMaxK = 16384;    // clusters the LDS histogram holds
constexpr int kKmSegRows = 256;   // sorted rows per wave in the segment sum
constexpr int kKmMaxT = 8;        // features per lane (f <= 512)

__global__ __launch_bounds__(256) void k_km_hist(const int32_t* __restrict__ assign, int64_t n,
                                                 int k, int nblk, int32_t* __restrict__ cnt) {
  __shared__ int32_t h[kKmMaxK];
  for (int i = threadIdx.x; i < k; i += 256) h[i] = 0;
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * kKmRows;
  const int64_t r1 = r0 + kKmRows < n ? r0 + kKmRows : n;
  for (int64_t r = r0 + threadIdx.x; r < r1; r += 256) atomicAdd(&h[assign[r]], 1);
  __syncthreads();
  for (int i = threadIdx.x; i < k; i += 256) cnt[(int64_t)i * nblk + blockIdx.x] = h[i];
}

__global__ __launch_bounds__(256) void k_km_scatter(const int32_t* __restrict__ assign, int64_t n,
                                                    int k, int nblk,
                                                    const int64_t* __restrict__ off,
                                                    int32_t* __restrict__ order,
                                                    int32_t* __restrict__ ocl) {
  __shared__ int32_t cur[kKmMaxK];
  for (int i = threadIdx.x; i < k; i += 256) cur[i] = (int32_t)off[(int64_t)i * nblk + blockIdx.x];
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * kKmRows;
  const int64_t r1 = r0 + kKmRows < n ? r0 + kKmRows : n;
  for (int64_t r = r0 + threadIdx.x; r < r1; r += 256) {
    const int c = assign[r];
    const int p = atomicAdd(&cur[c], 1);
    order[p] = (int32_t)r;
    ocl[p] = c;
  }
}

__global__ __launch_bounds__(256) void k_km_segsum(const float* __restrict__ X, int64_t n, int f,
                                                   const int32_t* __restrict__ order,
                                                   const int32_t* __restrict__ ocl,
                                                   float* __restrict__ sums) {
  const int lane = threadIdx.x & 63;
  const int64_t w = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int64_t p0 = w * kKmSegRows;
  if (p0 >= n) return;
  const int64_t p1 = p0 + kKmSegRows < n ? p0 + kKmSegRows : n;
  float acc[kKmMaxT];
#pragma unroll
  for (int t = 0; t < kKmMaxT; ++t) acc[t] = 0.f;
  int cur = -1;
  float cntc = 0.f;
  auto flush = [&]() {
    if (cur < 0) return;
    float* dst = sums + (int64_t)cur * (f + 1);
#pragma unroll
    for (int t = 0; t < kKmMaxT; ++t) {
      const int j = lane + 64 * t;
      if (j < f) atomicAdd(dst + j, acc[t]);
      acc[t] = 0.f;
    }
    if (lane == 0) atomicAdd(dst + f, cntc);
    cntc = 0.f;
  };
  for (int64_t b = p0; b < p1; b += 64) {
    // 64 sorted positions: one (row, cluster) pair per lane, then broadcast
    const bool ok = b + lane < p1;
    const int myrow = ok ? order[b + lane] : 0;
    const int mycl = ok ? ocl[b + lane] : -1;
    const int m = (int)(p1 - b < 64 ? p1 - b : 64);
    for (int i = 0; i < m; i += 4) {
      float v[4][kKmMaxT];
      int cl[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {  // four rows' loads in flight
        const int src = i + u < m ? i + u : i;
        const int row = __shfl(myrow, src, 64);
        cl[u] = i + u < m ? __shfl(mycl, src, 64) : -2;
        const float* xr = X + (int64_t)row * f;
#pragma unroll
        for (int t = 0; t < kKmMaxT; ++t) {
          const int j = lane + 64 * t;
          v[u][t] = j < f ? xr[j] : 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (cl[u] == -2) break;
        if (cl[u] != cur) {
          flush();
          cur = cl[u];
        }
#pragma unroll
        for (int t = 0; t < kKmMaxT; ++t) acc[t] += v[u][t];
        cntc += 1.f;
      }
    }
  }
  flush();
}

}  // namespace

// k-steps of 2 features; padded to the register-resident template widths so
// the packed X / C layouts and the kernel agree (padding columns are zero)
int kmeans_ks(int f) {
  const int ks = (f + 1) / 2;
  if (ks <= 8) return 8;
  if (ks <= 16) return 16;
  if (ks <= 32) return 32;
  if (ks <= 64) return 64;
  return ks;
}

void kmeans_pack_x(const float* X, int64_t n, int f, float* Xp, hipStream_t s) {
  const int ks = kmeans_ks(f);
  const int64_t total = (n + 31) / 32 * ks * 64;
  if (total <= 0) return;
  hipLaunchKernelGGL(k_pack_x, dim3(grid_for(total, 256)), dim3(256), 0, s, X, n, f, ks, Xp);
}

// the block-tiled kernel handles F <= 128; wider rows use the streamed kernel.
// NSUB = centroid subtiles of 32 per LDS chunk: 2 (measured 32.8 vs 27.2
// iter/s against 4 at 10M x 128, k=1000 -- two 32-wide subtiles keep more
// waves resident per CU than four).
static bool blocked(int f) { return kmeans_ks(f) <= 64; }
static constexpr int nsub() { return 2; }

int64_t kmeans_cp_elems(int k, int f) {
  const int ks = kmeans_ks(f);
  if (blocked(f)) {
    const int ch = 32 * nsub();
    return (int64_t)((k + ch - 1) / ch) * ks * 64 * nsub();
  }
  return (int64_t)((k + 31) / 32) * ks * 64;
}

void kmeans_pack_c(const float* C, int k, int f, float* Cp, hipStream_t s) {
  const int ks = kmeans_ks(f);
  if (blocked(f)) {
    const int ns = nsub(), nchunk = (k + 32 * ns - 1) / (32 * ns);
    const int64_t total = (int64_t)nchunk * ks * 64 * ns;
    hipLaunchKernelGGL(k_pack_cn, dim3(grid_for(total, 256)), dim3(256), 0, s, C, k, f, ks,
                       nchunk, ns, Cp);
    return;
  }
  const int nchunk = (k + 31) / 32;
  const int64_t total = (int64_t)nchunk * ks * 64;
  hipLaunchKernelGGL(k_pack_c, dim3(grid_for(total, 256)), dim3(256), 0, s, C, k, f, ks, nchunk,
                     Cp);
}

template <int NS>
static void launch_blk(int ks, dim3 grid, hipStream_t s, const float* Xp, int64_t n,
                       const float* Cp, int nchunk, int k, int32_t* assign, float* score) {
  const dim3 block(256);
  switch (ks) {
    case 8:
      hipLaunchKernelGGL((k_assign_blk<8, NS>), grid, block, 0, s, Xp, n, Cp, nchunk, k, assign,
                         score);
      break;
    case 16:
      hipLaunchKernelGGL((k_assign_blk<16, NS>), grid, block, 0, s, Xp, n, Cp, nchunk, k, assign,
                         score);
      break;
    case 32:
      hipLaunchKernelGGL((k_assign_blk<32, NS>), grid, block, 0, s, Xp, n, Cp, nchunk, k, assign,
                         score);
      break;
    default:
      hipLaunchKernelGGL((k_assign_blk<64, NS>), grid, block, 0, s, Xp, n, Cp, nchunk, k, assign,
                         score);
      break;
  }
}

void kmeans_assign(const float* Xp, int64_t n, int f, const float* Cp, int k, int32_t* assign,
                   float* score, hipStream_t s) {
  if (n <= 0) return;
  const int ks = kmeans_ks(f);
  const int64_t ntiles = (n + 31) / 32;
  if (blocked(f)) {
    const int ns = nsub(), nchunk = (k + 32 * ns - 1) / (32 * ns);
    const dim3 grid((unsigned)((ntiles + 3) / 4));
    launch_blk<nsub()>(ks, grid, s, Xp, n, Cp, nchunk, k, assign, score);
    return;
  }
  const int nchunk = (k + 31) / 32;
  const dim3 grid(grid_for(ntiles * 64, 256)), block(256);
  hipLaunchKernelGGL(k_assign<0>, grid, block, 0, s, Xp, n, ks, Cp, nchunk, k, assign, score);
}

void kmeans_accum(const float* X, int64_t n, int f, const int32_t* assign, float* sums,
                  hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_accum, dim3(grid_for(n * 64, 256)), dim3(256), 0, s, X, n, f, assign, sums);
}

namespace {
// Centroid update in one launch, one block per centroid (reference
// learn/kmeans/kmeans.cc: divide the summed rows by the count, then L2
// normalise): c = sums[r, f]; v = sums[r, :f] / c, or the previous centroid
// when the cluster is empty; out[r] = v * (float)(1 / ||v||) with the norm in
// double and rows of norm < 1e-6 left unscaled (models/kmeans.py
// normalize_rows); *nempty += the empty clusters. Replaces ~10 small torch
// launches per iteration.
__global__ __launch_bounds__(128) void k_km_update(const float* __restrict__ sums,
                                                   const float* __restrict__ C, int f,
                                                   float* __restrict__ out,
                                                   unsigned long long* nempty) {
  __shared__ double sh[2];
  const int r = blockIdx.x;
  const float c = sums[(int64_t)r * (f + 1) + f];
  const bool empty = c == 0.f;
  double ss = 0;
  for (int j = threadIdx.x; j < f; j += 128) {
    const float v = empty ? C[(int64_t)r * f + j] : sums[(int64_t)r * (f + 1) + j] / c;
    ss += (double)v * v;
  }
  ss = wave_sum_d(ss);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = ss;
  __syncthreads();
  const double nrm = sqrt(sh[0] + sh[1]);
  const float scale = nrm < 1e-6 ? 1.f : (float)(1.0 / nrm);
  for (int j = threadIdx.x; j < f; j += 128) {
    const float v = empty ? C[(int64_t)r * f + j] : sums[(int64_t)r * (f + 1) + j] / c;
    out[(int64_t)r * f + j] = v * scale;
  }
  if (threadIdx.x == 0 && empty) atomicAdd(nempty, 1ull);
}
}  // namespace

void kmeans_update(const float* sums, const float* C, int k, int f, float* out,
                   unsigned long long* nempty, hipStream_t s) {
  if (k <= 0) return;
  hipLaunchKernelGGL(k_km_update, dim3((unsigned)k), dim3(128), 0, s, sums, C, f, out, nempty);
}

// ---- sparse (CSR) input ---------------------------------------------------
// The reference clusters libsvm rows directly (learn/kmeans/kmeans.cc:108-130:
// Cos() walks a Row<unsigned>, only the K x F centroids are dense). Here the
// rows stay CSR in HBM; the centroids are read through their transpose Ct
// [F, Kp] (Kp = K rounded up to 4), so each non-zero (j, x) of a row gathers
// ONE contiguous centroid column Ct[j, :] -- float4 per lane, 1 KB per wave
// instruction -- and the wave accumulates x * Ct[j, k] for its row in double
// (the reference's `double rdot`), 4 * PER clusters per lane per pass. The
// argmax (ties: the smaller k, the reference's strict `>`) is a wave
// reduction; K beyond one pass re-walks the row per pass of 256 * PER
// clusters. ||x|| does not change a row's argmax and is not computed.
namespace {
constexpr int kCsrRows = 4;  // rows (waves) per 256-thread block

__device__ __forceinline__ bool km_better(double v, int k, double bv, int bk) {
  return v > bv || (v == bv && k < bk);
}

template <int PER>
__global__ __launch_bounds__(256) void k_assign_csr(const int64_t* __restrict__ off,
                                                    const int32_t* __restrict__ col,
                                                    const float* __restrict__ val, int64_t n,
                                                    const float* __restrict__ Ct, int K, int Kp,
                                                    int32_t* __restrict__ assign) {
  const int64_t row = (int64_t)blockIdx.x * kCsrRows + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  const int64_t b = off[row], e = off[row + 1];
  double best = -INFINITY;
  int bk = 0x7fffffff;
  for (int k0 = 0; k0 < K; k0 += 256 * PER) {
    double acc[PER][4];
#pragma unroll
    for (int g = 0; g < PER; ++g)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[g][q] = 0.0;
    for (int64_t j0 = b; j0 < e; j0 += 64) {
      const int m = e - j0 < 64 ? (int)(e - j0) : 64;
      const int c = lane < m ? col[j0 + lane] : 0;
      const float x = lane < m ? (val ? val[j0 + lane] : 1.f) : 0.f;
      // kCsrU non-zeros per step: their centroid-column loads are all issued
      // before the first accumulation (one dependent round trip per step)
      constexpr int kCsrU = 4;
      for (int t0 = 0; t0 < m; t0 += kCsrU) {
        float4 v[kCsrU][PER];
        double xj[kCsrU];
#pragma unroll
        for (int u = 0; u < kCsrU; ++u) {
          const int t = t0 + u < m ? t0 + u : m - 1;
          const int cj = __shfl(c, t, 64);
          xj[u] = t0 + u < m ? (double)__shfl(x, t, 64) : 0.0;
          const float* cr = Ct + (int64_t)cj * Kp + k0;
#pragma unroll
          for (int g = 0; g < PER; ++g) {
            const int kk = 4 * (lane + 64 * g);
            v[u][g] = k0 + kk < Kp ? *reinterpret_cast<const float4*>(cr + kk)
                                   : make_float4(0.f, 0.f, 0.f, 0.f);
          }
        }
#pragma unroll
        for (int u = 0; u < kCsrU; ++u)
#pragma unroll
          for (int g = 0; g < PER; ++g) {
            acc[g][0] += (double)v[u][g].x * xj[u];
            acc[g][1] += (double)v[u][g].y * xj[u];
            acc[g][2] += (double)v[u][g].z * xj[u];
            acc[g][3] += (double)v[u][g].w * xj[u];
          }
      }
    }
#pragma unroll
    for (int g = 0; g < PER; ++g)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int k = k0 + 4 * (lane + 64 * g) + q;
        if (k < K && km_better(acc[g][q], k, best, bk)) {
          best = acc[g][q];
          bk = k;
        }
      }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double v2 = __shfl_xor(best, o, 64);
    const int k2 = __shfl_xor(bk, o, 64);
    if (km_better(v2, k2, best, bk)) {
      best = v2;
      bk = k2;
    }
  }
  if (lane == 0) assign[row] = bk;
}

// sums[a, col] += x and sums[a, F] += 1 for each row (a = its cluster)
__global__ __launch_bounds__(256) void k_accum_csr(const int64_t* __restrict__ off,
                                                   const int32_t* __restrict__ col,
                                                   const float* __restrict__ val, int64_t n,
                                                   const int32_t* __restrict__ assign, int F,
                                                   float* __restrict__ sums) {
  const int64_t row = (int64_t)blockIdx.x * kCsrRows + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  const int64_t b = off[row], e = off[row + 1];
  float* sr = sums + (int64_t)assign[row] * (F + 1);
  if (lane == 0) atomicAdd(sr + F, 1.f);
  for (int64_t j = b + lane; j < e; j += 64) atomicAdd(sr + col[j], val ? val[j] : 1.f);
}
}  // namespace

int kmeans_csr_per(int K) {
  return K <= 256 ? 1 : K <= 512 ? 2 : K <= 1024 ? 4 : 8;
}

void kmeans_assign_csr(const int64_t* off, const int32_t* col, const float* val, int64_t n,
                       const float* Ct, int K, int Kp, int32_t* assign, hipStream_t s) {
  if (n <= 0) return;
  const dim3 grid((unsigned)((n + kCsrRows - 1) / kCsrRows)), block(256);
  switch (kmeans_csr_per(K)) {
    case 1: hipLaunchKernelGGL(k_assign_csr<1>, grid, block, 0, s, off, col, val, n, Ct, K, Kp, assign); break;
    case 2: hipLaunchKernelGGL(k_assign_csr<2>, grid, block, 0, s, off, col, val, n, Ct, K, Kp, assign); break;
    case 4: hipLaunchKernelGGL(k_assign_csr<4>, grid, block, 0, s, off, col, val, n, Ct, K, Kp, assign); break;
    default: hipLaunchKernelGGL(k_assign_csr<8>, grid, block, 0, s, off, col, val, n, Ct, K, Kp, assign); break;
  }
}

void kmeans_accum_csr(const int64_t* off, const int32_t* col, const float* val, int64_t n,
                      const int32_t* assign, int F, float* sums, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_accum_csr, dim3((unsigned)((n + kCsrRows - 1) / kCsrRows)), dim3(256), 0,
                     s, off, col, val, n, assign, F, sums);
}

}  // namespace wh

namespace wh {

int64_t kmeans_accum_scratch(int64_t n, int k) {
  // int32: cnt [k * nblk] ; int64: off [k * nblk + 1] + scan tmp ; int32: order, ocl [n]
  const int64_t nblk = (n + kKmRows - 1) / kKmRows;
  return nblk * k * 4 + (nblk * k + 1) * 8 + scan_tmp_elems(nblk * k) * 8 + 2 * n * 4 + 64;
}

bool kmeans_accum_sorted(const float* X, int64_t n, int f, int k, const int32_t* assign,
                         float* sums, void* scratch, hipStream_t s) {
  if (n <= 0) return true;
  if (k > kKmMaxK || f > 64 * kKmMaxT) return false;
  const int64_t nblk = (n + kKmRows - 1) / kKmRows;
  char* p = static_cast<char*>(scratch);
  int32_t* cnt = reinterpret_cast<int32_t*>(p);
  p += nblk * k * 4;
  p = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(p) + 7) & ~(uintptr_t)7);
  int64_t* off = reinterpret_cast<int64_t*>(p);
  p += (nblk * k + 1) * 8;
  int64_t* stmp = reinterpret_cast<int64_t*>(p);
  p += scan_tmp_elems(nblk * k) * 8;
  int32_t* order = reinterpret_cast<int32_t*>(p);
  int32_t* ocl = order + n;
  hipLaunchKernelGGL(k_km_hist, dim3((unsigned)nblk), dim3(256), 0, s, assign, n, k, (int)nblk,
                     cnt);
  scan_i32(cnt, off, nblk * k, stmp, s);
  hipLaunchKernelGGL(k_km_scatter, dim3((unsigned)nblk), dim3(256), 0, s, assign, n, k, (int)nblk,
                     off, order, ocl);
  const int64_t waves = (n + kKmSegRows - 1) / kKmSegRows;
  hipLaunchKernelGGL(k_km_segsum, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, X, n, f,
                     order, ocl, sums);
  return true;
}

}  // namespace wh

// ---- split-precision assignment (bf16 x 3 on the bf16 MFMA) ---------------
// x.c = (xh + xl).(ch + cl) ~ xh.ch + xh.cl + xl.ch with hi = bf16(v), lo =
// bf16(v - hi): three v_mfma_f32_32x32x16_bf16 per k-step of 16 features, at
// 16x the fp32 MFMA rate (5.3x the arithmetic for 3 products). The dropped /
// rounded terms are bounded by 3 * 2^-18 * |x| |c| plus the fp32 accumulation
// (eps * |x|, |c| <= 1 for the normalised centroids), so a row whose best
// and second-best approximate scores differ by at least 2 eps |x| has the
// exact argmax; every other row (a near-tie) is re-scored in fp32 by
// k_refine_rows. The result is the exact fp32 argmax, as the fp32 kernel's.
namespace wh {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ uint32_t bf16_rne(float v) {
  const uint32_t u = __float_as_uint(v);
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

// hi/lo bf16 pair of v packed as {hi, lo} 16-bit halves
__device__ __forceinline__ void split_bf16(float v, uint32_t& hi, uint32_t& lo) {
  hi = bf16_rne(v);
  lo = bf16_rne(v - __uint_as_float(hi << 16));
}

// Xp3[((tile * ks + s) * 2 + hl) * 64 + lane] = 8 bf16 (uint4): lane l holds
// X[row = tile*32 + (l&31)][16 s + 8 (l>>5) + j], j = 0..7 (the A-operand map
// of mfma_f32_32x32x16_bf16)
__global__ void k_pack_x3(const float* __restrict__ X, int64_t n, int f, int ks,
                          uint4* __restrict__ Xp) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t ntiles = (n + 31) / 32;
  if (t >= ntiles * ks * 64) return;
  const int lane = (int)(t & 63);
  const int64_t ts = t >> 6;
  const int s = (int)(ts % ks);
  const int64_t tile = ts / ks;
  const int64_t row = tile * 32 + (lane & 31);
  uint32_t h[8], l[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int col = 16 * s + 8 * (lane >> 5) + j;
    const float v = (row < n && col < f) ? X[row * f + col] : 0.f;
    split_bf16(v, h[j], l[j]);
  }
  const int64_t base = (tile * ks + s) * 2 * 64 + lane;
  Xp[base] = make_uint4(h[0] | h[1] << 16, h[2] | h[3] << 16, h[4] | h[5] << 16, h[6] | h[7] << 16);
  Xp[base + 64] =
      make_uint4(l[0] | l[1] << 16, l[2] | l[3] << 16, l[4] | l[5] << 16, l[6] | l[7] << 16);
}

// Cp3[(((chunk * ks + s) * nsub + j) * 2 + hl) * 64 + lane]: the B-operand map,
// centroid chunk * 32 nsub + 32 j + (lane & 31)
__global__ void k_pack_c3(const float* __restrict__ C, int k, int f, int ks, int nchunk, int nsub,
                          uint4* __restrict__ Cp) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)nchunk * ks * nsub * 64) return;
  const int lane = (int)(t & 63);
  int64_t q = t >> 6;
  const int j = (int)(q % nsub);
  q /= nsub;
  const int s = (int)(q % ks);
  const int chunk = (int)(q / ks);
  const int cl = chunk * 32 * nsub + 32 * j + (lane & 31);
  uint32_t h[8], l[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int col = 16 * s + 8 * (lane >> 5) + e;
    const float v = (cl < k && col < f) ? C[(int64_t)cl * f + col] : 0.f;
    split_bf16(v, h[e], l[e]);
  }
  const int64_t base = ((((int64_t)chunk * ks + s) * nsub + j) * 2) * 64 + lane;
  Cp[base] = make_uint4(h[0] | h[1] << 16, h[2] | h[3] << 16, h[4] | h[5] << 16, h[6] | h[7] << 16);
  Cp[base + 64] =
      make_uint4(l[0] | l[1] << 16, l[2] | l[3] << 16, l[4] | l[5] << 16, l[6] | l[7] << 16);
}

__device__ __forceinline__ bf16x8 as_bf16x8(uint4 v) { return __builtin_bit_cast(bf16x8, v); }

// 8 waves (256 rows) share each centroid chunk, streamed through a 3-slot
// LDS ring by LDS-DMA two chunks ahead: a chunk is only 48 MFMAs per wave
// (~0.6 us), less than an L2 round trip, so a double buffer drained by a
// full __syncthreads left the matrix pipe idle most of the time (21 ms/iter).
constexpr int kX3Waves = 8;
constexpr int kX3Threads = 64 * kX3Waves;

//
// PIPE: each chunk's MFMAs in two halves of NSUB / 2 subtiles, the top-2
// epilogue of one half issued between the other half's MFMAs (the previous
// chunk's second half under this chunk's first, this chunk's first under
// its second). Without it every chunk ends in a dependent epilogue: the
// VALU waits for the MFMA chain to drain, and the two waves of a SIMD --
// released together by the chunk barrier -- drain and rank at the same
// time, idling the matrix pipe (the MFMAs alone take 2.9 of the kernel's
// 8.0 ms at 10M x 128, k = 1000: profiles/round6_kmeans.txt). The B
// operands of the next k-step are loaded before the current one's MFMAs.
// Same accumulators (the pending half is carried across the chunk
// boundary), same result.
template <int KS, int NSUB, int SLOTS, bool PIPE>
__global__ __launch_bounds__(kX3Threads, 1) void k_assign_x3(const uint4* __restrict__ Xp,
                                                             const float* __restrict__ xnorm,
                                                             int64_t n,
                                                             const uint4* __restrict__ Cp,
                                                             int nchunk, int k, float eps,
                                                             int32_t* __restrict__ assign,
                                                             float* __restrict__ score,
                                                             int32_t* __restrict__ amb) {
  constexpr int CH = 32 * NSUB;
  constexpr int CF = KS * NSUB * 2 * 64;  // uint4 per chunk
  constexpr int PER = CF / kX3Threads;    // 16-byte DMA pieces per thread per chunk
  static_assert(PER * kX3Threads == CF, "chunk must split evenly");
  __shared__ uint4 lds[SLOTS * CF];
  __shared__ uint4 pf_sink[kX3Threads];  // L2-prefetch DMA target, never read
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t ntiles = (n + 31) / 32;
  const int64_t ngroups = (ntiles + kX3Waves - 1) / kX3Waves;
  // persistent: the workgroup walks row groups blockIdx.x, + gridDim.x, ...;
  // the C ring runs over the global chunk sequence q (chunk q % nchunk), so it
  // never drains between groups. The next group's A fragments are pulled into
  // L2 during the current group's last chunk (LDS-DMA into a scratch slot: no
  // registers held; VGPRs are at 222 of 256) and loaded into the A registers
  // right after the last chunk's MFMAs, under the top-2 epilogue (a fresh
  // workgroup per group left the matrix pipe idle for an HBM round trip and
  // the DMA prologue of every group)
  const int64_t mygroups =
      blockIdx.x < ngroups ? (ngroups - 1 - blockIdx.x) / gridDim.x + 1 : 0;
  const int64_t total = mygroups * nchunk;
  auto stage = [&](int slot, int c) {
    const uint4* src = Cp + (int64_t)c * CF;
    uint4* dst = lds + slot * CF;
#pragma unroll
    for (int i = 0; i < PER; ++i)
      __builtin_amdgcn_global_load_lds(
          src + i * kX3Threads + threadIdx.x,
          (__attribute__((address_space(3))) void*)(dst + i * kX3Threads + wid * 64), 16, 0, 0);
  };
  auto load_a = [&](int64_t g, bf16x8 (&h)[KS], bf16x8 (&l)[KS]) {
    const int64_t t = g * kX3Waves + wid;
    const bool lv = g < ngroups && t < ntiles;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int64_t b = (t * KS + s) * 2 * 64 + lane;
      h[s] = as_bf16x8(lv ? Xp[b] : make_uint4(0, 0, 0, 0));
      l[s] = as_bf16x8(lv ? Xp[b + 64] : make_uint4(0, 0, 0, 0));
    }
  };
  auto prefetch_a = [&](int64_t g) {
    const int64_t t = g * kX3Waves + wid;
    if (g >= ngroups || t >= ntiles) return;
#pragma unroll
    for (int i = 0; i < 2 * KS; ++i)
      __builtin_amdgcn_global_load_lds(
          Xp + t * KS * 2 * 64 + i * 64 + lane,
          (__attribute__((address_space(3))) void*)(pf_sink + wid * 64), 16, 0, 0);
  };
  bf16x8 ah[KS], al[KS];
  int64_t grp = blockIdx.x;
  load_a(grp, ah, al);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // A fragments before the DMA count
  if (total > 0) stage(0, 0);
  if (SLOTS == 3 && total > 1) stage(1, 1 % nchunk);
  float b1[16], b2[16];
  int i1[16];
  // (padded centroid columns >= k start their accumulators at -1e30, so no
  // per-score bounds test is needed; 5 VALU per score)
  auto top2 = [&](const f32x16 (&sc)[NSUB], int cbase, int j0 = 0, int j1 = NSUB) {
    const int col0 = cbase + (lane & 31);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int j = j0; j < j1; ++j) {
        const float v = sc[j][r];
        const bool nb = v > b1[r];
        b2[r] = fmaxf(b2[r], fminf(b1[r], v));
        i1[r] = nb ? col0 + 32 * j : i1[r];
        b1[r] = fmaxf(b1[r], v);
      }
    }
  };
  // MFMAs of subtiles [j0, j1) of chunk c with the ranking of the OTHER
  // half (columns from rbase) between them, in program order (sched_barrier
  // fences: left alone the compiler hoists the whole VALU block after the
  // MFMAs); the B operands double-buffered in registers one k-step ahead
  auto mfma_rank = [&](f32x16 (&acc)[NSUB], const uint4* cur, int c, int j0, int rbase) {
    constexpr int HN = NSUB / 2;
    const int o0 = j0 == 0 ? HN : 0;  // the other half's subtiles [o0, o0 + HN)
    constexpr int NU = 16 * HN;       // its score updates, spread over the groups
    constexpr int PER_G = (NU + 3 * KS - 1) / (3 * KS);
    const int col0 = rbase + (lane & 31);
    auto rank_upd = [&](int u) {
      if (u >= NU) return;
      const int r = u / HN, j = o0 + u % HN;
      const float v = acc[j][r];
      const bool nb = v > b1[r];
      b2[r] = fmaxf(b2[r], fminf(b1[r], v));
      i1[r] = nb ? col0 + 32 * j : i1[r];
      b1[r] = fmaxf(b1[r], v);
    };
#pragma unroll
    for (int jj = 0; jj < HN; ++jj) {
      const float init = c * CH + 32 * (j0 + jj) + (lane & 31) < k ? 0.f : -1e30f;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[j0 + jj][r] = init;
    }
    bf16x8 bh[2][HN], bl[2][HN];
    auto load_b = [&](int s, int buf) {
#pragma unroll
      for (int jj = 0; jj < HN; ++jj) {
        bh[buf][jj] = as_bf16x8(cur[((s * NSUB + j0 + jj) * 2) * 64 + lane]);
        bl[buf][jj] = as_bf16x8(cur[((s * NSUB + j0 + jj) * 2 + 1) * 64 + lane]);
      }
    };
    load_b(0, 0);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if (s + 1 < KS) load_b(s + 1, (s + 1) & 1);
#pragma unroll
      for (int g = 0; g < 3; ++g) {
#pragma unroll
        for (int jj = 0; jj < HN; ++jj)
          acc[j0 + jj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              g == 2 ? al[s] : ah[s], g == 1 ? bl[s & 1][jj] : bh[s & 1][jj], acc[j0 + jj], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < PER_G; ++t) rank_upd((s * 3 + g) * PER_G + t);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  f32x16 acc[NSUB];
#pragma unroll
  for (int j = 0; j < NSUB; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = -INFINITY;
  int64_t q = 0;
  for (; grp < ngroups; grp += gridDim.x) {
    const int64_t tile = grp * kX3Waves + wid;
    const bool live = tile < ntiles;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      b1[r] = -INFINITY;
      b2[r] = -INFINITY;
      i1[r] = 0x7fffffff;
    }
    for (int c = 0; c < nchunk; ++c, ++q) {
      // this wave's pieces of chunk q have landed once at most the next
      // chunk's PER pieces are outstanding; the barrier makes every wave's
      // pieces visible and marks the slot of chunk q-1 free for chunk q+2
      if (SLOTS == 3 && q + 1 < total) {
        static_assert(PER == 1 || PER == 2 || PER == 4 || PER == 8, "vmcnt immediates below");
        if (PER == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else if (PER == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else if (PER == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      // the next group's A fragments into L2, ahead of the C DMA (the wait
      // above -- all but the newest C pieces -- covers them a chunk later)
      if (c == nchunk - 1 && grp + gridDim.x < ngroups) prefetch_a(grp + gridDim.x);
#if !defined(WH_X3_VARIANT) || WH_X3_VARIANT != 2
      if (q + SLOTS - 1 < total) stage((int)((q + SLOTS - 1) % SLOTS), (int)((q + SLOTS - 1) % nchunk));
#endif
#if defined(WH_X3_VARIANT) && WH_X3_VARIANT == 2
      const uint4* cur = lds;  // (microbench: chunk 0 only, no DMA in the loop)
#else
      const uint4* cur = lds + (q % SLOTS) * CF;
#endif
      if constexpr (PIPE) {
        constexpr int H = NSUB / 2;
        mfma_rank(acc, cur, c, 0, (c > 0 ? c - 1 : 0) * CH);  // + the previous chunk's 2nd half
        mfma_rank(acc, cur, c, H, c * CH);                    // + this chunk's first half
        if (c == nchunk - 1 && grp + gridDim.x < ngroups) load_a(grp + gridDim.x, ah, al);
        if (c == nchunk - 1) {  // the group's last half, then -inf for the next group
          top2(acc, c * CH, H, NSUB);
#pragma unroll
          for (int j = H; j < NSUB; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[j][r] = -INFINITY;
        }
        continue;
      }
#pragma unroll
      for (int j = 0; j < NSUB; ++j) {
        const float init = c * CH + 32 * j + (lane & 31) < k ? 0.f : -1e30f;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = init;
      }
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        bf16x8 ch[NSUB], cl[NSUB];
#pragma unroll
        for (int j = 0; j < NSUB; ++j) {
          ch[j] = as_bf16x8(cur[((s * NSUB + j) * 2) * 64 + lane]);
          cl[j] = as_bf16x8(cur[((s * NSUB + j) * 2 + 1) * 64 + lane]);
        }
        // independent accumulators interleaved between dependent MFMAs
#pragma unroll
        for (int j = 0; j < NSUB; ++j)
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[s], ch[j], acc[j], 0, 0, 0);
#pragma unroll
        for (int j = 0; j < NSUB; ++j)
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[s], cl[j], acc[j], 0, 0, 0);
#pragma unroll
        for (int j = 0; j < NSUB; ++j)
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[s], ch[j], acc[j], 0, 0, 0);
      }
      // after the group's last MFMAs the A registers are free: the next
      // group's fragments (L2 hits) load under the epilogue
      if (c == nchunk - 1 && grp + gridDim.x < ngroups) load_a(grp + gridDim.x, ah, al);
#if defined(WH_X3_VARIANT) && WH_X3_VARIANT == 3
      // (microbench: a 1-VALU epilogue that keeps every accumulator live)
#pragma unroll
      for (int r = 0; r < 16; ++r)
#pragma unroll
        for (int j = 0; j < NSUB; ++j) b1[r] = fmaxf(b1[r], acc[j][r]);
#elif !defined(WH_X3_VARIANT) || WH_X3_VARIANT != 1
      top2(acc, c * CH);
#else
      if (acc[0][0] == 12345.f) b1[0] = 1.f;  // (microbench: no epilogue)
#endif
    }
    if (live) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float v1 = b1[r], v2 = b2[r];
        int kk = i1[r];
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) {
          const float o1 = __shfl_xor(v1, o, 64), o2 = __shfl_xor(v2, o, 64);
          const int ok = __shfl_xor(kk, o, 64);
          if (o1 > v1 || (o1 == v1 && ok < kk)) {
            v2 = fmaxf(v1, o2);
            v1 = o1;
            kk = ok;
          } else {
            v2 = fmaxf(v2, o1);
          }
        }
        if ((lane & 31) == 0) {
          const int64_t row = tile * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (row < n) {
            assign[row] = kk == 0x7fffffff ? 0 : kk;
            if (score) score[row] = v1;
#if defined(WH_X3_VARIANT)
            if (false) {  // (timing microbench: its scores are not the real ones)
#else
            if (!(v1 - v2 >= 2.f * eps * xnorm[row])) {  // a near-tie: exact re-score
#endif
              const int qq = atomicAdd(amb, 1);
              amb[1 + qq] = (int32_t)row;
            }
          }
        }
      }
    }
  }
}

// exact fp32 argmax over all k centroids for the near-tie rows: a wave takes
// 4 listed rows (their features in LDS, broadcast) and lane l the centroids
// l, l + 64, ... of the transposed C (coalesced 256-byte loads, each shared by
// the 4 rows); persistent over the device-counted list; ties -> lowest index.
constexpr int kRefRows = 4;
constexpr int kRefMaxF = 128;

__global__ void k_transpose_c(const float* __restrict__ C, int k, int f, float* __restrict__ CT) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)k * f) return;
  const int c = (int)(t / f), e = (int)(t % f);
  CT[(int64_t)e * k + c] = C[t];
}

__global__ __launch_bounds__(256) void k_refine_rows(const float* __restrict__ X, int f,
                                                     const float* __restrict__ CT, int k,
                                                     const int32_t* __restrict__ amb,
                                                     int32_t* __restrict__ assign,
                                                     float* __restrict__ score) {
  __shared__ float sx[4][kRefRows][kRefMaxF];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int cnt = amb[0];
  const int ngroups = (cnt + kRefRows - 1) / kRefRows;
  for (int g = blockIdx.x * 4 + wid; g < ngroups; g += gridDim.x * 4) {
    int64_t rows[kRefRows];
#pragma unroll
    for (int q = 0; q < kRefRows; ++q) {
      const int i = g * kRefRows + q;
      rows[q] = i < cnt ? amb[1 + i] : -1;
      for (int e = lane; e < kRefMaxF; e += 64)
        sx[wid][q][e] = (rows[q] >= 0 && e < f) ? X[rows[q] * f + e] : 0.f;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float bv[kRefRows];
    int bi[kRefRows];
#pragma unroll
    for (int q = 0; q < kRefRows; ++q) {
      bv[q] = -INFINITY;
      bi[q] = 0x7fffffff;
    }
    for (int c0 = 0; c0 < k; c0 += 64 * 4) {
      float d[kRefRows][4];
#pragma unroll
      for (int q = 0; q < kRefRows; ++q)
#pragma unroll
        for (int u = 0; u < 4; ++u) d[q][u] = 0.f;
      for (int e = 0; e < f; ++e) {
        float cv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int c = c0 + u * 64 + lane;
          cv[u] = c < k ? CT[(int64_t)e * k + c] : 0.f;
        }
#pragma unroll
        for (int q = 0; q < kRefRows; ++q) {
          const float xe = sx[wid][q][e];
#pragma unroll
          for (int u = 0; u < 4; ++u) d[q][u] = fmaf(xe, cv[u], d[q][u]);
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {  // centroid index increases with u: '>' keeps the lowest
        const int c = c0 + u * 64 + lane;
        if (c < k) {
#pragma unroll
          for (int q = 0; q < kRefRows; ++q)
            if (d[q][u] > bv[q]) {
              bv[q] = d[q][u];
              bi[q] = c;
            }
        }
      }
    }
#pragma unroll
    for (int q = 0; q < kRefRows; ++q) {
      float v = bv[q];
      int kk = bi[q];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(v, o, 64);
        const int ok = __shfl_xor(kk, o, 64);
        if (ov > v || (ov == v && ok < kk)) {
          v = ov;
          kk = ok;
        }
      }
      if (lane == 0 && rows[q] >= 0) {
        assign[rows[q]] = kk == 0x7fffffff ? 0 : kk;
        if (score) score[rows[q]] = v;
      }
    }
  }
}

#ifndef WH_X3_NSUB
#define WH_X3_NSUB 4
#endif
constexpr int kX3Nsub = WH_X3_NSUB;
constexpr int kX3Slots = kX3Nsub == 4 ? 2 : 3;  // LDS ring: SLOTS x (KS * NSUB * 2 KiB)

// the pipelined epilogue (PIPE) always; the unpipelined kernel only in the
// timing microbench builds (-DWH_X3_VARIANT=0..3, tools/variant_so.sh:
// 1 no epilogue, 2 no C DMA, 3 a one-VALU epilogue)
bool x3_pipe() {
#if defined(WH_X3_VARIANT)
  return false;
#else
  return true;
#endif
}

int x3_ks(int f) {  // k-steps of 16 features, padded to the template widths
  const int ks = (f + 15) / 16;
  return ks <= 2 ? 2 : ks <= 4 ? 4 : 8;
}

}  // namespace

bool kmeans_x3_supported(int f) { return f >= 1 && f <= 128; }

int64_t kmeans_x3_xp_bytes(int64_t n, int f) {
  return (n + 31) / 32 * x3_ks(f) * 2 * 64 * 16;
}

int64_t kmeans_x3_cp_bytes(int k, int f) {
  const int nchunk = (k + 32 * kX3Nsub - 1) / (32 * kX3Nsub);
  return (int64_t)nchunk * x3_ks(f) * kX3Nsub * 2 * 64 * 16;
}

void kmeans_pack_x3(const float* X, int64_t n, int f, void* Xp, hipStream_t s) {
  const int ks = x3_ks(f);
  const int64_t total = (n + 31) / 32 * ks * 64;
  if (total <= 0) return;
  hipLaunchKernelGGL(k_pack_x3, dim3(grid_for(total, 256)), dim3(256), 0, s, X, n, f, ks,
                     static_cast<uint4*>(Xp));
}

void kmeans_pack_c3(const float* C, int k, int f, void* Cp, hipStream_t s) {
  const int ks = x3_ks(f);
  const int nchunk = (k + 32 * kX3Nsub - 1) / (32 * kX3Nsub);
  const int64_t total = (int64_t)nchunk * ks * kX3Nsub * 64;
  hipLaunchKernelGGL(k_pack_c3, dim3(grid_for(total, 256)), dim3(256), 0, s, C, k, f, ks, nchunk,
                     kX3Nsub, static_cast<uint4*>(Cp));
}

void kmeans_assign_x3(const void* Xp, const float* xnorm, const float* X, int64_t n, int f,
                      const void* Cp, const float* C, int k, int32_t* assign, float* score,
                      int32_t* amb, float* ct, hipStream_t s) {
  if (n <= 0) return;
  const int ks = x3_ks(f);
  const int nchunk = (k + 32 * kX3Nsub - 1) / (32 * kX3Nsub);
  // persistent grid: one workgroup per CU (128 KiB of LDS each)
  const int64_t ngroups = ((n + 31) / 32 + kX3Waves - 1) / kX3Waves;
  static int ncu = [] {
    int dev = 0, v = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      v = 256;
    return v;
  }();
  const int64_t g = std::min<int64_t>(ngroups, ncu);
  const dim3 grid((unsigned)g), block(kX3Threads);
  // eps: 3 * 2^-18 for the split + 2^-24 * (3 * 16 * ks) for the fp32 sums, x2 margin
  const float eps = 2.f * (3.f / 262144.f + (48.f * ks) / 16777216.f);
  WH_HIP_CHECK(hipMemsetAsync(amb, 0, sizeof(int32_t), s));
  const uint4* xp = static_cast<const uint4*>(Xp);
  const uint4* cp = static_cast<const uint4*>(Cp);
  switch (ks) {
    case 2:
      if (x3_pipe())
        hipLaunchKernelGGL((k_assign_x3<2, kX3Nsub, kX3Slots, true>), grid, block, 0, s, xp, xnorm, n,
                           cp, nchunk, k, eps, assign, score, amb);
      else
        hipLaunchKernelGGL((k_assign_x3<2, kX3Nsub, kX3Slots, false>), grid, block, 0, s, xp, xnorm,
                           n, cp, nchunk, k, eps, assign, score, amb);
      break;
    case 4:
      if (x3_pipe())
        hipLaunchKernelGGL((k_assign_x3<4, kX3Nsub, kX3Slots, true>), grid, block, 0, s, xp, xnorm, n,
                           cp, nchunk, k, eps, assign, score, amb);
      else
        hipLaunchKernelGGL((k_assign_x3<4, kX3Nsub, kX3Slots, false>), grid, block, 0, s, xp, xnorm,
                           n, cp, nchunk, k, eps, assign, score, amb);
      break;
    default:
      if (x3_pipe())
        hipLaunchKernelGGL((k_assign_x3<8, kX3Nsub, kX3Slots, true>), grid, block, 0, s, xp, xnorm, n,
                           cp, nchunk, k, eps, assign, score, amb);
      else
        hipLaunchKernelGGL((k_assign_x3<8, kX3Nsub, kX3Slots, false>), grid, block, 0, s, xp, xnorm,
                           n, cp, nchunk, k, eps, assign, score, amb);
      break;
  }
  hipLaunchKernelGGL(k_transpose_c, dim3(grid_for((int64_t)k * f, 256)), dim3(256), 0, s, C, k, f,
                     ct);
  hipLaunchKernelGGL(k_refine_rows, dim3(1024), dim3(256), 0, s, X, f, ct, k, amb, assign, score);
}

}  // namespace wh
