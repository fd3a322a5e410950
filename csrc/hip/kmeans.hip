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
#include "wh_common.h"
#include "wh_kernels.h"

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

void kmeans_pack_c(const float* C, int k, int f, float* Cp, hipStream_t s) {
  const int ks = kmeans_ks(f);
  const int nchunk = (k + 31) / 32;
  const int64_t total = (int64_t)nchunk * ks * 64;
  hipLaunchKernelGGL(k_pack_c, dim3(grid_for(total, 256)), dim3(256), 0, s, C, k, f, ks, nchunk,
                     Cp);
}

void kmeans_assign(const float* Xp, int64_t n, int f, const float* Cp, int k, int32_t* assign,
                   float* score, hipStream_t s) {
  if (n <= 0) return;
  const int ks = kmeans_ks(f);
  const int nchunk = (k + 31) / 32;
  const int64_t ntiles = (n + 31) / 32;
  const dim3 grid(grid_for(ntiles * 64, 256)), block(256);
  // register-resident A for the common widths, streamed A beyond
  if (ks <= 8)
    hipLaunchKernelGGL(k_assign<8>, grid, block, 0, s, Xp, n, ks, Cp, nchunk, k, assign, score);
  else if (ks <= 16)
    hipLaunchKernelGGL(k_assign<16>, grid, block, 0, s, Xp, n, ks, Cp, nchunk, k, assign, score);
  else if (ks <= 32)
    hipLaunchKernelGGL(k_assign<32>, grid, block, 0, s, Xp, n, ks, Cp, nchunk, k, assign, score);
  else if (ks <= 64)
    hipLaunchKernelGGL(k_assign<64>, grid, block, 0, s, Xp, n, ks, Cp, nchunk, k, assign, score);
  else
    hipLaunchKernelGGL(k_assign<0>, grid, block, 0, s, Xp, n, ks, Cp, nchunk, k, assign, score);
}

void kmeans_accum(const float* X, int64_t n, int f, const int32_t* assign, float* sums,
                  hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_accum, dim3(grid_for(n * 64, 256)), dim3(256), 0, s, X, n, f, assign, sums);
}

}  // namespace wh
