// Microbenchmark: what bounds the GBDT histogram kernel (k_hist<true>) on
// Higgs-shaped data (11M rows x 28 uint8 bins, 255 bins, identity ridx).
// Variants, all with 1024-thread blocks, 1024 blocks of ~10.7K rows:
//   0  production: dword row loads, interleaved (g, h) fp32 LDS atomics
//   1  loads only (bins xor-reduced into a register)
//   2  LDS atomics only (bins from a hash, no global loads)
//   3  like 2 with ds_add_u32 (fixed-point) instead of ds_add_f32
//   4  production with planar g / h LDS arrays (bank = bin, not 2 * bin)
//   5  like 4, 256-thread blocks
//   6  LDS atomics only, ds_add_u64 (fixed point), hashed bins
//   7  production with int32 fixed point (ds_add_u32)
//   8  production with int64 fixed point (ds_add_u64, 2x LDS)
//   9  production, (g, h) packed into ONE ds_add_u64 per bin: qh * 2^32 + qg
//      (int32 fixed point each; the sum's low word is exactly sum(qg) while
//      |sum| < 2^31, the rest is sum(qh)) -- same LDS bytes as 7, half the
//      atomics
// 7p / 9p: 7 / 9 with a random permutation as the row index (the deep-level
// worst case of the partitioned row order)
// Build: hipcc -O3 --offload-arch=gfx950 -o /tmp/hb tools/microbench/hist_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <utility>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

constexpr int F = 28, NBIN = 255, D = F / 4, R = 64 / D, U = 4;

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352d; x ^= x >> 15; x *= 0x846ca68b; x ^= x >> 16;
  return x;
}

template <int MODE>
__global__ __launch_bounds__(1024) void k_hist(const uint8_t* B, const int* ridx, const float2* gp,
                                               int chunk, int n, float* out) {
  extern __shared__ float lds[];
  const int nl2 = 2 * F * NBIN * (MODE == 6 || MODE == 8 ? 2 : 1);
  for (int i = threadIdx.x; i < nl2; i += blockDim.x) lds[i] = 0.f;
  __syncthreads();
  const int rbeg = blockIdx.x * chunk, nrow = min(chunk, n - rbeg);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int ri = lane / D, dj = lane - ri * D;
  const bool act = ri < R;
  uint32_t acc = 0;
  for (int base = wave * R; base < nrow; base += nw * R * U) {
    uint32_t word[U];
    float2 g[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = base + u * nw * R + ri;
      const bool ok = act && r < nrow;
      if (MODE == 2 || MODE == 3 || MODE == 6) {
        word[u] = ok ? hash32(rbeg + r) : 0xffffffffu;
        g[u] = make_float2(1.f, 0.5f);
      } else {
        const int row = ok ? ridx[rbeg + r] : 0;
        word[u] = ok ? *reinterpret_cast<const uint32_t*>(B + (int64_t)row * F + 4 * dj) : 0xffffffffu;
        g[u] = ok ? gp[row] : make_float2(0.f, 0.f);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int b = (word[u] >> (8 * c)) & 255;
        const int fj = 4 * dj + c;
        if (MODE == 1) {
          acc ^= b + __float_as_uint(g[u].x);
        } else if (b != 255) {
          if (MODE == 9) {
            unsigned long long* l64 = reinterpret_cast<unsigned long long*>(lds);
            const long long qg = (int)(g[u].x * 1024), qh = (int)(g[u].y * 1024);
            atomicAdd(&l64[fj * NBIN + b], (unsigned long long)(qh * 4294967296LL + qg));
          } else if (MODE == 6 || MODE == 8) {
            unsigned long long* l64 = reinterpret_cast<unsigned long long*>(lds);
            atomicAdd(&l64[2 * (fj * NBIN + b)], (unsigned long long)(long long)(g[u].x * 1073741824.f));
            atomicAdd(&l64[2 * (fj * NBIN + b) + 1], (unsigned long long)(long long)(g[u].y * 1073741824.f));
          } else if (MODE == 3 || MODE == 7) {
            atomicAdd(reinterpret_cast<uint32_t*>(&lds[2 * (fj * NBIN + b)]), (uint32_t)(g[u].x * 1024));
            atomicAdd(reinterpret_cast<uint32_t*>(&lds[2 * (fj * NBIN + b) + 1]), (uint32_t)(g[u].y * 1024));
          } else if (MODE == 4 || MODE == 5) {
            atomicAdd(&lds[fj * NBIN + b], g[u].x);
            atomicAdd(&lds[F * NBIN + fj * NBIN + b], g[u].y);
          } else {
            atomicAdd(&lds[2 * (fj * NBIN + b)], g[u].x);
            atomicAdd(&lds[2 * (fj * NBIN + b) + 1], g[u].y);
          }
        }
      }
  }
  __syncthreads();
  if (MODE == 1) lds[threadIdx.x] = (float)acc;
  __syncthreads();
  for (int i = threadIdx.x; i < nl2; i += blockDim.x) out[(int64_t)blockIdx.x * nl2 + i] = lds[i];
}

template <int MODE>
float run(int threads, const uint8_t* B, const int* ridx, const float2* gp, int n, float* out) {
  const int nblk = 1024, chunk = (n + nblk - 1) / nblk;
  const size_t lds = 2 * F * NBIN * 4 * (MODE == 6 || MODE == 8 ? 2 : 1);
  CK(hipFuncSetAttribute((const void*)k_hist<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int it = 0; it < 2; ++it)
    hipLaunchKernelGGL(k_hist<MODE>, dim3(nblk), dim3(threads), lds, 0, B, ridx, gp, chunk, n, out);
  CK(hipEventRecord(a));
  const int reps = 10;
  for (int it = 0; it < reps; ++it)
    hipLaunchKernelGGL(k_hist<MODE>, dim3(nblk), dim3(threads), lds, 0, B, ridx, gp, chunk, n, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  const int n = 11000000;
  std::vector<uint8_t> hB((size_t)n * F);
  uint32_t s = 1;
  for (auto& v : hB) { s = s * 1664525u + 1013904223u; v = (uint8_t)((s >> 8) % NBIN); }
  std::vector<int> hr(n);
  for (int i = 0; i < n; ++i) hr[i] = i;
  std::vector<float2> hg(n, make_float2(0.3f, 0.2f));
  uint8_t* B; int* ridx; float2* gp; float* out;
  CK(hipMalloc(&B, hB.size()));
  CK(hipMalloc(&ridx, n * 4));
  CK(hipMalloc(&gp, n * 8));
  CK(hipMalloc(&out, (size_t)1024 * 4 * F * NBIN * 4));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  printf("sharedMemPerBlock %zu maxSharedMemoryPerMultiProcessor %zu\n", prop.sharedMemPerBlock, prop.maxSharedMemoryPerMultiProcessor);
  CK(hipMemcpy(B, hB.data(), hB.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(ridx, hr.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(gp, hg.data(), n * 8, hipMemcpyHostToDevice));
  printf("0 production         %.3f ms\n", run<0>(1024, B, ridx, gp, n, out));
  printf("1 loads only         %.3f ms\n", run<1>(1024, B, ridx, gp, n, out));
  printf("2 atomics only f32   %.3f ms\n", run<2>(1024, B, ridx, gp, n, out));
  printf("3 atomics only u32   %.3f ms\n", run<3>(1024, B, ridx, gp, n, out));
  printf("4 planar g/h         %.3f ms\n", run<4>(1024, B, ridx, gp, n, out));
  printf("5 planar, 256 thr    %.3f ms\n", run<5>(256, B, ridx, gp, n, out));
  printf("6 atomics only u64   %.3f ms\n", run<6>(1024, B, ridx, gp, n, out));
  printf("7 production u32     %.3f ms\n", run<7>(1024, B, ridx, gp, n, out));
  printf("8 production u64     %.3f ms\n", run<8>(1024, B, ridx, gp, n, out));
  printf("9 production packed  %.3f ms\n", run<9>(1024, B, ridx, gp, n, out));
  for (int i = n - 1; i > 0; --i) {  // Fisher-Yates with the LCG
    s = s * 1664525u + 1013904223u;
    const int j = (int)(((uint64_t)s * (uint64_t)(i + 1)) >> 32);
    std::swap(hr[i], hr[j]);
  }
  CK(hipMemcpy(ridx, hr.data(), n * 4, hipMemcpyHostToDevice));
  printf("7p u32, random ridx  %.3f ms\n", run<7>(1024, B, ridx, gp, n, out));
  printf("9p packed, random    %.3f ms\n", run<9>(1024, B, ridx, gp, n, out));
  return 0;
}
