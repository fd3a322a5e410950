// Localize CSC sort microbenchmark: stable sort of 3.9M (local id, row)
// int32 pairs on 20 key bits (a 100k-row Criteo minibatch, 515k unique ids),
// rocPRIM's default radix config vs onesweep configs with wider digits.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/microbench/sort_bench \
//        tools/microbench/sort_bench.hip
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__);    \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

template <class Cfg>
float run(const char* name, int* k, int* v, int* k2, int* v2, size_t n, int bits) {
  size_t bytes = 0;
  CK(rocprim::radix_sort_pairs<Cfg>(nullptr, bytes, k, k2, v, v2, n, 0, bits, 0));
  void* tmp;
  CK(hipMalloc(&tmp, bytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i)
    CK(rocprim::radix_sort_pairs<Cfg>(tmp, bytes, k, k2, v, v2, n, 0, bits, 0));
  CK(hipEventRecord(a, 0));
  const int it = 20;
  for (int i = 0; i < it; ++i)
    CK(rocprim::radix_sort_pairs<Cfg>(tmp, bytes, k, k2, v, v2, n, 0, bits, 0));
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  // verify sorted + stable
  std::vector<int> hk(n), hv(n);
  CK(hipMemcpy(hk.data(), k2, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hv.data(), v2, n * 4, hipMemcpyDeviceToHost));
  bool ok = true;
  for (size_t i = 1; i < n; ++i)
    if (hk[i] < hk[i - 1] || (hk[i] == hk[i - 1] && hv[i] < hv[i - 1])) { ok = false; break; }
  printf("%-40s %8.1f us  %s\n", name, 1000.f * ms / it, ok ? "ok" : "NOT SORTED/STABLE");
  CK(hipFree(tmp));
  return ms;
}

using namespace rocprim;
template <unsigned B, unsigned BS, unsigned IPT,
          block_radix_rank_algorithm A = block_radix_rank_algorithm::default_algorithm>
using OS = radix_sort_config<default_config, default_config,
                             radix_sort_onesweep_config<kernel_config<256, 12>,
                                                        kernel_config<BS, IPT>, B, A>,
                             0>;
constexpr auto kMatch = block_radix_rank_algorithm::match;

int main() {
  const size_t n = 3900000;
  const int U = 515000, bits = 20;
  std::vector<int> hk(n), hv(n);
  unsigned s = 12345;
  for (size_t i = 0; i < n; ++i) {
    s = s * 1664525u + 1013904223u;
    // power-law-ish ids
    const double u = (s >> 8) / 16777216.0;
    hk[i] = (int)(U * u * u * u) % U;
    hv[i] = (int)(i / 39);
  }
  int *k, *v, *k2, *v2;
  CK(hipMalloc(&k, n * 4));
  CK(hipMalloc(&v, n * 4));
  CK(hipMalloc(&k2, n * 4));
  CK(hipMalloc(&v2, n * 4));
  CK(hipMemcpy(k, hk.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(v, hv.data(), n * 4, hipMemcpyHostToDevice));
  run<default_config>("default", k, v, k2, v2, n, bits);
  run<OS<8, 256, 12>>("onesweep 8b 256x12", k, v, k2, v2, n, bits);
  run<OS<8, 256, 16, kMatch>>("onesweep 8b 256x16 match", k, v, k2, v2, n, bits);
  run<OS<10, 256, 12, kMatch>>("onesweep 10b 256x12 match", k, v, k2, v2, n, bits);
  run<OS<10, 512, 12, kMatch>>("onesweep 10b 512x12 match", k, v, k2, v2, n, bits);
  run<OS<10, 1024, 8, kMatch>>("onesweep 10b 1024x8 match", k, v, k2, v2, n, bits);
  run<OS<7, 256, 16, kMatch>>("onesweep 7b 256x16 match", k, v, k2, v2, n, bits);
  return 0;
}
