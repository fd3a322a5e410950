// Microbenchmark: what does the order of the 515K per-minibatch lookups into
// the 4 GB KV slot table (2^27 x 32 B) cost?  One 8-byte load per lookup
// (the probe of k_kv_find), followed by a dependent 16-byte read-modify-write
// of the same slot (what the push kernels do).
//   A  random slot order (hash order, as today)
//   B  the same slots, sorted ascending (table order)
//   C  random order inside a 64 MB table (TLB / DRAM-page reach check)
// Build: hipcc -O3 --offload-arch=gfx950 -o /tmp/kvl tools/microbench/kv_locality_bench.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

struct alignas(32) Slot { unsigned long long key; float w, z, sq, cnt; int vrow, pad; };

__global__ void k_probe(const int* idx, int n, Slot* t, float* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int s = idx[i];
  const unsigned long long k = __hip_atomic_load(&t[s].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  out[i] = (float)(k & 0xff);
}

__global__ void k_rmw(const int* idx, int n, Slot* t, const float* g) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Slot& sl = t[idx[i]];
  const float gi = g[i];
  sl.sq += gi * gi;
  sl.z += gi;
  sl.w = sl.z * 0.5f;
}

int main() {
  const int n = 515000;
  const long big = 1L << 27, small = 1L << 21;
  Slot* t;
  CK(hipMalloc(&t, big * sizeof(Slot)));
  CK(hipMemset(t, 0, big * sizeof(Slot)));
  int* idx;
  float *out, *g;
  CK(hipMalloc(&idx, n * 4));
  CK(hipMalloc(&out, n * 4));
  CK(hipMalloc(&g, n * 4));
  CK(hipMemset(g, 0, n * 4));
  std::mt19937_64 rng(1);
  std::vector<int> rnd(n), srt, rsm(n);
  for (int i = 0; i < n; ++i) rnd[i] = (int)(rng() % big);
  for (int i = 0; i < n; ++i) rsm[i] = (int)(rng() % small);
  srt = rnd;
  std::sort(srt.begin(), srt.end());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](const std::vector<int>& v, const char* name) {
    CK(hipMemcpy(idx, v.data(), n * 4, hipMemcpyHostToDevice));
    for (int w = 0; w < 3; ++w) {
      k_probe<<<(n + 255) / 256, 256>>>(idx, n, t, out);
      k_rmw<<<(n + 255) / 256, 256>>>(idx, n, t, g);
    }
    const int reps = 20;
    float ms1, ms2;
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) k_probe<<<(n + 255) / 256, 256>>>(idx, n, t, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms1, a, b));
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) k_rmw<<<(n + 255) / 256, 256>>>(idx, n, t, g);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms2, a, b));
    printf("%-28s probe %7.1f us   rmw %7.1f us\n", name, 1000 * ms1 / reps, 1000 * ms2 / reps);
  };
  run(rnd, "A random, 4 GB table");
  run(srt, "B sorted, 4 GB table");
  run(rsm, "C random, 64 MB table");
  return 0;
}
