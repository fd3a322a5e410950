// Microbenchmark of the split-precision k-means assign kernel variants
// (compile with -DWH_X3_VARIANT=0/1/2 and -DWH_X3_NSUB=2/4):
//   0 production, 1 no top-2 epilogue, 2 no LDS-DMA streaming (chunk 0 reused)
#include "../../csrc/hip/scan.hip"
#include "../../csrc/hip/kmeans.hip"
#include <cstdio>
#include <vector>

int main() {
  const int64_t n = 10000000;
  const int f = 128, k = 1000;
  float *X, *C, *xn, *sc, *ct;
  void *Xp, *Cp;
  int32_t *as, *amb;
  hipMalloc(&X, n * f * 4);
  hipMalloc(&C, (size_t)k * f * 4);
  hipMalloc(&xn, n * 4);
  hipMalloc(&sc, n * 4);
  hipMalloc(&ct, (size_t)k * f * 4);
  hipMalloc(&as, n * 4);
  hipMalloc(&amb, (n + 1) * 4);
  hipMalloc(&Xp, wh::kmeans_x3_xp_bytes(n, f));
  hipMalloc(&Cp, wh::kmeans_x3_cp_bytes(k, f));
  std::vector<float> h(k * f);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  hipMemcpy(C, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  hipMemset(X, 0, n * f * 4);
  hipMemset(xn, 0, n * 4);
  wh::kmeans_pack_x3(X, n, f, Xp, 0);
  wh::kmeans_pack_c3(C, k, f, Cp, 0);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int w = 0; w < 2; ++w)
    wh::kmeans_assign_x3(Xp, xn, X, n, f, Cp, C, k, as, sc, amb, ct, 0);
  hipEventRecord(a, 0);
  const int it = 10;
  for (int i = 0; i < it; ++i) wh::kmeans_assign_x3(Xp, xn, X, n, f, Cp, C, k, as, sc, amb, ct, 0);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  printf("variant %d nsub %d: %.3f ms per assign\n", WH_X3_VARIANT, WH_X3_NSUB, ms / it);
  return 0;
}
