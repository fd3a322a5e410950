// Host AUC timing (csrc/host/auc_host.h) on one 100k-row minibatch of
// sigmoid-shaped scores, 30 % positives.
// g++ -O3 -std=c++17 -Icsrc tools/microbench/auc_host.cc -o tools/microbench/auc_host_bench
#include "host/auc_host.h"
#include <chrono>
#include <cmath>
#include <cstdio>
#include <random>
int main() {
  const int n = 100000;
  std::vector<float> p(n), l(n);
  std::mt19937 g(1);
  std::uniform_real_distribution<float> u(0, 1);
  for (int i = 0; i < n; ++i) {
    p[i] = 1.f / (1.f + std::exp(-(u(g) * 8 - 4)));
    l[i] = u(g) < 0.3f;
  }
  std::vector<uint64_t> ws;
  double s = 0;
  for (int r = 0; r < 3; ++r) {
    auto t = std::chrono::steady_clock::now();
    for (int k = 0; k < 200; ++k) s += wh::auc_exact_host(p.data(), l.data(), n, ws);
    std::printf("%.3f ms per minibatch\n",
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count() / 200);
  }
  std::printf("checksum %.6f\n", s);
}
