// Exact AUC of one minibatch on the host, with the definition of the device
// chain in csrc/hip/metrics.hip: every example gets the key
// (order-preserving bits of its score, its index, its label bit); the AUC
// counts the (positive, negative) pairs whose positive key is the smaller
// (ties in score broken by index, so all-equal scores give 0.5 and no
// pair is counted twice), r = count / (P * N), AUC = max(r, 1 - r), and a
// minibatch with one class only counts 1 -- the reference's per-minibatch
// convention (learn/base/binary_class_evaluation.h:17-38, whose std::sort
// leaves the order of equal scores unspecified; the index fixes it here).
//
// Header-only: the device layer (csrc/bind/hip_ops.cc, which can run it on
// host threads from a pinned copy instead of the device chain:
// WH_AUC_HOST_THREADS) and the host runtime's binding (the CPU test against
// the plain-PyTorch oracle) compile the same code.
#pragma once

#include <cstdint>
#include <cstring>
#include <utility>
#include <vector>

namespace wh {

inline uint32_t auc_ord_bits(float f) {
  if (f == 0.f) f = 0.f;  // -0 ties with +0
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// A stable LSD radix sort of the keys' upper 32 bits (three passes of
// 11 / 11 / 10 bits, a pass whose digit is constant skipped) -- stable, so
// equal scores stay in index order -- then one sweep: 0.31 ms for 100k rows
// on the GPU box's EPYC 9575F (tools/microbench/auc_host.cc; a 2^16-bucket
// min/max-scaled variant that sorts only the mixed buckets measured 1.5 ms).
// ws: scratch reused between calls (2 n words)
inline double auc_exact_host(const float* py, const float* lab, int64_t n,
                              std::vector<uint64_t>& ws) {
  if (n <= 0) return 1.0;
  ws.resize(2 * (size_t)n);
  uint64_t* a = ws.data();
  uint64_t* b = a + n;
  static constexpr int kShift[3] = {32, 43, 54};
  static constexpr int kBits[3] = {11, 11, 10};
  std::vector<uint32_t> hist(3 * 2048, 0);
  int64_t tp = 0;
  for (int64_t i = 0; i < n; ++i) {
    const bool pos = lab[i] > 0.f;
    const uint64_t k = ((uint64_t)auc_ord_bits(py[i]) << 32) | ((uint64_t)i << 1) | (pos ? 1u : 0u);
    a[i] = k;
    tp += pos;
    for (int p = 0; p < 3; ++p) ++hist[p * 2048 + ((k >> kShift[p]) & ((1u << kBits[p]) - 1))];
  }
  if (tp == 0 || tp == n) return 1.0;
  for (int p = 0; p < 3; ++p) {
    uint32_t* h = hist.data() + p * 2048;
    const int nb = 1 << kBits[p];
    bool constant = false;
    uint32_t run = 0;
    for (int d = 0; d < nb; ++d) {
      if ((int64_t)h[d] == n) constant = true;
      const uint32_t c = h[d];
      h[d] = run;
      run += c;
    }
    if (constant) continue;
    const uint64_t m = (1u << kBits[p]) - 1;
    for (int64_t i = 0; i < n; ++i) b[h[(a[i] >> kShift[p]) & m]++] = a[i];
    std::swap(a, b);
  }
  uint64_t tot = 0, seen = 0;
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t pos = a[i] & 1u;
    seen += pos;
    tot += (pos ^ 1u) * seen;
  }
  const double r = (double)tot / ((double)tp * (double)(n - tp));
  return r < 0.5 ? 1 - r : r;
}

}  // namespace wh
