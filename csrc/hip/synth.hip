// Device-side synthetic data generators for benchmarks (no datasets are
// reachable from the benchmark boxes).
//
// synth_criteo: Criteo-1TB-shaped click logs. Each row has 13 integer + 26
// categorical fields; a field value is a power-law rank r in [0, card_f)
// (P(r) ~ 1/(r+1), drawn as r = floor(card^u) - 1), and the feature id is
// built exactly like the reference Criteo parser builds it from a token
// (learn/base/criteo_parser.h:69-70,81-82): (hash64(token) >> 10) | (field << 54).
// Labels come from a hidden logistic model over (field, rank) so the
// learners see real signal (logloss falls, AUC rises).
#include "wh_common.h"
#include "wh_kernels.h"

namespace wh {
namespace {

__global__ __launch_bounds__(256) void k_synth_criteo(int64_t nrows, uint64_t seed, uint64_t step,
                                                      const int64_t* card, int nfield,
                                                      uint64_t* keys, float* label,
                                                      int64_t* offset) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r > nrows) return;
  offset[r] = r * nfield;
  if (r == nrows) return;
  const uint64_t gid = step * (uint64_t)nrows + (uint64_t)r;
  float logit = -1.2f;
  for (int f = 0; f < nfield; ++f) {
    const float u = uhash01(seed, gid, (uint64_t)f);
    const double c = (double)card[f];
    int64_t rank = (int64_t)exp(log(c) * (double)u) - 1;
    if (rank < 0) rank = 0;
    if (rank >= card[f]) rank = card[f] - 1;
    const uint64_t tok = mix64(((uint64_t)f << 40) ^ (uint64_t)rank ^ 0x5bd1e995ull);
    keys[r * nfield + f] = (tok >> 10) | ((uint64_t)f << 54);
    // hidden weight of this (field, value); head values carry most signal
    const float th = uhash01(0x7e57ull, (uint64_t)f, (uint64_t)rank) - 0.5f;
    logit += th * 0.9f;
  }
  const float p = 1.f / (1.f + __expf(-logit));
  label[r] = uhash01(seed ^ 0xabcdefull, gid, 977) < p ? 1.f : 0.f;
}

}  // namespace

void synth_criteo(int64_t nrows, uint64_t seed, uint64_t step, const int64_t* card, int nfield,
                  uint64_t* keys, float* label, int64_t* offset, hipStream_t s) {
  hipLaunchKernelGGL(k_synth_criteo, dim3(grid_for(nrows + 1, 256)), dim3(256), 0, s, nrows, seed,
                     step, card, nfield, keys, label, offset);
}

}  // namespace wh
