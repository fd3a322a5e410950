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
#include <cstdio>
#include <cstdlib>

#include "wh_common.h"
#include "wh_kernels.h"

namespace wh {
namespace {

// A block owns kSynthRows whole rows; its threads stride over the rows'
// (row, field) elements, so key stores are contiguous and each row's label is
// summed from LDS. Rows per block are many enough that a thread has ~10
// independent elements in flight (one element per thread and 6 rows per block
// made the kernel a latency chain of 16k tiny blocks: 108 us per 100k rows).
// uniform in [0,1) from (seed, row, field) with 32-bit arithmetic (murmur3
// fmix32 rounds; the 64-bit multiplies of uhash01 made this generator
// ALU-bound at ~39 us per 100k rows)
__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}
__device__ __forceinline__ float uhash01_32(uint64_t seed, uint64_t gid, uint32_t f) {
  uint32_t h = fmix32((uint32_t)gid ^ (uint32_t)seed ^ 0x9e3779b9u);
  h = fmix32(h ^ (uint32_t)(gid >> 32) ^ (uint32_t)(seed >> 32) ^ (f * 0x27d4eb2du));
  return (float)(h >> 8) * (1.0f / 16777216.0f);
}

constexpr int kSynthThreads = 256;
constexpr int kSynthRows = 64;
constexpr int kMaxField = 64;

__global__ __launch_bounds__(kSynthThreads) void k_synth_criteo(int64_t nrows, uint64_t seed,
                                                                uint64_t step,
                                                                const int64_t* card, int nfield,
                                                                uint64_t* keys, float* label,
                                                                int64_t* offset) {
  __shared__ float th[kSynthRows * kMaxField];
  __shared__ float lc[kMaxField];
  __shared__ int64_t cd[kMaxField];
  for (int f = threadIdx.x; f < nfield; f += kSynthThreads) {
    cd[f] = card[f];
    lc[f] = log2f((float)cd[f]);
  }
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * kSynthRows;
  const int64_t nr = nrows - r0 < kSynthRows ? nrows - r0 : kSynthRows;
  const int ne = (int)nr * nfield;
  // (row, field) of element e, stepped instead of divided per element
  int lr = threadIdx.x / nfield, f = threadIdx.x - lr * nfield;
  const int dlr = kSynthThreads / nfield, df = kSynthThreads - dlr * nfield;
  for (int e = threadIdx.x; e < ne; e += kSynthThreads) {
    const int64_t r = r0 + lr;
    const uint64_t gid = step * (uint64_t)nrows + (uint64_t)r;
    const float u = uhash01_32(seed, gid, (uint32_t)f);
    // rank = floor(card^u) - 1 in single precision (a power law P(r) ~ 1 /
    // (r + 1); the double-precision exp was half of this kernel's time)
    int64_t rank = (int64_t)exp2f(lc[f] * u) - 1;
    if (rank < 0) rank = 0;
    if (rank >= cd[f]) rank = cd[f] - 1;
    const uint64_t tok = mix64(((uint64_t)f << 40) ^ (uint64_t)rank ^ 0x5bd1e995ull);
    keys[r0 * nfield + e] = (tok >> 10) | ((uint64_t)f << 54);
    // hidden weight of this (field, value) from the token hash's top bits;
    // head values carry most signal
    th[e] = ((float)(uint32_t)(tok >> 40) * (1.0f / 16777216.0f) - 0.5f) * 0.9f;
    lr += dlr;
    f += df;
    if (f >= nfield) {
      f -= nfield;
      ++lr;
    }
  }
  __syncthreads();
  if (threadIdx.x < nr) {
    const int64_t rr = r0 + threadIdx.x;
    float logit = -1.2f;
    for (int q = 0; q < nfield; ++q) logit += th[threadIdx.x * nfield + q];
    const float p = 1.f / (1.f + __expf(-logit));
    const uint64_t gid = step * (uint64_t)nrows + (uint64_t)rr;
    label[rr] = uhash01(seed ^ 0xabcdefull, gid, 977) < p ? 1.f : 0.f;
    offset[rr] = rr * nfield;
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) offset[nrows] = nrows * (int64_t)nfield;
}

}  // namespace

void synth_criteo(int64_t nrows, uint64_t seed, uint64_t step, const int64_t* card, int nfield,
                  uint64_t* keys, float* label, int64_t* offset, hipStream_t s) {
  if (nfield < 1 || nfield > kMaxField) {
    fprintf(stderr, "synth_criteo: nfield must be in [1, %d]\n", kMaxField);
    abort();
  }
  const int64_t nb = (nrows + kSynthRows - 1) / kSynthRows;
  hipLaunchKernelGGL(k_synth_criteo, dim3((unsigned)(nb > 0 ? nb : 1)), dim3(kSynthThreads), 0, s,
                     nrows, seed, step, card, nfield, keys, label, offset);
}

}  // namespace wh
