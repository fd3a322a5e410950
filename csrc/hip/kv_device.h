// Device helpers shared by the parameter-store kernels (kvstore.hip: the
// single-shard fused paths; psx.hip: the multi-shard exchange paths).
#pragma once
#include "wh_common.h"
#include "wh_kernels.h"

namespace wh {
namespace kvd {

constexpr int kThreads = 256;
// A probe sequence longer than this is a failed insert / lookup miss. The
// host keeps the load factor <= 0.7 (KVStore::reserve), where the expected
// probe length of linear probing is ~6, so hitting the bound means a broken
// table, and it is reported (stats[2]) instead of scanning the whole table.
constexpr int kMaxProbe = 256;
// pull / open tiles: 4 keys per thread
constexpr int kPullPer = 4;
constexpr int kPullTile = kThreads * kPullPer;
constexpr int kRowBatch = 8;   // row loads a G-lane group issues before its stores
constexpr int kPushBatch = 4;  // (V, VG, gV) row triples per G-lane group in the push

__device__ __forceinline__ uint64_t ld_relaxed(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int32_t ld_relaxed_i32(const int32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// counter `idx` of this wave's shard (see kStatShards)
__device__ __forceinline__ unsigned long long* stat_ptr(int64_t* stats, int idx) {
  const int shard =
      (int)((blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) & (kStatShards - 1));
  return reinterpret_cast<unsigned long long*>(stats + shard * kStatStride + idx);
}

// Find (insert=0) or find-or-insert (insert=1) key k whose home-slot key
// word was already loaded into `pv` (so callers can issue several home
// probes back to back). Returns the slot or -1; *created is set when this
// call inserted the key.
__device__ __forceinline__ int32_t probe_slot(KVSlot* sl, uint64_t mask, uint64_t k, uint64_t h,
                                              uint64_t pv, int insert, bool* created) {
  for (int probe = 0; probe < kMaxProbe; ++probe) {
    if (pv == k) return (int32_t)h;
    if (pv == kEmptyKey) {
      if (!insert) return -1;
      const uint64_t old = atomicCAS((unsigned long long*)(&sl[h].key),
                                     (unsigned long long)kEmptyKey, (unsigned long long)k);
      if (old == kEmptyKey) { *created = true; return (int32_t)h; }
      if (old == k) return (int32_t)h;
    }
    h = (h + 1) & mask;
    pv = ld_relaxed(&sl[h].key);
  }
  return -1;
}

// wave-aggregated bump allocation of V rows; returns the row or -1 (slab full)
__device__ __forceinline__ int32_t wave_alloc_rows(const KVTable& t, bool want) {
  const uint64_t m = __ballot(want);
  if (!m) return -1;
  const int lane = threadIdx.x & 63;
  int32_t base = 0;
  const int leader = __ffsll((unsigned long long)m) - 1;
  if (lane == leader) base = atomicAdd(t.vnext, (int)__popcll(m));
  base = __shfl(base, leader, 64);
  if (!want) return -1;
  const int32_t row = base + (int32_t)__popcll(m & ((1ull << lane) - 1));
  if (row >= t.vcap) {
    atomicAdd(stat_ptr(t.stats, 3), 1ull);
    return -1;
  }
  return row;
}

// the deterministic initial value of embedding element d of `key`
__device__ __forceinline__ float v_init_val(const DifactoHP& hp, uint64_t key, int d, int dim) {
  return d < dim ? (uhash01(hp.seed, key, (uint64_t)d) * 2.f - 1.f) * hp.v_init : 0.f;
}

__device__ __forceinline__ float4 v_init4(const DifactoHP& hp, uint64_t key, int c, int dim) {
  return make_float4(v_init_val(hp, key, c, dim), v_init_val(hp, key, c + 1, dim),
                     v_init_val(hp, key, c + 2, dim), v_init_val(hp, key, c + 3, dim));
}

__device__ __forceinline__ void init_v_row(const KVTable& t, uint64_t key, int32_t row, int gl,
                                           int G, const DifactoHP& hp) {
  float* V = t.V + (int64_t)row * t.vstride;
  float* VG = t.VG + (int64_t)row * t.vstride;
  for (int c = gl * 4; c < t.vstride; c += 4 * G) {
    *reinterpret_cast<float4*>(V + c) = v_init4(hp, key, c, t.dim);
    *reinterpret_cast<float4*>(VG + c) = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// FTRL step on w (reference UpdateW, learn/difacto/async_sgd.h:262-286);
// returns the new w and updates z / sq in place
__device__ __forceinline__ float difacto_ftrl(float w, float gw, float& sq, float& z,
                                              const DifactoHP& hp) {
  const float g = gw + hp.l2 * w;
  const float cg = sq;
  const float cg_new = sqrtf(cg * cg + g * g);
  sq = cg_new;
  z = z - (g - (cg_new - cg) / hp.alpha * w);
  if (z <= hp.l1 && z >= -hp.l1) return 0.f;
  const float eta = (hp.beta + cg_new) / hp.alpha;
  return (z > 0 ? z - hp.l1 : z + hp.l1) / eta;
}

// AdaGrad on 4 embedding elements (reference UpdateV, async_sgd.h:289-296)
__device__ __forceinline__ void adagrad4(float4& v, float4& cg, const float4& g,
                                         const DifactoHP& hp) {
  float* pv = &v.x;
  float* pc = &cg.x;
  const float* pg = &g.x;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const float gg = pg[e] + hp.v_l2 * pv[e];
    pc[e] = sqrtf(pc[e] * pc[e] + gg * gg);
    pv[e] -= hp.v_alpha / (pc[e] + hp.v_beta) * gg;
  }
}

__device__ __forceinline__ float l1l2_solve(float z, float eta, float l1, float l2) {
  // argmin_x 0.5*eta*(x - z/eta)^2 + l1|x| + l2 x^2 (soft threshold)
  // (reference L1L2::Solve, learn/linear/penalty.h:36-41)
  if (z <= l1 && z >= -l1) return 0.f;
  return (z > 0 ? z - l1 : z + l1) / (eta + l2);
}

// one linear-model push of gradient g into slot e (reference SGD / AdaGrad /
// FTRL handles, learn/linear/async_sgd.h:85-99, 123-135, 160-175); returns
// the new w. sgd_eta: SGD only, (beta + sqrt(t)) / alpha for this push.
__device__ __forceinline__ float linear_update(KVSlot& e, float g, const LinearHP& hp,
                                               float sgd_eta) {
  const float oldw = e.w;
  float neww;
  if (hp.algo == 1) {  // SGD
    neww = l1l2_solve(sgd_eta * oldw - g, sgd_eta, hp.l1, hp.l2);
  } else if (hp.algo == 2) {  // AdaGrad
    const float sq = sqrtf(e.sq * e.sq + g * g);
    e.sq = sq;
    const float eta = (sq + hp.beta) / hp.alpha;
    neww = l1l2_solve(eta * oldw - g, eta, hp.l1, hp.l2);
  } else if (hp.algo == 4) {  // DiFacto's FTRL on w (an embedding-free DiFacto
    // model over the linear wire format; reference UpdateW,
    // learn/difacto/async_sgd.h:262-286: l2 in the gradient, l1 threshold)
    const float gg = g + hp.l2 * oldw;
    const float cg = e.sq;
    const float cg_new = sqrtf(cg * cg + gg * gg);
    e.sq = cg_new;
    const float z = e.z - (gg - (cg_new - cg) / hp.alpha * oldw);
    e.z = z;
    neww = (z <= hp.l1 && z >= -hp.l1)
               ? 0.f
               : (z > 0 ? z - hp.l1 : z + hp.l1) / ((hp.beta + cg_new) / hp.alpha);
  } else {  // FTRL
    const float sq0 = e.sq;
    const float sq = sqrtf(sq0 * sq0 + g * g);
    e.sq = sq;
    const float sigma = (sq - sq0) / hp.alpha;
    const float z = e.z + g - sigma * oldw;
    e.z = z;
    neww = l1l2_solve(-z, (hp.beta + sq) / hp.alpha, hp.l1, hp.l2);
  }
  e.w = neww;
  return neww;
}

__device__ __forceinline__ void count_nnz_delta(float oldw, float neww, int64_t* stats) {
  const int d = (oldw == 0.f && neww != 0.f) ? 1 : ((oldw != 0.f && neww == 0.f) ? -1 : 0);
  long long s = wave_sum_ll(d);
  if ((threadIdx.x & 63) == 0 && s) atomicAdd(stat_ptr(stats, 0), (unsigned long long)s);
}

inline int lanes_per_key(int vstride) {
  if (vstride <= 0) return 1;
  int q = vstride / 4;
  return q >= 64 ? 64 : q;
}

}  // namespace kvd
}  // namespace wh

#define WH_DISPATCH_G(G, KERNEL, ...)                                            \
  switch (G) {                                                                   \
    case 1: hipLaunchKernelGGL(KERNEL<1>, __VA_ARGS__); break;                   \
    case 2: hipLaunchKernelGGL(KERNEL<2>, __VA_ARGS__); break;                   \
    case 4: hipLaunchKernelGGL(KERNEL<4>, __VA_ARGS__); break;                   \
    case 8: hipLaunchKernelGGL(KERNEL<8>, __VA_ARGS__); break;                   \
    case 16: hipLaunchKernelGGL(KERNEL<16>, __VA_ARGS__); break;                 \
    case 32: hipLaunchKernelGGL(KERNEL<32>, __VA_ARGS__); break;                 \
    default: hipLaunchKernelGGL(KERNEL<64>, __VA_ARGS__); break;                 \
  }
