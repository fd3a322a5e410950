// Single-shard linear step WITHOUT a localize: the minibatch's feature ids
// go straight to the parameter table, and gradients are summed per table
// slot. For one GPU (P = 1) the localize (unique ids + per-id occurrence
// lists) exists only to dedup the lookups and to order the transposed
// product; both jobs are done here per row tile in LDS:
//
//   k_ld_touch  per tile of rows: dedup the tile's ids in an LDS hash table,
//               find-or-insert each distinct id in the HBM table once, stamp
//               the slot with the step number (the first tile to stamp a
//               slot lists it in the tile's own part of the minibatch's slot
//               list), and write the slot of every non-zero (lid = slot).
//   (forward)   fm.hip k_lin_fwd reads w straight from the slots (stride 8).
//   k_ld_bwd    per tile: g = x * dual[row] accumulated per distinct slot in
//               LDS, then one float atomic per (tile, slot) into a dense
//               per-slot gradient array -- hot ids cost one atomic per tile,
//               not one per occurrence.
//   k_ld_push   per listed slot (a block per tile's list): take (and clear)
//               its summed gradient, apply
//               SGD / AdaGrad / FTRL (reference learn/linear/async_sgd.h:
//               71-180, penalty.h:36-41).
//
// No host synchronisation: the list length stays on the device (the push
// launches over the non-zero count, surplus lanes exit), so a 10000-row
// minibatch (the reference's published configuration) costs a handful of
// launches. The gradient sums use float atomics (order-free up to rounding);
// WH_DETERMINISTIC=1 keeps the localize path.
#include "wh_common.h"
#include "wh_kernels.h"
#include "kv_device.h"

#include <stdexcept>

namespace wh {
namespace {

using namespace kvd;

constexpr int kLdThreads = 256;
constexpr int kLdProbe = 64;            // LDS probe bound (a full table falls back to global)

// LDS hash entries per tile (T >= 2x the tile's ids; a tile holds ~T/2
// non-zeros). Small minibatches take small tiles: at the reference's 10000
// rows (390k non-zeros) 4096-entry tiles gave 193 workgroups at ~80 KB of LDS
// each -- fewer than the CUs, one resident per CU -- so each tile's chain of
// dependent probes was exposed; 1024-entry tiles give ~760 workgroups at
// ~20 KB, several resident per CU.
__host__ __device__ constexpr int ld_rows_cap(int T) { return T / 2 < 1024 ? T / 2 : 1024; }

// the tile's row range [r0, r1) and its non-zero range [j0, j1); row offsets
// of the tile staged in LDS (R + 1 entries) for the row of a non-zero
__device__ __forceinline__ int row_in_tile(const int64_t* so, int nr, int64_t j) {
  int lo = 0, hi = nr - 1;  // largest r with so[r] <= j
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (so[mid] <= j) lo = mid; else hi = mid - 1;
  }
  return lo;
}

template <int T>
__device__ __forceinline__ uint32_t lhash(uint64_t k) { return (uint32_t)(mix64(k) & (T - 1)); }

template <int T>
__global__ __launch_bounds__(kLdThreads) void k_ld_touch(
    KVTable t, const uint64_t* __restrict__ keys, const int64_t* __restrict__ off, int64_t nrows,
    int R, uint32_t stamp, int insert, int32_t* __restrict__ lid, int32_t* __restrict__ tlist,
    unsigned int* __restrict__ tcnt, int32_t* __restrict__ ovf, unsigned int* __restrict__ ovf_cnt) {
  __shared__ unsigned long long lk[T];
  __shared__ int32_t lslot[T];
  __shared__ int32_t lst[T];     // occupied entries, in insertion order
  __shared__ int32_t lfirst[T];  // slots this tile stamped first
  __shared__ unsigned int nlist, nfirst;
  const int64_t r0 = (int64_t)blockIdx.x * R;
  if (r0 >= nrows) return;
  const int64_t r1 = r0 + R < nrows ? r0 + R : nrows;
  const int64_t j0 = off[r0], j1 = off[r1];
  for (int e = threadIdx.x; e < T; e += kLdThreads) lk[e] = kEmptyKey;
  if (threadIdx.x == 0) nlist = nfirst = 0;
  __syncthreads();
  // phase A: distinct ids of the tile (LDS CAS); ids that do not fit are
  // resolved per occurrence in phase C
  for (int64_t j = j0 + threadIdx.x; j < j1; j += kLdThreads) {
    const uint64_t k = keys[j];
    if (k == kEmptyKey) continue;
    uint32_t h = lhash<T>(k);
    for (int p = 0; p < kLdProbe; ++p, h = (h + 1) & (T - 1)) {
      const unsigned long long o = atomicCAS(&lk[h], (unsigned long long)kEmptyKey,
                                             (unsigned long long)k);
      if (o == kEmptyKey) {
        lst[atomicAdd(&nlist, 1u)] = (int32_t)h;
        break;
      }
      if (o == k) break;
    }
  }
  __syncthreads();
  // phase B: one table probe per distinct id, kPullPer in flight per lane
  const int nl = (int)nlist;
  const uint64_t mask = (uint64_t)t.cap - 1;
  int created = 0, failed = 0;
  for (int b = threadIdx.x * kPullPer; b < nl; b += kLdThreads * kPullPer) {
    uint64_t k[kPullPer], h[kPullPer], pv[kPullPer];
    int32_t sl[kPullPer];
#pragma unroll
    for (int r = 0; r < kPullPer; ++r) {
      k[r] = b + r < nl ? lk[lst[b + r]] : kEmptyKey;
      h[r] = mix64(k[r]) & mask;
      pv[r] = k[r] != kEmptyKey ? ld_relaxed(&t.sl[h[r]].key) : 0;
    }
#pragma unroll
    for (int r = 0; r < kPullPer; ++r) {
      sl[r] = -1;
      if (k[r] == kEmptyKey) continue;
      bool cr = false;
      sl[r] = probe_slot(t.sl, mask, k[r], h[r], pv[r], insert, &cr);
      created += cr ? 1 : 0;
      if (insert && sl[r] < 0) ++failed;
      lslot[lst[b + r]] = sl[r];
    }
    // stamp: the first tile of this step to reach a slot lists it
    uint32_t old[kPullPer];
#pragma unroll
    for (int r = 0; r < kPullPer; ++r)
      old[r] = sl[r] >= 0 ? atomicExch(&t.sl[sl[r]].cnt, stamp) : stamp;
#pragma unroll
    for (int r = 0; r < kPullPer; ++r)
      if (old[r] != stamp) lfirst[atomicAdd(&nfirst, 1u)] = sl[r];
  }
  __syncthreads();
  // the tile's first-stamped slots are its part of the minibatch's slot list:
  // stored in the tile's own range with its count (no shared counter: one
  // same-address atomic per tile serialised ~770 of them, ~9 us at 10k rows)
  for (unsigned int i = threadIdx.x; i < nfirst; i += kLdThreads)
    tlist[(int64_t)blockIdx.x * T + i] = lfirst[i];
  if (threadIdx.x == 0) tcnt[blockIdx.x] = nfirst;
  const long long ci = wave_sum_ll(created), cf = wave_sum_ll(failed);
  if ((threadIdx.x & 63) == 0) {
    if (ci) atomicAdd(stat_ptr(t.stats, 4), (unsigned long long)ci);
    if (cf) atomicAdd(stat_ptr(t.stats, 2), (unsigned long long)cf);
  }
  __syncthreads();
  // phase C: the slot of every non-zero
  for (int64_t j = j0 + threadIdx.x; j < j1; j += kLdThreads) {
    const uint64_t k = keys[j];
    int32_t s = -1;
    if (k != kEmptyKey) {
      uint32_t h = lhash<T>(k);
      int p = 0;
      for (; p < kLdProbe; ++p, h = (h + 1) & (T - 1))
        if (lk[h] == k) break;
      if (p < kLdProbe) {
        s = lslot[h];
      } else {  // the tile overflowed its LDS table: resolve this one directly
        bool cr = false;
        const uint64_t hh = mix64(k) & mask;
        s = probe_slot(t.sl, mask, k, hh, ld_relaxed(&t.sl[hh].key), insert, &cr);
        if (cr) atomicAdd(stat_ptr(t.stats, 4), 1ull);
        if (insert && s >= 0 && atomicExch(&t.sl[s].cnt, stamp) != stamp)
          ovf[atomicAdd(ovf_cnt, 1u)] = s;  // (rare: a tile whose ids overflowed LDS)
      }
    }
    lid[j] = s;
  }
}

template <int T>
__global__ __launch_bounds__(kLdThreads) void k_ld_bwd(
    const int32_t* __restrict__ lid, const float* __restrict__ val,
    const int64_t* __restrict__ off, int64_t nrows, int R, const float* __restrict__ dual,
    float* __restrict__ grad) {
  constexpr int RC = ld_rows_cap(T);
  __shared__ int32_t ls[T];
  __shared__ float lg[T];
  __shared__ int32_t lst[T];
  __shared__ int64_t so[RC + 1];
  __shared__ float sd[RC];
  __shared__ unsigned int nlist;
  const int64_t r0 = (int64_t)blockIdx.x * R;
  if (r0 >= nrows) return;
  const int64_t r1 = r0 + R < nrows ? r0 + R : nrows;
  const int nr = (int)(r1 - r0);
  for (int e = threadIdx.x; e < T; e += kLdThreads) {
    ls[e] = -1;
    lg[e] = 0.f;
  }
  for (int r = threadIdx.x; r <= nr; r += kLdThreads) so[r] = off[r0 + r];
  for (int r = threadIdx.x; r < nr; r += kLdThreads) sd[r] = dual[r0 + r];
  if (threadIdx.x == 0) nlist = 0;
  __syncthreads();
  const int64_t j0 = so[0], j1 = so[nr];
  for (int64_t j = j0 + threadIdx.x; j < j1; j += kLdThreads) {
    const int32_t s = lid[j];
    if (s < 0) continue;
    const float g = (val ? val[j] : 1.f) * sd[row_in_tile(so, nr, j)];
    uint32_t h = (uint32_t)(mix64((uint64_t)s) & (T - 1));
    int p = 0;
    for (; p < kLdProbe; ++p, h = (h + 1) & (T - 1)) {
      const int32_t o = atomicCAS(&ls[h], -1, s);
      if (o == -1) {
        lst[atomicAdd(&nlist, 1u)] = (int32_t)h;
        break;
      }
      if (o == s) break;
    }
    if (p < kLdProbe) atomicAdd(&lg[h], g);
    else atomicAdd(&grad[s], g);  // (table full: straight to the slot)
  }
  __syncthreads();
  const int nl = (int)nlist;
  for (int i = threadIdx.x; i < nl; i += kLdThreads) {
    const int e = lst[i];
    atomicAdd(&grad[ls[e]], lg[e]);
  }
}

// block b < ntiles: tile b's listed slots; block ntiles: the overflow list
// (whose counter it re-zeroes for the next step, after reading it)
__global__ __launch_bounds__(kLdThreads) void k_ld_push(KVTable t, const int32_t* __restrict__ tlist,
                                                        const unsigned int* __restrict__ tcnt,
                                                        int T, const int32_t* __restrict__ ovf,
                                                        unsigned int* __restrict__ ovf_cnt,
                                                        float* __restrict__ grad, LinearHP hp) {
  const bool last = blockIdx.x == gridDim.x - 1;
  const unsigned int n = last ? *ovf_cnt : tcnt[blockIdx.x];
  const int32_t* list = last ? ovf : tlist + (int64_t)blockIdx.x * T;
  for (unsigned int i0 = 0; i0 < n; i0 += kLdThreads) {  // (block-uniform trips)
    const unsigned int i = i0 + threadIdx.x;
    float oldw = 0.f, neww = 0.f;
    if (i < n) {
      const int32_t s = list[i];
      const float g = grad[s];
      grad[s] = 0.f;  // the array is all-zero again after the push
      oldw = t.sl[s].w;
      neww = linear_update(t.sl[s], g, hp, hp.sgd_eta);
    }
    count_nnz_delta(oldw, neww, t.stats);
  }
  if (last) {
    __syncthreads();
    if (threadIdx.x == 0 && n) *ovf_cnt = 0u;
  }
}

}  // namespace

// the tile table for a minibatch of nnz non-zeros (see ld_rows_cap)
// (512-entry tiles: 70.0-70.3, 2048: 82.6-84.6 vs 77.2-83.8 M ex/s at 10k rows)
static int ld_table(int64_t nnz) { return nnz <= (int64_t)1 << 21 ? 1024 : 4096; }

int ld_rows_per_tile(int64_t nnz, int64_t nrows) {
  // ~T/2 non-zeros per tile, at most ld_rows_cap(T) rows (the tile's LDS
  // row offsets)
  const int T = ld_table(nnz);
  const int64_t avg = nrows > 0 ? (nnz + nrows - 1) / nrows : 1;
  int64_t R = (T / 2) / (avg > 0 ? avg : 1);
  const int64_t cap = ld_rows_cap(T);
  return (int)(R < 1 ? 1 : (R > cap ? cap : R));
}

int ld_tile_table(int64_t nnz) { return ld_table(nnz); }

void ld_touch(const KVTable& t, const uint64_t* keys, const int64_t* off, int64_t nrows,
              int64_t nnz, int R, uint32_t stamp, int insert, int32_t* lid, int32_t* tlist,
              unsigned int* tcnt, int32_t* ovf, unsigned int* ovf_cnt, hipStream_t s) {
  if (nrows <= 0) return;
  const int64_t nb = (nrows + R - 1) / R;
  const int T = ld_table(nnz);
  auto kern = T == 1024 ? k_ld_touch<1024> : k_ld_touch<4096>;
  hipLaunchKernelGGL(kern, dim3((unsigned)nb), dim3(kLdThreads), 0, s, t, keys, off, nrows, R,
                     stamp, insert, lid, tlist, tcnt, ovf, ovf_cnt);
}

void ld_backward(const int32_t* lid, const float* val, const int64_t* off, int64_t nrows,
                 int64_t nnz, int R, const float* dual, float* grad, hipStream_t s) {
  if (nrows <= 0) return;
  const int T = ld_table(nnz);
  if (R > ld_rows_cap(T)) throw std::runtime_error("ld_backward: tile rows exceed the LDS bound");
  const int64_t nb = (nrows + R - 1) / R;
  auto kern = T == 1024 ? k_ld_bwd<1024> : k_ld_bwd<4096>;
  hipLaunchKernelGGL(kern, dim3((unsigned)nb), dim3(kLdThreads), 0, s, lid, val, off, nrows, R,
                     dual, grad);
}

void ld_push(const KVTable& t, int64_t ntiles, int T, const int32_t* tlist,
             const unsigned int* tcnt, const int32_t* ovf, unsigned int* ovf_cnt, float* grad,
             LinearHP hp, hipStream_t s) {
  if (ntiles <= 0) return;
  hipLaunchKernelGGL(k_ld_push, dim3((unsigned)(ntiles + 1)), dim3(kLdThreads), 0, s, t, tlist,
                     tcnt, T, ovf, ovf_cnt, grad, hp);
}

}  // namespace wh
