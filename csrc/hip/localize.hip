// Minibatch localization on the GPU (K3 in SURVEY §2.5).
//
// Reference: learn/base/localizer.h:96-221 sorts (key, position) pairs with a
// thread-parallel std::sort, run-length encodes them and merge-joins back.
// Here the same map (uint64 feature id -> dense local id, plus per-id counts)
// is built with a device hash table, so no global sort is needed:
//
//   loc_count   : tiles of 1024 non-zeros de-duplicate in LDS first (so a
//                 hot feature costs one global atomic per tile, not one per
//                 occurrence), then insert the tile's unique ids into the
//                 batch table and add their tile counts.
//   loc_owner_hist / loc_assign : compact the occupied slots into local ids,
//                 grouped by owning shard so the id order IS the send order
//                 of the key exchange (no separate partition pass).
//   loc_csc     : per-id occurrence lists (CSC) for the atomic-free
//                 segmented backward; again LDS-aggregated per tile.
#include "wh_common.h"
#include "wh_kernels.h"

namespace wh {
namespace {

constexpr int kThreads = 256;
constexpr int kPer = 4;                       // items per thread
constexpr int kTileItems = kThreads * kPer;   // 1024
constexpr int kLds = 2 * kTileItems;          // LDS hash slots
constexpr int kMaxShard = 1024;

__device__ __forceinline__ uint64_t ld_relaxed(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int64_t table_insert(uint64_t* tkeys, uint64_t mask, uint64_t k) {
  uint64_t h = mix64(k) & mask;
  while (true) {
    uint64_t prev = ld_relaxed(tkeys + h);
    if (prev == k) return (int64_t)h;
    if (prev == kEmptyKey) {
      uint64_t old = atomicCAS((unsigned long long*)(tkeys + h), (unsigned long long)kEmptyKey,
                               (unsigned long long)k);
      if (old == kEmptyKey || old == k) return (int64_t)h;
    }
    h = (h + 1) & mask;
  }
}

__global__ __launch_bounds__(kThreads) void k_loc_count(const uint64_t* __restrict__ keys,
                                                        int64_t nnz, uint64_t* tkeys,
                                                        uint32_t* tcnt, uint64_t tmask,
                                                        int32_t* __restrict__ slot_of) {
  __shared__ unsigned long long sk[kLds];
  __shared__ uint32_t sc[kLds];
  __shared__ int32_t sg[kLds];
  for (int i = threadIdx.x; i < kLds; i += kThreads) {
    sk[i] = kEmptyKey;
    sc[i] = 0;
  }
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kTileItems;
  int ls[kPer];
#pragma unroll
  for (int r = 0; r < kPer; ++r) {
    const int64_t j = base + r * kThreads + threadIdx.x;
    ls[r] = -1;
    if (j < nnz) {
      const uint64_t k = keys[j];
      int h = (int)(mix64(k) & (kLds - 1));
      while (true) {
        unsigned long long prev = __hip_atomic_load(&sk[h], __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_WORKGROUP);
        if (prev == k) break;
        if (prev == kEmptyKey) {
          unsigned long long old = atomicCAS(&sk[h], (unsigned long long)kEmptyKey,
                                             (unsigned long long)k);
          if (old == kEmptyKey || old == k) break;
        }
        h = (h + 1) & (kLds - 1);
      }
      atomicAdd(&sc[h], 1u);
      ls[r] = h;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kLds; i += kThreads) {
    const uint64_t k = sk[i];
    if (k != kEmptyKey) {
      const int64_t g = table_insert(tkeys, tmask, k);
      atomicAdd(tcnt + g, sc[i]);
      sg[i] = (int32_t)g;
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kPer; ++r) {
    const int64_t j = base + r * kThreads + threadIdx.x;
    if (ls[r] >= 0) slot_of[j] = sg[ls[r]];
  }
}

__global__ __launch_bounds__(kThreads) void k_owner_hist(const uint64_t* __restrict__ tkeys,
                                                         int64_t tsize, int nshard,
                                                         int64_t* owner_cnt) {
  __shared__ int32_t h[kMaxShard];
  for (int i = threadIdx.x; i < nshard; i += kThreads) h[i] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < tsize;
       i += (int64_t)gridDim.x * kThreads) {
    const uint64_t k = tkeys[i];
    if (k != kEmptyKey) atomicAdd(&h[owner_of(k, nshard)], 1);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nshard; i += kThreads)
    if (h[i]) atomicAdd((unsigned long long*)(owner_cnt + i), (unsigned long long)h[i]);
}

constexpr int kAssignPer = 16;
__global__ __launch_bounds__(kThreads) void k_assign(const uint64_t* __restrict__ tkeys,
                                                     const uint32_t* __restrict__ tcnt,
                                                     int64_t tsize, int nshard,
                                                     int64_t* owner_cursor, int32_t* tlid,
                                                     uint64_t* uniq, int32_t* ucnt) {
  __shared__ int32_t lh[kMaxShard];
  __shared__ int64_t lb[kMaxShard];
  for (int i = threadIdx.x; i < nshard; i += kThreads) lh[i] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kThreads * kAssignPer;
  int own[kAssignPer], rk[kAssignPer];
#pragma unroll
  for (int r = 0; r < kAssignPer; ++r) {
    const int64_t i = base + (int64_t)r * kThreads + threadIdx.x;
    own[r] = -1;
    if (i < tsize) {
      const uint64_t k = tkeys[i];
      if (k != kEmptyKey) {
        own[r] = owner_of(k, nshard);
        rk[r] = atomicAdd(&lh[own[r]], 1);
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nshard; i += kThreads)
    if (lh[i])
      lb[i] = (int64_t)atomicAdd((unsigned long long*)(owner_cursor + i),
                                 (unsigned long long)lh[i]);
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kAssignPer; ++r) {
    if (own[r] >= 0) {
      const int64_t i = base + (int64_t)r * kThreads + threadIdx.x;
      const int64_t lid = lb[own[r]] + rk[r];
      tlid[i] = (int32_t)lid;
      uniq[lid] = tkeys[i];
      ucnt[lid] = (int32_t)tcnt[i];
    }
  }
}

__global__ void k_row_of(const int64_t* __restrict__ off, int64_t nrows, int32_t* row_of) {
  // one wave per row: lanes stride over the row's non-zeros
  const int64_t row = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (row >= nrows) return;
  for (int64_t j = off[row] + lane; j < off[row + 1]; j += 64) row_of[j] = (int32_t)row;
}

__global__ __launch_bounds__(kThreads) void k_loc_csc(const int32_t* __restrict__ slot_of,
                                                      const int32_t* __restrict__ tlid,
                                                      const int32_t* __restrict__ row_of,
                                                      const float* __restrict__ val,
                                                      int64_t nnz, int64_t* csc_cursor,
                                                      int32_t* __restrict__ lid_out,
                                                      int32_t* __restrict__ csc_row,
                                                      float* __restrict__ csc_val) {
  __shared__ int32_t sk[kLds];
  __shared__ int32_t sc[kLds];
  __shared__ int64_t sb[kLds];
  for (int i = threadIdx.x; i < kLds; i += kThreads) {
    sk[i] = -1;
    sc[i] = 0;
  }
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kTileItems;
  int ls[kPer];
  int32_t lid[kPer];
#pragma unroll
  for (int r = 0; r < kPer; ++r) {
    const int64_t j = base + r * kThreads + threadIdx.x;
    ls[r] = -1;
    if (j < nnz) {
      lid[r] = tlid[slot_of[j]];
      const uint32_t k = (uint32_t)lid[r];
      int h = (int)(mix64(k) & (kLds - 1));
      while (true) {
        int prev = __hip_atomic_load(&sk[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (prev == (int)k) break;
        if (prev == -1) {
          int old = atomicCAS(&sk[h], -1, (int)k);
          if (old == -1 || old == (int)k) break;
        }
        h = (h + 1) & (kLds - 1);
      }
      atomicAdd(&sc[h], 1);
      ls[r] = h;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kLds; i += kThreads) {
    const int k = sk[i];
    if (k >= 0) {
      sb[i] = (int64_t)atomicAdd((unsigned long long*)(csc_cursor + k),
                                 (unsigned long long)sc[i]);
      sc[i] = 0;  // reuse as the in-tile rank cursor
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kPer; ++r) {
    if (ls[r] >= 0) {
      const int64_t j = base + r * kThreads + threadIdx.x;
      const int64_t pos = sb[ls[r]] + atomicAdd(&sc[ls[r]], 1);
      lid_out[j] = lid[r];
      csc_row[pos] = row_of[j];
      if (csc_val) csc_val[pos] = val[j];
    }
  }
}

}  // namespace

void loc_count(const uint64_t* keys, int64_t nnz, uint64_t* tkeys, uint32_t* tcnt,
               int64_t tsize, int32_t* slot_of, hipStream_t s) {
  if (nnz <= 0) return;
  const int64_t nb = (nnz + kTileItems - 1) / kTileItems;
  hipLaunchKernelGGL(k_loc_count, dim3((unsigned)nb), dim3(kThreads), 0, s, keys, nnz, tkeys,
                     tcnt, (uint64_t)(tsize - 1), slot_of);
}

void loc_owner_hist(const uint64_t* tkeys, int64_t tsize, int nshard, int64_t* owner_cnt,
                    hipStream_t s) {
  hipLaunchKernelGGL(k_owner_hist, dim3(grid_for(tsize, kThreads, 2048)), dim3(kThreads), 0, s,
                     tkeys, tsize, nshard, owner_cnt);
}

void loc_assign(const uint64_t* tkeys, const uint32_t* tcnt, int64_t tsize, int nshard,
                int64_t* owner_cursor, int32_t* tlid, uint64_t* uniq, int32_t* ucnt,
                hipStream_t s) {
  const int64_t per_block = (int64_t)kThreads * kAssignPer;
  const int64_t nb = (tsize + per_block - 1) / per_block;
  hipLaunchKernelGGL(k_assign, dim3((unsigned)nb), dim3(kThreads), 0, s, tkeys, tcnt, tsize,
                     nshard, owner_cursor, tlid, uniq, ucnt);
}

void row_of_nnz(const int64_t* offset, int64_t nrows, int32_t* row_of, hipStream_t s) {
  if (nrows <= 0) return;
  const int64_t threads = nrows * 64;
  hipLaunchKernelGGL(k_row_of, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, offset,
                     nrows, row_of);
}

void loc_csc(const int32_t* slot_of, const int32_t* tlid, const int32_t* row_of,
             const float* val, int64_t nnz, int64_t* csc_cursor, int32_t* lid,
             int32_t* csc_row, float* csc_val, hipStream_t s) {
  if (nnz <= 0) return;
  const int64_t nb = (nnz + kTileItems - 1) / kTileItems;
  hipLaunchKernelGGL(k_loc_csc, dim3((unsigned)nb), dim3(kThreads), 0, s, slot_of, tlid, row_of,
                     val, nnz, csc_cursor, lid, csc_row, csc_val);
}

}  // namespace wh
