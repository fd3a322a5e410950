// Minibatch localization on the GPU (K3 in SURVEY §2.5).
//
// Reference: learn/base/localizer.h:96-221 sorts (key, position) pairs of
// 64-bit ids with a thread-parallel std::sort, run-length encodes them and
// merge-joins back. Here the same map (uint64 feature id -> dense local id,
// per-id counts, and per-id occurrence lists) is built without a 64-bit sort
// and without a per-occurrence global atomic:
//
//   loc_insert  : tiles of 1024 non-zeros de-duplicate in LDS first, then
//                 find-or-insert the tile's distinct ids into a batch hash
//                 table (one CAS per NEW id; hot ids cost one plain load per
//                 tile). Writes slot_of[nnz].
//   loc_owner_count / loc_assign : compact the occupied slots into local
//                 ids, grouped by owning shard so the id order IS the send
//                 order of the key exchange (no separate partition pass);
//                 per-block owner counts + one scan, no global atomics.
//   loc_rows_lid: lid[j] = tlid[slot_of[j]] (the nnz -> local id map) and
//                 the row of every non-zero, one wave per row;
//   loc_csc     : a radix sort of (lid, j) pairs on ceil(log2 U) bits
//                 (rocPRIM onesweep; stable, so every id's occurrence list
//                 comes out in row order -> a deterministic CSC), then
//                 csc_row/csc_val gathered through the sorted positions and
//                 csc_off/ucnt from the run boundaries of the sorted ids.
//
// Per-occurrence global atomics were the cost of the previous design (MI355X
// executes global atomics at the memory side, one 64-B request each; rocprof
// showed ~3.6M + 3M atomic requests per 100k-row minibatch).
#include <rocprim/device/device_radix_sort.hpp>

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

// returns the slot, or -1 once the probe sequence has visited every slot
// (table full: the caller flags an overflow and the host retries larger)
__device__ __forceinline__ int64_t table_insert_from(uint64_t* tkeys, uint64_t mask, uint64_t k,
                                                     uint64_t h) {
  for (uint64_t probe = 0; probe < mask; ++probe) {
    uint64_t prev = ld_relaxed(tkeys + h);
    if (prev == k) return (int64_t)h;
    if (prev == kEmptyKey) {
      uint64_t old = atomicCAS((unsigned long long*)(tkeys + h), (unsigned long long)kEmptyKey,
                               (unsigned long long)k);
      if (old == kEmptyKey || old == k) return (int64_t)h;
    }
    h = (h + 1) & mask;
  }
  return -1;
}

__global__ __launch_bounds__(kThreads) void k_loc_insert(const uint64_t* __restrict__ keys,
                                                         int64_t nnz, uint64_t* tkeys,
                                                         uint64_t tmask,
                                                         int32_t* __restrict__ slot_of,
                                                         int64_t* overflow) {
  __shared__ unsigned long long sk[kLds];
  __shared__ int32_t sg[kLds];
  for (int i = threadIdx.x; i < kLds; i += kThreads) sk[i] = kEmptyKey;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kTileItems;
  int ls[kPer];
  uint64_t kin[kPer];
#pragma unroll
  for (int r = 0; r < kPer; ++r) {  // all key loads in flight before the LDS work
    const int64_t j = base + r * kThreads + threadIdx.x;
    kin[r] = j < nnz ? keys[j] : kEmptyKey;
  }
#pragma unroll
  for (int r = 0; r < kPer; ++r) {
    const uint64_t k = kin[r];
    ls[r] = -1;
    if (k != kEmptyKey) {
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
      ls[r] = h;
    }
  }
  __syncthreads();
  // Global find-or-insert of the tile's distinct ids, batched so that every
  // thread has all its probes in flight at once: round 1 loads the home slot
  // of each id, round 2 CASes the ids whose home slot was empty; only ids
  // that met another id (load factor ~0.25: rare) walk the probe sequence.
  constexpr int kSlotsPer = kLds / kThreads;
  uint64_t gk[kSlotsPer], gh[kSlotsPer], gp[kSlotsPer];
#pragma unroll
  for (int q = 0; q < kSlotsPer; ++q) {
    gk[q] = sk[q * kThreads + threadIdx.x];
    gh[q] = mix64(gk[q]) & tmask;
    gp[q] = gk[q] != kEmptyKey ? ld_relaxed(tkeys + gh[q]) : 0;
  }
#pragma unroll
  for (int q = 0; q < kSlotsPer; ++q) {
    if (gk[q] != kEmptyKey && gp[q] == kEmptyKey)
      gp[q] = atomicCAS((unsigned long long*)(tkeys + gh[q]), (unsigned long long)kEmptyKey,
                        (unsigned long long)gk[q]);
    // gp[q] is now kEmptyKey (we inserted), gk[q] (present) or another id
  }
#pragma unroll
  for (int q = 0; q < kSlotsPer; ++q) {
    const uint64_t k = gk[q];
    if (k == kEmptyKey) continue;
    int64_t g = (int64_t)gh[q];
    if (gp[q] != kEmptyKey && gp[q] != k)
      g = table_insert_from(tkeys, tmask, k, (gh[q] + 1) & tmask);
    if (g < 0) atomicAdd((unsigned long long*)overflow, 1ull);
    sg[q * kThreads + threadIdx.x] = g >= 0 ? (int32_t)g : 0;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kPer; ++r) {
    const int64_t j = base + r * kThreads + threadIdx.x;
    if (ls[r] >= 0) slot_of[j] = sg[ls[r]];
  }
}

constexpr int kAssignPer = 16;
constexpr int64_t kAssignItems = (int64_t)kThreads * kAssignPer;  // table slots per block

// Per-block owner histogram of the occupied table slots, written owner-major
// (blkcnt[owner * nblk + block]) so that one exclusive scan gives every
// block's first local id in every owner group -- no same-address atomics
// (each costs ~12 ns serialised; 2K blocks x 2 passes were ~45 us).
__global__ __launch_bounds__(kThreads) void k_owner_count(const uint64_t* __restrict__ tkeys,
                                                          int64_t tsize, int nshard,
                                                          int64_t* __restrict__ blkcnt) {
  __shared__ int32_t h[kMaxShard];
  for (int i = threadIdx.x; i < nshard; i += kThreads) h[i] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kAssignItems;
#pragma unroll
  for (int r = 0; r < kAssignPer; ++r) {
    const int64_t i = base + (int64_t)r * kThreads + threadIdx.x;
    if (i < tsize) {
      const uint64_t k = tkeys[i];
      if (k != kEmptyKey) {
        if (nshard == 1) {
          const uint64_t b = __ballot(1);
          if ((threadIdx.x & 63) == __ffsll((unsigned long long)b) - 1)
            atomicAdd(&h[0], (int)__popcll(b));
        } else {
          atomicAdd(&h[owner_of(k, nshard)], 1);
        }
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nshard; i += kThreads)
    blkcnt[(int64_t)i * gridDim.x + blockIdx.x] = h[i];
}

// Single-block exclusive scan of n (<= a few 100K) int64 counts in place,
// then owner totals: owner_cnt[o] = sum of blkcnt[o * nblk .. (o+1) * nblk).
__global__ __launch_bounds__(1024) void k_owner_scan(int64_t* __restrict__ blk, int64_t nblk,
                                                     int nshard, int64_t* __restrict__ owner_cnt,
                                                     int64_t* __restrict__ ovf) {
  // the insert's overflow count travels with the owner counts (one host
  // read) and the persistent counter is re-armed for the next minibatch
  if (threadIdx.x == 0) {
    owner_cnt[nshard] = *ovf;
    *ovf = 0;
  }
  __shared__ int64_t part[1024];
  const int64_t n = nblk * nshard;
  const int64_t per = (n + 1023) / 1024;
  const int64_t b = threadIdx.x * per, e = b + per < n ? b + per : n;
  int64_t acc = 0;
  for (int64_t i = b; i < e; ++i) acc += blk[i];
  part[threadIdx.x] = acc;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan
    const int64_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  int64_t run = threadIdx.x ? part[threadIdx.x - 1] : 0;
  for (int64_t i = b; i < e; ++i) {
    const int64_t c = blk[i];
    blk[i] = run;
    run += c;
  }
  __syncthreads();
  const int64_t total = part[1023];
  for (int o = threadIdx.x; o < nshard; o += 1024) {
    const int64_t lo = blk[(int64_t)o * nblk];
    const int64_t hi = o + 1 < nshard ? blk[(int64_t)(o + 1) * nblk] : total;
    owner_cnt[o] = hi - lo;
  }
}

// lid of every occupied slot: the block's scanned offset in its owner group
// plus the slot's rank among the block's slots of that owner.
__global__ __launch_bounds__(kThreads) void k_assign(uint64_t* __restrict__ tkeys,
                                                     int64_t tsize, int nshard,
                                                     const int64_t* __restrict__ blkoff,
                                                     int32_t* tlid, uint64_t* uniq) {
  __shared__ int32_t lh[kMaxShard];
  for (int i = threadIdx.x; i < nshard; i += kThreads) lh[i] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kAssignItems;
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
#pragma unroll
  for (int r = 0; r < kAssignPer; ++r) {
    if (own[r] >= 0) {
      const int64_t i = base + (int64_t)r * kThreads + threadIdx.x;
      const int64_t lid = blkoff[(int64_t)own[r] * gridDim.x + blockIdx.x] + rk[r];
      tlid[i] = (int32_t)lid;
      uniq[lid] = tkeys[i];
      tkeys[i] = kEmptyKey;  // leave the persistent scratch table empty
    }
  }
}

// one wave per CSR row: the row id and the local id of each of its non-zeros
// (lid[j] = tlid[slot_of[j]]), plus the position payload for valued data
// A block owns kRowsPerBlk consecutive rows, i.e. one contiguous nnz range:
// every lane works (a wave per row left 25 of 64 lanes idle on 39-field rows)
// and each nnz finds its row by a binary search over the block's offsets in
// LDS; four slot -> local-id gathers per thread are in flight at once.
constexpr int kRowsPerBlk = 64;

__global__ __launch_bounds__(kThreads) void k_rows_lid(const int64_t* __restrict__ off,
                                                       int64_t nrows,
                                                       const int32_t* __restrict__ slot_of,
                                                       const int32_t* __restrict__ tlid,
                                                       int32_t* __restrict__ row_of,
                                                       int32_t* __restrict__ lid,
                                                       int32_t* __restrict__ pos) {
  __shared__ int64_t so[kRowsPerBlk + 1];
  const int64_t r0 = (int64_t)blockIdx.x * kRowsPerBlk;
  const int nr = (int)(nrows - r0 < kRowsPerBlk ? nrows - r0 : kRowsPerBlk);
  if (threadIdx.x <= nr) so[threadIdx.x] = off[r0 + threadIdx.x];
  __syncthreads();
  const int64_t j0 = so[0], j1 = so[nr];
  auto row_at = [&](int64_t j) {  // largest k < nr with so[k] <= j
    int lo = 0, hi = nr - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (so[mid] <= j) lo = mid;
      else hi = mid - 1;
    }
    return lo;
  };
  for (int64_t b = j0; b < j1; b += 4 * kThreads) {
    int sl[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t j = b + u * kThreads + threadIdx.x;
      sl[u] = j < j1 ? slot_of[j] : 0;
    }
    int li[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) li[u] = tlid[sl[u]];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t j = b + u * kThreads + threadIdx.x;
      if (j < j1) {
        row_of[j] = (int32_t)(r0 + row_at(j));
        lid[j] = li[u];
        if (pos) pos[j] = (int32_t)j;
      }
    }
  }
}

__global__ __launch_bounds__(kThreads) void k_loc_csc(const int32_t* __restrict__ slid,
                                                      const int32_t* __restrict__ spos,
                                                      const int32_t* __restrict__ row_of,
                                                      const float* __restrict__ val, int64_t nnz,
                                                      int64_t nuniq, int32_t* __restrict__ csc_row,
                                                      float* __restrict__ csc_val,
                                                      int64_t* __restrict__ csc_off) {
  const int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (p >= nnz) {
    if (p == nnz) csc_off[nuniq] = nnz;
    return;
  }
  if (spos) {  // valued data: rows and values gathered through the sorted positions
    const int32_t j = spos[p];
    csc_row[p] = row_of[j];
    csc_val[p] = val[j];
  }  // (binary data: the sort carried the row ids straight into csc_row)
  const int32_t k = slid[p];
  if (p == 0 || slid[p - 1] != k) csc_off[k] = p;  // every id occurs at least once
}

__global__ __launch_bounds__(kThreads) void k_ucnt(const int64_t* __restrict__ csc_off,
                                                   int64_t nuniq, int32_t* __restrict__ ucnt) {
  const int64_t k = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (k < nuniq) ucnt[k] = (int32_t)(csc_off[k + 1] - csc_off[k]);
}

__global__ __launch_bounds__(kThreads) void k_key_mod(uint64_t* keys, int64_t n, uint64_t m) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i < n) keys[i] %= m;
}

inline int bits_for(int64_t n) {
  int b = 1;
  while (b < 31 && ((int64_t)1 << b) < n) ++b;
  return b;
}

}  // namespace

void loc_insert(const uint64_t* keys, int64_t nnz, uint64_t* tkeys, int64_t tsize,
                int32_t* slot_of, int64_t* overflow, hipStream_t s) {
  if (nnz <= 0) return;
  const int64_t nb = (nnz + kTileItems - 1) / kTileItems;
  hipLaunchKernelGGL(k_loc_insert, dim3((unsigned)nb), dim3(kThreads), 0, s, keys, nnz, tkeys,
                     (uint64_t)(tsize - 1), slot_of, overflow);
}

int64_t loc_owner_blocks(int64_t tsize) { return (tsize + kAssignItems - 1) / kAssignItems; }

void loc_owner_count(const uint64_t* tkeys, int64_t tsize, int nshard, int64_t* blkcnt,
                     int64_t* owner_cnt, int64_t* overflow, hipStream_t s) {
  const int64_t nb = loc_owner_blocks(tsize);
  hipLaunchKernelGGL(k_owner_count, dim3((unsigned)nb), dim3(kThreads), 0, s, tkeys, tsize,
                     nshard, blkcnt);
  hipLaunchKernelGGL(k_owner_scan, dim3(1), dim3(1024), 0, s, blkcnt, nb, nshard, owner_cnt,
                     overflow);
}

void loc_assign(uint64_t* tkeys, int64_t tsize, int nshard, const int64_t* blkoff,
                int32_t* tlid, uint64_t* uniq, hipStream_t s) {
  const int64_t nb = loc_owner_blocks(tsize);
  hipLaunchKernelGGL(k_assign, dim3((unsigned)nb), dim3(kThreads), 0, s, tkeys, tsize, nshard,
                     blkoff, tlid, uniq);
}

void loc_rows_lid(const int64_t* offset, int64_t nrows, const int32_t* slot_of,
                  const int32_t* tlid, int32_t* row_of, int32_t* lid, int32_t* pos,
                  hipStream_t s) {
  if (nrows <= 0) return;
  static_assert(kRowsPerBlk < kThreads, "offset staging needs a thread per row");
  hipLaunchKernelGGL(k_rows_lid, dim3((unsigned)((nrows + kRowsPerBlk - 1) / kRowsPerBlk)),
                     dim3(kThreads), 0, s, offset, nrows, slot_of, tlid, row_of, lid, pos);
}

size_t loc_sort_tmp_bytes(int64_t nnz, int64_t nuniq) {
  size_t bytes = 0;
  WH_HIP_CHECK(rocprim::radix_sort_pairs(nullptr, bytes, (int32_t*)nullptr, (int32_t*)nullptr,
                                         (int32_t*)nullptr, (int32_t*)nullptr,
                                         (size_t)std::max<int64_t>(nnz, 1), 0, bits_for(nuniq),
                                         (hipStream_t)0));
  return bytes;
}

void loc_csc(const int32_t* row_of, const float* val, int64_t nnz, int64_t nuniq,
             int32_t* lid, int32_t* pos,
             int32_t* slid, int32_t* spos, void* sort_tmp, size_t sort_tmp_bytes,
             int64_t* csc_off, int32_t* ucnt, int32_t* csc_row, float* csc_val, hipStream_t s) {
  if (nnz <= 0) {
    hipLaunchKernelGGL(k_loc_csc, dim3(1), dim3(kThreads), 0, s, slid, spos, row_of, val,
                       (int64_t)0, nuniq, csc_row, csc_val, csc_off);
    return;
  }
  // binary data (no values): sort the row ids themselves as the payload,
  // straight into csc_row; valued data: sort positions, then gather
  int32_t* vin = val ? pos : const_cast<int32_t*>(row_of);
  int32_t* vout = val ? spos : csc_row;
  size_t bytes = sort_tmp_bytes;
  WH_HIP_CHECK(rocprim::radix_sort_pairs(sort_tmp, bytes, lid, slid, vin, vout, (size_t)nnz, 0,
                                         bits_for(nuniq), s));
  hipLaunchKernelGGL(k_loc_csc, dim3(grid_for(nnz + 1, kThreads)), dim3(kThreads), 0, s, slid,
                     val ? spos : nullptr, row_of, val, nnz, nuniq, csc_row, csc_val, csc_off);
  hipLaunchKernelGGL(k_ucnt, dim3(grid_for(nuniq, kThreads)), dim3(kThreads), 0, s, csc_off,
                     nuniq, ucnt);
}

}  // namespace wh

namespace wh {

void key_mod(uint64_t* keys, int64_t n, uint64_t m, hipStream_t s) {
  if (n <= 0 || m == 0) return;
  hipLaunchKernelGGL(k_key_mod, dim3(grid_for(n, kThreads)), dim3(kThreads), 0, s, keys, n, m);
}

}  // namespace wh
