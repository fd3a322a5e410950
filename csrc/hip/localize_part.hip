// Partitioned minibatch localization: the default K3 path.
//
// Same outputs as the hash-insert + radix-sort path of localize.hip
// (reference learn/base/localizer.h:96-221: unique ids, per-id counts, the
// nnz -> local id map and the per-id occurrence lists), built without ANY
// global atomic and without a sort:
//
//   part_hist    : tiles of R whole rows; per-tile histogram (LDS) of a
//                  partition digit d(key) = owner(key) * NPO + hash bits.
//   scan_i32     : digit-major exclusive scan of the tile histograms.
//   part_scatter : every non-zero (key, row, position) moves to its
//                  partition's range -- one radix-partition pass.
//   part_dedup   : one 1024-thread workgroup per partition: the partition's
//                  ~1K distinct ids de-duplicate in an LDS hash table, are
//                  counted there, get their local ids (partition order; the
//                  partition base by decoupled look-back) and occurrence
//                  offsets (partition range + LDS scan), and every non-zero
//                  is placed into the CSC and mapped back to its local id.
//
// The previous path paid ~3M random global operations per 100k-row
// minibatch (hash find-or-insert after LDS tile de-duplication, then three
// onesweep radix passes over (lid, row) pairs); MI355X serves random global
// accesses at ~20 (atomics) to ~100 (loads) per ns, which bounded it at
// ~350 us. Here every global access is a streaming or partition-local one.
//
// Because the digit is owner-major, local ids come out grouped by owning
// shard (the key exchange's send order) with no separate pass, and the owner
// counts are sums of partition counts. The order of occurrences inside an
// id's list and of ids inside a partition depends on LDS atomic timing
// (the hash path of localize.hip stays available as the deterministic one).
#include "wh_common.h"
#include "wh_kernels.h"
#include "wh_lookback.h"

#include <cstdlib>

namespace wh {
namespace {

constexpr int kPartThreads = 256;
constexpr int kDedupThreads = 1024;
constexpr int kDedupSlots = 4096;                        // LDS hash slots per partition
constexpr int kDedupPer = kDedupSlots / kDedupThreads;   // slots per thread in the scan
constexpr int kDedupMaxProbe = kDedupSlots;
constexpr int kDU = 4;  // non-zeros per thread per pass in the dedup loops

// Owner o's digits are [o * stride, (o + 1) * stride): groups of g = NPO /
// nho hashed digits, each followed by one heavy-id digit (interleaved, so
// that the hot ids' local ids -- and the backward's per-key work on them --
// are spread over the id range instead of packed at its end).
__device__ __forceinline__ int part_digit(uint64_t k, int nshard, int npo_bits, int stride,
                                          int gbits) {
  const int own = owner_of(k, nshard);
  const int sub = (int)((mix64(k) >> 40) & ((1ull << npo_bits) - 1ull));
  return own * stride + (sub >> gbits) * ((1 << gbits) + 1) + (sub & ((1 << gbits) - 1));
}

__device__ __forceinline__ int heavy_digit(int own, int q, int stride, int gbits) {
  return own * stride + q * ((1 << gbits) + 1) + (1 << gbits);
}

// Heavy ids (the previous minibatch's ids with >= thr occurrences) get
// single-id partitions of their own: owner o's digits are [o * stride,
// o * stride + NPO) for hashed ids and [o * stride + NPO, (o + 1) * stride)
// for its heavy ids. Without them a power-law head (one Criteo id is in 63%
// of the rows) lands in one hashed partition whose workgroup serialises the
// whole step (dedup timing: 50 us of 115 us in that one partition).
constexpr int kHeavySlots = 1024;  // LDS hash of <= kPartMaxHeavy ids
constexpr int kPartHeavyTotal = 128;  // heavy-id partitions over all owners (target)

__host__ __device__ __forceinline__ int log2_nho(int nho) {
  int b = 0;
  while ((2 << b) <= nho) ++b;
  return nho > 0 ? b : 0;
}

__device__ __forceinline__ void heavy_build(const PartHeavy& hv, int nshard, int npo_bits,
                                            int stride, int nho, unsigned long long* hk, int* hd) {
  for (int i = threadIdx.x; i < kHeavySlots; i += blockDim.x) hk[i] = kEmptyKey;
  __syncthreads();
  if (hv.nho == 0) return;
  for (int i = threadIdx.x; i < nshard * hv.nho; i += blockDim.x) {
    const int o = i / hv.nho, q = i - o * hv.nho;
    const uint32_t n = hv.cnt[o];
    if ((uint32_t)q >= n) continue;
    const uint64_t k = hv.keys[i];
    if (owner_of(k, nshard) != o) continue;  // (never, with a matching layout)
    int h = (int)((mix64(k) >> 8) & (kHeavySlots - 1));
    while (true) {
      const unsigned long long old =
          atomicCAS(&hk[h], (unsigned long long)kEmptyKey, (unsigned long long)k);
      if (old == kEmptyKey) {
        hd[h] = heavy_digit(o, q, stride, npo_bits - log2_nho(nho));
        break;
      }
      if (old == k) break;
      h = (h + 1) & (kHeavySlots - 1);
    }
  }
  __syncthreads();
}

__device__ __forceinline__ int digit_of(uint64_t k, const unsigned long long* hk, const int* hd,
                                        bool heavy_on, int nshard, int npo_bits, int stride,
                                        int nho) {
  if (heavy_on) {
    int h = (int)((mix64(k) >> 8) & (kHeavySlots - 1));
    while (true) {
      const unsigned long long v = hk[h];
      if (v == k) return hd[h];
      if (v == kEmptyKey) break;
      h = (h + 1) & (kHeavySlots - 1);
    }
  }
  return part_digit(k, nshard, npo_bits, stride, npo_bits - log2_nho(nho));
}

// tile t's row range [r0, r1)
__device__ __forceinline__ void tile_rows(int64_t t, int64_t nrows, int R, int64_t& r0,
                                          int64_t& r1) {
  r0 = t * R;
  r1 = r0 + R < nrows ? r0 + R : nrows;
}

__global__ __launch_bounds__(kPartThreads) void k_part_hist(const uint64_t* __restrict__ keys,
                                                            const int64_t* __restrict__ off,
                                                            int64_t nrows, int R, int nshard,
                                                            int npo_bits, int stride, int nho,
                                                            int ndig, PartHeavy hv,
                                                            uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[kPartMaxDigits];
  __shared__ unsigned long long hk[kHeavySlots];
  __shared__ int hd[kHeavySlots];
  for (int i = threadIdx.x; i < ndig; i += kPartThreads) h[i] = 0;
  if (blockIdx.x == 0 && hv.next_cnt)  // the heavy ids this minibatch elects start empty
    for (int i = threadIdx.x; i < nshard; i += kPartThreads) hv.next_cnt[i] = 0;
  heavy_build(hv, nshard, npo_bits, stride, nho, hk, hd);
  const bool hon = hv.nho > 0;
  int64_t r0, r1;
  tile_rows(blockIdx.x, nrows, R, r0, r1);
  const int64_t j0 = off[r0], j1 = off[r1];
  for (int64_t b = j0; b < j1; b += 4 * kPartThreads) {
    uint64_t k[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t j = b + u * kPartThreads + threadIdx.x;
      k[u] = j < j1 ? keys[j] : 0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t j = b + u * kPartThreads + threadIdx.x;
      if (j < j1) atomicAdd(&h[digit_of(k[u], hk, hd, hon, nshard, npo_bits, stride, nho)], 1u);
    }
  }
  __syncthreads();
  // tile-major: one coalesced row per tile (a digit-major layout made every
  // block store its ndig counters to ndig different cache lines)
  for (int i = threadIdx.x; i < ndig; i += kPartThreads)
    hist[(int64_t)blockIdx.x * ndig + i] = h[i];
}

// Partition offsets from the tile-major histogram without a transposing
// scan: off(t, d) = base[d] + gpre[t / kColTB][d] + hist'[t][d], where hist'
// is the exclusive prefix of digit d over the tiles of t's group (in place),
// gpre the exclusive prefix over groups and base the exclusive prefix of the
// digit totals (base[ndig] = nnz). Every access is a coalesced row.
constexpr int kColTB = 16;  // tiles per group

__global__ __launch_bounds__(256) void k_part_colpre(uint32_t* __restrict__ hist, int ntiles,
                                                     int ndig, uint32_t* __restrict__ gsum) {
  const int t0 = blockIdx.x * kColTB;
  const int t1 = t0 + kColTB < ntiles ? t0 + kColTB : ntiles;
  for (int d = threadIdx.x; d < ndig; d += 256) {
    uint32_t v[kColTB];
#pragma unroll
    for (int u = 0; u < kColTB; ++u) v[u] = t0 + u < t1 ? hist[(int64_t)(t0 + u) * ndig + d] : 0u;
    uint32_t run = 0;
#pragma unroll
    for (int u = 0; u < kColTB; ++u) {
      if (t0 + u < t1) hist[(int64_t)(t0 + u) * ndig + d] = run;
      run += v[u];
    }
    gsum[(int64_t)blockIdx.x * ndig + d] = run;
  }
}

__global__ __launch_bounds__(1024) void k_part_base(uint32_t* __restrict__ gsum, int ngroups,
                                                    int ndig, int64_t* __restrict__ base) {
  __shared__ uint32_t wt[16];
  const int d = threadIdx.x, lane = d & 63, w = d >> 6;
  uint32_t run = 0;
  if (d < ndig) {
    for (int g0 = 0; g0 < ngroups; g0 += 8) {  // 8 independent loads in flight
      uint32_t v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = g0 + u < ngroups ? gsum[(int64_t)(g0 + u) * ndig + d] : 0u;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (g0 + u < ngroups) gsum[(int64_t)(g0 + u) * ndig + d] = run;
        run += v[u];
      }
    }
  }
  // exclusive scan of the digit totals (ndig <= 1024 = blockDim)
  uint32_t x = run;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wt[w] = x;
  __syncthreads();
  uint32_t pre = 0;
  for (int q = 0; q < w; ++q) pre += wt[q];
  if (d < ndig) base[d] = (int64_t)(pre + x - run);
  if (d == ndig - 1) base[ndig] = (int64_t)(pre + x);
}

// Each tile's non-zeros go to [off(tile, d) ...) of their digit (off: see
// k_part_colpre). A tile is
// processed in chunks of kChunk non-zeros that are counting-sorted by digit
// in LDS first, so that consecutive lanes store consecutive addresses of a
// digit's run (scattered 4/8-byte stores cost one memory request each:
// storing in arrival order made this pass 140 us per 100k rows). The row of
// a non-zero comes from a binary search over the tile's row offsets in LDS
// (a tile owns whole rows); pos_of[j] (the non-zero's partition position) is
// stored in CSR order by the thread that loaded it.
constexpr int kScatThreads = 512;
constexpr int kScatPer = 8;
constexpr int kChunk = kScatThreads * kScatPer;  // 4096

size_t scatter_lds_bytes(int ndig, bool has_val) {
  return (size_t)3 * ndig * 4 + 8 + (size_t)(kPartMaxRows + 1) * 8 +
         (size_t)kChunk * (has_val ? 18 : 14);
}

__global__ __launch_bounds__(kScatThreads, 4) void k_part_scatter(
    const uint64_t* __restrict__ keys, const float* __restrict__ val,
    const int64_t* __restrict__ off, int64_t nrows, int R, int nshard, int npo_bits, int stride,
    int nho, int ndig, PartHeavy hv, const int64_t* __restrict__ base,
    const uint32_t* __restrict__ gpre, const uint32_t* __restrict__ tpre, uint64_t* __restrict__ pk,
    int32_t* __restrict__ pr, float* __restrict__ pv, int32_t* __restrict__ pos_of) {
  extern __shared__ __align__(16) unsigned char lds[];
  uint32_t* gbase = reinterpret_cast<uint32_t*>(lds);   // next free position per digit
  uint32_t* cnt = gbase + ndig;                          // chunk counts -> chunk starts
  uint32_t* lst = cnt + ndig;
  int64_t* so = reinterpret_cast<int64_t*>(lst + ndig + (ndig & 1));
  uint64_t* sk = reinterpret_cast<uint64_t*>(so + kPartMaxRows + 1);
  int32_t* sr = reinterpret_cast<int32_t*>(sk + kChunk);
  uint16_t* sd = reinterpret_cast<uint16_t*>(sr + kChunk);  // digit of each staged id
  float* sv = reinterpret_cast<float*>(sd + kChunk);
  __shared__ uint32_t wsum[kScatThreads / 64];
  __shared__ unsigned long long hk[kHeavySlots];
  __shared__ int hd[kHeavySlots];
  heavy_build(hv, nshard, npo_bits, stride, nho, hk, hd);
  const bool hon = hv.nho > 0;
  // neighbouring tiles write neighbouring runs of every partition (often the
  // same 128-byte lines): an XCD takes a contiguous range of tiles so those
  // partial-line writes merge in its L2
  const int64_t tile = xcd_swizzle(blockIdx.x, gridDim.x);
  int64_t r0, r1;
  tile_rows(tile, nrows, R, r0, r1);
  const int nr = (int)(r1 - r0);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < ndig; i += kScatThreads)
    gbase[i] = (uint32_t)base[i] + gpre[(tile / kColTB) * ndig + i] +
               tpre[tile * ndig + i];
  for (int i = threadIdx.x; i <= nr; i += kScatThreads) so[i] = off[r0 + i];
  __syncthreads();
  const int64_t j0 = so[0], j1 = so[nr];
  for (int64_t b = j0; b < j1; b += kChunk) {
    for (int i = threadIdx.x; i < ndig; i += kScatThreads) cnt[i] = 0;
    __syncthreads();
    uint64_t k[kScatPer];
    int d[kScatPer];
    uint32_t rk[kScatPer];
#pragma unroll
    for (int u = 0; u < kScatPer; ++u) {
      const int64_t j = b + u * kScatThreads + threadIdx.x;
      k[u] = j < j1 ? keys[j] : 0;
    }
#pragma unroll
    for (int u = 0; u < kScatPer; ++u) {
      const int64_t j = b + u * kScatThreads + threadIdx.x;
      d[u] = j < j1 ? digit_of(k[u], hk, hd, hon, nshard, npo_bits, stride, nho) : -1;
      rk[u] = d[u] >= 0 ? atomicAdd(&cnt[d[u]], 1u) : 0u;
    }
    __syncthreads();
    // exclusive scan of the chunk's digit counts (ndig <= kPartMaxDigits)
    constexpr int kDPer = kPartMaxDigits / kScatThreads;
    uint32_t c[kDPer], tsum = 0;
#pragma unroll
    for (int q = 0; q < kDPer; ++q) {
      const int i = threadIdx.x * kDPer + q;
      c[q] = i < ndig ? cnt[i] : 0u;
      tsum += c[q];
    }
    uint32_t inc = tsum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o, 64);
      if (lane >= o) inc += y;
    }
    if (lane == 63) wsum[wid] = inc;
    __syncthreads();
    uint32_t run = inc - tsum;
    for (int w = 0; w < wid; ++w) run += wsum[w];
#pragma unroll
    for (int q = 0; q < kDPer; ++q) {
      const int i = threadIdx.x * kDPer + q;
      if (i < ndig) lst[i] = run;
      run += c[q];
    }
    __syncthreads();
    // stage digit-sorted; every loading thread knows its partition position
#pragma unroll
    for (int u = 0; u < kScatPer; ++u) {
      if (d[u] < 0) continue;
      const int64_t j = b + u * kScatThreads + threadIdx.x;
      const uint32_t lp = lst[d[u]] + rk[u];
      int lo = 0, hi = nr - 1;  // largest row index with so[row] <= j
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (so[mid] <= j) lo = mid;
        else hi = mid - 1;
      }
      sk[lp] = k[u];
      sr[lp] = (int32_t)(r0 + lo);
      sd[lp] = (uint16_t)d[u];
      if (val) sv[lp] = val[j];
      pos_of[j] = (int32_t)(gbase[d[u]] + rk[u]);
    }
    __syncthreads();
    const int n = (int)(j1 - b < kChunk ? j1 - b : kChunk);
    for (int i = threadIdx.x; i < n; i += kScatThreads) {
      const int dd = sd[i];
      const uint32_t gp = gbase[dd] + (uint32_t)i - lst[dd];
      pk[gp] = sk[i];
      pr[gp] = sr[i];
      if (val) pv[gp] = sv[i];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < ndig; i += kScatThreads) gbase[i] += cnt[i];
    __syncthreads();
  }
}

__device__ __forceinline__ int dedup_slot0(uint64_t k) {
  return (int)((mix64(k) >> 16) & (kDedupSlots - 1));
}

// Find-or-insert in the LDS table; -1 once every slot was probed (full).
__device__ __forceinline__ int lds_insert(unsigned long long* sk, uint64_t k) {
  int h = dedup_slot0(k);
  for (int probe = 0; probe < kDedupMaxProbe; ++probe) {
    const unsigned long long prev =
        __hip_atomic_load(&sk[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (prev == k) return h;
    if (prev == kEmptyKey) {
      const unsigned long long old =
          atomicCAS(&sk[h], (unsigned long long)kEmptyKey, (unsigned long long)k);
      if (old == kEmptyKey || old == k) return h;
    }
    h = (h + 1) & (kDedupSlots - 1);
  }
  return -1;
}

__device__ __forceinline__ int lds_find(const unsigned long long* sk, uint64_t k) {
  int h = dedup_slot0(k);
  for (int probe = 0; probe < kDedupMaxProbe; ++probe) {
    const unsigned long long v = sk[h];
    if (v == k) return h;
    if (v == kEmptyKey) return -1;
    h = (h + 1) & (kDedupSlots - 1);
  }
  return -1;
}

// LDS counter add of 1 per active lane, returning each lane's old value.
// Hot ids put many lanes of one wave on ONE counter, and same-address LDS
// atomics serialise lane by lane, so the lanes of the two most common slots
// of the wave are aggregated first (one add of the group size each); the
// rest add individually. Broadcasts are v_readlane (no LDS round trip).
__device__ __forceinline__ uint32_t lds_ticket(uint32_t* cnt, int s, bool active) {
  const int lane = threadIdx.x & 63;
  const uint64_t lt = (1ull << lane) - 1ull;
  uint64_t act = __ballot(active);
  uint32_t got = 0;
  bool done = !active;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    if (!act) break;
    const int leader = __ffsll((unsigned long long)act) - 1;
    const int ls = __builtin_amdgcn_readlane(s, leader);
    const uint64_t peers = __ballot(!done && s == ls);
    uint32_t b = 0;
    if (lane == leader) b = atomicAdd(&cnt[ls], (uint32_t)__popcll(peers));
    b = (uint32_t)__builtin_amdgcn_readlane((int)b, leader);
    if (!done && s == ls) {
      got = b + (uint32_t)__popcll(peers & lt);
      done = true;
    }
    act &= ~peers;
  }
  if (!done) got = atomicAdd(&cnt[s], 1u);
  return got;
}

// The same count without the returned tickets: fire-and-forget adds, the
// wave's most common slot aggregated into one add.
__device__ __forceinline__ void lds_count(uint32_t* cnt, int s) {
  const int lane = threadIdx.x & 63;
  const uint64_t act = __ballot(s >= 0);
  if (!act) return;
  const int leader = __ffsll((unsigned long long)act) - 1;
  const int ls = __builtin_amdgcn_readlane(s, leader);
  const uint64_t peers = __ballot(s == ls);
  if (lane == leader) atomicAdd(&cnt[ls], (uint32_t)__popcll(peers));
  else if (s >= 0 && s != ls) atomicAdd(&cnt[s], 1u);
}

// A heavy id that qualifies again is appended to the next minibatch's list.
__device__ __forceinline__ void heavy_elect(const PartHeavy& hv, int own, uint64_t k, uint32_t c) {
  if (hv.next_cnt == nullptr || c < hv.thr || hv.nho_next == 0) return;
  const uint32_t q = atomicAdd(hv.next_cnt + own, 1u);
  if (q < (uint32_t)hv.nho_next) hv.next_keys[own * hv.nho_next + q] = k;
}

template <bool kVal>
__global__ __launch_bounds__(kDedupThreads, 8) void k_part_dedup(
    const uint64_t* __restrict__ pk, const int32_t* __restrict__ pr,
    const float* __restrict__ pv, const int64_t* __restrict__ base, int ntiles, int ndig,
    int nshard, int npo_bits, int stride, int nho, PartHeavy hv, Lookback lb, int64_t nnz,
    uint64_t* __restrict__ uniq, int32_t* __restrict__ ucnt, int64_t* __restrict__ csc_off,
    int32_t* __restrict__ csc_row, float* __restrict__ csc_val, int32_t* __restrict__ plid,
    unsigned long long* __restrict__ up, unsigned int* arrive, int64_t* __restrict__ owner_cnt,
    int64_t* __restrict__ tim) {
  __shared__ unsigned long long sk[kDedupSlots];
  __shared__ uint32_t sc[kDedupSlots];  // occurrence count, then the placement cursor
  __shared__ uint32_t sl[kDedupSlots];  // local id within the partition
  __shared__ uint32_t wtot[2][kDedupThreads / 64];
  __shared__ uint32_t sh_base;
  __shared__ int sh_tile, sh_ovf, sh_last;
  __shared__ int64_t ocnt[kPartMaxOwners + 1];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int p = lb_tile(lb, ndig, &sh_tile);
  if (tim && threadIdx.x == 0) tim[p * 4] = (int64_t)__builtin_amdgcn_s_memrealtime();
  const int own = p / stride;
  const int gsz = (1 << (npo_bits - log2_nho(nho))) + 1;
  const bool heavy = nho > 0 && (p - own * stride) % gsz == gsz - 1;  // a single-id partition
  const int64_t ps = base[p], pe = base[p + 1];
  uint32_t occ[kDedupPer], cnt[kDedupPer], so = 0, sn = 0, io = 0, in = 0;
  if (!heavy) {
    for (int i = threadIdx.x; i < kDedupSlots; i += kDedupThreads) {
      sk[i] = kEmptyKey;
      sc[i] = 0;
    }
    if (threadIdx.x == 0) sh_ovf = 0;
    __syncthreads();
    // 1. de-duplicate + count
    for (int64_t b = ps; b < pe; b += kDU * kDedupThreads) {
      uint64_t k[kDU];
#pragma unroll
      for (int u = 0; u < kDU; ++u) {
        const int64_t i = b + u * kDedupThreads + threadIdx.x;
        k[u] = i < pe ? pk[i] : 0;
      }
      // the home-slot probes of all kDU ids in flight together; only ids that
      // met an empty or foreign slot take the insert path
      unsigned long long h0[kDU];
#pragma unroll
      for (int u = 0; u < kDU; ++u)
        h0[u] = __hip_atomic_load(&sk[dedup_slot0(k[u])], __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
      for (int u = 0; u < kDU; ++u) {
        const int64_t i = b + u * kDedupThreads + threadIdx.x;
        int s = -1;
        if (i < pe) {
          s = h0[u] == k[u] ? dedup_slot0(k[u]) : lds_insert(sk, k[u]);
          if (s < 0) sh_ovf = 1;
        }
        lds_count(sc, s);
      }
    }
    __syncthreads();
    // 2. local ids and occurrence offsets: block scan over the slots (4 per
    // thread) of the occupancy flags and the counts
#pragma unroll
    for (int q = 0; q < kDedupPer; ++q) {
      const int s = threadIdx.x * kDedupPer + q;
      occ[q] = sk[s] != kEmptyKey ? 1u : 0u;
      cnt[q] = sc[s];
      so += occ[q];
      sn += cnt[q];
    }
    io = so;
    in = sn;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t a = __shfl_up(io, o, 64), c = __shfl_up(in, o, 64);
      if (lane >= o) { io += a; in += c; }
    }
    if (lane == 63) { wtot[0][wid] = io; wtot[1][wid] = in; }
  } else if (threadIdx.x == 0) {
    sh_ovf = 0;
    for (int w = 0; w < kDedupThreads / 64; ++w) wtot[0][w] = 0;
    wtot[0][0] = pe > ps ? 1u : 0u;
  }
  __syncthreads();
  if (tim && threadIdx.x == 0) tim[p * 4 + 1] = (int64_t)__builtin_amdgcn_s_memrealtime();
  uint32_t bo = 0, bn = 0, to = 0;
  for (int w = 0; w < kDedupThreads / 64; ++w) {
    if (w < wid) { bo += wtot[0][w]; bn += wtot[1][w]; }
    to += wtot[0][w];
  }
  if (wid == 0) {  // this partition's first global local id (look-back over partitions)
    const uint32_t base = lb_exclusive(lb, 0, p, to);
    if (lane == 0) {
      sh_base = base;
      // publish {overflow, unique count} for the owner totals, then arrive
      lb_store(up + p, ((unsigned long long)(sh_ovf ? 1u : 0u) << 32) | to);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned t = atomicAdd(arrive, 1u);
      sh_last = (int)t == ndig - 1;
    }
  }
  __syncthreads();
  const uint32_t gbase = sh_base;
  if (tim && threadIdx.x == 0) tim[p * 4 + 2] = (int64_t)__builtin_amdgcn_s_memrealtime();
  if (heavy) {
    // one id: its occurrences already form its CSC segment (any order)
    if (pe > ps) {
      const int32_t L = (int32_t)gbase;
      if (threadIdx.x == 0) {
        const uint64_t k = pk[ps];
        uniq[L] = k;
        ucnt[L] = (int32_t)(pe - ps);
        csc_off[L] = ps;
        heavy_elect(hv, own, k, (uint32_t)(pe - ps));
      }
      for (int64_t i = ps + threadIdx.x; i < pe; i += kDedupThreads) {
        csc_row[i] = pr[i];
        if (kVal) csc_val[i] = pv[i];
        plid[i] = L;
      }
    }
  } else {
    uint32_t eo = bo + io - so, en = bn + in - sn;
#pragma unroll
    for (int q = 0; q < kDedupPer; ++q) {
      const int s = threadIdx.x * kDedupPer + q;
      if (occ[q]) {
        const uint32_t L = gbase + eo;
        const uint64_t k = sk[s];
        sl[s] = eo;
        sc[s] = en;  // cursor = the id's first occurrence slot in the partition
        uniq[L] = k;
        ucnt[L] = (int32_t)cnt[q];
        csc_off[L] = ps + en;
        heavy_elect(hv, own, k, cnt[q]);
      }
      eo += occ[q];
      en += cnt[q];
    }
    __syncthreads();
    // 3. place every occurrence: CSC row (and value); its local id is stored
    // in partition order (plid), mapped back to CSR order by k_part_lid
    for (int64_t b = ps; b < pe; b += kDU * kDedupThreads) {
      uint64_t k[kDU];
      int32_t r[kDU];
      float v[kDU];
#pragma unroll
      for (int u = 0; u < kDU; ++u) {
        const int64_t i = b + u * kDedupThreads + threadIdx.x;
        const bool ok = i < pe;
        k[u] = ok ? pk[i] : 0;
        r[u] = ok ? pr[i] : 0;
        if (kVal) v[u] = ok ? pv[i] : 0.f;
      }
      unsigned long long h0[kDU];
#pragma unroll
      for (int u = 0; u < kDU; ++u) h0[u] = sk[dedup_slot0(k[u])];
#pragma unroll
      for (int u = 0; u < kDU; ++u) {
        const int64_t i = b + u * kDedupThreads + threadIdx.x;
        const int s = i >= pe ? -1 : h0[u] == k[u] ? dedup_slot0(k[u]) : lds_find(sk, k[u]);
        const uint32_t q = lds_ticket(sc, s, s >= 0);
        if (s >= 0) {
          const int64_t dst = ps + q;
          csc_row[dst] = r[u];
          if (kVal) csc_val[dst] = v[u];
          plid[i] = (int32_t)(gbase + sl[s]);
        }
      }
    }
  }
  if (tim) {
    __syncthreads();
    if (threadIdx.x == 0) tim[p * 4 + 3] = (int64_t)__builtin_amdgcn_s_memrealtime();
  }
  if (!sh_last) return;
  // 4. the last partition to arrive: owner totals (+ overflow count) for the
  // count exchange / host read, the CSC end marker, and re-arm the counter
  for (int i = threadIdx.x; i <= nshard; i += kDedupThreads) ocnt[i] = 0;
  __syncthreads();
  for (int d = threadIdx.x; d < ndig; d += kDedupThreads) {
    const unsigned long long v = lb_load(up + d);
    atomicAdd((unsigned long long*)&ocnt[d / stride], (unsigned long long)(uint32_t)v);
    if (v >> 32) atomicAdd((unsigned long long*)&ocnt[nshard], 1ull);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t U = 0;
    for (int o = 0; o < nshard; ++o) U += ocnt[o];
    csc_off[U] = nnz;
    __hip_atomic_store(arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  for (int i = threadIdx.x; i <= nshard; i += kDedupThreads) owner_cnt[i] = ocnt[i];
}

// lid[j] = plid[pos_of[j]]: CSR-order local ids. The reads of a wave are
// partly contiguous (a tile's non-zeros of one partition sit together).
__global__ __launch_bounds__(256) void k_part_lid(const int32_t* __restrict__ pos_of,
                                                  const int32_t* __restrict__ plid, int64_t nnz,
                                                  int32_t* __restrict__ lid) {
  // contiguous block ranges per XCD: the runs of pos_of a tile reads in
  // every partition sit next to its neighbour tiles' runs (same plid lines)
  const int64_t b = xcd_swizzle(blockIdx.x, gridDim.x);
  const int64_t j0 = (b * 256 + threadIdx.x) * 4;
  if (j0 + 3 < nnz) {
    const int4 p = *reinterpret_cast<const int4*>(pos_of + j0);
    *reinterpret_cast<int4*>(lid + j0) = make_int4(plid[p.x], plid[p.y], plid[p.z], plid[p.w]);
  } else {
    for (int64_t j = j0; j < nnz; ++j) lid[j] = plid[pos_of[j]];
  }
}

__global__ void k_part_empty(int nshard, int64_t* owner_cnt, int64_t* csc_off) {
  for (int i = threadIdx.x; i <= nshard; i += blockDim.x) owner_cnt[i] = 0;
  if (threadIdx.x == 0) csc_off[0] = 0;
}

}  // namespace

PartPlan loc_part_plan(int64_t nnz, int64_t nrows, int nshard, int64_t uest, bool heavy) {
  PartPlan pl;
  pl.ok = false;
  if (nnz <= 0 || nrows <= 0 || nshard < 1 || nshard > kPartMaxOwners) return pl;
  // hashed partitions: ~1-2K distinct ids each at the estimate (LDS table
  // 4096); few partitions keep each digit's run of a tile long (coalesced
  // scatter)
  // as few hashed partitions as fit: ~2K distinct ids each at the estimate
  // (<= 3K, i.e. LDS load <= 0.75 before the estimate's own 25% headroom)
  constexpr int64_t target = 2048;  // distinct ids per partition
  int npo_bits = 0;
  while (((int64_t)nshard << (npo_bits + 1)) * target <= uest) ++npo_bits;
  while (((int64_t)nshard << npo_bits) * 3072 < uest) ++npo_bits;
  // and enough partitions for the dedup's workgroups (one per partition) to
  // fill the GPU: <= ~16K non-zeros each. A minibatch of few distinct ids
  // (18.6K per 100K rows in bench_e2e.py's Criteo text) otherwise got 32
  // partitions of ~120K non-zeros: 0.66 ms of dedup on 32 workgroups.
  constexpr int64_t per_part = 16384;  // non-zeros per partition (target)
  while (((int64_t)nshard << npo_bits) * per_part < nnz &&
         ((int64_t)nshard << (npo_bits + 1)) <= kPartMaxDigits / 2)
    ++npo_bits;
  // and never fewer than 128 hashed partitions: the
  // linear step's 10K-row minibatch (390K non-zeros, ~94K distinct ids over
  // 8 owners) otherwise got 32, so 32 dedup workgroups (dedup 35 -> 30 us;
  // linear loopback 8 51.9 -> 54.5 M ex/s on one box, inside the
  // run-to-run spread on another; 256 measured no better)
  constexpr int64_t min_parts = 128;
  while (((int64_t)nshard << npo_bits) < min_parts &&
         ((int64_t)nshard << (npo_bits + 1)) <= kPartMaxDigits / 2)
    ++npo_bits;
  // heavy-id partitions per owner (a power of two, <= kPartMaxHeavy in all)
  int nho = 0;
  if (heavy) {
    // ~128 heavy ids over all owners: the power-law head is spread over the
    // owners by the hash, so 128 / nshard per owner covers the same ids as
    // 128 on one shard, and the digit count (hence the scatter's run length)
    // stays that of one shard
    constexpr int64_t htotal = kPartHeavyTotal;
    nho = (int)htotal;
    while (nho > 1 && (int64_t)nho * nshard > htotal) nho >>= 1;
    while (nho > 1 && (int64_t)nho * nshard > kPartMaxHeavy) nho >>= 1;
    if ((int64_t)nho * nshard > kPartMaxHeavy) nho = 0;
  }
  while (npo_bits > 0 && ((int64_t)nshard * ((1 << npo_bits) + nho)) > kPartMaxDigits) --npo_bits;
  while (nho > (1 << npo_bits)) nho >>= 1;  // one heavy digit per group of hashed digits
  pl.npo_bits = npo_bits;
  pl.nho = nho;
  pl.stride = (1 << npo_bits) + nho;
  pl.ndig = nshard * pl.stride;
  if (pl.ndig > kPartMaxDigits || uest > ((int64_t)nshard << npo_bits) * 3072) return pl;
  // tiles of R whole rows, ~4096 non-zeros each (8192 halves the histogram
  // but leaves too few workgroups: hist 28 -> 37 us, scatter 64 -> 80 us)
  // A small minibatch takes smaller tiles, down to 1024 non-zeros, for at
  // least 256 histogram / scatter workgroups: the linear step's 10K rows
  // made 96 tiles of 4096.
  constexpr int64_t min_tiles = 256;
  int64_t tile_nnz = nnz / min_tiles;
  tile_nnz = tile_nnz < 1024 ? 1024 : (tile_nnz > 4096 ? 4096 : tile_nnz);
  const int64_t avg = (nnz + nrows - 1) / nrows;
  int64_t R = tile_nnz / (avg > 0 ? avg : 1);
  R = R < 1 ? 1 : (R > kPartMaxRows ? kPartMaxRows : R);
  pl.R = (int)R;
  pl.ntiles = (nrows + R - 1) / R;
  if (pl.ntiles > (1 << 24)) return pl;
  pl.ok = true;
  return pl;
}

void loc_part_hist(const uint64_t* keys, const int64_t* offset, int64_t nrows, int nshard,
                   const PartPlan& pl, const PartHeavy& hv, uint32_t* hist, hipStream_t s) {
  hipLaunchKernelGGL(k_part_hist, dim3((unsigned)pl.ntiles), dim3(kPartThreads), 0, s, keys,
                     offset, nrows, pl.R, nshard, pl.npo_bits, pl.stride, pl.nho, pl.ndig, hv, hist);
}

int64_t loc_part_groups(const PartPlan& pl) { return (pl.ntiles + kColTB - 1) / kColTB; }

void loc_part_offsets(const PartPlan& pl, uint32_t* hist, uint32_t* gsum, int64_t* base,
                      hipStream_t s) {
  const int64_t ng = loc_part_groups(pl);
  hipLaunchKernelGGL(k_part_colpre, dim3((unsigned)ng), dim3(256), 0, s, hist, (int)pl.ntiles,
                     pl.ndig, gsum);
  hipLaunchKernelGGL(k_part_base, dim3(1), dim3(1024), 0, s, gsum, (int)ng, pl.ndig, base);
}

void loc_part_scatter(const uint64_t* keys, const float* val, const int64_t* offset,
                      int64_t nrows, int nshard, const PartPlan& pl, const PartHeavy& hv,
                      const int64_t* base, const uint32_t* gpre, const uint32_t* tpre,
                      uint64_t* pk, int32_t* pr, float* pv, int32_t* pos_of, hipStream_t s) {
  const size_t lds = scatter_lds_bytes(pl.ndig, val != nullptr) + 16;
  hipLaunchKernelGGL(k_part_scatter, dim3((unsigned)pl.ntiles), dim3(kScatThreads), lds, s, keys,
                     val, offset, nrows, pl.R, nshard, pl.npo_bits, pl.stride, pl.nho, pl.ndig, hv,
                     base, gpre, tpre, pk, pr, pv, pos_of);
}

void loc_part_dedup(const uint64_t* pk, const int32_t* pr, const float* pv, int64_t nnz,
                    int nshard, const PartPlan& pl, const PartHeavy& hv, const int64_t* base,
                    const Lookback& lb,
                    uint64_t* uniq, int32_t* ucnt, int64_t* csc_off, int32_t* csc_row,
                    float* csc_val, int32_t* plid, unsigned long long* up, unsigned int* arrive,
                    int64_t* owner_cnt, hipStream_t s, int64_t* tim) {
  auto kern = pv ? k_part_dedup<true> : k_part_dedup<false>;
  hipLaunchKernelGGL(kern, dim3((unsigned)pl.ndig), dim3(kDedupThreads), 0, s, pk, pr, pv, base,
                     (int)pl.ntiles, pl.ndig, nshard, pl.npo_bits, pl.stride, pl.nho, hv, lb, nnz, uniq,
                     ucnt, csc_off,
                     csc_row, csc_val, plid, up, arrive, owner_cnt, tim);
}

void loc_part_lid(const int32_t* pos_of, const int32_t* plid, int64_t nnz, int32_t* lid,
                  hipStream_t s) {
  hipLaunchKernelGGL(k_part_lid, dim3((unsigned)((nnz + 1023) / 1024)), dim3(256), 0, s, pos_of,
                     plid, nnz, lid);
}

void loc_part_empty(int nshard, int64_t* owner_cnt, int64_t* csc_off, hipStream_t s) {
  hipLaunchKernelGGL(k_part_empty, dim3(1), dim3(256), 0, s, nshard, owner_cnt, csc_off);
}

}  // namespace wh
