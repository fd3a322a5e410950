// Per-minibatch evaluation metrics (reference learn/base/binary_class_evaluation.h).
// Loss / objective / accuracy sums are fused into the forward kernel (fm.hip);
// this file holds the exact AUC rank-sum over predictions sorted ascending.
#include <rocprim/device/device_radix_sort.hpp>

#include "wh_common.h"
#include "wh_kernels.h"
#include "wh_lookback.h"

#include <algorithm>

namespace wh {
namespace {

constexpr int kThreads = 256;

__global__ void k_pos_flags(const float* lab, int64_t n, int32_t* flags) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i < n) flags[i] = lab[i] > 0.f ? 1 : 0;
}

// area = sum over negatives of #positives ranked strictly before them
__global__ __launch_bounds__(kThreads) void k_auc_area(const float* lab, const int64_t* excl,
                                                       int64_t n, double* out) {
  __shared__ double sh[kThreads / 64];
  double a = 0;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kThreads)
    if (!(lab[i] > 0.f)) a += (double)excl[i];
  const double r = block_sum_d(a, sh);
  if (threadIdx.x == 0) atomicAdd(out + 1, r);
}

__global__ void k_auc_final(const int64_t* excl, int64_t n, double* out) {
  const double tp = (double)excl[n];
  double auc;
  if (tp == 0 || tp == (double)n) {
    auc = 1.0;
  } else {
    double area = out[1] / (tp * ((double)n - tp));
    auc = area < 0.5 ? 1 - area : area;
  }
  out[0] = auc;
}

// ---------------------------------------------------------------------------
// Exact AUC without a full sort (5 short launches instead of a 10-launch
// radix sort + flag/scan/area passes).
//
// Every prediction gets a unique 64-bit key  ord(py) << 32 | i << 1 | pos
// (ord = order-preserving bits of the float, i = the example index, so ties
// are broken by index exactly like the stable sort of the reference path).
// Keys are bucketed linearly over [min, max] into kAucBuckets buckets; a
// negative's rank-sum term is  (#positives in lower buckets) + (#positives
// in its own bucket with a smaller key). Buckets hold a few keys each, and
// all-equal predictions (e.g. a zero model) spread evenly because the index
// is part of the key. Every count is an integer, so the result does not
// depend on atomic ordering. The bucket counters are left zeroed by the
// scan kernel and the min/max / area words by the last kernel, so the
// persistent workspace never needs a clearing launch.
constexpr int kAucBuckets = 16384;
constexpr int kAucScanThreads = 1024;

__device__ __forceinline__ uint64_t auc_key(float py, int64_t i, bool pos) {
  uint32_t u = __float_as_uint(py == 0.f ? 0.f : py);  // -0 ties with +0
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ((uint64_t)u << 32) | ((uint64_t)i << 1) | (pos ? 1u : 0u);
}

__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long t = __shfl_xor(v, o, 64);
    v = t < v ? t : v;
  }
  return v;
}
__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long t = __shfl_xor(v, o, 64);
    v = t > v ? t : v;
  }
  return v;
}

// min / max key: one pair of atomics per BLOCK (same-address atomics
// serialise at ~12 ns each, so per-wave atomics from 1000 waves cost 25 us)
__global__ __launch_bounds__(1024) void k_auc_minmax(const float* __restrict__ py,
                                                     const float* __restrict__ lab, int64_t n,
                                                     unsigned long long* lohi) {
  __shared__ unsigned long long slo[16], shi[16];
  unsigned long long lo = ~0ull, hi = 0ull;
  for (int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 1024) {
    const unsigned long long k = auc_key(py[i], i, lab[i] > 0.f) >> 32;
    lo = k < lo ? k : lo;
    hi = k > hi ? k : hi;
  }
  lo = wave_min_u64(lo);
  hi = wave_max_u64(hi);
  const int wid = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    slo[wid] = lo;
    shi[wid] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 16; ++w) {
      lo = slo[w] < lo ? slo[w] : lo;
      hi = shi[w] > hi ? shi[w] : hi;
    }
    atomicMin(lohi, lo);
    atomicMax(lohi + 1, hi);
  }
}

// Bucket of example i: linear in the prediction VALUE between the minibatch's
// min and max (double arithmetic: monotone non-decreasing in py, which is
// all the exact count needs); all-equal predictions bucket by index (also
// monotone in the key, whose high half is then constant). lo/hi are the
// order-preserving keys of the min / max prediction.
__device__ __forceinline__ float auc_unord(uint64_t k) {
  const uint32_t u = (uint32_t)k;
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}
__device__ __forceinline__ int auc_bucket(float py, int64_t i, int64_t n, uint64_t lo,
                                          uint64_t hi) {
  if (lo == hi) return (int)((i * kAucBuckets) / (n > 0 ? n : 1));
  const double flo = auc_unord(lo), fhi = auc_unord(hi);
  const double t = ((double)py - flo) * ((double)kAucBuckets / (fhi - flo));
  if (!(t >= 0.0)) return 0;
  return t < (double)(kAucBuckets - 1) ? (int)t : kAucBuckets - 1;
}

__global__ __launch_bounds__(kThreads) void k_auc_bucket(const float* __restrict__ py,
                                                         const float* __restrict__ lab, int64_t n,
                                                         const unsigned long long* lohi,
                                                         uint32_t* cnt, uint32_t* pcnt,
                                                         int2* br) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const bool pos = lab[i] > 0.f;
  const int b = auc_bucket(py[i], i, n, lohi[0], lohi[1]);
  const int r = (int)atomicAdd(cnt + b, 1u);
  if (pos) atomicAdd(pcnt + b, 1u);
  br[i] = make_int2(b, r);
}

// one block: exclusive scans of the bucket counts and positive counts
// (8 consecutive buckets per thread, 16-byte loads); leaves the counters
// zeroed, saves {lo, hi} and re-arms the min/max words
__global__ __launch_bounds__(kAucScanThreads) void k_auc_scan(uint32_t* cnt, uint32_t* pcnt,
                                                              unsigned long long* lohi,
                                                              uint32_t* off, uint32_t* poff,
                                                              unsigned long long* lw) {
  constexpr int kPer = kAucBuckets / kAucScanThreads;
  static_assert(kPer == 16, "scan assumes 16 buckets per thread");
  __shared__ uint32_t wa[16], wp[16];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  constexpr int kV = kPer / 4;  // uint4 per thread per array
  uint4* c4 = reinterpret_cast<uint4*>(cnt) + kV * t;
  uint4* p4 = reinterpret_cast<uint4*>(pcnt) + kV * t;
  uint32_t a[kPer], p[kPer];
#pragma unroll
  for (int v = 0; v < kV; ++v) {
    const uint4 x = c4[v], y = p4[v];
    a[4 * v] = x.x; a[4 * v + 1] = x.y; a[4 * v + 2] = x.z; a[4 * v + 3] = x.w;
    p[4 * v] = y.x; p[4 * v + 1] = y.y; p[4 * v + 2] = y.z; p[4 * v + 3] = y.w;
  }
  const uint4 z = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
  for (int v = 0; v < kV; ++v) { c4[v] = z; p4[v] = z; }
  uint32_t sa = 0, sp = 0;
#pragma unroll
  for (int j = 0; j < kPer; ++j) { sa += a[j]; sp += p[j]; }
  uint32_t ia = sa, ip = sp;  // wave inclusive scans
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t xa = __shfl_up(ia, o, 64), xp = __shfl_up(ip, o, 64);
    if (lane >= o) { ia += xa; ip += xp; }
  }
  if (lane == 63) { wa[wid] = ia; wp[wid] = ip; }
  __syncthreads();
  uint32_t ba = 0, bp = 0;
  for (int w = 0; w < wid; ++w) { ba += wa[w]; bp += wp[w]; }
  uint32_t ra = ba + ia - sa, rp = bp + ip - sp;
  uint32_t oa[kPer], op[kPer];
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    oa[j] = ra; op[j] = rp;
    ra += a[j]; rp += p[j];
  }
#pragma unroll
  for (int v = 0; v < kV; ++v) {
    reinterpret_cast<uint4*>(off)[kV * t + v] =
        make_uint4(oa[4 * v], oa[4 * v + 1], oa[4 * v + 2], oa[4 * v + 3]);
    reinterpret_cast<uint4*>(poff)[kV * t + v] =
        make_uint4(op[4 * v], op[4 * v + 1], op[4 * v + 2], op[4 * v + 3]);
  }
  if (t == kAucScanThreads - 1) {
    off[kAucBuckets] = ra;
    poff[kAucBuckets] = rp;
    lw[0] = lohi[0];
    lw[1] = lohi[1];
    lohi[0] = ~0ull;
    lohi[1] = 0ull;
  }
}

__global__ __launch_bounds__(kThreads) void k_auc_place(const float* __restrict__ py,
                                                        const float* __restrict__ lab, int64_t n,
                                                        const int2* __restrict__ br,
                                                        const uint32_t* __restrict__ off,
                                                        unsigned long long* sorted) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const int2 q = br[i];
  sorted[off[q.x] + q.y] = auc_key(py[i], i, lab[i] > 0.f);
}

__global__ __launch_bounds__(kThreads) void k_auc_count(const unsigned long long* __restrict__ sorted,
                                                        int64_t n, const uint32_t* __restrict__ off,
                                                        const uint32_t* __restrict__ poff,
                                                        const unsigned long long* __restrict__ lw,
                                                        unsigned long long* area,
                                                        unsigned int* ticket, double* auc_sum) {
  __shared__ int last;
  const int64_t q = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  unsigned long long a = 0;
  if (q < n) {
    const uint64_t k = sorted[q];
    if (!(k & 1)) {
      const int b = auc_bucket(auc_unord(k >> 32), (int64_t)((k & 0xffffffffull) >> 1), n, lw[0],
                               lw[1]);
      a = poff[b];
      const uint32_t e = off[b + 1];
      for (uint32_t j = off[b]; j < e; ++j) {
        const uint64_t o = sorted[j];
        a += (o & 1) && o < k;
      }
    }
  }
  // the block's count to its own word (a same-address atomic per wave
  // serialised ~1.5k of them at 100k rows), drained before the arrival
  __shared__ unsigned long long ws[kThreads / 64];
  a = wave_sum_ll((long long)a);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long b = 0;
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) b += ws[w];
    lb_store(area + blockIdx.x, b);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = arrive_last(ticket, blockIdx.x, gridDim.x);
  }
  __syncthreads();
  if (!last) return;
  unsigned long long t = 0;
  for (int b = threadIdx.x; b < (int)gridDim.x; b += kThreads) t += lb_load(area + b);
  t = (unsigned long long)wave_sum_ll((long long)t);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x != 0) return;
  unsigned long long at = 0;
#pragma unroll
  for (int w = 0; w < kThreads / 64; ++w) at += ws[w];
  const double tot = (double)at;
  const double tp = (double)poff[kAucBuckets];
  double auc = 1.0;
  if (tp != 0 && tp != (double)n) {
    const double r = tot / (tp * ((double)n - tp));
    auc = r < 0.5 ? 1 - r : r;
  }
  auc_sum[0] += auc;
}

// ---------------------------------------------------------------------------
// Small minibatches (n <= kAucSmallMax, e.g. the reference's 10000 rows): the
// same rank-sum by direct pair counting in ONE launch. Block (x, y) holds the
// positives of row chunk y in LDS (compacted, as keys) and each thread counts,
// for kAsJ negatives of tile x, the positives with a smaller key -- the
// identical integer as the bucketed path. Each block stores its count to its
// own word (no same-address atomics besides the arrival ticket) and the last
// block to arrive sums them. n^2 / 2 compares at n = 10000 spread over ~400
// workgroups; the five bucketed launches were ~40 us of mostly launch and
// single-workgroup scan latency.
constexpr int64_t kAucSmallMax = 24576;
constexpr int kAsThreads = 256;
constexpr int kAsJ = 2;
constexpr int kAsTileJ = kAsThreads * kAsJ;
constexpr int kAsTileI = 512;
constexpr int kAsMaxX = (int)((kAucSmallMax + kAsTileJ - 1) / kAsTileJ);
constexpr int kAsMaxY = (int)((kAucSmallMax + kAsTileI - 1) / kAsTileI);
constexpr int kAsUnroll = 8;  // LDS keys per batch of loads in flight

__global__ __launch_bounds__(kAsThreads) void k_auc_small(const float* __restrict__ py,
                                                          const float* __restrict__ lab,
                                                          int64_t n, unsigned long long* part,
                                                          unsigned int* ticket,
                                                          double* auc_sum) {
  __shared__ __attribute__((aligned(16))) unsigned long long pk[kAsTileI + kAsUnroll];
  __shared__ int wcnt[kAsThreads / 64];
  __shared__ unsigned long long wsum[kAsThreads / 64];
  __shared__ int last;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t i0 = (int64_t)blockIdx.y * kAsTileI;
  int np = 0;  // positives of the chunk staged so far (block-uniform)
#pragma unroll
  for (int r = 0; r < kAsTileI / kAsThreads; ++r) {
    const int64_t i = i0 + r * kAsThreads + tid;
    const bool pos = i < n && lab[i] > 0.f;
    const uint64_t m = __ballot(pos);
    if (lane == 0) wcnt[wid] = __popcll(m);
    __syncthreads();
    int off = np, tot = 0;
#pragma unroll
    for (int w = 0; w < kAsThreads / 64; ++w) {
      off += w < wid ? wcnt[w] : 0;
      tot += wcnt[w];
    }
    if (pos) pk[off + __popcll(m & ((1ull << lane) - 1ull))] = auc_key(py[i], i, true);
    np += tot;
    __syncthreads();
  }
  // pad to whole batches with keys no negative exceeds
  if (tid < kAsUnroll) pk[np + tid] = ~0ull;
  unsigned long long kj[kAsJ];
#pragma unroll
  for (int u = 0; u < kAsJ; ++u) {
    const int64_t j = (int64_t)blockIdx.x * kAsTileJ + u * kAsThreads + tid;
    kj[u] = (j < n && !(lab[j] > 0.f)) ? auc_key(py[j], j, false) : 0ull;  // 0: counts nothing
  }
  __syncthreads();
  uint32_t c[kAsJ] = {};
  const ulonglong2* pk2 = reinterpret_cast<const ulonglong2*>(pk);
  for (int p = 0; p < np; p += kAsUnroll) {
    ulonglong2 k[kAsUnroll / 2];
#pragma unroll
    for (int q = 0; q < kAsUnroll / 2; ++q) k[q] = pk2[p / 2 + q];
#pragma unroll
    for (int q = 0; q < kAsUnroll / 2; ++q)
#pragma unroll
      for (int u = 0; u < kAsJ; ++u) c[u] += (k[q].x < kj[u] ? 1u : 0u) + (k[q].y < kj[u] ? 1u : 0u);
  }
  unsigned long long a = 0;
#pragma unroll
  for (int u = 0; u < kAsJ; ++u) a += c[u];
  a = (unsigned long long)wave_sum_ll((long long)a);
  if (lane == 0) wsum[wid] = a;
  __syncthreads();
  const int nblk = (int)(gridDim.x * gridDim.y);
  if (tid == 0) {
    unsigned long long t = 0;
#pragma unroll
    for (int w = 0; w < kAsThreads / 64; ++w) t += wsum[w];
    // part[block] = this block's count; part[kAsMaxX * kAsMaxY + y] = the
    // positives of chunk y (from the x = 0 blocks); stores drained before
    // the ticket add, read back by the last block with agent-scope loads
    lb_store(part + blockIdx.y * gridDim.x + blockIdx.x, t);
    if (blockIdx.x == 0) lb_store(part + kAsMaxX * kAsMaxY + blockIdx.y, (unsigned long long)np);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = arrive_last(ticket, blockIdx.y * gridDim.x + blockIdx.x, (unsigned)nblk);
  }
  __syncthreads();
  if (!last) return;
  unsigned long long tot = 0, tp = 0;
  for (int b = tid; b < nblk; b += kAsThreads) tot += lb_load(part + b);
  for (int y = tid; y < (int)gridDim.y; y += kAsThreads) tp += lb_load(part + kAsMaxX * kAsMaxY + y);
  tot = (unsigned long long)wave_sum_ll((long long)tot);
  tp = (unsigned long long)wave_sum_ll((long long)tp);
  __syncthreads();
  if (lane == 0) {
    wsum[wid] = tot;
    wcnt[wid] = (int)tp;
  }
  __syncthreads();
  if (tid != 0) return;
  unsigned long long at = 0, pt = 0;
#pragma unroll
  for (int w = 0; w < kAsThreads / 64; ++w) {
    at += wsum[w];
    pt += (unsigned long long)wcnt[w];
  }
  const double area = (double)at, npos = (double)pt;
  double auc = 1.0;
  if (npos != 0 && npos != (double)n) {
    const double r = area / (npos * ((double)n - npos));
    auc = r < 0.5 ? 1 - r : r;
  }
  auc_sum[0] += auc;
}

}  // namespace

size_t auc_sort_tmp_bytes(int64_t n) {
  size_t bytes = 0;
  WH_HIP_CHECK(rocprim::radix_sort_pairs(nullptr, bytes, (float*)nullptr, (float*)nullptr,
                                         (float*)nullptr, (float*)nullptr,
                                         (size_t)std::max<int64_t>(n, 1), 0, 32, (hipStream_t)0));
  return bytes;
}

void sort_by_score(const float* py, const float* label, int64_t n, float* py_sorted,
                   float* label_sorted, void* tmp, size_t tmp_bytes, hipStream_t s) {
  if (n <= 0) return;
  size_t bytes = tmp_bytes;
  WH_HIP_CHECK(rocprim::radix_sort_pairs(tmp, bytes, py, py_sorted, label, label_sorted,
                                         (size_t)n, 0, 32, s));
}

void auc_from_sorted(const float* label_sorted, int64_t n, double* out, int64_t* tmp_i64,
                     hipStream_t s) {
  // tmp layout: [n int32 flags (as n/2+1 int64)] [n+1 excl] [scan tmp]
  int32_t* flags = reinterpret_cast<int32_t*>(tmp_i64);
  int64_t* excl = tmp_i64 + (n / 2 + 1);
  int64_t* stmp = excl + (n + 1);
  WH_HIP_CHECK(hipMemsetAsync(out, 0, 2 * sizeof(double), s));
  if (n <= 0) {
    hipLaunchKernelGGL(k_auc_final, dim3(1), dim3(1), 0, s, excl, (int64_t)0, out);
    return;
  }
  hipLaunchKernelGGL(k_pos_flags, dim3(grid_for(n, kThreads)), dim3(kThreads), 0, s, label_sorted,
                     n, flags);
  scan_i32(flags, excl, n, stmp, s);
  hipLaunchKernelGGL(k_auc_area, dim3(grid_for(n, kThreads, 1024)), dim3(kThreads), 0, s,
                     label_sorted, excl, n, out);
  hipLaunchKernelGGL(k_auc_final, dim3(1), dim3(1), 0, s, excl, n, out);
}

}  // namespace wh

namespace wh {

// persistent (zeroed once; lohi[0] = ~0): cnt, pcnt [NB] u32, lohi [2] u64,
// (unused) u64 [2], pair-path partials u64 [kAsMaxX kAsMaxY +
// kAsMaxY] (every word written before it is read).  scratch: off,
// poff [NB + 1] u32, {lo, width}, per-example (bucket, rank) and the
// bucket-ordered keys (none for the pair path).
int64_t auc_ws_bytes(int64_t n) {
  if (n <= kAucSmallMax) return 0;
  // ... + the count kernel's per-block partials
  return 2 * ((int64_t)kAucBuckets + 4) * 4 + 16 + 2 * 8 + 8 * n + 8 * n + 64 +
         8 * (int64_t)grid_for(n, kThreads);
}
// (+ the arrival ticket: kArriveWords u32 at the end)
static int64_t auc_ticket_offset() {
  return 2 * (int64_t)kAucBuckets * 4 + 4 * 8 + (int64_t)(kAsMaxX * kAsMaxY + kAsMaxY) * 8;
}
int64_t auc_ws_persistent_bytes() { return auc_ticket_offset() + (int64_t)kArriveWords * 4; }
int64_t auc_ws_lohi_offset() { return 2 * (int64_t)kAucBuckets * 4; }

void auc_accumulate(const float* py, const float* label, int64_t n, void* persist, void* scratch,
                    double* auc_sum, hipStream_t s) {
  if (n <= 0) return;
  char* base = static_cast<char*>(persist);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(base);
  uint32_t* pcnt = cnt + kAucBuckets;
  unsigned long long* lohi = reinterpret_cast<unsigned long long*>(pcnt + kAucBuckets);
  unsigned int* ticket = reinterpret_cast<unsigned int*>(base + auc_ticket_offset());
  if (n <= kAucSmallMax) {
    const dim3 grid((unsigned)((n + kAsTileJ - 1) / kAsTileJ),
                    (unsigned)((n + kAsTileI - 1) / kAsTileI));
    hipLaunchKernelGGL(k_auc_small, grid, dim3(kAsThreads), 0, s, py, label, n, lohi + 4, ticket,
                       auc_sum);
    return;
  }
  char* sc = static_cast<char*>(scratch);
  uint32_t* off = reinterpret_cast<uint32_t*>(sc);
  uint32_t* poff = off + kAucBuckets + 4;  // 16-byte aligned for the vector stores
  unsigned long long* lw = reinterpret_cast<unsigned long long*>(
      (reinterpret_cast<uintptr_t>(poff + kAucBuckets + 4) + 15) & ~(uintptr_t)15);
  int2* br = reinterpret_cast<int2*>(lw + 2);
  unsigned long long* sorted = reinterpret_cast<unsigned long long*>(br + n);
  unsigned long long* area = sorted + n;  // per-block counts of k_auc_count
  const int g = grid_for(n, kThreads);
  hipLaunchKernelGGL(k_auc_minmax, dim3(grid_for(n, 1024, 64)), dim3(1024), 0, s, py, label, n,
                     lohi);
  hipLaunchKernelGGL(k_auc_bucket, dim3(g), dim3(kThreads), 0, s, py, label, n, lohi, cnt, pcnt,
                     br);
  hipLaunchKernelGGL(k_auc_scan, dim3(1), dim3(kAucScanThreads), 0, s, cnt, pcnt, lohi, off, poff,
                     lw);
  hipLaunchKernelGGL(k_auc_place, dim3(g), dim3(kThreads), 0, s, py, label, n, br, off, sorted);
  hipLaunchKernelGGL(k_auc_count, dim3(g), dim3(kThreads), 0, s, sorted, n, off, poff, lw, area,
                     ticket, auc_sum);
}

}  // namespace wh
