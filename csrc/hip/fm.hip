// Fused factorization-machine / linear forward and backward on a localized
// minibatch (K4-K10 in SURVEY §2.5).
//
// Reference math (learn/difacto/loss.h:53-158, learn/linear/loss.h:92-157):
//   py   = X w + 0.5 * sum_d ((X V)_d^2 - ((X.*X)(V.*V))_d)
//   p    = dual(py)                       (logit: -y / (1 + exp(y py)))
//   gw   = X^T p
//   gV   = X^T diag(p) X V - diag((X.*X)^T p) V
// The reference does this with 2 SpMV + 4 SpMM passes and several
// elementwise loops; here it is ONE forward kernel (a lane group of
// G = vstride/4 lanes per row, float4 per lane: wave64 holds 64/G rows) that
// also emits loss/objective/accuracy sums and the dual, and ONE backward
// kernel that walks each key's occurrence list (the CSC produced by
// localize) so gradients are segmented sums, not scattered atomics. Only
// keys whose occurrence list is longer than one chunk (hot features) use
// float atomics, one per chunk.
//
// Variable-length model layout (the ZVPull/ZVPush value layout of
// learn/difacto/async_sgd.h:234-244, made dense): a pulled minibatch model is
//   hdr[U]  float2 {w, vidx}   vidx = bit-cast int32 row in vc, or -1
//   vc[m]   vstride floats     embedding rows of the keys that have one
// and the gradient mirrors it: gw[U] + gvc[m] (same vidx numbering). Only the
// m keys with an embedding move 256 bytes; the rest move 8 (pull) / 4 (push).
#include "wh_common.h"
#include <string>
#include "wh_kernels.h"
#include "wh_lookback.h"
#include "wh_loss.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace wh {
namespace {

constexpr int kThreads = 256;
constexpr int kChunk = 32;  // occurrences per backward work item
constexpr int kFwdBlocks = 2048;  // persistent forward grid: 8192 waves = 32 per CU

// Memory-level parallelism decides both FM kernels: every V / xv row is a
// dependent gather (index load -> header -> row), and 256-byte rows only
// reach the L2 / Infinity-Cache gather rates with many independent loads in
// flight per wave. tools/microbench/fm_gather_bench.hip measured the forward's
// 1 GB of row gathers per 100k-row minibatch at 189 us with G-lane groups
// issuing 8 rows at a time vs 65 us with ONE WAVE PER ROW issuing all its rows
// at once (15 TB/s), so both kernels use the wave-per-item shape:
//   lanes = SUB sub-groups x G lanes (G = vstride/4, a float4 slice each);
//   one wave-instruction gathers SUB rows; up to TI instructions in flight.
template <int G>
struct Shape {
  static constexpr int SUB = 64 / G;             // rows per wave-instruction
  static constexpr int NI = G;                   // instructions per 64 items
#ifndef WH_FM_TI
#define WH_FM_TI 4
#endif
  // instructions per gather batch: a batch only runs while it covers live
  // slots, so short rows / chunks issue ceil(n / (SUB * TI)) batches instead
  // of all NI instructions (rocprof: the forward was issue-bound at 43 %
  // instruction share with 64 slots per row for 39 non-zeros)
  static constexpr int TI = G < WH_FM_TI ? G : WH_FM_TI;
  static constexpr int VS = 4 * G;               // row stride in floats (= vstride)
};

// A gather slot without a row reads this zero row instead of branching
// around the load (a predicated load costs an exec-mask branch per gather).
__device__ float kZeroRow[256];

// Per-wave LDS staging of the 64 (row index, scalar) pairs of a pass, stored
// transposed ([sub][t]) so that lane (sub, gl) reads the pairs of its
// instructions t = 0.. as consecutive 8-byte entries (ds_read_b128 pairs,
// broadcast across the G lanes of the sub-group) instead of two ds_bpermute
// per gathered row.
template <int G>
__device__ __forceinline__ void stage_pairs(int2* st, int lane, int idx_val, float f) {
  using S = Shape<G>;
  st[(lane % S::SUB) * S::NI + lane / S::SUB] = make_int2(idx_val, __float_as_int(f));
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Forward staging: only the ids that HAVE an embedding row are staged,
// compacted to the front (the others contribute nothing to the
// second-order term). Slots past the returned count hold stale pairs: the
// reader masks them by position.
template <int G>
__device__ __forceinline__ int stage_pairs_compact(int2* st, int lane, int vid, float f) {
  using S = Shape<G>;
  const bool has = vid >= 0;
  const uint64_t m = __ballot(has);
  const int nv = __popcll(m);
  const int pos = __popcll(m & ((1ull << lane) - 1ull));
  if (has) st[(pos % S::SUB) * S::NI + pos / S::SUB] = make_int2(vid, __float_as_int(f));
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return nv;
}

template <int G>
__global__ __launch_bounds__(kThreads) void k_fm_fwd(int64_t nrows, const int64_t* __restrict__ off,
                                                     const int32_t* __restrict__ lid,
                                                     const float* __restrict__ val,
                                                     const float2* __restrict__ hdr,
                                                     const float* __restrict__ vc, int vstride,
                                                     const float* __restrict__ label, int loss,
                                                     float* __restrict__ py_out,
                                                     float* __restrict__ dual_out,
                                                     float* __restrict__ xv, double* part,
                                                     double* met, unsigned int* ticket, int acc5) {
  // Persistent waves, one example (row) at a time, software-pipelined over
  // the wave's rows so each row exposes ~one memory round trip instead of
  // four: while row i's embedding rows are gathered, the headers of row i+1,
  // the ids of row i+2 and the CSR bounds of row i+3 are in flight. The
  // gathers are issued first and the prefetches after them, so the in-order
  // vmcnt wait before the accumulation covers the gathers only.
  using S = Shape<G>;
  __shared__ double sh[kThreads / 64];
  __shared__ int2 stage[kThreads / 64][64];
  const int lane = threadIdx.x & 63, gl = lane & (G - 1), sub = lane / G;
  const int64_t nw = (int64_t)gridDim.x * (kThreads / 64);
  const int64_t w0 =
      __builtin_amdgcn_readfirstlane((int)(((int64_t)blockIdx.x * kThreads + threadIdx.x) >> 6));
  double m_objv = 0, m_objw = 0, m_corr = 0, m_n = 0;
  auto bounds = [&](int64_t r, int64_t& b, int64_t& e) {
    if (r < nrows) {
      b = off[r];
      e = off[r + 1];
    } else {
      b = e = 0;
    }
  };
  auto load_ids = [&](int64_t b, int64_t e, int& l, float& x) {
    const bool ok = b + lane < e;
    l = ok ? lid[b + lane] : -1;
    x = ok ? (val ? val[b + lane] : 1.f) : 0.f;
  };
  auto load_hdr = [&](int l) {
    return l >= 0 ? hdr[l] : make_float2(0.f, __int_as_float(-1));
  };
  // gather the embedding rows of one 64-id pass and accumulate them
  int2* st = stage[threadIdx.x >> 6];
  // gather the embedding rows of one 64-id pass and accumulate them
  auto gather = [&](int n, int vid, float x, float4& s, float4& q2, bool prefetch_first,
                    auto&& prefetch) {
    (void)n;
    n = stage_pairs_compact<G>(st, lane, vid, x);
#pragma unroll
    for (int t0 = 0; t0 < S::NI; t0 += S::TI) {
      if (t0 * S::SUB >= n) break;
      float4 v[S::TI];
      float xs[S::TI];
#pragma unroll
      for (int t = 0; t < S::TI; ++t) {
        const int2 e = st[sub * S::NI + t0 + t];
        const bool live = (t0 + t) * S::SUB + sub < n;  // compacted slots only
        xs[t] = live ? __int_as_float(e.y) : 0.f;
        const float* src = live ? vc + (uint32_t)e.x * (uint32_t)S::VS : kZeroRow;
        v[t] = reinterpret_cast<const float4*>(src)[gl];
      }
      if (t0 == 0 && prefetch_first) prefetch();
#pragma unroll
      for (int t = 0; t < S::TI; ++t) {
        const float xu = xs[t], xx = xu * xu;
        s.x += xu * v[t].x; s.y += xu * v[t].y; s.z += xu * v[t].z; s.w += xu * v[t].w;
        q2.x += xx * v[t].x * v[t].x; q2.y += xx * v[t].y * v[t].y;
        q2.z += xx * v[t].z * v[t].z; q2.w += xx * v[t].w * v[t].w;
      }
    }
  };
  int64_t r = w0;
  int64_t bc, ec, bn, en, b2, e2, b3 = 0, e3 = 0;
  bounds(r, bc, ec);
  bounds(r + nw, bn, en);
  bounds(r + 2 * nw, b2, e2);
  int lc, ln, l2 = -1;
  float xc, xn, x2 = 0.f;
  load_ids(bc, ec, lc, xc);
  float2 hc = load_hdr(lc), hn = make_float2(0.f, 0.f);
  load_ids(bn, en, ln, xn);
  for (; r < nrows; r += nw) {
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f), q2 = s;
    float wl = xc * hc.x;
    const int nc = (int)(ec - bc < 64 ? ec - bc : 64);
    bool fetched = false;
    auto prefetch = [&]() {
      hn = load_hdr(ln);
      load_ids(b2, e2, l2, x2);
      bounds(r + 3 * nw, b3, e3);
      fetched = true;
    };
    gather(nc, __float_as_int(hc.y), xc, s, q2, true, prefetch);
    if (!fetched) prefetch();  // empty row
    for (int64_t pb = bc + 64; pb < ec; pb += 64) {  // rest of a long row, unpipelined
      const int n = (int)(ec - pb < 64 ? ec - pb : 64);
      int l;
      float x;
      load_ids(pb, ec, l, x);
      const float2 h = load_hdr(l);
      wl += x * h.x;
      gather(n, __float_as_int(h.y), x, s, q2, false, prefetch);
    }
    // sum the SUB partial rows: lanes gl, gl+G, gl+2G, ... hold the same dims
#pragma unroll
    for (int o = G; o < 64; o <<= 1) {
      s.x += __shfl_xor(s.x, o, 64); s.y += __shfl_xor(s.y, o, 64);
      s.z += __shfl_xor(s.z, o, 64); s.w += __shfl_xor(s.w, o, 64);
      q2.x += __shfl_xor(q2.x, o, 64); q2.y += __shfl_xor(q2.y, o, 64);
      q2.z += __shfl_xor(q2.z, o, 64); q2.w += __shfl_xor(q2.w, o, 64);
    }
    const float wsum = wave_sum(wl);
    float pt = (s.x * s.x - q2.x) + (s.y * s.y - q2.y) + (s.z * s.z - q2.z) + (s.w * s.w - q2.w);
    pt = group_sum<G>(pt);
    if (sub == 0) reinterpret_cast<float4*>(xv + r * vstride)[gl] = s;
    if (lane == 0) {
      const float p = wsum + 0.5f * pt;
      const float y = label[r];
      const LossOut o = eval_loss(loss, y, p);
      const LossOut ow = eval_loss(loss, y, wsum);
      py_out[r] = p;
      dual_out[r] = o.dual;
      m_objv += o.objv;
      m_objw += ow.objv;
      m_corr += ((y > 0.f && p > 0.f) || (y <= 0.f && p <= 0.f)) ? 1.0 : 0.0;
      m_n += 1.0;
    }
    // rotate the pipeline
    bc = bn; ec = en; xc = xn; hc = hn;
    bn = b2; en = e2; ln = l2; xn = x2;
    b2 = b3; e2 = e3;
  }
  block_partials(part, sh, m_objv, m_objw, m_corr, m_n, met, ticket, acc5);
}

// linear model: G lanes stride over one row's non-zeros; persistent over rows
template <int G>
__global__ __launch_bounds__(kThreads) void k_lin_fwd(int64_t nrows, const int64_t* __restrict__ off,
                                                      const int32_t* __restrict__ lid,
                                                      const float* __restrict__ val,
                                                      const float* __restrict__ w, int wstride,
                                                      const float* __restrict__ label, int loss,
                                                      float* __restrict__ py_out,
                                                      float* __restrict__ dual_out, double* part,
                                                      double* met, unsigned int* ticket, int acc5) {
  __shared__ double sh[kThreads / 64];
  const int lane = threadIdx.x & 63, gl = lane & (G - 1);
  const int64_t ngroups = (int64_t)gridDim.x * (kThreads / G);
  double m_objv = 0, m_corr = 0, m_n = 0;
  for (int64_t row = ((int64_t)blockIdx.x * kThreads + threadIdx.x) / G; row < nrows;
       row += ngroups) {
    float acc = 0.f;
    const int64_t b = off[row], e = off[row + 1];
    for (int64_t j = b + gl; j < e; j += G) {
      const int32_t l = lid[j];
      if (wstride == 1) acc += (val ? val[j] : 1.f) * w[l];
      else if (l >= 0) acc += (val ? val[j] : 1.f) * w[(int64_t)l * wstride];  // (table slots)
    }
    acc = group_sum<G>(acc);
    if (gl == 0) {
      const float y = label[row];
      const LossOut o = eval_loss(loss, y, acc);
      py_out[row] = acc;
      dual_out[row] = o.dual;
      m_objv += o.objv;
      m_corr += ((y > 0.f && acc > 0.f) || (y <= 0.f && acc <= 0.f)) ? 1.0 : 0.0;
      m_n += 1.0;
    }
  }
  (void)lane;
  block_partials(part, sh, m_objv, m_objv, m_corr, m_n, met, ticket, acc5);
}

// ---------------------------------------------------------------- backward
// Two work lists over the CSC: keys WITHOUT an embedding are split into
// "scalar" chunks of <= kChunkS occurrences summed by one lane each (gw
// only); keys WITH an embedding into "V" chunks of <= kChunkV = 64
// occurrences, one WAVE each (gw, xxp and the 64-float gV row). A key with
// more than one chunk accumulates its chunks with float atomics.
constexpr int kChunkV = 64;

__global__ __launch_bounds__(kThreads) void k_chunk_count(int64_t nuniq,
                                                          const int64_t* __restrict__ csc_off,
                                                          const float2* __restrict__ hdr,
                                                          int64_t* cnt_s, int64_t* cnt_v) {
  const int64_t k = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (k < nuniq) {
    const int64_t c = csc_off[k + 1] - csc_off[k];
    const bool has_v = hdr && __float_as_int(hdr[k].y) >= 0;
    cnt_s[k] = has_v ? 0 : (c + kChunk - 1) / kChunk;
    cnt_v[k] = has_v ? (c + kChunkV - 1) / kChunkV : 0;
  }
}

// writes both chunk tables; zeroes the gradients of multi-chunk keys. Lane
// per key for single-chunk keys; a multi-chunk (hot) key is expanded by the
// whole wave, 64 chunks per round, so the hottest key does not serialise.
// V chunks get one packed int4 {key, csc begin, n | multi << 8, vidx} each,
// so the backward wave fetches a chunk's description in one load.
__global__ __launch_bounds__(kThreads) void k_chunk_fill(int64_t nuniq,
                                                         const int64_t* __restrict__ csc_off,
                                                         const int64_t* __restrict__ off_s,
                                                         const int64_t* __restrict__ off_v,
                                                         const float2* __restrict__ hdr,
                                                         int vstride, int32_t* key_s,
                                                         int32_t* beg_s, int4* meta_v, float* gw,
                                                         float* gvc) {
  const int lane = threadIdx.x & 63;
  const int64_t k = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  int64_t c0 = 0, nc = 0;
  int32_t b0 = 0, cnt = 0, vid = -1;
  int isv = 0;
  if (k < nuniq) {
    const int64_t ns = off_s[k + 1] - off_s[k];
    isv = ns == 0;
    c0 = isv ? off_v[k] : off_s[k];
    nc = isv ? off_v[k + 1] - c0 : ns;
    b0 = (int32_t)csc_off[k];
    cnt = (int32_t)(csc_off[k + 1] - b0);
    if (isv) vid = __float_as_int(hdr[k].y);
    if (nc == 1) {
      if (isv) {
        meta_v[c0] = make_int4((int)k, b0, cnt, vid);
      } else {
        key_s[c0] = (int32_t)k;
        beg_s[c0] = b0;
      }
    }
  }
  uint64_t m = __ballot(nc > 1);
  while (m) {
    const int src = __ffsll((unsigned long long)m) - 1;
    m &= m - 1;
    const int32_t jk = (int32_t)__shfl((int)k, src, 64);
    const int64_t jc0 = __shfl(c0, src, 64);
    const int64_t jnc = __shfl(nc, src, 64);
    const int32_t jb0 = __shfl(b0, src, 64);
    const int32_t jcnt = __shfl(cnt, src, 64);
    const int32_t jvid = __shfl(vid, src, 64);
    const int jv = __shfl(isv, src, 64);
    for (int64_t c = lane; c < jnc; c += 64) {
      if (jv) {
        const int32_t cb = (int32_t)(c * kChunkV);
        const int32_t n = jcnt - cb < kChunkV ? jcnt - cb : kChunkV;
        meta_v[jc0 + c] = make_int4(jk, jb0 + cb, n | (1 << 8), jvid);
      } else {
        key_s[jc0 + c] = jk;
        beg_s[jc0 + c] = jb0 + (int32_t)(c * kChunk);
      }
    }
    if (lane == 0) gw[jk] = 0.f;
    if (jv) {
      for (int d = lane * 4; d < vstride; d += 256)
        *reinterpret_cast<float4*>(gvc + (int64_t)jvid * vstride + d) =
            make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
}

// Single-pass version of k_chunk_count -> 2 scans -> k_chunk_fill: each tile
// of 1024 keys (4 per thread) counts its chunks, learns its chunk offsets
// (both lists) by decoupled look-back (wh_lookback.h) and fills its chunks
// in the same launch; the last tile writes the chunk totals to
// off_s[nuniq] / off_v[nuniq].
constexpr int kPlanPer = 4;
constexpr int kPlanTile = kThreads * kPlanPer;

__global__ __launch_bounds__(kThreads) void k_chunk_plan(int64_t nuniq,
                                                         const int64_t* __restrict__ csc_off,
                                                         const float2* __restrict__ hdr,
                                                         int vstride, Lookback lb, int ntiles,
                                                         int64_t* off_s_tot, int64_t* off_v_tot,
                                                         int32_t* key_s, int32_t* beg_s,
                                                         int4* meta_v, float* gw, float* gvc) {
  __shared__ uint32_t shs[16];
  __shared__ int sht;
  const int tile = lb_tile(lb, ntiles, &sht);
  const int lane = threadIdx.x & 63;
  const int64_t k0 = (int64_t)tile * kPlanTile + threadIdx.x * kPlanPer;
  int64_t co[kPlanPer + 1];
#pragma unroll
  for (int r = 0; r <= kPlanPer; ++r) co[r] = k0 + r <= nuniq ? csc_off[k0 + r] : 0;
  int32_t vid[kPlanPer];
#pragma unroll
  for (int r = 0; r < kPlanPer; ++r)
    vid[r] = (hdr && k0 + r < nuniq) ? __float_as_int(hdr[k0 + r].y) : -1;
  uint32_t c[2] = {0u, 0u};
  uint32_t nc[kPlanPer];
#pragma unroll
  for (int r = 0; r < kPlanPer; ++r) {
    nc[r] = 0;
    if (k0 + r < nuniq) {
      const int64_t cnt = co[r + 1] - co[r];
      nc[r] = vid[r] >= 0 ? (uint32_t)((cnt + kChunkV - 1) / kChunkV)
                          : (uint32_t)((cnt + kChunk - 1) / kChunk);
      c[vid[r] >= 0 ? 1 : 0] += nc[r];
    }
  }
  uint32_t ex[2], tot[2];
  lb_block_scan<2>(lb, tile, c, ex, tot, shs);
  if (tile == ntiles - 1 && threadIdx.x == 0) {
    *off_s_tot = tot[0];
    *off_v_tot = tot[1];
  }
#pragma unroll
  for (int r = 0; r < kPlanPer; ++r) {
    const int64_t k = k0 + r;
    const int isv = vid[r] >= 0;
    const int64_t c0 = isv ? ex[1] : ex[0];
    ex[isv ? 1 : 0] += nc[r];
    const int32_t b0 = (int32_t)co[r];
    const int32_t cnt = (int32_t)(co[r + 1] - co[r]);
    if (nc[r] == 1) {
      if (isv) {
        meta_v[c0] = make_int4((int)k, b0, cnt, vid[r]);
      } else {
        key_s[c0] = (int32_t)k;
        beg_s[c0] = b0;
      }
    }
    uint64_t m = __ballot(nc[r] > 1);
    while (m) {  // hot keys: the whole wave expands one key's chunk list
      const int src = __ffsll((unsigned long long)m) - 1;
      m &= m - 1;
      const int32_t jk = (int32_t)__shfl((int)k, src, 64);
      const int64_t jc0 = __shfl(c0, src, 64);
      const int64_t jnc = __shfl((int)nc[r], src, 64);
      const int32_t jb0 = __shfl(b0, src, 64);
      const int32_t jcnt = __shfl(cnt, src, 64);
      const int32_t jvid = __shfl(vid[r], src, 64);
      const int jv = __shfl(isv, src, 64);
      for (int64_t q = lane; q < jnc; q += 64) {
        if (jv) {
          const int32_t cb = (int32_t)(q * kChunkV);
          const int32_t n = jcnt - cb < kChunkV ? jcnt - cb : kChunkV;
          meta_v[jc0 + q] = make_int4(jk, jb0 + cb, n | (1 << 8), jvid);
        } else {
          key_s[jc0 + q] = jk;
          beg_s[jc0 + q] = jb0 + (int32_t)(q * kChunk);
        }
      }
      if (lane == 0) gw[jk] = 0.f;
      if (jv) {
        for (int d = lane * 4; d < vstride; d += 256)
          *reinterpret_cast<float4*>(gvc + (int64_t)jvid * vstride + d) =
              make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  }
}

// V-chunk order: chunks bucketed by the first row they touch (256 row
// windows of ~400 rows for a 100k minibatch), so the chunks in flight at any
// moment cover a narrow window of rows and their xv gathers hit in L2. A
// key-ordered list had every hot key's chunks sweep all rows concurrently:
// 31% L2 hit rate and 248 us in rocprof, vs 144 us bucketed. A three-kernel
// counting sort (block histograms -> bucket-major scan -> scatter); rocPRIM's
// radix_sort_pairs picks a 10-pass merge sort at this size (124 us).
constexpr int kBuckets = 256;
constexpr int kBucketBlocks = 128;
constexpr int kBucketU = 8;  // chunks per thread with loads in flight together

__device__ __forceinline__ int row_bucket(int row, int shift) {
  const int b = row >> shift;
  return b < kBuckets ? b : kBuckets - 1;
}

__global__ __launch_bounds__(kThreads) void k_vchunk_hist(const int64_t* __restrict__ nchunk_p,
                                                          const int4* __restrict__ meta,
                                                          const int32_t* __restrict__ csc_row,
                                                          int shift, int32_t* hist) {
  __shared__ int32_t h[kBuckets];
  for (int i = threadIdx.x; i < kBuckets; i += kThreads) h[i] = 0;
  __syncthreads();
  const int64_t n = *nchunk_p;
  const int64_t per = (n + gridDim.x - 1) / gridDim.x;
  const int64_t c0 = per * blockIdx.x, c1 = c0 + per < n ? c0 + per : n;
  // kBucketU independent meta -> row load chains in flight per thread (one
  // chain at a time left this kernel waiting on ~17 round trips)
  for (int64_t cb = c0 + threadIdx.x; cb < c1; cb += kThreads * kBucketU) {
    int idx[kBucketU], row[kBucketU];
#pragma unroll
    for (int u = 0; u < kBucketU; ++u) {
      const int64_t c = cb + (int64_t)u * kThreads;
      idx[u] = c < c1 ? meta[c].y : -1;
    }
#pragma unroll
    for (int u = 0; u < kBucketU; ++u) row[u] = idx[u] >= 0 ? csc_row[idx[u]] : -1;
#pragma unroll
    for (int u = 0; u < kBucketU; ++u)
      if (row[u] >= 0) atomicAdd(&h[row_bucket(row[u], shift)], 1);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kBuckets; i += kThreads) hist[blockIdx.x * kBuckets + i] = h[i];
}

// one block of 1024: hist[block][bucket] -> bucket-major exclusive offsets in
// place. Four threads per bucket each own a quarter of the blocks, so every
// load is independent (the serial per-bucket walk took ~15-20 us of load
// latency); the 256 bucket totals are scanned by the first four waves.
constexpr int kScanParts = 4;
constexpr int kScanPer = kBucketBlocks / kScanParts;

__global__ __launch_bounds__(kBuckets * kScanParts) void k_vchunk_scan(int32_t* hist) {
  __shared__ int32_t part[kScanParts][kBuckets];
  __shared__ int32_t excl[kBuckets];
  __shared__ int32_t wtot[kBuckets / 64];
  const int b = threadIdx.x & (kBuckets - 1), q = threadIdx.x / kBuckets;
  int32_t v[kScanPer];
#pragma unroll
  for (int i = 0; i < kScanPer; ++i) v[i] = hist[(q * kScanPer + i) * kBuckets + b];
  int32_t sum = 0;
#pragma unroll
  for (int i = 0; i < kScanPer; ++i) sum += v[i];
  part[q][b] = sum;
  __syncthreads();
  if (q == 0) {  // bucket totals -> wave-local inclusive scans
    int32_t t = 0;
#pragma unroll
    for (int r = 0; r < kScanParts; ++r) t += part[r][b];
    const int lane = b & 63;
    int32_t x = t;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int32_t y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) wtot[b >> 6] = x;
    excl[b] = x - t;
  }
  __syncthreads();
  int32_t base = excl[b];
  for (int w = 0; w < (b >> 6); ++w) base += wtot[w];
  for (int r = 0; r < q; ++r) base += part[r][b];
#pragma unroll
  for (int i = 0; i < kScanPer; ++i) {
    hist[(q * kScanPer + i) * kBuckets + b] = base;
    base += v[i];
  }
}

__global__ __launch_bounds__(kThreads) void k_vchunk_scatter(const int64_t* __restrict__ nchunk_p,
                                                             const int4* __restrict__ meta,
                                                             const int32_t* __restrict__ csc_row,
                                                             int shift,
                                                             const int32_t* __restrict__ hist,
                                                             int4* out) {
  __shared__ int32_t base[kBuckets];
  for (int i = threadIdx.x; i < kBuckets; i += kThreads) base[i] = hist[blockIdx.x * kBuckets + i];
  __syncthreads();
  const int64_t n = *nchunk_p;
  const int64_t per = (n + gridDim.x - 1) / gridDim.x;
  const int64_t c0 = per * blockIdx.x, c1 = c0 + per < n ? c0 + per : n;
  for (int64_t cb = c0 + threadIdx.x; cb < c1; cb += kThreads * kBucketU) {
    int4 m[kBucketU];
    int row[kBucketU];
#pragma unroll
    for (int u = 0; u < kBucketU; ++u) {
      const int64_t c = cb + (int64_t)u * kThreads;
      m[u] = c < c1 ? meta[c] : make_int4(0, -1, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < kBucketU; ++u) row[u] = m[u].y >= 0 ? csc_row[m[u].y] : -1;
#pragma unroll
    for (int u = 0; u < kBucketU; ++u)
      if (row[u] >= 0) out[atomicAdd(&base[row_bucket(row[u], shift)], 1)] = m[u];
  }
}

// scalar chunks: one lane sums dual_i * x_ik over <= kChunk occurrences
__global__ __launch_bounds__(kThreads) void k_bwd_scalar(const int64_t* __restrict__ nchunk_p,
                                                         const int32_t* __restrict__ chunk_key,
                                                         const int32_t* __restrict__ chunk_beg,
                                                         const int64_t* __restrict__ csc_off,
                                                         const int32_t* __restrict__ csc_row,
                                                         const float* __restrict__ csc_val,
                                                         const float* __restrict__ dual,
                                                         float* __restrict__ gw_out,
                                                         float* __restrict__ part_gw) {
  const int64_t c = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (c >= *nchunk_p) return;
  const int k = chunk_key[c];
  const int kb = (int)csc_off[k], ke = (int)csc_off[k + 1];
  const int b = chunk_beg[c];
  const int e = b + kChunk < ke ? b + kChunk : ke;
  float gw = 0.f;
  int p = b;
  for (; p + 3 < e; p += 4) {  // 4 independent row->dual chains in flight
    int i[4];
    float x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      i[u] = csc_row[p + u];
      x[u] = csc_val ? csc_val[p + u] : 1.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) gw += dual[i[u]] * x[u];
  }
  for (; p < e; ++p) gw += dual[csc_row[p]] * (csc_val ? csc_val[p] : 1.f);
  if (ke - kb <= kChunk) gw_out[k] = gw;
  else if (part_gw) part_gw[c] = gw;  // deterministic: summed in chunk order later
  else atomicAdd(gw_out + k, gw);
}

// V chunks: one wave per chunk, persistent over the (device-counted) list,
// software-pipelined like the forward: while chunk i's xv rows are gathered,
// the duals of chunk i+1, the CSC rows of chunk i+2 and the description of
// chunk i+3 are in flight.
template <int G>
__global__ __launch_bounds__(kThreads) void k_bwd_v(const int64_t* __restrict__ nchunk_p,
                                                    const int4* __restrict__ meta,
                                                    const int32_t* __restrict__ csc_row,
                                                    const float* __restrict__ csc_val,
                                                    const float* __restrict__ dual,
                                                    const float* __restrict__ xv,
                                                    const float* __restrict__ vc, int vstride,
                                                    float* __restrict__ gw_out,
                                                    float* __restrict__ gvc,
                                                    float* __restrict__ part_gw,
                                                    float* __restrict__ part_gv) {
  using S = Shape<G>;
  __shared__ int2 stage[kThreads / 64][64];
  int2* st = stage[threadIdx.x >> 6];
  const int lane = threadIdx.x & 63, gl = lane & (G - 1), sub = lane / G;
  const int64_t nch_all = *nchunk_p;
  const int64_t nch = nch_all, nw = (int64_t)gridDim.x * (kThreads / 64);
  const int64_t w0 =
      __builtin_amdgcn_readfirstlane((int)(((int64_t)blockIdx.x * kThreads + threadIdx.x) >> 6));
  auto get_meta = [&](int64_t c) {
    return c < nch ? meta[c] : make_int4(0, 0, 0, -1);
  };
  auto load_rows = [&](const int4& mt, int& r, float& x) {
    const bool ok = lane < (mt.z & 0xff);
    r = ok ? csc_row[mt.y + lane] : -1;
    x = ok ? (csc_val ? csc_val[mt.y + lane] : 1.f) : 0.f;
  };
  int64_t c = w0;
  int4 mc = get_meta(c), mn = get_meta(c + nw), m2 = get_meta(c + 2 * nw),
       m3 = make_int4(0, 0, 0, -1);
  int rc, rn, r2 = -1;
  float xc, xn, x2 = 0.f;
  load_rows(mc, rc, xc);
  float dc = rc >= 0 ? dual[rc] * xc : 0.f;
  load_rows(mn, rn, xn);
  float dn = 0.f;
  for (; c < nch; c += nw) {
    const int n = mc.z & 0xff;
    const bool multi = (mc.z >> 8) != 0;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    stage_pairs<G>(st, lane, rc, dc);
    // one gather batch of TB instructions starting at instruction t0
    auto batch = [&](auto tb, int t0) {
      constexpr int TB = decltype(tb)::value;
      float4 a[TB];
      float du[TB];
#pragma unroll
      for (int t = 0; t < TB; ++t) {
        const int2 e = st[sub * S::NI + t0 + t];
        du[t] = __int_as_float(e.y);
        const float* src = e.x >= 0 ? xv + (uint32_t)e.x * (uint32_t)S::VS : kZeroRow;
        a[t] = reinterpret_cast<const float4*>(src)[gl];
      }
      if (t0 == 0) {
        v = reinterpret_cast<const float4*>(vc + (uint32_t)mc.w * (uint32_t)S::VS)[gl];
        // prefetch the next stages behind the gathers
        dn = rn >= 0 ? dual[rn] * xn : 0.f;
        load_rows(m2, r2, x2);
        m3 = get_meta(c + 3 * nw);
      }
#pragma unroll
      for (int t = 0; t < TB; ++t) {
        acc.x += du[t] * a[t].x; acc.y += du[t] * a[t].y;
        acc.z += du[t] * a[t].z; acc.w += du[t] * a[t].w;
      }
    };
    // full chunks (hot keys) issue every instruction in one batch for the
    // most loads in flight; short chunks issue only the live instructions
    if (n > S::NI * S::SUB / 2) {
      batch(std::integral_constant<int, S::NI>(), 0);
    } else {
#pragma unroll
      for (int t0 = 0; t0 < S::NI; t0 += S::TI) {
        if (t0 * S::SUB >= n) break;
        batch(std::integral_constant<int, S::TI>(), t0);
      }
    }
    if (n == 0) {  // (chunks are never empty; keep the pipeline consistent anyway)
      dn = rn >= 0 ? dual[rn] * xn : 0.f;
      load_rows(m2, r2, x2);
      m3 = get_meta(c + 3 * nw);
    }
    const float gw = wave_sum(dc);
    const float xxp = wave_sum(dc * xc);
#pragma unroll
    for (int o = G; o < 64; o <<= 1) {
      acc.x += __shfl_xor(acc.x, o, 64); acc.y += __shfl_xor(acc.y, o, 64);
      acc.z += __shfl_xor(acc.z, o, 64); acc.w += __shfl_xor(acc.w, o, 64);
    }
    if (lane == 0) {
      if (!multi) gw_out[mc.x] = gw;
      else if (part_gw) part_gw[c] = gw;
      else atomicAdd(gw_out + mc.x, gw);
    }
    acc.x -= xxp * v.x; acc.y -= xxp * v.y; acc.z -= xxp * v.z; acc.w -= xxp * v.w;
    if (!multi || part_gv) {
      // single chunk: the row itself; deterministic mode: this chunk's
      // partial row (the list is key-major, unbucketed), summed in order later
      float* dst = multi ? part_gv + c * (int64_t)vstride : gvc + (int64_t)mc.w * vstride;
      if (sub == 0) *reinterpret_cast<float4*>(dst + gl * 4) = acc;
    } else {
      // every sub-group holds the whole row after the butterfly: lane l adds
      // dim l (+ 64 c), so each atomic wave-instruction covers 256
      // contiguous bytes (4 memory-side requests) instead of 16 lanes at a
      // 16-byte stride (16 requests per row)
      float* gv = gvc + (int64_t)mc.w * vstride;
#pragma unroll
      for (int c = 0; c < (S::VS + 63) / 64; ++c) {
        const int d = c * 64 + lane;
        const int src = (d >> 2) & (G - 1);
        const float ax = __shfl(acc.x, src, 64), ay = __shfl(acc.y, src, 64);
        const float az = __shfl(acc.z, src, 64), aw = __shfl(acc.w, src, 64);
        const int comp = d & 3;
        const float a = comp == 0 ? ax : comp == 1 ? ay : comp == 2 ? az : aw;
        if (d < S::VS) atomicAdd(gv + d, a);
      }
    }
    // rotate the pipeline
    mc = mn; rc = rn; xc = xn; dc = dn;
    mn = m2; rn = r2; xn = x2;
    m2 = m3;
  }
}

// Deterministic mode: the partials of every multi-chunk key, summed in chunk
// order (= occurrence order) by one wave per key, found at its first chunk.
__global__ __launch_bounds__(kThreads) void k_bwd_reduce_s(const int64_t* __restrict__ nchunk_p,
                                                           const int32_t* __restrict__ chunk_key,
                                                           const int32_t* __restrict__ chunk_beg,
                                                           const int64_t* __restrict__ csc_off,
                                                           const float* __restrict__ part_gw,
                                                           float* __restrict__ gw_out) {
  const int64_t c = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (c >= *nchunk_p) return;
  const int k = chunk_key[c];
  const int64_t kb = csc_off[k], cnt = csc_off[k + 1] - kb;
  if (cnt <= kChunk || chunk_beg[c] != kb) return;
  const int64_t n = (cnt + kChunk - 1) / kChunk;
  float s = 0.f;
  for (int64_t q = 0; q < n; ++q) s += part_gw[c + q];
  gw_out[k] = s;
}

__global__ __launch_bounds__(kThreads) void k_bwd_reduce_v(const int64_t* __restrict__ nchunk_p,
                                                           const int4* __restrict__ meta,
                                                           const int64_t* __restrict__ csc_off,
                                                           const float* __restrict__ part_gw,
                                                           const float* __restrict__ part_gv,
                                                           int vstride, float* __restrict__ gw_out,
                                                           float* __restrict__ gvc) {
  const int lane = threadIdx.x & 63;
  const int64_t c = ((int64_t)blockIdx.x * kThreads + threadIdx.x) >> 6;
  if (c >= *nchunk_p) return;
  const int4 m = meta[c];
  if ((m.z >> 8) == 0 || (int64_t)m.y != csc_off[m.x]) return;  // not a hot key's first chunk
  const int64_t cnt = csc_off[m.x + 1] - m.y;
  const int64_t n = (cnt + kChunkV - 1) / kChunkV;
  float g = 0.f;
  for (int64_t q = 0; q < n; ++q) g += part_gw[c + q];
  for (int d = lane; d < vstride; d += 64) {
    float a = 0.f;
    for (int64_t q = 0; q < n; ++q) a += part_gv[(c + q) * vstride + d];
    gvc[(int64_t)m.w * vstride + d] = a;
  }
  if (lane == 0) gw_out[m.x] = g;
}

// gradient clipping / dropout / normalisation on the m embedding-gradient
// rows (reference learn/difacto/loss.h:131-155); m is a device count
__global__ __launch_bounds__(kThreads) void k_grad_post(const int64_t* __restrict__ m_p,
                                                        float* gvc, int vstride, int dim,
                                                        float clip, float dropout, uint64_t seed,
                                                        double* sumsq) {
  // grid-stride (grid capped at 1024 blocks): one sumsq atomic per block
  __shared__ double sh[kThreads / 64];
  const int64_t total = *m_p * vstride;
  double ss = 0;
  for (int64_t t = (int64_t)blockIdx.x * kThreads + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * kThreads) {
    const int64_t r = t / vstride;
    const int d = (int)(t % vstride);
    if (d >= dim) continue;
    float v = gvc[t];
    if (clip > 0.f) v = fminf(fmaxf(v, -clip), clip);
    if (dropout > 0.f && uhash01(seed, (uint64_t)r, (uint64_t)d) > 1.f - dropout) v = 0.f;
    gvc[t] = v;
    ss += (double)v * v;
  }
  if (sumsq) {
    const double s = block_sum_d(ss, sh);
    if (threadIdx.x == 0) atomicAdd(sumsq, s);
  }
}

__global__ __launch_bounds__(kThreads) void k_grad_scale(const int64_t* __restrict__ m_p,
                                                         float* gvc, int vstride, int dim,
                                                         const double* sumsq) {
  const int64_t t = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  const double n2 = *sumsq;
  if (n2 < 1e-10 || t / vstride >= *m_p || (int)(t % vstride) >= dim) return;
  gvc[t] = (float)(gvc[t] / sqrt(n2));
}

}  // namespace

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

int64_t fm_fwd_partials() { return 4 * kFwdBlocks; }
int64_t fwd_ticket_words() { return kArriveWords; }

// CUs the persistent FM kernels leave free for concurrent collectives. A
// persistent grid that fills every CU's wave slots keeps RCCL's channel
// workgroups (all-to-all over xGMI, issued beside the compute) from being
// dispatched until the whole kernel drains, which serialises the transfer
// behind the compute instead of overlapping it. Set by the multi-rank step
// (kv/psx.py: WH_RCCL_CU_RESERVE); 0 on one GPU.
static int g_cu_reserve = 0;

void fm_set_cu_reserve(int cus) { g_cu_reserve = cus < 0 ? 0 : cus; }
int fm_cu_reserve() { return g_cu_reserve; }

static int device_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    WH_HIP_CHECK(hipGetDevice(&dev));
    WH_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  return std::max(1, cus - std::min(g_cu_reserve, cus / 2));
}

// Persistent grids are sized to what is actually resident: blocks per CU from
// the occupancy API (register-limited kernels fit fewer than 8) x CU count,
// so no block waits for a second round behind a full machine.
template <typename K>
static int resident_blocks(K kernel, int cap) {
  const int cus = device_cus();
  int per_cu = 0;
  WH_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kThreads, 0));
  const int n = std::max(1, per_cu) * cus;
  return n < cap ? n : cap;
}

#define WH_RESIDENT(G, KERNEL, CAP)                                            \
  ((G) == 1 ? resident_blocks(KERNEL<1>, CAP) : (G) == 2 ? resident_blocks(KERNEL<2>, CAP) \
   : (G) == 4 ? resident_blocks(KERNEL<4>, CAP) : (G) == 8 ? resident_blocks(KERNEL<8>, CAP) \
   : (G) == 16 ? resident_blocks(KERNEL<16>, CAP) : (G) == 32 ? resident_blocks(KERNEL<32>, CAP) \
   : resident_blocks(KERNEL<64>, CAP))

void fm_forward(int64_t nrows, const int64_t* offset, const int32_t* lid, const float* val,
                const float* w_or_hdr, const float* vc, int vstride, const float* label, int loss,
                float* py, float* dual, float* xv, double* met, double* part,
                unsigned int* ticket, hipStream_t s) {
  if (nrows <= 0) return;
  const int acc5 = (loss >> 8) & 1;  // kLossAcc5: met[4] += flipped accuracy
  loss &= 0xff;
  int nblk;
  if (vstride == 0) {
    constexpr int G = 8;
    nblk = grid_for(nrows * G, kThreads, kFwdBlocks);
    hipLaunchKernelGGL(k_lin_fwd<G>, dim3(nblk), dim3(kThreads), 0, s, nrows, offset, lid, val,
                       w_or_hdr, 1, label, loss, py, dual, part, met, ticket, acc5);
  } else {
    const int G = vstride / 4;  // vstride <= 256 enforced by the binding
    const float2* hdr = reinterpret_cast<const float2*>(w_or_hdr);
    nblk = grid_for(nrows * 64, kThreads, WH_RESIDENT(G, k_fm_fwd, kFwdBlocks));
    const dim3 grid(nblk), block(kThreads);
    WH_DISPATCH_G(G, k_fm_fwd, grid, block, 0, s, nrows, offset, lid, val, hdr, vc, vstride,
                  label, loss, py, dual, xv, part, met, ticket, acc5);
  }
}

void lin_forward_strided(int64_t nrows, const int64_t* offset, const int32_t* lid,
                         const float* val, const float* w, int wstride, const float* label,
                         int loss, float* py, float* dual, double* met, double* part,
                         unsigned int* ticket, hipStream_t s) {
  if (nrows <= 0) return;
  const int acc5 = (loss >> 8) & 1;
  loss &= 0xff;
  // 8 lanes per row (16: 80.3-81.0, 32: 75.4 vs 82.8 M ex/s at 10k rows)
  constexpr int G = 8;
  const int nblk = grid_for(nrows * G, kThreads, kFwdBlocks);
  hipLaunchKernelGGL(k_lin_fwd<G>, dim3(nblk), dim3(kThreads), 0, s, nrows, offset, lid, val, w,
                     wstride, label, loss, py, dual, part, met, ticket, acc5);
}

static int64_t scalar_cap(int64_t nuniq, int64_t nnz) { return nuniq + nnz / kChunk + 1; }
static int64_t v_cap(int64_t nuniq, int64_t nnz) { return nuniq + nnz / kChunkV + 1; }

int64_t fm_bwd_chunks_bound(int64_t nuniq, int64_t nnz) {
  return scalar_cap(nuniq, nnz) + v_cap(nuniq, nnz);
}

int64_t fm_bwd_meta_bound(int64_t nuniq, int64_t nnz) { return v_cap(nuniq, nnz); }

static int bucket_shift(int64_t nrows) {
  int shift = 0;
  while ((((nrows - 1) >> shift) >= kBuckets)) ++shift;
  return shift;
}

int64_t fm_bwd_bucket_scratch() { return (int64_t)kBuckets * kBucketBlocks; }

void fm_backward(int64_t nuniq, int64_t nnz, int64_t nrows, const int64_t* csc_off,
                 const int32_t* csc_row, const float* csc_val, const float* dual, const float* xv,
                 const float* hdr_f, const float* vc, int vstride, float* gw, float* gvc,
                 int32_t* chunk_key, int32_t* chunk_beg, int32_t* meta_v_i32, int32_t* bucket_hist,
                 int64_t* chunk_cnt, int64_t* chunk_off, int64_t* scan_tmp, const Lookback* lb,
                 hipStream_t s, float* det_part, int phase) {
  int4* meta_v = reinterpret_cast<int4*>(meta_v_i32);
  if (nuniq <= 0) return;
  const float2* hdr = vstride > 0 ? reinterpret_cast<const float2*>(hdr_f) : nullptr;
  int64_t* cnt_s = chunk_cnt;
  int64_t* cnt_v = chunk_cnt + nuniq;
  int64_t* off_s = chunk_off;
  int64_t* off_v = chunk_off + nuniq + 1;
  const int64_t cap_s = scalar_cap(nuniq, nnz);
  int32_t* key_s = chunk_key;
  int32_t* beg_s = chunk_beg;
  const int64_t ntiles = (nuniq + kPlanTile - 1) / kPlanTile;
  const int64_t vcap = v_cap(nuniq, nnz);
  // V chunks ordered by first-row bucket (meta_v[cap..2cap) receives the
  // list); deterministic mode keeps the key-major list (partials by index),
  // and so does a minibatch whose xv rows fit in L2 many times over (the
  // bucketing buys locality there is no need for: three launches of host
  // time in a launch-bound small step)
  const bool bucket = hdr && !det_part && nrows * (int64_t)vstride * 4 > ((int64_t)2 << 20);
  int4* meta_sorted = bucket ? meta_v + vcap : meta_v;
  if (phase != 2) {
  if (lb && ntiles <= kLbMaxTiles) {  // one launch
    hipLaunchKernelGGL(k_chunk_plan, dim3((unsigned)ntiles), dim3(kThreads), 0, s, nuniq, csc_off,
                       hdr, vstride, *lb, (int)ntiles, off_s + nuniq, off_v + nuniq, key_s, beg_s,
                       meta_v, gw, gvc);
  } else {
    hipLaunchKernelGGL(k_chunk_count, dim3(grid_for(nuniq, kThreads)), dim3(kThreads), 0, s,
                       nuniq, csc_off, hdr, cnt_s, cnt_v);
    scan_i64(cnt_s, off_s, nuniq, scan_tmp, s);
    if (hdr) scan_i64(cnt_v, off_v, nuniq, scan_tmp, s);
    hipLaunchKernelGGL(k_chunk_fill, dim3(grid_for(nuniq, kThreads)), dim3(kThreads), 0, s,
                       nuniq, csc_off, off_s, off_v, hdr, vstride, key_s, beg_s, meta_v, gw, gvc);
  }
  if (bucket) {
    const int shift = bucket_shift(std::max<int64_t>(nrows, 1));
    hipLaunchKernelGGL(k_vchunk_hist, dim3(kBucketBlocks), dim3(kThreads), 0, s, off_v + nuniq,
                       meta_v, csc_row, shift, bucket_hist);
    hipLaunchKernelGGL(k_vchunk_scan, dim3(1), dim3(kBuckets * kScanParts), 0, s, bucket_hist);
    hipLaunchKernelGGL(k_vchunk_scatter, dim3(kBucketBlocks), dim3(kThreads), 0, s, off_v + nuniq,
                       meta_v, csc_row, shift, bucket_hist, meta_sorted);
  }
  }
  if (phase == 1) return;
  // chunk counts are device values (off[nuniq]); the scalar kernel launches
  // over the host-side bound and surplus lanes exit; the V kernel is
  // persistent. No host synchronisation in the step.
  // deterministic scratch: [cap_s] scalar partials | [vcap] V-chunk gw | [vcap, vstride] rows
  float* pgs = det_part;
  float* pgv_w = det_part ? det_part + cap_s : nullptr;
  float* pgv = det_part ? pgv_w + vcap : nullptr;
  hipLaunchKernelGGL(k_bwd_scalar, dim3(grid_for(cap_s, kThreads)), dim3(kThreads), 0, s,
                     off_s + nuniq, key_s, beg_s, csc_off, csc_row, csc_val, dual, gw, pgs);
  if (det_part)
    hipLaunchKernelGGL(k_bwd_reduce_s, dim3(grid_for(cap_s, kThreads)), dim3(kThreads), 0, s,
                       off_s + nuniq, key_s, beg_s, csc_off, pgs, gw);
  if (!hdr) return;
  const int G = vstride / 4;
  int64_t vblk = std::min<int64_t>((v_cap(nuniq, nnz) + 3) / 4,
                                   WH_RESIDENT(G, k_bwd_v, 2048));
  // (an XCD-aware split of the chunk list -- group b % 8 of the blocks on
  // the b % 8-th eighth -- raised this kernel's L2 hit rate 44.5 -> 54.7 %
  // but cost the step 1.5 %: the groups' uneven ends leave a tail beside the
  // concurrent localize; measured round 4, removed)
  const dim3 grid((unsigned)vblk), block(kThreads);
  WH_DISPATCH_G(G, k_bwd_v, grid, block, 0, s, off_v + nuniq, meta_sorted, csc_row, csc_val,
                dual, xv, vc, vstride, gw, gvc, pgv_w, pgv);
  if (det_part)
    hipLaunchKernelGGL(k_bwd_reduce_v, dim3(grid_for(vcap * 64, kThreads)), dim3(kThreads), 0, s,
                       off_v + nuniq, meta_v, csc_off, pgv_w, pgv, vstride, gw, gvc);
}

int64_t fm_bwd_det_floats(int64_t nuniq, int64_t nnz, int vstride) {
  return scalar_cap(nuniq, nnz) + v_cap(nuniq, nnz) * (1 + (int64_t)vstride);
}

void fm_grad_post(const int64_t* m, int64_t m_cap, float* gvc, int vstride, int dim, float clip,
                  float dropout, uint64_t seed, double* sumsq, hipStream_t s) {
  if (m_cap <= 0 || vstride == 0) return;
  hipLaunchKernelGGL(k_grad_post, dim3(grid_for(m_cap * vstride, kThreads, 1024)), dim3(kThreads),
                     0, s, m, gvc, vstride, dim, clip, dropout, seed, sumsq);
}

void fm_grad_scale(const int64_t* m, int64_t m_cap, float* gvc, int vstride, int dim,
                   const double* sumsq, hipStream_t s) {
  if (m_cap <= 0 || vstride == 0) return;
  hipLaunchKernelGGL(k_grad_scale, dim3(grid_for(m_cap * vstride, kThreads)), dim3(kThreads), 0,
                     s, m, gvc, vstride, dim, sumsq);
}

}  // namespace wh
