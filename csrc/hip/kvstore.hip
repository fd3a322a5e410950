// Device-resident sharded parameter store and fused optimizer updates.
//
// Replaces the ps-lite OnlineServer/KVStore with per-GPU open-addressing
// tables in HBM (keys + SoA value arrays + an embedding slab), and the
// per-key server handles with fused kernels:
//   * linear SGD / AdaGrad / FTRL + L1L2 proximal step
//       (reference learn/linear/async_sgd.h:71-180, learn/linear/penalty.h:36-41)
//   * DiFacto: feature-count push with lazy V allocation, FTRL on w,
//     AdaGrad on V, variable-length pull
//       (reference learn/difacto/async_sgd.h:214-296)
// One lane group of G = vstride/4 lanes owns one key (float4 per lane), so a
// 64-dim embedding row is one 256-byte coalesced access per 16 lanes.
#include "wh_common.h"
#include "wh_kernels.h"
#include "wh_lookback.h"
#include "kv_device.h"

namespace wh {
namespace {

using namespace kvd;

__global__ __launch_bounds__(kThreads) void k_kv_find(const uint64_t* keys_in, int64_t n,
                                                      KVSlot* tsl, int64_t cap, int insert,
                                                      int32_t* slot, int64_t* stats) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  bool created = false, failed = false;
  if (i < n) {
    const uint64_t k = keys_in[i];
    const uint64_t mask = (uint64_t)cap - 1;
    const uint64_t h = mix64(k) & mask;
    const int32_t res = probe_slot(tsl, mask, k, h, ld_relaxed(&tsl[h].key), insert, &created);
    if (insert && res < 0) failed = true;
    slot[i] = (int32_t)res;
  }
  const uint64_t bc = __ballot(created), bf = __ballot(failed);
  if ((threadIdx.x & 63) == 0) {
    if (bc) atomicAdd(stat_ptr(stats, 4), (unsigned long long)__popcll(bc));
    if (bf) atomicAdd(stat_ptr(stats, 2), (unsigned long long)__popcll(bf));
  }
}

__global__ __launch_bounds__(kThreads) void k_kv_occupied(const KVSlot* tsl, int64_t cap,
                                                          int32_t* out, int64_t* out_n) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  const bool occ = i < cap && tsl[i].key != kEmptyKey;
  const uint64_t b = __ballot(occ);
  const int lane = threadIdx.x & 63;
  int64_t base = 0;
  if (lane == 0 && b)
    base = (int64_t)atomicAdd((unsigned long long*)out_n, (unsigned long long)__popcll(b));
  base = __shfl(base, 0, 64);
  if (occ) {
    const int rank = __popcll(b & ((1ull << lane) - 1));
    out[base + rank] = (int32_t)i;
  }
}

__global__ __launch_bounds__(kThreads) void k_linear_pull(const KVSlot* tsl, const int32_t* slot,
                                                          int64_t n, float* out) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i < n) {
    const int32_t s = slot[i];
    out[i] = s >= 0 ? tsl[s].w : 0.f;
  }
}

__global__ __launch_bounds__(kThreads) void k_linear_push(KVTable t, const int32_t* slot,
                                                          const float* grad, int64_t n,
                                                          LinearHP hp) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  float oldw = 0.f, neww = 0.f;
  if (i < n) {
    const int32_t s = slot[i];
    if (s >= 0) {
      oldw = t.sl[s].w;
      neww = linear_update(t.sl[s], grad[i], hp, hp.sgd_eta);
    }
  }
  count_nnz_delta(oldw, neww, t.stats);
}


// ---------------------------------------------------------------- difacto
// Layout of the work: ONE LANE PER KEY for everything scalar (count add,
// FTRL on w, the allocation decision), then the wave cooperatively runs the
// per-key embedding-row jobs (init a new V row / AdaGrad an existing one /
// copy a row out) with G = vstride/4 lanes per row, 64/G rows at a time.
// Most keys of a power-law minibatch have no V, so lane-per-key keeps all 64
// lanes busy on the scalar part instead of 1 of every G.

template <int G>
__global__ __launch_bounds__(kThreads) void k_difacto_push_cnt(KVTable t, const int32_t* slot,
                                                               const float* cnt,
                                                               const int32_t* cnti, int64_t n,
                                                               DifactoHP hp) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  int32_t s = -1;
  bool want = false;
  if (i < n) {
    s = slot[i];
    if (s >= 0) {
      const uint32_t c = t.sl[s].cnt + (cnt ? (uint32_t)cnt[i] : (uint32_t)cnti[i]);
      t.sl[s].cnt = c;
      want = t.vstride > 0 && c > hp.threshold && t.sl[s].vrow < 0 &&
             (!hp.l1_shrk || t.sl[s].w != 0.f);
    }
  }
  if (t.vstride == 0) return;
  const int32_t row = wave_alloc_rows(t, want);
  if (row >= 0) t.sl[s].vrow = row;
  long long newv = row >= 0 ? t.dim : 0;
  for_each_row_job<G>(row >= 0, [&](int src, int gl) {
    const int sl = src >= 0 ? src : lane;
    const int32_t js = __shfl(s, sl, 64), jr = __shfl(row, sl, 64);
    if (src >= 0) init_v_row(t, t.sl[js].key, jr, gl, G, hp);
  });
  newv = wave_sum_ll(newv);
  if (lane == 0 && newv) atomicAdd(stat_ptr(t.stats, 1), (unsigned long long)newv);
}

__global__ __launch_bounds__(kThreads) void k_difacto_pull_hdr(KVTable t, const int32_t* slot,
                                                               int64_t n, int l1_shrk,
                                                               float2* hdr, int32_t* vflag) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const int32_t s = slot[i];
  float w = 0.f;
  int32_t row = -1;
  if (s >= 0) {
    w = t.sl[s].w;
    row = t.vstride > 0 ? t.sl[s].vrow : -1;
    if (l1_shrk && w == 0.f) row = -1;
  }
  hdr[i] = make_float2(w, __int_as_float(-1));
  vflag[i] = row >= 0 ? 1 : 0;
}

// copy the V rows of flagged keys into their compact position
template <int G>
__global__ __launch_bounds__(kThreads) void k_difacto_pull_rows(KVTable t, const int32_t* slot,
                                                                int64_t n,
                                                                const int32_t* __restrict__ vflag,
                                                                const int64_t* __restrict__ vpos,
                                                                float2* hdr, float* vc) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  int32_t row = -1, vp = -1;
  if (i < n && vflag[i]) {
    row = t.sl[slot[i]].vrow;
    vp = (int32_t)vpos[i];
    hdr[i].y = __int_as_float(vp);
  }
  for_each_row_job<G>(row >= 0, [&](int src, int gl) {
    const int sl = src >= 0 ? src : lane;
    const int32_t jr = __shfl(row, sl, 64), jp = __shfl(vp, sl, 64);
    if (src >= 0) {
      const float* V = t.V + (int64_t)jr * t.vstride;
      float* o = vc + (int64_t)jp * t.vstride;
      for (int c = gl * 4; c < t.vstride; c += 4 * G)
        *reinterpret_cast<float4*>(o + c) = *reinterpret_cast<const float4*>(V + c);
    }
  });
}

// Fused variable-length pull: header, V-flag scan (decoupled look-back)
// and row copy in ONE launch (was: header kernel, 3-launch scan, row kernel).
// A tile is 1024 consecutive keys, 4 per thread (vector loads of the slot
// ids, 32-byte header stores), so a 515k-key minibatch is ~500 tiles and the
// look-back finishes in ~2 windows.

template <int G>
__global__ __launch_bounds__(kThreads) void k_difacto_pull(KVTable t, const int32_t* slot,
                                                           int64_t n, int l1_shrk, Lookback lb,
                                                           int ntiles, float2* hdr, int64_t* vpos,
                                                           float* vc) {
  __shared__ uint32_t shs[16];
  __shared__ int sht;
  const int tile = lb_tile(lb, ntiles, &sht);
  const int lane = threadIdx.x & 63;
  const int64_t i0 = (int64_t)tile * kPullTile + threadIdx.x * kPullPer;
  int32_t sl[kPullPer];
  bool vec = false;
  if constexpr (kPullPer == 4) {
    if (i0 + kPullPer <= n && (reinterpret_cast<uintptr_t>(slot) & 15) == 0) {
      const int4 q = *reinterpret_cast<const int4*>(slot + i0);
      sl[0] = q.x; sl[1] = q.y; sl[2] = q.z; sl[3] = q.w;
      vec = true;
    }
  }
  if (!vec) {
#pragma unroll
    for (int r = 0; r < kPullPer; ++r) sl[r] = i0 + r < n ? slot[i0 + r] : -1;
  }
  float w[kPullPer];
  int32_t row[kPullPer];
#pragma unroll
  for (int r = 0; r < kPullPer; ++r) {  // all slot loads in flight together
    w[r] = sl[r] >= 0 ? t.sl[sl[r]].w : 0.f;
    row[r] = (sl[r] >= 0 && t.vstride > 0) ? t.sl[sl[r]].vrow : -1;
  }
  uint32_t f[1] = {0u}, ex[1], tot[1];
#pragma unroll
  for (int r = 0; r < kPullPer; ++r) {
    if (l1_shrk && w[r] == 0.f) row[r] = -1;
    f[0] += row[r] >= 0 ? 1u : 0u;
  }
  lb_block_scan<1>(lb, tile, f, ex, tot, shs);
  int32_t vp[kPullPer];
  uint32_t run = ex[0];
#pragma unroll
  for (int r = 0; r < kPullPer; ++r) {
    vp[r] = row[r] >= 0 ? (int32_t)run : -1;
    if (i0 + r < n) {
      hdr[i0 + r] = make_float2(w[r], __int_as_float(vp[r]));
      vpos[i0 + r] = run;
    }
    run += row[r] >= 0 ? 1u : 0u;
  }
  if (tile == ntiles - 1 && threadIdx.x == 0) vpos[n] = tot[0];
  if (t.vstride == 0) return;
#pragma unroll
  for (int r = 0; r < kPullPer; ++r) {
    for_each_row_job<G>(row[r] >= 0, [&](int src, int gl) {
      const int sl2 = src >= 0 ? src : lane;
      const int32_t jr = __shfl(row[r], sl2, 64), jp = __shfl(vp[r], sl2, 64);
      if (src >= 0) {
        const float* V = t.V + (int64_t)jr * t.vstride;
        float* o = vc + (int64_t)jp * t.vstride;
        for (int c = gl * 4; c < t.vstride; c += 4 * G)
          *reinterpret_cast<float4*>(o + c) = *reinterpret_cast<const float4*>(V + c);
      }
    });
  }
}

// One-launch minibatch open on a single shard: find-or-insert every key,
// (data pass 0) add its feature count and lazily allocate + initialise its
// embedding row, then the variable-length pull (look-back scan of the V
// flags, header, compact rows). Replaces kv_find -> difacto_push_cnt ->
// difacto_pull: the three passes re-visited the same 32-byte slot of every
// key. Keys must be distinct (one worker's minibatch).
template <int G>
__global__ __launch_bounds__(kThreads) void k_difacto_open_pull(
    KVTable t, const uint64_t* __restrict__ keys, int64_t n, const int32_t* __restrict__ cnt,
    DifactoHP hp, int insert, Lookback lb, int ntiles, int32_t* __restrict__ slot_out,
    float2* hdr, int64_t* vpos, float* vc) {
  __shared__ uint32_t shs[16];
  __shared__ int sht;
  const int tile = lb_tile(lb, ntiles, &sht);
  const int lane = threadIdx.x & 63;
  const int64_t i0 = (int64_t)tile * kPullTile + threadIdx.x * kPullPer;
  const uint64_t mask = (uint64_t)t.cap - 1;
  uint64_t k[kPullPer];
  int32_t sl[kPullPer];
  uint64_t h[kPullPer], prev[kPullPer];
#pragma unroll
  for (int r = 0; r < kPullPer; ++r) k[r] = i0 + r < n ? keys[i0 + r] : kEmptyKey;
#pragma unroll
  for (int r = 0; r < kPullPer; ++r) {  // all home-slot probes in flight together
    h[r] = mix64(k[r]) & mask;
    prev[r] = k[r] != kEmptyKey ? ld_relaxed(&t.sl[h[r]].key) : 0;
  }
  int created = 0, failed = 0;
#pragma unroll
  for (int r = 0; r < kPullPer; ++r) {
    sl[r] = -1;
    if (k[r] == kEmptyKey) continue;
    bool cr = false;
    sl[r] = probe_slot(t.sl, mask, k[r], h[r], prev[r], insert, &cr);
    created += cr ? 1 : 0;
    if (insert && sl[r] < 0) ++failed;
    if (i0 + r < n) slot_out[i0 + r] = sl[r];
  }
  float w[kPullPer];
  int32_t row[kPullPer];
  bool fresh[kPullPer];
#pragma unroll
  for (int r = 0; r < kPullPer; ++r) {
    w[r] = 0.f;
    row[r] = -1;
    fresh[r] = false;
    if (sl[r] < 0) continue;
    KVSlot& e = t.sl[sl[r]];
    w[r] = e.w;
    row[r] = t.vstride > 0 ? e.vrow : -1;
    if (cnt) {
      const uint32_t c = e.cnt + (uint32_t)cnt[i0 + r];
      e.cnt = c;
      fresh[r] = t.vstride > 0 && c > hp.threshold && row[r] < 0 &&
                 (!hp.l1_shrk || w[r] != 0.f);
    }
  }
  long long newv = 0;
  if (cnt && t.vstride > 0) {
#pragma unroll
    for (int r = 0; r < kPullPer; ++r) {
      const int32_t nr = wave_alloc_rows(t, fresh[r]);
      fresh[r] = nr >= 0;
      if (nr >= 0) {
        t.sl[sl[r]].vrow = nr;
        row[r] = nr;
        newv += t.dim;
      }
    }
  }
  uint32_t f[1] = {0u}, ex[1], tot[1];
#pragma unroll
  for (int r = 0; r < kPullPer; ++r) {
    if (hp.l1_shrk && w[r] == 0.f) row[r] = -1;  // (a fresh row has w != 0)
    f[0] += row[r] >= 0 ? 1u : 0u;
  }
  // direct (vc == null): the header points at the table's own V rows; only
  // the count of pulled rows is scanned (vpos[n])
  const bool direct = vc == nullptr;
  lb_block_scan<1>(lb, tile, f, ex, tot, shs);
  int32_t vp[kPullPer];
  uint32_t run = ex[0];
#pragma unroll
  for (int r = 0; r < kPullPer; ++r) {
    vp[r] = row[r] >= 0 ? (int32_t)run : -1;
    if (i0 + r < n) {
      hdr[i0 + r] = make_float2(w[r], __int_as_float(direct ? row[r] : vp[r]));
      if (!direct) vpos[i0 + r] = run;
    }
    run += row[r] >= 0 ? 1u : 0u;
  }
  if (tile == ntiles - 1 && threadIdx.x == 0) vpos[n] = tot[0];
  // event counters: inserts / failed inserts / new embedding weights
  const long long ci = wave_sum_ll(created), cf = wave_sum_ll(failed), cv = wave_sum_ll(newv);
  if (lane == 0) {
    if (ci) atomicAdd(stat_ptr(t.stats, 4), (unsigned long long)ci);
    if (cf) atomicAdd(stat_ptr(t.stats, 2), (unsigned long long)cf);
    if (cv) atomicAdd(stat_ptr(t.stats, 1), (unsigned long long)cv);
  }
  if (t.vstride == 0) return;
  // row jobs: a fresh row is initialised into the table AND written to its
  // pull position from the same registers; an existing row is copied.
  if (t.vstride == 4 * G) {
    // Batched: the wave's jobs (up to kPullPer x 64) are listed in LDS and
    // every G-lane group issues kRowBatch row loads before its stores, so the
    // wave waits ~jobs / (64/G * kRowBatch) memory round trips instead of one
    // per 64/G jobs (the load -> store chain of each job serialised them).
    constexpr int NG = 64 / G;
    __shared__ int4 jobs[kThreads / 64][kPullPer * 64];
    int4* jl = jobs[threadIdx.x >> 6];
    int nj = 0;
#pragma unroll
    for (int r = 0; r < kPullPer; ++r) {
      const bool has = row[r] >= 0 && (!direct || fresh[r]);  // direct: initialise only
      const uint64_t m = __ballot(has);
      if (has)
        jl[nj + __popcll(m & ((1ull << lane) - 1ull))] =
            make_int4(row[r], vp[r] | (fresh[r] ? (int)0x80000000 : 0), (int)(uint32_t)k[r],
                      (int)(uint32_t)(k[r] >> 32));
      nj += __popcll(m);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int grp = lane / G, gl = lane & (G - 1), c = gl * 4;
    for (int j0 = 0; j0 < nj; j0 += NG * kRowBatch) {
      float4 v[kRowBatch];
#pragma unroll
      for (int b = 0; b < kRowBatch; ++b) {
        const int jj = j0 + b * NG + grp;
        v[b] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (jj < nj) {
          const int4 d = jl[jj];
          if (d.y >= 0) v[b] = *reinterpret_cast<const float4*>(t.V + (int64_t)d.x * t.vstride + c);
        }
      }
#pragma unroll
      for (int b = 0; b < kRowBatch; ++b) {
        const int jj = j0 + b * NG + grp;
        if (jj >= nj) continue;
        const int4 d = jl[jj];
        const int jp = d.y & 0x7fffffff;
        if (d.y < 0) {  // fresh
          const uint64_t jk = (uint64_t)(uint32_t)d.z | ((uint64_t)(uint32_t)d.w << 32);
          v[b] = v_init4(hp, jk, c, t.dim);
          *reinterpret_cast<float4*>(t.V + (int64_t)d.x * t.vstride + c) = v[b];
          *reinterpret_cast<float4*>(t.VG + (int64_t)d.x * t.vstride + c) =
              make_float4(0.f, 0.f, 0.f, 0.f);
        }
        if (!direct) *reinterpret_cast<float4*>(vc + (int64_t)jp * t.vstride + c) = v[b];
      }
    }
    return;
  }
#pragma unroll
  for (int r = 0; r < kPullPer; ++r) {
    for_each_row_job<G>(row[r] >= 0 && (!direct || fresh[r]), [&](int src, int gl) {
      const int s2 = src >= 0 ? src : lane;
      const int32_t jr = __shfl(row[r], s2, 64), jp = __shfl(vp[r], s2, 64);
      const int jf = __shfl((int)fresh[r], s2, 64);
      const uint64_t jk = __shfl(k[r], s2, 64);
      if (src < 0) return;
      float* V = t.V + (int64_t)jr * t.vstride;
      float* o = vc + (int64_t)jp * t.vstride;
      if (jf) {
        float* VG = t.VG + (int64_t)jr * t.vstride;
        for (int c = gl * 4; c < t.vstride; c += 4 * G) {
          const float4 v = v_init4(hp, jk, c, t.dim);
          *reinterpret_cast<float4*>(V + c) = v;
          *reinterpret_cast<float4*>(VG + c) = make_float4(0.f, 0.f, 0.f, 0.f);
          if (!direct) *reinterpret_cast<float4*>(o + c) = v;
        }
      } else {
        for (int c = gl * 4; c < t.vstride; c += 4 * G)
          *reinterpret_cast<float4*>(o + c) = *reinterpret_cast<const float4*>(V + c);
      }
    });
  }
}

// worker side of a multi-shard pull, fused: flag -> scan -> renumber
__global__ __launch_bounds__(kThreads) void k_vidx_renumber(float2* hdr, int64_t n, Lookback lb,
                                                            int ntiles, int64_t* count) {
  __shared__ uint32_t shs[16];
  __shared__ int sht;
  const int tile = lb_tile(lb, ntiles, &sht);
  const int64_t i = (int64_t)tile * kThreads + threadIdx.x;
  const bool has = i < n && __float_as_int(hdr[i].y) >= 0;
  uint32_t f[1] = {has ? 1u : 0u}, ex[1], tot[1];
  lb_block_scan<1>(lb, tile, f, ex, tot, shs);
  if (has) hdr[i].y = __int_as_float((int32_t)ex[0]);
  if (tile == ntiles - 1 && threadIdx.x == 0) *count = tot[0];
}

__global__ __launch_bounds__(kThreads) void k_vidx_flag(const float2* hdr, int64_t n,
                                                        int32_t* flag) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i < n) flag[i] = __float_as_int(hdr[i].y) >= 0 ? 1 : 0;
}

__global__ __launch_bounds__(kThreads) void k_vidx_set(float2* hdr, int64_t n,
                                                       const int32_t* flag, const int64_t* pos) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i < n && flag[i]) hdr[i].y = __int_as_float((int32_t)pos[i]);
}

template <int G>
__global__ __launch_bounds__(kThreads) void k_difacto_push(KVTable t, const int32_t* slot,
                                                           const float2* __restrict__ hdr,
                                                           const float* __restrict__ gw,
                                                           const float* __restrict__ gvc,
                                                           int64_t n, DifactoHP hp) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  float oldw = 0.f, neww = 0.f;
  bool want = false;
  int32_t s = -1, row = -1, gvid = -1;
  if (i < n) {
    s = slot[i];
    if (s >= 0) {
      if (t.vstride > 0) gvid = __float_as_int(hdr[i].y);
      // FTRL on w (reference UpdateW, learn/difacto/async_sgd.h:262-286)
      const float w = t.sl[s].w;
      const float g = gw[i] + hp.l2 * w;
      const float cg = t.sl[s].sq;
      const float cg_new = sqrtf(cg * cg + g * g);
      t.sl[s].sq = cg_new;
      const float z = t.sl[s].z - (g - (cg_new - cg) / hp.alpha * w);
      t.sl[s].z = z;
      float nw;
      if (z <= hp.l1 && z >= -hp.l1) {
        nw = 0.f;
      } else {
        const float eta = (hp.beta + cg_new) / hp.alpha;
        nw = (z > 0 ? z - hp.l1 : z + hp.l1) / eta;
      }
      t.sl[s].w = nw;
      oldw = w;
      neww = nw;
      if (t.vstride > 0) {
        row = t.sl[s].vrow;
        if (w == 0.f && nw != 0.f) want = t.sl[s].cnt > hp.threshold && row < 0;
      }
    }
  }
  count_nnz_delta(oldw, neww, t.stats);
  if (t.vstride == 0) return;
  // job kinds: 1 = initialise a freshly allocated row, 2 = AdaGrad step
  const int32_t nrow = wave_alloc_rows(t, want);
  int kind = 0;
  if (nrow >= 0) {
    t.sl[s].vrow = nrow;
    row = nrow;
    kind = 1;
  } else if (gvid >= 0 && row >= 0) {
    kind = 2;
  }
  long long newv = kind == 1 ? t.dim : 0;
  if (t.vstride == 4 * G) {
    // Batched as in k_difacto_open_pull: jobs listed in LDS, kPushBatch jobs'
    // loads (V, VG, gV rows) in flight per G-lane group before the updates
    constexpr int NG = 64 / G;
    __shared__ int4 jobs[kThreads / 64][64];
    int4* jl = jobs[threadIdx.x >> 6];
    const uint64_t m = __ballot(kind != 0);
    if (kind != 0) jl[__popcll(m & ((1ull << lane) - 1ull))] = make_int4(row, gvid, kind, s);
    const int nj = __popcll(m);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int grp = lane / G, gl = lane & (G - 1), c = gl * 4;
    for (int j0 = 0; j0 < nj; j0 += NG * kPushBatch) {
      float4 v[kPushBatch], cg[kPushBatch], g[kPushBatch];
      uint64_t kk[kPushBatch];
#pragma unroll
      for (int b = 0; b < kPushBatch; ++b) {
        const int jj = j0 + b * NG + grp;
        kk[b] = 0;
        if (jj >= nj) continue;
        const int4 d = jl[jj];
        if (d.z == 2) {
          v[b] = *reinterpret_cast<const float4*>(t.V + (int64_t)d.x * t.vstride + c);
          cg[b] = *reinterpret_cast<const float4*>(t.VG + (int64_t)d.x * t.vstride + c);
          g[b] = *reinterpret_cast<const float4*>(gvc + (int64_t)d.y * t.vstride + c);
        } else {
          kk[b] = t.sl[d.w].key;
        }
      }
#pragma unroll
      for (int b = 0; b < kPushBatch; ++b) {
        const int jj = j0 + b * NG + grp;
        if (jj >= nj) continue;
        const int4 d = jl[jj];
        float* V = t.V + (int64_t)d.x * t.vstride + c;
        float* VG = t.VG + (int64_t)d.x * t.vstride + c;
        if (d.z == 1) {
          *reinterpret_cast<float4*>(V) = v_init4(hp, kk[b], c, t.dim);
          *reinterpret_cast<float4*>(VG) = make_float4(0.f, 0.f, 0.f, 0.f);
          continue;
        }
        // AdaGrad on V (reference UpdateV, learn/difacto/async_sgd.h:289-296)
        float* pv = &v[b].x;
        float* pc = &cg[b].x;
        const float* pg = &g[b].x;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float gg = pg[e] + hp.v_l2 * pv[e];
          pc[e] = sqrtf(pc[e] * pc[e] + gg * gg);
          pv[e] -= hp.v_alpha / (pc[e] + hp.v_beta) * gg;
        }
        *reinterpret_cast<float4*>(V) = v[b];
        *reinterpret_cast<float4*>(VG) = cg[b];
      }
    }
    newv = wave_sum_ll(newv);
    if (lane == 0 && newv) atomicAdd(stat_ptr(t.stats, 1), (unsigned long long)newv);
    return;
  }
  for_each_row_job<G>(kind != 0, [&](int src, int gl) {
    const int sl = src >= 0 ? src : lane;
    const int32_t js = __shfl(s, sl, 64), jr = __shfl(row, sl, 64);
    const int jk = __shfl(kind, sl, 64), jv = __shfl(gvid, sl, 64);
    if (src < 0) return;
    if (jk == 1) {
      init_v_row(t, t.sl[js].key, jr, gl, G, hp);
      return;
    }
    // AdaGrad on V (reference UpdateV, learn/difacto/async_sgd.h:289-296)
    float* V = t.V + (int64_t)jr * t.vstride;
    float* VG = t.VG + (int64_t)jr * t.vstride;
    const float* gv = gvc + (int64_t)jv * t.vstride;
    for (int c = gl * 4; c < t.vstride; c += 4 * G) {
      float4 v = *reinterpret_cast<float4*>(V + c);
      float4 cg = *reinterpret_cast<float4*>(VG + c);
      const float4 g = *reinterpret_cast<const float4*>(gv + c);
      float* pv = &v.x;
      float* pc = &cg.x;
      const float* pg = &g.x;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float gg = pg[e] + hp.v_l2 * pv[e];
        pc[e] = sqrtf(pc[e] * pc[e] + gg * gg);
        pv[e] -= hp.v_alpha / (pc[e] + hp.v_beta) * gg;
      }
      *reinterpret_cast<float4*>(V + c) = v;
      *reinterpret_cast<float4*>(VG + c) = cg;
    }
  });
  newv = wave_sum_ll(newv);
  if (lane == 0 && newv) atomicAdd(stat_ptr(t.stats, 1), (unsigned long long)newv);
}

__global__ __launch_bounds__(kThreads) void k_gather_rows(const float* in, const int32_t* idx,
                                                          int64_t n, int width, float* out) {
  // width in floats; vectorised when width % 4 == 0
  const int64_t tid = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (width % 4 == 0) {
    const int q = width / 4;
    const int64_t r = tid / q, c = tid % q;
    if (r >= n) return;
    reinterpret_cast<float4*>(out + r * width)[c] =
        reinterpret_cast<const float4*>(in + (int64_t)idx[r] * width)[c];
  } else {
    const int64_t r = tid / width, c = tid % width;
    if (r >= n) return;
    out[r * width + c] = in[(int64_t)idx[r] * width + c];
  }
}

}  // namespace

void kv_find(const KVTable& t, const uint64_t* keys, int64_t n, int insert, int32_t* slot,
             hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_kv_find, dim3(grid_for(n, kThreads)), dim3(kThreads), 0, s, keys, n,
                     t.sl, t.cap, insert, slot, t.stats);
}

void kv_occupied(const KVTable& t, int32_t* out_slots, int64_t* out_n, hipStream_t s) {
  hipLaunchKernelGGL(k_kv_occupied, dim3(grid_for(t.cap, kThreads)), dim3(kThreads), 0, s,
                     t.sl, t.cap, out_slots, out_n);
}

void linear_pull(const KVTable& t, const int32_t* slot, int64_t n, float* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_linear_pull, dim3(grid_for(n, kThreads)), dim3(kThreads), 0, s, t.sl,
                     slot, n, out);
}

void linear_push(const KVTable& t, const int32_t* slot, const float* grad, int64_t n,
                 LinearHP hp, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_linear_push, dim3(grid_for(n, kThreads)), dim3(kThreads), 0, s, t, slot,
                     grad, n, hp);
}

void difacto_push_cnt(const KVTable& t, const int32_t* slot, const float* cnt,
                      const int32_t* cnti, int64_t n, DifactoHP hp, hipStream_t s) {
  if (n <= 0) return;
  const int G = lanes_per_key(t.vstride);
  const dim3 grid(grid_for(n, kThreads)), block(kThreads);  // lane per key
  WH_DISPATCH_G(G, k_difacto_push_cnt, grid, block, 0, s, t, slot, cnt, cnti, n, hp);
}

void difacto_pull_hdr(const KVTable& t, const int32_t* slot, int64_t n, int l1_shrk, float* hdr,
                      int32_t* vflag, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_difacto_pull_hdr, dim3(grid_for(n, kThreads)), dim3(kThreads), 0, s, t,
                     slot, n, l1_shrk, reinterpret_cast<float2*>(hdr), vflag);
}

void difacto_pull_rows(const KVTable& t, const int32_t* slot, int64_t n, const int32_t* vflag,
                       const int64_t* vpos, float* hdr, float* vc, hipStream_t s) {
  if (n <= 0 || t.vstride == 0) return;
  const int G = lanes_per_key(t.vstride);
  const dim3 grid(grid_for(n, kThreads)), block(kThreads);  // lane per key
  WH_DISPATCH_G(G, k_difacto_pull_rows, grid, block, 0, s, t, slot, n, vflag, vpos,
                reinterpret_cast<float2*>(hdr), vc);
}

void difacto_push(const KVTable& t, const int32_t* slot, const float* hdr, const float* gw,
                  const float* gvc, int64_t n, DifactoHP hp, hipStream_t s) {
  if (n <= 0) return;
  const int G = lanes_per_key(t.vstride);
  const dim3 grid(grid_for(n, kThreads)), block(kThreads);  // lane per key
  WH_DISPATCH_G(G, k_difacto_push, grid, block, 0, s, t, slot,
                reinterpret_cast<const float2*>(hdr), gw, gvc, n, hp);
}

void vidx_renumber(float* hdr, int64_t n, int32_t* flag_tmp, int64_t* pos_tmp, int64_t* scan_tmp,
                   hipStream_t s) {
  if (n <= 0) return;
  float2* h = reinterpret_cast<float2*>(hdr);
  hipLaunchKernelGGL(k_vidx_flag, dim3(grid_for(n, kThreads)), dim3(kThreads), 0, s, h, n,
                     flag_tmp);
  scan_i32(flag_tmp, pos_tmp, n, scan_tmp, s);
  hipLaunchKernelGGL(k_vidx_set, dim3(grid_for(n, kThreads)), dim3(kThreads), 0, s, h, n,
                     flag_tmp, pos_tmp);
}

void gather_rows(const float* in, const int32_t* idx, int64_t n, int width, float* out,
                 hipStream_t s) {
  if (n <= 0) return;
  const int64_t work = (width % 4 == 0) ? n * (width / 4) : n * width;
  hipLaunchKernelGGL(k_gather_rows, dim3((unsigned)((work + kThreads - 1) / kThreads)),
                     dim3(kThreads), 0, s, in, idx, n, width, out);
}

}  // namespace wh

namespace wh {

bool difacto_pull_fused(const KVTable& t, const int32_t* slot, int64_t n, int l1_shrk,
                        const Lookback& lb, float* hdr, int64_t* vpos, float* vc, hipStream_t s) {
  const int64_t ntiles = (n + kPullTile - 1) / kPullTile;
  if (n <= 0 || ntiles > kLbMaxTiles) return false;
  const int G = lanes_per_key(t.vstride);
  const dim3 grid((unsigned)ntiles), block(kThreads);
  WH_DISPATCH_G(G, k_difacto_pull, grid, block, 0, s, t, slot, n, l1_shrk, lb, (int)ntiles,
                reinterpret_cast<float2*>(hdr), vpos, vc);
  return true;
}

bool vidx_renumber_fused(float* hdr, int64_t n, const Lookback& lb, int64_t* count,
                         hipStream_t s) {
  const int64_t ntiles = (n + kThreads - 1) / kThreads;
  if (n <= 0 || ntiles > kLbMaxTiles) return false;
  hipLaunchKernelGGL(k_vidx_renumber, dim3((unsigned)ntiles), dim3(kThreads), 0, s,
                     reinterpret_cast<float2*>(hdr), n, lb, (int)ntiles, count);
  return true;
}

}  // namespace wh

namespace wh {

bool difacto_open_pull(const KVTable& t, const uint64_t* keys, int64_t n, const int32_t* cnt,
                       DifactoHP hp, int insert, const Lookback& lb, int32_t* slot, float* hdr,
                       int64_t* vpos, float* vc, hipStream_t s) {
  const int64_t ntiles = (n + kPullTile - 1) / kPullTile;
  if (n <= 0 || ntiles > kLbMaxTiles) return false;
  const int G = lanes_per_key(t.vstride);
  const dim3 grid((unsigned)ntiles), block(kThreads);
  WH_DISPATCH_G(G, k_difacto_open_pull, grid, block, 0, s, t, keys, n, cnt, hp, insert, lb,
                (int)ntiles, slot, reinterpret_cast<float2*>(hdr), vpos, vc);
  return true;
}

}  // namespace wh

// ------------------------------------------------------------ growth / health
namespace wh {
namespace {

using namespace kvd;

// Re-insert every occupied slot of `old` into the (larger, empty) table
// `nt`; remap[old slot] = new slot (or -1 for an empty old slot), so the
// slot ids held by in-flight minibatch sessions can be translated. Slots are
// copied whole (w, FTRL/AdaGrad state, count, V row, chain tag); the V slab
// is untouched.
__global__ __launch_bounds__(kThreads) void k_kv_rehash(const KVSlot* __restrict__ old,
                                                        int64_t oldcap, KVSlot* nt, int64_t newcap,
                                                        int32_t* remap, int64_t* stats) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  bool failed = false;
  if (i < oldcap) {
    const KVSlot e = old[i];
    int32_t ns = -1;
    if (e.key != kEmptyKey) {
      const uint64_t mask = (uint64_t)newcap - 1;
      const uint64_t h = mix64(e.key) & mask;
      bool created = false;
      ns = probe_slot(nt, mask, e.key, h, ld_relaxed(&nt[h].key), 1, &created);
      if (ns >= 0) {
        // the key word is already published by the CAS; copy the rest
        nt[ns].w = e.w;
        nt[ns].z = e.z;
        nt[ns].sq = e.sq;
        nt[ns].cnt = e.cnt;
        nt[ns].vrow = e.vrow;
        nt[ns].tag = e.tag;
      } else {
        failed = true;
      }
    }
    remap[i] = ns;
  }
  const uint64_t bf = __ballot(failed);
  if ((threadIdx.x & 63) == 0 && bf) atomicAdd(stat_ptr(stats, 2), (unsigned long long)__popcll(bf));
}

// out[0..3] = {keys in the table, failed inserts, V-slab overflows, V rows used}
__global__ __launch_bounds__(64) void k_kv_summary(const int64_t* stats, const int32_t* vnext,
                                                   int64_t* out) {
  const int lane = threadIdx.x;
  long long a = 0, b = 0, c = 0;
  for (int s = lane; s < kStatShards; s += 64) {
    a += stats[s * kStatStride + 4];
    b += stats[s * kStatStride + 2];
    c += stats[s * kStatStride + 3];
  }
  a = wave_sum_ll(a);
  b = wave_sum_ll(b);
  c = wave_sum_ll(c);
  if (lane == 0) {
    out[0] = a;
    out[1] = b;
    out[2] = c;
    out[3] = vnext ? (int64_t)*vnext : 0;
  }
}

}  // namespace

void kv_rehash(const KVSlot* old, int64_t oldcap, KVSlot* nt, int64_t newcap, int32_t* remap,
               int64_t* stats, hipStream_t s) {
  if (oldcap <= 0) return;
  hipLaunchKernelGGL(k_kv_rehash, dim3(grid_for(oldcap, kThreads)), dim3(kThreads), 0, s, old,
                     oldcap, nt, newcap, remap, stats);
}

void kv_summary(const KVTable& t, int64_t* out, hipStream_t s) {
  hipLaunchKernelGGL(k_kv_summary, dim3(1), dim3(64), 0, s, t.stats, t.vnext, out);
}

}  // namespace wh
