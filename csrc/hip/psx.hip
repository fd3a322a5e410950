// Multi-shard parameter-server exchange: owner- and worker-side kernels of
// the lean DiFacto step over P > 1 shards (P ranks over RCCL, or P virtual
// shards on one GPU for the loopback rehearsal).
//
// Reference flow (learn/difacto/async_sgd.h:372-424): ZPush(feature counts)
// -> ZVPull(w, V) -> ZVPush(gw, gV), each a ps-lite request per server.
// Here a minibatch is FOUR collectives on the wire, none of which the host
// has to wait for inside the step:
//   C0  tiny all-to-all: {key count, table overflow, V rows of the previous
//       step's pull} per peer (rides on localize's count exchange)
//   C1  keys (+ counts in data pass 0) as 12-byte records
//   C2  pull reply: per peer ONE contiguous region of vstride-float rows
//       [H_p header rows | v_p embedding rows]
//   C3  push: the same regions in reverse, [gw | gV rows]
//
// Row-aligned regions. With S_p / HS_p the prefix sums of the per-peer key
// counts n_p and header rows H_p = ceil(2 n_p / vstride), and VS_p the prefix
// of the per-peer embedding-row counts, region p starts at row HS_p + VS_p.
// The owner's open kernel writes the embedding row of key i (segment p) at
// row HS_{p+1} + vpos(i) -- VS_p cancels out -- so rows go straight from the
// table into the wire buffer in the same launch that decides them; only the
// 8-byte headers need VS_p and are packed by a second small kernel. The
// worker consumes the received buffer IN PLACE: its header unpack rewrites
// each key's row id to the row inside that buffer, the FM kernels gather
// from it, and the backward writes gV rows at the same positions, so the
// gradient buffer already has the push layout (pack_gw only adds gw).
//
// Duplicates. Unlike one worker's minibatch, the keys an owner receives from
// different peers overlap (hot features). The open kernel therefore counts
// with atomics and allocates an embedding row with a CAS on the slot's vrow
// (exactly one winner initialises it; any other lane that sees a row created
// in this launch computes the identical initial values from the key hash
// instead of reading half-written memory). It also threads each key's
// duplicates into a forward chain: every lane swaps its (epoch, index) tag
// into the slot's tag word; the lane that finds no tag of this launch is the
// key's head, every other lane links itself behind the lane it displaced.
// The tags are never cleared per minibatch (a stale tag carries an older
// epoch); the host sweeps the table's tags once per 255 minibatches, before
// the 8-bit epoch wraps. The push kernel lets only a head lane update its
// key, over its chain in ascending index = peer-rank order, so each worker's
// push is applied as one sequential update, deterministically (like the
// ps-lite server handling requests one at a time), in ONE launch.
#include "wh_common.h"
#include "wh_kernels.h"
#include "wh_lookback.h"
#include "kv_device.h"

namespace wh {
namespace {

using namespace kvd;

constexpr int kMaxSeg = 256;  // peers (LDS copies of the segment tables)

// chain[i] = index + 1 of the next duplicate of key i (0 = end; zeroed
// before the open, written only by that successor); head[i] = 1 when lane i
// heads its key's chain (written only by lane i)

// segment of item i: largest p with S[p] <= i (S in LDS, P+1 entries)
__device__ __forceinline__ int seg_of(const int64_t* S, int P, int64_t i) {
  int lo = 0, hi = P - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (S[mid] <= i) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ void load_seg(const int64_t* g, int64_t* sh, int P) {
  for (int p = threadIdx.x; p <= P; p += blockDim.x) sh[p] = g[p];
}

// the new {cnt, tag} word of lane `idx` (index idx + 1 in the chain tag)
__device__ __forceinline__ unsigned long long next_ct(unsigned long long cur, uint32_t epoch,
                                                      int64_t idx, uint32_t add, int chains) {
  const uint32_t mine = (epoch << 24) | (uint32_t)(idx + 1);
  const uint32_t nt = chains ? mine : (uint32_t)(cur >> 32);
  return ((unsigned long long)nt << 32) | (uint32_t)((uint32_t)cur + add);
}

// a segment's V-row prefix published by k_ps_open (tagged granule; a spin
// past its bound sets *err like the look-back and yields 0)
__device__ __forceinline__ uint32_t seg_granule(const unsigned long long* g,
                                                unsigned long long tag, unsigned int* err) {
  unsigned long long v = lb_load(g);
  unsigned spins = 0;
  while ((v & 0xffffffff00000000ull) != tag) {
    if (++spins > (1u << 22)) {
      atomicOr(err, 1u);
      return 0;
    }
    __builtin_amdgcn_s_sleep(1);
    v = lb_load(g);
  }
  return (uint32_t)v;
}

// ---------------------------------------------------------------- owner open
// keys: u64 [n] (rec == null) or 12-byte records rec [n x 3] int32 {key lo,
// key hi, count}. Writes slot[n], w_out[n], vpos[n+1], chain[n] (train) and
// the embedding rows into rbuf.
template <int G>
__global__ __launch_bounds__(kThreads) void k_ps_open(
    KVTable t, const uint64_t* __restrict__ keys, const int32_t* __restrict__ rec, int64_t n,
    DifactoHP hp, int insert, int use_cnt, int chains, uint32_t epoch,
    const int32_t* __restrict__ vbase_p, const int64_t* __restrict__ segS,
    const int64_t* __restrict__ segHS, int P, Lookback lb, int ntiles, int32_t* __restrict__ slot_out,
    float* __restrict__ w_out, int64_t* __restrict__ vpos, uint32_t* __restrict__ chain,
    uint8_t* __restrict__ head, float* __restrict__ rbuf, int64_t* __restrict__ vcnt) {
  __shared__ uint32_t shs[16];
  __shared__ int sht;
  __shared__ int64_t sS[kMaxSeg + 1], sHS[kMaxSeg + 1];
  load_seg(segS, sS, P);
  load_seg(segHS, sHS, P);
  const int tile = lb_tile(lb, ntiles, &sht);  // (syncs the block)
  const int lane = threadIdx.x & 63;
  const int64_t i0 = (int64_t)tile * kPullTile + threadIdx.x * kPullPer;
  const uint64_t mask = (uint64_t)t.cap - 1;
  const int32_t vbase = *vbase_p;
  uint64_t k[kPullPer], h[kPullPer], prev[kPullPer];
  int32_t c[kPullPer], sl[kPullPer];
#pragma unroll
  for (int r = 0; r < kPullPer; ++r) {
    const int64_t i = i0 + r;
    k[r] = kEmptyKey;
    c[r] = 0;
    if (i < n) {
      if (rec) {
        const uint32_t lo = (uint32_t)rec[3 * i], hi = (uint32_t)rec[3 * i + 1];
        k[r] = ((uint64_t)hi << 32) | lo;
        c[r] = use_cnt ? rec[3 * i + 2] : 0;
      } else {
        k[r] = keys[i];
      }
    }
  }
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
  bool want[kPullPer];
  // {cnt, tag} in one 64-bit CAS: add the count and swap in this lane's
  // chain tag. The kPullPer keys' slot reads, first CAS attempts and (rare)
  // retries are issued phase by phase, so their memory round trips overlap
  // instead of running key after key.
  const bool ctag = use_cnt || chains;
  unsigned long long cur[kPullPer], seen[kPullPer];
#pragma unroll
  for (int r = 0; r < kPullPer; ++r) {
    w[r] = 0.f;
    row[r] = -1;
    want[r] = false;
    cur[r] = seen[r] = 0ull;
    if (sl[r] < 0) continue;
    KVSlot& e = t.sl[sl[r]];
    w[r] = e.w;
    row[r] = t.vstride > 0 ? ld_relaxed_i32(&e.vrow) : -1;
    if (ctag)
      cur[r] = __hip_atomic_load(reinterpret_cast<unsigned long long*>(&e.cnt), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
  }
  if (ctag) {
#pragma unroll
    for (int r = 0; r < kPullPer; ++r)
      if (sl[r] >= 0)
        seen[r] = atomicCAS(reinterpret_cast<unsigned long long*>(&t.sl[sl[r]].cnt), cur[r],
                            next_ct(cur[r], epoch, i0 + r, use_cnt ? (uint32_t)c[r] : 0u, chains));
#pragma unroll
    for (int r = 0; r < kPullPer; ++r) {
      if (sl[r] < 0) continue;
      unsigned long long* ct = reinterpret_cast<unsigned long long*>(&t.sl[sl[r]].cnt);
      while (seen[r] != cur[r]) {  // another lane of this launch updated the word
        cur[r] = seen[r];
        seen[r] = atomicCAS(ct, cur[r],
                            next_ct(cur[r], epoch, i0 + r, use_cnt ? (uint32_t)c[r] : 0u, chains));
      }
      const uint32_t add = use_cnt ? (uint32_t)c[r] : 0u;
      const uint32_t old = (uint32_t)cur[r], pv = (uint32_t)(cur[r] >> 32);
      // Only the lane whose add crosses the threshold may allocate: with a
      // key's duplicates adding concurrently, exactly one lane crosses (a
      // key that crossed while l1_shrk held w at 0 is allocated by the push
      // that makes w non-zero).
      want[r] = use_cnt && t.vstride > 0 && old <= hp.threshold && old + add > hp.threshold &&
                row[r] < 0 && (!hp.l1_shrk || w[r] != 0.f);
      if (chains) {
        const uint32_t j = (pv & 0xffffffu) - 1;
        const bool linked = (pv >> 24) == epoch && (int64_t)j < n && (int64_t)j != i0 + r;
        if (linked) chain[j] = (uint32_t)(i0 + r + 1);  // behind the lane we displaced
        head[i0 + r] = linked ? 0 : 1;
      }
    }
  }
  // allocation: exactly one CAS winner per key initialises the row
  bool mine_fresh[kPullPer];
  long long newv = 0;
#pragma unroll
  for (int r = 0; r < kPullPer; ++r) {
    mine_fresh[r] = false;
    if (!use_cnt || t.vstride == 0) continue;
    const int32_t nr = wave_alloc_rows(t, want[r]);
    if (nr >= 0) {
      const int32_t o = atomicCAS(&t.sl[sl[r]].vrow, -1, nr);
      if (o == -1) {
        row[r] = nr;
        mine_fresh[r] = true;
        newv += t.dim;
      } else {
        row[r] = o;  // another peer's duplicate won (nr stays unused)
      }
    }
  }
  uint32_t f[1] = {0u}, ex[1], tot[1];
#pragma unroll
  for (int r = 0; r < kPullPer; ++r) {
    if (hp.l1_shrk && w[r] == 0.f) row[r] = -1;
    f[0] += row[r] >= 0 ? 1u : 0u;
  }
  lb_block_scan<1>(lb, tile, f, ex, tot, shs);
  int32_t orow[kPullPer];  // output row in rbuf
  uint32_t run = ex[0];
#pragma unroll
  for (int r = 0; r < kPullPer; ++r) {
    orow[r] = -1;
    if (i0 + r < n) {
      w_out[i0 + r] = w[r];
      vpos[i0 + r] = run;
      if (row[r] >= 0) {
        const int p = seg_of(sS, P, i0 + r);
        orow[r] = (int32_t)(sHS[p + 1] + run);
      }
    }
    run += row[r] >= 0 ? 1u : 0u;
  }
  if (tile == ntiles - 1 && threadIdx.x == 0) vpos[n] = tot[0];
  if (t.vstride > 0) {
    // The headers {w, row inside the peer's V block} of this tile's keys, in
    // this launch (a separate pack kernel after the open cost a launch on
    // the step's critical chain): a header goes to float (HS_p + VS_p) *
    // vstride + 2 (i - S_p), and VS_p = vpos[S_p] is known to the tile
    // holding item S_p once its look-back is done. That tile publishes it as
    // a tagged granule (look-back channel 1, status 3: earlier launches'
    // granules never match); readers wait only on tiles that took their
    // ticket earlier (resident or finished), as the look-back itself does.
    __shared__ uint32_t sv[kPullTile];
    unsigned long long* sg = lb.gran + (size_t)kLbMaxTiles;
    const unsigned long long tag = (unsigned long long)((lb.epoch << 2) | 3u) << 32;
    const int64_t t0 = (int64_t)tile * kPullTile;
    {
      uint32_t rr = ex[0];
#pragma unroll
      for (int r = 0; r < kPullPer; ++r) {
        sv[threadIdx.x * kPullPer + r] = rr;
        rr += row[r] >= 0 ? 1u : 0u;
      }
    }
    __syncthreads();
    for (int p = threadIdx.x; p <= P; p += blockDim.x) {
      const int64_t sp = sS[p];
      if (sp >= t0 && sp < t0 + kPullTile && sp < n)
        lb_store(sg + p, tag | sv[sp - t0]);
      else if (sp >= n && tile == ntiles - 1)
        lb_store(sg + p, tag | tot[0]);
    }
    int cp = -1;
    uint32_t cvs = 0;
#pragma unroll
    for (int r = 0; r < kPullPer; ++r) {
      const int64_t i = i0 + r;
      if (i >= n) break;
      const int p = seg_of(sS, P, i);
      if (p != cp) {
        cp = p;
        cvs = seg_granule(sg + p, tag, lb.err);
      }
      const int32_t j = row[r] >= 0 ? (int32_t)(sv[threadIdx.x * kPullPer + r] - cvs) : -1;
      *reinterpret_cast<float2*>(rbuf + (sHS[p] + cvs) * t.vstride + 2 * (i - sS[p])) =
          make_float2(w[r], __int_as_float(j));
    }
    if (tile == ntiles - 1)
      for (int p = threadIdx.x; p < P; p += blockDim.x)
        vcnt[p] = (int64_t)seg_granule(sg + p + 1, tag, lb.err) -
                  (int64_t)seg_granule(sg + p, tag, lb.err);
  }
  const long long ci = wave_sum_ll(created), cf = wave_sum_ll(failed), cv = wave_sum_ll(newv);
  if (lane == 0) {
    if (ci) atomicAdd(stat_ptr(t.stats, 4), (unsigned long long)ci);
    if (cf) atomicAdd(stat_ptr(t.stats, 2), (unsigned long long)cf);
    if (cv) atomicAdd(stat_ptr(t.stats, 1), (unsigned long long)cv);
  }
  if (t.vstride == 0) return;
  // row jobs: 0 copy from the slab, 1 initialise (CAS winner: table + wire),
  // 2 recompute the initial values (a row another lane created in this launch)
  if (t.vstride == 4 * G) {
    // batched through a per-wave LDS job list, as k_difacto_open_pull
    // (kvstore.hip): kRowBatch slab loads in flight per G-lane group
    constexpr int NG = 64 / G;
    __shared__ int4 jobs[kThreads / 64][kPullPer * 64];
    int4* jl = jobs[threadIdx.x >> 6];
    int nj = 0;
#pragma unroll
    for (int r = 0; r < kPullPer; ++r) {
      const int kind = mine_fresh[r] ? 1 : (row[r] >= vbase ? 2 : 0);
      const bool has = orow[r] >= 0;
      const uint64_t m = __ballot(has);
      if (has)
        jl[nj + __popcll(m & ((1ull << lane) - 1ull))] =
            make_int4(row[r] | (kind << 30), orow[r], (int)(uint32_t)k[r],
                      (int)(uint32_t)(k[r] >> 32));
      nj += __popcll(m);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int grp = lane / G, c = (lane & (G - 1)) * 4;
    for (int j0 = 0; j0 < nj; j0 += NG * kRowBatch) {
      float4 v[kRowBatch];
#pragma unroll
      for (int b = 0; b < kRowBatch; ++b) {
        const int jj = j0 + b * NG + grp;
        v[b] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (jj < nj) {
          const int4 d = jl[jj];
          if ((d.x >> 30) == 0)
            v[b] = *reinterpret_cast<const float4*>(t.V + (int64_t)d.x * t.vstride + c);
        }
      }
#pragma unroll
      for (int b = 0; b < kRowBatch; ++b) {
        const int jj = j0 + b * NG + grp;
        if (jj >= nj) continue;
        const int4 d = jl[jj];
        const int kind = (d.x >> 30) & 3, jr = d.x & 0x3fffffff;
        if (kind != 0) {
          const uint64_t jk = (uint64_t)(uint32_t)d.z | ((uint64_t)(uint32_t)d.w << 32);
          v[b] = v_init4(hp, jk, c, t.dim);
          if (kind == 1) {
            *reinterpret_cast<float4*>(t.V + (int64_t)jr * t.vstride + c) = v[b];
            *reinterpret_cast<float4*>(t.VG + (int64_t)jr * t.vstride + c) =
                make_float4(0.f, 0.f, 0.f, 0.f);
          }
        }
        *reinterpret_cast<float4*>(rbuf + (int64_t)d.y * t.vstride + c) = v[b];
      }
    }
    return;
  }
#pragma unroll
  for (int r = 0; r < kPullPer; ++r) {
    const int kind = mine_fresh[r] ? 1 : (row[r] >= vbase ? 2 : 0);
    for_each_row_job<G>(orow[r] >= 0, [&](int src, int gl) {
      const int s2 = src >= 0 ? src : lane;
      const int32_t jr = __shfl(row[r], s2, 64), jo = __shfl(orow[r], s2, 64);
      const int jk = __shfl(kind, s2, 64);
      const uint64_t jkey = __shfl(k[r], s2, 64);
      if (src < 0) return;
      float* V = t.V + (int64_t)jr * t.vstride;
      float* o = rbuf + (int64_t)jo * t.vstride;
      for (int cc = gl * 4; cc < t.vstride; cc += 4 * G) {
        float4 v;
        if (jk == 0) {
          v = *reinterpret_cast<const float4*>(V + cc);
        } else {
          v = v_init4(hp, jkey, cc, t.dim);
          if (jk == 1) {
            *reinterpret_cast<float4*>(V + cc) = v;
            *reinterpret_cast<float4*>(t.VG + (int64_t)jr * t.vstride + cc) =
                make_float4(0.f, 0.f, 0.f, 0.f);
          }
        }
        *reinterpret_cast<float4*>(o + cc) = v;
      }
    });
  }
}

// header pack (owner, after the open): {w, row index inside the peer's V
// block or -1} at float (HS_p + VS_p) * vstride + 2 (i - S_p), and the
// per-peer V row counts
__global__ __launch_bounds__(kThreads) void k_ps_pack_hdr(
    const float* __restrict__ w_out, const int64_t* __restrict__ vpos, int64_t n, int vstride,
    const int64_t* __restrict__ segS, const int64_t* __restrict__ segHS, int P,
    float* __restrict__ rbuf, int64_t* __restrict__ vcnt) {
  __shared__ int64_t sS[kMaxSeg + 1], sHS[kMaxSeg + 1];
  load_seg(segS, sS, P);
  load_seg(segHS, sHS, P);
  __syncthreads();
  if (blockIdx.x == 0)
    for (int p = threadIdx.x; p < P; p += blockDim.x) vcnt[p] = vpos[sS[p + 1]] - vpos[sS[p]];
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= n) return;
  const int p = seg_of(sS, P, i);
  const int64_t vs0 = vpos[sS[p]];
  const int64_t v = vpos[i];
  const bool has = vpos[i + 1] > v;
  const int32_t j = has ? (int32_t)(v - vs0) : -1;
  *reinterpret_cast<float2*>(rbuf + (sHS[p] + vs0) * vstride + 2 * (i - sS[p])) =
      make_float2(w_out[i], __int_as_float(j));
}

// before an open: zero the chain links and snapshot the V-row bump pointer
// (rows at or above it are created by the coming launch)
__global__ __launch_bounds__(kThreads) void k_ps_prep(uint32_t* __restrict__ chain, int64_t n,
                                                      const int32_t* __restrict__ vnext,
                                                      int32_t* __restrict__ vbase) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i < n) chain[i] = 0u;
  if (i == 0) *vbase = *vnext;
}

// clear every slot's chain tag (once per 255 opens, before the epoch wraps).
// Read-mostly: only the slots the cycle's minibatches touched carry a tag,
// so every tag word is read (four loads in flight per lane) and only the set
// ones are written back; an unconditional 4-byte store into every 32-byte
// slot took 1.7 ms on the linear loopback-8 bench's 134M-slot table.
constexpr int kSweepU = 4;
__global__ __launch_bounds__(kThreads) void k_ps_sweep_tags(KVSlot* sl, int64_t cap) {
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i0 = (int64_t)blockIdx.x * kThreads + threadIdx.x; i0 < cap;
       i0 += kSweepU * stride) {
    uint32_t t[kSweepU];
#pragma unroll
    for (int u = 0; u < kSweepU; ++u) {
      const int64_t i = i0 + u * stride;
      t[u] = i < cap ? sl[i].tag : 0u;
    }
#pragma unroll
    for (int u = 0; u < kSweepU; ++u)
      if (t[u] != 0u) sl[i0 + u * stride].tag = 0u;
  }
}

// worker: 12-byte key records {lo, hi, count} of the C1 exchange
__global__ __launch_bounds__(kThreads) void k_ps_records(const uint64_t* __restrict__ uniq,
                                                         const int32_t* __restrict__ ucnt,
                                                         int64_t U, int32_t* __restrict__ rec) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= U) return;
  const uint64_t k = uniq[i];
  rec[3 * i] = (int32_t)(uint32_t)k;
  rec[3 * i + 1] = (int32_t)(uint32_t)(k >> 32);
  rec[3 * i + 2] = ucnt ? ucnt[i] : 0;
}

// C0: send[4p..] = {keys for p (0 for a peer that owns no shard: p >= S),
// own table-overflow flag, V rows for p, this rank's has-data flag};
// payload = [owner_cnt (S+1) | received 4P (filled by the exchange) | vcnt P]
__global__ __launch_bounds__(256) void k_ps_c0(const int64_t* __restrict__ owner_cnt,
                                               const int64_t* __restrict__ vcnt, int S, int P,
                                               int64_t flag, int64_t* __restrict__ send,
                                               int64_t* __restrict__ payload, int loop) {
  for (int p = threadIdx.x; p <= S; p += blockDim.x) payload[p] = owner_cnt[p];
  for (int p = threadIdx.x; p < P; p += blockDim.x) {
    const int64_t v = vcnt ? vcnt[p] : 0;
    const int64_t m[4] = {p < S ? owner_cnt[p] : 0, owner_cnt[S], v, flag};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      send[4 * p + k] = m[k];
      // loopback identity: what peer p would send this rank is what it sends
      if (loop) payload[S + 1 + 4 * p + k] = m[k];
    }
    payload[S + 1 + 4 * P + p] = v;
  }
}

// ---------------------------------------------------------------- worker side
// hdr[k] = {w, row of key k's embedding inside the received buffer or -1};
// rows_total[0] = rows of the received buffer
__global__ __launch_bounds__(kThreads) void k_ps_unpack(
    const float* __restrict__ rbuf, int64_t U, int vstride, const int64_t* __restrict__ segS,
    const int64_t* __restrict__ segHS, const int64_t* __restrict__ vrecv, int P,
    float2* __restrict__ hdr, int64_t* __restrict__ rows_total) {
  __shared__ int64_t sS[kMaxSeg + 1], sHS[kMaxSeg + 1], sVS[kMaxSeg + 1];
  load_seg(segS, sS, P);
  load_seg(segHS, sHS, P);
  if (threadIdx.x == 0) {  // P is small (peers): a serial prefix is fine
    int64_t a = 0;
    for (int p = 0; p < P; ++p) { sVS[p] = a; a += vrecv[p]; }
    sVS[P] = a;
  }
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0) rows_total[0] = sHS[P] + sVS[P];
  const int64_t k = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (k >= U) return;
  const int q = seg_of(sS, P, k);
  const float2 e =
      *reinterpret_cast<const float2*>(rbuf + (sHS[q] + sVS[q]) * vstride + 2 * (k - sS[q]));
  const int32_t j = __float_as_int(e.y);
  const int32_t vid = j >= 0 ? (int32_t)(sHS[q + 1] + sVS[q] + j) : -1;
  hdr[k] = make_float2(e.x, __int_as_float(vid));
}

// gw[k] into the header rows of its owner's region of the push buffer
__global__ __launch_bounds__(kThreads) void k_ps_pack_gw(
    const float* __restrict__ gw, int64_t U, int vstride, const int64_t* __restrict__ segS,
    const int64_t* __restrict__ segHS, const int64_t* __restrict__ vrecv, int P,
    float* __restrict__ gbuf) {
  __shared__ int64_t sS[kMaxSeg + 1], sHS[kMaxSeg + 1], sVS[kMaxSeg + 1];
  load_seg(segS, sS, P);
  load_seg(segHS, sHS, P);
  if (threadIdx.x == 0) {
    int64_t a = 0;
    for (int p = 0; p < P; ++p) { sVS[p] = a; a += vrecv[p]; }
    sVS[P] = a;
  }
  __syncthreads();
  const int64_t k = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (k >= U) return;
  const int q = seg_of(sS, P, k);
  gbuf[(sHS[q] + sVS[q]) * vstride + (k - sS[q])] = gw[k];
}

// ---------------------------------------------------------------- owner push
// next element of a chain in ascending index order after `last` (the chains
// hold at most one entry per peer, so a selection walk is cheap)
__device__ __forceinline__ int64_t chain_next_after(const uint32_t* chain, int64_t head,
                                                    int64_t last) {
  int64_t best = -1;
  for (int64_t e = head; e >= 0;) {
    if (e > last && (best < 0 || e < best)) best = e;
    const uint32_t nx = chain[e];
    e = nx ? (int64_t)nx - 1 : -1;
  }
  return best;
}

// the next open's prep (PsPrep), folded into a push launch
__device__ __forceinline__ void ps_prep_in(const PsPrep& pr, const int32_t* vnext) {
  if (pr.vbase && blockIdx.x == 0 && threadIdx.x == 0) *pr.vbase = *vnext;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < pr.n;
       i += (int64_t)gridDim.x * blockDim.x)
    pr.chain[i] = 0u;
}

template <int G>
__global__ __launch_bounds__(kThreads) void k_ps_push(
    KVTable t, const int32_t* __restrict__ slot, const int64_t* __restrict__ vpos,
    const uint32_t* __restrict__ chain, const uint8_t* __restrict__ headf, int64_t n,
    const int64_t* __restrict__ segS, const int64_t* __restrict__ segHS, int P,
    const float* __restrict__ gbuf, DifactoHP hp, PsPrep prep) {
  ps_prep_in(prep, t.vnext);  // (before any row of this push is allocated)
  __shared__ int64_t sS[kMaxSeg + 1], sHS[kMaxSeg + 1], sVS[kMaxSeg + 1];
  load_seg(segS, sS, P);
  load_seg(segHS, sHS, P);
  __syncthreads();
  for (int p = threadIdx.x; p <= P; p += blockDim.x) sVS[p] = vpos[sS[p]];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  float w0 = 0.f, w = 0.f;
  int32_t s = -1, row = -1;
  bool head = false, any_v = false, alloc = false, single = true;
  int64_t gvrow = -1;  // singleton: the gradient row of this key
  if (i < n) {
    s = slot[i];
    head = s >= 0 && (!chain || headf[i]);
    single = !chain || chain[i] == 0u;
  }
  if (head) {
    KVSlot& e = t.sl[s];
    w0 = w = e.w;
    float z = e.z, sq = e.sq;
    bool up = false;  // w went 0 -> non-zero at some push of the chain
    if (single) {  // the common case: one peer pushed this key
      const int p = seg_of(sS, P, i);
      const float g = gbuf[(sHS[p] + sVS[p]) * t.vstride + (i - sS[p])];
      w = difacto_ftrl(w, g, sq, z, hp);
      up = w0 == 0.f && w != 0.f;
      const int64_t v0 = vpos[i];
      any_v = vpos[i + 1] > v0;
      gvrow = sHS[p + 1] + v0;
    } else {
      for (int64_t el = chain_next_after(chain, i, -1); el >= 0;
           el = chain_next_after(chain, i, el)) {
        const int p = seg_of(sS, P, el);
        const float g = gbuf[(sHS[p] + sVS[p]) * t.vstride + (el - sS[p])];
        const float nw = difacto_ftrl(w, g, sq, z, hp);
        up |= (w == 0.f && nw != 0.f);
        w = nw;
        any_v |= vpos[el + 1] > vpos[el];
      }
    }
    e.w = w;
    e.z = z;
    e.sq = sq;
    if (t.vstride > 0) {
      row = e.vrow;
      alloc = up && row < 0 && e.cnt > hp.threshold;
    }
  }
  count_nnz_delta(w0, w, t.stats);
  if (t.vstride == 0) return;
  const int32_t nrow = wave_alloc_rows(t, alloc);
  int kind = 0;  // 1 initialise a new row, 2 AdaGrad over the chain's gradients
  if (nrow >= 0) {
    t.sl[s].vrow = nrow;
    row = nrow;
    kind = 1;
  } else if (head && row >= 0 && any_v) {
    kind = 2;
  }
  long long newv = kind == 1 ? t.dim : 0;
  bool rest = kind != 0;
  if (t.vstride == 4 * G) {
    // initialisations and single-peer AdaGrad steps batched through an LDS
    // job list (as k_difacto_push); keys pushed by several peers (chains)
    // take the general loop below
    constexpr int NG = 64 / G;
    __shared__ int4 jobs[kThreads / 64][64];
    int4* jl = jobs[threadIdx.x >> 6];
    const bool bat = kind == 1 || (kind == 2 && single);
    rest = kind != 0 && !bat;
    const uint64_t m = __ballot(bat);
    if (bat) jl[__popcll(m & ((1ull << lane) - 1ull))] = make_int4(row, (int)gvrow, kind, s);
    const int nj = __popcll(m);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int grp = lane / G, c = (lane & (G - 1)) * 4;
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
          g[b] = *reinterpret_cast<const float4*>(gbuf + (int64_t)d.y * t.vstride + c);
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
        adagrad4(v[b], cg[b], g[b], hp);
        *reinterpret_cast<float4*>(V) = v[b];
        *reinterpret_cast<float4*>(VG) = cg[b];
      }
    }
  }
  for_each_row_job<G>(rest, [&](int src, int gl) {
    const int s2 = src >= 0 ? src : lane;
    const int32_t jr = __shfl(row, s2, 64), jk = __shfl(kind, s2, 64);
    const int32_t js = __shfl(s, s2, 64);
    const int64_t ji = __shfl(i, s2, 64);
    const int64_t jg = __shfl(single ? gvrow : -1, s2, 64);
    if (src < 0) return;
    if (jk == 1) {
      init_v_row(t, t.sl[js].key, jr, gl, G, hp);
      return;
    }
    float* V = t.V + (int64_t)jr * t.vstride;
    float* VG = t.VG + (int64_t)jr * t.vstride;
    if (jg >= 0) {  // singleton: one gradient row, known to the key's lane
      const float* gv = gbuf + jg * t.vstride;
      for (int cc = gl * 4; cc < t.vstride; cc += 4 * G) {
        float4 v = *reinterpret_cast<float4*>(V + cc);
        float4 cg = *reinterpret_cast<float4*>(VG + cc);
        adagrad4(v, cg, *reinterpret_cast<const float4*>(gv + cc), hp);
        *reinterpret_cast<float4*>(V + cc) = v;
        *reinterpret_cast<float4*>(VG + cc) = cg;
      }
      return;
    }
    for (int cc = gl * 4; cc < t.vstride; cc += 4 * G) {
      float4 v = *reinterpret_cast<float4*>(V + cc);
      float4 cg = *reinterpret_cast<float4*>(VG + cc);
      for (int64_t el = chain ? chain_next_after(chain, ji, -1) : ji; el >= 0;
           el = chain ? chain_next_after(chain, ji, el) : -1) {
        if (vpos[el + 1] <= vpos[el]) continue;  // that peer pulled no V row
        const int p = seg_of(sS, P, el);
        const float4 g = *reinterpret_cast<const float4*>(
            gbuf + (sHS[p + 1] + vpos[el]) * t.vstride + cc);
        adagrad4(v, cg, g, hp);
      }
      *reinterpret_cast<float4*>(V + cc) = v;
      *reinterpret_cast<float4*>(VG + cc) = cg;
    }
  });
  newv = wave_sum_ll(newv);
  if (lane == 0 && newv) atomicAdd(stat_ptr(t.stats, 1), (unsigned long long)newv);
}

// Linear model (vstride 0): the owner's push. g[i] is the gradient a peer
// pushed for key i of this owner's received list (segments in peer order).
// Only a key's chain head updates it, over the chain in ascending index =
// peer order, so each worker's push lands as one sequential request (the
// ps-lite server handles requests one at a time). SGD's t counts requests:
// segment p of this batch is request t0 + p + 1.
__global__ __launch_bounds__(kThreads) void k_psl_push(
    KVTable t, const int32_t* __restrict__ slot, const uint32_t* __restrict__ chain,
    const uint8_t* __restrict__ headf, int64_t n, const int64_t* __restrict__ segS, int P,
    const float* __restrict__ g, LinearHP hp, double t0, PsPrep prep) {
  ps_prep_in(prep, t.vnext);
  __shared__ int64_t sS[kMaxSeg + 1];
  load_seg(segS, sS, P);
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  float w0 = 0.f, w = 0.f;
  if (i < n) {
    const int32_t s = slot[i];
    const bool head = s >= 0 && (!chain || headf[i]);
    if (head) {
      KVSlot& e = t.sl[s];
      w0 = w = e.w;
      const bool single = !chain || chain[i] == 0u;
      for (int64_t el = single ? i : chain_next_after(chain, i, -1); el >= 0;
           el = single ? -1 : chain_next_after(chain, i, el)) {
        float eta = 0.f;
        if (hp.algo == 1) eta = (float)((hp.beta + sqrt(t0 + seg_of(sS, P, el) + 1.0)) / hp.alpha);
        w = linear_update(e, g[el], hp, eta);
      }
    }
  }
  count_nnz_delta(w0, w, t.stats);
}

}  // namespace

bool ps_push_linear(const KVTable& t, const int32_t* slot, const uint32_t* chain,
                    const uint8_t* head, int64_t n, const int64_t* segS, int P, const float* g,
                    LinearHP hp, double t0, hipStream_t s, PsPrep prep) {
  if (P < 1 || P > kMaxSeg || t.vstride != 0) return false;
  if (n <= 0 && prep.n <= 0 && !prep.vbase) return true;
  hipLaunchKernelGGL(k_psl_push, dim3(grid_for(n > prep.n ? n : prep.n, kThreads)),
                     dim3(kThreads), 0, s, t, slot, chain, head, n, segS, P, g, hp, t0, prep);
  return true;
}

bool ps_open(const KVTable& t, const uint64_t* keys, const int32_t* rec, int64_t n, int use_cnt,
             DifactoHP hp, int insert, int chains, uint32_t epoch, int32_t* vbase,
             const int64_t* segS, const int64_t* segHS, int P, const Lookback& lb, int32_t* slot,
             float* w_out, int64_t* vpos, uint32_t* chain, uint8_t* head, float* rbuf,
             int64_t* vcnt, hipStream_t s, int prepped) {
  const int64_t ntiles = (n + kPullTile - 1) / kPullTile;
  if (P < 1 || P > kMaxSeg || ntiles > kLbMaxTiles || n >= (1 << 24) || epoch < 1 ||
      epoch > 255)
    return false;
  if (!prepped)
    hipLaunchKernelGGL(k_ps_prep, dim3(grid_for(n, kThreads)), dim3(kThreads), 0, s, chain,
                       chains ? n : 0, t.vnext, vbase);
  if (epoch == 1) {  // a new epoch cycle: no tag of the previous cycle may survive
    hipLaunchKernelGGL(k_ps_sweep_tags, dim3(grid_for(t.cap, kThreads, 8192)), dim3(kThreads), 0,
                       s, t.sl, t.cap);
  }
  if (n > 0) {
    const int G = lanes_per_key(t.vstride);
    WH_DISPATCH_G(G, k_ps_open, dim3((unsigned)ntiles), dim3(kThreads), 0, s, t, keys, rec, n, hp,
                  insert, use_cnt, chains, epoch, vbase, segS, segHS, P, lb, (int)ntiles, slot,
                  w_out, vpos, chain, head, rbuf, vcnt);
  } else {
    WH_HIP_CHECK(hipMemsetAsync(vpos, 0, sizeof(int64_t), s));
    // (no keys: only the per-peer V row counts, all zero)
    if (t.vstride > 0)
      hipLaunchKernelGGL(k_ps_pack_hdr, dim3(1), dim3(kThreads), 0, s, w_out, vpos, n,
                         t.vstride, segS, segHS, P, rbuf, vcnt);
  }
  // linear (vstride 0): the reply is w_out itself, one float per key; the
  // headers of the embedding model are written by the open
  return true;
}

bool ps_push(const KVTable& t, const int32_t* slot, const int64_t* vpos, const uint32_t* chain,
             const uint8_t* head, int64_t n, const int64_t* segS, const int64_t* segHS, int P,
             const float* gbuf, DifactoHP hp, hipStream_t s, PsPrep prep) {
  if (P < 1 || P > kMaxSeg || t.vstride == 0) return false;
  if (n <= 0 && prep.n <= 0 && !prep.vbase) return true;
  const int G = lanes_per_key(t.vstride);
  WH_DISPATCH_G(G, k_ps_push, dim3(grid_for(n > prep.n ? n : prep.n, kThreads)), dim3(kThreads),
                0, s, t, slot, vpos, chain, head, n, segS, segHS, P, gbuf, hp, prep);
  return true;
}

void ps_records(const uint64_t* uniq, const int32_t* ucnt, int64_t U, int32_t* rec,
                hipStream_t s) {
  if (U <= 0) return;
  hipLaunchKernelGGL(k_ps_records, dim3(grid_for(U, kThreads)), dim3(kThreads), 0, s, uniq, ucnt,
                     U, rec);
}

bool ps_c0(const int64_t* owner_cnt, const int64_t* vcnt, int S, int P, int64_t flag,
           int64_t* send, int64_t* payload, hipStream_t s, int loop) {
  if (P < 1 || P > 4096 || S < 1 || S > P) return false;
  hipLaunchKernelGGL(k_ps_c0, dim3(1), dim3(256), 0, s, owner_cnt, vcnt, S, P, flag, send,
                     payload, loop);
  return true;
}

bool ps_unpack(const float* rbuf, int64_t U, int vstride, const int64_t* segS,
               const int64_t* segHS, const int64_t* vrecv, int P, float* hdr, int64_t* rows_total,
               hipStream_t s) {
  if (P < 1 || P > kMaxSeg) return false;
  hipLaunchKernelGGL(k_ps_unpack, dim3(grid_for(U, kThreads)), dim3(kThreads), 0, s, rbuf, U,
                     vstride, segS, segHS, vrecv, P, reinterpret_cast<float2*>(hdr), rows_total);
  return true;
}

bool ps_pack_gw(const float* gw, int64_t U, int vstride, const int64_t* segS,
                const int64_t* segHS, const int64_t* vrecv, int P, float* gbuf, hipStream_t s) {
  if (P < 1 || P > kMaxSeg) return false;
  if (U <= 0) return true;
  hipLaunchKernelGGL(k_ps_pack_gw, dim3(grid_for(U, kThreads)), dim3(kThreads), 0, s, gw, U,
                     vstride, segS, segHS, vrecv, P, gbuf);
  return true;
}

}  // namespace wh
