// Single-pass device-wide exclusive scan by decoupled look-back, as a
// building block that kernels embed: a tile computes its items, publishes its
// aggregate, learns its exclusive prefix from its predecessors' published
// values, and then runs its own epilogue in the SAME launch. This replaces
// the reduce -> scan-partials -> rescan triple (3 dependent launches of ~5 us
// each at minibatch sizes) and lets the producer / consumer of a scan fuse
// around it (pull header + row copy, backward chunk planning).
//
// Cross-workgroup visibility on gfx950 (8 XCDs, private non-coherent L2s):
// every published word is an 8-byte granule {tag, value} written by ONE
// agent-scope atomic store and read by agent-scope atomic loads (the
// "data is the flag" form: no fences, no separate flag word). The tag is
// (epoch << 2 | status), status 1 = aggregate, 2 = inclusive prefix. The
// epoch is a per-call host counter, so granules left by earlier scans never
// need clearing. Tiles are taken in order from a ticket counter (a tile
// only ever waits for tiles that were handed out before it, which are
// resident or done); the tile that takes the last ticket resets it.
// A spin that exceeds its bound sets *err and gives up (wrong result, no hang).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "wh_kernels.h"  // struct Lookback, kLbMaxTiles, kLbChannels

namespace wh {

__device__ __forceinline__ unsigned long long lb_load(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Arrival ticket in two levels: blocks count in at kArriveGroups counters
// (bid % groups, one 64-byte line each), the last of each group at the final
// counter; true in the one block (of nb) that arrives last, which may then
// read every block's drained partials. Same-address atomics serialise at
// ~11 ns each, so ONE counter cost ~3.5 us at 313 blocks and ~14 us at 1250
// once every block finishes at about the same time (a short kernel).
// ticket: kArriveWords zeroed words, left zeroed. Called by one thread per
// block, after its partials were stored and drained (s_waitcnt vmcnt(0)).
constexpr int kArriveGroups = 16;
constexpr int kArriveStride = 16;  // words: one cache line per group counter
constexpr int kArriveWords = (kArriveGroups + 1) * kArriveStride;
__device__ __forceinline__ bool arrive_last(unsigned int* ticket, unsigned bid, unsigned nb) {
  const unsigned ng = nb < (unsigned)kArriveGroups ? nb : (unsigned)kArriveGroups;
  const unsigned g = bid % ng, gsize = (nb - g + ng - 1) / ng;
  unsigned int* gc = ticket + g * kArriveStride;
  if (atomicAdd(gc, 1u) != gsize - 1) return false;
  __hip_atomic_store(gc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned int* fc = ticket + kArriveGroups * kArriveStride;
  if (atomicAdd(fc, 1u) != ng - 1) return false;
  __hip_atomic_store(fc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

// Block-wide: the tile index of this block (ticket order). `sh` is one
// shared int. Must be called by every thread of the block.
__device__ __forceinline__ int lb_tile(const Lookback& lb, int ntiles, int* sh) {
  if (threadIdx.x == 0) {
    const unsigned t = atomicAdd(lb.ticket, 1u);
    if ((int)t == ntiles - 1)
      __hip_atomic_store(lb.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *sh = (int)t;
  }
  __syncthreads();
  return *sh;
}

__device__ __forceinline__ uint32_t lb_wave_sum(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Wave-level (call from ONE full wave): exclusive prefix of `agg` over all
// tiles before `tile` in channel `ch`; publishes this tile's inclusive value.
// Each look-back step reads a window of 256 predecessors (4 granules per
// lane, all loads in flight together): every step is one memory round trip
// (~1-2 us for write-through data another XCD just published), so the
// window, not the tile count, bounds the latency.
__device__ __forceinline__ uint32_t lb_exclusive(const Lookback& lb, int ch, int tile,
                                                 uint32_t agg) {
  constexpr int kW = 4;  // granules per lane per step
  const int lane = threadIdx.x & 63;
  unsigned long long* g = lb.gran + (size_t)ch * kLbMaxTiles;
  const unsigned long long tag_a = (unsigned long long)((lb.epoch << 2) | 1u) << 32;
  const unsigned long long tag_i = (unsigned long long)((lb.epoch << 2) | 2u) << 32;
  const unsigned long long hi = 0xffffffff00000000ull;
  if (tile == 0) {
    if (lane == 0) lb_store(g, tag_i | agg);
    return 0;
  }
  if (lane == 0) lb_store(g + tile, tag_a | agg);
  uint32_t run = 0;
  int base = tile - 1;
  while (true) {
    // lane l, slot j covers tile base - (j * 64 + l): slot-major, so slot 0
    // holds the 64 nearest predecessors
    unsigned long long v[kW];
#pragma unroll
    for (int j = 0; j < kW; ++j) {
      const int t = base - (j * 64 + lane);
      v[j] = t >= 0 ? lb_load(g + t) : tag_i;  // before tile 0: an inclusive zero
    }
    unsigned spins = 0;
    while (true) {
      bool ready = true;
#pragma unroll
      for (int j = 0; j < kW; ++j) {
        const unsigned long long tg = v[j] & hi;
        ready &= tg == tag_a || tg == tag_i;
      }
      if (__all(ready)) break;
      if (++spins > (1u << 22)) {
        if (lane == 0) atomicOr(lb.err, 1u);
#pragma unroll
        for (int j = 0; j < kW; ++j) v[j] = tag_i;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
#pragma unroll
      for (int j = 0; j < kW; ++j) {
        const unsigned long long tg = v[j] & hi;
        const int t = base - (j * 64 + lane);
        if (tg != tag_a && tg != tag_i && t >= 0) v[j] = lb_load(g + t);
      }
    }
    // nearest inclusive predecessor (slot-major order = distance order)
    bool done = false;
#pragma unroll
    for (int j = 0; j < kW; ++j) {
      if (done) break;
      const uint64_t inc = __ballot((v[j] & hi) == tag_i);
      const int first = inc ? __ffsll((unsigned long long)inc) - 1 : 63;
      run += lb_wave_sum(lane <= first ? (uint32_t)v[j] : 0u);
      done = inc != 0;
    }
    if (done) break;
    base -= 64 * kW;
  }
  if (lane == 0) lb_store(g + tile, tag_i | (uint32_t)(run + agg));
  return run;
}

// Block-wide exclusive scan of one uint32 per thread for NV channels.
// Returns each thread's exclusive prefix WITHIN the whole scan (block
// prefix from the look-back included) and writes the grand totals (valid
// only in the last tile) to total[]. `sh` needs 16 + 2*NV uint32 of LDS.
template <int NV>
__device__ __forceinline__ void lb_block_scan(const Lookback& lb, int tile, const uint32_t (&v)[NV],
                                              uint32_t (&excl)[NV], uint32_t (&total)[NV],
                                              uint32_t* sh) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  uint32_t inc[NV];
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    uint32_t x = v[c];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    inc[c] = x;
    if (lane == 63) sh[c * 4 + wid] = x;
  }
  __syncthreads();
  uint32_t wbase[NV], btot[NV];
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    wbase[c] = 0;
    btot[c] = 0;
    for (int i = 0; i < nw; ++i) {
      const uint32_t s = sh[c * 4 + i];
      if (i < wid) wbase[c] += s;
      btot[c] += s;
    }
  }
  if (wid == 0) {
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const uint32_t p = lb_exclusive(lb, c, tile, btot[c]);
      if (lane == 0) sh[8 + c] = p;
    }
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const uint32_t p = sh[8 + c];
    excl[c] = p + wbase[c] + inc[c] - v[c];
    total[c] = p + btot[c];
  }
}

}  // namespace wh
