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
#include "wh_kernels.h"

namespace wh {
namespace {

constexpr int kThreads = 256;
constexpr int kChunk = 32;  // occurrences per backward work item

struct LossOut {
  float objv, dual;
};

__device__ __forceinline__ float softplus(float x) {  // log(1 + exp(x)), stable
  return x > 0.f ? x + log1pf(__expf(-x)) : log1pf(__expf(x));
}

__device__ __forceinline__ LossOut eval_loss(int loss, float label, float py) {
  LossOut o;
  if (loss == 1) {  // square: 0.5 (p - y)^2
    const float d = py - label;
    o.objv = 0.5f * d * d;
    o.dual = d;
  } else if (loss == 4) {  // squared hinge: max(0, 1 - y p)^2
    const float y = label > 0.f ? 1.f : -1.f;
    const float t = fmaxf(1.f - y * py, 0.f);
    o.objv = t * t;
    o.dual = -2.f * y * t;
  } else {  // logit
    const float y = label > 0.f ? 1.f : -1.f;
    o.objv = softplus(-y * py);
    o.dual = -y / (1.f + __expf(y * py));
  }
  return o;
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
                                                     float* __restrict__ xv, double* met) {
  // G lanes own one row. Per round the group loads G of the row's non-zeros
  // cooperatively (coalesced local ids, G independent header gathers), then
  // walks the ones that carry an embedding four at a time, every lane
  // gathering its float4 slice of each V row (four 16-byte loads in flight).
  __shared__ double sh[kThreads / 64];
  const int lane = threadIdx.x & 63, gl = lane & (G - 1), gbase = lane - gl;
  const int64_t row = ((int64_t)blockIdx.x * kThreads + threadIdx.x) / G;
  const uint64_t gmask = G == 64 ? ~0ull : (((1ull << G) - 1ull) << gbase);
  double m_objv = 0, m_objw = 0, m_corr = 0, m_n = 0;
  const bool live = row < nrows;
  float wl = 0.f;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f), q = s;
  int64_t b = 0, e = 0;
  if (live) {
    b = off[row];
    e = off[row + 1];
  }
  for (int64_t base = b; base < e; base += G) {
    const int64_t j = base + gl;
    const bool valid = j < e;
    int vid = -1;
    float x = 0.f;
    float2 h = make_float2(0.f, 0.f);
    if (valid) {
      const int k = lid[j];
      x = val ? val[j] : 1.f;
      h = hdr[k];
      vid = __float_as_int(h.y);
    }
    wl += x * h.x;
    uint64_t mg = __ballot(valid && vid >= 0) & gmask;
    while (mg) {
      int t[4];
      float keep[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (mg) {
          t[u] = __ffsll((unsigned long long)mg) - 1;
          mg &= mg - 1;
          keep[u] = 1.f;
        } else {
          t[u] = t[0];
          keep[u] = 0.f;
        }
      }
      float4 v[4];
      float xs[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int vu = __shfl(vid, t[u], 64);
        xs[u] = __shfl(x, t[u], 64) * keep[u];
        v[u] = reinterpret_cast<const float4*>(vc + (int64_t)vu * vstride)[gl];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float xu = xs[u], xx = xu * xu;
        s.x += xu * v[u].x; s.y += xu * v[u].y; s.z += xu * v[u].z; s.w += xu * v[u].w;
        q.x += xx * v[u].x * v[u].x; q.y += xx * v[u].y * v[u].y;
        q.z += xx * v[u].z * v[u].z; q.w += xx * v[u].w * v[u].w;
      }
    }
  }
  const float wsum = group_sum<G>(wl);
  float part = (s.x * s.x - q.x) + (s.y * s.y - q.y) + (s.z * s.z - q.z) + (s.w * s.w - q.w);
  part = group_sum<G>(part);
  if (live) {
    reinterpret_cast<float4*>(xv + row * vstride)[gl] = s;
    if (gl == 0) {
      const float p = wsum + 0.5f * part;
      const float y = label[row];
      const LossOut o = eval_loss(loss, y, p);
      const LossOut ow = eval_loss(loss, y, wsum);
      py_out[row] = p;
      dual_out[row] = o.dual;
      m_objv = o.objv;
      m_objw = ow.objv;
      m_corr = ((y > 0.f && p > 0.f) || (y <= 0.f && p <= 0.f)) ? 1.0 : 0.0;
      m_n = 1.0;
    }
  }
  double r;
  r = block_sum_d(m_objv, sh); if (threadIdx.x == 0) atomicAdd(met + 0, r); __syncthreads();
  r = block_sum_d(m_objw, sh); if (threadIdx.x == 0) atomicAdd(met + 1, r); __syncthreads();
  r = block_sum_d(m_corr, sh); if (threadIdx.x == 0) atomicAdd(met + 2, r); __syncthreads();
  r = block_sum_d(m_n, sh); if (threadIdx.x == 0) atomicAdd(met + 3, r);
}

// linear model: G lanes stride over one row's non-zeros
template <int G>
__global__ __launch_bounds__(kThreads) void k_lin_fwd(int64_t nrows, const int64_t* __restrict__ off,
                                                      const int32_t* __restrict__ lid,
                                                      const float* __restrict__ val,
                                                      const float* __restrict__ w,
                                                      const float* __restrict__ label, int loss,
                                                      float* __restrict__ py_out,
                                                      float* __restrict__ dual_out, double* met) {
  __shared__ double sh[kThreads / 64];
  const int lane = threadIdx.x & 63, gl = lane & (G - 1);
  const int64_t row = ((int64_t)blockIdx.x * kThreads + threadIdx.x) / G;
  double m_objv = 0, m_corr = 0, m_n = 0;
  float acc = 0.f;
  if (row < nrows) {
    const int64_t b = off[row], e = off[row + 1];
    for (int64_t j = b + gl; j < e; j += G) acc += (val ? val[j] : 1.f) * w[lid[j]];
  }
  acc = group_sum<G>(acc);
  if (row < nrows && gl == 0) {
    const float y = label[row];
    const LossOut o = eval_loss(loss, y, acc);
    py_out[row] = acc;
    dual_out[row] = o.dual;
    m_objv = o.objv;
    m_corr = ((y > 0.f && acc > 0.f) || (y <= 0.f && acc <= 0.f)) ? 1.0 : 0.0;
    m_n = 1.0;
  }
  double r;
  r = block_sum_d(m_objv, sh); if (threadIdx.x == 0) { atomicAdd(met + 0, r); atomicAdd(met + 1, r); }
  __syncthreads();
  r = block_sum_d(m_corr, sh); if (threadIdx.x == 0) atomicAdd(met + 2, r); __syncthreads();
  r = block_sum_d(m_n, sh); if (threadIdx.x == 0) atomicAdd(met + 3, r);
}

// ---------------------------------------------------------------- backward
__global__ void k_chunk_count(int64_t nuniq, const int64_t* csc_off, int64_t* chunk_cnt) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < nuniq) {
    const int64_t c = csc_off[k + 1] - csc_off[k];
    chunk_cnt[k] = c > 0 ? (c + kChunk - 1) / kChunk : 0;
  }
}

// writes the chunk table; zeroes the gradients of multi-chunk keys (they
// are accumulated with atomics). Lane per key for the common single-chunk
// key; a multi-chunk (hot) key is expanded by the whole wave, 64 chunks per
// round, so the hottest key does not serialise on one lane.
__global__ __launch_bounds__(kThreads) void k_chunk_fill(int64_t nuniq,
                                                         const int64_t* __restrict__ csc_off,
                                                         const int64_t* __restrict__ chunk_off,
                                                         const float2* __restrict__ hdr,
                                                         int vstride, int32_t* chunk_key,
                                                         int32_t* chunk_beg, float* gw,
                                                         float* gvc) {
  const int lane = threadIdx.x & 63;
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t c0 = 0, nc = 0;
  int32_t b0 = 0;
  if (k < nuniq) {
    c0 = chunk_off[k];
    nc = chunk_off[k + 1] - c0;
    b0 = (int32_t)csc_off[k];
    if (nc == 1) {
      chunk_key[c0] = (int32_t)k;
      chunk_beg[c0] = b0;
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
    for (int64_t c = lane; c < jnc; c += 64) {
      chunk_key[jc0 + c] = jk;
      chunk_beg[jc0 + c] = jb0 + (int32_t)(c * kChunk);
    }
    if (lane == 0) gw[jk] = 0.f;
    if (vstride > 0) {
      const int vid = __float_as_int(hdr[jk].y);
      if (vid >= 0)
        for (int d = lane * 4; d < vstride; d += 256)
          *reinterpret_cast<float4*>(gvc + (int64_t)vid * vstride + d) =
              make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
}

template <int G>
__global__ __launch_bounds__(kThreads) void k_fm_bwd(const int64_t* __restrict__ nchunk_p, const int32_t* __restrict__ chunk_key,
                                                     const int32_t* __restrict__ chunk_beg,
                                                     const int64_t* __restrict__ csc_off,
                                                     const int32_t* __restrict__ csc_row,
                                                     const float* __restrict__ csc_val,
                                                     const float* __restrict__ dual,
                                                     const float* __restrict__ xv,
                                                     const float2* __restrict__ hdr,
                                                     const float* __restrict__ vc, int vstride,
                                                     float* __restrict__ gw_out,
                                                     float* __restrict__ gvc) {
  // ONE LANE PER CHUNK computes the scalar sums (gw, xxp) of its <= kChunk
  // occurrences; the wave then runs the embedding-gradient jobs of the
  // chunks whose key has V, G lanes per job (float4 slice of each xv row).
  const int lane = threadIdx.x & 63;
  const int64_t nch = *nchunk_p;
  const int64_t c = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  const bool live = c < nch;
  int k = 0, b = 0, e = 0, vid = -1;
  bool multi = false;
  float gw = 0.f, xxp = 0.f;
  if (live) {
    k = chunk_key[c];
    const int kb = (int)csc_off[k], ke = (int)csc_off[k + 1];
    b = chunk_beg[c];
    e = b + kChunk < ke ? b + kChunk : ke;
    multi = (ke - kb) > kChunk;
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
      for (int u = 0; u < 4; ++u) {
        const float d = dual[i[u]] * x[u];
        gw += d;
        xxp += d * x[u];
      }
    }
    for (; p < e; ++p) {
      const float x = csc_val ? csc_val[p] : 1.f;
      const float d = dual[csc_row[p]] * x;
      gw += d;
      xxp += d * x;
    }
    vid = __float_as_int(hdr[k].y);
    if (!multi) gw_out[k] = gw;
    else atomicAdd(gw_out + k, gw);
  }
  for_each_row_job<G>(live && vid >= 0, [&](int src, int gl) {
    const int sl = src >= 0 ? src : lane;
    const int jv = __shfl(vid, sl, 64), jb = __shfl(b, sl, 64), je = __shfl(e, sl, 64);
    const float jx = __shfl(xxp, sl, 64);
    const int jm = __shfl((int)multi, sl, 64);
    if (src < 0) return;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int p = jb;
    for (; p + 3 < je; p += 4) {
      float d[4];
      float4 a[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = csc_row[p + u];
        d[u] = dual[i] * (csc_val ? csc_val[p + u] : 1.f);
        a[u] = reinterpret_cast<const float4*>(xv + (int64_t)i * vstride)[gl];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        acc.x += d[u] * a[u].x; acc.y += d[u] * a[u].y;
        acc.z += d[u] * a[u].z; acc.w += d[u] * a[u].w;
      }
    }
    for (; p < je; ++p) {
      const int i = csc_row[p];
      const float d = dual[i] * (csc_val ? csc_val[p] : 1.f);
      const float4 a = reinterpret_cast<const float4*>(xv + (int64_t)i * vstride)[gl];
      acc.x += d * a.x; acc.y += d * a.y; acc.z += d * a.z; acc.w += d * a.w;
    }
    const float4 v = reinterpret_cast<const float4*>(vc + (int64_t)jv * vstride)[gl];
    acc.x -= jx * v.x; acc.y -= jx * v.y; acc.z -= jx * v.z; acc.w -= jx * v.w;
    float* gv = gvc + (int64_t)jv * vstride + gl * 4;
    if (!jm) {
      *reinterpret_cast<float4*>(gv) = acc;
    } else {
      atomicAdd(gv + 0, acc.x); atomicAdd(gv + 1, acc.y);
      atomicAdd(gv + 2, acc.z); atomicAdd(gv + 3, acc.w);
    }
  });
}

__global__ __launch_bounds__(kThreads) void k_lin_bwd(const int64_t* __restrict__ nchunk_p, const int32_t* __restrict__ chunk_key,
                                                      const int32_t* __restrict__ chunk_beg,
                                                      const int64_t* __restrict__ csc_off,
                                                      const int32_t* __restrict__ csc_row,
                                                      const float* __restrict__ csc_val,
                                                      const float* __restrict__ dual,
                                                      float* __restrict__ grad) {
  const int64_t c = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (c >= *nchunk_p) return;
  const int k = chunk_key[c];
  const int64_t kb = csc_off[k], ke = csc_off[k + 1];
  const int64_t b = chunk_beg[c];
  const int64_t e = b + kChunk < ke ? b + kChunk : ke;
  float gw = 0.f;
  for (int64_t p = b; p < e; ++p) gw += dual[csc_row[p]] * (csc_val ? csc_val[p] : 1.f);
  if ((ke - kb) > kChunk) atomicAdd(grad + k, gw);
  else grad[k] = gw;
}

// gradient clipping / dropout / normalisation on the m embedding-gradient
// rows (reference learn/difacto/loss.h:131-155); m is a device count
__global__ __launch_bounds__(kThreads) void k_grad_post(const int64_t* __restrict__ m_p,
                                                        float* gvc, int vstride, int dim,
                                                        float clip, float dropout, uint64_t seed,
                                                        double* sumsq) {
  __shared__ double sh[kThreads / 64];
  const int64_t t = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  const int64_t r = t / vstride;
  const int d = (int)(t % vstride);
  const int64_t m = *m_p;
  double ss = 0;
  if (r < m && d < dim) {
    float v = gvc[t];
    if (clip > 0.f) v = fminf(fmaxf(v, -clip), clip);
    if (dropout > 0.f && uhash01(seed, (uint64_t)r, (uint64_t)d) > 1.f - dropout) v = 0.f;
    gvc[t] = v;
    ss = (double)v * v;
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

void fm_forward(int64_t nrows, const int64_t* offset, const int32_t* lid, const float* val,
                const float* w_or_hdr, const float* vc, int vstride, const float* label, int loss,
                float* py, float* dual, float* xv, double* met, hipStream_t s) {
  if (nrows <= 0) return;
  if (vstride == 0) {
    constexpr int G = 8;
    hipLaunchKernelGGL(k_lin_fwd<G>, dim3(grid_for(nrows * G, kThreads)), dim3(kThreads), 0, s,
                       nrows, offset, lid, val, w_or_hdr, label, loss, py, dual, met);
    return;
  }
  const int G = vstride / 4;  // vstride <= 256 enforced by the binding
  const float2* hdr = reinterpret_cast<const float2*>(w_or_hdr);
  const dim3 grid(grid_for(nrows * G, kThreads)), block(kThreads);
  WH_DISPATCH_G(G, k_fm_fwd, grid, block, 0, s, nrows, offset, lid, val, hdr, vc, vstride, label,
                loss, py, dual, xv, met);
}

int64_t fm_bwd_chunks_bound(int64_t nuniq, int64_t nnz) { return nuniq + nnz / kChunk + 1; }

void fm_backward(int64_t nuniq, const int64_t* csc_off, const int32_t* csc_row,
                 const float* csc_val, const float* dual, const float* xv, const float* hdr_f,
                 const float* vc, int vstride, float* gw, float* gvc, int32_t* chunk_key,
                 int32_t* chunk_beg, int64_t* chunk_cnt, int64_t* chunk_off, int64_t* scan_tmp,
                 int64_t chunk_cap, hipStream_t s) {
  if (nuniq <= 0) return;
  const float2* hdr = reinterpret_cast<const float2*>(hdr_f);
  hipLaunchKernelGGL(k_chunk_count, dim3(grid_for(nuniq, kThreads)), dim3(kThreads), 0, s, nuniq,
                     csc_off, chunk_cnt);
  scan_i64(chunk_cnt, chunk_off, nuniq, scan_tmp, s);
  hipLaunchKernelGGL(k_chunk_fill, dim3(grid_for(nuniq, kThreads)), dim3(kThreads), 0, s, nuniq,
                     csc_off, chunk_off, hdr, vstride, chunk_key, chunk_beg, gw, gvc);
  // the chunk count is data dependent (device value chunk_off[nuniq]); launch
  // over the host-side bound and let surplus work items exit, so the whole
  // step stays free of host synchronisation.
  const int64_t* nchunk_p = chunk_off + nuniq;
  if (vstride == 0) {
    hipLaunchKernelGGL(k_lin_bwd, dim3(grid_for(chunk_cap, kThreads)), dim3(kThreads), 0, s,
                       nchunk_p, chunk_key, chunk_beg, csc_off, csc_row, csc_val, dual, gw);
    return;
  }
  const int G = vstride / 4;
  const dim3 grid(grid_for(chunk_cap, kThreads)), block(kThreads);  // lane per chunk
  WH_DISPATCH_G(G, k_fm_bwd, grid, block, 0, s, nchunk_p, chunk_key, chunk_beg, csc_off,
                csc_row, csc_val, dual, xv, hdr, vc, vstride, gw, gvc);
}

void fm_grad_post(const int64_t* m, int64_t m_cap, float* gvc, int vstride, int dim, float clip,
                  float dropout, uint64_t seed, double* sumsq, hipStream_t s) {
  if (m_cap <= 0 || vstride == 0) return;
  hipLaunchKernelGGL(k_grad_post, dim3(grid_for(m_cap * vstride, kThreads)), dim3(kThreads), 0,
                     s, m, gvc, vstride, dim, clip, dropout, seed, sumsq);
}

void fm_grad_scale(const int64_t* m, int64_t m_cap, float* gvc, int vstride, int dim,
                   const double* sumsq, hipStream_t s) {
  if (m_cap <= 0 || vstride == 0) return;
  hipLaunchKernelGGL(k_grad_scale, dim3(grid_for(m_cap * vstride, kThreads)), dim3(kThreads), 0,
                     s, m, gvc, vstride, dim, sumsq);
}

}  // namespace wh
