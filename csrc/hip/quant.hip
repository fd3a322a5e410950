// Fixed-point payload compression for the key-value exchange: the ps-lite
// FIXING_FLOAT filter of the reference (learn/difacto/async_sgd.h:429-446,
// config `fixed_bytes` = 1, 2 or 3, "convert floating-points into fixed-point
// integers with n bytes ... randomly round"), re-designed for the xGMI
// all-to-all of embedding rows.
//
// A row of W floats travels as ONE packed record of 4 + n*W bytes (rounded up
// to 4): a float32 scale = max|x| / (2^(8n-1) - 1), then W signed n-byte
// integers q = floor(x / scale + u), u ~ U[0,1) from a counter-based hash of
// (seed, row, column), so E[q * scale] = x (unbiased stochastic rounding, as
// ps-lite's random rounding). One wave per row, a float4 slice per lane for
// W = 64.
#include "wh_common.h"
#include "wh_kernels.h"

namespace wh {
namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ float qmax(int nb) {
  return nb == 1 ? 127.f : nb == 2 ? 32767.f : 8388607.f;
}

__global__ __launch_bounds__(kThreads) void k_quant_rows(const float* __restrict__ x, int64_t rows,
                                                         int w, int nb, uint64_t seed,
                                                         int64_t rec_bytes,
                                                         uint8_t* __restrict__ out) {
  const int64_t r = ((int64_t)blockIdx.x * kThreads + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const float* xr = x + r * w;
  float m = 0.f;
  for (int c = lane; c < w; c += 64) m = fmaxf(m, fabsf(xr[c]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  const float scale = m > 0.f ? m / qmax(nb) : 1.f;
  const float inv = 1.f / scale;
  uint8_t* o = out + r * rec_bytes;
  if (lane == 0) *reinterpret_cast<float*>(o) = scale;
  uint8_t* q = o + 4;
  const float lim = qmax(nb);
  for (int c = lane; c < w; c += 64) {
    const float u = uhash01(seed, (uint64_t)r, (uint64_t)c);
    float v = floorf(xr[c] * inv + u);
    v = fminf(fmaxf(v, -lim), lim);
    const int32_t iv = (int32_t)v;
    for (int b = 0; b < nb; ++b) q[c * nb + b] = (uint8_t)((uint32_t)iv >> (8 * b));
  }
}

__global__ __launch_bounds__(kThreads) void k_dequant_rows(const uint8_t* __restrict__ in,
                                                           int64_t rows, int w, int nb,
                                                           int64_t rec_bytes,
                                                           float* __restrict__ x) {
  const int64_t r = ((int64_t)blockIdx.x * kThreads + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const uint8_t* o = in + r * rec_bytes;
  const float scale = *reinterpret_cast<const float*>(o);
  const uint8_t* q = o + 4;
  for (int c = lane; c < w; c += 64) {
    uint32_t u = 0;
    for (int b = 0; b < nb; ++b) u |= (uint32_t)q[c * nb + b] << (8 * b);
    const int sh = 32 - 8 * nb;
    const int32_t iv = (int32_t)(u << sh) >> sh;  // sign-extend
    x[r * w + c] = (float)iv * scale;
  }
}

// feature counts -> uint8, saturating (the reference's TRUNCATE_FLOAT(1) on
// the count push)
__global__ __launch_bounds__(kThreads) void k_trunc_u8(const int32_t* __restrict__ c, int64_t n,
                                                       uint8_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i < n) {
    const int32_t v = c[i];
    out[i] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
  }
}

// ---- region payload filter of the multi-shard exchange (kv/psx.py) -------
// The C2 / C3 buffers are per-peer regions. Peer p's region (desc row p of
// int64 {sf, a, vf, nf, sq, ha}) holds, in the float layout, `a` floats sent
// bit-exact at [sf, sf + a) (the 8-byte {w, vidx} headers / gradients) and
// `nf` floats quantised at [sf + vf, sf + vf + nf) (the embedding rows, or
// the linear model's per-key gradients) ; on the wire it is ha rows of R
// bytes carrying the raw floats, then ceil(nf / W) records {scale, W nb-byte
// ints} of R = quant_record_bytes(W, nb) bytes each, from wire row sq. The
// last record of a region may be partial (its missing floats read as 0). One
// wave per wire row; the peer of a row by binary search over the sq column.
constexpr int kQDesc = 6;

__device__ __forceinline__ int qregion_peer(const int64_t* __restrict__ desc, int P, int64_t row) {
  int lo = 0, hi = P - 1;  // last p with sq_p <= row
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (desc[(int64_t)mid * kQDesc + 4] <= row) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__global__ __launch_bounds__(kThreads) void k_qregion_pack(const float* __restrict__ x,
                                                           const int64_t* __restrict__ desc, int P,
                                                           int64_t rows, int W, int nb,
                                                           int64_t R, uint64_t seed,
                                                           uint8_t* __restrict__ out) {
  const int64_t r = ((int64_t)blockIdx.x * kThreads + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const int p = qregion_peer(desc, P, r);
  const int64_t* d = desc + (int64_t)p * kQDesc;
  const int64_t sf = d[0], a = d[1], vf = d[2], nf = d[3], j = r - d[4], ha = d[5];
  uint8_t* o = out + r * R;
  if (j < ha) {  // raw words of the exact part
    const int64_t wpr = R / 4, w0 = j * wpr;
    for (int64_t c = lane; c < wpr; c += 64) {
      const int64_t f = w0 + c;
      reinterpret_cast<float*>(o)[c] = f < a ? x[sf + f] : 0.f;
    }
    return;
  }
  const int64_t q0 = (j - ha) * W;  // first quantised float of this record
  const float* xr = x + sf + vf + q0;
  const int64_t nw = nf - q0 < W ? nf - q0 : W;
  float m = 0.f;
  for (int c = lane; c < nw; c += 64) m = fmaxf(m, fabsf(xr[c]));
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) m = fmaxf(m, __shfl_xor(m, s, 64));
  const float lim = qmax(nb);
  const float scale = m > 0.f ? m / lim : 1.f;
  const float inv = 1.f / scale;
  if (lane == 0) *reinterpret_cast<float*>(o) = scale;
  uint8_t* q = o + 4;
  for (int c = lane; c < W; c += 64) {
    int32_t iv = 0;
    if (c < nw) {
      const float u = uhash01(seed, (uint64_t)r, (uint64_t)c);
      iv = (int32_t)fminf(fmaxf(floorf(xr[c] * inv + u), -lim), lim);
    }
    for (int b = 0; b < nb; ++b) q[c * nb + b] = (uint8_t)((uint32_t)iv >> (8 * b));
  }
}

__global__ __launch_bounds__(kThreads) void k_qregion_unpack(const uint8_t* __restrict__ in,
                                                             const int64_t* __restrict__ desc,
                                                             int P, int64_t rows, int W, int nb,
                                                             int64_t R, float* __restrict__ x) {
  const int64_t r = ((int64_t)blockIdx.x * kThreads + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const int p = qregion_peer(desc, P, r);
  const int64_t* d = desc + (int64_t)p * kQDesc;
  const int64_t sf = d[0], a = d[1], vf = d[2], nf = d[3], j = r - d[4], ha = d[5];
  const uint8_t* o = in + r * R;
  if (j < ha) {
    const int64_t wpr = R / 4, w0 = j * wpr;
    for (int64_t c = lane; c < wpr; c += 64) {
      const int64_t f = w0 + c;
      if (f < a) x[sf + f] = reinterpret_cast<const float*>(o)[c];
    }
    return;
  }
  const int64_t q0 = (j - ha) * W;
  const int64_t nw = nf - q0 < W ? nf - q0 : W;
  const float scale = *reinterpret_cast<const float*>(o);
  const uint8_t* q = o + 4;
  float* xr = x + sf + vf + q0;
  for (int c = lane; c < nw; c += 64) {
    uint32_t u = 0;
    for (int b = 0; b < nb; ++b) u |= (uint32_t)q[c * nb + b] << (8 * b);
    const int sh = 32 - 8 * nb;
    xr[c] = (float)((int32_t)(u << sh) >> sh) * scale;
  }
}

}  // namespace

int64_t quant_record_bytes(int w, int nb) { return (4 + (int64_t)w * nb + 3) / 4 * 4; }

void qregion_pack(const float* x, const int64_t* desc, int P, int64_t rows, int W, int nb,
                  uint64_t seed, uint8_t* out, hipStream_t s) {
  if (rows <= 0) return;
  hipLaunchKernelGGL(k_qregion_pack, dim3(grid_for(rows * 64, kThreads)), dim3(kThreads), 0, s, x,
                     desc, P, rows, W, nb, quant_record_bytes(W, nb), seed, out);
}

void qregion_unpack(const uint8_t* in, const int64_t* desc, int P, int64_t rows, int W, int nb,
                    float* x, hipStream_t s) {
  if (rows <= 0) return;
  hipLaunchKernelGGL(k_qregion_unpack, dim3(grid_for(rows * 64, kThreads)), dim3(kThreads), 0, s,
                     in, desc, P, rows, W, nb, quant_record_bytes(W, nb), x);
}

void quant_rows(const float* x, int64_t rows, int w, int nb, uint64_t seed, uint8_t* out,
                hipStream_t s) {
  if (rows <= 0) return;
  hipLaunchKernelGGL(k_quant_rows, dim3(grid_for(rows * 64, kThreads)), dim3(kThreads), 0, s, x,
                     rows, w, nb, seed, quant_record_bytes(w, nb), out);
}

void dequant_rows(const uint8_t* in, int64_t rows, int w, int nb, float* x, hipStream_t s) {
  if (rows <= 0) return;
  hipLaunchKernelGGL(k_dequant_rows, dim3(grid_for(rows * 64, kThreads)), dim3(kThreads), 0, s,
                     in, rows, w, nb, quant_record_bytes(w, nb), x);
}

void trunc_u8(const int32_t* c, int64_t n, uint8_t* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_trunc_u8, dim3(grid_for(n, kThreads)), dim3(kThreads), 0, s, c, n, out);
}

}  // namespace wh
