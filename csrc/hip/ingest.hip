// Device-side text ingest (Criteo, libsvm) (K1 in SURVEY §2.5): raw bytes of whole
// lines are copied to the GPU and tokenized there, every field hashed with
// CityHash64 exactly as the host parser does (csrc/host/parsers.cc
// ParseCriteo, reference learn/base/criteo_parser.h:64-86):
//   key = (CityHash64(field bytes) >> 10) | (field index << 54)
// for the 13 integer and 26 categorical fields, empty fields skipped; the
// label is the first field (training data).
//
//   k_nl_count / k_nl_fill : line starts (per 4 KiB tile newline counts ->
//                            scan -> positions), no host pass over the bytes
//   k_criteo_fields        : one wave per line: 64-byte windows are loaded
//                            lane-parallel and tab / newline positions found by
//                            ballot; lane f then hashes field f
//   k_criteo_compact       : the per-line keys packed into the CSR minibatch
//                            (row offsets = scan of the per-line counts)
//   k_libsvm_count / _fill : libsvm lines, one wave per line: token starts by
//                            ballot, the lane at a token start parses it
//                            (index exactly, value strtof-compatible)
// The host only splits the file into whole-line batches (memchr) and copies
// them into pinned memory.
#include "wh_common.h"
#include "wh_kernels.h"

namespace wh {
namespace {

// ---- CityHash64 (v1.1), device port of csrc/host/cityhash.cc -------------
// Bytes are assembled one at a time: fields start at arbitrary offsets.
constexpr uint64_t kC0 = 0xc3a5c85c97cb3127ULL;
constexpr uint64_t kC1 = 0xb492b66fbe98f273ULL;
constexpr uint64_t kC2 = 0x9ae16a3b2f90404fULL;

__device__ __forceinline__ uint64_t dfetch64(const uint8_t* p) {
  uint64_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r |= (uint64_t)p[i] << (8 * i);
  return r;
}
__device__ __forceinline__ uint32_t dfetch32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
__device__ __forceinline__ uint64_t drot(uint64_t v, int s) {
  return s == 0 ? v : ((v >> s) | (v << (64 - s)));
}
__device__ __forceinline__ uint64_t dshiftmix(uint64_t v) { return v ^ (v >> 47); }
__device__ __forceinline__ uint64_t dbswap(uint64_t x) {
  return ((x & 0xffull) << 56) | ((x & 0xff00ull) << 40) | ((x & 0xff0000ull) << 24) |
         ((x & 0xff000000ull) << 8) | ((x >> 8) & 0xff000000ull) | ((x >> 24) & 0xff0000ull) |
         ((x >> 40) & 0xff00ull) | (x >> 56);
}
__device__ __forceinline__ uint64_t dlen16(uint64_t u, uint64_t v, uint64_t mul) {
  uint64_t a = (u ^ v) * mul;
  a ^= (a >> 47);
  uint64_t b = (v ^ a) * mul;
  b ^= (b >> 47);
  return b * mul;
}
__device__ __forceinline__ uint64_t dlen16(uint64_t u, uint64_t v) {
  return dlen16(u, v, 0x9ddfea08eb382d69ULL);
}

__device__ uint64_t dcity_0to16(const uint8_t* s, uint32_t len) {
  if (len >= 8) {
    const uint64_t mul = kC2 + len * 2;
    const uint64_t a = dfetch64(s) + kC2;
    const uint64_t b = dfetch64(s + len - 8);
    const uint64_t c = drot(b, 37) * mul + a;
    const uint64_t d = (drot(a, 25) + b) * mul;
    return dlen16(c, d, mul);
  }
  if (len >= 4) {
    const uint64_t mul = kC2 + len * 2;
    const uint64_t a = dfetch32(s);
    return dlen16(len + (a << 3), dfetch32(s + len - 4), mul);
  }
  if (len > 0) {
    const uint8_t a = s[0], b = s[len >> 1], c = s[len - 1];
    const uint32_t y = (uint32_t)a + ((uint32_t)b << 8);
    const uint32_t z = len + ((uint32_t)c << 2);
    return dshiftmix(y * kC2 ^ z * kC0) * kC2;
  }
  return kC2;
}

__device__ uint64_t dcity_17to32(const uint8_t* s, uint32_t len) {
  const uint64_t mul = kC2 + len * 2;
  const uint64_t a = dfetch64(s) * kC1;
  const uint64_t b = dfetch64(s + 8);
  const uint64_t c = dfetch64(s + len - 8) * mul;
  const uint64_t d = dfetch64(s + len - 16) * kC2;
  return dlen16(drot(a + b, 43) + drot(c, 30) + d, a + drot(b + kC2, 18) + c, mul);
}

__device__ __forceinline__ void dweak32(uint64_t w, uint64_t x, uint64_t y, uint64_t z,
                                        uint64_t a, uint64_t b, uint64_t& o1, uint64_t& o2) {
  a += w;
  b = drot(b + a + z, 21);
  const uint64_t c = a;
  a += x;
  a += y;
  b += drot(a, 44);
  o1 = a + z;
  o2 = b + c;
}
__device__ __forceinline__ void dweak32(const uint8_t* s, uint64_t a, uint64_t b, uint64_t& o1,
                                        uint64_t& o2) {
  dweak32(dfetch64(s), dfetch64(s + 8), dfetch64(s + 16), dfetch64(s + 24), a, b, o1, o2);
}

__device__ uint64_t dcity_33to64(const uint8_t* s, uint32_t len) {
  const uint64_t mul = kC2 + len * 2;
  uint64_t a = dfetch64(s) * kC2;
  uint64_t b = dfetch64(s + 8);
  const uint64_t c = dfetch64(s + len - 24);
  const uint64_t d = dfetch64(s + len - 32);
  const uint64_t e = dfetch64(s + 16) * kC2;
  const uint64_t f = dfetch64(s + 24) * 9;
  const uint64_t g = dfetch64(s + len - 8);
  const uint64_t h = dfetch64(s + len - 16) * mul;
  const uint64_t u = drot(a + g, 43) + (drot(b, 30) + c) * 9;
  const uint64_t v = ((a + g) ^ d) + f + 1;
  const uint64_t w = dbswap((u + v) * mul) + h;
  const uint64_t x = drot(e + f, 42) + c;
  const uint64_t y = (dbswap((v + w) * mul) + g) * mul;
  const uint64_t z = e + f + c;
  a = dbswap((x + z) * mul + y) + b;
  b = dshiftmix((z + a) * mul + d + h) * mul;
  return b + x;
}

__device__ uint64_t dcityhash64(const uint8_t* s, uint32_t len) {
  if (len <= 32) return len <= 16 ? dcity_0to16(s, len) : dcity_17to32(s, len);
  if (len <= 64) return dcity_33to64(s, len);
  uint64_t x = dfetch64(s + len - 40);
  uint64_t y = dfetch64(s + len - 16) + dfetch64(s + len - 56);
  uint64_t z = dlen16(dfetch64(s + len - 48) + len, dfetch64(s + len - 24));
  uint64_t v1, v2, w1, w2;
  dweak32(s + len - 64, len, z, v1, v2);
  dweak32(s + len - 32, y + kC1, x, w1, w2);
  x = x * kC1 + dfetch64(s);
  len = (len - 1) & ~63u;
  do {
    x = drot(x + y + v1 + dfetch64(s + 8), 37) * kC1;
    y = drot(y + v2 + dfetch64(s + 48), 42) * kC1;
    x ^= w2;
    y += v1 + dfetch64(s + 40);
    z = drot(z + w1, 33) * kC1;
    uint64_t nv1, nv2, nw1, nw2;
    dweak32(s, v2 * kC1, x + w1, nv1, nv2);
    dweak32(s + 32, z + w2, y + dfetch64(s + 16), nw1, nw2);
    v1 = nv1, v2 = nv2, w1 = nw1, w2 = nw2;
    const uint64_t t = z;
    z = x;
    x = t;
    s += 64;
    len -= 64;
  } while (len != 0);
  return dlen16(dlen16(v1, w1) + dshiftmix(y) * kC1 + z, dlen16(v2, w2) + x);
}

// ---- line starts -----------------------------------------------------------
constexpr int kNlTile = 4096;

// a line ends at a newline that follows a non-newline byte: empty lines are
// skipped as the host parser skips them (a batch starts right after a newline,
// so byte 0 never ends a line)
__device__ __forceinline__ bool is_end(const uint8_t* t, int64_t j) {
  return t[j] == '\n' && j > 0 && t[j - 1] != '\n';
}

__global__ __launch_bounds__(256) void k_nl_count(const uint8_t* __restrict__ t, int64_t n,
                                                  int32_t* __restrict__ cnt) {
  __shared__ int sc;
  if (threadIdx.x == 0) sc = 0;
  __syncthreads();
  const int64_t b = (int64_t)blockIdx.x * kNlTile;
  int c = 0;
  for (int i = threadIdx.x; i < kNlTile; i += 256) {
    const int64_t j = b + i;
    if (j < n && is_end(t, j)) ++c;
  }
  c = (int)wave_sum((float)c);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(&sc, c);
  __syncthreads();
  if (threadIdx.x == 0) cnt[blockIdx.x] = sc;
}

// line k starts after its predecessor's end; line 0 at 0. A final line
// without a newline (the host batcher always appends one) is not counted.
__global__ __launch_bounds__(256) void k_nl_fill(const uint8_t* __restrict__ t, int64_t n,
                                                 const int64_t* __restrict__ off,
                                                 int64_t* __restrict__ start) {
  const int64_t b = (int64_t)blockIdx.x * kNlTile;
  if (blockIdx.x == 0 && threadIdx.x == 0) start[0] = 0;
  // wave-ordered: each wave scans a contiguous 1 KiB slice in 64-byte steps
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t base = off[blockIdx.x];
  __shared__ int wc[4];
  int c = 0;
  for (int i = 0; i < kNlTile / 4; i += 64) {
    const int64_t j = b + w * (kNlTile / 4) + i + lane;
    c += (j < n && is_end(t, j)) ? 1 : 0;
  }
  c = (int)wave_sum((float)c);
  if (lane == 0) wc[w] = c;
  __syncthreads();
  for (int q = 0; q < w; ++q) base += wc[q];
  for (int i = 0; i < kNlTile / 4; i += 64) {
    const int64_t j = b + w * (kNlTile / 4) + i + lane;
    const bool nl = j < n && is_end(t, j);
    const uint64_t m = __ballot(nl);
    if (nl) start[base + 1 + __popcll(m & ((1ull << lane) - 1ull))] = j + 1;
    base += __popcll(m);
  }
}

// 16 bytes per thread (one 16-byte load; the byte before them by one more):
// the same ends as k_nl_count / k_nl_fill with a sixteenth of the load
// instructions -- those scanned a byte per lane and loaded every byte twice
// (it and its predecessor). Needs a 16-byte aligned text.
__device__ __forceinline__ uint32_t nl_ends16(const uint8_t* __restrict__ t, int64_t n, int64_t j0) {
  uint8_t c[16];
  if (j0 + 16 <= n) {
    const uint4 v = *reinterpret_cast<const uint4*>(t + j0);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 16; ++k) c[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
  } else {
#pragma unroll
    for (int k = 0; k < 16; ++k) c[k] = j0 + k < n ? t[j0 + k] : (uint8_t)0;
  }
  uint8_t prev = j0 > 0 && j0 - 1 < n ? t[j0 - 1] : (uint8_t)'\n';
  uint32_t m = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    // is_end: a newline after a non-newline byte (byte 0 never ends a line)
    if (j0 + k < n && j0 + k > 0 && c[k] == '\n' && prev != '\n') m |= 1u << k;
    prev = c[k];
  }
  return m;
}

__global__ __launch_bounds__(256) void k_nl_count16(const uint8_t* __restrict__ t, int64_t n,
                                                    int32_t* __restrict__ cnt) {
  __shared__ int wc[4];
  const int64_t j0 = (int64_t)blockIdx.x * kNlTile + threadIdx.x * 16;
  int c = __popc(nl_ends16(t, n, j0));
  c = (int)wave_sum((float)c);
  if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) cnt[blockIdx.x] = wc[0] + wc[1] + wc[2] + wc[3];
}

__global__ __launch_bounds__(256) void k_nl_fill16(const uint8_t* __restrict__ t, int64_t n,
                                                   const int64_t* __restrict__ off,
                                                   int64_t* __restrict__ start) {
  __shared__ int wc[4];
  if (blockIdx.x == 0 && threadIdx.x == 0) start[0] = 0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t j0 = (int64_t)blockIdx.x * kNlTile + threadIdx.x * 16;
  const uint32_t m = nl_ends16(t, n, j0);
  const int c = __popc(m);
  int x = c;  // wave inclusive scan of the per-thread counts
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wc[w] = x;
  __syncthreads();
  int64_t base = off[blockIdx.x] + x - c;
  for (int q = 0; q < w; ++q) base += wc[q];
  uint32_t mm = m;
  while (mm) {
    const int k = __ffs(mm) - 1;
    mm &= mm - 1;
    start[++base] = j0 + k + 1;
  }
}

// ---- fields ---------------------------------------------------------------
constexpr int kCriteoFields = 39;
constexpr int kMaxLine = 1 << 16;
constexpr int kStage = 1024;  // LDS bytes per wave (a Criteo line is ~250)

// label: the first field as a decimal (Criteo: "0" / "1"); strtof-compatible
// for plain integers and simple decimals
__device__ float parse_label(const uint8_t* s, int len) {
  float v = 0.f, frac = 0.f, scale = 1.f;
  bool neg = false, dot = false;
  for (int i = 0; i < len; ++i) {
    const uint8_t c = s[i];
    if (i == 0 && (c == '-' || c == '+')) {
      neg = c == '-';
      continue;
    }
    if (c == '.') {
      dot = true;
      continue;
    }
    if (c < '0' || c > '9') break;
    if (dot) {
      scale *= 0.1f;
      frac += (c - '0') * scale;
    } else {
      v = v * 10.f + (c - '0');
    }
  }
  v += frac;
  return neg ? -v : v;
}

__global__ __launch_bounds__(256) void k_criteo_fields(const uint8_t* __restrict__ t, int64_t n,
                                                       const int64_t* __restrict__ start,
                                                       int64_t nlines, int train,
                                                       uint64_t* __restrict__ keys,
                                                       int32_t* __restrict__ cnt,
                                                       float* __restrict__ label) {
  const int lane = threadIdx.x & 63;
  const int64_t line = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  if (line >= nlines) return;
  int64_t b = start[line];
  int64_t e = start[line + 1] - 1;  // the newline
  if (e > n) e = n;
  while (b < e && (t[b] == '\n' || t[b] == '\r')) ++b;  // empty lines before this one
  while (e > b && t[e - 1] == '\r') --e;
  // field boundaries: tab positions by ballot over 64-byte windows; lane q
  // ends up holding the start of field q (and field q+1's start - 1 = its end).
  // The scanned bytes are staged in LDS and hashed from there.
  __shared__ uint8_t sl[4][kStage];
  uint8_t* my = sl[threadIdx.x >> 6];
  const int nf = kCriteoFields + (train ? 1 : 0);
  int my_start = lane == 0 ? 0 : -1;  // relative to b
  int ntabs = 0;
  const int len = (int)(e - b < kMaxLine ? e - b : kMaxLine);
  // the line's first kStage bytes staged in LDS up front: all of a lane's
  // byte loads in flight together (the window loop below then scans LDS;
  // loading each 64-byte window inside it made every line a chain of ~5
  // dependent global round trips)
  {
    const int lim = len < kStage ? len : kStage;
    uint8_t pre[kStage / 64];
#pragma unroll
    for (int u = 0; u < kStage / 64; ++u) {
      const int i = u * 64 + lane;
      pre[u] = i < lim ? t[b + i] : (uint8_t)0;
    }
#pragma unroll
    for (int u = 0; u < kStage / 64; ++u) my[u * 64 + lane] = pre[u];
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  int w0 = 0;
  for (; w0 < len && ntabs < nf; w0 += 64) {
    const int i = w0 + lane;
    const uint8_t c = i < len ? (i < kStage ? my[i] : t[b + i]) : (uint8_t)0;
    const uint64_t m = __ballot(i < len && c == '\t');
    // the k-th tab of the line starts field k: lane k takes its position
    uint64_t mm = m;
    while (mm) {
      const int src = __ffsll((unsigned long long)mm) - 1;
      mm &= mm - 1;
      ++ntabs;
      if (lane == ntabs && ntabs < 64) my_start = w0 + src + 1;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  // every hashed byte lies in a scanned window (scanning stops only after the
  // tab that ends the last used field)
  const uint8_t* src = w0 <= kStage ? my : t + b;
  // field q spans [start_q, start_{q+1} - 1); the last field ends at len
  int nxt = __shfl_down(my_start, 1, 64);
  if (lane == 63 || lane + 1 > ntabs) nxt = len + 1;
  const bool have = lane <= ntabs && my_start >= 0 && lane < nf;
  const int fs = my_start, fe = nxt - 1;  // [fs, fe)
  // label (training): field 0; features: fields 1.. (train) or 0..
  if (train && lane == 0) label[line] = have ? parse_label(src + fs, fe - fs) : 0.f;
  if (!train && lane == 0) label[line] = 0.f;
  const int fi = lane - (train ? 1 : 0);  // feature field index
  uint64_t key = kEmptyKey;
  if (have && fi >= 0 && fi < kCriteoFields && fe > fs)
    key = (dcityhash64(src + fs, (uint32_t)(fe - fs)) >> 10) | ((uint64_t)fi << 54);
  // compact this line's present keys in field order
  const bool k_ok = key != kEmptyKey;
  const uint64_t km = __ballot(k_ok);
  if (k_ok) keys[line * kCriteoFields + __popcll(km & ((1ull << lane) - 1ull))] = key;
  if (lane == 0) cnt[line] = __popcll(km);
}

__global__ __launch_bounds__(256) void k_criteo_compact(const uint64_t* __restrict__ padded,
                                                        const int64_t* __restrict__ off,
                                                        int64_t nlines,
                                                        uint64_t* __restrict__ keys) {
  const int lane = threadIdx.x & 63;
  const int64_t line = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  if (line >= nlines) return;
  const int64_t o = off[line], c = off[line + 1] - o;
  if (lane < c) keys[o + lane] = padded[line * kCriteoFields + lane];
}


// ---- libsvm ----------------------------------------------------------------
// label[:weight] idx[:value] ... separated by blanks; the host parser is
// csrc/host/parsers.cc ParseLibSVM (dmlc LibSVMParser semantics). Numbers are
// converted as strtoull / strtof do: integers exactly; decimals correctly
// rounded when the significand has <= 7 digits and |exponent| <= 10 (one
// exact float operation, Clinger's fast path) -- every value the usual
// libsvm writers print -- and via one correctly rounded double otherwise
// (which can differ from strtof in the last bit only at a double-rounding
// tie, probability ~2^-29 per value).
__device__ __forceinline__ bool is_blank(uint8_t c) { return c == ' ' || c == '\t'; }
__device__ __forceinline__ bool is_digit(uint8_t c) { return c >= '0' && c <= '9'; }

__device__ const uint8_t* parse_u64(const uint8_t* s, const uint8_t* e, uint64_t* v) {
  uint64_t m = 0;
  while (s < e && is_digit(*s)) m = m * 10 + (*s++ - '0');
  *v = m;
  return s;
}

__device__ const uint8_t* parse_f32(const uint8_t* s, const uint8_t* e, float* out) {
  const uint8_t* s0 = s;
  bool neg = false;
  if (s < e && (*s == '-' || *s == '+')) neg = *s++ == '-';
  uint64_t m = 0;
  int nd = 0, e10 = 0;
  bool any = false, trunc = false;
  for (; s < e && is_digit(*s); ++s) {
    const int d = *s - '0';
    any = true;
    if (m == 0 && d == 0) continue;
    if (nd < 19) m = m * 10 + d, ++nd;
    else ++e10, trunc |= d != 0;
  }
  if (s < e && *s == '.') {
    for (++s; s < e && is_digit(*s); ++s) {
      const int d = *s - '0';
      any = true;
      if (m == 0 && d == 0) {
        --e10;
        continue;
      }
      if (nd < 19) m = m * 10 + d, ++nd, --e10;
      else trunc |= d != 0;
    }
  }
  if (!any) {
    *out = 0.f;
    return s0;
  }
  if (s < e && (*s == 'e' || *s == 'E')) {
    const uint8_t* q = s + 1;
    bool eneg = false;
    if (q < e && (*q == '-' || *q == '+')) eneg = *q++ == '-';
    if (q < e && is_digit(*q)) {
      int x = 0;
      for (; q < e && is_digit(*q); ++q) x = x < 100000 ? x * 10 + (*q - '0') : x;
      e10 += eneg ? -x : x;
      s = q;
    }
  }
  float f;
  if (m == 0) {
    f = 0.f;
  } else if (!trunc && m < (1ull << 24) && e10 >= -10 && e10 <= 10) {
    const float p10[11] = {1e0f, 1e1f, 1e2f, 1e3f, 1e4f, 1e5f, 1e6f, 1e7f, 1e8f, 1e9f, 1e10f};
    f = e10 >= 0 ? (float)m * p10[e10] : (float)m / p10[-e10];
  } else {
    double d = (double)m;
    int x = e10;
    if (x > 400) x = 400;
    if (x < -400) x = -400;
    while (x > 22) d *= 1e22, x -= 22;
    while (x < -22) d /= 1e22, x += 22;
    const double p22[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                            1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
    d = x >= 0 ? d * p22[x] : d / p22[-x];
    f = (float)d;
  }
  *out = neg ? -f : f;
  return s;
}

// the content of line `line`: [b, e) without leading newlines and trailing
// carriage returns
__device__ __forceinline__ void line_span(const uint8_t* t, int64_t n, const int64_t* start,
                                          int64_t line, int64_t& b, int64_t& e) {
  b = start[line];
  e = start[line + 1] - 1;
  if (e > n) e = n;
  while (b < e && (t[b] == '\n' || t[b] == '\r')) ++b;
  while (e > b && t[e - 1] == '\r') --e;
}

// token starts of a 64-byte window: a non-blank byte after a blank (the byte
// before the line counts as blank); `prev` carries the last byte's blankness
__device__ __forceinline__ uint64_t token_starts(const uint8_t* t, int64_t b, int64_t len,
                                                 int64_t w0, int lane, uint64_t& prev) {
  const int64_t i = w0 + lane;
  const bool blank = i >= len || is_blank(t[b + i]);
  const uint64_t bm = __ballot(blank);
  const uint64_t st = ~bm & ((bm << 1) | prev);
  prev = bm >> 63;
  return st;
}

__global__ __launch_bounds__(256) void k_libsvm_count(const uint8_t* __restrict__ t, int64_t n,
                                                      const int64_t* __restrict__ start,
                                                      int64_t nlines, int32_t* __restrict__ cnt) {
  const int lane = threadIdx.x & 63;
  const int64_t line = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  if (line >= nlines) return;
  int64_t b, e;
  line_span(t, n, start, line, b, e);
  const int64_t len = e - b;
  uint64_t prev = 1;
  int ntok = 0;
  for (int64_t w0 = 0; w0 < len; w0 += 64) ntok += __popcll(token_starts(t, b, len, w0, lane, prev));
  if (lane == 0) cnt[line] = ntok > 0 ? ntok - 1 : 0;
}

// flags[0] = 1 if any value != 1, flags[1] = 1 if any line has a weight
__global__ __launch_bounds__(256) void k_libsvm_fill(
    const uint8_t* __restrict__ t, int64_t n, const int64_t* __restrict__ start, int64_t nlines,
    const int64_t* __restrict__ off, uint64_t* __restrict__ keys, float* __restrict__ val,
    float* __restrict__ label, float* __restrict__ weight, int32_t* __restrict__ flags) {
  const int lane = threadIdx.x & 63;
  const int64_t line = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  if (line >= nlines) return;
  int64_t b, e;
  line_span(t, n, start, line, b, e);
  const int64_t len = e - b;
  const uint8_t* le = t + e;
  const int64_t o = off[line];
  uint64_t prev = 1;
  int tok = 0;
  bool anyv = false, anyw = false;
  for (int64_t w0 = 0; w0 < len; w0 += 64) {
    const uint64_t st = token_starts(t, b, len, w0, lane, prev);
    if ((st >> lane) & 1) {
      const int k = tok + __popcll(st & ((1ull << lane) - 1ull));
      const uint8_t* p = t + b + w0 + lane;
      if (k == 0) {  // the label lane
        float lab = 0.f, w = 1.f;
        p = parse_f32(p, le, &lab);
        if (p < le && *p == ':') {
          parse_f32(p + 1, le, &w);
          anyw = true;
        }
        label[line] = lab;
        weight[line] = w;
      } else {
        uint64_t idx;
        p = parse_u64(p, le, &idx);
        float v = 1.f;
        if (p < le && *p == ':') parse_f32(p + 1, le, &v);
        keys[o + k - 1] = idx;
        val[o + k - 1] = v;
        anyv |= v != 1.f;
      }
    }
    tok += __popcll(st);
  }
  const uint64_t vm = __ballot(anyv), wm = __ballot(anyw);
  if (vm && lane == 0) flags[0] = 1;
  if (wm && lane == 0) flags[1] = 1;
  if (tok == 0 && lane == 0) label[line] = 0.f, weight[line] = 1.f;  // a blank line
}

// rows sel[i] of a CSR block -> row i of a new CSR block (noff: its offsets);
// 16 lanes per row (a Criteo row is 39 keys: a whole wave per row left 25 of
// its 64 lanes idle), the device half of the shuffle buffer
constexpr int kGatherLanes = 16;
__global__ __launch_bounds__(256) void k_csr_gather(
    const int64_t* __restrict__ off, const uint64_t* __restrict__ keys,
    const float* __restrict__ val, const float* __restrict__ label,
    const int64_t* __restrict__ sel, int64_t nsel, const int64_t* __restrict__ noff,
    uint64_t* __restrict__ okeys, float* __restrict__ oval, float* __restrict__ olabel) {
  const int sub = threadIdx.x & (kGatherLanes - 1);
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) / kGatherLanes;
  if (i >= nsel) return;
  const int64_t r = sel[i];
  const int64_t a = off[r], c = off[r + 1] - a, o = noff[i];
  for (int64_t j = sub; j < c; j += kGatherLanes) {
    okeys[o + j] = keys[a + j];
    if (val) oval[o + j] = val[a + j];
  }
  if (sub == 0) olabel[i] = label[r];
}

}  // namespace

void csr_gather(const int64_t* off, const uint64_t* keys, const float* val, const float* label,
                const int64_t* sel, int64_t nsel, const int64_t* noff, uint64_t* okeys,
                float* oval, float* olabel, hipStream_t s) {
  if (nsel <= 0) return;
  const int64_t rows_per_block = 256 / kGatherLanes;
  hipLaunchKernelGGL(k_csr_gather, dim3((unsigned)((nsel + rows_per_block - 1) / rows_per_block)),
                     dim3(256), 0, s, off, keys,
                     val, label, sel, nsel, noff, okeys, oval, olabel);
}

int64_t text_lines(const uint8_t* text, int64_t nbytes, int32_t* tile_cnt, int64_t* tile_off,
                     int64_t* scan_tmp, int64_t* start, hipStream_t s) {
  const int64_t ntile = (nbytes + kNlTile - 1) / kNlTile;
  if (ntile <= 0) return 0;
  const bool v16 = (reinterpret_cast<uintptr_t>(text) & 15) == 0;
  if (v16)
    hipLaunchKernelGGL(k_nl_count16, dim3((unsigned)ntile), dim3(256), 0, s, text, nbytes, tile_cnt);
  else
    hipLaunchKernelGGL(k_nl_count, dim3((unsigned)ntile), dim3(256), 0, s, text, nbytes, tile_cnt);
  scan_i32(tile_cnt, tile_off, ntile, scan_tmp, s);
  if (v16)
    hipLaunchKernelGGL(k_nl_fill16, dim3((unsigned)ntile), dim3(256), 0, s, text, nbytes, tile_off,
                       start);
  else
    hipLaunchKernelGGL(k_nl_fill, dim3((unsigned)ntile), dim3(256), 0, s, text, nbytes, tile_off,
                       start);
  return ntile;
}

int64_t text_tiles(int64_t nbytes) { return (nbytes + kNlTile - 1) / kNlTile; }

void criteo_fields(const uint8_t* text, int64_t nbytes, const int64_t* start, int64_t nlines,
                   bool train, uint64_t* padded, int32_t* cnt, float* label, hipStream_t s) {
  if (nlines <= 0) return;
  hipLaunchKernelGGL(k_criteo_fields, dim3((unsigned)((nlines + 3) / 4)), dim3(256), 0, s, text,
                     nbytes, start, nlines, train ? 1 : 0, padded, cnt, label);
}

int64_t libsvm_count(const uint8_t* text, int64_t nbytes, const int64_t* start, int64_t nlines,
                     int32_t* cnt, hipStream_t s) {
  if (nlines <= 0) return 0;
  hipLaunchKernelGGL(k_libsvm_count, dim3((unsigned)((nlines + 3) / 4)), dim3(256), 0, s, text,
                     nbytes, start, nlines, cnt);
  return nlines;
}

void libsvm_fill(const uint8_t* text, int64_t nbytes, const int64_t* start, int64_t nlines,
                 const int64_t* off, uint64_t* keys, float* val, float* label, float* weight,
                 int32_t* flags, hipStream_t s) {
  if (nlines <= 0) return;
  hipLaunchKernelGGL(k_libsvm_fill, dim3((unsigned)((nlines + 3) / 4)), dim3(256), 0, s, text,
                     nbytes, start, nlines, off, keys, val, label, weight, flags);
}

void criteo_compact(const uint64_t* padded, const int64_t* off, int64_t nlines, uint64_t* keys,
                    hipStream_t s) {
  if (nlines <= 0) return;
  hipLaunchKernelGGL(k_criteo_compact, dim3((unsigned)((nlines + 3) / 4)), dim3(256), 0, s,
                     padded, off, nlines, keys);
}

}  // namespace wh
