// Microbenchmark: the FM forward's embedding-row gathers on Criteo-shaped
// data (100k rows x 39 fields, power-law ranks), to find what bounds
// k_fm_fwd. Variants (all compute sum_j x_j v_j per row, 64-dim fp32):
//   A  G=16 lanes/row, 8 rows in flight per group          (production shape)
//   B  same, no V gathers (index + header traffic only)
//   C  same, V index masked to 1024 rows (L2-resident V)
//   D  one wave per row, 4 V rows per wave-instruction, all 39 rows issued
//      before any use (max MLP)
//   E  like A but rows of a wave sorted so that G-groups read the SAME field
// Build: hipcc -O3 --offload-arch=gfx950 -o /tmp/fmgb tools/microbench/fm_gather_bench.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
#include <unordered_map>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

constexpr int NF = 39, DIM = 64, G = 16;

template <int MODE>
__global__ __launch_bounds__(256) void k_a(int nrows, const int* lid, const float2* hdr,
                                           const float* vc, float* out) {
  const int lane = threadIdx.x & 63, gl = lane & (G - 1), gbase = lane - gl;
  const int row = (blockIdx.x * 256 + threadIdx.x) / G;
  if (row >= nrows) return;  // nrows multiple of 16 here
  int vq[3];
  float wl = 0.f;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int i = q * G + gl;
    int l = i < NF ? lid[row * NF + i] : -1;
    float2 h = l >= 0 ? hdr[l] : make_float2(0.f, __int_as_float(-1));
    wl += h.x;
    vq[q] = __float_as_int(h.y);
    if (MODE == 2 && vq[q] >= 0) vq[q] &= 1023;
  }
  float4 s = make_float4(0, 0, 0, 0);
  if (MODE != 1) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
#pragma unroll
      for (int i0 = 0; i0 < G; i0 += 8) {
        if (q * G + i0 >= NF) break;
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int vu = __shfl(vq[q], gbase + i0 + u, 64);
          v[u] = vu >= 0 ? reinterpret_cast<const float4*>(vc + (size_t)vu * DIM)[gl]
                         : make_float4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) { s.x += v[u].x; s.y += v[u].y; s.z += v[u].z; s.w += v[u].w; }
      }
    }
  }
  reinterpret_cast<float4*>(out + (size_t)row * DIM)[gl] = make_float4(s.x + wl, s.y, s.z, s.w);
}

// one wave per row: lane = (sub, gl): sub in 0..3 picks the V row within an
// instruction, gl the float4 slice; 10 instructions cover 40 >= 39 rows
__global__ __launch_bounds__(256) void k_d(int nrows, const int* lid, const float2* hdr,
                                           const float* vc, float* out) {
  const int lane = threadIdx.x & 63, gl = lane & 15, sub = lane >> 4;
  const int row = (blockIdx.x * 256 + threadIdx.x) / 64;
  if (row >= nrows) return;
  int l = lane < NF ? lid[row * NF + lane] : -1;
  float2 h = l >= 0 ? hdr[l] : make_float2(0.f, __int_as_float(-1));
  const int vid = __float_as_int(h.y);
  float4 v[10];
#pragma unroll
  for (int t = 0; t < 10; ++t) {
    const int vu = __shfl(vid, t * 4 + sub, 64);
    v[t] = vu >= 0 ? reinterpret_cast<const float4*>(vc + (size_t)vu * DIM)[gl]
                   : make_float4(0, 0, 0, 0);
  }
  float4 s = make_float4(0, 0, 0, 0);
#pragma unroll
  for (int t = 0; t < 10; ++t) { s.x += v[t].x; s.y += v[t].y; s.z += v[t].z; s.w += v[t].w; }
  // reduce the 4 subs
  for (int o = 16; o < 64; o <<= 1) {
    s.x += __shfl_xor(s.x, o, 64); s.y += __shfl_xor(s.y, o, 64);
    s.z += __shfl_xor(s.z, o, 64); s.w += __shfl_xor(s.w, o, 64);
  }
  if (sub == 0) reinterpret_cast<float4*>(out + (size_t)row * DIM)[gl] = s;
}

int main() {
  const int nrows = 100000;
  const long card[NF] = {64, 3000, 2000, 500, 200000, 10000, 3000, 500, 6000, 20, 200, 1000, 600,
                         39884406, 39043, 17289, 7420, 20263, 3, 7120, 1543, 63, 38532951,
                         2953546, 403346, 10, 2208, 11938, 155, 4, 976, 14, 39979771, 25641295,
                         39664984, 585935, 12972, 108, 36};
  std::mt19937_64 rng(1);
  std::uniform_real_distribution<double> U(0, 1);
  // local ids: (field, rank) -> dense id by first appearance
  std::vector<int> lid(nrows * NF);
  std::vector<std::vector<std::pair<long, int>>> maps(NF);
  std::vector<std::unordered_map<long, int>*> mp(NF);
  for (int f = 0; f < NF; ++f) mp[f] = new std::unordered_map<long, int>();
  int nu = 0;
  for (int r = 0; r < nrows; ++r)
    for (int f = 0; f < NF; ++f) {
      long rank = (long)std::exp(std::log((double)card[f]) * U(rng)) - 1;
      if (rank < 0) rank = 0;
      auto it = mp[f]->find(rank);
      int id;
      if (it == mp[f]->end()) { id = nu++; (*mp[f])[rank] = id; } else id = it->second;
      lid[r * NF + f] = id;
    }
  // every key has a V row (worst case); vidx = random permutation
  std::vector<float2> hdr(nu);
  std::vector<int> perm(nu);
  for (int i = 0; i < nu; ++i) perm[i] = i;
  std::shuffle(perm.begin(), perm.end(), rng);
  for (int i = 0; i < nu; ++i) { hdr[i].x = 0.01f; hdr[i].y = *(float*)&perm[i]; }
  printf("nrows %d nnz %d unique %d  V bytes gathered %.1f MB\n", nrows, nrows * NF, nu,
         nrows * NF * 256.0 / 1e6);
  int* d_lid; float2* d_hdr; float* d_vc; float* d_out;
  CK(hipMalloc(&d_lid, lid.size() * 4));
  CK(hipMalloc(&d_hdr, nu * 8));
  CK(hipMalloc(&d_vc, (size_t)nu * DIM * 4));
  CK(hipMalloc(&d_out, (size_t)nrows * DIM * 4));
  CK(hipMemcpy(d_lid, lid.data(), lid.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_hdr, hdr.data(), nu * 8, hipMemcpyHostToDevice));
  CK(hipMemset(d_vc, 0, (size_t)nu * DIM * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    const int it = 20;
    for (int i = 0; i < it; ++i) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    const double us = 1000.0 * ms / it;
    printf("%-44s %8.1f us   %6.2f TB/s of V rows\n", name, us, nrows * NF * 256.0 / (us * 1e-6) / 1e12);
  };
  const int gA = (nrows * G + 255) / 256, gD = (nrows * 64 + 255) / 256;
  run("A  G=16, 8 in flight (production shape)", [&] { k_a<0><<<gA, 256>>>(nrows, d_lid, d_hdr, d_vc, d_out); });
  run("B  no V gathers", [&] { k_a<1><<<gA, 256>>>(nrows, d_lid, d_hdr, d_vc, d_out); });
  run("C  V index & 1023 (L2 resident)", [&] { k_a<2><<<gA, 256>>>(nrows, d_lid, d_hdr, d_vc, d_out); });
  run("D  wave/row, 10 instr (40 rows) in flight", [&] { k_d<<<gD, 256>>>(nrows, d_lid, d_hdr, d_vc, d_out); });
  return 0;
}
