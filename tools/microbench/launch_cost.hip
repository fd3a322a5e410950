// Host cost of the HIP calls a small-minibatch step is made of, on one
// MI355X: an empty kernel launch (1 and 8 arguments), an event record, a
// stream wait on an event, a small async D2H copy into pinned memory, and
// the same 25-launch sequence captured once in a hipGraph and replayed.
//
//   hipcc -O3 --offload-arch=gfx950 -o launch_cost launch_cost.hip && ./launch_cost
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                  \
      std::exit(1);                                                         \
    }                                                                       \
  } while (0)

__global__ void k_empty() {}
__global__ void k_args(const long* a, long* b, long n, int c, float d, const int* e, int* f,
                       long g) {
  if (n < 0 && threadIdx.x == 0) b[0] = a[0] + c + (long)d + e[0] + f[0] + g;
}

using clk = std::chrono::steady_clock;
static double us_since(clk::time_point t0, int n) {
  return std::chrono::duration<double, std::micro>(clk::now() - t0).count() / n;
}

int main() {
  hipStream_t s, s2;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  long *a, *b;
  int* e;
  CK(hipMalloc(&a, 4096));
  CK(hipMalloc(&b, 4096));
  CK(hipMalloc(&e, 4096));
  CK(hipMemset(a, 0, 4096));
  CK(hipMemset(e, 0, 4096));
  long* host;
  CK(hipHostMalloc(&host, 4096, hipHostMallocDefault));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const int N = 20000;
  for (int i = 0; i < 2000; ++i) k_empty<<<1, 64, 0, s>>>();
  CK(hipStreamSynchronize(s));

  auto t0 = clk::now();
  for (int i = 0; i < N; ++i) k_empty<<<1, 64, 0, s>>>();
  double t_empty = us_since(t0, N);
  CK(hipStreamSynchronize(s));

  t0 = clk::now();
  for (int i = 0; i < N; ++i) k_args<<<256, 256, 0, s>>>(a, b, -1, 3, 1.f, e, e + 1, 7);
  double t_args = us_since(t0, N);
  CK(hipStreamSynchronize(s));

  t0 = clk::now();
  for (int i = 0; i < N; ++i) CK(hipEventRecord(ev, s));
  double t_rec = us_since(t0, N);
  CK(hipStreamSynchronize(s));

  t0 = clk::now();
  for (int i = 0; i < N; ++i) CK(hipStreamWaitEvent(s2, ev, 0));
  double t_wait = us_since(t0, N);
  CK(hipStreamSynchronize(s2));

  t0 = clk::now();
  for (int i = 0; i < N; ++i) CK(hipMemcpyAsync(host, a, 64, hipMemcpyDeviceToHost, s));
  double t_d2h = us_since(t0, N);
  CK(hipStreamSynchronize(s));

  // the same on the NULL stream (torch's default current stream)
  t0 = clk::now();
  for (int i = 0; i < N; ++i) k_args<<<256, 256, 0, 0>>>(a, b, -1, 3, 1.f, e, e + 1, 7);
  double t_args0 = us_since(t0, N);
  CK(hipDeviceSynchronize());
  t0 = clk::now();
  for (int i = 0; i < N; ++i) CK(hipEventRecord(ev, 0));
  double t_rec0 = us_since(t0, N);
  CK(hipDeviceSynchronize());
  t0 = clk::now();
  for (int i = 0; i < N; ++i) CK(hipStreamWaitEvent(0, ev, 0));
  double t_wait0 = us_since(t0, N);
  CK(hipDeviceSynchronize());
  t0 = clk::now();
  for (int i = 0; i < N; ++i) {
    CK(hipEventRecord(ev, 0));
    CK(hipStreamWaitEvent(s2, ev, 0));
  }
  double t_recwait0 = us_since(t0, N);
  CK(hipDeviceSynchronize());
  t0 = clk::now();
  for (int i = 0; i < N; ++i) {
    CK(hipEventRecord(ev, s));
    CK(hipStreamWaitEvent(s2, ev, 0));
  }
  double t_recwait = us_since(t0, N);
  CK(hipDeviceSynchronize());
  t0 = clk::now();
  for (int i = 0; i < N; ++i) CK(hipMemsetAsync(b, 0, 8, s));
  double t_memset = us_since(t0, N);
  CK(hipDeviceSynchronize());

  // round trip: launch + D2H + sync (a step's one host read)
  const int R = 2000;
  t0 = clk::now();
  for (int i = 0; i < R; ++i) {
    k_empty<<<1, 64, 0, s>>>();
    CK(hipMemcpyAsync(host, a, 64, hipMemcpyDeviceToHost, s));
    CK(hipEventRecord(ev, s));
    CK(hipEventSynchronize(ev));
  }
  double t_rt = us_since(t0, R);

  // 25 launches captured once, replayed
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < 25; ++i) k_args<<<256, 256, 0, s>>>(a, b, -1, i, 1.f, e, e + 1, 7);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int i = 0; i < 100; ++i) CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  const int G = 2000;
  t0 = clk::now();
  for (int i = 0; i < G; ++i) CK(hipGraphLaunch(ge, s));
  double t_graph = us_since(t0, G);
  CK(hipStreamSynchronize(s));
  t0 = clk::now();
  for (int i = 0; i < G; ++i) CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  double t_graph_gpu = us_since(t0, G);
  t0 = clk::now();
  for (int i = 0; i < G; ++i)
    for (int j = 0; j < 25; ++j) k_args<<<256, 256, 0, s>>>(a, b, -1, j, 1.f, e, e + 1, 7);
  CK(hipStreamSynchronize(s));
  double t_25_gpu = us_since(t0, G);

  std::printf("host us per call: empty launch %.2f | 8-arg 256-block launch %.2f | event record %.2f | "
              "stream wait %.2f | 64 B D2H async %.2f\n",
              t_empty, t_args, t_rec, t_wait, t_d2h);
  std::printf("NULL stream: 8-arg launch %.2f | event record %.2f | wait on NULL %.2f | record on NULL + "
              "wait on other %.2f || created streams: record + wait %.2f | 8 B memset async %.2f\n",
              t_args0, t_rec0, t_wait0, t_recwait0, t_recwait, t_memset);
  std::printf("launch + D2H + event sync round trip %.2f us\n", t_rt);
  std::printf("25-launch hipGraph: %.2f us host per replay, %.2f us per replay incl. GPU; "
              "25 plain launches incl. GPU %.2f us\n",
              t_graph, t_graph_gpu, t_25_gpu);
  return 0;
}
