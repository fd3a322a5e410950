// Host cost of the torch-side calls around a small-minibatch native step
// (csrc/bind/difacto_step.inl): caching-allocator allocations, recordStream,
// stream / device guards, views, next to a plain kernel launch.
// Built by tools/microbench/build_torch_host_cost.sh (g++ against libtorch,
// no Python); run on the GPU box: ./bin/torch_host_cost
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

using clk = std::chrono::steady_clock;
template <class F>
static double per_call_us(int n, F&& f) {
  for (int i = 0; i < n / 10; ++i) f(i);
  const auto t0 = clk::now();
  for (int i = 0; i < n; ++i) f(i);
  return std::chrono::duration<double, std::micro>(clk::now() - t0).count() / n;
}

int main() {
  const int N = 20000;
  auto opt = at::TensorOptions().device(at::kCUDA, 0).dtype(at::kFloat);
  at::Tensor t = at::empty({1 << 20}, opt);
  hipStream_t raw;
  (void)hipStreamCreateWithFlags(&raw, hipStreamNonBlocking);
  auto side = c10::hip::getStreamFromExternal(raw, 0);
  hipEvent_t ev;
  (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  std::vector<double> r;
  std::printf("start\n");
  std::fflush(stdout);
  const char* names[] = {"at::empty 4 KiB",        "at::empty 4 MiB",
                         "recordStream",           "HIPStreamGuard",
                         "c10::DeviceGuard",       "getCurrentHIPStream",
                         "narrow + view",          "event record + stream wait",
                         "at::zeros 8 B",          "empty + 3 narrow/view + drop"};
  r.push_back(per_call_us(N, [&](int) { auto x = at::empty({1024}, opt); }));
  r.push_back(per_call_us(N, [&](int) { auto x = at::empty({1 << 20}, opt); }));
  r.push_back(per_call_us(N, [&](int) {
    c10::hip::HIPCachingAllocator::recordStream(t.storage().data_ptr(), side);
  }));
  r.push_back(per_call_us(N, [&](int) { c10::hip::HIPStreamGuard g(side); }));
  r.push_back(per_call_us(N, [&](int) { c10::DeviceGuard g(t.device()); }));
  r.push_back(per_call_us(N, [&](int) {
    volatile auto s = c10::hip::getCurrentHIPStream(0).stream();
    (void)s;
  }));
  r.push_back(per_call_us(N, [&](int i) { auto v = t.narrow(0, i & 1023, 256).view(at::kInt); }));
  r.push_back(per_call_us(N, [&](int) {
    (void)hipEventRecord(ev, c10::hip::getCurrentHIPStream(0).stream());
    (void)hipStreamWaitEvent(raw, ev, 0);
  }));
  r.push_back(per_call_us(N, [&](int) { auto x = at::zeros({1}, opt.dtype(at::kDouble)); }));
  r.push_back(per_call_us(N, [&](int) {
    auto b = at::empty({65536}, opt.dtype(at::kByte));
    auto a = b.narrow(0, 0, 4096).view(at::kFloat);
    auto c = b.narrow(0, 4096, 4096).view(at::kInt);
    auto d = b.narrow(0, 8192, 8192).view(at::kLong);
  }));
  (void)hipDeviceSynchronize();
  for (size_t i = 0; i < r.size(); ++i) std::printf("%-32s %7.2f us\n", names[i], r[i]);
  std::fflush(stdout);
  std::_Exit(0);  // (no static teardown of the HIP runtime / allocator)
}
