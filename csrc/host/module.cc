// pybind11 module entry of the native host runtime (wormhole_amd._host).
#include <torch/extension.h>

#include <execinfo.h>
#include <unistd.h>

#include <cstdlib>
#include <exception>

namespace wh { namespace host { void register_all(pybind11::module& m); } }

namespace {
// std::terminate in a worker (a joinable std::thread destroyed, a forced
// unwind through a noexcept frame) otherwise dies with one line and no
// location: print the native stack to stderr first, then abort as before.
std::terminate_handler g_prev_terminate = nullptr;
void terminate_with_stack() {
  static const char msg[] = "[wormhole_amd] std::terminate; native stack:\n";
  ssize_t r = write(2, msg, sizeof(msg) - 1);
  (void)r;
  void* frames[64];
  const int n = backtrace(frames, 64);
  backtrace_symbols_fd(frames, n, 2);
  if (g_prev_terminate) g_prev_terminate();
  std::abort();
}
}  // namespace

PYBIND11_MODULE(_host, m) {
  m.doc() = "wormhole_amd native host runtime";
  g_prev_terminate = std::set_terminate(terminate_with_stack);
  wh::host::register_all(m);
}
