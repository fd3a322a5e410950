// pybind11 module entry of the native host runtime (wormhole_amd._host).
#include <torch/extension.h>

namespace wh { namespace host { void register_all(pybind11::module& m); } }

PYBIND11_MODULE(_host, m) {
  m.doc() = "wormhole_amd native host runtime";
  wh::host::register_all(m);
}
