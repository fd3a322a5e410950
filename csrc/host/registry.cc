#include <torch/extension.h>
namespace wh { namespace host {
void register_all(pybind11::module& m) { (void)m; }
} }
