#include <pybind11/pybind11.h>
namespace py = pybind11;
namespace bgc_py {
void register_gpu(py::module_& m) {}
}  // namespace bgc_py
