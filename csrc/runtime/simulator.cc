// MI355X execution simulator + MCMC strategy search (filled in below).
#include <pybind11/pybind11.h>
namespace py = pybind11;
void register_sim(py::module_& m) {}
