// bindings.cpp — the `DPE_MVS._dpe` pybind11 module: `dpe_mvs(...)` with the signature and error
// behaviour of the reference's binding (csrc/bindings.cpp:31-43): returns 0, raises RuntimeError
// on a nonzero pipeline result.  The pipeline itself is libdpe_host (C++), the GIL is released
// while it runs.  std::cout / std::cerr go to Python's sys.stdout / sys.stderr as in the reference
// (csrc/bindings.cpp:23-24); pybind's pythonbuf takes the GIL back on each flush.
#include <pybind11/iostream.h>
#include <pybind11/pybind11.h>

#include <iostream>

#include <stdexcept>
#include <string>

#include "../../include/dpe_host.h"

namespace py = pybind11;

static int dpe_mvs(const std::string& dense_folder, int gpu_index, bool verbose, bool fusion, bool viz, bool depth,
                   bool normal, bool weak, bool edge) {
  DpePipelineOptions o;
  dpe_pipeline_default_options(&o);
  o.gpu_index = gpu_index;
  o.verbose = verbose; o.fusion = fusion; o.viz = viz;
  o.depth = depth; o.normal = normal; o.weak = weak; o.edge = edge;
  py::scoped_ostream_redirect out(std::cout);
  py::scoped_ostream_redirect err(std::cerr, py::module_::import("sys").attr("stderr"));
  int rc;
  {
    py::gil_scoped_release release;
    rc = dpe_run_pipeline(dense_folder.c_str(), &o);
  }
  if (rc != 0) throw std::runtime_error(std::string("DPE pipeline failed: ") + dpe_pipeline_last_error());
  return rc;
}

PYBIND11_MODULE(_dpe, m) {
  m.doc() = "MI355X-native DPE-MVS pipeline (C++ host over the HIP PatchMatch C-ABI)";
  m.def("dpe_mvs", &dpe_mvs, py::arg("dense_folder"), py::arg("gpu_index") = 0, py::arg("verbose") = true,
        py::arg("fusion") = false, py::arg("viz") = false, py::arg("depth") = true, py::arg("normal") = false,
        py::arg("weak") = false, py::arg("edge") = false);
}
