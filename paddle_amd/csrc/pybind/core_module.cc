// `paddle_amd_core`: the CPython extension module over the native C++ framework
// (csrc/native), the counterpart of the reference's pybind core
// (paddle/fluid/pybind/pybind.cc:89-708: core.Scope / core.LoDTensor /
// core.Executor / ProgramDesc / places; tensor_py.h numpy bridges).
//
// It binds the C++ classes themselves (no C ABI in between): ProgramDesc parsed
// from the framework.proto bytes Python's Program serialises, Scope trees,
// LoDTensor with numpy round trips and zero-copy lending of caller memory (a
// torch tensor's storage, host or device), and Executor running blocks on the
// host or a HIP device with the shared kernel library.  The GIL is released
// around Executor.run so Python threads keep running while a block executes.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "../native/framework.h"

namespace py = pybind11;

namespace {

pa::DT dt_of(const py::dtype& d) {
  switch (d.kind()) {
    case 'b':
      return pa::DT::BOOL;
    case 'f':
      if (d.itemsize() == 4) return pa::DT::FP32;
      if (d.itemsize() == 8) return pa::DT::FP64;
      if (d.itemsize() == 2) return pa::DT::FP16;
      break;
    case 'i':
      if (d.itemsize() == 8) return pa::DT::INT64;
      if (d.itemsize() == 4) return pa::DT::INT32;
      if (d.itemsize() == 2) return pa::DT::INT16;
      if (d.itemsize() == 1) return pa::DT::INT8;
      break;
    case 'u':
      if (d.itemsize() == 1) return pa::DT::UINT8;
      if (d.itemsize() == 2) return pa::DT::BF16;  // bf16 travels as uint16 bits
      break;
  }
  throw py::type_error("unsupported numpy dtype for a LoDTensor");
}

py::dtype np_of(pa::DT t) {
  switch (t) {
    case pa::DT::BOOL: return py::dtype::of<bool>();
    case pa::DT::INT16: return py::dtype::of<int16_t>();
    case pa::DT::INT32: return py::dtype::of<int32_t>();
    case pa::DT::INT64: return py::dtype::of<int64_t>();
    case pa::DT::FP16: return py::dtype("float16");
    case pa::DT::FP32: return py::dtype::of<float>();
    case pa::DT::FP64: return py::dtype::of<double>();
    case pa::DT::UINT8: return py::dtype::of<uint8_t>();
    case pa::DT::INT8: return py::dtype::of<int8_t>();
    case pa::DT::BF16: return py::dtype::of<uint16_t>();
  }
  throw py::type_error("unknown tensor dtype");
}

void set_from_numpy(pa::Tensor& t, py::array a, int device) {
  a = py::array::ensure(a, py::array::c_style);
  std::vector<int64_t> dims(a.shape(), a.shape() + a.ndim());
  pa::Tensor h;
  void* p = h.alloc(dt_of(a.dtype()), dims, -1);
  std::memcpy(p, a.data(), h.nbytes());
  t = device >= 0 ? h.to(device) : h;
}

py::array to_numpy(const pa::Tensor& t) {
  if (!t.initialized()) throw py::value_error("tensor is not initialised");
  pa::Tensor h = t.device >= 0 ? t.to(-1) : t;
  py::array out(np_of(h.dtype), std::vector<py::ssize_t>(h.dims.begin(), h.dims.end()));
  std::memcpy(out.mutable_data(), h.raw(), h.nbytes());
  return out;
}

}  // namespace

PYBIND11_MODULE(paddle_amd_core, m) {
  m.doc() = "paddle_amd native core (C++ ProgramDesc / Scope / LoDTensor / Executor)";
  py::register_exception<pa::Error>(m, "EnforceNotMet");

  py::enum_<pa::DT>(m, "VarType")
      .value("BOOL", pa::DT::BOOL).value("INT16", pa::DT::INT16).value("INT32", pa::DT::INT32)
      .value("INT64", pa::DT::INT64).value("FP16", pa::DT::FP16).value("FP32", pa::DT::FP32)
      .value("FP64", pa::DT::FP64).value("UINT8", pa::DT::UINT8).value("INT8", pa::DT::INT8)
      .value("BF16", pa::DT::BF16);

  py::class_<pa::ProgramDesc>(m, "ProgramDesc")
      .def(py::init([](py::bytes b) { return pa::ProgramDesc::Parse(std::string(b)); }), py::arg("binary_str"))
      .def_static("load", &pa::ProgramDesc::Load)
      .def("num_blocks", [](const pa::ProgramDesc& p) { return p.blocks.size(); })
      .def("num_ops", [](const pa::ProgramDesc& p, int b) { return p.Block(b).ops.size(); }, py::arg("block") = 0)
      .def("op_types", [](const pa::ProgramDesc& p, int b) {
        std::vector<std::string> v;
        for (auto& o : p.Block(b).ops) v.push_back(o.type);
        return v;
      }, py::arg("block") = 0)
      .def("var_names", [](const pa::ProgramDesc& p, int b) {
        std::vector<std::string> v;
        for (auto& x : p.Block(b).vars) v.push_back(x.name);
        return v;
      }, py::arg("block") = 0);

  py::class_<pa::Tensor>(m, "LoDTensor")
      .def(py::init<>())
      .def("shape", [](const pa::Tensor& t) { return t.dims; })
      .def("dtype", [](const pa::Tensor& t) { return t.dtype; })
      .def("device", [](const pa::Tensor& t) { return t.device; })
      .def("lod", [](const pa::Tensor& t) { return t.lod; })
      .def("set_lod", [](pa::Tensor& t, const pa::LoD& l) { t.lod = l; })
      .def("_is_initialized", &pa::Tensor::initialized)
      .def("set", &set_from_numpy, py::arg("array"), py::arg("device") = -1)
      .def("numpy", &to_numpy)
      .def("__array__", [](const pa::Tensor& t, py::args, py::kwargs) { return to_numpy(t); })
      .def("data_ptr", [](const pa::Tensor& t) { return reinterpret_cast<uintptr_t>(t.raw()); })
      // zero-copy: the tensor views caller-owned memory (e.g. torch storage); the
      // caller keeps it alive and the framework never frees it
      .def("share_external", [](pa::Tensor& t, uintptr_t ptr, pa::DT dt, std::vector<int64_t> dims, int device) {
        t.dtype = dt;
        t.dims = std::move(dims);
        t.device = device;
        t.buf = std::make_shared<pa::Buffer>(reinterpret_cast<void*>(ptr), t.nbytes(), device);
      }, py::arg("ptr"), py::arg("dtype"), py::arg("dims"), py::arg("device"));

  py::class_<pa::Variable>(m, "Variable")
      .def("get_tensor", [](pa::Variable& v) -> pa::Tensor& { return v.tensor; }, py::return_value_policy::reference_internal)
      .def("is_initialized", [](const pa::Variable& v) { return v.tensor.initialized(); })
      .def("kind", [](const pa::Variable& v) { return v.kind; });

  py::class_<pa::Scope>(m, "Scope")
      .def(py::init<>())
      .def("var", &pa::Scope::Var, py::return_value_policy::reference_internal)
      .def("find_var", &pa::Scope::Find, py::return_value_policy::reference_internal)
      .def("find_local_var", &pa::Scope::FindLocal, py::return_value_policy::reference_internal)
      .def("new_scope", &pa::Scope::NewScope, py::return_value_policy::reference_internal)
      .def("erase", &pa::Scope::Erase)
      .def("local_var_names", &pa::Scope::LocalNames);

  py::class_<pa::Executor>(m, "Executor")
      .def(py::init<int>(), py::arg("device") = -1)
      .def("run", [](pa::Executor& e, const pa::ProgramDesc& p, pa::Scope& s, int block) {
        py::gil_scoped_release nogil;
        e.Run(p, &s, block);
        e.Sync();
      }, py::arg("program"), py::arg("scope"), py::arg("block_id") = 0)
      .def("set_fallback", [](pa::Executor& e, py::object fn) {
        if (fn.is_none()) {
          e.fallback = nullptr;
          return;
        }
        // called from RunBlock with the GIL released by run(): take it for the callback
        auto keep = std::make_shared<py::object>(fn);
        e.fallback = [keep](const pa::OpDesc& op, pa::Scope& s, int block, int idx) {
          py::gil_scoped_acquire gil;
          (*keep)(block, idx, py::cast(&s, py::return_value_policy::reference));
        };
      }, py::arg("fn"))
      .def("set_stream", [](pa::Executor& e, uintptr_t st) { e.SetStream(reinterpret_cast<void*>(st)); },
           py::arg("stream"))
      .def("sync", &pa::Executor::Sync)
      .def_readonly("embedder_fallbacks", &pa::Executor::embedder_fallbacks)
      .def_readwrite("profile", &pa::Executor::profile)
      .def_readonly("op_time_ms", &pa::Executor::op_time_ms)
      .def_readonly("host_fallbacks", &pa::Executor::host_fallbacks);

  m.def("registered_ops", [](bool device) {
    pa::link_host_kernels();
    if (device) pa::link_device_kernels();
    auto v = pa::registered_ops(device);
    std::sort(v.begin(), v.end());
    return v;
  }, py::arg("device") = false);
  m.def("load_persistables", [](const pa::ProgramDesc& p, pa::Scope& s, const std::string& dir,
                                const std::string& combined, int device) {
    pa::load_persistables(p, &s, dir, combined, device, nullptr);
  }, py::arg("program"), py::arg("scope"), py::arg("dirname"), py::arg("combined_file") = "", py::arg("device") = -1);
}
