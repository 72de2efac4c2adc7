// C++ entry for the hottest framework tensor ops (elementwise add / scale / cast /
// copy / fill on contiguous same-shape device tensors): unpacks the torch tensors in
// C++ and launches the kernel library's flat elementwise kernel (tensor_ops.hip
// pa_ew_flat) on the caller's stream.  The Python dispatch path pays ~5 us per call in
// argument marshalling (profiles/r5_dispatch_cost.md); this entry is what
// ops/aten_native.py's hot path and the framework's direct callers (oplib.add_ /
// fill_, the eager engine's gradient accumulation) use when it is built.
// Returns false when the call does not fit (the caller takes the general path).
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

extern "C" int pa_ew_flat(int op, int cdt, int nin, long n, void* out, int odt, const void* x, int xdt,
                          const void* y, int ydt, const void* z, int zdt, double a, double b, void* st);

namespace {

int dt_code(c10::ScalarType s) {
  switch (s) {
    case c10::ScalarType::Float: return 0;
    case c10::ScalarType::BFloat16: return 1;
    case c10::ScalarType::Half: return 2;
    case c10::ScalarType::Double: return 3;
    case c10::ScalarType::Long: return 4;
    case c10::ScalarType::Int: return 5;
    case c10::ScalarType::Short: return 6;
    case c10::ScalarType::Char: return 7;
    case c10::ScalarType::Byte: return 8;
    case c10::ScalarType::Bool: return 9;
    default: return -1;
  }
}

// compute type: 0 fp32 (every float type but double), 1 fp64, 2 integer
int cdt_of(c10::ScalarType s) {
  if (s == c10::ScalarType::Double) return 1;
  if (c10::isFloatingType(s)) return 0;
  return 2;
}

bool fits(const at::Tensor& out, const at::Tensor* ins, int nin) {
  if (!out.is_cuda() || !out.is_contiguous() || dt_code(out.scalar_type()) < 0) return false;
  for (int i = 0; i < nin; ++i) {
    const at::Tensor& t = ins[i];
    if (!t.is_cuda() || !t.is_contiguous() || t.sizes() != out.sizes() || dt_code(t.scalar_type()) < 0 ||
        t.device() != out.device())
      return false;
  }
  return true;
}

bool launch(int op, int cdt, const at::Tensor& out, const at::Tensor* ins, int nin, double a, double b,
            int64_t stream) {
  if (!fits(out, ins, nin)) return false;
  const long n = out.numel();
  if (n == 0) return true;
  if (cdt < 0) cdt = cdt_of(nin ? ins[0].scalar_type() : out.scalar_type());
  const void* p[3] = {nullptr, nullptr, nullptr};
  int d[3] = {0, 0, 0};
  for (int i = 0; i < nin; ++i) {
    p[i] = ins[i].data_ptr();
    d[i] = dt_code(ins[i].scalar_type());
  }
  const int rc = pa_ew_flat(op, cdt, nin, n, out.data_ptr(), dt_code(out.scalar_type()), p[0], d[0], p[1], d[1],
                            p[2], d[2], a, b, reinterpret_cast<void*>(stream));
  TORCH_CHECK(rc == 0, "pa_ew_flat failed (rc=", rc, ", op=", op, ")");
  return true;
}

bool ew0(int op, int cdt, const at::Tensor& out, double a, double b, int64_t stream) {
  return launch(op, cdt, out, nullptr, 0, a, b, stream);
}

bool ew1(int op, int cdt, const at::Tensor& out, const at::Tensor& x, double a, double b, int64_t stream) {
  return launch(op, cdt, out, &x, 1, a, b, stream);
}

bool ew2(int op, int cdt, const at::Tensor& out, const at::Tensor& x, const at::Tensor& y, double a, double b,
         int64_t stream) {
  const at::Tensor ins[2] = {x, y};
  return launch(op, cdt, out, ins, 2, a, b, stream);
}

bool ew3(int op, int cdt, const at::Tensor& out, const at::Tensor& x, const at::Tensor& y, const at::Tensor& z,
         double a, double b, int64_t stream) {
  const at::Tensor ins[3] = {x, y, z};
  return launch(op, cdt, out, ins, 3, a, b, stream);
}

void* current_stream(const at::Tensor& t) { return c10::hip::getCurrentHIPStream(t.get_device()).stream(); }

// The binary hot path of the native dispatch (add / sub / mul, out-of-place or in
// place): every check, the allocation and the launch in C++, on the current stream.
// Returns None when the call does not fit (the Python handler's general path).
py::object bin(int op, const at::Tensor& self, const at::Tensor& other, double alpha, bool inplace) {
  const auto dt = self.scalar_type();
  if ((dt != c10::ScalarType::Float && dt != c10::ScalarType::BFloat16) || other.scalar_type() != dt ||
      !self.is_cuda() || !other.is_cuda() || self.dim() == 0 || self.sizes() != other.sizes() ||
      !self.is_contiguous() || !other.is_contiguous() || self.device() != other.device())
    return py::none();
  at::Tensor dst = inplace ? self : at::empty_like(self, at::MemoryFormat::Contiguous);
  const int code = dt_code(dt);
  const int rc = pa_ew_flat(op, 0, 2, dst.numel(), dst.data_ptr(), code, self.data_ptr(), code, other.data_ptr(), code,
                            nullptr, 0, alpha, 0.0, current_stream(self));
  TORCH_CHECK(rc == 0, "pa_ew_flat failed (rc=", rc, ")");
  return py::cast(dst);
}

c10::ScalarType from_code(int c) {
  switch (c) {
    case 0: return c10::ScalarType::Float;
    case 1: return c10::ScalarType::BFloat16;
    case 2: return c10::ScalarType::Half;
    case 3: return c10::ScalarType::Double;
    case 4: return c10::ScalarType::Long;
    case 5: return c10::ScalarType::Int;
    case 6: return c10::ScalarType::Short;
    case 7: return c10::ScalarType::Char;
    case 8: return c10::ScalarType::Byte;
    case 9: return c10::ScalarType::Bool;
    default: return c10::ScalarType::Undefined;
  }
}

// The cast / copy hot path of the native dispatch (_to_copy / clone of a contiguous
// device tensor into dtype code `dc`): allocation and launch in C++.  None when the
// call does not fit.
py::object cast(const at::Tensor& self, int dc) {
  const auto odt = from_code(dc);
  const int sc = dt_code(self.scalar_type());
  if (odt == c10::ScalarType::Undefined || sc < 0 || !self.is_cuda() || self.dim() == 0 || !self.is_contiguous())
    return py::none();
  at::Tensor dst = at::empty(self.sizes(), self.options().dtype(odt));
  if (self.numel() == 0) return py::cast(dst);
  // compute in the source's class unless a float is written from an integer source
  const int cdt = c10::isFloatingType(self.scalar_type()) || !c10::isFloatingType(odt) ? cdt_of(self.scalar_type())
                                                                                      : cdt_of(odt);
  const int rc = pa_ew_flat(0, cdt, 1, dst.numel(), dst.data_ptr(), dc, self.data_ptr(), sc, nullptr, 0, nullptr, 0,
                            0.0, 0.0, current_stream(self));
  TORCH_CHECK(rc == 0, "pa_ew_flat failed (rc=", rc, ")");
  return py::cast(dst);
}

// Direct framework callers: a += alpha * b, t[...] = v (current stream).
bool add_(const at::Tensor& a, const at::Tensor& b, double alpha) {
  const at::Tensor ins[2] = {a, b};
  return a.is_cuda() && launch(50, -1, a, ins, 2, alpha, 0.0, reinterpret_cast<int64_t>(current_stream(a)));
}

bool fill_(const at::Tensor& t, double v) {
  return t.is_cuda() && launch(1, -1, t, nullptr, 0, v, 0.0, reinterpret_cast<int64_t>(current_stream(t)));
}

}  // namespace

PYBIND11_MODULE(pa_fastops, m) {
  m.def("bin", &bin, "binary hot path (op, self, other, alpha, inplace) -> tensor or None");
  m.def("cast", &cast, "contiguous copy / cast into dtype code -> tensor or None");
  m.def("add_", &add_, "a += alpha * b on the current stream");
  m.def("fill_", &fill_, "t[...] = v on the current stream");
  m.doc() = "C++ launch entry for the framework's flat elementwise kernels";
  m.def("ew0", &ew0, "out = op() (fill / iota)");
  m.def("ew1", &ew1, "out = op(x)");
  m.def("ew2", &ew2, "out = op(x, y)");
  m.def("ew3", &ew3, "out = op(x, y, z)");
}
