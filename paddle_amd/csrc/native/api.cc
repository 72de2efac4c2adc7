// NativePaddlePredictor (reference inference/api/api_impl.cc: Init / Run / Clone,
// SetFeed / GetFetch) on the native executor, plus the C ABI the Python side uses
// (paddle_amd/native.py) to drive predictors, programs and scopes.
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <mutex>

#include "framework.h"
#include "paddle_inference_api.h"

namespace paddle {

// ---------------------------------------------------------------- PaddleBuf
PaddleBuf::PaddleBuf(PaddleBuf&& o) : data_(o.data_), length_(o.length_), memory_owned_(o.memory_owned_) {
  o.data_ = nullptr;
  o.length_ = 0;
  o.memory_owned_ = false;
}
PaddleBuf::PaddleBuf(const PaddleBuf& o) { *this = o; }
PaddleBuf& PaddleBuf::operator=(const PaddleBuf& o) {
  if (this == &o) return *this;
  Resize(o.length_);
  if (o.length_) memcpy(data_, o.data_, o.length_);
  return *this;
}
PaddleBuf& PaddleBuf::operator=(PaddleBuf&& o) {
  if (this == &o) return *this;
  Free();
  data_ = o.data_;
  length_ = o.length_;
  memory_owned_ = o.memory_owned_;
  o.data_ = nullptr;
  o.length_ = 0;
  o.memory_owned_ = false;
  return *this;
}
void PaddleBuf::Resize(size_t length) {
  if (length_ == length && memory_owned_) return;
  Free();
  data_ = length ? new char[length] : nullptr;
  length_ = length;
  memory_owned_ = true;
}
void PaddleBuf::Reset(void* data, size_t length) {
  Free();
  data_ = data;
  length_ = length;
  memory_owned_ = false;
}
void PaddleBuf::Free() {
  if (memory_owned_ && data_) delete[] static_cast<char*>(data_);
  data_ = nullptr;
  length_ = 0;
}

int PaddleDtypeSize(PaddleDType t) {
  switch (t) {
    case FLOAT32: return 4;
    case INT64: return 8;
    case INT32: return 4;
  }
  return 0;
}

static thread_local std::string g_last_error;
const std::string& LastError() { return g_last_error; }

namespace {
pa::DT to_dt(PaddleDType t) {
  switch (t) {
    case FLOAT32: return pa::DT::FP32;
    case INT64: return pa::DT::INT64;
    case INT32: return pa::DT::INT32;
  }
  pa::fail("unknown PaddleDType %d", (int)t);
}
PaddleDType from_dt(pa::DT t) {
  switch (t) {
    case pa::DT::FP32: return FLOAT32;
    case pa::DT::INT64: return INT64;
    case pa::DT::INT32: return INT32;
    default: pa::fail("output dtype %s has no PaddleDType", pa::dt_name(t));
  }
}

std::string dirname_of(const std::string& p) {
  auto k = p.find_last_of('/');
  return k == std::string::npos ? "." : p.substr(0, k);
}

// fc fusion (framework/ir/fc_fuse_pass.cc): mul(X, W) -> elementwise_add(., b) with
// a 1-D bias and no other reader of the mul output becomes one fc op.
void fuse_fc(pa::ProgramDesc* prog) {
  auto& ops = prog->blocks[0].ops;
  std::vector<pa::OpDesc> out;
  for (size_t i = 0; i < ops.size(); ++i) {
    const pa::OpDesc& m = ops[i];
    if (m.type == "mul" && i + 1 < ops.size() && ops[i + 1].type == "elementwise_add") {
      const pa::OpDesc& a = ops[i + 1];
      const std::string tmp = m.Output("Out");
      int readers = 0;
      for (auto& o : ops)
        for (auto& s : o.inputs)
          for (auto& n : s.second) readers += n == tmp;
      const pa::VarDesc* bv = prog->blocks[0].FindVar(a.Input("Y"));
      if (a.Input("X") == tmp && readers == 1 && m.GetInt("y_num_col_dims", 1) == 1 && bv && bv->persistable &&
          bv->dims.size() == 1) {
        pa::OpDesc fc;
        fc.type = "fc";
        fc.inputs = {{"Input", {m.Input("X")}}, {"W", {m.Input("Y")}}, {"Bias", {a.Input("Y")}}};
        fc.outputs = {{"Out", {a.Output("Out")}}};
        pa::Attr nc;
        nc.name = "in_num_col_dims";
        nc.type = pa::A_INT;
        nc.i = m.GetInt("x_num_col_dims", 1);
        fc.attrs[nc.name] = nc;
        out.push_back(std::move(fc));
        ++i;
        continue;
      }
    }
    out.push_back(m);
  }
  ops.swap(out);
}

class NativePredictor : public PaddlePredictor {
 public:
  NativePredictor(const NativeConfig& cfg, bool ir_optim) : cfg_(cfg) {
    const std::string prog_path = !cfg.prog_file.empty() ? cfg.prog_file : cfg.model_dir + "/__model__";
    prog_ = std::make_shared<pa::ProgramDesc>(pa::ProgramDesc::Load(prog_path));
    if (ir_optim) fuse_fc(prog_.get());
    device_ = cfg.use_gpu ? cfg.device : -1;
    if (device_ >= 0) PA_CHECK(pa::device_count() > device_, "use_gpu: HIP device %d not present", device_);
    exe_.reset(new pa::Executor(device_));
    exe_->context().is_test = true;
    params_ = std::make_shared<pa::Scope>();
    const std::string dir = !cfg.model_dir.empty() ? cfg.model_dir : dirname_of(prog_path);
    const std::string combined = cfg.param_file.empty() ? "" : cfg.param_file;
    pa::load_persistables(*prog_, params_.get(), dir, combined, device_, exe_->context().stream);
    init_io();
  }

  NativePredictor(const NativePredictor& o)
      : cfg_(o.cfg_), prog_(o.prog_), params_(o.params_), device_(o.device_), feeds_(o.feeds_), fetches_(o.fetches_) {
    exe_.reset(new pa::Executor(device_));
    exe_->context().is_test = true;
    local_.reset(new pa::Scope(params_.get()));
  }

  bool Run(const std::vector<PaddleTensor>& inputs, std::vector<PaddleTensor>* outputs, int) override {
    try {
      pa::Variable* feed = local_->Var("feed");
      feed->kind = pa::VK_FEED_MINIBATCH;
      feed->list.assign(feeds_.size(), pa::Tensor());
      PA_CHECK(inputs.size() == feeds_.size() || cfg_.specify_input_name, "Run: %zu inputs for %zu feed targets",
               inputs.size(), feeds_.size());
      for (size_t i = 0; i < inputs.size(); ++i) {
        const PaddleTensor& in = inputs[i];
        size_t col = i;
        if (cfg_.specify_input_name) {
          auto it = std::find(feeds_.begin(), feeds_.end(), in.name);
          PA_CHECK(it != feeds_.end(), "Run: no feed target named %s", in.name.c_str());
          col = (size_t)(it - feeds_.begin());
        }
        PA_CHECK(col < feeds_.size(), "Run: input %zu has no feed target", i);
        pa::Tensor t;
        std::vector<int64_t> dims(in.shape.begin(), in.shape.end());
        void* p = t.alloc(to_dt(in.dtype), dims, -1);
        PA_CHECK(in.data.length() >= t.nbytes(), "Run: input %s holds %zu bytes, shape needs %zu", in.name.c_str(),
                 in.data.length(), t.nbytes());
        memcpy(p, in.data.data(), t.nbytes());
        t.lod = in.lod;
        feed->list[col] = device_ >= 0 ? t.to(device_, exe_->context().stream) : t;
      }
      exe_->Run(*prog_, params_.get(), 0, local_.get());
      exe_->Sync();
      pa::Variable* fetch = local_->Find("fetch");
      PA_CHECK(fetch != nullptr, "Run: program has no fetch holder");
      outputs->clear();
      outputs->resize(fetches_.size());
      for (size_t i = 0; i < fetches_.size(); ++i) {
        PA_CHECK(i < fetch->list.size() && fetch->list[i].initialized(), "Run: fetch %zu not produced", i);
        const pa::Tensor& t = fetch->list[i];
        PaddleTensor& o = (*outputs)[i];
        o.name = fetches_[i];
        o.shape.assign(t.dims.begin(), t.dims.end());
        o.dtype = from_dt(t.dtype);
        o.lod = t.lod;
        o.data.Resize(t.nbytes());
        memcpy(o.data.data(), t.raw(), t.nbytes());
      }
      return true;
    } catch (const std::exception& e) {
      g_last_error = e.what();
      fprintf(stderr, "[paddle_amd predictor] %s\n", e.what());
      return false;
    }
  }

  std::unique_ptr<PaddlePredictor> Clone() override {
    return std::unique_ptr<PaddlePredictor>(new NativePredictor(*this));
  }

  pa::Executor& executor() { return *exe_; }

 private:
  void init_io() {
    local_.reset(new pa::Scope(params_.get()));
    const auto& ops = prog_->Block(0).ops;
    for (auto& op : ops) {
      if (op.type == "feed") {
        const size_t col = (size_t)op.GetInt("col");
        if (feeds_.size() <= col) feeds_.resize(col + 1);
        feeds_[col] = op.Output("Out");
      } else if (op.type == "fetch") {
        const size_t col = (size_t)op.GetInt("col");
        if (fetches_.size() <= col) fetches_.resize(col + 1);
        fetches_[col] = op.Input("X");
      }
    }
  }

  NativeConfig cfg_;
  std::shared_ptr<pa::ProgramDesc> prog_;
  std::shared_ptr<pa::Scope> params_;
  std::unique_ptr<pa::Scope> local_;
  std::unique_ptr<pa::Executor> exe_;
  int device_ = -1;
  std::vector<std::string> feeds_, fetches_;
};

std::unique_ptr<PaddlePredictor> make(const NativeConfig& c, bool ir) {
  try {
    return std::unique_ptr<PaddlePredictor>(new NativePredictor(c, ir));
  } catch (const std::exception& e) {
    g_last_error = e.what();
    fprintf(stderr, "[paddle_amd predictor] %s\n", e.what());
    return nullptr;
  }
}
}  // namespace

template <>
std::unique_ptr<PaddlePredictor> CreatePaddlePredictor<NativeConfig, PaddleEngineKind::kNative>(
    const NativeConfig& config) {
  return make(config, false);
}

template <>
std::unique_ptr<PaddlePredictor> CreatePaddlePredictor<NativeConfig, PaddleEngineKind::kAnalysis>(
    const NativeConfig& config) {
  return make(config, true);
}

template <>
std::unique_ptr<PaddlePredictor> CreatePaddlePredictor<AnalysisConfig, PaddleEngineKind::kAnalysis>(
    const AnalysisConfig& config) {
  return make(config, config.enable_ir_optim);
}

}  // namespace paddle

// ==================================================================== C ABI
#define PA_NAT_EXPORT extern "C" __attribute__((visibility("default")))

namespace {
struct CPredictor {
  std::unique_ptr<paddle::PaddlePredictor> p;
  std::vector<paddle::PaddleTensor> outs;
};
thread_local std::string c_err;

template <class F> int guard(F f) {
  try {
    return f();
  } catch (const std::exception& e) {
    c_err = e.what();
    return -1;
  }
}
}  // namespace

PA_NAT_EXPORT const char* pa_nat_last_error() {
  return !c_err.empty() ? c_err.c_str() : paddle::LastError().c_str();
}

PA_NAT_EXPORT void* pa_nat_create(const char* model_dir, const char* prog_file, const char* param_file, int use_gpu,
                                  int device, int ir_optim) {
  paddle::NativeConfig c;
  c.model_dir = model_dir ? model_dir : "";
  c.prog_file = prog_file ? prog_file : "";
  c.param_file = param_file ? param_file : "";
  c.use_gpu = use_gpu != 0;
  c.device = device;
  c.specify_input_name = false;
  auto p = ir_optim ? paddle::CreatePaddlePredictor<paddle::NativeConfig, paddle::PaddleEngineKind::kAnalysis>(c)
                    : paddle::CreatePaddlePredictor<paddle::NativeConfig>(c);
  if (!p) {
    c_err = paddle::LastError();
    return nullptr;
  }
  auto* h = new CPredictor();
  h->p = std::move(p);
  return h;
}

PA_NAT_EXPORT void* pa_nat_clone(void* h) {
  auto* c = new CPredictor();
  c->p = static_cast<CPredictor*>(h)->p->Clone();
  return c;
}

PA_NAT_EXPORT void pa_nat_destroy(void* h) { delete static_cast<CPredictor*>(h); }

// inputs: n tensors; dims flattened; lod: per input `lod_len[i]` level-1 offsets
// (0 = no LoD) flattened in `lod`.
PA_NAT_EXPORT int pa_nat_run(void* h, int n, const int* dtypes, const int* ndims, const int64_t* dims,
                             const void* const* data, const int64_t* lod, const int* lod_len) {
  return guard([&] {
    auto* c = static_cast<CPredictor*>(h);
    std::vector<paddle::PaddleTensor> ins((size_t)n);
    const int64_t* d = dims;
    const int64_t* l = lod;
    for (int i = 0; i < n; ++i) {
      auto& t = ins[(size_t)i];
      t.dtype = (paddle::PaddleDType)dtypes[i];
      size_t numel = 1;
      for (int k = 0; k < ndims[i]; ++k) {
        t.shape.push_back((int)d[k]);
        numel *= (size_t)d[k];
      }
      d += ndims[i];
      t.data.Reset(const_cast<void*>(data[i]), numel * (size_t)paddle::PaddleDtypeSize(t.dtype));
      if (lod_len && lod_len[i] > 0) {
        t.lod.push_back(std::vector<size_t>(l, l + lod_len[i]));
        l += lod_len[i];
      }
    }
    if (!c->p->Run(ins, &c->outs)) {
      c_err = paddle::LastError();
      return -1;
    }
    c_err.clear();
    return (int)c->outs.size();
  });
}

PA_NAT_EXPORT int pa_nat_output(void* h, int i, int* dtype, int* ndim, int64_t* dims, int dims_cap,
                                const void** data, size_t* nbytes) {
  auto* c = static_cast<CPredictor*>(h);
  if (i < 0 || (size_t)i >= c->outs.size()) return -1;
  auto& t = c->outs[(size_t)i];
  if ((int)t.shape.size() > dims_cap) return -1;
  *dtype = (int)t.dtype;
  *ndim = (int)t.shape.size();
  for (size_t k = 0; k < t.shape.size(); ++k) dims[k] = t.shape[k];
  *data = t.data.data();
  *nbytes = t.data.length();
  return 0;
}

// ------------------------------------------------------------ programs / scopes / executor
PA_NAT_EXPORT void* pa_nat_program_load(const char* path) {
  try {
    return new pa::ProgramDesc(pa::ProgramDesc::Load(path));
  } catch (const std::exception& e) {
    c_err = e.what();
    return nullptr;
  }
}
PA_NAT_EXPORT void* pa_nat_program_parse(const char* bytes, size_t n) {
  try {
    return new pa::ProgramDesc(pa::ProgramDesc::Parse(std::string(bytes, n)));
  } catch (const std::exception& e) {
    c_err = e.what();
    return nullptr;
  }
}
PA_NAT_EXPORT void pa_nat_program_free(void* p) { delete static_cast<pa::ProgramDesc*>(p); }
PA_NAT_EXPORT int pa_nat_program_num_ops(void* p, int block) {
  return (int)static_cast<pa::ProgramDesc*>(p)->Block(block).ops.size();
}

PA_NAT_EXPORT void* pa_nat_scope_new() { return new pa::Scope(); }
PA_NAT_EXPORT void pa_nat_scope_free(void* s) { delete static_cast<pa::Scope*>(s); }

PA_NAT_EXPORT void* pa_nat_executor_new(int device) {
  try {
    return new pa::Executor(device);
  } catch (const std::exception& e) {
    c_err = e.what();
    return nullptr;
  }
}
PA_NAT_EXPORT void pa_nat_executor_free(void* e) { delete static_cast<pa::Executor*>(e); }

PA_NAT_EXPORT int pa_nat_executor_run(void* e, void* prog, void* scope, int block) {
  return guard([&] {
    auto* ex = static_cast<pa::Executor*>(e);
    ex->Run(*static_cast<pa::ProgramDesc*>(prog), static_cast<pa::Scope*>(scope), block);
    ex->Sync();
    return 0;
  });
}

PA_NAT_EXPORT int pa_nat_scope_set(void* s, const char* name, int dtype, int ndim, const int64_t* dims,
                                   const void* data, int device) {
  return guard([&] {
    pa::Tensor t;
    void* p = t.alloc((pa::DT)dtype, std::vector<int64_t>(dims, dims + ndim), -1);
    memcpy(p, data, t.nbytes());
    pa::Variable* v = static_cast<pa::Scope*>(s)->Var(name);
    v->tensor = device >= 0 ? t.to(device) : t;
    return 0;
  });
}

// binds `name` to memory the caller owns (a torch tensor's storage): kernels read and
// update it in place; the executor never frees it
PA_NAT_EXPORT int pa_nat_scope_share(void* s, const char* name, int dtype, int ndim, const int64_t* dims, void* data,
                                     int device) {
  return guard([&] {
    pa::Tensor t;
    t.dtype = (pa::DT)dtype;
    t.dims.assign(dims, dims + ndim);
    t.device = device;
    t.buf = std::make_shared<pa::Buffer>(data, t.nbytes(), device);
    pa::Variable* v = static_cast<pa::Scope*>(s)->Var(name);
    v->tensor = t;
    return 0;
  });
}

// describes `name` without copying: 1 found (fields filled), 0 absent / uninitialised
PA_NAT_EXPORT int pa_nat_scope_info(void* s, const char* name, int* dtype, int* ndim, int64_t* dims, int dims_cap,
                                    void** data, int* device) {
  pa::Variable* v = static_cast<pa::Scope*>(s)->Find(name);
  if (!v || !v->tensor.initialized() || (int)v->tensor.dims.size() > dims_cap) return 0;
  const pa::Tensor& t = v->tensor;
  *dtype = (int)t.dtype;
  *ndim = (int)t.dims.size();
  for (size_t k = 0; k < t.dims.size(); ++k) dims[k] = t.dims[k];
  *data = t.raw();
  *device = t.device;
  return 1;
}

// synchronous copy between host (-1) / device memories
PA_NAT_EXPORT int pa_nat_copy(void* dst, int dst_dev, const void* src, int src_dev, size_t n) {
  return guard([&] {
    pa::device_copy(dst, dst_dev, src, src_dev, n, nullptr);
    if (dst_dev >= 0 && src_dev >= 0) pa::device_synchronize(dst_dev);
    return 0;
  });
}

// "type count" lines of the ops a device executor ran on host copies
PA_NAT_EXPORT int pa_nat_executor_fallbacks(void* e, char* buf, int cap) {
  std::string s;
  for (auto& kv : static_cast<pa::Executor*>(e)->host_fallbacks) s += kv.first + " " + std::to_string(kv.second) + "\n";
  if ((int)s.size() + 1 > cap) return -(int)s.size() - 1;
  memcpy(buf, s.c_str(), s.size() + 1);
  return (int)s.size();
}

// copies the tensor to host (kept alive in the scope variable `name@HOST` until the next call)
PA_NAT_EXPORT int pa_nat_scope_get(void* s, const char* name, int* dtype, int* ndim, int64_t* dims, int dims_cap,
                                   const void** data, size_t* nbytes) {
  return guard([&] {
    auto* sc = static_cast<pa::Scope*>(s);
    pa::Variable* v = sc->Find(name);
    PA_CHECK(v && v->tensor.initialized(), "variable %s not found or empty", name);
    pa::Variable* h = sc->Var(std::string(name) + "@HOST");
    h->tensor = v->tensor.device >= 0 ? v->tensor.to(-1) : v->tensor;
    const pa::Tensor& t = h->tensor;
    PA_CHECK((int)t.dims.size() <= dims_cap, "rank too large");
    *dtype = (int)t.dtype;
    *ndim = (int)t.dims.size();
    for (size_t k = 0; k < t.dims.size(); ++k) dims[k] = t.dims[k];
    *data = t.raw();
    *nbytes = t.nbytes();
    return 0;
  });
}

PA_NAT_EXPORT int pa_nat_load_persistables(void* prog, void* scope, const char* dir, const char* combined,
                                           int device) {
  return guard([&] {
    pa::load_persistables(*static_cast<pa::ProgramDesc*>(prog), static_cast<pa::Scope*>(scope), dir ? dir : "",
                          combined ? combined : "", device, nullptr);
    return 0;
  });
}

PA_NAT_EXPORT int pa_nat_registered_ops(char* buf, int cap, int device) {
  pa::link_host_kernels();
  if (device) pa::link_device_kernels();
  std::string s;
  auto v = pa::registered_ops(device != 0);
  std::sort(v.begin(), v.end());
  for (auto& n : v) s += n + "\n";
  if ((int)s.size() + 1 > cap) return -(int)s.size() - 1;
  memcpy(buf, s.c_str(), s.size() + 1);
  return (int)s.size();
}
