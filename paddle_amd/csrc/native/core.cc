// Native executor core: error reporting, dtypes, ProgramDesc wire-format decoding,
// tensors / scopes, host worker pool, kernel registry, Executor, LoDTensor IO.
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <fstream>
#include <set>
#include <sstream>
#include <thread>

#include "framework.h"

namespace pa {

void fail(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  throw Error(buf);
}

size_t dt_size(DT t) {
  switch (t) {
    case DT::BOOL: case DT::UINT8: case DT::INT8: return 1;
    case DT::INT16: case DT::FP16: case DT::BF16: return 2;
    case DT::INT32: case DT::FP32: return 4;
    case DT::INT64: case DT::FP64: return 8;
  }
  fail("unsupported dtype %d", (int)t);
}

const char* dt_name(DT t) {
  switch (t) {
    case DT::BOOL: return "bool";
    case DT::INT16: return "int16";
    case DT::INT32: return "int32";
    case DT::INT64: return "int64";
    case DT::FP16: return "float16";
    case DT::FP32: return "float32";
    case DT::FP64: return "float64";
    case DT::UINT8: return "uint8";
    case DT::INT8: return "int8";
    case DT::BF16: return "bfloat16";
  }
  return "?";
}

// ================================================================ OpDesc accessors
static const std::vector<std::string> kEmpty;

const std::vector<std::string>& OpDesc::Inputs(const std::string& slot) const {
  for (auto& kv : inputs)
    if (kv.first == slot) return kv.second;
  return kEmpty;
}
const std::vector<std::string>& OpDesc::Outputs(const std::string& slot) const {
  for (auto& kv : outputs)
    if (kv.first == slot) return kv.second;
  return kEmpty;
}
std::string OpDesc::Input(const std::string& slot) const {
  auto& v = Inputs(slot);
  return v.empty() ? "" : v[0];
}
std::string OpDesc::Output(const std::string& slot) const {
  auto& v = Outputs(slot);
  return v.empty() ? "" : v[0];
}
int64_t OpDesc::GetInt(const std::string& a, int64_t def) const {
  auto it = attrs.find(a);
  if (it == attrs.end()) return def;
  if (it->second.type == A_FLOAT) return (int64_t)it->second.f;
  return it->second.i;
}
float OpDesc::GetFloat(const std::string& a, float def) const {
  auto it = attrs.find(a);
  if (it == attrs.end()) return def;
  if (it->second.type == A_FLOAT) return it->second.f;
  return (float)it->second.i;
}
bool OpDesc::GetBool(const std::string& a, bool def) const {
  auto it = attrs.find(a);
  return it == attrs.end() ? def : it->second.i != 0;
}
std::string OpDesc::GetString(const std::string& a, const std::string& def) const {
  auto it = attrs.find(a);
  return it == attrs.end() ? def : it->second.s;
}
std::vector<int64_t> OpDesc::GetInts(const std::string& a) const {
  auto it = attrs.find(a);
  if (it == attrs.end()) return {};
  if (it->second.type == A_INT || it->second.type == A_LONG) return {it->second.i};
  return it->second.ints;
}
std::vector<float> OpDesc::GetFloats(const std::string& a) const {
  auto it = attrs.find(a);
  return it == attrs.end() ? std::vector<float>{} : it->second.floats;
}

const VarDesc* BlockDesc::FindVar(const std::string& n) const {
  for (auto& v : vars)
    if (v.name == n) return &v;
  return nullptr;
}

// ================================================================ proto2 decoding
// Minimal wire-format reader: varint (0), fixed64 (1), length-delimited (2),
// fixed32 (5).  Repeated scalars are accepted both packed and unpacked.
namespace {
struct Reader {
  const unsigned char* p;
  const unsigned char* end;

  bool more() const { return p < end; }
  uint64_t varint() {
    uint64_t v = 0;
    for (int shift = 0; shift < 64; shift += 7) {
      PA_CHECK(p < end, "ProgramDesc: truncated varint");
      uint8_t b = *p++;
      v |= (uint64_t)(b & 0x7f) << shift;
      if (!(b & 0x80)) return v;
    }
    fail("ProgramDesc: varint too long");
  }
  Reader sub() {
    uint64_t n = varint();
    PA_CHECK(n <= (uint64_t)(end - p), "ProgramDesc: length %llu runs past the message",
             (unsigned long long)n);
    Reader r{p, p + n};
    p += n;
    return r;
  }
  std::string str() {
    Reader r = sub();
    return std::string((const char*)r.p, (size_t)(r.end - r.p));
  }
  float f32() {
    PA_CHECK(end - p >= 4, "ProgramDesc: truncated fixed32");
    float f;
    memcpy(&f, p, 4);
    p += 4;
    return f;
  }
  void skip(int wt) {
    switch (wt) {
      case 0: varint(); break;
      case 1: PA_CHECK(end - p >= 8, "ProgramDesc: truncated fixed64"); p += 8; break;
      case 2: sub(); break;
      case 5: PA_CHECK(end - p >= 4, "ProgramDesc: truncated fixed32"); p += 4; break;
      default: fail("ProgramDesc: unsupported wire type %d", wt);
    }
  }
  template <class F> void ints(int wt, F push) {  // repeated varint field
    if (wt == 2) {
      Reader r = sub();
      while (r.more()) push((int64_t)r.varint());
    } else {
      push((int64_t)varint());
    }
  }
};

int64_t zz32(uint64_t v) { return (int64_t)(int32_t)(uint32_t)v; }  // int32 stored as varint

Attr parse_attr(Reader r) {
  Attr a;
  while (r.more()) {
    uint64_t tag = r.varint();
    int fn = (int)(tag >> 3), wt = (int)(tag & 7);
    switch (fn) {
      case 1: a.name = r.str(); break;
      case 2: a.type = (int)r.varint(); break;
      case 3: a.i = zz32(r.varint()); break;
      case 4: a.f = r.f32(); break;
      case 5: a.s = r.str(); break;
      case 6: r.ints(wt, [&](int64_t v) { a.ints.push_back((int64_t)(int32_t)v); }); break;
      case 7:
        if (wt == 2) {
          Reader s = r.sub();
          while (s.more()) a.floats.push_back(s.f32());
        } else {
          a.floats.push_back(r.f32());
        }
        break;
      case 8: a.strings.push_back(r.str()); break;
      case 10: a.i = (int64_t)r.varint(); break;
      case 11: r.ints(wt, [&](int64_t v) { a.ints.push_back(v != 0); }); break;
      case 12: a.i = zz32(r.varint()); break;
      case 13: a.i = (int64_t)r.varint(); break;
      case 14: r.ints(wt, [&](int64_t v) { a.ints.push_back(v); }); break;
      default: r.skip(wt);
    }
  }
  return a;
}

std::pair<std::string, std::vector<std::string>> parse_opvar(Reader r) {
  std::pair<std::string, std::vector<std::string>> v;
  while (r.more()) {
    uint64_t tag = r.varint();
    int fn = (int)(tag >> 3), wt = (int)(tag & 7);
    if (fn == 1) v.first = r.str();
    else if (fn == 2) v.second.push_back(r.str());
    else r.skip(wt);
  }
  return v;
}

OpDesc parse_op(Reader r) {
  OpDesc op;
  while (r.more()) {
    uint64_t tag = r.varint();
    int fn = (int)(tag >> 3), wt = (int)(tag & 7);
    switch (fn) {
      case 1: op.inputs.push_back(parse_opvar(r.sub())); break;
      case 2: op.outputs.push_back(parse_opvar(r.sub())); break;
      case 3: op.type = r.str(); break;
      case 4: {
        Attr a = parse_attr(r.sub());
        std::string n = a.name;
        op.attrs[n] = std::move(a);
        break;
      }
      default: r.skip(wt);
    }
  }
  return op;
}

void parse_tensor_desc(Reader r, VarDesc* v) {
  while (r.more()) {
    uint64_t tag = r.varint();
    int fn = (int)(tag >> 3), wt = (int)(tag & 7);
    if (fn == 1) v->dtype = (DT)r.varint();
    else if (fn == 2) r.ints(wt, [&](int64_t d) { v->dims.push_back(d); });
    else r.skip(wt);
  }
}

void parse_lod_desc(Reader r, VarDesc* v) {
  while (r.more()) {
    uint64_t tag = r.varint();
    int fn = (int)(tag >> 3), wt = (int)(tag & 7);
    if (fn == 1) parse_tensor_desc(r.sub(), v);
    else if (fn == 2) v->lod_level = (int)r.varint();
    else r.skip(wt);
  }
}

void parse_vartype(Reader r, VarDesc* v) {
  while (r.more()) {
    uint64_t tag = r.varint();
    int fn = (int)(tag >> 3), wt = (int)(tag & 7);
    if (fn == 1) v->type = (int)r.varint();
    else if (fn == 2) parse_tensor_desc(r.sub(), v);  // selected_rows
    else if (fn == 3 || fn == 4) parse_lod_desc(r.sub(), v);  // lod_tensor / tensor_array
    else r.skip(wt);
  }
}

VarDesc parse_var(Reader r) {
  VarDesc v;
  while (r.more()) {
    uint64_t tag = r.varint();
    int fn = (int)(tag >> 3), wt = (int)(tag & 7);
    if (fn == 1) v.name = r.str();
    else if (fn == 2) parse_vartype(r.sub(), &v);
    else if (fn == 3) v.persistable = r.varint() != 0;
    else r.skip(wt);
  }
  return v;
}

BlockDesc parse_block(Reader r) {
  BlockDesc b;
  while (r.more()) {
    uint64_t tag = r.varint();
    int fn = (int)(tag >> 3), wt = (int)(tag & 7);
    switch (fn) {
      case 1: b.idx = (int)zz32(r.varint()); break;
      case 2: b.parent_idx = (int)zz32(r.varint()); break;
      case 3: b.vars.push_back(parse_var(r.sub())); break;
      case 4: b.ops.push_back(parse_op(r.sub())); break;
      case 5: b.forward_block_idx = (int)zz32(r.varint()); break;
      default: r.skip(wt);
    }
  }
  return b;
}
}  // namespace

ProgramDesc ProgramDesc::Parse(const std::string& bytes) {
  ProgramDesc prog;
  Reader r{(const unsigned char*)bytes.data(), (const unsigned char*)bytes.data() + bytes.size()};
  while (r.more()) {
    uint64_t tag = r.varint();
    if ((tag >> 3) == 1 && (tag & 7) == 2) prog.blocks.push_back(parse_block(r.sub()));
    else r.skip((int)(tag & 7));
  }
  PA_CHECK(!prog.blocks.empty(), "ProgramDesc: no blocks");
  return prog;
}

ProgramDesc ProgramDesc::Load(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  PA_CHECK((bool)f, "cannot open program file %s", path.c_str());
  std::stringstream ss;
  ss << f.rdbuf();
  return Parse(ss.str());
}

// ================================================================ buffers / tensors
Buffer::Buffer(size_t n, int dev) : bytes(n), device(dev) {
  size_t sz = n ? n : 1;
  if (dev < 0) {
    ptr = aligned_alloc(64, (sz + 63) / 64 * 64);
    PA_CHECK(ptr != nullptr, "host allocation of %zu bytes failed", n);
  } else {
    ptr = device_alloc(sz, dev);
  }
}

Buffer::~Buffer() {
  if (!owned) return;
  if (device < 0) free(ptr);
  else device_free(ptr, device);
}

int64_t Tensor::numel() const {
  int64_t n = 1;
  for (auto d : dims) n *= d;
  return n;
}

void* Tensor::alloc(DT t, const std::vector<int64_t>& d, int dev) {
  for (auto x : d) PA_CHECK(x >= 0, "negative dimension in %s", shape_str().c_str());
  dtype = t;
  dims = d;
  const size_t need = nbytes();
  if (!buf || buf->device != dev || buf->bytes < need || buf.use_count() > 1)
    buf = std::make_shared<Buffer>(need, dev);
  device = dev;
  return buf->ptr;
}

template <class T> T* Tensor::alloc(const std::vector<int64_t>& d, int dev) {
  DT t = std::is_same<T, float>::value ? DT::FP32
         : std::is_same<T, int64_t>::value ? DT::INT64
         : std::is_same<T, int32_t>::value ? DT::INT32
         : std::is_same<T, double>::value ? DT::FP64
         : std::is_same<T, uint8_t>::value ? DT::UINT8
                                           : DT::BOOL;
  return static_cast<T*>(alloc(t, d, dev));
}
template float* Tensor::alloc<float>(const std::vector<int64_t>&, int);
template int64_t* Tensor::alloc<int64_t>(const std::vector<int64_t>&, int);
template int32_t* Tensor::alloc<int32_t>(const std::vector<int64_t>&, int);
template double* Tensor::alloc<double>(const std::vector<int64_t>&, int);
template uint8_t* Tensor::alloc<uint8_t>(const std::vector<int64_t>&, int);

Tensor Tensor::to(int dev, void* stream) const {
  Tensor o;
  o.lod = lod;
  o.alloc(dtype, dims, dev);
  if (nbytes()) device_copy(o.raw(), dev, raw(), device, nbytes(), stream);
  return o;
}

std::string Tensor::shape_str() const {
  std::string s = "[";
  for (size_t i = 0; i < dims.size(); ++i) s += (i ? ", " : "") + std::to_string(dims[i]);
  return s + "]";
}

// ================================================================ scopes
Variable* Scope::Var(const std::string& name) {
  std::lock_guard<std::mutex> g(mu_);
  auto& v = vars_[name];
  if (!v) v.reset(new Variable());
  return v.get();
}

Variable* Scope::FindLocal(const std::string& name) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = vars_.find(name);
  return it == vars_.end() ? nullptr : it->second.get();
}

Variable* Scope::Find(const std::string& name) const {
  for (const Scope* s = this; s; s = s->parent_) {
    Variable* v = s->FindLocal(name);
    if (v) return v;
  }
  return nullptr;
}

Scope& Scope::NewScope() {
  std::lock_guard<std::mutex> g(mu_);
  kids_.emplace_back(new Scope(this));
  return *kids_.back();
}

void Scope::DropKid(Scope* kid) {
  std::lock_guard<std::mutex> g(mu_);
  for (auto it = kids_.begin(); it != kids_.end(); ++it)
    if (it->get() == kid) {
      kids_.erase(it);
      return;
    }
}

void Scope::Erase(const std::string& name) {
  std::lock_guard<std::mutex> g(mu_);
  vars_.erase(name);
}

Scope& Scope::Root() {
  Scope* s = this;
  while (s->parent_) s = const_cast<Scope*>(s->parent_);
  return *s;
}

std::vector<std::string> Scope::LocalNames() const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::string> out;
  for (auto& kv : vars_) out.push_back(kv.first);
  return out;
}

// ================================================================ host worker pool
// Each parallel_for publishes one Job; a worker takes a reference to the job under
// the pool mutex and only ever touches that job's own counters, so a worker that
// wakes late (after its job finished, or while the next job is being published)
// can neither run a finished job's functor nor mix two jobs' chunk geometry.
struct ThreadPool {
  struct Job {
    const std::function<void(int64_t, int64_t)>* fn;
    int64_t n, chunk;
    std::atomic<int64_t> next{0};
    int active = 0;  // workers inside drain(), guarded by the pool mutex
  };
  std::vector<std::thread> workers;
  std::mutex mu;
  std::condition_variable cv, done_cv;
  std::shared_ptr<Job> cur;  // guarded by mu
  bool stop = false;
  std::mutex run_mu;  // one parallel_for at a time (nested calls run serially)

  explicit ThreadPool(int nt) {
    for (int i = 0; i < nt; ++i) workers.emplace_back([this] { loop(); });
  }
  ~ThreadPool() {
    {
      std::lock_guard<std::mutex> g(mu);
      stop = true;
    }
    cv.notify_all();
    for (auto& t : workers) t.join();
  }
  static void drain(Job& j) {
    for (;;) {
      const int64_t b = j.next.fetch_add(j.chunk);
      if (b >= j.n) return;
      (*j.fn)(b, std::min(j.n, b + j.chunk));
    }
  }
  void loop() {
    const Job* last = nullptr;
    for (;;) {
      std::shared_ptr<Job> j;
      {
        std::unique_lock<std::mutex> l(mu);
        cv.wait(l, [&] { return stop || (cur && cur.get() != last); });
        if (stop) return;
        j = cur;
        last = j.get();
        ++j->active;
      }
      drain(*j);
      {
        std::lock_guard<std::mutex> g(mu);
        if (--j->active == 0) done_cv.notify_all();
      }
    }
  }
  void run(int64_t total, int64_t ch, const std::function<void(int64_t, int64_t)>& fn) {
    std::unique_lock<std::mutex> busy(run_mu, std::try_to_lock);
    if (!busy.owns_lock() || workers.empty()) {  // nested or single-threaded
      fn(0, total);
      return;
    }
    auto j = std::make_shared<Job>();
    j->fn = &fn;
    j->n = total;
    j->chunk = ch;
    {
      std::lock_guard<std::mutex> g(mu);
      cur = j;
    }
    cv.notify_all();
    drain(*j);
    std::unique_lock<std::mutex> l(mu);
    done_cv.wait(l, [&] { return j->active == 0; });
    cur.reset();
  }
};

static int pool_threads() {
  const char* e = getenv("PADDLE_NUM_THREADS");
  int n = e ? atoi(e) : (int)std::thread::hardware_concurrency();
  if (n > 32) n = 32;  // host kernels are a fallback path: bounded footprint
  return n > 1 ? n - 1 : 0;
}

ThreadPool& host_pool() {
  static ThreadPool pool(pool_threads());
  return pool;
}

void parallel_for(int64_t n, int64_t grain, const std::function<void(int64_t, int64_t)>& fn) {
  if (n <= 0) return;
  ThreadPool& p = host_pool();
  const int64_t nt = (int64_t)p.workers.size() + 1;
  if (n < 2 * grain || nt == 1) {
    fn(0, n);
    return;
  }
  int64_t chunk = std::max<int64_t>(grain, (n + 4 * nt - 1) / (4 * nt));
  p.run(n, chunk, fn);
}

// ================================================================ registry
namespace {
std::unordered_map<std::string, Kernel>& reg(bool device) {
  static std::unordered_map<std::string, Kernel> host, dev;
  return device ? dev : host;
}
}  // namespace

void register_kernel(const std::string& type, bool device, Kernel k) { reg(device)[type] = std::move(k); }

// FLAGS_native_py_ops=a,b,...: these op types run on the embedder's fallback (the
// Python op library) even where a C++ kernel exists -- for bisecting an engine
// divergence one op family at a time (fluid/native_engine.py reads the same flag)
static const std::set<std::string>& forced_fallback() {
  static const std::set<std::string> s = [] {
    std::set<std::string> out;
    const char* e = getenv("FLAGS_native_py_ops");
    std::string cur;
    for (const char* c = e ? e : ""; ; ++c) {
      if (*c == ',' || *c == 0) {
        if (!cur.empty()) out.insert(cur);
        cur.clear();
        if (*c == 0) break;
      } else {
        cur += *c;
      }
    }
    return out;
  }();
  return s;
}

const Kernel* find_kernel(const std::string& type, bool device) {
  if (!forced_fallback().empty() && forced_fallback().count(type)) return nullptr;
  auto& r = reg(device);
  auto it = r.find(type);
  return it == r.end() ? nullptr : &it->second;
}

std::vector<std::string> registered_ops(bool device) {
  std::vector<std::string> out;
  for (auto& kv : reg(device))
    if (!forced_fallback().count(kv.first)) out.push_back(kv.first);
  return out;
}

// ================================================================ OpRun helpers
Variable* OpRun::var(const std::string& name) const {
  Variable* v = scope.Find(name);
  PA_CHECK(v != nullptr, "%s: variable %s not found", op.type.c_str(), name.c_str());
  return v;
}

Tensor& OpRun::in(const std::string& slot, size_t i) const {
  auto& names = op.Inputs(slot);
  PA_CHECK(i < names.size(), "%s: missing input %s[%zu]", op.type.c_str(), slot.c_str(), i);
  Tensor& t = var(names[i])->tensor;
  PA_CHECK(t.initialized(), "%s: input %s (%s) is not initialised", op.type.c_str(), slot.c_str(),
           names[i].c_str());
  return t;
}

Tensor* OpRun::in_opt(const std::string& slot, size_t i) const {
  auto& names = op.Inputs(slot);
  if (i >= names.size()) return nullptr;
  Variable* v = scope.Find(names[i]);
  return v && v->tensor.initialized() ? &v->tensor : nullptr;
}

std::vector<Tensor*> OpRun::ins(const std::string& slot) const {
  std::vector<Tensor*> out;
  for (size_t i = 0; i < op.Inputs(slot).size(); ++i) out.push_back(&in(slot, i));
  return out;
}

Tensor* OpRun::out(const std::string& slot, size_t i) const {
  Variable* v = out_var(slot, i);
  return v ? &v->tensor : nullptr;
}

Variable* OpRun::in_var(const std::string& slot, size_t i) const {
  auto& names = op.Inputs(slot);
  PA_CHECK(i < names.size(), "%s: missing input %s[%zu]", op.type.c_str(), slot.c_str(), i);
  return var(names[i]);
}

Variable* OpRun::out_var(const std::string& slot, size_t i) const {
  auto& names = op.Outputs(slot);
  if (i >= names.size() || names[i].empty() || names[i] == "@EMPTY@") return nullptr;
  Variable* v = scope.Find(names[i]);
  if (!v) v = scope.Var(names[i]);
  return v;
}

// ================================================================ executor
Executor::Executor(int device) {
  ctx_.device = device;
  const char* sn = getenv("FLAGS_strict_native");
  strict_native = sn && (strcmp(sn, "1") == 0 || strcmp(sn, "true") == 0 || strcmp(sn, "True") == 0);
  if (device >= 0) {
    link_device_kernels();
    own_stream_ = ctx_.stream = device_stream_create(device);
  }
  link_host_kernels();
  link_control_kernels();
  link_rnn_kernels();
  link_struct_kernels();
  link_beam_kernels();
  link_optim_kernels();
  link_seq_kernels();
  link_io_kernels();
  link_tensor_kernels();
  link_rnn_unit_kernels();
  link_conv3d_kernels();
  link_loss_kernels();
  link_misc_kernels();
  link_more_kernels();
  link_extra_kernels();
}

Executor::~Executor() {
  if (own_stream_) device_stream_destroy(own_stream_);
}

void Executor::SetStream(void* stream) {
  if (ctx_.device < 0) return;
  ctx_.stream = stream ? stream : own_stream_;
}

bool Executor::ReadBool(const Tensor& t) {
  PA_CHECK(t.initialized() && t.numel() >= 1, "control flow: condition tensor is empty");
  if (t.device < 0) {
    switch (t.dtype) {
      case DT::BOOL: case DT::UINT8: case DT::INT8: return *t.data<uint8_t>() != 0;
      case DT::INT32: return *t.data<int32_t>() != 0;
      case DT::INT64: return *t.data<int64_t>() != 0;
      case DT::FP32: return *t.data<float>() != 0.f;
      default: fail("control flow: unsupported condition dtype %s", dt_name(t.dtype));
    }
  }
  Tensor h = t.to(-1, ctx_.stream);
  device_stream_sync(ctx_.stream);
  return ReadBool(h);
}

// while_op.cc: run the sub-block while Condition holds; variables of enclosing
// scopes are updated in place.  Inference (is_test, or no StepScopes output): one
// child scope holds the body's temporaries for the whole loop.  Training: every
// iteration runs in a fresh child scope that is KEPT in the StepScopes variable
// (kStepScopes), so the step-local activations survive for while_grad; the scopes
// of the previous run are dropped when the loop runs again.
void Executor::RunWhile(const ProgramDesc& prog, const OpDesc& op, Scope* scope) {
  const int sb = (int)op.GetInt("sub_block", -1);
  PA_CHECK(sb >= 0 && sb < (int)prog.blocks.size(), "while: bad sub_block %d", sb);
  const std::string cond = op.Input("Condition");
  Variable* cv = scope->Find(cond);
  PA_CHECK(cv != nullptr, "while: condition %s not found", cond.c_str());
  const BlockDesc& blk = prog.Block(sb);
  auto declare = [&](Scope& s) {
    for (const VarDesc& v : blk.vars)
      if (!scope->Find(v.name)) s.Var(v.name)->kind = v.type;
  };
  const std::string ss = op.Output("StepScopes");
  const bool keep = !ss.empty() && !op.GetBool("is_test", false) && !ctx_.is_test;
  int64_t iters = 0;
  if (!keep) {
    Scope& body = scope->NewScope();
    declare(body);
    while (ReadBool(cv->tensor)) {
      RunBlock(prog, blk, &body);
      PA_CHECK(++iters < (int64_t)1 << 40, "while: runaway loop");
    }
    scope->DropKid(&body);  // device buffers of the body's temporaries are stream-ordered frees
    return;
  }
  Variable* sv = scope->Find(ss);
  if (!sv) sv = scope->Var(ss);
  sv->kind = VK_STEP_SCOPES;
  for (Scope* s : sv->steps) sv->steps_owner->DropKid(s);
  sv->steps.clear();
  sv->steps_owner = scope;
  while (ReadBool(cv->tensor)) {
    Scope& step = scope->NewScope();
    sv->steps.push_back(&step);
    declare(step);
    RunBlock(prog, blk, &step);
    PA_CHECK(++iters < (int64_t)1 << 40, "while: runaway loop");
  }
}

namespace {
// acc += x for fp32 tensors on one place; an empty `acc` takes a private copy of x
void accumulate_into(Tensor& acc, const Tensor& x, void* stream) {
  PA_CHECK(x.dtype == DT::FP32, "while_grad: gradient %s is not float32", dt_name(x.dtype));
  if (!acc.initialized()) {
    acc.alloc(DT::FP32, x.dims, x.device);
    device_copy(acc.raw(), x.device, x.raw(), x.device, x.nbytes(), stream);
    return;
  }
  PA_CHECK(acc.numel() == x.numel() && acc.device == x.device, "while_grad: step gradients differ in shape");
  if (x.device >= 0) {
    device_add_f32(stream, acc.data<float>(), x.data<float>(), x.numel());
  } else {
    float* a = acc.data<float>();
    const float* b = x.data<float>();
    for (int64_t i = 0; i < x.numel(); ++i) a[i] += b[i];
  }
}
}  // namespace

// while_op.cc WhileGradOp::RunImpl: the grad block runs once per kept step scope,
// last step first, each time in a fresh child of that step scope (so it reads the
// step's forward activations).  Gradients of tensor ARRAYS (DynamicRNN memories and
// outputs) are ONE variable in the enclosing scope shared by every step (slot t
// written by reverse step t is read by reverse step t - 1); gradients of dense
// loop-invariant inputs (parameters, static inputs) are step-local and summed into
// the enclosing X@GRAD; an input no step produced a gradient for gets zeros.
void Executor::RunWhileGrad(const ProgramDesc& prog, const OpDesc& op, Scope* scope) {
  const int sb = (int)op.GetInt("sub_block", -1);
  PA_CHECK(sb >= 0 && sb < (int)prog.blocks.size(), "while_grad: bad sub_block %d", sb);
  const BlockDesc& blk = prog.Block(sb);
  const auto& xs = op.Inputs("X");
  const auto& xgs = op.Outputs("X@GRAD");
  Variable* sv = scope->Find(op.Input("StepScopes"));
  PA_CHECK(sv != nullptr, "while_grad: step scopes %s not found", op.Input("StepScopes").c_str());
  std::set<std::string> arrays, shared;
  auto note_array = [&](const std::string& n) {
    Variable* v = scope->Find(n);
    if (!v || v->kind != VK_LOD_TENSOR_ARRAY) return;
    arrays.insert(n);
    const std::string gn = n + "@GRAD";
    Variable* gv = scope->Find(gn);
    if (!gv) gv = scope->Var(gn);
    if (gv->kind != VK_LOD_TENSOR_ARRAY) {
      gv->kind = VK_LOD_TENSOR_ARRAY;
      gv->list.clear();
      gv->tensor = Tensor();
    }
    shared.insert(gn);
  };
  for (auto& n : xs) note_array(n);
  for (auto& n : op.Inputs("Out")) note_array(n);
  // incoming output gradients live in the enclosing scope: never shadowed per step
  const std::set<std::string> out_grads(op.Inputs("Out@GRAD").begin(), op.Inputs("Out@GRAD").end());
  std::map<std::string, Tensor> acc;
  for (size_t k = sv->steps.size(); k-- > 0;) {
    Scope* s = sv->steps[k];
    Scope& gs = s->NewScope();
    for (const VarDesc& v : blk.vars)
      if (!v.persistable && !shared.count(v.name) && !out_grads.count(v.name)) gs.Var(v.name)->kind = v.type;
    for (size_t i = 0; i < xs.size() && i < xgs.size(); ++i)
      if (xgs[i] != "@EMPTY@" && !arrays.count(xs[i]) && !gs.FindLocal(xgs[i])) gs.Var(xgs[i]);
    RunBlock(prog, blk, &gs);
    for (size_t i = 0; i < xs.size() && i < xgs.size(); ++i) {
      if (xgs[i] == "@EMPTY@" || arrays.count(xs[i])) continue;
      Variable* g = gs.FindLocal(xgs[i]);
      if (g && g->tensor.initialized()) accumulate_into(acc[xgs[i]], g->tensor, ctx_.stream);
    }
    s->DropKid(&gs);
  }
  for (size_t i = 0; i < xs.size() && i < xgs.size(); ++i) {
    if (xgs[i] == "@EMPTY@" || arrays.count(xs[i])) continue;
    Variable* x = scope->Find(xs[i]);
    Variable* out = scope->Find(xgs[i]);
    if (!out) out = scope->Var(xgs[i]);
    out->kind = VK_LOD_TENSOR;
    auto it = acc.find(xgs[i]);
    if (it != acc.end()) {
      out->tensor = it->second;
      if (x) out->tensor.lod = x->tensor.lod;
    } else if (x && x->tensor.initialized() && x->tensor.dtype == DT::FP32) {
      Tensor z;
      z.alloc(DT::FP32, x->tensor.dims, x->tensor.device);
      if (z.device >= 0) device_fill(ctx_.stream, z.raw(), DT::FP32, z.numel(), 0.0);
      else std::fill_n(z.data<float>(), z.numel(), 0.f);
      z.lod = x->tensor.lod;
      out->tensor = z;
    }
  }
}

namespace {
const std::vector<std::string>& str_attr(const OpDesc& op, const char* name) {
  static const std::vector<std::string> none;
  auto it = op.attrs.find(name);
  return it == op.attrs.end() ? none : it->second.strings;
}

// a [T, ...] tensor's row t as a fresh tensor on its own place
Tensor time_row(const Tensor& x, int64_t t, void* stream) {
  Tensor r;
  std::vector<int64_t> d(x.dims.begin() + 1, x.dims.end());
  r.alloc(x.dtype, d, x.device);
  const size_t rb = r.nbytes();
  device_copy(r.raw(), r.device, static_cast<const char*>(x.raw()) + (size_t)t * rb, x.device, rb, stream);
  return r;
}

// dst[t] = src, allocating dst as [T] + src.dims (zero-filled) on the first write
void put_row(Tensor& dst, int64_t T, int64_t t, const Tensor& src, void* stream) {
  std::vector<int64_t> d{T};
  d.insert(d.end(), src.dims.begin(), src.dims.end());
  if (!dst.initialized() || dst.dims != d || dst.device != src.device || dst.dtype != src.dtype) {
    dst = Tensor();
    dst.alloc(src.dtype, d, src.device);
    if (dst.device >= 0) device_fill(stream, dst.raw(), dst.dtype, dst.numel(), 0.0);
    else memset(dst.raw(), 0, dst.nbytes());
  }
  const size_t rb = src.nbytes();
  device_copy(static_cast<char*>(dst.raw()) + (size_t)t * rb, dst.device, src.raw(), src.device, rb, stream);
}

Tensor zeros_like_f32(const Tensor& x, void* stream) {
  Tensor z;
  z.alloc(DT::FP32, x.dims, x.device);
  if (z.device >= 0) device_fill(stream, z.raw(), DT::FP32, z.numel(), 0.0);
  else std::fill_n(z.data<float>(), z.numel(), 0.f);
  return z;
}
}  // namespace

// recurrent_op.cc RecurrentOp::RunImpl (StaticRNN): step t of the time-major inputs
// runs the sub-block in its own child scope, where the block-local variables named
// like the outer `inputs` hold row t, the ex-states hold the previous step's states
// (initial_states at the first step) and the `outputs` rows are stacked back into
// the outer [T, ...] outputs.  reverse: t runs T-1 .. 0.  Training keeps the step
// scopes (StepScopes output) for recurrent_grad.
void Executor::RunRecurrent(const ProgramDesc& prog, const OpDesc& op, Scope* scope) {
  const int sb = (int)op.GetInt("sub_block", -1);
  PA_CHECK(sb >= 0 && sb < (int)prog.blocks.size(), "recurrent: bad sub_block %d", sb);
  const BlockDesc& blk = prog.Block(sb);
  const auto& xs = op.Inputs("inputs");
  const auto& inits = op.Inputs("initial_states");
  const auto& outs = op.Outputs("outputs");
  const auto& ex = str_attr(op, "ex_states");
  const auto& st = str_attr(op, "states");
  PA_CHECK(ex.size() == st.size() && ex.size() == inits.size(), "recurrent: %zu ex_states, %zu states, %zu initial",
           ex.size(), st.size(), inits.size());
  PA_CHECK(!xs.empty(), "recurrent: no inputs");
  const bool reverse = op.GetBool("reverse", false);
  Variable* x0 = scope->Find(xs[0]);
  PA_CHECK(x0 && x0->tensor.initialized() && !x0->tensor.dims.empty(), "recurrent: input %s is empty", xs[0].c_str());
  const int64_t T = x0->tensor.dims[0];
  const std::string ss = op.Output("step_scopes");
  const bool keep = !ss.empty() && !ctx_.is_test && !op.GetBool("is_test", false);
  Variable* sv = nullptr;
  if (keep) {
    sv = scope->Find(ss);
    if (!sv) sv = scope->Var(ss);
    sv->kind = VK_STEP_SCOPES;
    for (Scope* s : sv->steps) sv->steps_owner->DropKid(s);
    sv->steps.clear();
    sv->steps_owner = scope;
  }
  std::vector<Tensor> prev(ex.size());
  for (size_t i = 0; i < inits.size(); ++i) {
    Variable* v = scope->Find(inits[i]);
    PA_CHECK(v && v->tensor.initialized(), "recurrent: initial state %s is empty", inits[i].c_str());
    prev[i] = v->tensor;
  }
  std::vector<Tensor> stacked(outs.size());
  for (int64_t k = 0; k < T; ++k) {
    const int64_t t = reverse ? T - 1 - k : k;
    Scope& s = scope->NewScope();
    for (const VarDesc& v : blk.vars)
      if (!v.persistable) s.Var(v.name)->kind = v.type;
    for (auto& n : xs) {
      Variable* x = scope->Find(n);
      PA_CHECK(x && x->tensor.initialized() && x->tensor.dims.size() >= 1 && x->tensor.dims[0] == T,
               "recurrent: input %s is not [%lld, ...]", n.c_str(), (long long)T);
      s.Var(n)->tensor = time_row(x->tensor, t, ctx_.stream);
    }
    for (size_t i = 0; i < ex.size(); ++i) s.Var(ex[i])->tensor = prev[i];
    RunBlock(prog, blk, &s);
    for (size_t i = 0; i < st.size(); ++i) {
      Variable* v = s.FindLocal(st[i]);
      PA_CHECK(v && v->tensor.initialized(), "recurrent: state %s not produced at step %lld", st[i].c_str(),
               (long long)t);
      prev[i] = v->tensor;
    }
    for (size_t j = 0; j < outs.size(); ++j) {
      Variable* v = s.FindLocal(outs[j]);
      PA_CHECK(v && v->tensor.initialized(), "recurrent: output %s not produced at step %lld", outs[j].c_str(),
               (long long)t);
      put_row(stacked[j], T, t, v->tensor, ctx_.stream);
    }
    if (keep) sv->steps.push_back(&s);
    else scope->DropKid(&s);
  }
  for (size_t j = 0; j < outs.size(); ++j) {
    Variable* o = scope->Find(outs[j]);
    if (!o) o = scope->Var(outs[j]);
    o->kind = VK_LOD_TENSOR;
    o->tensor = stacked[j];
  }
}

// recurrent_op.cc RecurrentGradOp::RunImpl: the grad block runs in a child of every
// kept step scope, last step first.  Per step the block-local output gradients hold
// row t of the outer ones, each state's gradient additionally takes the ex-state
// gradient the later step produced (the link the forward made between them); row t
// of every input gradient is copied out, parameter gradients are summed over the
// steps, and the first step's ex-state gradients are the initial-state gradients.
void Executor::RunRecurrentGrad(const ProgramDesc& prog, const OpDesc& op, Scope* scope) {
  const int sb = (int)op.GetInt("sub_block", -1);
  PA_CHECK(sb >= 0 && sb < (int)prog.blocks.size(), "recurrent_grad: bad sub_block %d", sb);
  const BlockDesc& blk = prog.Block(sb);
  const auto& xs = op.Inputs("inputs");
  const auto& inits = op.Inputs("initial_states");
  const auto& params = op.Inputs("parameters");
  const auto& outs = op.Inputs("outputs");
  const auto& ogs = op.Inputs("outputs@GRAD");
  const auto& xgs = op.Outputs("inputs@GRAD");
  const auto& igs = op.Outputs("initial_states@GRAD");
  const auto& pgs = op.Outputs("parameters@GRAD");
  const auto& ex = str_attr(op, "ex_states");
  const auto& st = str_attr(op, "states");
  const bool reverse = op.GetBool("reverse", false);
  Variable* sv = scope->Find(op.Input("step_scopes"));
  PA_CHECK(sv != nullptr, "recurrent_grad: step scopes %s not found", op.Input("step_scopes").c_str());
  const int64_t T = (int64_t)sv->steps.size();
  auto g = [](const std::string& n) { return n + "@GRAD"; };
  auto live = [](const std::vector<std::string>& v, size_t i) { return i < v.size() && v[i] != "@EMPTY@" && !v[i].empty(); };
  // outer output gradients by output position (the slot lists only differentiable ones)
  std::map<std::string, Tensor> og_outer;
  for (auto& n : ogs) {
    Variable* v = scope->Find(n);
    if (v && v->tensor.initialized()) og_outer[n] = v->tensor;
  }
  std::vector<Tensor> carry(ex.size()), xg_acc(xs.size());
  std::map<std::string, Tensor> pacc;
  for (int64_t k = T; k-- > 0;) {
    const int64_t t = reverse ? T - 1 - k : k;
    Scope* s = sv->steps[k];
    Scope& gs = s->NewScope();
    for (const VarDesc& v : blk.vars)
      if (!v.persistable) gs.Var(v.name)->kind = v.type;
    // <name>@GRAD@EXT of every step output / state: row t of its outer gradient plus
    // the later step's ex-state gradient, zeros when neither exists (the grad block
    // adds it to its own contributions: fluid/backward.py _recurrent_grad_descs)
    std::vector<std::string> linked(st.begin(), st.end());
    for (auto& o : outs)
      if (std::find(linked.begin(), linked.end(), o) == linked.end()) linked.push_back(o);
    for (auto& n : linked) {
      Tensor ext;
      auto it = og_outer.find(g(n));
      if (it != og_outer.end()) ext = time_row(it->second, t, ctx_.stream);
      auto si = std::find(st.begin(), st.end(), n);
      if (si != st.end() && carry[si - st.begin()].initialized())
        accumulate_into(ext, carry[si - st.begin()], ctx_.stream);  // += or a private copy
      if (!ext.initialized()) {
        Variable* fv = s->FindLocal(n);
        PA_CHECK(fv && fv->tensor.initialized(), "recurrent_grad: step variable %s not kept", n.c_str());
        ext = zeros_like_f32(fv->tensor, ctx_.stream);
      }
      gs.Var(g(n) + "@EXT")->tensor = ext;
    }
    RunBlock(prog, blk, &gs);
    for (size_t j = 0; j < xs.size(); ++j) {
      if (!live(xgs, j)) continue;
      Variable* v = gs.FindLocal(g(xs[j]));
      Tensor r = v && v->tensor.initialized() ? v->tensor : Tensor();
      if (!r.initialized()) {
        Variable* x = scope->Find(xs[j]);
        r = zeros_like_f32(time_row(x->tensor, t, ctx_.stream), ctx_.stream);
      }
      put_row(xg_acc[j], T, t, r, ctx_.stream);
    }
    for (size_t j = 0; j < params.size(); ++j) {
      if (!live(pgs, j)) continue;
      Variable* v = gs.FindLocal(g(params[j]));
      if (v && v->tensor.initialized()) accumulate_into(pacc[pgs[j]], v->tensor, ctx_.stream);
    }
    for (size_t i = 0; i < ex.size(); ++i) {
      Variable* v = gs.FindLocal(g(ex[i]));
      carry[i] = Tensor();
      if (v && v->tensor.initialized()) accumulate_into(carry[i], v->tensor, ctx_.stream);
    }
    s->DropKid(&gs);
  }
  auto set_out = [&](const std::string& name, const Tensor& val, const std::string& like) {
    Variable* o = scope->Find(name);
    if (!o) o = scope->Var(name);
    o->kind = VK_LOD_TENSOR;
    if (val.initialized()) {
      o->tensor = val;
    } else {
      Variable* x = scope->Find(like);
      if (x && x->tensor.initialized() && x->tensor.dtype == DT::FP32) o->tensor = zeros_like_f32(x->tensor, ctx_.stream);
    }
  };
  for (size_t j = 0; j < xs.size(); ++j)
    if (live(xgs, j)) set_out(xgs[j], xg_acc[j], xs[j]);
  for (size_t j = 0; j < params.size(); ++j)
    if (live(pgs, j)) set_out(pgs[j], pacc.count(pgs[j]) ? pacc[pgs[j]] : Tensor(), params[j]);
  for (size_t i = 0; i < inits.size(); ++i)
    if (live(igs, i)) set_out(igs[i], i < carry.size() ? carry[i] : Tensor(), inits[i]);
}

// conditional_block_op.cc: run the sub-block once when the condition holds
// (is_scalar_condition: Cond[0] != 0; else: every Input is non-empty).
void Executor::RunConditionalBlock(const ProgramDesc& prog, const OpDesc& op, Scope* scope) {
  const int sb = (int)op.GetInt("sub_block", -1);
  PA_CHECK(sb >= 0 && sb < (int)prog.blocks.size(), "conditional_block: bad sub_block %d", sb);
  bool run = true;
  if (op.GetBool("is_scalar_condition", false)) {
    Variable* cv = scope->Find(op.Input("Cond"));
    PA_CHECK(cv != nullptr, "conditional_block: condition not found");
    run = ReadBool(cv->tensor);
  } else {
    for (auto& n : op.Inputs("Cond")) {
      Variable* v = scope->Find(n);
      if (!v || !v->tensor.initialized() || v->tensor.numel() == 0) run = false;
    }
  }
  // training programs keep the block's scope in the Scope output for
  // conditional_block_grad (empty when the block did not run)
  const std::string sn = op.Output("Scope");
  Variable* kept = (!sn.empty() && !ctx_.is_test) ? scope->Find(sn) : nullptr;
  if (!sn.empty() && !ctx_.is_test && !kept) kept = scope->Var(sn);
  if (kept) {
    kept->kind = VK_STEP_SCOPES;
    for (Scope* s : kept->steps) kept->steps_owner->DropKid(s);
    kept->steps.clear();
    kept->steps_owner = scope;
  }
  if (!run) return;
  Scope& body = scope->NewScope();
  const BlockDesc& blk = prog.Block(sb);
  for (const VarDesc& v : blk.vars)
    if (!scope->Find(v.name)) body.Var(v.name)->kind = v.type;
  RunBlock(prog, blk, &body);
  if (kept) kept->steps.push_back(&body);
  else scope->DropKid(&body);
}

// conditional_block_op.cc ConditionalBlockGradOp: when the forward ran, the grad
// block runs in a child of the kept scope and the block-local input gradients are
// copied to the enclosing X@GRAD (AssignLocalGradientToGlobal); else zeros
void Executor::RunConditionalBlockGrad(const ProgramDesc& prog, const OpDesc& op, Scope* scope) {
  const int sb = (int)op.GetInt("sub_block", -1);
  PA_CHECK(sb >= 0 && sb < (int)prog.blocks.size(), "conditional_block_grad: bad sub_block %d", sb);
  const BlockDesc& blk = prog.Block(sb);
  const auto& xs = op.Inputs("X");
  const auto& xgs = op.Outputs("X@GRAD");
  Variable* kept = scope->Find(op.Input("Scope"));
  std::map<std::string, Tensor> got;
  if (kept && !kept->steps.empty()) {
    Scope* s = kept->steps[0];
    Scope& gs = s->NewScope();
    // the block's locals, except the incoming output gradients (held outside)
    const auto& ogs = op.Inputs("Out@GRAD");
    for (const VarDesc& v : blk.vars)
      if (!v.persistable && std::find(ogs.begin(), ogs.end(), v.name) == ogs.end()) gs.Var(v.name)->kind = v.type;
    for (size_t i = 0; i < xs.size() && i < xgs.size(); ++i)
      if (xgs[i] != "@EMPTY@" && !gs.FindLocal(xgs[i])) gs.Var(xgs[i]);
    RunBlock(prog, blk, &gs);
    for (size_t i = 0; i < xs.size() && i < xgs.size(); ++i) {
      if (xgs[i] == "@EMPTY@") continue;
      Variable* g = gs.FindLocal(xgs[i]);
      if (g && g->tensor.initialized()) accumulate_into(got[xgs[i]], g->tensor, ctx_.stream);
    }
    s->DropKid(&gs);
  }
  for (size_t i = 0; i < xs.size() && i < xgs.size(); ++i) {
    if (xgs[i] == "@EMPTY@") continue;
    Variable* x = scope->Find(xs[i]);
    Variable* out = scope->Find(xgs[i]);
    if (!out) out = scope->Var(xgs[i]);
    out->kind = VK_LOD_TENSOR;
    auto it = got.find(xgs[i]);
    if (it != got.end()) {
      out->tensor = it->second;
      if (x) out->tensor.lod = x->tensor.lod;
    } else if (x && x->tensor.initialized() && x->tensor.dtype == DT::FP32) {
      Tensor z;
      z.alloc(DT::FP32, x->tensor.dims, x->tensor.device);
      if (z.device >= 0) device_fill(ctx_.stream, z.raw(), DT::FP32, z.numel(), 0.0);
      else std::fill_n(z.data<float>(), z.numel(), 0.f);
      z.lod = x->tensor.lod;
      out->tensor = z;
    }
  }
}

void Executor::Sync() {
  if (ctx_.stream) device_stream_sync(ctx_.stream);
}

void Executor::RunBlock(const ProgramDesc& prog, const BlockDesc& block, Scope* scope) {
  const bool dev = ctx_.device >= 0;
  // kernels that only move metadata / holders work on tensors of any device
  static const std::set<std::string> agnostic = {"feed", "fetch", "reshape", "reshape2", "flatten", "flatten2",
                                                 "squeeze", "squeeze2", "unsqueeze", "unsqueeze2", "delete_var",
                                                 "reshape_grad", "reshape2_grad"};
  // loop counters / flags: a declined device kernel takes the host kernel (a few
  // bytes each way), not the embedder's
  static const std::set<std::string> host_scalar = {"fill_constant", "increment", "less_than", "less_equal",
                                                    "greater_than", "greater_equal", "equal", "not_equal",
                                                    "logical_and", "logical_or", "logical_xor", "logical_not"};
  // every input is an initialised host tensor (and there is at least one)
  auto host_inputs = [&](const OpDesc& op) {
    int n = 0;
    for (auto& slot : op.inputs)
      for (auto& name : slot.second) {
        Variable* v = scope->Find(name);
        if (!v || !v->tensor.initialized() || v->tensor.device >= 0) return false;
        ++n;
      }
    return n > 0;
  };
  // a loop-control op mixing host and device SCALARS (a force_cpu counter against a
  // device-filled bound, a host condition and-ed with a device is_empty flag): its
  // kernel place is the host (the reference's compare / logical ops with force_cpu
  // and their data transform), so the device scalars are read over and the result
  // stays on the host where the loop reads it
  auto host_scalar_mix = [&](const OpDesc& op) {
    int host = 0, n = 0;
    for (auto& slot : op.inputs)
      for (auto& name : slot.second) {
        Variable* v = scope->Find(name);
        if (!v || v->kind != VK_LOD_TENSOR || !v->tensor.initialized() || v->tensor.numel() > 1) return false;
        host += v->tensor.device < 0;
        ++n;
      }
    return n > 0 && host > 0;
  };
  auto run_host_scalars = [&](const OpDesc& op, const Kernel* k) {
    Scope& tmp = scope->NewScope();
    for (auto& slot : op.inputs)
      for (auto& name : slot.second) {
        Variable* v = scope->Find(name);
        if (v->tensor.device >= 0) {
          Variable* h = tmp.Var(name);
          h->kind = v->kind;
          h->tensor = v->tensor.to(-1, ctx_.stream);
        }
      }
    device_stream_sync(ctx_.stream);
    ExecContext hctx = ctx_;
    hctx.device = -1;
    (*k)(OpRun{op, tmp, hctx});
    // an output that shadows a copied input (in place) moves out as a host tensor
    for (auto& slot : op.outputs)
      for (auto& name : slot.second) {
        Variable* h = tmp.FindLocal(name);
        if (!h || !h->tensor.initialized()) continue;
        Variable* v = scope->Find(name);
        if (!v) v = scope->Var(name);
        v->tensor = h->tensor;
      }
    scope->DropKid(&tmp);
  };
  // the reference's InferShape ShareLoD("X", "Out") default (the Python op library's
  // register_op share_lod=True): an output with no LoD and as many rows as the first
  // LoD-carrying input takes that input's LoD; the ops registered share_lod=False there
  // are exempt (their kernels set the output LoD themselves)
  auto share_lod = [&](const OpDesc& op) {
    static const std::set<std::string> exempt = {
        "array_to_lod_tensor", "array_to_lod_tensor_grad", "attention_lstm", "conditional_block",
        "conditional_block_grad", "feed", "fetch", "fusion_seqexpand_concat_fc", "go", "gru_unit",
        "hierarchical_sigmoid", "linear_chain_crf", "lod_rank_table", "lod_reset", "lod_tensor_to_array",
        "lod_tensor_to_array_grad", "lstm_unit", "merge_lod_tensor", "nce", "parallel_do", "read",
        "read_from_array", "read_from_array_grad", "recurrent", "recurrent_grad", "reorder_lod_tensor_by_rank",
        "reorder_lod_tensor_by_rank_grad", "select", "sequence_concat", "sequence_erase", "sequence_expand",
        "sequence_expand_as", "sequence_pad", "sequence_pool", "sequence_reshape", "sequence_scatter",
        "sequence_slice", "sequence_unpad", "shrink_rnn_memory", "shrink_rnn_memory_grad", "split_lod_tensor",
        "warpctc", "while", "while_grad", "write_to_array", "write_to_array_grad", "beam_search",
        "beam_search_decode", "crf_decoding"};
    if (exempt.count(op.type)) return;
    const Tensor* first = nullptr;
    for (auto& slot : op.inputs) {
      if (slot.second.empty()) continue;
      Variable* v = scope->Find(slot.second[0]);
      if (v && v->kind == VK_LOD_TENSOR && v->tensor.initialized() && !v->tensor.lod.empty()) {
        first = &v->tensor;
        break;
      }
    }
    if (!first || first->dims.empty()) return;
    const LoD lod = first->lod;
    const int64_t rows = first->dims[0];
    for (auto& slot : op.outputs)
      for (auto& n : slot.second) {
        Variable* v = scope->Find(n);
        if (v && v->kind == VK_LOD_TENSOR && v->tensor.initialized() && v->tensor.lod.empty() &&
            !v->tensor.dims.empty() && v->tensor.dims[0] == rows)
          v->tensor.lod = lod;
      }
  };
  auto timed = [&](const OpDesc& op, const std::function<void()>& fn) {
    if (!profile) {
      fn();
      share_lod(op);
      return;
    }
    Sync();
    auto t0 = std::chrono::steady_clock::now();
    fn();
    share_lod(op);
    Sync();
    auto& e = op_time_ms[op.type];
    e.first += 1;
    e.second += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  };
  // host kernel on host copies of the device inputs; results go back to HBM
  auto host_fallback = [&](const OpDesc& op, const Kernel* k) {
    PA_CHECK(!strict_native, "FLAGS_strict_native: op '%s' has no device kernel for this configuration and "
             "would run on host copies of its device inputs", op.type.c_str());
    host_fallbacks[op.type] += 1;
    Scope& tmp = scope->NewScope();
    for (auto& slot : op.inputs)
      for (auto& n : slot.second) {
        Variable* v = scope->Find(n);
        if (v && v->tensor.initialized() && v->tensor.device >= 0) {
          Variable* h = tmp.Var(n);
          h->kind = v->kind;
          h->tensor = v->tensor.to(-1, ctx_.stream);
        }
      }
    device_stream_sync(ctx_.stream);
    for (auto& slot : op.outputs)
      for (auto& n : slot.second) {
        Variable* v = scope->Find(n);
        if (v && !tmp.FindLocal(n)) {
          Variable* h = tmp.Var(n);
          h->kind = v->kind;
          h->list = v->list;
          if (v->tensor.initialized()) h->tensor = v->tensor.to(-1, ctx_.stream);
        }
      }
    device_stream_sync(ctx_.stream);
    ExecContext hctx = ctx_;
    hctx.device = -1;
    (*k)(OpRun{op, tmp, hctx});
    for (auto& slot : op.outputs)
      for (auto& n : slot.second) {
        Variable* h = tmp.FindLocal(n);
        if (!h) continue;
        Variable* v = scope->Find(n);
        if (!v) v = scope->Var(n);
        v->kind = h->kind;
        v->list = h->list;
        if (!h->tensor.initialized()) continue;
        if (h->kind == VK_FETCH_LIST) {
          v->tensor = h->tensor;
        } else if (v->tensor.initialized() && v->tensor.buf && !v->tensor.buf->owned &&
                   v->tensor.device == ctx_.device && v->tensor.nbytes() == h->tensor.nbytes() &&
                   v->tensor.dtype == h->tensor.dtype) {
          // lent (embedder-owned) buffer: update it in place so the embedder sees the result
          device_copy(v->tensor.raw(), ctx_.device, h->tensor.raw(), -1, h->tensor.nbytes(), ctx_.stream);
          v->tensor.dims = h->tensor.dims;
          v->tensor.lod = h->tensor.lod;
        } else {
          v->tensor = h->tensor.to(ctx_.device, ctx_.stream);
        }
      }
  };
  // an op's outputs start without LoD (the reference's InferShape ShareLoD runs every
  // time): temporaries keep their buffers from run to run, and a LoD left over from
  // the previous batch must not survive into an output whose kernel does not set one
  // (share_lod fills it from the inputs afterwards).  In-place outputs keep theirs.
  auto clear_out_lod = [&](const OpDesc& op) {
    for (auto& slot : op.outputs)
      for (auto& n : slot.second) {
        if (n.empty() || n == "@EMPTY@") continue;
        bool inplace = false;
        for (auto& is : op.inputs)
          for (auto& m : is.second) inplace = inplace || m == n;
        if (inplace) continue;
        Variable* v = scope->Find(n);
        if (v && v->kind == VK_LOD_TENSOR && !v->tensor.lod.empty()) v->tensor.lod.clear();
      }
  };
  int op_idx = -1;
  for (const OpDesc& op : block.ops) {
    ++op_idx;
    if (op.type != "while" && op.type != "conditional_block" && op.type != "while_grad" &&
        op.type != "conditional_block_grad" && op.type != "recurrent" && op.type != "recurrent_grad" &&
        op.type != "feed" && op.type != "fetch")
      clear_out_lod(op);
    if (op.type == "while") {
      timed(op, [&] { RunWhile(prog, op, scope); });
      continue;
    }
    if (op.type == "conditional_block") {
      timed(op, [&] { RunConditionalBlock(prog, op, scope); });
      continue;
    }
    if (op.type == "while_grad") {
      timed(op, [&] { RunWhileGrad(prog, op, scope); });
      continue;
    }
    if (op.type == "conditional_block_grad") {
      timed(op, [&] { RunConditionalBlockGrad(prog, op, scope); });
      continue;
    }
    if (op.type == "recurrent") {
      timed(op, [&] { RunRecurrent(prog, op, scope); });
      continue;
    }
    if (op.type == "recurrent_grad") {
      timed(op, [&] { RunRecurrentGrad(prog, op, scope); });
      continue;
    }
    // loop counters / bounds that live on the host (fill_constant force_cpu,
    // max_sequence_len, lod_array_length): the host kernel IS their kernel on a device
    // place too (the reference's CPU-pinned control tensors), no round trip
    if (dev && host_scalar.count(op.type) && host_inputs(op)) {
      if (const Kernel* hk = find_kernel(op.type, false)) {
        timed(op, [&] { (*hk)(OpRun{op, *scope, ctx_}); });
        continue;
      }
    }
    if (dev && host_scalar.count(op.type) && host_scalar_mix(op)) {
      if (const Kernel* hk = find_kernel(op.type, false)) {
        timed(op, [&] { run_host_scalars(op, hk); });
        continue;
      }
    }
    const Kernel* dk = dev ? find_kernel(op.type, true) : nullptr;
    if (dk) {
      try {
        timed(op, [&] { (*dk)(OpRun{op, *scope, ctx_}); });
        continue;
      } catch (const Decline&) {
        // the embedder's kernel runs on the device too: prefer it to a host round
        // trip (place-agnostic host kernels -- fill / shape ops -- stay native)
        const Kernel* hk = find_kernel(op.type, false);
        if (fallback && !(hk && (agnostic.count(op.type) || host_scalar.count(op.type)))) {
          embedder_fallbacks[op.type] += 1;
          timed(op, [&] { fallback(op, *scope, block.idx, op_idx); });
          continue;
        }
      }
    }
    const Kernel* k = find_kernel(op.type, false);
    if (k == nullptr && fallback) {
      embedder_fallbacks[op.type] += 1;
      timed(op, [&] { fallback(op, *scope, block.idx, op_idx); });
      continue;
    }
    PA_CHECK(k != nullptr, dk ? "op '%s' declined its device kernel and has no host kernel"
                              : "no kernel registered for op type '%s'", op.type.c_str());
    try {
      if (dev && !agnostic.count(op.type))
        timed(op, [&] { host_fallback(op, k); });
      else
        timed(op, [&] { (*k)(OpRun{op, *scope, ctx_}); });
    } catch (const Decline&) {
      // the host kernel does not cover these dtypes / this configuration
      PA_CHECK(fallback != nullptr, "op '%s': no kernel covers this configuration (dtype / layout)",
               op.type.c_str());
      embedder_fallbacks[op.type] += 1;
      timed(op, [&] { fallback(op, *scope, block.idx, op_idx); });
    }
  }
}

void Executor::Run(const ProgramDesc& prog, Scope* scope, int block_id, Scope* local) {
  const BlockDesc& block = prog.Block(block_id);
  Scope* tmp = local ? local : scope;
  for (const VarDesc& v : block.vars) {
    // feed / fetch holders are per-run state: they live with the temporaries so
    // predictors sharing one parameter scope never share them
    const bool io = v.type == VK_FEED_MINIBATCH || v.type == VK_FETCH_LIST;
    Scope* s = v.persistable && !io ? scope : tmp;
    if (Variable* have = tmp->Find(v.name)) {
      // temporaries start every run empty (the reference drops its local scope after
      // a run): a tensor array left from the previous batch would be appended to /
      // accumulated into with stale shapes
      if (!v.persistable && have->kind == VK_LOD_TENSOR_ARRAY) have->list.clear();
      continue;
    }
    Variable* var = s->Var(v.name);
    var->kind = v.type;
  }
  RunBlock(prog, block, tmp);
}

// ================================================================ LoDTensor IO
// LoDTensor := u32 version | u64 lod_level | lod_level x (u64 nbytes | u64[]) | Tensor
// Tensor    := u32 version | i32 desc_size | TensorDesc proto | raw data
bool read_lod_tensor(FILE* f, Tensor* t) {
  uint32_t ver;
  size_t got = fread(&ver, 1, 4, f);
  if (got == 0) return false;
  PA_CHECK(got == 4, "LoDTensor: truncated header");
  uint64_t ll;
  PA_CHECK(fread(&ll, 8, 1, f) == 1 && ll <= 16, "LoDTensor: bad lod level");
  t->lod.assign(ll, {});
  for (uint64_t i = 0; i < ll; ++i) {
    uint64_t nb;
    PA_CHECK(fread(&nb, 8, 1, f) == 1 && nb % 8 == 0 && nb <= (1ull << 36), "LoDTensor: bad lod size");
    std::vector<uint64_t> tmp(nb / 8);
    PA_CHECK(fread(tmp.data(), 8, tmp.size(), f) == tmp.size(), "LoDTensor: truncated lod");
    t->lod[i].assign(tmp.begin(), tmp.end());
  }
  int32_t dsz;
  PA_CHECK(fread(&ver, 4, 1, f) == 1 && fread(&dsz, 4, 1, f) == 1 && dsz >= 0 && dsz < (1 << 16),
           "LoDTensor: bad tensor desc");
  std::string desc((size_t)dsz, '\0');
  PA_CHECK(fread(&desc[0], 1, desc.size(), f) == desc.size(), "LoDTensor: truncated desc");
  VarDesc vd;
  parse_tensor_desc(Reader{(const unsigned char*)desc.data(), (const unsigned char*)desc.data() + desc.size()},
                    &vd);
  // element count and byte total with overflow checks (dims like [2^33, 2^31] must not
  // wrap numel to a small value), capped at 2^40 bytes and at what the file still holds
  uint64_t count = 1;
  for (auto d : vd.dims) {
    PA_CHECK(d >= 0 && d < (1ll << 40), "LoDTensor: implausible dim");
    PA_CHECK(!__builtin_mul_overflow(count, (uint64_t)d, &count), "LoDTensor: element count overflows");
  }
  uint64_t bytes = 0;
  PA_CHECK(!__builtin_mul_overflow(count, (uint64_t)dt_size(vd.dtype), &bytes) && bytes <= (1ull << 40),
           "LoDTensor: implausible byte size");
  {
    const long here = ftell(f);
    if (here >= 0 && fseek(f, 0, SEEK_END) == 0) {
      const long end = ftell(f);
      PA_CHECK(fseek(f, here, SEEK_SET) == 0, "LoDTensor: seek failed");
      PA_CHECK(end >= here && bytes <= (uint64_t)(end - here), "LoDTensor: declared size %llu beyond end of file",
               (unsigned long long)bytes);
    }
  }
  LoD lod = t->lod;
  t->alloc(vd.dtype, vd.dims, -1);
  t->lod = lod;
  PA_CHECK(fread(t->raw(), 1, t->nbytes(), f) == t->nbytes(), "LoDTensor: truncated data");
  return true;
}

void write_lod_tensor(FILE* f, const Tensor& t0) {
  Tensor t = t0.device >= 0 ? t0.to(-1) : t0;
  uint32_t ver = 0;
  uint64_t ll = t.lod.size();
  fwrite(&ver, 4, 1, f);
  fwrite(&ll, 8, 1, f);
  for (auto& lv : t.lod) {
    uint64_t nb = lv.size() * 8;
    fwrite(&nb, 8, 1, f);
    std::vector<uint64_t> tmp(lv.begin(), lv.end());
    fwrite(tmp.data(), 8, tmp.size(), f);
  }
  std::string desc;
  auto put = [&](uint64_t v) {
    while (v >= 0x80) {
      desc.push_back((char)(v | 0x80));
      v >>= 7;
    }
    desc.push_back((char)v);
  };
  desc.push_back(0x08);
  put((uint64_t)t.dtype);
  for (auto d : t.dims) {
    desc.push_back(0x10);
    put((uint64_t)d);
  }
  int32_t dsz = (int32_t)desc.size();
  fwrite(&ver, 4, 1, f);
  fwrite(&dsz, 4, 1, f);
  fwrite(desc.data(), 1, desc.size(), f);
  fwrite(t.raw(), 1, t.nbytes(), f);
}

void load_persistables(const ProgramDesc& prog, Scope* scope, const std::string& dir,
                       const std::string& combined_file, int device, void* stream) {
  std::vector<const VarDesc*> vars;
  for (const VarDesc& v : prog.Block(0).vars) {
    if (!v.persistable || v.type == VK_FEED_MINIBATCH || v.type == VK_FETCH_LIST || v.type == VK_RAW ||
        v.type == VK_READER)
      continue;
    vars.push_back(&v);
  }
  auto place = [&](const VarDesc* v, Tensor&& host) {
    Variable* var = scope->Var(v->name);
    var->kind = v->type;
    var->tensor = device >= 0 ? host.to(device, stream) : std::move(host);
  };
  if (!combined_file.empty()) {
    // save_combine writes the variables sorted by name (fluid/io.py save_vars)
    std::sort(vars.begin(), vars.end(), [](const VarDesc* a, const VarDesc* b) { return a->name < b->name; });
    FILE* f = fopen(combined_file.c_str(), "rb");
    PA_CHECK(f != nullptr, "cannot open params file %s", combined_file.c_str());
    try {
      for (const VarDesc* v : vars) {
        Tensor t;
        PA_CHECK(read_lod_tensor(f, &t), "params file %s ends before %s", combined_file.c_str(), v->name.c_str());
        place(v, std::move(t));
      }
    } catch (...) {
      fclose(f);
      throw;
    }
    fclose(f);
  } else {
    for (const VarDesc* v : vars) {
      const std::string path = dir + "/" + v->name;
      FILE* f = fopen(path.c_str(), "rb");
      PA_CHECK(f != nullptr, "cannot open parameter file %s", path.c_str());
      Tensor t;
      bool ok = false;
      try {
        ok = read_lod_tensor(f, &t);
      } catch (...) {
        fclose(f);
        throw;
      }
      fclose(f);
      PA_CHECK(ok, "empty parameter file %s", path.c_str());
      place(v, std::move(t));
    }
  }
  if (device >= 0) device_stream_sync(stream);
}

}  // namespace pa
