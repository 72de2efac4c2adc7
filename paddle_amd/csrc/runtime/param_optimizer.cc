// Parameter optimizer library with a C ABI -- the counterpart of the reference's
// paddle/legacy/optimizer (optimizer.h: paddle_create_optimizer /
// paddle_update_parameter / paddle_optimizer_get_weights / paddle_optimizer_get_state
// / paddle_release_optimizer), the update rules the Go pserver runs through cgo.
//
// * config: an OptimizerConfig message (proto/OptimizerConfig.proto) in protobuf wire
//   format -- SGD (momentum, decay, nesterov), Adadelta, Adagrad, Adam; Const / Linear
//   learning-rate policy over the number of updates;
// * state: the <Kind>OptimizerState message (lr_state, num_sample_passed, parameter
//   and the accumulators as TensorProto).  TensorProto.content is written as ONE
//   entry holding the raw little-endian float32 block (exact); the reference writes
//   one decimal string per element (6 significant digits) -- both forms are read;
// * the parameter buffer is owned by the optimizer (copied in at create).
//
// Exported with the pa_ prefix (the runtime library's namespace) plus the
// reference's paddle_* names as aliases.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "runtime.h"

namespace {

// ------------------------------------------------------------------ proto2 wire
struct Reader {
  const uint8_t* p;
  const uint8_t* e;
  bool ok = true;
  bool more() const { return ok && p < e; }
  uint64_t varint() {
    uint64_t r = 0;
    for (int s = 0; s < 64 && p < e; s += 7) {
      const uint8_t b = *p++;
      r |= (uint64_t)(b & 0x7f) << s;
      if (!(b & 0x80)) return r;
    }
    ok = false;
    return 0;
  }
  double f64() {
    double d = 0;
    if (e - p < 8) { ok = false; return 0; }
    std::memcpy(&d, p, 8);
    p += 8;
    return d;
  }
  std::string bytes() {
    const uint64_t n = varint();
    if (!ok || (uint64_t)(e - p) < n) { ok = false; return {}; }
    std::string s((const char*)p, (size_t)n);
    p += n;
    return s;
  }
  void skip(int wt) {
    if (wt == 0) varint();
    else if (wt == 1) { if (e - p < 8) ok = false; else p += 8; }
    else if (wt == 5) { if (e - p < 4) ok = false; else p += 4; }
    else if (wt == 2) bytes();
    else ok = false;
  }
};

struct Writer {
  std::string s;
  void varint(uint64_t v) {
    while (v >= 0x80) { s.push_back((char)(v | 0x80)); v >>= 7; }
    s.push_back((char)v);
  }
  void key(int num, int wt) { varint(((uint64_t)num << 3) | (uint64_t)wt); }
  void f64(int num, double d) {
    key(num, 1);
    char b[8];
    std::memcpy(b, &d, 8);
    s.append(b, 8);
  }
  void u64(int num, uint64_t v) { key(num, 0); varint(v); }
  void bytes(int num, const std::string& b) { key(num, 2); varint(b.size()); s += b; }
};

struct Lr {
  int policy = 0;  // 0 const, 1 linear
  double lr = 0.1, a = 0, b = 0;
  double at(double n) const { return policy == 1 ? std::max(lr - a * n, b) : lr; }
  std::string state() const {
    Writer w;
    w.f64(1, lr);
    w.f64(2, a);
    w.f64(3, b);
    return w.s;
  }
  void load(const std::string& st) {
    Reader r{(const uint8_t*)st.data(), (const uint8_t*)st.data() + st.size()};
    while (r.more()) {
      const uint64_t k = r.varint();
      const int num = (int)(k >> 3), wt = (int)(k & 7);
      if (wt == 1 && num >= 1 && num <= 3) {
        const double v = r.f64();
        (num == 1 ? lr : num == 2 ? a : b) = v;
      } else {
        r.skip(wt);
      }
    }
  }
};

struct Opt {
  int kind = 1;  // 1 SGD, 2 Adadelta, 3 Adagrad, 4 Adam
  Lr lr;
  double momentum = 0, decay = 0, rho = 0.9, eps = 1e-5, beta1 = 0.9, beta2 = 0.999;
  bool nesterov = false;
  double num_sample_passed = 0;
  std::vector<float> param, a0, a1, a2;  // accumulators per kind
};

// sub-message of a config: field -> (double fields by number, bool)
void parse_sub(const std::string& m, Opt& o, int which) {
  Reader r{(const uint8_t*)m.data(), (const uint8_t*)m.data() + m.size()};
  while (r.more()) {
    const uint64_t k = r.varint();
    const int num = (int)(k >> 3), wt = (int)(k & 7);
    if (wt == 1) {
      const double v = r.f64();
      switch (which) {
        case 3:  // SGDConfig
          if (num == 21) o.momentum = v;
          else if (num == 23) o.decay = v;
          break;
        case 4:  // AdadeltaConfig
          if (num == 33) o.rho = v;
          else if (num == 31) o.eps = v;
          else if (num == 32) o.decay = v;
          break;
        case 5:  // AdagradConfig
          if (num == 41) o.eps = v;
          else if (num == 42) o.decay = v;
          break;
        case 6:  // AdamConfig
          if (num == 41) o.beta1 = v;
          else if (num == 42) o.beta2 = v;
          else if (num == 43) o.eps = v;
          else if (num == 44) o.decay = v;
          break;
        case 12:  // ConstLrConfig
          if (num == 1) o.lr.lr = v;
          break;
        case 13:  // LinearLrConfig
          if (num == 1) o.lr.lr = v;
          else if (num == 2) o.lr.a = v;
          else if (num == 3) o.lr.b = v;
          break;
      }
    } else if (wt == 0) {
      const uint64_t v = r.varint();
      if (which == 3 && num == 24) o.nesterov = v != 0;
    } else {
      r.skip(wt);
    }
  }
}

bool parse_config(const uint8_t* buf, int len, Opt& o) {
  Reader r{buf, buf + len};
  std::string subs[14];
  bool lr_set = false;
  while (r.more()) {
    const uint64_t k = r.varint();
    const int num = (int)(k >> 3), wt = (int)(k & 7);
    if (wt == 0 && num == 1) o.kind = (int)r.varint();
    else if (wt == 0 && num == 11) { o.lr.policy = (int)r.varint(); lr_set = true; }
    else if (wt == 2 && num >= 3 && num <= 13) subs[num] = r.bytes();
    else r.skip(wt);
  }
  if (!r.ok || o.kind < 1 || o.kind > 4) return false;
  // proto2 defaults of OptimizerConfig.proto: AdamConfig declares none (0), Adagrad /
  // Adadelta epsilon 1e-5, Adadelta rho 0.9
  if (o.kind == 4) { o.beta1 = 0.0; o.beta2 = 0.0; o.eps = 0.0; }
  if (o.kind == 3) o.eps = 1e-5;
  for (int w : {3, 4, 5, 6}) parse_sub(subs[w], o, w);
  // an unset lr_policy reads as Const (the enum's first value), so the reference's
  // "ConstLr(0.1)" fallback never runs: ConstLrConfig / LinearLrConfig default to
  // learning_rate 1.0 (parameter_optimizer.cc:32-43, OptimizerConfig.proto:70-79)
  (void)lr_set;
  o.lr.lr = 1.0;
  o.lr.a = o.lr.b = 0.0;
  parse_sub(subs[o.lr.policy == 1 ? 13 : 12], o, o.lr.policy == 1 ? 13 : 12);
  return true;
}

// TensorProto: data_type = 1, content = 2 (repeated bytes)
std::string tensor_proto(const std::vector<float>& t) {
  Writer w;
  w.u64(1, 4);  // PADDLE_ELEMENT_TYPE_FLOAT32
  if (t.size() == 1) {  // one element: the decimal form (a 4-byte raw block would be ambiguous)
    char b[32];
    std::snprintf(b, sizeof(b), "%.9g", (double)t[0]);
    w.bytes(2, b);
  } else {
    w.bytes(2, std::string((const char*)t.data(), t.size() * sizeof(float)));
  }
  return w.s;
}

bool load_tensor(const std::string& m, std::vector<float>& t) {
  Reader r{(const uint8_t*)m.data(), (const uint8_t*)m.data() + m.size()};
  std::vector<std::string> content;
  while (r.more()) {
    const uint64_t k = r.varint();
    const int num = (int)(k >> 3), wt = (int)(k & 7);
    if (num == 2 && wt == 2) content.push_back(r.bytes());
    else r.skip(wt);
  }
  if (!r.ok) return false;
  if (content.size() == 1 && content[0].size() == t.size() * sizeof(float) && t.size() != 1) {
    std::memcpy(t.data(), content[0].data(), content[0].size());  // raw block
    return true;
  }
  if (content.size() != t.size()) return false;
  for (size_t i = 0; i < t.size(); ++i) t[i] = std::strtof(content[i].c_str(), nullptr);  // decimal per element
  return true;
}

// state field numbers per kind: accumulators after parameter (= 1)
std::string state_of(const Opt& o) {
  Writer w;
  w.bytes(101, o.lr.state());
  w.f64(104, o.num_sample_passed);
  w.bytes(1, tensor_proto(o.param));
  if (o.kind == 1) w.bytes(2, tensor_proto(o.a0));
  if (o.kind == 2) { w.bytes(2, tensor_proto(o.a0)); w.bytes(3, tensor_proto(o.a1)); w.bytes(4, tensor_proto(o.a2)); }
  if (o.kind == 3) w.bytes(2, tensor_proto(o.a0));
  if (o.kind == 4) { w.bytes(2, tensor_proto(o.a0)); w.bytes(3, tensor_proto(o.a1)); }
  return w.s;
}

bool load_state(const char* st, int len, Opt& o) {
  Reader r{(const uint8_t*)st, (const uint8_t*)st + len};
  while (r.more()) {
    const uint64_t k = r.varint();
    const int num = (int)(k >> 3), wt = (int)(k & 7);
    if (num == 101 && wt == 2) o.lr.load(r.bytes());
    else if (num == 104 && wt == 1) o.num_sample_passed = r.f64();
    else if (wt == 2 && num >= 1 && num <= 4) {
      const std::string m = r.bytes();
      std::vector<float>* t = num == 1 ? &o.param : num == 2 ? &o.a0 : num == 3 ? &o.a1 : &o.a2;
      if (!load_tensor(m, *t)) return false;
    } else {
      r.skip(wt);
    }
  }
  return r.ok;
}

void update(Opt& o, const float* g) {
  o.num_sample_passed += 1;
  const double n = o.num_sample_passed;
  const double lr = o.lr.at(n);
  float* p = o.param.data();
  const size_t N = o.param.size();
  switch (o.kind) {
    case 1: {  // SGD (+ momentum, nesterov)
      float* m = o.a0.data();
      for (size_t i = 0; i < N; ++i) {
        double v;
        if (o.momentum == 0.0) {
          v = -lr * g[i] - lr * o.decay * p[i];
        } else {
          m[i] = (float)(o.momentum * m[i] - lr * g[i] - lr * o.decay * p[i]);
          v = m[i];
        }
        p[i] = (float)(o.nesterov ? p[i] + o.momentum * v - lr * g[i] : p[i] + v);
      }
      break;
    }
    case 2: {  // Adadelta
      float *ag = o.a0.data(), *ad = o.a1.data(), *ud = o.a2.data();
      for (size_t i = 0; i < N; ++i) {
        ag[i] = (float)(o.rho * ag[i] + (1.0 - o.rho) * g[i] * g[i]);
        ud[i] = (float)(std::sqrt(ad[i] + o.eps) / std::sqrt(ag[i] + o.eps) * g[i]);
        ad[i] = (float)(o.rho * ad[i] + (1.0 - o.rho) * ud[i] * ud[i]);
        p[i] = (float)(p[i] - lr * ud[i] - lr * o.decay * p[i]);
      }
      break;
    }
    case 3: {  // Adagrad (descent; the reference's adagrad_optimizer.cc adds the step)
      float* ag = o.a0.data();
      for (size_t i = 0; i < N; ++i) {
        ag[i] += g[i] * g[i];
        p[i] = (float)(p[i] - lr * g[i] / std::sqrt(ag[i] + o.eps) - lr * o.decay * p[i]);
      }
      break;
    }
    case 4: {  // Adam (bias corrections folded into the step size)
      const double c1 = 1.0 - std::pow(o.beta1, n), c2 = 1.0 - std::pow(o.beta2, n);
      const double a = lr * std::sqrt(c2) / c1;
      float *m = o.a0.data(), *v = o.a1.data();
      for (size_t i = 0; i < N; ++i) {
        m[i] = (float)(o.beta1 * m[i] + (1.0 - o.beta1) * g[i]);
        v[i] = (float)(o.beta2 * v[i] + (1.0 - o.beta2) * g[i] * g[i]);
        p[i] = (float)(p[i] - a * (m[i] / std::sqrt(v[i] + o.eps) + o.decay * p[i]));
      }
      break;
    }
  }
}

struct Handle {
  Opt o;
  std::string state;  // buffer of the last get_state
};

}  // namespace

PA_RT_EXPORT void* pa_opt_create(const unsigned char* config, int config_len, int dtype, void* param, int num_bytes,
                                 const char* state, int state_len) {
  if (dtype != 4 || !config || num_bytes < 0 || num_bytes % 4) return nullptr;  // float32 only, as the reference
  auto h = std::make_unique<Handle>();
  if (!parse_config(config, config_len, h->o)) return nullptr;
  const size_t n = (size_t)num_bytes / 4;
  h->o.param.assign(n, 0.f);
  if (param) std::memcpy(h->o.param.data(), param, (size_t)num_bytes);
  const int nacc = h->o.kind == 2 ? 3 : h->o.kind == 4 ? 2 : 1;
  h->o.a0.assign(n, 0.f);
  if (nacc > 1) h->o.a1.assign(n, 0.f);
  if (nacc > 2) h->o.a2.assign(n, 0.f);
  if (state && state_len > 0 && !load_state(state, state_len, h->o)) return nullptr;
  return h.release();
}

PA_RT_EXPORT int pa_opt_release(void* h) {
  delete (Handle*)h;
  return 0;
}

PA_RT_EXPORT int pa_opt_update(void* h, int dtype, const void* grad, int num_bytes) {
  auto* H = (Handle*)h;
  if (!H || dtype != 4 || (size_t)num_bytes != H->o.param.size() * 4) return -1;
  update(H->o, (const float*)grad);
  return 0;
}

PA_RT_EXPORT int pa_opt_get_weights(void* h, void** buf) {
  auto* H = (Handle*)h;
  *buf = H->o.param.data();
  return (int)H->o.param.size();
}

PA_RT_EXPORT int pa_opt_get_state(void* h, const char** st) {
  auto* H = (Handle*)h;
  H->state = state_of(H->o);
  *st = H->state.data();
  return (int)H->state.size();
}

// the reference's C names (optimizer.h)
PA_RT_EXPORT void* paddle_create_optimizer(const unsigned char* config, const int config_len, const int dtype,
                                           void* param, int num_bytes, const char* state, const int state_len) {
  return pa_opt_create(config, config_len, dtype, param, num_bytes, state, state_len);
}
PA_RT_EXPORT int paddle_release_optimizer(void* o) { return pa_opt_release(o); }
PA_RT_EXPORT int paddle_update_parameter(void* o, const int dtype, const void* g, int num_bytes) {
  return pa_opt_update(o, dtype, g, num_bytes);
}
PA_RT_EXPORT int paddle_optimizer_get_weights(void* o, void** buf) { return pa_opt_get_weights(o, buf); }
PA_RT_EXPORT int paddle_optimizer_get_state(void* o, const char** st) { return pa_opt_get_state(o, st); }
