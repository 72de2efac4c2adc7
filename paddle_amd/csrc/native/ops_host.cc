// Host (CPU) kernels of the native executor.  Semantics follow the reference
// operators (paddle/fluid/operators/*_op.{h,cc}); the file:line of the behaviour
// each kernel mirrors is cited at the kernel.  fp32 compute, int64 ids/labels.
#include <math.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <limits>
#include <numeric>

#include "framework.h"

namespace pa {
namespace {

using Dims = std::vector<int64_t>;

int64_t prod(const Dims& d, size_t b = 0, size_t e = (size_t)-1) {
  int64_t n = 1;
  for (size_t i = b; i < std::min(e, d.size()); ++i) n *= d[i];
  return n;
}

// a dtype the host kernels do not cover declines the op (the executor then runs the
// embedder's kernel for it, or reports the op as unsupported)
float* f32(Tensor& t) {
  if (t.dtype != DT::FP32) throw Decline{};
  return t.data<float>();
}

std::vector<int64_t> ids_of(const Tensor& t) {
  std::vector<int64_t> v((size_t)t.numel());
  if (t.dtype == DT::INT64) memcpy(v.data(), t.raw(), v.size() * 8);
  else if (t.dtype == DT::INT32)
    for (size_t i = 0; i < v.size(); ++i) v[i] = t.data<int32_t>()[i];
  else throw Decline{};  // not an integer index tensor
  return v;
}

// ------------------------------------------------------------ feed / fetch (feed_op.cc, fetch_op.cc)
void k_feed(const OpRun& r) {
  Variable* x = r.var(r.op.Input("X"));
  const int64_t col = r.op.GetInt("col");
  PA_CHECK(col >= 0 && col < (int64_t)x->list.size(), "feed: column %lld not fed", (long long)col);
  r.out("Out")->share(x->list[(size_t)col]);
}

void k_fetch(const OpRun& r) {
  Tensor& x = r.in("X");
  Variable* out = r.var(r.op.Output("Out"));
  out->kind = VK_FETCH_LIST;
  const size_t col = (size_t)r.op.GetInt("col");
  if (out->list.size() <= col) out->list.resize(col + 1);
  out->list[col] = x.device >= 0 ? x.to(-1, r.ctx.stream) : x;
}

// ------------------------------------------------------------ initialisers
void k_fill_constant(const OpRun& r) {
  Tensor* o = r.out("Out");
  const DT dt = (DT)r.op.GetInt("dtype", (int)DT::FP32);
  const double v = r.op.Has("str_value") && !r.op.GetString("str_value").empty()
                       ? atof(r.op.GetString("str_value").c_str())
                       : (double)r.op.GetFloat("value");
  o->alloc(dt, r.op.GetInts("shape"), -1);
  const int64_t n = o->numel();
  switch (dt) {
    case DT::FP32: std::fill_n(o->data<float>(), n, (float)v); break;
    case DT::FP64: std::fill_n(o->data<double>(), n, v); break;
    case DT::INT64: std::fill_n(o->data<int64_t>(), n, (int64_t)v); break;
    case DT::INT32: std::fill_n(o->data<int32_t>(), n, (int32_t)v); break;
    case DT::BOOL: case DT::UINT8: std::fill_n(o->data<uint8_t>(), n, (uint8_t)v); break;
    default: fail("fill_constant: dtype %s", dt_name(dt));
  }
}

// the shape attr; the *_batch_size_like forms take shape[output_dim_idx] from
// Input.dims[input_dim_idx] (batch_size_like.h)
Dims random_shape(const OpRun& r) {
  Dims shape = r.op.GetInts("shape");
  if (r.op.type.find("batch_size_like") == std::string::npos) return shape;
  const Tensor& in = r.in("Input");
  const size_t oi = (size_t)r.op.GetInt("output_dim_idx", 0), ii = (size_t)r.op.GetInt("input_dim_idx", 0);
  PA_CHECK(oi < shape.size() && ii < in.dims.size(), "%s: dim index out of range", r.op.type.c_str());
  shape[oi] = in.dims[ii];
  return shape;
}

void k_uniform_random(const OpRun& r) {
  Tensor* o = r.out("Out");
  float* p = o->alloc<float>(random_shape(r), -1);
  const int64_t seed = r.op.GetInt("seed");
  std::mt19937_64 g(seed ? (uint64_t)seed : r.ctx.rng());
  std::uniform_real_distribution<float> d(r.op.GetFloat("min", -1.f), r.op.GetFloat("max", 1.f));
  for (int64_t i = 0; i < o->numel(); ++i) p[i] = d(g);
}

void k_gaussian_random(const OpRun& r) {
  Tensor* o = r.out("Out");
  float* p = o->alloc<float>(random_shape(r), -1);
  const int64_t seed = r.op.GetInt("seed");
  std::mt19937_64 g(seed ? (uint64_t)seed : r.ctx.rng());
  std::normal_distribution<float> d(r.op.GetFloat("mean", 0.f), r.op.GetFloat("std", 1.f));
  for (int64_t i = 0; i < o->numel(); ++i) p[i] = d(g);
}

void k_assign(const OpRun& r) {
  Tensor& x = r.in("X");
  Tensor* o = r.out("Out");
  LoD lod = x.lod;
  o->alloc(x.dtype, x.dims, -1);
  memcpy(o->raw(), x.raw(), x.nbytes());
  o->lod = lod;
}

void k_shape(const OpRun& r) {
  Tensor& x = r.in("Input");
  Tensor* o = r.out("Out");
  Dims d = x.dims;
  int32_t* p = o->alloc<int32_t>({(int64_t)d.size()}, -1);
  for (size_t i = 0; i < d.size(); ++i) p[i] = (int32_t)d[i];
}

// bf16 / fp16 <-> float on the host (round to nearest even; fp16 with subnormals)
float bf16_to_f(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
uint16_t f_to_bf16(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
float f16_to_f(uint16_t h) {
  const uint32_t s = (uint32_t)(h & 0x8000) << 16, e = (h >> 10) & 0x1f, m = h & 0x3ff;
  float v;
  if (e == 0) v = std::ldexp((float)m, -24);
  else if (e == 31) v = m ? std::numeric_limits<float>::quiet_NaN() : std::numeric_limits<float>::infinity();
  else v = std::ldexp((float)(m | 0x400), (int)e - 25);
  return s ? -v : v;
}
uint16_t f_to_f16(float f) {
  const uint16_t s = std::signbit(f) ? 0x8000 : 0;
  const float a = std::fabs(f);
  if (std::isnan(f)) return (uint16_t)(s | 0x7e00);
  if (a >= 65520.f) return (uint16_t)(s | 0x7c00);
  if (a < 6.103515625e-05f) return (uint16_t)(s | (uint16_t)std::nearbyint(a * 16777216.f));  // subnormal
  int e;
  const float fr = std::frexp(a, &e);  // a = fr * 2^e, fr in [0.5, 1)
  uint32_t m = (uint32_t)std::nearbyint(fr * 2048.f);  // 11 significant bits
  if (m == 2048) { m = 1024; ++e; }
  const uint32_t he = (uint32_t)(e + 14);
  if (he >= 31) return (uint16_t)(s | 0x7c00);
  return (uint16_t)(s | (he << 10) | (m & 0x3ff));
}

void k_cast(const OpRun& r) {
  // everything read from X before r.out(): creating Out may invalidate the reference
  const Tensor& x = r.in("X");
  const DT out = (DT)r.op.GetInt("out_dtype", (int)DT::FP32);
  const int64_t n = x.numel();
  std::vector<double> tmp((size_t)n);
  switch (x.dtype) {
    case DT::FP32: for (int64_t i = 0; i < n; ++i) tmp[i] = x.data<float>()[i]; break;
    case DT::FP64: for (int64_t i = 0; i < n; ++i) tmp[i] = x.data<double>()[i]; break;
    case DT::INT64: for (int64_t i = 0; i < n; ++i) tmp[i] = (double)x.data<int64_t>()[i]; break;
    case DT::INT32: for (int64_t i = 0; i < n; ++i) tmp[i] = x.data<int32_t>()[i]; break;
    case DT::BOOL: case DT::UINT8: for (int64_t i = 0; i < n; ++i) tmp[i] = x.data<uint8_t>()[i]; break;
    case DT::BF16: for (int64_t i = 0; i < n; ++i) tmp[i] = bf16_to_f(x.data<uint16_t>()[i]); break;
    case DT::FP16: for (int64_t i = 0; i < n; ++i) tmp[i] = f16_to_f(x.data<uint16_t>()[i]); break;
    default: throw Decline{};
  }
  const LoD lod = x.lod;
  const Dims d = x.dims;
  Tensor* o = r.out("Out");
  switch (out) {
    case DT::FP32: case DT::FP64: case DT::INT64: case DT::INT32: case DT::BOOL: case DT::UINT8: case DT::BF16:
    case DT::FP16: break;
    default: throw Decline{};
  }
  o->alloc(out, d, -1);
  o->lod = lod;
  switch (out) {
    case DT::FP32: for (int64_t i = 0; i < n; ++i) o->data<float>()[i] = (float)tmp[i]; break;
    case DT::FP64: for (int64_t i = 0; i < n; ++i) o->data<double>()[i] = tmp[i]; break;
    case DT::INT64: for (int64_t i = 0; i < n; ++i) o->data<int64_t>()[i] = (int64_t)tmp[i]; break;
    case DT::INT32: for (int64_t i = 0; i < n; ++i) o->data<int32_t>()[i] = (int32_t)tmp[i]; break;
    case DT::BOOL: case DT::UINT8: for (int64_t i = 0; i < n; ++i) o->data<uint8_t>()[i] = tmp[i] != 0; break;
    case DT::BF16: for (int64_t i = 0; i < n; ++i) o->data<uint16_t>()[i] = f_to_bf16((float)tmp[i]); break;
    case DT::FP16: for (int64_t i = 0; i < n; ++i) o->data<uint16_t>()[i] = f_to_f16((float)tmp[i]); break;
    default: break;
  }
}

// ------------------------------------------------------------ mul / matmul / fc
// mul_op.cc: X flattened to [prod(x[:xnc]), prod(x[xnc:])], Y to [prod(y[:ync]), ...]
void k_mul(const OpRun& r) {
  Tensor& x = r.in("X");
  Tensor& y = r.in("Y");
  const size_t xnc = (size_t)r.op.GetInt("x_num_col_dims", 1), ync = (size_t)r.op.GetInt("y_num_col_dims", 1);
  const int64_t M = prod(x.dims, 0, xnc), K = prod(x.dims, xnc), N = prod(y.dims, ync);
  PA_CHECK(prod(y.dims, 0, ync) == K, "mul: X %s and Y %s do not match", x.shape_str().c_str(),
           y.shape_str().c_str());
  Dims od(x.dims.begin(), x.dims.begin() + xnc);
  od.insert(od.end(), y.dims.begin() + ync, y.dims.end());
  LoD lod = x.lod;
  Tensor* o = r.out("Out");
  float* c = o->alloc<float>(od, -1);
  sgemm(false, false, M, N, K, 1.f, f32(x), K, f32(y), N, 0.f, c, N);
  o->lod = lod;
}

void k_mul_grad(const OpRun& r) {
  Tensor& x = r.in("X");
  Tensor& y = r.in("Y");
  Tensor& dout = r.in("Out@GRAD");
  const size_t xnc = (size_t)r.op.GetInt("x_num_col_dims", 1), ync = (size_t)r.op.GetInt("y_num_col_dims", 1);
  const int64_t M = prod(x.dims, 0, xnc), K = prod(x.dims, xnc), N = prod(y.dims, ync);
  if (Tensor* dx = r.out("X@GRAD")) {
    Dims d = x.dims;
    sgemm(false, true, M, K, N, 1.f, f32(dout), N, f32(y), N, 0.f, dx->alloc<float>(d, -1), K);
  }
  if (Tensor* dy = r.out("Y@GRAD")) {
    Dims d = y.dims;
    sgemm(true, false, K, N, M, 1.f, f32(x), K, f32(dout), N, 0.f, dy->alloc<float>(d, -1), N);
  }
}

// matmul_op.cc: batched, optional transposes, alpha; rank-1 operands promoted
void k_matmul(const OpRun& r) {
  Tensor& x = r.in("X");
  Tensor& y = r.in("Y");
  const bool tx = r.op.GetBool("transpose_X"), ty = r.op.GetBool("transpose_Y");
  const float alpha = r.op.GetFloat("alpha", 1.f);
  Dims xd = x.dims, yd = y.dims;
  const bool xv = xd.size() == 1, yv = yd.size() == 1;
  if (xv) xd = tx ? Dims{xd[0], 1} : Dims{1, xd[0]};
  if (yv) yd = ty ? Dims{1, yd[0]} : Dims{yd[0], 1};
  const int64_t xr = xd[xd.size() - 2], xc = xd.back(), yr = yd[yd.size() - 2], yc = yd.back();
  const int64_t M = tx ? xc : xr, K = tx ? xr : xc, N = ty ? yr : yc;
  PA_CHECK((ty ? yc : yr) == K, "matmul: inner dims differ (%s x %s)", x.shape_str().c_str(),
           y.shape_str().c_str());
  const int64_t bx = prod(xd, 0, xd.size() - 2), by = prod(yd, 0, yd.size() - 2);
  PA_CHECK(bx == by || bx == 1 || by == 1, "matmul: batch dims differ");
  const int64_t B = std::max(bx, by);
  Dims od(xd.size() >= yd.size() ? xd.begin() : yd.begin(),
          xd.size() >= yd.size() ? xd.end() - 2 : yd.end() - 2);
  if (bx == 1 && by > 1) od.assign(yd.begin(), yd.end() - 2);
  if (!xv) od.push_back(M);
  if (!yv) od.push_back(N);
  if (od.empty()) od.push_back(1);
  Tensor* o = r.out("Out");
  float* c = o->alloc<float>(od, -1);
  const float* a = f32(x);
  const float* b = f32(y);
  for (int64_t i = 0; i < B; ++i)
    sgemm(tx, ty, M, N, K, alpha, a + (bx == 1 ? 0 : i * M * K), tx ? M : K, b + (by == 1 ? 0 : i * K * N),
          ty ? K : N, 0.f, c + i * M * N, N);
}

// fc_op.cc (fused by fc_fuse_pass): Input [.., K] x W [K, N] + Bias
void k_fc(const OpRun& r) {
  Tensor& x = r.in("Input");
  Tensor& w = r.in("W");
  Tensor* b = r.in_opt("Bias");
  const size_t nc = (size_t)r.op.GetInt("in_num_col_dims", 1);
  const int64_t M = prod(x.dims, 0, nc), K = prod(x.dims, nc), N = w.dims[1];
  Dims od(x.dims.begin(), x.dims.begin() + nc);
  od.push_back(N);
  Tensor* o = r.out("Out");
  float* c = o->alloc<float>(od, -1);
  if (b) {
    const float* bp = f32(*b);
    for (int64_t i = 0; i < M; ++i) memcpy(c + i * N, bp, sizeof(float) * N);
  }
  sgemm(false, false, M, N, K, 1.f, f32(x), K, f32(w), N, b ? 1.f : 0.f, c, N);
  const std::string act = r.op.GetString("activation_type");
  if (act == "relu")
    for (int64_t i = 0; i < M * N; ++i) c[i] = c[i] > 0 ? c[i] : 0;
  else if (act == "tanh")
    for (int64_t i = 0; i < M * N; ++i) c[i] = tanhf(c[i]);
  else if (act == "sigmoid")
    for (int64_t i = 0; i < M * N; ++i) c[i] = 1.f / (1.f + expf(-c[i]));
  else if (act == "gelu")
    for (int64_t i = 0; i < M * N; ++i) c[i] = 0.5f * c[i] * (1.f + erff(c[i] * 0.70710678f));
  else if (!act.empty())
    throw Decline{};
}

// ------------------------------------------------------------ elementwise (elementwise_op_function.h)
// Y is aligned to X at `axis` (trailing size-1 dims of Y trimmed); the common case
// is X [pre, n, post] with Y [n].  Anything else goes through the strided path.
struct Bc {
  Dims out, sx, sy;  // out shape, x/y strides in out index space (0 = broadcast)
};

Bc broadcast(const Dims& x, const Dims& y0, int64_t axis) {
  Dims y = y0;
  const int64_t xr = (int64_t)x.size();
  if (axis < 0) axis = xr - (int64_t)y.size();
  if (axis < 0) {  // Y has the larger rank: numpy-style right alignment
    axis = 0;
  }
  Dims yf((size_t)std::max<int64_t>(xr, (int64_t)y.size()), 1);
  Dims xf = x;
  if ((int64_t)y.size() > xr) {
    xf.insert(xf.begin(), y.size() - x.size(), 1);
    yf = y;
  } else {
    for (size_t i = 0; i < y.size(); ++i) yf[(size_t)axis + i] = y[i];
  }
  Bc b;
  const size_t R = xf.size();
  b.out.resize(R);
  for (size_t i = 0; i < R; ++i) {
    PA_CHECK(xf[i] == yf[i] || xf[i] == 1 || yf[i] == 1, "elementwise: shapes do not broadcast");
    b.out[i] = std::max(xf[i], yf[i]);
  }
  b.sx.assign(R, 0);
  b.sy.assign(R, 0);
  int64_t s1 = 1, s2 = 1;
  for (size_t i = R; i-- > 0;) {
    b.sx[i] = xf[i] == 1 ? 0 : s1;
    b.sy[i] = yf[i] == 1 ? 0 : s2;
    s1 *= xf[i];
    s2 *= yf[i];
  }
  return b;
}

template <class T, class F> void ew_apply(const Bc& b, const T* x, const T* y, T* o, F f) {
  const int64_t n = prod(b.out);
  const size_t R = b.out.size();
  if (R == 0) {
    o[0] = f(x[0], y[0]);
    return;
  }
  const int64_t inner = b.out[R - 1], ix = b.sx[R - 1], iy = b.sy[R - 1];
  const int64_t rows = n / std::max<int64_t>(inner, 1);
  parallel_for(rows, 64, [&](int64_t r0, int64_t r1) {
    for (int64_t row = r0; row < r1; ++row) {
      int64_t rem = row, ox = 0, oy = 0;
      for (size_t d = R - 1; d-- > 0;) {
        const int64_t k = rem % b.out[d];
        rem /= b.out[d];
        ox += k * b.sx[d];
        oy += k * b.sy[d];
      }
      T* op = o + row * inner;
      if (ix == 1 && iy == 1)
        for (int64_t j = 0; j < inner; ++j) op[j] = f(x[ox + j], y[oy + j]);
      else if (ix == 1 && iy == 0) {
        const T yv = y[oy];
        for (int64_t j = 0; j < inner; ++j) op[j] = f(x[ox + j], yv);
      } else
        for (int64_t j = 0; j < inner; ++j) op[j] = f(x[ox + j * ix], y[oy + j * iy]);
    }
  });
}

template <class F> Kernel ew_kernel(F f) {
  return [f](const OpRun& r) {
    Tensor& x = r.in("X");
    Tensor& y = r.in("Y");
    const Bc b = broadcast(x.dims, y.dims, r.op.GetInt("axis", -1));
    LoD lod = x.lod;
    Tensor* o = r.out("Out");
    Tensor xs = x, ys = y;  // keep inputs alive if Out aliases one of them
    if (xs.dtype == DT::FP32 || ys.dtype != xs.dtype || xs.device >= 0 || ys.device >= 0) {
      ew_apply(b, f32(xs), f32(ys), o->alloc<float>(b.out, -1), f);
    } else if (xs.dtype == DT::INT64) {  // integer index arithmetic (elementwise_op.h int kernels)
      ew_apply(b, xs.data<int64_t>(), ys.data<int64_t>(), static_cast<int64_t*>(o->alloc(DT::INT64, b.out, -1)), f);
    } else if (xs.dtype == DT::INT32) {
      ew_apply(b, xs.data<int32_t>(), ys.data<int32_t>(), static_cast<int32_t*>(o->alloc(DT::INT32, b.out, -1)), f);
    } else {
      throw Decline{};
    }
    o->lod = lod;
  };
}

// sum of g (shape b.out) onto a tensor with strides s (shape = b.out where s != 0)
void reduce_to(const Bc& b, const Dims& s, const float* g, float* dst, int64_t dst_n, float sign) {
  memset(dst, 0, sizeof(float) * dst_n);
  const size_t R = b.out.size();
  const int64_t n = prod(b.out);
  std::vector<int64_t> idx(R, 0);
  for (int64_t i = 0; i < n; ++i) {
    int64_t off = 0;
    for (size_t d = 0; d < R; ++d) off += idx[d] * s[d];
    dst[off] += sign * g[i];
    for (size_t d = R; d-- > 0;) {
      if (++idx[d] < b.out[d]) break;
      idx[d] = 0;
    }
  }
}

// elementwise_{add,sub,mul,div}_grad (elementwise_*_op.h)
template <int KIND>  // 0 add, 1 sub, 2 mul, 3 div
void k_ew_grad(const OpRun& r) {
  Tensor& x = r.in("X");
  Tensor& y = r.in("Y");
  Tensor& g = r.in("Out@GRAD");
  const Bc b = broadcast(x.dims, y.dims, r.op.GetInt("axis", -1));
  const int64_t n = prod(b.out);
  std::vector<float> gx((size_t)n), gy((size_t)n);
  const float* gp = f32(g);
  // expand x / y to the output shape where needed
  std::vector<float> xe, ye;
  if (KIND >= 2) {
    xe.resize((size_t)n);
    ye.resize((size_t)n);
    ew_apply(b, f32(x), f32(y), xe.data(), [](float a, float) { return a; });
    ew_apply(b, f32(x), f32(y), ye.data(), [](float, float c) { return c; });
  }
  for (int64_t i = 0; i < n; ++i) {
    switch (KIND) {
      case 0: gx[i] = gp[i]; gy[i] = gp[i]; break;
      case 1: gx[i] = gp[i]; gy[i] = -gp[i]; break;
      case 2: gx[i] = gp[i] * ye[i]; gy[i] = gp[i] * xe[i]; break;
      case 3: gx[i] = gp[i] / ye[i]; gy[i] = -gp[i] * xe[i] / (ye[i] * ye[i]); break;
    }
  }
  if (Tensor* dx = r.out("X@GRAD")) {
    Dims d = x.dims;
    reduce_to(b, b.sx, gx.data(), dx->alloc<float>(d, -1), prod(d), 1.f);
  }
  if (Tensor* dy = r.out("Y@GRAD")) {
    Dims d = y.dims;
    reduce_to(b, b.sy, gy.data(), dy->alloc<float>(d, -1), prod(d), 1.f);
  }
}

// ------------------------------------------------------------ unary activations (activation_op.h)
template <class F> Kernel unary(F f) {
  return [f](const OpRun& r) {
    Tensor& x = r.in("X");
    Tensor xs = x;
    Tensor* o = r.out("Out");
    LoD lod = x.lod;
    Dims d = x.dims;
    float* op = o->alloc<float>(d, -1);
    const float* xp = f32(xs);
    parallel_for(xs.numel(), 4096, [&](int64_t a, int64_t e) {
      for (int64_t i = a; i < e; ++i) op[i] = f(xp[i], r.op);
    });
    o->lod = lod;
  };
}

// grad kernels taking (x, out, dout) -> dx
template <class F> Kernel unary_grad(F f) {
  return [f](const OpRun& r) {
    Tensor* x = r.in_opt("X");
    Tensor* out = r.in_opt("Out");
    Tensor& g = r.in("Out@GRAD");
    Tensor* dx = r.out("X@GRAD");
    if (!dx) return;
    Dims d = g.dims;
    Tensor gs = g;
    float* dp = dx->alloc<float>(d, -1);
    const float* xp = x ? f32(*x) : nullptr;
    const float* opp = out ? f32(*out) : nullptr;
    const float* gp = f32(gs);
    for (int64_t i = 0; i < gs.numel(); ++i) dp[i] = f(xp ? xp[i] : 0.f, opp ? opp[i] : 0.f, gp[i], r.op);
  };
}

float sigm(float v) { return 1.f / (1.f + expf(-v)); }

// ------------------------------------------------------------ scale / sum / mean / reductions
void k_scale(const OpRun& r) {
  const float s = r.op.GetFloat("scale", 1.f), bias = r.op.GetFloat("bias", 0.f);
  const bool after = r.op.GetBool("bias_after_scale", true);
  unary([s, bias, after](float v, const OpDesc&) { return after ? v * s + bias : (v + bias) * s; })(r);
}

void k_scale_grad(const OpRun& r) {  // dX = scale * dOut (bias drops out)
  Tensor& g = r.in("Out@GRAD");
  Tensor gs = g;
  Tensor* dx = r.out("X@GRAD");
  if (!dx) return;
  const float s = r.op.GetFloat("scale", 1.f);
  const LoD lod = gs.lod;
  const Dims d = gs.dims;
  float* o = dx->alloc<float>(d, -1);
  const float* gp = f32(gs);
  for (int64_t i = 0; i < gs.numel(); ++i) o[i] = s * gp[i];
  dx->lod = lod;
}

void k_sum(const OpRun& r) {
  if (selected_rows_sum(r)) return;
  auto xs = r.ins("X");
  PA_CHECK(!xs.empty(), "sum: no inputs");
  std::vector<Tensor> keep;
  for (auto* t : xs) keep.push_back(*t);
  Dims d = keep[0].dims;
  LoD lod = keep[0].lod;
  Tensor* o = r.out("Out");
  float* op = o->alloc<float>(d, -1);
  const int64_t n = prod(d);
  std::vector<float> acc((size_t)n, 0.f);
  for (auto& t : keep) {
    PA_CHECK(t.numel() == n, "sum: input sizes differ");
    const float* p = f32(t);
    for (int64_t i = 0; i < n; ++i) acc[i] += p[i];
  }
  memcpy(op, acc.data(), sizeof(float) * n);
  o->lod = lod;
}

void k_mean(const OpRun& r) {
  Tensor& x = r.in("X");
  const float* p = f32(x);
  double s = 0;
  for (int64_t i = 0; i < x.numel(); ++i) s += p[i];
  r.out("Out")->alloc<float>({1}, -1)[0] = (float)(s / std::max<int64_t>(1, x.numel()));
}

void k_mean_grad(const OpRun& r) {
  Tensor& x = r.in("X");
  const float g = f32(r.in("Out@GRAD"))[0];
  Dims d = x.dims;
  const int64_t n = prod(d);
  std::fill_n(r.out("X@GRAD")->alloc<float>(d, -1), n, g / (float)std::max<int64_t>(1, n));
}

// reduce_op.h: dim (list), keep_dim, reduce_all
template <int KIND>  // 0 sum, 1 mean, 2 max, 3 min, 4 prod
void k_reduce(const OpRun& r) {
  Tensor& x = r.in("X");
  const Dims xd = x.dims;
  const int64_t R = (int64_t)xd.size();
  std::vector<bool> red((size_t)R, r.op.GetBool("reduce_all"));
  for (int64_t a : r.op.GetInts("dim")) red[(size_t)(a < 0 ? a + R : a)] = true;
  Dims od, kd;
  for (int64_t i = 0; i < R; ++i) {
    if (!red[(size_t)i]) od.push_back(xd[(size_t)i]);
    kd.push_back(red[(size_t)i] ? 1 : xd[(size_t)i]);
  }
  const bool keep = r.op.GetBool("keep_dim");
  Dims outd = keep ? kd : (od.empty() ? Dims{1} : od);
  const int64_t on = prod(kd);
  std::vector<double> acc((size_t)on, KIND == 2 ? -INFINITY : KIND == 3 ? INFINITY : KIND == 4 ? 1.0 : 0.0);
  std::vector<int64_t> cnt((size_t)on, 0);
  const float* p = f32(x);
  const int64_t n = prod(xd);
  std::vector<int64_t> idx((size_t)R, 0);
  for (int64_t i = 0; i < n; ++i) {
    int64_t o = 0;
    for (int64_t d = 0; d < R; ++d) o = o * kd[(size_t)d] + (red[(size_t)d] ? 0 : idx[(size_t)d]);
    const double v = p[i];
    switch (KIND) {
      case 0: case 1: acc[o] += v; break;
      case 2: acc[o] = std::max(acc[o], v); break;
      case 3: acc[o] = std::min(acc[o], v); break;
      case 4: acc[o] *= v; break;
    }
    cnt[o]++;
    for (int64_t d = R; d-- > 0;) {
      if (++idx[(size_t)d] < xd[(size_t)d]) break;
      idx[(size_t)d] = 0;
    }
  }
  float* op = r.out("Out")->alloc<float>(outd, -1);
  for (int64_t i = 0; i < on; ++i) op[i] = (float)(KIND == 1 ? acc[i] / std::max<int64_t>(1, cnt[i]) : acc[i]);
}

// ------------------------------------------------------------ softmax / cross entropy
void softmax_rows(const float* x, float* y, int64_t rows, int64_t n) {
  parallel_for(rows, 16, [&](int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i) {
      const float* xr = x + i * n;
      float* yr = y + i * n;
      float m = -INFINITY;
      for (int64_t j = 0; j < n; ++j) m = std::max(m, xr[j]);
      double s = 0;
      for (int64_t j = 0; j < n; ++j) s += (yr[j] = expf(xr[j] - m));
      const float inv = (float)(1.0 / s);
      for (int64_t j = 0; j < n; ++j) yr[j] *= inv;
    }
  });
}

void k_softmax(const OpRun& r) {
  Tensor x = r.in("X");
  int64_t axis = r.op.GetInt("axis", -1);
  if (axis < 0) axis += (int64_t)x.dims.size();
  PA_CHECK(axis == (int64_t)x.dims.size() - 1, "softmax: only the last axis is supported on the host");
  const int64_t n = x.dims.back();
  Tensor* o = r.out("Out");
  Dims d = x.dims;
  softmax_rows(f32(x), o->alloc<float>(d, -1), x.numel() / n, n);
  o->lod = x.lod;
}

void k_softmax_grad(const OpRun& r) {
  Tensor& y = r.in("Out");
  Tensor& g = r.in("Out@GRAD");
  const int64_t n = y.dims.back(), rows = y.numel() / n;
  Dims d = y.dims;
  float* dx = r.out("X@GRAD")->alloc<float>(d, -1);
  const float* yp = f32(y);
  const float* gp = f32(g);
  for (int64_t i = 0; i < rows; ++i) {
    double dot = 0;
    for (int64_t j = 0; j < n; ++j) dot += (double)yp[i * n + j] * gp[i * n + j];
    for (int64_t j = 0; j < n; ++j) dx[i * n + j] = yp[i * n + j] * (gp[i * n + j] - (float)dot);
  }
}

// cross_entropy_op.h (hard labels): Y = -log(X[label])
void k_cross_entropy(const OpRun& r) {
  Tensor& x = r.in("X");
  Tensor& l = r.in("Label");
  PA_CHECK(!r.op.GetBool("soft_label"), "cross_entropy: soft labels not supported on the host");
  const int64_t n = x.dims.back(), rows = x.numel() / n;
  auto lab = ids_of(l);
  const int64_t ignore = r.op.GetInt("ignore_index", -100);
  Dims od(x.dims.begin(), x.dims.end() - 1);
  od.push_back(1);
  float* y = r.out("Y")->alloc<float>(od, -1);
  const float* p = f32(x);
  for (int64_t i = 0; i < rows; ++i) {
    const int64_t c = lab[(size_t)i];
    y[i] = c == ignore ? 0.f : -logf(std::max(p[i * n + c], 1e-20f));
  }
}

void k_cross_entropy_grad(const OpRun& r) {
  Tensor& x = r.in("X");
  Tensor& l = r.in("Label");
  Tensor& g = r.in("Y@GRAD");
  const int64_t n = x.dims.back(), rows = x.numel() / n;
  auto lab = ids_of(l);
  const int64_t ignore = r.op.GetInt("ignore_index", -100);
  Dims d = x.dims;
  float* dx = r.out("X@GRAD")->alloc<float>(d, -1);
  memset(dx, 0, sizeof(float) * rows * n);
  const float* p = f32(x);
  for (int64_t i = 0; i < rows; ++i) {
    const int64_t c = lab[(size_t)i];
    if (c != ignore) dx[i * n + c] = -f32(g)[i] / std::max(p[i * n + c], 1e-20f);
  }
}

// softmax_with_cross_entropy_op.h (hard labels)
void k_softmax_ce(const OpRun& r) {
  Tensor& x = r.in("Logits");
  Tensor& l = r.in("Label");
  const int64_t n = x.dims.back(), rows = x.numel() / n;
  auto lab = ids_of(l);
  const int64_t ignore = r.op.GetInt("ignore_index", -100);
  Dims d = x.dims;
  float* sm = r.out("Softmax")->alloc<float>(d, -1);
  softmax_rows(f32(x), sm, rows, n);
  Dims od(d.begin(), d.end() - 1);
  od.push_back(1);
  float* loss = r.out("Loss")->alloc<float>(od, -1);
  for (int64_t i = 0; i < rows; ++i) {
    const int64_t c = lab[(size_t)i];
    loss[i] = c == ignore ? 0.f : -logf(std::max(sm[i * n + c], 1e-20f));
  }
}

void k_softmax_ce_grad(const OpRun& r) {
  Tensor& sm = r.in("Softmax");
  Tensor& l = r.in("Label");
  Tensor& g = r.in("Loss@GRAD");
  const int64_t n = sm.dims.back(), rows = sm.numel() / n;
  auto lab = ids_of(l);
  const int64_t ignore = r.op.GetInt("ignore_index", -100);
  Dims d = sm.dims;
  float* dx = r.out("Logits@GRAD")->alloc<float>(d, -1);
  const float* s = f32(sm);
  const float* gp = f32(g);
  for (int64_t i = 0; i < rows; ++i) {
    const int64_t c = lab[(size_t)i];
    for (int64_t j = 0; j < n; ++j)
      dx[i * n + j] = c == ignore ? 0.f : gp[i] * (s[i * n + j] - (j == c ? 1.f : 0.f));
  }
}

// accuracy_op.h: Out (top-k indices) vs Label
void k_accuracy(const OpRun& r) {
  Tensor& idx = r.in("Indices");
  Tensor& lab = r.in("Label");
  const int64_t k = idx.dims.back(), rows = idx.numel() / k;
  auto ii = ids_of(idx);
  auto ll = ids_of(lab);
  int64_t correct = 0;
  for (int64_t i = 0; i < rows; ++i)
    for (int64_t j = 0; j < k; ++j)
      if (ii[(size_t)(i * k + j)] == ll[(size_t)i]) {
        ++correct;
        break;
      }
  r.out("Accuracy")->alloc<float>({1}, -1)[0] = rows ? (float)correct / (float)rows : 0.f;
  if (Tensor* c = r.out("Correct")) c->alloc<int32_t>({1}, -1)[0] = (int32_t)correct;
  if (Tensor* t = r.out("Total")) t->alloc<int32_t>({1}, -1)[0] = (int32_t)rows;
}

// top_k_op.h: last axis, values + int64 indices
void k_top_k(const OpRun& r) {
  Tensor& x = r.in("X");
  const int64_t k = r.op.GetInt("k", 1);
  const int64_t n = x.dims.back(), rows = x.numel() / n;
  Dims od = x.dims;
  od.back() = k;
  const float* p = f32(x);
  Tensor xs = x;
  float* v = r.out("Out")->alloc<float>(od, -1);
  int64_t* ix = r.out("Indices")->alloc<int64_t>(od, -1);
  std::vector<int64_t> ord((size_t)n);
  for (int64_t i = 0; i < rows; ++i) {
    std::iota(ord.begin(), ord.end(), 0);
    const float* row = p + i * n;
    std::partial_sort(ord.begin(), ord.begin() + k, ord.end(),
                      [row](int64_t a, int64_t b) { return row[a] > row[b] || (row[a] == row[b] && a < b); });
    for (int64_t j = 0; j < k; ++j) {
      v[i * k + j] = row[ord[(size_t)j]];
      ix[i * k + j] = ord[(size_t)j];
    }
  }
}

void k_arg_max(const OpRun& r) {
  Tensor& x = r.in("X");
  int64_t axis = r.op.GetInt("axis", -1);
  if (axis < 0) axis += (int64_t)x.dims.size();
  const int64_t pre = prod(x.dims, 0, (size_t)axis), n = x.dims[(size_t)axis], post = prod(x.dims, (size_t)axis + 1);
  Dims od;
  for (size_t i = 0; i < x.dims.size(); ++i)
    if ((int64_t)i != axis) od.push_back(x.dims[i]);
  if (od.empty()) od.push_back(1);
  const float* p = f32(x);
  Tensor xs = x;
  int64_t* o = r.out("Out")->alloc<int64_t>(od, -1);
  for (int64_t a = 0; a < pre; ++a)
    for (int64_t c = 0; c < post; ++c) {
      int64_t best = 0;
      for (int64_t j = 1; j < n; ++j)
        if (p[(a * n + j) * post + c] > p[(a * n + best) * post + c]) best = j;
      o[a * post + c] = best;
    }
}

// ------------------------------------------------------------ shape ops
Dims infer_shape(const Dims& in, const std::vector<int64_t>& shape) {
  Dims out(shape.size());
  int64_t known = 1, neg = -1;
  for (size_t i = 0; i < shape.size(); ++i) {
    if (shape[i] == -1) {
      PA_CHECK(neg < 0, "reshape: more than one -1");
      neg = (int64_t)i;
      out[i] = 1;
    } else if (shape[i] == 0) {
      PA_CHECK(i < in.size(), "reshape: 0 refers past the input rank");
      out[i] = in[i];
    } else {
      out[i] = shape[i];
    }
    if (shape[i] != -1) known *= out[i];
  }
  const int64_t n = prod(in);
  if (neg >= 0) {
    PA_CHECK(known > 0 && n % known == 0, "reshape: cannot infer -1");
    out[(size_t)neg] = n / known;
  }
  PA_CHECK(prod(out) == n, "reshape: element count changes");
  return out;
}

void k_reshape(const OpRun& r) {
  Tensor x = r.in("X");
  std::vector<int64_t> shape = r.op.GetInts("shape");
  if (Tensor* st = r.in_opt("Shape")) {
    Tensor h = st->device >= 0 ? st->to(-1, r.ctx.stream) : *st;
    shape.clear();
    for (int64_t i = 0; i < h.numel(); ++i) shape.push_back(h.data<int32_t>()[i]);
  }
  Tensor* o = r.out("Out");
  Dims nd = infer_shape(x.dims, shape);
  *o = x;  // shares the buffer
  o->dims = nd;
  // the LoD travels only while the rows it indexes do (ShareLoD of an unchanged batch)
  if (nd.empty() || x.dims.empty() || nd[0] != x.dims[0]) o->lod.clear();
  if (Tensor* xs = r.out("XShape")) {
    Dims d{0};
    d.insert(d.end(), x.dims.begin(), x.dims.end());
    xs->dtype = x.dtype;
    xs->dims = d;
  }
}

void k_reshape_grad(const OpRun& r) {  // reshape_grad / reshape2_grad
  Tensor g = r.in("Out@GRAD");
  Dims d;
  if (Tensor* xs = r.in_opt("XShape")) d.assign(xs->dims.begin() + 1, xs->dims.end());
  else d = r.in("X").dims;
  Tensor* dx = r.out("X@GRAD");
  *dx = g;
  dx->dims = d;
}

void k_flatten(const OpRun& r) {
  Tensor x = r.in("X");
  const size_t axis = (size_t)r.op.GetInt("axis", 1);
  Tensor* o = r.out("Out");
  *o = x;
  o->dims = {prod(x.dims, 0, axis), prod(x.dims, axis)};
  if (Tensor* xs = r.out("XShape")) {
    Dims d{0};
    d.insert(d.end(), x.dims.begin(), x.dims.end());
    xs->dims = d;
  }
}

void k_squeeze(const OpRun& r) {
  Tensor x = r.in("X");
  auto axes = r.op.GetInts("axes");
  Dims d;
  const int64_t R = (int64_t)x.dims.size();
  for (int64_t i = 0; i < R; ++i) {
    bool drop = false;
    if (axes.empty()) drop = x.dims[(size_t)i] == 1;
    for (auto a : axes) drop |= ((a < 0 ? a + R : a) == i) && x.dims[(size_t)i] == 1;
    if (!drop) d.push_back(x.dims[(size_t)i]);
  }
  Tensor* o = r.out("Out");
  *o = x;
  o->dims = d;
}

void k_unsqueeze(const OpRun& r) {
  Tensor x = r.in("X");
  Dims d = x.dims;
  for (auto a : r.op.GetInts("axes")) {
    int64_t cur = (int64_t)d.size();
    int64_t p = a < 0 ? a + cur + 1 : a;
    d.insert(d.begin() + p, 1);
  }
  Tensor* o = r.out("Out");
  *o = x;
  o->dims = d;
}

void permute(const Tensor& x, const std::vector<int64_t>& perm, Tensor* o) {
  const size_t R = x.dims.size();
  Dims od(R), sx(R);
  int64_t s = 1;
  for (size_t i = R; i-- > 0;) {
    sx[i] = s;
    s *= x.dims[i];
  }
  for (size_t i = 0; i < R; ++i) od[i] = x.dims[(size_t)perm[i]];
  const size_t es = dt_size(x.dtype);
  Tensor xs = x;
  char* op = (char*)o->alloc(x.dtype, od, -1);
  const char* ip = (const char*)xs.raw();
  const int64_t n = prod(od);
  std::vector<int64_t> idx(R, 0);
  for (int64_t i = 0; i < n; ++i) {
    int64_t off = 0;
    for (size_t d = 0; d < R; ++d) off += idx[d] * sx[(size_t)perm[d]];
    memcpy(op + i * es, ip + off * es, es);
    for (size_t d = R; d-- > 0;) {
      if (++idx[d] < od[d]) break;
      idx[d] = 0;
    }
  }
}

void k_transpose(const OpRun& r) {
  Tensor x = r.in("X");
  permute(x, r.op.GetInts("axis"), r.out("Out"));
  if (Tensor* xs = r.out("XShape")) {
    Dims d{0};
    d.insert(d.end(), x.dims.begin(), x.dims.end());
    xs->dims = d;
  }
}

void k_concat(const OpRun& r) {
  auto xs = r.ins("X");
  std::vector<Tensor> keep;
  for (auto* t : xs) keep.push_back(*t);
  int64_t axis = r.op.GetInt("axis", 0);
  const int64_t R = (int64_t)keep[0].dims.size();
  if (axis < 0) axis += R;
  Dims od = keep[0].dims;
  od[(size_t)axis] = 0;
  for (auto& t : keep) od[(size_t)axis] += t.dims[(size_t)axis];
  const int64_t pre = prod(od, 0, (size_t)axis), post = prod(od, (size_t)axis + 1);
  const size_t es = dt_size(keep[0].dtype);
  char* o = (char*)r.out("Out")->alloc(keep[0].dtype, od, -1);
  int64_t off = 0;
  for (auto& t : keep) {
    const int64_t w = t.dims[(size_t)axis] * post;
    for (int64_t p = 0; p < pre; ++p)
      memcpy(o + (p * od[(size_t)axis] * post + off) * es, (const char*)t.raw() + p * w * es, w * es);
    off += w;
  }
}

void k_split(const OpRun& r) {
  Tensor x = r.in("X");
  int64_t axis = r.op.GetInt("axis", 0);
  const int64_t R = (int64_t)x.dims.size();
  if (axis < 0) axis += R;
  auto& outs = r.op.Outputs("Out");
  std::vector<int64_t> sec = r.op.GetInts("sections");
  const int64_t num = r.op.GetInt("num", 0);
  if (sec.empty()) sec.assign(outs.size(), x.dims[(size_t)axis] / (num ? num : (int64_t)outs.size()));
  const int64_t pre = prod(x.dims, 0, (size_t)axis), post = prod(x.dims, (size_t)axis + 1);
  const size_t es = dt_size(x.dtype);
  int64_t off = 0;
  for (size_t i = 0; i < outs.size(); ++i) {
    Dims od = x.dims;
    od[(size_t)axis] = sec[i];
    char* o = (char*)r.out("Out", i)->alloc(x.dtype, od, -1);
    const int64_t w = sec[i] * post;
    for (int64_t p = 0; p < pre; ++p)
      memcpy(o + p * w * es, (const char*)x.raw() + (p * x.dims[(size_t)axis] * post + off) * es, w * es);
    off += w;
  }
}

// ------------------------------------------------------------ lookup_table (lookup_table_op.h)
void k_lookup_table(const OpRun& r) {
  Tensor& w = r.in("W");
  Tensor& ids = r.in("Ids");
  const int64_t V = w.dims[0], D = w.dims[1];
  const int64_t pad = r.op.GetInt("padding_idx", -1);
  auto id = ids_of(ids);
  Dims od = ids.dims;
  if (od.size() > 1 && od.back() == 1) od.back() = D;
  else od.push_back(D);
  LoD lod = ids.lod;
  Tensor* o = r.out("Out");
  float* op = o->alloc<float>(od, -1);
  const float* wp = f32(w);
  for (size_t i = 0; i < id.size(); ++i) {
    if (id[i] == pad) {
      memset(op + i * D, 0, sizeof(float) * D);
      continue;
    }
    PA_CHECK(id[i] >= 0 && id[i] < V, "lookup_table: id %lld out of range [0, %lld)", (long long)id[i],
             (long long)V);
    memcpy(op + i * D, wp + id[i] * D, sizeof(float) * D);
  }
  o->lod = lod;
}

void k_lookup_table_grad(const OpRun& r) {  // dense W@GRAD, or SelectedRows when is_sparse
  if (r.op.GetBool("is_sparse")) return lookup_table_grad_sparse(r);
  Tensor& w = r.in("W");
  Tensor& ids = r.in("Ids");
  Tensor& g = r.in("Out@GRAD");
  const int64_t D = w.dims[1];
  const int64_t pad = r.op.GetInt("padding_idx", -1);
  auto id = ids_of(ids);
  Dims d = w.dims;
  float* dw = r.out("W@GRAD")->alloc<float>(d, -1);
  memset(dw, 0, sizeof(float) * prod(d));
  const float* gp = f32(g);
  for (size_t i = 0; i < id.size(); ++i)
    if (id[i] != pad)
      for (int64_t j = 0; j < D; ++j) dw[id[i] * D + j] += gp[i * D + j];
}

// ------------------------------------------------------------ conv / pool / batch norm (NCHW)
// conv_op.h: im2col + GEMM per (image, group)
void im2col(const float* x, int64_t C, int64_t H, int64_t W, int64_t kh, int64_t kw, int64_t sh, int64_t sw,
            int64_t ph, int64_t pw, int64_t dh, int64_t dw, int64_t OH, int64_t OW, float* col) {
  for (int64_t c = 0; c < C; ++c)
    for (int64_t i = 0; i < kh; ++i)
      for (int64_t j = 0; j < kw; ++j) {
        float* row = col + ((c * kh + i) * kw + j) * OH * OW;
        for (int64_t oh = 0; oh < OH; ++oh) {
          const int64_t ih = oh * sh - ph + i * dh;
          for (int64_t ow = 0; ow < OW; ++ow) {
            const int64_t iw = ow * sw - pw + j * dw;
            row[oh * OW + ow] = (ih >= 0 && ih < H && iw >= 0 && iw < W) ? x[(c * H + ih) * W + iw] : 0.f;
          }
        }
      }
}

void k_conv2d(const OpRun& r) {
  Tensor x = r.in("Input");
  Tensor& w = r.in("Filter");
  auto st = r.op.GetInts("strides"), pd = r.op.GetInts("paddings"), dl = r.op.GetInts("dilations");
  if (st.empty()) st = {1, 1};
  if (pd.empty()) pd = {0, 0};
  if (dl.empty()) dl = {1, 1};
  const int64_t g = std::max<int64_t>(1, r.op.GetInt("groups", 1));
  const int64_t N = x.dims[0], C = x.dims[1], H = x.dims[2], W = x.dims[3];
  const int64_t OC = w.dims[0], kh = w.dims[2], kw = w.dims[3];
  PA_CHECK(w.dims[1] * g == C, "conv2d: filter %s vs input %s with groups %lld", w.shape_str().c_str(),
           x.shape_str().c_str(), (long long)g);
  const int64_t OH = (H + 2 * pd[0] - (dl[0] * (kh - 1) + 1)) / st[0] + 1;
  const int64_t OW = (W + 2 * pd[1] - (dl[1] * (kw - 1) + 1)) / st[1] + 1;
  float* o = r.out("Output")->alloc<float>({N, OC, OH, OW}, -1);
  const int64_t Cg = C / g, OCg = OC / g, Kc = Cg * kh * kw, P = OH * OW;
  const float* xp = f32(x);
  const float* wp = f32(w);
  std::vector<float> col((size_t)(Kc * P));
  for (int64_t n = 0; n < N; ++n)
    for (int64_t gi = 0; gi < g; ++gi) {
      im2col(xp + (n * C + gi * Cg) * H * W, Cg, H, W, kh, kw, st[0], st[1], pd[0], pd[1], dl[0], dl[1], OH, OW,
             col.data());
      sgemm(false, false, OCg, P, Kc, 1.f, wp + gi * OCg * Kc, Kc, col.data(), P, 0.f,
            o + (n * OC + gi * OCg) * P, P);
    }
}

// pool_op.h / math/pooling.cc
void k_pool2d(const OpRun& r) {
  Tensor x = r.in("X");
  const bool is_max = r.op.GetString("pooling_type", "max") == "max";
  auto ks = r.op.GetInts("ksize"), st = r.op.GetInts("strides"), pd = r.op.GetInts("paddings");
  if (st.empty()) st = {1, 1};
  if (pd.empty()) pd = {0, 0};
  const int64_t N = x.dims[0], C = x.dims[1], H = x.dims[2], W = x.dims[3];
  if (r.op.GetBool("global_pooling")) {
    ks = {H, W};
    pd = {0, 0};
  }
  const bool ceil = r.op.GetBool("ceil_mode"), excl = r.op.GetBool("exclusive", true);
  auto osz = [&](int64_t in, int64_t k, int64_t p, int64_t s) {
    return ceil ? (in - k + 2 * p + s - 1) / s + 1 : (in - k + 2 * p) / s + 1;
  };
  const int64_t OH = osz(H, ks[0], pd[0], st[0]), OW = osz(W, ks[1], pd[1], st[1]);
  float* o = r.out("Out")->alloc<float>({N, C, OH, OW}, -1);
  const float* xp = f32(x);
  parallel_for(N * C, 4, [&](int64_t a, int64_t b) {
    for (int64_t nc = a; nc < b; ++nc) {
      const float* xi = xp + nc * H * W;
      for (int64_t oh = 0; oh < OH; ++oh)
        for (int64_t ow = 0; ow < OW; ++ow) {
          const int64_t h0 = oh * st[0] - pd[0], w0 = ow * st[1] - pd[1];
          const int64_t h1 = std::min(h0 + ks[0], H), w1 = std::min(w0 + ks[1], W);
          const int64_t hs = std::max<int64_t>(h0, 0), ws = std::max<int64_t>(w0, 0);
          float acc = is_max ? -INFINITY : 0.f;
          for (int64_t h = hs; h < h1; ++h)
            for (int64_t w = ws; w < w1; ++w) acc = is_max ? std::max(acc, xi[h * W + w]) : acc + xi[h * W + w];
          if (!is_max) {
            const int64_t cnt = excl ? (h1 - hs) * (w1 - ws) : ks[0] * ks[1];
            acc /= (float)std::max<int64_t>(1, cnt);
          }
          o[(nc * OH + oh) * OW + ow] = acc;
        }
    }
  });
}

// batch_norm_op.cc: inference normalisation with the running statistics; in
// training (is_test false and not forced) batch statistics are used and the
// running ones updated with `momentum`.
void k_batch_norm(const OpRun& r) {
  Tensor x = r.in("X");
  Tensor& sc = r.in("Scale");
  Tensor& bi = r.in("Bias");
  Tensor& mean = r.in("Mean");
  Tensor& var = r.in("Variance");
  const float eps = r.op.GetFloat("epsilon", 1e-5f), mom = r.op.GetFloat("momentum", 0.9f);
  const bool test = r.ctx.is_test || r.op.GetBool("is_test") || r.op.GetBool("use_global_stats");
  const bool nhwc = r.op.GetString("data_layout", "NCHW") == "NHWC";
  const int64_t N = x.dims[0], C = nhwc ? x.dims.back() : x.dims[1];
  const int64_t HW = x.numel() / (N * C);
  const float* xp = f32(x);
  auto at = [&](int64_t n, int64_t c, int64_t i) { return nhwc ? (n * HW + i) * C + c : (n * C + c) * HW + i; };
  std::vector<float> m(C), v(C);
  if (test) {
    memcpy(m.data(), f32(mean), sizeof(float) * C);
    memcpy(v.data(), f32(var), sizeof(float) * C);
  } else {
    for (int64_t c = 0; c < C; ++c) {
      double s = 0, s2 = 0;
      for (int64_t n = 0; n < N; ++n)
        for (int64_t i = 0; i < HW; ++i) {
          const double t = xp[at(n, c, i)];
          s += t;
          s2 += t * t;
        }
      const double cnt = (double)N * HW;
      m[c] = (float)(s / cnt);
      v[c] = (float)std::max(0.0, s2 / cnt - (s / cnt) * (s / cnt));
    }
    float* rm = f32(mean);
    float* rv = f32(var);
    for (int64_t c = 0; c < C; ++c) {
      rm[c] = rm[c] * mom + m[c] * (1 - mom);
      rv[c] = rv[c] * mom + v[c] * (1 - mom);
    }
    if (Tensor* sm = r.out("SavedMean")) memcpy(sm->alloc<float>({C}, -1), m.data(), sizeof(float) * C);
    if (Tensor* sv = r.out("SavedVariance")) {
      float* p = sv->alloc<float>({C}, -1);
      for (int64_t c = 0; c < C; ++c) p[c] = 1.f / sqrtf(v[c] + eps);
    }
  }
  Dims d = x.dims;
  float* y = r.out("Y")->alloc<float>(d, -1);
  const float* s = f32(sc);
  const float* b = f32(bi);
  for (int64_t c = 0; c < C; ++c) {
    const float a = s[c] / sqrtf(v[c] + eps), sh = b[c] - m[c] * a;
    for (int64_t n = 0; n < N; ++n)
      for (int64_t i = 0; i < HW; ++i) y[at(n, c, i)] = xp[at(n, c, i)] * a + sh;
  }
}

// dropout_op.h: downgrade_in_infer scales by (1-p) at inference, upscale_in_train not
void k_dropout(const OpRun& r) {
  Tensor x = r.in("X");
  const float p = r.op.GetFloat("dropout_prob", 0.5f);
  const bool upscale = r.op.GetString("dropout_implementation", "downgrade_in_infer") == "upscale_in_train";
  const bool test = r.ctx.is_test || r.op.GetBool("is_test");
  Dims d = x.dims;
  LoD lod = x.lod;
  Tensor* o = r.out("Out");
  float* op = o->alloc<float>(d, -1);
  const float* xp = f32(x);
  const int64_t n = x.numel();
  if (test) {
    const float s = upscale ? 1.f : 1.f - p;
    for (int64_t i = 0; i < n; ++i) op[i] = xp[i] * s;
  } else {
    Tensor* mt = r.out("Mask");
    float* mk = mt ? mt->alloc<float>(d, -1) : nullptr;
    std::uniform_real_distribution<float> u(0.f, 1.f);
    for (int64_t i = 0; i < n; ++i) {
      // Mask holds 0 / 1 (dropout_op.h); the upscale factor applies to Out and, in
      // dropout_grad, to the gradient
      const bool keep = u(r.ctx.rng) >= p;
      if (mk) mk[i] = keep ? 1.f : 0.f;
      op[i] = keep ? xp[i] * (upscale && p < 1.f ? 1.f / (1.f - p) : 1.f) : 0.f;
    }
  }
  o->lod = lod;
}

// ------------------------------------------------------------ conv / pool / batch-norm gradients
// conv_op.h GemmConvGradKernel: per (image, group) dcol = W^T dY scattered back by
// col2im, dW += dY col(X)^T; dBias = per-channel sums of dY
void col2im_add(const float* col, int64_t C, int64_t H, int64_t W, int64_t kh, int64_t kw, int64_t sh, int64_t sw,
                int64_t ph, int64_t pw, int64_t dh, int64_t dw, int64_t OH, int64_t OW, float* x) {
  for (int64_t c = 0; c < C; ++c)
    for (int64_t i = 0; i < kh; ++i)
      for (int64_t j = 0; j < kw; ++j) {
        const float* row = col + ((c * kh + i) * kw + j) * OH * OW;
        for (int64_t oh = 0; oh < OH; ++oh) {
          const int64_t ih = oh * sh - ph + i * dh;
          if (ih < 0 || ih >= H) continue;
          for (int64_t ow = 0; ow < OW; ++ow) {
            const int64_t iw = ow * sw - pw + j * dw;
            if (iw >= 0 && iw < W) x[(c * H + ih) * W + iw] += row[oh * OW + ow];
          }
        }
      }
}

void k_conv2d_grad(const OpRun& r) {
  Tensor x = r.in("Input");
  Tensor& w = r.in("Filter");
  Tensor dy = r.in("Output@GRAD");
  auto st = r.op.GetInts("strides"), pd = r.op.GetInts("paddings"), dl = r.op.GetInts("dilations");
  if (st.empty()) st = {1, 1};
  if (pd.empty()) pd = {0, 0};
  if (dl.empty()) dl = {1, 1};
  const int64_t g = std::max<int64_t>(1, r.op.GetInt("groups", 1));
  const int64_t N = x.dims[0], C = x.dims[1], H = x.dims[2], W = x.dims[3];
  const int64_t OC = w.dims[0], kh = w.dims[2], kw = w.dims[3];
  const int64_t OH = dy.dims[2], OW = dy.dims[3];
  const int64_t Cg = C / g, OCg = OC / g, Kc = Cg * kh * kw, P = OH * OW;
  PA_CHECK(dy.numel() == N * OC * P, "conv2d_grad: Output@GRAD %s does not match", dy.shape_str().c_str());
  const float* xp = f32(x);
  const float* wp = f32(w);
  const float* gp = f32(dy);
  Tensor* dxt = r.out("Input@GRAD");
  Tensor* dwt = r.out("Filter@GRAD");
  Tensor* dbt = r.out("Bias@GRAD");
  float* dx = dxt ? dxt->alloc<float>(x.dims, -1) : nullptr;
  float* dw = dwt ? dwt->alloc<float>(w.dims, -1) : nullptr;
  if (dx) memset(dx, 0, sizeof(float) * x.numel());
  if (dw) memset(dw, 0, sizeof(float) * w.numel());
  std::vector<float> col((size_t)(Kc * P));
  for (int64_t n = 0; n < N; ++n)
    for (int64_t gi = 0; gi < g; ++gi) {
      const float* dyg = gp + (n * OC + gi * OCg) * P;
      if (dw) {
        im2col(xp + (n * C + gi * Cg) * H * W, Cg, H, W, kh, kw, st[0], st[1], pd[0], pd[1], dl[0], dl[1], OH, OW,
               col.data());
        sgemm(false, true, OCg, Kc, P, 1.f, dyg, P, col.data(), P, 1.f, dw + gi * OCg * Kc, Kc);
      }
      if (dx) {
        sgemm(true, false, Kc, P, OCg, 1.f, wp + gi * OCg * Kc, Kc, dyg, P, 0.f, col.data(), P);
        col2im_add(col.data(), Cg, H, W, kh, kw, st[0], st[1], pd[0], pd[1], dl[0], dl[1], OH, OW,
                   dx + (n * C + gi * Cg) * H * W);
      }
    }
  if (dbt) {
    float* db = dbt->alloc<float>({OC}, -1);
    for (int64_t c = 0; c < OC; ++c) {
      double s = 0;
      for (int64_t n = 0; n < N; ++n)
        for (int64_t i = 0; i < P; ++i) s += gp[(n * OC + c) * P + i];
      db[c] = (float)s;
    }
  }
}

// pool_op.h PoolGradKernel / math/pooling.cc: max routes dOut to the window's first
// maximum, avg spreads it over the counted window
void k_pool2d_grad(const OpRun& r) {
  Tensor x = r.in("X");
  Tensor dy = r.in("Out@GRAD");
  const bool is_max = r.op.GetString("pooling_type", "max") == "max";
  auto ks = r.op.GetInts("ksize"), st = r.op.GetInts("strides"), pd = r.op.GetInts("paddings");
  if (st.empty()) st = {1, 1};
  if (pd.empty()) pd = {0, 0};
  const int64_t N = x.dims[0], C = x.dims[1], H = x.dims[2], W = x.dims[3];
  if (r.op.GetBool("global_pooling")) {
    ks = {H, W};
    pd = {0, 0};
  }
  const bool excl = r.op.GetBool("exclusive", true);
  const int64_t OH = dy.dims[2], OW = dy.dims[3];
  Tensor* dxt = r.out("X@GRAD");
  if (!dxt) return;
  float* dx = dxt->alloc<float>(x.dims, -1);
  memset(dx, 0, sizeof(float) * x.numel());
  const float* xp = f32(x);
  const float* gp = f32(dy);
  parallel_for(N * C, 4, [&](int64_t a, int64_t b) {
    for (int64_t nc = a; nc < b; ++nc) {
      const float* xi = xp + nc * H * W;
      float* di = dx + nc * H * W;
      for (int64_t oh = 0; oh < OH; ++oh)
        for (int64_t ow = 0; ow < OW; ++ow) {
          const int64_t h0 = oh * st[0] - pd[0], w0 = ow * st[1] - pd[1];
          const int64_t h1 = std::min(h0 + ks[0], H), w1 = std::min(w0 + ks[1], W);
          const int64_t hs = std::max<int64_t>(h0, 0), ws = std::max<int64_t>(w0, 0);
          const float g = gp[(nc * OH + oh) * OW + ow];
          if (is_max) {
            int64_t best = -1;
            float bv = -INFINITY;
            for (int64_t h = hs; h < h1; ++h)
              for (int64_t w = ws; w < w1; ++w)
                if (best < 0 || xi[h * W + w] > bv) {
                  bv = xi[h * W + w];
                  best = h * W + w;
                }
            if (best >= 0) di[best] += g;
          } else {
            const int64_t cnt = excl ? (h1 - hs) * (w1 - ws) : ks[0] * ks[1];
            const float v = g / (float)std::max<int64_t>(1, cnt);
            for (int64_t h = hs; h < h1; ++h)
              for (int64_t w = ws; w < w1; ++w) di[h * W + w] += v;
          }
        }
    }
  });
}

// batch_norm_op.cc BatchNormGradKernel (NCHW / NHWC) from SavedMean and
// SavedVariance (= 1 / sqrt(var + eps)):
//   dx = scale * rstd * (dy - mean(dy) - xhat * mean(dy * xhat))
void k_batch_norm_grad(const OpRun& r) {
  Tensor x = r.in("X");
  Tensor dy = r.in("Y@GRAD");
  Tensor& sc = r.in("Scale");
  const float* mean = f32(r.in("SavedMean"));
  const float* rstd = f32(r.in("SavedVariance"));
  const bool nhwc = r.op.GetString("data_layout", "NCHW") == "NHWC";
  const bool relu = r.op.GetBool("fuse_with_relu");
  const int64_t N = x.dims[0], C = nhwc ? x.dims.back() : x.dims[1], HW = x.numel() / (N * C);
  auto at = [&](int64_t n, int64_t c, int64_t i) { return nhwc ? (n * HW + i) * C + c : (n * C + c) * HW + i; };
  const float* xp = f32(x);
  const float* gp = f32(dy);
  const float* yp = relu ? f32(r.in("Y")) : nullptr;
  std::vector<float> ds((size_t)C), db((size_t)C);
  const double M = (double)N * HW;
  Tensor* dxt = r.out("X@GRAD");
  float* dx = dxt ? dxt->alloc<float>(x.dims, -1) : nullptr;
  const float* s = f32(sc);
  for (int64_t c = 0; c < C; ++c) {
    double sg = 0, sgx = 0;
    for (int64_t n = 0; n < N; ++n)
      for (int64_t i = 0; i < HW; ++i) {
        const int64_t k = at(n, c, i);
        const double g = (yp && yp[k] <= 0.f) ? 0.0 : gp[k];
        sg += g;
        sgx += g * (xp[k] - mean[c]) * rstd[c];
      }
    db[(size_t)c] = (float)sg;
    ds[(size_t)c] = (float)sgx;
    if (!dx) continue;
    for (int64_t n = 0; n < N; ++n)
      for (int64_t i = 0; i < HW; ++i) {
        const int64_t k = at(n, c, i);
        const double g = (yp && yp[k] <= 0.f) ? 0.0 : gp[k];
        const double xh = (xp[k] - mean[c]) * rstd[c];
        dx[k] = (float)(s[c] * rstd[c] * (g - sg / M - xh * sgx / M));
      }
  }
  if (Tensor* t = r.out("Scale@GRAD")) memcpy(t->alloc<float>(sc.dims, -1), ds.data(), sizeof(float) * C);
  if (Tensor* t = r.out("Bias@GRAD")) memcpy(t->alloc<float>(r.in("Bias").dims, -1), db.data(), sizeof(float) * C);
}

void k_fill_zeros_like(const OpRun& r) {
  // read X's shape and dtype before r.out(): creating the output variable may
  // rehash the scope and invalidate the reference r.in() returned
  const Tensor& x = r.in("X");
  const Dims d = x.dims;
  const DT dt = x.dtype;
  Tensor* o = r.out("Out");
  void* dst = o->alloc(dt, d, -1);  // (not inside memset's argument list: o->nbytes() must see the new dims)
  memset(dst, 0, o->nbytes());
}

// ------------------------------------------------------------ optimizers (sgd_op.h, momentum_op.h, adam_op.h)
// the update target of `in_slot` -> `out_slot`: in place, or a copy of the input
float* opt_target(const OpRun& r, const char* in_slot, const char* out_slot) {
  Tensor& in = r.in(in_slot);
  if (r.op.Output(out_slot) == r.op.Input(in_slot)) return f32(in);
  const Dims d = in.dims;
  const float* src = f32(in);
  const size_t bytes = in.nbytes();
  Tensor keep = in;  // holds the source buffer while the output is allocated
  float* dst = r.out(out_slot)->alloc<float>(d, -1);
  memcpy(dst, src, bytes);
  return dst;
}

void k_sgd(const OpRun& r) {
  if (selected_rows_sgd(r)) return;
  Tensor& p = r.in("Param");
  Tensor& g = r.in("Grad");
  const float lr = f32(r.in("LearningRate"))[0];
  Tensor* po = r.out("ParamOut");
  if (po->raw() != p.raw()) {
    Dims d = p.dims;
    Tensor src = p;
    float* dst = po->alloc<float>(d, -1);
    memcpy(dst, src.raw(), src.nbytes());
  }
  float* w = f32(*po);
  const float* gp = f32(g);
  for (int64_t i = 0; i < p.numel(); ++i) w[i] -= lr * gp[i];
}

void k_momentum(const OpRun& r) {
  Tensor& p = r.in("Param");
  Tensor& g = r.in("Grad");
  Tensor& v = r.in("Velocity");
  const float lr = f32(r.in("LearningRate"))[0], mu = r.op.GetFloat("mu");
  const bool nesterov = r.op.GetBool("use_nesterov");
  float* w = f32(*r.out("ParamOut"));
  float* vel = f32(*r.out("VelocityOut"));
  if (!(w == f32(p) && vel == f32(v))) throw Decline{};  // out-of-place update: not covered here
  const float* gp = f32(g);
  for (int64_t i = 0; i < p.numel(); ++i) {
    vel[i] = vel[i] * mu + gp[i];
    w[i] -= nesterov ? (gp[i] + mu * vel[i]) * lr : lr * vel[i];
  }
}

void k_adam(const OpRun& r) {
  if (selected_rows_adam(r)) return;
  Tensor& p = r.in("Param");
  Tensor& g = r.in("Grad");
  const float lr = f32(r.in("LearningRate"))[0];
  const float b1p = f32(r.in("Beta1Pow"))[0], b2p = f32(r.in("Beta2Pow"))[0];
  const float b1 = r.op.GetFloat("beta1", 0.9f), b2 = r.op.GetFloat("beta2", 0.999f),
              eps = r.op.GetFloat("epsilon", 1e-8f);
  const float* gp = f32(g);
  Tensor gkeep = g;
  (void)p;
  float* w = opt_target(r, "Param", "ParamOut");  // out-of-place outputs (op tests) start as copies
  float* m1 = opt_target(r, "Moment1", "Moment1Out");
  float* m2 = opt_target(r, "Moment2", "Moment2Out");
  const float lr_t = lr * sqrtf(1 - b2p) / (1 - b1p);
  for (int64_t i = 0; i < gkeep.numel(); ++i) {
    m1[i] = b1 * m1[i] + (1 - b1) * gp[i];
    m2[i] = b2 * m2[i] + (1 - b2) * gp[i] * gp[i];
    w[i] -= lr_t * m1[i] / (sqrtf(m2[i]) + eps);
  }
}

// ------------------------------------------------------------ misc
void k_increment(const OpRun& r) {
  Tensor& x = r.in("X");
  const float step = r.op.GetFloat("step", 1.f);
  Tensor* o = r.out("Out");
  if (x.dtype == DT::INT64) {
    const int64_t v = x.data<int64_t>()[0];
    o->alloc<int64_t>({1}, -1)[0] = v + (int64_t)step;
  } else {
    const float v = f32(x)[0];
    o->alloc<float>({1}, -1)[0] = v + step;
  }
}

// compare_op.cc / logical_op.cc: elementwise comparisons and logic into BOOL.  Y
// broadcasts as a trailing block of X (the common scalar-bound loop counter case);
// values are compared as double (exact for the int32 / int64 counters and fp32).
double load_d(const Tensor& t, int64_t i) {
  switch (t.dtype) {
    case DT::FP32: return t.data<float>()[i];
    case DT::FP64: return t.data<double>()[i];
    case DT::INT64: return (double)t.data<int64_t>()[i];
    case DT::INT32: return t.data<int32_t>()[i];
    case DT::BOOL: case DT::UINT8: return t.data<uint8_t>()[i];
    default: fail("compare/logical: input dtype %s", dt_name(t.dtype));
  }
}

template <class F>
void k_binary_bool(const OpRun& r, F f) {
  Tensor& x = r.in("X");
  Tensor* yp = r.in_opt("Y");
  const int64_t n = x.numel();
  const int64_t ny = yp ? yp->numel() : 1;
  PA_CHECK(!yp || (ny > 0 && n % ny == 0), "%s: Y (%s) does not broadcast into X (%s)", r.op.type.c_str(),
           yp ? yp->shape_str().c_str() : "", x.shape_str().c_str());
  Tensor xs = x;  // keep the input alive when Out aliases it
  Tensor ys = yp ? *yp : Tensor();
  Tensor* o = r.out("Out");
  LoD lod = x.lod;
  Dims d = x.dims;
  uint8_t* p = static_cast<uint8_t*>(o->alloc(DT::BOOL, d, -1));
  o->lod = lod;
  for (int64_t i = 0; i < n; ++i) p[i] = f(load_d(xs, i), yp ? load_d(ys, i % ny) : 0.0) ? 1 : 0;
}

void k_less_than(const OpRun& r) { k_binary_bool(r, [](double a, double b) { return a < b; }); }
void k_less_equal(const OpRun& r) { k_binary_bool(r, [](double a, double b) { return a <= b; }); }
void k_greater_than(const OpRun& r) { k_binary_bool(r, [](double a, double b) { return a > b; }); }
void k_greater_equal(const OpRun& r) { k_binary_bool(r, [](double a, double b) { return a >= b; }); }
void k_equal(const OpRun& r) { k_binary_bool(r, [](double a, double b) { return a == b; }); }
void k_not_equal(const OpRun& r) { k_binary_bool(r, [](double a, double b) { return a != b; }); }
void k_logical_and(const OpRun& r) { k_binary_bool(r, [](double a, double b) { return a != 0 && b != 0; }); }
void k_logical_or(const OpRun& r) { k_binary_bool(r, [](double a, double b) { return a != 0 || b != 0; }); }
void k_logical_xor(const OpRun& r) { k_binary_bool(r, [](double a, double b) { return (a != 0) != (b != 0); }); }
void k_logical_not(const OpRun& r) { k_binary_bool(r, [](double a, double) { return a == 0; }); }

void k_delete_var(const OpRun& r) {
  for (auto& n : r.op.Inputs("X"))
    if (Variable* v = r.scope.Find(n)) v->tensor = Tensor();
}

}  // namespace

// ---------------------------------------------------------------- registration

std::vector<int64_t> sequence_expand_rows(const Tensor& x, const Tensor& y, int ref_level, LoD* out_lod) {
  PA_CHECK(!y.lod.empty(), "sequence_expand: Y has no LoD");
  const int ref = ref_level < 0 ? (int)y.lod.size() - 1 : ref_level;
  PA_CHECK(ref < (int)y.lod.size(), "sequence_expand: ref_level %d out of range", ref);
  const auto& yoff = y.lod[(size_t)ref];
  const int64_t rows_x = x.dims.empty() ? 0 : x.dims[0];
  std::vector<int64_t> rows;
  out_lod->clear();
  if (yoff.size() <= 1) {  // nothing to expand against: Out = X
    rows.resize((size_t)rows_x);
    std::iota(rows.begin(), rows.end(), int64_t{0});
    *out_lod = x.lod;
    return rows;
  }
  std::vector<size_t> xoff;
  if (x.lod.size() == 1) {
    xoff = x.lod[0];
  } else {  // every row is one sequence; the output carries no LoD
    xoff.resize((size_t)rows_x + 1);
    std::iota(xoff.begin(), xoff.end(), size_t{0});
  }
  PA_CHECK(xoff.size() == yoff.size(), "sequence_expand: X has %zu sequences, Y's level %d has %zu",
           xoff.size() - 1, ref, yoff.size() - 1);
  std::vector<size_t> oo{0};
  for (size_t i = 0; i + 1 < yoff.size(); ++i)
    for (size_t k = yoff[i]; k < yoff[i + 1]; ++k) {
      for (size_t t = xoff[i]; t < xoff[i + 1]; ++t) rows.push_back((int64_t)t);
      oo.push_back(rows.size());
    }
  if (x.lod.size() == 1) out_lod->push_back(std::move(oo));
  return rows;
}

std::vector<int64_t> sequence_expand_as_rows(const Tensor& x, const Tensor& y, LoD* out_lod) {
  PA_CHECK(!y.lod.empty(), "sequence_expand_as: Y has no LoD");
  const auto& yoff = y.lod[0];
  PA_CHECK(!x.dims.empty() && (int64_t)yoff.size() == x.dims[0] + 1,
           "sequence_expand_as: X has %lld rows, Y has %zu sequences", (long long)(x.dims.empty() ? 0 : x.dims[0]),
           yoff.size() - 1);
  std::vector<int64_t> rows;
  rows.reserve(yoff.back());
  for (size_t i = 0; i + 1 < yoff.size(); ++i)
    for (size_t k = yoff[i]; k < yoff[i + 1]; ++k) rows.push_back((int64_t)i);
  *out_lod = LoD{yoff};
  return rows;
}

std::vector<std::vector<int64_t>> sequence_concat_rows(const std::vector<Tensor*>& xs, LoD* out_lod) {
  PA_CHECK(!xs.empty(), "sequence_concat: no inputs");
  std::vector<const std::vector<size_t>*> offs;
  for (const Tensor* x : xs) {
    PA_CHECK(!x->lod.empty() && !x->dims.empty(), "sequence_concat: an input has no LoD");
    offs.push_back(&x->lod.back());
    PA_CHECK(offs.back()->size() == offs[0]->size(), "sequence_concat: inputs hold different sequence counts");
    PA_CHECK((int64_t)offs.back()->back() == x->dims[0], "sequence_concat: LoD does not cover the rows");
    PA_CHECK(x->lod.size() == xs[0]->lod.size(), "sequence_concat: inputs differ in LoD levels");
  }
  std::vector<std::vector<int64_t>> dst(xs.size());
  for (size_t k = 0; k < xs.size(); ++k) dst[k].resize((size_t)xs[k]->dims[0]);
  std::vector<size_t> oo{0};
  int64_t row = 0;
  for (size_t i = 0; i + 1 < offs[0]->size(); ++i) {
    for (size_t k = 0; k < xs.size(); ++k)
      for (size_t t = (*offs[k])[i]; t < (*offs[k])[i + 1]; ++t) dst[k][t] = row++;
    oo.push_back((size_t)row);
  }
  // reference ConcatLoD at level 0: the upper levels are X[0]'s, the finest level
  // holds the summed sequence lengths (sequence_concat_op.h ConcatLoD)
  *out_lod = xs[0]->lod;
  out_lod->back() = oo;
  return dst;
}

namespace {
// the row map of sequence_expand (AS=false) / sequence_expand_as (AS=true)
template <bool AS>
std::vector<int64_t> expand_rows(const OpRun& r, LoD* ol) {
  return AS ? sequence_expand_as_rows(r.in("X"), r.in("Y"), ol)
            : sequence_expand_rows(r.in("X"), r.in("Y"), r.op.GetInt("ref_level", -1), ol);
}
}  // namespace

namespace {
// ---------------------------------------------------------------- sequence (LoD) ops
// sequence_pool_op.h / math/sequence_pooling.cc over the last LoD level; an empty
// sequence pools to 0.  Out drops the last level; MaxIndex (int32) for MAX.
// the finest LoD level; a tensor without LoD is ONE sequence of all its rows (the
// Python op library's _last_level)
std::vector<size_t> last_level(const Tensor& x, const char* op) {
  (void)op;
  if (x.lod.empty()) return {0, (size_t)(x.dims.empty() ? 0 : x.dims[0])};
  return x.lod.back();
}

void k_sequence_pool(const OpRun& r) {
  Tensor& x = r.in("X");
  const auto off = last_level(x, "sequence_pool");
  const std::string pt = r.op.GetString("pooltype", "AVERAGE");
  const int64_t n = (int64_t)off.size() - 1, D = x.dims[0] ? x.numel() / x.dims[0] : 0;
  Dims od = x.dims;
  od[0] = n;
  Tensor* o = r.out("Out");
  float* y = o->alloc<float>(od, -1);
  int32_t* mi = nullptr;
  if (Tensor* m = r.out("MaxIndex")) {  // always produced (a gradient program reads its shape)
    int32_t* p = m->alloc<int32_t>(od, -1);
    std::fill_n(p, n * D, 0);
    if (pt == "MAX") mi = p;
  }
  const float* xp = f32(x);
  parallel_for(n, 4, [&](int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i) {
      const int64_t s = (int64_t)off[(size_t)i], e = (int64_t)off[(size_t)i + 1], len = e - s;
      for (int64_t d = 0; d < D; ++d) {
        float v = 0.f;
        if (len > 0) {
          if (pt == "SUM" || pt == "AVERAGE" || pt == "SQRT") {
            double acc = 0;
            for (int64_t t = s; t < e; ++t) acc += xp[t * D + d];
            v = (float)(pt == "SUM" ? acc : pt == "AVERAGE" ? acc / (double)len : acc / std::sqrt((double)len));
          } else if (pt == "MAX") {
            int64_t best = s;
            for (int64_t t = s + 1; t < e; ++t)
              if (xp[t * D + d] > xp[best * D + d]) best = t;
            v = xp[best * D + d];
            if (mi) mi[i * D + d] = (int32_t)best;
          } else if (pt == "LAST") {
            v = xp[(e - 1) * D + d];
          } else if (pt == "FIRST") {
            v = xp[s * D + d];
          } else {
            fail("sequence_pool: unknown pooltype %s", pt.c_str());
          }
        } else if (mi) {
          mi[i * D + d] = -1;
        }
        y[i * D + d] = v;
      }
    }
  });
  if (!x.lod.empty()) o->lod.assign(x.lod.begin(), x.lod.end() - 1);
}

// the MAX gradient goes to the first maximum, recomputed from X (the forward's
// MaxIndex may come from another kernel)
void k_sequence_pool_grad(const OpRun& r) {
  Tensor& x = r.in("X");
  Tensor& g = r.in("Out@GRAD");
  const auto off = last_level(x, "sequence_pool_grad");
  const std::string pt = r.op.GetString("pooltype", "AVERAGE");
  const int64_t n = (int64_t)off.size() - 1, D = x.dims[0] ? x.numel() / x.dims[0] : 0;
  Tensor* dxt = r.out("X@GRAD");
  Dims d0 = x.dims;
  float* dx = dxt->alloc<float>(d0, -1);
  std::fill_n(dx, x.numel(), 0.f);
  const float* xp = f32(x);
  const float* gp = f32(g);
  parallel_for(n, 4, [&](int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i) {
      const int64_t s = (int64_t)off[(size_t)i], e = (int64_t)off[(size_t)i + 1], len = e - s;
      if (len <= 0) continue;
      for (int64_t d = 0; d < D; ++d) {
        const float gv = gp[i * D + d];
        if (pt == "SUM" || pt == "AVERAGE" || pt == "SQRT") {
          const float v = pt == "SUM" ? gv : pt == "AVERAGE" ? gv / (float)len : gv / std::sqrt((float)len);
          for (int64_t t = s; t < e; ++t) dx[t * D + d] = v;
        } else if (pt == "MAX") {
          int64_t best = s;
          for (int64_t t = s + 1; t < e; ++t)
            if (xp[t * D + d] > xp[best * D + d]) best = t;
          dx[best * D + d] = gv;
        } else if (pt == "LAST") {
          dx[(e - 1) * D + d] = gv;
        } else {
          dx[s * D + d] = gv;
        }
      }
    }
  });
  dxt->lod = x.lod;
}

void k_sequence_softmax(const OpRun& r) {
  Tensor& x = r.in("X");
  const auto& off = last_level(x, "sequence_softmax");
  Tensor* o = r.out("Out");
  Dims d = x.dims;
  float* y = o->alloc<float>(d, -1);
  const float* xp = f32(x);
  for (size_t i = 0; i + 1 < off.size(); ++i) {
    const int64_t s = (int64_t)off[i], e = (int64_t)off[i + 1];
    if (e > s) softmax_rows(xp + s, y + s, 1, e - s);
  }
  o->lod = x.lod;
}

void k_sequence_softmax_grad(const OpRun& r) {
  Tensor& y = r.in("Out");
  Tensor& g = r.in("Out@GRAD");
  Tensor* xl = r.in_opt("X");
  const LoD& lod = !y.lod.empty() ? y.lod : (xl ? xl->lod : y.lod);
  PA_CHECK(!lod.empty(), "sequence_softmax_grad: no LoD");
  const auto& off = lod.back();
  Tensor* dxt = r.out("X@GRAD");
  Dims d = y.dims;
  float* dx = dxt->alloc<float>(d, -1);
  const float* yp = f32(y);
  const float* gp = f32(g);
  for (size_t i = 0; i + 1 < off.size(); ++i) {
    const int64_t s = (int64_t)off[i], e = (int64_t)off[i + 1];
    double dot = 0;
    for (int64_t t = s; t < e; ++t) dot += (double)yp[t] * gp[t];
    for (int64_t t = s; t < e; ++t) dx[t] = yp[t] * (gp[t] - (float)dot);
  }
  dxt->lod = lod;
}

template <bool AS>
void k_sequence_expand(const OpRun& r) {
  Tensor& x = r.in("X");
  LoD ol;
  const auto rows = expand_rows<AS>(r, &ol);
  const int64_t D = x.dims[0] ? x.numel() / x.dims[0] : 0;
  Dims od = x.dims;
  od[0] = (int64_t)rows.size();
  Tensor* o = r.out("Out");
  float* y = o->alloc<float>(od, -1);
  const float* xp = f32(x);
  parallel_for((int64_t)rows.size(), 16, [&](int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i) std::copy_n(xp + rows[(size_t)i] * D, D, y + i * D);
  });
  o->lod = ol;
}

// X@GRAD[row] = sum of Out@GRAD over the output rows copied from it
template <bool AS>
void k_sequence_expand_grad(const OpRun& r) {
  Tensor& x = r.in("X");
  Tensor& g = r.in("Out@GRAD");
  LoD ol;
  const auto rows = expand_rows<AS>(r, &ol);
  const int64_t D = x.dims[0] ? x.numel() / x.dims[0] : 0;
  PA_CHECK(g.numel() == (int64_t)rows.size() * D, "sequence_expand_grad: Out@GRAD has %lld elements, expected %lld",
           (long long)g.numel(), (long long)rows.size() * D);
  Tensor* dxt = r.out("X@GRAD");
  float* dx = dxt->alloc<float>(x.dims, -1);
  std::fill_n(dx, x.numel(), 0.f);
  const float* gp = f32(g);
  for (size_t i = 0; i < rows.size(); ++i)
    for (int64_t d = 0; d < D; ++d) dx[rows[i] * D + d] += gp[(int64_t)i * D + d];
  dxt->lod = x.lod;
  if (Tensor* dy = r.out("Y@GRAD")) {  // Y only shapes the expansion
    Tensor& yt = r.in("Y");
    std::fill_n(dy->alloc<float>(yt.dims, -1), yt.numel(), 0.f);
    dy->lod = yt.lod;
  }
}

int64_t row_width(const Tensor& t) { return t.dims.empty() || t.dims[0] == 0 ? 0 : t.numel() / t.dims[0]; }

// sequence_reshape (sequence_reshape_op.h): the same buffer viewed as [-1, new_dim];
// offsets scale by width / new_dim.  No data moves, so one kernel serves host and
// device tensors.
void k_sequence_reshape(const OpRun& r) {
  Tensor x = r.in("X");
  const auto& off = last_level(x, "sequence_reshape");
  const int64_t D = row_width(x), nd = r.op.GetInt("new_dim", 1);
  PA_CHECK(nd > 0 && x.dims.size() == 2, "sequence_reshape: X must be 2-D and new_dim positive");
  LoD ol{{}};
  for (size_t o : off) {
    PA_CHECK(((int64_t)o * D) % nd == 0, "sequence_reshape: a sequence of width %lld does not split into rows of %lld",
             (long long)D, (long long)nd);
    ol[0].push_back((size_t)((int64_t)o * D / nd));
  }
  Tensor* o = r.out("Out");
  o->share(x);
  o->dims = {x.numel() / nd, nd};
  o->lod = ol;
}

void k_sequence_reshape_grad(const OpRun& r) {
  Tensor x = r.in("X");
  Tensor g = r.in("Out@GRAD");
  PA_CHECK(g.numel() == x.numel(), "sequence_reshape_grad: Out@GRAD does not match X");
  Tensor* dx = r.out("X@GRAD");
  dx->share(g);
  dx->dims = x.dims;
  dx->lod = x.lod;
}

// axis 0 at LoD level 0 only (the finest level); other forms run the Python kernel
void seq_concat_attrs_ok(const OpRun& r) {
  if (r.op.GetInt("axis", 0) != 0 || r.op.GetInt("level", 0) != 0) throw Decline{};
}

void k_sequence_concat(const OpRun& r) {
  seq_concat_attrs_ok(r);
  auto xs = r.ins("X");
  LoD ol;
  const auto dst = sequence_concat_rows(xs, &ol);
  const int64_t D = row_width(*xs[0]);
  Dims od = xs[0]->dims;
  od[0] = (int64_t)ol.back().back();
  for (Tensor* x : xs) PA_CHECK(row_width(*x) == D, "sequence_concat: inputs differ in row width");
  Tensor* o = r.out("Out");
  float* y = o->alloc<float>(od, -1);
  for (size_t k = 0; k < xs.size(); ++k) {
    const float* xp = f32(*xs[k]);
    for (size_t t = 0; t < dst[k].size(); ++t) std::copy_n(xp + (int64_t)t * D, D, y + dst[k][t] * D);
  }
  o->lod = ol;
}

void k_sequence_concat_grad(const OpRun& r) {
  seq_concat_attrs_ok(r);
  auto xs = r.ins("X");
  Tensor& g = r.in("Out@GRAD");
  LoD ol;
  const auto dst = sequence_concat_rows(xs, &ol);
  const float* gp = f32(g);
  for (size_t k = 0; k < xs.size(); ++k) {
    Tensor* dxt = r.out("X@GRAD", k);
    if (!dxt) continue;
    const int64_t D = row_width(*xs[k]);
    float* dx = dxt->alloc<float>(xs[k]->dims, -1);
    for (size_t t = 0; t < dst[k].size(); ++t) std::copy_n(gp + dst[k][t] * D, D, dx + (int64_t)t * D);
    dxt->lod = xs[k]->lod;
  }
}
}  // namespace

PA_HOST_KERNEL(feed, k_feed);
PA_HOST_KERNEL(fetch, k_fetch);
PA_HOST_KERNEL(fill_constant, k_fill_constant);
PA_HOST_KERNEL(uniform_random, k_uniform_random);
PA_HOST_KERNEL(gaussian_random, k_gaussian_random);
PA_HOST_KERNEL(uniform_random_batch_size_like, k_uniform_random);
PA_HOST_KERNEL(gaussian_random_batch_size_like, k_gaussian_random);
PA_HOST_KERNEL(assign, k_assign);
PA_HOST_KERNEL(shape, k_shape);
PA_HOST_KERNEL(cast, k_cast);
PA_HOST_KERNEL(mul, k_mul);
PA_HOST_KERNEL(mul_grad, k_mul_grad);
PA_HOST_KERNEL(matmul, k_matmul);
PA_HOST_KERNEL(fc, k_fc);
PA_HOST_KERNEL(elementwise_add, ew_kernel([](auto a, auto b) { return a + b; }));
PA_HOST_KERNEL(elementwise_sub, ew_kernel([](auto a, auto b) { return a - b; }));
PA_HOST_KERNEL(elementwise_mul, ew_kernel([](auto a, auto b) { return a * b; }));
PA_HOST_KERNEL(elementwise_div, ew_kernel([](auto a, auto b) { return a / b; }));
PA_HOST_KERNEL(elementwise_max, ew_kernel([](auto a, auto b) { return a > b ? a : b; }));
PA_HOST_KERNEL(elementwise_min, ew_kernel([](auto a, auto b) { return a < b ? a : b; }));
PA_HOST_KERNEL(elementwise_pow, ew_kernel([](auto a, auto b) { return (decltype(a))powf((float)a, (float)b); }));
PA_HOST_KERNEL(elementwise_add_grad, k_ew_grad<0>);
PA_HOST_KERNEL(elementwise_sub_grad, k_ew_grad<1>);
PA_HOST_KERNEL(elementwise_mul_grad, k_ew_grad<2>);
PA_HOST_KERNEL(elementwise_div_grad, k_ew_grad<3>);
PA_HOST_KERNEL(relu, unary([](float v, const OpDesc&) { return v > 0 ? v : 0.f; }));
PA_HOST_KERNEL(sigmoid, unary([](float v, const OpDesc&) { return sigm(v); }));
PA_HOST_KERNEL(logsigmoid, unary([](float v, const OpDesc&) { return -log1pf(expf(-v)); }));
PA_HOST_KERNEL(tanh, unary([](float v, const OpDesc&) { return tanhf(v); }));
PA_HOST_KERNEL(exp, unary([](float v, const OpDesc&) { return expf(v); }));
PA_HOST_KERNEL(log, unary([](float v, const OpDesc&) { return logf(v); }));
PA_HOST_KERNEL(sqrt, unary([](float v, const OpDesc&) { return sqrtf(v); }));
PA_HOST_KERNEL(abs, unary([](float v, const OpDesc&) { return fabsf(v); }));
PA_HOST_KERNEL(square, unary([](float v, const OpDesc&) { return v * v; }));
PA_HOST_KERNEL(reciprocal, unary([](float v, const OpDesc&) { return 1.f / v; }));
PA_HOST_KERNEL(ceil, unary([](float v, const OpDesc&) { return ceilf(v); }));
PA_HOST_KERNEL(floor, unary([](float v, const OpDesc&) { return floorf(v); }));
PA_HOST_KERNEL(round, unary([](float v, const OpDesc&) { return nearbyintf(v); }));  // half to even
PA_HOST_KERNEL(softplus, unary([](float v, const OpDesc&) { return v > 20.f ? v : log1pf(expf(v)); }));
PA_HOST_KERNEL(softsign, unary([](float v, const OpDesc&) { return v / (1.f + fabsf(v)); }));
PA_HOST_KERNEL(gelu, unary([](float v, const OpDesc&) { return 0.5f * v * (1.f + erff(v * 0.70710678f)); }));
PA_HOST_KERNEL(leaky_relu, unary([](float v, const OpDesc& o) { return v > 0 ? v : v * o.GetFloat("alpha", 0.02f); }));
PA_HOST_KERNEL(relu6, unary([](float v, const OpDesc& o) {
                 return std::min(std::max(v, 0.f), o.GetFloat("threshold", 6.f));
               }));
PA_HOST_KERNEL(brelu, unary([](float v, const OpDesc& o) {
                 return std::min(std::max(v, o.GetFloat("t_min", 0.f)), o.GetFloat("t_max", 24.f));
               }));
PA_HOST_KERNEL(elu, unary([](float v, const OpDesc& o) { return v > 0 ? v : o.GetFloat("alpha", 1.f) * (expf(v) - 1.f); }));
PA_HOST_KERNEL(hard_sigmoid, unary([](float v, const OpDesc& o) {
                 return std::min(1.f, std::max(0.f, v * o.GetFloat("slope", 0.2f) + o.GetFloat("offset", 0.5f)));
               }));
PA_HOST_KERNEL(swish, unary([](float v, const OpDesc& o) { return v * sigm(o.GetFloat("beta", 1.f) * v); }));
PA_HOST_KERNEL(pow, unary([](float v, const OpDesc& o) { return powf(v, o.GetFloat("factor", 1.f)); }));
PA_HOST_KERNEL(scale, k_scale);
PA_HOST_KERNEL(scale_grad, k_scale_grad);
// the rest of the activation table of fluid_ops.hip (act_f / act_df), on the host
PA_HOST_KERNEL(cos, unary([](float v, const OpDesc&) { return cosf(v); }));
PA_HOST_KERNEL(sin, unary([](float v, const OpDesc&) { return sinf(v); }));
PA_HOST_KERNEL(rsqrt, unary([](float v, const OpDesc&) { return 1.f / sqrtf(v); }));
PA_HOST_KERNEL(silu, unary([](float v, const OpDesc&) { return v * sigm(v); }));
PA_HOST_KERNEL(tanh_shrink, unary([](float v, const OpDesc&) { return v - tanhf(v); }));
PA_HOST_KERNEL(hard_shrink, unary([](float v, const OpDesc& o) {
                 const float t = o.GetFloat("threshold", 0.5f);
                 return (v > t || v < -t) ? v : 0.f;
               }));
PA_HOST_KERNEL(softshrink, unary([](float v, const OpDesc& o) {
                 const float l = o.GetFloat("lambda", 0.5f);
                 return v > l ? v - l : (v < -l ? v + l : 0.f);
               }));
PA_HOST_KERNEL(soft_relu, unary([](float v, const OpDesc& o) {
                 const float t = o.GetFloat("threshold", 40.f);
                 return log1pf(expf(std::min(std::max(v, -t), t)));
               }));
PA_HOST_KERNEL(stanh, unary([](float v, const OpDesc& o) {
                 return o.GetFloat("scale_b", 1.7159f) * tanhf(o.GetFloat("scale_a", 2.f / 3.f) * v);
               }));
PA_HOST_KERNEL(thresholded_relu, unary([](float v, const OpDesc& o) { return v > o.GetFloat("threshold", 1.f) ? v : 0.f; }));
PA_HOST_KERNEL(abs_grad, unary_grad([](float x, float, float g, const OpDesc&) {
                 return g * (x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f));
               }));
PA_HOST_KERNEL(ceil_grad, unary_grad([](float, float, float, const OpDesc&) { return 0.f; }));
PA_HOST_KERNEL(floor_grad, unary_grad([](float, float, float, const OpDesc&) { return 0.f; }));
PA_HOST_KERNEL(round_grad, unary_grad([](float, float, float, const OpDesc&) { return 0.f; }));
PA_HOST_KERNEL(cos_grad, unary_grad([](float x, float, float g, const OpDesc&) { return -g * sinf(x); }));
PA_HOST_KERNEL(sin_grad, unary_grad([](float x, float, float g, const OpDesc&) { return g * cosf(x); }));
PA_HOST_KERNEL(sqrt_grad, unary_grad([](float, float y, float g, const OpDesc&) { return g * 0.5f / y; }));
PA_HOST_KERNEL(rsqrt_grad, unary_grad([](float, float y, float g, const OpDesc&) { return -0.5f * g * y * y * y; }));
PA_HOST_KERNEL(reciprocal_grad, unary_grad([](float, float y, float g, const OpDesc&) { return -g * y * y; }));
PA_HOST_KERNEL(log_grad, unary_grad([](float x, float, float g, const OpDesc&) { return g / x; }));
PA_HOST_KERNEL(logsigmoid_grad, unary_grad([](float x, float, float g, const OpDesc&) { return g * sigm(-x); }));
PA_HOST_KERNEL(softplus_grad, unary_grad([](float x, float, float g, const OpDesc&) { return g * sigm(x); }));
PA_HOST_KERNEL(softsign_grad, unary_grad([](float x, float, float g, const OpDesc&) {
                 const float d = 1.f + fabsf(x);
                 return g / (d * d);
               }));
PA_HOST_KERNEL(silu_grad, unary_grad([](float x, float, float g, const OpDesc&) {
                 const float s = sigm(x);
                 return g * s * (1.f + x * (1.f - s));
               }));
PA_HOST_KERNEL(gelu_grad, unary_grad([](float x, float, float g, const OpDesc&) {
                 return g * (0.5f * (1.f + erff(x * 0.70710678118654752f)) +
                             x * 0.3989422804014327f * expf(-0.5f * x * x));
               }));
PA_HOST_KERNEL(tanh_shrink_grad, unary_grad([](float x, float, float g, const OpDesc&) {
                 const float t = tanhf(x);
                 return g * t * t;
               }));
PA_HOST_KERNEL(hard_shrink_grad, unary_grad([](float x, float, float g, const OpDesc& o) {
                 const float t = o.GetFloat("threshold", 0.5f);
                 return (x > t || x < -t) ? g : 0.f;
               }));
PA_HOST_KERNEL(softshrink_grad, unary_grad([](float x, float, float g, const OpDesc& o) {
                 const float l = o.GetFloat("lambda", 0.5f);
                 return (x > l || x < -l) ? g : 0.f;
               }));
PA_HOST_KERNEL(brelu_grad, unary_grad([](float x, float, float g, const OpDesc& o) {
                 return (x > o.GetFloat("t_min", 0.f) && x < o.GetFloat("t_max", 24.f)) ? g : 0.f;
               }));
PA_HOST_KERNEL(leaky_relu_grad, unary_grad([](float x, float, float g, const OpDesc& o) {
                 return x > 0.f ? g : g * o.GetFloat("alpha", 0.02f);
               }));
PA_HOST_KERNEL(soft_relu_grad, unary_grad([](float x, float y, float g, const OpDesc& o) {
                 const float t = o.GetFloat("threshold", 40.f);
                 return (x > -t && x < t) ? g * (1.f - expf(-y)) : 0.f;
               }));
PA_HOST_KERNEL(elu_grad, unary_grad([](float x, float y, float g, const OpDesc& o) {
                 return x > 0.f ? g : g * (y + o.GetFloat("alpha", 1.f));
               }));
PA_HOST_KERNEL(relu6_grad, unary_grad([](float x, float, float g, const OpDesc& o) {
                 return (x > 0.f && x < o.GetFloat("threshold", 6.f)) ? g : 0.f;
               }));
PA_HOST_KERNEL(pow_grad, unary_grad([](float x, float, float g, const OpDesc& o) {
                 const float f = o.GetFloat("factor", 1.f);
                 return g * f * powf(x, f - 1.f);
               }));
PA_HOST_KERNEL(stanh_grad, unary_grad([](float x, float, float g, const OpDesc& o) {
                 const float a = o.GetFloat("scale_a", 2.f / 3.f), b = o.GetFloat("scale_b", 1.7159f);
                 const float t = tanhf(a * x);
                 return g * a * b * (1.f - t * t);
               }));
PA_HOST_KERNEL(thresholded_relu_grad, unary_grad([](float x, float, float g, const OpDesc& o) {
                 return x > o.GetFloat("threshold", 1.f) ? g : 0.f;
               }));
PA_HOST_KERNEL(hard_sigmoid_grad, unary_grad([](float x, float, float g, const OpDesc& o) {
                 const float t = o.GetFloat("slope", 0.2f) * x + o.GetFloat("offset", 0.5f);
                 return (t > 0.f && t < 1.f) ? g * o.GetFloat("slope", 0.2f) : 0.f;
               }));
PA_HOST_KERNEL(swish_grad, unary_grad([](float x, float, float g, const OpDesc& o) {
                 const float b = o.GetFloat("beta", 1.f), s = sigm(b * x);
                 return g * (s + b * x * s * (1.f - s));
               }));
PA_HOST_KERNEL(relu_grad, unary_grad([](float, float y, float g, const OpDesc&) { return y > 0 ? g : 0.f; }));
PA_HOST_KERNEL(sigmoid_grad, unary_grad([](float, float y, float g, const OpDesc&) { return g * y * (1.f - y); }));
PA_HOST_KERNEL(tanh_grad, unary_grad([](float, float y, float g, const OpDesc&) { return g * (1.f - y * y); }));
PA_HOST_KERNEL(square_grad, unary_grad([](float x, float, float g, const OpDesc&) { return 2.f * x * g; }));
PA_HOST_KERNEL(exp_grad, unary_grad([](float, float y, float g, const OpDesc&) { return g * y; }));
PA_HOST_KERNEL(sum, k_sum);
PA_HOST_KERNEL(mean, k_mean);
PA_HOST_KERNEL(mean_grad, k_mean_grad);
PA_HOST_KERNEL(reduce_sum, k_reduce<0>);
PA_HOST_KERNEL(reduce_mean, k_reduce<1>);
PA_HOST_KERNEL(reduce_max, k_reduce<2>);
PA_HOST_KERNEL(reduce_min, k_reduce<3>);
PA_HOST_KERNEL(reduce_prod, k_reduce<4>);
PA_HOST_KERNEL(softmax, k_softmax);
PA_HOST_KERNEL(softmax_grad, k_softmax_grad);
PA_HOST_KERNEL(cross_entropy, k_cross_entropy);
PA_HOST_KERNEL(cross_entropy_grad, k_cross_entropy_grad);
PA_HOST_KERNEL(softmax_with_cross_entropy, k_softmax_ce);
PA_HOST_KERNEL(softmax_with_cross_entropy_grad, k_softmax_ce_grad);
PA_HOST_KERNEL(accuracy, k_accuracy);
PA_HOST_KERNEL(top_k, k_top_k);
PA_HOST_KERNEL(arg_max, k_arg_max);
PA_HOST_KERNEL(reshape, k_reshape);
PA_HOST_KERNEL(reshape2, k_reshape);
PA_HOST_KERNEL(reshape_grad, k_reshape_grad);
PA_HOST_KERNEL(reshape2_grad, k_reshape_grad);
PA_HOST_KERNEL(flatten, k_flatten);
PA_HOST_KERNEL(flatten2, k_flatten);
PA_HOST_KERNEL(squeeze, k_squeeze);
PA_HOST_KERNEL(squeeze2, k_squeeze);
PA_HOST_KERNEL(unsqueeze, k_unsqueeze);
PA_HOST_KERNEL(unsqueeze2, k_unsqueeze);
PA_HOST_KERNEL(transpose, k_transpose);
PA_HOST_KERNEL(transpose2, k_transpose);
PA_HOST_KERNEL(concat, k_concat);
PA_HOST_KERNEL(split, k_split);
PA_HOST_KERNEL(lookup_table, k_lookup_table);
PA_HOST_KERNEL(lookup_table_grad, k_lookup_table_grad);
PA_HOST_KERNEL(conv2d, k_conv2d);
PA_HOST_KERNEL(depthwise_conv2d, k_conv2d);
PA_HOST_KERNEL(pool2d, k_pool2d);
PA_HOST_KERNEL(batch_norm, k_batch_norm);
PA_HOST_KERNEL(conv2d_grad, k_conv2d_grad);
PA_HOST_KERNEL(depthwise_conv2d_grad, k_conv2d_grad);
PA_HOST_KERNEL(pool2d_grad, k_pool2d_grad);
PA_HOST_KERNEL(batch_norm_grad, k_batch_norm_grad);
PA_HOST_KERNEL(fill_zeros_like, k_fill_zeros_like);
PA_HOST_KERNEL(dropout, k_dropout);
PA_HOST_KERNEL(sgd, k_sgd);
PA_HOST_KERNEL(momentum, k_momentum);
PA_HOST_KERNEL(adam, k_adam);
PA_HOST_KERNEL(increment, k_increment);
PA_HOST_KERNEL(less_than, k_less_than);
PA_HOST_KERNEL(less_equal, k_less_equal);
PA_HOST_KERNEL(greater_than, k_greater_than);
PA_HOST_KERNEL(greater_equal, k_greater_equal);
PA_HOST_KERNEL(equal, k_equal);
PA_HOST_KERNEL(not_equal, k_not_equal);
PA_HOST_KERNEL(logical_and, k_logical_and);
PA_HOST_KERNEL(logical_or, k_logical_or);
PA_HOST_KERNEL(logical_xor, k_logical_xor);
PA_HOST_KERNEL(logical_not, k_logical_not);
PA_HOST_KERNEL(delete_var, k_delete_var);
PA_HOST_KERNEL(sequence_pool, k_sequence_pool);
PA_HOST_KERNEL(sequence_pool_grad, k_sequence_pool_grad);
PA_HOST_KERNEL(sequence_softmax, k_sequence_softmax);
PA_HOST_KERNEL(sequence_softmax_grad, k_sequence_softmax_grad);
PA_HOST_KERNEL(sequence_expand, k_sequence_expand<false>);
PA_HOST_KERNEL(sequence_expand_grad, k_sequence_expand_grad<false>);
PA_HOST_KERNEL(sequence_expand_as, k_sequence_expand<true>);
PA_HOST_KERNEL(sequence_expand_as_grad, k_sequence_expand_grad<true>);
PA_HOST_KERNEL(sequence_concat, k_sequence_concat);
PA_HOST_KERNEL(sequence_concat_grad, k_sequence_concat_grad);
PA_HOST_KERNEL(sequence_reshape, k_sequence_reshape);
PA_HOST_KERNEL(sequence_reshape_grad, k_sequence_reshape_grad);
PA_DEVICE_KERNEL(sequence_reshape, k_sequence_reshape);
PA_DEVICE_KERNEL(sequence_reshape_grad, k_sequence_reshape_grad);

void link_host_kernels() {}

}  // namespace pa
