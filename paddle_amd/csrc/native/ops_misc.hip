// Pointwise losses, clipping and small tensor ops of the native executor, host AND
// device from one source (any_place.h): sign, clip (+grad), clip_by_norm, minus
// (+grad), label_smooth (+grad), sigmoid_cross_entropy_with_logits (+grad), huber_loss
// (+grad), log_loss (+grad), smooth_l1_loss (+grad), squared_l2_norm (+grad),
// squared_l2_distance (+grad), cumsum (+grad), gather (+grad), scatter, one_hot,
// log_softmax (+grad).
//
// Semantics: reference operators/{sign,clip,clip_by_norm,minus,label_smooth,
// sigmoid_cross_entropy_with_logits,huber_loss,log_loss,smooth_l1_loss,
// squared_l2_norm,squared_l2_distance,cumsum,gather,scatter,one_hot}_op.h and
// log_softmax; the Python kernels of operators/{math,nn,tensor}_ops.py compute the
// same functions, and their VJPs are the gradients below (clamp passes the gradient
// where min <= x <= max; a sigmoid CE element whose label equals ignore_index has
// zero loss and gradient).  fp32 only (other dtypes decline to the embedder's kernel).
// Reductions (squared_l2_norm, clip_by_norm's norm) sum per-chunk partials with one
// float atomic per chunk on a device and in order on the host.
#include <hip/hip_runtime.h>
#include <math.h>

#include <vector>

#include "any_place.h"

namespace pa {
namespace {

using any::f32;
using Dims = std::vector<int64_t>;

constexpr int64_t kSerial = int64_t(1) << 60;

__host__ __device__ inline void acc_add(float* p, float v) {
#if defined(__HIP_DEVICE_COMPILE__)
  atomicAdd(p, v);
#else
  *p += v;
#endif
}

__host__ __device__ inline float sigm(float v) { return 1.f / (1.f + expf(-v)); }

int place_of(const OpRun& r) { return r.ctx.device >= 0 ? r.ctx.device : -1; }

// output `slot` shaped like `like` (LoD kept)
float* out_like(const OpRun& r, const char* slot, const Tensor& like, Tensor* keep) {
  float* p = keep->alloc<float>(like.dims, place_of(r));
  keep->lod = like.lod;
  (void)slot;
  return p;
}

void decline_if_requested(const OpRun& r, const char* slot) {
  if (r.op.Outputs(slot).empty()) return;
  if (r.out_var(slot)) throw Decline{};
}

// ---------------------------------------------------------------- sign / clip / minus
struct Sign {
  const float* x;
  float* y;
  __host__ __device__ void operator()(int64_t i) const { y[i] = x[i] > 0.f ? 1.f : (x[i] < 0.f ? -1.f : 0.f); }
};

void k_sign(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("X");
  Tensor o;
  float* y = out_like(r, "Out", x, &o);
  any::run(r, dev, x.numel(), Sign{f32(x, dev), y});
  *r.out("Out") = o;
}

struct Clip {
  const float* x;
  float* y;
  float lo, hi;
  __host__ __device__ void operator()(int64_t i) const { y[i] = fminf(fmaxf(x[i], lo), hi); }
};
struct ClipGrad {
  const float *x, *g;
  float* dx;
  float lo, hi;
  __host__ __device__ void operator()(int64_t i) const { dx[i] = (x[i] >= lo && x[i] <= hi) ? g[i] : 0.f; }
};

void k_clip(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("X");
  Tensor o;
  float* y = out_like(r, "Out", x, &o);
  any::run(r, dev, x.numel(), Clip{f32(x, dev), y, r.op.GetFloat("min", -1e30f), r.op.GetFloat("max", 1e30f)});
  *r.out("Out") = o;
}

void k_clip_grad(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("X");
  Tensor& g = r.in("Out@GRAD");
  Tensor o;
  float* dx = out_like(r, "X@GRAD", x, &o);
  any::run(r, dev, x.numel(),
           ClipGrad{f32(x, dev), f32(g, dev), dx, r.op.GetFloat("min", -1e30f), r.op.GetFloat("max", 1e30f)});
  *r.out("X@GRAD") = o;
}

// sum of squares of chunk c into out[0] (zeroed)
struct SumSq {
  const float* x;
  float* out;
  int64_t n, chunk;
  __host__ __device__ void operator()(int64_t c) const {
    float s = 0.f;
    const int64_t e = (c + 1) * chunk < n ? (c + 1) * chunk : n;
    for (int64_t i = c * chunk; i < e; ++i) s += x[i] * x[i];
    acc_add(out, s);
  }
};

float* sumsq(const OpRun& r, bool dev, const float* x, int64_t n, const char* ws, std::vector<float>* host) {
  float* out = any::scratch(r, dev, ws, 1, host);
  any::zero(r, dev, out, 1);
  const int64_t chunk = 1024;
  any::run(r, dev, (n + chunk - 1) / chunk, SumSq{x, out, n, chunk}, dev ? 4096 : kSerial);
  return out;
}

struct ClipNorm {
  const float *x, *ss;
  float* y;
  float mx;
  __host__ __device__ void operator()(int64_t i) const {
    const float n = sqrtf(ss[0]);
    y[i] = n > mx ? x[i] * (mx / n) : x[i];
  }
};

void k_clip_by_norm(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("X");
  std::vector<float> hs;
  float* ss = sumsq(r, dev, f32(x, dev), x.numel(), "@clipnorm_ss@", &hs);
  Tensor o;
  float* y = out_like(r, "Out", x, &o);
  any::run(r, dev, x.numel(), ClipNorm{f32(x, dev), ss, y, r.op.GetFloat("max_norm", 1.f)});
  *r.out("Out") = o;
}

struct Dot {  // chunk c of sum x * g into out[0]
  const float *x, *g;
  float* out;
  int64_t n, chunk;
  __host__ __device__ void operator()(int64_t c) const {
    float s = 0.f;
    const int64_t e = (c + 1) * chunk < n ? (c + 1) * chunk : n;
    for (int64_t i = c * chunk; i < e; ++i) s += x[i] * g[i];
    acc_add(out, s);
  }
};
struct ClipNormGrad {  // n > mx: dx = (mx / n) g - mx x (x . g) / n^3
  const float *x, *g, *ss, *dot;
  float* dx;
  float mx;
  __host__ __device__ void operator()(int64_t i) const {
    const float n = sqrtf(ss[0]);
    dx[i] = n > mx ? (mx / n) * g[i] - mx * x[i] * dot[0] / (n * n * n) : g[i];
  }
};

void k_clip_by_norm_grad(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("X");
  Tensor& g = r.in("Out@GRAD");
  const int64_t n = x.numel(), chunk = 1024;
  std::vector<float> hs, hd;
  float* ss = sumsq(r, dev, f32(x, dev), n, "@clipnorm_ss@", &hs);
  float* dot = any::scratch(r, dev, "@clipnorm_dot@", 1, &hd);
  any::zero(r, dev, dot, 1);
  any::run(r, dev, (n + chunk - 1) / chunk, Dot{f32(x, dev), f32(g, dev), dot, n, chunk}, dev ? 4096 : kSerial);
  Tensor o;
  any::run(r, dev, n, ClipNormGrad{f32(x, dev), f32(g, dev), ss, dot, out_like(r, "X@GRAD", x, &o),
                                   r.op.GetFloat("max_norm", 1.f)});
  *r.out("X@GRAD") = o;
}

struct Sub {
  const float *x, *y;
  float* o;
  float sy;
  __host__ __device__ void operator()(int64_t i) const { o[i] = x[i] + sy * y[i]; }
};
struct ScaleCopy {
  const float* g;
  float* o;
  float s;
  __host__ __device__ void operator()(int64_t i) const { o[i] = s * g[i]; }
};

void k_minus(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("X");
  Tensor& y = r.in("Y");
  if (x.numel() != y.numel()) throw Decline{};
  Tensor o;
  float* p = out_like(r, "Out", x, &o);
  any::run(r, dev, x.numel(), Sub{f32(x, dev), f32(y, dev), p, -1.f});
  *r.out("Out") = o;
}

void k_minus_grad(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& g = r.in("Out@GRAD");
  if (r.out_var("X@GRAD")) {
    Tensor o;
    any::run(r, dev, g.numel(), ScaleCopy{f32(g, dev), out_like(r, "X@GRAD", r.in("X"), &o), 1.f});
    *r.out("X@GRAD") = o;
  }
  if (r.out_var("Y@GRAD")) {
    Tensor o;
    any::run(r, dev, g.numel(), ScaleCopy{f32(g, dev), out_like(r, "Y@GRAD", r.in("Y"), &o), -1.f});
    *r.out("Y@GRAD") = o;
  }
}

// ---------------------------------------------------------------- label_smooth
struct LabelSmooth {
  const float *x, *prior;
  float* o;
  float e;
  int64_t C;
  __host__ __device__ void operator()(int64_t i) const {
    o[i] = (1.f - e) * x[i] + (prior ? e * prior[i % C] : e / (float)C);
  }
};

void k_label_smooth(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("X");
  Tensor* pr = r.in_opt("PriorDist");
  const int64_t C = x.dims.back();
  if (pr && pr->numel() != C) throw Decline{};
  Tensor o;
  float* p = out_like(r, "Out", x, &o);
  any::run(r, dev, x.numel(), LabelSmooth{f32(x, dev), pr ? f32(*pr, dev) : nullptr, p, r.op.GetFloat("epsilon", 0.f), C});
  *r.out("Out") = o;
}

void k_label_smooth_grad(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  decline_if_requested(r, "PriorDist@GRAD");
  Tensor& g = r.in("Out@GRAD");
  Tensor o;
  any::run(r, dev, g.numel(),
           ScaleCopy{f32(g, dev), out_like(r, "X@GRAD", r.in("X"), &o), 1.f - r.op.GetFloat("epsilon", 0.f)});
  *r.out("X@GRAD") = o;
}

// ---------------------------------------------------------------- pointwise losses
struct SigmoidCE {
  const float *x, *z;
  float* o;
  float ignore;
  __host__ __device__ void operator()(int64_t i) const {
    const float v = x[i], t = z[i];
    o[i] = t == ignore ? 0.f : fmaxf(v, 0.f) - v * t + log1pf(expf(-fabsf(v)));
  }
};
struct SigmoidCEGrad {
  const float *x, *z, *g;
  float *dx, *dz;
  float ignore;
  __host__ __device__ void operator()(int64_t i) const {
    const bool ig = z[i] == ignore;
    if (dx) dx[i] = ig ? 0.f : (sigm(x[i]) - z[i]) * g[i];
    if (dz) dz[i] = ig ? 0.f : -x[i] * g[i];
  }
};

void k_sigmoid_ce(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("X");
  Tensor& z = r.in("Label");
  if (z.numel() != x.numel()) throw Decline{};
  Tensor o;
  any::run(r, dev, x.numel(),
           SigmoidCE{f32(x, dev), f32(z, dev), out_like(r, "Out", x, &o), (float)r.op.GetInt("ignore_index", -100)});
  *r.out("Out") = o;
}

void k_sigmoid_ce_grad(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("X");
  Tensor& z = r.in("Label");
  Tensor& g = r.in("Out@GRAD");
  Tensor dX, dZ;
  float* dx = r.out_var("X@GRAD") ? out_like(r, "X@GRAD", x, &dX) : nullptr;
  float* dz = r.out_var("Label@GRAD") ? out_like(r, "Label@GRAD", z, &dZ) : nullptr;
  any::run(r, dev, x.numel(),
           SigmoidCEGrad{f32(x, dev), f32(z, dev), f32(g, dev), dx, dz, (float)r.op.GetInt("ignore_index", -100)});
  if (dx) *r.out("X@GRAD") = dX;
  if (dz) *r.out("Label@GRAD") = dZ;
}

struct Huber {
  const float *x, *y;
  float *res, *o;
  float d;
  __host__ __device__ void operator()(int64_t i) const {
    const float rr = y[i] - x[i], a = fabsf(rr);
    res[i] = rr;
    o[i] = a <= d ? 0.5f * rr * rr : d * (a - 0.5f * d);
  }
};
struct HuberGrad {
  const float *res, *g;
  float *dx, *dy;
  float d;
  __host__ __device__ void operator()(int64_t i) const {
    const float rr = res[i];
    const float dr = fabsf(rr) <= d ? rr : (rr > 0.f ? d : -d);  // d out / d residual
    if (dx) dx[i] = -dr * g[i];
    if (dy) dy[i] = dr * g[i];
  }
};

void k_huber(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("X");
  Tensor& y = r.in("Y");
  if (x.numel() != y.numel()) throw Decline{};
  Tensor res, o;
  float* rp = out_like(r, "Residual", x, &res);
  any::run(r, dev, x.numel(), Huber{f32(x, dev), f32(y, dev), rp, out_like(r, "Out", x, &o), r.op.GetFloat("delta", 1.f)});
  if (Tensor* t = r.out("Residual")) *t = res;
  *r.out("Out") = o;
}

void k_huber_grad(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("X");
  Tensor& res = r.in("Residual");
  Tensor& g = r.in("Out@GRAD");
  Tensor dX, dY;
  float* dx = r.out_var("X@GRAD") ? out_like(r, "X@GRAD", x, &dX) : nullptr;
  float* dy = r.out_var("Y@GRAD") ? out_like(r, "Y@GRAD", r.in("Y"), &dY) : nullptr;
  any::run(r, dev, x.numel(), HuberGrad{f32(res, dev), f32(g, dev), dx, dy, r.op.GetFloat("delta", 1.f)});
  if (dx) *r.out("X@GRAD") = dX;
  if (dy) *r.out("Y@GRAD") = dY;
}

struct LogLoss {
  const float *p, *y;
  float* o;
  float e;
  __host__ __device__ void operator()(int64_t i) const {
    o[i] = -y[i] * logf(p[i] + e) - (1.f - y[i]) * logf(1.f - p[i] + e);
  }
};
struct LogLossGrad {
  const float *p, *y, *g;
  float *dp, *dy;
  float e;
  __host__ __device__ void operator()(int64_t i) const {
    if (dp) dp[i] = g[i] * (-y[i] / (p[i] + e) + (1.f - y[i]) / (1.f - p[i] + e));
    if (dy) dy[i] = g[i] * (-logf(p[i] + e) + logf(1.f - p[i] + e));
  }
};

void k_log_loss(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& p = r.in("Predicted");
  Tensor& y = r.in("Labels");
  if (p.numel() != y.numel()) throw Decline{};
  Tensor o;
  any::run(r, dev, p.numel(), LogLoss{f32(p, dev), f32(y, dev), out_like(r, "Loss", p, &o), r.op.GetFloat("epsilon", 1e-4f)});
  *r.out("Loss") = o;
}

void k_log_loss_grad(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& p = r.in("Predicted");
  Tensor& y = r.in("Labels");
  Tensor& g = r.in("Loss@GRAD");
  Tensor dP, dY;
  float* dp = r.out_var("Predicted@GRAD") ? out_like(r, "Predicted@GRAD", p, &dP) : nullptr;
  float* dy = r.out_var("Labels@GRAD") ? out_like(r, "Labels@GRAD", y, &dY) : nullptr;
  any::run(r, dev, p.numel(), LogLossGrad{f32(p, dev), f32(y, dev), f32(g, dev), dp, dy, r.op.GetFloat("epsilon", 1e-4f)});
  if (dp) *r.out("Predicted@GRAD") = dP;
  if (dy) *r.out("Labels@GRAD") = dY;
}

// smooth_l1: d = (x - y) * iw; v = |d| < 1/s2 ? s2 d^2 / 2 : |d| - 1/(2 s2); Out[n] = sum_row v * ow
struct SmoothL1Row {
  const float *x, *y, *iw, *ow;
  float *diff, *out;
  int64_t D;
  float s2;
  __host__ __device__ void operator()(int64_t n) const {
    float s = 0.f;
    for (int64_t j = 0; j < D; ++j) {
      const int64_t i = n * D + j;
      float d = x[i] - y[i];
      if (iw) d *= iw[i];
      diff[i] = d;
      const float a = fabsf(d);
      float v = a < 1.f / s2 ? 0.5f * d * d * s2 : a - 0.5f / s2;
      if (ow) v *= ow[i];
      s += v;
    }
    out[n] = s;
  }
};
struct SmoothL1Grad {
  const float *diff, *iw, *ow, *g;
  float *dx, *dy;
  int64_t D;
  float s2;
  __host__ __device__ void operator()(int64_t i) const {
    const float d = diff[i];
    float v = fabsf(d) < 1.f / s2 ? d * s2 : (d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f));
    if (ow) v *= ow[i];
    if (iw) v *= iw[i];
    v *= g[i / D];
    if (dx) dx[i] = v;
    if (dy) dy[i] = -v;
  }
};

void k_smooth_l1(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("X");
  Tensor& y = r.in("Y");
  Tensor* iw = r.in_opt("InsideWeight");
  Tensor* ow = r.in_opt("OutsideWeight");
  const int64_t N = x.dims[0], D = x.numel() / std::max<int64_t>(N, 1);
  if (y.numel() != x.numel() || (iw && iw->numel() != x.numel()) || (ow && ow->numel() != x.numel())) throw Decline{};
  const float s = r.op.GetFloat("sigma", 1.f);
  Tensor diff, o;
  float* dp = out_like(r, "Diff", x, &diff);
  float* op = o.alloc<float>({N, 1}, place_of(r));
  any::run(r, dev, N,
           SmoothL1Row{f32(x, dev), f32(y, dev), iw ? f32(*iw, dev) : nullptr, ow ? f32(*ow, dev) : nullptr, dp, op, D,
                       s * s},
           64);
  if (Tensor* t = r.out("Diff")) *t = diff;
  *r.out("Out") = o;
}

void k_smooth_l1_grad(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  decline_if_requested(r, "InsideWeight@GRAD");
  decline_if_requested(r, "OutsideWeight@GRAD");
  Tensor& x = r.in("X");
  Tensor* iw = r.in_opt("InsideWeight");
  Tensor* ow = r.in_opt("OutsideWeight");
  Tensor& diff = r.in("Diff");
  Tensor& g = r.in("Out@GRAD");
  const int64_t N = x.dims[0], D = x.numel() / std::max<int64_t>(N, 1);
  const float s = r.op.GetFloat("sigma", 1.f);
  Tensor dX, dY;
  float* dx = r.out_var("X@GRAD") ? out_like(r, "X@GRAD", x, &dX) : nullptr;
  float* dy = r.out_var("Y@GRAD") ? out_like(r, "Y@GRAD", r.in("Y"), &dY) : nullptr;
  any::run(r, dev, x.numel(),
           SmoothL1Grad{f32(diff, dev), iw ? f32(*iw, dev) : nullptr, ow ? f32(*ow, dev) : nullptr, f32(g, dev), dx, dy, D,
                        s * s});
  if (dx) *r.out("X@GRAD") = dX;
  if (dy) *r.out("Y@GRAD") = dY;
}

// ---------------------------------------------------------------- squared L2
struct ScaleBy {  // o[i] = s * x[i] * g[0]
  const float *x, *g;
  float* o;
  float s;
  __host__ __device__ void operator()(int64_t i) const { o[i] = s * x[i] * g[0]; }
};

void k_sq_l2_norm(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("X");
  Tensor o;
  float* op = o.alloc<float>({1}, place_of(r));
  any::zero(r, dev, op, 1);
  const int64_t n = x.numel(), chunk = 1024;
  any::run(r, dev, (n + chunk - 1) / chunk, SumSq{f32(x, dev), op, n, chunk}, dev ? 4096 : kSerial);
  *r.out("Out") = o;
}

void k_sq_l2_norm_grad(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("X");
  Tensor& g = r.in("Out@GRAD");
  Tensor o;
  any::run(r, dev, x.numel(), ScaleBy{f32(x, dev), f32(g, dev), out_like(r, "X@GRAD", x, &o), 2.f});
  *r.out("X@GRAD") = o;
}

struct SqDist {  // row n: sub = x - y (y row 0 when broadcast), out = sum sub^2
  const float *x, *y;
  float *sub, *out;
  int64_t D, yrows;
  __host__ __device__ void operator()(int64_t n) const {
    float s = 0.f;
    const float* yr = y + (yrows == 1 ? 0 : n * D);
    for (int64_t j = 0; j < D; ++j) {
      const float d = x[n * D + j] - yr[j];
      sub[n * D + j] = d;
      s += d * d;
    }
    out[n] = s;
  }
};
struct SqDistGradX {
  const float *sub, *g;
  float* dx;
  int64_t D;
  __host__ __device__ void operator()(int64_t i) const { dx[i] = 2.f * sub[i] * g[i / D]; }
};
struct SqDistGradY {  // broadcast y: column sums of -2 sub g
  const float *sub, *g;
  float* dy;
  int64_t N, D;
  __host__ __device__ void operator()(int64_t j) const {
    float s = 0.f;
    for (int64_t n = 0; n < N; ++n) s += -2.f * sub[n * D + j] * g[n];
    dy[j] = s;
  }
};

void k_sq_l2_dist(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("X");
  Tensor& y = r.in("Y");
  const int64_t N = x.dims[0], D = x.numel() / std::max<int64_t>(N, 1);
  const int64_t yrows = y.dims[0];
  if (y.numel() != yrows * D || (yrows != N && yrows != 1)) throw Decline{};
  Tensor sub, o;
  float* sp = out_like(r, "sub_result", x, &sub);
  float* op = o.alloc<float>({N, 1}, place_of(r));
  any::run(r, dev, N, SqDist{f32(x, dev), f32(y, dev), sp, op, D, yrows}, 64);
  if (Tensor* t = r.out("sub_result")) *t = sub;
  *r.out("Out") = o;
}

void k_sq_l2_dist_grad(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("X");
  Tensor& y = r.in("Y");
  Tensor& sub = r.in("sub_result");
  Tensor& g = r.in("Out@GRAD");
  const int64_t N = x.dims[0], D = x.numel() / std::max<int64_t>(N, 1);
  if (r.out_var("X@GRAD")) {
    Tensor o;
    any::run(r, dev, x.numel(), SqDistGradX{f32(sub, dev), f32(g, dev), out_like(r, "X@GRAD", x, &o), D});
    *r.out("X@GRAD") = o;
  }
  if (r.out_var("Y@GRAD")) {
    Tensor o;
    float* dy = out_like(r, "Y@GRAD", y, &o);
    if (y.dims[0] == N && N != 1) {
      any::run(r, dev, x.numel(), SqDistGradX{f32(sub, dev), f32(g, dev), dy, D});
      any::run(r, dev, x.numel(), ScaleCopy{dy, dy, -1.f});
    } else {
      any::run(r, dev, D, SqDistGradY{f32(sub, dev), f32(g, dev), dy, N, D}, 64);
    }
    *r.out("Y@GRAD") = o;
  }
}

// ---------------------------------------------------------------- cumsum
struct Cumsum {  // one (outer, inner) line of length L along the axis
  const float* x;
  float* o;
  int64_t L, inner;
  int excl, rev;
  __host__ __device__ void operator()(int64_t line) const {
    const int64_t a = line / inner, b = line % inner;
    const float* xs = x + a * L * inner + b;
    float* os = o + a * L * inner + b;
    float s = 0.f;
    for (int64_t k = 0; k < L; ++k) {
      const int64_t t = rev ? L - 1 - k : k;
      const float v = xs[t * inner];
      os[t * inner] = excl ? s : s + v;
      s += v;
    }
  }
};

struct Axis {
  int64_t L, inner, outer;
};

Axis axis_of(const Tensor& x, int64_t axis) {
  const int64_t R = (int64_t)x.dims.size();
  if (axis < 0) axis += R;
  PA_CHECK(axis >= 0 && axis < R, "axis out of range");
  Axis a{x.dims[(size_t)axis], 1, 1};
  for (int64_t k = axis + 1; k < R; ++k) a.inner *= x.dims[(size_t)k];
  for (int64_t k = 0; k < axis; ++k) a.outer *= x.dims[(size_t)k];
  return a;
}

void k_cumsum(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("X");
  const Axis a = axis_of(x, r.op.GetInt("axis", -1));
  Tensor o;
  any::run(r, dev, a.outer * a.inner,
           Cumsum{f32(x, dev), out_like(r, "Out", x, &o), a.L, a.inner, r.op.GetBool("exclusive", false) ? 1 : 0,
                  r.op.GetBool("reverse", false) ? 1 : 0},
           64);
  *r.out("Out") = o;
}

// d cumsum: the cumsum of Out@GRAD in the opposite direction (same exclusivity)
void k_cumsum_grad(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& g = r.in("Out@GRAD");
  const Axis a = axis_of(g, r.op.GetInt("axis", -1));
  Tensor o;
  any::run(r, dev, a.outer * a.inner,
           Cumsum{f32(g, dev), out_like(r, "X@GRAD", r.in("X"), &o), a.L, a.inner,
                  r.op.GetBool("exclusive", false) ? 1 : 0, r.op.GetBool("reverse", false) ? 0 : 1},
           64);
  *r.out("X@GRAD") = o;
}

// ---------------------------------------------------------------- gather / scatter / one_hot
template <class I>
struct GatherRows {
  const float* x;
  const I* idx;
  float* o;
  int64_t W, rows;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t k = i / W;
    const int64_t src = (int64_t)idx[k];
    o[i] = (src >= 0 && src < rows) ? x[src * W + i % W] : 0.f;
  }
};
template <class I>
struct ScatterAddRows {
  const float* g;
  const I* idx;
  float* o;
  int64_t W, rows;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t k = i / W, dst = (int64_t)idx[k];
    if (dst >= 0 && dst < rows) acc_add(o + dst * W + i % W, g[i]);
  }
};

template <class F64, class F32>
void by_index(const Tensor& idx, F64 f64, F32 f32_) {
  if (idx.dtype == DT::INT64) f64(idx.data<int64_t>());
  else if (idx.dtype == DT::INT32) f32_(idx.data<int32_t>());
  else throw Decline{};
}

void k_gather(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("X");
  Tensor& idx = r.in("Index");
  if ((idx.device >= 0) != dev) throw Decline{};
  const int64_t rows = x.dims[0], W = x.numel() / std::max<int64_t>(rows, 1), n = idx.numel();
  Dims od = x.dims;
  od[0] = n;
  Tensor o;
  float* op = o.alloc<float>(od, place_of(r));
  const float* xp = f32(x, dev);
  by_index(idx, [&](const int64_t* p) { any::run(r, dev, n * W, GatherRows<int64_t>{xp, p, op, W, rows}); },
           [&](const int32_t* p) { any::run(r, dev, n * W, GatherRows<int32_t>{xp, p, op, W, rows}); });
  *r.out("Out") = o;
}

void k_gather_grad(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  // (an integer Index has no gradient: Index@GRAD stays unset, as in the interpreter)
  Tensor& x = r.in("X");
  Tensor& idx = r.in("Index");
  Tensor& g = r.in("Out@GRAD");
  if ((idx.device >= 0) != dev) throw Decline{};
  const int64_t rows = x.dims[0], W = x.numel() / std::max<int64_t>(rows, 1), n = idx.numel();
  Tensor o;
  float* dx = out_like(r, "X@GRAD", x, &o);
  any::zero(r, dev, dx, x.numel());
  const float* gp = f32(g, dev);
  const int64_t grain = dev ? 4096 : kSerial;
  by_index(idx, [&](const int64_t* p) { any::run(r, dev, n * W, ScatterAddRows<int64_t>{gp, p, dx, W, rows}, grain); },
           [&](const int32_t* p) { any::run(r, dev, n * W, ScatterAddRows<int32_t>{gp, p, dx, W, rows}, grain); });
  *r.out("X@GRAD") = o;
}

template <class I>
struct ScatterRows {  // overwrite: the LAST update of a repeated id wins (index_put's host order)
  const float* up;
  const I* idx;
  float* o;
  int64_t W, rows, n;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t k = i / W, dst = (int64_t)idx[k];
    for (int64_t j = k + 1; j < n; ++j)  // a later write to the same row owns it (parallel-safe)
      if ((int64_t)idx[j] == dst) return;
    if (dst >= 0 && dst < rows) o[dst * W + i % W] = up[i];
  }
};

void k_scatter(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("X");
  Tensor& idx = r.in("Ids");
  Tensor& up = r.in("Updates");
  if ((idx.device >= 0) != dev) throw Decline{};
  const bool overwrite = r.op.GetBool("overwrite", true);
  const int64_t rows = x.dims[0], W = x.numel() / std::max<int64_t>(rows, 1), n = idx.numel();
  if (up.numel() != n * W) throw Decline{};
  Tensor o;
  float* op = out_like(r, "Out", x, &o);
  any::copy(r, dev, op, f32(x, dev), x.numel());
  const float* upp = f32(up, dev);
  const int64_t grain = dev ? 4096 : kSerial;
  if (overwrite) {
    by_index(idx, [&](const int64_t* p) { any::run(r, dev, n * W, ScatterRows<int64_t>{upp, p, op, W, rows, n}, grain); },
             [&](const int32_t* p) { any::run(r, dev, n * W, ScatterRows<int32_t>{upp, p, op, W, rows, n}, grain); });
  } else {
    by_index(idx, [&](const int64_t* p) { any::run(r, dev, n * W, ScatterAddRows<int64_t>{upp, p, op, W, rows}, grain); },
             [&](const int32_t* p) { any::run(r, dev, n * W, ScatterAddRows<int32_t>{upp, p, op, W, rows}, grain); });
  }
  *r.out("Out") = o;
}

template <class I>
struct OneHot {
  const I* x;
  float* o;
  int64_t depth;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t k = i / depth, c = i % depth;
    o[i] = (int64_t)x[k] == c ? 1.f : 0.f;
  }
};

void k_one_hot(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("X");
  if ((x.device >= 0) != dev || r.op.GetInt("dtype", 5) != 5) throw Decline{};  // fp32 output only
  const int64_t depth = r.op.GetInt("depth", 1), n = x.numel();
  Dims od = x.dims;
  if (od.size() > 1 && od.back() == 1) od.back() = depth;
  else od.push_back(depth);
  Tensor o;
  float* op = o.alloc<float>(od, place_of(r));
  o.lod = x.lod;
  by_index(x, [&](const int64_t* p) { any::run(r, dev, n * depth, OneHot<int64_t>{p, op, depth}); },
           [&](const int32_t* p) { any::run(r, dev, n * depth, OneHot<int32_t>{p, op, depth}); });
  *r.out("Out") = o;
}

// ---------------------------------------------------------------- log_softmax (last axis)
struct LogSoftmaxRow {
  const float* x;
  float* o;
  int64_t C;
  __host__ __device__ void operator()(int64_t n) const {
    const float* xr = x + n * C;
    float m = -INFINITY;
    for (int64_t c = 0; c < C; ++c) m = fmaxf(m, xr[c]);
    float s = 0.f;
    for (int64_t c = 0; c < C; ++c) s += expf(xr[c] - m);
    const float l = m + logf(s);
    for (int64_t c = 0; c < C; ++c) o[n * C + c] = xr[c] - l;
  }
};
struct LogSoftmaxGradRow {  // dx = g - softmax * sum(g)
  const float *y, *g;
  float* dx;
  int64_t C;
  __host__ __device__ void operator()(int64_t n) const {
    float s = 0.f;
    for (int64_t c = 0; c < C; ++c) s += g[n * C + c];
    for (int64_t c = 0; c < C; ++c) dx[n * C + c] = g[n * C + c] - expf(y[n * C + c]) * s;
  }
};

int64_t last_axis_rows(const OpRun& r, const Tensor& x) {
  int64_t ax = r.op.GetInt("axis", -1);
  if (ax < 0) ax += (int64_t)x.dims.size();
  if (ax != (int64_t)x.dims.size() - 1) throw Decline{};
  return x.numel() / std::max<int64_t>(x.dims.back(), 1);
}

void k_log_softmax(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("X");
  const int64_t N = last_axis_rows(r, x);
  Tensor o;
  any::run(r, dev, N, LogSoftmaxRow{f32(x, dev), out_like(r, "Out", x, &o), x.dims.back()}, 16);
  *r.out("Out") = o;
}

void k_log_softmax_grad(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& y = r.in("Out");
  Tensor& g = r.in("Out@GRAD");
  const int64_t N = last_axis_rows(r, y);
  Tensor o;
  any::run(r, dev, N, LogSoftmaxGradRow{f32(y, dev), f32(g, dev), out_like(r, "X@GRAD", r.in("X"), &o), y.dims.back()}, 16);
  *r.out("X@GRAD") = o;
}

}  // namespace

#define PA_ANY_KERNEL(name, fn) \
  PA_HOST_KERNEL(name, fn);     \
  PA_DEVICE_KERNEL(name, fn)
PA_ANY_KERNEL(sign, k_sign);
PA_ANY_KERNEL(clip, k_clip);
PA_ANY_KERNEL(clip_grad, k_clip_grad);
PA_ANY_KERNEL(clip_by_norm, k_clip_by_norm);
PA_ANY_KERNEL(clip_by_norm_grad, k_clip_by_norm_grad);
PA_ANY_KERNEL(minus, k_minus);
PA_ANY_KERNEL(minus_grad, k_minus_grad);
PA_ANY_KERNEL(label_smooth, k_label_smooth);
PA_ANY_KERNEL(label_smooth_grad, k_label_smooth_grad);
PA_ANY_KERNEL(sigmoid_cross_entropy_with_logits, k_sigmoid_ce);
PA_ANY_KERNEL(sigmoid_cross_entropy_with_logits_grad, k_sigmoid_ce_grad);
PA_ANY_KERNEL(huber_loss, k_huber);
PA_ANY_KERNEL(huber_loss_grad, k_huber_grad);
PA_ANY_KERNEL(log_loss, k_log_loss);
PA_ANY_KERNEL(log_loss_grad, k_log_loss_grad);
PA_ANY_KERNEL(smooth_l1_loss, k_smooth_l1);
PA_ANY_KERNEL(smooth_l1_loss_grad, k_smooth_l1_grad);
PA_ANY_KERNEL(squared_l2_norm, k_sq_l2_norm);
PA_ANY_KERNEL(squared_l2_norm_grad, k_sq_l2_norm_grad);
PA_ANY_KERNEL(squared_l2_distance, k_sq_l2_dist);
PA_ANY_KERNEL(squared_l2_distance_grad, k_sq_l2_dist_grad);
PA_ANY_KERNEL(cumsum, k_cumsum);
PA_ANY_KERNEL(cumsum_grad, k_cumsum_grad);
PA_ANY_KERNEL(gather, k_gather);
PA_ANY_KERNEL(gather_grad, k_gather_grad);
PA_ANY_KERNEL(scatter, k_scatter);
PA_ANY_KERNEL(one_hot, k_one_hot);
PA_ANY_KERNEL(log_softmax, k_log_softmax);
PA_ANY_KERNEL(log_softmax_grad, k_log_softmax_grad);
#undef PA_ANY_KERNEL

void link_misc_kernels() {}

}  // namespace pa
