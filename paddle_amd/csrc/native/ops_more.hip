// More pointwise losses, shape ops and optimizers of the native executor, host AND
// device from one source (any_place.h): hinge_loss (+grad), modified_huber_loss
// (+grad), rank_loss (+grad), margin_rank_loss (+grad), l1_norm (+grad), reverse
// (+grad), pad (+grad), pad_constant_like (+grad), prelu (+grad), iou_similarity,
// arg_min, fill, assign_value, proximal_gd, proximal_adagrad, matmul_grad, cos_sim
// (+grad), multiplex (+grad), crop (+grad), norm (+grad), conv_shift (+grad),
// bilinear_tensor_product (+grad), maxout (+grad), fake_quantize_abs_max,
// fake_dequantize_max_abs (+grad), rnn_memory_helper (+grad), lod_reset_grad,
// scatter_grad, polygon_box_transform, argsort, row_conv (+grad), lrn (+grad),
// split_lod_tensor / merge_lod_tensor (IfElse), max_pool2d_with_index / unpool (+grads),
// box_coder, mean_iou, bilinear / nearest interpolation (+grads), pad2d (+grad),
// im2sequence (+grad), fc_grad.
//
// Semantics: reference operators/{hinge_loss,modified_huber_loss,rank_loss,
// margin_rank_loss,l1_norm,reverse,pad,pad_constant_like,prelu,iou_similarity,
// arg_min_max_base,fill,assign_value,proximal_gd,proximal_adagrad}_op.h; the Python
// kernels of operators/{nn,math,tensor,detection,optimizer}_ops.py compute the same
// functions and the auto-VJP grad ops their derivatives (slots: the forward inputs,
// outputs and Out@GRAD; <input>@GRAD out).  fp32 data (other dtypes decline to the
// embedder's kernel); index tensors int64 / int32.
#include <hip/hip_runtime.h>
#include <math.h>

#include <vector>

#include "any_place.h"

namespace pa {
namespace {

using any::f32;
using Dims = std::vector<int64_t>;

__host__ __device__ inline void acc_add(float* p, float v) {
#if defined(__HIP_DEVICE_COMPILE__)
  atomicAdd(p, v);
#else
  *p += v;
#endif
}

int place_of(const OpRun& r) { return r.ctx.device >= 0 ? r.ctx.device : -1; }
bool on_dev(const OpRun& r) { return r.ctx.device >= 0; }

float* new_like(const OpRun& r, const Tensor& like, Tensor* keep) {
  float* p = keep->alloc<float>(like.dims, place_of(r));
  keep->lod = like.lod;
  return p;
}

// an optional gradient output: its tensor when the grad op asks for it, else null
float* grad_out(const OpRun& r, const char* slot, const Tensor& like, Tensor* keep) {
  if (r.op.Outputs(slot).empty() || !r.out_var(slot)) return nullptr;
  return new_like(r, like, keep);
}

void set(const OpRun& r, const char* slot, const Tensor& t) {
  if (Tensor* o = r.out(slot)) *o = t;
}

// ---------------------------------------------------------------- pointwise losses
struct Hinge {
  const float *x, *y;
  float* o;
  __host__ __device__ void operator()(int64_t i) const { o[i] = fmaxf(0.f, 1.f - x[i] * (2.f * y[i] - 1.f)); }
};
struct HingeGrad {
  const float *x, *y, *g;
  float* dx;
  __host__ __device__ void operator()(int64_t i) const {
    const float s = 2.f * y[i] - 1.f;
    dx[i] = x[i] * s < 1.f ? -s * g[i] : 0.f;
  }
};

void k_hinge(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("Logits");
  Tensor& y = r.in("Labels");
  if (x.numel() != y.numel()) throw Decline{};
  Tensor o;
  any::run(r, dev, x.numel(), Hinge{f32(x, dev), f32(y, dev), new_like(r, x, &o)});
  set(r, "Loss", o);
}

void k_hinge_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("Logits");
  Tensor d;
  float* dx = grad_out(r, "Logits@GRAD", x, &d);
  if (dx) any::run(r, dev, x.numel(), HingeGrad{f32(x, dev), f32(r.in("Labels"), dev), f32(r.in("Loss@GRAD"), dev), dx});
  if (dx) set(r, "Logits@GRAD", d);
}

struct ModHuber {
  const float *x, *y;
  float *z, *o;
  __host__ __device__ void operator()(int64_t i) const {
    const float v = x[i] * (2.f * y[i] - 1.f);
    z[i] = v;
    o[i] = v < -1.f ? -4.f * v : (v < 1.f ? (1.f - v) * (1.f - v) : 0.f);
  }
};
struct ModHuberGrad {
  const float *y, *z, *g;
  float* dx;
  __host__ __device__ void operator()(int64_t i) const {
    const float v = z[i], s = 2.f * y[i] - 1.f;
    dx[i] = g[i] * (v < -1.f ? -4.f * s : (v < 1.f ? -2.f * (1.f - v) * s : 0.f));
  }
};

void k_mod_huber(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  Tensor& y = r.in("Y");
  if (x.numel() != y.numel()) throw Decline{};
  Tensor z, o;
  any::run(r, dev, x.numel(), ModHuber{f32(x, dev), f32(y, dev), new_like(r, x, &z), new_like(r, x, &o)});
  set(r, "IntermediateVal", z);
  set(r, "Out", o);
}

void k_mod_huber_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  Tensor d;
  float* dx = grad_out(r, "X@GRAD", x, &d);
  if (!dx) return;
  any::run(r, dev, x.numel(),
           ModHuberGrad{f32(r.in("Y"), dev), f32(r.in("IntermediateVal"), dev), f32(r.in("Out@GRAD"), dev), dx});
  set(r, "X@GRAD", d);
}

// rank_loss: log(1 + e^(l - r)) - label (l - r)
struct RankLoss {
  const float *lab, *l, *rt;
  float* o;
  __host__ __device__ void operator()(int64_t i) const {
    const float d = l[i] - rt[i];
    o[i] = log1pf(expf(d)) - lab[i] * d;
  }
};
struct RankLossGrad {
  const float *lab, *l, *rt, *g;
  float *dl, *dr;
  __host__ __device__ void operator()(int64_t i) const {
    const float d = l[i] - rt[i];
    const float s = 1.f / (1.f + expf(-d)) - lab[i];
    if (dl) dl[i] = g[i] * s;
    if (dr) dr[i] = -g[i] * s;
  }
};

struct RankLabelGrad {
  const float *l, *rt, *g;
  float* o;
  __host__ __device__ void operator()(int64_t i) const { o[i] = -(l[i] - rt[i]) * g[i]; }
};

void k_rank_loss(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& l = r.in("Left");
  Tensor o;
  if (r.in("Right").numel() != l.numel() || r.in("Label").numel() != l.numel()) throw Decline{};
  any::run(r, dev, l.numel(), RankLoss{f32(r.in("Label"), dev), f32(l, dev), f32(r.in("Right"), dev), new_like(r, l, &o)});
  set(r, "Out", o);
}

void k_rank_loss_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& l = r.in("Left");
  Tensor dL, dR, dLab;
  float* dl = grad_out(r, "Left@GRAD", l, &dL);
  float* dr = grad_out(r, "Right@GRAD", r.in("Right"), &dR);
  float* dlab = grad_out(r, "Label@GRAD", r.in("Label"), &dLab);
  any::run(r, dev, l.numel(),
           RankLossGrad{f32(r.in("Label"), dev), f32(l, dev), f32(r.in("Right"), dev), f32(r.in("Out@GRAD"), dev), dl, dr});
  if (dlab) {  // d/dlabel = -(l - r) g
    any::run(r, dev, l.numel(), RankLabelGrad{f32(l, dev), f32(r.in("Right"), dev), f32(r.in("Out@GRAD"), dev), dlab});
    set(r, "Label@GRAD", dLab);
  }
  if (dl) set(r, "Left@GRAD", dL);
  if (dr) set(r, "Right@GRAD", dR);
}

// margin_rank_loss: relu(-label (x1 - x2) + margin); Activated = 1 where positive
struct MarginRank {
  const float *x1, *x2, *lab;
  float *o, *act;
  float margin;
  __host__ __device__ void operator()(int64_t i) const {
    const float v = -lab[i] * (x1[i] - x2[i]) + margin;
    o[i] = fmaxf(v, 0.f);
    act[i] = v > 0.f ? 1.f : 0.f;
  }
};
struct MarginRankGrad {
  const float *x1, *x2, *lab, *g;
  float *d1, *d2, *dlab;
  float margin;
  __host__ __device__ void operator()(int64_t i) const {
    const float v = -lab[i] * (x1[i] - x2[i]) + margin;
    const float a = v > 0.f ? g[i] : 0.f;
    if (d1) d1[i] = -lab[i] * a;
    if (d2) d2[i] = lab[i] * a;
    if (dlab) dlab[i] = -(x1[i] - x2[i]) * a;
  }
};

void k_margin_rank(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x1 = r.in("X1");
  if (r.in("X2").numel() != x1.numel() || r.in("Label").numel() != x1.numel()) throw Decline{};
  Tensor o, a;
  any::run(r, dev, x1.numel(),
           MarginRank{f32(x1, dev), f32(r.in("X2"), dev), f32(r.in("Label"), dev), new_like(r, x1, &o),
                      new_like(r, x1, &a), r.op.GetFloat("margin", 0.f)});
  set(r, "Out", o);
  set(r, "Activated", a);
}

void k_margin_rank_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x1 = r.in("X1");
  Tensor d1, d2, dl;
  float* p1 = grad_out(r, "X1@GRAD", x1, &d1);
  float* p2 = grad_out(r, "X2@GRAD", r.in("X2"), &d2);
  float* pl = grad_out(r, "Label@GRAD", r.in("Label"), &dl);
  any::run(r, dev, x1.numel(),
           MarginRankGrad{f32(x1, dev), f32(r.in("X2"), dev), f32(r.in("Label"), dev), f32(r.in("Out@GRAD"), dev), p1, p2,
                          pl, r.op.GetFloat("margin", 0.f)});
  if (p1) set(r, "X1@GRAD", d1);
  if (p2) set(r, "X2@GRAD", d2);
  if (pl) set(r, "Label@GRAD", dl);
}

// ---------------------------------------------------------------- l1_norm
struct AbsSumChunk {
  const float* x;
  float* out;
  int64_t n, chunk;
  __host__ __device__ void operator()(int64_t c) const {
    float s = 0.f;
    const int64_t a = c * chunk, b = a + chunk < n ? a + chunk : n;
    for (int64_t i = a; i < b; ++i) s += fabsf(x[i]);
    acc_add(out, s);
  }
};

void k_l1_norm(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  Tensor o;
  float* op = o.alloc<float>({1}, place_of(r));
  any::zero(r, dev, op, 1);
  const int64_t n = x.numel(), chunk = 4096, nc = (n + chunk - 1) / chunk;
  // host: chunks in order on one thread (deterministic sum); device: one atomic per chunk
  if (dev) any::run(r, dev, nc, AbsSumChunk{f32(x, dev), op, n, chunk});
  else AbsSumChunk{f32(x, dev), op, n, n > 0 ? n : 1}(0);
  set(r, "Out", o);
}

struct L1Grad {
  const float *x, *g;
  float* dx;
  __host__ __device__ void operator()(int64_t i) const {
    dx[i] = g[0] * (x[i] > 0.f ? 1.f : (x[i] < 0.f ? -1.f : 0.f));
  }
};

void k_l1_norm_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  Tensor d;
  float* dx = grad_out(r, "X@GRAD", x, &d);
  if (!dx) return;
  any::run(r, dev, x.numel(), L1Grad{f32(x, dev), f32(r.in("Out@GRAD"), dev), dx});
  set(r, "X@GRAD", d);
}

// ---------------------------------------------------------------- N-d index maps
constexpr int kMaxD = 8;
struct Shape {
  int nd;
  int64_t d[kMaxD];
};

Shape shape_of(const Dims& d) {
  PA_CHECK((int)d.size() <= kMaxD, "tensor rank %d above %d", (int)d.size(), kMaxD);
  Shape s{(int)d.size(), {}};
  for (int i = 0; i < s.nd; ++i) s.d[i] = d[i];
  return s;
}

// out[o] = in[i] with, per dim, i_k = flip_k ? D_k - 1 - o_k : o_k - off_k; outside the
// input: `fill` (pad) -- one functor for reverse, pad, pad_constant_like, their grads
struct Remap {
  const float* in;
  float* out;
  Shape os, is;
  int64_t off[kMaxD];
  int flip[kMaxD];
  float fill;
  __host__ __device__ void operator()(int64_t o) const {
    int64_t rem = o, idx = 0, stride = 1;
    bool inside = true;
    int64_t coord[kMaxD];
    for (int k = os.nd - 1; k >= 0; --k) {
      coord[k] = rem % os.d[k];
      rem /= os.d[k];
    }
    for (int k = os.nd - 1; k >= 0; --k) {
      const int64_t c = flip[k] ? is.d[k] - 1 - coord[k] : coord[k] - off[k];
      if (c < 0 || c >= is.d[k]) inside = false;
      idx += c * stride;
      stride *= is.d[k];
    }
    out[o] = inside ? in[idx] : fill;
  }
};

void remap(const OpRun& r, const Tensor& in, const Dims& odims, const std::vector<int64_t>& off,
           const std::vector<int>& flip, float fill, Tensor* out) {
  const bool dev = on_dev(r);
  Remap m{f32(in, dev), out->alloc<float>(odims, place_of(r)), shape_of(odims), shape_of(in.dims), {}, {}, fill};
  for (int k = 0; k < kMaxD; ++k) {
    m.off[k] = k < (int)off.size() ? off[k] : 0;
    m.flip[k] = k < (int)flip.size() ? flip[k] : 0;
  }
  any::run(r, dev, out->numel(), m);
}

std::vector<int> flip_axes(const OpRun& r, int nd) {
  std::vector<int> f(nd, 0);
  for (int64_t a : r.op.GetInts("axis")) {
    const int k = (int)(a < 0 ? a + nd : a);
    PA_CHECK(k >= 0 && k < nd, "reverse: axis %lld out of range", (long long)a);
    f[k] = 1;
  }
  return f;
}

void k_reverse(const OpRun& r) {
  Tensor& x = r.in("X");
  Tensor o;
  remap(r, x, x.dims, {}, flip_axes(r, (int)x.dims.size()), 0.f, &o);
  o.lod = x.lod;
  set(r, "Out", o);
}

void k_reverse_grad(const OpRun& r) {
  Tensor& g = r.in("Out@GRAD");
  if (r.op.Outputs("X@GRAD").empty() || !r.out_var("X@GRAD")) return;
  Tensor o;
  remap(r, g, g.dims, {}, flip_axes(r, (int)g.dims.size()), 0.f, &o);
  set(r, "X@GRAD", o);
}

void k_pad(const OpRun& r) {
  Tensor& x = r.in("X");
  const auto p = r.op.GetInts("paddings");
  const int nd = (int)x.dims.size();
  if ((int)p.size() != 2 * nd) throw Decline{};
  Dims od(nd);
  std::vector<int64_t> off(nd);
  for (int k = 0; k < nd; ++k) {
    od[k] = x.dims[k] + p[2 * k] + p[2 * k + 1];
    off[k] = p[2 * k];
  }
  Tensor o;
  remap(r, x, od, off, {}, r.op.GetFloat("pad_value", 0.f), &o);
  set(r, "Out", o);
}

// pad's gradient: the window of Out@GRAD the input occupies
void k_pad_grad(const OpRun& r) {
  Tensor& x = r.in("X");
  Tensor& g = r.in("Out@GRAD");
  if (r.op.Outputs("X@GRAD").empty() || !r.out_var("X@GRAD")) return;
  const auto p = r.op.GetInts("paddings");
  const int nd = (int)x.dims.size();
  if ((int)p.size() != 2 * nd) throw Decline{};
  std::vector<int64_t> off(nd);
  for (int k = 0; k < nd; ++k) off[k] = -p[2 * k];
  Tensor o;
  remap(r, g, x.dims, off, {}, 0.f, &o);
  set(r, "X@GRAD", o);
}

// pad_constant_like: Y padded at the end of every dim up to X's shape
void k_pad_constant_like(const OpRun& r) {
  Tensor& x = r.in("X");
  Tensor& y = r.in("Y");
  if (x.dims.size() != y.dims.size()) throw Decline{};
  Tensor o;
  remap(r, y, x.dims, {}, {}, r.op.GetFloat("pad_value", 0.f), &o);
  set(r, "Out", o);
}

void k_pad_constant_like_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& y = r.in("Y");
  Tensor& g = r.in("Out@GRAD");
  if (!r.op.Outputs("Y@GRAD").empty() && r.out_var("Y@GRAD")) {
    Tensor o;
    remap(r, g, y.dims, {}, {}, 0.f, &o);
    set(r, "Y@GRAD", o);
  }
  Tensor dx;
  if (float* p = grad_out(r, "X@GRAD", r.in("X"), &dx)) {  // X only gives the shape
    any::zero(r, dev, p, dx.numel());
    set(r, "X@GRAD", dx);
  }
}

// ---------------------------------------------------------------- prelu
// alpha index of element i: 0 (all), channel (i / inner) % C, element i % (C * inner)
struct PRelu {
  const float *x, *a;
  float* o;
  int mode;
  int64_t C, inner;
  __host__ __device__ int64_t ai(int64_t i) const {
    return mode == 0 ? 0 : (mode == 1 ? (i / inner) % C : i % (C * inner));
  }
  __host__ __device__ void operator()(int64_t i) const { o[i] = x[i] > 0.f ? x[i] : a[ai(i)] * x[i]; }
};
struct PReluGradX {
  PRelu p;
  const float* g;
  float* dx;
  __host__ __device__ void operator()(int64_t i) const { dx[i] = g[i] * (p.x[i] > 0.f ? 1.f : p.a[p.ai(i)]); }
};
// dAlpha[j] = sum over the elements using alpha j of g x (x <= 0); one lane per alpha
struct PReluGradA {
  PRelu p;
  const float* g;
  float* da;
  int64_t n, per;  // elements, elements per alpha (all: n)
  __host__ __device__ void operator()(int64_t j) const {
    float s = 0.f;
    if (p.mode == 0) {
      for (int64_t i = 0; i < n; ++i) s += p.x[i] > 0.f ? 0.f : g[i] * p.x[i];
    } else if (p.mode == 1) {
      for (int64_t b = 0; b < n / (p.C * p.inner); ++b)
        for (int64_t k = 0; k < p.inner; ++k) {
          const int64_t i = (b * p.C + j) * p.inner + k;
          s += p.x[i] > 0.f ? 0.f : g[i] * p.x[i];
        }
    } else {
      for (int64_t i = j; i < n; i += per) s += p.x[i] > 0.f ? 0.f : g[i] * p.x[i];
    }
    da[j] = s;
  }
};

PRelu prelu_of(const OpRun& r, bool dev, float* out) {
  Tensor& x = r.in("X");
  Tensor& a = r.in("Alpha");
  const std::string mode = r.op.GetString("mode", "all");
  PRelu p{f32(x, dev), f32(a, dev), out, 0, 1, 1};
  if (mode == "channel") {
    if (x.dims.size() < 2) throw Decline{};
    p.mode = 1;
    p.C = x.dims[1];
    for (size_t k = 2; k < x.dims.size(); ++k) p.inner *= x.dims[k];
    if (a.numel() != p.C) throw Decline{};
  } else if (mode == "element") {
    p.mode = 2;
    p.C = x.dims.empty() ? 1 : x.numel() / x.dims[0];
    if (a.numel() != p.C) throw Decline{};
  } else if (a.numel() < 1) {
    throw Decline{};
  }
  return p;
}

void k_prelu(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  Tensor o;
  float* op = new_like(r, x, &o);
  any::run(r, dev, x.numel(), prelu_of(r, dev, op));
  set(r, "Out", o);
}

void k_prelu_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  const float* g = f32(r.in("Out@GRAD"), dev);
  PRelu p = prelu_of(r, dev, nullptr);
  Tensor dX, dA;
  if (float* dx = grad_out(r, "X@GRAD", x, &dX)) {
    any::run(r, dev, x.numel(), PReluGradX{p, g, dx});
    set(r, "X@GRAD", dX);
  }
  if (float* da = grad_out(r, "Alpha@GRAD", r.in("Alpha"), &dA)) {
    const int64_t na = r.in("Alpha").numel();
    any::run(r, dev, p.mode == 0 ? 1 : na, PReluGradA{p, g, da, x.numel(), p.mode == 2 ? p.C : x.numel()}, 1);
    set(r, "Alpha@GRAD", dA);
  }
}

// ---------------------------------------------------------------- iou_similarity
struct Iou {
  const float *a, *b;
  float* o;
  int64_t M;
  float one;
  __host__ __device__ void operator()(int64_t k) const {
    const float* p = a + (k / M) * 4;
    const float* q = b + (k % M) * 4;
    const float aa = (p[2] - p[0] + one) * (p[3] - p[1] + one);
    const float ab = (q[2] - q[0] + one) * (q[3] - q[1] + one);
    const float w = fmaxf(fminf(p[2], q[2]) - fmaxf(p[0], q[0]) + one, 0.f);
    const float h = fmaxf(fminf(p[3], q[3]) - fmaxf(p[1], q[1]) + one, 0.f);
    const float in = w * h;
    o[k] = in / fmaxf(aa + ab - in, 1e-10f);
  }
};

void k_iou(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  Tensor& y = r.in("Y");
  if (x.dims.size() != 2 || y.dims.size() != 2 || x.dims[1] != 4 || y.dims[1] != 4) throw Decline{};
  Tensor o;
  float* op = o.alloc<float>({x.dims[0], y.dims[0]}, place_of(r));
  o.lod = x.lod;
  any::run(r, dev, x.dims[0] * y.dims[0],
           Iou{f32(x, dev), f32(y, dev), op, y.dims[0], r.op.GetBool("box_normalized", true) ? 0.f : 1.f});
  set(r, "Out", o);
}

// ---------------------------------------------------------------- arg_min
struct ArgMin {
  const float* x;
  int64_t* o;
  int64_t outer, n, inner;
  __host__ __device__ void operator()(int64_t t) const {
    const int64_t a = t / inner, b = t % inner;
    const float* p = x + a * n * inner + b;
    int64_t best = 0;
    float bv = p[0];
    for (int64_t k = 1; k < n; ++k)
      if (p[k * inner] < bv) {
        bv = p[k * inner];
        best = k;
      }
    o[t] = best;
  }
};

void k_arg_min(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  const int nd = (int)x.dims.size();
  int64_t ax = r.op.GetInt("axis", 0);
  if (ax < 0) ax += nd;
  if (nd == 0 || ax < 0 || ax >= nd || x.dims[ax] == 0) throw Decline{};
  int64_t outer = 1, inner = 1;
  for (int k = 0; k < ax; ++k) outer *= x.dims[k];
  for (int k = (int)ax + 1; k < nd; ++k) inner *= x.dims[k];
  Dims od;
  for (int k = 0; k < nd; ++k)
    if (k != ax) od.push_back(x.dims[k]);
  Tensor o;
  int64_t* op = static_cast<int64_t*>(o.alloc(DT::INT64, od, place_of(r)));
  any::run(r, dev, outer * inner, ArgMin{f32(x, dev), op, outer, x.dims[ax], inner});
  set(r, "Out", o);
}

// ---------------------------------------------------------------- fill / assign_value
// a host constant of the op's dtype written to the op's place
void write_values(const OpRun& r, DT dt, const Dims& shape, const std::vector<double>& vals, const char* slot) {
  Tensor o;
  void* p = o.alloc(dt, shape, place_of(r));
  const int64_t n = o.numel();
  if ((int64_t)vals.size() != n) fail("%s: %zu values for %lld elements", r.op.type.c_str(), vals.size(), (long long)n);
  std::vector<char> h((size_t)o.nbytes());
  for (int64_t i = 0; i < n; ++i) {
    switch (dt) {
      case DT::FP32: reinterpret_cast<float*>(h.data())[i] = (float)vals[i]; break;
      case DT::FP64: reinterpret_cast<double*>(h.data())[i] = vals[i]; break;
      case DT::INT32: reinterpret_cast<int32_t*>(h.data())[i] = (int32_t)vals[i]; break;
      case DT::INT64: reinterpret_cast<int64_t*>(h.data())[i] = (int64_t)vals[i]; break;
      case DT::BOOL: case DT::UINT8: reinterpret_cast<uint8_t*>(h.data())[i] = (uint8_t)(vals[i] != 0); break;
      default: throw Decline{};
    }
  }
  if (n) device_copy(p, o.device, h.data(), -1, o.nbytes(), r.ctx.stream);
  set(r, slot, o);
}

void k_fill(const OpRun& r) {
  std::vector<double> v;
  for (float f : r.op.GetFloats("value")) v.push_back(f);
  write_values(r, (DT)r.op.GetInt("dtype", 5), r.op.GetInts("shape"), v, "Out");
}

void k_assign_value(const OpRun& r) {
  std::vector<double> v;
  for (float f : r.op.GetFloats("fp32_values")) v.push_back(f);
  if (v.empty())
    for (int64_t i : r.op.GetInts("int32_values")) v.push_back((double)i);
  write_values(r, (DT)r.op.GetInt("dtype", 5), r.op.GetInts("shape"), v, "Out");
}

// ---------------------------------------------------------------- proximal optimizers
struct ProxGD {
  const float *p, *g, *lr;
  float* out;
  float l1, l2;
  __host__ __device__ void operator()(int64_t i) const {
    const float a = lr[0], prox = p[i] - a * g[i];
    const float s = prox > 0.f ? 1.f : (prox < 0.f ? -1.f : 0.f);
    out[i] = s * fmaxf(fabsf(prox) - a * l1, 0.f) / (1.f + a * l2);
  }
};
struct ProxAdagrad {
  const float *p, *m, *g, *lr;
  float *out, *mout;
  float l1, l2;
  __host__ __device__ void operator()(int64_t i) const {
    const float m2 = m[i] + g[i] * g[i];
    const float a = lr[0] / sqrtf(m2), prox = p[i] - a * g[i];
    const float s = prox > 0.f ? 1.f : (prox < 0.f ? -1.f : 0.f);
    out[i] = s * fmaxf(fabsf(prox) - a * l1, 0.f) / (1.f + a * l2);
    mout[i] = m2;
  }
};

// an in-place output keeps its buffer (ParamOut = Param)
float* inplace_out(const OpRun& r, const char* slot, const Tensor& like) {
  Tensor* o = r.out(slot);
  if (o->raw() == like.raw() && o->initialized()) return o->data<float>();
  return o->alloc<float>(like.dims, place_of(r));
}

void k_proximal_gd(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& p = r.in("Param");
  Tensor& g = r.in("Grad");
  if (g.numel() != p.numel()) throw Decline{};
  const float* lr = f32(r.in("LearningRate"), dev);
  const float *pp = f32(p, dev), *gp = f32(g, dev);
  any::run(r, dev, p.numel(), ProxGD{pp, gp, lr, inplace_out(r, "ParamOut", p), r.op.GetFloat("l1", 0.f),
                                     r.op.GetFloat("l2", 0.f)});
}

void k_proximal_adagrad(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& p = r.in("Param");
  Tensor& m = r.in("Moment");
  Tensor& g = r.in("Grad");
  if (g.numel() != p.numel() || m.numel() != p.numel()) throw Decline{};
  const float* lr = f32(r.in("LearningRate"), dev);
  const float *pp = f32(p, dev), *mp = f32(m, dev), *gp = f32(g, dev);
  any::run(r, dev, p.numel(),
           ProxAdagrad{pp, mp, gp, lr, inplace_out(r, "ParamOut", p), inplace_out(r, "MomentOut", m),
                       r.op.GetFloat("l1", 0.f), r.op.GetFloat("l2", 0.f)});
}

// ---------------------------------------------------------------- matmul_grad
// Out = alpha op(X) op(Y) per batch (rank-1 operands promoted, a batch of 1 broadcast):
//   d op(X) = alpha dOut op(Y)^T, d op(Y) = alpha op(X)^T dOut, stored back through
//   the transposes; a broadcast operand's gradient sums over the batches
void k_matmul_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  Tensor& y = r.in("Y");
  Tensor& g = r.in("Out@GRAD");
  const bool tx = r.op.GetBool("transpose_X"), ty = r.op.GetBool("transpose_Y");
  const float alpha = r.op.GetFloat("alpha", 1.f);
  Dims xd = x.dims, yd = y.dims;
  if (xd.size() == 1) xd = tx ? Dims{xd[0], 1} : Dims{1, xd[0]};
  if (yd.size() == 1) yd = ty ? Dims{1, yd[0]} : Dims{yd[0], 1};
  const int64_t xr = xd[xd.size() - 2], xc = xd.back(), yr = yd[yd.size() - 2], yc = yd.back();
  const int64_t M = tx ? xc : xr, K = tx ? xr : xc, N = ty ? yr : yc;
  if ((ty ? yc : yr) != K) throw Decline{};
  int64_t bx = 1, by = 1;
  for (size_t i = 0; i + 2 < xd.size(); ++i) bx *= xd[i];
  for (size_t i = 0; i + 2 < yd.size(); ++i) by *= yd[i];
  if (!(bx == by || bx == 1 || by == 1)) throw Decline{};
  const int64_t B = bx > by ? bx : by;
  if (g.numel() != B * M * N) throw Decline{};
  const float *xp = f32(x, dev), *yp = f32(y, dev), *gp = f32(g, dev);
  Tensor dX, dY;
  if (float* dx = grad_out(r, "X@GRAD", x, &dX)) {
    for (int64_t b = 0; b < B; ++b) {
      const float* gb = gp + b * M * N;
      const float* yb = yp + (by == 1 ? 0 : b * K * N);
      float* db = dx + (bx == 1 ? 0 : b * M * K);
      const float beta = (bx == 1 && b > 0) ? 1.f : 0.f;
      if (!tx)  // dX [M, K] = g op(Y)^T
        any::gemm(r, dev, false, !ty, M, K, N, alpha, gb, N, yb, ty ? K : N, beta, db, K);
      else      // dX [K, M] = op(Y) g^T
        any::gemm(r, dev, ty, true, K, M, N, alpha, yb, ty ? K : N, gb, N, beta, db, M);
    }
    set(r, "X@GRAD", dX);
  }
  if (float* dy = grad_out(r, "Y@GRAD", y, &dY)) {
    for (int64_t b = 0; b < B; ++b) {
      const float* gb = gp + b * M * N;
      const float* xb = xp + (bx == 1 ? 0 : b * M * K);
      float* db = dy + (by == 1 ? 0 : b * K * N);
      const float beta = (by == 1 && b > 0) ? 1.f : 0.f;
      if (!ty)  // dY [K, N] = op(X)^T g
        any::gemm(r, dev, !tx, false, K, N, M, alpha, xb, tx ? M : K, gb, N, beta, db, N);
      else      // dY [N, K] = g^T op(X)
        any::gemm(r, dev, true, tx, N, K, M, alpha, gb, N, xb, tx ? M : K, beta, db, K);
    }
    set(r, "Y@GRAD", dY);
  }
}

// ---------------------------------------------------------------- cos_sim
// Out[i] = <x_i, y_i> / (|x_i| |y_i|) over rows (Y may be one row, broadcast)
struct CosSim {
  const float *x, *y;
  float *o, *xn, *yn;
  int64_t D, ybc;
  __host__ __device__ void operator()(int64_t i) const {
    const float* a = x + i * D;
    const float* b = y + (ybc ? 0 : i * D);
    float ab = 0.f, aa = 0.f, bb = 0.f;
    for (int64_t k = 0; k < D; ++k) {
      ab += a[k] * b[k];
      aa += a[k] * a[k];
      bb += b[k] * b[k];
    }
    xn[i] = sqrtf(aa);
    if (!ybc || i == 0) yn[ybc ? 0 : i] = sqrtf(bb);
    o[i] = ab / (sqrtf(aa) * sqrtf(bb));
  }
};
// dx_i = g_i (y_i / (|x||y|) - out_i x_i / |x|^2); dy likewise (summed over rows when broadcast)
struct CosSimGradX {
  const float *x, *y, *o, *xn, *yn, *g;
  float* dx;
  int64_t D, ybc;
  __host__ __device__ void operator()(int64_t t) const {
    const int64_t i = t / D, k = t % D;
    const float a = x[t], b = y[(ybc ? 0 : i * D) + k];
    const float nx = xn[i], ny = yn[ybc ? 0 : i];
    dx[t] = g[i] * (b / (nx * ny) - o[i] * a / (nx * nx));
  }
};
struct CosSimGradY {
  const float *x, *y, *o, *xn, *yn, *g;
  float* dy;
  int64_t D, rows, ybc;
  __host__ __device__ void operator()(int64_t t) const {
    if (!ybc) {
      const int64_t i = t / D;
      const float a = x[t], b = y[t], nx = xn[i], ny = yn[i];
      dy[t] = g[i] * (a / (nx * ny) - o[i] * b / (ny * ny));
      return;
    }
    const int64_t k = t;  // one lane per column of the broadcast row
    const float b = y[k], ny = yn[0];
    float s = 0.f;
    for (int64_t i = 0; i < rows; ++i) s += g[i] * (x[i * D + k] / (xn[i] * ny) - o[i] * b / (ny * ny));
    dy[k] = s;
  }
};

void k_cos_sim(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  Tensor& y = r.in("Y");
  if (x.dims.empty() || y.dims.empty()) throw Decline{};
  const int64_t rows = x.dims[0], D = rows ? x.numel() / rows : 0;
  const int64_t yrows = y.dims[0];
  if (y.numel() != yrows * D || !(yrows == rows || yrows == 1)) throw Decline{};
  Tensor o, xn, yn;
  float* op = o.alloc<float>({rows, 1}, place_of(r));
  float* xp = xn.alloc<float>({rows, 1}, place_of(r));
  float* yp = yn.alloc<float>({yrows, 1}, place_of(r));
  o.lod = x.lod;
  any::run(r, dev, rows, CosSim{f32(x, dev), f32(y, dev), op, xp, yp, D, yrows == 1 && rows > 1 ? 1 : 0});
  set(r, "Out", o);
  set(r, "XNorm", xn);
  set(r, "YNorm", yn);
}

void k_cos_sim_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  Tensor& y = r.in("Y");
  const int64_t rows = x.dims[0], D = rows ? x.numel() / rows : 0;
  const int64_t ybc = y.dims[0] == 1 && rows > 1 ? 1 : 0;
  const float *xp = f32(x, dev), *yp = f32(y, dev), *op = f32(r.in("Out"), dev);
  const float *xn = f32(r.in("XNorm"), dev), *yn = f32(r.in("YNorm"), dev), *gp = f32(r.in("Out@GRAD"), dev);
  Tensor dX, dY;
  if (float* dx = grad_out(r, "X@GRAD", x, &dX)) {
    any::run(r, dev, x.numel(), CosSimGradX{xp, yp, op, xn, yn, gp, dx, D, ybc});
    set(r, "X@GRAD", dX);
  }
  if (float* dy = grad_out(r, "Y@GRAD", y, &dY)) {
    any::run(r, dev, ybc ? D : y.numel(), CosSimGradY{xp, yp, op, xn, yn, gp, dy, D, rows, ybc});
    set(r, "Y@GRAD", dY);
  }
}

// ---------------------------------------------------------------- multiplex
// Out[i] = X[ids[i]][i]; the candidates' row pointers go in a small table
struct Multiplex {
  const int64_t* ids;
  const float* const* xs;
  float* o;
  int64_t D;
  __host__ __device__ void operator()(int64_t t) const { o[t] = xs[ids[t / D]][t]; }
};
struct MultiplexGrad {
  const int64_t* ids;
  float* const* dxs;  // null entries: no gradient wanted
  const float* g;
  int64_t K, D;
  __host__ __device__ void operator()(int64_t t) const {
    const int64_t sel = ids[t / D];
    for (int64_t k = 0; k < K; ++k)
      if (dxs[k]) dxs[k][t] = k == sel ? g[t] : 0.f;
  }
};

template <class P>
P* ptr_table(const OpRun& r, bool dev, const char* name, const std::vector<P>& v, std::vector<P>* keep) {
  *keep = v;
  if (!dev) return keep->data();
  return (P*)device_upload(r, name, keep->data(), keep->size() * sizeof(P));
}

void k_multiplex(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& ids = r.in("Ids");
  auto xs = r.ins("X");
  if (xs.empty() || ids.dtype != DT::INT64 || (ids.device >= 0) != dev) throw Decline{};
  const Tensor& x0 = *xs[0];
  const int64_t rows = x0.dims.empty() ? 0 : x0.dims[0], D = rows ? x0.numel() / rows : 0;
  if (ids.numel() != rows) throw Decline{};
  std::vector<const float*> ptrs;
  for (Tensor* t : xs) {
    if (t->numel() != x0.numel()) throw Decline{};
    ptrs.push_back(f32(*t, dev));
  }
  std::vector<const float*> keep;
  const float* const* tab = ptr_table(r, dev, "@mpx_ptrs@", ptrs, &keep);
  Tensor o;
  float* op = new_like(r, x0, &o);
  any::run(r, dev, rows * D, Multiplex{ids.data<int64_t>(), tab, op, D});
  set(r, "Out", o);
}

void k_multiplex_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& ids = r.in("Ids");
  auto xs = r.ins("X");
  if (xs.empty() || ids.dtype != DT::INT64 || (ids.device >= 0) != dev) throw Decline{};
  const int64_t rows = xs[0]->dims[0], D = rows ? xs[0]->numel() / rows : 0;
  const auto& gnames = r.op.Outputs("X@GRAD");
  std::vector<Tensor> grads(xs.size());
  std::vector<float*> ptrs(xs.size(), nullptr);
  for (size_t k = 0; k < xs.size() && k < gnames.size(); ++k)
    if (gnames[k] != "@EMPTY@" && !gnames[k].empty()) ptrs[k] = new_like(r, *xs[k], &grads[k]);
  std::vector<float*> keep;
  float* const* tab = ptr_table(r, dev, "@mpxg_ptrs@", ptrs, &keep);
  any::run(r, dev, rows * D, MultiplexGrad{ids.data<int64_t>(), tab, f32(r.in("Out@GRAD"), dev), (int64_t)xs.size(), D});
  for (size_t k = 0; k < xs.size() && k < gnames.size(); ++k)
    if (ptrs[k]) *r.out("X@GRAD", k) = grads[k];
}

// ---------------------------------------------------------------- crop
void k_crop(const OpRun& r) {
  Tensor& x = r.in("X");
  Dims shape;
  if (Tensor* y = r.in_opt("Y")) shape = y->dims;
  else shape = r.op.GetInts("shape");
  auto off = r.op.GetInts("offsets");
  if (shape.size() != x.dims.size()) throw Decline{};
  if (off.empty()) off.assign(x.dims.size(), 0);
  std::vector<int64_t> neg(off.size());
  for (size_t k = 0; k < off.size(); ++k) neg[k] = -off[k];
  Tensor o;
  remap(r, x, shape, neg, {}, 0.f, &o);
  set(r, "Out", o);
}

void k_crop_grad(const OpRun& r) {
  Tensor& x = r.in("X");
  Tensor& g = r.in("Out@GRAD");
  if (r.op.Outputs("X@GRAD").empty() || !r.out_var("X@GRAD")) return;
  auto off = r.op.GetInts("offsets");
  if (off.empty()) off.assign(x.dims.size(), 0);
  Tensor o;
  remap(r, g, x.dims, off, {}, 0.f, &o);
  set(r, "X@GRAD", o);
}

// ---------------------------------------------------------------- norm (L2 along an axis)
struct NormFwd {
  const float* x;
  float *o, *n;
  int64_t A, inner;
  float eps;
  __host__ __device__ void operator()(int64_t t) const {  // t = outer * inner + j
    const int64_t a0 = (t / inner) * A * inner + t % inner;
    float s = 0.f;
    for (int64_t k = 0; k < A; ++k) s += x[a0 + k * inner] * x[a0 + k * inner];
    const float nv = sqrtf(s + eps);
    n[t] = nv;
    for (int64_t k = 0; k < A; ++k) o[a0 + k * inner] = x[a0 + k * inner] / nv;
  }
};
struct NormBwd {
  const float *x, *n, *g;
  float* dx;
  int64_t A, inner;
  __host__ __device__ void operator()(int64_t t) const {
    const int64_t a0 = (t / inner) * A * inner + t % inner;
    const float nv = n[t];
    float dot = 0.f;
    for (int64_t k = 0; k < A; ++k) dot += g[a0 + k * inner] * x[a0 + k * inner];
    for (int64_t k = 0; k < A; ++k) {
      const float xv = x[a0 + k * inner];
      dx[a0 + k * inner] = g[a0 + k * inner] / nv - xv * dot / (nv * nv * nv);
    }
  }
};

void norm_geom(const Tensor& x, int64_t ax, int64_t* outer, int64_t* A, int64_t* inner) {
  const int nd = (int)x.dims.size();
  if (ax < 0) ax += nd;
  if (ax < 0 || ax >= nd) throw Decline{};
  *outer = 1;
  *inner = 1;
  for (int k = 0; k < ax; ++k) *outer *= x.dims[k];
  for (int k = (int)ax + 1; k < nd; ++k) *inner *= x.dims[k];
  *A = x.dims[ax];
}

void k_norm(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  int64_t outer, A, inner;
  norm_geom(x, r.op.GetInt("axis", 1), &outer, &A, &inner);
  Tensor o, n;
  Dims nd = x.dims;
  int64_t ax = r.op.GetInt("axis", 1);
  if (ax < 0) ax += (int64_t)nd.size();
  nd[ax] = 1;
  float* np_ = n.alloc<float>(nd, place_of(r));
  any::run(r, dev, outer * inner, NormFwd{f32(x, dev), new_like(r, x, &o), np_, A, inner, r.op.GetFloat("epsilon", 1e-10f)});
  set(r, "Out", o);
  set(r, "Norm", n);
}

void k_norm_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  int64_t outer, A, inner;
  norm_geom(x, r.op.GetInt("axis", 1), &outer, &A, &inner);
  Tensor d;
  float* dx = grad_out(r, "X@GRAD", x, &d);
  if (!dx) return;
  any::run(r, dev, outer * inner, NormBwd{f32(x, dev), f32(r.in("Norm"), dev), f32(r.in("Out@GRAD"), dev), dx, A, inner});
  set(r, "X@GRAD", d);
}

// ---------------------------------------------------------------- conv_shift (circular)
struct ConvShift {
  const float *x, *y;
  float* o;
  int64_t M, N;
  __host__ __device__ void operator()(int64_t t) const {
    const int64_t b = t / M, i = t % M, half = (N - 1) / 2;
    float s = 0.f;
    for (int64_t j = 0; j < N; ++j) s += x[b * M + ((i + j - half) % M + M) % M] * y[b * N + j];
    o[t] = s;
  }
};
struct ConvShiftGradX {
  const float *y, *g;
  float* dx;
  int64_t M, N;
  __host__ __device__ void operator()(int64_t t) const {
    const int64_t b = t / M, m = t % M, half = (N - 1) / 2;
    float s = 0.f;
    for (int64_t j = 0; j < N; ++j) s += g[b * M + ((m - j + half) % M + M) % M] * y[b * N + j];
    dx[t] = s;
  }
};
struct ConvShiftGradY {
  const float *x, *g;
  float* dy;
  int64_t M, N;
  __host__ __device__ void operator()(int64_t t) const {
    const int64_t b = t / N, j = t % N, half = (N - 1) / 2;
    float s = 0.f;
    for (int64_t i = 0; i < M; ++i) s += g[b * M + i] * x[b * M + ((i + j - half) % M + M) % M];
    dy[t] = s;
  }
};

void k_conv_shift(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  Tensor& y = r.in("Y");
  if (x.dims.size() != 2 || y.dims.size() != 2 || x.dims[0] != y.dims[0]) throw Decline{};
  Tensor o;
  any::run(r, dev, x.numel(), ConvShift{f32(x, dev), f32(y, dev), new_like(r, x, &o), x.dims[1], y.dims[1]});
  set(r, "Out", o);
}

void k_conv_shift_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  Tensor& y = r.in("Y");
  const float* g = f32(r.in("Out@GRAD"), dev);
  Tensor dX, dY;
  if (float* dx = grad_out(r, "X@GRAD", x, &dX)) {
    any::run(r, dev, x.numel(), ConvShiftGradX{f32(y, dev), g, dx, x.dims[1], y.dims[1]});
    set(r, "X@GRAD", dX);
  }
  if (float* dy = grad_out(r, "Y@GRAD", y, &dY)) {
    any::run(r, dev, y.numel(), ConvShiftGradY{f32(x, dev), g, dy, x.dims[1], y.dims[1]});
    set(r, "Y@GRAD", dY);
  }
}

// ---------------------------------------------------------------- bilinear_tensor_product
// out[b, k] = x_b^T W_k y_b (+ bias[k])
struct Btp {
  const float *x, *y, *w, *bias;
  float* o;
  int64_t K, I, J;
  __host__ __device__ void operator()(int64_t t) const {
    const int64_t b = t / K, k = t % K;
    float s = bias ? bias[k] : 0.f;
    for (int64_t i = 0; i < I; ++i) {
      float t2 = 0.f;
      for (int64_t j = 0; j < J; ++j) t2 += w[(k * I + i) * J + j] * y[b * J + j];
      s += x[b * I + i] * t2;
    }
    o[t] = s;
  }
};
struct BtpGradX {
  const float *y, *w, *g;
  float* dx;
  int64_t K, I, J;
  __host__ __device__ void operator()(int64_t t) const {
    const int64_t b = t / I, i = t % I;
    float s = 0.f;
    for (int64_t k = 0; k < K; ++k) {
      float t2 = 0.f;
      for (int64_t j = 0; j < J; ++j) t2 += w[(k * I + i) * J + j] * y[b * J + j];
      s += g[b * K + k] * t2;
    }
    dx[t] = s;
  }
};
struct BtpGradY {
  const float *x, *w, *g;
  float* dy;
  int64_t K, I, J;
  __host__ __device__ void operator()(int64_t t) const {
    const int64_t b = t / J, j = t % J;
    float s = 0.f;
    for (int64_t k = 0; k < K; ++k) {
      float t2 = 0.f;
      for (int64_t i = 0; i < I; ++i) t2 += x[b * I + i] * w[(k * I + i) * J + j];
      s += g[b * K + k] * t2;
    }
    dy[t] = s;
  }
};
struct BtpGradW {
  const float *x, *y, *g;
  float* dw;
  int64_t B, K, I, J;
  __host__ __device__ void operator()(int64_t t) const {
    const int64_t k = t / (I * J), i = (t / J) % I, j = t % J;
    float s = 0.f;
    for (int64_t b = 0; b < B; ++b) s += g[b * K + k] * x[b * I + i] * y[b * J + j];
    dw[t] = s;
  }
};

void k_btp(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  Tensor& y = r.in("Y");
  Tensor& w = r.in("Weight");
  Tensor* bias = r.in_opt("Bias");
  if (x.dims.size() != 2 || y.dims.size() != 2 || w.dims.size() != 3) throw Decline{};
  const int64_t B = x.dims[0], K = w.dims[0], I = w.dims[1], J = w.dims[2];
  if (x.dims[1] != I || y.dims[1] != J || y.dims[0] != B) throw Decline{};
  Tensor o;
  float* op = o.alloc<float>({B, K}, place_of(r));
  any::run(r, dev, B * K, Btp{f32(x, dev), f32(y, dev), f32(w, dev), bias ? f32(*bias, dev) : nullptr, op, K, I, J});
  set(r, "Out", o);
}

void k_btp_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  Tensor& y = r.in("Y");
  Tensor& w = r.in("Weight");
  const int64_t B = x.dims[0], K = w.dims[0], I = w.dims[1], J = w.dims[2];
  const float *xp = f32(x, dev), *yp = f32(y, dev), *wp = f32(w, dev), *g = f32(r.in("Out@GRAD"), dev);
  Tensor dX, dY, dW, dB;
  if (float* p = grad_out(r, "X@GRAD", x, &dX)) {
    any::run(r, dev, B * I, BtpGradX{yp, wp, g, p, K, I, J});
    set(r, "X@GRAD", dX);
  }
  if (float* p = grad_out(r, "Y@GRAD", y, &dY)) {
    any::run(r, dev, B * J, BtpGradY{xp, wp, g, p, K, I, J});
    set(r, "Y@GRAD", dY);
  }
  if (float* p = grad_out(r, "Weight@GRAD", w, &dW)) {
    any::run(r, dev, K * I * J, BtpGradW{xp, yp, g, p, B, K, I, J});
    set(r, "Weight@GRAD", dW);
  }
  if (Tensor* bt = r.in_opt("Bias")) {
    if (float* p = grad_out(r, "Bias@GRAD", *bt, &dB)) {
      any::run(r, dev, K, any::ColSum{g, p, B, K, 0});
      set(r, "Bias@GRAD", dB);
    }
  }
}

// ---------------------------------------------------------------- maxout
struct Maxout {
  const float* x;
  float* o;
  int64_t Co, G, HW;
  __host__ __device__ void operator()(int64_t t) const {  // t over [N, Co, HW]
    const int64_t n = t / (Co * HW), c = (t / HW) % Co, s = t % HW;
    const float* p = x + ((n * Co + c) * G) * HW + s;
    float m = p[0];
    for (int64_t k = 1; k < G; ++k) m = fmaxf(m, p[k * HW]);
    o[t] = m;
  }
};
struct MaxoutGrad {
  const float *x, *o, *g;
  float* dx;
  int64_t Co, G, HW;
  __host__ __device__ void operator()(int64_t t) const {
    const int64_t n = t / (Co * HW), c = (t / HW) % Co, s = t % HW;
    const int64_t base = ((n * Co + c) * G) * HW + s;
    bool done = false;  // the gradient goes to the first maximal element
    for (int64_t k = 0; k < G; ++k) {
      const bool hit = !done && x[base + k * HW] == o[t];
      dx[base + k * HW] = hit ? g[t] : 0.f;
      done = done || hit;
    }
  }
};

void k_maxout(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  const int64_t G = r.op.GetInt("groups", 1);
  if (x.dims.size() != 4 || G <= 0 || x.dims[1] % G) throw Decline{};
  const int64_t N = x.dims[0], Co = x.dims[1] / G, HW = x.dims[2] * x.dims[3];
  Tensor o;
  float* op = o.alloc<float>({N, Co, x.dims[2], x.dims[3]}, place_of(r));
  any::run(r, dev, N * Co * HW, Maxout{f32(x, dev), op, Co, G, HW});
  set(r, "Out", o);
}

void k_maxout_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  const int64_t G = r.op.GetInt("groups", 1);
  if (x.dims.size() != 4 || G <= 0 || x.dims[1] % G) throw Decline{};
  const int64_t N = x.dims[0], Co = x.dims[1] / G, HW = x.dims[2] * x.dims[3];
  Tensor d;
  float* dx = grad_out(r, "X@GRAD", x, &d);
  if (!dx) return;
  any::run(r, dev, N * Co * HW, MaxoutGrad{f32(x, dev), f32(r.in("Out"), dev), f32(r.in("Out@GRAD"), dev), dx, Co, G, HW});
  set(r, "X@GRAD", d);
}

// ---------------------------------------------------------------- fake (de)quantisation
struct AbsMaxChunk {
  const float* x;
  float* part;
  int64_t n, chunk;
  __host__ __device__ void operator()(int64_t c) const {
    float m = 0.f;
    const int64_t a = c * chunk, b = a + chunk < n ? a + chunk : n;
    for (int64_t i = a; i < b; ++i) m = fmaxf(m, fabsf(x[i]));
    part[c] = m;
  }
};
struct MaxOf {
  const float* part;
  float* out;
  int64_t nc;
  __host__ __device__ void operator()(int64_t) const {
    float m = 0.f;
    for (int64_t c = 0; c < nc; ++c) m = fmaxf(m, part[c]);
    out[0] = m;
  }
};
struct Quant {
  const float *x, *s;
  float* o;
  float bins;
  __host__ __device__ void operator()(int64_t i) const { o[i] = rintf(x[i] / fmaxf(s[0], 1e-30f) * bins); }
};

void k_fake_quant_abs_max(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  const int64_t n = x.numel(), chunk = 4096, nc = (n + chunk - 1) / chunk;
  std::vector<float> hp;
  float* part = any::scratch(r, dev, "@fq_part@", nc, &hp);
  Tensor sc, o;
  float* sp = sc.alloc<float>({1}, place_of(r));
  any::run(r, dev, nc, AbsMaxChunk{f32(x, dev), part, n, chunk});
  any::run(r, dev, 1, MaxOf{part, sp, nc});
  const float bins = (float)((1 << (r.op.GetInt("bit_length", 8) - 1)) - 1);
  any::run(r, dev, n, Quant{f32(x, dev), sp, new_like(r, x, &o), bins});
  set(r, "Out", o);
  set(r, "OutScale", sc);
}

struct Dequant {
  const float *x, *s;
  float* o;
  float inv;
  __host__ __device__ void operator()(int64_t i) const { o[i] = x[i] * s[0] * inv; }
};
struct DequantGradScale {
  const float *x, *g;
  float* ds;
  int64_t n;
  float inv;
  __host__ __device__ void operator()(int64_t) const {
    float s = 0.f;
    for (int64_t i = 0; i < n; ++i) s += g[i] * x[i];
    ds[0] = s * inv;
  }
};

void k_fake_dequant(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  Tensor o;
  any::run(r, dev, x.numel(), Dequant{f32(x, dev), f32(r.in("Scale"), dev), new_like(r, x, &o),
                                      1.f / r.op.GetFloat("max_range", 127.f)});
  set(r, "Out", o);
}

void k_fake_dequant_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  const float inv = 1.f / r.op.GetFloat("max_range", 127.f);
  const float* g = f32(r.in("Out@GRAD"), dev);
  Tensor dX, dS;
  if (float* p = grad_out(r, "X@GRAD", x, &dX)) {
    any::run(r, dev, x.numel(), Dequant{g, f32(r.in("Scale"), dev), p, inv});
    set(r, "X@GRAD", dX);
  }
  if (float* p = grad_out(r, "Scale@GRAD", r.in("Scale"), &dS)) {
    any::run(r, dev, 1, DequantGradScale{f32(x, dev), g, p, x.numel(), inv});
    set(r, "Scale@GRAD", dS);
  }
}

// ---------------------------------------------------------------- identity-like grads
void copy_out(const OpRun& r, const Tensor& src, const char* slot, const LoD& lod) {
  const bool dev = on_dev(r);
  Tensor o;
  any::copy(r, dev, o.alloc<float>(src.dims, place_of(r)), f32(src, dev), src.numel());
  o.lod = lod;
  set(r, slot, o);
}

// rnn_memory_helper: Out shares X (StaticRNN memories); its gradient passes through
void k_rnn_memory_helper(const OpRun& r) { *r.out("Out") = r.in("X"); }

void k_rnn_memory_helper_grad(const OpRun& r) {
  if (r.op.Outputs("X@GRAD").empty() || !r.out_var("X@GRAD")) return;
  Tensor& x = r.in("X");
  if (Tensor* g = r.in_opt("Out@GRAD")) {
    copy_out(r, *g, "X@GRAD", x.lod);
  } else {
    Tensor z;
    any::zero(r, on_dev(r), new_like(r, x, &z), x.numel());
    set(r, "X@GRAD", z);
  }
}

// lod_reset's gradient: Out@GRAD with X's LoD
void k_lod_reset_grad(const OpRun& r) {
  if (r.op.Outputs("X@GRAD").empty() || !r.out_var("X@GRAD")) return;
  copy_out(r, r.in("Out@GRAD"), "X@GRAD", r.in("X").lod);
}

// scatter's gradient: dX = g (rows written by an overwriting scatter zeroed), dUpdates = g[ids]
struct RowGather {
  const float* g;
  const int64_t* ids;
  float* o;
  int64_t D;
  __host__ __device__ void operator()(int64_t t) const { o[t] = g[ids[t / D] * D + t % D]; }
};
struct RowZero {
  const int64_t* ids;
  float* o;
  int64_t D;
  __host__ __device__ void operator()(int64_t t) const { o[ids[t / D] * D + t % D] = 0.f; }
};

void k_scatter_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& ids = r.in("Ids");
  Tensor& g = r.in("Out@GRAD");
  if (ids.dtype != DT::INT64 || (ids.device >= 0) != dev || g.dims.empty()) throw Decline{};
  const int64_t D = g.numel() / g.dims[0], n = ids.numel();
  Tensor dX, dU;
  if (float* p = grad_out(r, "X@GRAD", r.in("X"), &dX)) {
    any::copy(r, dev, p, f32(g, dev), g.numel());
    if (r.op.GetBool("overwrite", true)) any::run(r, dev, n * D, RowZero{ids.data<int64_t>(), p, D});
    set(r, "X@GRAD", dX);
  }
  if (float* p = grad_out(r, "Updates@GRAD", r.in("Updates"), &dU)) {
    any::run(r, dev, n * D, RowGather{f32(g, dev), ids.data<int64_t>(), p, D});
    set(r, "Updates@GRAD", dU);
  }
}

// ---------------------------------------------------------------- polygon_box_transform
struct PolyBox {
  const float* x;
  float* o;
  int64_t C, H, W;
  __host__ __device__ void operator()(int64_t t) const {
    const int64_t w = t % W, h = (t / W) % H, c = (t / (W * H)) % C;
    o[t] = (c % 2 == 0 ? (float)w : (float)h) - x[t];
  }
};

void k_polygon_box(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("Input");
  if (x.dims.size() != 4) throw Decline{};
  Tensor o;
  any::run(r, dev, x.numel(), PolyBox{f32(x, dev), new_like(r, x, &o), x.dims[1], x.dims[2], x.dims[3]});
  set(r, "Output", o);
}

// ---------------------------------------------------------------- argsort
// ascending along `axis`, one lane per line: stable insertion sort of (value, index)
struct ArgSort {
  const float* x;
  float* v;
  int64_t* idx;
  int64_t n, inner;
  __host__ __device__ void operator()(int64_t t) const {
    const int64_t base = (t / inner) * n * inner + t % inner;
    for (int64_t k = 0; k < n; ++k) {
      const float xv = x[base + k * inner];
      int64_t j = k;
      while (j > 0 && v[base + (j - 1) * inner] > xv) {
        v[base + j * inner] = v[base + (j - 1) * inner];
        idx[base + j * inner] = idx[base + (j - 1) * inner];
        --j;
      }
      v[base + j * inner] = xv;
      idx[base + j * inner] = k;
    }
  }
};

void k_argsort(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  const int nd = (int)x.dims.size();
  int64_t ax = r.op.GetInt("axis", -1);
  if (ax < 0) ax += nd;
  if (nd == 0 || ax < 0 || ax >= nd) throw Decline{};
  int64_t outer = 1, inner = 1;
  for (int k = 0; k < ax; ++k) outer *= x.dims[k];
  for (int k = (int)ax + 1; k < nd; ++k) inner *= x.dims[k];
  Tensor v, i;
  float* vp = new_like(r, x, &v);
  int64_t* ip = static_cast<int64_t*>(i.alloc(DT::INT64, x.dims, place_of(r)));
  any::run(r, dev, outer * inner, ArgSort{f32(x, dev), vp, ip, x.dims[ax], inner});
  set(r, "Out", v);
  set(r, "Indices", i);
}

// ---------------------------------------------------------------- row_conv (lookahead)
// out[t] = sum_{k < ctx, t + k in t's sequence} x[t + k] * w[k]   (elementwise per feature)
struct RowConv {
  const float *x, *w;
  const int* seq_end;  // end row of each row's sequence
  float* o;
  int64_t D, ctx;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t t = i / D, d = i % D, e = seq_end[t];
    float s = 0.f;
    for (int64_t k = 0; k < ctx && t + k < e; ++k) s += x[(t + k) * D + d] * w[k * D + d];
    o[i] = s;
  }
};
struct RowConvGradX {
  const float *g, *w;
  const int* seq_start;
  float* dx;
  int64_t D, ctx;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t t = i / D, d = i % D, st = seq_start[t];
    float s = 0.f;
    for (int64_t k = 0; k < ctx && t - k >= st; ++k) s += g[(t - k) * D + d] * w[k * D + d];
    dx[i] = s;
  }
};
struct RowConvGradW {
  const float *g, *x;
  const int* seq_end;
  float* dw;
  int64_t T, D;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t k = i / D, d = i % D;
    float s = 0.f;
    for (int64_t t = 0; t < T; ++t)
      if (t + k < seq_end[t]) s += g[t * D + d] * x[(t + k) * D + d];
    dw[i] = s;
  }
};

void row_bounds(const Tensor& x, std::vector<int>* st, std::vector<int>* en) {
  const int64_t T = x.dims[0];
  std::vector<size_t> off = x.lod.empty() ? std::vector<size_t>{0, (size_t)T} : x.lod[0];
  st->assign((size_t)T, 0);
  en->assign((size_t)T, 0);
  for (size_t s = 0; s + 1 < off.size(); ++s)
    for (size_t t = off[s]; t < off[s + 1] && (int64_t)t < T; ++t) {
      (*st)[t] = (int)off[s];
      (*en)[t] = (int)off[s + 1];
    }
}

void k_row_conv(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  Tensor& w = r.in("Filter");
  if (x.dims.size() != 2 || w.dims.size() != 2 || w.dims[1] != x.dims[1]) throw Decline{};
  std::vector<int> st, en;
  row_bounds(x, &st, &en);
  Tensor o;
  any::run(r, dev, x.numel(),
           RowConv{f32(x, dev), f32(w, dev), any::ints(r, dev, "@rowconv_end@", en), new_like(r, x, &o), x.dims[1],
                   w.dims[0]});
  set(r, "Out", o);
}

void k_row_conv_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  Tensor& w = r.in("Filter");
  const float* g = f32(r.in("Out@GRAD"), dev);
  std::vector<int> st, en;
  row_bounds(x, &st, &en);
  Tensor dX, dW;
  if (float* p = grad_out(r, "X@GRAD", x, &dX)) {
    any::run(r, dev, x.numel(),
             RowConvGradX{g, f32(w, dev), any::ints(r, dev, "@rowconv_start@", st), p, x.dims[1], w.dims[0]});
    set(r, "X@GRAD", dX);
  }
  if (float* p = grad_out(r, "Filter@GRAD", w, &dW)) {
    any::run(r, dev, w.numel(),
             RowConvGradW{g, f32(x, dev), any::ints(r, dev, "@rowconv_end2@", en), p, x.dims[0], x.dims[1]});
    set(r, "Filter@GRAD", dW);
  }
}

// ---------------------------------------------------------------- lrn (across channels)
// mid = k + alpha * sum_{c' in [c - (n-1)/2, c + n/2]} x_c'^2, out = x mid^-beta
struct Lrn {
  const float* x;
  float *o, *mid;
  int64_t C, HW, n;
  float k, alpha, beta;
  __host__ __device__ void operator()(int64_t t) const {
    const int64_t c = (t / HW) % C, base = t - c * HW;
    float s = 0.f;
    for (int64_t q = c - (n - 1) / 2; q <= c + n / 2; ++q)
      if (q >= 0 && q < C) s += x[base + q * HW] * x[base + q * HW];
    const float m = k + alpha * s;
    mid[t] = m;
    o[t] = x[t] * powf(m, -beta);
  }
};
// dx_c = g_c mid_c^-b - 2 a b x_c sum_{c': c in window(c')} g_c' out_c' / mid_c'
struct LrnGrad {
  const float *x, *o, *mid, *g;
  float* dx;
  int64_t C, HW, n;
  float alpha, beta;
  __host__ __device__ void operator()(int64_t t) const {
    const int64_t c = (t / HW) % C, base = t - c * HW;
    float s = 0.f;
    for (int64_t q = c - n / 2; q <= c + (n - 1) / 2; ++q)
      if (q >= 0 && q < C) s += g[base + q * HW] * o[base + q * HW] / mid[base + q * HW];
    dx[t] = g[t] * powf(mid[t], -beta) - 2.f * alpha * beta * x[t] * s;
  }
};

void k_lrn(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  if (x.dims.size() != 4) throw Decline{};
  Tensor o, m;
  any::run(r, dev, x.numel(),
           Lrn{f32(x, dev), new_like(r, x, &o), new_like(r, x, &m), x.dims[1], x.dims[2] * x.dims[3],
               r.op.GetInt("n", 5), r.op.GetFloat("k", 2.f), r.op.GetFloat("alpha", 1e-4f), r.op.GetFloat("beta", 0.75f)});
  set(r, "Out", o);
  set(r, "MidOut", m);
}

void k_lrn_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  if (x.dims.size() != 4) throw Decline{};
  Tensor d;
  float* dx = grad_out(r, "X@GRAD", x, &d);
  if (!dx) return;
  any::run(r, dev, x.numel(),
           LrnGrad{f32(x, dev), f32(r.in("Out"), dev), f32(r.in("MidOut"), dev), f32(r.in("Out@GRAD"), dev), dx,
                   x.dims[1], x.dims[2] * x.dims[3], r.op.GetInt("n", 5), r.op.GetFloat("alpha", 1e-4f),
                   r.op.GetFloat("beta", 0.75f)});
  set(r, "X@GRAD", d);
}

// ---------------------------------------------------------------- IfElse row routing
// split_lod_tensor: the rows of X where Mask holds / does not, in order; the row maps
// are built on the host from the (small) mask
std::vector<uint8_t> host_mask(const OpRun& r, const Tensor& m) {
  std::vector<uint8_t> h((size_t)m.numel());
  Tensor hm = m.device >= 0 ? m.to(-1, r.ctx.stream) : m;
  if (m.device >= 0) device_stream_sync(r.ctx.stream);
  for (int64_t i = 0; i < m.numel(); ++i) {
    switch (hm.dtype) {
      case DT::BOOL: case DT::UINT8: case DT::INT8: h[i] = hm.data<uint8_t>()[i] != 0; break;
      case DT::INT32: h[i] = hm.data<int32_t>()[i] != 0; break;
      case DT::INT64: h[i] = hm.data<int64_t>()[i] != 0; break;
      case DT::FP32: h[i] = hm.data<float>()[i] != 0.f; break;
      default: throw Decline{};
    }
  }
  return h;
}

struct RowCopy {  // dst row k = src row rows[k]
  const float* src;
  const int* rows;
  float* dst;
  int64_t D;
  __host__ __device__ void operator()(int64_t t) const { dst[t] = src[(int64_t)rows[t / D] * D + t % D]; }
};
struct RowPut {  // dst row rows[k] = src row k
  const float* src;
  const int* rows;
  float* dst;
  int64_t D;
  __host__ __device__ void operator()(int64_t t) const { dst[(int64_t)rows[t / D] * D + t % D] = src[t]; }
};

void k_split_lod_tensor(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  const auto m = host_mask(r, r.in("Mask"));
  if (x.dims.empty() || (int64_t)m.size() != x.dims[0]) throw Decline{};
  const int64_t D = x.numel() / x.dims[0];
  std::vector<int> tr, fl;
  for (size_t i = 0; i < m.size(); ++i) (m[i] ? tr : fl).push_back((int)i);
  for (int side = 0; side < 2; ++side) {
    const auto& rows = side ? fl : tr;
    Dims d = x.dims;
    d[0] = (int64_t)rows.size();
    Tensor o;
    float* op = o.alloc<float>(d, place_of(r));
    any::run(r, dev, (int64_t)rows.size() * D,
             RowCopy{f32(x, dev), any::ints(r, dev, side ? "@split_f@" : "@split_t@", rows), op, D});
    set(r, side ? "OutFalse" : "OutTrue", o);
  }
}

void k_merge_lod_tensor(const OpRun& r) {
  const bool dev = on_dev(r);
  const auto m = host_mask(r, r.in("Mask"));
  Tensor* t = r.in_opt("InTrue");
  Tensor* f = r.in_opt("InFalse");
  const Tensor* ref = t && t->numel() ? t : f;
  if (!ref || ref->dims.empty()) throw Decline{};
  const int64_t D = ref->numel() / ref->dims[0];
  std::vector<int> tr, fl;
  for (size_t i = 0; i < m.size(); ++i) (m[i] ? tr : fl).push_back((int)i);
  Dims d = ref->dims;
  d[0] = (int64_t)m.size();
  Tensor o;
  float* op = o.alloc<float>(d, place_of(r));
  any::zero(r, dev, op, o.numel());
  if (t && t->numel()) {
    if (t->dims[0] != (int64_t)tr.size()) throw Decline{};
    any::run(r, dev, (int64_t)tr.size() * D, RowPut{f32(*t, dev), any::ints(r, dev, "@merge_t@", tr), op, D});
  }
  if (f && f->numel()) {
    if (f->dims[0] != (int64_t)fl.size()) throw Decline{};
    any::run(r, dev, (int64_t)fl.size() * D, RowPut{f32(*f, dev), any::ints(r, dev, "@merge_f@", fl), op, D});
  }
  set(r, "Out", o);
}

// their gradients: split's is the merge of the two branch gradients (a missing one
// contributes zeros), merge's the split of Out@GRAD (X only gives the row count)
void k_split_lod_tensor_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  const auto m = host_mask(r, r.in("Mask"));
  Tensor d;
  float* dx = grad_out(r, "X@GRAD", x, &d);
  if (!dx) return;
  if (x.dims.empty() || (int64_t)m.size() != x.dims[0]) throw Decline{};
  const int64_t D = x.numel() / x.dims[0];
  any::zero(r, dev, dx, x.numel());
  std::vector<int> tr, fl;
  for (size_t i = 0; i < m.size(); ++i) (m[i] ? tr : fl).push_back((int)i);
  Tensor* gt = r.in_opt("OutTrue@GRAD");
  Tensor* gf = r.in_opt("OutFalse@GRAD");
  if (gt && gt->numel() && !tr.empty())
    any::run(r, dev, (int64_t)tr.size() * D, RowPut{f32(*gt, dev), any::ints(r, dev, "@splitg_t@", tr), dx, D});
  if (gf && gf->numel() && !fl.empty())
    any::run(r, dev, (int64_t)fl.size() * D, RowPut{f32(*gf, dev), any::ints(r, dev, "@splitg_f@", fl), dx, D});
  d.lod = x.lod;
  set(r, "X@GRAD", d);
}

void k_merge_lod_tensor_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& g = r.in("Out@GRAD");
  const auto m = host_mask(r, r.in("Mask"));
  if (g.dims.empty() || (int64_t)m.size() != g.dims[0]) throw Decline{};
  const int64_t D = g.numel() / g.dims[0];
  std::vector<int> tr, fl;
  for (size_t i = 0; i < m.size(); ++i) (m[i] ? tr : fl).push_back((int)i);
  for (int side = 0; side < 2; ++side) {
    const char* slot = side ? "InFalse@GRAD" : "InTrue@GRAD";
    if (r.op.Outputs(slot).empty() || !r.out_var(slot)) continue;
    const auto& rows = side ? fl : tr;
    Dims dd = g.dims;
    dd[0] = (int64_t)rows.size();
    Tensor o;
    float* op = o.alloc<float>(dd, place_of(r));
    any::run(r, dev, (int64_t)rows.size() * D, RowCopy{f32(g, dev), any::ints(r, dev, side ? "@mergeg_f@" : "@mergeg_t@", rows), op, D});
    set(r, slot, o);
  }
  Tensor dx;
  if (float* p = grad_out(r, "X@GRAD", r.in("X"), &dx)) {
    any::zero(r, dev, p, dx.numel());
    set(r, "X@GRAD", dx);
  }
}

// ---------------------------------------------------------------- max_pool2d_with_index / unpool
struct MaxPoolIdx {
  const float* x;
  float* o;
  int32_t* mask;
  int64_t H, W, OH, OW, kh, kw, sh, sw, ph, pw;
  __host__ __device__ void operator()(int64_t t) const {
    const int64_t ow = t % OW, oh = (t / OW) % OH, plane = t / (OW * OH);
    const float* p = x + plane * H * W;
    float best = -INFINITY;
    int64_t bi = -1;
    for (int64_t i = 0; i < kh; ++i)
      for (int64_t j = 0; j < kw; ++j) {
        const int64_t h = oh * sh - ph + i, w = ow * sw - pw + j;
        if (h < 0 || h >= H || w < 0 || w >= W) continue;
        const float v = p[h * W + w];
        if (bi < 0 || v > best) {
          best = v;
          bi = h * W + w;
        }
      }
    o[t] = best;
    mask[t] = (int32_t)bi;
  }
};
// scatter-add of the pooled gradient to the recorded positions (windows may overlap)
struct MaxPoolIdxGrad {
  const float* g;
  const int32_t* mask;
  float* dx;
  int64_t HW, OHW;
  __host__ __device__ void operator()(int64_t t) const {
    const int64_t plane = t / OHW;
    if (mask[t] >= 0) acc_add(dx + plane * HW + mask[t], g[t]);
  }
};

void pool_attrs(const OpRun& r, const Tensor& x, int64_t* kh, int64_t* kw, int64_t* sh, int64_t* sw, int64_t* ph,
                int64_t* pw) {
  auto k = r.op.GetInts("ksize"), st = r.op.GetInts("strides"), pd = r.op.GetInts("paddings");
  if (k.size() != 2 || st.size() != 2 || pd.size() != 2 || x.dims.size() != 4) throw Decline{};
  *kh = k[0], *kw = k[1], *sh = st[0], *sw = st[1], *ph = pd[0], *pw = pd[1];
  if (r.op.GetBool("global_pooling", false)) {
    *kh = x.dims[2], *kw = x.dims[3], *ph = 0, *pw = 0;
  }
}

void k_max_pool2d_idx(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  int64_t kh, kw, sh, sw, ph, pw;
  pool_attrs(r, x, &kh, &kw, &sh, &sw, &ph, &pw);
  const int64_t H = x.dims[2], W = x.dims[3], OH = (H + 2 * ph - kh) / sh + 1, OW = (W + 2 * pw - kw) / sw + 1;
  Tensor o, m;
  float* op = o.alloc<float>({x.dims[0], x.dims[1], OH, OW}, place_of(r));
  int32_t* mp = static_cast<int32_t*>(m.alloc(DT::INT32, {x.dims[0], x.dims[1], OH, OW}, place_of(r)));
  any::run(r, dev, o.numel(), MaxPoolIdx{f32(x, dev), op, mp, H, W, OH, OW, kh, kw, sh, sw, ph, pw});
  set(r, "Out", o);
  set(r, "Mask", m);
}

void k_max_pool2d_idx_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  Tensor& m = r.in("Mask");
  Tensor& g = r.in("Out@GRAD");
  if (m.dtype != DT::INT32 || (m.device >= 0) != dev) throw Decline{};
  Tensor d;
  float* dx = grad_out(r, "X@GRAD", x, &d);
  if (!dx) return;
  any::zero(r, dev, dx, x.numel());
  any::run(r, dev, g.numel(),
           MaxPoolIdxGrad{f32(g, dev), m.data<int32_t>(), dx, x.dims[2] * x.dims[3], g.dims[2] * g.dims[3]}, 1 << 30);
  set(r, "X@GRAD", d);
}

struct Unpool {
  const float* x;
  const int32_t* idx;
  float* o;
  int64_t HW, OHW;
  __host__ __device__ void operator()(int64_t t) const { o[(t / HW) * OHW + idx[t]] = x[t]; }
};
struct UnpoolGrad {
  const float* g;
  const int32_t* idx;
  float* dx;
  int64_t HW, OHW;
  __host__ __device__ void operator()(int64_t t) const { dx[t] = g[(t / HW) * OHW + idx[t]]; }
};

void unpool_geom(const OpRun& r, const Tensor& x, int64_t* OH, int64_t* OW) {
  auto k = r.op.GetInts("ksize"), st = r.op.GetInts("strides"), pd = r.op.GetInts("paddings");
  if (k.size() != 2 || st.size() != 2 || pd.size() != 2 || x.dims.size() != 4) throw Decline{};
  *OH = (x.dims[2] - 1) * st[0] - 2 * pd[0] + k[0];
  *OW = (x.dims[3] - 1) * st[1] - 2 * pd[1] + k[1];
}

void k_unpool(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  Tensor& idx = r.in("Indices");
  if (idx.dtype != DT::INT32 || (idx.device >= 0) != dev || idx.numel() != x.numel()) throw Decline{};
  int64_t OH, OW;
  unpool_geom(r, x, &OH, &OW);
  Tensor o;
  float* op = o.alloc<float>({x.dims[0], x.dims[1], OH, OW}, place_of(r));
  any::zero(r, dev, op, o.numel());
  any::run(r, dev, x.numel(), Unpool{f32(x, dev), idx.data<int32_t>(), op, x.dims[2] * x.dims[3], OH * OW});
  set(r, "Out", o);
}

void k_unpool_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  Tensor& idx = r.in("Indices");
  if (idx.dtype != DT::INT32 || (idx.device >= 0) != dev) throw Decline{};
  int64_t OH, OW;
  unpool_geom(r, x, &OH, &OW);
  Tensor d;
  float* dx = grad_out(r, "X@GRAD", x, &d);
  if (!dx) return;
  any::run(r, dev, x.numel(),
           UnpoolGrad{f32(r.in("Out@GRAD"), dev), idx.data<int32_t>(), dx, x.dims[2] * x.dims[3], OH * OW});
  set(r, "X@GRAD", d);
}

// ---------------------------------------------------------------- box_coder
struct BoxCoder {
  const float *prior, *var, *tgt;
  float* o;
  int64_t M, tgt3;
  int encode;
  float one;
  __host__ __device__ void operator()(int64_t t) const {  // t over [N, M]
    const int64_t n = t / M, m = t % M;
    const float* p = prior + m * 4;
    const float pw = p[2] - p[0] + one, ph = p[3] - p[1] + one;
    const float pcx = (p[0] + p[2]) / 2.f, pcy = (p[1] + p[3]) / 2.f;
    float* out = o + t * 4;
    if (encode) {
      const float* b = tgt + n * 4;
      const float tw = b[2] - b[0] + one, th = b[3] - b[1] + one;
      const float tcx = (b[0] + b[2]) / 2.f, tcy = (b[1] + b[3]) / 2.f;
      float v[4] = {(tcx - pcx) / pw, (tcy - pcy) / ph, logf(fabsf(tw / pw)), logf(fabsf(th / ph))};
      for (int k = 0; k < 4; ++k) out[k] = var ? v[k] / var[m * 4 + k] : v[k];
    } else {
      const float* d = tgt + (tgt3 ? t * 4 : n * 4);
      const float v0 = var ? var[m * 4] : 1.f, v1 = var ? var[m * 4 + 1] : 1.f;
      const float v2 = var ? var[m * 4 + 2] : 1.f, v3 = var ? var[m * 4 + 3] : 1.f;
      const float cx = v0 * d[0] * pw + pcx, cy = v1 * d[1] * ph + pcy;
      const float w = expf(v2 * d[2]) * pw, h = expf(v3 * d[3]) * ph;
      out[0] = cx - w / 2.f;
      out[1] = cy - h / 2.f;
      out[2] = cx + w / 2.f - one;
      out[3] = cy + h / 2.f - one;
    }
  }
};

void k_box_coder(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& prior = r.in("PriorBox");
  Tensor& tgt = r.in("TargetBox");
  Tensor* var = r.in_opt("PriorBoxVar");
  const std::string ct = r.op.GetString("code_type", "encode_center_size");
  const bool encode = ct.rfind("encode", 0) == 0 || ct.rfind("Encode", 0) == 0;
  if (prior.dims.size() != 2 || prior.dims[1] != 4 || tgt.dims.empty() || tgt.dims.back() != 4) throw Decline{};
  if (var && var->numel() != prior.numel()) throw Decline{};
  const int64_t M = prior.dims[0], N = tgt.dims[0];
  const bool t3 = tgt.dims.size() == 3;
  if (t3 && (encode || tgt.dims[1] != M)) throw Decline{};
  Tensor o;
  float* op = o.alloc<float>({N, M, 4}, place_of(r));
  o.lod = tgt.lod;
  any::run(r, dev, N * M,
           BoxCoder{f32(prior, dev), var ? f32(*var, dev) : nullptr, f32(tgt, dev), op, M, t3 ? 1 : 0, encode ? 1 : 0,
                    r.op.GetBool("box_normalized", true) ? 0.f : 1.f});
  set(r, "OutputBox", o);
}

// ---------------------------------------------------------------- mean_iou
__host__ __device__ inline void acc_add_i(int32_t* p, int32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  atomicAdd(p, v);
#else
  *p += v;
#endif
}
template <class T>
struct IouHist {
  const T *p, *l;
  int32_t *correct, *wrong;
  int64_t C;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t a = (int64_t)p[i], b = (int64_t)l[i];
    if (a == b) {
      if (b >= 0 && b < C) acc_add_i(correct + b, 1);
    } else {
      if (a >= 0 && a < C) acc_add_i(wrong + a, 1);
      if (b >= 0 && b < C) acc_add_i(wrong + b, 1);
    }
  }
};
struct IouAdd {
  const int32_t* in;
  int32_t* acc;
  __host__ __device__ void operator()(int64_t c) const { acc[c] += in[c]; }
};
struct IouMean {
  const int32_t *correct, *wrong;
  const float* const* extra;
  int64_t C, nextra;
  float* out;
  __host__ __device__ void operator()(int64_t) const {
    double s = 0.0;
    int64_t n = 0;
    for (int64_t c = 0; c < C; ++c) {
      const int64_t den = (int64_t)correct[c] + wrong[c];
      if (den > 0) {
        s += (double)correct[c] / (double)den;
        ++n;
      }
    }
    double m = n ? s / (double)n : 0.0;
    for (int64_t k = 0; k < nextra; ++k) m += (double)extra[k][0];
    out[0] = (float)m;
  }
};

void k_mean_iou(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& p = r.in("Predictions");
  Tensor& l = r.in("Labels");
  const int64_t C = r.op.GetInt("num_classes", 2);
  if (p.numel() != l.numel() || p.dtype != l.dtype || (p.device >= 0) != dev || (l.device >= 0) != dev) throw Decline{};
  Tensor co, wr, mi;
  int32_t* cp = static_cast<int32_t*>(co.alloc(DT::INT32, {C}, place_of(r)));
  int32_t* wp = static_cast<int32_t*>(wr.alloc(DT::INT32, {C}, place_of(r)));
  if (dev) {
    PA_HIPCHK(hipMemsetAsync(cp, 0, C * 4, dev_stream(r)));
    PA_HIPCHK(hipMemsetAsync(wp, 0, C * 4, dev_stream(r)));
  } else {
    memset(cp, 0, C * 4);
    memset(wp, 0, C * 4);
  }
  const int64_t serial = int64_t(1) << 60;  // host: one thread (plain increments)
  if (p.dtype == DT::INT32) any::run(r, dev, p.numel(), IouHist<int32_t>{p.data<int32_t>(), l.data<int32_t>(), cp, wp, C}, serial);
  else if (p.dtype == DT::INT64) any::run(r, dev, p.numel(), IouHist<int64_t>{p.data<int64_t>(), l.data<int64_t>(), cp, wp, C}, serial);
  else throw Decline{};
  for (Tensor* t : r.ins("InWrongs")) {
    if (t->dtype != DT::INT32 || t->numel() != C) throw Decline{};
    any::run(r, dev, C, IouAdd{t->data<int32_t>(), wp}, serial);
  }
  for (Tensor* t : r.ins("InCorrects")) {
    if (t->dtype != DT::INT32 || t->numel() != C) throw Decline{};
    any::run(r, dev, C, IouAdd{t->data<int32_t>(), cp}, serial);
  }
  std::vector<const float*> ex;
  for (Tensor* t : r.ins("InMeanIou")) ex.push_back(f32(*t, dev));
  std::vector<const float*> keep;
  const float* const* tab = ex.empty() ? nullptr : ptr_table(r, dev, "@miou_ptrs@", ex, &keep);
  float* mp = mi.alloc<float>({1}, place_of(r));
  any::run(r, dev, 1, IouMean{cp, wp, tab, C, (int64_t)ex.size(), mp});
  set(r, "OutMeanIou", mi);
  set(r, "OutWrong", wr);
  set(r, "OutCorrect", co);
}

// ---------------------------------------------------------------- bilinear / nearest interpolation
// torch conventions (what the Python kernel computes): align_corners: src = dst (in-1)/(out-1);
// else src = (dst + 0.5) in/out - 0.5 clamped at 0; nearest: src = floor(dst in/out)
struct Interp {
  const float* x;
  float* o;
  int64_t H, W, OH, OW;
  int bilinear, align;
  __host__ __device__ void coord(int64_t d, int64_t in, int64_t out, int64_t* i0, int64_t* i1, float* l) const {
    if (!bilinear) {
      int64_t s = (int64_t)floorf((float)d * (float)in / (float)out);
      *i0 = *i1 = s < in - 1 ? s : in - 1;
      *l = 0.f;
      return;
    }
    float src = align ? (out > 1 ? (float)d * (float)(in - 1) / (float)(out - 1) : 0.f)
                      : fmaxf(((float)d + 0.5f) * (float)in / (float)out - 0.5f, 0.f);
    int64_t a = (int64_t)floorf(src);
    if (a > in - 1) a = in - 1;
    *i0 = a;
    *i1 = a + 1 < in ? a + 1 : in - 1;
    *l = src - (float)a;
  }
  __host__ __device__ void operator()(int64_t t) const {
    const int64_t ow = t % OW, oh = (t / OW) % OH, plane = t / (OW * OH);
    int64_t y0, y1, x0, x1;
    float ly, lx;
    coord(oh, H, OH, &y0, &y1, &ly);
    coord(ow, W, OW, &x0, &x1, &lx);
    const float* p = x + plane * H * W;
    o[t] = (1.f - ly) * ((1.f - lx) * p[y0 * W + x0] + lx * p[y0 * W + x1]) +
           ly * ((1.f - lx) * p[y1 * W + x0] + lx * p[y1 * W + x1]);
  }
};
struct InterpGrad {
  Interp f;
  const float* g;
  float* dx;
  __host__ __device__ void operator()(int64_t t) const {
    const int64_t ow = t % f.OW, oh = (t / f.OW) % f.OH, plane = t / (f.OW * f.OH);
    int64_t y0, y1, x0, x1;
    float ly, lx;
    f.coord(oh, f.H, f.OH, &y0, &y1, &ly);
    f.coord(ow, f.W, f.OW, &x0, &x1, &lx);
    float* p = dx + plane * f.H * f.W;
    const float gv = g[t];
    acc_add(p + y0 * f.W + x0, gv * (1.f - ly) * (1.f - lx));
    acc_add(p + y0 * f.W + x1, gv * (1.f - ly) * lx);
    acc_add(p + y1 * f.W + x0, gv * ly * (1.f - lx));
    acc_add(p + y1 * f.W + x1, gv * ly * lx);
  }
};

Interp interp_of(const OpRun& r, const Tensor& x, int64_t* oh, int64_t* ow) {
  if (x.dims.size() != 4) throw Decline{};
  if (Tensor* os = r.in_opt("OutSize")) {
    Tensor h = os->device >= 0 ? os->to(-1, r.ctx.stream) : *os;
    if (os->device >= 0) device_stream_sync(r.ctx.stream);
    if (h.numel() != 2 || h.dtype != DT::INT32) throw Decline{};
    *oh = h.data<int32_t>()[0];
    *ow = h.data<int32_t>()[1];
  } else {
    *oh = r.op.GetInt("out_h", -1);
    *ow = r.op.GetInt("out_w", -1);
    const float sc = r.op.GetFloat("scale", 0.f);
    if ((*oh <= 0 || *ow <= 0) && sc > 0.f) {
      *oh = (int64_t)(x.dims[2] * sc);
      *ow = (int64_t)(x.dims[3] * sc);
    }
  }
  if (*oh <= 0 || *ow <= 0) throw Decline{};
  return Interp{nullptr, nullptr, x.dims[2], x.dims[3], *oh, *ow,
                r.op.GetString("interp_method", "bilinear") == "bilinear" ? 1 : 0,
                r.op.GetBool("align_corners", true) ? 1 : 0};
}

void k_interp(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  int64_t oh, ow;
  Interp f = interp_of(r, x, &oh, &ow);
  Tensor o;
  f.x = f32(x, dev);
  f.o = o.alloc<float>({x.dims[0], x.dims[1], oh, ow}, place_of(r));
  any::run(r, dev, o.numel(), f);
  set(r, "Out", o);
}

void k_interp_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  int64_t oh, ow;
  Interp f = interp_of(r, x, &oh, &ow);
  Tensor d;
  float* dx = grad_out(r, "X@GRAD", x, &d);
  if (!dx) return;
  any::zero(r, dev, dx, x.numel());
  Tensor& g = r.in("Out@GRAD");
  any::run(r, dev, g.numel(), InterpGrad{f, f32(g, dev), dx}, int64_t(1) << 60);
  set(r, "X@GRAD", d);
}

// ---------------------------------------------------------------- pad2d
// constant / reflect / edge padding of [N, C, H, W] (or NHWC); gradient: the adjoint
struct Pad2d {
  const float* x;
  float* o;
  int64_t C, H, W, OH, OW, pt, pl;
  int mode, nhwc;
  float value;
  __host__ __device__ int64_t src(int64_t i, int64_t n) const {  // -1: constant pad
    if (i >= 0 && i < n) return i;
    if (mode == 0) return -1;
    if (mode == 1) {  // reflect (no edge repeat)
      i = i < 0 ? -i : 2 * (n - 1) - i;
      return i;
    }
    return i < 0 ? 0 : n - 1;  // edge
  }
  __host__ __device__ int64_t in_index(int64_t t, int64_t* out_ok) const {
    int64_t n, c, h, w;
    if (nhwc) {
      c = t % C;
      w = (t / C) % OW;
      h = (t / (C * OW)) % OH;
      n = t / (C * OW * OH);
    } else {
      w = t % OW;
      h = (t / OW) % OH;
      c = (t / (OW * OH)) % C;
      n = t / (OW * OH * C);
    }
    const int64_t sh = src(h - pt, H), sw = src(w - pl, W);
    *out_ok = sh >= 0 && sw >= 0;
    if (!*out_ok) return 0;
    return nhwc ? ((n * H + sh) * W + sw) * C + c : ((n * C + c) * H + sh) * W + sw;
  }
  __host__ __device__ void operator()(int64_t t) const {
    int64_t ok;
    const int64_t i = in_index(t, &ok);
    o[t] = ok ? x[i] : value;
  }
};
struct Pad2dGrad {
  Pad2d f;
  const float* g;
  float* dx;
  __host__ __device__ void operator()(int64_t t) const {
    int64_t ok;
    const int64_t i = f.in_index(t, &ok);
    if (ok) acc_add(dx + i, g[t]);
  }
};

Pad2d pad2d_of(const OpRun& r, const Tensor& x) {
  auto p = r.op.GetInts("paddings");
  if (x.dims.size() != 4 || p.size() != 4) throw Decline{};
  const std::string mode = r.op.GetString("mode", "constant");
  const bool nhwc = r.op.GetString("data_format", "NCHW") == "NHWC";
  const int64_t C = nhwc ? x.dims[3] : x.dims[1], H = nhwc ? x.dims[1] : x.dims[2], W = nhwc ? x.dims[2] : x.dims[3];
  Pad2d f{nullptr, nullptr, C, H, W, H + p[0] + p[1], W + p[2] + p[3], p[0], p[2],
          mode == "constant" ? 0 : (mode == "reflect" ? 1 : 2), nhwc ? 1 : 0, r.op.GetFloat("pad_value", 0.f)};
  if (f.mode == 1 && (p[0] >= H || p[1] >= H || p[2] >= W || p[3] >= W)) throw Decline{};
  return f;
}

void k_pad2d(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  Pad2d f = pad2d_of(r, x);
  Dims od = f.nhwc ? Dims{x.dims[0], f.OH, f.OW, f.C} : Dims{x.dims[0], f.C, f.OH, f.OW};
  Tensor o;
  f.x = f32(x, dev);
  f.o = o.alloc<float>(od, place_of(r));
  any::run(r, dev, o.numel(), f);
  set(r, "Out", o);
}

void k_pad2d_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  Pad2d f = pad2d_of(r, x);
  Tensor d;
  float* dx = grad_out(r, "X@GRAD", x, &d);
  if (!dx) return;
  any::zero(r, dev, dx, x.numel());
  Tensor& g = r.in("Out@GRAD");
  any::run(r, dev, g.numel(), Pad2dGrad{f, f32(g, dev), dx}, int64_t(1) << 60);
  set(r, "X@GRAD", d);
}

// ---------------------------------------------------------------- im2sequence
// Out[n L + l, (c kh + i) kw + j] = xpad[n, c, oh sh + i, ow sw + j], LoD [0, L, 2L, ...]
struct Im2Seq {
  const float* x;
  float* o;
  int64_t C, H, W, OH, OW, kh, kw, sh, sw, pt, pl;
  __host__ __device__ int64_t src(int64_t t) const {
    const int64_t CK = C * kh * kw, col = t % CK, row = t / CK;
    const int64_t L = OH * OW, n = row / L, l = row % L, oh = l / OW, ow = l % OW;
    const int64_t c = col / (kh * kw), i = (col / kw) % kh, j = col % kw;
    const int64_t h = oh * sh + i - pt, w = ow * sw + j - pl;
    if (h < 0 || h >= H || w < 0 || w >= W) return -1;
    return ((n * C + c) * H + h) * W + w;
  }
  __host__ __device__ void operator()(int64_t t) const {
    const int64_t s = src(t);
    o[t] = s >= 0 ? x[s] : 0.f;
  }
};
struct Im2SeqGrad {
  Im2Seq f;
  const float* g;
  float* dx;
  __host__ __device__ void operator()(int64_t t) const {
    const int64_t s = f.src(t);
    if (s >= 0) acc_add(dx + s, g[t]);
  }
};

Im2Seq im2seq_of(const OpRun& r, const Tensor& x) {
  auto k = r.op.GetInts("kernels"), st = r.op.GetInts("strides"), p = r.op.GetInts("paddings");
  if (x.dims.size() != 4 || k.size() != 2 || st.size() != 2 || p.size() != 4) throw Decline{};
  const int64_t H = x.dims[2], W = x.dims[3];
  const int64_t OH = (H + p[0] + p[2] - k[0]) / st[0] + 1, OW = (W + p[1] + p[3] - k[1]) / st[1] + 1;
  return Im2Seq{nullptr, nullptr, x.dims[1], H, W, OH, OW, k[0], k[1], st[0], st[1], p[0], p[1]};
}

void k_im2sequence(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  Im2Seq f = im2seq_of(r, x);
  const int64_t N = x.dims[0], L = f.OH * f.OW;
  Tensor o;
  f.x = f32(x, dev);
  f.o = o.alloc<float>({N * L, f.C * f.kh * f.kw}, place_of(r));
  std::vector<size_t> lod;
  for (int64_t n = 0; n <= N; ++n) lod.push_back((size_t)(n * L));
  o.lod = {lod};
  any::run(r, dev, o.numel(), f);
  set(r, "Out", o);
}

void k_im2sequence_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("X");
  Im2Seq f = im2seq_of(r, x);
  Tensor d;
  float* dx = grad_out(r, "X@GRAD", x, &d);
  if (!dx) return;
  any::zero(r, dev, dx, x.numel());
  Tensor& g = r.in("Out@GRAD");
  any::run(r, dev, g.numel(), Im2SeqGrad{f, f32(g, dev), dx}, int64_t(1) << 60);
  set(r, "X@GRAD", d);
}

// ---------------------------------------------------------------- fc_grad
// Out = act(flatten(Input) W + Bias), act in {none, relu}
struct ReluMask {
  const float *g, *out;
  float* d;
  __host__ __device__ void operator()(int64_t i) const { d[i] = out[i] > 0.f ? g[i] : 0.f; }
};

void k_fc_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  Tensor& x = r.in("Input");
  Tensor& w = r.in("W");
  const std::string act = r.op.GetString("activation_type", "");
  if (!act.empty() && act != "relu") throw Decline{};
  const size_t nc = (size_t)r.op.GetInt("in_num_col_dims", 1);
  int64_t M = 1;
  for (size_t k = 0; k < nc && k < x.dims.size(); ++k) M *= x.dims[k];
  const int64_t K = M ? x.numel() / M : 0, N = w.dims.size() == 2 ? w.dims[1] : 0;
  if (w.dims.size() != 2 || w.dims[0] != K) throw Decline{};
  const float* g = f32(r.in("Out@GRAD"), dev);
  std::vector<float> hs;
  if (act == "relu") {
    float* m = any::scratch(r, dev, "@fcg_mask@", M * N, &hs);
    any::run(r, dev, M * N, ReluMask{g, f32(r.in("Out"), dev), m});
    g = m;
  }
  Tensor dX, dW, dB;
  if (float* p = grad_out(r, "Input@GRAD", x, &dX)) {
    any::gemm(r, dev, false, true, M, K, N, 1.f, g, N, f32(w, dev), N, 0.f, p, K);
    set(r, "Input@GRAD", dX);
  }
  if (float* p = grad_out(r, "W@GRAD", w, &dW)) {
    any::gemm(r, dev, true, false, K, N, M, 1.f, f32(x, dev), K, g, N, 0.f, p, N);
    set(r, "W@GRAD", dW);
  }
  if (Tensor* b = r.in_opt("Bias")) {
    if (float* p = grad_out(r, "Bias@GRAD", *b, &dB)) {
      any::run(r, dev, N, any::ColSum{g, p, M, N, 0});
      set(r, "Bias@GRAD", dB);
    }
  }
}

}  // namespace

#define PA_ANY_KERNEL(name, fn) \
  PA_HOST_KERNEL(name, fn);     \
  PA_DEVICE_KERNEL(name, fn)

PA_ANY_KERNEL(hinge_loss, k_hinge);
PA_ANY_KERNEL(hinge_loss_grad, k_hinge_grad);
PA_ANY_KERNEL(modified_huber_loss, k_mod_huber);
PA_ANY_KERNEL(modified_huber_loss_grad, k_mod_huber_grad);
PA_ANY_KERNEL(rank_loss, k_rank_loss);
PA_ANY_KERNEL(rank_loss_grad, k_rank_loss_grad);
PA_ANY_KERNEL(margin_rank_loss, k_margin_rank);
PA_ANY_KERNEL(margin_rank_loss_grad, k_margin_rank_grad);
PA_ANY_KERNEL(l1_norm, k_l1_norm);
PA_ANY_KERNEL(l1_norm_grad, k_l1_norm_grad);
PA_ANY_KERNEL(reverse, k_reverse);
PA_ANY_KERNEL(reverse_grad, k_reverse_grad);
PA_ANY_KERNEL(pad, k_pad);
PA_ANY_KERNEL(pad_grad, k_pad_grad);
PA_ANY_KERNEL(pad_constant_like, k_pad_constant_like);
PA_ANY_KERNEL(pad_constant_like_grad, k_pad_constant_like_grad);
PA_ANY_KERNEL(prelu, k_prelu);
PA_ANY_KERNEL(prelu_grad, k_prelu_grad);
PA_ANY_KERNEL(iou_similarity, k_iou);
PA_ANY_KERNEL(arg_min, k_arg_min);
PA_ANY_KERNEL(fill, k_fill);
PA_ANY_KERNEL(assign_value, k_assign_value);
PA_ANY_KERNEL(proximal_gd, k_proximal_gd);
PA_ANY_KERNEL(proximal_adagrad, k_proximal_adagrad);
PA_ANY_KERNEL(matmul_grad, k_matmul_grad);
PA_ANY_KERNEL(cos_sim, k_cos_sim);
PA_ANY_KERNEL(cos_sim_grad, k_cos_sim_grad);
PA_ANY_KERNEL(multiplex, k_multiplex);
PA_ANY_KERNEL(multiplex_grad, k_multiplex_grad);
PA_ANY_KERNEL(crop, k_crop);
PA_ANY_KERNEL(crop_grad, k_crop_grad);
PA_ANY_KERNEL(norm, k_norm);
PA_ANY_KERNEL(norm_grad, k_norm_grad);
PA_ANY_KERNEL(conv_shift, k_conv_shift);
PA_ANY_KERNEL(conv_shift_grad, k_conv_shift_grad);
PA_ANY_KERNEL(bilinear_tensor_product, k_btp);
PA_ANY_KERNEL(bilinear_tensor_product_grad, k_btp_grad);
PA_ANY_KERNEL(maxout, k_maxout);
PA_ANY_KERNEL(maxout_grad, k_maxout_grad);
PA_ANY_KERNEL(fake_quantize_abs_max, k_fake_quant_abs_max);
PA_ANY_KERNEL(fake_dequantize_max_abs, k_fake_dequant);
PA_ANY_KERNEL(fake_dequantize_max_abs_grad, k_fake_dequant_grad);
PA_ANY_KERNEL(rnn_memory_helper, k_rnn_memory_helper);
PA_ANY_KERNEL(rnn_memory_helper_grad, k_rnn_memory_helper_grad);
PA_ANY_KERNEL(lod_reset_grad, k_lod_reset_grad);
PA_ANY_KERNEL(scatter_grad, k_scatter_grad);
PA_ANY_KERNEL(polygon_box_transform, k_polygon_box);
PA_ANY_KERNEL(argsort, k_argsort);
PA_ANY_KERNEL(row_conv, k_row_conv);
PA_ANY_KERNEL(row_conv_grad, k_row_conv_grad);
PA_ANY_KERNEL(lrn, k_lrn);
PA_ANY_KERNEL(lrn_grad, k_lrn_grad);
PA_ANY_KERNEL(split_lod_tensor, k_split_lod_tensor);
PA_ANY_KERNEL(merge_lod_tensor, k_merge_lod_tensor);
PA_ANY_KERNEL(split_lod_tensor_grad, k_split_lod_tensor_grad);
PA_ANY_KERNEL(merge_lod_tensor_grad, k_merge_lod_tensor_grad);
PA_ANY_KERNEL(max_pool2d_with_index, k_max_pool2d_idx);
PA_ANY_KERNEL(max_pool2d_with_index_grad, k_max_pool2d_idx_grad);
PA_ANY_KERNEL(unpool, k_unpool);
PA_ANY_KERNEL(unpool_grad, k_unpool_grad);
PA_ANY_KERNEL(box_coder, k_box_coder);
PA_ANY_KERNEL(mean_iou, k_mean_iou);
PA_ANY_KERNEL(bilinear_interp, k_interp);
PA_ANY_KERNEL(bilinear_interp_grad, k_interp_grad);
PA_ANY_KERNEL(nearest_interp, k_interp);
PA_ANY_KERNEL(nearest_interp_grad, k_interp_grad);
PA_ANY_KERNEL(pad2d, k_pad2d);
PA_ANY_KERNEL(pad2d_grad, k_pad2d_grad);
PA_ANY_KERNEL(im2sequence, k_im2sequence);
PA_ANY_KERNEL(im2sequence_grad, k_im2sequence_grad);
PA_ANY_KERNEL(fc_grad, k_fc_grad);

void link_more_kernels() {}

}  // namespace pa
