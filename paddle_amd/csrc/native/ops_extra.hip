// Detection priors, pyramid pooling, fused elementwise activation, metrics and the
// remaining random / quantisation / averaging ops of the native executor, host AND
// device from one source (any_place.h): prior_box, anchor_generator, spp (+grad),
// fused_elemwise_activation (+grad), auc, precision_recall, positive_negative_pair,
// average_accumulates, fake_quantize_range_abs_max, bipartite_match, target_assign,
// reduce_*_grad, elementwise_{max,min,pow}_grad, elementwise_{floordiv,mod},
// sequence_reverse / sequence_scatter (+grads), kldiv_loss / bpr_loss (+grads),
// shuffle_channel / scale_sub_region (+grads), size, lars_momentum,
// max_pool3d_with_index (+grad), chunk_eval, sampling_id, random_crop, print; plus the
// host twins of the device-only layer_norm (+grad) and dropout_grad.
//
// Semantics: reference operators/detection/{prior_box,anchor_generator,
// bipartite_match,target_assign}_op.h, operators/{spp,fused_elemwise_activation,auc,
// precision_recall,positive_negative_pair,average_accumulates,fake_quantize,
// layer_norm,dropout}_op.h; the Python kernels of operators/{detection,nn,math,
// metric,optimizer}_ops.py compute the same functions (the interpreter the tests
// compare against) and the auto-VJP grad ops their derivatives (slots: the forward
// inputs, outputs and Out@GRAD; <input>@GRAD out).  The sequential parts (greedy
// matching, metric reductions over a batch) run as one work item per image or one
// work item in total: on a HIP place that is a single lane of a grid-stride kernel,
// which keeps the op on the device stream (no host round trip) for these small
// bookkeeping ops.
#include <hip/hip_runtime.h>
#include <math.h>

#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <map>
#include <random>
#include <string>
#include <vector>

#include "any_place.h"

namespace pa {
namespace {

using any::f32;
using Dims = std::vector<int64_t>;

int place_of(const OpRun& r) { return r.ctx.device >= 0 ? r.ctx.device : -1; }
bool on_dev(const OpRun& r) { return r.ctx.device >= 0; }

void set(const OpRun& r, const char* slot, const Tensor& t) {
  if (Tensor* o = r.out(slot)) *o = t;
}

bool wants(const OpRun& r, const char* slot) { return !r.op.Outputs(slot).empty() && r.out_var(slot); }

// Y's [pre, n, post] placement in X (elementwise_op_function.h); below
bool bc_geo(const Dims& xd, const Dims& yd0, int64_t axis, int64_t* pre, int64_t* n, int64_t* post);

// an int64 / int32 index tensor of the op's place
struct Idx {
  const int64_t* l;
  const int32_t* i;
  __host__ __device__ int64_t operator[](int64_t k) const { return l ? l[k] : (int64_t)i[k]; }
};
Idx idx_of(const Tensor& t, bool dev) {
  if ((t.device >= 0) != dev) throw Decline{};
  if (t.dtype == DT::INT64) return Idx{t.data<int64_t>(), nullptr};
  if (t.dtype == DT::INT32) return Idx{nullptr, t.data<int32_t>()};
  throw Decline{};
}

std::vector<int> offsets_of(const Tensor& t, int64_t rows) {
  std::vector<int> o;
  if (!t.lod.empty())
    for (size_t v : t.lod.back()) o.push_back((int)v);
  else
    o = {0, (int)rows};
  return o;
}

// ---------------------------------------------------------------- prior_box / anchor_generator
// one (h, w, prior) box per work item: [xmin, ymin, xmax, ymax] plus its variances
struct Priors {
  const float *bw, *bh, *var;
  float *box, *vo;
  int64_t W, P;
  float sw, sh, off, iw, ih;
  int clip, anchor;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t p = i % P, w = (i / P) % W, h = i / (P * W);
    float b[4];
    if (anchor) {  // anchor_generator_op.h: pixel centres w * stride + offset * (stride - 1)
      const float xc = (float)w * sw + off * (sw - 1.f), yc = (float)h * sh + off * (sh - 1.f);
      const float hw = 0.5f * (bw[p] - 1.f), hh = 0.5f * (bh[p] - 1.f);
      b[0] = xc - hw; b[1] = yc - hh; b[2] = xc + hw; b[3] = yc + hh;
    } else {  // prior_box_op.h: normalised by the image extent, optionally clipped
      const float cx = ((float)w + off) * sw, cy = ((float)h + off) * sh;
      const float hw = bw[p] / 2.f, hh = bh[p] / 2.f;
      b[0] = (cx - hw) / iw; b[1] = (cy - hh) / ih; b[2] = (cx + hw) / iw; b[3] = (cy + hh) / ih;
      if (clip)
        for (int k = 0; k < 4; ++k) b[k] = fminf(fmaxf(b[k], 0.f), 1.f);
    }
    for (int k = 0; k < 4; ++k) {
      box[i * 4 + k] = b[k];
      vo[i * 4 + k] = var[k];
    }
  }
};

std::vector<double> expand_ars(const std::vector<float>& ars, bool flip) {
  std::vector<double> out = {1.0};
  for (float a : ars) {
    const double cand[2] = {(double)a, 1.0 / (double)a};
    for (int k = 0; k < (flip ? 2 : 1); ++k) {
      bool fresh = true;
      for (double c : out) fresh = fresh && fabs(cand[k] - c) > 1e-6;
      if (fresh) out.push_back(cand[k]);
    }
  }
  return out;
}

void run_priors(const OpRun& r, const Tensor& feat, std::vector<float> bw, std::vector<float> bh, float sw, float sh,
                float off, float iw, float ih, int clip, int anchor, const char* box_slot) {
  const bool dev = on_dev(r);
  PA_CHECK(feat.dims.size() == 4, "%s: NCHW Input expected", r.op.type.c_str());
  if ((feat.device >= 0) != dev) throw Decline{};
  std::vector<float> var = r.op.GetFloats("variances");
  if (var.empty()) var = {0.1f, 0.1f, 0.2f, 0.2f};
  PA_CHECK(var.size() == 4, "%s: 4 variances expected", r.op.type.c_str());
  const int64_t H = feat.dims[2], W = feat.dims[3], P = (int64_t)bw.size();
  PA_CHECK(P > 0, "%s: no box sizes", r.op.type.c_str());
  std::vector<float> tab(bw);
  tab.insert(tab.end(), bh.begin(), bh.end());
  tab.insert(tab.end(), var.begin(), var.end());
  const float* t = tab.data();
  if (dev) {
    std::vector<int> raw(tab.size());
    memcpy(raw.data(), tab.data(), tab.size() * sizeof(float));
    t = (const float*)any::ints(r, dev, "@priors_tab@", raw);
  }
  Tensor box, vo;
  float* bp = box.alloc<float>({H, W, P, 4}, place_of(r));
  float* vp = vo.alloc<float>({H, W, P, 4}, place_of(r));
  any::run(r, dev, H * W * P, Priors{t, t + P, t + 2 * P, bp, vp, W, P, sw, sh, off, iw, ih, clip, anchor});
  set(r, box_slot, box);
  set(r, "Variances", vo);
}

void k_prior_box(const OpRun& r) {
  const Tensor& feat = r.in("Input");
  const Tensor& img = r.in("Image");
  PA_CHECK(img.dims.size() == 4, "prior_box: NCHW Image expected");
  const int64_t H = feat.dims[2], W = feat.dims[3], IH = img.dims[2], IW = img.dims[3];
  const std::vector<float> mins = r.op.GetFloats("min_sizes"), maxs = r.op.GetFloats("max_sizes");
  const auto ars = expand_ars(r.op.GetFloats("aspect_ratios"), r.op.GetBool("flip", true));
  const bool mm_order = r.op.GetBool("min_max_aspect_ratios_order");
  std::vector<float> bw, bh;
  for (size_t k = 0; k < mins.size(); ++k) {
    const double m = mins[k];
    auto with_ars = [&](bool skip_one) {
      for (double a : ars) {
        if (skip_one && fabs(a - 1.0) <= 1e-6) continue;
        bw.push_back((float)(m * sqrt(a)));
        bh.push_back((float)(m / sqrt(a)));
      }
    };
    auto with_max = [&]() {
      if (maxs.empty()) return;
      const double s = sqrt(m * (double)maxs[k]);
      bw.push_back((float)s);
      bh.push_back((float)s);
    };
    if (mm_order) {
      bw.push_back((float)m);
      bh.push_back((float)m);
      with_max();
      with_ars(true);
    } else {
      with_ars(false);
      with_max();
    }
  }
  float sw = r.op.GetFloat("step_w"), sh = r.op.GetFloat("step_h");
  if (sw == 0.f) sw = (float)((double)IW / (double)W);
  if (sh == 0.f) sh = (float)((double)IH / (double)H);
  run_priors(r, feat, bw, bh, sw, sh, r.op.GetFloat("offset", 0.5f), (float)IW, (float)IH,
             r.op.GetBool("clip", true) ? 1 : 0, 0, "Boxes");
}

void k_anchor_generator(const OpRun& r) {
  const Tensor& feat = r.in("Input");
  std::vector<float> stride = r.op.GetFloats("stride");
  if (stride.empty()) stride = {16.f, 16.f};
  PA_CHECK(stride.size() == 2, "anchor_generator: 2 strides expected");
  const double sw = stride[0], sh = stride[1];
  std::vector<float> ws, hs;
  for (float ar : r.op.GetFloats("aspect_ratios"))
    for (float size : r.op.GetFloats("anchor_sizes")) {
      const double base_w = nearbyint(sqrt(sw * sh / (double)ar));  // round half to even, as Python's round
      const double base_h = nearbyint(base_w * (double)ar);
      ws.push_back((float)((double)size / sw * base_w));
      hs.push_back((float)((double)size / sh * base_h));
    }
  run_priors(r, feat, ws, hs, (float)sw, (float)sh, r.op.GetFloat("offset", 0.5f), 1.f, 1.f, 0, 1, "Anchors");
}

// ---------------------------------------------------------------- spp
// spp_op.h: level l pools into 2^l x 2^l bins, kernel = ceil(size / bins), stride =
// kernel, padding (kernel * bins - size + 1) / 2; max over the window's in-image
// pixels, avg divides by their count.  Out [N, C * sum_l 4^l], level-major.
struct SppGeo {
  int64_t N, C, H, W, levels, width;
};
__host__ __device__ inline void spp_win(const SppGeo& g, int64_t lvl, int64_t* kh, int64_t* kw, int64_t* ph,
                                        int64_t* pw, int64_t* col0) {
  const int64_t bins = (int64_t)1 << lvl;
  *kh = (g.H + bins - 1) / bins;
  *kw = (g.W + bins - 1) / bins;
  *ph = (*kh * bins - g.H + 1) / 2;
  *pw = (*kw * bins - g.W + 1) / 2;
  *col0 = g.C * (((int64_t)1 << (2 * lvl)) - 1) / 3;  // C * sum_{j<l} 4^j
}

struct SppFwd {
  const float* x;
  float* o;
  SppGeo g;
  int avg;
  __host__ __device__ void operator()(int64_t i) const {
    // i over N * width
    const int64_t n = i / g.width, col = i % g.width;
    int64_t lvl = 0, kh, kw, ph, pw, c0;
    while (lvl + 1 < g.levels && g.C * (((int64_t)1 << (2 * (lvl + 1))) - 1) / 3 <= col) ++lvl;
    spp_win(g, lvl, &kh, &kw, &ph, &pw, &c0);
    const int64_t bins = (int64_t)1 << lvl, rel = col - c0, c = rel / (bins * bins), bi = (rel / bins) % bins,
                  bj = rel % bins;
    const int64_t h0 = bi * kh - ph, w0 = bj * kw - pw;
    const float* xc = x + (n * g.C + c) * g.H * g.W;
    float acc = avg ? 0.f : -INFINITY;
    int64_t cnt = 0;
    for (int64_t h = h0 < 0 ? 0 : h0; h < h0 + kh && h < g.H; ++h)
      for (int64_t w = w0 < 0 ? 0 : w0; w < w0 + kw && w < g.W; ++w) {
        const float v = xc[h * g.W + w];
        acc = avg ? acc + v : (v > acc ? v : acc);
        ++cnt;
      }
    o[i] = avg ? (cnt ? acc / (float)cnt : 0.f) : acc;
  }
};

// X@GRAD per input pixel: each level's unique window holding it routes its gradient
// (max: to the window's first maximum; avg: 1 / count)
struct SppBwd {
  const float *x, *go;
  float* dx;
  SppGeo g;
  int avg;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t w = i % g.W, h = (i / g.W) % g.H, c = (i / (g.W * g.H)) % g.C, n = i / (g.W * g.H * g.C);
    const float* xc = x + (n * g.C + c) * g.H * g.W;
    float s = 0.f;
    for (int64_t lvl = 0; lvl < g.levels; ++lvl) {
      int64_t kh, kw, ph, pw, c0;
      spp_win(g, lvl, &kh, &kw, &ph, &pw, &c0);
      const int64_t bins = (int64_t)1 << lvl, bi = (h + ph) / kh, bj = (w + pw) / kw;
      if (bi >= bins || bj >= bins) continue;
      const int64_t h0 = bi * kh - ph, w0 = bj * kw - pw;
      const float gv = go[n * g.width + c0 + (c * bins + bi) * bins + bj];
      int64_t cnt = 0, best = -1;
      float bv = -INFINITY;
      for (int64_t hh = h0 < 0 ? 0 : h0; hh < h0 + kh && hh < g.H; ++hh)
        for (int64_t ww = w0 < 0 ? 0 : w0; ww < w0 + kw && ww < g.W; ++ww) {
          const float v = xc[hh * g.W + ww];
          if (best < 0 || v > bv) {
            bv = v;
            best = hh * g.W + ww;
          }
          ++cnt;
        }
      if (avg) s += gv / (float)(cnt ? cnt : 1);
      else if (best == h * g.W + w) s += gv;
    }
    dx[i] = s;
  }
};

SppGeo spp_geo(const OpRun& r, const Tensor& x) {
  PA_CHECK(x.dims.size() == 4, "spp: NCHW input expected");
  SppGeo g{x.dims[0], x.dims[1], x.dims[2], x.dims[3], std::max<int64_t>(1, r.op.GetInt("pyramid_height", 1)), 0};
  PA_CHECK(((int64_t)1 << (g.levels - 1)) <= std::min(g.H, g.W), "spp: more bins than pixels");
  g.width = g.C * (((int64_t)1 << (2 * g.levels)) - 1) / 3;
  return g;
}

void k_spp(const OpRun& r) {
  const bool dev = on_dev(r);
  const Tensor& x = r.in("X");
  const SppGeo g = spp_geo(r, x);
  Tensor o;
  float* op = o.alloc<float>({g.N, g.width}, place_of(r));
  any::run(r, dev, g.N * g.width, SppFwd{f32(x, dev), op, g, r.op.GetString("pooling_type", "max") == "avg"}, 64);
  set(r, "Out", o);
}

void k_spp_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  const Tensor& x = r.in("X");
  if (!wants(r, "X@GRAD")) return;
  const SppGeo g = spp_geo(r, x);
  Tensor d;
  float* dx = d.alloc<float>(x.dims, place_of(r));
  any::run(r, dev, x.numel(),
           SppBwd{f32(x, dev), f32(r.in("Out@GRAD"), dev), dx, g, r.op.GetString("pooling_type", "max") == "avg"},
           64);
  set(r, "X@GRAD", d);
}

// ---------------------------------------------------------------- fused_elemwise_activation
// functor_list {binary, unary}: Out = binary(X, unary(Y)); {unary, binary}: Out =
// unary(binary(X, Y)); binary in {elementwise_add, elementwise_mul}, unary in {relu,
// scale}; Y broadcasts over X as elementwise_op's axis rule ([pre, n, post] with Y
// covering the n span).  IntermediateOut = the inner function's value.
struct FusedGeo {
  int64_t n, post;  // Y index of X element i: (i / post) % n
  int outer_binary, mul, relu;
  float scale;
  __host__ __device__ int64_t yi(int64_t i) const { return (i / post) % n; }
  __host__ __device__ float un(float v) const { return relu ? (v > 0.f ? v : 0.f) : v * scale; }
  __host__ __device__ float dun(float v) const { return relu ? (v > 0.f ? 1.f : 0.f) : scale; }
  __host__ __device__ float bin(float a, float b) const { return mul ? a * b : a + b; }
};

struct FusedFwd {
  const float *x, *y;
  float *o, *inter;
  FusedGeo g;
  __host__ __device__ void operator()(int64_t i) const {
    const float yv = y[g.yi(i)];
    float in, out;
    if (g.outer_binary) {
      in = g.un(yv);
      out = g.bin(x[i], in);
    } else {
      in = g.bin(x[i], yv);
      out = g.un(in);
    }
    o[i] = out;
    if (inter) inter[i] = in;
  }
};

// dX per X element; d(inner) of binary-outer stored per X element for the Y reduction
struct FusedBwdX {
  const float *x, *y, *go;
  float *dx, *dyfull;
  FusedGeo g;
  __host__ __device__ void operator()(int64_t i) const {
    const float yv = y[g.yi(i)], gv = go[i];
    if (g.outer_binary) {  // Out = bin(X, u(Y))
      const float u = g.un(yv);
      if (dx) dx[i] = g.mul ? gv * u : gv;
      if (dyfull) dyfull[i] = (g.mul ? gv * x[i] : gv) * g.dun(yv);
    } else {  // Out = u(bin(X, Y))
      const float d = gv * g.dun(g.bin(x[i], yv));
      if (dx) dx[i] = g.mul ? d * yv : d;
      if (dyfull) dyfull[i] = g.mul ? d * x[i] : d;
    }
  }
};

// dY[j] = sum over the X elements broadcasting Y[j]
struct FusedReduceY {
  const float* full;
  float* dy;
  int64_t pre, n, post;
  __host__ __device__ void operator()(int64_t j) const {
    float s = 0.f;
    for (int64_t a = 0; a < pre; ++a)
      for (int64_t b = 0; b < post; ++b) s += full[(a * n + j) * post + b];
    dy[j] = s;
  }
};

FusedGeo fused_geo(const OpRun& r, const Tensor& x, const Tensor& y, int64_t* pre) {
  const auto it = r.op.attrs.find("functor_list");
  const std::vector<std::string> fl =
      it == r.op.attrs.end() ? std::vector<std::string>{"elementwise_add", "relu"} : it->second.strings;
  PA_CHECK(fl.size() == 2, "fused_elemwise_activation: functor_list of 2 expected");
  FusedGeo g;
  g.outer_binary = fl[0].rfind("elementwise_", 0) == 0;
  const std::string& bn = g.outer_binary ? fl[0] : fl[1];
  const std::string& un = g.outer_binary ? fl[1] : fl[0];
  if ((bn != "elementwise_add" && bn != "elementwise_mul") || (un != "relu" && un != "scale")) throw Decline{};
  g.mul = bn == "elementwise_mul";
  g.relu = un == "relu";
  g.scale = r.op.GetFloat("scale", 0.f);
  // Y's dims, trailing 1s dropped, sit at `axis` of X's dims
  Dims yd = y.dims;
  while (yd.size() > 1 && yd.back() == 1) yd.pop_back();
  int64_t axis = r.op.GetInt("axis", -1);
  if (axis < 0) axis = (int64_t)x.dims.size() - (int64_t)yd.size();
  PA_CHECK(axis >= 0 && axis + (int64_t)yd.size() <= (int64_t)x.dims.size(), "fused_elemwise_activation: bad axis");
  int64_t p = 1, n = 1, q = 1;
  for (int64_t k = 0; k < (int64_t)x.dims.size(); ++k) {
    if (k < axis) p *= x.dims[(size_t)k];
    else if (k < axis + (int64_t)yd.size()) {
      PA_CHECK(x.dims[(size_t)k] == yd[(size_t)(k - axis)], "fused_elemwise_activation: Y does not broadcast");
      n *= x.dims[(size_t)k];
    } else q *= x.dims[(size_t)k];
  }
  g.n = n;
  g.post = q;
  *pre = p;
  return g;
}

void k_fused_ew(const OpRun& r) {
  const bool dev = on_dev(r);
  const Tensor& x = r.in("X");
  const Tensor& y = r.in("Y");
  int64_t pre;
  const FusedGeo g = fused_geo(r, x, y, &pre);
  Tensor o, it;
  float* op = o.alloc<float>(x.dims, place_of(r));
  o.lod = x.lod;
  float* ip = wants(r, "IntermediateOut") ? it.alloc<float>(x.dims, place_of(r)) : nullptr;
  any::run(r, dev, x.numel(), FusedFwd{f32(x, dev), f32(y, dev), op, ip, g});
  set(r, "Out", o);
  if (ip) set(r, "IntermediateOut", it);
}

void k_fused_ew_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  const Tensor& x = r.in("X");
  const Tensor& y = r.in("Y");
  int64_t pre;
  const FusedGeo g = fused_geo(r, x, y, &pre);
  Tensor dxt, dyt;
  float* dx = wants(r, "X@GRAD") ? dxt.alloc<float>(x.dims, place_of(r)) : nullptr;
  float* dy = wants(r, "Y@GRAD") ? dyt.alloc<float>(y.dims, place_of(r)) : nullptr;
  std::vector<float> hfull;
  float* full = dy ? any::scratch(r, dev, "@fused_ew_dy@", x.numel(), &hfull) : nullptr;
  if (!dx && !dy) return;
  any::run(r, dev, x.numel(), FusedBwdX{f32(x, dev), f32(y, dev), f32(r.in("Out@GRAD"), dev), dx, full, g});
  if (dy) any::run(r, dev, g.n, FusedReduceY{full, dy, pre, g.n, g.post}, 16);
  if (dx) set(r, "X@GRAD", dxt);
  if (dy) set(r, "Y@GRAD", dyt);
}

// ---------------------------------------------------------------- auc
// auc_op.h: thresholds k / (n - 1) with -1e-7 and 1 + 1e-7 at the ends; per
// threshold the TP / FN / FP / TN counts (plus the carried-in state), then the
// trapezoid area under ROC (fpr, tpr) or PR (tpr, precision) in double
struct AucCount {
  const float* score;
  Idx lab;
  const int64_t *tp0, *fn0, *fp0, *tn0;
  int64_t *tp, *fn, *fp, *tn;
  int64_t N, stride, nth;
  __host__ __device__ void operator()(int64_t k) const {
    const double th = k == 0 ? -1e-7 : (k == nth - 1 ? 1.0 + 1e-7 : (double)k / (double)(nth - 1));
    int64_t a = 0, b = 0, c = 0, d = 0;
    for (int64_t i = 0; i < N; ++i) {
      const bool ge = (double)score[i * stride] >= th, pos = lab[i] != 0;
      a += ge && pos;
      b += !ge && pos;
      c += ge && !pos;
      d += !ge && !pos;
    }
    tp[k] = a + (tp0 ? tp0[k] : 0);
    fn[k] = b + (fn0 ? fn0[k] : 0);
    fp[k] = c + (fp0 ? fp0[k] : 0);
    tn[k] = d + (tn0 ? tn0[k] : 0);
  }
};
struct AucArea {
  const int64_t *tp, *fn, *fp, *tn;
  double* out;
  int64_t nth;
  int pr;
  __host__ __device__ void operator()(int64_t) const {
    const double eps = 1e-6;
    double s = 0.0, ptpr = 0.0, pfpr = 0.0, pprec = 0.0;
    for (int64_t k = 0; k < nth; ++k) {
      const double TP = (double)tp[k], FN = (double)fn[k], FP = (double)fp[k], TN = (double)tn[k];
      const double tpr = (TP + eps) / (TP + FN + eps), fpr = FP / (FP + TN + eps), prec = (TP + eps) / (TP + FP + eps);
      if (k > 0) s += pr ? (tpr - ptpr) * (prec + pprec) / 2.0 : (pfpr - fpr) * (ptpr + tpr) / 2.0;
      ptpr = tpr;
      pfpr = fpr;
      pprec = prec;
    }
    out[0] = s;
  }
};

void k_auc(const OpRun& r) {
  const bool dev = on_dev(r);
  const Tensor& p = r.in("Predict");
  const Tensor& lab = r.in("Label");
  const int64_t nth = r.op.GetInt("num_thresholds", 200);
  PA_CHECK(nth >= 2, "auc: num_thresholds must be >= 2");
  const bool two = p.dims.size() == 2 && p.dims[1] > 1;
  const int64_t N = two ? p.dims[0] : p.numel(), stride = two ? p.dims[1] : 1;
  PA_CHECK(lab.numel() == N, "auc: Label does not match Predict");
  const float* sp = f32(p, dev) + (two ? 1 : 0);
  const char* slots[4] = {"TP", "FN", "FP", "TN"};
  const int64_t* prev[4];
  for (int k = 0; k < 4; ++k) {
    Tensor* t = r.in_opt(slots[k]);
    prev[k] = nullptr;
    if (t && t->numel() == nth) {
      if (t->dtype != DT::INT64 || (t->device >= 0) != dev) throw Decline{};
      prev[k] = t->data<int64_t>();
    }
  }
  Tensor cnt[4], auc;
  int64_t* c[4];
  for (int k = 0; k < 4; ++k) c[k] = cnt[k].alloc<int64_t>({nth}, place_of(r));
  double* ap = auc.alloc<double>({1}, place_of(r));
  any::run(r, dev, nth, AucCount{sp, idx_of(lab, dev), prev[0], prev[1], prev[2], prev[3], c[0], c[1], c[2], c[3], N,
                                 stride, nth}, 8);
  any::run(r, dev, 1, AucArea{c[0], c[1], c[2], c[3], ap, nth, r.op.GetString("curve", "ROC") == "PR"});
  set(r, "TPOut", cnt[0]);
  set(r, "FNOut", cnt[1]);
  set(r, "FPOut", cnt[2]);
  set(r, "TNOut", cnt[3]);
  set(r, "AUC", auc);
}

// ---------------------------------------------------------------- precision_recall
// precision_recall_op.h: per-class weighted TP / FP / TN / FN of the batch, the
// accumulated states, and macro / micro precision, recall and F1 of both
struct PrecRecall {
  Idx pred, lab;
  const float *w, *st0;
  float *batch, *accum, *st;
  double* work;  // [2, C, 4]
  int64_t N, C;
  __host__ __device__ static void metrics(const double* s, int64_t C, float* out) {
    double mp = 0.0, mr = 0.0, TP = 0.0, FP = 0.0, FN = 0.0;
    for (int64_t c = 0; c < C; ++c) {
      const double tp = s[c * 4], fp = s[c * 4 + 1], fn = s[c * 4 + 3];
      mp += tp + fp > 0.0 ? tp / fmax(tp + fp, 1e-12) : 1.0;
      mr += tp + fn > 0.0 ? tp / fmax(tp + fn, 1e-12) : 1.0;
      TP += tp;
      FP += fp;
      FN += fn;
    }
    mp /= (double)C;
    mr /= (double)C;
    const double mf = mp + mr > 0.0 ? 2.0 * mp * mr / (mp + mr) : 0.0;
    const double up = TP + FP > 0.0 ? TP / (TP + FP) : 1.0, ur = TP + FN > 0.0 ? TP / (TP + FN) : 1.0;
    const double uf = up + ur > 0.0 ? 2.0 * up * ur / (up + ur) : 0.0;
    const double v[6] = {mp, mr, mf, up, ur, uf};
    for (int k = 0; k < 6; ++k) out[k] = (float)v[k];
  }
  __host__ __device__ void operator()(int64_t) const {
    double* b = work;
    double* a = work + C * 4;
    for (int64_t k = 0; k < C * 4; ++k) b[k] = 0.0;
    for (int64_t i = 0; i < N; ++i) {
      const int64_t p = pred[i], l = lab[i];
      const double wv = w ? (double)w[i] : 1.0;
      for (int64_t c = 0; c < C; ++c) {
        const bool pc = p == c, lc = l == c;
        b[c * 4 + (pc ? (lc ? 0 : 1) : (lc ? 3 : 2))] += wv;
      }
    }
    for (int64_t k = 0; k < C * 4; ++k) {
      a[k] = b[k] + (st0 ? (double)st0[k] : 0.0);
      st[k] = (float)a[k];
    }
    metrics(b, C, batch);
    metrics(a, C, accum);
  }
};

void k_precision_recall(const OpRun& r) {
  const bool dev = on_dev(r);
  const Tensor& ind = r.in("Indices");
  const Tensor& lab = r.in("Labels");
  const int64_t C = r.op.GetInt("class_number", 2), N = ind.numel();
  PA_CHECK(lab.numel() == N, "precision_recall: Labels does not match Indices");
  Tensor* w = r.in_opt("Weights");
  Tensor* s0 = r.in_opt("StatesInfo");
  if (s0) PA_CHECK(s0->numel() == C * 4, "precision_recall: StatesInfo must be [class_number, 4]");
  Tensor bt, at, st;
  float* bp = bt.alloc<float>({6}, place_of(r));
  float* ap = at.alloc<float>({6}, place_of(r));
  float* sp = st.alloc<float>({C, 4}, place_of(r));
  std::vector<float> hw;
  double* work = (double*)any::scratch(r, dev, "@prec_recall@", 2 * (2 * C * 4), &hw);
  any::run(r, dev, 1, PrecRecall{idx_of(ind, dev), idx_of(lab, dev), w ? f32(*w, dev) : nullptr,
                                 s0 ? f32(*s0, dev) : nullptr, bp, ap, sp, work, N, C});
  set(r, "BatchMetrics", bt);
  set(r, "AccumMetrics", at);
  set(r, "AccumStatesInfo", st);
}

// ---------------------------------------------------------------- positive_negative_pair
// positive_negative_pair_op.h: over every pair of a query with different labels,
// weight (w_i + w_j) / 2 into positive (score order agrees with label order),
// negative, or neutral (equal scores); plus the accumulated inputs
struct PnPair {
  const float *score, *lab, *w, *acc[3];
  Idx q;
  float* out[3];
  int64_t N, stride;
  __host__ __device__ void operator()(int64_t) const {
    double pos = 0.0, neg = 0.0, neu = 0.0;
    for (int64_t i = 0; i < N; ++i)
      for (int64_t j = i + 1; j < N; ++j) {
        if (q[i] != q[j] || lab[i] == lab[j]) continue;
        const double ww = w ? ((double)w[i] + (double)w[j]) / 2.0 : 1.0;
        const float si = score[i * stride], sj = score[j * stride];
        if (si == sj) neu += ww;
        else if ((si > sj) == (lab[i] > lab[j])) pos += ww;
        else neg += ww;
      }
    const double v[3] = {pos, neg, neu};
    for (int k = 0; k < 3; ++k) out[k][0] = (float)(v[k] + (acc[k] ? (double)acc[k][0] : 0.0));
  }
};

void k_pn_pair(const OpRun& r) {
  const bool dev = on_dev(r);
  const Tensor& s = r.in("Score");
  const Tensor& lab = r.in("Label");
  const Tensor& q = r.in("QueryID");
  const bool two = s.dims.size() == 2;
  int64_t col = r.op.GetInt("column", 0);
  const int64_t N = two ? s.dims[0] : s.numel(), stride = two ? s.dims[1] : 1;
  if (col < 0) col += stride;
  PA_CHECK(col >= 0 && col < stride, "positive_negative_pair: column out of range");
  PA_CHECK(lab.numel() == N && q.numel() == N, "positive_negative_pair: Label / QueryID do not match Score");
  Tensor* w = r.in_opt("Weight");
  const char* accs[3] = {"AccumulatePositivePair", "AccumulateNegativePair", "AccumulateNeutralPair"};
  const char* outs[3] = {"PositivePair", "NegativePair", "NeutralPair"};
  PnPair f;
  Tensor ot[3];
  for (int k = 0; k < 3; ++k) {
    Tensor* a = r.in_opt(accs[k]);
    f.acc[k] = a ? f32(*a, dev) : nullptr;
    f.out[k] = ot[k].alloc<float>({1}, place_of(r));
  }
  f.score = f32(s, dev) + (two ? col : 0);
  f.lab = f32(lab, dev);
  f.w = w ? f32(*w, dev) : nullptr;
  f.q = idx_of(q, dev);
  f.N = N;
  f.stride = stride;
  any::run(r, dev, 1, f);
  for (int k = 0; k < 3; ++k) set(r, outs[k], ot[k]);
}

// ---------------------------------------------------------------- average_accumulates
// average_accumulates_op.h (ModelAverage): sum_1 += param; every 16384 updates sum_1
// folds into sum_2; once the window is full sum_3 = sum_1 + sum_2 and both restart.
// The counters step on the op's place (one work item), the sums read its flags.
struct AvgCounters {
  Idx na0, ona0, nu0;
  int64_t *na, *ona, *nu;
  float* flags;  // [fold into sum_2, restart window]
  int64_t min_w, max_w;
  float win;
  __host__ __device__ void operator()(int64_t) const {
    int64_t a = na0[0] + 1, o = ona0[0], u = nu0[0] + 1;
    flags[0] = u % 16384 == 0 ? 1.f : 0.f;
    const double lim = (double)u * (double)win;
    const bool roll = a >= min_w && (double)a >= (lim < (double)max_w ? lim : (double)max_w);
    flags[1] = roll ? 1.f : 0.f;
    if (roll) {
      o = a;
      a = 0;
    }
    na[0] = a;
    ona[0] = o;
    nu[0] = u;
  }
};
struct AvgSums {
  const float *p, *s1, *s2, *s3, *flags;
  float *o1, *o2, *o3;
  __host__ __device__ void operator()(int64_t i) const {
    float a = s1[i] + p[i], b = s2[i];
    if (flags[0] != 0.f) {
      b += a;
      a = 0.f;
    }
    float c = s3[i];
    if (flags[1] != 0.f) {
      c = a + b;
      a = 0.f;
      b = 0.f;
    }
    o1[i] = a;
    o2[i] = b;
    o3[i] = c;
  }
};

void k_average_accumulates(const OpRun& r) {
  const bool dev = on_dev(r);
  const Tensor& p = r.in("param");
  const Tensor& s1 = r.in("in_sum_1");
  const Tensor& s2 = r.in("in_sum_2");
  const Tensor& s3 = r.in("in_sum_3");
  PA_CHECK(s1.numel() == p.numel() && s2.numel() == p.numel() && s3.numel() == p.numel(),
           "average_accumulates: sums must match param");
  std::vector<float> hf;
  float* flags = any::scratch(r, dev, "@avg_acc_flags@", 2, &hf);
  Tensor c[3], o[3];
  int64_t* cp[3];
  for (int k = 0; k < 3; ++k) cp[k] = c[k].alloc<int64_t>({1}, place_of(r));
  any::run(r, dev, 1, AvgCounters{idx_of(r.in("in_num_accumulates"), dev), idx_of(r.in("in_old_num_accumulates"), dev),
                                  idx_of(r.in("in_num_updates"), dev), cp[0], cp[1], cp[2], flags,
                                  r.op.GetInt("min_average_window", 10000), r.op.GetInt("max_average_window", 10000),
                                  r.op.GetFloat("average_window", 0.f)});
  float* op[3];
  for (int k = 0; k < 3; ++k) op[k] = o[k].alloc<float>(p.dims, place_of(r));
  any::run(r, dev, p.numel(), AvgSums{f32(p, dev), f32(s1, dev), f32(s2, dev), f32(s3, dev), flags, op[0], op[1],
                                      op[2]});
  set(r, "out_sum_1", o[0]);
  set(r, "out_sum_2", o[1]);
  set(r, "out_sum_3", o[2]);
  set(r, "out_num_accumulates", c[0]);
  set(r, "out_old_num_accumulates", c[1]);
  set(r, "out_num_updates", c[2]);
}

// ---------------------------------------------------------------- fake_quantize_range_abs_max
// fake_quantize_op.h FindRangeAbsMax: scale = max(|X|max, InScale) in training,
// InScale at test; Out = round(clip(X, -s, s) / s * (2^(bits-1) - 1))
struct AbsMaxPart {
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
struct RangeScale {
  const float *part, *in;
  float* out;
  int64_t nc;
  int test;
  __host__ __device__ void operator()(int64_t) const {
    float m = 0.f;
    for (int64_t c = 0; c < nc; ++c) m = fmaxf(m, part[c]);
    out[0] = test ? in[0] : fmaxf(m, in[0]);
  }
};
struct RangeQuant {
  const float *x, *s;
  float* o;
  float bins;
  __host__ __device__ void operator()(int64_t i) const {
    const float sc = s[0], v = fminf(fmaxf(x[i], -sc), sc);
    o[i] = rintf(v / fmaxf(sc, 1e-30f) * bins);
  }
};
struct Broadcast1 {
  const float* s;
  float* o;
  __host__ __device__ void operator()(int64_t i) const { o[i] = s[0]; }
};

void k_fake_quant_range(const OpRun& r) {
  const bool dev = on_dev(r);
  const Tensor& x = r.in("X");
  const Tensor& in_s = r.in("InScale");
  PA_CHECK(in_s.numel() >= 1, "fake_quantize_range_abs_max: empty InScale");
  const int64_t n = x.numel(), chunk = 4096, nc = std::max<int64_t>(1, (n + chunk - 1) / chunk);
  std::vector<float> hp;
  float* part = any::scratch(r, dev, "@fq_range_part@", nc, &hp);
  Tensor sc, o;
  float* sp = sc.alloc<float>({1}, place_of(r));
  any::run(r, dev, nc, AbsMaxPart{f32(x, dev), part, n, chunk});
  any::run(r, dev, 1, RangeScale{part, f32(in_s, dev), sp, nc, (r.ctx.is_test || r.op.GetBool("is_test")) ? 1 : 0});
  const float bins = (float)((1 << (r.op.GetInt("bit_length", 8) - 1)) - 1);
  float* op = o.alloc<float>(x.dims, place_of(r));
  any::run(r, dev, n, RangeQuant{f32(x, dev), sp, op, bins});
  set(r, "Out", o);
  if (wants(r, "OutScales")) {
    const int64_t ws = r.op.GetInt("window_size", 10000);
    Tensor ss;
    any::run(r, dev, ws, Broadcast1{sp, ss.alloc<float>({ws}, place_of(r))});
    set(r, "OutScales", ss);
  }
  set(r, "OutScale", sc);
}

// ---------------------------------------------------------------- bipartite_match
// bipartite_match_op.cc: per image (LoD of DistMat) the greedy global-maximum
// matching of rows (ground truth) to columns (priors) while the best remaining
// distance is positive; per_prediction then matches every unmatched column to its
// best row when that distance reaches dist_threshold.  One work item per image.
struct Bipartite {
  const float* d;
  float* work;
  const int* off;
  int* idx;
  float* dist;
  int64_t M;
  int per_pred;
  float thr;
  __host__ __device__ void operator()(int64_t b) const {
    const int64_t r0 = off[b], R = off[b + 1] - off[b];
    int* ib = idx + b * M;
    float* db = dist + b * M;
    for (int64_t c = 0; c < M; ++c) {
      ib[c] = -1;
      db[c] = 0.f;
    }
    if (R <= 0) return;
    const float* dm = d + r0 * M;
    float* w = work + r0 * M;
    for (int64_t k = 0; k < R * M; ++k) w[k] = dm[k];
    for (;;) {
      int64_t best = 0;
      for (int64_t k = 1; k < R * M; ++k)
        if (w[k] > w[best]) best = k;
      if (!(w[best] > 0.f)) break;
      const int64_t rr = best / M, cc = best % M;
      ib[cc] = (int)rr;
      db[cc] = dm[best];
      for (int64_t c = 0; c < M; ++c) w[rr * M + c] = -1.f;
      for (int64_t q = 0; q < R; ++q) w[q * M + cc] = -1.f;
    }
    if (!per_pred) return;
    for (int64_t c = 0; c < M; ++c) {
      if (ib[c] >= 0) continue;
      int64_t br = 0;
      for (int64_t q = 1; q < R; ++q)
        if (dm[q * M + c] > dm[br * M + c]) br = q;
      if (dm[br * M + c] >= thr) {
        ib[c] = (int)br;
        db[c] = dm[br * M + c];
      }
    }
  }
};

void k_bipartite_match(const OpRun& r) {
  const bool dev = on_dev(r);
  const Tensor& d = r.in("DistMat");
  PA_CHECK(d.dims.size() == 2, "bipartite_match: 2-D DistMat expected");
  const int64_t M = d.dims[1];
  const std::vector<int> off = offsets_of(d, d.dims[0]);
  const int64_t B = (int64_t)off.size() - 1;
  const std::string mt = r.op.GetString("match_type", "bipartite");
  std::vector<float> hw;
  float* work = any::scratch(r, dev, "@bipartite_work@", d.numel(), &hw);
  Tensor it, dt;
  int* ip = it.alloc<int>({B, M}, place_of(r));
  float* dp = dt.alloc<float>({B, M}, place_of(r));
  any::run(r, dev, B, Bipartite{f32(d, dev), work, any::ints(r, dev, "@bipartite_off@", off), ip, dp, M,
                                mt == "per_prediction" ? 1 : 0, r.op.GetFloat("dist_threshold", 0.5f)}, 1);
  set(r, "ColToRowMatchIndices", it);
  set(r, "ColToRowMatchDist", dt);
}

// ---------------------------------------------------------------- target_assign
// target_assign_op.h: Out[b, p] = X[lod(b) + match(b, p), p % cols] for matched
// priors (weight 1), mismatch_value otherwise (weight 0); NegIndices (LoD per image)
// then mark their priors weight 1 with mismatch_value.
struct TargetAssign {
  const float* x;
  Idx mi;
  const int* xo;
  float *o, *w;
  int64_t P, K, cols;
  float mis;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t k = i % K, bp = i / K, p = bp % P, b = bp / P;
    const int64_t m = mi[bp];
    if (m >= 0) {
      o[i] = x[((xo[b] + m) * cols + (cols > 1 ? p % cols : 0)) * K + k];
      if (k == 0) w[bp] = 1.f;
    } else {
      o[i] = mis;
      if (k == 0) w[bp] = 0.f;
    }
  }
};
struct TargetNeg {
  Idx neg;
  const int* no;
  float *o, *w;
  int64_t B, P, K;
  float mis;
  __host__ __device__ void operator()(int64_t e) const {
    int64_t b = 0;
    while (b + 1 < B && no[b + 1] <= e) ++b;
    const int64_t p = neg[e];
    if (p < 0 || p >= P) return;
    w[b * P + p] = 1.f;
    for (int64_t k = 0; k < K; ++k) o[(b * P + p) * K + k] = mis;
  }
};

void k_target_assign(const OpRun& r) {
  const bool dev = on_dev(r);
  const Tensor& x = r.in("X");
  const Tensor& mi = r.in("MatchIndices");
  PA_CHECK(mi.dims.size() == 2 && x.dims.size() >= 2, "target_assign: X [rows, (cols,) K], MatchIndices [N, P]");
  const int64_t N = mi.dims[0], P = mi.dims[1], K = x.dims.back(), cols = x.numel() / (x.dims[0] * K);
  const std::vector<int> xo = offsets_of(x, x.dims[0]);
  PA_CHECK((int64_t)xo.size() == N + 1, "target_assign: X LoD does not match MatchIndices");
  const float mis = (float)r.op.GetInt("mismatch_value", 0);
  Tensor ot, wt;
  float* op = ot.alloc<float>({N, P, K}, place_of(r));
  float* wp = wt.alloc<float>({N, P, 1}, place_of(r));
  any::run(r, dev, N * P * K, TargetAssign{f32(x, dev), idx_of(mi, dev), any::ints(r, dev, "@ta_xo@", xo), op, wp, P,
                                           K, cols, mis});
  if (Tensor* neg = r.in_opt("NegIndices")) {
    const std::vector<int> no = offsets_of(*neg, neg->numel());
    PA_CHECK((int64_t)no.size() == N + 1, "target_assign: NegIndices LoD does not match MatchIndices");
    any::run(r, dev, neg->numel(), TargetNeg{idx_of(*neg, dev), any::ints(r, dev, "@ta_no@", no), op, wp, N, P, K,
                                             mis});
  }
  set(r, "Out", ot);
  set(r, "OutWeight", wt);
}

// ---------------------------------------------------------------- host layer_norm / dropout_grad
// (their HIP kernels live in ops_gpu.hip on the norm / mask kernels of the library)
void ln_geom(const OpRun& r, const Tensor& x, int64_t* rows, int64_t* H) {
  const int64_t ax = r.op.GetInt("begin_norm_axis", 1);
  PA_CHECK(ax >= 1 && ax <= (int64_t)x.dims.size(), "layer_norm: begin_norm_axis out of range");
  *rows = 1;
  for (int64_t k = 0; k < ax; ++k) *rows *= x.dims[(size_t)k];
  *H = x.numel() / std::max<int64_t>(*rows, 1);
}

struct LnFwd {
  const float *x, *w, *b;
  float *y, *mean, *var;
  int64_t H;
  float eps;
  __host__ __device__ void operator()(int64_t i) const {
    const float* xr = x + i * H;
    double s = 0.0;
    for (int64_t j = 0; j < H; ++j) s += xr[j];
    const double mu = s / (double)H;
    double v = 0.0;
    for (int64_t j = 0; j < H; ++j) v += ((double)xr[j] - mu) * ((double)xr[j] - mu);
    v /= (double)H;
    const float m = (float)mu, rs = (float)(1.0 / sqrt(v + (double)eps));
    for (int64_t j = 0; j < H; ++j) {
      float o = (xr[j] - m) * rs;
      if (w) o *= w[j];
      if (b) o += b[j];
      y[i * H + j] = o;
    }
    mean[i] = m;
    var[i] = (float)v;
  }
};
struct LnBwdX {
  const float *x, *g, *mean, *var, *w;
  float* dx;
  int64_t H;
  float eps;
  __host__ __device__ void operator()(int64_t i) const {
    const float rs = 1.f / sqrtf(var[i] + eps), m = mean[i];
    const float *xr = x + i * H, *gr = g + i * H;
    double sg = 0.0, sgx = 0.0;
    for (int64_t j = 0; j < H; ++j) {
      const float gx = w ? gr[j] * w[j] : gr[j];
      sg += gx;
      sgx += (double)gx * (double)((xr[j] - m) * rs);
    }
    const float mg = (float)(sg / (double)H), mgx = (float)(sgx / (double)H);
    for (int64_t j = 0; j < H; ++j) {
      const float gx = w ? gr[j] * w[j] : gr[j], xh = (xr[j] - m) * rs;
      dx[i * H + j] = rs * (gx - mg - xh * mgx);
    }
  }
};
struct LnBwdW {
  const float *x, *g, *mean, *var;
  float *dw, *db;
  int64_t rows, H;
  float eps;
  __host__ __device__ void operator()(int64_t j) const {
    double sw = 0.0, sb = 0.0;
    for (int64_t i = 0; i < rows; ++i) {
      const float rs = 1.f / sqrtf(var[i] + eps), gv = g[i * H + j];
      sw += (double)gv * (double)((x[i * H + j] - mean[i]) * rs);
      sb += gv;
    }
    if (dw) dw[j] = (float)sw;
    if (db) db[j] = (float)sb;
  }
};

}  // namespace

// layer_norm (+grad) on either place, one work item per row (per column for the
// parameter gradients): the host kernel, and the device path for the shapes the
// fused norm kernel of the library does not take (ops_gpu.hip k_layer_norm)
void layer_norm_any(const OpRun& r) {
  const bool dev = on_dev(r);
  const Tensor& x = r.in("X");
  int64_t rows, H;
  ln_geom(r, x, &rows, &H);
  Tensor* sc = r.in_opt("Scale");
  Tensor* bi = r.in_opt("Bias");
  Tensor y, mt, vt;
  float* yp = y.alloc<float>(x.dims, place_of(r));
  y.lod = x.lod;
  any::run(r, dev, rows, LnFwd{f32(x, dev), sc ? f32(*sc, dev) : nullptr, bi ? f32(*bi, dev) : nullptr, yp,
                               mt.alloc<float>({rows}, place_of(r)), vt.alloc<float>({rows}, place_of(r)), H,
                               r.op.GetFloat("epsilon", 1e-5f)}, 8);
  set(r, "Y", y);
  set(r, "Mean", mt);
  set(r, "Variance", vt);
}

void layer_norm_grad_any(const OpRun& r) {
  const bool dev = on_dev(r);
  const Tensor& x = r.in("X");
  int64_t rows, H;
  ln_geom(r, x, &rows, &H);
  Tensor* sc = r.in_opt("Scale");
  Tensor* bi = r.in_opt("Bias");
  const float eps = r.op.GetFloat("epsilon", 1e-5f);
  const float *xp = f32(x, dev), *gp = f32(r.in("Y@GRAD"), dev), *mp = f32(r.in("Mean"), dev),
              *vp = f32(r.in("Variance"), dev);
  Tensor dxt, dwt, dbt;
  float* dx = wants(r, "X@GRAD") ? dxt.alloc<float>(x.dims, place_of(r)) : nullptr;
  float* dw = (sc && wants(r, "Scale@GRAD")) ? dwt.alloc<float>(sc->dims, place_of(r)) : nullptr;
  float* db = (bi && wants(r, "Bias@GRAD")) ? dbt.alloc<float>(bi->dims, place_of(r)) : nullptr;
  if (dx) any::run(r, dev, rows, LnBwdX{xp, gp, mp, vp, sc ? f32(*sc, dev) : nullptr, dx, H, eps}, 8);
  if (dw || db) any::run(r, dev, H, LnBwdW{xp, gp, mp, vp, dw, db, rows, H, eps}, 64);
  if (dx) set(r, "X@GRAD", dxt);
  if (dw) set(r, "Scale@GRAD", dwt);
  if (db) set(r, "Bias@GRAD", dbt);
}

// integer elementwise_{add,sub,mul,div,max,min} on either place (index arithmetic;
// the float kernels live in ops_host.cc / ops_gpu.hip); Y broadcast as [pre, n, post]
template <class T>
struct EwInt {
  const T *x, *y;
  T* o;
  int64_t n, post;
  int op;
  __host__ __device__ void operator()(int64_t i) const {
    const T a = x[i], b = y[(i / post) % n];
    T v;
    switch (op) {
      case 0: v = a + b; break;
      case 1: v = a - b; break;
      case 2: v = a * b; break;
      case 3: v = b ? a / b : 0; break;
      case 4: v = a > b ? a : b; break;
      default: v = a < b ? a : b; break;
    }
    o[i] = v;
  }
};

void elementwise_int_any(const OpRun& r, int op) {
  const bool dev = on_dev(r);
  const Tensor& x = r.in("X");
  const Tensor& y = r.in("Y");
  int64_t pre, n, post;
  if (op > 5 || x.dtype != y.dtype || (x.device >= 0) != dev || (y.device >= 0) != dev ||
      !bc_geo(x.dims, y.dims, r.op.GetInt("axis", -1), &pre, &n, &post))
    throw Decline{};
  Tensor o;
  void* p = o.alloc(x.dtype, x.dims, place_of(r));
  o.lod = x.lod;
  if (x.dtype == DT::INT64)
    any::run(r, dev, x.numel(), EwInt<int64_t>{x.data<int64_t>(), y.data<int64_t>(), (int64_t*)p, n, post, op});
  else if (x.dtype == DT::INT32)
    any::run(r, dev, x.numel(), EwInt<int32_t>{x.data<int32_t>(), y.data<int32_t>(), (int32_t*)p, n, post, op});
  else
    throw Decline{};
  set(r, "Out", o);
}

namespace {

void k_dropout_grad_host(const OpRun& r) {
  const Tensor& m = r.in("Mask");
  const Tensor& d = r.in("Out@GRAD");
  const float* gp = f32(d, false);
  PA_CHECK(m.numel() == d.numel(), "dropout_grad: Mask does not match Out@GRAD");
  const float p = r.op.GetFloat("dropout_prob", 0.5f);
  const bool upscale = r.op.GetString("dropout_implementation", "downgrade_in_infer") == "upscale_in_train";
  const float scale = (upscale && p < 1.f) ? 1.f / (1.f - p) : 1.f;
  if (m.device >= 0) throw Decline{};
  Tensor o;
  float* dx = o.alloc<float>(d.dims, -1);
  o.lod = d.lod;
  const int64_t n = d.numel();
  if (m.dtype == DT::FP32) {
    const float* mp = m.data<float>();
    for (int64_t i = 0; i < n; ++i) dx[i] = gp[i] * mp[i] * scale;
  } else if (m.dtype == DT::UINT8 || m.dtype == DT::BOOL) {
    const uint8_t* mp = m.data<uint8_t>();
    for (int64_t i = 0; i < n; ++i) dx[i] = mp[i] ? gp[i] * scale : 0.f;
  } else {
    throw Decline{};
  }
  set(r, "X@GRAD", o);
}

// ---------------------------------------------------------------- reduce_*_grad
// reduce_op.h ReduceGradKernel over X's dims with the reduced axes flagged (dim,
// reduce_all; an empty dim list reduces everything, as the Python kernel): sum ->
// g; mean -> g / |group|; max / min -> g split evenly over the group's elements equal
// to Out (torch amax / amin's rule, which the interpreter's autograd follows); prod ->
// g * prod of the group's other elements
struct RGeo {
  int R;
  int64_t xd[8], kst[8];  // X dims; strides of the kept-dims (Out) index per axis (0: reduced)
  int red[8];
  int64_t gsize;
  __host__ __device__ int64_t out_of(int64_t i) const {
    int64_t o = 0;
    for (int d = R - 1; d >= 0; --d) {
      const int64_t c = i % xd[d];
      i /= xd[d];
      o += c * kst[d];
    }
    return o;
  }
  // X index of member j of the group of X element i (i's kept coordinates, j over the reduced ones)
  __host__ __device__ int64_t member(int64_t i, int64_t j) const {
    int64_t idx = 0, mul = 1;
    for (int d = R - 1; d >= 0; --d) {
      int64_t c = i % xd[d];
      i /= xd[d];
      if (red[d]) {
        c = j % xd[d];
        j /= xd[d];
      }
      idx += c * mul;
      mul *= xd[d];
    }
    return idx;
  }
};

template <int KIND>  // 0 sum, 1 mean, 2 max, 3 min, 4 prod
struct ReduceGrad {
  const float *x, *out, *g;
  float* dx;
  RGeo geo;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t o = geo.out_of(i);
    const float gv = g[o];
    if (KIND == 0) {
      dx[i] = gv;
    } else if (KIND == 1) {
      dx[i] = gv / (float)geo.gsize;
    } else if (KIND == 2 || KIND == 3) {
      if (x[i] != out[o]) {
        dx[i] = 0.f;
        return;
      }
      int64_t ties = 0;
      for (int64_t j = 0; j < geo.gsize; ++j) ties += x[geo.member(i, j)] == out[o];
      dx[i] = gv / (float)ties;
    } else {
      float p = 1.f;
      for (int64_t j = 0; j < geo.gsize; ++j) {
        const int64_t m = geo.member(i, j);
        if (m != i) p *= x[m];
      }
      dx[i] = gv * p;
    }
  }
};

template <int KIND>
void k_reduce_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  const Tensor& x = r.in("X");
  if (!wants(r, "X@GRAD")) return;
  const int R = (int)x.dims.size();
  if (R > 8) throw Decline{};
  RGeo geo;
  geo.R = R;
  std::vector<int64_t> dims = r.op.GetInts("dim");
  const bool all = r.op.GetBool("reduce_all") || dims.empty();
  for (int d = 0; d < R; ++d) {
    geo.xd[d] = x.dims[(size_t)d];
    geo.red[d] = all ? 1 : 0;
  }
  for (int64_t a : dims) {
    const int64_t d = a < 0 ? a + R : a;
    PA_CHECK(d >= 0 && d < R, "%s: dim out of range", r.op.type.c_str());
    geo.red[d] = 1;
  }
  int64_t st = 1;
  geo.gsize = 1;
  for (int d = R - 1; d >= 0; --d) {
    geo.kst[d] = geo.red[d] ? 0 : st;
    if (!geo.red[d]) st *= geo.xd[d];
    else geo.gsize *= geo.xd[d];
  }
  const Tensor& g = r.in("Out@GRAD");
  PA_CHECK(g.numel() == st, "%s: Out@GRAD %s does not match", r.op.type.c_str(), g.shape_str().c_str());
  const float* outp = (KIND == 2 || KIND == 3) ? f32(r.in("Out"), dev) : nullptr;
  Tensor d;
  float* dx = d.alloc<float>(x.dims, place_of(r));
  d.lod = x.lod;
  const float* xp = KIND >= 2 ? f32(x, dev) : nullptr;
  any::run(r, dev, x.numel(), ReduceGrad<KIND>{xp, outp, f32(g, dev), dx, geo});
  set(r, "X@GRAD", d);
}

// ---------------------------------------------------------------- elementwise max / min / pow grads
// Y broadcast into X as elementwise_op_function.h's [pre, n, post] (Y's dims,
// trailing 1s dropped, at `axis`).  max / min follow torch.maximum / minimum's rule
// (ties split the gradient in half); pow: dX = g y x^(y-1), dY = g x^y ln x.
bool bc_geo(const Dims& xd, const Dims& yd0, int64_t axis, int64_t* pre, int64_t* n, int64_t* post) {
  Dims yd = yd0;
  while (yd.size() > 1 && yd.back() == 1) yd.pop_back();
  *pre = *n = *post = 1;
  if (yd.size() == 1 && yd[0] == 1) {  // a scalar Y
    for (int64_t d : xd) *pre *= d;
    return true;
  }
  if (axis < 0) axis = (int64_t)xd.size() - (int64_t)yd.size();
  if (axis < 0 || axis + (int64_t)yd.size() > (int64_t)xd.size()) return false;
  for (int64_t k = 0; k < (int64_t)xd.size(); ++k) {
    if (k < axis) *pre *= xd[(size_t)k];
    else if (k < axis + (int64_t)yd.size()) {
      if (xd[(size_t)k] != yd[(size_t)(k - axis)]) return false;
      *n *= xd[(size_t)k];
    } else *post *= xd[(size_t)k];
  }
  return true;
}

template <int KIND>  // 0 max, 1 min, 2 pow
struct EwGrad3 {
  const float *x, *y, *g;
  float *dx, *dyf;
  int64_t n, post;
  __host__ __device__ void operator()(int64_t i) const {
    const float a = x[i], b = y[(i / post) % n], gv = g[i];
    float gx, gy;
    if (KIND == 2) {
      gx = gv * b * powf(a, b - 1.f);
      gy = gv * powf(a, b) * logf(a);
    } else {
      const bool win = KIND == 0 ? a > b : a < b;
      gx = a == b ? gv * 0.5f : (win ? gv : 0.f);
      gy = gv - gx;
    }
    if (dx) dx[i] = gx;
    if (dyf) dyf[i] = gy;
  }
};

template <int KIND>
void k_ew_grad3(const OpRun& r) {
  const bool dev = on_dev(r);
  const Tensor& x = r.in("X");
  const Tensor& y = r.in("Y");
  const Tensor& g = r.in("Out@GRAD");
  int64_t pre, n, post;
  if (g.numel() != x.numel() || !bc_geo(x.dims, y.dims, r.op.GetInt("axis", -1), &pre, &n, &post)) throw Decline{};
  Tensor dxt, dyt;
  float* dx = wants(r, "X@GRAD") ? dxt.alloc<float>(x.dims, place_of(r)) : nullptr;
  float* dy = wants(r, "Y@GRAD") ? dyt.alloc<float>(y.dims, place_of(r)) : nullptr;
  if (!dx && !dy) return;
  dxt.lod = x.lod;
  std::vector<float> hf;
  float* full = dy ? (pre * post == 1 ? dy : any::scratch(r, dev, "@ew_grad3@", x.numel(), &hf)) : nullptr;
  any::run(r, dev, x.numel(), EwGrad3<KIND>{f32(x, dev), f32(y, dev), f32(g, dev), dx, full, n, post});
  if (dy && pre * post != 1) any::run(r, dev, n, FusedReduceY{full, dy, pre, n, post}, 16);
  if (dx) set(r, "X@GRAD", dxt);
  if (dy) set(r, "Y@GRAD", dyt);
}

// elementwise_floordiv / elementwise_mod (torch floor division / remainder: the
// result takes the divisor's sign) over int64, int32 and fp32
template <class T, bool MOD>
struct FloorDivMod {
  const T *x, *y;
  T* o;
  int64_t n, post;
  __host__ __device__ void operator()(int64_t i) const {
    const T a = x[i], b = y[(i / post) % n];
    if (MOD) {
      T m = a % b;
      if (m != 0 && ((m < 0) != (b < 0))) m += b;
      o[i] = m;
    } else {
      T q = a / b;
      if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
      o[i] = q;
    }
  }
};
template <bool MOD>
struct FloorDivModF {
  const float *x, *y;
  float* o;
  int64_t n, post;
  __host__ __device__ void operator()(int64_t i) const {
    const float a = x[i], b = y[(i / post) % n];
    if (MOD) {
      float m = fmodf(a, b);
      if (m != 0.f && ((m < 0.f) != (b < 0.f))) m += b;
      o[i] = m;
    } else {
      o[i] = floorf(a / b);
    }
  }
};

template <bool MOD>
void k_floordiv_mod(const OpRun& r) {
  const bool dev = on_dev(r);
  const Tensor& x = r.in("X");
  const Tensor& y = r.in("Y");
  int64_t pre, n, post;
  if (x.dtype != y.dtype || (x.device >= 0) != dev || (y.device >= 0) != dev ||
      !bc_geo(x.dims, y.dims, r.op.GetInt("axis", -1), &pre, &n, &post))
    throw Decline{};
  Tensor o;
  void* op = o.alloc(x.dtype, x.dims, place_of(r));
  o.lod = x.lod;
  switch (x.dtype) {
    case DT::INT64:
      any::run(r, dev, x.numel(), FloorDivMod<int64_t, MOD>{x.data<int64_t>(), y.data<int64_t>(), (int64_t*)op, n, post});
      break;
    case DT::INT32:
      any::run(r, dev, x.numel(), FloorDivMod<int32_t, MOD>{x.data<int32_t>(), y.data<int32_t>(), (int32_t*)op, n, post});
      break;
    case DT::FP32:
      any::run(r, dev, x.numel(), FloorDivModF<MOD>{x.data<float>(), y.data<float>(), (float*)op, n, post});
      break;
    default:
      throw Decline{};
  }
  set(r, "Out", o);
}

// ---------------------------------------------------------------- sequence_reverse / sequence_scatter
// sequence_reverse: rows of every last-level sequence reversed (an involution, so the
// gradient is the same gather of Y@GRAD)
struct SeqReverse {
  const float* x;
  float* y;
  const int* off;
  int64_t W, nseq;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t row = i / W;
    int64_t lo = 0, hi = nseq;  // the sequence holding `row`: off[s] <= row < off[s + 1]
    while (hi - lo > 1) {
      const int64_t mid = (lo + hi) / 2;
      if (off[mid] <= row) lo = mid;
      else hi = mid;
    }
    const int64_t src = off[lo] + off[lo + 1] - 1 - row;
    y[i] = x[src * W + i % W];
  }
};

void seq_reverse(const OpRun& r, const Tensor& x, const Tensor& lod_src, const char* out_slot) {
  const bool dev = on_dev(r);
  PA_CHECK(!x.dims.empty(), "%s: empty input", r.op.type.c_str());
  const std::vector<int> off = offsets_of(lod_src, x.dims[0]);
  PA_CHECK(off.back() == x.dims[0], "%s: LoD does not match the rows", r.op.type.c_str());
  Tensor o;
  float* yp = o.alloc<float>(x.dims, place_of(r));
  o.lod = lod_src.lod;
  const int64_t W = x.dims[0] ? x.numel() / x.dims[0] : 0;
  any::run(r, dev, x.numel(), SeqReverse{f32(x, dev), yp, any::ints(r, dev, "@seq_rev_off@", off), W,
                                         (int64_t)off.size() - 1});
  set(r, out_slot, o);
}

void k_seq_reverse(const OpRun& r) { seq_reverse(r, r.in("X"), r.in("X"), "Y"); }
void k_seq_reverse_grad(const OpRun& r) {
  if (wants(r, "X@GRAD")) seq_reverse(r, r.in("Y@GRAD"), r.in("X"), "X@GRAD");
}

// sequence_scatter: Out = X; Out[i, Ids[k]] += Updates[k] for the k of sequence i
// (Ids / Updates share the LoD).  One work item per output element sums its matches
// (deterministic); Updates@GRAD[k] = g[i, Ids[k]].
struct SeqScatter {
  const float *x, *up;
  Idx ids;
  const int* off;
  float* o;
  int64_t W;
  __host__ __device__ void operator()(int64_t e) const {
    const int64_t i = e / W, c = e % W;
    float v = x[e];
    for (int64_t k = off[i]; k < off[i + 1]; ++k)
      if (ids[k] == c) v += up[k];
    o[e] = v;
  }
};
struct SeqScatterGradUp {
  const float* g;
  Idx ids;
  const int* off;
  float* du;
  int64_t W, nseq;
  __host__ __device__ void operator()(int64_t k) const {
    int64_t lo = 0, hi = nseq;
    while (hi - lo > 1) {
      const int64_t mid = (lo + hi) / 2;
      if (off[mid] <= k) lo = mid;
      else hi = mid;
    }
    const int64_t c = ids[k];
    du[k] = (c >= 0 && c < W) ? g[lo * W + c] : 0.f;
  }
};

void k_seq_scatter(const OpRun& r) {
  const bool dev = on_dev(r);
  const Tensor& x = r.in("X");
  const Tensor& ids = r.in("Ids");
  const Tensor& up = r.in("Updates");
  PA_CHECK(x.dims.size() == 2 && !ids.lod.empty(), "sequence_scatter: 2-D X and LoD Ids expected");
  const std::vector<int> off(ids.lod[0].begin(), ids.lod[0].end());
  PA_CHECK((int64_t)off.size() - 1 == x.dims[0] && up.numel() == ids.numel(), "sequence_scatter: shapes mismatch");
  Tensor o;
  float* op = o.alloc<float>(x.dims, place_of(r));
  any::run(r, dev, x.numel(), SeqScatter{f32(x, dev), f32(up, dev), idx_of(ids, dev),
                                         any::ints(r, dev, "@seq_scatter_off@", off), op, x.dims[1]});
  set(r, "Out", o);
}

void k_seq_scatter_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  const Tensor& x = r.in("X");
  const Tensor& ids = r.in("Ids");
  const Tensor& g = r.in("Out@GRAD");
  if (wants(r, "X@GRAD")) {
    Tensor d;
    any::copy(r, dev, d.alloc<float>(x.dims, place_of(r)), f32(g, dev), x.numel());
    set(r, "X@GRAD", d);
  }
  if (wants(r, "Updates@GRAD")) {
    const Tensor& up = r.in("Updates");
    const std::vector<int> off(ids.lod[0].begin(), ids.lod[0].end());
    Tensor d;
    float* du = d.alloc<float>(up.dims, place_of(r));
    d.lod = up.lod;
    any::run(r, dev, up.numel(), SeqScatterGradUp{f32(g, dev), idx_of(ids, dev),
                                                  any::ints(r, dev, "@seq_scatter_off@", off), du, x.dims[1],
                                                  (int64_t)off.size() - 1});
    set(r, "Updates@GRAD", d);
  }
}

// ---------------------------------------------------------------- kldiv_loss / bpr_loss
// kldiv_loss_op.h: l = t (log t - x) where t > 0; reduction none / sum / mean /
// batchmean (the sums reduce in fixed chunks, then one lane adds the chunks)
struct KlElem {
  const float *x, *t;
  float* l;
  __host__ __device__ void operator()(int64_t i) const {
    const float tv = t[i];
    l[i] = tv > 0.f ? tv * (logf(fmaxf(tv, 1e-30f)) - x[i]) : 0.f;
  }
};
struct SumChunk {
  const float* v;
  float* part;
  int64_t n, chunk;
  __host__ __device__ void operator()(int64_t c) const {
    float s = 0.f;
    const int64_t a = c * chunk, b = a + chunk < n ? a + chunk : n;
    for (int64_t i = a; i < b; ++i) s += v[i];
    part[c] = s;
  }
};
struct SumParts {
  const float* part;
  float* out;
  int64_t nc;
  float div;
  __host__ __device__ void operator()(int64_t) const {
    float s = 0.f;
    for (int64_t c = 0; c < nc; ++c) s += part[c];
    out[0] = s / div;
  }
};
struct KlGrad {
  const float *x, *t, *g;
  float *dx, *dt;
  int scalar;
  float div;
  __host__ __device__ void operator()(int64_t i) const {
    const float gv = (scalar ? g[0] : g[i]) / div, tv = t[i];
    if (dx) dx[i] = tv > 0.f ? -tv * gv : 0.f;
    if (dt) dt[i] = tv > 0.f ? (logf(fmaxf(tv, 1e-30f)) + 1.f - x[i]) * gv : 0.f;
  }
};

float kl_div(const OpRun& r, const Tensor& x) {
  const std::string red = r.op.GetString("reduction", "mean");
  if (red == "mean") return (float)std::max<int64_t>(1, x.numel());
  if (red == "batchmean") return (float)std::max<int64_t>(1, x.dims.empty() ? 1 : x.dims[0]);
  return 1.f;
}

void k_kldiv(const OpRun& r) {
  const bool dev = on_dev(r);
  const Tensor& x = r.in("X");
  const Tensor& t = r.in("Target");
  PA_CHECK(t.numel() == x.numel(), "kldiv_loss: Target does not match X");
  const bool none = r.op.GetString("reduction", "mean") == "none";
  Tensor o;
  std::vector<float> hl, hp;
  if (none) {
    any::run(r, dev, x.numel(), KlElem{f32(x, dev), f32(t, dev), o.alloc<float>(x.dims, place_of(r))});
  } else {
    const int64_t n = x.numel(), chunk = 4096, nc = std::max<int64_t>(1, (n + chunk - 1) / chunk);
    float* l = any::scratch(r, dev, "@kldiv_l@", n, &hl);
    float* part = any::scratch(r, dev, "@kldiv_part@", nc, &hp);
    any::run(r, dev, n, KlElem{f32(x, dev), f32(t, dev), l});
    any::run(r, dev, nc, SumChunk{l, part, n, chunk});
    any::run(r, dev, 1, SumParts{part, o.alloc<float>({1}, place_of(r)), nc, kl_div(r, x)});
  }
  set(r, "Loss", o);
}

void k_kldiv_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  const Tensor& x = r.in("X");
  const Tensor& t = r.in("Target");
  const bool none = r.op.GetString("reduction", "mean") == "none";
  Tensor dxt, dtt;
  float* dx = wants(r, "X@GRAD") ? dxt.alloc<float>(x.dims, place_of(r)) : nullptr;
  float* dt = wants(r, "Target@GRAD") ? dtt.alloc<float>(t.dims, place_of(r)) : nullptr;
  if (!dx && !dt) return;
  any::run(r, dev, x.numel(), KlGrad{f32(x, dev), f32(t, dev), f32(r.in("Loss@GRAD"), dev), dx, dt, none ? 0 : 1,
                                     none ? 1.f : kl_div(r, x)});
  if (dx) set(r, "X@GRAD", dxt);
  if (dt) set(r, "Target@GRAD", dtt);
}

// bpr_loss_op.h: Y_i = sum_{j != l_i} softplus(x_ij - x_il) / (C - 1)
__host__ __device__ inline float softplus(float v) { return fmaxf(v, 0.f) + log1pf(expf(-fabsf(v))); }
__host__ __device__ inline float sigm(float v) { return 1.f / (1.f + expf(-v)); }
struct Bpr {
  const float* x;
  Idx lab;
  float* y;
  int64_t C;
  __host__ __device__ void operator()(int64_t i) const {
    const float* xr = x + i * C;
    const int64_t l = lab[i];
    float s = 0.f;
    for (int64_t j = 0; j < C; ++j)
      if (j != l) s += softplus(xr[j] - xr[l]);
    y[i] = s / (float)(C > 1 ? C - 1 : 1);
  }
};
struct BprGrad {
  const float *x, *g;
  Idx lab;
  float* dx;
  int64_t C;
  __host__ __device__ void operator()(int64_t i) const {
    const float* xr = x + i * C;
    const int64_t l = lab[i];
    const float gv = g[i] / (float)(C > 1 ? C - 1 : 1);
    float sl = 0.f;
    for (int64_t j = 0; j < C; ++j) {
      if (j == l) continue;
      const float d = sigm(xr[j] - xr[l]) * gv;
      dx[i * C + j] = d;
      sl -= d;
    }
    if (l >= 0 && l < C) dx[i * C + l] = sl;
  }
};

void k_bpr(const OpRun& r) {
  const bool dev = on_dev(r);
  const Tensor& x = r.in("X");
  PA_CHECK(x.dims.size() == 2, "bpr_loss: 2-D X expected");
  Tensor o;
  float* yp = o.alloc<float>({x.dims[0], 1}, place_of(r));
  o.lod = x.lod;
  any::run(r, dev, x.dims[0], Bpr{f32(x, dev), idx_of(r.in("Label"), dev), yp, x.dims[1]}, 16);
  set(r, "Y", o);
}

void k_bpr_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  const Tensor& x = r.in("X");
  if (!wants(r, "X@GRAD")) return;
  Tensor d;
  float* dx = d.alloc<float>(x.dims, place_of(r));
  any::run(r, dev, x.dims[0], BprGrad{f32(x, dev), f32(r.in("Y@GRAD"), dev), idx_of(r.in("Label"), dev), dx, x.dims[1]},
           16);
  set(r, "X@GRAD", d);
}

// ---------------------------------------------------------------- shuffle_channel / scale_sub_region / size
// shuffle_channel_op.h: [N, g, C/g, H, W] -> [N, C/g, g, H, W]; the gradient is the
// inverse permutation
struct Shuffle {
  const float* x;
  float* o;
  int64_t C, HW, g, inv;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t s = i % HW, c = (i / HW) % C, n = i / (HW * C), cg = C / g;
    // forward: out channel c = j * g + k reads input channel k * cg + j
    const int64_t src = inv ? (c % cg) * g + c / cg : (c % g) * cg + c / g;
    o[i] = x[(n * C + src) * HW + s];
  }
};

void k_shuffle_channel(const OpRun& r) {
  const bool dev = on_dev(r);
  const bool grad = r.op.type == "shuffle_channel_grad";
  const Tensor& x = r.in(grad ? "Out@GRAD" : "X");
  const char* out = grad ? "X@GRAD" : "Out";
  if (grad && !wants(r, out)) return;
  PA_CHECK(x.dims.size() == 4, "shuffle_channel: NCHW input expected");
  const int64_t g = r.op.GetInt("group", 1), C = x.dims[1];
  PA_CHECK(g > 0 && C % g == 0, "shuffle_channel: group must divide the channels");
  Tensor o;
  any::run(r, dev, x.numel(), Shuffle{f32(x, dev), o.alloc<float>(x.dims, place_of(r)), C, x.dims[2] * x.dims[3], g,
                                      grad ? 1 : 0});
  set(r, out, o);
}

// scale_sub_region: X * value inside the 1-based inclusive box [c0, c1] x [h0, h1] x
// [w0, w1] of each sample (Indices [N, 6]); the gradient scales the same box
struct ScaleSub {
  const float* x;
  Idx ind;
  float* o;
  int64_t C, H, W;
  float v;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t w = i % W, h = (i / W) % H, c = (i / (W * H)) % C, n = i / (W * H * C);
    const int64_t b = n * 6;
    const bool in = c + 1 >= ind[b] && c + 1 <= ind[b + 1] && h + 1 >= ind[b + 2] && h + 1 <= ind[b + 3] &&
                    w + 1 >= ind[b + 4] && w + 1 <= ind[b + 5];
    o[i] = in ? x[i] * v : x[i];
  }
};

void k_scale_sub_region(const OpRun& r) {
  const bool dev = on_dev(r);
  const bool grad = r.op.type == "scale_sub_region_grad";
  const Tensor& x = r.in(grad ? "Out@GRAD" : "X");
  const char* out = grad ? "X@GRAD" : "Out";
  if (grad && !wants(r, out)) return;
  PA_CHECK(x.dims.size() == 4, "scale_sub_region: [N, C, H, W] input expected");
  const Tensor& ind = r.in("Indices");
  PA_CHECK(ind.numel() == x.dims[0] * 6, "scale_sub_region: Indices must be [N, 6]");
  Tensor o;
  any::run(r, dev, x.numel(), ScaleSub{f32(x, dev), idx_of(ind, dev), o.alloc<float>(x.dims, place_of(r)), x.dims[1],
                                       x.dims[2], x.dims[3], r.op.GetFloat("value", 1.f)});
  set(r, out, o);
}

struct Fill64 {
  int64_t* o;
  int64_t v;
  __host__ __device__ void operator()(int64_t) const { o[0] = v; }
};
void k_size(const OpRun& r) {
  Tensor o;
  any::run(r, on_dev(r), 1, Fill64{o.alloc<int64_t>({1}, place_of(r)), r.in("Input").numel()});
  set(r, "Out", o);
}

// ---------------------------------------------------------------- lars_momentum
// lars_momentum_op.h: local_lr = lr * coeff * |p| / (|g| + wd |p| + 1e-12);
// v' = mu v + local_lr (g + wd p); p' = p - v'
struct SqChunk {
  const float *a, *b;
  float* part;  // [2, nc]
  int64_t n, chunk, nc;
  __host__ __device__ void operator()(int64_t c) const {
    float sa = 0.f, sb = 0.f;
    const int64_t lo = c * chunk, hi = lo + chunk < n ? lo + chunk : n;
    for (int64_t i = lo; i < hi; ++i) {
      sa += a[i] * a[i];
      sb += b[i] * b[i];
    }
    part[c] = sa;
    part[nc + c] = sb;
  }
};
struct LarsLocal {
  const float *part, *lr;
  float* local;
  int64_t nc;
  float coeff, wd;
  __host__ __device__ void operator()(int64_t) const {
    float sp = 0.f, sg = 0.f;
    for (int64_t c = 0; c < nc; ++c) {
      sp += part[c];
      sg += part[nc + c];
    }
    const float pn = sqrtf(sp), gn = sqrtf(sg);
    local[0] = lr[0] * coeff * pn / (gn + wd * pn + 1e-12f);
  }
};
struct LarsUpdate {
  const float *p, *g, *v, *local;
  float *po, *vo;
  float mu, wd;
  __host__ __device__ void operator()(int64_t i) const {
    const float nv = mu * v[i] + local[0] * (g[i] + wd * p[i]);
    vo[i] = nv;
    po[i] = p[i] - nv;
  }
};

void k_lars_momentum(const OpRun& r) {
  const bool dev = on_dev(r);
  const Tensor& p = r.in("Param");
  const Tensor& g = r.in("Grad");
  const Tensor& v = r.in("Velocity");
  PA_CHECK(g.numel() == p.numel() && v.numel() == p.numel(), "lars_momentum: Grad / Velocity must match Param");
  const int64_t n = p.numel(), chunk = 4096, nc = std::max<int64_t>(1, (n + chunk - 1) / chunk);
  std::vector<float> hp, hl;
  float* part = any::scratch(r, dev, "@lars_part@", 2 * nc, &hp);
  float* local = any::scratch(r, dev, "@lars_local@", 1, &hl);
  const float wd = r.op.GetFloat("lars_weight_decay", 0.0005f);
  any::run(r, dev, nc, SqChunk{f32(p, dev), f32(g, dev), part, n, chunk, nc});
  any::run(r, dev, 1, LarsLocal{part, f32(r.in("LearningRate"), dev), local, nc, r.op.GetFloat("lars_coeff", 0.001f), wd});
  Tensor po, vo;
  any::run(r, dev, n, LarsUpdate{f32(p, dev), f32(g, dev), f32(v, dev), local, po.alloc<float>(p.dims, place_of(r)),
                                 vo.alloc<float>(v.dims, place_of(r)), r.op.GetFloat("mu", 0.9f), wd});
  set(r, "ParamOut", po);
  set(r, "VelocityOut", vo);
}

// ---------------------------------------------------------------- max_pool3d_with_index
// pooling_op.h MaxPool3dWithIndexFunctor: the window's first maximum and its flat
// index inside the [D, H, W] volume; the gradient scatters back through that index
__host__ __device__ inline void acc_add(float* p, float v) {
#if defined(__HIP_DEVICE_COMPILE__)
  atomicAdd(p, v);
#else
  *p += v;
#endif
}
struct MaxPool3Idx {
  const float* x;
  float* o;
  int32_t* mask;
  int64_t in[3], out[3], k[3], st[3], pd[3];
  __host__ __device__ void operator()(int64_t t) const {
    const int64_t ow = t % out[2], oh = (t / out[2]) % out[1], od = (t / (out[2] * out[1])) % out[0],
                  plane = t / (out[0] * out[1] * out[2]);
    const float* p = x + plane * in[0] * in[1] * in[2];
    float best = -INFINITY;
    int64_t bi = -1;
    for (int64_t a = 0; a < k[0]; ++a)
      for (int64_t b = 0; b < k[1]; ++b)
        for (int64_t c = 0; c < k[2]; ++c) {
          const int64_t d = od * st[0] - pd[0] + a, h = oh * st[1] - pd[1] + b, w = ow * st[2] - pd[2] + c;
          if (d < 0 || d >= in[0] || h < 0 || h >= in[1] || w < 0 || w >= in[2]) continue;
          const int64_t at = (d * in[1] + h) * in[2] + w;
          if (bi < 0 || p[at] > best) {
            best = p[at];
            bi = at;
          }
        }
    o[t] = best;
    mask[t] = (int32_t)bi;
  }
};
struct MaxPool3IdxGrad {
  const float* g;
  const int32_t* mask;
  float* dx;
  int64_t I, O;
  __host__ __device__ void operator()(int64_t t) const {
    if (mask[t] >= 0) acc_add(dx + (t / O) * I + mask[t], g[t]);
  }
};

MaxPool3Idx pool3_idx_geo(const OpRun& r, const Tensor& x) {
  PA_CHECK(x.dims.size() == 5, "max_pool3d_with_index: NCDHW input expected");
  auto k = r.op.GetInts("ksize"), st = r.op.GetInts("strides"), pd = r.op.GetInts("paddings");
  if (k.size() != 3 || st.size() != 3 || pd.size() != 3) throw Decline{};
  MaxPool3Idx g{};
  for (int i = 0; i < 3; ++i) {
    g.in[i] = x.dims[(size_t)i + 2];
    g.k[i] = r.op.GetBool("global_pooling") ? g.in[i] : k[(size_t)i];
    g.st[i] = st[(size_t)i];
    g.pd[i] = r.op.GetBool("global_pooling") ? 0 : pd[(size_t)i];
    g.out[i] = (g.in[i] + 2 * g.pd[i] - g.k[i]) / g.st[i] + 1;
    PA_CHECK(g.out[i] > 0, "max_pool3d_with_index: empty output");
  }
  return g;
}

void k_max_pool3d_idx(const OpRun& r) {
  const bool dev = on_dev(r);
  const Tensor& x = r.in("X");
  MaxPool3Idx g = pool3_idx_geo(r, x);
  const Dims od = {x.dims[0], x.dims[1], g.out[0], g.out[1], g.out[2]};
  Tensor o, m;
  g.x = f32(x, dev);
  g.o = o.alloc<float>(od, place_of(r));
  g.mask = static_cast<int32_t*>(m.alloc(DT::INT32, od, place_of(r)));
  any::run(r, dev, o.numel(), g);
  set(r, "Out", o);
  set(r, "Mask", m);
}

void k_max_pool3d_idx_grad(const OpRun& r) {
  const bool dev = on_dev(r);
  const Tensor& x = r.in("X");
  const Tensor& m = r.in("Mask");
  const Tensor& g = r.in("Out@GRAD");
  if (m.dtype != DT::INT32 || (m.device >= 0) != dev || !wants(r, "X@GRAD")) {
    if (!wants(r, "X@GRAD")) return;
    throw Decline{};
  }
  Tensor d;
  float* dx = d.alloc<float>(x.dims, place_of(r));
  any::zero(r, dev, dx, x.numel());
  const int64_t I = x.dims[2] * x.dims[3] * x.dims[4], O = g.dims[2] * g.dims[3] * g.dims[4];
  any::run(r, dev, g.numel(), MaxPool3IdxGrad{f32(g, dev), m.data<int32_t>(), dx, I, O}, 1 << 30);
  set(r, "X@GRAD", d);
}

// ---------------------------------------------------------------- chunk_eval
// chunk_eval_op.h: chunks (begin, end, type) of every sequence under the IOB / IOE /
// IOBES / plain tagging scheme (label = tag + n_tags * type, type == num_chunk_types
// is "outside"), excluded types dropped; counts of inferred, labelled and matching
// chunks, then precision / recall / F1.  One work item per sequence; the chunks of
// the inference are listed in a per-sequence scratch and matched by a merge (both
// lists come out ordered by begin).
struct ChunkScheme {
  int64_t ntag, tb, ti, te, ts, other;
  const int* excl;
  int nexcl;
  __host__ __device__ bool ends(int64_t pt, int64_t pty, int64_t t, int64_t ty) const {
    if (pty == other) return false;
    if (ty == other || ty != pty) return true;
    if (pt == tb || pt == ti) return t == tb || t == ts;
    return pt == te || pt == ts;
  }
  __host__ __device__ bool begins(int64_t pt, int64_t pty, int64_t t, int64_t ty) const {
    if (pty == other) return ty != other;
    if (ty == other) return false;
    if (ty != pty || t == tb || t == ts) return true;
    if (t == ti || t == te) return pt == te || pt == ts;
    return false;
  }
  __host__ __device__ bool kept(int64_t ty) const {
    for (int k = 0; k < nexcl; ++k)
      if (excl[k] == ty) return false;
    return true;
  }
  // calls emit(begin, end, type) for every kept chunk of labels[a, b)
  template <class E>
  __host__ __device__ void scan(Idx v, int64_t a, int64_t b, E& emit) const {
    int64_t tag = -1, typ = other, start = 0;
    bool inside = false;
    for (int64_t i = a; i < b; ++i) {
      const int64_t pt = tag, pty = typ, lab = v[i];
      tag = lab % ntag;
      typ = lab / ntag;
      if (inside && ends(pt, pty, tag, typ)) {
        if (kept(pty)) emit(start, i - 1, pty);
        inside = false;
      }
      if (begins(pt, pty, tag, typ)) {
        start = i;
        inside = true;
      }
    }
    if (inside && kept(typ)) emit(start, b - 1, typ);
  }
};
struct ChunkList {
  int64_t* buf;
  int64_t n;
  __host__ __device__ void operator()(int64_t s, int64_t e, int64_t t) {
    buf[3 * n] = s;
    buf[3 * n + 1] = e;
    buf[3 * n + 2] = t;
    ++n;
  }
};
struct ChunkMatch {
  const int64_t* buf;
  int64_t n, k, nl, nc;
  __host__ __device__ void operator()(int64_t s, int64_t e, int64_t t) {
    ++nl;
    while (k < n && buf[3 * k] < s) ++k;
    if (k < n && buf[3 * k] == s && buf[3 * k + 1] == e && buf[3 * k + 2] == t) ++nc;
  }
};
struct ChunkSeq {
  Idx inf, lab;
  const int* off;
  int64_t* scratch;  // 3 per token
  int64_t* counts;   // [nseq, 3]
  ChunkScheme sc;
  __host__ __device__ void operator()(int64_t q) const {
    const int64_t a = off[q], b = off[q + 1];
    ChunkList li{scratch + 3 * a, 0};
    sc.scan(inf, a, b, li);
    ChunkMatch m{li.buf, li.n, 0, 0, 0};
    sc.scan(lab, a, b, m);
    counts[3 * q] = li.n;
    counts[3 * q + 1] = m.nl;
    counts[3 * q + 2] = m.nc;
  }
};
struct ChunkTotals {
  const int64_t* counts;
  int64_t nseq;
  float *p, *rc, *f1;
  int64_t *ni, *nl, *nc;
  __host__ __device__ void operator()(int64_t) const {
    int64_t a = 0, b = 0, c = 0;
    for (int64_t q = 0; q < nseq; ++q) {
      a += counts[3 * q];
      b += counts[3 * q + 1];
      c += counts[3 * q + 2];
    }
    const double pr = a ? (double)c / (double)a : 0.0, re = b ? (double)c / (double)b : 0.0;
    p[0] = (float)pr;
    rc[0] = (float)re;
    f1[0] = c ? (float)(2.0 * pr * re / (pr + re)) : 0.f;
    ni[0] = a;
    nl[0] = b;
    nc[0] = c;
  }
};

void k_chunk_eval(const OpRun& r) {
  const bool dev = on_dev(r);
  const Tensor& inf = r.in("Inference");
  const Tensor& lab = r.in("Label");
  PA_CHECK(inf.numel() == lab.numel(), "chunk_eval: Inference does not match Label");
  const std::vector<int> off = offsets_of(lab, lab.numel());
  const int64_t nseq = (int64_t)off.size() - 1;
  const std::string scheme = r.op.GetString("chunk_scheme", "IOB");
  ChunkScheme sc;
  if (scheme == "IOB") sc = {2, 0, 1, -1, -1, 0, nullptr, 0};
  else if (scheme == "IOE") sc = {2, -1, 0, 1, -1, 0, nullptr, 0};
  else if (scheme == "IOBES") sc = {4, 0, 1, 2, 3, 0, nullptr, 0};
  else if (scheme == "plain") sc = {1, -1, -1, -1, -1, 0, nullptr, 0};
  else PA_CHECK(false, "chunk_eval: unknown chunk_scheme %s", scheme.c_str());
  sc.other = r.op.GetInt("num_chunk_types", 1);
  std::vector<int> excl;
  for (int64_t t : r.op.GetInts("excluded_chunk_types")) excl.push_back((int)t);
  sc.excl = any::ints(r, dev, "@chunk_excl@", excl);
  sc.nexcl = (int)excl.size();
  Tensor work, cnt;
  int64_t* wp = work.alloc<int64_t>({std::max<int64_t>(1, 3 * inf.numel())}, place_of(r));
  int64_t* cp = cnt.alloc<int64_t>({std::max<int64_t>(1, 3 * nseq)}, place_of(r));
  any::run(r, dev, nseq, ChunkSeq{idx_of(inf, dev), idx_of(lab, dev), any::ints(r, dev, "@chunk_off@", off), wp, cp, sc},
           1);
  Tensor pt, rt, ft, it, lt, ct;
  any::run(r, dev, 1, ChunkTotals{cp, nseq, pt.alloc<float>({1}, place_of(r)), rt.alloc<float>({1}, place_of(r)),
                                  ft.alloc<float>({1}, place_of(r)), it.alloc<int64_t>({1}, place_of(r)),
                                  lt.alloc<int64_t>({1}, place_of(r)), ct.alloc<int64_t>({1}, place_of(r))});
  set(r, "Precision", pt);
  set(r, "Recall", rt);
  set(r, "F1-Score", ft);
  set(r, "NumInferChunks", it);
  set(r, "NumLabelChunks", lt);
  set(r, "NumCorrectChunks", ct);
}

// ---------------------------------------------------------------- sampling_id / random_crop
// sampling_id_op.h: per row, the first column whose running probability sum reaches a
// uniform draw in [min, max) (draws from the executor's RNG, or `seed`)
struct SampleRow {
  const float *x, *u;
  int64_t* o;
  int64_t C;
  __host__ __device__ void operator()(int64_t i) const {
    float s = 0.f;
    int64_t pick = C - 1;
    for (int64_t j = 0; j < C; ++j) {
      s += x[i * C + j];
      if (s >= u[i]) {
        pick = j;
        break;
      }
    }
    o[i] = pick;
  }
};

void k_sampling_id(const OpRun& r) {
  const bool dev = on_dev(r);
  const Tensor& x = r.in("X");
  PA_CHECK(x.dims.size() == 2, "sampling_id: 2-D X expected");
  const int64_t N = x.dims[0], seed = r.op.GetInt("seed");
  std::mt19937_64 g(seed ? (uint64_t)seed : r.ctx.rng());
  std::uniform_real_distribution<float> d(r.op.GetFloat("min", 0.f), r.op.GetFloat("max", 1.f));
  std::vector<int> u((size_t)N);
  for (auto& v : u) {
    const float f = d(g);
    memcpy(&v, &f, sizeof(float));
  }
  Tensor o;
  any::run(r, dev, N, SampleRow{f32(x, dev), (const float*)any::ints(r, dev, "@sampling_u@", u),
                                o.alloc<int64_t>({N}, place_of(r)), x.dims[1]}, 64);
  set(r, "Out", o);
}

// random_crop_op.h: a random window of `shape` over the trailing dims of every
// instance (offsets from the executor's RNG); SeedOut carries the seed on
struct CropND {
  const float* x;
  float* o;
  int R;
  int64_t xd[8], od[8], st[8];
  __host__ __device__ void operator()(int64_t i) const {
    int64_t src = 0, mul = 1, rem = i;
    for (int d = R - 1; d >= 0; --d) {
      const int64_t c = rem % od[d];
      rem /= od[d];
      src += (c + st[d]) * mul;
      mul *= xd[d];
    }
    o[i] = x[src];
  }
};

void k_random_crop(const OpRun& r) {
  const bool dev = on_dev(r);
  const Tensor& x = r.in("X");
  const auto shape = r.op.GetInts("shape");
  const int R = (int)x.dims.size(), k = (int)shape.size();
  PA_CHECK(R <= 8 && k <= R, "random_crop: shape longer than X");
  CropND f{};
  f.x = f32(x, dev);
  f.R = R;
  Dims od = x.dims;
  for (int d = 0; d < R; ++d) {
    f.xd[d] = x.dims[(size_t)d];
    f.st[d] = 0;
  }
  for (int i = 0; i < k; ++i) {
    const int d = R - k + i;
    PA_CHECK(shape[(size_t)i] <= x.dims[(size_t)d], "random_crop: crop larger than X");
    od[(size_t)d] = shape[(size_t)i];
    std::uniform_int_distribution<int64_t> u(0, x.dims[(size_t)d] - shape[(size_t)i]);
    f.st[d] = u(r.ctx.rng);
  }
  for (int d = 0; d < R; ++d) f.od[d] = od[(size_t)d];
  Tensor o;
  f.o = o.alloc<float>(od, place_of(r));
  any::run(r, dev, o.numel(), f);
  set(r, "Out", o);
  if (Tensor* so = r.out("SeedOut")) *so = r.in("Seed");
}

// ---------------------------------------------------------------- print
// print_op.cc: message, name, shape, LoD and the first `summarize` values of In
// (a host copy on a HIP place); Out shares In
void k_print(const OpRun& r) {
  const Tensor& in = r.in("In");
  const Tensor h = in.device >= 0 ? in.to(-1, r.ctx.stream) : in;
  int64_t n = h.numel();
  const int64_t lim = r.op.GetInt("summarize", -1);
  if (lim > 0 && lim < n) n = lim;
  std::string s = r.op.GetString("message") + " " + r.op.Input("In") + " shape=" + in.shape_str() + " data=[";
  char buf[64];
  for (int64_t i = 0; i < n; ++i) {
    switch (h.dtype) {
      case DT::FP32: snprintf(buf, sizeof buf, "%g", (double)h.data<float>()[i]); break;
      case DT::FP64: snprintf(buf, sizeof buf, "%g", h.data<double>()[i]); break;
      case DT::INT64: snprintf(buf, sizeof buf, "%lld", (long long)h.data<int64_t>()[i]); break;
      case DT::INT32: snprintf(buf, sizeof buf, "%d", h.data<int32_t>()[i]); break;
      default: snprintf(buf, sizeof buf, "?"); break;
    }
    s += (i ? ", " : "") + std::string(buf);
  }
  printf("%s]\n", s.c_str());
  fflush(stdout);
  if (Tensor* o = r.out("Out")) *o = in;
}

// ---------------------------------------------------------------- multiclass_nms / mine_hard_examples
// Variable-length outputs decided by sequential greedy loops: the reference runs
// both on the CPU only (multiclass_nms_op.cc, mine_hard_examples_op.cc).  Here the
// host computes them; on a HIP place the (small) inputs are staged to the host on
// the op's stream and the result is uploaded back.
Tensor host_view(const OpRun& r, const Tensor& t) { return t.device >= 0 ? t.to(-1, r.ctx.stream) : t; }
void put(const OpRun& r, const char* slot, Tensor h, const LoD& lod) {
  Tensor o = on_dev(r) ? h.to(r.ctx.device, r.ctx.stream) : h;
  o.lod = lod;
  set(r, slot, o);
}

float box_iou(const float* a, const float* b, bool norm) {
  const float one = norm ? 0.f : 1.f;
  const float aa = (a[2] - a[0] + one) * (a[3] - a[1] + one), ab = (b[2] - b[0] + one) * (b[3] - b[1] + one);
  const float w = std::max(std::min(a[2], b[2]) - std::max(a[0], b[0]) + one, 0.f);
  const float h = std::max(std::min(a[3], b[3]) - std::max(a[1], b[1]) + one, 0.f);
  const float inter = w * h;
  return inter / std::max(aa + ab - inter, 1e-10f);
}

// multiclass_nms: per image and non-background class, greedy NMS over the boxes
// scoring above score_threshold (nms_top_k best first, adaptive threshold with
// nms_eta); the image's detections [label, score, x0, y0, x1, y1] sorted by score,
// keep_top_k kept; one row of -1 when nothing survives anywhere
void k_multiclass_nms(const OpRun& r) {
  const Tensor bt = host_view(r, r.in("BBoxes"));
  const Tensor st = host_view(r, r.in("Scores"));
  PA_CHECK(st.dims.size() == 3 && bt.dims.size() == 3 && bt.dims[2] == 4, "multiclass_nms: [N, C, M] scores and "
           "[N, M, 4] boxes expected");
  if (r.ctx.device >= 0) PA_HIPCHK(hipStreamSynchronize((hipStream_t)r.ctx.stream));
  const float* boxes = f32(bt, false);
  const float* scores = f32(st, false);
  const int64_t N = st.dims[0], C = st.dims[1], M = st.dims[2];
  const int64_t bg = r.op.GetInt("background_label", 0), top_k = r.op.GetInt("nms_top_k", 400),
                keep_k = r.op.GetInt("keep_top_k", 200);
  const float sthr = r.op.GetFloat("score_threshold", 0.01f), nthr = r.op.GetFloat("nms_threshold", 0.3f),
              eta = r.op.GetFloat("nms_eta", 1.f);
  const bool norm = r.op.GetBool("normalized", true);
  std::vector<float> rows;
  std::vector<size_t> off = {0};
  for (int64_t b = 0; b < N; ++b) {
    struct Det {
      float c, s;
      int64_t i;
    };
    std::vector<Det> dets;
    const float* bb = boxes + b * M * 4;
    for (int64_t c = 0; c < C; ++c) {
      if (c == bg) continue;
      const float* sc = scores + (b * C + c) * M;
      std::vector<int64_t> order;
      for (int64_t m = 0; m < M; ++m)
        if (sc[m] > sthr) order.push_back(m);
      std::stable_sort(order.begin(), order.end(), [&](int64_t u, int64_t v) { return sc[u] > sc[v]; });
      if (top_k > -1 && (int64_t)order.size() > top_k) order.resize((size_t)top_k);
      float adaptive = nthr;
      std::vector<int64_t> kept;
      for (size_t q = 0; q < order.size(); ++q) {
        const int64_t i = order[q];
        bool ok = true;
        for (int64_t j : kept)
          if (box_iou(bb + i * 4, bb + j * 4, norm) > adaptive) {
            ok = false;
            break;
          }
        if (!ok) continue;
        kept.push_back(i);
        if (eta < 1.f && adaptive > 0.5f) adaptive *= eta;
      }
      for (int64_t i : kept) dets.push_back({(float)c, sc[i], i});
    }
    std::stable_sort(dets.begin(), dets.end(), [](const Det& u, const Det& v) { return u.s > v.s; });
    if (keep_k > -1 && (int64_t)dets.size() > keep_k) dets.resize((size_t)keep_k);
    for (const Det& d : dets) {
      rows.push_back(d.c);
      rows.push_back(d.s);
      for (int k = 0; k < 4; ++k) rows.push_back(bb[d.i * 4 + k]);
    }
    off.push_back(rows.size() / 6);
  }
  if (rows.empty()) {
    rows.assign(6, -1.f);
    off = {0, 1};
  }
  Tensor h;
  memcpy(h.alloc<float>({(int64_t)rows.size() / 6, 6}, -1), rows.data(), rows.size() * sizeof(float));
  put(r, "Out", h, {off});
}

// mine_hard_examples: max_negative takes, per image, the unmatched priors under
// neg_dist_threshold with the largest classification loss, neg_pos_ratio per
// positive; hard_example takes the sample_size largest (cls + loc) losses and unmatches
// the positives left out.  NegIndices (LoD per image, ascending) and the updated
// match indices
void k_mine_hard_examples(const OpRun& r) {
  const Tensor cl = host_view(r, r.in("ClsLoss"));
  Tensor* locp = r.in_opt("LocLoss");
  const Tensor loc = locp ? host_view(r, *locp) : Tensor();
  const Tensor mi0 = host_view(r, r.in("MatchIndices"));
  const Tensor md = host_view(r, r.in("MatchDist"));
  if (r.ctx.device >= 0) PA_HIPCHK(hipStreamSynchronize((hipStream_t)r.ctx.stream));
  PA_CHECK(mi0.dims.size() == 2, "mine_hard_examples: [N, P] MatchIndices expected");
  const int64_t N = mi0.dims[0], P = mi0.dims[1];
  const float* cls = f32(cl, false);
  const float* lp = locp ? f32(loc, false) : nullptr;
  const float* dist = f32(md, false);
  const Idx mi = idx_of(mi0, false);
  const std::string kind = r.op.GetString("mining_type", "max_negative");
  const float ratio = r.op.GetFloat("neg_pos_ratio", 1.f), dthr = r.op.GetFloat("neg_dist_threshold", 0.5f);
  const int64_t sample = r.op.GetInt("sample_size", 0);
  Tensor upd;
  int32_t* up = static_cast<int32_t*>(upd.alloc(DT::INT32, {N, P}, -1));
  for (int64_t k = 0; k < N * P; ++k) up[k] = (int32_t)mi[k];
  std::vector<int32_t> negs;
  std::vector<size_t> off = {0};
  for (int64_t b = 0; b < N; ++b) {
    std::vector<float> loss((size_t)P);
    for (int64_t p = 0; p < P; ++p)
      loss[(size_t)p] = cls[b * P + p] + ((lp && kind == "hard_example") ? lp[b * P + p] : 0.f);
    std::vector<int64_t> cand;
    int64_t k;
    if (kind == "max_negative") {
      int64_t npos = 0;
      for (int64_t p = 0; p < P; ++p) {
        if (up[b * P + p] >= 0) ++npos;
        else if (dist[b * P + p] < dthr) cand.push_back(p);
      }
      k = std::min<int64_t>((int64_t)((float)npos * ratio), (int64_t)cand.size());
    } else {
      for (int64_t p = 0; p < P; ++p) cand.push_back(p);
      k = std::min<int64_t>(sample, P);
    }
    std::stable_sort(cand.begin(), cand.end(), [&](int64_t u, int64_t v) { return loss[(size_t)u] > loss[(size_t)v]; });
    cand.resize((size_t)std::max<int64_t>(k, 0));
    std::sort(cand.begin(), cand.end());
    if (kind == "hard_example") {
      std::vector<char> keep((size_t)P, 0);
      for (int64_t p : cand) keep[(size_t)p] = 1;
      for (int64_t p = 0; p < P; ++p)
        if (up[b * P + p] >= 0 && !keep[(size_t)p]) up[b * P + p] = -1;
      std::vector<int64_t> neg;
      for (int64_t p : cand)
        if (up[b * P + p] < 0) neg.push_back(p);
      cand.swap(neg);
    }
    for (int64_t p : cand) negs.push_back((int32_t)p);
    off.push_back(negs.size());
  }
  Tensor nt;
  int32_t* np_ = static_cast<int32_t*>(nt.alloc(DT::INT32, {(int64_t)negs.size(), 1}, -1));
  if (!negs.empty()) memcpy(np_, negs.data(), negs.size() * sizeof(int32_t));
  put(r, "NegIndices", nt, {off});
  put(r, "UpdatedMatchIndices", upd, {});
}

// ---------------------------------------------------------------- fusion_lstm / fusion_gru
// fusion_{lstm,gru}_op.cc: XX = X WeightX (+ Bias for the GRU) in one GEMM over all
// time steps, then the recurrence of lstm / gru over XX with WeightH.  The recurrence
// is the registered lstm / gru kernel of this place, run on a derived op desc (same
// scope, same stream): XX lands in the XX output (or a scope temporary), the
// recurrence writes Hidden (and Cell).
void k_fusion_rnn(const OpRun& r) {
  const bool dev = on_dev(r);
  const bool gru = r.op.type == "fusion_gru";
  const Tensor& x = r.in("X");
  const Tensor& wx = r.in("WeightX");
  PA_CHECK(x.dims.size() == 2 && wx.dims.size() == 2 && wx.dims[0] == x.dims[1], "%s: X [T, M], WeightX [M, G]",
           r.op.type.c_str());
  const int64_t T = x.dims[0], M = x.dims[1], G = wx.dims[1];
  std::string xx_name = r.op.Output("XX");
  if (xx_name.empty()) xx_name = r.op.Output("Hidden") + "@fusion_xx";
  Tensor& xx = r.scope.Var(xx_name)->tensor;
  float* xp = xx.alloc<float>({T, G}, place_of(r));
  any::gemm(r, dev, false, false, T, G, M, 1.f, f32(x, dev), M, f32(wx, dev), G, 0.f, xp, G);
  Tensor* bias = r.in_opt("Bias");
  if (gru && bias) {
    PA_CHECK(bias->numel() == G, "fusion_gru: Bias must be [1, 3D]");
    any::run(r, dev, T * G, FusedFwd{xp, f32(*bias, dev), xp, nullptr, FusedGeo{G, 1, 1, 0, 0, 1.f}});
  }
  xx.lod = x.lod;
  OpDesc sub;
  sub.type = gru ? "gru" : "lstm";
  auto pass = [&](const char* from, const char* to, std::vector<std::pair<std::string, std::vector<std::string>>>& v,
                  bool input) {
    const auto& names = input ? r.op.Inputs(from) : r.op.Outputs(from);
    if (!names.empty()) v.push_back({to, names});
  };
  sub.inputs.push_back({"Input", {xx_name}});
  pass("H0", "H0", sub.inputs, true);
  pass("WeightH", "Weight", sub.inputs, true);
  if (!gru) {
    pass("C0", "C0", sub.inputs, true);
    pass("Bias", "Bias", sub.inputs, true);
    pass("Cell", "Cell", sub.outputs, false);
  }
  pass("Hidden", "Hidden", sub.outputs, false);
  sub.attrs = r.op.attrs;
  const Kernel* k = find_kernel(sub.type, dev);
  if (!k) throw Decline{};
  (*k)(OpRun{sub, r.scope, r.ctx});
}

// ---------------------------------------------------------------- fusion_seqexpand_concat_fc
// fusion_seqexpand_concat_fc_op.cc: X[0] [T, M0] carries the sequences, X[k>0] [N,
// Mk] one row per sequence expanded over its steps; FCOut = concat(...) FCWeight (+
// FCBias), Out = act(FCOut) with act in identity / relu / sigmoid / tanh
struct ExpandConcat {
  const float* const* xs;  // device / host array of the inputs
  const int* widths;       // Mk, prefix-summed: [0, M0, M0 + M1, ...]
  const int* off;          // sequence offsets of X[0]
  float* o;
  int64_t nx, nseq, W;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t t = i / W, c = i % W;
    int64_t k = 0;
    while (k + 1 < nx && widths[k + 1] <= c) ++k;
    const int64_t col = c - widths[k], mk = widths[k + 1] - widths[k];
    if (k == 0) {
      o[i] = xs[0][t * mk + col];
      return;
    }
    int64_t lo = 0, hi = nseq;
    while (hi - lo > 1) {
      const int64_t mid = (lo + hi) / 2;
      if (off[mid] <= t) lo = mid;
      else hi = mid;
    }
    o[i] = xs[k][lo * mk + col];
  }
};
struct BiasAct {
  const float* b;
  float *fc, *out;
  int64_t N;
  int act;  // 0 identity 1 relu 2 sigmoid 3 tanh
  __host__ __device__ void operator()(int64_t i) const {
    float v = fc[i] + (b ? b[i % N] : 0.f);
    fc[i] = v;
    out[i] = act == 1 ? fmaxf(v, 0.f) : act == 2 ? 1.f / (1.f + expf(-v)) : act == 3 ? tanhf(v) : v;
  }
};

void k_seqexpand_concat_fc(const OpRun& r) {
  const bool dev = on_dev(r);
  const std::vector<Tensor*> xs = r.ins("X");
  PA_CHECK(!xs.empty() && xs[0]->dims.size() == 2, "fusion_seqexpand_concat_fc: 2-D X[0] expected");
  const int64_t T = xs[0]->dims[0];
  const std::vector<int> off = offsets_of(*xs[0], T);
  const int64_t nseq = (int64_t)off.size() - 1;
  std::vector<int> widths = {0};
  std::vector<int> ptrs;  // the input pointers, as int pairs for the upload helper
  for (size_t k = 0; k < xs.size(); ++k) {
    PA_CHECK(xs[k]->dims.size() == 2 && (k == 0 || xs[k]->dims[0] == nseq),
             "fusion_seqexpand_concat_fc: X[%d] must have one row per sequence", (int)k);
    widths.push_back(widths.back() + (int)xs[k]->dims[1]);
    const float* p = f32(*xs[k], dev);
    int pair[2];
    memcpy(pair, &p, sizeof(p));
    ptrs.push_back(pair[0]);
    ptrs.push_back(pair[1]);
  }
  const int64_t W = widths.back();
  const Tensor& w = r.in("FCWeight");
  PA_CHECK(w.dims.size() == 2 && w.dims[0] == W, "fusion_seqexpand_concat_fc: FCWeight must be [sum M, N]");
  const int64_t N = w.dims[1];
  std::vector<float> hcat;
  float* cat = any::scratch(r, dev, "@seqexpand_cat@", T * W, &hcat);
  any::run(r, dev, T * W, ExpandConcat{(const float* const*)any::ints(r, dev, "@seqexpand_ptrs@", ptrs),
                                       any::ints(r, dev, "@seqexpand_w@", widths),
                                       any::ints(r, dev, "@seqexpand_off@", off), cat, (int64_t)xs.size(), nseq, W});
  Tensor fc, out;
  float* fp = fc.alloc<float>({T, N}, place_of(r));
  float* op = out.alloc<float>({T, N}, place_of(r));
  any::gemm(r, dev, false, false, T, N, W, 1.f, cat, W, f32(w, dev), N, 0.f, fp, N);
  const std::string a = r.op.GetString("fc_activation", "identity");
  const int act = a == "relu" ? 1 : a == "sigmoid" ? 2 : a == "tanh" ? 3 : 0;
  PA_CHECK(act || a == "identity" || a.empty(), "fusion_seqexpand_concat_fc: activation %s", a.c_str());
  Tensor* b = r.in_opt("FCBias");
  any::run(r, dev, T * N, BiasAct{b ? f32(*b, dev) : nullptr, fp, op, N, act});
  out.lod = xs[0]->lod;
  set(r, "FCOut", fc);
  set(r, "Out", out);
}

// ---------------------------------------------------------------- detection_map
// detection_map_op.h (VOC mAP): per image and class, detections by descending score
// claim the unused ground truth of best IoU >= overlap_threshold (difficult ground
// truth skipped unless evaluate_difficult); per class AP from the cumulative TP / FP
// curve ("integral" or "11point"), MAP their mean over non-background classes with
// positives.  Outputs the per-class positive counts and the (score, tp) / (score, fp)
// records.  Host loops as the reference's CPU kernel; staged through the host on a HIP
// place.
double iou_plain(const double* a, const double* b) {
  const double ix = std::max(0.0, std::min(a[2], b[2]) - std::max(a[0], b[0]));
  const double iy = std::max(0.0, std::min(a[3], b[3]) - std::max(a[1], b[1]));
  const double inter = ix * iy;
  const double ua = (a[2] - a[0]) * (a[3] - a[1]) + (b[2] - b[0]) * (b[3] - b[1]) - inter;
  return ua > 0 ? inter / ua : 0.0;
}

void k_detection_map(const OpRun& r) {
  const Tensor dt = host_view(r, r.in("DetectRes"));
  const Tensor gt = host_view(r, r.in("Label"));
  if (r.ctx.device >= 0) PA_HIPCHK(hipStreamSynchronize((hipStream_t)r.ctx.stream));
  PA_CHECK(dt.dims.size() == 2 && dt.dims[1] == 6 && gt.dims.size() == 2 && (gt.dims[1] == 5 || gt.dims[1] == 6),
           "detection_map: DetectRes [D, 6] and Label [G, 5 or 6] expected");
  const float* det = f32(dt, false);
  const float* lab = f32(gt, false);
  const int64_t GW = gt.dims[1];
  const bool has_diff = GW == 6, eval_diff = r.op.GetBool("evaluate_difficult", true);
  const double thr = r.op.GetFloat("overlap_threshold", 0.5f);
  const int64_t bg = r.op.GetInt("background_label", 0);
  const std::vector<int> doff = offsets_of(dt, dt.dims[0]), goff = offsets_of(gt, gt.dims[0]);
  std::map<int64_t, int64_t> pos;
  std::map<int64_t, std::vector<std::pair<double, int>>> rec;
  for (size_t i = 0; i + 1 < goff.size(); ++i) {
    const int64_t g0 = goff[i], g1 = goff[i + 1];
    const int64_t d0 = i + 1 < doff.size() ? doff[i] : 0, d1 = i + 1 < doff.size() ? doff[i + 1] : 0;
    for (int64_t g = g0; g < g1; ++g) {
      const bool diff = has_diff && lab[g * GW + 1] != 0.f;
      if (eval_diff || !diff) ++pos[(int64_t)lab[g * GW]];
    }
    std::map<int64_t, std::vector<int64_t>> by_class;
    for (int64_t d = d0; d < d1; ++d) by_class[(int64_t)det[d * 6]].push_back(d);
    for (auto& kv : by_class) {
      const int64_t c = kv.first;
      std::vector<int64_t>& ds = kv.second;
      std::stable_sort(ds.begin(), ds.end(), [&](int64_t a, int64_t b) { return det[a * 6 + 1] > det[b * 6 + 1]; });
      std::vector<int64_t> gs;
      for (int64_t g = g0; g < g1; ++g)
        if ((int64_t)lab[g * GW] == c) gs.push_back(g);
      std::vector<char> used(gs.size(), 0);
      for (int64_t d : ds) {
        double box[4], best = -1.0;
        for (int k = 0; k < 4; ++k) box[k] = det[d * 6 + 2 + k];
        int64_t bj = -1;
        for (size_t j = 0; j < gs.size(); ++j) {
          double gb[4];
          for (int k = 0; k < 4; ++k) gb[k] = lab[gs[j] * GW + GW - 4 + k];
          const double o = iou_plain(box, gb);
          if (o > best) {
            best = o;
            bj = (int64_t)j;
          }
        }
        int tp = 0;
        if (best >= thr) {
          const bool diff = has_diff && lab[gs[(size_t)bj] * GW + 1] != 0.f;
          if (!eval_diff && diff) continue;
          if (!used[(size_t)bj]) {
            tp = 1;
            used[(size_t)bj] = 1;
          }
        }
        rec[c].push_back({(double)det[d * 6 + 1], tp});
      }
    }
  }
  const bool eleven = r.op.GetString("ap_type", "integral") == "11point";
  double ap_sum = 0.0;
  int64_t n_ap = 0;
  for (const auto& kv : pos) {
    const int64_t c = kv.first, npos = kv.second;
    if (c == bg || npos == 0) continue;
    std::vector<std::pair<double, int>> rs = rec.count(c) ? rec[c] : std::vector<std::pair<double, int>>();
    std::stable_sort(rs.begin(), rs.end(), [](const std::pair<double, int>& a, const std::pair<double, int>& b) {
      return a.first > b.first;
    });
    std::vector<double> recall, prec;
    double tps = 0, fps = 0;
    for (const auto& e : rs) {
      tps += e.second;
      fps += 1 - e.second;
      recall.push_back(tps / (double)npos);
      prec.push_back(tps / std::max(tps + fps, 1e-12));
    }
    double ap = 0.0;
    if (eleven) {
      for (int t = 0; t <= 10; ++t) {
        double m = 0.0;
        bool any = false;
        for (size_t k = 0; k < recall.size(); ++k)
          if (recall[k] >= t * 0.1) {  // np.linspace(0, 1, 11)
            m = any ? std::max(m, prec[k]) : prec[k];
            any = true;
          }
        ap += m;
      }
      ap /= 11.0;
    } else {
      double prev = 0.0;
      for (size_t k = 0; k < recall.size(); ++k) {
        ap += prec[k] * (recall[k] - prev);
        prev = recall[k];
      }
    }
    ap_sum += ap;
    ++n_ap;
  }
  Tensor mt, pt, tt, ft;
  mt.alloc<float>({1}, -1)[0] = n_ap ? (float)(ap_sum / (double)n_ap) : 0.f;
  const int64_t npc = std::max<int64_t>(1, (int64_t)pos.size());
  int32_t* pp = static_cast<int32_t*>(pt.alloc(DT::INT32, {npc, 1}, -1));
  pp[0] = 0;
  int64_t q = 0;
  for (const auto& kv : pos) pp[q++] = (int32_t)kv.second;
  int64_t nrec = 0;
  for (const auto& kv : rec) nrec += (int64_t)kv.second.size();
  float* tp = tt.alloc<float>({std::max<int64_t>(1, nrec), 2}, -1);
  float* fp = ft.alloc<float>({std::max<int64_t>(1, nrec), 2}, -1);
  tp[0] = tp[1] = fp[0] = fp[1] = 0.f;
  q = 0;
  for (const auto& kv : rec)
    for (const auto& e : kv.second) {
      tp[2 * q] = fp[2 * q] = (float)e.first;
      tp[2 * q + 1] = (float)e.second;
      fp[2 * q + 1] = (float)(1 - e.second);
      ++q;
    }
  put(r, "MAP", mt, {});
  put(r, "AccumPosCount", pt, {});
  put(r, "AccumTruePos", tt, {});
  put(r, "AccumFalsePos", ft, {});
}

// ---------------------------------------------------------------- attention_lstm
// attention_lstm_op.cc: per step, attention scores relu(x_l . aw[:M] (+ ab) + c . aw[M:])
// (optionally scaled and re-biased through relu) softmaxed over the sequence, the
// attended input lx = sum_l a_l x_l, then an LSTM step with gates {forget, input,
// output, candidate} from lx W[D:] + h W[:D] + b.  One work item per sequence runs all
// its steps (the batch-wide step count, state frozen past the sequence's end, as the
// reference's last-step intermediates see it).
__host__ __device__ inline float act_of(int a, float v) {
  switch (a) {
    case 0: return 1.f / (1.f + expf(-v));
    case 1: return tanhf(v);
    case 2: return fmaxf(v, 0.f);
    default: return v;
  }
}
int act_code(const std::string& s) {
  if (s == "sigmoid") return 0;
  if (s == "tanh") return 1;
  if (s == "relu") return 2;
  PA_CHECK(s == "identity" || s.empty(), "attention_lstm: activation %s", s.c_str());
  return 3;
}
struct AttLstm {
  const float *x, *ax, *aw, *sc, *scb, *W, *b, *c0, *h0;
  const int* off;
  float *H, *C, *work, *fc_last, *lx_last, *g_last;
  int64_t N, M, D, L;
  int ag, ac, acand;
  __host__ __device__ void operator()(int64_t n) const {
    const int64_t a = off[n], len = off[n + 1] - off[n];
    float* fc = work + n * (L + M + 6 * D);
    float* lx = fc + L;
    float* g = lx + M;
    float* c = g + 4 * D;
    float* h = c + D;
    for (int64_t d = 0; d < D; ++d) {
      c[d] = c0[n * D + d];
      h[d] = h0 ? h0[n * D + d] : 0.f;
    }
    for (int64_t t = 0; t < L; ++t) {
      float cb = 0.f;
      for (int64_t d = 0; d < D; ++d) cb += c[d] * aw[M + d];
      float mx = -INFINITY;
      for (int64_t l = 0; l < len; ++l) {
        float v = fmaxf(ax[a + l] + cb, 0.f);
        if (sc) {
          v *= sc[0];
          v = fmaxf(v + (scb ? scb[0] : 0.f), 0.f);
        }
        fc[l] = v;
        mx = fmaxf(mx, v);
      }
      float den = 0.f;
      for (int64_t l = 0; l < len; ++l) {
        fc[l] = expf(fc[l] - mx);
        den += fc[l];
      }
      for (int64_t l = 0; l < L; ++l) fc[l] = l < len ? fc[l] / den : 0.f;
      for (int64_t m = 0; m < M; ++m) {
        float v = 0.f;
        for (int64_t l = 0; l < len; ++l) v += fc[l] * x[(a + l) * M + m];
        lx[m] = v;
      }
      for (int64_t j = 0; j < 4 * D; ++j) {
        float v = 0.f;
        for (int64_t m = 0; m < M; ++m) v += lx[m] * W[(D + m) * 4 * D + j];
        for (int64_t d = 0; d < D; ++d) v += h[d] * W[d * 4 * D + j];
        g[j] = v + b[j];
      }
      const bool alive = t < len;
      for (int64_t d = 0; d < D; ++d) {
        const float f = act_of(ag, g[d]), i = act_of(ag, g[D + d]), o = act_of(ag, g[2 * D + d]),
                    cand = act_of(acand, g[3 * D + d]);
        const float cn = f * c[d] + i * cand, hn = act_of(ac, cn) * o;
        if (alive) {
          H[(a + t) * D + d] = hn;
          C[(a + t) * D + d] = cn;
          c[d] = cn;
          h[d] = hn;
        }
      }
    }
    if (n == N - 1) {
      for (int64_t l = 0; l < L; ++l) fc_last[l] = fc[l];
      for (int64_t m = 0; m < M; ++m) lx_last[m] = lx[m];
      for (int64_t j = 0; j < 4 * D; ++j) g_last[j] = g[j];
    }
  }
};
struct AttScore {
  const float *x, *aw, *ab;
  float* ax;
  int64_t M;
  __host__ __device__ void operator()(int64_t t) const {
    float v = ab ? ab[0] : 0.f;
    for (int64_t m = 0; m < M; ++m) v += x[t * M + m] * aw[m];
    ax[t] = v;
  }
};

void k_attention_lstm(const OpRun& r) {
  const bool dev = on_dev(r);
  const Tensor& x = r.in("X");
  PA_CHECK(x.dims.size() == 2 && !x.lod.empty(), "attention_lstm: LoD X [T, M] expected");
  const std::vector<int> off = offsets_of(x, x.dims[0]);
  const int64_t T = x.dims[0], M = x.dims[1], N = (int64_t)off.size() - 1;
  const Tensor& W = r.in("LSTMWeight");
  const int64_t D = W.dims[1] / 4;
  PA_CHECK(W.dims.size() == 2 && W.dims[0] == D + M, "attention_lstm: LSTMWeight must be [D + M, 4D]");
  int64_t L = 0;
  for (int64_t n = 0; n < N; ++n) L = std::max<int64_t>(L, off[(size_t)n + 1] - off[(size_t)n]);
  auto opt = [&](const char* slot) -> const float* {
    Tensor* t = r.in_opt(slot);
    return t ? f32(*t, dev) : nullptr;
  };
  Tensor ax, H, C, fcl, lxl, gl;
  float* axp = ax.alloc<float>({T, 1}, place_of(r));
  const float* aw = f32(r.in("AttentionWeight"), dev);
  any::run(r, dev, T, AttScore{f32(x, dev), aw, opt("AttentionBias"), axp, M}, 64);
  std::vector<float> hw;
  float* work = any::scratch(r, dev, "@att_lstm_work@", N * (L + M + 6 * D), &hw);
  AttLstm f{f32(x, dev), axp, aw, opt("AttentionScalar"), opt("AttentionScalarBias"), f32(W, dev),
            f32(r.in("LSTMBias"), dev), f32(r.in("C0"), dev), opt("H0"), any::ints(r, dev, "@att_lstm_off@", off),
            H.alloc<float>({T, D}, place_of(r)), C.alloc<float>({T, D}, place_of(r)), work,
            fcl.alloc<float>({L, 1}, place_of(r)), lxl.alloc<float>({1, M}, place_of(r)),
            gl.alloc<float>({1, 4 * D}, place_of(r)), N, M, D, L,
            act_code(r.op.GetString("gate_activation", "sigmoid")), act_code(r.op.GetString("cell_activation", "tanh")),
            act_code(r.op.GetString("candidate_activation", "tanh"))};
  any::run(r, dev, N, f, 1);
  H.lod = x.lod;
  C.lod = x.lod;
  set(r, "Hidden", H);
  set(r, "Cell", C);
  set(r, "AttentionedX", ax);
  set(r, "AttentionFCOut", fcl);
  set(r, "LSTMX", lxl);
  set(r, "LSTMOUT", gl);
}

// ---------------------------------------------------------------- generate_proposals
// generate_proposals_op.cc (RPN): per image, the pre_nms_topN best anchors decode
// their deltas (x Variances), clip to the image, drop boxes under min_size * scale,
// greedy NMS (pixel IoU, adaptive eta), post_nms_topN kept.  Host loops as the
// reference's CPU kernel; staged through the host on a HIP place.
std::vector<int64_t> greedy_nms(const std::vector<std::array<float, 4>>& boxes, const std::vector<float>& sc,
                                float thr, float eta) {
  std::vector<int64_t> order(boxes.size());
  for (size_t i = 0; i < order.size(); ++i) order[i] = (int64_t)i;
  std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return sc[(size_t)a] > sc[(size_t)b]; });
  std::vector<int64_t> keep;
  float adaptive = thr;
  while (!order.empty()) {
    const int64_t i = order[0];
    keep.push_back(i);
    std::vector<int64_t> rest;
    for (size_t q = 1; q < order.size(); ++q)
      if (box_iou(boxes[(size_t)i].data(), boxes[(size_t)order[q]].data(), false) <= adaptive) rest.push_back(order[q]);
    order.swap(rest);
    if (eta < 1.f && adaptive > 0.5f) adaptive *= eta;
  }
  return keep;
}

void k_generate_proposals(const OpRun& r) {
  const Tensor st = host_view(r, r.in("Scores"));
  const Tensor dt = host_view(r, r.in("BboxDeltas"));
  const Tensor it = host_view(r, r.in("ImInfo"));
  const Tensor at = host_view(r, r.in("Anchors"));
  Tensor* vp = r.in_opt("Variances");
  const Tensor vt = vp ? host_view(r, *vp) : Tensor();
  if (r.ctx.device >= 0) PA_HIPCHK(hipStreamSynchronize((hipStream_t)r.ctx.stream));
  PA_CHECK(st.dims.size() == 4, "generate_proposals: Scores [N, A, H, W] expected");
  const int64_t N = st.dims[0], A = st.dims[1], H = st.dims[2], W = st.dims[3], K = A * H * W;
  PA_CHECK(dt.numel() == N * 4 * K && at.numel() == 4 * K, "generate_proposals: deltas / anchors do not match");
  const float *sp = f32(st, false), *dp = f32(dt, false), *ip = f32(it, false), *ap = f32(at, false);
  const float* var = vp ? f32(vt, false) : nullptr;
  const int64_t pre = r.op.GetInt("pre_nms_topN", 6000), post = r.op.GetInt("post_nms_topN", 1000);
  const float nthr = r.op.GetFloat("nms_thresh", 0.5f), eta = r.op.GetFloat("eta", 1.f);
  const float clampv = (float)log(1000.0 / 16);
  std::vector<float> rois, probs;
  std::vector<size_t> off = {0};
  const int64_t IW = it.dims.back();
  for (int64_t b = 0; b < N; ++b) {
    std::vector<float> s((size_t)K);
    for (int64_t a = 0; a < A; ++a)
      for (int64_t hw = 0; hw < H * W; ++hw) s[(size_t)(hw * A + a)] = sp[(b * A + a) * H * W + hw];
    std::vector<int64_t> order((size_t)K);
    for (int64_t i = 0; i < K; ++i) order[(size_t)i] = i;
    std::stable_sort(order.begin(), order.end(), [&](int64_t u, int64_t v) { return s[(size_t)u] > s[(size_t)v]; });
    if (pre > 0 && (int64_t)order.size() > pre) order.resize((size_t)pre);
    const float ih = ip[b * IW], iw = ip[b * IW + 1];
    const float ms = (float)((double)r.op.GetFloat("min_size", 0.1f) * (double)ip[b * IW + 2]);
    std::vector<std::array<float, 4>> boxes;
    std::vector<float> ss;
    for (int64_t i : order) {
      const int64_t a = i % A, hw = i / A;
      const float* an = ap + i * 4;
      float d[4];
      for (int k = 0; k < 4; ++k) d[k] = dp[((b * A + a) * 4 + k) * H * W + hw] * (var ? var[i * 4 + k] : 1.f);
      const float aw = an[2] - an[0] + 1.f, ah = an[3] - an[1] + 1.f;
      const float acx = an[0] + 0.5f * aw, acy = an[1] + 0.5f * ah;
      const float cx = d[0] * aw + acx, cy = d[1] * ah + acy;
      const float w = expf(std::min(d[2], clampv)) * aw, h = expf(std::min(d[3], clampv)) * ah;
      std::array<float, 4> bx = {cx - w / 2, cy - h / 2, cx + w / 2 - 1, cy + h / 2 - 1};
      bx[0] = std::min(std::max(bx[0], 0.f), iw - 1);
      bx[2] = std::min(std::max(bx[2], 0.f), iw - 1);
      bx[1] = std::min(std::max(bx[1], 0.f), ih - 1);
      bx[3] = std::min(std::max(bx[3], 0.f), ih - 1);
      if (bx[2] - bx[0] + 1 >= ms && bx[3] - bx[1] + 1 >= ms) {
        boxes.push_back(bx);
        ss.push_back(s[(size_t)i]);
      }
    }
    std::vector<int64_t> keep = greedy_nms(boxes, ss, nthr, eta);
    if (post > 0 && (int64_t)keep.size() > post) keep.resize((size_t)post);
    for (int64_t k : keep) {
      for (int q = 0; q < 4; ++q) rois.push_back(boxes[(size_t)k][(size_t)q]);
      probs.push_back(ss[(size_t)k]);
    }
    off.push_back(probs.size());
  }
  Tensor ro, pr;
  float* rp = ro.alloc<float>({(int64_t)probs.size(), 4}, -1);
  float* pp = pr.alloc<float>({(int64_t)probs.size(), 1}, -1);
  if (!probs.empty()) {
    memcpy(rp, rois.data(), rois.size() * sizeof(float));
    memcpy(pp, probs.data(), probs.size() * sizeof(float));
  }
  put(r, "RpnRois", ro, {off});
  put(r, "RpnRoiProbs", pr, {off});
}

// ---------------------------------------------------------------- ctc_align
// ctc_align_op.h: per sequence, drop blanks and (merge_repeated) repeats of the
// previous token; a single -1 when everything was removed.  Variable-length output:
// host loop (the reference's CPU kernel), staged through the host on a HIP place.
void k_ctc_align(const OpRun& r) {
  const Tensor in = host_view(r, r.in("Input"));
  if (r.ctx.device >= 0) PA_HIPCHK(hipStreamSynchronize((hipStream_t)r.ctx.stream));
  const Idx x = idx_of(in, false);
  const std::vector<int> off = offsets_of(in, in.numel());
  const int64_t blank = r.op.GetInt("blank", 0);
  const bool merge = r.op.GetBool("merge_repeated", true);
  std::vector<int64_t> out;
  std::vector<size_t> noff = {0};
  for (size_t q = 0; q + 1 < off.size(); ++q) {
    bool have_prev = false;
    int64_t prev = 0;
    for (int64_t i = off[q]; i < off[q + 1]; ++i) {
      const int64_t v = x[i];
      if (v != blank && !(merge && have_prev && v == prev)) out.push_back(v);
      prev = v;
      have_prev = true;
    }
    noff.push_back(out.size());
  }
  if (out.empty()) {
    out = {-1};
    noff = {0, 1};
  }
  Tensor h;
  memcpy(h.alloc<int64_t>({(int64_t)out.size(), 1}, -1), out.data(), out.size() * sizeof(int64_t));
  put(r, "Output", h, {noff});
}

}  // namespace

#define PA_ANY_KERNEL(name, fn) \
  PA_HOST_KERNEL(name, fn);     \
  PA_DEVICE_KERNEL(name, fn)

PA_ANY_KERNEL(prior_box, k_prior_box);
PA_ANY_KERNEL(anchor_generator, k_anchor_generator);
PA_ANY_KERNEL(spp, k_spp);
PA_ANY_KERNEL(spp_grad, k_spp_grad);
PA_ANY_KERNEL(fused_elemwise_activation, k_fused_ew);
PA_ANY_KERNEL(fused_elemwise_activation_grad, k_fused_ew_grad);
PA_ANY_KERNEL(auc, k_auc);
PA_ANY_KERNEL(precision_recall, k_precision_recall);
PA_ANY_KERNEL(positive_negative_pair, k_pn_pair);
PA_ANY_KERNEL(average_accumulates, k_average_accumulates);
PA_ANY_KERNEL(fake_quantize_range_abs_max, k_fake_quant_range);
PA_ANY_KERNEL(bipartite_match, k_bipartite_match);
PA_ANY_KERNEL(target_assign, k_target_assign);
PA_HOST_KERNEL(layer_norm, layer_norm_any);
PA_HOST_KERNEL(layer_norm_grad, layer_norm_grad_any);
PA_HOST_KERNEL(dropout_grad, k_dropout_grad_host);

PA_ANY_KERNEL(reduce_sum_grad, k_reduce_grad<0>);
PA_ANY_KERNEL(reduce_mean_grad, k_reduce_grad<1>);
PA_ANY_KERNEL(reduce_max_grad, k_reduce_grad<2>);
PA_ANY_KERNEL(reduce_min_grad, k_reduce_grad<3>);
PA_ANY_KERNEL(reduce_prod_grad, k_reduce_grad<4>);
PA_ANY_KERNEL(elementwise_max_grad, k_ew_grad3<0>);
PA_ANY_KERNEL(elementwise_min_grad, k_ew_grad3<1>);
PA_ANY_KERNEL(elementwise_pow_grad, k_ew_grad3<2>);
PA_ANY_KERNEL(elementwise_floordiv, k_floordiv_mod<false>);
PA_ANY_KERNEL(elementwise_mod, k_floordiv_mod<true>);
PA_ANY_KERNEL(sequence_reverse, k_seq_reverse);
PA_ANY_KERNEL(sequence_reverse_grad, k_seq_reverse_grad);
PA_ANY_KERNEL(sequence_scatter, k_seq_scatter);
PA_ANY_KERNEL(sequence_scatter_grad, k_seq_scatter_grad);
PA_ANY_KERNEL(kldiv_loss, k_kldiv);
PA_ANY_KERNEL(kldiv_loss_grad, k_kldiv_grad);
PA_ANY_KERNEL(bpr_loss, k_bpr);
PA_ANY_KERNEL(bpr_loss_grad, k_bpr_grad);
PA_ANY_KERNEL(shuffle_channel, k_shuffle_channel);
PA_ANY_KERNEL(shuffle_channel_grad, k_shuffle_channel);
PA_ANY_KERNEL(scale_sub_region, k_scale_sub_region);
PA_ANY_KERNEL(scale_sub_region_grad, k_scale_sub_region);
PA_ANY_KERNEL(size, k_size);
PA_ANY_KERNEL(lars_momentum, k_lars_momentum);
PA_ANY_KERNEL(max_pool3d_with_index, k_max_pool3d_idx);
PA_ANY_KERNEL(max_pool3d_with_index_grad, k_max_pool3d_idx_grad);
PA_ANY_KERNEL(chunk_eval, k_chunk_eval);
PA_ANY_KERNEL(sampling_id, k_sampling_id);
PA_ANY_KERNEL(random_crop, k_random_crop);
PA_ANY_KERNEL(print, k_print);
PA_ANY_KERNEL(multiclass_nms, k_multiclass_nms);
PA_ANY_KERNEL(mine_hard_examples, k_mine_hard_examples);
PA_ANY_KERNEL(fusion_lstm, k_fusion_rnn);
PA_ANY_KERNEL(fusion_gru, k_fusion_rnn);
PA_ANY_KERNEL(fusion_seqexpand_concat_fc, k_seqexpand_concat_fc);
PA_ANY_KERNEL(detection_map, k_detection_map);
PA_ANY_KERNEL(attention_lstm, k_attention_lstm);
PA_ANY_KERNEL(generate_proposals, k_generate_proposals);
PA_ANY_KERNEL(ctc_align, k_ctc_align);

void link_extra_kernels() {}

}  // namespace pa
