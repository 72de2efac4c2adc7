// conv3d / conv3d_grad, pool3d / pool3d_grad (NCDHW) and the transposed convolutions
// conv2d_transpose / depthwise_conv2d_transpose / conv3d_transpose (+grads) on the
// native executor, host AND device.
//
// Semantics: reference operators/conv_op.h GemmConvKernel / GemmConvGradKernel with
// math/vol2col.{cc,cu} (a column matrix of [C/g * kd * kh * kw, OD * OH * OW] per
// image and group, the filter GEMM over it), operators/pool_op.h with
// math/pooling.{cc,cu} Pool3dFunctor (max routes the gradient to the window's first
// maximum; avg divides by the in-image window, or with exclusive = False by the
// window clipped to the padded volume; ceil_mode rounds the output extent up while
// the last window still starts inside the padded input).
// Device: the kernel library's pa_vol2col / pa_col2vol / pa_sgemm (exact-fp32 MFMA,
// images x groups on the GEMM batch) / pa_pool_* launchers -- the same ones the
// Python operators call, so both engines agree bit for bit on a HIP place.  Host:
// the loops below over the worker pool plus the blocked sgemm.
#include <hip/hip_runtime.h>
#include <math.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "device_util.h"
#include "kernel_lib.h"

namespace pa {
namespace {

using Dims = std::vector<int64_t>;

std::vector<int64_t> ints3(const OpRun& r, const char* name, int64_t def) {
  auto v = r.op.GetInts(name);
  if (v.empty()) v.assign(3, def);
  PA_CHECK(v.size() == 3, "%s: %s must have 3 values", r.op.type.c_str(), name);
  return v;
}

struct Conv3 {
  int64_t N, C, D, H, W, OC, kd, kh, kw, OD, OH, OW, G, Cg, OCg, K, S, I;
  int64_t st[3], pd[3], dl[3];
  int geo[19];
};

// the GEMM-conv geometry of input [N, C, D, H, W] and filter [OC, C/g, kd, kh, kw]
Conv3 conv3_make(const char* op, const Dims& xd, const Dims& wd, const Dims& st, const Dims& pd, const Dims& dl,
                 int64_t G) {
  PA_CHECK(xd.size() == 5 && wd.size() == 5, "%s: NCDHW input and [OC, C/g, kd, kh, kw] filter expected", op);
  Conv3 c;
  c.G = std::max<int64_t>(1, G);
  c.N = xd[0]; c.C = xd[1]; c.D = xd[2]; c.H = xd[3]; c.W = xd[4];
  c.OC = wd[0]; c.kd = wd[2]; c.kh = wd[3]; c.kw = wd[4];
  PA_CHECK(wd[1] * c.G == c.C && c.OC % c.G == 0, "%s: filter / input channel mismatch", op);
  const int64_t k[3] = {c.kd, c.kh, c.kw}, in[3] = {c.D, c.H, c.W};
  int64_t o[3];
  for (int i = 0; i < 3; ++i) {
    c.st[i] = st[(size_t)i];
    c.pd[i] = pd[(size_t)i];
    c.dl[i] = dl[(size_t)i];
    o[i] = (in[i] + 2 * pd[(size_t)i] - (dl[(size_t)i] * (k[i] - 1) + 1)) / st[(size_t)i] + 1;
    PA_CHECK(o[i] > 0, "%s: empty output", op);
  }
  c.OD = o[0]; c.OH = o[1]; c.OW = o[2];
  c.Cg = c.C / c.G; c.OCg = c.OC / c.G;
  c.K = c.Cg * c.kd * c.kh * c.kw;
  c.S = c.OD * c.OH * c.OW;
  c.I = c.D * c.H * c.W;
  const int64_t g[19] = {c.C, c.D, c.H, c.W, c.OD, c.OH, c.OW, c.kd, c.kh, c.kw, st[0], st[1], st[2],
                         pd[0], pd[1], pd[2], dl[0], dl[1], dl[2]};
  for (int i = 0; i < 19; ++i) c.geo[i] = (int)g[i];
  return c;
}

Conv3 conv3_of(const OpRun& r, const Dims& xd, const Dims& wd) {
  return conv3_make("conv3d", xd, wd, ints3(r, "strides", 1), ints3(r, "paddings", 0), ints3(r, "dilations", 1),
                    r.op.GetInt("groups", 1));
}

// ---------------------------------------------------------------- host vol2col
// col[(c, i, j, l), (od, oh, ow)] of one image's channel block [Cg, D, H, W]
void vol2col(const Conv3& c, const float* x, float* col) {
  parallel_for(c.Cg * c.kd * c.kh * c.kw, 4, [&](int64_t a, int64_t b) {
    for (int64_t row = a; row < b; ++row) {
      const int64_t l = row % c.kw, j = (row / c.kw) % c.kh, i = (row / (c.kw * c.kh)) % c.kd,
                    ch = row / (c.kw * c.kh * c.kd);
      float* out = col + row * c.S;
      for (int64_t od = 0; od < c.OD; ++od) {
        const int64_t id = od * c.st[0] - c.pd[0] + i * c.dl[0];
        for (int64_t oh = 0; oh < c.OH; ++oh) {
          const int64_t ih = oh * c.st[1] - c.pd[1] + j * c.dl[1];
          for (int64_t ow = 0; ow < c.OW; ++ow) {
            const int64_t iw = ow * c.st[2] - c.pd[2] + l * c.dl[2];
            const bool in = id >= 0 && id < c.D && ih >= 0 && ih < c.H && iw >= 0 && iw < c.W;
            out[(od * c.OH + oh) * c.OW + ow] = in ? x[((ch * c.D + id) * c.H + ih) * c.W + iw] : 0.f;
          }
        }
      }
    }
  });
}

// x += col2vol(col) for one image's channel block (channels in parallel, rows of a
// channel serially: a channel's rows write only that channel)
void col2vol_add(const Conv3& c, const float* col, float* x) {
  const int64_t per = c.kd * c.kh * c.kw;
  parallel_for(c.Cg, 1, [&](int64_t a, int64_t b) {
    for (int64_t ch = a; ch < b; ++ch)
      for (int64_t q = 0; q < per; ++q) {
        const int64_t l = q % c.kw, j = (q / c.kw) % c.kh, i = q / (c.kw * c.kh);
        const float* in = col + (ch * per + q) * c.S;
        for (int64_t od = 0; od < c.OD; ++od) {
          const int64_t id = od * c.st[0] - c.pd[0] + i * c.dl[0];
          if (id < 0 || id >= c.D) continue;
          for (int64_t oh = 0; oh < c.OH; ++oh) {
            const int64_t ih = oh * c.st[1] - c.pd[1] + j * c.dl[1];
            if (ih < 0 || ih >= c.H) continue;
            for (int64_t ow = 0; ow < c.OW; ++ow) {
              const int64_t iw = ow * c.st[2] - c.pd[2] + l * c.dl[2];
              if (iw >= 0 && iw < c.W) x[((ch * c.D + id) * c.H + ih) * c.W + iw] += in[(od * c.OH + oh) * c.OW + ow];
            }
          }
        }
      }
  });
}

float* f32h(const Tensor& t) {
  if (t.dtype != DT::FP32 || t.device >= 0) throw Decline{};
  return t.data<float>();
}

// The three GEMM-conv passes, parameterised by role so that conv3d and the
// transposed convolutions (whose forward is a conv's data gradient) share them.
// y = conv(x, w) (+ bias)
void conv_fwd_h(const Conv3& c, const float* xp, const float* wp, const float* bp, float* y) {
  std::vector<float> col((size_t)(c.K * c.S));
  for (int64_t n = 0; n < c.N; ++n)
    for (int64_t g = 0; g < c.G; ++g) {
      vol2col(c, xp + (n * c.C + g * c.Cg) * c.I, col.data());
      float* yo = y + (n * c.OC + g * c.OCg) * c.S;
      sgemm(false, false, c.OCg, c.S, c.K, 1.f, wp + g * c.OCg * c.K, c.K, col.data(), c.S, 0.f, yo, c.S);
      if (bp)
        for (int64_t o = 0; o < c.OCg; ++o)
          for (int64_t s = 0; s < c.S; ++s) yo[o * c.S + s] += bp[g * c.OCg + o];
    }
}

// dx = conv's data gradient of dy (dx overwritten)
void conv_dx_h(const Conv3& c, const float* wp, const float* gp, float* dx) {
  memset(dx, 0, sizeof(float) * (size_t)(c.N * c.C * c.I));
  std::vector<float> col((size_t)(c.K * c.S));
  for (int64_t n = 0; n < c.N; ++n)
    for (int64_t g = 0; g < c.G; ++g) {
      sgemm(true, false, c.K, c.S, c.OCg, 1.f, wp + g * c.OCg * c.K, c.K, gp + (n * c.OC + g * c.OCg) * c.S, c.S,
            0.f, col.data(), c.S);
      col2vol_add(c, col.data(), dx + (n * c.C + g * c.Cg) * c.I);
    }
}

// dw = conv's filter gradient of (x, dy) (dw overwritten)
void conv_dw_h(const Conv3& c, const float* xp, const float* gp, float* dw) {
  memset(dw, 0, sizeof(float) * (size_t)(c.OC * c.K));
  std::vector<float> col((size_t)(c.K * c.S));
  for (int64_t n = 0; n < c.N; ++n)
    for (int64_t g = 0; g < c.G; ++g) {
      vol2col(c, xp + (n * c.C + g * c.Cg) * c.I, col.data());
      sgemm(false, true, c.OCg, c.K, c.S, 1.f, gp + (n * c.OC + g * c.OCg) * c.S, c.S, col.data(), c.S, 1.f,
            dw + g * c.OCg * c.K, c.K);
    }
}

void k_conv3d_host(const OpRun& r) {
  Tensor x = r.in("Input");
  Tensor w = r.in("Filter");
  Tensor* b = r.in_opt("Bias");
  const Conv3 c = conv3_of(r, x.dims, w.dims);
  const float *xp = f32h(x), *wp = f32h(w), *bp = b ? f32h(*b) : nullptr;
  conv_fwd_h(c, xp, wp, bp, r.out("Output")->alloc<float>({c.N, c.OC, c.OD, c.OH, c.OW}, -1));
}

void k_conv3d_grad_host(const OpRun& r) {
  Tensor x = r.in("Input");
  Tensor w = r.in("Filter");
  Tensor dy = r.in("Output@GRAD");
  const Conv3 c = conv3_of(r, x.dims, w.dims);
  PA_CHECK(dy.numel() == c.N * c.OC * c.S, "conv3d_grad: Output@GRAD %s does not match", dy.shape_str().c_str());
  const float *xp = f32h(x), *wp = f32h(w), *gp = f32h(dy);
  Tensor* dxt = r.out("Input@GRAD");
  Tensor* dwt = r.out("Filter@GRAD");
  Tensor* dbt = r.out("Bias@GRAD");
  if (dxt) conv_dx_h(c, wp, gp, dxt->alloc<float>(x.dims, -1));
  if (dwt) conv_dw_h(c, xp, gp, dwt->alloc<float>(w.dims, -1));
  if (dbt) {
    float* db = dbt->alloc<float>({c.OC}, -1);
    for (int64_t o = 0; o < c.OC; ++o) {
      double s = 0;
      for (int64_t n = 0; n < c.N; ++n)
        for (int64_t i = 0; i < c.S; ++i) s += gp[(n * c.OC + o) * c.S + i];
      db[o] = (float)s;
    }
  }
}

// ---------------------------------------------------------------- device conv3d
constexpr int64_t kColBudget = int64_t(1) << 28;  // floats per column chunk (1 GiB)

int64_t chunk(const Conv3& c) {
  int64_t nb = std::max<int64_t>(1, std::min<int64_t>(c.N, kColBudget / std::max<int64_t>(c.C * c.K / c.Cg * c.S, 1)));
  return std::max<int64_t>(1, std::min<int64_t>(nb, 65535 / std::max<int64_t>(c.G, 1)));
}

void sg(const OpRun& r, const float* A, long sam, long sak, const float* B, long sbk, long sbn, float* C, long ldc,
        long M, long N, long K, int Z1, int Z2, long a1, long b1, long c1, long a2, long b2, long c2, int kb = 1,
        long kbA = 0, long kbB = 0, const float* bias = nullptr, long bsb = 0, int atomic = 0) {
  PA_CHECK((int64_t)Z1 * Z2 <= 65535, "conv3d: batch x groups too large");
  PA_KL(pa_sgemm(A, sam, sak, B, sbk, sbn, C, ldc, M, N, K, Z1, Z2, a1, b1, c1, a2, b2, c2, kb, kbA, kbB, bias, bsb,
                 1.f, 0.f, atomic, nullptr, dev_stream(r)));
}

void conv_fwd_d(const OpRun& r, const Conv3& c, const float* xp, const float* wp, const float* bp, float* y) {
  const int64_t nb = chunk(c), rows = c.C * c.kd * c.kh * c.kw;
  float* col = device_workspace(r, "@conv_col@", nb * rows * c.S);
  for (int64_t n0 = 0; n0 < c.N; n0 += nb) {
    const int m = (int)std::min(nb, c.N - n0);
    PA_KL(pa_vol2col(0, xp + n0 * c.C * c.I, col, c.geo, m, dev_stream(r)));
    sg(r, wp, c.K, 1, col, c.S, 1, y + n0 * c.OC * c.S, c.S, c.OCg, c.S, c.K, m, (int)c.G, 0, rows * c.S,
       c.OC * c.S, c.OCg * c.K, c.K * c.S, c.OCg * c.S, 1, 0, 0, bp, c.OCg);
  }
}

void conv_dx_d(const OpRun& r, const Conv3& c, const float* wp, const float* gp, float* dx) {
  const int64_t nb = chunk(c), rows = c.C * c.kd * c.kh * c.kw;
  float* col = device_workspace(r, "@conv_col@", nb * rows * c.S);
  for (int64_t n0 = 0; n0 < c.N; n0 += nb) {
    const int m = (int)std::min(nb, c.N - n0);
    sg(r, wp, 1, c.K, gp + n0 * c.OC * c.S, c.S, 1, col, c.S, c.K, c.S, c.OCg, m, (int)c.G, 0, c.OC * c.S,
       rows * c.S, c.OCg * c.K, c.OCg * c.S, c.K * c.S);
    PA_KL(pa_col2vol(col, dx + n0 * c.C * c.I, c.geo, m, 0, dev_stream(r)));
  }
}

void conv_dw_d(const OpRun& r, const Conv3& c, const float* xp, const float* gp, float* dw) {
  const int64_t nb = chunk(c), rows = c.C * c.kd * c.kh * c.kw;
  float* col = device_workspace(r, "@conv_col@", nb * rows * c.S);
  PA_HIPCHK(hipMemsetAsync(dw, 0, sizeof(float) * (size_t)(c.OC * c.K), dev_stream(r)));
  for (int64_t n0 = 0; n0 < c.N; n0 += nb) {
    const int m = (int)std::min(nb, c.N - n0);
    PA_KL(pa_vol2col(0, xp + n0 * c.C * c.I, col, c.geo, m, dev_stream(r)));
    sg(r, gp + n0 * c.OC * c.S, c.S, 1, col, 1, c.S, dw, c.K, c.OCg, c.K, c.S, 1, (int)c.G, 0, 0, 0,
       c.OCg * c.S, c.K * c.S, c.OCg * c.K, m, c.OC * c.S, rows * c.S, nullptr, 0, 1);
  }
}

void k_conv3d_dev(const OpRun& r) {
  Tensor x = r.in("Input");
  Tensor w = r.in("Filter");
  Tensor* b = r.in_opt("Bias");
  const Conv3 c = conv3_of(r, x.dims, w.dims);
  float* y = r.out("Output")->alloc<float>({c.N, c.OC, c.OD, c.OH, c.OW}, dev_id(r));
  conv_fwd_d(r, c, dev_f32(x), dev_f32(w), b ? dev_f32(*b) : nullptr, y);
}

void k_conv3d_grad_dev(const OpRun& r) {
  Tensor x = r.in("Input");
  Tensor w = r.in("Filter");
  Tensor dy = r.in("Output@GRAD");
  const Conv3 c = conv3_of(r, x.dims, w.dims);
  PA_CHECK(dy.numel() == c.N * c.OC * c.S, "conv3d_grad: Output@GRAD %s does not match", dy.shape_str().c_str());
  const float *xp = dev_f32(x), *wp = dev_f32(w), *gp = dev_f32(dy);
  Tensor* dxt = r.out("Input@GRAD");
  Tensor* dwt = r.out("Filter@GRAD");
  Tensor* dbt = r.out("Bias@GRAD");
  if (dxt) conv_dx_d(r, c, wp, gp, dxt->alloc<float>(x.dims, dev_id(r)));
  if (dwt) conv_dw_d(r, c, xp, gp, dwt->alloc<float>(w.dims, dev_id(r)));
  if (dbt) PA_KL(pa_chan_sum(gp, dbt->alloc<float>({c.OC}, dev_id(r)), (int)c.N, (int)c.OC, c.S, 0, dev_stream(r)));
}

// ---------------------------------------------------------------- transposed convolution
// conv{2,3}d_transpose / depthwise_conv2d_transpose (reference operators/
// conv_transpose_op.h: col = W^T x per image and group, col2im into the output).
// Input [N, Cin, (D,) H, W], Filter [Cin, OC/g, (kd,) kh, kw]; the output extent is
// (in - 1) * stride - 2 pad + dilation (k - 1) + 1.  Computed as the data gradient of
// the conv that maps the output back onto the input (that conv's filter is exactly
// Filter), so forward = conv dgrad, Input@GRAD = conv forward of Output@GRAD and
// Filter@GRAD = that conv's wgrad of (Output@GRAD, Input).  2-D ops run as depth 1.
struct ConvT {
  Conv3 c;       // the conv from the transposed op's output to its input
  Dims out;      // the transposed op's output dims
};

ConvT convt_of(const OpRun& r, const Dims& xd0, const Dims& wd0) {
  const bool two = xd0.size() == 4;
  const char* op = r.op.type.c_str();
  PA_CHECK((two && wd0.size() == 4) || (xd0.size() == 5 && wd0.size() == 5),
           "%s: NC(D)HW input and [Cin, OC/g, (kd,) kh, kw] filter expected", op);
  const size_t nd = two ? 2 : 3;
  auto attr = [&](const char* name, int64_t def) {
    auto v = r.op.GetInts(name);
    if (v.empty()) v.assign(nd, def);
    PA_CHECK(v.size() == nd, "%s: %s must have %d values", op, name, (int)nd);
    if (two) v.insert(v.begin(), name[0] == 'p' ? 0 : 1);
    return v;
  };
  const Dims st = attr("strides", 1), pd = attr("paddings", 0), dl = attr("dilations", 1);
  Dims xd = xd0, wd = wd0;
  if (two) {
    xd.insert(xd.begin() + 2, 1);
    wd.insert(wd.begin() + 2, 1);
  }
  const int64_t G = std::max<int64_t>(1, r.op.GetInt("groups", 1));
  Dims yd = {xd[0], wd[1] * G};
  for (int i = 0; i < 3; ++i) {
    const int64_t o = (xd[(size_t)i + 2] - 1) * st[(size_t)i] - 2 * pd[(size_t)i] +
                      dl[(size_t)i] * (wd[(size_t)i + 2] - 1) + 1;
    PA_CHECK(o > 0, "%s: empty output", op);
    yd.push_back(o);
  }
  const auto osz = r.op.GetInts("output_size");
  for (size_t i = 0; i < osz.size(); ++i)
    if (osz[i] != yd[yd.size() - osz.size() + i]) throw Decline{};  // trimmed output sizes: the embedder's kernel
  ConvT t;
  t.c = conv3_make(op, yd, wd, st, pd, dl, G);
  PA_CHECK(t.c.OD == xd[2] && t.c.OH == xd[3] && t.c.OW == xd[4] && t.c.OC == xd[1], "%s: geometry mismatch", op);
  t.out = yd;
  if (two) t.out.erase(t.out.begin() + 2);
  return t;
}

void k_convt(const OpRun& r) {
  Tensor x = r.in("Input");
  Tensor w = r.in("Filter");
  const ConvT t = convt_of(r, x.dims, w.dims);
  const bool dev = x.device >= 0;
  float* y = r.out("Output")->alloc<float>(t.out, dev ? dev_id(r) : -1);
  if (dev) conv_dx_d(r, t.c, dev_f32(w), dev_f32(x), y);
  else conv_dx_h(t.c, f32h(w), f32h(x), y);
}

void k_convt_grad(const OpRun& r) {
  Tensor x = r.in("Input");
  Tensor w = r.in("Filter");
  Tensor dy = r.in("Output@GRAD");
  const ConvT t = convt_of(r, x.dims, w.dims);
  PA_CHECK(dy.numel() == t.c.N * t.c.C * t.c.I, "%s: Output@GRAD %s does not match", r.op.type.c_str(),
           dy.shape_str().c_str());
  const bool dev = x.device >= 0;
  Tensor* dxt = r.op.Outputs("Input@GRAD").empty() ? nullptr : r.out("Input@GRAD");
  Tensor* dwt = r.op.Outputs("Filter@GRAD").empty() ? nullptr : r.out("Filter@GRAD");
  if (dev) {
    if (dxt) conv_fwd_d(r, t.c, dev_f32(dy), dev_f32(w), nullptr, dxt->alloc<float>(x.dims, dev_id(r)));
    if (dwt) conv_dw_d(r, t.c, dev_f32(dy), dev_f32(x), dwt->alloc<float>(w.dims, dev_id(r)));
  } else {
    if (dxt) conv_fwd_h(t.c, f32h(dy), f32h(w), nullptr, dxt->alloc<float>(x.dims, -1));
    if (dwt) conv_dw_h(t.c, f32h(dy), f32h(x), dwt->alloc<float>(w.dims, -1));
  }
}

// ---------------------------------------------------------------- pool3d
struct Pool3 {
  int64_t N, C, in[3], out[3], k[3], st[3], pd[3];
  int type, exclusive;
  int geo[15];
};

Pool3 pool3_of(const OpRun& r, const Dims& xd) {
  PA_CHECK(xd.size() == 5, "pool3d: NCDHW input expected");
  Pool3 p;
  p.N = xd[0];
  p.C = xd[1];
  auto ks = ints3(r, "ksize", 1), st = ints3(r, "strides", 1), pd = ints3(r, "paddings", 0);
  if (r.op.GetBool("global_pooling")) {
    ks = {xd[2], xd[3], xd[4]};
    pd = {0, 0, 0};
  }
  const bool ceil = r.op.GetBool("ceil_mode");
  for (int i = 0; i < 3; ++i) {
    p.in[i] = xd[(size_t)i + 2];
    p.k[i] = ks[(size_t)i];
    p.st[i] = st[(size_t)i];
    p.pd[i] = pd[(size_t)i];
    int64_t o = ceil ? (p.in[i] - p.k[i] + 2 * p.pd[i] + p.st[i] - 1) / p.st[i] + 1
                     : (p.in[i] - p.k[i] + 2 * p.pd[i]) / p.st[i] + 1;
    if (ceil && (o - 1) * p.st[i] >= p.in[i] + p.pd[i]) --o;  // the last window must start in the input
    PA_CHECK(o > 0, "pool3d: empty output");
    p.out[i] = o;
  }
  p.type = r.op.GetString("pooling_type", "max") == "max" ? 0 : 1;
  p.exclusive = r.op.GetBool("exclusive", true) ? 1 : 0;
  const int64_t g[15] = {p.in[0], p.in[1], p.in[2], p.out[0], p.out[1], p.out[2], p.k[0], p.k[1], p.k[2],
                         p.st[0], p.st[1], p.st[2], p.pd[0], p.pd[1], p.pd[2]};
  for (int i = 0; i < 15; ++i) p.geo[i] = (int)g[i];
  return p;
}

// one window of the host pooling: [lo, hi) per axis inside the image, and the avg divisor
struct Win {
  int64_t lo[3], hi[3];
  float div;
};

Win window(const Pool3& p, int64_t od, int64_t oh, int64_t ow) {
  Win w;
  const int64_t o[3] = {od, oh, ow};
  int64_t cnt = 1, padded = 1;
  for (int i = 0; i < 3; ++i) {
    const int64_t s = o[i] * p.st[i] - p.pd[i];
    const int64_t e = std::min(s + p.k[i], p.in[i] + p.pd[i]);
    padded *= e - s;
    w.lo[i] = std::max<int64_t>(s, 0);
    w.hi[i] = std::min(e, p.in[i]);
    cnt *= std::max<int64_t>(w.hi[i] - w.lo[i], 0);
  }
  w.div = (float)std::max<int64_t>(1, p.exclusive ? cnt : padded);
  return w;
}

void k_pool3d_host(const OpRun& r) {
  Tensor x = r.in("X");
  const Pool3 p = pool3_of(r, x.dims);
  const int64_t I = p.in[0] * p.in[1] * p.in[2], O = p.out[0] * p.out[1] * p.out[2];
  float* y = r.out("Out")->alloc<float>({p.N, p.C, p.out[0], p.out[1], p.out[2]}, -1);
  const float* xp = f32h(x);
  parallel_for(p.N * p.C, 1, [&](int64_t a, int64_t b) {
    for (int64_t nc = a; nc < b; ++nc) {
      const float* xi = xp + nc * I;
      for (int64_t od = 0; od < p.out[0]; ++od)
        for (int64_t oh = 0; oh < p.out[1]; ++oh)
          for (int64_t ow = 0; ow < p.out[2]; ++ow) {
            const Win w = window(p, od, oh, ow);
            float acc = p.type == 0 ? -INFINITY : 0.f;
            for (int64_t d = w.lo[0]; d < w.hi[0]; ++d)
              for (int64_t h = w.lo[1]; h < w.hi[1]; ++h)
                for (int64_t q = w.lo[2]; q < w.hi[2]; ++q) {
                  const float v = xi[(d * p.in[1] + h) * p.in[2] + q];
                  acc = p.type == 0 ? (v > acc ? v : acc) : acc + v;
                }
            y[nc * O + (od * p.out[1] + oh) * p.out[2] + ow] = p.type == 0 ? acc : acc / w.div;
          }
    }
  });
}

void k_pool3d_grad_host(const OpRun& r) {
  Tensor x = r.in("X");
  Tensor dy = r.in("Out@GRAD");
  const Pool3 p = pool3_of(r, x.dims);
  const int64_t I = p.in[0] * p.in[1] * p.in[2], O = p.out[0] * p.out[1] * p.out[2];
  Tensor* dxt = r.out("X@GRAD");
  if (!dxt) return;
  float* dx = dxt->alloc<float>(x.dims, -1);
  memset(dx, 0, sizeof(float) * (size_t)x.numel());
  const float *xp = f32h(x), *gp = f32h(dy);
  parallel_for(p.N * p.C, 1, [&](int64_t a, int64_t b) {
    for (int64_t nc = a; nc < b; ++nc) {
      const float* xi = xp + nc * I;
      float* di = dx + nc * I;
      for (int64_t od = 0; od < p.out[0]; ++od)
        for (int64_t oh = 0; oh < p.out[1]; ++oh)
          for (int64_t ow = 0; ow < p.out[2]; ++ow) {
            const Win w = window(p, od, oh, ow);
            const float g = gp[nc * O + (od * p.out[1] + oh) * p.out[2] + ow];
            int64_t best = -1;
            float bv = -INFINITY;
            for (int64_t d = w.lo[0]; d < w.hi[0]; ++d)
              for (int64_t h = w.lo[1]; h < w.hi[1]; ++h)
                for (int64_t q = w.lo[2]; q < w.hi[2]; ++q) {
                  const int64_t at = (d * p.in[1] + h) * p.in[2] + q;
                  if (p.type == 0) {
                    if (best < 0 || xi[at] > bv) {
                      bv = xi[at];
                      best = at;
                    }
                  } else {
                    di[at] += g / w.div;
                  }
                }
            if (p.type == 0 && best >= 0) di[best] += g;
          }
    }
  });
}

int* pool3_mask(const OpRun& r, const std::string& out_name, const Pool3& p) {
  Variable* v = r.scope.Var(out_name + "@MASK");
  return static_cast<int*>(v->tensor.alloc(DT::INT32, {p.N, p.C, p.out[0], p.out[1], p.out[2]}, dev_id(r)));
}

void k_pool3d_dev(const OpRun& r) {
  Tensor x = r.in("X");
  const Pool3 p = pool3_of(r, x.dims);
  float* o = r.out("Out")->alloc<float>({p.N, p.C, p.out[0], p.out[1], p.out[2]}, dev_id(r));
  int* mask = p.type == 0 ? pool3_mask(r, r.op.Output("Out"), p) : nullptr;
  PA_KL(pa_pool_fwd(0, dev_f32(x), o, mask, p.N * p.C, p.geo, p.type, p.exclusive, dev_stream(r)));
}

void k_pool3d_grad_dev(const OpRun& r) {
  Tensor x = r.in("X");
  Tensor dy = r.in("Out@GRAD");
  const Pool3 p = pool3_of(r, x.dims);
  Tensor* dx = r.out("X@GRAD");
  if (!dx) return;
  const int* mask = nullptr;
  if (p.type == 0) {
    Variable* mv = r.scope.Find(r.op.Input("Out") + "@MASK");
    if (mv && mv->tensor.initialized() && mv->tensor.device == dev_id(r) && mv->tensor.numel() == dy.numel()) {
      mask = mv->tensor.data<int>();
    } else {  // forward ran elsewhere: rebuild the argmax
      int* m = pool3_mask(r, r.op.Input("Out"), p);
      float* tmp = device_workspace(r, "@pool_tmp@", dy.numel());
      PA_KL(pa_pool_fwd(0, dev_f32(x), tmp, m, p.N * p.C, p.geo, 0, p.exclusive, dev_stream(r)));
      mask = m;
    }
  }
  float* dxp = dx->alloc<float>(x.dims, dev_id(r));
  PA_KL(pa_pool_bwd(0, dev_f32(dy), mask, dxp, p.N * p.C, p.geo, p.type, p.exclusive, dev_stream(r)));
}

}  // namespace

PA_HOST_KERNEL(conv3d, k_conv3d_host);
PA_HOST_KERNEL(conv3d_grad, k_conv3d_grad_host);
PA_HOST_KERNEL(pool3d, k_pool3d_host);
PA_HOST_KERNEL(pool3d_grad, k_pool3d_grad_host);
PA_DEVICE_KERNEL(conv3d, k_conv3d_dev);
PA_DEVICE_KERNEL(conv3d_grad, k_conv3d_grad_dev);
PA_DEVICE_KERNEL(pool3d, k_pool3d_dev);
PA_DEVICE_KERNEL(pool3d_grad, k_pool3d_grad_dev);
#define PA_CONVT(name)             \
  PA_HOST_KERNEL(name, k_convt);   \
  PA_DEVICE_KERNEL(name, k_convt); \
  PA_HOST_KERNEL(name##_grad, k_convt_grad); \
  PA_DEVICE_KERNEL(name##_grad, k_convt_grad)
PA_CONVT(conv2d_transpose);
PA_CONVT(depthwise_conv2d_transpose);
PA_CONVT(conv3d_transpose);

void link_conv3d_kernels() {}

}  // namespace pa
