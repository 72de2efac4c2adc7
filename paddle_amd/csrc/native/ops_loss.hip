// Structured / sampled losses and ROI pooling of the native executor, host AND
// device: warpctc (+grad), edit_distance, nce (+grad), hierarchical_sigmoid (+grad),
// roi_pool (+grad).
//
// Semantics (the Python kernels of operators/structured_ops.py, nn_ops.py compute
// the same functions):
//   * warpctc (reference warpctc_op.h): Loss = -log p(label | softmax(logits)) per
//     LoD sequence by the alpha / beta lattice over the blank-extended label; an
//     impossible alignment gives loss 0 and gradient 0; norm_by_times scales only the
//     gradient by 1 / T.  The grad op recomputes the lattice (it does not trust a
//     WarpCTCGrad that another engine may have left empty).
//   * edit_distance (edit_distance_op.h): Levenshtein distance per (hyp, ref) pair,
//     divided by the reference length when normalized.
//   * nce (nce_op.h): logits of the true labels and num_neg_samples negatives
//     (custom_neg_classes, else a counter-based uniform sampler keyed on `seed` --
//     the interpreter draws from torch's generator, so only custom negatives give
//     the same samples on both engines), o = sigmoid(logit), b = k / C,
//     cost = sum_true -log(o / (o + b)) + sum_neg -log(b / (o + b)), times SampleWeight.
//   * hierarchical_sigmoid (hierarchical_sigmoid_op.h with math/matrix_bit_code.h
//     SimpleCode): code c = label + C, node of bit j = (c >> (j + 1)) - 1, branch bit
//     (c >> j) & 1, length floor(log2 c); pre = x . W[node] + b[node] clipped to
//     [-40, 40]; Out = sum_j softplus(pre) - bit * pre.
//   * roi_pool (roi_pool_op.h): max over bins of the scaled, rounded ROI; Argmax is
//     the in-map flat index (-1 for an empty bin).
// Device: warpctc / edit_distance / roi_pool on the kernel library's seqdet.hip
// launchers (the ones the Python operators use on a HIP place); nce / hsigmoid as
// one-source functors (any_place.h) with float atomics for the weight rows.
#include <hip/hip_runtime.h>
#include <math.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "any_place.h"
#include "kernel_lib.h"

extern "C" {
int pa_ctc_loss(const float* x, const int* xoff, const int* labels, const int* loff, int N, int Ttot, int C, int Smax,
                int blank, float* lse, float* alpha, float* beta, float* loss, float* grad, hipStream_t st);
int pa_roi_pool_fwd(const float* x, const float* rois, const int* bid, int R, int C, int H, int W, int PH, int PW,
                    float scale, float* out, long long* argmax, hipStream_t st);
int pa_roi_pool_bwd(const float* dy, const long long* argmax, const int* bid, int R, int C, int H, int W, int PH,
                    int PW, float* dx, hipStream_t st);
int pa_edit_distance(const long long* hyp, const int* hoff, const long long* ref, const int* roff, int N, int wsw,
                     int* ws, int normalized, float* out, hipStream_t st);
}

namespace pa {
namespace {

constexpr int64_t kSerial = int64_t(1) << 60;  // any::run grain that keeps a host loop on one thread

__host__ __device__ inline void acc_add(float* p, float v) {
#if defined(__HIP_DEVICE_COMPILE__)
  atomicAdd(p, v);
#else
  *p += v;
#endif
}

Tensor host_of(const OpRun& r, const Tensor& t) {
  if (t.device < 0) return t;
  Tensor h = t.to(-1, r.ctx.stream);
  device_stream_sync(r.ctx.stream);
  return h;
}

std::vector<int64_t> ids_of(const Tensor& h) {
  std::vector<int64_t> v((size_t)h.numel());
  if (h.dtype == DT::INT64) memcpy(v.data(), h.raw(), v.size() * 8);
  else if (h.dtype == DT::INT32)
    for (size_t i = 0; i < v.size(); ++i) v[i] = h.data<int32_t>()[i];
  else fail("expected integer ids, got %s", dt_name(h.dtype));
  return v;
}

const std::vector<size_t>& lod_of(const Tensor& t, const char* what) {
  PA_CHECK(!t.lod.empty(), "%s has no LoD", what);
  return t.lod.back();
}

// ---------------------------------------------------------------- warpctc (host lattice)
inline float lse2(float a, float b) {
  if (a == -INFINITY) return b;
  if (b == -INFINITY) return a;
  const float m = a > b ? a : b;
  return m + log1pf(expf(-fabsf(a - b)));
}

// loss of one sequence; grad rows [T, C] when g != nullptr (d loss / d logits)
float ctc_one(const float* x, int64_t T, int64_t C, const int64_t* lab, int64_t L, int64_t blank, float* g) {
  if (T <= 0) {
    if (g) memset(g, 0, sizeof(float) * (size_t)(T * C));
    return 0.f;
  }
  const int64_t S = 2 * L + 1;
  std::vector<float> lp((size_t)(T * C)), al((size_t)(T * S), -INFINITY), be((size_t)(T * S), -INFINITY);
  for (int64_t t = 0; t < T; ++t) {
    const float* xr = x + t * C;
    float m = -INFINITY;
    for (int64_t c = 0; c < C; ++c) m = std::max(m, xr[c]);
    double s = 0;
    for (int64_t c = 0; c < C; ++c) s += exp((double)(xr[c] - m));
    const float ls = m + (float)log(s);
    for (int64_t c = 0; c < C; ++c) lp[(size_t)(t * C + c)] = xr[c] - ls;
  }
  auto sym = [&](int64_t s) { return (s & 1) ? lab[s >> 1] : blank; };
  al[0] = lp[(size_t)blank];
  if (S > 1) al[1] = lp[(size_t)sym(1)];
  for (int64_t t = 1; t < T; ++t)
    for (int64_t s = 0; s < S; ++s) {
      float v = al[(size_t)((t - 1) * S + s)];
      if (s >= 1) v = lse2(v, al[(size_t)((t - 1) * S + s - 1)]);
      if (s >= 2 && sym(s) != blank && sym(s) != sym(s - 2)) v = lse2(v, al[(size_t)((t - 1) * S + s - 2)]);
      al[(size_t)(t * S + s)] = v == -INFINITY ? v : v + lp[(size_t)(t * C + sym(s))];
    }
  const float lpz = S >= 2 ? lse2(al[(size_t)((T - 1) * S + S - 1)], al[(size_t)((T - 1) * S + S - 2)])
                           : al[(size_t)((T - 1) * S + S - 1)];
  if (lpz == -INFINITY) {
    if (g) memset(g, 0, sizeof(float) * (size_t)(T * C));
    return 0.f;
  }
  if (!g) return -lpz;
  be[(size_t)((T - 1) * S + S - 1)] = lp[(size_t)((T - 1) * C + sym(S - 1))];
  if (S > 1) be[(size_t)((T - 1) * S + S - 2)] = lp[(size_t)((T - 1) * C + sym(S - 2))];
  for (int64_t t = T - 2; t >= 0; --t)
    for (int64_t s = S - 1; s >= 0; --s) {
      float v = be[(size_t)((t + 1) * S + s)];
      if (s + 1 < S) v = lse2(v, be[(size_t)((t + 1) * S + s + 1)]);
      if (s + 2 < S && sym(s) != blank && sym(s) != sym(s + 2)) v = lse2(v, be[(size_t)((t + 1) * S + s + 2)]);
      be[(size_t)(t * S + s)] = v == -INFINITY ? v : v + lp[(size_t)(t * C + sym(s))];
    }
  std::vector<float> acc((size_t)C);
  for (int64_t t = 0; t < T; ++t) {
    std::fill(acc.begin(), acc.end(), -INFINITY);
    for (int64_t s = 0; s < S; ++s) {
      const float v = al[(size_t)(t * S + s)] + be[(size_t)(t * S + s)];
      if (v != -INFINITY) acc[(size_t)sym(s)] = lse2(acc[(size_t)sym(s)], v);
    }
    for (int64_t c = 0; c < C; ++c) {
      const float l = lp[(size_t)(t * C + c)];
      const float occ = acc[(size_t)c] == -INFINITY ? 0.f : expf(acc[(size_t)c] - l + lpz * -1.f);
      g[t * C + c] = expf(l) - occ;
    }
  }
  return -lpz;
}

struct Ctc {
  std::vector<size_t> xo, lo;
  std::vector<int64_t> lab;
  int64_t N, C, blank;
  bool norm;
};

Ctc ctc_of(const OpRun& r, const Tensor& x, const Tensor& label) {
  Ctc c;
  c.xo = lod_of(x, "warpctc: Logits");
  c.lo = lod_of(label, "warpctc: Label");
  PA_CHECK(c.xo.size() == c.lo.size(), "warpctc: Logits and Label hold different sequence counts");
  c.lab = ids_of(host_of(r, label));
  c.N = (int64_t)c.xo.size() - 1;
  c.C = x.dims[1];
  c.blank = r.op.GetInt("blank", 0);
  c.norm = r.op.GetBool("norm_by_times", false);
  PA_CHECK(c.blank >= 0 && c.blank < c.C, "warpctc: blank out of range");
  return c;
}

// device lattice: loss [N] and (grad != nullptr) d loss / d logits [Ttot, C]
void ctc_device(const OpRun& r, const Ctc& c, const float* x, int64_t Ttot, float* loss, float* grad) {
  int64_t Lmax = 0;
  for (int64_t n = 0; n < c.N; ++n) Lmax = std::max<int64_t>(Lmax, (int64_t)(c.lo[(size_t)n + 1] - c.lo[(size_t)n]));
  const int64_t Smax = 2 * Lmax + 1;
  PA_CHECK(Smax <= 8192, "warpctc: label too long for the device lattice");
  std::vector<int> offs;
  for (size_t v : c.xo) offs.push_back((int)v);
  for (size_t v : c.lo) offs.push_back((int)v);
  for (int64_t v : c.lab) offs.push_back((int)v);
  const int* d = (const int*)device_upload(r, "@ctc_meta@", offs.data(), offs.size() * sizeof(int));
  const int* xoff = d;
  const int* loff = d + c.xo.size();
  const int* labels = d + c.xo.size() + c.lo.size();
  float* lse = device_workspace(r, "@ctc_lse@", std::max<int64_t>(Ttot, 1));
  float* alpha = device_workspace(r, "@ctc_alpha@", std::max<int64_t>(Ttot * Smax, 1));
  float* beta = device_workspace(r, "@ctc_beta@", std::max<int64_t>(Ttot * Smax, 1));
  PA_KL(pa_ctc_loss(x, xoff, labels, loff, (int)c.N, (int)Ttot, (int)c.C, (int)Smax, (int)c.blank, lse, alpha, beta,
                    loss, grad, dev_stream(r)));
}

void k_warpctc(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor x = r.in("Logits");
  const Ctc c = ctc_of(r, x, r.in("Label"));
  const int64_t Ttot = x.dims[0];
  const float* xp = any::f32(x, dev);
  const int place = dev ? r.ctx.device : -1;
  Tensor loss, grad;
  float* lp = loss.alloc<float>({c.N, 1}, place);
  Tensor* gt = r.out("WarpCTCGrad");
  float* gp = gt ? grad.alloc<float>(x.dims, place) : nullptr;
  if (dev) {
    ctc_device(r, c, xp, Ttot, lp, gp);
  } else {
    parallel_for(c.N, 1, [&](int64_t a, int64_t b) {
      for (int64_t n = a; n < b; ++n) {
        const int64_t t0 = (int64_t)c.xo[(size_t)n], T = (int64_t)c.xo[(size_t)n + 1] - t0;
        const int64_t l0 = (int64_t)c.lo[(size_t)n], L = (int64_t)c.lo[(size_t)n + 1] - l0;
        lp[n] = ctc_one(xp + t0 * c.C, T, c.C, c.lab.data() + l0, L, c.blank, gp ? gp + t0 * c.C : nullptr);
      }
    });
  }
  *r.out("Loss") = loss;
  if (gt) *gt = grad;
}

struct CtcScale {  // g[row] *= dloss[seq(row)] (/ T when norm)
  float* g;
  const float* dloss;
  const int* seq;
  const int* len;
  int64_t C;
  int norm;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t row = i / C;
    const int s = seq[row];
    float w = dloss ? dloss[s] : 0.f;
    if (norm) w /= (float)(len[s] > 0 ? len[s] : 1);
    g[i] *= w;
  }
};

void k_warpctc_grad(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor x = r.in("Logits");
  const Ctc c = ctc_of(r, x, r.in("Label"));
  Tensor* dl = r.in_opt("Loss@GRAD");
  const int64_t Ttot = x.dims[0];
  const float* xp = any::f32(x, dev);
  const int place = dev ? r.ctx.device : -1;
  Tensor grad;
  float* gp = grad.alloc<float>(x.dims, place);
  if (dev) {
    float* loss = device_workspace(r, "@ctc_loss@", std::max<int64_t>(c.N, 1));
    ctc_device(r, c, xp, Ttot, loss, gp);
  } else {
    parallel_for(c.N, 1, [&](int64_t a, int64_t b) {
      for (int64_t n = a; n < b; ++n) {
        const int64_t t0 = (int64_t)c.xo[(size_t)n], T = (int64_t)c.xo[(size_t)n + 1] - t0;
        const int64_t l0 = (int64_t)c.lo[(size_t)n], L = (int64_t)c.lo[(size_t)n + 1] - l0;
        ctc_one(xp + t0 * c.C, T, c.C, c.lab.data() + l0, L, c.blank, gp + t0 * c.C);
      }
    });
  }
  std::vector<int> meta((size_t)(Ttot + c.N));
  for (int64_t n = 0; n < c.N; ++n) {
    for (size_t t = c.xo[(size_t)n]; t < c.xo[(size_t)n + 1]; ++t) meta[t] = (int)n;
    meta[(size_t)(Ttot + n)] = (int)(c.xo[(size_t)n + 1] - c.xo[(size_t)n]);
  }
  const int* m = any::ints(r, dev, "@ctc_rowseq@", meta);
  any::run(r, dev, Ttot * c.C, CtcScale{gp, dl ? any::f32(*dl, dev) : nullptr, m, m + Ttot, c.C, c.norm ? 1 : 0});
  grad.lod = x.lod;
  *r.out("Logits@GRAD") = grad;
}

// ---------------------------------------------------------------- edit_distance
int levenshtein(const int64_t* a, int64_t la, const int64_t* b, int64_t lb) {
  std::vector<int> prev((size_t)lb + 1), cur((size_t)lb + 1);
  for (int64_t j = 0; j <= lb; ++j) prev[(size_t)j] = (int)j;
  for (int64_t i = 1; i <= la; ++i) {
    cur[0] = (int)i;
    for (int64_t j = 1; j <= lb; ++j)
      cur[(size_t)j] = std::min(std::min(prev[(size_t)j] + 1, cur[(size_t)j - 1] + 1),
                                prev[(size_t)j - 1] + (a[i - 1] != b[j - 1] ? 1 : 0));
    std::swap(prev, cur);
  }
  return prev[(size_t)lb];
}

void k_edit_distance(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& hyp = r.in("Hyps");
  Tensor& ref = r.in("Refs");
  const auto& ho = lod_of(hyp, "edit_distance: Hyps");
  const auto& ro = lod_of(ref, "edit_distance: Refs");
  PA_CHECK(ho.size() == ro.size(), "edit_distance: Hyps and Refs hold different sequence counts");
  const int64_t N = (int64_t)ho.size() - 1;
  const bool norm = r.op.GetBool("normalized", false);
  const int place = dev ? r.ctx.device : -1;
  Tensor out, num;
  float* op = out.alloc<float>({N, 1}, place);
  if (dev && hyp.dtype == DT::INT64 && ref.dtype == DT::INT64 && hyp.device >= 0 && ref.device >= 0 && N > 0) {
    int64_t lbmax = 0;
    std::vector<int> offs;
    for (size_t v : ho) offs.push_back((int)v);
    for (size_t i = 0; i < ro.size(); ++i) {
      offs.push_back((int)ro[i]);
      if (i) lbmax = std::max<int64_t>(lbmax, (int64_t)(ro[i] - ro[i - 1]));
    }
    const int* d = (const int*)device_upload(r, "@ed_off@", offs.data(), offs.size() * sizeof(int));
    const int wsw = (int)lbmax + 1;
    int* ws = (int*)device_workspace(r, "@ed_ws@", N * 2 * wsw);
    PA_KL(pa_edit_distance((const long long*)hyp.raw(), d, (const long long*)ref.raw(), d + ho.size(), (int)N, wsw, ws,
                           norm ? 1 : 0, op, dev_stream(r)));
  } else {
    const std::vector<int64_t> h = ids_of(host_of(r, hyp)), f = ids_of(host_of(r, ref));
    std::vector<float> d((size_t)N);
    for (int64_t n = 0; n < N; ++n) {
      const int64_t la = (int64_t)(ho[(size_t)n + 1] - ho[(size_t)n]), lb = (int64_t)(ro[(size_t)n + 1] - ro[(size_t)n]);
      float v = (float)levenshtein(h.data() + ho[(size_t)n], la, f.data() + ro[(size_t)n], lb);
      if (norm) v /= (float)std::max<int64_t>(lb, 1);
      d[(size_t)n] = v;
    }
    if (dev) {
      if (N) device_copy(op, place, d.data(), -1, sizeof(float) * (size_t)N, r.ctx.stream);
      device_stream_sync(r.ctx.stream);
    } else if (N) {
      memcpy(op, d.data(), sizeof(float) * (size_t)N);
    }
  }
  Tensor hn;
  *hn.alloc<int64_t>({1}, -1) = N;
  if (dev) {
    num.alloc<int64_t>({1}, place);
    device_copy(num.raw(), place, hn.raw(), -1, 8, r.ctx.stream);
    device_stream_sync(r.ctx.stream);
  } else {
    num = hn;
  }
  *r.out("Out") = out;
  *r.out("SequenceNum") = num;
}

// ---------------------------------------------------------------- nce
__host__ __device__ inline uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

struct NceFwd {  // one (n, j) sample: logit, sigmoid, sampled label
  const float *x, *W, *b;
  const int64_t *lab, *custom;
  int64_t *labels;
  float* o;
  int64_t D, nt, k, C, ncustom;
  uint64_t seed;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t n = i / (nt + k), j = i % (nt + k);
    int64_t l;
    if (j < nt) l = lab[n * nt + j];
    else if (ncustom) l = custom[(j - nt) % ncustom];
    else l = (int64_t)(mix64(seed * 0x100000001b3ull + (uint64_t)(n * k + (j - nt))) % (uint64_t)C);
    labels[i] = l;
    float z = b ? b[l] : 0.f;
    for (int64_t d = 0; d < D; ++d) z += x[n * D + d] * W[l * D + d];
    o[i] = 1.f / (1.f + expf(-z));
  }
};

struct NceCost {
  const float *o, *sw;
  float* cost;
  int64_t nt, k;
  float bb;
  __host__ __device__ void operator()(int64_t n) const {
    float s = 0.f;
    for (int64_t j = 0; j < nt + k; ++j) {
      const float v = o[n * (nt + k) + j];
      s += j < nt ? -logf(v / (v + bb)) : -logf(bb / (v + bb));
    }
    cost[n] = sw ? s * sw[n] : s;
  }
};

void k_nce(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("Input");
  Tensor& W = r.in("Weight");
  Tensor* Bt = r.in_opt("Bias");
  Tensor* SW = r.in_opt("SampleWeight");
  const int64_t N = x.dims[0], D = x.dims[1];
  const std::vector<int64_t> lab = ids_of(host_of(r, r.in("Label")));
  PA_CHECK(N > 0 && (int64_t)lab.size() % N == 0, "nce: Label rows must match Input");
  const int64_t nt = (int64_t)lab.size() / N, k = r.op.GetInt("num_neg_samples", 10);
  const int64_t C = r.op.GetInt("num_total_classes", 2);
  const auto custom = r.op.GetInts("custom_neg_classes");
  const int place = dev ? r.ctx.device : -1;
  const int64_t* labp = lab.data();
  const int64_t* cus = custom.data();
  if (dev) {
    labp = (const int64_t*)device_upload(r, "@nce_lab@", lab.data(), lab.size() * 8);
    cus = custom.empty() ? nullptr : (const int64_t*)device_upload(r, "@nce_custom@", custom.data(), custom.size() * 8);
  }
  Tensor cost, logits, labels;
  float* cp = cost.alloc<float>({N, 1}, place);
  float* op = logits.alloc<float>({N, nt + k}, place);
  int64_t* lp = labels.alloc<int64_t>({N, nt + k}, place);
  any::run(r, dev, N * (nt + k),
           NceFwd{any::f32(x, dev), any::f32(W, dev), Bt ? any::f32(*Bt, dev) : nullptr, labp, cus, lp, op, D, nt, k, C,
                  (int64_t)custom.size(), (uint64_t)r.op.GetInt("seed", 0)},
           64);
  any::run(r, dev, N, NceCost{op, SW ? any::f32(*SW, dev) : nullptr, cp, nt, k, (float)k / (float)C}, 64);
  *r.out("Cost") = cost;
  if (Tensor* t = r.out("SampleLogits")) *t = logits;
  if (Tensor* t = r.out("SampleLabels")) *t = labels;
}

struct NceDz {  // dz[n, j] = d cost / d logit
  const float *o, *dcost, *sw;
  float* dz;
  int64_t nt, k;
  float bb;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t n = i / (nt + k), j = i % (nt + k);
    const float v = o[i];
    float g = j < nt ? -(1.f - v) * bb / (v + bb) : v * (1.f - v) / (v + bb);
    float w = dcost ? dcost[n] : 0.f;
    if (sw) w *= sw[n];
    dz[i] = g * w;
  }
};

struct NceBack {  // one (n, j): dX[n] += dz W[l]; dW[l] += dz x[n]; dB[l] += dz
  const float *x, *W, *dz;
  const int64_t* labels;
  float *dx, *dW, *dB;
  int64_t D, nt, k;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t n = i / (nt + k);
    const int64_t l = labels[i];
    const float g = dz[i];
    for (int64_t d = 0; d < D; ++d) {
      if (dx) acc_add(dx + n * D + d, g * W[l * D + d]);
      if (dW) acc_add(dW + l * D + d, g * x[n * D + d]);
    }
    if (dB) acc_add(dB + l, g);
  }
};

void k_nce_grad(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("Input");
  Tensor& W = r.in("Weight");
  Tensor* Bt = r.in_opt("Bias");
  Tensor* SW = r.in_opt("SampleWeight");
  Tensor& o = r.in("SampleLogits");
  Tensor& labels = r.in("SampleLabels");
  Tensor* dc = r.in_opt("Cost@GRAD");
  const int64_t N = x.dims[0], D = x.dims[1], k = r.op.GetInt("num_neg_samples", 10);
  const int64_t C = r.op.GetInt("num_total_classes", 2);
  const int64_t nt = o.dims[1] - k;
  PA_CHECK(labels.dtype == DT::INT64 && (labels.device >= 0) == dev, "nce_grad: SampleLabels must be int64 on the place");
  const int place = dev ? r.ctx.device : -1;
  Tensor dz, dX, dWt, dBt;
  float* dzp = dz.alloc<float>({N, nt + k}, place);
  any::run(r, dev, N * (nt + k),
           NceDz{any::f32(o, dev), dc ? any::f32(*dc, dev) : nullptr, SW ? any::f32(*SW, dev) : nullptr, dzp, nt, k,
                 (float)k / (float)C});
  Tensor* dxo = r.out("Input@GRAD");
  Tensor* dwo = r.out("Weight@GRAD");
  Tensor* dbo = Bt ? r.out("Bias@GRAD") : nullptr;
  float* dx = dxo ? dX.alloc<float>(x.dims, place) : nullptr;
  float* dw = dwo ? dWt.alloc<float>(W.dims, place) : nullptr;
  float* db = dbo ? dBt.alloc<float>(Bt->dims, place) : nullptr;
  if (dx) any::zero(r, dev, dx, x.numel());
  if (dw) any::zero(r, dev, dw, W.numel());
  if (db) any::zero(r, dev, db, Bt->numel());
  // host: one chunk (the scatter into W rows is not partitioned); device: atomics
  any::run(r, dev, N * (nt + k),
           NceBack{any::f32(x, dev), any::f32(W, dev), dzp, labels.data<int64_t>(), dx, dw, db, D, nt, k},
           dev ? 4096 : kSerial);
  if (dxo) *dxo = dX;
  if (dwo) *dwo = dWt;
  if (dbo) *dbo = dBt;
}

// ---------------------------------------------------------------- hierarchical_sigmoid
struct HsPre {  // pre[n, j] (unclipped when raw) over the code of label n
  const float *x, *W, *b;
  const int64_t* lab;
  float* pre;
  int64_t D, L, C;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t n = i / L, j = i % L;
    const int64_t c = lab[n] + C;
    int64_t len = 0;
    while ((c >> (len + 1)) > 0) ++len;  // floor(log2 c)
    if (j >= len) {
      pre[i] = 0.f;
      return;
    }
    const int64_t node = (c >> (j + 1)) - 1;
    float z = b ? b[node] : 0.f;
    for (int64_t d = 0; d < D; ++d) z += x[n * D + d] * W[node * D + d];
    pre[i] = z;
  }
};

__host__ __device__ inline float softplus_t(float v) { return v > 20.f ? v : log1pf(expf(v)); }

struct HsOut {
  const float* raw;
  const int64_t* lab;
  float *pre, *out;
  int64_t L, C;
  __host__ __device__ void operator()(int64_t n) const {
    const int64_t c = lab[n] + C;
    float s = 0.f;
    for (int64_t j = 0; j < L; ++j) {
      int64_t len = 0;
      while ((c >> (len + 1)) > 0) ++len;
      const float p = j < len ? fminf(fmaxf(raw[n * L + j], -40.f), 40.f) : 0.f;
      if (pre) pre[n * L + j] = p;
      if (j < len) s += softplus_t(p) - (float)((c >> j) & 1) * p;
    }
    out[n] = s;
  }
};

int64_t code_len(int64_t C) {
  int64_t L = 0;
  while ((int64_t(1) << L) < C) ++L;  // bit_length(C - 1)
  return L;
}

void k_hsigmoid(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("X");
  Tensor& W = r.in("W");
  Tensor* Bt = r.in_opt("Bias");
  Tensor& lab = r.in("Label");
  PA_CHECK(lab.dtype == DT::INT64, "hierarchical_sigmoid: int64 Label expected");
  const int64_t N = x.dims[0], D = x.dims[1], C = r.op.GetInt("num_classes", 2), L = code_len(C);
  const int place = dev ? r.ctx.device : -1;
  Tensor raw, pre, out;
  float* rp = raw.alloc<float>({N, L}, place);
  float* pp = pre.alloc<float>({N, L}, place);
  float* op = out.alloc<float>({N, 1}, place);
  const int64_t* lp = lab.data<int64_t>();
  PA_CHECK((lab.device >= 0) == dev, "hierarchical_sigmoid: Label on another place");
  any::run(r, dev, N * L, HsPre{any::f32(x, dev), any::f32(W, dev), Bt ? any::f32(*Bt, dev) : nullptr, lp, rp, D, L, C}, 64);
  any::run(r, dev, N, HsOut{rp, lp, pp, op, L, C}, 64);
  *r.out("Out") = out;
  if (Tensor* t = r.out("PreOut")) *t = pre;
}

struct HsBack {  // dpre of (n, j), then the row scatters
  const float *x, *W, *raw, *dout;
  const int64_t* lab;
  float *dx, *dW, *dB;
  int64_t D, L, C;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t n = i / L, j = i % L;
    const int64_t c = lab[n] + C;
    int64_t len = 0;
    while ((c >> (len + 1)) > 0) ++len;
    if (j >= len) return;
    const float z = raw[i];
    if (z < -40.f || z > 40.f) return;  // clipped: no gradient
    const float s = 1.f / (1.f + expf(-z));
    const float g = (dout ? dout[n] : 0.f) * (s - (float)((c >> j) & 1));
    const int64_t node = (c >> (j + 1)) - 1;
    for (int64_t d = 0; d < D; ++d) {
      if (dx) acc_add(dx + n * D + d, g * W[node * D + d]);
      if (dW) acc_add(dW + node * D + d, g * x[n * D + d]);
    }
    if (dB) acc_add(dB + node, g);
  }
};

void k_hsigmoid_grad(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("X");
  Tensor& W = r.in("W");
  Tensor* Bt = r.in_opt("Bias");
  Tensor& lab = r.in("Label");
  Tensor* dout = r.in_opt("Out@GRAD");
  const int64_t N = x.dims[0], D = x.dims[1], C = r.op.GetInt("num_classes", 2), L = code_len(C);
  const int place = dev ? r.ctx.device : -1;
  const float *xp = any::f32(x, dev), *wp = any::f32(W, dev), *bp = Bt ? any::f32(*Bt, dev) : nullptr;
  const int64_t* lp = lab.data<int64_t>();
  Tensor raw, dX, dWt, dBt;
  float* rp = raw.alloc<float>({N, L}, place);
  any::run(r, dev, N * L, HsPre{xp, wp, bp, lp, rp, D, L, C}, 64);
  Tensor* dxo = r.out("X@GRAD");
  Tensor* dwo = r.out("W@GRAD");
  Tensor* dbo = Bt ? r.out("Bias@GRAD") : nullptr;
  float* dx = dxo ? dX.alloc<float>(x.dims, place) : nullptr;
  float* dw = dwo ? dWt.alloc<float>(W.dims, place) : nullptr;
  float* db = dbo ? dBt.alloc<float>(Bt->dims, place) : nullptr;
  if (dx) any::zero(r, dev, dx, x.numel());
  if (dw) any::zero(r, dev, dw, W.numel());
  if (db) any::zero(r, dev, db, Bt->numel());
  any::run(r, dev, N * L, HsBack{xp, wp, rp, dout ? any::f32(*dout, dev) : nullptr, lp, dx, dw, db, D, L, C},
           dev ? 4096 : kSerial);
  if (dxo) *dxo = dX;
  if (dwo) *dwo = dWt;
  if (dbo) *dbo = dBt;
}

// ---------------------------------------------------------------- roi_pool
std::vector<int> roi_batch_ids(const Tensor& rois) {
  std::vector<int> ids;
  if (rois.lod.empty()) {
    ids.assign((size_t)rois.dims[0], 0);
    return ids;
  }
  const auto& off = rois.lod[0];
  for (size_t b = 0; b + 1 < off.size(); ++b)
    for (size_t i = off[b]; i < off[b + 1]; ++i) ids.push_back((int)b);
  PA_CHECK((int64_t)ids.size() == rois.dims[0], "roi_pool: ROIs LoD does not cover its rows");
  return ids;
}

inline int64_t round_away(float v) { return (int64_t)(v < 0 ? -floorf(-v + 0.5f) : floorf(v + 0.5f)); }

void k_roi_pool(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("X");
  Tensor& rois = r.in("ROIs");
  const int64_t B = x.dims[0], C = x.dims[1], H = x.dims[2], W = x.dims[3], R = rois.dims[0];
  const int64_t PH = r.op.GetInt("pooled_height", 1), PW = r.op.GetInt("pooled_width", 1);
  const float sc = r.op.GetFloat("spatial_scale", 1.f);
  const std::vector<int> bid = roi_batch_ids(rois);
  for (int b : bid) PA_CHECK(b < B, "roi_pool: ROI batch index out of range");
  const int place = dev ? r.ctx.device : -1;
  Tensor out, am;
  float* op = out.alloc<float>({R, C, PH, PW}, place);
  int64_t* ap = am.alloc<int64_t>({R, C, PH, PW}, place);
  if (dev) {
    const int* db = (const int*)device_upload(r, "@roi_bid@", bid.data(), bid.size() * sizeof(int));
    PA_KL(pa_roi_pool_fwd(any::f32(x, true), any::f32(rois, true), db, (int)R, (int)C, (int)H, (int)W, (int)PH,
                          (int)PW, sc, op, (long long*)ap, dev_stream(r)));
  } else {
    const float *xp = any::f32(x, false), *rp = any::f32(rois, false);
    parallel_for(R, 1, [&](int64_t a, int64_t e) {
      for (int64_t i = a; i < e; ++i) {
        const int64_t x1 = round_away(rp[i * 4] * sc), y1 = round_away(rp[i * 4 + 1] * sc);
        const int64_t x2 = round_away(rp[i * 4 + 2] * sc), y2 = round_away(rp[i * 4 + 3] * sc);
        const int64_t rw = std::max<int64_t>(x2 - x1 + 1, 1), rh = std::max<int64_t>(y2 - y1 + 1, 1);
        for (int64_t py = 0; py < PH; ++py) {
          const int64_t hs = std::min(std::max<int64_t>((int64_t)floor((double)(py * rh) / PH) + y1, 0), H);
          const int64_t he = std::min(std::max<int64_t>((int64_t)ceil((double)((py + 1) * rh) / PH) + y1, 0), H);
          for (int64_t px = 0; px < PW; ++px) {
            const int64_t ws = std::min(std::max<int64_t>((int64_t)floor((double)(px * rw) / PW) + x1, 0), W);
            const int64_t we = std::min(std::max<int64_t>((int64_t)ceil((double)((px + 1) * rw) / PW) + x1, 0), W);
            for (int64_t c = 0; c < C; ++c) {
              const int64_t o = ((i * C + c) * PH + py) * PW + px;
              if (he <= hs || we <= ws) {
                op[o] = 0.f;
                ap[o] = -1;
                continue;
              }
              const float* plane = xp + ((int64_t)bid[(size_t)i] * C + c) * H * W;
              float best = -INFINITY;
              int64_t at = -1;
              for (int64_t h = hs; h < he; ++h)
                for (int64_t w = ws; w < we; ++w)
                  if (at < 0 || plane[h * W + w] > best) {
                    best = plane[h * W + w];
                    at = h * W + w;
                  }
              op[o] = best;
              ap[o] = at;
            }
          }
        }
      }
    });
  }
  *r.out("Out") = out;
  if (Tensor* t = r.out("Argmax")) *t = am;
}

void k_roi_pool_grad(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("X");
  Tensor& rois = r.in("ROIs");
  Tensor& am = r.in("Argmax");
  Tensor* dy = r.in_opt("Out@GRAD");
  const int64_t C = x.dims[1], H = x.dims[2], W = x.dims[3], R = rois.dims[0];
  const int64_t PH = r.op.GetInt("pooled_height", 1), PW = r.op.GetInt("pooled_width", 1);
  PA_CHECK(am.dtype == DT::INT64 && am.numel() == R * C * PH * PW, "roi_pool_grad: Argmax does not match");
  const std::vector<int> bid = roi_batch_ids(rois);
  const int place = dev ? r.ctx.device : -1;
  Tensor dX;
  float* dx = dX.alloc<float>(x.dims, place);
  any::zero(r, dev, dx, x.numel());
  if (dy && R) {
    if (dev) {
      const int* db = (const int*)device_upload(r, "@roi_bid@", bid.data(), bid.size() * sizeof(int));
      PA_KL(pa_roi_pool_bwd(any::f32(*dy, true), (const long long*)am.raw(), db, (int)R, (int)C, (int)H, (int)W,
                            (int)PH, (int)PW, dx, dev_stream(r)));
    } else {
      const float* gp = any::f32(*dy, false);
      const int64_t* ap = am.data<int64_t>();
      for (int64_t i = 0; i < R * C * PH * PW; ++i) {
        if (ap[i] < 0) continue;
        const int64_t c = (i / (PW * PH)) % C, roi = i / (PW * PH * C);
        dx[((int64_t)bid[(size_t)roi] * C + c) * H * W + ap[i]] += gp[i];
      }
    }
  }
  *r.out("X@GRAD") = dX;
}

}  // namespace

#define PA_ANY_KERNEL(name, fn) \
  PA_HOST_KERNEL(name, fn);     \
  PA_DEVICE_KERNEL(name, fn)
PA_ANY_KERNEL(warpctc, k_warpctc);
PA_ANY_KERNEL(warpctc_grad, k_warpctc_grad);
PA_ANY_KERNEL(edit_distance, k_edit_distance);
PA_ANY_KERNEL(nce, k_nce);
PA_ANY_KERNEL(nce_grad, k_nce_grad);
PA_ANY_KERNEL(hierarchical_sigmoid, k_hsigmoid);
PA_ANY_KERNEL(hierarchical_sigmoid_grad, k_hsigmoid_grad);
PA_ANY_KERNEL(roi_pool, k_roi_pool);
PA_ANY_KERNEL(roi_pool_grad, k_roi_pool_grad);
#undef PA_ANY_KERNEL

void link_loss_kernels() {}

}  // namespace pa
