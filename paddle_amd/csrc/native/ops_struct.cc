// Host kernels of the structured-prediction operators: linear_chain_crf /
// linear_chain_crf_grad and crf_decoding.
//
// Semantics (reference operators/linear_chain_crf_op.h:54-190, crf_decoding_op.h;
// the Python kernels of operators/structured_ops.py compute the same functions):
// Transition is [D + 2, D]: row 0 the start weights, row 1 the end weights, rows
// 2.. the tag -> tag matrix.  LogLikelihood is -log p(label | emission) per
// sequence (the NEGATIVE log-likelihood, the cost the book model minimises).
// The gradient is the marginal-minus-indicator form from the forward / backward
// recursions in log space.  crf_decoding is Viterbi; with Label it outputs 1 where
// the decoded tag matches.
#include <math.h>
#include <string.h>

#include <algorithm>
#include <limits>
#include <vector>

#include "framework.h"
#include "struct_common.h"

namespace pa {
namespace crf {

void forward_backward(const float* em, const float* tr, const int64_t* y, int64_t L, int64_t D, double* alpha,
                      double* beta, double* nll_out) {
  const float *start = tr, *end = tr + D, *T = tr + 2 * D;
  for (int64_t j = 0; j < D; ++j) alpha[j] = (double)start[j] + em[j];
  for (int64_t t = 1; t < L; ++t)
    for (int64_t j = 0; j < D; ++j) {
      double m = -std::numeric_limits<double>::infinity();
      for (int64_t i = 0; i < D; ++i) m = std::max(m, alpha[(t - 1) * D + i] + T[i * D + j]);
      double s = 0;
      for (int64_t i = 0; i < D; ++i) s += exp(alpha[(t - 1) * D + i] + T[i * D + j] - m);
      alpha[t * D + j] = m + log(s) + em[t * D + j];
    }
  double m = -std::numeric_limits<double>::infinity();
  for (int64_t j = 0; j < D; ++j) m = std::max(m, alpha[(L - 1) * D + j] + end[j]);
  double s = 0;
  for (int64_t j = 0; j < D; ++j) s += exp(alpha[(L - 1) * D + j] + end[j] - m);
  const double logz = m + log(s);
  double score = (double)start[y[0]] + em[y[0]];
  for (int64_t t = 1; t < L; ++t) score += (double)T[y[t - 1] * D + y[t]] + em[t * D + y[t]];
  score += end[y[L - 1]];
  *nll_out = logz - score;
  if (!beta) return;
  for (int64_t j = 0; j < D; ++j) beta[(L - 1) * D + j] = end[j];
  for (int64_t t = L - 2; t >= 0; --t)
    for (int64_t i = 0; i < D; ++i) {
      double mm = -std::numeric_limits<double>::infinity();
      for (int64_t j = 0; j < D; ++j) mm = std::max(mm, T[i * D + j] + em[(t + 1) * D + j] + beta[(t + 1) * D + j]);
      double ss = 0;
      for (int64_t j = 0; j < D; ++j) ss += exp(T[i * D + j] + em[(t + 1) * D + j] + beta[(t + 1) * D + j] - mm);
      beta[t * D + i] = mm + log(ss);
    }
  // stash logZ for the gradient in nll's slot pair: the caller recomputes it
}

}  // namespace crf

namespace {

float* f32(Tensor& t) {
  if (t.dtype != DT::FP32) throw Decline{};
  return t.data<float>();
}

std::vector<int64_t> labels_of(const Tensor& t) {
  std::vector<int64_t> v((size_t)t.numel());
  if (t.dtype == DT::INT64) memcpy(v.data(), t.raw(), v.size() * 8);
  else if (t.dtype == DT::INT32)
    for (size_t i = 0; i < v.size(); ++i) v[i] = t.data<int32_t>()[i];
  else throw Decline{};
  return v;
}

const std::vector<size_t> seq_off(const Tensor& x) {
  if (!x.lod.empty()) return x.lod.back();
  return {0, (size_t)x.dims[0]};
}

// Python-kernel-compatible intermediates (EmissionExps = exp(em - rowmax),
// TransitionExps = exp(tr), Alpha = row softmax of em)
void crf_intermediates(const OpRun& r, const float* em, const float* tr, int64_t T, int64_t D, const Tensor& trt) {
  if (Tensor* ee = r.out("EmissionExps")) {
    float* o = ee->alloc<float>({T, D}, -1);
    for (int64_t t = 0; t < T; ++t) {
      float m = em[t * D];
      for (int64_t j = 1; j < D; ++j) m = std::max(m, em[t * D + j]);
      for (int64_t j = 0; j < D; ++j) o[t * D + j] = expf(em[t * D + j] - m);
    }
  }
  if (Tensor* te = r.out("TransitionExps")) {
    float* o = te->alloc<float>(trt.dims, -1);
    for (int64_t i = 0; i < trt.numel(); ++i) o[i] = expf(tr[i]);
  }
  if (Tensor* al = r.out("Alpha")) {
    float* o = al->alloc<float>({T, D}, -1);
    for (int64_t t = 0; t < T; ++t) {
      float m = em[t * D];
      for (int64_t j = 1; j < D; ++j) m = std::max(m, em[t * D + j]);
      double s = 0;
      for (int64_t j = 0; j < D; ++j) s += exp((double)em[t * D + j] - m);
      for (int64_t j = 0; j < D; ++j) o[t * D + j] = (float)(exp((double)em[t * D + j] - m) / s);
    }
  }
}

void k_linear_chain_crf(const OpRun& r) {
  Tensor& emt = r.in("Emission");
  Tensor& trt = r.in("Transition");
  const int64_t T = emt.dims[0], D = emt.dims[1];
  PA_CHECK(trt.dims.size() == 2 && trt.dims[0] == D + 2 && trt.dims[1] == D, "linear_chain_crf: Transition [D+2, D]");
  const float *em = f32(emt), *tr = f32(trt);
  const std::vector<int64_t> y = labels_of(r.in("Label"));
  const auto off = seq_off(emt);
  const int64_t N = (int64_t)off.size() - 1;
  float* nll = r.out("LogLikelihood")->alloc<float>({N, 1}, -1);
  parallel_for(N, 1, [&](int64_t a, int64_t b) {
    std::vector<double> alpha;
    for (int64_t s = a; s < b; ++s) {
      const int64_t s0 = (int64_t)off[(size_t)s], L = (int64_t)off[(size_t)s + 1] - s0;
      if (L <= 0) {
        nll[s] = 0.f;
        continue;
      }
      alpha.resize((size_t)(L * D));
      double v;
      crf::forward_backward(em + s0 * D, tr, y.data() + s0, L, D, alpha.data(), nullptr, &v);
      nll[s] = (float)v;
    }
  });
  crf_intermediates(r, em, tr, T, D, trt);
}

void k_linear_chain_crf_grad(const OpRun& r) {
  Tensor& emt = r.in("Emission");
  Tensor& trt = r.in("Transition");
  Tensor* g = r.in_opt("LogLikelihood@GRAD");
  const int64_t T = emt.dims[0], D = emt.dims[1];
  const float *em = f32(emt), *tr = f32(trt);
  const float* gp = g ? f32(*g) : nullptr;
  const std::vector<int64_t> y = labels_of(r.in("Label"));
  const auto off = seq_off(emt);
  const int64_t N = (int64_t)off.size() - 1;
  std::vector<float> dem((size_t)(T * D), 0.f);
  std::vector<double> dtr((size_t)((D + 2) * D), 0.0);
  std::vector<double> alpha, beta;
  const float* Tm = tr + 2 * D;
  for (int64_t s = 0; s < N; ++s) {
    const int64_t s0 = (int64_t)off[(size_t)s], L = (int64_t)off[(size_t)s + 1] - s0;
    const double gs = gp ? gp[s] : 1.0;
    if (L <= 0 || gs == 0.0) continue;
    alpha.resize((size_t)(L * D));
    beta.resize((size_t)(L * D));
    const float* e = em + s0 * D;
    const int64_t* ys = y.data() + s0;
    double nll;
    crf::forward_backward(e, tr, ys, L, D, alpha.data(), beta.data(), &nll);
    // log Z from alpha (nll = logZ - score; recompute Z directly)
    double m = -1e300;
    for (int64_t j = 0; j < D; ++j) m = std::max(m, alpha[(size_t)((L - 1) * D + j)] + tr[D + j]);
    double z = 0;
    for (int64_t j = 0; j < D; ++j) z += exp(alpha[(size_t)((L - 1) * D + j)] + tr[D + j] - m);
    const double logz = m + log(z);
    for (int64_t t = 0; t < L; ++t)
      for (int64_t j = 0; j < D; ++j) {
        const double mg = exp(alpha[(size_t)(t * D + j)] + beta[(size_t)(t * D + j)] - logz);
        dem[(size_t)((s0 + t) * D + j)] = (float)(gs * (mg - (ys[t] == j ? 1.0 : 0.0)));
        if (t == 0) dtr[(size_t)j] += gs * (mg - (ys[0] == j ? 1.0 : 0.0));
        if (t == L - 1) dtr[(size_t)(D + j)] += gs * (mg - (ys[L - 1] == j ? 1.0 : 0.0));
      }
    for (int64_t t = 1; t < L; ++t) {
      for (int64_t i = 0; i < D; ++i)
        for (int64_t j = 0; j < D; ++j) {
          const double pr = exp(alpha[(size_t)((t - 1) * D + i)] + Tm[i * D + j] + e[t * D + j] +
                                beta[(size_t)(t * D + j)] - logz);
          dtr[(size_t)((2 + i) * D + j)] += gs * pr;
        }
      dtr[(size_t)((2 + ys[t - 1]) * D + ys[t])] -= gs;
    }
  }
  if (Tensor* de = r.out("Emission@GRAD")) {
    memcpy(de->alloc<float>(emt.dims, -1), dem.data(), dem.size() * sizeof(float));
    de->lod = emt.lod;
  }
  if (Tensor* dt = r.out("Transition@GRAD")) {
    float* o = dt->alloc<float>(trt.dims, -1);
    for (size_t i = 0; i < dtr.size(); ++i) o[i] = (float)dtr[i];
  }
}

void k_crf_decoding(const OpRun& r) {
  Tensor& emt = r.in("Emission");
  Tensor& trt = r.in("Transition");
  Tensor* lab = r.in_opt("Label");
  const int64_t T = emt.dims[0], D = emt.dims[1];
  const float *em = f32(emt), *tr = f32(trt);
  const auto off = seq_off(emt);
  const int64_t N = (int64_t)off.size() - 1;
  Tensor* out = r.out("ViterbiPath");
  int64_t* path = out->alloc<int64_t>({T, 1}, -1);
  std::fill_n(path, T, (int64_t)0);
  parallel_for(N, 1, [&](int64_t a, int64_t b) {
    std::vector<float> score, nxt;
    std::vector<int32_t> back;
    for (int64_t s = a; s < b; ++s) {
      const int64_t s0 = (int64_t)off[(size_t)s], L = (int64_t)off[(size_t)s + 1] - s0;
      if (L > 0) crf::viterbi(em + s0 * D, tr, L, D, score, nxt, back, path + s0);
    }
  });
  if (lab) {
    const std::vector<int64_t> y = labels_of(*lab);
    for (int64_t t = 0; t < T; ++t) path[t] = path[t] == y[(size_t)t] ? 1 : 0;
  }
  out->lod = emt.lod;
}

}  // namespace

namespace crf {
void viterbi(const float* em, const float* tr, int64_t L, int64_t D, std::vector<float>& score,
             std::vector<float>& nxt, std::vector<int32_t>& back, int64_t* path) {
  const float *start = tr, *end = tr + D, *T = tr + 2 * D;
  score.resize((size_t)D);
  nxt.resize((size_t)D);
  back.assign((size_t)(L * D), 0);
  for (int64_t j = 0; j < D; ++j) score[(size_t)j] = start[j] + em[j];
  for (int64_t t = 1; t < L; ++t) {
    for (int64_t j = 0; j < D; ++j) {
      float best = score[0] + T[j];
      int32_t arg = 0;
      for (int64_t i = 1; i < D; ++i) {
        const float c = score[(size_t)i] + T[i * D + j];
        if (c > best) {
          best = c;
          arg = (int32_t)i;
        }
      }
      nxt[(size_t)j] = best + em[t * D + j];
      back[(size_t)(t * D + j)] = arg;
    }
    score.swap(nxt);
  }
  int64_t best = 0;
  for (int64_t j = 1; j < D; ++j)
    if (score[(size_t)j] + end[j] > score[(size_t)best] + end[best]) best = j;
  for (int64_t t = L - 1; t >= 0; --t) {
    path[t] = best;
    if (t > 0) best = back[(size_t)(t * D + best)];
  }
}
}  // namespace crf

PA_HOST_KERNEL(linear_chain_crf, k_linear_chain_crf);
PA_HOST_KERNEL(linear_chain_crf_grad, k_linear_chain_crf_grad);
PA_HOST_KERNEL(crf_decoding, k_crf_decoding);

void link_struct_kernels() {}

}  // namespace pa
