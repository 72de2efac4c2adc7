// Host kernels of the LoD recurrent operators: lstm / lstm_grad, gru / gru_grad.
//
// Semantics (reference operators/lstm_op.h:40-160, math/detail/lstm_kernel.h:36-40,
// operators/gru_op.h:40-180, math/detail/gru_kernel.h:62; the Python kernels of
// operators/rnn_ops.py compute the same functions):
//   * LSTM gates {candidate, input, forget, output} in the 4D axis of Input / Weight;
//     with use_peepholes the bias is [1, 7D] = {b_c, b_i, b_f, b_o, W_ic, W_fc, W_oc},
//     i / f see c_{t-1}, o sees c_t.  BatchGate holds the ACTIVATED gates per LoD
//     row, BatchCellPreAct the cell state, which is what lstm_grad consumes.
//   * GRU gates {update, reset, candidate}; Weight [D, 3D] = {W_u | W_r | W_c};
//     h = h_prev - u h_prev + u c.  BatchGate holds the activated {u, r, c},
//     BatchResetHiddenPrev r * h_prev.
//   * is_reverse processes every sequence from its end; H0 / C0 are per sequence.
//
// Execution follows the reference's LoDTensor2Batch (math/sequence2batch.cc): the
// sequences are ordered longest first, so time step t covers a prefix of them; each
// step is one GEMM over the live sequences' previous hidden rows plus an elementwise
// cell pass.  The backward walks the steps in reverse and accumulates dW with one
// GEMM per step.  fp32.
#include <math.h>
#include <string.h>

#include <algorithm>
#include <numeric>

#include "framework.h"
#include "rnn_common.h"

namespace pa {
namespace rnn {

int act_id(const OpDesc& op, const char* name, int def) {
  auto it = op.attrs.find(name);
  if (it == op.attrs.end()) return def;
  const Attr& a = it->second;
  if (a.type == A_STRING) {
    const std::string& s = a.s;
    if (s == "identity" || s == "linear" || s.empty()) return ACT_IDENTITY;
    if (s == "sigmoid") return ACT_SIGMOID;
    if (s == "tanh") return ACT_TANH;
    if (s == "relu") return ACT_RELU;
    fail("%s: unsupported activation '%s'", op.type.c_str(), s.c_str());
  }
  PA_CHECK(a.i >= 0 && a.i <= 3, "%s: activation id %lld", op.type.c_str(), (long long)a.i);
  return (int)a.i;
}

SeqBatch make_batch(const std::vector<size_t>& off, bool reverse) {
  SeqBatch b;
  const int64_t N = (int64_t)off.size() - 1;
  std::vector<int64_t> len((size_t)N);
  for (int64_t i = 0; i < N; ++i) len[(size_t)i] = (int64_t)(off[(size_t)i + 1] - off[(size_t)i]);
  b.order.resize((size_t)N);
  std::iota(b.order.begin(), b.order.end(), 0);
  std::stable_sort(b.order.begin(), b.order.end(), [&](int64_t x, int64_t y) { return len[(size_t)x] > len[(size_t)y]; });
  const int64_t L = N ? len[(size_t)b.order[0]] : 0;
  b.step_begin.assign((size_t)L + 1, 0);
  for (int64_t t = 0; t < L; ++t) {
    b.step_begin[(size_t)t] = (int64_t)b.rows.size();
    for (int64_t k = 0; k < N && len[(size_t)b.order[(size_t)k]] > t; ++k) {
      const int64_t s = b.order[(size_t)k];
      const int64_t row = (int64_t)off[(size_t)s] + (reverse ? len[(size_t)s] - 1 - t : t);
      b.rows.push_back(row);
      b.seq.push_back(s);
      b.prev.push_back(t == 0 ? -1 : (int64_t)off[(size_t)s] + (reverse ? len[(size_t)s] - t : t - 1));
    }
  }
  b.step_begin[(size_t)L] = (int64_t)b.rows.size();
  return b;
}

}  // namespace rnn

namespace {

using rnn::act;
using rnn::dact;

float* f32(Tensor& t) {
  if (t.dtype != DT::FP32) throw Decline{};
  return t.data<float>();
}

const std::vector<size_t>& seq_offsets(const Tensor& x, const char* op) {
  PA_CHECK(!x.lod.empty(), "%s: Input has no LoD", op);
  return x.lod.back();
}

// ---------------------------------------------------------------- lstm (lstm_op.h LSTMKernel)
void k_lstm(const OpRun& r) {
  Tensor& x = r.in("Input");
  Tensor& W = r.in("Weight");
  Tensor& Bt = r.in("Bias");
  Tensor* H0 = r.in_opt("H0");
  Tensor* C0 = r.in_opt("C0");
  const int64_t D = W.dims[0], T = x.dims[0];
  const bool peep = r.op.GetBool("use_peepholes", true), rev = r.op.GetBool("is_reverse", false);
  const int ag = rnn::act_id(r.op, "gate_activation", rnn::ACT_SIGMOID);
  const int ac = rnn::act_id(r.op, "cell_activation", rnn::ACT_TANH);
  const int an = rnn::act_id(r.op, "candidate_activation", rnn::ACT_TANH);
  PA_CHECK(x.dims.size() == 2 && x.dims[1] == 4 * D && W.dims[1] == 4 * D, "lstm: Input [T, 4D], Weight [D, 4D]");
  PA_CHECK(Bt.numel() == (peep ? 7 : 4) * D, "lstm: Bias must hold %lld values", (long long)((peep ? 7 : 4) * D));
  const auto& off = seq_offsets(x, "lstm");
  const rnn::SeqBatch sb = rnn::make_batch(off, rev);
  const int64_t N = (int64_t)off.size() - 1;
  const float *xp = f32(x), *wp = f32(W), *bp = f32(Bt);
  float* hp = r.out("Hidden")->alloc<float>({T, D}, -1);
  float* cp = r.out("Cell")->alloc<float>({T, D}, -1);
  float* gp = r.out("BatchGate") ? r.out("BatchGate")->alloc<float>({T, 4 * D}, -1) : nullptr;
  float* pp = r.out("BatchCellPreAct") ? r.out("BatchCellPreAct")->alloc<float>({T, D}, -1) : nullptr;
  std::vector<float> gates(gp ? 0 : (size_t)(T * 4 * D));
  if (!gp) gp = gates.data();
  const float* h0 = H0 ? f32(*H0) : nullptr;
  const float* c0 = C0 ? f32(*C0) : nullptr;
  std::vector<float> hprev, G;
  for (size_t t = 0; t + 1 < sb.step_begin.size(); ++t) {
    const int64_t a = sb.step_begin[t], nb = sb.step_begin[t + 1] - a;
    // G = x + b + h_prev W  (h_prev of each live sequence gathered into [nb, D])
    G.assign((size_t)(nb * 4 * D), 0.f);
    hprev.assign((size_t)(nb * D), 0.f);
    bool any_h = false;
    for (int64_t k = 0; k < nb; ++k) {
      const int64_t row = sb.rows[(size_t)(a + k)], pr = sb.prev[(size_t)(a + k)], s = sb.seq[(size_t)(a + k)];
      for (int64_t j = 0; j < 4 * D; ++j) G[(size_t)(k * 4 * D + j)] = xp[row * 4 * D + j] + bp[j];
      const float* src = pr >= 0 ? hp + pr * D : (h0 ? h0 + s * D : nullptr);
      if (src) {
        memcpy(&hprev[(size_t)(k * D)], src, sizeof(float) * D);
        any_h = true;
      }
    }
    if (any_h) sgemm(false, false, nb, 4 * D, D, 1.f, hprev.data(), D, wp, 4 * D, 1.f, G.data(), 4 * D);
    parallel_for(nb, 8, [&](int64_t k0, int64_t k1) {
      for (int64_t k = k0; k < k1; ++k) {
        const int64_t row = sb.rows[(size_t)(a + k)], pr = sb.prev[(size_t)(a + k)], s = sb.seq[(size_t)(a + k)];
        const float* cprev = pr >= 0 ? cp + pr * D : (c0 ? c0 + s * D : nullptr);
        const float* g = &G[(size_t)(k * 4 * D)];
        float* go = gp + row * 4 * D;
        for (int64_t d = 0; d < D; ++d) {
          const float c_1 = cprev ? cprev[d] : 0.f;
          float gi = g[D + d], gf = g[2 * D + d], gop = g[3 * D + d];
          if (peep) {
            gi += c_1 * bp[4 * D + d];
            gf += c_1 * bp[5 * D + d];
          }
          const float cand = act(an, g[d]), i = act(ag, gi), f = act(ag, gf);
          const float c = cand * i + c_1 * f;
          if (peep) gop += c * bp[6 * D + d];
          const float o = act(ag, gop);
          cp[row * D + d] = c;
          hp[row * D + d] = o * act(ac, c);
          go[d] = cand;
          go[D + d] = i;
          go[2 * D + d] = f;
          go[3 * D + d] = o;
          if (pp) pp[row * D + d] = c;
        }
      }
    });
  }
  r.out("Hidden")->lod = x.lod;
  r.out("Cell")->lod = x.lod;
  (void)N;
}

// lstm_op.h LSTMGradKernel: backward through time from the kept activated gates and
// cell states (no recomputation of the forward GEMMs).
void k_lstm_grad(const OpRun& r) {
  Tensor& x = r.in("Input");
  Tensor& W = r.in("Weight");
  Tensor& Bt = r.in("Bias");
  Tensor* H0 = r.in_opt("H0");
  Tensor* C0 = r.in_opt("C0");
  Tensor& Hd = r.in("Hidden");
  Tensor& Cl = r.in("Cell");
  Tensor& BG = r.in("BatchGate");
  Tensor* dH = r.in_opt("Hidden@GRAD");
  Tensor* dC = r.in_opt("Cell@GRAD");
  const int64_t D = W.dims[0], T = x.dims[0];
  const bool peep = r.op.GetBool("use_peepholes", true), rev = r.op.GetBool("is_reverse", false);
  const int ag = rnn::act_id(r.op, "gate_activation", rnn::ACT_SIGMOID);
  const int ac = rnn::act_id(r.op, "cell_activation", rnn::ACT_TANH);
  const int an = rnn::act_id(r.op, "candidate_activation", rnn::ACT_TANH);
  const auto& off = seq_offsets(x, "lstm_grad");
  const rnn::SeqBatch sb = rnn::make_batch(off, rev);
  const int64_t N = (int64_t)off.size() - 1;
  const float *wp = f32(W), *bp = f32(Bt), *hp = f32(Hd), *cp = f32(Cl), *gp = f32(BG);
  const float* dhp = dH ? f32(*dH) : nullptr;
  const float* dcp = dC ? f32(*dC) : nullptr;
  const float* h0 = H0 ? f32(*H0) : nullptr;
  const float* c0 = C0 ? f32(*C0) : nullptr;
  std::vector<float> dG_all((size_t)(T * 4 * D), 0.f);
  std::vector<float> dh_next((size_t)(N * D), 0.f), dc_next((size_t)(N * D), 0.f);
  std::vector<float> dW((size_t)(D * 4 * D), 0.f), dpeep(peep ? (size_t)(3 * D) : 0, 0.f);
  std::vector<float> hprev, dG, dhp_b;
  for (int64_t t = (int64_t)sb.step_begin.size() - 2; t >= 0; --t) {
    const int64_t a = sb.step_begin[(size_t)t], nb = sb.step_begin[(size_t)t + 1] - a;
    dG.assign((size_t)(nb * 4 * D), 0.f);
    for (int64_t k = 0; k < nb; ++k) {
      const int64_t row = sb.rows[(size_t)(a + k)], pr = sb.prev[(size_t)(a + k)], s = sb.seq[(size_t)(a + k)];
      const float* cprev = pr >= 0 ? cp + pr * D : (c0 ? c0 + s * D : nullptr);
      const float* g = gp + row * 4 * D;
      float* dg = &dG[(size_t)(k * 4 * D)];
      for (int64_t d = 0; d < D; ++d) {
        const float cand = g[d], i = g[D + d], f = g[2 * D + d], o = g[3 * D + d];
        const float c = cp[row * D + d], c_1 = cprev ? cprev[d] : 0.f;
        const float dh = (dhp ? dhp[row * D + d] : 0.f) + dh_next[(size_t)(s * D + d)];
        float dc = (dcp ? dcp[row * D + d] : 0.f) + dc_next[(size_t)(s * D + d)];
        const float acv = act(ac, c);
        const float dgo = dh * acv * dact(ag, o);
        dc += dh * o * dact(ac, acv);
        if (peep) dc += dgo * bp[6 * D + d];
        const float dgc = dc * i * dact(an, cand);
        const float dgi = dc * cand * dact(ag, i);
        const float dgf = dc * c_1 * dact(ag, f);
        float dcp_ = dc * f;
        if (peep) {
          dcp_ += dgi * bp[4 * D + d] + dgf * bp[5 * D + d];
          dpeep[(size_t)d] += dgi * c_1;
          dpeep[(size_t)(D + d)] += dgf * c_1;
          dpeep[(size_t)(2 * D + d)] += dgo * c;
        }
        dc_next[(size_t)(s * D + d)] = dcp_;
        dg[d] = dgc;
        dg[D + d] = dgi;
        dg[2 * D + d] = dgf;
        dg[3 * D + d] = dgo;
      }
      memcpy(&dG_all[(size_t)(row * 4 * D)], dg, sizeof(float) * 4 * D);
    }
    // dh_prev = dG W^T ; dW += h_prev^T dG
    dhp_b.assign((size_t)(nb * D), 0.f);
    sgemm(false, true, nb, D, 4 * D, 1.f, dG.data(), 4 * D, wp, 4 * D, 0.f, dhp_b.data(), D);
    hprev.assign((size_t)(nb * D), 0.f);
    bool any_h = false;
    for (int64_t k = 0; k < nb; ++k) {
      const int64_t pr = sb.prev[(size_t)(a + k)], s = sb.seq[(size_t)(a + k)];
      memcpy(&dh_next[(size_t)(s * D)], &dhp_b[(size_t)(k * D)], sizeof(float) * D);
      const float* src = pr >= 0 ? hp + pr * D : (h0 ? h0 + s * D : nullptr);
      if (src) {
        memcpy(&hprev[(size_t)(k * D)], src, sizeof(float) * D);
        any_h = true;
      }
    }
    if (any_h) sgemm(true, false, D, 4 * D, nb, 1.f, hprev.data(), D, dG.data(), 4 * D, 1.f, dW.data(), 4 * D);
  }
  if (Tensor* dx = r.out("Input@GRAD")) {
    memcpy(dx->alloc<float>({T, 4 * D}, -1), dG_all.data(), dG_all.size() * sizeof(float));
    dx->lod = x.lod;
  }
  if (Tensor* dw = r.out("Weight@GRAD")) memcpy(dw->alloc<float>(W.dims, -1), dW.data(), dW.size() * sizeof(float));
  if (Tensor* db = r.out("Bias@GRAD")) {
    float* o = db->alloc<float>(Bt.dims, -1);
    std::fill_n(o, Bt.numel(), 0.f);
    for (int64_t row = 0; row < T; ++row)
      for (int64_t j = 0; j < 4 * D; ++j) o[j] += dG_all[(size_t)(row * 4 * D + j)];
    if (peep) memcpy(o + 4 * D, dpeep.data(), sizeof(float) * 3 * D);
  }
  // the gradients reaching the initial states are what step 0 passed back
  if (Tensor* dh0 = r.out("H0@GRAD"))
    if (H0) memcpy(dh0->alloc<float>(H0->dims, -1), dh_next.data(), sizeof(float) * N * D);
  if (Tensor* dc0 = r.out("C0@GRAD"))
    if (C0) memcpy(dc0->alloc<float>(C0->dims, -1), dc_next.data(), sizeof(float) * N * D);
}

// ---------------------------------------------------------------- gru (gru_op.h GRUKernel)
void k_gru(const OpRun& r) {
  Tensor& x = r.in("Input");
  Tensor& W = r.in("Weight");
  Tensor* Bt = r.in_opt("Bias");
  Tensor* H0 = r.in_opt("H0");
  const int64_t D = W.dims[0], T = x.dims[0];
  const bool rev = r.op.GetBool("is_reverse", false);
  const int an = rnn::act_id(r.op, "activation", rnn::ACT_TANH);
  const int ag = rnn::act_id(r.op, "gate_activation", rnn::ACT_SIGMOID);
  PA_CHECK(x.dims.size() == 2 && x.dims[1] == 3 * D && W.dims[1] == 3 * D, "gru: Input [T, 3D], Weight [D, 3D]");
  const auto& off = seq_offsets(x, "gru");
  const rnn::SeqBatch sb = rnn::make_batch(off, rev);
  const float *xp = f32(x), *wp = f32(W), *bp = Bt ? f32(*Bt) : nullptr, *h0 = H0 ? f32(*H0) : nullptr;
  float* hp = r.out("Hidden")->alloc<float>({T, D}, -1);
  std::vector<float> gbuf, rbuf;
  float* gp = r.out("BatchGate") ? r.out("BatchGate")->alloc<float>({T, 3 * D}, -1) : (gbuf.resize((size_t)(T * 3 * D)), gbuf.data());
  float* rp = r.out("BatchResetHiddenPrev") ? r.out("BatchResetHiddenPrev")->alloc<float>({T, D}, -1)
                                            : (rbuf.resize((size_t)(T * D)), rbuf.data());
  std::vector<float> hprev, G, RH, C;
  for (size_t t = 0; t + 1 < sb.step_begin.size(); ++t) {
    const int64_t a = sb.step_begin[t], nb = sb.step_begin[t + 1] - a;
    G.assign((size_t)(nb * 3 * D), 0.f);
    hprev.assign((size_t)(nb * D), 0.f);
    for (int64_t k = 0; k < nb; ++k) {
      const int64_t row = sb.rows[(size_t)(a + k)], pr = sb.prev[(size_t)(a + k)], s = sb.seq[(size_t)(a + k)];
      for (int64_t j = 0; j < 3 * D; ++j) G[(size_t)(k * 3 * D + j)] = xp[row * 3 * D + j] + (bp ? bp[j] : 0.f);
      const float* src = pr >= 0 ? hp + pr * D : (h0 ? h0 + s * D : nullptr);
      if (src) memcpy(&hprev[(size_t)(k * D)], src, sizeof(float) * D);
    }
    // [u | r] pre-activations += h_prev W_{u,r}
    sgemm(false, false, nb, 2 * D, D, 1.f, hprev.data(), D, wp, 3 * D, 1.f, G.data(), 3 * D);
    RH.assign((size_t)(nb * D), 0.f);
    for (int64_t k = 0; k < nb; ++k)
      for (int64_t d = 0; d < D; ++d) {
        float* g = &G[(size_t)(k * 3 * D)];
        g[d] = act(ag, g[d]);
        g[D + d] = act(ag, g[D + d]);
        RH[(size_t)(k * D + d)] = g[D + d] * hprev[(size_t)(k * D + d)];
      }
    // candidate pre-activation += (r * h_prev) W_c
    sgemm(false, false, nb, D, D, 1.f, RH.data(), D, wp + 2 * D, 3 * D, 1.f, G.data() + 2 * D, 3 * D);
    for (int64_t k = 0; k < nb; ++k) {
      const int64_t row = sb.rows[(size_t)(a + k)];
      float* g = &G[(size_t)(k * 3 * D)];
      for (int64_t d = 0; d < D; ++d) {
        const float c = act(an, g[2 * D + d]), u = g[d], hpv = hprev[(size_t)(k * D + d)];
        hp[row * D + d] = hpv - u * hpv + u * c;
        gp[row * 3 * D + d] = u;
        gp[row * 3 * D + D + d] = g[D + d];
        gp[row * 3 * D + 2 * D + d] = c;
        rp[row * D + d] = RH[(size_t)(k * D + d)];
      }
    }
  }
  r.out("Hidden")->lod = x.lod;
  if (Tensor* bh = r.out("BatchHidden")) {
    memcpy(bh->alloc<float>({T, D}, -1), hp, sizeof(float) * T * D);
  }
}

// gru_op.h GRUGradKernel from the kept activated gates
void k_gru_grad(const OpRun& r) {
  Tensor& x = r.in("Input");
  Tensor& W = r.in("Weight");
  Tensor* Bt = r.in_opt("Bias");
  Tensor* H0 = r.in_opt("H0");
  Tensor& Hd = r.in("Hidden");
  Tensor& BG = r.in("BatchGate");
  Tensor* dH = r.in_opt("Hidden@GRAD");
  const int64_t D = W.dims[0], T = x.dims[0];
  const bool rev = r.op.GetBool("is_reverse", false);
  const int an = rnn::act_id(r.op, "activation", rnn::ACT_TANH);
  const int ag = rnn::act_id(r.op, "gate_activation", rnn::ACT_SIGMOID);
  const auto& off = seq_offsets(x, "gru_grad");
  const rnn::SeqBatch sb = rnn::make_batch(off, rev);
  const int64_t N = (int64_t)off.size() - 1;
  const float *wp = f32(W), *hp = f32(Hd), *gp = f32(BG), *h0 = H0 ? f32(*H0) : nullptr;
  const float* dhp = dH ? f32(*dH) : nullptr;
  std::vector<float> dG_all((size_t)(T * 3 * D), 0.f), dh_next((size_t)(N * D), 0.f), dW((size_t)(D * 3 * D), 0.f);
  std::vector<float> hprev, dG, drh, dhprev, RH;
  for (int64_t t = (int64_t)sb.step_begin.size() - 2; t >= 0; --t) {
    const int64_t a = sb.step_begin[(size_t)t], nb = sb.step_begin[(size_t)t + 1] - a;
    hprev.assign((size_t)(nb * D), 0.f);
    dG.assign((size_t)(nb * 3 * D), 0.f);
    dhprev.assign((size_t)(nb * D), 0.f);
    RH.assign((size_t)(nb * D), 0.f);
    for (int64_t k = 0; k < nb; ++k) {
      const int64_t row = sb.rows[(size_t)(a + k)], pr = sb.prev[(size_t)(a + k)], s = sb.seq[(size_t)(a + k)];
      const float* src = pr >= 0 ? hp + pr * D : (h0 ? h0 + s * D : nullptr);
      if (src) memcpy(&hprev[(size_t)(k * D)], src, sizeof(float) * D);
      const float* g = gp + row * 3 * D;
      float* dg = &dG[(size_t)(k * 3 * D)];
      for (int64_t d = 0; d < D; ++d) {
        const float u = g[d], rr = g[D + d], c = g[2 * D + d], hpv = hprev[(size_t)(k * D + d)];
        const float dh = (dhp ? dhp[row * D + d] : 0.f) + dh_next[(size_t)(s * D + d)];
        dg[2 * D + d] = dh * u * dact(an, c);            // d candidate pre-activation
        dg[d] = dh * (c - hpv) * dact(ag, u);            // d update pre-activation
        dhprev[(size_t)(k * D + d)] = dh * (1.f - u);   // direct path
        RH[(size_t)(k * D + d)] = rr * hpv;
      }
    }
    // d(r h_prev) = dc W_c^T ; dW_c += (r h_prev)^T dc
    drh.assign((size_t)(nb * D), 0.f);
    sgemm(false, true, nb, D, D, 1.f, dG.data() + 2 * D, 3 * D, wp + 2 * D, 3 * D, 0.f, drh.data(), D);
    sgemm(true, false, D, D, nb, 1.f, RH.data(), D, dG.data() + 2 * D, 3 * D, 1.f, dW.data() + 2 * D, 3 * D);
    for (int64_t k = 0; k < nb; ++k) {
      const int64_t row = sb.rows[(size_t)(a + k)];
      const float* g = gp + row * 3 * D;
      for (int64_t d = 0; d < D; ++d) {
        const float rr = g[D + d], hpv = hprev[(size_t)(k * D + d)], dr = drh[(size_t)(k * D + d)];
        dG[(size_t)(k * 3 * D + D + d)] = dr * hpv * dact(ag, rr);  // d reset pre-activation
        dhprev[(size_t)(k * D + d)] += dr * rr;
      }
    }
    // dh_prev += d[u | r] W_{u,r}^T ; dW_{u,r} += h_prev^T d[u | r]
    sgemm(false, true, nb, D, 2 * D, 1.f, dG.data(), 3 * D, wp, 3 * D, 1.f, dhprev.data(), D);
    sgemm(true, false, D, 2 * D, nb, 1.f, hprev.data(), D, dG.data(), 3 * D, 1.f, dW.data(), 3 * D);
    for (int64_t k = 0; k < nb; ++k) {
      const int64_t row = sb.rows[(size_t)(a + k)], s = sb.seq[(size_t)(a + k)];
      memcpy(&dh_next[(size_t)(s * D)], &dhprev[(size_t)(k * D)], sizeof(float) * D);
      memcpy(&dG_all[(size_t)(row * 3 * D)], &dG[(size_t)(k * 3 * D)], sizeof(float) * 3 * D);
    }
  }
  if (Tensor* dx = r.out("Input@GRAD")) {
    memcpy(dx->alloc<float>({T, 3 * D}, -1), dG_all.data(), dG_all.size() * sizeof(float));
    dx->lod = x.lod;
  }
  if (Tensor* dw = r.out("Weight@GRAD")) memcpy(dw->alloc<float>(W.dims, -1), dW.data(), dW.size() * sizeof(float));
  if (Tensor* db = r.out("Bias@GRAD"))
    if (Bt) {
      float* o = db->alloc<float>(Bt->dims, -1);
      std::fill_n(o, Bt->numel(), 0.f);
      for (int64_t row = 0; row < T; ++row)
        for (int64_t j = 0; j < 3 * D; ++j) o[j] += dG_all[(size_t)(row * 3 * D + j)];
    }
  if (Tensor* dh0 = r.out("H0@GRAD"))
    if (H0) memcpy(dh0->alloc<float>(H0->dims, -1), dh_next.data(), sizeof(float) * N * D);
}

}  // namespace

PA_HOST_KERNEL(lstm, k_lstm);
PA_HOST_KERNEL(lstm_grad, k_lstm_grad);
PA_HOST_KERNEL(gru, k_gru);
PA_HOST_KERNEL(gru_grad, k_gru_grad);

void link_rnn_kernels() {}

}  // namespace pa
