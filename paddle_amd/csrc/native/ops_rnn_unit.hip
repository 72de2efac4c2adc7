// Single-step and projected recurrent operators of the native executor, host AND
// device from one source (any_place.h): gru_unit / gru_unit_grad, lstm_unit /
// lstm_unit_grad, lstmp / lstmp_grad.
//
// Semantics (reference operators/gru_unit_op.h:40-200, lstm_unit_op.h:38-160,
// lstmp_op.h:60-400; the Python kernels of operators/rnn_ops.py compute the same
// functions):
//   * gru_unit: Gate = {u, r, c} activated, u / r = act_gate(x_{u,r} + h W_{u,r}),
//     c = act(x_c + (r h) W_c), Hidden = h - u h + u c; activation ids are
//     {identity, sigmoid, tanh, relu}.
//   * lstm_unit: X = {i, f, o, g} pre-activations, c = sig(f + forget_bias) c_prev +
//     sig(i) tanh(g), h = sig(o) tanh(c).
//   * lstmp: the LoD LSTM of ops_rnn.cc whose recurrent state is the projection
//     r_t = proj_act(h_t ProjWeight) ([T, P], Weight is [P, 4D]); with H0 the initial
//     projection is proj_act(H0 ProjWeight) (OrderedP0).  BatchHidden holds r.
// The backward of lstmp walks the LoDTensor2Batch steps in reverse (one GEMM back
// through the projection and one through the recurrent weight per step) and forms
// dWeight, dProjWeight as single GEMMs over all rows at the end.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "any_place.h"
#include "rnn_common.h"

namespace pa {
namespace {

using rnn::act;
using rnn::dact;

// ---------------------------------------------------------------- gru_unit
struct GruGateUR {  // G[:, :2D] activated in place, RH = r * h
  float *G, *RH;
  const float* h;
  int64_t D;
  int ag;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t k = i / D, d = i % D;
    float* g = G + k * 3 * D;
    g[d] = act(ag, g[d]);
    g[D + d] = act(ag, g[D + d]);
    RH[i] = g[D + d] * h[i];
  }
};

struct GruOut {
  float *G, *H;
  const float* h;
  int64_t D;
  int an;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t k = i / D, d = i % D;
    float* g = G + k * 3 * D;
    const float c = act(an, g[2 * D + d]), u = g[d];
    g[2 * D + d] = c;
    H[i] = h[i] - u * h[i] + u * c;
  }
};

struct AddBias {  // out[k, j] = x[k, j] + b[j]
  float* out;
  const float *x, *b;
  int64_t W;
  __host__ __device__ void operator()(int64_t i) const { out[i] = x[i] + (b ? b[i % W] : 0.f); }
};

void k_gru_unit(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("Input");
  Tensor& hp = r.in("HiddenPrev");
  Tensor& W = r.in("Weight");
  Tensor* Bt = r.in_opt("Bias");
  const int64_t B = x.dims[0], D = W.dims[0];
  PA_CHECK(x.dims.size() == 2 && x.dims[1] == 3 * D && W.dims[1] == 3 * D && hp.numel() == B * D,
           "gru_unit: Input [B, 3D], HiddenPrev [B, D], Weight [D, 3D]");
  const int an = rnn::act_id(r.op, "activation", rnn::ACT_TANH), ag = rnn::act_id(r.op, "gate_activation", rnn::ACT_SIGMOID);
  const float *xp = any::f32(x, dev), *h = any::f32(hp, dev), *wp = any::f32(W, dev);
  const float* bp = Bt ? any::f32(*Bt, dev) : nullptr;
  const int place = dev ? r.ctx.device : -1;
  Tensor G, RH, H;
  float* g = G.alloc<float>({B, 3 * D}, place);
  float* rh = RH.alloc<float>({B, D}, place);
  float* ho = H.alloc<float>({B, D}, place);
  any::run(r, dev, B * 3 * D, AddBias{g, xp, bp, 3 * D});
  any::gemm(r, dev, false, false, B, 2 * D, D, 1.f, h, D, wp, 3 * D, 1.f, g, 3 * D);
  any::run(r, dev, B * D, GruGateUR{g, rh, h, D, ag});
  any::gemm(r, dev, false, false, B, D, D, 1.f, rh, D, wp + 2 * D, 3 * D, 1.f, g + 2 * D, 3 * D);
  any::run(r, dev, B * D, GruOut{g, ho, h, D, an});
  if (Tensor* o = r.out("Gate")) *o = G;
  if (Tensor* o = r.out("ResetHiddenPrev")) *o = RH;
  *r.out("Hidden") = H;
}

struct GruBwd1 {  // dG_u, dG_c and the direct dh_prev path
  const float *G, *dH, *h;
  float *dG, *dhp;
  int64_t D;
  int an, ag;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t k = i / D, d = i % D;
    const float* g = G + k * 3 * D;
    const float u = g[d], c = g[2 * D + d], dh = dH ? dH[i] : 0.f;
    dG[k * 3 * D + 2 * D + d] = dh * u * dact(an, c);
    dG[k * 3 * D + d] = dh * (c - h[i]) * dact(ag, u);
    dhp[i] = dh * (1.f - u);
  }
};

struct GruBwd2 {  // dG_r from d(r h); dh_prev += d(r h) r
  const float *G, *drh, *h;
  float *dG, *dhp;
  int64_t D;
  int ag;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t k = i / D, d = i % D;
    const float rr = G[k * 3 * D + D + d];
    dG[k * 3 * D + D + d] = drh[i] * h[i] * dact(ag, rr);
    dhp[i] += drh[i] * rr;
  }
};

void k_gru_unit_grad(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("Input");
  Tensor& hp = r.in("HiddenPrev");
  Tensor& W = r.in("Weight");
  Tensor* Bt = r.in_opt("Bias");
  Tensor& Gt = r.in("Gate");
  Tensor& RHt = r.in("ResetHiddenPrev");
  Tensor* dHt = r.in_opt("Hidden@GRAD");
  const int64_t B = x.dims[0], D = W.dims[0];
  const int an = rnn::act_id(r.op, "activation", rnn::ACT_TANH), ag = rnn::act_id(r.op, "gate_activation", rnn::ACT_SIGMOID);
  const float *h = any::f32(hp, dev), *wp = any::f32(W, dev), *g = any::f32(Gt, dev), *rh = any::f32(RHt, dev);
  const float* dh = dHt ? any::f32(*dHt, dev) : nullptr;
  const int place = dev ? r.ctx.device : -1;
  Tensor dG, dHP, dRH;
  float* dg = dG.alloc<float>({B, 3 * D}, place);
  float* dhp = dHP.alloc<float>(hp.dims, place);
  float* drh = dRH.alloc<float>({B, D}, place);
  any::run(r, dev, B * D, GruBwd1{g, dh, h, dg, dhp, D, an, ag});
  any::gemm(r, dev, false, true, B, D, D, 1.f, dg + 2 * D, 3 * D, wp + 2 * D, 3 * D, 0.f, drh, D);
  any::run(r, dev, B * D, GruBwd2{g, drh, h, dg, dhp, D, ag});
  any::gemm(r, dev, false, true, B, D, 2 * D, 1.f, dg, 3 * D, wp, 3 * D, 1.f, dhp, D);
  if (Tensor* dw = r.out("Weight@GRAD")) {
    float* p = dw->alloc<float>(W.dims, place);
    any::gemm(r, dev, true, false, D, 2 * D, B, 1.f, h, D, dg, 3 * D, 0.f, p, 3 * D);
    any::gemm(r, dev, true, false, D, D, B, 1.f, rh, D, dg + 2 * D, 3 * D, 0.f, p + 2 * D, 3 * D);
  }
  if (Tensor* db = r.out("Bias@GRAD"))
    if (Bt) any::run(r, dev, 3 * D, any::ColSum{dg, db->alloc<float>(Bt->dims, place), B, 3 * D, 0}, 64);
  if (Tensor* dx = r.out("Input@GRAD")) {
    *dx = dG;
    dx->dims = x.dims;
  }
  if (Tensor* o = r.out("HiddenPrev@GRAD")) *o = dHP;
}

// ---------------------------------------------------------------- lstm_unit
__host__ __device__ inline float sigm(float v) { return 1.f / (1.f + expf(-v)); }

struct LstmUnitFwd {
  const float *x, *cp;
  float *c, *h;
  int64_t D;
  float fb;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t k = i / D, d = i % D;
    const float* xr = x + k * 4 * D;
    const float ii = sigm(xr[d]), f = sigm(xr[D + d] + fb), o = sigm(xr[2 * D + d]), g = tanhf(xr[3 * D + d]);
    const float cv = f * cp[i] + ii * g;
    c[i] = cv;
    h[i] = o * tanhf(cv);
  }
};

void k_lstm_unit(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("X");
  Tensor& cp = r.in("C_prev");
  const int64_t B = cp.dims[0], D = cp.dims[1];
  PA_CHECK(x.numel() == B * 4 * D, "lstm_unit: X must be [B, 4D] for C_prev [B, D]");
  const int place = dev ? r.ctx.device : -1;
  Tensor C, H;
  float* c = C.alloc<float>({B, D}, place);
  float* h = H.alloc<float>({B, D}, place);
  any::run(r, dev, B * D, LstmUnitFwd{any::f32(x, dev), any::f32(cp, dev), c, h, D, r.op.GetFloat("forget_bias", 0.f)});
  *r.out("C") = C;
  *r.out("H") = H;
}

struct LstmUnitBwd {
  const float *x, *cp, *c, *dC, *dH;
  float *dx, *dcp;
  int64_t D;
  float fb;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t k = i / D, d = i % D;
    const float* xr = x + k * 4 * D;
    const float ii = sigm(xr[d]), f = sigm(xr[D + d] + fb), o = sigm(xr[2 * D + d]), g = tanhf(xr[3 * D + d]);
    const float tc = tanhf(c[i]);
    const float dh = dH ? dH[i] : 0.f;
    const float dc = (dC ? dC[i] : 0.f) + dh * o * (1.f - tc * tc);
    float* dr = dx + k * 4 * D;
    dr[d] = dc * g * ii * (1.f - ii);
    dr[D + d] = dc * cp[i] * f * (1.f - f);
    dr[2 * D + d] = dh * tc * o * (1.f - o);
    dr[3 * D + d] = dc * ii * (1.f - g * g);
    if (dcp) dcp[i] = dc * f;
  }
};

void k_lstm_unit_grad(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("X");
  Tensor& cp = r.in("C_prev");
  Tensor& C = r.in("C");
  Tensor* dC = r.in_opt("C@GRAD");
  Tensor* dH = r.in_opt("H@GRAD");
  const int64_t B = cp.dims[0], D = cp.dims[1];
  const int place = dev ? r.ctx.device : -1;
  Tensor dX, dCP;
  float* dx = dX.alloc<float>(x.dims, place);
  Tensor* dcp_out = r.out("C_prev@GRAD");
  float* dcp = dcp_out ? dCP.alloc<float>(cp.dims, place) : nullptr;
  any::run(r, dev, B * D,
           LstmUnitBwd{any::f32(x, dev), any::f32(cp, dev), any::f32(C, dev), dC ? any::f32(*dC, dev) : nullptr,
                       dH ? any::f32(*dH, dev) : nullptr, dx, dcp, D, r.op.GetFloat("forget_bias", 0.f)});
  if (Tensor* o = r.out("X@GRAD")) *o = dX;
  if (dcp_out) *dcp_out = dCP;
}

// ---------------------------------------------------------------- lstmp
struct Sched {
  const int *rows, *seq, *prev;
};

Sched sched(const OpRun& r, bool dev, const rnn::SeqBatch& sb, std::vector<int>* keep) {
  const size_t n = sb.rows.size();
  keep->resize(3 * n);
  for (size_t i = 0; i < n; ++i) {
    (*keep)[i] = (int)sb.rows[i];
    (*keep)[n + i] = (int)sb.seq[i];
    (*keep)[2 * n + i] = (int)sb.prev[i];
  }
  const int* p = any::ints(r, dev, "@lstmp_sched@", *keep);
  return Sched{p, p + n, p + 2 * n};
}

struct GatherX {
  const float *x, *b;
  float* G;
  Sched sc;
  int64_t a, W;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t k = i / W, j = i % W;
    G[i] = x[(int64_t)sc.rows[a + k] * W + j] + b[j];
  }
};

// out[k] = R[prev[a+k]] | r0[seq[a+k]] | 0   (rows of width P)
struct GatherPrev {
  const float *R, *r0;
  float* out;
  Sched sc;
  int64_t a, P;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t k = i / P, j = i % P;
    const int pr = sc.prev[a + k];
    out[i] = pr >= 0 ? R[(int64_t)pr * P + j] : (r0 ? r0[(int64_t)sc.seq[a + k] * P + j] : 0.f);
  }
};

struct LstmpCell {
  const float *G, *b, *c0;
  float *C, *BG, *hb;
  Sched sc;
  int64_t a, D;
  int ag, ac, an, peep;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t k = i / D, d = i % D;
    const int row = sc.rows[a + k], pr = sc.prev[a + k];
    const float c_1 = pr >= 0 ? C[(int64_t)pr * D + d] : (c0 ? c0[(int64_t)sc.seq[a + k] * D + d] : 0.f);
    const float* g = G + k * 4 * D;
    float gi = g[D + d], gf = g[2 * D + d], go = g[3 * D + d];
    if (peep) {
      gi += c_1 * b[4 * D + d];
      gf += c_1 * b[5 * D + d];
    }
    const float cand = act(an, g[d]), ii = act(ag, gi), f = act(ag, gf);
    const float c = cand * ii + c_1 * f;
    if (peep) go += c * b[6 * D + d];
    const float o = act(ag, go);
    C[(int64_t)row * D + d] = c;
    hb[i] = o * act(ac, c);
    float* bg = BG + (int64_t)row * 4 * D;
    bg[d] = cand;
    bg[D + d] = ii;
    bg[2 * D + d] = f;
    bg[3 * D + d] = o;
  }
};

struct ProjAct {  // R[rows[a+k]] = pact(tmp[k])   (scatter == false: in place on tmp)
  const float* tmp;
  float* R;
  const int* rows;
  int64_t a, P;
  int pact;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t k = i / P, j = i % P;
    const float v = act(pact, tmp[i]);
    if (rows) R[(int64_t)rows[a + k] * P + j] = v;
    else R[i] = v;
  }
};

struct Lstmp {
  int64_t D, P, T, N;
  bool peep, rev;
  int ag, ac, an, pact;
};

Lstmp lstmp_dims(const OpRun& r, const Tensor& x, const Tensor& W, const Tensor& PW, const Tensor& Bt) {
  Lstmp L;
  L.D = PW.dims[0];
  L.P = PW.dims[1];
  L.T = x.dims[0];
  L.peep = r.op.GetBool("use_peepholes", true);
  L.rev = r.op.GetBool("is_reverse", false);
  L.ag = rnn::act_id(r.op, "gate_activation", rnn::ACT_SIGMOID);
  L.ac = rnn::act_id(r.op, "cell_activation", rnn::ACT_TANH);
  L.an = rnn::act_id(r.op, "candidate_activation", rnn::ACT_TANH);
  L.pact = rnn::act_id(r.op, "proj_activation", rnn::ACT_TANH);
  PA_CHECK(!x.lod.empty(), "lstmp: Input has no LoD");
  PA_CHECK(x.dims.size() == 2 && x.dims[1] == 4 * L.D && W.dims[0] == L.P && W.dims[1] == 4 * L.D,
           "lstmp: Input [T, 4D], Weight [P, 4D], ProjWeight [D, P]");
  PA_CHECK(Bt.numel() == (L.peep ? 7 : 4) * L.D, "lstmp: Bias must hold %lld values",
           (long long)((L.peep ? 7 : 4) * L.D));
  L.N = (int64_t)x.lod.back().size() - 1;
  return L;
}

void k_lstmp(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("Input");
  Tensor& W = r.in("Weight");
  Tensor& PW = r.in("ProjWeight");
  Tensor& Bt = r.in("Bias");
  Tensor* H0 = r.in_opt("H0");
  Tensor* C0 = r.in_opt("C0");
  const Lstmp L = lstmp_dims(r, x, W, PW, Bt);
  const int64_t D = L.D, P = L.P, T = L.T, N = L.N;
  const float *xp = any::f32(x, dev), *wp = any::f32(W, dev), *pwp = any::f32(PW, dev), *bp = any::f32(Bt, dev);
  const float* c0 = C0 ? any::f32(*C0, dev) : nullptr;
  const int place = dev ? r.ctx.device : -1;
  Tensor R, C, BG, R0;
  float* rp = R.alloc<float>({T, P}, place);
  float* cp = C.alloc<float>({T, D}, place);
  float* bg = BG.alloc<float>({T, 4 * D}, place);
  float* r0 = nullptr;
  if (H0) {  // OrderedP0 = pact(H0 ProjWeight)
    r0 = R0.alloc<float>({N, P}, place);
    any::gemm(r, dev, false, false, N, P, D, 1.f, any::f32(*H0, dev), D, pwp, P, 0.f, r0, P);
    any::run(r, dev, N * P, ProjAct{r0, r0, nullptr, 0, P, L.pact});
  }
  const rnn::SeqBatch sb = rnn::make_batch(x.lod.back(), L.rev);
  std::vector<int> keep;
  const Sched sc = sched(r, dev, sb, &keep);
  std::vector<float> hG, hRB, hHB, hTP;
  float* G = any::scratch(r, dev, "@lstmp_G@", N * 4 * D, &hG);
  float* rb = any::scratch(r, dev, "@lstmp_rb@", N * P, &hRB);
  float* hb = any::scratch(r, dev, "@lstmp_hb@", N * D, &hHB);
  float* tp = any::scratch(r, dev, "@lstmp_tp@", N * P, &hTP);
  for (size_t t = 0; t + 1 < sb.step_begin.size(); ++t) {
    const int64_t a = sb.step_begin[t], nb = sb.step_begin[t + 1] - a;
    any::run(r, dev, nb * 4 * D, GatherX{xp, bp, G, sc, a, 4 * D});
    if (t > 0 || r0) {
      any::run(r, dev, nb * P, GatherPrev{rp, r0, rb, sc, a, P});
      any::gemm(r, dev, false, false, nb, 4 * D, P, 1.f, rb, P, wp, 4 * D, 1.f, G, 4 * D);
    }
    any::run(r, dev, nb * D, LstmpCell{G, bp, c0, cp, bg, hb, sc, a, D, L.ag, L.ac, L.an, L.peep});
    any::gemm(r, dev, false, false, nb, P, D, 1.f, hb, D, pwp, P, 0.f, tp, P);
    any::run(r, dev, nb * P, ProjAct{tp, rp, sc.rows, a, P, L.pact});
  }
  R.lod = x.lod;
  C.lod = x.lod;
  if (Tensor* o = r.out("BatchGate")) *o = BG;
  if (Tensor* o = r.out("BatchCellPreAct")) *o = C;
  if (Tensor* o = r.out("BatchHidden")) *o = R;
  if (Tensor* o = r.out("OrderedP0"))
    if (H0) *o = R0;
  *r.out("Projection") = R;
  *r.out("Cell") = C;
}

// dpre[k] = (dR[rows[a+k]] + dr_next[seq[a+k]]) * dpact(R[rows[a+k]]); also into dPre_all
struct LstmpBwdProj {
  const float *R, *dR;
  float *dr_next, *dpre, *dpre_all;
  Sched sc;
  int64_t a, P;
  int pact;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t k = i / P, j = i % P;
    const int row = sc.rows[a + k], s = sc.seq[a + k];
    const float g = (dR ? dR[(int64_t)row * P + j] : 0.f) + dr_next[(int64_t)s * P + j];
    const float v = g * dact(pact, R[(int64_t)row * P + j]);
    dpre[i] = v;
    dpre_all[(int64_t)row * P + j] = v;
  }
};

struct LstmpCellBwd {
  const float *b, *c0, *C, *BG, *dh, *dC;
  float *dG, *dGb, *dc_next;
  Sched sc;
  int64_t a, D;
  int ag, ac, an, peep;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t k = i / D, d = i % D;
    const int row = sc.rows[a + k], pr = sc.prev[a + k], s = sc.seq[a + k];
    const float* g = BG + (int64_t)row * 4 * D;
    const float cand = g[d], ii = g[D + d], f = g[2 * D + d], o = g[3 * D + d];
    const float c = C[(int64_t)row * D + d];
    const float c_1 = pr >= 0 ? C[(int64_t)pr * D + d] : (c0 ? c0[(int64_t)s * D + d] : 0.f);
    const float dhv = dh[i];
    float dc = (dC ? dC[(int64_t)row * D + d] : 0.f) + dc_next[(int64_t)s * D + d];
    const float acv = act(ac, c);
    const float dgo = dhv * acv * dact(ag, o);
    dc += dhv * o * dact(ac, acv);
    if (peep) dc += dgo * b[6 * D + d];
    const float dgc = dc * ii * dact(an, cand);
    const float dgi = dc * cand * dact(ag, ii);
    const float dgf = dc * c_1 * dact(ag, f);
    float dcp = dc * f;
    if (peep) dcp += dgi * b[4 * D + d] + dgf * b[5 * D + d];
    dc_next[(int64_t)s * D + d] = dcp;
    float* o1 = dG + (int64_t)row * 4 * D;
    float* o2 = dGb + k * 4 * D;
    o1[d] = o2[d] = dgc;
    o1[D + d] = o2[D + d] = dgi;
    o1[2 * D + d] = o2[2 * D + d] = dgf;
    o1[3 * D + d] = o2[3 * D + d] = dgo;
  }
};

struct ScatterSeq {  // dst[seq[a+k]] = src[k]
  const float* src;
  float* dst;
  const int* seq;
  int64_t a, W;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t k = i / W, j = i % W;
    dst[(int64_t)seq[a + k] * W + j] = src[i];
  }
};

struct HiddenOf {  // h[row] = o * act_cell(c)   (the un-projected hidden, recomputed)
  const float *BG, *C;
  float* h;
  int64_t D;
  int ac;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t row = i / D, d = i % D;
    h[i] = BG[row * 4 * D + 3 * D + d] * act(ac, C[i]);
  }
};

struct PrevRows {  // out[rows[k]] = R[prev[k]] | r0[seq[k]] | 0 over all n schedule slots
  const float *R, *r0;
  float* out;
  Sched sc;
  int64_t P;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t k = i / P, j = i % P;
    const int pr = sc.prev[k];
    out[(int64_t)sc.rows[k] * P + j] = pr >= 0 ? R[(int64_t)pr * P + j] : (r0 ? r0[(int64_t)sc.seq[k] * P + j] : 0.f);
  }
};

struct CPrevRows {
  const float *C, *c0;
  float* out;
  Sched sc;
  int64_t D;
  __host__ __device__ void operator()(int64_t i) const {
    const int64_t k = i / D, j = i % D;
    const int pr = sc.prev[k];
    out[(int64_t)sc.rows[k] * D + j] = pr >= 0 ? C[(int64_t)pr * D + j] : (c0 ? c0[(int64_t)sc.seq[k] * D + j] : 0.f);
  }
};

struct PeepGrad {  // out = {sum dgi c_prev, sum dgf c_prev, sum dgo c}
  const float *dG, *C, *Cp;
  float* out;
  int64_t T, D;
  __host__ __device__ void operator()(int64_t d) const {
    float si = 0.f, sf = 0.f, so = 0.f;
    for (int64_t t = 0; t < T; ++t) {
      si += dG[t * 4 * D + D + d] * Cp[t * D + d];
      sf += dG[t * 4 * D + 2 * D + d] * Cp[t * D + d];
      so += dG[t * 4 * D + 3 * D + d] * C[t * D + d];
    }
    out[4 * D + d] = si;
    out[5 * D + d] = sf;
    out[6 * D + d] = so;
  }
};

struct MulDact {  // v[i] *= dact(a, y[i])
  float* v;
  const float* y;
  int a;
  __host__ __device__ void operator()(int64_t i) const { v[i] *= dact(a, y[i]); }
};

void k_lstmp_grad(const OpRun& r) {
  const bool dev = r.ctx.device >= 0;
  Tensor& x = r.in("Input");
  Tensor& W = r.in("Weight");
  Tensor& PW = r.in("ProjWeight");
  Tensor& Bt = r.in("Bias");
  Tensor* H0 = r.in_opt("H0");
  Tensor* C0 = r.in_opt("C0");
  const Lstmp L = lstmp_dims(r, x, W, PW, Bt);
  const int64_t D = L.D, P = L.P, T = L.T, N = L.N;
  const float *wp = any::f32(W, dev), *pwp = any::f32(PW, dev), *bp = any::f32(Bt, dev);
  const float *Rp = any::f32(r.in("Projection"), dev), *Cp = any::f32(r.in("Cell"), dev);
  const float* BGp = any::f32(r.in("BatchGate"), dev);
  Tensor* dRt = r.in_opt("Projection@GRAD");
  Tensor* dCt = r.in_opt("Cell@GRAD");
  const float* dR = dRt ? any::f32(*dRt, dev) : nullptr;
  const float* dC = dCt ? any::f32(*dCt, dev) : nullptr;
  const float* c0 = C0 ? any::f32(*C0, dev) : nullptr;
  const float* h0 = H0 ? any::f32(*H0, dev) : nullptr;
  const int place = dev ? r.ctx.device : -1;
  const rnn::SeqBatch sb = rnn::make_batch(x.lod.back(), L.rev);
  std::vector<int> keep;
  const Sched sc = sched(r, dev, sb, &keep);
  // r0 recomputed (OrderedP0 is optional in the program)
  Tensor R0;
  float* r0 = nullptr;
  if (h0) {
    r0 = R0.alloc<float>({N, P}, place);
    any::gemm(r, dev, false, false, N, P, D, 1.f, h0, D, pwp, P, 0.f, r0, P);
    any::run(r, dev, N * P, ProjAct{r0, r0, nullptr, 0, P, L.pact});
  }
  Tensor dG, dPre;
  float* dg = dG.alloc<float>({T, 4 * D}, place);
  float* dpre_all = dPre.alloc<float>({T, P}, place);
  std::vector<float> h1, h2, h3, h4, h5, h6;
  float* dr_next = any::scratch(r, dev, "@lstmp_drn@", N * P, &h1);
  float* dc_next = any::scratch(r, dev, "@lstmp_dcn@", N * D, &h2);
  float* dpre = any::scratch(r, dev, "@lstmp_dpre@", N * P, &h3);
  float* dh = any::scratch(r, dev, "@lstmp_dh@", N * D, &h4);
  float* dGb = any::scratch(r, dev, "@lstmp_dGb@", N * 4 * D, &h5);
  float* drb = any::scratch(r, dev, "@lstmp_drb@", N * P, &h6);
  any::zero(r, dev, dr_next, N * P);
  any::zero(r, dev, dc_next, N * D);
  for (int64_t t = (int64_t)sb.step_begin.size() - 2; t >= 0; --t) {
    const int64_t a = sb.step_begin[(size_t)t], nb = sb.step_begin[(size_t)t + 1] - a;
    any::run(r, dev, nb * P, LstmpBwdProj{Rp, dR, dr_next, dpre, dpre_all, sc, a, P, L.pact});
    any::gemm(r, dev, false, true, nb, D, P, 1.f, dpre, P, pwp, P, 0.f, dh, D);
    any::run(r, dev, nb * D, LstmpCellBwd{bp, c0, Cp, BGp, dh, dC, dg, dGb, dc_next, sc, a, D, L.ag, L.ac, L.an, L.peep});
    any::gemm(r, dev, false, true, nb, P, 4 * D, 1.f, dGb, 4 * D, wp, 4 * D, 0.f, drb, P);
    any::run(r, dev, nb * P, ScatterSeq{drb, dr_next, sc.seq, a, P});
  }
  // (what step 0 passed back reaches r0 / C0)
  if (Tensor* dw = r.out("Weight@GRAD")) {
    Tensor Rprev;
    float* rprev = Rprev.alloc<float>({T, P}, place);
    any::run(r, dev, T * P, PrevRows{Rp, r0, rprev, sc, P});
    any::gemm(r, dev, true, false, P, 4 * D, T, 1.f, rprev, P, dg, 4 * D, 0.f, dw->alloc<float>(W.dims, place), 4 * D);
  }
  Tensor dR0;
  if (h0) {  // d r0 -> d pre-activation of the initial projection
    float* d0 = dR0.alloc<float>({N, P}, place);
    any::copy(r, dev, d0, dr_next, N * P);
    any::run(r, dev, N * P, MulDact{d0, r0, L.pact});
  }
  if (Tensor* dpw = r.out("ProjWeight@GRAD")) {
    Tensor Hh;
    float* hh = Hh.alloc<float>({T, D}, place);
    any::run(r, dev, T * D, HiddenOf{BGp, Cp, hh, D, L.ac});
    float* p = dpw->alloc<float>(PW.dims, place);
    any::gemm(r, dev, true, false, D, P, T, 1.f, hh, D, dpre_all, P, 0.f, p, P);
    if (h0) any::gemm(r, dev, true, false, D, P, N, 1.f, h0, D, dR0.data<float>(), P, 1.f, p, P);
  }
  if (Tensor* db = r.out("Bias@GRAD")) {
    float* o = db->alloc<float>(Bt.dims, place);
    any::run(r, dev, 4 * D, any::ColSum{dg, o, T, 4 * D, 0}, 64);
    if (L.peep) {
      Tensor Cprev;
      float* cpv = Cprev.alloc<float>({T, D}, place);
      any::run(r, dev, T * D, CPrevRows{Cp, c0, cpv, sc, D});
      any::run(r, dev, D, PeepGrad{dg, Cp, cpv, o, T, D}, 64);
    }
  }
  if (Tensor* dh0 = r.out("H0@GRAD"))
    if (h0) any::gemm(r, dev, false, true, N, D, P, 1.f, dR0.data<float>(), P, pwp, P, 0.f,
                      dh0->alloc<float>(H0->dims, place), D);
  if (Tensor* dc0 = r.out("C0@GRAD"))
    if (C0) any::copy(r, dev, dc0->alloc<float>(C0->dims, place), dc_next, N * D);
  if (Tensor* dx = r.out("Input@GRAD")) {
    *dx = dG;
    dx->lod = x.lod;
  }
}

}  // namespace

#define PA_ANY_KERNEL(name, fn) \
  PA_HOST_KERNEL(name, fn);     \
  PA_DEVICE_KERNEL(name, fn)
PA_ANY_KERNEL(gru_unit, k_gru_unit);
PA_ANY_KERNEL(gru_unit_grad, k_gru_unit_grad);
PA_ANY_KERNEL(lstm_unit, k_lstm_unit);
PA_ANY_KERNEL(lstm_unit_grad, k_lstm_unit_grad);
PA_ANY_KERNEL(lstmp, k_lstmp);
PA_ANY_KERNEL(lstmp_grad, k_lstmp_grad);
#undef PA_ANY_KERNEL

void link_rnn_unit_kernels() {}

}  // namespace pa
