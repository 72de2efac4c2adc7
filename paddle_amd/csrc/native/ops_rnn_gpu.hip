// gfx950 device kernels of the LoD recurrent operators: lstm / lstm_grad, gru /
// gru_grad (semantics and step schedule: ops_rnn.cc, rnn_common.h).
//
// Each time step is one pa_sgemm (exact-fp32 MFMA) over the live sequences'
// previous hidden rows plus one fused elementwise kernel for the cell, as the
// reference's LoDTensor2Batch + math/detail/lstm_gpu_kernel.h / gru_gpu_kernel.h.
// The step schedule (rows / sequence / previous row per batch slot) is built on the
// host from the LoD and uploaded once per op.  The weight gradients are not
// accumulated per step: dW = H_prev^T dG over ALL rows is one GEMM at the end (the
// per-row previous hidden states are gathered once), and the bias / peephole
// gradients are column reductions of dG.
#include <hip/hip_runtime.h>

#include <vector>

#include "device_util.h"
#include "kernel_lib.h"
#include "rnn_common.h"

namespace pa {
namespace {

using rnn::act;
using rnn::dact;

struct Sched {
  const int* rows;
  const int* seq;
  const int* prev;
};

Sched upload_sched(const OpRun& r, const rnn::SeqBatch& sb, const char* tag) {
  const size_t n = sb.rows.size();
  std::vector<int> h(3 * n);
  for (size_t i = 0; i < n; ++i) {
    h[i] = (int)sb.rows[i];
    h[n + i] = (int)sb.seq[i];
    h[2 * n + i] = (int)sb.prev[i];
  }
  const int* d = (const int*)device_upload(r, tag, h.data(), h.size() * sizeof(int));
  return Sched{d, d + n, d + 2 * n};
}

// G[k, :W] = x[rows[a + k], :W] + b ; hb[k] = H[prev] | h0[seq] | 0
__global__ void rnn_gather_kernel(const float* __restrict__ x, const float* __restrict__ b, int W,
                                  const float* __restrict__ H, const float* __restrict__ h0, int D, Sched sc, int a,
                                  int nb, float* __restrict__ G, float* __restrict__ hb) {
  const int64_t n1 = (int64_t)nb * W, n2 = (int64_t)nb * D;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n1 + n2; i += (int64_t)gridDim.x * blockDim.x) {
    if (i < n1) {
      const int k = (int)(i / W), j = (int)(i % W);
      G[i] = x[(int64_t)sc.rows[a + k] * W + j] + (b ? b[j] : 0.f);
    } else {
      const int64_t q = i - n1;
      const int k = (int)(q / D), d = (int)(q % D);
      const int pr = sc.prev[a + k];
      hb[q] = pr >= 0 ? H[(int64_t)pr * D + d] : (h0 ? h0[(int64_t)sc.seq[a + k] * D + d] : 0.f);
    }
  }
}

// ---------------------------------------------------------------- lstm
struct LstmArgs {
  int D, ag, ac, an, peep;
  const float *b, *c0;
  float *H, *C, *BG, *P;
};

__global__ void lstm_cell_kernel(const float* __restrict__ G, LstmArgs A, Sched sc, int a, int nb) {
  const int D = A.D;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < (int64_t)nb * D;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(i / D), d = (int)(i % D);
    const int row = sc.rows[a + k], pr = sc.prev[a + k];
    const float c_1 = pr >= 0 ? A.C[(int64_t)pr * D + d] : (A.c0 ? A.c0[(int64_t)sc.seq[a + k] * D + d] : 0.f);
    const float* g = G + (int64_t)k * 4 * D;
    float gi = g[D + d], gf = g[2 * D + d], go = g[3 * D + d];
    if (A.peep) {
      gi += c_1 * A.b[4 * D + d];
      gf += c_1 * A.b[5 * D + d];
    }
    const float cand = act(A.an, g[d]), ii = act(A.ag, gi), f = act(A.ag, gf);
    const float c = cand * ii + c_1 * f;
    if (A.peep) go += c * A.b[6 * D + d];
    const float o = act(A.ag, go);
    A.C[(int64_t)row * D + d] = c;
    A.H[(int64_t)row * D + d] = o * act(A.ac, c);
    float* bg = A.BG + (int64_t)row * 4 * D;
    bg[d] = cand;
    bg[D + d] = ii;
    bg[2 * D + d] = f;
    bg[3 * D + d] = o;
    if (A.P) A.P[(int64_t)row * D + d] = c;
  }
}

void k_lstm(const OpRun& r) {
  Tensor& x = r.in("Input");
  Tensor& W = r.in("Weight");
  Tensor& Bt = r.in("Bias");
  Tensor* H0 = r.in_opt("H0");
  Tensor* C0 = r.in_opt("C0");
  const int64_t D = W.dims[0], T = x.dims[0];
  const bool peep = r.op.GetBool("use_peepholes", true), rev = r.op.GetBool("is_reverse", false);
  if (x.lod.empty() || x.dims.size() != 2 || x.dims[1] != 4 * D || Bt.numel() != (peep ? 7 : 4) * D) throw Decline{};
  const float *xp = dev_f32(x), *wp = dev_f32(W), *bp = dev_f32(Bt);
  const float* h0 = H0 ? dev_f32(*H0) : nullptr;
  LstmArgs A;
  A.D = (int)D;
  A.ag = rnn::act_id(r.op, "gate_activation", rnn::ACT_SIGMOID);
  A.ac = rnn::act_id(r.op, "cell_activation", rnn::ACT_TANH);
  A.an = rnn::act_id(r.op, "candidate_activation", rnn::ACT_TANH);
  A.peep = peep;
  A.b = bp;
  A.c0 = C0 ? dev_f32(*C0) : nullptr;
  const rnn::SeqBatch sb = rnn::make_batch(x.lod.back(), rev);
  const int dev = dev_id(r);
  A.H = r.out("Hidden")->alloc<float>({T, D}, dev);
  A.C = r.out("Cell")->alloc<float>({T, D}, dev);
  A.BG = r.out("BatchGate") ? r.out("BatchGate")->alloc<float>({T, 4 * D}, dev)
                            : device_workspace(r, "@lstm_bg@", T * 4 * D);
  A.P = r.out("BatchCellPreAct") ? r.out("BatchCellPreAct")->alloc<float>({T, D}, dev) : nullptr;
  r.out("Hidden")->lod = x.lod;
  r.out("Cell")->lod = x.lod;
  const int64_t N = (int64_t)x.lod.back().size() - 1;
  if (T == 0 || N == 0) return;
  const Sched sc = upload_sched(r, sb, "@lstm_sched@");
  float* G = device_workspace(r, "@lstm_G@", N * 4 * D);
  float* hb = device_workspace(r, "@lstm_hb@", N * D);
  hipStream_t s = dev_stream(r);
  for (size_t t = 0; t + 1 < sb.step_begin.size(); ++t) {
    const int a = (int)sb.step_begin[t], nb = (int)(sb.step_begin[t + 1] - a);
    hipLaunchKernelGGL(rnn_gather_kernel, dim3(dev_grid((int64_t)nb * 5 * D)), dim3(256), 0, s, xp, bp, (int)(4 * D),
                       (const float*)A.H, h0, (int)D, sc, a, nb, G, hb);
    if (t > 0 || h0) device_sgemm(s, false, false, nb, 4 * D, D, 1.f, hb, D, wp, 4 * D, 1.f, G, 4 * D);
    hipLaunchKernelGGL(lstm_cell_kernel, dim3(dev_grid((int64_t)nb * D)), dim3(256), 0, s, (const float*)G, A, sc, a,
                       nb);
  }
  PA_HIPCHK(hipGetLastError());
}

struct LstmBwdArgs {
  int D, ag, ac, an, peep;
  const float *b, *c0, *C, *BG, *dH, *dC;
  float *dG, *dGb, *dh_next, *dc_next;
};

__global__ void lstm_cell_bwd_kernel(LstmBwdArgs A, Sched sc, int a, int nb) {
  const int D = A.D;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < (int64_t)nb * D;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(i / D), d = (int)(i % D);
    const int row = sc.rows[a + k], pr = sc.prev[a + k], s = sc.seq[a + k];
    const float* g = A.BG + (int64_t)row * 4 * D;
    const float cand = g[d], ii = g[D + d], f = g[2 * D + d], o = g[3 * D + d];
    const float c = A.C[(int64_t)row * D + d];
    const float c_1 = pr >= 0 ? A.C[(int64_t)pr * D + d] : (A.c0 ? A.c0[(int64_t)s * D + d] : 0.f);
    const float dh = (A.dH ? A.dH[(int64_t)row * D + d] : 0.f) + A.dh_next[(int64_t)s * D + d];
    float dc = (A.dC ? A.dC[(int64_t)row * D + d] : 0.f) + A.dc_next[(int64_t)s * D + d];
    const float acv = act(A.ac, c);
    const float dgo = dh * acv * dact(A.ag, o);
    dc += dh * o * dact(A.ac, acv);
    if (A.peep) dc += dgo * A.b[6 * D + d];
    const float dgc = dc * ii * dact(A.an, cand);
    const float dgi = dc * cand * dact(A.ag, ii);
    const float dgf = dc * c_1 * dact(A.ag, f);
    float dcp = dc * f;
    if (A.peep) dcp += dgi * A.b[4 * D + d] + dgf * A.b[5 * D + d];
    A.dc_next[(int64_t)s * D + d] = dcp;
    float* dg = A.dG + (int64_t)row * 4 * D;
    float* dgb = A.dGb + (int64_t)k * 4 * D;
    dg[d] = dgb[d] = dgc;
    dg[D + d] = dgb[D + d] = dgi;
    dg[2 * D + d] = dgb[2 * D + d] = dgf;
    dg[3 * D + d] = dgb[3 * D + d] = dgo;
  }
}

// dh_next[seq[a + k]] = dhb[k]
__global__ void rnn_scatter_seq_kernel(const float* __restrict__ dhb, float* __restrict__ dst, int D, Sched sc, int a,
                                       int nb) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < (int64_t)nb * D;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(i / D), d = (int)(i % D);
    dst[(int64_t)sc.seq[a + k] * D + d] = dhb[i];
  }
}

// per LoD row: the hidden state the row's step started from (H[prev] | h0[seq] | 0)
__global__ void rnn_prev_rows_kernel(const float* __restrict__ H, const float* __restrict__ h0, int D, Sched sc,
                                     int n, float* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < (int64_t)n * D;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(i / D), d = (int)(i % D);
    const int pr = sc.prev[k];
    out[(int64_t)sc.rows[k] * D + d] = pr >= 0 ? H[(int64_t)pr * D + d] : (h0 ? h0[(int64_t)sc.seq[k] * D + d] : 0.f);
  }
}

// out[j] (+)= sum over rows of X[row, j]   (one thread per column; T is small)
__global__ void colsum_kernel(const float* __restrict__ X, int64_t T, int W, int ld, float* __restrict__ out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= W) return;
  float s = 0.f;
  for (int64_t t = 0; t < T; ++t) s += X[t * ld + j];
  out[j] = s;
}

// peephole gradients: dW_ic = sum dgi c_prev, dW_fc = sum dgf c_prev, dW_oc = sum dgo c
__global__ void lstm_peep_grad_kernel(const float* __restrict__ dG, const float* __restrict__ C,
                                      const float* __restrict__ Cprev, int64_t T, int D, float* __restrict__ out) {
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= D) return;
  float si = 0.f, sf = 0.f, so = 0.f;
  for (int64_t t = 0; t < T; ++t) {
    const float cp = Cprev[t * D + d];
    si += dG[t * 4 * D + D + d] * cp;
    sf += dG[t * 4 * D + 2 * D + d] * cp;
    so += dG[t * 4 * D + 3 * D + d] * C[t * D + d];
  }
  out[d] = si;
  out[D + d] = sf;
  out[2 * D + d] = so;
}

void k_lstm_grad(const OpRun& r) {
  Tensor& x = r.in("Input");
  Tensor& W = r.in("Weight");
  Tensor& Bt = r.in("Bias");
  Tensor* H0 = r.in_opt("H0");
  Tensor* C0 = r.in_opt("C0");
  Tensor* dH = r.in_opt("Hidden@GRAD");
  Tensor* dC = r.in_opt("Cell@GRAD");
  const int64_t D = W.dims[0], T = x.dims[0];
  const bool peep = r.op.GetBool("use_peepholes", true), rev = r.op.GetBool("is_reverse", false);
  if (x.lod.empty()) throw Decline{};
  LstmBwdArgs A;
  A.D = (int)D;
  A.ag = rnn::act_id(r.op, "gate_activation", rnn::ACT_SIGMOID);
  A.ac = rnn::act_id(r.op, "cell_activation", rnn::ACT_TANH);
  A.an = rnn::act_id(r.op, "candidate_activation", rnn::ACT_TANH);
  A.peep = peep;
  const float* wp = dev_f32(W);
  A.b = dev_f32(Bt);
  A.c0 = C0 ? dev_f32(*C0) : nullptr;
  const float* hp = dev_f32(r.in("Hidden"));
  A.C = dev_f32(r.in("Cell"));
  A.BG = dev_f32(r.in("BatchGate"));
  A.dH = dH ? dev_f32(*dH) : nullptr;
  A.dC = dC ? dev_f32(*dC) : nullptr;
  const float* h0 = H0 ? dev_f32(*H0) : nullptr;
  const int dev = dev_id(r);
  const int64_t N = (int64_t)x.lod.back().size() - 1;
  const rnn::SeqBatch sb = rnn::make_batch(x.lod.back(), rev);
  hipStream_t s = dev_stream(r);
  Tensor* dxt = r.out("Input@GRAD");
  A.dG = dxt ? dxt->alloc<float>({T, 4 * D}, dev) : device_workspace(r, "@lstm_dG@", T * 4 * D);
  if (dxt) dxt->lod = x.lod;
  A.dGb = device_workspace(r, "@lstm_dGb@", std::max<int64_t>(N, 1) * 4 * D);
  A.dh_next = device_workspace(r, "@lstm_dhn@", std::max<int64_t>(N, 1) * D);
  A.dc_next = device_workspace(r, "@lstm_dcn@", std::max<int64_t>(N, 1) * D);
  float* dhb = device_workspace(r, "@lstm_dhb@", std::max<int64_t>(N, 1) * D);
  PA_HIPCHK(hipMemsetAsync(A.dh_next, 0, sizeof(float) * N * D, s));
  PA_HIPCHK(hipMemsetAsync(A.dc_next, 0, sizeof(float) * N * D, s));
  if (T > 0 && N > 0) {
    const Sched sc = upload_sched(r, sb, "@lstmg_sched@");
    for (int64_t t = (int64_t)sb.step_begin.size() - 2; t >= 0; --t) {
      const int a = (int)sb.step_begin[(size_t)t], nb = (int)(sb.step_begin[(size_t)t + 1] - a);
      hipLaunchKernelGGL(lstm_cell_bwd_kernel, dim3(dev_grid((int64_t)nb * D)), dim3(256), 0, s, A, sc, a, nb);
      device_sgemm(s, false, true, nb, D, 4 * D, 1.f, A.dGb, 4 * D, wp, 4 * D, 0.f, dhb, D);
      hipLaunchKernelGGL(rnn_scatter_seq_kernel, dim3(dev_grid((int64_t)nb * D)), dim3(256), 0, s, (const float*)dhb,
                         A.dh_next, (int)D, sc, a, nb);
    }
    const int n = (int)sb.rows.size();
    float* hprev = device_workspace(r, "@lstm_hprev@", T * D);
    hipLaunchKernelGGL(rnn_prev_rows_kernel, dim3(dev_grid((int64_t)n * D)), dim3(256), 0, s, hp, h0, (int)D, sc, n,
                       hprev);
    if (Tensor* dw = r.out("Weight@GRAD"))
      device_sgemm(s, true, false, D, 4 * D, T, 1.f, hprev, D, A.dG, 4 * D, 0.f, dw->alloc<float>(W.dims, dev), 4 * D);
    if (Tensor* db = r.out("Bias@GRAD")) {
      float* o = db->alloc<float>(Bt.dims, dev);
      hipLaunchKernelGGL(colsum_kernel, dim3(dev_grid(4 * D)), dim3(256), 0, s, (const float*)A.dG, T, (int)(4 * D),
                         (int)(4 * D), o);
      if (peep) {
        float* cprev = device_workspace(r, "@lstm_cprev@", T * D);
        hipLaunchKernelGGL(rnn_prev_rows_kernel, dim3(dev_grid((int64_t)n * D)), dim3(256), 0, s, A.C, A.c0, (int)D,
                           sc, n, cprev);
        hipLaunchKernelGGL(lstm_peep_grad_kernel, dim3(dev_grid(D)), dim3(256), 0, s, (const float*)A.dG, A.C,
                           (const float*)cprev, T, (int)D, o + 4 * D);
      }
    }
  } else {
    if (Tensor* dw = r.out("Weight@GRAD")) PA_HIPCHK(hipMemsetAsync(dw->alloc<float>(W.dims, dev), 0, W.nbytes(), s));
    if (Tensor* db = r.out("Bias@GRAD")) PA_HIPCHK(hipMemsetAsync(db->alloc<float>(Bt.dims, dev), 0, Bt.nbytes(), s));
  }
  if (Tensor* dh0 = r.out("H0@GRAD"))
    if (H0) PA_HIPCHK(hipMemcpyAsync(dh0->alloc<float>(H0->dims, dev), A.dh_next, sizeof(float) * N * D,
                                     hipMemcpyDeviceToDevice, s));
  if (Tensor* dc0 = r.out("C0@GRAD"))
    if (C0) PA_HIPCHK(hipMemcpyAsync(dc0->alloc<float>(C0->dims, dev), A.dc_next, sizeof(float) * N * D,
                                     hipMemcpyDeviceToDevice, s));
  PA_HIPCHK(hipGetLastError());
}

// ---------------------------------------------------------------- gru
// after G[:, :2D] += h_prev W_{u,r}: activate u, r in place; RHb = r * h_prev
__global__ void gru_gate_kernel(float* __restrict__ G, const float* __restrict__ hb, float* __restrict__ rhb, int D,
                                int ag, int nb) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < (int64_t)nb * D;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(i / D), d = (int)(i % D);
    float* g = G + (int64_t)k * 3 * D;
    g[d] = act(ag, g[d]);
    const float rr = act(ag, g[D + d]);
    g[D + d] = rr;
    rhb[i] = rr * hb[i];
  }
}

struct GruOut {
  int D, an;
  float *H, *BG, *RHP;
};

__global__ void gru_out_kernel(const float* __restrict__ G, const float* __restrict__ hb, const float* __restrict__ rhb,
                               GruOut A, Sched sc, int a, int nb) {
  const int D = A.D;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < (int64_t)nb * D;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(i / D), d = (int)(i % D);
    const int row = sc.rows[a + k];
    const float* g = G + (int64_t)k * 3 * D;
    const float u = g[d], c = act(A.an, g[2 * D + d]), hpv = hb[i];
    A.H[(int64_t)row * D + d] = hpv - u * hpv + u * c;
    float* bg = A.BG + (int64_t)row * 3 * D;
    bg[d] = u;
    bg[D + d] = g[D + d];
    bg[2 * D + d] = c;
    A.RHP[(int64_t)row * D + d] = rhb[i];
  }
}

void k_gru(const OpRun& r) {
  Tensor& x = r.in("Input");
  Tensor& W = r.in("Weight");
  Tensor* Bt = r.in_opt("Bias");
  Tensor* H0 = r.in_opt("H0");
  const int64_t D = W.dims[0], T = x.dims[0];
  if (x.lod.empty() || x.dims.size() != 2 || x.dims[1] != 3 * D) throw Decline{};
  const bool rev = r.op.GetBool("is_reverse", false);
  const int an = rnn::act_id(r.op, "activation", rnn::ACT_TANH);
  const int ag = rnn::act_id(r.op, "gate_activation", rnn::ACT_SIGMOID);
  const float *xp = dev_f32(x), *wp = dev_f32(W), *bp = Bt ? dev_f32(*Bt) : nullptr, *h0 = H0 ? dev_f32(*H0) : nullptr;
  const int dev = dev_id(r);
  GruOut A;
  A.D = (int)D;
  A.an = an;
  A.H = r.out("Hidden")->alloc<float>({T, D}, dev);
  A.BG = r.out("BatchGate") ? r.out("BatchGate")->alloc<float>({T, 3 * D}, dev)
                            : device_workspace(r, "@gru_bg@", T * 3 * D);
  A.RHP = r.out("BatchResetHiddenPrev") ? r.out("BatchResetHiddenPrev")->alloc<float>({T, D}, dev)
                                        : device_workspace(r, "@gru_rhp@", T * D);
  r.out("Hidden")->lod = x.lod;
  const int64_t N = (int64_t)x.lod.back().size() - 1;
  hipStream_t s = dev_stream(r);
  if (T > 0 && N > 0) {
    const rnn::SeqBatch sb = rnn::make_batch(x.lod.back(), rev);
    const Sched sc = upload_sched(r, sb, "@gru_sched@");
    float* G = device_workspace(r, "@gru_G@", N * 3 * D);
    float* hb = device_workspace(r, "@gru_hb@", N * D);
    float* rhb = device_workspace(r, "@gru_rhb@", N * D);
    for (size_t t = 0; t + 1 < sb.step_begin.size(); ++t) {
      const int a = (int)sb.step_begin[t], nb = (int)(sb.step_begin[t + 1] - a);
      hipLaunchKernelGGL(rnn_gather_kernel, dim3(dev_grid((int64_t)nb * 4 * D)), dim3(256), 0, s, xp, bp,
                         (int)(3 * D), (const float*)A.H, h0, (int)D, sc, a, nb, G, hb);
      device_sgemm(s, false, false, nb, 2 * D, D, 1.f, hb, D, wp, 3 * D, 1.f, G, 3 * D);
      hipLaunchKernelGGL(gru_gate_kernel, dim3(dev_grid((int64_t)nb * D)), dim3(256), 0, s, G, (const float*)hb, rhb,
                         (int)D, ag, nb);
      device_sgemm(s, false, false, nb, D, D, 1.f, rhb, D, wp + 2 * D, 3 * D, 1.f, G + 2 * D, 3 * D);
      hipLaunchKernelGGL(gru_out_kernel, dim3(dev_grid((int64_t)nb * D)), dim3(256), 0, s, (const float*)G,
                         (const float*)hb, (const float*)rhb, A, sc, a, nb);
    }
  }
  if (Tensor* bh = r.out("BatchHidden"))
    PA_HIPCHK(hipMemcpyAsync(bh->alloc<float>({T, D}, dev), A.H, sizeof(float) * T * D, hipMemcpyDeviceToDevice, s));
  PA_HIPCHK(hipGetLastError());
}

struct GruBwd {
  int D, an, ag;
  const float *BG, *dH, *H, *h0;
  float *dG, *dGb, *dh_next, *dhprev, *hb;
};

// d candidate / d update pre-activations, the direct dh_prev path, h_prev batch
__global__ void gru_bwd1_kernel(GruBwd A, Sched sc, int a, int nb) {
  const int D = A.D;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < (int64_t)nb * D;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(i / D), d = (int)(i % D);
    const int row = sc.rows[a + k], pr = sc.prev[a + k], s = sc.seq[a + k];
    const float hpv = pr >= 0 ? A.H[(int64_t)pr * D + d] : (A.h0 ? A.h0[(int64_t)s * D + d] : 0.f);
    A.hb[i] = hpv;
    const float* g = A.BG + (int64_t)row * 3 * D;
    const float u = g[d], c = g[2 * D + d];
    const float dh = (A.dH ? A.dH[(int64_t)row * D + d] : 0.f) + A.dh_next[(int64_t)s * D + d];
    float* dgb = A.dGb + (int64_t)k * 3 * D;
    dgb[2 * D + d] = dh * u * dact(A.an, c);
    dgb[d] = dh * (c - hpv) * dact(A.ag, u);
    A.dhprev[i] = dh * (1.f - u);
  }
}

// d reset pre-activation from d(r h_prev); dh_prev += d(r h_prev) r; dG rows out
__global__ void gru_bwd2_kernel(GruBwd A, const float* __restrict__ drh, Sched sc, int a, int nb) {
  const int D = A.D;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < (int64_t)nb * D;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(i / D), d = (int)(i % D);
    const int row = sc.rows[a + k];
    const float rr = A.BG[(int64_t)row * 3 * D + D + d];
    float* dgb = A.dGb + (int64_t)k * 3 * D;
    dgb[D + d] = drh[i] * A.hb[i] * dact(A.ag, rr);
    A.dhprev[i] += drh[i] * rr;
    float* dg = A.dG + (int64_t)row * 3 * D;
    dg[d] = dgb[d];
    dg[D + d] = dgb[D + d];
    dg[2 * D + d] = dgb[2 * D + d];
  }
}

void k_gru_grad(const OpRun& r) {
  Tensor& x = r.in("Input");
  Tensor& W = r.in("Weight");
  Tensor* Bt = r.in_opt("Bias");
  Tensor* H0 = r.in_opt("H0");
  Tensor* dH = r.in_opt("Hidden@GRAD");
  const int64_t D = W.dims[0], T = x.dims[0];
  if (x.lod.empty()) throw Decline{};
  const bool rev = r.op.GetBool("is_reverse", false);
  GruBwd A;
  A.D = (int)D;
  A.an = rnn::act_id(r.op, "activation", rnn::ACT_TANH);
  A.ag = rnn::act_id(r.op, "gate_activation", rnn::ACT_SIGMOID);
  const float* wp = dev_f32(W);
  A.BG = dev_f32(r.in("BatchGate"));
  A.H = dev_f32(r.in("Hidden"));
  A.h0 = H0 ? dev_f32(*H0) : nullptr;
  A.dH = dH ? dev_f32(*dH) : nullptr;
  const float* rhp = dev_f32(r.in("BatchResetHiddenPrev"));
  const int dev = dev_id(r);
  const int64_t N = (int64_t)x.lod.back().size() - 1, Nm = std::max<int64_t>(N, 1);
  hipStream_t s = dev_stream(r);
  Tensor* dxt = r.out("Input@GRAD");
  A.dG = dxt ? dxt->alloc<float>({T, 3 * D}, dev) : device_workspace(r, "@gru_dG@", T * 3 * D);
  if (dxt) dxt->lod = x.lod;
  A.dGb = device_workspace(r, "@gru_dGb@", Nm * 3 * D);
  A.dh_next = device_workspace(r, "@gru_dhn@", Nm * D);
  A.dhprev = device_workspace(r, "@gru_dhp@", Nm * D);
  A.hb = device_workspace(r, "@gru_hbb@", Nm * D);
  float* drh = device_workspace(r, "@gru_drh@", Nm * D);
  PA_HIPCHK(hipMemsetAsync(A.dh_next, 0, sizeof(float) * N * D, s));
  if (T > 0 && N > 0) {
    const rnn::SeqBatch sb = rnn::make_batch(x.lod.back(), rev);
    const Sched sc = upload_sched(r, sb, "@grug_sched@");
    for (int64_t t = (int64_t)sb.step_begin.size() - 2; t >= 0; --t) {
      const int a = (int)sb.step_begin[(size_t)t], nb = (int)(sb.step_begin[(size_t)t + 1] - a);
      const dim3 g(dev_grid((int64_t)nb * D));
      hipLaunchKernelGGL(gru_bwd1_kernel, g, dim3(256), 0, s, A, sc, a, nb);
      device_sgemm(s, false, true, nb, D, D, 1.f, A.dGb + 2 * D, 3 * D, wp + 2 * D, 3 * D, 0.f, drh, D);
      hipLaunchKernelGGL(gru_bwd2_kernel, g, dim3(256), 0, s, A, (const float*)drh, sc, a, nb);
      device_sgemm(s, false, true, nb, D, 2 * D, 1.f, A.dGb, 3 * D, wp, 3 * D, 1.f, A.dhprev, D);
      hipLaunchKernelGGL(rnn_scatter_seq_kernel, g, dim3(256), 0, s, (const float*)A.dhprev, A.dh_next, (int)D, sc,
                         a, nb);
    }
    if (Tensor* dw = r.out("Weight@GRAD")) {
      float* o = dw->alloc<float>(W.dims, dev);
      const int n = (int)sb.rows.size();
      float* hprev = device_workspace(r, "@gru_hprev@", T * D);
      hipLaunchKernelGGL(rnn_prev_rows_kernel, dim3(dev_grid((int64_t)n * D)), dim3(256), 0, s, A.H, A.h0, (int)D,
                         sc, n, hprev);
      device_sgemm(s, true, false, D, 2 * D, T, 1.f, hprev, D, A.dG, 3 * D, 0.f, o, 3 * D);
      device_sgemm(s, true, false, D, D, T, 1.f, rhp, D, A.dG + 2 * D, 3 * D, 0.f, o + 2 * D, 3 * D);
    }
    if (Tensor* db = r.out("Bias@GRAD"))
      if (Bt)
        hipLaunchKernelGGL(colsum_kernel, dim3(dev_grid(3 * D)), dim3(256), 0, s, (const float*)A.dG, T, (int)(3 * D),
                           (int)(3 * D), db->alloc<float>(Bt->dims, dev));
  } else {
    if (Tensor* dw = r.out("Weight@GRAD")) PA_HIPCHK(hipMemsetAsync(dw->alloc<float>(W.dims, dev), 0, W.nbytes(), s));
    if (Tensor* db = r.out("Bias@GRAD"))
      if (Bt) PA_HIPCHK(hipMemsetAsync(db->alloc<float>(Bt->dims, dev), 0, Bt->nbytes(), s));
  }
  if (Tensor* dh0 = r.out("H0@GRAD"))
    if (H0) PA_HIPCHK(hipMemcpyAsync(dh0->alloc<float>(H0->dims, dev), A.dh_next, sizeof(float) * N * D,
                                     hipMemcpyDeviceToDevice, s));
  PA_HIPCHK(hipGetLastError());
}

}  // namespace

PA_DEVICE_KERNEL(lstm, k_lstm);
PA_DEVICE_KERNEL(lstm_grad, k_lstm_grad);
PA_DEVICE_KERNEL(gru, k_gru);
PA_DEVICE_KERNEL(gru_grad, k_gru_grad);

}  // namespace pa
