// Persistent LSTM forward/backward for gfx950 (MI355X).
//
// A recurrent step is a [B x H] x [H x 4H] product plus pointwise gates: far too
// small to fill the chip, so a per-step launch (MIOpen, or an op-by-op loop) pays a
// kernel boundary and a re-read of W_hh every step.  Here ONE launch walks all T
// steps: H/16 workgroups each own 16 hidden units; their slice of W_hh lives in
// VGPRs (as MFMA B fragments) for the whole sequence, and the only per-step
// traffic is the new hidden state, exchanged through a ping-pong buffer with a
// grid-wide counter barrier (agent-scope release/acquire, bounded spins -- guide
// cdna_hip_programming.md Guideline 16, MI355X_MICROARCH.md "barrier-counter").
//
// Reference behaviour (what, not how): operators/lstm_op.{cc,h} +
// math/detail/lstm_gpu_kernel.h run one kernel per time step over the
// length-sorted LoD batch (sequence2batch), gate order in the reference is
// {c~, i, f, o}; here the torch/paddle-2 order {i, f, g, o} is used and LoD
// lengths are handled by freezing (h, c) past each sequence's end, so h[T-1] is
// every sequence's last state (sequence_pool "last").
//
// Layouts: xproj [T, B, 4H] fp32 (= x W_ih + b), W_hh [H, 4H] bf16 row-major,
// hs/cs [T, B, H] fp32, gates [T, B, 4H] bf16 (post-activation), dgates
// [T, BP, 4H] bf16 (pre-activation gradients; rows >= B are zero),
// hbuf [2, BP, H] bf16.  B <= 128 (BP = 16, 32, 64 or 128), H / 32 in {4, 8, 16, 32}.
#include "common.h"

namespace pa {

typedef __bf16 bf16x8r __attribute__((ext_vector_type(8)));
typedef unsigned int __attribute__((address_space(1))) gu32;

__device__ __forceinline__ f32x4 rnn_mfma(u16x8 a, u16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8r, a), __builtin_bit_cast(bf16x8r, b),
                                                 c, 0, 0, 0);
}

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }
__device__ __forceinline__ float tanh_f(float x) {
  const float e = __expf(-2.f * fabsf(x));
  const float t = (1.f - e) / (1.f + e);
  return copysignf(t, x);
}

constexpr unsigned kSpinLimit = 1u << 22;

// Publish this workgroup's stores of the step and arrive on the counter.
__device__ __forceinline__ void rnn_arrive(unsigned* cnt) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add((gu32*)cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Wait until the counter reaches `target`; false on timeout (err word set, every
// thread of the workgroup returns false so the grid drains).
__device__ __forceinline__ bool rnn_wait(unsigned* cnt, unsigned target, unsigned* err, int* abort_s) {
  if (threadIdx.x == 0) {
    unsigned spins = 0;
    int ok = 1;
    while (__hip_atomic_load((gu32*)cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > kSpinLimit) {
        __hip_atomic_store((gu32*)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
      if (__hip_atomic_load((gu32*)err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
        ok = 0;
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    *abort_s = !ok;
  }
  __syncthreads();
  return *abort_s == 0;
}

struct LstmArgs {
  const float* xproj;
  const u16* whh;
  const int* lens;
  u16* hbuf;
  float* hs;
  float* cs;
  u16* gates;
  const float* h0;  // [B, H] or null
  const float* c0;
  // backward
  const float* dhs;     // [T, B, H] or null: gradient into every h_t output
  const float* dcs;     // [T, B, H] or null: gradient into every c_t output
  const float* dh_last; // [B, H] or null: gradient into h[T-1]
  const float* dc_last; // [B, H] or null
  u16* dgates;          // [T, BP, 4H]
  float* dh0;           // [B, H] or null
  float* dc0;
  unsigned* cnt;
  unsigned* err;
  int T, B, BP, H;
};

// -------------------------------------------------------------------- forward
// grid = (H/16 unit blocks, row blocks of 16 NRT batch rows); wave w computes gate w
// of the 16 units.  Row blocks never exchange data (a row's recurrence only reads
// its own row), so each row block has its own barrier counter.
template <int NRT, int KS>  // row tiles per workgroup; k-steps = H / 32
__global__ __launch_bounds__(256) void lstm_fwd_persistent(LstmArgs a) {
  __shared__ float gs[4][NRT * 16][16];
  __shared__ int abort_s;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j = blockIdx.x, H = a.H, G = 4 * H, B = a.B, BP = a.BP;
  const int row0 = blockIdx.y * NRT * 16;
  unsigned* cnt = a.cnt + 16 * blockIdx.y;
  const int n = lane & 15, kq = lane >> 4;
  const int col = w * H + 16 * j + n;  // this lane's W_hh / gate column
  // resident W_hh fragments: B[k][n] = W_hh[k][col], k = 32 ks + 8 kq + e
  u16x8 wf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    u16x8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = a.whh[(long)(32 * ks + 8 * kq + e) * G + col];
    wf[ks] = v;
  }
  // pointwise ownership: local pairs p = tid + 256 r over (row, unit)
  constexpr int NP = NRT;  // NRT * 16 rows * 16 units / 256 threads
  float creg[NP], hreg[NP];
#pragma unroll
  for (int r = 0; r < NP; ++r) {
    const int p = threadIdx.x + 256 * r;
    const int b = row0 + (p >> 4), u = 16 * j + (p & 15);
    creg[r] = (b < B && a.c0) ? a.c0[(long)b * H + u] : 0.f;
    hreg[r] = (b < B && a.h0) ? a.h0[(long)b * H + u] : 0.f;
  }
  if (threadIdx.x == 0) abort_s = 0;
  for (int t = 0; t < a.T; ++t) {
    // this step's input projection does not depend on other workgroups: issue it
    // before the barrier so its latency hides behind the wait
    float xv[NRT][4];
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int b = row0 + 16 * rt + 4 * kq + i;
        xv[rt][i] = b < B ? a.xproj[((long)t * B + b) * G + col] : 0.f;
      }
    if (t > 0 && !rnn_wait(cnt, (unsigned)(gridDim.x * t), a.err, &abort_s)) return;
    const u16* hin = a.hbuf + (long)(t & 1) * BP * H + (long)row0 * H;
    f32x4 acc[NRT];
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt) acc[rt] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
      for (int rt = 0; rt < NRT; ++rt) {
        const u16x8 av = *reinterpret_cast<const u16x8*>(hin + (long)(16 * rt + n) * H + 32 * ks + 8 * kq);
        acc[rt] = rnn_mfma(av, wf[ks], acc[rt]);
      }
    }
    // epilogue: + x W_ih + b, activation, to LDS (local row 16 rt + 4 kq + i, unit n)
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v = acc[rt][i] + xv[rt][i];
        gs[w][16 * rt + 4 * kq + i][n] = (w == 2) ? tanh_f(v) : sigm(v);
      }
    }
    __syncthreads();
    u16* hout = a.hbuf + (long)((t + 1) & 1) * BP * H;
#pragma unroll
    for (int r = 0; r < NP; ++r) {
      const int p = threadIdx.x + 256 * r;
      const int lb = p >> 4, nn = p & 15, u = 16 * j + nn, b = row0 + lb;
      if (b < B) {
        const float ig = gs[0][lb][nn], fg = gs[1][lb][nn], gg = gs[2][lb][nn], og = gs[3][lb][nn];
        if (t < a.lens[b]) {
          creg[r] = fg * creg[r] + ig * gg;
          hreg[r] = og * tanh_f(creg[r]);
        }
        const long o = ((long)t * B + b) * H + u;
        a.hs[o] = hreg[r];
        a.cs[o] = creg[r];
        u16* gp = a.gates + ((long)t * B + b) * G + u;
        gp[0] = f2bf(ig);
        gp[H] = f2bf(fg);
        gp[2 * H] = f2bf(gg);
        gp[3 * H] = f2bf(og);
      }
      hout[(long)b * H + u] = f2bf(b < B ? hreg[r] : 0.f);
    }
    rnn_arrive(cnt);
  }
}

// -------------------------------------------------------------------- backward
// Wave w owns the K (= gate column) quarter [w G/4, (w+1) G/4) of the recurrent
// product dh_{t-1}[b, u] = sum_G dgates_t[b, G] W_hh[u, G].
template <int NRT, int KS>
__global__ __launch_bounds__(256) void lstm_bwd_persistent(LstmArgs a) {
  __shared__ float red[4][NRT * 16][16];
  __shared__ int abort_s;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j = blockIdx.x, H = a.H, G = 4 * H, B = a.B, BP = a.BP;
  const int row0 = blockIdx.y * NRT * 16;
  unsigned* cnt = a.cnt + 16 * blockIdx.y;
  const int n = lane & 15, kq = lane >> 4;
  const int u_mine = 16 * j + n;
  const int KQ = G / 4;  // K range per wave (= H = 32 KS)
  u16x8 wf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
    wf[ks] = *reinterpret_cast<const u16x8*>(a.whh + (long)u_mine * G + w * KQ + 32 * ks + 8 * kq);
  constexpr int NP = NRT;
  float dh[NP], dc[NP];
#pragma unroll
  for (int r = 0; r < NP; ++r) {
    const int p = threadIdx.x + 256 * r;
    const int b = row0 + (p >> 4), u = 16 * j + (p & 15);
    dh[r] = (b < B && a.dh_last) ? a.dh_last[(long)b * H + u] : 0.f;
    dc[r] = (b < B && a.dc_last) ? a.dc_last[(long)b * H + u] : 0.f;
  }
  if (threadIdx.x == 0) abort_s = 0;
  int steps = 0;
  for (int t = a.T - 1; t >= 0; --t, ++steps) {
    bool act[NP];
    // pointwise: dgates_t for own units
#pragma unroll
    for (int r = 0; r < NP; ++r) {
      const int p = threadIdx.x + 256 * r;
      const int b = row0 + (p >> 4), u = 16 * j + (p & 15);
      act[r] = false;
      u16* dg = a.dgates + ((long)t * BP + b) * G + u;
      if (b >= B) {
        dg[0] = 0; dg[H] = 0; dg[2 * H] = 0; dg[3 * H] = 0;
        continue;
      }
      if (a.dhs) dh[r] += a.dhs[((long)t * B + b) * H + u];
      if (a.dcs) dc[r] += a.dcs[((long)t * B + b) * H + u];
      act[r] = t < a.lens[b];
      if (!act[r]) {
        dg[0] = 0; dg[H] = 0; dg[2 * H] = 0; dg[3 * H] = 0;
        continue;
      }
      const u16* gp = a.gates + ((long)t * B + b) * G + u;
      const float ig = bf2f(gp[0]), fg = bf2f(gp[H]), gg = bf2f(gp[2 * H]), og = bf2f(gp[3 * H]);
      const float c = a.cs[((long)t * B + b) * H + u];
      const float cp = t > 0 ? a.cs[((long)(t - 1) * B + b) * H + u] : (a.c0 ? a.c0[(long)b * H + u] : 0.f);
      const float tc = tanh_f(c);
      const float dO = dh[r] * tc;
      const float dct = dc[r] + dh[r] * og * (1.f - tc * tc);
      const float dI = dct * gg, dG = dct * ig, dF = dct * cp;
      dc[r] = dct * fg;
      dg[0] = f2bf(dI * ig * (1.f - ig));
      dg[H] = f2bf(dF * fg * (1.f - fg));
      dg[2 * H] = f2bf(dG * (1.f - gg * gg));
      dg[3 * H] = f2bf(dO * og * (1.f - og));
    }
    rnn_arrive(cnt);
    if (!rnn_wait(cnt, (unsigned)(gridDim.x * (steps + 1)), a.err, &abort_s)) return;
    // recurrent product over this wave's K quarter
    const u16* dgt = a.dgates + ((long)t * BP + row0) * G;
    f32x4 acc[NRT];
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt) acc[rt] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
      for (int rt = 0; rt < NRT; ++rt) {
        const u16x8 av = *reinterpret_cast<const u16x8*>(dgt + (long)(16 * rt + n) * G + w * KQ + 32 * ks + 8 * kq);
        acc[rt] = rnn_mfma(av, wf[ks], acc[rt]);
      }
    }
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[w][16 * rt + 4 * kq + i][n] = acc[rt][i];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < NP; ++r) {
      const int p = threadIdx.x + 256 * r;
      const int lb = p >> 4, nn = p & 15;
      if (row0 + lb >= B) continue;
      if (act[r]) dh[r] = red[0][lb][nn] + red[1][lb][nn] + red[2][lb][nn] + red[3][lb][nn];
      // inactive step: h_t == h_{t-1}, the gradient passes through unchanged
    }
    __syncthreads();  // red is rewritten next step
  }
#pragma unroll
  for (int r = 0; r < NP; ++r) {
    const int p = threadIdx.x + 256 * r;
    const int b = row0 + (p >> 4), u = 16 * j + (p & 15);
    if (b >= B) continue;
    if (a.dh0) a.dh0[(long)b * H + u] = dh[r];
    if (a.dc0) a.dc0[(long)b * H + u] = dc[r];
  }
}

}  // namespace pa

using namespace pa;

// ws: >= 512 bytes of device scratch: err word + one barrier counter per row block
// (64-B lines), zeroed here every call.
PA_EXPORT int pa_lstm_persistent(int backward, const float* xproj, const void* whh, const int* lens, void* hbuf,
                                 float* hs, float* cs, void* gates, const float* h0, const float* c0,
                                 const float* dhs, const float* dcs, const float* dh_last, const float* dc_last,
                                 void* dgates, float* dh0, float* dc0, unsigned* ws, int T, int B, int H,
                                 hipStream_t st) {
  const int KS = H / 32;
  if (H % 32 || !(KS == 4 || KS == 8 || KS == 16 || KS == 32) || B < 1 || B > 128 || T < 1)
    return (int)hipErrorInvalidValue;
  const int NRT_ALL = B <= 16 ? 1 : B <= 32 ? 2 : B <= 64 ? 4 : 8;  // BP = 16 NRT_ALL rows
  const int NRT = NRT_ALL < 2 ? NRT_ALL : 2;                         // rows per workgroup / 16
  LstmArgs a;
  a.xproj = xproj; a.whh = (const u16*)whh; a.lens = lens; a.hbuf = (u16*)hbuf;
  a.hs = hs; a.cs = cs; a.gates = (u16*)gates; a.h0 = h0; a.c0 = c0;
  a.dhs = dhs; a.dcs = dcs; a.dh_last = dh_last; a.dc_last = dc_last; a.dgates = (u16*)dgates;
  a.dh0 = dh0; a.dc0 = dc0;
  a.err = ws; a.cnt = ws + 16;  // counters at ws[16 (1 + y)], one 64-B line each
  a.T = T; a.B = B; a.BP = 16 * NRT_ALL; a.H = H;
  hipError_t e = hipMemsetAsync(ws, 0, 512, st);
  if (e != hipSuccess) return (int)e;
  const dim3 grid(H / 16, NRT_ALL / NRT), blk(256);
#define PA_LSTM_K(R, K)                                                                   \
  if (backward) hipLaunchKernelGGL((lstm_bwd_persistent<R, K>), grid, blk, 0, st, a);     \
  else hipLaunchKernelGGL((lstm_fwd_persistent<R, K>), grid, blk, 0, st, a);
#define PA_LSTM(R)                                    \
  switch (KS) {                                       \
    case 4: PA_LSTM_K(R, 4) break;                    \
    case 8: PA_LSTM_K(R, 8) break;                    \
    case 16: PA_LSTM_K(R, 16) break;                  \
    default: PA_LSTM_K(R, 32) break;                  \
  }
  if (NRT == 1) {
    PA_LSTM(1)
  } else {
    PA_LSTM(2)
  }
#undef PA_LSTM
#undef PA_LSTM_K
  PA_LAUNCH_CHECK();
}

// ============================================================================
// Attention-LSTM decoder step kernels (seq2seq, reference
// benchmark/fluid/models/machine_translation.py: simple_attention + lstm_step).
// The decoder loop itself is driven from ops/rnn.py (4 launches per step forward,
// 4 backward, all graph-capturable); these fuse what would otherwise be ~15
// elementwise / reduction kernels per step.
// ============================================================================
namespace pa {

// score[b, s] = sum_a w[a] tanh(ep[b, s, a] + sp[b, a]) over s < len[b]; att = softmax;
// ctx[b, :] = sum_s att[s] enc[b, s, :].  One workgroup (256) per batch row; wave per
// source position for the scores (8 a per lane per 512-chunk), thread per 4 ctx columns.
__global__ __launch_bounds__(1024) void add_attn_fwd(const u16* __restrict__ ep, const u16* __restrict__ sp,
                                                      const float* __restrict__ w, const u16* __restrict__ enc,
                                                      const int* __restrict__ lens, u16* __restrict__ ctx, long ctx_ld,
                                                      float* __restrict__ att, int Ts, int A, int E) {
  extern __shared__ float sm[];  // [Ts] scores -> probabilities | [4][E] ctx partials
  float* part = sm + Ts;
  const int b = blockIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int L = min(lens[b], Ts);
  for (int s = wv; s < Ts; s += 16) {
    float acc = 0.f;
    if (s < L) {
      for (int a0 = 8 * lane; a0 < A; a0 += 512) {
        float e8[8], s8[8], w8[8];
        load8(ep + ((long)b * Ts + s) * A + a0, e8);
        load8(sp + (long)b * A + a0, s8);
        load8(w + a0, w8);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += w8[k] * tanhf(e8[k] + s8[k]);
      }
      acc = wave_sum(acc);
    }
    if (lane == 0) sm[s] = s < L ? acc : -INFINITY;
  }
  __syncthreads();
  if (wv == 0) {
    float m = -INFINITY;
    for (int s = lane; s < Ts; s += 64) m = fmaxf(m, sm[s]);
    m = wave_max(m);
    float z = 0.f;
    for (int s = lane; s < Ts; s += 64) z += (sm[s] == -INFINITY) ? 0.f : __expf(sm[s] - m);
    z = wave_sum(z);
    const float inv = z > 0.f ? 1.f / z : 0.f;
    for (int s = lane; s < Ts; s += 64) {
      const float p = (sm[s] == -INFINITY) ? 0.f : __expf(sm[s] - m) * inv;
      sm[s] = p;
      att[(long)b * Ts + s] = p;
    }
  }
  __syncthreads();
  // ctx: 4 thread groups split the source positions (s = g mod 4), 4 columns per thread
  const int g = threadIdx.x >> 8, tt = threadIdx.x & 255;
  for (int e0 = 4 * tt; e0 < E; e0 += 1024) {
    float c4[4] = {0.f, 0.f, 0.f, 0.f};
    for (int s = g; s < L; s += 4) {
      const float p = sm[s];
      const u16x4 v = *reinterpret_cast<const u16x4*>(enc + ((long)b * Ts + s) * E + e0);
#pragma unroll
      for (int k = 0; k < 4; ++k) c4[k] += p * bf2f(v[k]);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) part[g * E + e0 + k] = c4[k];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < E; e += 1024)
    ctx[(long)b * ctx_ld + e] = f2bf(part[e] + part[E + e] + part[2 * E + e] + part[3 * E + e]);
}

// Backward of add_attn_fwd for one decoder step (enc's gradient is formed once,
// after the loop, as att^T dctx; not here):
//   da[s] = dctx . enc[b, s, :];  de = att * (da - sum att da)
//   dz[s, a] = de[s] w[a] (1 - tanh^2(ep + sp)):  dep_acc += dz (fp32, across steps),
//   dsp[b, a] = sum_s dz;  dw_acc[a] += sum_{b, s} de[s] tanh(ep + sp)
__global__ __launch_bounds__(1024) void add_attn_bwd(const u16* __restrict__ dctx, long dctx_ld,
                                                     const float* __restrict__ att, const u16* __restrict__ ep,
                                                     const u16* __restrict__ sp, const float* __restrict__ w,
                                                     const u16* __restrict__ enc, const int* __restrict__ lens,
                                                     float* __restrict__ dep_acc, u16* __restrict__ dsp,
                                                     float* __restrict__ dw_acc, int Ts, int A, int E) {
  extern __shared__ float sm[];  // [Ts] de | [16][A] dsp partial | [16][A] dw partial
  float* de = sm;
  float* pd = sm + Ts;
  float* pw = pd + 16 * A;
  const int b = blockIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int L = min(lens[b], Ts);
  // da[s] (wave per s, 8 columns per lane per 512-chunk)
  for (int s = wv; s < Ts; s += 16) {
    float acc = 0.f;
    if (s < L) {
      for (int e0 = 8 * lane; e0 < E; e0 += 512) {
        float d8[8], x8[8];
        load8(dctx + (long)b * dctx_ld + e0, d8);
        load8(enc + ((long)b * Ts + s) * E + e0, x8);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += d8[k] * x8[k];
      }
      acc = wave_sum(acc);
    }
    if (lane == 0) de[s] = acc;
  }
  __syncthreads();
  if (wv == 0) {
    float sad = 0.f;
    for (int s = lane; s < L; s += 64) sad += att[(long)b * Ts + s] * de[s];
    sad = wave_sum(sad);
    for (int s = lane; s < Ts; s += 64) de[s] = s < L ? att[(long)b * Ts + s] * (de[s] - sad) : 0.f;
  }
  for (int i = threadIdx.x; i < 32 * A; i += 1024) pd[i] = 0.f;  // pd and pw
  __syncthreads();
  for (int a0 = 8 * lane; a0 < A; a0 += 512) {
    float s8[8], w8[8], accd[8], accw[8];
    load8(sp + (long)b * A + a0, s8);
    load8(w + a0, w8);
#pragma unroll
    for (int k = 0; k < 8; ++k) accd[k] = accw[k] = 0.f;
    for (int s = wv; s < L; s += 16) {
      const float d = de[s];
      float e8[8], g8[8];
      load8(ep + ((long)b * Ts + s) * A + a0, e8);
      float* dp = dep_acc + ((long)b * Ts + s) * A + a0;
      load8(dp, g8);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float t = tanhf(e8[k] + s8[k]);
        const float dz = d * w8[k] * (1.f - t * t);
        g8[k] += dz;
        accd[k] += dz;
        accw[k] += d * t;
      }
      store8(dp, g8);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      pd[wv * A + a0 + k] = accd[k];
      pw[wv * A + a0 + k] = accw[k];
    }
  }
  __syncthreads();
  for (int a = threadIdx.x; a < A; a += 1024) {
    float d = 0.f, g = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      d += pd[k * A + a];
      g += pw[k * A + a];
    }
    dsp[(long)b * A + a] = f2bf(d);
    if (g != 0.f) atomicAdd(dw_acc + a, g);
  }
}

// gates = gp[b, :] (+ y[b, :]); i f g o; c = f c_prev + i g; h = o tanh(c).
// Writes c (fp32), post-activation gates (bf16) and h (bf16) to up to two places.
__global__ __launch_bounds__(256) void lstm_cell_fwd(const u16* __restrict__ gp, const float* __restrict__ y,
                                                      const float* __restrict__ cp, float* __restrict__ c_out,
                                                      u16* __restrict__ gates, u16* __restrict__ h1, long ld1,
                                                      u16* __restrict__ h2, long ld2, int B, int H) {
  const long n = (long)B * H;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int b = (int)(i / H), j = (int)(i % H);
    const long g0 = (long)b * 4 * H + j;
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = bf2f(gp[g0 + k * H]) + (y ? y[g0 + k * H] : 0.f);
    const float ig = 1.f / (1.f + __expf(-v[0])), fg = 1.f / (1.f + __expf(-v[1]));
    const float gg = tanhf(v[2]), og = 1.f / (1.f + __expf(-v[3]));
    const float c = fg * (cp ? cp[i] : 0.f) + ig * gg;
    const float h = og * tanhf(c);
    c_out[i] = c;
    gates[g0] = f2bf(ig);
    gates[g0 + H] = f2bf(fg);
    gates[g0 + 2 * H] = f2bf(gg);
    gates[g0 + 3 * H] = f2bf(og);
    h1[(long)b * ld1 + j] = f2bf(h);
    if (h2) h2[(long)b * ld2 + j] = f2bf(h);
  }
}

// dh = dh_out (+ dh_rec, row stride ld_rec); pre-activation gate grads -> dgp (bf16);
// dc (fp32, in place) becomes dc_prev.
__global__ __launch_bounds__(256) void lstm_cell_bwd(const u16* __restrict__ dh_out, const u16* __restrict__ dh_rec,
                                                      long ld_rec, float* __restrict__ dc, const u16* __restrict__ gates,
                                                      const float* __restrict__ c, const float* __restrict__ cp,
                                                      u16* __restrict__ dgp, int B, int H) {
  const long n = (long)B * H;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int b = (int)(i / H), j = (int)(i % H);
    const long g0 = (long)b * 4 * H + j;
    const float dh = (dh_out ? bf2f(dh_out[i]) : 0.f) + (dh_rec ? bf2f(dh_rec[(long)b * ld_rec + j]) : 0.f);
    const float ig = bf2f(gates[g0]), fg = bf2f(gates[g0 + H]), gg = bf2f(gates[g0 + 2 * H]),
                og = bf2f(gates[g0 + 3 * H]);
    const float tc = tanhf(c[i]);
    const float dct = dc[i] + dh * og * (1.f - tc * tc);
    const float cpv = cp ? cp[i] : 0.f;
    dgp[g0] = f2bf(dct * gg * ig * (1.f - ig));
    dgp[g0 + H] = f2bf(dct * cpv * fg * (1.f - fg));
    dgp[g0 + 2 * H] = f2bf(dct * ig * (1.f - gg * gg));
    dgp[g0 + 3 * H] = f2bf(dh * tc * og * (1.f - og));
    dc[i] = dct * fg;
  }
}

}  // namespace pa

PA_EXPORT int pa_add_attn_fwd(const void* ep, const void* sp, const float* w, const void* enc, const int* lens,
                              void* ctx, long ctx_ld, float* att, int B, int Ts, int A, int E, hipStream_t st) {
  if (A % 512 || E % 1024 || Ts < 1 || (Ts + 4 * E) * 4 > 160 * 1024) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(add_attn_fwd, dim3(B), dim3(1024), (Ts + 4 * E) * sizeof(float), st, (const u16*)ep, (const u16*)sp, w,
                     (const u16*)enc, lens, (u16*)ctx, ctx_ld, att, Ts, A, E);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_add_attn_bwd(const void* dctx, long dctx_ld, const float* att, const void* ep, const void* sp,
                              const float* w, const void* enc, const int* lens, float* dep_acc, void* dsp,
                              float* dw_acc, int B, int Ts, int A, int E, hipStream_t st) {
  if (A % 512 || E % 512 || Ts < 1) return (int)hipErrorInvalidValue;
  const size_t lds = (Ts + 32 * A) * sizeof(float);
  if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(add_attn_bwd, dim3(B), dim3(1024), lds, st, (const u16*)dctx, dctx_ld, att, (const u16*)ep,
                     (const u16*)sp, w, (const u16*)enc, lens, dep_acc, (u16*)dsp, dw_acc, Ts, A, E);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_lstm_cell_fwd(const void* gp, const float* y, const float* cp, float* c_out, void* gates, void* h1,
                               long ld1, void* h2, long ld2, int B, int H, hipStream_t st) {
  const int g = stream_grid((long)B * H, 256);
  hipLaunchKernelGGL(lstm_cell_fwd, dim3(g), dim3(256), 0, st, (const u16*)gp, y, cp, c_out, (u16*)gates, (u16*)h1,
                     ld1, (u16*)h2, ld2, B, H);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_lstm_cell_bwd(const void* dh_out, const void* dh_rec, long ld_rec, float* dc, const void* gates,
                               const float* c, const float* cp, void* dgp, int B, int H, hipStream_t st) {
  const int g = stream_grid((long)B * H, 256);
  hipLaunchKernelGGL(lstm_cell_bwd, dim3(g), dim3(256), 0, st, (const u16*)dh_out, (const u16*)dh_rec, ld_rec, dc,
                     (const u16*)gates, c, cp, (u16*)dgp, B, H);
  PA_LAUNCH_CHECK();
}
