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
// grid = H/16 workgroups x 256 threads; wave w computes gate w of the 16 units.
template <int NRT, int KS>  // row tiles = BP / 16; k-steps = H / 32
__global__ __launch_bounds__(256) void lstm_fwd_persistent(LstmArgs a) {
  __shared__ float gs[4][NRT * 16][16];
  __shared__ int abort_s;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j = blockIdx.x, H = a.H, G = 4 * H, B = a.B, BP = NRT * 16;
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
  // pointwise ownership: pairs p = tid + 256 r over (b, u) with b < BP
  constexpr int NP = (NRT * 16 * 16 + 255) / 256;
  float creg[NP], hreg[NP];
#pragma unroll
  for (int r = 0; r < NP; ++r) {
    const int p = threadIdx.x + 256 * r;
    const int b = p >> 4, u = 16 * j + (p & 15);
    creg[r] = (b < B && a.c0) ? a.c0[(long)b * H + u] : 0.f;
    hreg[r] = (b < B && a.h0) ? a.h0[(long)b * H + u] : 0.f;
  }
  if (threadIdx.x == 0) abort_s = 0;
  for (int t = 0; t < a.T; ++t) {
    if (t > 0 && !rnn_wait(a.cnt, (unsigned)(gridDim.x * t), a.err, &abort_s)) return;
    const u16* hin = a.hbuf + (long)(t & 1) * BP * H;
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
    // epilogue: + x W_ih + b, activation, to LDS (row b = 16 rt + 4 kq + i, unit n)
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int b = 16 * rt + 4 * kq + i;
        float v = acc[rt][i];
        if (b < B) v += a.xproj[((long)t * B + b) * G + col];
        gs[w][b][n] = (w == 2) ? tanh_f(v) : sigm(v);
      }
    }
    __syncthreads();
    u16* hout = a.hbuf + (long)((t + 1) & 1) * BP * H;
#pragma unroll
    for (int r = 0; r < NP; ++r) {
      const int p = threadIdx.x + 256 * r;
      const int b = p >> 4, nn = p & 15, u = 16 * j + nn;
      if (b >= BP) continue;
      if (b < B) {
        const float ig = gs[0][b][nn], fg = gs[1][b][nn], gg = gs[2][b][nn], og = gs[3][b][nn];
        const bool active = t < a.lens[b];
        if (active) {
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
    rnn_arrive(a.cnt);
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
  const int j = blockIdx.x, H = a.H, G = 4 * H, B = a.B, BP = NRT * 16;
  const int n = lane & 15, kq = lane >> 4;
  const int u_mine = 16 * j + n;
  const int KQ = G / 4;  // K range per wave (= H = 32 KS)
  u16x8 wf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
    wf[ks] = *reinterpret_cast<const u16x8*>(a.whh + (long)u_mine * G + w * KQ + 32 * ks + 8 * kq);
  constexpr int NP = (NRT * 16 * 16 + 255) / 256;
  float dh[NP], dc[NP];
#pragma unroll
  for (int r = 0; r < NP; ++r) {
    const int p = threadIdx.x + 256 * r;
    const int b = p >> 4, u = 16 * j + (p & 15);
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
      const int b = p >> 4, u = 16 * j + (p & 15);
      act[r] = false;
      if (b >= BP) continue;
      u16* dg = a.dgates + ((long)t * BP + b) * G + u;
      if (b >= B) {
        dg[0] = 0; dg[H] = 0; dg[2 * H] = 0; dg[3 * H] = 0;
        continue;
      }
      if (a.dhs) dh[r] += a.dhs[((long)t * B + b) * H + u];
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
    rnn_arrive(a.cnt);
    if (!rnn_wait(a.cnt, (unsigned)(gridDim.x * (steps + 1)), a.err, &abort_s)) return;
    // recurrent product over this wave's K quarter
    const u16* dgt = a.dgates + (long)t * BP * G;
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
      const int b = p >> 4, nn = p & 15;
      if (b >= B) continue;
      if (act[r]) dh[r] = red[0][b][nn] + red[1][b][nn] + red[2][b][nn] + red[3][b][nn];
      // inactive step: h_t == h_{t-1}, the gradient passes through unchanged
    }
    __syncthreads();  // red is rewritten next step
  }
#pragma unroll
  for (int r = 0; r < NP; ++r) {
    const int p = threadIdx.x + 256 * r;
    const int b = p >> 4, u = 16 * j + (p & 15);
    if (b >= B) continue;
    if (a.dh0) a.dh0[(long)b * H + u] = dh[r];
    if (a.dc0) a.dc0[(long)b * H + u] = dc[r];
  }
}

}  // namespace pa

using namespace pa;

// ws: >= 64 bytes of device scratch for {cnt, err} (zeroed here).
PA_EXPORT int pa_lstm_persistent(int backward, const float* xproj, const void* whh, const int* lens, void* hbuf,
                                 float* hs, float* cs, void* gates, const float* h0, const float* c0,
                                 const float* dhs, const float* dh_last, const float* dc_last, void* dgates,
                                 float* dh0, float* dc0, unsigned* ws, int T, int B, int H, hipStream_t st) {
  const int KS = H / 32;
  if (H % 32 || !(KS == 4 || KS == 8 || KS == 16 || KS == 32) || B < 1 || B > 128 || T < 1)
    return (int)hipErrorInvalidValue;
  const int NRT = B <= 16 ? 1 : B <= 32 ? 2 : B <= 64 ? 4 : 8;  // row tiles; BP = 16 NRT
  const int BP = 16 * NRT;
  LstmArgs a;
  a.xproj = xproj; a.whh = (const u16*)whh; a.lens = lens; a.hbuf = (u16*)hbuf;
  a.hs = hs; a.cs = cs; a.gates = (u16*)gates; a.h0 = h0; a.c0 = c0;
  a.dhs = dhs; a.dh_last = dh_last; a.dc_last = dc_last; a.dgates = (u16*)dgates;
  a.dh0 = dh0; a.dc0 = dc0;
  a.cnt = ws; a.err = ws + 16;  // separate 64-B lines
  a.T = T; a.B = B; a.BP = BP; a.H = H;
  hipError_t e = hipMemsetAsync(ws, 0, 128, st);
  if (e != hipSuccess) return (int)e;
  const dim3 grid(H / 16), blk(256);
#define PA_LSTM_K(NRT, K)                                                                   \
  if (backward) hipLaunchKernelGGL((lstm_bwd_persistent<NRT, K>), grid, blk, 0, st, a);     \
  else hipLaunchKernelGGL((lstm_fwd_persistent<NRT, K>), grid, blk, 0, st, a);
#define PA_LSTM(NRT)                                  \
  switch (KS) {                                       \
    case 4: PA_LSTM_K(NRT, 4) break;                  \
    case 8: PA_LSTM_K(NRT, 8) break;                  \
    case 16: PA_LSTM_K(NRT, 16) break;                \
    default: PA_LSTM_K(NRT, 32) break;                \
  }
  switch (NRT) {
    case 1: PA_LSTM(1) break;
    case 2: PA_LSTM(2) break;
    case 4: PA_LSTM(4) break;
    default: PA_LSTM(8) break;
  }
#undef PA_LSTM
#undef PA_LSTM_K
  PA_LAUNCH_CHECK();
}
