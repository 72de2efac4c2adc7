// RMSNorm / LayerNorm forward + backward for gfx950.
//
// Parity: reference layer_norm (paddle/fluid/operators/layer_norm_op.cu:66-406,
// one block per row with cub BlockReduce, 3 backward kernels).  Redesigned for
// CDNA4: one wave64 per row, the whole row lives in VGPRs (H/512 x 16-byte
// vectors per lane), reductions are pure in-wave shuffles (no LDS, no barrier),
// and the residual add of a pre-norm transformer block is fused in
// (h = x + residual; y = norm(h)) so the residual stream is read once.
// dgamma/dbeta are accumulated in registers across the rows a wave owns,
// folded across the block's waves with LDS float atomics and written as one
// fp32 partial row per block; a second tiny kernel sums the partials.
#include <stdlib.h>

#include "common.h"

namespace pa {

template <typename T, int MAXV, bool RMS, bool HAS_RES, bool HAS_BIAS>
__global__ __launch_bounds__(256) void norm_fwd_kernel(
    const T* __restrict__ x, const T* __restrict__ res, const T* __restrict__ w,
    const T* __restrict__ b, T* __restrict__ y, T* __restrict__ hout,
    float* __restrict__ mean_out, float* __restrict__ rstd_out, long N, int H, float eps) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= N) return;
  const T* xr = x + row * H;
  float v[MAXV][8];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (c < H) {
      load8(xr + c, v[k]);
      if (HAS_RES) {
        float r[8];
        load8(res + row * H + c, r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[k][j] += r[j];
        if (hout) store8(hout + row * H + c, v[k]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += RMS ? v[k][j] * v[k][j] : v[k][j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[k][j] = 0.f;
    }
  }
  s = wave_sum(s);
  float mean = 0.f, rstd;
  if (RMS) {
    rstd = rsqrtf(s / H + eps);
  } else {
    mean = s / H;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int c = (k * 64 + lane) * 8;
      if (c < H) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { float d = v[k][j] - mean; q += d * d; }
      }
    }
    q = wave_sum(q);
    rstd = rsqrtf(q / H + eps);
  }
  if (lane == 0) {
    rstd_out[row] = rstd;
    if (!RMS && mean_out) mean_out[row] = mean;
  }
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (c < H) {
      float g[8], o[8];
      load8(w + c, g);
      if (HAS_BIAS) {
        float bb[8];
        load8(b + c, bb);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (v[k][j] - mean) * rstd * g[j] + bb[j];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (v[k][j] - mean) * rstd * g[j];
      }
      store8(y + row * H + c, o);
    }
  }
}

// Backward.  dx = rstd*(g*dy - mean(g*dy) [LN only] - xhat*mean(g*dy*xhat)) + dres
// Each block owns a contiguous range of rows; waves take rows round-robin.  The
// row's h and dy stay in VGPRs in their storage dtype (packed bf16 = 4 VGPRs per
// 8 elements); gamma is re-read from L1 each row.  dgamma/dbeta accumulate in
// registers; rows wider than 4096 are split over two waves (WPR) to keep that.
template <typename T> struct Raw8;
template <> struct Raw8<u16> {
  u16x8 v;
  __device__ __forceinline__ void load(const u16* p) { v = *reinterpret_cast<const u16x8*>(p); }
  __device__ __forceinline__ float operator[](int j) const { return bf2f(v[j]); }
};
template <> struct Raw8<float> {
  f32x4 a, b;
  __device__ __forceinline__ void load(const float* p) {
    a = *reinterpret_cast<const f32x4*>(p);
    b = *reinterpret_cast<const f32x4*>(p + 4);
  }
  __device__ __forceinline__ float operator[](int j) const { return j < 4 ? a[j] : b[j - 4]; }
};

template <typename T, int MAXV, bool RMS, bool HAS_DRES, int WPR>
__global__ __launch_bounds__(256) void norm_bwd_kernel(
    const T* __restrict__ dy, const T* __restrict__ h, const T* __restrict__ w,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    const T* __restrict__ dres, T* __restrict__ dx, float* __restrict__ dw_part,
    float* __restrict__ db_part, long N, int H, long rows_per_block) {
  // WPR waves share one row (WPR = 2 for 4096 < H <= 8192): every lane then holds
  // at most 8 x 8 elements, so dgamma/dbeta stay in registers instead of per-row
  // LDS atomics (8-way bank-conflicted with the 8-float lane stride).
  constexpr bool ACC_REG = MAXV <= 8;
  constexpr int AV = ACC_REG ? MAXV : 1;
  constexpr int RPI = 4 / WPR;  // rows in flight per block iteration
  extern __shared__ __attribute__((aligned(16))) float sm[];  // [2*H] dw, db; [8] row partials
  float* xred = sm + 2 * H;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int tir = (wv % WPR) * 64 + lane, rg = wv / WPR;
  for (int i = threadIdx.x; i < 2 * H; i += 256) sm[i] = 0.f;
  __syncthreads();
  float aw[AV][8], ab[AV][8];
#pragma unroll
  for (int k = 0; k < AV; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) { aw[k][j] = 0.f; ab[k][j] = 0.f; }
  const long r0 = (long)blockIdx.x * rows_per_block;
  const long r1 = min(N, r0 + rows_per_block);
  // block-uniform trip count: the WPR > 1 exchange below has a barrier
  const long iters = (r1 - r0 + RPI - 1) / RPI;
  for (long it = 0; it < iters; ++it) {
    const long row = r0 + it * RPI + rg;
    const bool live = row < r1;
    const float rstd = live ? rstd_in[row] : 0.f;
    const float mean = (RMS || !live) ? 0.f : mean_in[row];
    Raw8<T> hx[MAXV], dd[MAXV];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int c = (k * 64 * WPR + tir) * 8;
      if (live && c < H) {
        hx[k].load(h + row * H + c);
        dd[k].load(dy + row * H + c);
        float g[8];
        load8(w + c, g);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = (hx[k][j] - mean) * rstd;
          const float gd = g[j] * dd[k][j];
          s1 += gd;
          s2 += gd * xh;
          if (ACC_REG) {
            aw[ACC_REG ? k : 0][j] += dd[k][j] * xh;
            ab[ACC_REG ? k : 0][j] += dd[k][j];
          } else {
            atomicAdd(&sm[c + j], dd[k][j] * xh);
            if (!RMS) atomicAdd(&sm[H + c + j], dd[k][j]);
          }
        }
      }
    }
    s2 = wave_sum(s2);
    if (!RMS) s1 = wave_sum(s1);
    if (WPR > 1) {
      if (lane == 0) { xred[wv * 2] = s1; xred[wv * 2 + 1] = s2; }
      __syncthreads();
      float t1 = 0.f, t2 = 0.f;
#pragma unroll
      for (int q = 0; q < WPR; ++q) { t1 += xred[(rg * WPR + q) * 2]; t2 += xred[(rg * WPR + q) * 2 + 1]; }
      s1 = t1; s2 = t2;
      __syncthreads();  // xred is rewritten next iteration
    }
    s2 /= H;
    s1 /= H;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int c = (k * 64 * WPR + tir) * 8;
      if (live && c < H) {
        float o[8], g[8];
        load8(w + c, g);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = (hx[k][j] - mean) * rstd;
          o[j] = rstd * (g[j] * dd[k][j] - (RMS ? 0.f : s1) - xh * s2);
        }
        if (HAS_DRES) {
          float r[8];
          load8(dres + row * H + c, r);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += r[j];
        }
        store8(dx + row * H + c, o);
      }
    }
  }
  if (ACC_REG) {
#pragma unroll
    for (int k = 0; k < AV; ++k) {
      const int c = (k * 64 * WPR + tir) * 8;
      if (c < H) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          atomicAdd(&sm[c + j], aw[k][j]);
          if (!RMS) atomicAdd(&sm[H + c + j], ab[k][j]);
        }
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < H; i += 256) {
    dw_part[(long)blockIdx.x * H + i] = sm[i];
    if (!RMS) db_part[(long)blockIdx.x * H + i] = sm[H + i];
  }
}

// Column sum of a [G, H] fp32 partial matrix into out[H] (dtype T).  Each block
// owns 64 columns; its 4 waves split the G rows and fold through LDS, so H/64
// blocks x 4 waves cover the chip even for H = 4096 (64 blocks).
// 16 waves per 64 columns (each sums G/16 partial rows, fixed order), grid.y = 1 or
// 2 partial sets (dW, and dB for LayerNorm) in one launch: with 4 waves the 128
// dependent loads per thread at G = 512 left this pass latency-bound (~38 us at H 5120).
template <typename T>
__global__ __launch_bounds__(1024) void colsum_kernel(const float* __restrict__ part0, T* __restrict__ out0,
                                                      const float* __restrict__ part1, T* __restrict__ out1, int G,
                                                      int H) {
  __shared__ float red[16][64];
  const float* part = blockIdx.y ? part1 : part0;
  T* out = blockIdx.y ? out1 : out0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (c < H)
    for (int g = w; g < G; g += 16) s += part[(long)g * H + c];
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && c < H) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[i][lane];
    IO<T>::st(out, c, t);
  }
}

template <typename T, int MAXV>
static int launch_fwd(bool rms, const void* x, const void* res, const void* w, const void* b,
                      void* y, void* hout, float* mean, float* rstd, long N, int H, float eps,
                      hipStream_t st) {
  dim3 grid((N + 3) / 4), blk(256);
  const T *X = (const T*)x, *R = (const T*)res, *W = (const T*)w, *B = (const T*)b;
  T *Y = (T*)y, *HO = (T*)hout;
#define PA_NF(RMS_, RES_, BIAS_) \
  hipLaunchKernelGGL((norm_fwd_kernel<T, MAXV, RMS_, RES_, BIAS_>), grid, blk, 0, st, X, R, W, B, Y, HO, mean, rstd, N, H, eps)
  if (rms) {
    if (res) PA_NF(true, true, false); else PA_NF(true, false, false);
  } else {
    if (res) { if (b) PA_NF(false, true, true); else PA_NF(false, true, false); }
    else { if (b) PA_NF(false, false, true); else PA_NF(false, false, false); }
  }
#undef PA_NF
  PA_LAUNCH_CHECK();
}

// backward variant knobs for A/B runs (benchmarks/norm_bwd_ab.py): PA_NORM_BWD_G =
// block count cap, PA_NORM_BWD_WPR2 = 1 (default) splits rows of 2049-4096 over two waves too
static int env_int(const char* k, int def) {
  const char* v = getenv(k);
  return v && *v ? atoi(v) : def;
}

template <typename T, int MAXV, int WPR>
static void launch_bwd_k(bool rms, const T* DY, const T* Hh, const T* W, const float* mean, const float* rstd,
                         const T* DR, T* DX, float* dwp, float* dbp, long N, int H, long rpb, int G, size_t shm,
                         hipStream_t st) {
#define PA_NB(RMS_, DRES_) \
  hipLaunchKernelGGL((norm_bwd_kernel<T, MAXV, RMS_, DRES_, WPR>), dim3(G), dim3(256), shm, st, DY, Hh, W, mean, rstd, DR, DX, dwp, dbp, N, H, rpb)
  if (rms) { if (DR) PA_NB(true, true); else PA_NB(true, false); }
  else { if (DR) PA_NB(false, true); else PA_NB(false, false); }
#undef PA_NB
}

template <typename T, int MAXV>
static int launch_bwd(bool rms, const void* dy, const void* h, const void* w, const float* mean,
                      const float* rstd, const void* dres, void* dx, void* dw, void* db,
                      float* ws, long N, int H, hipStream_t st) {
  // (capped at 1024: callers size the workspace for 1024 partial rows)
  static const int gcap = env_int("PA_NORM_BWD_G", 512) < 1024 ? env_int("PA_NORM_BWD_G", 512) : 1024;
  static const int wpr2 = env_int("PA_NORM_BWD_WPR2", 1);  // default: profiles/r5_norm_bwd_ab.log (-6 %)
  // rows per block >= PA_NORM_BWD_RPB (default 16): [16384, 4096] 0.158 ms at 512 blocks,
  // [4096, 5120] LayerNorm 0.081 ms at 256 blocks vs 0.114 at 512 / 0.116 at 128
  // (profiles/r5_norm_bwd_rpb_ab.log)
  static const int rpb_min = env_int("PA_NORM_BWD_RPB", 16) > 0 ? env_int("PA_NORM_BWD_RPB", 16) : 4;
  long G0 = (N + rpb_min - 1) / rpb_min; int G = (int)(G0 < gcap ? G0 : gcap);
  if (G < 1) G = 1;
  long rpb = (N + G - 1) / G;
  G = (int)((N + rpb - 1) / rpb);
  float* dwp = ws;
  float* dbp = ws + (long)G * H;
  // (2H+8) fp32 of dynamic LDS: 65,568 B at H = 8192.  That is over the 64 KiB
  // per-workgroup limit of older CDNA parts, so this launcher is gfx950-only
  // (160 KB of LDS per CU, up to 160 KB per workgroup); the build targets gfx950
  // exclusively and the launch below fails loudly (hipError) rather than falling
  // back if it ever ran on a part with less LDS.
  size_t shm = (2 * H + 8) * sizeof(float);
  // rows wider than 4096 elements: two waves per row, 8 vectors per lane
  constexpr int WPR = MAXV > 8 ? 2 : 1;
  constexpr int MV = MAXV > 8 ? MAXV / 2 : MAXV;
  const T *DY = (const T*)dy, *Hh = (const T*)h, *W = (const T*)w, *DR = (const T*)dres;
  T* DX = (T*)dx;
  if (MAXV == 8 && wpr2)
    launch_bwd_k<T, 4, 2>(rms, DY, Hh, W, mean, rstd, DR, DX, dwp, dbp, N, H, rpb, G, shm, st);
  else
    launch_bwd_k<T, MV, WPR>(rms, DY, Hh, W, mean, rstd, DR, DX, dwp, dbp, N, H, rpb, G, shm, st);
  const bool two = !rms && db;
  hipLaunchKernelGGL((colsum_kernel<T>), dim3((H + 63) / 64, two ? 2 : 1), dim3(1024), 0, st, dwp, (T*)dw,
                     two ? dbp : dwp, two ? (T*)db : (T*)dw, G, H);
  PA_LAUNCH_CHECK();
}

}  // namespace pa

using namespace pa;

// dtype: 0 = fp32, 1 = bf16.  Returns hipError_t.  H must be a multiple of 8, <= 8192.
PA_EXPORT int pa_norm_fwd(int dtype, int rms, const void* x, const void* res, const void* w,
                          const void* b, void* y, void* hout, float* mean, float* rstd, long N,
                          int H, float eps, hipStream_t st) {
  const int nv = (H + 511) / 512;
#define PA_D(T)                                                                          \
  if (nv <= 1) return launch_fwd<T, 1>(rms, x, res, w, b, y, hout, mean, rstd, N, H, eps, st); \
  if (nv <= 2) return launch_fwd<T, 2>(rms, x, res, w, b, y, hout, mean, rstd, N, H, eps, st); \
  if (nv <= 4) return launch_fwd<T, 4>(rms, x, res, w, b, y, hout, mean, rstd, N, H, eps, st); \
  if (nv <= 8) return launch_fwd<T, 8>(rms, x, res, w, b, y, hout, mean, rstd, N, H, eps, st); \
  if (nv <= 16) return launch_fwd<T, 16>(rms, x, res, w, b, y, hout, mean, rstd, N, H, eps, st);
  if (dtype == 1) { PA_D(u16) } else { PA_D(float) }
#undef PA_D
  return (int)hipErrorInvalidValue;
}

// Workspace: ws must hold 2 * min(512, ceil(N/4)) * H floats.
PA_EXPORT int pa_norm_bwd(int dtype, int rms, const void* dy, const void* h, const void* w,
                          const float* mean, const float* rstd, const void* dres, void* dx,
                          void* dw, void* db, float* ws, long N, int H, hipStream_t st) {
  const int nv = (H + 511) / 512;
#define PA_D(T)                                                                                 \
  if (nv <= 1) return launch_bwd<T, 1>(rms, dy, h, w, mean, rstd, dres, dx, dw, db, ws, N, H, st); \
  if (nv <= 2) return launch_bwd<T, 2>(rms, dy, h, w, mean, rstd, dres, dx, dw, db, ws, N, H, st); \
  if (nv <= 4) return launch_bwd<T, 4>(rms, dy, h, w, mean, rstd, dres, dx, dw, db, ws, N, H, st); \
  if (nv <= 8) return launch_bwd<T, 8>(rms, dy, h, w, mean, rstd, dres, dx, dw, db, ws, N, H, st); \
  if (nv <= 16) return launch_bwd<T, 16>(rms, dy, h, w, mean, rstd, dres, dx, dw, db, ws, N, H, st);
  if (dtype == 1) { PA_D(u16) } else { PA_D(float) }
#undef PA_D
  return (int)hipErrorInvalidValue;
}
