// NHWC (channels-last) bf16 kernels around the implicit-GEMM convolution of
// gemm.hip: im2col for the weight gradient / tiny-C stems, BatchNorm forward and
// backward (fp32 statistics, optional fused ReLU), max pooling with a per-element
// argmax byte, and global average pooling.
//
// Reference: paddle/fluid/operators/math/im2col.cu (im2col / col2im for NCHW),
// batch_norm_op.cu.cc:170 (cuDNN BN), math/pooling.cu:25-189 (pool2d fwd/bwd).
// Layout here is NHWC throughout, so a 16-byte vector is 8 consecutive channels
// of one pixel; every kernel moves 16 B per lane (guide Guideline 13).
#include <cstdlib>

#include "common.h"

namespace pa {

// ---------------------------------------------------------------------- im2col
// col[(n, oy, ox)][(kh, kw, c)] (row pitch Kp >= KH*KW*C, padding columns zeroed)
template <bool VEC8>
__global__ void im2col_nhwc_kernel(const u16* __restrict__ x, u16* __restrict__ col, int N, int H, int W, int C,
                                   int OH, int OW, int KH, int KW, int sy, int sx, int py, int px, int dy, int dx,
                                   int Kp) {
  const int K = KH * KW * C;
  const int per_row = VEC8 ? Kp / 8 : Kp;
  const long total = (long)N * OH * OW * per_row;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const long row = idx / per_row;
    const int e = (int)(idx - row * per_row) * (VEC8 ? 8 : 1);
    const int ox = (int)(row % OW);
    const long t = row / OW;
    const int oy = (int)(t % OH), n = (int)(t / OH);
    u16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (e < K) {
      const int c = e % C, tap = e / C;
      const int kh = tap / KW, kw = tap - kh * KW;
      const int iy = oy * sy - py + kh * dy, ix = ox * sx - px + kw * dx;
      if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W) {
        const u16* src = x + (((long)n * H + iy) * W + ix) * C + c;
        if (VEC8) {
          v = *reinterpret_cast<const u16x8*>(src);
        } else {
          v[0] = *src;
        }
      }
    }
    if (VEC8) {
      *reinterpret_cast<u16x8*>(col + row * Kp + e) = v;
    } else {
      col[row * Kp + e] = v[0];
    }
  }
}

// ------------------------------------------------------------------ BatchNorm
// Rows = N*H*W pixels, C channels (C % 8 == 0).  Threads of a block are laid out
// (row_sub, chunk): chunk = 8 channels.  Per-thread fp32 sums are shifted by the
// first pixel's value (variance without catastrophic cancellation); blocks write
// partial sums, a finalize kernel combines them in fp64.
constexpr int BN_T = 256;

__host__ __device__ __forceinline__ void bn_layout(int C, int& chunks, int& rsub) {
  chunks = C / 8;
  rsub = chunks >= BN_T ? 1 : BN_T / chunks;
}

// partial[g][0][c] = sum(x - shift), partial[g][1][c] = sum((x - shift)^2)   (fwd)
// partial[g][0][c] = sum(dy'),       partial[g][1][c] = sum(dy' * (x - mean)) (bwd)
// with dy' = dy * (y > 0) when relu.
// Per-channel affine of the forward (sc = rstd * w, sf = b - mean * sc) for 8 channels:
// the ReLU mask of relu(BN(x)) is recomputed in backward as fmaf(x, sc, sf) > 0 --
// the same expression bn_apply_kernel evaluated -- instead of reading y back.
// 8 per-channel values from c0 (a multiple of 8): two 16-B loads for fp32 / one for bf16
// when the base is 16-B aligned (every framework allocation is), else element loads
__device__ __forceinline__ void chan8(const void* __restrict__ p, int bf16, int c0, float def, float (&o)[8]) {
  if (!p) {
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = def;
  } else if (((uintptr_t)p & 15) == 0) {
    if (bf16) {
      const u16x8 v = *reinterpret_cast<const u16x8*>((const u16*)p + c0);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = bf2f(v[j]);
    } else {
      const f32x4 a = *reinterpret_cast<const f32x4*>((const float*)p + c0);
      const f32x4 b = *reinterpret_cast<const f32x4*>((const float*)p + c0 + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        o[j] = a[j];
        o[4 + j] = b[j];
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = bf16 ? bf2f(((const u16*)p)[c0 + j]) : ((const float*)p)[c0 + j];
  }
}

__device__ __forceinline__ void bn_affine8(int ch, const float* __restrict__ mean, const float* __restrict__ rstd,
                                           const void* __restrict__ w, const void* __restrict__ b, int wdt,
                                           float (&sc)[8], float (&sf)[8]) {
  float ww[8], bb[8], mm[8], rr[8];
  chan8(w, wdt, ch * 8, 1.f, ww);
  chan8(b, wdt, ch * 8, 0.f, bb);
  chan8(mean, 0, ch * 8, 0.f, mm);
  chan8(rstd, 0, ch * 8, 0.f, rr);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = rr[j] * ww[j];
    sf[j] = bb[j] - mm[j] * sc[j];
  }
}

struct BnMask {  // relu-mask source of the backward kernels
  const u16* y;  // forward output (residual layers), or null: recompute from x
  const float* rstd;
  const void* w;
  const void* b;
  int wdt;
};

// UNR (backward only): two rows' loads in flight per thread before their sums
template <bool BWD, bool UNR = false>
__global__ __launch_bounds__(BN_T) void bn_reduce_kernel(const u16* __restrict__ x, const u16* __restrict__ dy,
                                                          BnMask mk, const float* __restrict__ mean,
                                                          float* __restrict__ partial, long rows, int C, int relu) {
  const u16* __restrict__ y = mk.y;
  int chunks, rsub;
  bn_layout(C, chunks, rsub);
  extern __shared__ __attribute__((aligned(16))) float red[];  // [rsub][C] x 2
  const int tid = threadIdx.x;
  const int chunk_per_iter = rsub == 1 ? BN_T : chunks;
  for (int cb = 0; cb < chunks; cb += chunk_per_iter) {
    const int ch = cb + tid % chunk_per_iter;
    const int rs = tid / chunk_per_iter;
    const bool active = ch < chunks && rs < rsub;
    float s0[8], s1[8], sh[8], msc[8], msf[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s0[j] = s1[j] = msc[j] = msf[j] = 0.f;
    if (active) {
      if (BWD) {
#pragma unroll
        for (int j = 0; j < 8; ++j) sh[j] = mean[ch * 8 + j];
        if (relu && !y) bn_affine8(ch, mean, mk.rstd, mk.w, mk.b, mk.wdt, msc, msf);
      } else {
        load8(x + ch * 8, sh);  // first pixel = shift
      }
      long r = (long)blockIdx.x * rsub + rs;
      const long step = (long)gridDim.x * rsub;
      if constexpr (BWD && UNR) {
        for (; r + step < rows; r += 2 * step) {
          u16x8 xa[2], ga[2], ya[2];
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const long o = (r + u * step) * C + ch * 8;
            xa[u] = *reinterpret_cast<const u16x8*>(x + o);
            ga[u] = *reinterpret_cast<const u16x8*>(dy + o);
            if (relu && y) ya[u] = *reinterpret_cast<const u16x8*>(y + o);
          }
#pragma unroll
          for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const float a = bf2f(xa[u][j]);
              float g = bf2f(ga[u][j]);
              if (relu && y) g = bf2f(ya[u][j]) > 0.f ? g : 0.f;
              else if (relu) g = fmaf(a, msc[j], msf[j]) > 0.f ? g : 0.f;
              s0[j] += g;
              s1[j] += g * (a - sh[j]);
            }
        }
      }
      for (; r < rows; r += step) {
        float a[8];
        load8(x + r * C + ch * 8, a);
        if (BWD) {
          float g[8];
          load8(dy + r * C + ch * 8, g);
          if (relu && y) {
            float yy[8];
            load8(y + r * C + ch * 8, yy);
#pragma unroll
            for (int j = 0; j < 8; ++j) g[j] = yy[j] > 0.f ? g[j] : 0.f;
          } else if (relu) {
#pragma unroll
            for (int j = 0; j < 8; ++j) g[j] = fmaf(a[j], msc[j], msf[j]) > 0.f ? g[j] : 0.f;
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            s0[j] += g[j];
            s1[j] += g[j] * (a[j] - sh[j]);
          }
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float d = a[j] - sh[j];
            s0[j] += d;
            s1[j] += d * d;
          }
        }
      }
    }
    __syncthreads();
    if (active) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        red[(rs * C + ch * 8 + j) * 2] = s0[j];
        red[(rs * C + ch * 8 + j) * 2 + 1] = s1[j];
      }
    }
    __syncthreads();
    // reduce over row_sub, one thread per channel
    for (int c = tid; c < C && c < (cb + chunk_per_iter) * 8; c += BN_T) {
      if (c < cb * 8) continue;
      float a0 = 0.f, a1 = 0.f;
      for (int r = 0; r < rsub; ++r) {
        a0 += red[(r * C + c) * 2];
        a1 += red[(r * C + c) * 2 + 1];
      }
      partial[((long)blockIdx.x * 2) * C + c] = a0;
      partial[((long)blockIdx.x * 2 + 1) * C + c] = a1;
    }
    __syncthreads();
  }
}

// forward finalize: mean, rstd (saved for backward), running stats update
// (running = m * running + (1 - m) * batch, unbiased variance), one thread per channel
// sum the G block partials of channel c: 1024 threads = 16 channels x 64 slices
// (64 independent fp64 chains per channel: latency-bound G of several thousand --
// the per-tile partials of the conv epilogue -- stays a few microseconds), tree
// over the slices in LDS
__device__ __forceinline__ bool bn_sum_partials(const float* __restrict__ partial, int G, int C, int& c, double& s0,
                                                double& s1) {
  __shared__ double red[2][64][16];
  const int cl = threadIdx.x & 15, sl = threadIdx.x >> 4;
  c = blockIdx.x * 16 + cl;
  double a0 = 0.0, a1 = 0.0;
  if (c < C)
    for (int g = sl; g < G; g += 64) {
      a0 += partial[((long)g * 2) * C + c];
      a1 += partial[((long)g * 2 + 1) * C + c];
    }
  red[0][sl][cl] = a0;
  red[1][sl][cl] = a1;
  __syncthreads();
  for (int h = 32; h > 0; h >>= 1) {
    if (sl < h) {
      red[0][sl][cl] += red[0][sl + h][cl];
      red[1][sl][cl] += red[1][sl + h][cl];
    }
    __syncthreads();
  }
  if (sl != 0 || c >= C) return false;
  s0 = red[0][0][cl];
  s1 = red[1][0][cl];
  return true;
}

__global__ __launch_bounds__(1024) void bn_finalize_fwd_kernel(const float* __restrict__ partial, int G,
                                                               const u16* __restrict__ x,
                                                               const float* __restrict__ shiftf, int C, long rows,
                                                               float eps, float momentum, float* __restrict__ mean_out,
                                                               float* __restrict__ rstd_out,
                                                               float* __restrict__ run_mean,
                                                               float* __restrict__ run_var, int update_running) {
  int c;
  double s0, s1;
  if (!bn_sum_partials(partial, G, C, c, s0, s1)) return;
  // the shift the partials were taken about: the first pixel (bn_reduce) or a given
  // per-channel value (conv epilogue statistics; null = 0)
  const double shift = x ? (double)bf2f(x[c]) : shiftf ? (double)shiftf[c] : 0.0;
  const double n = (double)rows;
  const double md = s0 / n;
  double var = s1 / n - md * md;
  if (var < 0.0) var = 0.0;
  const double mean = shift + md;
  mean_out[c] = (float)mean;
  rstd_out[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (update_running) {
    const double unbiased = rows > 1 ? var * n / (n - 1.0) : var;
    run_mean[c] = (float)(momentum * run_mean[c] + (1.0 - momentum) * mean);
    run_var[c] = (float)(momentum * run_var[c] + (1.0 - momentum) * unbiased);
  }
}

// y = (x - mean) * rstd * w + b (+ relu); w, b fp32 or bf16 per `wdt` (0 f32, 1 bf16).
// The launch makes the thread count a multiple of C/8, so a thread keeps one channel
// chunk for its whole grid-stride loop and folds (mean, rstd, w, b) into one FMA.
// U chunks in flight per thread; NT: non-temporal stores (the output is read by the next
// conv, not by this kernel: keep it out of the way of the streaming loads)
template <int U, bool NT>
__global__ void bn_apply_kernel(const u16* __restrict__ x, u16* __restrict__ y, const float* __restrict__ mean,
                                const float* __restrict__ rstd, const void* __restrict__ w, const void* __restrict__ b,
                                int wdt, long rows, int C, int relu, const u16* __restrict__ res) {
  const int chunks = C / 8;
  const long total = rows * chunks;
  const long stride = (long)gridDim.x * blockDim.x;  // multiple of chunks
  const long i0 = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const int ch = (int)(i0 % chunks);
  float sc[8], sf[8];
  bn_affine8(ch, mean, rstd, w, b, wdt, sc, sf);
  // U chunks in flight per thread: every load of a group is issued before the first
  // store (y may alias nothing the loads read, but the compiler cannot know that)
  long i = i0;
  for (; i + (U - 1) * stride < total; i += U * stride) {
    u16x8 xa[U], ra[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      xa[u] = *reinterpret_cast<const u16x8*>(x + (i + u * stride) * 8);
      if (res) ra[u] = *reinterpret_cast<const u16x8*>(res + (i + u * stride) * 8);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float a[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = fmaf(bf2f(xa[u][j]), sc[j], sf[j]) + (res ? bf2f(ra[u][j]) : 0.f);
        a[j] = relu ? fmaxf(v, 0.f) : v;
      }
      if constexpr (NT) {
        u16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = f2bf(a[j]);
        __builtin_nontemporal_store(o, reinterpret_cast<u16x8*>(y + (i + u * stride) * 8));
      } else {
        store8(y + (i + u * stride) * 8, a);
      }
    }
  }
  for (; i < total; i += stride) {
    float a[8], r[8];
    load8(x + i * 8, a);
    if (res) {
      load8(res + i * 8, r);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = fmaf(a[j], sc[j], sf[j]) + r[j];
      a[j] = relu ? fmaxf(v, 0.f) : v;
    }
    store8(y + i * 8, a);
  }
}

// A/B knob PA_BN_RED_UNR: 1 = two rows in flight in the backward statistics pass
static int bn_red_unroll() {
  static const int v = [] {
    const char* e = getenv("PA_BN_RED_UNR");
    return e && *e ? atoi(e) : 0;
  }();
  return v;
}

// A/B knob PA_BN_DX: 1 = 4 chunks in flight + non-temporal stores, 0 (default) = one
// at a time -- the unrolled form measured 2 % slower on ResNet-50 (profiles/r5_bn_ew_ab.md)
static int bn_dx_unroll() {
  static const int v = [] {
    const char* e = getenv("PA_BN_DX");
    return e && *e ? atoi(e) : 0;
  }();
  return v;
}

// A/B knob PA_BN_APPLY: 0 = 4 chunks in flight, 1 = 8, 2 = 4 + non-temporal stores,
// 3 = 8 + non-temporal stores
static int bn_apply_variant() {
  static const int v = [] {
    const char* e = getenv("PA_BN_APPLY");
    return e && *e ? atoi(e) : 2;  // default: 4 in flight + non-temporal stores (benchmarks/bn_apply_ab.py)
  }();
  return v;
}

static void launch_bn_apply(dim3 g, dim3 blk, hipStream_t st, const u16* x, u16* y, const float* mean,
                            const float* rstd, const void* w, const void* b, int wdt, long rows, int C, int relu,
                            const u16* res) {
  switch (bn_apply_variant()) {
    case 1: hipLaunchKernelGGL((bn_apply_kernel<8, false>), g, blk, 0, st, x, y, mean, rstd, w, b, wdt, rows, C, relu, res); break;
    case 2: hipLaunchKernelGGL((bn_apply_kernel<4, true>), g, blk, 0, st, x, y, mean, rstd, w, b, wdt, rows, C, relu, res); break;
    case 3: hipLaunchKernelGGL((bn_apply_kernel<8, true>), g, blk, 0, st, x, y, mean, rstd, w, b, wdt, rows, C, relu, res); break;
    default: hipLaunchKernelGGL((bn_apply_kernel<4, false>), g, blk, 0, st, x, y, mean, rstd, w, b, wdt, rows, C, relu, res);
  }
}

// backward finalize: dw = rstd * sum(dy' (x - mean)), db = sum(dy'); also writes the
// per-channel coefficients k1 = w*rstd, k2 = db/M, k3 = w*rstd^3*sum(dy'(x-mean))/M
__global__ __launch_bounds__(1024) void bn_finalize_bwd_kernel(const float* __restrict__ partial, int G, int C,
                                                               long rows, const float* __restrict__ rstd,
                                                               const void* __restrict__ w, int wdt,
                                                               float* __restrict__ dw, float* __restrict__ db,
                                                               float* __restrict__ coef) {
  int c;
  double s0, s1;
  if (!bn_sum_partials(partial, G, C, c, s0, s1)) return;
  const double r = rstd[c];
  const double ww = w ? (wdt ? bf2f(((const u16*)w)[c]) : ((const float*)w)[c]) : 1.0;
  dw[c] = (float)(s1 * r);
  db[c] = (float)s0;
  coef[c] = (float)(ww * r);
  coef[C + c] = (float)(s0 / rows);
  coef[2 * C + c] = (float)(ww * r * r * r * s1 / rows);
}

// dx = k1 * dy' - k1 * k2 - k3 * (x - mean)   (fixed channel chunk per thread, as bn_apply)
__global__ void bn_dx_kernel(const u16* __restrict__ x, const u16* __restrict__ dy, BnMask mk,
                             const float* __restrict__ mean, const float* __restrict__ coef, u16* __restrict__ dx,
                             long rows, int C, int relu, u16* __restrict__ dres, int unroll) {
  const u16* __restrict__ y = mk.y;
  const int chunks = C / 8;
  const long total = rows * chunks;
  const long stride = (long)gridDim.x * blockDim.x;
  const long i0 = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const int ch = (int)(i0 % chunks);
  float k1[8], k0[8], k3[8], k2[8], mm[8];
  chan8(coef, 0, ch * 8, 0.f, k1);
  chan8(coef + C, 0, ch * 8, 0.f, k2);
  chan8(coef + 2 * C, 0, ch * 8, 0.f, k3);
  chan8(mean, 0, ch * 8, 0.f, mm);
#pragma unroll
  for (int j = 0; j < 8; ++j) k0[j] = -k1[j] * k2[j] + k3[j] * mm[j];  // constant part
  float msc[8], msf[8];
  if (relu && !y) bn_affine8(ch, mean, mk.rstd, mk.w, mk.b, mk.wdt, msc, msf);
  long i = i0;
  // 4 chunks in flight (all loads of a group before its stores), non-temporal stores
  constexpr int U = 4;
  for (; unroll && i + (U - 1) * stride < total; i += U * stride) {
    u16x8 xa[U], ga[U], ya[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      xa[u] = *reinterpret_cast<const u16x8*>(x + (i + u * stride) * 8);
      ga[u] = *reinterpret_cast<const u16x8*>(dy + (i + u * stride) * 8);
      if (relu && y) ya[u] = *reinterpret_cast<const u16x8*>(y + (i + u * stride) * 8);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float a[8], g[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        a[j] = bf2f(xa[u][j]);
        g[j] = bf2f(ga[u][j]);
        if (relu && y) g[j] = bf2f(ya[u][j]) > 0.f ? g[j] : 0.f;
        else if (relu) g[j] = fmaf(a[j], msc[j], msf[j]) > 0.f ? g[j] : 0.f;
      }
      const long o = (i + u * stride) * 8;
      if (dres) {
        u16x8 r;
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = f2bf(g[j]);
        __builtin_nontemporal_store(r, reinterpret_cast<u16x8*>(dres + o));
      }
      u16x8 d;
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] = f2bf(fmaf(k1[j], g[j], fmaf(-k3[j], a[j], k0[j])));
      __builtin_nontemporal_store(d, reinterpret_cast<u16x8*>(dx + o));
    }
  }
  for (; i < total; i += stride) {
    float a[8], g[8];
    load8(x + i * 8, a);
    load8(dy + i * 8, g);
    if (relu && y) {
      float yy[8];
      load8(y + i * 8, yy);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = yy[j] > 0.f ? g[j] : 0.f;
    } else if (relu) {
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = fmaf(a[j], msc[j], msf[j]) > 0.f ? g[j] : 0.f;
    }
    if (dres) store8(dres + i * 8, g);  // gradient of the residual input of relu(bn(x) + res)
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = fmaf(k1[j], g[j], fmaf(-k3[j], a[j], k0[j]));
    store8(dx + i * 8, a);
  }
}

// ------------------------------------------------------------------- max pool
// out / idx: [N, OH, OW, C]; idx = window position (kh*KW + kw) of the max (0xff:
// the window held no valid pixel)
__global__ void maxpool_fwd_kernel(const u16* __restrict__ x, u16* __restrict__ y, unsigned char* __restrict__ idx,
                                   int N, int H, int W, int C, int OH, int OW, int KH, int KW, int sy, int sx, int py,
                                   int px) {
  const int chunks = C / 8;
  const long total = (long)N * OH * OW * chunks;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int ch = (int)(i % chunks);
    long t = i / chunks;
    const int ox = (int)(t % OW);
    t /= OW;
    const int oy = (int)(t % OH), n = (int)(t / OH);
    float best[8];
    unsigned char bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      best[j] = -INFINITY;
      bi[j] = 0xff;
    }
    for (int kh = 0; kh < KH; ++kh) {
      const int iy = oy * sy - py + kh;
      if ((unsigned)iy >= (unsigned)H) continue;
      for (int kw = 0; kw < KW; ++kw) {
        const int ix = ox * sx - px + kw;
        if ((unsigned)ix >= (unsigned)W) continue;
        float a[8];
        load8(x + (((long)n * H + iy) * W + ix) * C + ch * 8, a);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (a[j] > best[j] || bi[j] == 0xff) {
            best[j] = a[j];
            bi[j] = (unsigned char)(kh * KW + kw);
          }
      }
    }
    store8(y + i * 8, best);
    uint2 packed;
    packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((unsigned)bi[3] << 24);
    packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((unsigned)bi[7] << 24);
    *reinterpret_cast<uint2*>(idx + i * 8) = packed;
  }
}

// gather form: each input pixel sums the dy of the outputs whose argmax it is
__global__ void maxpool_bwd_kernel(const u16* __restrict__ dy, const unsigned char* __restrict__ idx,
                                   u16* __restrict__ dx, int N, int H, int W, int C, int OH, int OW, int KH, int KW,
                                   int sy, int sx, int py, int px) {
  const int chunks = C / 8;
  const long total = (long)N * H * W * chunks;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int ch = (int)(i % chunks);
    long t = i / chunks;
    const int ix = (int)(t % W);
    t /= W;
    const int iy = (int)(t % H), n = (int)(t / H);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // outputs with oy*sy - py <= iy <= oy*sy - py + KH - 1
    const int oy_lo = max(0, (iy + py - KH + sy) / sy), oy_hi = min(OH - 1, (iy + py) / sy);
    const int ox_lo = max(0, (ix + px - KW + sx) / sx), ox_hi = min(OW - 1, (ix + px) / sx);
    for (int oy = oy_lo; oy <= oy_hi; ++oy) {
      const int kh = iy - (oy * sy - py);
      if (kh < 0 || kh >= KH) continue;
      for (int ox = ox_lo; ox <= ox_hi; ++ox) {
        const int kw = ix - (ox * sx - px);
        if (kw < 0 || kw >= KW) continue;
        const long o = (((long)n * OH + oy) * OW + ox) * C + ch * 8;
        const uint2 pk = *reinterpret_cast<const uint2*>(idx + o);
        float g[8];
        load8(dy + o, g);
        const unsigned want = (unsigned)(kh * KW + kw);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const unsigned b = ((j < 4 ? pk.x : pk.y) >> (8 * (j & 3))) & 0xff;
          if (b == want) acc[j] += g[j];
        }
      }
    }
    store8(dx + i * 8, acc);
  }
}

// ------------------------------------------------------------ global avg pool
__global__ void gap_fwd_kernel(const u16* __restrict__ x, u16* __restrict__ y, int N, int HW, int C) {
  const int chunks = C / 8;
  const long total = (long)N * chunks;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int ch = (int)(i % chunks), n = (int)(i / chunks);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int p = 0; p < HW; ++p) {
      float a[8];
      load8(x + ((long)n * HW + p) * C + ch * 8, a);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += a[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] *= 1.f / HW;
    store8(y + i * 8, acc);
  }
}

__global__ void gap_bwd_kernel(const u16* __restrict__ dy, u16* __restrict__ dx, int N, int HW, int C) {
  const int chunks = C / 8;
  const long total = (long)N * HW * chunks;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int ch = (int)(i % chunks);
    const int n = (int)(i / chunks / HW);
    float g[8];
    load8(dy + ((long)n * C) + ch * 8, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] *= 1.f / HW;
    store8(dx + i * 8, g);
  }
}

// Running-statistics update for running mean / var kept in another dtype than the
// fp32 the finalize kernel updates (a bf16-cast model): var recovered from rstd, one
// launch for all channels instead of a chain of elementwise ops per statistic.
template <typename T>
__global__ void bn_running_kernel(T* __restrict__ rm, T* __restrict__ rv, const float* __restrict__ mean,
                                  const float* __restrict__ rstd, int C, long rows, float eps, float momentum) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double r = rstd[c];
  const double var = 1.0 / (r * r) - (double)eps;
  const double n = (double)rows;
  const double unb = rows > 1 ? var * n / (n - 1.0) : var;
  IO<T>::st(rm, c, (float)(momentum * (double)IO<T>::ld(rm, c) + (1.0 - momentum) * (double)mean[c]));
  IO<T>::st(rv, c, (float)(momentum * (double)IO<T>::ld(rv, c) + (1.0 - momentum) * unb));
}

}  // namespace pa

using namespace pa;

// dt: 0 fp32, 1 bf16 running statistics
PA_EXPORT int pa_bn_running_update(int dt, void* rm, void* rv, const float* mean, const float* rstd, int C, long rows,
                                   float eps, float momentum, hipStream_t st) {
  if (C <= 0) return 0;
  const int grid = (C + 255) / 256;
  if (dt == 1)
    hipLaunchKernelGGL(bn_running_kernel<u16>, dim3(grid), dim3(256), 0, st, (u16*)rm, (u16*)rv, mean, rstd, C, rows,
                       eps, momentum);
  else
    hipLaunchKernelGGL(bn_running_kernel<float>, dim3(grid), dim3(256), 0, st, (float*)rm, (float*)rv, mean, rstd, C,
                       rows, eps, momentum);
  PA_LAUNCH_CHECK();
}

// C < 8 (image stems): compile-time C; a thread writes 8 consecutive columns of
// one row (one 16-byte store) and walks (kh, kw, c) incrementally, no divisions.
template <int CC>
__global__ void im2col_smallc_kernel(const u16* __restrict__ x, u16* __restrict__ col, int N, int H, int W, int OH,
                                     int OW, int KH, int KW, int sy, int sx, int py, int px, int dy, int dx, int Kp) {
  const int K = KH * KW * CC;
  const int per_row = Kp / 8;
  const long total = (long)N * OH * OW * per_row;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const long row = idx / per_row;
    const int e0 = (int)(idx - row * per_row) * 8;
    const int ox = (int)(row % OW);
    const long t = row / OW;
    const int oy = (int)(t % OH), n = (int)(t / OH);
    int tap = e0 / CC, c = e0 - tap * CC;
    int kh = tap / KW, kw = tap - kh * KW;
    const u16* img = x + (long)n * H * W * CC;
    u16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int iy = oy * sy - py + kh * dy, ix = ox * sx - px + kw * dx;
      const bool ok = e0 + j < K && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
      v[j] = ok ? img[((long)iy * W + ix) * CC + c] : (u16)0;
      if (++c == CC) {
        c = 0;
        if (++kw == KW) {
          kw = 0;
          ++kh;
        }
      }
    }
    *reinterpret_cast<u16x8*>(col + row * Kp + e0) = v;
  }
}

PA_EXPORT int pa_im2col_nhwc(const void* x, void* col, int N, int H, int W, int C, int OH, int OW, int KH, int KW,
                             int sy, int sx, int py, int px, int dy, int dx, int Kp, hipStream_t st) {
  const long rows = (long)N * OH * OW;
  const bool vec = C % 8 == 0 && Kp % 8 == 0;
  const long work = rows * (vec ? Kp / 8 : Kp);
  const int grid = stream_grid(work, 256) * 4;
  if (!vec && C <= 4 && Kp % 8 == 0) {
    const long work8 = rows * (Kp / 8);
    const dim3 g(stream_grid(work8, 256) * 4), b(256);
#define PA_SMALLC(CC)                                                                                              \
  hipLaunchKernelGGL(im2col_smallc_kernel<CC>, g, b, 0, st, (const u16*)x, (u16*)col, N, H, W, OH, OW, KH, KW, sy, \
                     sx, py, px, dy, dx, Kp)
    if (C == 1) PA_SMALLC(1);
    else if (C == 2) PA_SMALLC(2);
    else if (C == 3) PA_SMALLC(3);
    else PA_SMALLC(4);
#undef PA_SMALLC
    PA_LAUNCH_CHECK();
  }
  if (vec)
    hipLaunchKernelGGL(im2col_nhwc_kernel<true>, dim3(grid), dim3(256), 0, st, (const u16*)x, (u16*)col, N, H, W, C,
                       OH, OW, KH, KW, sy, sx, py, px, dy, dx, Kp);
  else
    hipLaunchKernelGGL(im2col_nhwc_kernel<false>, dim3(grid), dim3(256), 0, st, (const u16*)x, (u16*)col, N, H, W,
                       C, OH, OW, KH, KW, sy, sx, py, px, dy, dx, Kp);
  PA_LAUNCH_CHECK();
}

// elementwise BN launch: block size a multiple of C/8 (or C/8 a multiple of the block)
// and a thread count that is a multiple of C/8, so each thread keeps one chunk
static void bn_ew_launch(long rows, int C, int& grid, int& block) {
  const int chunks = C / 8;
  block = chunks >= 256 ? 256 : 256 / chunks * chunks;
  long threads_needed = rows * chunks;
  long g = (threads_needed + block - 1) / block;
  // block cap (PA_BN_EW_CAP, default 2048): each thread loads its 8 channels'
  // parameters once, so fewer, longer-running threads amortise that prologue -- 8192
  // measured 11 % slower end to end on ResNet-50 (profiles/r5_bn_ew_ab.md)
  static const long cap = [] {
    const char* e = getenv("PA_BN_EW_CAP");
    return e && *e ? atol(e) : 2048L;
  }();
  if (g > cap) g = cap;
  // total threads must be a multiple of chunks
  while (((long)g * block) % chunks) ++g;
  grid = (int)g;
}

// number of reduce blocks (partials buffer = G * 2 * C floats)
PA_EXPORT int pa_bn_blocks(long rows, int C) {
  int chunks, rsub;
  bn_layout(C, chunks, rsub);
  // >= 16 rows per thread, up to 4 blocks per CU: small (late-stage) layers keep
  // every CU streaming instead of a few hundred blocks
  long g = (rows + rsub * 16 - 1) / (rsub * 16);
  if (g > 1024) g = 1024;
  if (g < 1) g = 1;
  return (int)g;
}

static size_t bn_shm(int C) {
  int chunks, rsub;
  bn_layout(C, chunks, rsub);
  return (size_t)rsub * C * 2 * sizeof(float);
}

// training forward: y = BN(x) (+ relu); writes mean / rstd for backward and updates
// the running statistics.  part: >= pa_bn_blocks * 2 * C floats of workspace.
// res (optional): y = relu(BN(x) + res) -- the residual add of a bottleneck block
PA_EXPORT int pa_bn_fwd_train(const void* x, void* y, const void* w, const void* b, int wdt, float* run_mean,
                              float* run_var, float* mean, float* rstd, float* part, long rows, int C, float eps,
                              float momentum, int relu, const void* res, hipStream_t st) {
  if (C % 8) return -1;
  const int G = pa_bn_blocks(rows, C);
  hipLaunchKernelGGL(bn_reduce_kernel<false>, dim3(G), dim3(BN_T), bn_shm(C), st, (const u16*)x, nullptr,
                     BnMask{nullptr, nullptr, nullptr, nullptr, 0}, nullptr, part, rows, C, 0);
  hipLaunchKernelGGL(bn_finalize_fwd_kernel, dim3((C + 15) / 16), dim3(1024), 0, st, part, G, (const u16*)x,
                     (const float*)nullptr, C, rows, eps, momentum, mean, rstd, run_mean, run_var, run_mean != nullptr);
  int eg, eb;
  bn_ew_launch(rows, C, eg, eb);
  launch_bn_apply(dim3(eg), dim3(eb), st, (const u16*)x, (u16*)y, mean, rstd, w, b, wdt, rows,
                     C, relu, (const u16*)res);
  PA_LAUNCH_CHECK();
}

// training forward from statistics the producing convolution already emitted
// (pa_conv_sn's epilogue: part[G][2][C] about `shift`): no statistics pass over x
PA_EXPORT int pa_bn_fwd_stats(const float* part, int G, const float* shift, const void* x, void* y, const void* w,
                              const void* b, int wdt, float* run_mean, float* run_var, float* mean, float* rstd,
                              long rows, int C, float eps, float momentum, int relu, const void* res, hipStream_t st) {
  if (C % 8) return -1;
  hipLaunchKernelGGL(bn_finalize_fwd_kernel, dim3((C + 15) / 16), dim3(1024), 0, st, part, G, (const u16*)nullptr,
                     shift, C, rows, eps, momentum, mean, rstd, run_mean, run_var, run_mean != nullptr);
  int eg, eb;
  bn_ew_launch(rows, C, eg, eb);
  launch_bn_apply(dim3(eg), dim3(eb), st, (const u16*)x, (u16*)y, mean, rstd, w, b, wdt, rows,
                     C, relu, (const u16*)res);
  PA_LAUNCH_CHECK();
}

// inference forward with given statistics (mean / rstd precomputed by the caller)
PA_EXPORT int pa_bn_apply(const void* x, void* y, const float* mean, const float* rstd, const void* w, const void* b,
                          int wdt, long rows, int C, int relu, hipStream_t st) {
  if (C % 8) return -1;
  int eg, eb;
  bn_ew_launch(rows, C, eg, eb);
  launch_bn_apply(dim3(eg), dim3(eb), st, (const u16*)x, (u16*)y, mean, rstd, w, b, wdt, rows,
                     C, relu, (const u16*)nullptr);
  PA_LAUNCH_CHECK();
}

// backward: dx, dw, db (fp32) from x, dy, the saved mean / rstd and (relu) the output y.
// coef: 3*C floats of workspace, part: pa_bn_blocks * 2 * C floats.
// dres (optional): also write the residual gradient (= dY masked by the ReLU)
// y == null with relu: the ReLU mask is recomputed from x and (mean, rstd, w, b)
// (non-residual layers need not keep their output for backward)
PA_EXPORT int pa_bn_bwd2(const void* x, const void* dy, const void* y, const float* mean, const float* rstd,
                         const void* w, const void* b, int wdt, void* dx, float* dw, float* db, float* coef,
                         float* part, long rows, int C, int relu, void* dres, hipStream_t st) {
  if (C % 8) return -1;
  const int G = pa_bn_blocks(rows, C);
  const BnMask mk{(const u16*)y, rstd, w, b, wdt};
if (bn_red_unroll())
      hipLaunchKernelGGL((bn_reduce_kernel<true, true>), dim3(G), dim3(BN_T), bn_shm(C), st, (const u16*)x, (const u16*)dy,
                     mk, mean, part, rows, C, relu);
  else
      hipLaunchKernelGGL(bn_reduce_kernel<true>, dim3(G), dim3(BN_T), bn_shm(C), st, (const u16*)x, (const u16*)dy,
                     mk, mean, part, rows, C, relu);
  hipLaunchKernelGGL(bn_finalize_bwd_kernel, dim3((C + 15) / 16), dim3(1024), 0, st, part, G, C, rows, rstd, w, wdt,
                     dw, db, coef);
  int eg, eb;
  bn_ew_launch(rows, C, eg, eb);
  hipLaunchKernelGGL(bn_dx_kernel, dim3(eg), dim3(eb), 0, st, (const u16*)x, (const u16*)dy, mk, mean, coef,
                     (u16*)dx, rows, C, relu, (u16*)dres, bn_dx_unroll());
  PA_LAUNCH_CHECK();
}

// pa_bn_bwd2 with the reduction already done: part [G][2][C] of sum dy', sum dy' (x - mean)
// emitted by the epilogue of the convolution that produced dy (pa_conv_sn_bnbwd /
// pa_conv_gemm_bnbwd), so only the finalize and the dx pass run.
PA_EXPORT int pa_bn_bwd_part(const float* part, int G, const void* x, const void* dy, const void* y,
                             const float* mean, const float* rstd, const void* w, const void* b, int wdt, void* dx,
                             float* dw, float* db, float* coef, long rows, int C, int relu, void* dres,
                             hipStream_t st) {
  if (C % 8 || G <= 0) return -1;
  const BnMask mk{(const u16*)y, rstd, w, b, wdt};
  hipLaunchKernelGGL(bn_finalize_bwd_kernel, dim3((C + 15) / 16), dim3(1024), 0, st, part, G, C, rows, rstd, w, wdt,
                     dw, db, coef);
  int eg, eb;
  bn_ew_launch(rows, C, eg, eb);
  hipLaunchKernelGGL(bn_dx_kernel, dim3(eg), dim3(eb), 0, st, (const u16*)x, (const u16*)dy, mk, mean, coef,
                     (u16*)dx, rows, C, relu, (u16*)dres, bn_dx_unroll());
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_bn_bwd(const void* x, const void* dy, const void* y, const float* mean, const float* rstd,
                        const void* w, int wdt, void* dx, float* dw, float* db, float* coef, float* part, long rows,
                        int C, int relu, void* dres, hipStream_t st) {
  if (relu && !y) return -1;  // the mask source: y, or pa_bn_bwd2 with the bias
  return pa_bn_bwd2(x, dy, y, mean, rstd, w, nullptr, wdt, dx, dw, db, coef, part, rows, C, relu, dres, st);
}

PA_EXPORT int pa_maxpool_nhwc_fwd(const void* x, void* y, void* idx, int N, int H, int W, int C, int OH, int OW,
                                  int KH, int KW, int sy, int sx, int py, int px, hipStream_t st) {
  if (C % 8 || KH * KW > 255) return -1;
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(stream_grid((long)N * OH * OW * (C / 8), 256) * 4), dim3(256), 0, st,
                     (const u16*)x, (u16*)y, (unsigned char*)idx, N, H, W, C, OH, OW, KH, KW, sy, sx, py, px);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_maxpool_nhwc_bwd(const void* dy, const void* idx, void* dx, int N, int H, int W, int C, int OH,
                                  int OW, int KH, int KW, int sy, int sx, int py, int px, hipStream_t st) {
  if (C % 8) return -1;
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(stream_grid((long)N * H * W * (C / 8), 256) * 4), dim3(256), 0, st,
                     (const u16*)dy, (const unsigned char*)idx, (u16*)dx, N, H, W, C, OH, OW, KH, KW, sy, sx, py,
                     px);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_gap_nhwc_fwd(const void* x, void* y, int N, int HW, int C, hipStream_t st) {
  if (C % 8) return -1;
  hipLaunchKernelGGL(gap_fwd_kernel, dim3(stream_grid((long)N * (C / 8), 256)), dim3(256), 0, st, (const u16*)x,
                     (u16*)y, N, HW, C);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_gap_nhwc_bwd(const void* dy, void* dx, int N, int HW, int C, hipStream_t st) {
  if (C % 8) return -1;
  hipLaunchKernelGGL(gap_bwd_kernel, dim3(stream_grid((long)N * HW * (C / 8), 256) * 4), dim3(256), 0, st,
                     (const u16*)dy, (u16*)dx, N, HW, C);
  PA_LAUNCH_CHECK();
}

// out[i] (+)= sum_s part[s * n + i]   (split-K partials, fp32, n % 4 == 0)
__global__ void splitk_reduce_kernel(const float* __restrict__ part, float* __restrict__ out, long n4, int S,
                                     int accumulate) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    f32x4 acc = accumulate ? reinterpret_cast<const f32x4*>(out)[i] : f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < S; ++s) acc += reinterpret_cast<const f32x4*>(part + (long)s * n4 * 4)[i];
    reinterpret_cast<f32x4*>(out)[i] = acc;
  }
}

PA_EXPORT int pa_splitk_reduce(const float* part, float* out, long n, int S, int accumulate, hipStream_t st) {
  if (n % 4) return -1;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(stream_grid(n / 4, 256)), dim3(256), 0, st, part, out, n / 4, S,
                     accumulate);
  PA_LAUNCH_CHECK();
}
