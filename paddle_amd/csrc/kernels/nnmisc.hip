// Small Fluid NN kernels on gfx950: cos_sim (row-wise, optional broadcast Y row),
// bilinear / nearest interpolation (align_corners both ways), conv_shift (NTM
// circular convolution) and lstm_unit, each with its backward.  fp32 or bf16 data
// (T = float | u16), fp32 math, wave64.
//
// Reference behaviour: operators/cos_sim_op.h + math/cos_sim_functor.cu,
// bilinear_interp_op.cu (KeBilinearInterpFw / Bw), conv_shift_op.cu,
// lstm_unit_op.cu (gate order i, f, o, g; forget_bias inside the sigmoid).
#include "common.h"

namespace pa {
namespace {

inline int grid_for(long n, int block = 256) {
  long g = (n + block - 1) / block;
  return (int)(g < 1 ? 1 : (g > 16384 ? 16384 : g));
}

#define GRID_STRIDE(i, n) for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < (n); i += (long)gridDim.x * blockDim.x)

__device__ __forceinline__ float sigm(float v) { return 1.f / (1.f + __expf(-v)); }

// ---------------------------------------------------------------- cos_sim
// one wave per row; y_rows == 1 broadcasts the single Y row
template <typename T>
__global__ __launch_bounds__(256) void cos_sim_fwd_kernel(const T* __restrict__ x, const T* __restrict__ y,
                                                          T* __restrict__ out, float* __restrict__ xn,
                                                          float* __restrict__ yn, long rows, int D, int y_rows) {
  const int lane = threadIdx.x & 63;
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const T* xr = x + r * D;
  const T* yr = y + (y_rows == 1 ? 0 : r) * D;
  float xy = 0.f, xx = 0.f, yy = 0.f;
  for (int d = lane; d < D; d += 64) {
    const float a = IO<T>::ld(xr, d), b = IO<T>::ld(yr, d);
    xy += a * b;
    xx += a * a;
    yy += b * b;
  }
  xy = wave_sum(xy);
  xx = wave_sum(xx);
  yy = wave_sum(yy);
  if (lane == 0) {
    const float nx = sqrtf(xx), ny = sqrtf(yy);
    IO<T>::st(out, r, xy / (nx * ny));
    xn[r] = nx;
    yn[r] = ny;
  }
}

// dx = g (y / (|x||y|) - out x / |x|^2); dy likewise (fp32 atomics into dy when Y
// is one broadcast row)
template <typename T>
__global__ __launch_bounds__(256) void cos_sim_bwd_kernel(const T* __restrict__ x, const T* __restrict__ y,
                                                          const T* __restrict__ out, const float* __restrict__ xn,
                                                          const float* __restrict__ yn, const T* __restrict__ dout,
                                                          T* __restrict__ dx, float* __restrict__ dy, long rows, int D,
                                                          int y_rows) {
  const int lane = threadIdx.x & 63;
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const T* xr = x + r * D;
  const T* yr = y + (y_rows == 1 ? 0 : r) * D;
  const float nx = xn[r], ny = yn[r], o = IO<T>::ld(out, r), g = IO<T>::ld(dout, r);
  const float inv = 1.f / (nx * ny), ox = o / (nx * nx), oy = o / (ny * ny);
  for (int d = lane; d < D; d += 64) {
    const float a = IO<T>::ld(xr, d), b = IO<T>::ld(yr, d);
    if (dx) IO<T>::st(dx, r * D + d, g * (b * inv - a * ox));
    if (dy) {
      const float v = g * (a * inv - b * oy);
      if (y_rows == 1) atomicAdd(dy + d, v);
      else dy[r * D + d] = v;
    }
  }
}

// ---------------------------------------------------------------- interpolation (NCHW)
// src coordinate of destination o: align_corners -> o * (in - 1) / (out - 1);
// otherwise half-pixel (o + 0.5) * in / out - 0.5 clamped at 0 (F.interpolate)
__device__ __forceinline__ float src_coord(int o, int in, int outn, int align) {
  if (align) return outn > 1 ? (float)o * (float)(in - 1) / (float)(outn - 1) : 0.f;
  const float s = ((float)o + 0.5f) * (float)in / (float)outn - 0.5f;
  return s < 0.f ? 0.f : s;
}

template <typename T>
__global__ void interp_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, long NC, int H, int W, int OH, int OW,
                                  int nearest, int align) {
  GRID_STRIDE(i, NC * OH * OW) {
    const int ow = (int)(i % OW), oh = (int)((i / OW) % OH);
    const long nc = i / ((long)OH * OW);
    const T* p = x + nc * H * W;
    if (nearest) {
      const int sh = min((int)floorf((float)oh * (float)H / (float)OH), H - 1);
      const int sw = min((int)floorf((float)ow * (float)W / (float)OW), W - 1);
      IO<T>::st(y, i, IO<T>::ld(p, (long)sh * W + sw));
      continue;
    }
    const float fh = src_coord(oh, H, OH, align), fw = src_coord(ow, W, OW, align);
    const int h0 = min((int)fh, H - 1), w0 = min((int)fw, W - 1);
    const int h1 = min(h0 + 1, H - 1), w1 = min(w0 + 1, W - 1);
    const float lh = fh - h0, lw = fw - w0;
    const float v = (1.f - lh) * ((1.f - lw) * IO<T>::ld(p, (long)h0 * W + w0) + lw * IO<T>::ld(p, (long)h0 * W + w1)) +
                    lh * ((1.f - lw) * IO<T>::ld(p, (long)h1 * W + w0) + lw * IO<T>::ld(p, (long)h1 * W + w1));
    IO<T>::st(y, i, v);
  }
}

// dx (fp32, zeroed) += weights * dy (float atomics: several outputs share inputs)
template <typename T>
__global__ void interp_bwd_kernel(const T* __restrict__ dy, float* __restrict__ dx, long NC, int H, int W, int OH,
                                  int OW, int nearest, int align) {
  GRID_STRIDE(i, NC * OH * OW) {
    const int ow = (int)(i % OW), oh = (int)((i / OW) % OH);
    const long nc = i / ((long)OH * OW);
    float* p = dx + nc * H * W;
    const float g = IO<T>::ld(dy, i);
    if (nearest) {
      const int sh = min((int)floorf((float)oh * (float)H / (float)OH), H - 1);
      const int sw = min((int)floorf((float)ow * (float)W / (float)OW), W - 1);
      atomicAdd(p + (long)sh * W + sw, g);
      continue;
    }
    const float fh = src_coord(oh, H, OH, align), fw = src_coord(ow, W, OW, align);
    const int h0 = min((int)fh, H - 1), w0 = min((int)fw, W - 1);
    const int h1 = min(h0 + 1, H - 1), w1 = min(w0 + 1, W - 1);
    const float lh = fh - h0, lw = fw - w0;
    atomicAdd(p + (long)h0 * W + w0, g * (1.f - lh) * (1.f - lw));
    atomicAdd(p + (long)h0 * W + w1, g * (1.f - lh) * lw);
    atomicAdd(p + (long)h1 * W + w0, g * lh * (1.f - lw));
    atomicAdd(p + (long)h1 * W + w1, g * lh * lw);
  }
}

// ---------------------------------------------------------------- conv_shift
// out[b][i] = sum_j x[b][(i + j - half) mod M] y[b][j], half = (N - 1) / 2
template <typename T>
__global__ void conv_shift_fwd_kernel(const T* __restrict__ x, const T* __restrict__ y, T* __restrict__ out, int B,
                                      int M, int N) {
  const int half = (N - 1) / 2;
  GRID_STRIDE(t, (long)B * M) {
    const long b = t / M;
    const int i = (int)(t % M);
    float acc = 0.f;
    for (int j = 0; j < N; ++j) {
      int k = (i + j - half) % M;
      if (k < 0) k += M;
      acc += IO<T>::ld(x, b * M + k) * IO<T>::ld(y, b * N + j);
    }
    IO<T>::st(out, t, acc);
  }
}

// dx[b][k] = sum_j g[b][(k - j + half) mod M] y[b][j];  dy[b][j] = sum_i g[b][i] x[b][(i + j - half) mod M]
template <typename T>
__global__ void conv_shift_bwd_kernel(const T* __restrict__ x, const T* __restrict__ y, const T* __restrict__ g,
                                      T* __restrict__ dx, T* __restrict__ dy, int B, int M, int N) {
  const int half = (N - 1) / 2;
  GRID_STRIDE(t, (long)B * (M + N)) {
    const long b = t / (M + N);
    const int r = (int)(t % (M + N));
    if (r < M) {
      if (!dx) continue;
      float acc = 0.f;
      for (int j = 0; j < N; ++j) {
        int i = (r - j + half) % M;
        if (i < 0) i += M;
        acc += IO<T>::ld(g, b * M + i) * IO<T>::ld(y, b * N + j);
      }
      IO<T>::st(dx, b * M + r, acc);
    } else {
      if (!dy) continue;
      const int j = r - M;
      float acc = 0.f;
      for (int i = 0; i < M; ++i) {
        int k = (i + j - half) % M;
        if (k < 0) k += M;
        acc += IO<T>::ld(g, b * M + i) * IO<T>::ld(x, b * M + k);
      }
      IO<T>::st(dy, b * N + j, acc);
    }
  }
}

// ---------------------------------------------------------------- lstm_unit
// x [B, 4D] gates (i, f, o, g); c = sig(f + fb) c_prev + sig(i) tanh(g); h = sig(o) tanh(c)
template <typename T>
__global__ void lstm_unit_fwd_kernel(const T* __restrict__ x, const T* __restrict__ cp, T* __restrict__ c,
                                     T* __restrict__ h, long B, int D, float fb) {
  GRID_STRIDE(t, B * D) {
    const long b = t / D;
    const int d = (int)(t % D);
    const T* xr = x + b * 4 * D;
    const float i = sigm(IO<T>::ld(xr, d)), f = sigm(IO<T>::ld(xr, D + d) + fb), o = sigm(IO<T>::ld(xr, 2 * D + d));
    const float gg = tanhf(IO<T>::ld(xr, 3 * D + d));
    const float cv = f * IO<T>::ld(cp, t) + i * gg;
    IO<T>::st(c, t, cv);
    IO<T>::st(h, t, o * tanhf(cv));
  }
}

template <typename T>
__global__ void lstm_unit_bwd_kernel(const T* __restrict__ x, const T* __restrict__ cp, const T* __restrict__ c,
                                     const T* __restrict__ dc, const T* __restrict__ dh, T* __restrict__ dx,
                                     T* __restrict__ dcp, long B, int D, float fb) {
  GRID_STRIDE(t, B * D) {
    const long b = t / D;
    const int d = (int)(t % D);
    const T* xr = x + b * 4 * D;
    const float i = sigm(IO<T>::ld(xr, d)), f = sigm(IO<T>::ld(xr, D + d) + fb), o = sigm(IO<T>::ld(xr, 2 * D + d));
    const float gg = tanhf(IO<T>::ld(xr, 3 * D + d));
    const float tc = tanhf(IO<T>::ld(c, t));
    const float gh = dh ? IO<T>::ld(dh, t) : 0.f;
    const float gc = (dc ? IO<T>::ld(dc, t) : 0.f) + gh * o * (1.f - tc * tc);
    const float cpv = IO<T>::ld(cp, t);
    T* dxr = dx + b * 4 * D;
    IO<T>::st(dxr, d, gc * gg * i * (1.f - i));
    IO<T>::st(dxr, D + d, gc * cpv * f * (1.f - f));
    IO<T>::st(dxr, 2 * D + d, gh * tc * o * (1.f - o));
    IO<T>::st(dxr, 3 * D + d, gc * i * (1.f - gg * gg));
    if (dcp) IO<T>::st(dcp, t, gc * f);
  }
}


// ---------------------------------------------------------------- cross_entropy on probabilities
// hard labels: y = -log(x[label]) (0 for ignore_index); soft: y = -sum lab * log(x)
// (math/cross_entropy.cu CrossEntropyKernel / SoftCrossEntropyKernel); one wave per row
template <typename T>
__global__ __launch_bounds__(256) void xent_fwd_kernel(const T* __restrict__ x, const long* __restrict__ label,
                                                       const T* __restrict__ soft, T* __restrict__ y, long rows, int D,
                                                       long ignore) {
  const int lane = threadIdx.x & 63;
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  if (!soft) {
    if (lane == 0) {
      const long l = label[r];
      float v = 0.f;
      if (l != ignore && l >= 0 && l < D) v = -logf(IO<T>::ld(x, r * D + l));
      IO<T>::st(y, r, v);
    }
    return;
  }
  float acc = 0.f;
  for (int d = lane; d < D; d += 64) acc -= IO<T>::ld(soft, r * D + d) * logf(IO<T>::ld(x, r * D + d));
  acc = wave_sum(acc);
  if (lane == 0) IO<T>::st(y, r, acc);
}

template <typename T>
__global__ void xent_bwd_kernel(const T* __restrict__ x, const long* __restrict__ label, const T* __restrict__ soft,
                                const T* __restrict__ dy, T* __restrict__ dx, long rows, int D, long ignore) {
  GRID_STRIDE(i, rows * D) {
    const long r = i / D;
    const int d = (int)(i % D);
    const float g = IO<T>::ld(dy, r);
    float v;
    if (soft) {
      v = -g * IO<T>::ld(soft, i) / IO<T>::ld(x, i);
    } else {
      const long l = label[r];
      v = (l == d && l != ignore) ? -g / IO<T>::ld(x, i) : 0.f;
    }
    IO<T>::st(dx, i, v);
  }
}

}  // namespace

PA_EXPORT int pa_cross_entropy(int dt, int backward, const void* x, const long* label, const void* soft,
                               const void* dy, void* out, long rows, int D, long ignore, hipStream_t st) {
  if (rows <= 0 || D <= 0) return 0;
  if (!backward) {
    const dim3 g((unsigned)((rows + 3) / 4));
    if (dt == 1)
      hipLaunchKernelGGL(xent_fwd_kernel<u16>, g, dim3(256), 0, st, (const u16*)x, label, (const u16*)soft, (u16*)out,
                         rows, D, ignore);
    else
      hipLaunchKernelGGL(xent_fwd_kernel<float>, g, dim3(256), 0, st, (const float*)x, label, (const float*)soft,
                         (float*)out, rows, D, ignore);
  } else {
    if (dt == 1)
      hipLaunchKernelGGL(xent_bwd_kernel<u16>, dim3(grid_for(rows * D)), dim3(256), 0, st, (const u16*)x, label,
                         (const u16*)soft, (const u16*)dy, (u16*)out, rows, D, ignore);
    else
      hipLaunchKernelGGL(xent_bwd_kernel<float>, dim3(grid_for(rows * D)), dim3(256), 0, st, (const float*)x, label,
                         (const float*)soft, (const float*)dy, (float*)out, rows, D, ignore);
  }
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_cos_sim(int dt, const void* x, const void* y, void* out, float* xn, float* yn, long rows, int D,
                         int y_rows, hipStream_t st) {
  if (rows <= 0 || D <= 0) return 0;
  const dim3 g((unsigned)((rows + 3) / 4));
  if (dt == 1)
    hipLaunchKernelGGL(cos_sim_fwd_kernel<u16>, g, dim3(256), 0, st, (const u16*)x, (const u16*)y, (u16*)out, xn, yn,
                       rows, D, y_rows);
  else
    hipLaunchKernelGGL(cos_sim_fwd_kernel<float>, g, dim3(256), 0, st, (const float*)x, (const float*)y, (float*)out,
                       xn, yn, rows, D, y_rows);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_cos_sim_bwd(int dt, const void* x, const void* y, const void* out, const float* xn, const float* yn,
                             const void* dout, void* dx, float* dy, long rows, int D, int y_rows, hipStream_t st) {
  if (rows <= 0 || D <= 0) return 0;
  const dim3 g((unsigned)((rows + 3) / 4));
  if (dt == 1)
    hipLaunchKernelGGL(cos_sim_bwd_kernel<u16>, g, dim3(256), 0, st, (const u16*)x, (const u16*)y, (const u16*)out, xn,
                       yn, (const u16*)dout, (u16*)dx, dy, rows, D, y_rows);
  else
    hipLaunchKernelGGL(cos_sim_bwd_kernel<float>, g, dim3(256), 0, st, (const float*)x, (const float*)y,
                       (const float*)out, xn, yn, (const float*)dout, (float*)dx, dy, rows, D, y_rows);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_interp(int dt, int backward, const void* src, void* dst, long NC, int H, int W, int OH, int OW,
                        int nearest, int align, hipStream_t st) {
  const long total = NC * OH * OW;
  if (total <= 0 || H <= 0 || W <= 0) return 0;
  if (!backward) {
    if (dt == 1)
      hipLaunchKernelGGL(interp_fwd_kernel<u16>, dim3(grid_for(total)), dim3(256), 0, st, (const u16*)src, (u16*)dst,
                         NC, H, W, OH, OW, nearest, align);
    else
      hipLaunchKernelGGL(interp_fwd_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, (const float*)src,
                         (float*)dst, NC, H, W, OH, OW, nearest, align);
  } else {
    if (dt == 1)
      hipLaunchKernelGGL(interp_bwd_kernel<u16>, dim3(grid_for(total)), dim3(256), 0, st, (const u16*)src,
                         (float*)dst, NC, H, W, OH, OW, nearest, align);
    else
      hipLaunchKernelGGL(interp_bwd_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, (const float*)src,
                         (float*)dst, NC, H, W, OH, OW, nearest, align);
  }
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_conv_shift(int dt, const void* x, const void* y, const void* g, void* out, void* dx, void* dy, int B,
                            int M, int N, hipStream_t st) {
  if (B <= 0 || M <= 0 || N <= 0) return 0;
  if (!g) {
    if (dt == 1)
      hipLaunchKernelGGL(conv_shift_fwd_kernel<u16>, dim3(grid_for((long)B * M)), dim3(256), 0, st, (const u16*)x,
                         (const u16*)y, (u16*)out, B, M, N);
    else
      hipLaunchKernelGGL(conv_shift_fwd_kernel<float>, dim3(grid_for((long)B * M)), dim3(256), 0, st,
                         (const float*)x, (const float*)y, (float*)out, B, M, N);
  } else {
    if (dt == 1)
      hipLaunchKernelGGL(conv_shift_bwd_kernel<u16>, dim3(grid_for((long)B * (M + N))), dim3(256), 0, st,
                         (const u16*)x, (const u16*)y, (const u16*)g, (u16*)dx, (u16*)dy, B, M, N);
    else
      hipLaunchKernelGGL(conv_shift_bwd_kernel<float>, dim3(grid_for((long)B * (M + N))), dim3(256), 0, st,
                         (const float*)x, (const float*)y, (const float*)g, (float*)dx, (float*)dy, B, M, N);
  }
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_lstm_unit(int dt, int backward, const void* x, const void* cp, void* c, void* h, const void* dc,
                           const void* dh, void* dx, void* dcp, long B, int D, float fb, hipStream_t st) {
  const long total = B * D;
  if (total <= 0) return 0;
  if (!backward) {
    if (dt == 1)
      hipLaunchKernelGGL(lstm_unit_fwd_kernel<u16>, dim3(grid_for(total)), dim3(256), 0, st, (const u16*)x,
                         (const u16*)cp, (u16*)c, (u16*)h, B, D, fb);
    else
      hipLaunchKernelGGL(lstm_unit_fwd_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, (const float*)x,
                         (const float*)cp, (float*)c, (float*)h, B, D, fb);
  } else {
    if (dt == 1)
      hipLaunchKernelGGL(lstm_unit_bwd_kernel<u16>, dim3(grid_for(total)), dim3(256), 0, st, (const u16*)x,
                         (const u16*)cp, (const u16*)c, (const u16*)dc, (const u16*)dh, (u16*)dx, (u16*)dcp, B, D, fb);
    else
      hipLaunchKernelGGL(lstm_unit_bwd_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, (const float*)x,
                         (const float*)cp, (const float*)c, (const float*)dc, (const float*)dh, (float*)dx,
                         (float*)dcp, B, D, fb);
  }
  PA_LAUNCH_CHECK();
}

}  // namespace pa
