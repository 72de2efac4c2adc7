// Softmax and fused softmax-with-cross-entropy for gfx950.
//
// Parity: softmax_with_cross_entropy (paddle/fluid/operators/
// softmax_with_cross_entropy_op.cu:109-311: three row-reduction kernels with
// cub::BlockReduce, warp32) and softmax (operators/math/softmax.cu, cuDNN).
// Redesigned: one 256-thread block per row, a single online (running max +
// rescaled sum) pass over 16-byte vectors for the forward, wave64 shuffles +
// one LDS hop for the block reduction; backward is one streaming pass that
// can run in place over the logits (saves a vocab-sized buffer for LLM heads).
#include "common.h"

namespace pa {

struct MS {
  float m, s;
};
__device__ __forceinline__ MS ms_merge(MS a, MS b) {
  const float m = fmaxf(a.m, b.m);
  if (m == -INFINITY) return {m, 0.f};
  return {m, a.s * __expf(a.m - m) + b.s * __expf(b.m - m)};
}
__device__ __forceinline__ MS wave_ms(MS v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    MS t{__shfl_xor(v.m, o, 64), __shfl_xor(v.s, o, 64)};
    v = ms_merge(v, t);
  }
  return v;
}
__device__ __forceinline__ MS block_ms(MS v, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_ms(v);
  __syncthreads();
  if (lane == 0) { red[2 * w] = v.m; red[2 * w + 1] = v.s; }
  __syncthreads();
  MS t{red[0], red[1]};
#pragma unroll
  for (int i = 1; i < 4; ++i) t = ms_merge(t, MS{red[2 * i], red[2 * i + 1]});
  return t;
}

// Row log-sum-exp over V columns (online pass).  VEC: columns % 8 == 0.
template <typename T, bool VEC>
__device__ __forceinline__ MS row_ms(const T* __restrict__ x, int V) {
  MS acc{-INFINITY, 0.f};
  if (VEC) {
    for (int c = threadIdx.x * 8; c < V; c += 256 * 8) {
      float v[8];
      load8(x + c, v);
      float m = v[0];
#pragma unroll
      for (int j = 1; j < 8; ++j) m = fmaxf(m, v[j]);
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) s += __expf(v[j] - m);
      acc = ms_merge(acc, MS{m, s});
    }
  } else {
    for (int c = threadIdx.x; c < V; c += 256) acc = ms_merge(acc, MS{IO<T>::ld(x, c), 1.f});
  }
  return acc;
}

// loss[r] = lse - x[label]; lse saved for backward.  soft_label: label is a [N,V]
// distribution (same dtype as logits) and loss = -sum(p * log_softmax).
template <typename T, bool VEC>
__global__ __launch_bounds__(256) void softmax_ce_fwd_kernel(
    const T* __restrict__ logits, const long* __restrict__ label, const T* __restrict__ soft,
    float* __restrict__ loss, float* __restrict__ lse_out, long N, int V, long ignore_index) {
  __shared__ float red[8];
  const long r = blockIdx.x;
  const T* x = logits + r * (long)V;
  MS ms = block_ms(row_ms<T, VEC>(x, V), red);
  const float lse = ms.m + __logf(ms.s);
  if (soft) {
    float acc = 0.f;
    for (int c = threadIdx.x; c < V; c += 256)
      acc += IO<T>::ld(soft, r * (long)V + c) * (IO<T>::ld(x, c) - lse);
    __syncthreads();
    acc = block_sum<256>(acc, red);
    if (threadIdx.x == 0) { loss[r] = -acc; lse_out[r] = lse; }
    return;
  }
  if (threadIdx.x == 0) {
    const long lb = label[r];
    lse_out[r] = lse;
    loss[r] = (lb == ignore_index || lb < 0 || lb >= V) ? 0.f : lse - IO<T>::ld(x, lb);
  }
}

// dlogits = (softmax - onehot) * dloss[r]   (may alias logits)
template <typename T, bool VEC>
__global__ __launch_bounds__(256) void softmax_ce_bwd_kernel(
    const T* logits, const long* __restrict__ label, const T* __restrict__ soft,
    const float* __restrict__ lse_in, const float* __restrict__ dloss, T* dlogits, long N, int V,
    long ignore_index, float dloss_scale) {
  const long r = blockIdx.x;
  const float lse = lse_in[r];
  long lb = soft ? -1 : label[r];
  float g = dloss ? dloss[r] * dloss_scale : dloss_scale;
  if (!soft && (lb == ignore_index || lb < 0 || lb >= V)) { g = 0.f; lb = -1; }
  const T* x = logits + r * (long)V;
  T* dx = dlogits + r * (long)V;
  if (VEC && !soft) {
    for (int c = threadIdx.x * 8; c < V; c += 256 * 8) {
      float v[8];
      load8(x + c, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (__expf(v[j] - lse) - ((c + j) == lb ? 1.f : 0.f)) * g;
      store8(dx + c, v);
    }
  } else {
    for (int c = threadIdx.x; c < V; c += 256) {
      const float p = __expf(IO<T>::ld(x, c) - lse);
      const float t = soft ? IO<T>::ld(soft, r * (long)V + c) : (c == lb ? 1.f : 0.f);
      IO<T>::st(dx, c, (p - t) * g);
    }
  }
}

// Plain row softmax (last axis): y = exp(x - lse)
template <typename T, bool VEC>
__global__ __launch_bounds__(256) void softmax_fwd_kernel(const T* __restrict__ x_,
                                                          T* __restrict__ y_, long N, int V,
                                                          int log_softmax) {
  __shared__ float red[8];
  const long r = blockIdx.x;
  const T* x = x_ + r * (long)V;
  T* y = y_ + r * (long)V;
  MS ms = block_ms(row_ms<T, VEC>(x, V), red);
  const float lse = ms.m + __logf(ms.s);
  if (VEC) {
    for (int c = threadIdx.x * 8; c < V; c += 256 * 8) {
      float v[8];
      load8(x + c, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = log_softmax ? v[j] - lse : __expf(v[j] - lse);
      store8(y + c, v);
    }
  } else {
    for (int c = threadIdx.x; c < V; c += 256) {
      const float v = IO<T>::ld(x, c);
      IO<T>::st(y, c, log_softmax ? v - lse : __expf(v - lse));
    }
  }
}

// dx = y * (dy - sum(dy * y))   (softmax)   or  dx = dy - exp(y) * sum(dy) (log_softmax)
template <typename T>
__global__ __launch_bounds__(256) void softmax_bwd_kernel(const T* __restrict__ y_,
                                                          const T* __restrict__ dy_,
                                                          T* __restrict__ dx_, long N, int V,
                                                          int log_softmax) {
  __shared__ float red[8];
  const long r = blockIdx.x;
  const T* y = y_ + r * (long)V;
  const T* dy = dy_ + r * (long)V;
  T* dx = dx_ + r * (long)V;
  float acc = 0.f;
  for (int c = threadIdx.x; c < V; c += 256)
    acc += log_softmax ? IO<T>::ld(dy, c) : IO<T>::ld(dy, c) * IO<T>::ld(y, c);
  acc = block_sum<256>(acc, red);
  for (int c = threadIdx.x; c < V; c += 256) {
    const float yv = IO<T>::ld(y, c), g = IO<T>::ld(dy, c);
    IO<T>::st(dx, c, log_softmax ? g - __expf(yv) * acc : yv * (g - acc));
  }
}

}  // namespace pa

using namespace pa;

#define PA_VEC_DISPATCH(KERNEL, ...)                                                     \
  do {                                                                                   \
    const bool vec = (V % 8) == 0;                                                       \
    if (dtype == 1) {                                                                    \
      if (vec) hipLaunchKernelGGL((KERNEL<u16, true>), dim3(N), dim3(256), 0, st, __VA_ARGS__); \
      else hipLaunchKernelGGL((KERNEL<u16, false>), dim3(N), dim3(256), 0, st, __VA_ARGS__);   \
    } else {                                                                             \
      if (vec) hipLaunchKernelGGL((KERNEL<float, true>), dim3(N), dim3(256), 0, st, __VA_ARGS__); \
      else hipLaunchKernelGGL((KERNEL<float, false>), dim3(N), dim3(256), 0, st, __VA_ARGS__);   \
    }                                                                                    \
  } while (0)

PA_EXPORT int pa_softmax_ce_fwd(int dtype, const void* logits, const long* label, const void* soft,
                                float* loss, float* lse, long N, int V, long ignore_index,
                                hipStream_t st) {
  if (N == 0) return 0;
  if (dtype == 1) {
    if (V % 8 == 0) hipLaunchKernelGGL((softmax_ce_fwd_kernel<u16, true>), dim3(N), dim3(256), 0, st, (const u16*)logits, label, (const u16*)soft, loss, lse, N, V, ignore_index);
    else hipLaunchKernelGGL((softmax_ce_fwd_kernel<u16, false>), dim3(N), dim3(256), 0, st, (const u16*)logits, label, (const u16*)soft, loss, lse, N, V, ignore_index);
  } else {
    if (V % 8 == 0) hipLaunchKernelGGL((softmax_ce_fwd_kernel<float, true>), dim3(N), dim3(256), 0, st, (const float*)logits, label, (const float*)soft, loss, lse, N, V, ignore_index);
    else hipLaunchKernelGGL((softmax_ce_fwd_kernel<float, false>), dim3(N), dim3(256), 0, st, (const float*)logits, label, (const float*)soft, loss, lse, N, V, ignore_index);
  }
  PA_LAUNCH_CHECK();
}

// dloss may be null (then every row's upstream grad = dloss_scale).
PA_EXPORT int pa_softmax_ce_bwd(int dtype, const void* logits, const long* label, const void* soft,
                                const float* lse, const float* dloss, void* dlogits, long N, int V,
                                long ignore_index, float dloss_scale, hipStream_t st) {
  if (N == 0) return 0;
  if (dtype == 1) {
    if (V % 8 == 0) hipLaunchKernelGGL((softmax_ce_bwd_kernel<u16, true>), dim3(N), dim3(256), 0, st, (const u16*)logits, label, (const u16*)soft, lse, dloss, (u16*)dlogits, N, V, ignore_index, dloss_scale);
    else hipLaunchKernelGGL((softmax_ce_bwd_kernel<u16, false>), dim3(N), dim3(256), 0, st, (const u16*)logits, label, (const u16*)soft, lse, dloss, (u16*)dlogits, N, V, ignore_index, dloss_scale);
  } else {
    if (V % 8 == 0) hipLaunchKernelGGL((softmax_ce_bwd_kernel<float, true>), dim3(N), dim3(256), 0, st, (const float*)logits, label, (const float*)soft, lse, dloss, (float*)dlogits, N, V, ignore_index, dloss_scale);
    else hipLaunchKernelGGL((softmax_ce_bwd_kernel<float, false>), dim3(N), dim3(256), 0, st, (const float*)logits, label, (const float*)soft, lse, dloss, (float*)dlogits, N, V, ignore_index, dloss_scale);
  }
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_softmax_fwd(int dtype, const void* x, void* y, long N, int V, int log_softmax,
                             hipStream_t st) {
  if (N == 0) return 0;
  if (dtype == 1) {
    if (V % 8 == 0) hipLaunchKernelGGL((softmax_fwd_kernel<u16, true>), dim3(N), dim3(256), 0, st, (const u16*)x, (u16*)y, N, V, log_softmax);
    else hipLaunchKernelGGL((softmax_fwd_kernel<u16, false>), dim3(N), dim3(256), 0, st, (const u16*)x, (u16*)y, N, V, log_softmax);
  } else {
    if (V % 8 == 0) hipLaunchKernelGGL((softmax_fwd_kernel<float, true>), dim3(N), dim3(256), 0, st, (const float*)x, (float*)y, N, V, log_softmax);
    else hipLaunchKernelGGL((softmax_fwd_kernel<float, false>), dim3(N), dim3(256), 0, st, (const float*)x, (float*)y, N, V, log_softmax);
  }
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_softmax_bwd(int dtype, const void* y, const void* dy, void* dx, long N, int V,
                             int log_softmax, hipStream_t st) {
  if (N == 0) return 0;
  if (dtype == 1)
    hipLaunchKernelGGL(softmax_bwd_kernel<u16>, dim3(N), dim3(256), 0, st, (const u16*)y, (const u16*)dy, (u16*)dx, N, V, log_softmax);
  else
    hipLaunchKernelGGL(softmax_bwd_kernel<float>, dim3(N), dim3(256), 0, st, (const float*)y, (const float*)dy, (float*)dx, N, V, log_softmax);
  PA_LAUNCH_CHECK();
}

// ---------------------------------------------------------------- mean reduction
// out[0] = sum_r loss[r] / max(1, #rows with a valid label); cnt[0] = that count.
// One block; the fused CE + mean node of the framework tape (no framework ops
// between the kernel and the scalar loss).
__global__ __launch_bounds__(1024) void ce_mean_fwd_kernel(const float* __restrict__ loss,
                                                           const long* __restrict__ label, long N, int V,
                                                           long ignore_index, float* __restrict__ out,
                                                           float* __restrict__ cnt) {
  __shared__ float red[16];
  float s = 0.f, c = 0.f;
  for (long r = threadIdx.x; r < N; r += blockDim.x) {
    const long lb = label[r];
    const bool ok = !(lb == ignore_index || lb < 0 || lb >= V);
    s += loss[r];
    c += ok ? 1.f : 0.f;
  }
  s = block_sum<1024>(s, red);
  __syncthreads();
  c = block_sum<1024>(c, red);
  if (threadIdx.x == 0) {
    cnt[0] = c;
    out[0] = s / fmaxf(c, 1.f);
  }
}

__global__ void ce_mean_bwd_rows_kernel(const float* __restrict__ g, const float* __restrict__ cnt,
                                        float* __restrict__ dl, long N) {
  const float v = g[0] / fmaxf(cnt[0], 1.f);
  for (long r = (long)blockIdx.x * blockDim.x + threadIdx.x; r < N; r += (long)gridDim.x * blockDim.x) dl[r] = v;
}

PA_EXPORT int pa_ce_mean_fwd(const float* loss, const long* label, long N, int V, long ignore_index, float* out,
                             float* cnt, hipStream_t st) {
  hipLaunchKernelGGL(ce_mean_fwd_kernel, dim3(1), dim3(1024), 0, st, loss, label, N, V, ignore_index, out, cnt);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_ce_mean_bwd_rows(const float* g, const float* cnt, float* dl, long N, hipStream_t st) {
  if (N <= 0) return 0;
  hipLaunchKernelGGL(ce_mean_bwd_rows_kernel, dim3(stream_grid(N, 256)), dim3(256), 0, st, g, cnt, dl, N);
  PA_LAUNCH_CHECK();
}
