// Remaining Fluid op-library kernels on gfx950 (SURVEY §2.8 "misc" / concat-split /
// argsort-accuracy / one_hot rows).  fp32 or bf16 (T = float | u16) data, wave64.
//
// Reference behaviour: operators/one_hot_op.cu, pad2d_op.cu (constant / reflect /
// edge, NCHW / NHWC), lrn_op.cu (cross-channel, mid = k + alpha * sum x^2),
// row_conv_op.cu (lookahead conv per LoD sequence), concat_op / split_op
// (math/concat.cu), argsort_op.cu, accuracy_op.cu.
#include "common.h"

namespace pa {
namespace {

inline int grid_for(long n, int block = 256) {
  long g = (n + block - 1) / block;
  return (int)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

#define GRID_STRIDE(i, n) for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < (n); i += (long)gridDim.x * blockDim.x)

// ---------------------------------------------------------------- one_hot
__global__ void one_hot_kernel(const long* __restrict__ x, float* __restrict__ out, long n, int depth,
                               int* __restrict__ bad) {
  GRID_STRIDE(i, n * depth) {
    const long r = i / depth;
    const int c = (int)(i % depth);
    const long v = x[r];
    if (c == 0 && (v < 0 || v >= depth)) *bad = 1;
    out[i] = (v == c) ? 1.f : 0.f;
  }
}

// ---------------------------------------------------------------- pad2d
// mode 0 constant, 1 reflect, 2 edge; layout 0 NCHW, 1 NHWC
__device__ __forceinline__ int pad_src(int o, int pad, int n, int mode) {
  int s = o - pad;
  if (s >= 0 && s < n) return s;
  if (mode == 0) return -1;
  if (mode == 2) return s < 0 ? 0 : n - 1;
  // reflect (no edge repeat): -1 -> 1, n -> n - 2
  if (n == 1) return 0;
  const int period = 2 * (n - 1);
  s = s % period;
  if (s < 0) s += period;
  return s < n ? s : period - s;
}

template <typename T>
__global__ void pad2d_kernel(const T* __restrict__ x, T* __restrict__ y, int N, int C, int H, int W, int OH, int OW,
                             int pt, int pl, int mode, float val, int nhwc) {
  const long total = (long)N * C * OH * OW;
  GRID_STRIDE(i, total) {
    int n, c, oh, ow;
    if (nhwc) {
      c = (int)(i % C);
      long t = i / C;
      ow = (int)(t % OW);
      t /= OW;
      oh = (int)(t % OH);
      n = (int)(t / OH);
    } else {
      ow = (int)(i % OW);
      long t = i / OW;
      oh = (int)(t % OH);
      t /= OH;
      c = (int)(t % C);
      n = (int)(t / C);
    }
    const int sh = pad_src(oh, pt, H, mode), sw = pad_src(ow, pl, W, mode);
    float v = val;
    if (sh >= 0 && sw >= 0) {
      const long si = nhwc ? (((long)n * H + sh) * W + sw) * C + c : (((long)n * C + c) * H + sh) * W + sw;
      v = IO<T>::ld(x, si);
    }
    IO<T>::st(y, i, v);
  }
}

// dx (fp32, zeroed) += dy at the mapped source (reflect / edge: several outputs map
// to one input -> float atomics; constant: plain crop, no collisions)
template <typename T>
__global__ void pad2d_bwd_kernel(const T* __restrict__ dy, float* __restrict__ dx, int N, int C, int H, int W, int OH,
                                 int OW, int pt, int pl, int mode, int nhwc) {
  const long total = (long)N * C * OH * OW;
  GRID_STRIDE(i, total) {
    int n, c, oh, ow;
    if (nhwc) {
      c = (int)(i % C);
      long t = i / C;
      ow = (int)(t % OW);
      t /= OW;
      oh = (int)(t % OH);
      n = (int)(t / OH);
    } else {
      ow = (int)(i % OW);
      long t = i / OW;
      oh = (int)(t % OH);
      t /= OH;
      c = (int)(t % C);
      n = (int)(t / C);
    }
    const int sh = pad_src(oh, pt, H, mode), sw = pad_src(ow, pl, W, mode);
    if (sh < 0 || sw < 0) continue;
    const long si = nhwc ? (((long)n * H + sh) * W + sw) * C + c : (((long)n * C + c) * H + sh) * W + sw;
    const float g = IO<T>::ld(dy, i);
    if (mode == 0) dx[si] = g;
    else atomicAdd(dx + si, g);
  }
}

// ---------------------------------------------------------------- LRN (NCHW, across channels)
// mid = k + alpha * sum_{c' in [c - pre, c - pre + n)} x^2, pre = (n - 1) / 2
// (operators/lrn_op.cc: start = -(n - 1) / 2, end = start + n); out = x * mid^-beta
template <typename T>
__global__ void lrn_fwd_kernel(const T* __restrict__ x, T* __restrict__ out, float* __restrict__ mid, int N, int C,
                               long HW, int n, float k, float alpha, float beta) {
  const long total = (long)N * C * HW;
  const int pre = (n - 1) / 2;
  GRID_STRIDE(i, total) {
    const int c = (int)((i / HW) % C);
    const long base = i - (long)c * HW;  // (n, 0, hw)
    float s = 0.f;
    for (int j = c - pre; j < c - pre + n; ++j)
      if (j >= 0 && j < C) {
        const float v = IO<T>::ld(x, base + (long)j * HW);
        s += v * v;
      }
    const float m = k + alpha * s;
    mid[i] = m;
    IO<T>::st(out, i, IO<T>::ld(x, i) * __powf(m, -beta));
  }
}

// dx_c = dy_c * mid_c^-beta - 2 alpha beta x_c * sum_{j: c in window(j)} dy_j x_j mid_j^(-beta-1)
template <typename T>
__global__ void lrn_bwd_kernel(const T* __restrict__ x, const T* __restrict__ dy, const float* __restrict__ mid,
                               T* __restrict__ dx, int N, int C, long HW, int n, float alpha, float beta) {
  const long total = (long)N * C * HW;
  const int pre = (n - 1) / 2;
  GRID_STRIDE(i, total) {
    const int c = (int)((i / HW) % C);
    const long base = i - (long)c * HW;
    // window(j) = [j - pre, j - pre + n): c is inside it for j in (c + pre - n, c + pre]
    float acc = 0.f;
    for (int j = c + pre - n + 1; j <= c + pre; ++j)
      if (j >= 0 && j < C) {
        const long o = base + (long)j * HW;
        acc += IO<T>::ld(dy, o) * IO<T>::ld(x, o) * __powf(mid[o], -beta - 1.f);
      }
    const float g = IO<T>::ld(dy, i) * __powf(mid[i], -beta) - 2.f * alpha * beta * IO<T>::ld(x, i) * acc;
    IO<T>::st(dx, i, g);
  }
}

// ---------------------------------------------------------------- row_conv (LoD sequences)
// out[t, d] = sum_{k < K, t + k < end(seq(t))} x[t + k, d] * w[k, d]
template <typename T>
__global__ void row_conv_fwd_kernel(const T* __restrict__ x, const T* __restrict__ w, const int* __restrict__ seq_end,
                                    T* __restrict__ out, long rows, int D, int K) {
  GRID_STRIDE(i, rows * D) {
    const long t = i / D;
    const int d = (int)(i % D);
    const long end = seq_end[t];
    float s = 0.f;
    for (int k = 0; k < K && t + k < end; ++k) s += IO<T>::ld(x, (t + k) * D + d) * IO<T>::ld(w, (long)k * D + d);
    IO<T>::st(out, i, s);
  }
}

// dx[t, d] = sum_{k, t - k >= start(seq(t))} dy[t - k, d] * w[k, d]
template <typename T>
__global__ void row_conv_dx_kernel(const T* __restrict__ dy, const T* __restrict__ w, const int* __restrict__ seq_start,
                                   T* __restrict__ dx, long rows, int D, int K) {
  GRID_STRIDE(i, rows * D) {
    const long t = i / D;
    const int d = (int)(i % D);
    const long st = seq_start[t];
    float s = 0.f;
    for (int k = 0; k < K && t - k >= st; ++k) s += IO<T>::ld(dy, (t - k) * D + d) * IO<T>::ld(w, (long)k * D + d);
    IO<T>::st(dx, i, s);
  }
}

// dw[k, d] = sum_t dy[t, d] * x[t + k, d] (t + k in the same sequence): one block per
// (k, d-chunk of 64), wave-strided over t, block reduction in LDS
template <typename T>
__global__ __launch_bounds__(256) void row_conv_dw_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                          const int* __restrict__ seq_end, float* __restrict__ dw,
                                                          long rows, int D) {
  const int k = blockIdx.y;
  const int d = blockIdx.x * 64 + (threadIdx.x & 63);
  const int tw = threadIdx.x >> 6;  // 4 row lanes
  float s = 0.f;
  if (d < D)
    for (long t = tw; t < rows; t += 4)
      if (t + k < seq_end[t]) s += IO<T>::ld(dy, t * D + d) * IO<T>::ld(x, (t + k) * D + d);
  __shared__ float red[4][64];
  red[tw][threadIdx.x & 63] = s;
  __syncthreads();
  if (tw == 0 && d < D) dw[(long)k * D + d] = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
}

// ---------------------------------------------------------------- argsort (per row, n <= 2048)
// Bitonic sort of (key, index) pairs in LDS, one block per row; ascending keys, ties
// by index (stable order).  Padding keys are +inf with index n (sorted last).
template <typename T>
__global__ __launch_bounds__(1024) void argsort_rows_kernel(const T* __restrict__ x, T* __restrict__ vals,
                                                            long* __restrict__ idx, int n, int P, int desc) {
  extern __shared__ char sm[];
  float* key = reinterpret_cast<float*>(sm);
  int* id = reinterpret_cast<int*>(key + P);
  const long row = blockIdx.x;
  const T* xr = x + row * n;
  for (int i = threadIdx.x; i < P; i += blockDim.x) {
    const float v = i < n ? IO<T>::ld(xr, i) : INFINITY;
    key[i] = (i < n && desc) ? -v : v;
    id[i] = i;
  }
  __syncthreads();
  for (int size = 2; size <= P; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < P; i += blockDim.x) {
        const int j = i ^ stride;
        if (j > i) {
          const bool up = (i & size) == 0;
          const float ki = key[i], kj = key[j];
          const int ii = id[i], ij = id[j];
          const bool gt = ki > kj || (ki == kj && ii > ij);
          if (gt == up) {
            key[i] = kj; key[j] = ki;
            id[i] = ij; id[j] = ii;
          }
        }
      }
      __syncthreads();
    }
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    IO<T>::st(vals + row * n, i, desc ? -key[i] : key[i]);
    idx[row * n + i] = id[i];
  }
}

// ---------------------------------------------------------------- accuracy
// correct = #rows whose label appears among the row's k indices
__global__ __launch_bounds__(256) void accuracy_kernel(const long* __restrict__ ind, const long* __restrict__ lab,
                                                       long rows, int k, int* __restrict__ correct) {
  int c = 0;
  for (long r = blockIdx.x * (long)blockDim.x + threadIdx.x; r < rows; r += (long)gridDim.x * blockDim.x) {
    const long l = lab[r];
    bool hit = false;
    for (int j = 0; j < k; ++j) hit |= ind[r * k + j] == l;
    c += hit ? 1 : 0;
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(correct, c);
}

__global__ void accuracy_finish_kernel(const int* __restrict__ correct, long rows, float* __restrict__ acc,
                                       int* __restrict__ total) {
  if (threadIdx.x == 0) {
    acc[0] = rows ? (float)correct[0] / (float)rows : 0.f;
    total[0] = (int)rows;
  }
}

}  // namespace
}  // namespace pa

using namespace pa;

#define DT_DISPATCH(dt, KERNEL, ...)                                   \
  do {                                                                 \
    if ((dt) == 1) hipLaunchKernelGGL(KERNEL<u16>, __VA_ARGS__);       \
    else hipLaunchKernelGGL(KERNEL<float>, __VA_ARGS__);               \
  } while (0)

PA_EXPORT int pa_one_hot(const long* x, float* out, long n, int depth, int* bad, hipStream_t st) {
  hipLaunchKernelGGL(one_hot_kernel, dim3(grid_for(n * depth)), dim3(256), 0, st, x, out, n, depth, bad);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_pad2d(int dt, const void* x, void* y, int N, int C, int H, int W, int pt, int pb, int pl, int pr,
                       int mode, float val, int nhwc, hipStream_t st) {
  const int OH = H + pt + pb, OW = W + pl + pr;
  if (mode == 1 && (pt >= H || pb >= H || pl >= W || pr >= W)) return -1;  // reflect needs pad < size
  const long total = (long)N * C * OH * OW;
  if (dt == 1)
    hipLaunchKernelGGL(pad2d_kernel<u16>, dim3(grid_for(total)), dim3(256), 0, st, (const u16*)x, (u16*)y, N, C, H, W,
                       OH, OW, pt, pl, mode, val, nhwc);
  else
    hipLaunchKernelGGL(pad2d_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, (const float*)x, (float*)y, N, C,
                       H, W, OH, OW, pt, pl, mode, val, nhwc);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_pad2d_bwd(int dt, const void* dy, float* dx, int N, int C, int H, int W, int pt, int pb, int pl,
                           int pr, int mode, int nhwc, hipStream_t st) {
  const int OH = H + pt + pb, OW = W + pl + pr;
  const long total = (long)N * C * OH * OW;
  if (dt == 1)
    hipLaunchKernelGGL(pad2d_bwd_kernel<u16>, dim3(grid_for(total)), dim3(256), 0, st, (const u16*)dy, dx, N, C, H, W,
                       OH, OW, pt, pl, mode, nhwc);
  else
    hipLaunchKernelGGL(pad2d_bwd_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, (const float*)dy, dx, N, C,
                       H, W, OH, OW, pt, pl, mode, nhwc);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_lrn_fwd(int dt, const void* x, void* out, float* mid, int N, int C, long HW, int n, float k,
                         float alpha, float beta, hipStream_t st) {
  const long total = (long)N * C * HW;
  if (dt == 1)
    hipLaunchKernelGGL(lrn_fwd_kernel<u16>, dim3(grid_for(total)), dim3(256), 0, st, (const u16*)x, (u16*)out, mid, N,
                       C, HW, n, k, alpha, beta);
  else
    hipLaunchKernelGGL(lrn_fwd_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, (const float*)x, (float*)out,
                       mid, N, C, HW, n, k, alpha, beta);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_lrn_bwd(int dt, const void* x, const void* dy, const float* mid, void* dx, int N, int C, long HW,
                         int n, float alpha, float beta, hipStream_t st) {
  const long total = (long)N * C * HW;
  if (dt == 1)
    hipLaunchKernelGGL(lrn_bwd_kernel<u16>, dim3(grid_for(total)), dim3(256), 0, st, (const u16*)x, (const u16*)dy,
                       mid, (u16*)dx, N, C, HW, n, alpha, beta);
  else
    hipLaunchKernelGGL(lrn_bwd_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, (const float*)x,
                       (const float*)dy, mid, (float*)dx, N, C, HW, n, alpha, beta);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_row_conv_fwd(int dt, const void* x, const void* w, const int* seq_end, void* out, long rows, int D,
                              int K, hipStream_t st) {
  if (dt == 1)
    hipLaunchKernelGGL(row_conv_fwd_kernel<u16>, dim3(grid_for(rows * D)), dim3(256), 0, st, (const u16*)x,
                       (const u16*)w, seq_end, (u16*)out, rows, D, K);
  else
    hipLaunchKernelGGL(row_conv_fwd_kernel<float>, dim3(grid_for(rows * D)), dim3(256), 0, st, (const float*)x,
                       (const float*)w, seq_end, (float*)out, rows, D, K);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_row_conv_bwd(int dt, const void* dy, const void* x, const void* w, const int* seq_start,
                              const int* seq_end, void* dx, float* dw, long rows, int D, int K, hipStream_t st) {
  if (dx) {
    if (dt == 1)
      hipLaunchKernelGGL(row_conv_dx_kernel<u16>, dim3(grid_for(rows * D)), dim3(256), 0, st, (const u16*)dy,
                         (const u16*)w, seq_start, (u16*)dx, rows, D, K);
    else
      hipLaunchKernelGGL(row_conv_dx_kernel<float>, dim3(grid_for(rows * D)), dim3(256), 0, st, (const float*)dy,
                         (const float*)w, seq_start, (float*)dx, rows, D, K);
  }
  if (dw) {
    dim3 g((unsigned)((D + 63) / 64), (unsigned)K);
    if (dt == 1)
      hipLaunchKernelGGL(row_conv_dw_kernel<u16>, g, dim3(256), 0, st, (const u16*)dy, (const u16*)x, seq_end, dw, rows,
                         D);
    else
      hipLaunchKernelGGL(row_conv_dw_kernel<float>, g, dim3(256), 0, st, (const float*)dy, (const float*)x, seq_end, dw,
                         rows, D);
  }
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_argsort_rows(int dt, const void* x, void* vals, long* idx, long rows, int n, int desc,
                              hipStream_t st) {
  if (n <= 0 || n > 2048 || rows <= 0) return -1;
  int P = 1;
  while (P < n) P <<= 1;
  const size_t sh = (size_t)P * 8;
  const int threads = P < 1024 ? (P < 64 ? 64 : P) : 1024;
  if (dt == 1)
    hipLaunchKernelGGL(argsort_rows_kernel<u16>, dim3((unsigned)rows), dim3(threads), sh, st, (const u16*)x,
                       (u16*)vals, idx, n, P, desc);
  else
    hipLaunchKernelGGL(argsort_rows_kernel<float>, dim3((unsigned)rows), dim3(threads), sh, st, (const float*)x,
                       (float*)vals, idx, n, P, desc);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_accuracy(const long* ind, const long* lab, long rows, int k, int* correct, float* acc, int* total,
                          hipStream_t st) {
  if (hipMemsetAsync(correct, 0, sizeof(int), st) != hipSuccess) return -1;
  hipLaunchKernelGGL(accuracy_kernel, dim3(grid_for(rows)), dim3(256), 0, st, ind, lab, rows, k, correct);
  hipLaunchKernelGGL(accuracy_finish_kernel, dim3(1), dim3(64), 0, st, correct, rows, acc, total);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_copy2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width, size_t height,
                        hipStream_t st) {
  if (!width || !height) return 0;
  return (int)hipMemcpy2DAsync(dst, dpitch, src, spitch, width, height, hipMemcpyDeviceToDevice, st);
}
