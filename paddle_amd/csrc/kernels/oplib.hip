// The general GPU operator library of the Fluid op set on gfx950: broadcast binary
// ops, axis reductions, Philox dropout, top-k, SGD / Adagrad (dense and
// SelectedRows), row gather / scatter-add (sequence expand / pad / unpad, sparse
// gradient merge), sequence pooling and the fused GRU gate math.
//
// Reference kernels these replace (behaviour, not code):
//   operators/elementwise_op_function.h (broadcast via (pre, n, post) + functors),
//   operators/reduce_op.h (Eigen reductions), operators/dropout_op.cu:27 (curand
//   mask), operators/top_k_op.cu:313, operators/sgd_op.cu / adagrad_op.cu,
//   math/selected_rows_functor.cu (MergeAdd), math/sequence_pooling.cu,
//   math/sequence_padding.cu, math/detail/gru_gpu_kernel.h:32.
//
// MI355X shape: wave64 reductions (common.h), grid-stride loops capped by
// stream_grid, fp32 accumulation for bf16 data, 16-B vectors on the contiguous
// same-shape paths; dtype T is float or u16 (bf16 bits).
#include "common.h"

namespace pa {
namespace oplib {

// ------------------------------------------------------------------ binary
constexpr int kMaxDims = 6;
struct BShape {
  int nd;
  long size[kMaxDims];
  long sx[kMaxDims];  // element strides of x / y in the output index space (0: broadcast)
  long sy[kMaxDims];
};

template <int OP>
__device__ __forceinline__ float bop(float a, float b) {
  if constexpr (OP == 0) return a + b;
  if constexpr (OP == 1) return a - b;
  if constexpr (OP == 2) return a * b;
  if constexpr (OP == 3) return a / b;
  if constexpr (OP == 4) return fmaxf(a, b);
  if constexpr (OP == 5) return fminf(a, b);
  return powf(a, b);
}

template <typename T, int OP>
__global__ void binary_bcast_kernel(const T* __restrict__ x, const T* __restrict__ y, T* __restrict__ out, long n,
                                    BShape s) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    long r = i, ox = 0, oy = 0;
#pragma unroll
    for (int d = kMaxDims - 1; d >= 0; --d) {
      if (d < s.nd) {
        const long c = r % s.size[d];
        r /= s.size[d];
        ox += c * s.sx[d];
        oy += c * s.sy[d];
      }
    }
    IO<T>::st(out, i, bop<OP>(IO<T>::ld(x, ox), IO<T>::ld(y, oy)));
  }
}

// same shape, both contiguous: 8 elements per thread-step
template <typename T, int OP>
__global__ void binary_same_kernel(const T* __restrict__ x, const T* __restrict__ y, T* __restrict__ out, long n8) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    float a[8], b[8], o[8];
    load8(x + i * 8, a);
    load8(y + i * 8, b);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = bop<OP>(a[e], b[e]);
    store8(out + i * 8, o);
  }
}

// ------------------------------------------------------------------ reduce
// x viewed as [pre, R, post]; op: 0 sum, 1 mean, 2 max, 3 min, 4 prod
template <int OP>
__device__ __forceinline__ float rinit() {
  if constexpr (OP == 2) return -INFINITY;
  if constexpr (OP == 3) return INFINITY;
  if constexpr (OP == 4) return 1.f;
  return 0.f;
}
template <int OP>
__device__ __forceinline__ float rcomb(float a, float b) {
  if constexpr (OP == 2) return fmaxf(a, b);
  if constexpr (OP == 3) return fminf(a, b);
  if constexpr (OP == 4) return a * b;
  return a + b;
}

template <int OP>
__device__ __forceinline__ float block_reduce(float v, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = rcomb<OP>(v, __shfl_xor(v, o, 64));
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = rinit<OP>();
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t = rcomb<OP>(t, red[i]);
  return t;
}

// post == 1: one block per row
template <typename T, int OP>
__global__ __launch_bounds__(256) void reduce_rows_kernel(const T* __restrict__ x, T* __restrict__ out, long R) {
  __shared__ float red[4];
  const long row = blockIdx.x;
  const T* xr = x + row * R;
  float acc = rinit<OP>();
  for (long j = threadIdx.x; j < R; j += blockDim.x) acc = rcomb<OP>(acc, IO<T>::ld(xr, j));
  acc = block_reduce<OP>(acc, red);
  if (threadIdx.x == 0) IO<T>::st(out, row, OP == 1 ? acc / (float)R : acc);
}

// post > 1: one thread per (pre, post) output, coalesced along post
template <typename T, int OP>
__global__ void reduce_cols_kernel(const T* __restrict__ x, T* __restrict__ out, long pre, long R, long post) {
  const long n = pre * post;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long p = i / post, q = i - p * post;
    const T* xp = x + p * R * post + q;
    float acc = rinit<OP>();
    for (long j = 0; j < R; ++j) acc = rcomb<OP>(acc, IO<T>::ld(xp, j * post));
    IO<T>::st(out, i, OP == 1 ? acc / (float)R : acc);
  }
}

// ------------------------------------------------------------------ dropout (Philox4x32-10)
__device__ __forceinline__ void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[1] = (uint32_t)p1;
    c[3] = (uint32_t)p0;
    c[0] = n0;
    c[2] = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

// element i uses word (i & 3) of the Philox block at counter (offset + i / 4)
template <typename T>
__global__ void dropout_kernel(const T* __restrict__ x, T* __restrict__ out, uint8_t* __restrict__ mask, long n,
                               float p, float scale, uint64_t seed, uint64_t offset) {
  const long nb = (n + 3) / 4;
  for (long b = (long)blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += (long)gridDim.x * blockDim.x) {
    const uint64_t ctr = offset + (uint64_t)b;
    uint32_t c[4] = {(uint32_t)ctr, (uint32_t)(ctr >> 32), 0u, 0u};
    philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long i = b * 4 + j;
      if (i < n) {
        const float u = (float)(c[j] >> 8) * (1.f / 16777216.f);
        const bool keep = u >= p;
        mask[i] = keep;
        IO<T>::st(out, i, keep ? IO<T>::ld(x, i) * scale : 0.f);
      }
    }
  }
}

template <typename T>
__global__ void mask_mul_kernel(const T* __restrict__ d, const uint8_t* __restrict__ mask, T* __restrict__ out,
                                long n, float scale) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    IO<T>::st(out, i, mask[i] ? IO<T>::ld(d, i) * scale : 0.f);
}

// ------------------------------------------------------------------ top-k (last axis)
// One wave per row.  Selection j takes the largest (value, -index) strictly below the
// previous pick in that order, so no "already taken" set is kept: k passes over the
// row (k <= 64; rows of any length).  Ties resolve to the smaller index (torch.topk).
template <typename T>
__global__ __launch_bounds__(256) void topk_kernel(const T* __restrict__ x, T* __restrict__ vals,
                                                   long* __restrict__ idx, long rows, int n, int k) {
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int lane = threadIdx.x & 63;
  const T* xr = x + r * n;
  float pv = INFINITY;
  int pi = -1;
  for (int j = 0; j < k; ++j) {
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int c = lane; c < n; c += 64) {
      const float v = IO<T>::ld(xr, c);
      const bool below = v < pv || (v == pv && c > pi);  // strictly after the previous pick
      const bool better = v > bv || (v == bv && c < bi);
      if (below && better) {
        bv = v;
        bi = c;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > bv || (ov == bv && oi < bi)) {
        bv = ov;
        bi = oi;
      }
    }
    if (lane == 0) {
      IO<T>::st(vals, r * k + j, bv);
      idx[r * k + j] = bi;
    }
    pv = bv;
    pi = bi;
  }
}

// ------------------------------------------------------------------ optimizers
template <typename T>
__global__ void sgd_kernel(T* __restrict__ p, const T* __restrict__ g, const float* __restrict__ lr, long n) {
  const float a = lr[0];
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    IO<T>::st(p, i, IO<T>::ld(p, i) - a * IO<T>::ld(g, i));
}

// Param[rows[r], :] -= lr * Values[r, :] (float atomics: rows may repeat)
__global__ void sgd_sparse_kernel(float* __restrict__ p, const long* __restrict__ rows, const float* __restrict__ v,
                                  const float* __restrict__ lr, long nrows, int D) {
  const float a = lr[0];
  const long n = nrows * D;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / D;
    const int d = (int)(i - r * D);
    atomicAdd(p + rows[r] * D + d, -a * v[i]);
  }
}

__global__ void adagrad_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                               const float* __restrict__ lr, long n, float eps) {
  const float a = lr[0];
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float gi = g[i];
    const float mi = m[i] + gi * gi;
    m[i] = mi;
    p[i] -= a * gi / (sqrtf(mi) + eps);
  }
}

// ------------------------------------------------------------------ row gather / scatter-add
// out[i, :] = idx[i] >= 0 ? src[idx[i], :] : fill ; D % 8 == 0 for the vector path
template <typename T>
__global__ void gather_rows_kernel(const T* __restrict__ src, const int* __restrict__ idx, T* __restrict__ out,
                                   long nrows, int D, float fill) {
  const long n = nrows * D;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / D;
    const int d = (int)(i - r * D);
    const int s = idx[r];
    IO<T>::st(out, i, s >= 0 ? IO<T>::ld(src, (long)s * D + d) : fill);
  }
}

// out[idx[i], :] += v[i, :] (fp32, float atomics; idx < 0 skipped)
__global__ void scatter_add_rows_kernel(const float* __restrict__ v, const int* __restrict__ idx,
                                        float* __restrict__ out, long nrows, int D) {
  const long n = nrows * D;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / D;
    const int d = (int)(i - r * D);
    const int t = idx[r];
    if (t >= 0) atomicAdd(out + (long)t * D + d, v[i]);
  }
}

// ------------------------------------------------------------------ sequence pooling
// x: [T, D] rows grouped by offsets[0..nseq]; one block per sequence, threads over D.
// type: 0 SUM, 1 AVERAGE, 2 SQRT, 3 MAX (argmax row -> maxi), 4 LAST, 5 FIRST
template <typename T>
__global__ __launch_bounds__(256) void seq_pool_kernel(const T* __restrict__ x, const int* __restrict__ off,
                                                       T* __restrict__ out, int* __restrict__ maxi, int D, int type,
                                                       float pad) {
  const int s = blockIdx.x;
  const int a = off[s], b = off[s + 1], len = b - a;
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float v;
    if (len == 0) {
      v = pad;
      if (type == 3) maxi[(long)s * D + d] = -1;
    } else if (type == 4) {
      v = IO<T>::ld(x, (long)(b - 1) * D + d);
    } else if (type == 5) {
      v = IO<T>::ld(x, (long)a * D + d);
    } else if (type == 3) {
      v = -INFINITY;
      int am = a;
      for (int r = a; r < b; ++r) {
        const float t = IO<T>::ld(x, (long)r * D + d);
        if (t > v) {
          v = t;
          am = r;
        }
      }
      maxi[(long)s * D + d] = am;
    } else {
      v = 0.f;
      for (int r = a; r < b; ++r) v += IO<T>::ld(x, (long)r * D + d);
      if (type == 1) v /= (float)len;
      if (type == 2) v /= sqrtf((float)len);
    }
    IO<T>::st(out, (long)s * D + d, v);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void seq_pool_grad_kernel(const T* __restrict__ dout, const int* __restrict__ off,
                                                            const int* __restrict__ maxi, T* __restrict__ dx, int D,
                                                            int type) {
  const int s = blockIdx.x;
  const int a = off[s], b = off[s + 1], len = b - a;
  if (len == 0) return;
  const float sc = type == 1 ? 1.f / (float)len : type == 2 ? rsqrtf((float)len) : 1.f;
  for (int r = a; r < b; ++r)
    for (int d = threadIdx.x; d < D; d += blockDim.x) {
      const float g = IO<T>::ld(dout, (long)s * D + d);
      float v;
      if (type == 3) v = maxi[(long)s * D + d] == r ? g : 0.f;
      else if (type == 4) v = r == b - 1 ? g : 0.f;
      else if (type == 5) v = r == a ? g : 0.f;
      else v = g * sc;
      IO<T>::st(dx, (long)r * D + d, v);
    }
}

// ------------------------------------------------------------------ GRU gates
// ur: [B, 2D] pre-activations (x-projection + bias + h W_ur); h: [B, D]
//   u = sigmoid(ur[:, :D]), r = sigmoid(ur[:, D:]), rh = r * h
// c_pre: [B, D] (x_c + bias_c + rh W_c); h' = h + u * (tanh(c_pre) - h)
__device__ __forceinline__ float sigm(float v) { return 1.f / (1.f + __expf(-v)); }

__global__ void gru_gate_kernel(const float* __restrict__ ur, const float* __restrict__ h, float* __restrict__ u,
                                float* __restrict__ r, float* __restrict__ rh, long B, int D) {
  const long n = B * D;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long b = i / D;
    const int d = (int)(i - b * D);
    const float uu = sigm(ur[b * 2 * D + d]), rr = sigm(ur[b * 2 * D + D + d]);
    u[i] = uu;
    r[i] = rr;
    rh[i] = rr * h[i];
  }
}

__global__ void gru_out_kernel(const float* __restrict__ cpre, const float* __restrict__ u,
                               const float* __restrict__ h, float* __restrict__ c, float* __restrict__ hn, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float cc = tanhf(cpre[i]);
    c[i] = cc;
    hn[i] = h[i] + u[i] * (cc - h[i]);
  }
}

// backward of gru_out: dcpre = dhn * u * (1 - c^2), du = dhn * (c - h), dh (partial) = dhn * (1 - u)
__global__ void gru_out_bwd_kernel(const float* __restrict__ dhn, const float* __restrict__ u,
                                   const float* __restrict__ h, const float* __restrict__ c, float* __restrict__ dcpre,
                                   float* __restrict__ du, float* __restrict__ dh, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float g = dhn[i], uu = u[i], cc = c[i];
    dcpre[i] = g * uu * (1.f - cc * cc);
    du[i] = g * (cc - h[i]);
    dh[i] = g * (1.f - uu);
  }
}

// backward of gru_gate: dur[:, :D] = du * u(1-u), dur[:, D:] = drh * h * r(1-r), dh += drh * r
__global__ void gru_gate_bwd_kernel(const float* __restrict__ du, const float* __restrict__ drh,
                                    const float* __restrict__ u, const float* __restrict__ r,
                                    const float* __restrict__ h, float* __restrict__ dur, float* __restrict__ dh,
                                    long B, int D) {
  const long n = B * D;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long b = i / D;
    const int d = (int)(i - b * D);
    const float uu = u[i], rr = r[i];
    dur[b * 2 * D + d] = du[i] * uu * (1.f - uu);
    dur[b * 2 * D + D + d] = drh[i] * h[i] * rr * (1.f - rr);
    dh[i] += drh[i] * rr;
  }
}

}  // namespace oplib
}  // namespace pa

using namespace pa;
using namespace pa::oplib;

#define PA_GRID(n) dim3(stream_grid((n), 256)), dim3(256), 0, st

// dt: 0 fp32, 1 bf16.  op: 0 add 1 sub 2 mul 3 div 4 max 5 min 6 pow.
// size/sx/sy: nd entries (outer -> inner); same == 1: contiguous equal shapes.
PA_EXPORT int pa_binary(int dt, int op, const void* x, const void* y, void* out, long n, int nd, const long* size,
                        const long* sx, const long* sy, int same, hipStream_t st) {
  if (n <= 0) return 0;
  if (nd > kMaxDims || op < 0 || op > 6 || dt < 0 || dt > 1) return -1;
#define PA_B(T, OP)                                                                                       \
  if (same && n % 8 == 0) {                                                                               \
    hipLaunchKernelGGL((binary_same_kernel<T, OP>), PA_GRID(n / 8), (const T*)x, (const T*)y, (T*)out, n / 8); \
  } else {                                                                                                \
    BShape s{};                                                                                           \
    s.nd = nd;                                                                                            \
    for (int d = 0; d < nd; ++d) {                                                                        \
      s.size[d] = size[d];                                                                                \
      s.sx[d] = sx[d];                                                                                    \
      s.sy[d] = sy[d];                                                                                    \
    }                                                                                                     \
    hipLaunchKernelGGL((binary_bcast_kernel<T, OP>), PA_GRID(n), (const T*)x, (const T*)y, (T*)out, n, s); \
  }                                                                                                       \
  PA_LAUNCH_CHECK();
#define PA_BOPS(T)                 \
  switch (op) {                    \
    case 0: { PA_B(T, 0) }         \
    case 1: { PA_B(T, 1) }         \
    case 2: { PA_B(T, 2) }         \
    case 3: { PA_B(T, 3) }         \
    case 4: { PA_B(T, 4) }         \
    case 5: { PA_B(T, 5) }         \
    default: { PA_B(T, 6) }        \
  }
  if (dt == 0) { PA_BOPS(float) }
  PA_BOPS(u16)
#undef PA_BOPS
#undef PA_B
}

// op: 0 sum 1 mean 2 max 3 min 4 prod over the middle axis of [pre, R, post]
PA_EXPORT int pa_reduce(int dt, int op, const void* x, void* out, long pre, long R, long post, hipStream_t st) {
  if (pre <= 0 || post <= 0) return 0;
  if (R <= 0 || op < 0 || op > 4 || dt < 0 || dt > 1) return -1;
#define PA_R(T, OP)                                                                                             \
  if (post == 1)                                                                                                \
    hipLaunchKernelGGL((reduce_rows_kernel<T, OP>), dim3((unsigned)pre), dim3(256), 0, st, (const T*)x, (T*)out, R); \
  else                                                                                                          \
    hipLaunchKernelGGL((reduce_cols_kernel<T, OP>), PA_GRID(pre * post), (const T*)x, (T*)out, pre, R, post);   \
  PA_LAUNCH_CHECK();
#define PA_ROPS(T)          \
  switch (op) {             \
    case 0: { PA_R(T, 0) }  \
    case 1: { PA_R(T, 1) }  \
    case 2: { PA_R(T, 2) }  \
    case 3: { PA_R(T, 3) }  \
    default: { PA_R(T, 4) } \
  }
  if (dt == 0) { PA_ROPS(float) }
  PA_ROPS(u16)
#undef PA_ROPS
#undef PA_R
}

PA_EXPORT int pa_dropout(int dt, const void* x, void* out, void* mask, long n, float p, float scale,
                         unsigned long long seed, unsigned long long offset, hipStream_t st) {
  if (n <= 0) return 0;
  if (dt == 0)
    hipLaunchKernelGGL(dropout_kernel<float>, PA_GRID((n + 3) / 4), (const float*)x, (float*)out, (uint8_t*)mask, n,
                       p, scale, (uint64_t)seed, (uint64_t)offset);
  else
    hipLaunchKernelGGL(dropout_kernel<u16>, PA_GRID((n + 3) / 4), (const u16*)x, (u16*)out, (uint8_t*)mask, n, p,
                       scale, (uint64_t)seed, (uint64_t)offset);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_mask_mul(int dt, const void* d, const void* mask, void* out, long n, float scale, hipStream_t st) {
  if (n <= 0) return 0;
  if (dt == 0)
    hipLaunchKernelGGL(mask_mul_kernel<float>, PA_GRID(n), (const float*)d, (const uint8_t*)mask, (float*)out, n,
                       scale);
  else
    hipLaunchKernelGGL(mask_mul_kernel<u16>, PA_GRID(n), (const u16*)d, (const uint8_t*)mask, (u16*)out, n, scale);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_topk(int dt, const void* x, void* vals, long* idx, long rows, int n, int k, hipStream_t st) {
  if (rows <= 0) return 0;
  if (k <= 0 || k > n || k > 64) return -1;
  const dim3 g((unsigned)((rows + 3) / 4));
  if (dt == 0)
    hipLaunchKernelGGL(topk_kernel<float>, g, dim3(256), 0, st, (const float*)x, (float*)vals, idx, rows, n, k);
  else
    hipLaunchKernelGGL(topk_kernel<u16>, g, dim3(256), 0, st, (const u16*)x, (u16*)vals, idx, rows, n, k);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_sgd(int dt, void* p, const void* g, const float* lr, long n, hipStream_t st) {
  if (n <= 0) return 0;
  if (dt == 0) hipLaunchKernelGGL(sgd_kernel<float>, PA_GRID(n), (float*)p, (const float*)g, lr, n);
  else hipLaunchKernelGGL(sgd_kernel<u16>, PA_GRID(n), (u16*)p, (const u16*)g, lr, n);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_sgd_sparse(float* p, const long* rows, const float* v, const float* lr, long nrows, int D,
                            hipStream_t st) {
  if (nrows <= 0) return 0;
  hipLaunchKernelGGL(sgd_sparse_kernel, PA_GRID(nrows * D), p, rows, v, lr, nrows, D);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_adagrad(float* p, const float* g, float* m, const float* lr, long n, float eps, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(adagrad_kernel, PA_GRID(n), p, g, m, lr, n, eps);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_gather_rows(int dt, const void* src, const int* idx, void* out, long nrows, int D, float fill,
                             hipStream_t st) {
  if (nrows <= 0 || D <= 0) return 0;
  if (dt == 0)
    hipLaunchKernelGGL(gather_rows_kernel<float>, PA_GRID(nrows * D), (const float*)src, idx, (float*)out, nrows, D,
                       fill);
  else
    hipLaunchKernelGGL(gather_rows_kernel<u16>, PA_GRID(nrows * D), (const u16*)src, idx, (u16*)out, nrows, D, fill);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_scatter_add_rows(const float* v, const int* idx, float* out, long nrows, int D, hipStream_t st) {
  if (nrows <= 0 || D <= 0) return 0;
  hipLaunchKernelGGL(scatter_add_rows_kernel, PA_GRID(nrows * D), v, idx, out, nrows, D);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_seq_pool(int dt, const void* x, const int* off, void* out, int* maxi, int nseq, int D, int type,
                          float pad, hipStream_t st) {
  if (nseq <= 0) return 0;
  if (type < 0 || type > 5) return -1;
  if (dt == 0)
    hipLaunchKernelGGL(seq_pool_kernel<float>, dim3(nseq), dim3(256), 0, st, (const float*)x, off, (float*)out, maxi,
                       D, type, pad);
  else
    hipLaunchKernelGGL(seq_pool_kernel<u16>, dim3(nseq), dim3(256), 0, st, (const u16*)x, off, (u16*)out, maxi, D,
                       type, pad);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_seq_pool_grad(int dt, const void* dout, const int* off, const int* maxi, void* dx, int nseq, int D,
                               int type, hipStream_t st) {
  if (nseq <= 0) return 0;
  if (dt == 0)
    hipLaunchKernelGGL(seq_pool_grad_kernel<float>, dim3(nseq), dim3(256), 0, st, (const float*)dout, off, maxi,
                       (float*)dx, D, type);
  else
    hipLaunchKernelGGL(seq_pool_grad_kernel<u16>, dim3(nseq), dim3(256), 0, st, (const u16*)dout, off, maxi,
                       (u16*)dx, D, type);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_gru_gate(const float* ur, const float* h, float* u, float* r, float* rh, long B, int D,
                          hipStream_t st) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL(gru_gate_kernel, PA_GRID(B * D), ur, h, u, r, rh, B, D);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_gru_out(const float* cpre, const float* u, const float* h, float* c, float* hn, long n,
                         hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(gru_out_kernel, PA_GRID(n), cpre, u, h, c, hn, n);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_gru_out_bwd(const float* dhn, const float* u, const float* h, const float* c, float* dcpre, float* du,
                             float* dh, long n, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(gru_out_bwd_kernel, PA_GRID(n), dhn, u, h, c, dcpre, du, dh, n);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_gru_gate_bwd(const float* du, const float* drh, const float* u, const float* r, const float* h,
                              float* dur, float* dh, long B, int D, hipStream_t st) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL(gru_gate_bwd_kernel, PA_GRID(B * D), du, drh, u, r, h, dur, dh, B, D);
  PA_LAUNCH_CHECK();
}
