// Fluid operator-library rows on gfx950: activations (forward and backward),
// softmax-with-cross-entropy producing the Softmax output and its grad from it,
// dtype cast, an n-d strided gather (transpose / reverse / slice / expand / tile /
// crop all lower to it), Philox uniform / gaussian random, the pointwise loss
// family, and LoD sequence softmax.
//
// Reference rows (paddle/fluid/operators): activation_op.h:877-906 (functor table,
// grad from X or Out), softmax_with_cross_entropy_op.cu:109-311, cast_op.h,
// transpose_op.h / math_function.cu Transpose, reverse_op.h, slice_op.h,
// expand_op.h, uniform_random_op.cu, gaussian_random_op.cu (thrust + minstd),
// hinge_loss_op.h, huber_loss_op.h, smooth_l1_loss_op.h, log_loss_op.h,
// modified_huber_loss_op.h, sigmoid_cross_entropy_with_logits_op.h,
// sequence_softmax_cudnn_op.cu.cc.
//
// MI355X design: every elementwise kernel is a grid-stride loop over 8 elements
// per lane per trip (16-byte bf16 vectors, two 16-byte fp32 vectors) with a
// scalar tail; grids from stream_grid() (<= 2048 blocks of 256: 8 blocks / CU).
// Random numbers are counter-based Philox4x32-10 keyed by (seed, element index),
// so a tensor is reproducible for any grid and across devices.
#include "common.h"

namespace pa {
namespace fo {

// ------------------------------------------------------------------ element IO
template <typename T> struct E;
template <> struct E<float> {
  static __device__ __forceinline__ float ld(const float* p, long i) { return p[i]; }
  static __device__ __forceinline__ void st(float* p, long i, float v) { p[i] = v; }
};
template <> struct E<u16> {  // bf16 bits
  static __device__ __forceinline__ float ld(const u16* p, long i) { return bf2f(p[i]); }
  static __device__ __forceinline__ void st(u16* p, long i, float v) { p[i] = f2bf(v); }
};

// ------------------------------------------------------------------ activations
enum Act {
  RELU = 0, SIGMOID, LOGSIGMOID, EXP, TANH, TANH_SHRINK, SOFTSHRINK, SQRT, RSQRT, ABS, CEIL, FLOOR, COS, SIN,
  ROUND, RECIPROCAL, LOG, SQUARE, SOFTPLUS, SOFTSIGN, BRELU, LEAKY_RELU, SOFT_RELU, ELU, RELU6, POW, STANH,
  HARD_SHRINK, THRESHOLDED_RELU, HARD_SIGMOID, SWISH, GELU, SILU, NUM_ACT
};

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

__device__ __forceinline__ float act_f(int op, float x, float a, float b) {
  switch (op) {
    case RELU: return fmaxf(x, 0.f);
    case SIGMOID: return sigm(x);
    case LOGSIGMOID: return -(fmaxf(-x, 0.f) + log1pf(__expf(-fabsf(x))));
    case EXP: return __expf(x);
    case TANH: return tanhf(x);
    case TANH_SHRINK: return x - tanhf(x);
    case SOFTSHRINK: return x > a ? x - a : (x < -a ? x + a : 0.f);
    case SQRT: return sqrtf(x);
    case RSQRT: return rsqrtf(x);
    case ABS: return fabsf(x);
    case CEIL: return ceilf(x);
    case FLOOR: return floorf(x);
    case COS: return cosf(x);
    case SIN: return sinf(x);
    case ROUND: return rintf(x);
    case RECIPROCAL: return 1.f / x;
    case LOG: return __logf(x);
    case SQUARE: return x * x;
    case SOFTPLUS: return fmaxf(x, 0.f) + log1pf(__expf(-fabsf(x)));
    case SOFTSIGN: return x / (1.f + fabsf(x));
    case BRELU: return fminf(fmaxf(x, a), b);
    case LEAKY_RELU: return x > 0.f ? x : a * x;
    case SOFT_RELU: { const float t = fminf(fmaxf(x, -a), a); return log1pf(__expf(t)); }
    case ELU: return x > 0.f ? x : a * (__expf(x) - 1.f);
    case RELU6: return fminf(fmaxf(x, 0.f), a);
    case POW: return powf(x, a);
    case STANH: return b * tanhf(a * x);
    case HARD_SHRINK: return (x > a || x < -a) ? x : 0.f;
    case THRESHOLDED_RELU: return x > a ? x : 0.f;
    case HARD_SIGMOID: return fminf(fmaxf(a * x + b, 0.f), 1.f);
    case SWISH: return x * sigm(a * x);
    case GELU: return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
    case SILU: return x * sigm(x);
  }
  return x;
}

// dOut/dX at (x, y = f(x)); the Fluid grad ops hand over whichever of X / Out the
// functor needs (activation_op.h FDDepType), both are passed here (null -> unused)
__device__ __forceinline__ float act_df(int op, float x, float y, float a, float b) {
  switch (op) {
    case RELU: return y > 0.f ? 1.f : 0.f;
    case SIGMOID: return y * (1.f - y);
    case LOGSIGMOID: return sigm(-x);
    case EXP: return y;
    case TANH: return 1.f - y * y;
    case TANH_SHRINK: { const float t = tanhf(x); return t * t; }
    case SOFTSHRINK: return (x > a || x < -a) ? 1.f : 0.f;
    case SQRT: return 0.5f / y;
    case RSQRT: return -0.5f * y * y * y;
    case ABS: return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f);
    case CEIL: case FLOOR: case ROUND: return 0.f;
    case COS: return -sinf(x);
    case SIN: return cosf(x);
    case RECIPROCAL: return -y * y;
    case LOG: return 1.f / x;
    case SQUARE: return 2.f * x;
    case SOFTPLUS: return sigm(x);
    case SOFTSIGN: { const float d = 1.f + fabsf(x); return 1.f / (d * d); }
    case BRELU: return (x > a && x < b) ? 1.f : 0.f;
    case LEAKY_RELU: return x > 0.f ? 1.f : a;
    case SOFT_RELU: return (x > -a && x < a) ? 1.f - __expf(-y) : 0.f;
    case ELU: return x > 0.f ? 1.f : y + a;
    case RELU6: return (x > 0.f && x < a) ? 1.f : 0.f;
    case POW: return a * powf(x, a - 1.f);
    case STANH: { const float t = tanhf(a * x); return a * b * (1.f - t * t); }
    case HARD_SHRINK: return (x > a || x < -a) ? 1.f : 0.f;
    case THRESHOLDED_RELU: return x > a ? 1.f : 0.f;
    case HARD_SIGMOID: { const float t = a * x + b; return (t > 0.f && t < 1.f) ? a : 0.f; }
    case SWISH: { const float s = sigm(a * x); return s + a * x * s * (1.f - s); }
    case GELU: return 0.5f * (1.f + erff(x * 0.70710678118654752f)) + x * 0.3989422804014327f * __expf(-0.5f * x * x);
    case SILU: { const float s = sigm(x); return s * (1.f + x * (1.f - s)); }
  }
  return 1.f;
}

template <typename T>
__global__ __launch_bounds__(256) void act_fwd_kernel(int op, const T* __restrict__ x, T* __restrict__ y, long n,
                                                      float a, float b) {
  const long stride = (long)gridDim.x * 256 * 8;
  for (long base = ((long)blockIdx.x * 256 + threadIdx.x) * 8; base < n; base += stride) {
    if (base + 8 <= n) {
      float v[8];
      load8(x + base, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = act_f(op, v[j], a, b);
      store8(y + base, v);
    } else {
      for (long i = base; i < n; ++i) E<T>::st(y, i, act_f(op, E<T>::ld(x, i), a, b));
    }
  }
}

// dx = dy * f'(x, y); x or y may be null (the functor does not read it)
template <typename T>
__global__ __launch_bounds__(256) void act_bwd_kernel(int op, const T* __restrict__ x, const T* __restrict__ y,
                                                      const T* __restrict__ dy, T* __restrict__ dx, long n, float a,
                                                      float b) {
  const long stride = (long)gridDim.x * 256 * 8;
  for (long base = ((long)blockIdx.x * 256 + threadIdx.x) * 8; base < n; base += stride) {
    if (base + 8 <= n) {
      float xv[8], yv[8], gv[8];
      if (x) load8(x + base, xv); else for (int j = 0; j < 8; ++j) xv[j] = 0.f;
      if (y) load8(y + base, yv); else for (int j = 0; j < 8; ++j) yv[j] = 0.f;
      load8(dy + base, gv);
#pragma unroll
      for (int j = 0; j < 8; ++j) gv[j] *= act_df(op, xv[j], yv[j], a, b);
      store8(dx + base, gv);
    } else {
      for (long i = base; i < n; ++i) {
        const float xv = x ? E<T>::ld(x, i) : 0.f, yv = y ? E<T>::ld(y, i) : 0.f;
        E<T>::st(dx, i, E<T>::ld(dy, i) * act_df(op, xv, yv, a, b));
      }
    }
  }
}

// ------------------------------------------------------------------ softmax + CE
// One 256-thread block per row: pass 1 online max / sum, pass 2 writes the
// probabilities and the row loss (hard label: -log p[label], ignore -> 0; soft:
// -sum_j q_j log p_j).
template <typename T>
__global__ __launch_bounds__(256) void softmax_ce_prob_fwd_kernel(const T* __restrict__ x, const long* __restrict__ label,
                                                                  const T* __restrict__ soft, T* __restrict__ prob,
                                                                  T* __restrict__ loss, int V, long ignore_index) {
  __shared__ float red[8];
  const long row = blockIdx.x;
  const T* xr = x + row * V;
  float m = -INFINITY, s = 0.f;
  for (int c = threadIdx.x; c < V; c += 256) {
    const float v = E<T>::ld(xr, c);
    const float nm = fmaxf(m, v);
    s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + __expf(v - nm);
    m = nm;
  }
  // block merge of (m, s)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
    const float nm = fmaxf(m, om);
    s = (nm == -INFINITY) ? 0.f : s * __expf(m - nm) + os * __expf(om - nm);
    m = nm;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) { red[2 * w] = m; red[2 * w + 1] = s; }
  __syncthreads();
  float M = red[0], S = red[1];
  for (int i = 1; i < 4; ++i) {
    const float om = red[2 * i], os = red[2 * i + 1];
    const float nm = fmaxf(M, om);
    S = (nm == -INFINITY) ? 0.f : S * __expf(M - nm) + os * __expf(om - nm);
    M = nm;
  }
  const float lse = M + __logf(S);
  __syncthreads();
  float part = 0.f;
  for (int c = threadIdx.x; c < V; c += 256) {
    const float lp = E<T>::ld(xr, c) - lse;
    E<T>::st(prob + row * V, c, __expf(lp));
    if (soft) part -= E<T>::ld(soft + row * V, c) * lp;
  }
  if (soft) {
    part = wave_sum(part);
    if (lane == 0) red[w] = part;
    __syncthreads();
    if (threadIdx.x == 0) E<T>::st(loss, row, red[0] + red[1] + red[2] + red[3]);
  } else if (threadIdx.x == 0) {
    const long l = label[row];
    E<T>::st(loss, row, (l == ignore_index || l < 0 || l >= V) ? 0.f : lse - E<T>::ld(xr, (int)l));
  }
}

// dlogits = (p - onehot(label) | q) * dloss[row]  (ignored rows -> 0)
template <typename T>
__global__ __launch_bounds__(256) void softmax_ce_prob_bwd_kernel(const T* __restrict__ prob, const long* __restrict__ label,
                                                                  const T* __restrict__ soft, const T* __restrict__ dloss,
                                                                  T* __restrict__ dx, int V, long ignore_index) {
  const long row = blockIdx.x;
  const float g = E<T>::ld(dloss, row);
  const long l = soft ? -1 : label[row];
  const bool ign = !soft && (l == ignore_index || l < 0 || l >= V);
  for (int c = threadIdx.x; c < V; c += 256) {
    float v = E<T>::ld(prob + row * V, c);
    v -= soft ? E<T>::ld(soft + row * V, c) : (c == l ? 1.f : 0.f);
    E<T>::st(dx + row * V, c, ign ? 0.f : v * g);
  }
}

// ------------------------------------------------------------------ cast
// dtype codes: 0 f32, 1 bf16, 2 f16, 3 f64, 4 i32, 5 i64, 6 u8/bool, 7 i8, 8 i16
template <int C> struct Ty;
template <> struct Ty<0> { typedef float t; };
template <> struct Ty<1> { typedef u16 t; };
template <> struct Ty<2> { typedef _Float16 t; };
template <> struct Ty<3> { typedef double t; };
template <> struct Ty<4> { typedef int t; };
template <> struct Ty<5> { typedef long t; };
template <> struct Ty<6> { typedef unsigned char t; };
template <> struct Ty<7> { typedef signed char t; };
template <> struct Ty<8> { typedef short t; };

template <int C> __device__ __forceinline__ double to_d(typename Ty<C>::t v) { return (double)v; }
template <> __device__ __forceinline__ double to_d<1>(u16 v) { return (double)bf2f(v); }
template <int C> __device__ __forceinline__ typename Ty<C>::t from_d(double v) { return (typename Ty<C>::t)v; }
// bf16 rounds through fp32, fp16 directly from the source value (the device
// conversion order PyTorch-ROCm uses, so casts agree bit for bit)
template <> __device__ __forceinline__ u16 from_d<1>(double v) { return f2bf((float)v); }
template <> __device__ __forceinline__ unsigned char from_d<6>(double v) { return (unsigned char)(long)v; }
template <int C> constexpr bool is_int_code() { return C >= 4; }

template <int S, int D>
__global__ __launch_bounds__(256) void cast_kernel(const void* __restrict__ src, void* __restrict__ dst, long n,
                                                   int to_bool) {
  const typename Ty<S>::t* a = (const typename Ty<S>::t*)src;
  typename Ty<D>::t* b = (typename Ty<D>::t*)dst;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    if constexpr (is_int_code<S>() && is_int_code<D>()) {
      // integer -> integer: two's-complement truncation, exact for every int64
      const long v = (long)a[i];
      b[i] = (typename Ty<D>::t)(to_bool ? (v != 0) : v);
    } else {
      const double v = to_d<S>(a[i]);
      b[i] = from_d<D>(to_bool ? (v != 0.0 ? 1.0 : 0.0) : v);
    }
  }
}

// ------------------------------------------------------------------ strided gather
// out[i] (dense, nd dims of size[]) = in[base + sum_d coord_d * stride_d]; strides
// may be zero (expand / tile via a size-r axis) or negative (reverse).
struct Gather {
  long size[8];
  long stride[8];
  long base;
  int nd;
};

template <int BYTES>
__global__ __launch_bounds__(256) void gather_kernel(const char* __restrict__ in, char* __restrict__ out, long n,
                                                     Gather g) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    long r = i, off = g.base;
    for (int d = g.nd - 1; d >= 0; --d) {
      const long c = r % g.size[d];
      r /= g.size[d];
      off += c * g.stride[d];
    }
    if constexpr (BYTES == 1) out[i] = in[off];
    else if constexpr (BYTES == 2) ((u16*)out)[i] = ((const u16*)in)[off];
    else if constexpr (BYTES == 4) ((unsigned*)out)[i] = ((const unsigned*)in)[off];
    else ((unsigned long long*)out)[i] = ((const unsigned long long*)in)[off];
  }
}

// ------------------------------------------------------------------ Philox4x32-10
__device__ __forceinline__ void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)M0 * c[0], p1 = (uint64_t)M1 * c[2];
    const uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0, h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
    const uint32_t n0 = h1 ^ c[1] ^ k0, n2 = h0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = l1; c[2] = n2; c[3] = l0;
    k0 += W0; k1 += W1;
  }
}
__device__ __forceinline__ float u01(uint32_t v) { return ((v >> 8) + 0.5f) * (1.f / 16777216.f); }

// kind 0: uniform [a, b); kind 1: gaussian N(a, b^2) (Box-Muller on pairs);
// element i draws from counter block i / 4 (4 values per Philox call)
template <typename T>
__global__ __launch_bounds__(256) void random_kernel(T* __restrict__ out, long n, int kind, float a, float b,
                                                     unsigned long long seed) {
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  for (long blk = (long)blockIdx.x * 256 + threadIdx.x; blk * 4 < n; blk += (long)gridDim.x * 256) {
    uint32_t c[4] = {(uint32_t)blk, (uint32_t)((unsigned long long)blk >> 32), 0x5EEDu, 0u};
    philox(c, k0, k1);
    float v[4];
    if (kind == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = a + (b - a) * u01(c[j]);
    } else {
#pragma unroll
      for (int j = 0; j < 4; j += 2) {
        const float r = sqrtf(-2.f * __logf(u01(c[j]))), t = 6.283185307179586f * u01(c[j + 1]);
        v[j] = a + b * r * __cosf(t);
        v[j + 1] = a + b * r * __sinf(t);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (blk * 4 + j < n) E<T>::st(out, blk * 4 + j, v[j]);
  }
}

// ------------------------------------------------------------------ pointwise losses
enum Loss { HINGE = 0, HUBER, SMOOTH_L1, LOG_LOSS, MODIFIED_HUBER, SIGMOID_CE };

// forward: out_i = loss(x_i, y_i); residual r_i saved where the grad wants it
__device__ __forceinline__ float loss_f(int op, float x, float y, float a, float* res) {
  switch (op) {
    case HINGE: return fmaxf(0.f, 1.f - x * (2.f * y - 1.f));  // x: logits, y: {0,1}
    case HUBER: { const float r = y - x; *res = r; const float ar = fabsf(r); return ar <= a ? 0.5f * r * r : a * (ar - 0.5f * a); }
    case SMOOTH_L1: { const float d = x - y; *res = d; const float ad = fabsf(d), s2 = a * a;
      return ad < 1.f / s2 ? 0.5f * d * d * s2 : ad - 0.5f / s2; }
    case LOG_LOSS: return -y * __logf(x + a) - (1.f - y) * __logf(1.f - x + a);  // x: prob
    case MODIFIED_HUBER: { const float z = x * (2.f * y - 1.f); *res = z;
      return z < -1.f ? -4.f * z : (z < 1.f ? (1.f - z) * (1.f - z) : 0.f); }
    case SIGMOID_CE: return fmaxf(x, 0.f) - x * y + log1pf(__expf(-fabsf(x)));
  }
  return 0.f;
}
// d loss / d x at the same point (times the upstream grad g)
__device__ __forceinline__ float loss_dx(int op, float x, float y, float a, float res) {
  switch (op) {
    case HINGE: { const float s = 2.f * y - 1.f; return x * s < 1.f ? -s : 0.f; }
    case HUBER: { const float r = res; return fabsf(r) <= a ? -r : (r > 0.f ? -a : a); }
    case SMOOTH_L1: { const float d = res, s2 = a * a; return fabsf(d) < 1.f / s2 ? d * s2 : (d > 0.f ? 1.f : -1.f); }
    case LOG_LOSS: return -y / (x + a) + (1.f - y) / (1.f - x + a);
    case MODIFIED_HUBER: { const float z = res, s = 2.f * y - 1.f;
      return z < -1.f ? -4.f * s : (z < 1.f ? -2.f * (1.f - z) * s : 0.f); }
    case SIGMOID_CE: return sigm(x) - y;
  }
  return 0.f;
}

template <typename T>
__global__ __launch_bounds__(256) void loss_fwd_kernel(int op, const T* __restrict__ x, const T* __restrict__ y,
                                                       T* __restrict__ out, T* __restrict__ res, long n, float a) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    float r = 0.f;
    const float v = loss_f(op, E<T>::ld(x, i), E<T>::ld(y, i), a, &r);
    E<T>::st(out, i, v);
    if (res) E<T>::st(res, i, r);
  }
}

// dx_i = g[i / gdiv] * dloss/dx (gdiv > 1: one upstream grad per row of gdiv elements)
template <typename T>
__global__ __launch_bounds__(256) void loss_bwd_kernel(int op, const T* __restrict__ x, const T* __restrict__ y,
                                                       const T* __restrict__ res, const T* __restrict__ g,
                                                       T* __restrict__ dx, long n, long gdiv, float a) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float r = res ? E<T>::ld(res, i) : 0.f;
    E<T>::st(dx, i, E<T>::ld(g, i / gdiv) * loss_dx(op, E<T>::ld(x, i), E<T>::ld(y, i), a, r));
  }
}

// ------------------------------------------------------------------ sequence softmax
// x is a flat [total] column; sequence s spans [off[s], off[s+1]); one block each
template <typename T>
__global__ __launch_bounds__(256) void seq_softmax_fwd_kernel(const T* __restrict__ x, const long* __restrict__ off,
                                                              T* __restrict__ y) {
  __shared__ float red[4];
  const long b = off[blockIdx.x], e = off[blockIdx.x + 1];
  float m = -INFINITY;
  for (long i = b + threadIdx.x; i < e; i += 256) m = fmaxf(m, E<T>::ld(x, i));
  m = block_max<256>(m, red);
  float s = 0.f;
  for (long i = b + threadIdx.x; i < e; i += 256) s += __expf(E<T>::ld(x, i) - m);
  s = block_sum<256>(s, red);
  const float inv = s > 0.f ? 1.f / s : 0.f;
  for (long i = b + threadIdx.x; i < e; i += 256) E<T>::st(y, i, __expf(E<T>::ld(x, i) - m) * inv);
}

template <typename T>
__global__ __launch_bounds__(256) void seq_softmax_bwd_kernel(const T* __restrict__ y, const T* __restrict__ dy,
                                                              const long* __restrict__ off, T* __restrict__ dx) {
  __shared__ float red[4];
  const long b = off[blockIdx.x], e = off[blockIdx.x + 1];
  float s = 0.f;
  for (long i = b + threadIdx.x; i < e; i += 256) s += E<T>::ld(y, i) * E<T>::ld(dy, i);
  s = block_sum<256>(s, red);
  for (long i = b + threadIdx.x; i < e; i += 256) E<T>::st(dx, i, E<T>::ld(y, i) * (E<T>::ld(dy, i) - s));
}

}  // namespace fo
}  // namespace pa

using namespace pa;
using namespace pa::fo;

#define FO_DISPATCH(dtype, KERNEL, grid, ...)                                                  \
  do {                                                                                         \
    if ((dtype) == 1) hipLaunchKernelGGL((KERNEL<u16>), dim3(grid), dim3(256), 0, st, __VA_ARGS__); \
    else if ((dtype) == 0) hipLaunchKernelGGL((KERNEL<float>), dim3(grid), dim3(256), 0, st, __VA_ARGS__); \
    else return -1;                                                                            \
  } while (0)

PA_EXPORT int pa_act_fwd(int op, int dtype, const void* x, void* y, long n, float a, float b, hipStream_t st) {
  if (n <= 0) return 0;
  if (op < 0 || op >= NUM_ACT) return -1;
  const int g = stream_grid((n + 7) / 8, 256);
  if (dtype == 1) hipLaunchKernelGGL((act_fwd_kernel<u16>), dim3(g), dim3(256), 0, st, op, (const u16*)x, (u16*)y, n, a, b);
  else if (dtype == 0) hipLaunchKernelGGL((act_fwd_kernel<float>), dim3(g), dim3(256), 0, st, op, (const float*)x, (float*)y, n, a, b);
  else return -1;
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_act_bwd(int op, int dtype, const void* x, const void* y, const void* dy, void* dx, long n, float a,
                         float b, hipStream_t st) {
  if (n <= 0) return 0;
  if (op < 0 || op >= NUM_ACT) return -1;
  const int g = stream_grid((n + 7) / 8, 256);
  if (dtype == 1)
    hipLaunchKernelGGL((act_bwd_kernel<u16>), dim3(g), dim3(256), 0, st, op, (const u16*)x, (const u16*)y, (const u16*)dy, (u16*)dx, n, a, b);
  else if (dtype == 0)
    hipLaunchKernelGGL((act_bwd_kernel<float>), dim3(g), dim3(256), 0, st, op, (const float*)x, (const float*)y, (const float*)dy, (float*)dx, n, a, b);
  else return -1;
  PA_LAUNCH_CHECK();
}

// label: int64 [N] (hard) or null with soft [N, V]
PA_EXPORT int pa_softmax_ce_prob_fwd(int dtype, const void* x, const long* label, const void* soft, void* prob,
                                     void* loss, long N, int V, long ignore_index, hipStream_t st) {
  if (N <= 0) return 0;
  if (V <= 0 || (!label && !soft)) return -1;
  if (dtype == 1) hipLaunchKernelGGL((softmax_ce_prob_fwd_kernel<u16>), dim3(N), dim3(256), 0, st, (const u16*)x, label, (const u16*)soft, (u16*)prob, (u16*)loss, V, ignore_index);
  else if (dtype == 0) hipLaunchKernelGGL((softmax_ce_prob_fwd_kernel<float>), dim3(N), dim3(256), 0, st, (const float*)x, label, (const float*)soft, (float*)prob, (float*)loss, V, ignore_index);
  else return -1;
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_softmax_ce_prob_bwd(int dtype, const void* prob, const long* label, const void* soft,
                                     const void* dloss, void* dx, long N, int V, long ignore_index, hipStream_t st) {
  if (N <= 0) return 0;
  if (V <= 0 || (!label && !soft)) return -1;
  if (dtype == 1) hipLaunchKernelGGL((softmax_ce_prob_bwd_kernel<u16>), dim3(N), dim3(256), 0, st, (const u16*)prob, label, (const u16*)soft, (const u16*)dloss, (u16*)dx, V, ignore_index);
  else if (dtype == 0) hipLaunchKernelGGL((softmax_ce_prob_bwd_kernel<float>), dim3(N), dim3(256), 0, st, (const float*)prob, label, (const float*)soft, (const float*)dloss, (float*)dx, V, ignore_index);
  else return -1;
  PA_LAUNCH_CHECK();
}

template <int S>
static int cast_from(int dst, const void* src, void* out, long n, int to_bool, int g, hipStream_t st) {
  switch (dst) {
#define PA_CAST_CASE(D) \
    case D: hipLaunchKernelGGL((cast_kernel<S, D>), dim3(g), dim3(256), 0, st, src, out, n, to_bool); break;
    PA_CAST_CASE(0) PA_CAST_CASE(1) PA_CAST_CASE(2) PA_CAST_CASE(3) PA_CAST_CASE(4) PA_CAST_CASE(5) PA_CAST_CASE(6)
    PA_CAST_CASE(7) PA_CAST_CASE(8)
#undef PA_CAST_CASE
    default: return -1;
  }
  return (int)hipGetLastError();
}

PA_EXPORT int pa_cast_any(int src_dt, int dst_dt, const void* src, void* dst, long n, int to_bool, hipStream_t st) {
  if (n <= 0) return 0;
  const int g = stream_grid(n, 256);
  switch (src_dt) {
    case 0: return cast_from<0>(dst_dt, src, dst, n, to_bool, g, st);
    case 1: return cast_from<1>(dst_dt, src, dst, n, to_bool, g, st);
    case 2: return cast_from<2>(dst_dt, src, dst, n, to_bool, g, st);
    case 3: return cast_from<3>(dst_dt, src, dst, n, to_bool, g, st);
    case 4: return cast_from<4>(dst_dt, src, dst, n, to_bool, g, st);
    case 5: return cast_from<5>(dst_dt, src, dst, n, to_bool, g, st);
    case 6: return cast_from<6>(dst_dt, src, dst, n, to_bool, g, st);
    case 7: return cast_from<7>(dst_dt, src, dst, n, to_bool, g, st);
    case 8: return cast_from<8>(dst_dt, src, dst, n, to_bool, g, st);
  }
  return -1;
}

// sizes / strides in elements; the caller guarantees every reachable source offset
// lies inside the source allocation (the Python wrapper checks min / max offsets)
PA_EXPORT int pa_strided_gather(int elem_bytes, const void* src, void* dst, int nd, const long* sizes,
                                const long* strides, long base, hipStream_t st) {
  if (nd < 1 || nd > 8) return -1;
  Gather g{};
  long n = 1;
  for (int d = 0; d < nd; ++d) {
    if (sizes[d] < 0) return -1;
    g.size[d] = sizes[d];
    g.stride[d] = strides[d];
    n *= sizes[d];
  }
  g.nd = nd;
  g.base = base;
  if (n == 0) return 0;
  const int grid = stream_grid(n, 256);
  switch (elem_bytes) {
    case 1: hipLaunchKernelGGL((gather_kernel<1>), dim3(grid), dim3(256), 0, st, (const char*)src, (char*)dst, n, g); break;
    case 2: hipLaunchKernelGGL((gather_kernel<2>), dim3(grid), dim3(256), 0, st, (const char*)src, (char*)dst, n, g); break;
    case 4: hipLaunchKernelGGL((gather_kernel<4>), dim3(grid), dim3(256), 0, st, (const char*)src, (char*)dst, n, g); break;
    case 8: hipLaunchKernelGGL((gather_kernel<8>), dim3(grid), dim3(256), 0, st, (const char*)src, (char*)dst, n, g); break;
    default: return -1;
  }
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_random(int dtype, void* out, long n, int kind, float a, float b, unsigned long long seed,
                        hipStream_t st) {
  if (n <= 0) return 0;
  if (kind != 0 && kind != 1) return -1;
  const int g = stream_grid((n + 3) / 4, 256);
  if (dtype == 1) hipLaunchKernelGGL((random_kernel<u16>), dim3(g), dim3(256), 0, st, (u16*)out, n, kind, a, b, seed);
  else if (dtype == 0) hipLaunchKernelGGL((random_kernel<float>), dim3(g), dim3(256), 0, st, (float*)out, n, kind, a, b, seed);
  else return -1;
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_loss_fwd(int op, int dtype, const void* x, const void* y, void* out, void* res, long n, float a,
                          hipStream_t st) {
  if (n <= 0) return 0;
  if (op < 0 || op > SIGMOID_CE) return -1;
  const int g = stream_grid(n, 256);
  if (dtype == 1) hipLaunchKernelGGL((loss_fwd_kernel<u16>), dim3(g), dim3(256), 0, st, op, (const u16*)x, (const u16*)y, (u16*)out, (u16*)res, n, a);
  else if (dtype == 0) hipLaunchKernelGGL((loss_fwd_kernel<float>), dim3(g), dim3(256), 0, st, op, (const float*)x, (const float*)y, (float*)out, (float*)res, n, a);
  else return -1;
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_loss_bwd(int op, int dtype, const void* x, const void* y, const void* res, const void* g, void* dx,
                          long n, long gdiv, float a, hipStream_t st) {
  if (n <= 0) return 0;
  if (op < 0 || op > SIGMOID_CE || gdiv < 1) return -1;
  const int grid = stream_grid(n, 256);
  if (dtype == 1) hipLaunchKernelGGL((loss_bwd_kernel<u16>), dim3(grid), dim3(256), 0, st, op, (const u16*)x, (const u16*)y, (const u16*)res, (const u16*)g, (u16*)dx, n, gdiv, a);
  else if (dtype == 0) hipLaunchKernelGGL((loss_bwd_kernel<float>), dim3(grid), dim3(256), 0, st, op, (const float*)x, (const float*)y, (const float*)res, (const float*)g, (float*)dx, n, gdiv, a);
  else return -1;
  PA_LAUNCH_CHECK();
}

// off: device int64 [nseq + 1]
PA_EXPORT int pa_seq_softmax_fwd(int dtype, const void* x, const long* off, void* y, long nseq, hipStream_t st) {
  if (nseq <= 0) return 0;
  if (dtype == 1) hipLaunchKernelGGL((seq_softmax_fwd_kernel<u16>), dim3(nseq), dim3(256), 0, st, (const u16*)x, off, (u16*)y);
  else if (dtype == 0) hipLaunchKernelGGL((seq_softmax_fwd_kernel<float>), dim3(nseq), dim3(256), 0, st, (const float*)x, off, (float*)y);
  else return -1;
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_seq_softmax_bwd(int dtype, const void* y, const void* dy, const long* off, void* dx, long nseq,
                                 hipStream_t st) {
  if (nseq <= 0) return 0;
  if (dtype == 1) hipLaunchKernelGGL((seq_softmax_bwd_kernel<u16>), dim3(nseq), dim3(256), 0, st, (const u16*)y, (const u16*)dy, off, (u16*)dx);
  else if (dtype == 0) hipLaunchKernelGGL((seq_softmax_bwd_kernel<float>), dim3(nseq), dim3(256), 0, st, (const float*)y, (const float*)dy, off, (float*)dx);
  else return -1;
  PA_LAUNCH_CHECK();
}
