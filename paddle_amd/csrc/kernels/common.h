// Shared device helpers for the paddle_amd CDNA4 (gfx950) kernel library.
//
// Everything here is written for wave64: lane = threadIdx.x & 63, reductions
// span 64 lanes via DPP/ds_swizzle-backed __shfl_xor, and bf16 data is always
// moved as 16-byte vectors (8 x bf16) per lane (guide: Guideline 13).
//
// Reference parity notes: the reference's block reductions hard-code a 32-lane
// warp (paddle/fluid/platform/cuda_device_function.h:83-110); these helpers are
// re-derived for 64-lane waves instead.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PA_EXPORT extern "C" __attribute__((visibility("default")))

namespace pa {

typedef __bf16 bf16;
typedef unsigned short u16;
typedef u16 u16x8 __attribute__((ext_vector_type(8)));
typedef u16 u16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short i16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(u16 v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
// Round-to-nearest-even f32 -> bf16 (NaN preserved as quiet NaN).
__device__ __forceinline__ u16 f2bf(float f) {
  __bf16 b = (__bf16)f;  // lowers to v_cvt_pk_bf16_f32 on gfx950
  return __builtin_bit_cast(u16, b);
}
__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

// dtype-generic load/store of one scalar: T is float or u16 (bf16 bits) or _Float16 bits
template <typename T> struct IO;
template <> struct IO<float> {
  static __device__ __forceinline__ float ld(const float* p, long i) { return p[i]; }
  static __device__ __forceinline__ void st(float* p, long i, float v) { p[i] = v; }
};
template <> struct IO<u16> {
  static __device__ __forceinline__ float ld(const u16* p, long i) { return bf2f(p[i]); }
  static __device__ __forceinline__ void st(u16* p, long i, float v) { p[i] = f2bf(v); }
};

// Load 8 consecutive elements as floats (16 B for bf16, 32 B for f32).
__device__ __forceinline__ void load8(const u16* p, float (&o)[8]) {
  u16x8 v = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = bf2f(v[j]);
}
__device__ __forceinline__ void load8(const float* p, float (&o)[8]) {
  f32x4 a = *reinterpret_cast<const f32x4*>(p);
  f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) { o[j] = a[j]; o[j + 4] = b[j]; }
}
__device__ __forceinline__ void store8(u16* p, const float (&o)[8]) {
  u16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = f2bf(o[j]);
  *reinterpret_cast<u16x8*>(p) = v;
}
__device__ __forceinline__ void store8(float* p, const float (&o)[8]) {
  f32x4 a, b;
#pragma unroll
  for (int j = 0; j < 4; ++j) { a[j] = o[j]; b[j] = o[j + 4]; }
  *reinterpret_cast<f32x4*>(p) = a;
  *reinterpret_cast<f32x4*>(p + 4) = b;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64). `red` must hold NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_sum(v);
  if (NT == 64) return v;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += red[i];
  return t;
}
template <int NT>
__device__ __forceinline__ float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_max(v);
  if (NT == 64) return v;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = -INFINITY;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t = fmaxf(t, red[i]);
  return t;
}

// BatchNorm backward statistics taken in the epilogue of the convolution whose data
// gradient dY' is the gradient of the BN output y = relu(BN(x) [+ res]):
//   part[tile][0][c] = sum g,  part[tile][1][c] = sum g * (x - mean),  g = dY' * mask
// mask: y > 0 (residual layers, y kept), fmaf(x, rstd*w, b - mean*rstd*w) > 0 (relu,
// recomputed as the forward evaluated it), or 1 (no relu) -- what bn_reduce_kernel<true>
// computes, so the BN backward skips its reduction pass over dY and x.
struct BnBwdSrc {
  const u16* x;       // BN input [rows, C] (null: statistics off)
  const u16* y;       // BN output (mask source) or null
  const float* mean;  // [C]
  const float* rstd;  // [C]
  const void* w;      // [C] fp32 / bf16 per wdt, or null (1)
  const void* b;      // [C] or null (0)
  int wdt;
  int relu;
};

// per-channel (mean, mask scale, mask shift) of channel c
__device__ __forceinline__ void bn_bwd_coef(const BnBwdSrc& s, int c, float& mean, float& sc, float& sf) {
  mean = s.mean[c];
  const float ww = s.w ? (s.wdt ? bf2f(((const u16*)s.w)[c]) : ((const float*)s.w)[c]) : 1.f;
  const float bb = s.b ? (s.wdt ? bf2f(((const u16*)s.b)[c]) : ((const float*)s.b)[c]) : 0.f;
  sc = s.rstd[c] * ww;
  sf = bb - mean * sc;
}

// Grid size for memory-bound grid-stride kernels (guide Guideline 11).
static inline int stream_grid(long work_items, int block) {
  long g = (work_items + block - 1) / block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace pa

#define PA_LAUNCH_CHECK() return (int)hipGetLastError()
