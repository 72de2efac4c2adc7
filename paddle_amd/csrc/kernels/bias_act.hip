// Bias-gradient and GELU(tanh) kernels for the biased linear layers (GPT / ERNIE
// blocks) on gfx950.
//
// Parity: the reference's fc/elementwise_add backward reduces the bias gradient
// with a generic column reduction (paddle/fluid/operators/elementwise_op_function.h
// ElemwiseGradCompute / math/math_function.cu ColwiseSum) and runs the activation
// backward as a separate pass (activation_op.h GeluGradFunctor lineage).  Here the
// activation backward and the bias reduction are ONE pass over dY:
//   dZ = dY * gelu'(Z)   (written once, consumed by the dX / dW GEMMs)
//   db = sum_rows(dZ)    (fp32 partial rows per row-block, then a column sum)
// Each wave streams 1 KB of a row per load (8 bf16 per lane, 512 columns per
// block), rows split over a 2-D grid sized to fill all 256 CUs; partial sums stay
// in registers, fold through LDS once per block.
#include "common.h"

namespace pa {

constexpr float kGeluK0 = 0.7978845608028654f;  // sqrt(2/pi)
constexpr float kGeluK1 = 0.044715f;

__device__ __forceinline__ float gelu_tanh(float z) {
  const float u = kGeluK0 * (z + kGeluK1 * z * z * z);
  const float t = 1.f - 2.f / (1.f + __expf(2.f * u));
  return 0.5f * z * (1.f + t);
}

__device__ __forceinline__ float gelu_tanh_grad(float z) {
  const float z2 = z * z;
  const float u = kGeluK0 * z * (1.f + kGeluK1 * z2);
  const float t = 1.f - 2.f / (1.f + __expf(2.f * u));
  return 0.5f * (1.f + t) + 0.5f * z * (1.f - t * t) * kGeluK0 * (1.f + 3.f * kGeluK1 * z2);
}

template <typename T>
__global__ __launch_bounds__(256) void gelu_fwd_kernel(const T* __restrict__ z, T* __restrict__ g, long n8) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    float v[8], o[8];
    load8(z + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = gelu_tanh(v[j]);
    store8(g + i * 8, o);
  }
}

// grid (ceil(H/512), G); block 256 = 4 waves striding the block's rows.
template <typename T, bool ACT>
__global__ __launch_bounds__(256) void bias_act_bwd_kernel(
    const T* __restrict__ dy, const T* __restrict__ z, T* __restrict__ dz,
    float* __restrict__ part, long N, int H, long rpb) {
  __shared__ __attribute__((aligned(16))) float red[4][512];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * 512 + lane * 8;
  const long r0 = (long)blockIdx.y * rpb;
  const long r1 = min(N, r0 + rpb);
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  if (c < H) {
    long r = r0 + wv;
    // two rows per trip: two independent 16-byte loads in flight per lane
    for (; r + 4 < r1; r += 8) {
      float d0[8], d1[8];
      load8(dy + r * H + c, d0);
      load8(dy + (r + 4) * H + c, d1);
      if (ACT) {
        float v0[8], v1[8];
        load8(z + r * H + c, v0);
        load8(z + (r + 4) * H + c, v1);
#pragma unroll
        for (int j = 0; j < 8; ++j) { d0[j] *= gelu_tanh_grad(v0[j]); d1[j] *= gelu_tanh_grad(v1[j]); }
        store8(dz + r * H + c, d0);
        store8(dz + (r + 4) * H + c, d1);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += d0[j] + d1[j];
    }
    if (r < r1) {
      float d0[8];
      load8(dy + r * H + c, d0);
      if (ACT) {
        float v0[8];
        load8(z + r * H + c, v0);
#pragma unroll
        for (int j = 0; j < 8; ++j) d0[j] *= gelu_tanh_grad(v0[j]);
        store8(dz + r * H + c, d0);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += d0[j];
    }
  }
  *reinterpret_cast<f32x4*>(&red[wv][lane * 8]) = f32x4{acc[0], acc[1], acc[2], acc[3]};
  *reinterpret_cast<f32x4*>(&red[wv][lane * 8 + 4]) = f32x4{acc[4], acc[5], acc[6], acc[7]};
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 256) {
    const int cc = blockIdx.x * 512 + i;
    if (cc < H) part[(long)blockIdx.y * H + cc] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
  }
}

// out[c] = sum_g part[g, c]; 64 columns per block, 4 waves split the G rows.
template <typename T>
__global__ __launch_bounds__(256) void part_colsum_kernel(const float* __restrict__ part, T* __restrict__ out, int G, int H) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (c < H)
    for (int g = w; g < G; g += 4) s += part[(long)g * H + c];
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && c < H) IO<T>::st(out, c, red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane]);
}

}  // namespace pa

using namespace pa;

// Row-block count for an [N, H] bias reduction: ~2048 blocks over the chip, at
// least 32 rows per block (the fp32 partials stay <= 1/16 of dY's bytes).  The host sizes `part` as G * H floats with this.
PA_EXPORT int pa_bias_grad_blocks(long N, int H) {
  const long tiles = (H + 511) / 512;
  long G = 2048 / tiles;
  const long gmax = (N + 31) / 32;
  if (G > gmax) G = gmax;
  if (G < 1) G = 1;
  const long rpb = (N + G - 1) / G;
  return (int)((N + rpb - 1) / rpb);
}

PA_EXPORT int pa_gelu_fwd(int dtype, const void* z, void* g, long n, hipStream_t st) {
  if (n % 8) return (int)hipErrorInvalidValue;
  const int grid = stream_grid(n / 8, 256);
  if (dtype == 1)
    hipLaunchKernelGGL(gelu_fwd_kernel<u16>, dim3(grid), dim3(256), 0, st, (const u16*)z, (u16*)g, n / 8);
  else
    hipLaunchKernelGGL(gelu_fwd_kernel<float>, dim3(grid), dim3(256), 0, st, (const float*)z, (float*)g, n / 8);
  PA_LAUNCH_CHECK();
}

// act: 0 = none (db = colsum(dy); z, dz unused), 1 = gelu(tanh) (dz = dy * gelu'(z)).
// part: fp32 workspace of pa_bias_grad_blocks(N, H) * H floats.  H % 8 == 0.
PA_EXPORT int pa_bias_act_bwd(int dtype, int act, const void* dy, const void* z, void* dz, void* db,
                              float* part, long N, int H, hipStream_t st) {
  if (H % 8 || N < 1) return (int)hipErrorInvalidValue;
  const int G = pa_bias_grad_blocks(N, H);
  const long rpb = (N + G - 1) / G;
  dim3 grid((H + 511) / 512, G);
#define PA_B(T_, ACT_) \
  hipLaunchKernelGGL((bias_act_bwd_kernel<T_, ACT_>), grid, dim3(256), 0, st, (const T_*)dy, (const T_*)z, (T_*)dz, part, N, H, rpb)
  if (dtype == 1) { if (act) PA_B(u16, true); else PA_B(u16, false); }
  else { if (act) PA_B(float, true); else PA_B(float, false); }
#undef PA_B
  if (db) {
    if (dtype == 1)
      hipLaunchKernelGGL(part_colsum_kernel<u16>, dim3((H + 63) / 64), dim3(256), 0, st, part, (u16*)db, G, H);
    else
      hipLaunchKernelGGL(part_colsum_kernel<float>, dim3((H + 63) / 64), dim3(256), 0, st, part, (float*)db, G, H);
  }
  PA_LAUNCH_CHECK();
}
