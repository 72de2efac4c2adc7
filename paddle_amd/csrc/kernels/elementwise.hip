// Memory-bound fused elementwise kernels for gfx950: rotary embedding, SwiGLU,
// embedding gather/scatter-add, and cast.  All of them move 16 B per lane per
// access (guide Guideline 13) and use grid-stride loops capped at 2048 blocks.
//
// Parity: the reference has no rotary/SwiGLU (north-star ops); embedding
// follows lookup_table (paddle/fluid/operators/lookup_table_op.cu:89-166,
// dense grad by atomics) re-derived for wave64 with 16-byte row vectors.
#include "common.h"

namespace pa {

// ---------------------------------------------------------------- rotary
// x: [B*S tokens, nh_total heads, D] with token stride x_ts (elements), head stride D;
// heads [0, n_rot) are rotated, heads [n_rot, nh_total) are copied unchanged (used
// to repack [q|k|v] -> rotated [q|k] + v in one pass).  y may alias x (in place).
// neox / rotate-half convention: pairs (i, i + D/2).  cos/sin tables: [S, D/2] fp32.
// pos: optional int64 [B*S] position ids (null => position = s).
// sign = +1 forward, -1 backward (rotation by -theta).  TI/TO allow fp32 -> bf16
// (fused dq-accumulator cast + inverse rotation in the attention backward).
template <typename TI, typename TO>
__global__ void rope_kernel(const TI* x, long x_ts, TO* y, long y_ts,
                            const float* __restrict__ cosT, const float* __restrict__ sinT,
                            const long* __restrict__ pos, long B, long S, int nh, int n_rot,
                            int D, float sign) {
  const int half = D / 2;
  const int cpp = half / 8;  // 8-wide chunks per head half
  const long total = B * S * nh * cpp;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % cpp);
    long t = i / cpp;
    const int h = (int)(t % nh);
    t /= nh;  // token index b*S + s
    const TI* xb = x + t * x_ts + (long)h * D + c * 8;
    TO* yb = y + t * y_ts + (long)h * D + c * 8;
    float a[8], b[8];
    load8(xb, a);
    load8(xb + half, b);
    if (h < n_rot) {
      const long s = t % S;
      const long p = pos ? pos[t] : s;
      float co[8], si[8];
      load8(cosT + p * half + c * 8, co);
      load8(sinT + p * half + c * 8, si);
      float oa[8], ob[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float sn = sign * si[j];
        oa[j] = a[j] * co[j] - b[j] * sn;
        ob[j] = b[j] * co[j] + a[j] * sn;
      }
      store8(yb, oa);
      store8(yb + half, ob);
    } else {
      store8(yb, a);
      store8(yb + half, b);
    }
  }
}

// ---------------------------------------------------------------- SwiGLU
// gu: [N, 2I] = [gate | up]; out: [N, I] = silu(gate) * up
template <typename T>
__global__ void swiglu_fwd_kernel(const T* __restrict__ gu, T* __restrict__ out, long N, int I) {
  const int cpr = I / 8;
  const long total = N * cpr;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long r = i / cpr;
    const int c = (int)(i % cpr) * 8;
    float g[8], u[8], o[8];
    load8(gu + r * 2 * I + c, g);
    load8(gu + r * 2 * I + I + c, u);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = g[j] / (1.f + __expf(-g[j])) * u[j];
    store8(out + r * I + c, o);
  }
}

template <typename T>
__global__ void swiglu_bwd_kernel(const T* __restrict__ gu, const T* __restrict__ dout,
                                  T* __restrict__ dgu, long N, int I) {
  const int cpr = I / 8;
  const long total = N * cpr;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long r = i / cpr;
    const int c = (int)(i % cpr) * 8;
    float g[8], u[8], d[8], dg[8], du[8];
    load8(gu + r * 2 * I + c, g);
    load8(gu + r * 2 * I + I + c, u);
    load8(dout + r * I + c, d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float sg = 1.f / (1.f + __expf(-g[j]));
      const float silu = g[j] * sg;
      du[j] = d[j] * silu;
      dg[j] = d[j] * u[j] * sg * (1.f + g[j] * (1.f - sg));
    }
    store8(dgu + r * 2 * I + c, dg);
    store8(dgu + r * 2 * I + I + c, du);
  }
}

// ---------------------------------------------------------------- embedding
template <typename T>
__global__ void embedding_fwd_kernel(const long* __restrict__ ids, const T* __restrict__ W,
                                     T* __restrict__ out, long N, int H, long padding_idx) {
  const int cpr = H / 8;
  const long total = N * cpr;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long r = i / cpr;
    const int c = (int)(i % cpr) * 8;
    const long id = ids[r];
    float v[8];
    if (id == padding_idx) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = 0.f;
    } else {
      load8(W + id * H + c, v);
    }
    store8(out + r * H + c, v);
  }
}

// dW (fp32 accumulator) += scatter(dout).  One wave per token row: each lane adds
// 4 contiguous floats -> a wave instruction covers 256 contiguous bytes, the
// shape that runs at the full float-atomic rate (MI355X_MICROARCH Global float atomics).
template <typename T>
__global__ void embedding_bwd_kernel(const long* __restrict__ ids, const T* __restrict__ dout,
                                     float* __restrict__ dW, long N, int H, long padding_idx) {
  const int lane = threadIdx.x & 63;
  const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long nwaves = ((long)gridDim.x * blockDim.x) >> 6;
  for (long r = wave; r < N; r += nwaves) {
    const long id = ids[r];
    if (id == padding_idx) continue;
    for (int c = lane * 4; c < H; c += 256) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (c + j < H) atomicAdd(&dW[id * H + c + j], IO<T>::ld(dout, r * H + c + j));
    }
  }
}

template <typename TI, typename TO>
__global__ void cast_kernel(const TI* __restrict__ in, TO* __restrict__ out, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    IO<TO>::st(out, i, IO<TI>::ld(in, i));
}

}  // namespace pa

using namespace pa;

// in/out dtype: 0 fp32, 1 bf16
PA_EXPORT int pa_rope(int in_dtype, int out_dtype, const void* x, long x_ts, void* y, long y_ts,
                      const float* cosT, const float* sinT, const long* pos, long B, long S,
                      int nh, int n_rot, int D, int backward, hipStream_t st) {
  if (D % 16) return (int)hipErrorInvalidValue;
  const long work = B * S * nh * (D / 16);
  const int g = stream_grid(work, 256);
  const float sign = backward ? -1.f : 1.f;
#define PA_R(TI, TO) \
  hipLaunchKernelGGL((rope_kernel<TI, TO>), dim3(g), dim3(256), 0, st, (const TI*)x, x_ts, (TO*)y, y_ts, cosT, sinT, pos, B, S, nh, n_rot, D, sign)
  if (in_dtype == 1 && out_dtype == 1) PA_R(u16, u16);
  else if (in_dtype == 0 && out_dtype == 1) PA_R(float, u16);
  else if (in_dtype == 0 && out_dtype == 0) PA_R(float, float);
  else PA_R(u16, float);
#undef PA_R
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_swiglu_fwd(int dtype, const void* gu, void* out, long N, int I, hipStream_t st) {
  if (I % 8) return (int)hipErrorInvalidValue;
  const int g = stream_grid(N * (I / 8), 256);
  if (dtype == 1)
    hipLaunchKernelGGL(swiglu_fwd_kernel<u16>, dim3(g), dim3(256), 0, st, (const u16*)gu, (u16*)out, N, I);
  else
    hipLaunchKernelGGL(swiglu_fwd_kernel<float>, dim3(g), dim3(256), 0, st, (const float*)gu, (float*)out, N, I);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_swiglu_bwd(int dtype, const void* gu, const void* dout, void* dgu, long N, int I,
                            hipStream_t st) {
  if (I % 8) return (int)hipErrorInvalidValue;
  const int g = stream_grid(N * (I / 8), 256);
  if (dtype == 1)
    hipLaunchKernelGGL(swiglu_bwd_kernel<u16>, dim3(g), dim3(256), 0, st, (const u16*)gu, (const u16*)dout, (u16*)dgu, N, I);
  else
    hipLaunchKernelGGL(swiglu_bwd_kernel<float>, dim3(g), dim3(256), 0, st, (const float*)gu, (const float*)dout, (float*)dgu, N, I);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_embedding_fwd(int dtype, const long* ids, const void* W, void* out, long N, int H,
                               long padding_idx, hipStream_t st) {
  if (H % 8) return (int)hipErrorInvalidValue;
  const int g = stream_grid(N * (H / 8), 256);
  if (dtype == 1)
    hipLaunchKernelGGL(embedding_fwd_kernel<u16>, dim3(g), dim3(256), 0, st, ids, (const u16*)W, (u16*)out, N, H, padding_idx);
  else
    hipLaunchKernelGGL(embedding_fwd_kernel<float>, dim3(g), dim3(256), 0, st, ids, (const float*)W, (float*)out, N, H, padding_idx);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_embedding_bwd(int dtype, const long* ids, const void* dout, float* dW, long N,
                               int H, long padding_idx, hipStream_t st) {
  long g = (N + 3) / 4;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  if (dtype == 1)
    hipLaunchKernelGGL(embedding_bwd_kernel<u16>, dim3(g), dim3(256), 0, st, ids, (const u16*)dout, dW, N, H, padding_idx);
  else
    hipLaunchKernelGGL(embedding_bwd_kernel<float>, dim3(g), dim3(256), 0, st, ids, (const float*)dout, dW, N, H, padding_idx);
  PA_LAUNCH_CHECK();
}

// in_dtype/out_dtype: 0 fp32, 1 bf16
PA_EXPORT int pa_cast(int in_dtype, int out_dtype, const void* in, void* out, long n, hipStream_t st) {
  const int g = stream_grid(n, 256);
  if (in_dtype == 0 && out_dtype == 1)
    hipLaunchKernelGGL((cast_kernel<float, u16>), dim3(g), dim3(256), 0, st, (const float*)in, (u16*)out, n);
  else if (in_dtype == 1 && out_dtype == 0)
    hipLaunchKernelGGL((cast_kernel<u16, float>), dim3(g), dim3(256), 0, st, (const u16*)in, (float*)out, n);
  else
    return (int)hipErrorInvalidValue;
  PA_LAUNCH_CHECK();
}
