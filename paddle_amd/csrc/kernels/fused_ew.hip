// fused_elemwise_activation (reference operators/fused_elemwise_activation_op.h,
// CompoundFunctors): Out = Binary(X, Unary(Y)) ("elementwise_*, act") or
// Out = Unary(Binary(X, Y)) ("act, elementwise_*") with Binary in {add, mul},
// Unary in {relu, scale}, Y broadcast over X as [pre, n, post] (Paddle axis rule).
// One pass forward (optionally storing IntermediateOut) and one pass backward that
// writes dX and an X-shaped dY (the caller folds the broadcast dims).
#include "common.h"

namespace pa {
namespace {

__device__ __forceinline__ float un(int uop, float v, float s) { return uop == 0 ? fmaxf(v, 0.f) : v * s; }
__device__ __forceinline__ float dun(int uop, float v, float s) { return uop == 0 ? (v > 0.f ? 1.f : 0.f) : s; }
__device__ __forceinline__ float bin(int bop, float a, float b) { return bop == 0 ? a + b : a * b; }

template <typename T>
__global__ __launch_bounds__(256) void few_fwd(int mode, int bop, int uop, float s, const T* __restrict__ x,
                                               const T* __restrict__ y, T* __restrict__ out, T* __restrict__ inter,
                                               long n, long ny, long post) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float xv = IO<T>::ld(x, i), yv = IO<T>::ld(y, (i / post) % ny);
    float it, o;
    if (mode == 0) {
      it = un(uop, yv, s);
      o = bin(bop, xv, it);
    } else {
      it = bin(bop, xv, yv);
      o = un(uop, it, s);
    }
    IO<T>::st(out, i, o);
    if (inter) IO<T>::st(inter, i, it);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void few_bwd(int mode, int bop, int uop, float s, const T* __restrict__ x,
                                               const T* __restrict__ y, const T* __restrict__ dout,
                                               T* __restrict__ dx, float* __restrict__ dyf, long n, long ny,
                                               long post) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float xv = IO<T>::ld(x, i), yv = IO<T>::ld(y, (i / post) % ny), d = IO<T>::ld(dout, i);
    float gx, gy;
    if (mode == 0) {
      const float it = un(uop, yv, s);
      const float di = bop == 0 ? d : d * xv;
      gx = bop == 0 ? d : d * it;
      gy = di * dun(uop, yv, s);
    } else {
      const float it = bin(bop, xv, yv);
      const float di = d * dun(uop, it, s);
      gx = bop == 0 ? di : di * yv;
      gy = bop == 0 ? di : di * xv;
    }
    if (dx) IO<T>::st(dx, i, gx);
    if (dyf) dyf[i] = gy;
  }
}

}  // namespace
}  // namespace pa

using namespace pa;

// dtype 0 f32, 1 bf16; mode 0: Binary(X, Unary(Y)), 1: Unary(Binary(X, Y));
// bop 0 add, 1 mul; uop 0 relu, 1 scale.  inter may be null.
PA_EXPORT int pa_fused_ew_act(int dtype, int mode, int bop, int uop, float s, const void* x, const void* y, void* out,
                              void* inter, long n, long ny, long post, hipStream_t st) {
  if (n < 0 || ny <= 0 || post <= 0 || mode < 0 || mode > 1 || bop < 0 || bop > 1 || uop < 0 || uop > 1) return -1;
  if (n == 0) return 0;
  const dim3 g(stream_grid(n, 256));
  if (dtype == 0)
    hipLaunchKernelGGL(few_fwd<float>, g, dim3(256), 0, st, mode, bop, uop, s, (const float*)x, (const float*)y,
                       (float*)out, (float*)inter, n, ny, post);
  else if (dtype == 1)
    hipLaunchKernelGGL(few_fwd<u16>, g, dim3(256), 0, st, mode, bop, uop, s, (const u16*)x, (const u16*)y, (u16*)out,
                       (u16*)inter, n, ny, post);
  else
    return -1;
  PA_LAUNCH_CHECK();
}

// dyf: fp32, X-shaped (null when dY is not needed); dx may be null
PA_EXPORT int pa_fused_ew_act_bwd(int dtype, int mode, int bop, int uop, float s, const void* x, const void* y,
                                  const void* dout, void* dx, float* dyf, long n, long ny, long post, hipStream_t st) {
  if (n < 0 || ny <= 0 || post <= 0 || mode < 0 || mode > 1 || bop < 0 || bop > 1 || uop < 0 || uop > 1) return -1;
  if (n == 0) return 0;
  const dim3 g(stream_grid(n, 256));
  if (dtype == 0)
    hipLaunchKernelGGL(few_bwd<float>, g, dim3(256), 0, st, mode, bop, uop, s, (const float*)x, (const float*)y,
                       (const float*)dout, (float*)dx, dyf, n, ny, post);
  else if (dtype == 1)
    hipLaunchKernelGGL(few_bwd<u16>, g, dim3(256), 0, st, mode, bop, uop, s, (const u16*)x, (const u16*)y,
                       (const u16*)dout, (u16*)dx, dyf, n, ny, post);
  else
    return -1;
  PA_LAUNCH_CHECK();
}
