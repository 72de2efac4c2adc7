// Fused optimizer updates for gfx950 over flat (multi-tensor) buffers.
//
// Parity: reference adam/momentum/sgd ops (paddle/fluid/operators/adam_op.h:35-321
// ForRange<AdamFunctor> 1024-thread blocks; momentum_op.cu:67; sgd_op.cu:73).
// Redesigned: parameters, grads and optimizer state live in ONE flat buffer each
// (the fused-parameter layout the sharded DP engine uses), so a whole model's
// step is one grid-stride launch; bf16 grads are read and the bf16 model copy is
// written in the same pass as the fp32 master update (no separate cast kernel).
// lr / beta-pow may come from device memory (static-graph ops) or by value.
#include <stdlib.h>

#include <algorithm>

#include "common.h"

namespace pa {

template <typename TG, typename TP>
__global__ void adamw_kernel(float* __restrict__ p, const TG* __restrict__ g, float* __restrict__ m,
                             float* __restrict__ v, TP* __restrict__ pout, long n, float lr,
                             const float* __restrict__ lr_ptr, float b1, float b2, float eps,
                             float wd, float bc1, float bc2, const float* __restrict__ b1pow,
                             const float* __restrict__ b2pow, long decay_end, float gscale,
                             const float* __restrict__ gscale_ptr, int lr_t_eps) {
  float lr_ = lr_ptr ? lr_ptr[0] : lr;
  float c1 = b1pow ? 1.f - b1pow[0] : bc1;
  float c2 = b2pow ? 1.f - b2pow[0] : bc2;
  const float gs = gscale_ptr ? gscale_ptr[0] * gscale : gscale;
  const float step = lr_ / c1;
  const float rc2 = rsqrtf(c2);
  // lr_t_eps: Kingma/Paddle form lr_t = lr*sqrt(c2)/c1, p -= lr_t*m/(sqrt(v)+eps)
  // (adam_op.h); otherwise eps is added to the bias-corrected sqrt(v/c2) (AdamW form).
  const float eps_ = lr_t_eps ? eps * rc2 : eps;
  const long n4 = n / 4;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (long)gridDim.x * blockDim.x) {
    const long e = i * 4;
    f32x4 pp = *reinterpret_cast<f32x4*>(p + e);
    f32x4 mm = *reinterpret_cast<f32x4*>(m + e);
    f32x4 vv = *reinterpret_cast<f32x4*>(v + e);
    float gg[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) gg[j] = IO<TG>::ld(g, e + j) * gs;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      mm[j] = b1 * mm[j] + (1.f - b1) * gg[j];
      vv[j] = b2 * vv[j] + (1.f - b2) * gg[j] * gg[j];
      const float decay = (e + j) < decay_end ? wd : 0.f;
      pp[j] = pp[j] * (1.f - lr_ * decay) - step * mm[j] / (sqrtf(vv[j]) * rc2 + eps_);
    }
    *reinterpret_cast<f32x4*>(p + e) = pp;
    *reinterpret_cast<f32x4*>(m + e) = mm;
    *reinterpret_cast<f32x4*>(v + e) = vv;
    if (pout) {
#pragma unroll
      for (int j = 0; j < 4; ++j) IO<TP>::st(pout, e + j, pp[j]);
    }
  }
  // tail
  for (long e = n4 * 4 + (long)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (long)gridDim.x * blockDim.x) {
    const float gg = IO<TG>::ld(g, e) * gs;
    float mm = b1 * m[e] + (1.f - b1) * gg;
    float vv = b2 * v[e] + (1.f - b2) * gg * gg;
    const float decay = e < decay_end ? wd : 0.f;
    float pp = p[e] * (1.f - lr_ * decay) - step * mm / (sqrtf(vv) * rc2 + eps_);
    p[e] = pp; m[e] = mm; v[e] = vv;
    if (pout) IO<TP>::st(pout, e, pp);
  }
}

// Streaming AdamW, 8 elements per lane per trip: every operand of a trip (2 x 16 B
// of p, m, v and g, or one 16 B bf16 g) is loaded before any arithmetic, so each lane
// keeps 7-8 vector loads in flight; the state is touched exactly once per step, so
// NT loads / stores would keep it from evicting the GEMM operands' L2 lines
// (nontemporal == 1; measured slower, kept as an A/B arm).  fp32 master + fp32 m / v are 28 of the 30 B per element.
template <typename T, int NT>
__device__ __forceinline__ T ld_s(const T* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <typename T, int NT>
__device__ __forceinline__ void st_s(T v, T* p) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

typedef unsigned short u16x8_t __attribute__((ext_vector_type(8)));

template <typename TG, typename TP, int NT>
__global__ __launch_bounds__(256) void adamw8_kernel(float* __restrict__ p, const TG* __restrict__ g,
                                                     float* __restrict__ m, float* __restrict__ v,
                                                     TP* __restrict__ pout, long n8, float lr,
                                                     const float* __restrict__ lr_ptr, float b1, float b2,
                                                     float eps, float wd, float bc1, float bc2,
                                                     const float* __restrict__ b1pow,
                                                     const float* __restrict__ b2pow, long decay_end,
                                                     float gscale, const float* __restrict__ gscale_ptr,
                                                     int lr_t_eps) {
  const float lr_ = lr_ptr ? lr_ptr[0] : lr;
  const float c1 = b1pow ? 1.f - b1pow[0] : bc1;
  const float c2 = b2pow ? 1.f - b2pow[0] : bc2;
  const float gs = gscale_ptr ? gscale_ptr[0] * gscale : gscale;
  const float step = lr_ / c1;
  const float rc2 = rsqrtf(c2);
  const float eps_ = lr_t_eps ? eps * rc2 : eps;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    const long e = i * 8;
    f32x4 p0 = ld_s<f32x4, NT>(reinterpret_cast<const f32x4*>(p + e));
    f32x4 p1 = ld_s<f32x4, NT>(reinterpret_cast<const f32x4*>(p + e + 4));
    f32x4 m0 = ld_s<f32x4, NT>(reinterpret_cast<const f32x4*>(m + e));
    f32x4 m1 = ld_s<f32x4, NT>(reinterpret_cast<const f32x4*>(m + e + 4));
    f32x4 v0 = ld_s<f32x4, NT>(reinterpret_cast<const f32x4*>(v + e));
    f32x4 v1 = ld_s<f32x4, NT>(reinterpret_cast<const f32x4*>(v + e + 4));
    float gg[8];
    if constexpr (sizeof(TG) == 4) {
      const f32x4 g0 = ld_s<f32x4, NT>(reinterpret_cast<const f32x4*>(g + e));
      const f32x4 g1 = ld_s<f32x4, NT>(reinterpret_cast<const f32x4*>(g + e + 4));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        gg[j] = g0[j] * gs;
        gg[4 + j] = g1[j] * gs;
      }
    } else {
      const u16x8_t gb = ld_s<u16x8_t, NT>(reinterpret_cast<const u16x8_t*>(g + e));
#pragma unroll
      for (int j = 0; j < 8; ++j) gg[j] = bf2f(gb[j]) * gs;
    }
    float pp[8], mm[8], vv[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pp[j] = p0[j]; pp[4 + j] = p1[j];
      mm[j] = m0[j]; mm[4 + j] = m1[j];
      vv[j] = v0[j]; vv[4 + j] = v1[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mm[j] = b1 * mm[j] + (1.f - b1) * gg[j];
      vv[j] = b2 * vv[j] + (1.f - b2) * gg[j] * gg[j];
      const float decay = (e + j) < decay_end ? wd : 0.f;
      pp[j] = pp[j] * (1.f - lr_ * decay) - step * mm[j] / (sqrtf(vv[j]) * rc2 + eps_);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      p0[j] = pp[j]; p1[j] = pp[4 + j];
      m0[j] = mm[j]; m1[j] = mm[4 + j];
      v0[j] = vv[j]; v1[j] = vv[4 + j];
    }
    st_s<f32x4, NT>(p0, reinterpret_cast<f32x4*>(p + e));
    st_s<f32x4, NT>(p1, reinterpret_cast<f32x4*>(p + e + 4));
    st_s<f32x4, NT>(m0, reinterpret_cast<f32x4*>(m + e));
    st_s<f32x4, NT>(m1, reinterpret_cast<f32x4*>(m + e + 4));
    st_s<f32x4, NT>(v0, reinterpret_cast<f32x4*>(v + e));
    st_s<f32x4, NT>(v1, reinterpret_cast<f32x4*>(v + e + 4));
    if (pout) {
      if constexpr (sizeof(TP) == 2) {
        u16x8_t o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = f2bf(pp[j]);
        st_s<u16x8_t, NT>(o, reinterpret_cast<u16x8_t*>(pout + e));
      } else {
        st_s<f32x4, NT>(p0, reinterpret_cast<f32x4*>(pout + e));
        st_s<f32x4, NT>(p1, reinterpret_cast<f32x4*>(pout + e + 4));
      }
    }
  }
}

// Momentum (optionally Nesterov) and plain SGD; fp32 velocity, parameters fp32 or
// bf16 updated in place (bf16: read, fp32 update, one rounding on the store -- no
// fp32 staging copy of a bf16 model).
template <typename TG, typename TP>
__global__ void momentum_kernel(TP* __restrict__ p, const TG* __restrict__ g,
                                float* __restrict__ vel, long n, float lr,
                                const float* __restrict__ lr_ptr, float mu, int nesterov, float wd,
                                float gscale) {
  const float lr_ = lr_ptr ? lr_ptr[0] : lr;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x) {
    const float pi = IO<TP>::ld(p, i);
    const float gg = IO<TG>::ld(g, i) * gscale + wd * pi;
    float po;
    if (vel) {
      const float v = mu * vel[i] + gg;
      vel[i] = v;
      po = pi - (nesterov ? lr_ * (gg + mu * v) : lr_ * v);
    } else {
      po = pi - lr_ * gg;
    }
    IO<TP>::st(p, i, po);
  }
}

// Multi-tensor Momentum: every parameter of a model in ONE launch (a DyGraph model
// has hundreds of small parameters; one launch + host call each dominates the step
// of a conv net).  A device table describes each tensor; block b updates chunk
// b - chunk0 (MCHUNK elements) of the tensor whose chunk range holds b (binary
// search over the table).  Per tensor: L2 decay `wd` on the updated value, an lr
// multiplier, and an optional second output (the bf16 model copy of an fp32 master).
struct MomT {
  void* t;         // updated tensor: fp32 master, or the fp32 / bf16 parameter itself
  void* out;       // optional model copy written with the new value (null: none)
  const void* g;   // gradient (fp32 / bf16)
  float* vel;      // fp32 velocity
  long n;
  long chunk0;     // first chunk index of this tensor
  float wd, lr_scale;
  int tdt, odt, gdt, pad;  // dtypes: 0 fp32, 1 bf16
};
constexpr int MCHUNK = 4096;

__global__ __launch_bounds__(256) void momentum_multi_kernel(const MomT* __restrict__ tab, int nt, float lr,
                                                             const float* __restrict__ lr_ptr, float mu,
                                                             int nesterov, float gscale) {
  const long b = blockIdx.x;
  int lo = 0, hi = nt - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (tab[mid].chunk0 <= b) lo = mid; else hi = mid - 1;
  }
  const MomT e = tab[lo];
  const float lr_ = (lr_ptr ? lr_ptr[0] : lr) * e.lr_scale;
  const long base = (b - e.chunk0) * MCHUNK;
  const long end = base + MCHUNK < e.n ? base + MCHUNK : e.n;
  for (long i = base + threadIdx.x; i < end; i += blockDim.x) {
    const float pi = e.tdt ? bf2f(((const u16*)e.t)[i]) : ((const float*)e.t)[i];
    const float gi = e.gdt ? bf2f(((const u16*)e.g)[i]) : ((const float*)e.g)[i];
    const float gg = gi * gscale + e.wd * pi;
    const float v = mu * e.vel[i] + gg;
    e.vel[i] = v;
    const float po = pi - lr_ * (nesterov ? gg + mu * v : v);
    if (e.tdt) ((u16*)e.t)[i] = f2bf(po); else ((float*)e.t)[i] = po;
    if (e.out) {
      if (e.odt) ((u16*)e.out)[i] = f2bf(po); else ((float*)e.out)[i] = po;
    }
  }
}

// sum of squares (for global-norm clipping): out[0] += sum(x^2); 16-B vector loads,
// one fp32 atomic per block.
template <typename T>
__global__ __launch_bounds__(256) void sumsq_kernel(const T* __restrict__ x, long n, float* __restrict__ out) {
  __shared__ float red[4];
  float s = 0.f;
  const long n8 = n / 8;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    float v[8];
    load8(x + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[j] * v[j];
  }
  for (long i = n8 * 8 + (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float v = IO<T>::ld(x, i);
    s += v * v;
  }
  s = block_sum<256>(s, red);
  if (threadIdx.x == 0) atomicAdd(out, s);
}

}  // namespace pa

using namespace pa;

// gdtype: grad dtype (0 fp32, 1 bf16); pdtype: model-copy dtype (0 fp32, 1 bf16, -1 none)
PA_EXPORT int pa_adamw(int gdtype, int pdtype, float* p, const void* g, float* m, float* v,
                       void* pout, long n, float lr, const float* lr_ptr, float b1, float b2,
                       float eps, float wd, float bc1, float bc2, const float* b1pow,
                       const float* b2pow, long decay_end, float gscale, const float* gscale_ptr,
                       int lr_t_eps, hipStream_t st) {
  if (n == 0) return 0;
  // PA_ADAMW_MODE: 0 the 4-wide kernel, 1 (default) the 8-wide kernel, 2 8-wide with
  // non-temporal state traffic.  1e9 elements (benchmarks/adamw_bw.py, 30 B / element):
  // 4.65 / 4.77 / 3.15 TB/s -- NT stores cost a third here.  The 8-wide kernel takes
  // the 16 B-aligned body; the 4-wide kernel finishes the (< 8 element) tail.
  static const int mode = [] {
    const char* s = getenv("PA_ADAMW_MODE");
    return s ? atoi(s) : 1;
  }();
  const bool aligned = ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(m) |
                         reinterpret_cast<uintptr_t>(v) | reinterpret_cast<uintptr_t>(g) |
                         reinterpret_cast<uintptr_t>(pout)) & 15) == 0;
  if (mode > 0 && aligned && n >= 8) {
    const long n8 = n / 8;
    const int grid8 = (int)std::min<long>((n8 + 255) / 256, 8192);
#define PA_A8(TG, TP, NTV) \
  hipLaunchKernelGGL((adamw8_kernel<TG, TP, NTV>), dim3(grid8), dim3(256), 0, st, p, (const TG*)g, m, v, (TP*)pout, n8, lr, lr_ptr, b1, b2, eps, wd, bc1, bc2, b1pow, b2pow, decay_end, gscale, gscale_ptr, lr_t_eps)
#define PA_A8N(TG, TP) \
  if (mode == 2) PA_A8(TG, TP, 1); else PA_A8(TG, TP, 0)
    if (gdtype == 1) { if (pdtype == 1) { PA_A8N(u16, u16); } else { PA_A8N(u16, float); } }
    else { if (pdtype == 1) { PA_A8N(float, u16); } else { PA_A8N(float, float); } }
#undef PA_A8N
#undef PA_A8
    const long done = n8 * 8;
    if (done == n) PA_LAUNCH_CHECK();
    // tail on the 4-wide kernel (its own tail loop covers the last < 4 elements)
    const int gs = gdtype == 1 ? 2 : 4, ps = pdtype == 1 ? 2 : 4;
    p += done;
    m += done;
    v += done;
    g = (const char*)g + done * gs;
    if (pout) pout = (char*)pout + done * ps;
    n -= done;
    decay_end -= done;
  }
  const int grid = stream_grid((n + 3) / 4, 256);
#define PA_A(TG, TP) \
  hipLaunchKernelGGL((adamw_kernel<TG, TP>), dim3(grid), dim3(256), 0, st, p, (const TG*)g, m, v, (TP*)pout, n, lr, lr_ptr, b1, b2, eps, wd, bc1, bc2, b1pow, b2pow, decay_end, gscale, gscale_ptr, lr_t_eps)
  if (gdtype == 1) { if (pdtype == 1) PA_A(u16, u16); else PA_A(u16, float); }
  else { if (pdtype == 1) PA_A(float, u16); else PA_A(float, float); }
#undef PA_A
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_momentum(int gdtype, float* p, const void* g, float* vel, long n, float lr,
                          const float* lr_ptr, float mu, int nesterov, float wd, float gscale,
                          hipStream_t st) {
  if (n == 0) return 0;
  const int grid = stream_grid(n, 256);
  if (gdtype == 1)
    hipLaunchKernelGGL((momentum_kernel<u16, float>), dim3(grid), dim3(256), 0, st, p, (const u16*)g, vel, n, lr, lr_ptr, mu, nesterov, wd, gscale);
  else
    hipLaunchKernelGGL((momentum_kernel<float, float>), dim3(grid), dim3(256), 0, st, p, (const float*)g, vel, n, lr, lr_ptr, mu, nesterov, wd, gscale);
  PA_LAUNCH_CHECK();
}

// pdtype: 0 fp32, 1 bf16 parameters (updated in place)
PA_EXPORT int pa_momentum_p(int gdtype, int pdtype, void* p, const void* g, float* vel, long n, float lr,
                            const float* lr_ptr, float mu, int nesterov, float wd, float gscale,
                            hipStream_t st) {
  if (n == 0) return 0;
  const int grid = stream_grid(n, 256);
#define PA_M(TG, TP) \
  hipLaunchKernelGGL((momentum_kernel<TG, TP>), dim3(grid), dim3(256), 0, st, (TP*)p, (const TG*)g, vel, n, lr, lr_ptr, mu, nesterov, wd, gscale)
  if (gdtype == 1) { if (pdtype == 1) PA_M(u16, u16); else PA_M(u16, float); }
  else { if (pdtype == 1) PA_M(float, u16); else PA_M(float, float); }
#undef PA_M
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_sumsq(int dtype, const void* x, long n, float* out, hipStream_t st) {
  if (n == 0) return 0;
  const int grid = stream_grid((n + 7) / 8, 256);
  if (dtype == 1)
    hipLaunchKernelGGL(sumsq_kernel<u16>, dim3(grid), dim3(256), 0, st, (const u16*)x, n, out);
  else
    hipLaunchKernelGGL(sumsq_kernel<float>, dim3(grid), dim3(256), 0, st, (const float*)x, n, out);
  PA_LAUNCH_CHECK();
}

// Global-norm clip coefficient on the device (no host sync, no framework scalar ops):
// coef = min(1, max_norm / (sqrt(sumsq) * norm_scale + 1e-6)).
__global__ void clip_coef_kernel(const float* __restrict__ sumsq, float norm_scale, float max_norm,
                                 float* __restrict__ coef) {
  if (threadIdx.x == 0) coef[0] = fminf(1.f, max_norm / (sqrtf(sumsq[0]) * norm_scale + 1e-6f));
}

PA_EXPORT int pa_clip_coef(const float* sumsq, float norm_scale, float max_norm, float* coef, hipStream_t st) {
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(64), 0, st, sumsq, norm_scale, max_norm, coef);
  PA_LAUNCH_CHECK();
}

// Fold a bf16 / fp32 gradient into the fp32 main_grad: dst = (fresh ? 0 : dst) + g.
// The sharded optimizer's post-accumulate hook runs this for parameters whose
// backward returned a plain gradient (biases, norm weights) instead of writing
// main_grad in a GEMM epilogue.
template <typename T>
__global__ void fold_grad_kernel(float* __restrict__ dst, const T* __restrict__ g, long n, int fresh) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    dst[i] = (fresh ? 0.f : dst[i]) + IO<T>::ld(g, i);
}

PA_EXPORT int pa_fold_grad(int gdtype, float* dst, const void* g, long n, int fresh, hipStream_t st) {
  if (n == 0) return 0;
  const int grid = stream_grid(n, 256);
  if (gdtype == 1)
    hipLaunchKernelGGL(fold_grad_kernel<u16>, dim3(grid), dim3(256), 0, st, dst, (const u16*)g, n, fresh);
  else
    hipLaunchKernelGGL(fold_grad_kernel<float>, dim3(grid), dim3(256), 0, st, dst, (const float*)g, n, fresh);
  PA_LAUNCH_CHECK();
}

// tab: device array of nt MomT entries (chunk0 ascending), total_chunks = sum of
// ceil(n / MCHUNK); see ops/optim.py momentum_multi
PA_EXPORT int pa_momentum_multi(const void* tab, int nt, long total_chunks, float lr, const float* lr_ptr, float mu,
                                int nesterov, float gscale, hipStream_t st) {
  if (nt <= 0 || total_chunks <= 0) return 0;
  if (total_chunks > 0x7fffffffL) return -1;
  hipLaunchKernelGGL(momentum_multi_kernel, dim3((unsigned)total_chunks), dim3(256), 0, st, (const MomT*)tab, nt, lr,
                     lr_ptr, mu, nesterov, gscale);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_momentum_multi_entry_bytes() { return (int)sizeof(MomT); }
PA_EXPORT int pa_momentum_multi_chunk() { return MCHUNK; }

