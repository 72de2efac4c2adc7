// The remaining Fluid optimizer update ops as single-pass fp32 kernels (reference
// operators/{adamax,decayed_adagrad,adadelta,rmsprop,ftrl,proximal_gd,
// proximal_adagrad,lars_momentum}_op.h: Eigen expressions there).  Every kernel
// updates parameter and state in place in one read / one write of each array; the
// learning rate (and beta-pow) is read from device memory, so an optimizer step
// never syncs with the host.  LARS needs ||p|| and ||g||: a first pass folds both
// squared norms into two fp32 accumulators, the update pass reads them.
#include "common.h"

namespace pa {
namespace {

#define GRID_STRIDE(i, n) for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < (n); i += (long)gridDim.x * blockDim.x)

__global__ __launch_bounds__(256) void adamax_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                     float* __restrict__ m, float* __restrict__ u,
                                                     const float* __restrict__ lr, const float* __restrict__ bp1,
                                                     float b1, float b2, float eps, long n) {
  const float step = lr[0] / (1.f - bp1[0]);
  GRID_STRIDE(i, n) {
    const float gi = g[i];
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float ui = fmaxf(b2 * u[i] + eps, fabsf(gi));
    m[i] = mi;
    u[i] = ui;
    p[i] -= step * mi / ui;
  }
}

__global__ __launch_bounds__(256) void decayed_adagrad_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                              float* __restrict__ m, const float* __restrict__ lr,
                                                              float decay, float eps, long n) {
  const float l = lr[0];
  GRID_STRIDE(i, n) {
    const float gi = g[i];
    const float mi = decay * m[i] + (1.f - decay) * gi * gi;
    m[i] = mi;
    p[i] -= l * gi / (sqrtf(mi) + eps);
  }
}

__global__ __launch_bounds__(256) void adadelta_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                       float* __restrict__ ag, float* __restrict__ au, float rho,
                                                       float eps, long n) {
  GRID_STRIDE(i, n) {
    const float gi = g[i];
    const float a = rho * ag[i] + (1.f - rho) * gi * gi;
    const float upd = -sqrtf((au[i] + eps) / (a + eps)) * gi;
    ag[i] = a;
    au[i] = rho * au[i] + (1.f - rho) * upd * upd;
    p[i] += upd;
  }
}

__global__ __launch_bounds__(256) void rmsprop_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                      float* __restrict__ ms, float* __restrict__ mom,
                                                      float* __restrict__ mg, const float* __restrict__ lr, float rho,
                                                      float mu, float eps, long n) {
  const float l = lr[0];
  GRID_STRIDE(i, n) {
    const float gi = g[i];
    const float s = rho * ms[i] + (1.f - rho) * gi * gi;
    ms[i] = s;
    float den;
    if (mg) {
      const float a = rho * mg[i] + (1.f - rho) * gi;
      mg[i] = a;
      den = s - a * a + eps;
    } else {
      den = s + eps;
    }
    const float v = mu * mom[i] + l * gi / sqrtf(den);
    mom[i] = v;
    p[i] -= v;
  }
}

__global__ __launch_bounds__(256) void ftrl_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ sq, float* __restrict__ lin,
                                                   const float* __restrict__ lr, float l1, float l2, float lr_power,
                                                   long n) {
  const float l = lr[0];
  GRID_STRIDE(i, n) {
    const float gi = g[i], s0 = sq[i];
    const float s1 = s0 + gi * gi;
    float sigma, y;
    if (lr_power == -0.5f) {
      sigma = (sqrtf(s1) - sqrtf(s0)) / l;
      y = sqrtf(s1) / l + 2.f * l2;
    } else {
      sigma = (powf(s1, -lr_power) - powf(s0, -lr_power)) / l;
      y = powf(s1, -lr_power) / l + 2.f * l2;
    }
    const float nl = lin[i] + gi - sigma * p[i];
    sq[i] = s1;
    lin[i] = nl;
    p[i] = fabsf(nl) > l1 ? (fminf(fmaxf(nl, -l1), l1) - nl) / y : 0.f;
  }
}

// m == nullptr: proximal_gd; else proximal_adagrad (lr_t = lr / sqrt(m + g^2))
__global__ __launch_bounds__(256) void proximal_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                       float* __restrict__ m, const float* __restrict__ lr, float l1,
                                                       float l2, long n) {
  const float l = lr[0];
  GRID_STRIDE(i, n) {
    const float gi = g[i];
    float lt = l;
    if (m) {
      const float mi = m[i] + gi * gi;
      m[i] = mi;
      lt = l / sqrtf(mi);
    }
    const float prox = p[i] - lt * gi;
    const float mag = fmaxf(fabsf(prox) - lt * l1, 0.f);
    p[i] = copysignf(mag, prox) * (prox != 0.f) / (1.f + lt * l2);
  }
}

__global__ __launch_bounds__(256) void sqnorm2_kernel(const float* __restrict__ p, const float* __restrict__ g, long n,
                                                      float* __restrict__ acc) {
  __shared__ float red[4];
  float a = 0.f, b = 0.f;
  GRID_STRIDE(i, n) {
    a += p[i] * p[i];
    b += g[i] * g[i];
  }
  a = block_sum<256>(a, red);
  b = block_sum<256>(b, red);
  if (threadIdx.x == 0) {
    atomicAdd(acc, a);
    atomicAdd(acc + 1, b);
  }
}

__global__ __launch_bounds__(256) void lars_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ v, const float* __restrict__ lr,
                                                   const float* __restrict__ acc, float mu, float coeff, float wd,
                                                   long n) {
  const float pn = sqrtf(acc[0]), gn = sqrtf(acc[1]);
  const float local = lr[0] * coeff * pn / (gn + wd * pn + 1e-12f);
  GRID_STRIDE(i, n) {
    const float vi = mu * v[i] + local * (g[i] + wd * p[i]);
    v[i] = vi;
    p[i] -= vi;
  }
}

}  // namespace
}  // namespace pa

using namespace pa;

#define LAUNCH(k, n, ...)                                                                       \
  do {                                                                                          \
    if ((n) <= 0) return 0;                                                                     \
    hipLaunchKernelGGL(k, dim3(stream_grid((n), 256)), dim3(256), 0, st, __VA_ARGS__);          \
  } while (0)

PA_EXPORT int pa_opt_adamax(float* p, const float* g, float* m, float* u, const float* lr, const float* bp1, float b1,
                            float b2, float eps, long n, hipStream_t st) {
  LAUNCH(adamax_kernel, n, p, g, m, u, lr, bp1, b1, b2, eps, n);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_opt_decayed_adagrad(float* p, const float* g, float* m, const float* lr, float decay, float eps,
                                     long n, hipStream_t st) {
  LAUNCH(decayed_adagrad_kernel, n, p, g, m, lr, decay, eps, n);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_opt_adadelta(float* p, const float* g, float* ag, float* au, float rho, float eps, long n,
                              hipStream_t st) {
  LAUNCH(adadelta_kernel, n, p, g, ag, au, rho, eps, n);
  PA_LAUNCH_CHECK();
}

// mg == nullptr: plain RMSProp; else centered
PA_EXPORT int pa_opt_rmsprop(float* p, const float* g, float* ms, float* mom, float* mg, const float* lr, float rho,
                             float mu, float eps, long n, hipStream_t st) {
  LAUNCH(rmsprop_kernel, n, p, g, ms, mom, mg, lr, rho, mu, eps, n);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_opt_ftrl(float* p, const float* g, float* sq, float* lin, const float* lr, float l1, float l2,
                          float lr_power, long n, hipStream_t st) {
  LAUNCH(ftrl_kernel, n, p, g, sq, lin, lr, l1, l2, lr_power, n);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_opt_proximal(float* p, const float* g, float* m, const float* lr, float l1, float l2, long n,
                              hipStream_t st) {
  LAUNCH(proximal_kernel, n, p, g, m, lr, l1, l2, n);
  PA_LAUNCH_CHECK();
}

// acc: two zeroed fp32 workspace floats
PA_EXPORT int pa_opt_lars(float* p, const float* g, float* v, const float* lr, float* acc, float mu, float coeff,
                          float wd, long n, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(sqnorm2_kernel, dim3(stream_grid(n, 256)), dim3(256), 0, st, p, g, n, acc);
  LAUNCH(lars_kernel, n, p, g, v, lr, acc, mu, coeff, wd, n);
  PA_LAUNCH_CHECK();
}
