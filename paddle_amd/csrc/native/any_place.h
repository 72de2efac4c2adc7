// One-source host + device kernels for the native executor's HIP translation units.
//
// An op written against these helpers runs the same algorithm on either place: an
// elementwise functor (a struct with a __host__ __device__ operator()(int64_t)) runs
// over the worker pool on the host or as a grid-stride HIP kernel on the op's stream,
// GEMMs go to the blocked host sgemm or to pa_sgemm (exact-fp32 MFMA), and integer
// schedules built on the host from LoD metadata are uploaded through the op's pinned
// staging buffer.  Used by ops_rnn_unit.hip, ops_loss.hip and ops_tensor.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <string.h>

#include <vector>

#include "device_util.h"

namespace pa {
namespace any {

template <class F>
__global__ void ew_kernel(F f, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) f(i);
}

// f(i) for i in [0, n) on the op's place
template <class F>
void run(const OpRun& r, bool dev, int64_t n, const F& f, int64_t grain = 4096) {
  if (n <= 0) return;
  if (dev) {
    hipLaunchKernelGGL(ew_kernel<F>, dim3(dev_grid(n)), dim3(256), 0, dev_stream(r), f, n);
    PA_HIPCHK(hipGetLastError());
  } else {
    parallel_for(n, grain, [&](int64_t a, int64_t b) {
      for (int64_t i = a; i < b; ++i) f(i);
    });
  }
}

inline void gemm(const OpRun& r, bool dev, bool ta, bool tb, int64_t M, int64_t N, int64_t K, float alpha,
                 const float* A, int64_t lda, const float* B, int64_t ldb, float beta, float* C, int64_t ldc) {
  if (M <= 0 || N <= 0) return;
  if (K <= 0) {
    // C = beta C (the GEMM libraries are not asked to handle an empty reduction)
    struct Scale {
      float* c;
      int64_t n, ldc;
      float beta;
      __host__ __device__ void operator()(int64_t i) const {
        float& v = c[(i / n) * ldc + i % n];
        v = beta == 0.f ? 0.f : v * beta;
      }
    };
    run(r, dev, M * N, Scale{C, N, ldc, beta});
    return;
  }
  if (dev) device_sgemm(r.ctx.stream, ta, tb, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc);
  else sgemm(ta, tb, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc);
}

// fp32 input of the op's place, or decline (the executor then tries the next kernel)
inline float* f32(const Tensor& t, bool dev) {
  if (t.dtype != DT::FP32 || (t.device >= 0) != dev) throw Decline{};
  return t.data<float>();
}

// a scratch buffer of n floats on the op's place: a root-scope workspace on the
// device, a vector owned by `host` on the host
inline float* scratch(const OpRun& r, bool dev, const char* name, int64_t n, std::vector<float>* host) {
  if (dev) return device_workspace(r, name, n < 1 ? 1 : n);
  host->assign((size_t)(n < 1 ? 1 : n), 0.f);
  return host->data();
}

// int32 table on the op's place (host: a pointer into `keep`)
inline const int* ints(const OpRun& r, bool dev, const char* name, const std::vector<int>& v) {
  if (v.empty()) return nullptr;
  if (dev) return (const int*)device_upload(r, name, v.data(), v.size() * sizeof(int));
  return v.data();
}

inline void zero(const OpRun& r, bool dev, float* p, int64_t n) {
  if (n <= 0) return;
  if (dev) PA_HIPCHK(hipMemsetAsync(p, 0, (size_t)n * sizeof(float), dev_stream(r)));
  else memset(p, 0, (size_t)n * sizeof(float));
}

inline void copy(const OpRun& r, bool dev, float* dst, const float* src, int64_t n) {
  if (n <= 0 || dst == src) return;
  if (dev) PA_HIPCHK(hipMemcpyAsync(dst, src, (size_t)n * sizeof(float), hipMemcpyDeviceToDevice, dev_stream(r)));
  else memcpy(dst, src, (size_t)n * sizeof(float));
}

// out[j] = sum_t X[t * ld + j] (+ out[j] when acc) for j < W
struct ColSum {
  const float* x;
  float* out;
  int64_t T, ld;
  int acc;
  __host__ __device__ void operator()(int64_t j) const {
    float s = acc ? out[j] : 0.f;
    for (int64_t t = 0; t < T; ++t) s += x[t * ld + j];
    out[j] = s;
  }
};

}  // namespace any
}  // namespace pa
