// Device-side helpers shared by the native executor's HIP translation units
// (ops_gpu.hip defines them; ops_rnn_gpu.hip, ops_struct_gpu.hip use them).
#pragma once

#include <hip/hip_runtime.h>

#include "framework.h"

namespace pa {

#define PA_HIPCHK(x)                                                               \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) ::pa::fail("%s failed: %s", #x, hipGetErrorString(e_)); \
  } while (0)

// host array -> the op's device scratch `name` through a pinned staging buffer
void* device_upload(const OpRun& r, const char* name, const void* src, size_t bytes);
// root-scope device scratch of >= n floats, reused across ops and runs
float* device_workspace(const OpRun& r, const char* name, int64_t n);
void device_sgemm(void* stream, bool ta, bool tb, int64_t M, int64_t N, int64_t K, float alpha, const float* A,
                  int64_t lda, const float* B, int64_t ldb, float beta, float* C, int64_t ldc);

inline hipStream_t dev_stream(const OpRun& r) { return (hipStream_t)r.ctx.stream; }
inline int dev_id(const OpRun& r) { return r.ctx.device; }
inline int dev_grid(int64_t n, int block = 256) {
  int64_t g = (n + block - 1) / block;
  return (int)(g < 1 ? 1 : (g > 4096 ? 4096 : g));
}
// fp32 device tensor or decline (the executor then runs the host kernel on copies)
inline float* dev_f32(const Tensor& t) {
  if (t.dtype != DT::FP32 || t.device < 0) throw Decline{};
  return t.data<float>();
}

}  // namespace pa
