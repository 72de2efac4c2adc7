// HIP device memory / streams for the native executor (HBM tensors, one stream per
// executor).  Tensors keep their buffers across runs (Tensor::alloc reuses a block
// that is large enough), so steady-state predictor runs do not allocate.
#include <hip/hip_runtime_api.h>

#include <string.h>

#include "framework.h"

namespace pa {

#define HIPCHK(x)                                                                  \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) ::pa::fail("%s failed: %s", #x, hipGetErrorString(e_)); \
  } while (0)

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

void* device_alloc(size_t n, int dev) {
  HIPCHK(hipSetDevice(dev));
  void* p = nullptr;
  HIPCHK(hipMalloc(&p, n));
  return p;
}

void device_free(void* p, int dev) {
  if (!p) return;
  hipSetDevice(dev);
  hipFree(p);  // hipFree synchronises the device: blocks are never freed under a running kernel
}

void device_copy(void* dst, int dst_dev, const void* src, int src_dev, size_t n, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  hipMemcpyKind kind = dst_dev < 0 ? (src_dev < 0 ? hipMemcpyHostToHost : hipMemcpyDeviceToHost)
                                   : (src_dev < 0 ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice);
  if (kind == hipMemcpyHostToHost) {
    memcpy(dst, src, n);
    return;
  }
  HIPCHK(hipMemcpyAsync(dst, src, n, kind, s));
  // host buffers may be temporaries: complete copies that touch host memory
  if (kind != hipMemcpyDeviceToDevice) HIPCHK(hipStreamSynchronize(s));
}

void* device_stream_create(int dev) {
  HIPCHK(hipSetDevice(dev));
  hipStream_t s;
  HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  return s;
}

void device_stream_destroy(void* s) { hipStreamDestroy((hipStream_t)s); }

void device_stream_sync(void* s) {
  if (s) HIPCHK(hipStreamSynchronize((hipStream_t)s));
}

void device_synchronize(int dev) {
  HIPCHK(hipSetDevice(dev));
  HIPCHK(hipDeviceSynchronize());
}

}  // namespace pa
