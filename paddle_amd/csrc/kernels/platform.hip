// Platform layer of the kernel library (reference platform/enforce.h, init.cc
// InitP2P, gpu_info.cc): HIP error names for the Python enforce layer, peer
// access set-up between the node's GPUs, peer copies and device memory info.
#include "common.h"

PA_EXPORT const char* pa_error_name(int e) { return hipGetErrorName((hipError_t)e); }
PA_EXPORT const char* pa_error_string(int e) { return hipGetErrorString((hipError_t)e); }

PA_EXPORT int pa_device_count(int* n) { return (int)hipGetDeviceCount(n); }

PA_EXPORT int pa_can_access_peer(int dev, int peer, int* can) { return (int)hipDeviceCanAccessPeer(can, dev, peer); }

// Enables dev -> peer access (idempotent: "already enabled" is success).
PA_EXPORT int pa_enable_peer_access(int dev, int peer) {
  int prev = 0;
  hipGetDevice(&prev);
  hipError_t e = hipSetDevice(dev);
  if (e == hipSuccess) {
    e = hipDeviceEnablePeerAccess(peer, 0);
    if (e == hipErrorPeerAccessAlreadyEnabled) {
      (void)hipGetLastError();
      e = hipSuccess;
    }
  }
  hipSetDevice(prev);
  return (int)e;
}

PA_EXPORT int pa_memcpy_peer_async(void* dst, int dst_dev, const void* src, int src_dev, size_t bytes,
                                   hipStream_t st) {
  return (int)hipMemcpyPeerAsync(dst, dst_dev, src, src_dev, bytes, st);
}

PA_EXPORT int pa_mem_info(int dev, size_t* free_b, size_t* total_b) {
  int prev = 0;
  hipGetDevice(&prev);
  hipError_t e = hipSetDevice(dev);
  if (e == hipSuccess) e = hipMemGetInfo(free_b, total_b);
  hipSetDevice(prev);
  return (int)e;
}

// Reads and clears the thread's last HIP error (a failed runtime call leaves it
// set; torch's launch checks would otherwise report it at its next launch).
PA_EXPORT int pa_clear_error() { return (int)hipGetLastError(); }
