// Device contexts (reference: platform/device_context.h:39-179 DeviceContext /
// CUDADeviceContext / DeviceContextPool).  MI355X design: per
// HIP device one context owning
//   * a compute stream, a communication stream and an auxiliary stream (all
//     non-blocking; the comm stream at high priority so bucketed collectives
//     overtake queued compute; aux for side work such as an overlapped optimizer
//     update),
//   * an event pool (events are recycled instead of created per use),
// created lazily per device and kept for the process lifetime (pool semantics:
// DeviceContextPool::Get(place)).  The framework wraps the streams as torch
// external streams, so every kernel it launches runs on a stream owned here.
#include <hip/hip_runtime_api.h>

#include <mutex>
#include <vector>

#include "runtime.h"

#pragma GCC diagnostic ignored "-Wunused-result"

namespace {

struct DeviceContext {
  int device = 0;
  hipStream_t compute = nullptr, comm = nullptr, aux = nullptr;
  std::vector<hipEvent_t> free_events;
  std::mutex mu;
  long events_created = 0;
};

std::mutex g_mu;
std::vector<DeviceContext*> g_pool;  // index = device

}  // namespace

// The context of HIP device `device` (created on first use); null on error.
PA_RT_EXPORT void* pa_dc_get(int device) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (device < 0 || device > 1024) return nullptr;
  if ((int)g_pool.size() <= device) g_pool.resize(device + 1, nullptr);
  if (!g_pool[device]) {
    int prev = 0;
    hipGetDevice(&prev);
    if (hipSetDevice(device) != hipSuccess) {
      pa_rt_set_error("device context: no HIP device %d", device);
      return nullptr;
    }
    auto* dc = new DeviceContext();
    dc->device = device;
    int lo = 0, hi = 0;
    hipDeviceGetStreamPriorityRange(&lo, &hi);  // hi = greatest priority (numerically lowest)
    bool ok = hipStreamCreateWithPriority(&dc->compute, hipStreamNonBlocking, lo) == hipSuccess &&
              hipStreamCreateWithPriority(&dc->comm, hipStreamNonBlocking, hi) == hipSuccess &&
              hipStreamCreateWithPriority(&dc->aux, hipStreamNonBlocking, lo) == hipSuccess;
    hipSetDevice(prev);
    if (!ok) {
      pa_rt_set_error("device context: stream creation failed on device %d", device);
      delete dc;
      return nullptr;
    }
    g_pool[device] = dc;
  }
  return g_pool[device];
}

hipStream_t pick(DeviceContext* dc, int which) { return which == 1 ? dc->comm : which == 2 ? dc->aux : dc->compute; }

// which: 0 compute, 1 comm, 2 aux
PA_RT_EXPORT void* pa_dc_stream(void* h, int which) { return (void*)pick(static_cast<DeviceContext*>(h), which); }

PA_RT_EXPORT int pa_dc_device(void* h) { return static_cast<DeviceContext*>(h)->device; }

// An event from the pool (timing disabled), or a new one.
PA_RT_EXPORT void* pa_dc_event_acquire(void* h) {
  auto* dc = static_cast<DeviceContext*>(h);
  std::lock_guard<std::mutex> lk(dc->mu);
  if (!dc->free_events.empty()) {
    hipEvent_t e = dc->free_events.back();
    dc->free_events.pop_back();
    return e;
  }
  int prev = 0;
  hipGetDevice(&prev);
  hipSetDevice(dc->device);
  hipEvent_t e = nullptr;
  hipError_t rc = hipEventCreateWithFlags(&e, hipEventDisableTiming);
  hipSetDevice(prev);
  if (rc != hipSuccess) {
    pa_rt_set_error("device context: event creation failed");
    return nullptr;
  }
  ++dc->events_created;
  return e;
}

// Back to the pool once the caller no longer waits on it (a recorded event may be
// re-recorded: HIP events carry their latest record only).
PA_RT_EXPORT void pa_dc_event_release(void* h, void* ev) {
  auto* dc = static_cast<DeviceContext*>(h);
  std::lock_guard<std::mutex> lk(dc->mu);
  dc->free_events.push_back(static_cast<hipEvent_t>(ev));
}

// stream `waiter` waits on the device for everything queued so far on stream `other`.
PA_RT_EXPORT int pa_dc_stream_wait(void* h, int waiter, int other) {
  auto* dc = static_cast<DeviceContext*>(h);
  hipEvent_t e = static_cast<hipEvent_t>(pa_dc_event_acquire(h));
  if (!e) return -1;
  hipStream_t o = pick(dc, other), w = pick(dc, waiter);
  int rc = (hipEventRecord(e, o) == hipSuccess && hipStreamWaitEvent(w, e, 0) == hipSuccess) ? 0 : -1;
  pa_dc_event_release(h, e);
  return rc;
}

// DeviceContext::Wait(): the host blocks until every stream of the context drained.
PA_RT_EXPORT int pa_dc_wait(void* h) {
  auto* dc = static_cast<DeviceContext*>(h);
  return (hipStreamSynchronize(dc->compute) == hipSuccess && hipStreamSynchronize(dc->comm) == hipSuccess &&
          hipStreamSynchronize(dc->aux) == hipSuccess) ? 0 : -1;
}

PA_RT_EXPORT long pa_dc_events_created(void* h) { return static_cast<DeviceContext*>(h)->events_created; }
PA_RT_EXPORT long pa_dc_events_pooled(void* h) {
  auto* dc = static_cast<DeviceContext*>(h);
  std::lock_guard<std::mutex> lk(dc->mu);
  return (long)dc->free_events.size();
}
