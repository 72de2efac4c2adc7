// Double-buffered device reader behind fluid py_reader / double_buffer.
//
// Reference: operators/reader/lod_tensor_blocking_queue.h (the py_reader queue),
// operators/reader/buffered_reader.cc:26-110 (a prefetch thread copying the next
// batches to the device on its own CUDA stream, one event per buffer) and
// create_double_buffer_reader_op.cc.  MI355X design:
//
//   producer (Python thread) --push--> [bounded queue of batches in pinned host
//   memory] --prefetch thread--> hipMemcpyAsync H2D on a private non-blocking
//   stream into one of `nslots` device slots, ready event per slot
//   --consume(stream)--> the consumer's stream waits on the ready event and copies
//   the slot into its own tensors (device-to-device, stream ordered), then records
//   the slot's free event; the prefetch thread makes its copy stream wait on that
//   free event before overwriting the slot.
//
// No host thread ever blocks on the GPU on the hot path: slot reuse is ordered by
// events on the device, pinned staging buffers are recycled once their copy's
// event has completed (polled).  device < 0 runs the same pipeline on host memory
// (memcpy) so the queue logic is exercised without a GPU.
#include <hip/hip_runtime_api.h>
#include <stdlib.h>
#include <string.h>

// status codes of the HIP calls on the prefetch path are folded into `ok` where they
// matter; bookkeeping calls (event record / destroy) are best effort
#pragma GCC diagnostic ignored "-Wunused-result"

#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "runtime.h"

namespace {

struct Staged {  // one batch in pinned (or plain) host memory
  std::vector<void*> buf;
  std::vector<size_t> cap, bytes;
};

struct Slot {
  std::vector<void*> dev;
  std::vector<size_t> cap, bytes;
  hipEvent_t ready = nullptr, freed = nullptr;
  bool freed_recorded = false;
};

struct DBR {
  int device = -1, nslots = 2;
  size_t capacity = 2;
  hipStream_t copy_stream = nullptr;
  std::mutex mu;
  std::condition_variable cv;
  std::deque<Staged> queue;               // pushed, not yet prefetched
  std::deque<int> ready;                  // prefetched slots, in order
  std::vector<int> free_slots;            // slots not holding a batch
  std::vector<Slot> slots;
  std::vector<Staged> pinned_pool;        // recyclable host buffers
  std::deque<std::pair<hipEvent_t, Staged>> in_flight;  // host buffers under an H2D copy
  bool closed = false, stop = false, failed = false;
  int in_prefetch = 0;                    // batches taken by the prefetch thread, not yet ready
  std::thread th;
};

bool host_mode(const DBR* d) { return d->device < 0; }

void* host_alloc(DBR* d, size_t n) {
  if (host_mode(d)) return malloc(n ? n : 1);
  void* p = nullptr;
  if (hipHostMalloc(&p, n ? n : 1, hipHostMallocDefault) != hipSuccess) return nullptr;
  return p;
}

void host_free(DBR* d, void* p) {
  if (!p) return;
  if (host_mode(d))
    free(p);
  else
    hipHostFree(p);
}

void recycle_in_flight(DBR* d, bool wait) {  // caller holds mu
  while (!d->in_flight.empty()) {
    auto& f = d->in_flight.front();
    if (wait)
      hipEventSynchronize(f.first);
    else if (hipEventQuery(f.first) != hipSuccess)
      break;
    hipEventDestroy(f.first);
    d->pinned_pool.push_back(std::move(f.second));
    d->in_flight.pop_front();
  }
}

// a staged batch able to hold `bytes` (pool reuse when every field fits)
bool take_staging(DBR* d, const std::vector<size_t>& bytes, Staged& out) {
  for (size_t i = 0; i < d->pinned_pool.size(); ++i) {
    Staged& s = d->pinned_pool[i];
    if (s.buf.size() != bytes.size()) continue;
    bool fits = true;
    for (size_t f = 0; f < bytes.size(); ++f) fits = fits && s.cap[f] >= bytes[f];
    if (!fits) continue;
    out = std::move(s);
    d->pinned_pool.erase(d->pinned_pool.begin() + i);
    out.bytes = bytes;
    return true;
  }
  out.buf.assign(bytes.size(), nullptr);
  out.cap = bytes;
  out.bytes = bytes;
  for (size_t f = 0; f < bytes.size(); ++f)
    if (!(out.buf[f] = host_alloc(d, bytes[f]))) return false;
  return true;
}

void prefetch_loop(DBR* d) {
  if (!host_mode(d)) hipSetDevice(d->device);
  for (;;) {
    Staged b;
    int s = -1;
    {
      std::unique_lock<std::mutex> lk(d->mu);
      d->cv.wait(lk, [&] { return d->stop || (!d->queue.empty() && !d->free_slots.empty()) ||
                                  (d->closed && d->queue.empty()); });
      if (d->stop || (d->closed && d->queue.empty())) {
        d->cv.notify_all();
        return;
      }
      b = std::move(d->queue.front());
      d->queue.pop_front();
      d->in_prefetch = 1;
      s = d->free_slots.back();
      d->free_slots.pop_back();
      d->cv.notify_all();  // a producer may be waiting for queue room
    }
    Slot& sl = d->slots[s];
    const size_t nf = b.bytes.size();
    bool ok = true;
    if (sl.dev.size() != nf) {
      sl.dev.resize(nf, nullptr);
      sl.cap.resize(nf, 0);
    }
    sl.bytes = b.bytes;
    if (!host_mode(d) && sl.freed_recorded) hipStreamWaitEvent(d->copy_stream, sl.freed, 0);
    for (size_t f = 0; f < nf && ok; ++f) {
      if (sl.cap[f] < b.bytes[f]) {  // grow (rare: first batch / a larger batch)
        if (host_mode(d)) {
          free(sl.dev[f]);
          sl.dev[f] = malloc(b.bytes[f] ? b.bytes[f] : 1);
          ok = sl.dev[f] != nullptr;
        } else {
          if (sl.dev[f]) {
            hipStreamSynchronize(d->copy_stream);  // prior copies into the old buffer
            hipFree(sl.dev[f]);
          }
          ok = hipMalloc(&sl.dev[f], b.bytes[f] ? b.bytes[f] : 1) == hipSuccess;
        }
        sl.cap[f] = b.bytes[f];
      }
      if (!ok) break;
      if (host_mode(d))
        memcpy(sl.dev[f], b.buf[f], b.bytes[f]);
      else
        ok = hipMemcpyAsync(sl.dev[f], b.buf[f], b.bytes[f], hipMemcpyHostToDevice, d->copy_stream) == hipSuccess;
    }
    std::lock_guard<std::mutex> lk(d->mu);
    if (!ok) {
      d->failed = true;
      pa_rt_set_error("double-buffer reader: device copy / allocation failed");
    }
    if (host_mode(d)) {
      d->pinned_pool.push_back(std::move(b));
    } else {
      hipEventRecord(sl.ready, d->copy_stream);
      hipEvent_t done = nullptr;
      hipEventCreateWithFlags(&done, hipEventDisableTiming);
      hipEventRecord(done, d->copy_stream);
      d->in_flight.emplace_back(done, std::move(b));
      recycle_in_flight(d, false);
    }
    d->ready.push_back(s);
    d->in_prefetch = 0;
    d->cv.notify_all();
  }
}

void stop_thread(DBR* d) {
  {
    std::lock_guard<std::mutex> lk(d->mu);
    d->stop = true;
    d->cv.notify_all();
  }
  if (d->th.joinable()) d->th.join();
  if (!host_mode(d)) hipStreamSynchronize(d->copy_stream);
  std::lock_guard<std::mutex> lk(d->mu);
  recycle_in_flight(d, true);
}

}  // namespace

PA_RT_EXPORT void* pa_dbr_create(int nslots, size_t capacity, int device) {
  DBR* d = new DBR();
  d->device = device;
  d->nslots = nslots < 1 ? 1 : nslots;
  d->capacity = capacity < 1 ? 1 : capacity;
  d->slots.resize(d->nslots);
  for (int i = d->nslots - 1; i >= 0; --i) d->free_slots.push_back(i);
  if (device >= 0) {
    if (hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithFlags(&d->copy_stream, hipStreamNonBlocking) != hipSuccess) {
      pa_rt_set_error("double-buffer reader: no HIP device %d", device);
      delete d;
      return nullptr;
    }
    for (auto& s : d->slots) {
      hipEventCreateWithFlags(&s.ready, hipEventDisableTiming);
      hipEventCreateWithFlags(&s.freed, hipEventDisableTiming);
    }
  }
  d->th = std::thread(prefetch_loop, d);
  return d;
}

// Blocks while `capacity` batches wait; -1 once closed.
PA_RT_EXPORT int pa_dbr_push(void* h, int nfields, const void* const* ptrs, const int64_t* nbytes) {
  DBR* d = static_cast<DBR*>(h);
  std::vector<size_t> bytes(nfields);
  for (int f = 0; f < nfields; ++f) bytes[f] = (size_t)nbytes[f];
  Staged b;
  {
    std::unique_lock<std::mutex> lk(d->mu);
    d->cv.wait(lk, [&] { return d->closed || d->stop || d->queue.size() < d->capacity; });
    if (d->closed || d->stop) return -1;
    if (!host_mode(d)) recycle_in_flight(d, false);
    if (!take_staging(d, bytes, b)) {
      pa_rt_set_error("double-buffer reader: pinned host allocation failed");
      return -2;
    }
  }
  for (int f = 0; f < nfields; ++f) memcpy(b.buf[f], ptrs[f], bytes[f]);  // off the lock
  std::lock_guard<std::mutex> lk(d->mu);
  if (d->closed || d->stop) {
    d->pinned_pool.push_back(std::move(b));
    return -1;
  }
  d->queue.push_back(std::move(b));
  d->cv.notify_all();
  return 0;
}

// End of data: the consumer drains what is queued, then sees EOF.
PA_RT_EXPORT void pa_dbr_close(void* h) {
  DBR* d = static_cast<DBR*>(h);
  std::lock_guard<std::mutex> lk(d->mu);
  d->closed = true;
  d->cv.notify_all();
}

// Next prefetched batch: slot id (>= 0) with its field sizes in nbytes_out, -1 at
// EOF, -2 on timeout (timeout_ms < 0: wait forever), -3 after a failed copy.
PA_RT_EXPORT int pa_dbr_next(void* h, int64_t* nbytes_out, int max_fields, int timeout_ms) {
  DBR* d = static_cast<DBR*>(h);
  std::unique_lock<std::mutex> lk(d->mu);
  auto pred = [&] {
    return d->failed || !d->ready.empty() || (d->closed && d->queue.empty() && d->in_prefetch == 0);
  };
  if (timeout_ms < 0)
    d->cv.wait(lk, pred);
  else if (!d->cv.wait_for(lk, std::chrono::milliseconds(timeout_ms), pred))
    return -2;
  if (d->failed) return -3;
  if (d->ready.empty()) return -1;
  const int s = d->ready.front();
  d->ready.pop_front();
  const Slot& sl = d->slots[s];
  for (int f = 0; f < max_fields && f < (int)sl.bytes.size(); ++f) nbytes_out[f] = (int64_t)sl.bytes[f];
  return s;
}

// Hand slot `s` to the consumer: `stream` waits for its H2D copy, copies each field
// into dst[f] (device-to-device, or memcpy in host mode; a null dst skips it),
// then records the slot's free event so the prefetcher reuses it after these
// copies on the device -- no host synchronisation.
PA_RT_EXPORT int pa_dbr_consume(void* h, int s, void* const* dst, void* stream) {
  DBR* d = static_cast<DBR*>(h);
  if (s < 0 || s >= d->nslots) return -1;
  Slot& sl = d->slots[s];
  hipStream_t st = static_cast<hipStream_t>(stream);
  int rc = 0;
  if (host_mode(d)) {
    for (size_t f = 0; f < sl.bytes.size(); ++f)
      if (dst[f]) memcpy(dst[f], sl.dev[f], sl.bytes[f]);
  } else {
    if (hipStreamWaitEvent(st, sl.ready, 0) != hipSuccess) rc = -2;
    for (size_t f = 0; f < sl.bytes.size() && rc == 0; ++f)
      if (dst[f] && hipMemcpyAsync(dst[f], sl.dev[f], sl.bytes[f], hipMemcpyDeviceToDevice, st) != hipSuccess)
        rc = -2;
    hipEventRecord(sl.freed, st);
    sl.freed_recorded = true;
  }
  std::lock_guard<std::mutex> lk(d->mu);
  d->free_slots.push_back(s);
  d->cv.notify_all();
  if (rc) pa_rt_set_error("double-buffer reader: consume failed");
  return rc;
}

PA_RT_EXPORT size_t pa_dbr_queued(void* h) {
  DBR* d = static_cast<DBR*>(h);
  std::lock_guard<std::mutex> lk(d->mu);
  return d->queue.size() + d->ready.size() + (size_t)d->in_prefetch;
}

// Drop everything queued / prefetched and reopen (py_reader.reset()).
PA_RT_EXPORT void pa_dbr_reset(void* h) {
  DBR* d = static_cast<DBR*>(h);
  stop_thread(d);
  {
    std::lock_guard<std::mutex> lk(d->mu);
    for (auto& b : d->queue) d->pinned_pool.push_back(std::move(b));
    d->queue.clear();
    d->ready.clear();
    d->free_slots.clear();
    for (int i = d->nslots - 1; i >= 0; --i) d->free_slots.push_back(i);
    d->closed = d->stop = d->failed = false;
    d->in_prefetch = 0;
  }
  d->th = std::thread(prefetch_loop, d);
}

PA_RT_EXPORT void pa_dbr_destroy(void* h) {
  DBR* d = static_cast<DBR*>(h);
  stop_thread(d);
  for (auto& b : d->queue)
    for (void* p : b.buf) host_free(d, p);
  for (auto& b : d->pinned_pool)
    for (void* p : b.buf) host_free(d, p);
  for (auto& sl : d->slots) {
    for (void* p : sl.dev) {
      if (!p) continue;
      if (host_mode(d))
        free(p);
      else
        hipFree(p);
    }
    if (sl.ready) hipEventDestroy(sl.ready);
    if (sl.freed) hipEventDestroy(sl.freed);
  }
  if (d->copy_stream) hipStreamDestroy(d->copy_stream);
  delete d;
}
