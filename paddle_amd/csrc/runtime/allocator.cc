// Buddy allocator over HIP device (or host) arenas.
//
// Reference: memory/detail/buddy_allocator.{h,cc} (Alloc :52, RefillPool :185) on a
// SystemAllocator (hipMalloc / posix_memalign); first device chunk =
// FLAGS_fraction_of_gpu_memory_to_use of free memory.  MI355X version: arenas are
// large power-of-two hipMalloc regions (288 GB HBM -> few, huge arenas), blocks are
// split/merged by order with per-order free sets, 256-B minimum block (matches the
// 256-B alignment the gfx950 kernels rely on for 16-B vector loads).  Exposes the
// torch "pluggable allocator" entry points so PyTorch tensors can live in it
// (FLAGS_allocator_strategy=buddy).
#include <hip/hip_runtime_api.h>
#include <stdlib.h>
#include <string.h>

#include <map>
#include <mutex>
#include <set>
#include <unordered_map>
#include <vector>

#include "runtime.h"

namespace {
constexpr int kMinOrder = 8;  // 256 B

struct Arena {
  char* base;
  int order;  // arena size = 1 << order
  std::vector<std::set<size_t>> free_by_order;  // offsets
};

struct Buddy {
  int device = -1;  // -1 = host
  size_t chunk = 1ull << 30;
  bool init_mem = false;
  std::vector<Arena> arenas;
  std::unordered_map<char*, std::pair<int, int>> live;  // ptr -> (arena, order)
  // Large requests skip the power-of-two buddy (up to 2x waste at these sizes):
  // they get exact-size blocks (2 MiB granularity) cached by size for reuse
  // (reference buddy_allocator.cc: requests above max_chunk_size go straight to
  // the system allocator).
  size_t large = 32ull << 20;
  std::multimap<size_t, char*> large_free;       // size -> block
  std::unordered_map<char*, size_t> large_live;  // block -> size
  size_t used = 0, reserved = 0, peak = 0;
  std::mutex mu;

  static int order_for(size_t n) {
    int o = kMinOrder;
    while ((1ull << o) < n) ++o;
    return o;
  }

  char* sys_alloc(size_t sz) {
    char* p = nullptr;
    if (device >= 0) {
      int prev;
      hipGetDevice(&prev);
      hipSetDevice(device);
      hipError_t e = hipMalloc((void**)&p, sz);
      hipSetDevice(prev);
      if (e != hipSuccess) {
        hipGetLastError();  // clear the sticky OOM so the caller can retry
        pa_rt_set_error("hipMalloc(%zu) failed: %d", sz, (int)e);
        return nullptr;
      }
    } else if (posix_memalign((void**)&p, 4096, sz) != 0) {
      pa_rt_set_error("posix_memalign(%zu) failed", sz);
      return nullptr;
    }
    return p;
  }

  void sys_free(char* p) {
    if (device >= 0) hipFree(p);
    else free(p);
  }

  // gives cached large blocks and wholly free arenas back to the system
  bool trim() {
    bool any = !large_free.empty();
    for (auto& kv : large_free) {
      sys_free(kv.second);
      reserved -= kv.first;
    }
    large_free.clear();
    for (size_t ai = 0; ai < arenas.size(); ++ai) {
      Arena& a = arenas[ai];
      if (a.base && a.free_by_order[a.order].count(0)) {
        sys_free(a.base);
        reserved -= 1ull << a.order;
        a.base = nullptr;  // slot kept so live (arena index) entries stay valid
        a.free_by_order.assign(a.order + 1, {});
        any = true;
      }
    }
    return any;
  }

  bool refill(int need_order) {
    int o = order_for(chunk);
    if (o < need_order) o = need_order;
    size_t sz = 1ull << o;
    char* p = sys_alloc(sz);
    if (!p && trim()) p = sys_alloc(sz);
    if (!p) return false;
    for (auto& a : arenas)  // reuse a trimmed slot
      if (!a.base) {
        a.base = p;
        a.order = o;
        a.free_by_order.assign(o + 1, {});
        a.free_by_order[o].insert(0);
        reserved += sz;
        return true;
      }
    Arena a;
    a.base = p;
    a.order = o;
    a.free_by_order.resize(o + 1);
    a.free_by_order[o].insert(0);
    arenas.push_back(std::move(a));
    reserved += sz;
    return true;
  }

  void* alloc_large(size_t n) {
    const size_t sz = (n + (2ull << 20) - 1) & ~((2ull << 20) - 1);
    // best fit within 1/8 slack
    auto it = large_free.lower_bound(sz);
    if (it != large_free.end() && it->first <= sz + sz / 8) {
      char* p = it->second;
      const size_t have = it->first;
      large_free.erase(it);
      large_live[p] = have;
      used += have;
      if (used > peak) peak = used;
      return p;
    }
    char* p = sys_alloc(sz);
    if (!p && trim()) p = sys_alloc(sz);
    if (!p) return nullptr;
    reserved += sz;
    large_live[p] = sz;
    used += sz;
    if (used > peak) peak = used;
    return p;
  }

  void* alloc(size_t n) {
    std::lock_guard<std::mutex> g(mu);
    if (n >= large) return alloc_large(n);
    int want = order_for(n ? n : 1);
    for (int pass = 0; pass < 2; ++pass) {
      for (size_t ai = 0; ai < arenas.size(); ++ai) {
        Arena& a = arenas[ai];
        if (!a.base) continue;
        for (int o = want; o <= a.order; ++o) {
          if (a.free_by_order[o].empty()) continue;
          size_t off = *a.free_by_order[o].begin();
          a.free_by_order[o].erase(a.free_by_order[o].begin());
          while (o > want) {  // split, keep lower half
            --o;
            a.free_by_order[o].insert(off + (1ull << o));
          }
          char* p = a.base + off;
          live[p] = {(int)ai, want};
          used += 1ull << want;
          if (used > peak) peak = used;
          if (init_mem && device < 0) memset(p, 0xCD, 1ull << want);
          return p;
        }
      }
      if (pass == 0 && !refill(want)) return nullptr;
    }
    return nullptr;
  }

  int release(void* ptr) {
    std::lock_guard<std::mutex> g(mu);
    auto lg = large_live.find((char*)ptr);
    if (lg != large_live.end()) {
      used -= lg->second;
      large_free.emplace(lg->second, lg->first);
      large_live.erase(lg);
      return 0;
    }
    auto it = live.find((char*)ptr);
    if (it == live.end()) {
      pa_rt_set_error("free of unknown pointer");
      return -1;
    }
    int ai = it->second.first, o = it->second.second;
    live.erase(it);
    used -= 1ull << o;
    Arena& a = arenas[ai];
    size_t off = (char*)ptr - a.base;
    while (o < a.order) {  // merge with buddy while it is free
      size_t bud = off ^ (1ull << o);
      auto f = a.free_by_order[o].find(bud);
      if (f == a.free_by_order[o].end()) break;
      a.free_by_order[o].erase(f);
      off = off < bud ? off : bud;
      ++o;
    }
    a.free_by_order[o].insert(off);
    return 0;
  }

  ~Buddy() {
    for (auto& a : arenas)
      if (a.base) sys_free(a.base);
    for (auto& kv : large_free) sys_free(kv.second);
    for (auto& kv : large_live) sys_free(kv.first);
  }
};

std::mutex g_mu;
std::map<int, Buddy*> g_torch;  // device -> allocator used by the torch hook
size_t g_torch_chunk = 4ull << 30;

// Stream-ordered release for the torch hook: a freed block may still be read by
// kernels queued on its stream, so free() records an event there and the block
// returns to the buddy pool once the event has completed (polled on the next
// allocation; all pending events are waited for only when an allocation would
// otherwise fail) -- no host synchronisation on the free path.
struct Pending {
  void* ptr;
  hipEvent_t ev;
};
std::map<int, std::vector<Pending>> g_pending;
std::vector<hipEvent_t> g_event_pool;

hipEvent_t take_event() {
  if (!g_event_pool.empty()) {
    hipEvent_t e = g_event_pool.back();
    g_event_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  hipEventCreateWithFlags(&e, hipEventDisableTiming);
  return e;
}

// caller holds g_mu; wait == true blocks on every pending event
void drain(int device, Buddy* b, bool wait) {
  auto& pend = g_pending[device];
  size_t keep = 0;
  for (size_t i = 0; i < pend.size(); ++i) {
    Pending& q = pend[i];
    const hipError_t st = wait ? hipEventSynchronize(q.ev) : hipEventQuery(q.ev);
    if (st == hipSuccess) {
      b->release(q.ptr);
      g_event_pool.push_back(q.ev);
    } else {
      pend[keep++] = q;
    }
  }
  pend.resize(keep);
}
}  // namespace

PA_RT_EXPORT void* pa_buddy_create(int device, size_t chunk_bytes, int init_mem) {
  Buddy* b = new Buddy();
  b->device = device;
  if (chunk_bytes) b->chunk = chunk_bytes;
  b->init_mem = init_mem != 0;
  return b;
}

PA_RT_EXPORT void pa_buddy_destroy(void* h) { delete (Buddy*)h; }
PA_RT_EXPORT void* pa_buddy_alloc(void* h, size_t n) { return ((Buddy*)h)->alloc(n); }
PA_RT_EXPORT int pa_buddy_free(void* h, void* p) { return ((Buddy*)h)->release(p); }

PA_RT_EXPORT void pa_buddy_stats(void* h, size_t* used, size_t* reserved, size_t* peak, size_t* narenas) {
  Buddy* b = (Buddy*)h;
  std::lock_guard<std::mutex> g(b->mu);
  *used = b->used;
  *reserved = b->reserved;
  *peak = b->peak;
  *narenas = b->arenas.size();
}

// ---- torch CUDAPluggableAllocator hooks (HIP build of torch uses hipStream_t)
PA_RT_EXPORT void pa_torch_set_chunk(size_t bytes) { g_torch_chunk = bytes; }

PA_RT_EXPORT void* pa_torch_malloc(ssize_t size, int device, hipStream_t) {
  std::lock_guard<std::mutex> g(g_mu);
  Buddy* b;
  auto it = g_torch.find(device);
  if (it == g_torch.end()) {
    b = new Buddy();
    b->device = device;
    b->chunk = g_torch_chunk;
    g_torch[device] = b;
  } else {
    b = it->second;
  }
  drain(device, b, false);
  void* p = b->alloc((size_t)size);
  if (!p && !g_pending[device].empty()) {  // blocks still in flight: wait for them, retry
    drain(device, b, true);
    p = b->alloc((size_t)size);
  }
  return p;
}

PA_RT_EXPORT void pa_torch_free(void* ptr, ssize_t, int device, hipStream_t stream) {
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_torch.find(device);
  if (it == g_torch.end() || !ptr) return;
  hipEvent_t ev = take_event();
  if (ev && hipEventRecord(ev, stream) == hipSuccess) {
    g_pending[device].push_back({ptr, ev});
  } else {  // no event: fall back to a synchronous release
    if (ev) g_event_pool.push_back(ev);
    if (stream) hipStreamSynchronize(stream);
    it->second->release(ptr);
  }
}

PA_RT_EXPORT void pa_torch_stats(int device, size_t* used, size_t* reserved, size_t* peak) {
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_torch.find(device);
  if (it == g_torch.end()) {
    *used = *reserved = *peak = 0;
    return;
  }
  size_t n;
  pa_buddy_stats(it->second, used, reserved, peak, &n);
}
