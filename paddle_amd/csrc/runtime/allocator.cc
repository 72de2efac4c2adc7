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
  struct Blk {
    size_t size;
    int seg;
    bool free;
  };
  std::map<char*, Blk> blocks;                  // every large block by address
  std::set<std::pair<size_t, char*>> free_set;  // free large blocks by (size, address)
  std::vector<std::pair<char*, size_t>> segs;   // large segments (base, size); base null once trimmed
  size_t seg_min = 1ull << 30;                  // segments of at least 1 GiB (exact for larger requests)
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
        (void)hipGetLastError();  // clear the sticky OOM so the caller can retry
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

  // gives wholly free large segments and arenas back to the system
  bool trim() {
    bool any = false;
    for (size_t si = 0; si < segs.size(); ++si) {
      char* base = segs[si].first;
      if (!base) continue;
      auto it = blocks.find(base);
      if (it == blocks.end() || !it->second.free || it->second.size != segs[si].second) continue;
      free_set.erase({it->second.size, base});
      blocks.erase(it);
      sys_free(base);
      reserved -= segs[si].second;
      segs[si].first = nullptr;
      any = true;
    }
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

  // Large pool: best-fit over free blocks of the segments, split on allocation,
  // coalesced with free neighbours of the same segment on release (the
  // reference buddy_allocator.cc pool semantics, at 512-B granularity).
  void* alloc_large(size_t n) {
    const size_t sz = (n + 511) & ~(size_t)511;
    auto it = free_set.lower_bound({sz, nullptr});
    if (it == free_set.end()) {
      size_t seg_sz = std::max<size_t>(seg_min, (sz + (2ull << 20) - 1) & ~((size_t)(2ull << 20) - 1));
      char* base = sys_alloc(seg_sz);
      if (!base && trim()) base = sys_alloc(seg_sz);
      if (!base && seg_sz > sz) {  // no room for a full segment: an exact one
        seg_sz = sz;
        base = sys_alloc(seg_sz);
      }
      if (!base) return nullptr;
      segs.push_back({base, seg_sz});
      reserved += seg_sz;
      blocks[base] = {seg_sz, (int)segs.size() - 1, true};
      it = free_set.insert({seg_sz, base}).first;
    }
    char* p = it->second;
    Blk b = blocks[p];
    free_set.erase(it);
    if (b.size - sz >= (1ull << 20)) {  // split: remainder stays free
      char* rest = p + sz;
      blocks[rest] = {b.size - sz, b.seg, true};
      free_set.insert({b.size - sz, rest});
      b.size = sz;
    }
    b.free = false;
    blocks[p] = b;
    used += b.size;
    if (used > peak) peak = used;
    return p;
  }

  bool release_large(char* p) {
    auto it = blocks.find(p);
    if (it == blocks.end() || it->second.free) return false;
    used -= it->second.size;
    it->second.free = true;
    // merge with the next block of the same segment
    auto nx = std::next(it);
    if (nx != blocks.end() && nx->second.free && nx->second.seg == it->second.seg && it->first + it->second.size == nx->first) {
      free_set.erase({nx->second.size, nx->first});
      it->second.size += nx->second.size;
      blocks.erase(nx);
    }
    // merge into the previous block of the same segment
    if (it != blocks.begin()) {
      auto pv = std::prev(it);
      if (pv->second.free && pv->second.seg == it->second.seg && pv->first + pv->second.size == it->first) {
        free_set.erase({pv->second.size, pv->first});
        pv->second.size += it->second.size;
        blocks.erase(it);
        it = pv;
      }
    }
    free_set.insert({it->second.size, it->first});
    return true;
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
    if (release_large((char*)ptr)) return 0;
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
    for (auto& sg : segs)
      if (sg.first) sys_free(sg.first);
  }
};

std::mutex g_mu;
size_t g_torch_chunk = 4ull << 30;
// Torch hook pools: one allocator per (device, stream).  torch's pluggable
// allocator frees a block with the stream it was allocated on, and a block only
// ever returns to its own stream's pool, so reuse is ordered by that stream and a
// plain free needs no event or host synchronisation.  A block that was also used
// on other streams (Tensor.record_stream -> pa_torch_record_stream) is released
// only after an event recorded on each of those streams at free time has
// completed -- the caching allocator's record_stream contract.
std::map<std::pair<int, hipStream_t>, Buddy*> g_torch;
std::unordered_map<void*, std::vector<hipStream_t>> g_uses;  // ptr -> extra streams
struct Deferred {
  void* ptr;
  int device;
  hipStream_t stream;
  std::vector<hipEvent_t> events;
};
std::vector<Deferred> g_deferred;

Buddy* torch_pool(int device, hipStream_t s) {
  auto& b = g_torch[{device, s}];
  if (!b) {
    b = new Buddy();
    b->device = device;
    b->chunk = g_torch_chunk;
  }
  return b;
}

void release_now(void* ptr, int device, hipStream_t stream) {
  auto it = g_torch.find({device, stream});
  if (it != g_torch.end() && it->second->release(ptr) == 0) return;
  for (auto& kv : g_torch)  // defensive: a block freed with another stream
    if (kv.first.first == device && kv.second->release(ptr) == 0) return;
}

// releases the deferred blocks whose events have all completed (wait: block on them)
void drain_deferred(bool wait) {
  size_t keep = 0;
  for (size_t i = 0; i < g_deferred.size(); ++i) {
    Deferred& d = g_deferred[i];
    bool done = true;
    for (hipEvent_t e : d.events) {
      hipError_t q = wait ? hipEventSynchronize(e) : hipEventQuery(e);
      if (q == hipErrorNotReady) {
        done = false;
        break;
      }
      if (q != hipSuccess) (void)hipGetLastError();  // a failed event: treat as completed
    }
    if (done) {
      for (hipEvent_t e : d.events) hipEventDestroy(e);
      release_now(d.ptr, d.device, d.stream);
    } else {
      g_deferred[keep++] = std::move(d);
    }
  }
  g_deferred.resize(keep);
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

PA_RT_EXPORT void* pa_torch_malloc(ssize_t size, int device, hipStream_t stream) {
  std::lock_guard<std::mutex> g(g_mu);
  if (!g_deferred.empty()) drain_deferred(false);
  Buddy* b = torch_pool(device, stream);
  void* p = b->alloc((size_t)size);
  if (!p && !g_deferred.empty()) {  // blocks still waiting on other streams: wait for them
    drain_deferred(true);
    p = b->alloc((size_t)size);
  }
  if (!p) {  // out of memory: return other streams' wholly free segments, retry
    for (auto& kv : g_torch)
      if (kv.first.first == device && kv.second != b) {
        std::lock_guard<std::mutex> gb(kv.second->mu);
        kv.second->trim();
      }
    p = b->alloc((size_t)size);
  }
  return p;
}

PA_RT_EXPORT void pa_torch_record_stream(void* ptr, hipStream_t stream) {
  if (!ptr) return;
  std::lock_guard<std::mutex> g(g_mu);
  auto& v = g_uses[ptr];
  for (hipStream_t s : v)
    if (s == stream) return;
  v.push_back(stream);
}

PA_RT_EXPORT void pa_torch_free(void* ptr, ssize_t, int device, hipStream_t stream) {
  if (!ptr) return;
  std::lock_guard<std::mutex> g(g_mu);
  auto u = g_uses.find(ptr);
  if (u != g_uses.end()) {
    Deferred d{ptr, device, stream, {}};
    int prev;
    hipGetDevice(&prev);
    hipSetDevice(device);
    for (hipStream_t s : u->second) {
      if (s == stream) continue;
      hipEvent_t e;
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
        (void)hipGetLastError();
        hipStreamSynchronize(s);  // no event: order the reuse by waiting now
        continue;
      }
      hipEventRecord(e, s);
      d.events.push_back(e);
    }
    hipSetDevice(prev);
    g_uses.erase(u);
    if (!d.events.empty()) {
      g_deferred.push_back(std::move(d));
      return;
    }
  }
  release_now(ptr, device, stream);
}

PA_RT_EXPORT size_t pa_torch_deferred_frees() {
  std::lock_guard<std::mutex> g(g_mu);
  return g_deferred.size();
}

PA_RT_EXPORT void pa_torch_stats(int device, size_t* used, size_t* reserved, size_t* peak) {
  std::lock_guard<std::mutex> g(g_mu);
  *used = *reserved = *peak = 0;
  for (auto& kv : g_torch)
    if (kv.first.first == device) {
      size_t u, r, pk, n;
      pa_buddy_stats(kv.second, &u, &r, &pk, &n);
      *used += u;
      *reserved += r;
      *peak += pk;  // sum of per-stream peaks (an upper bound of the joint peak)
    }
}
