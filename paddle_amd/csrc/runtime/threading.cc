// Threading primitives of the runtime:
//  * BlockingQueue of byte records (reference: operators/reader/
//    lod_tensor_blocking_queue.h, framework/blocking_queue.h) with close semantics;
//  * RecordIO prefetcher: N reader threads stream record files into a queue
//    (reference: open_files_op.cc multi-thread file reader), off the Python thread;
//  * DAG scheduler: dependency-counting executor over a thread pool with an
//    exception holder (reference: details/threaded_ssa_graph_executor.cc:36-129,
//    exception_holder.h) -- the ParallelExecutor's SSA-graph engine;
//  * profiler event buffers: per-thread RAII push/pop ranges, chrome-trace dump
//    (reference: platform/profiler.cc:36-160 EventList, tools/timeline.py).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "runtime.h"

extern "C" {
void* pa_rio_scanner_open(const char* path);
int pa_rio_scanner_next(void* h, const char** data, size_t* len);
void pa_rio_scanner_close(void* h);
}

namespace {
struct BQ {
  size_t cap;
  std::deque<std::string> q;
  std::mutex mu;
  std::condition_variable not_full, not_empty;
  bool closed = false;
  std::vector<std::thread> producers;
  std::atomic<int> live_producers{0};
};
}  // namespace

PA_RT_EXPORT void* pa_bq_create(size_t capacity) {
  BQ* b = new BQ();
  b->cap = capacity ? capacity : 1;
  return b;
}

// Returns 0 ok, 1 if the queue is closed.
PA_RT_EXPORT int pa_bq_push(void* h, const char* data, size_t len) {
  BQ* b = (BQ*)h;
  std::unique_lock<std::mutex> l(b->mu);
  b->not_full.wait(l, [b] { return b->closed || b->q.size() < b->cap; });
  if (b->closed) return 1;
  b->q.emplace_back(data, len);
  b->not_empty.notify_one();
  return 0;
}

// Pops one record into a malloc'd buffer (free with pa_rt_free).  Returns 1 ok,
// 0 when closed and drained, -1 on timeout.
PA_RT_EXPORT int pa_bq_pop(void* h, char** out, size_t* len, int timeout_ms) {
  BQ* b = (BQ*)h;
  std::unique_lock<std::mutex> l(b->mu);
  auto ready = [b] { return !b->q.empty() || b->closed; };
  if (timeout_ms < 0) b->not_empty.wait(l, ready);
  else if (!b->not_empty.wait_for(l, std::chrono::milliseconds(timeout_ms), ready)) return -1;
  if (b->q.empty()) return 0;
  std::string s = std::move(b->q.front());
  b->q.pop_front();
  b->not_full.notify_one();
  l.unlock();
  *out = (char*)malloc(s.size() ? s.size() : 1);
  memcpy(*out, s.data(), s.size());
  *len = s.size();
  return 1;
}

PA_RT_EXPORT size_t pa_bq_size(void* h) {
  BQ* b = (BQ*)h;
  std::lock_guard<std::mutex> l(b->mu);
  return b->q.size();
}

PA_RT_EXPORT void pa_bq_close(void* h) {
  BQ* b = (BQ*)h;
  std::lock_guard<std::mutex> l(b->mu);
  b->closed = true;
  b->not_full.notify_all();
  b->not_empty.notify_all();
}

PA_RT_EXPORT void pa_bq_destroy(void* h) {
  BQ* b = (BQ*)h;
  pa_bq_close(h);
  for (auto& t : b->producers)
    if (t.joinable()) t.join();
  delete b;
}

PA_RT_EXPORT void pa_rt_free(void* p) { free(p); }

// Start `nthreads` readers over `npaths` RecordIO files (round-robin), `passes`
// passes; the queue is closed when every reader finishes.
PA_RT_EXPORT int pa_bq_start_recordio_readers(void* h, const char** paths, int npaths, int nthreads, int passes) {
  BQ* b = (BQ*)h;
  std::vector<std::string> files(paths, paths + npaths);
  if (nthreads < 1) nthreads = 1;
  b->live_producers = nthreads;
  for (int t = 0; t < nthreads; ++t) {
    b->producers.emplace_back([b, files, t, nthreads, passes] {
      for (int p = 0; p < passes; ++p) {
        for (size_t i = t; i < files.size(); i += nthreads) {
          void* s = pa_rio_scanner_open(files[i].c_str());
          if (!s) continue;
          const char* d;
          size_t n;
          while (pa_rio_scanner_next(s, &d, &n) == 1) {
            if (pa_bq_push(b, d, n) != 0) {
              pa_rio_scanner_close(s);
              goto done;
            }
          }
          pa_rio_scanner_close(s);
        }
      }
    done:
      if (--b->live_producers == 0) pa_bq_close(b);
    });
  }
  return 0;
}

// ------------------------------------------------------------------ DAG scheduler
typedef int (*pa_node_fn)(int node, void* user);

// CSR successor lists: succ[succ_off[i] .. succ_off[i+1]).  Runs every node once,
// respecting dependencies, on `nthreads` workers; the first failing node's rc is
// returned after in-flight nodes drain (exception-holder semantics).
PA_RT_EXPORT int pa_dag_run(int n, const int* indeg_in, const int* succ_off, const int* succ, int nthreads,
                            pa_node_fn fn, void* user) {
  std::vector<std::atomic<int>> indeg(n);
  for (int i = 0; i < n; ++i) indeg[i] = indeg_in[i];
  std::deque<int> ready;
  std::mutex mu;
  std::condition_variable cv;
  int done = 0, inflight = 0, err = 0;
  for (int i = 0; i < n; ++i)
    if (indeg_in[i] == 0) ready.push_back(i);
  auto worker = [&]() {
    for (;;) {
      int node;
      {
        std::unique_lock<std::mutex> l(mu);
        cv.wait(l, [&] { return !ready.empty() || done == n || (err && inflight == 0); });
        if (done == n || (err && inflight == 0) || (err && ready.empty())) {
          cv.notify_all();
          return;
        }
        if (err) {  // stop scheduling new work
          ready.clear();
          cv.notify_all();
          return;
        }
        node = ready.front();
        ready.pop_front();
        inflight++;
      }
      int rc = fn(node, user);
      {
        std::lock_guard<std::mutex> l(mu);
        inflight--;
        done++;
        if (rc != 0 && !err) err = rc;
        if (!err)
          for (int k = succ_off[node]; k < succ_off[node + 1]; ++k)
            if (--indeg[succ[k]] == 0) ready.push_back(succ[k]);
      }
      cv.notify_all();
    }
  };
  if (nthreads < 1) nthreads = 1;
  std::vector<std::thread> ts;
  for (int t = 1; t < nthreads; ++t) ts.emplace_back(worker);
  worker();
  for (auto& t : ts) t.join();
  if (!err && done != n) {
    pa_rt_set_error("dependency cycle: %d of %d nodes ran", done, n);
    return -1;
  }
  return err;
}

// ------------------------------------------------------------------ profiler buffers
namespace {
struct Ev {
  int name;
  uint64_t t0, t1;
  uint64_t tid;
};
struct ThreadBuf {
  std::vector<Ev> done;
  std::vector<std::pair<int, uint64_t>> stack;
  uint64_t tid;
};
std::atomic<bool> g_prof_on{false};
std::mutex g_prof_mu;
std::vector<std::string> g_names;
// owned here (freed at exit); a thread keeps a raw pointer to its own buffer
std::vector<std::unique_ptr<ThreadBuf>> g_bufs;
thread_local ThreadBuf* t_buf = nullptr;
uint64_t now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}
int name_id(const char* s) {
  std::lock_guard<std::mutex> l(g_prof_mu);
  for (size_t i = 0; i < g_names.size(); ++i)
    if (g_names[i] == s) return (int)i;
  g_names.emplace_back(s);
  return (int)g_names.size() - 1;
}
ThreadBuf* buf() {
  if (!t_buf) {
    t_buf = new ThreadBuf();
    t_buf->tid = std::hash<std::thread::id>()(std::this_thread::get_id());
    std::lock_guard<std::mutex> l(g_prof_mu);
    g_bufs.emplace_back(t_buf);
  }
  return t_buf;
}
}  // namespace

PA_RT_EXPORT void pa_prof_enable(int on) { g_prof_on = on != 0; }

PA_RT_EXPORT void pa_prof_push(const char* name) {
  if (!g_prof_on) return;
  buf()->stack.emplace_back(name_id(name), now_ns());
}

PA_RT_EXPORT void pa_prof_pop() {
  if (!g_prof_on) return;
  ThreadBuf* b = buf();
  if (b->stack.empty()) return;
  auto e = b->stack.back();
  b->stack.pop_back();
  b->done.push_back({e.first, e.second, now_ns(), b->tid});
}

PA_RT_EXPORT void pa_prof_reset() {
  std::lock_guard<std::mutex> l(g_prof_mu);
  for (auto& b : g_bufs) {
    b->done.clear();
    b->stack.clear();
  }
}

// Writes a chrome://tracing JSON; returns the number of events.
PA_RT_EXPORT long pa_prof_dump(const char* path) {
  std::lock_guard<std::mutex> l(g_prof_mu);
  FILE* f = fopen(path, "w");
  if (!f) return -1;
  fprintf(f, "{\"traceEvents\":[");
  long n = 0;
  for (auto& b : g_bufs)
    for (auto& e : b->done) {
      fprintf(f, "%s{\"name\":\"%s\",\"ph\":\"X\",\"pid\":0,\"tid\":%llu,\"ts\":%.3f,\"dur\":%.3f}", n ? "," : "",
              g_names[e.name].c_str(), (unsigned long long)(e.tid % 1000000), e.t0 / 1e3, (e.t1 - e.t0) / 1e3);
      n++;
    }
  fprintf(f, "]}\n");
  fclose(f);
  return n;
}
