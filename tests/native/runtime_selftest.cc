// Self-test of the native runtime (paddle_amd/csrc/runtime) built together with the
// runtime sources under AddressSanitizer + UBSan (and, separately, ThreadSanitizer)
// by tests/test_native_sanitizers_cpu.py.  SURVEY §5.2: the reference has no
// sanitizer builds at all; this is the host-side half of that gap (GPU ASan is not
// available on this machine pool).
//
// Exercises: buddy allocator (host place) with split/merge + init_mem poisoning,
// RecordIO round trip (gzip + plain), LoDTensor stream round trip, blocking queue
// with concurrent producers/consumers and close, DAG scheduler on a diamond graph
// with a failing node, profiler buffers from several threads, the parameter
// optimizer (config parse, updates, state save / resume, truncated inputs).
#include <atomic>
#include <cassert>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../paddle_amd/csrc/runtime/runtime.h"

extern "C" {
void* pa_buddy_create(int device, size_t chunk_bytes, int init_mem);
void pa_buddy_destroy(void* h);
void* pa_buddy_alloc(void* h, size_t n);
int pa_buddy_free(void* h, void* p);
void pa_buddy_stats(void* h, size_t* used, size_t* reserved, size_t* peak, size_t* narenas);
void* pa_rio_writer_open(const char* path, int compressor, int max_records);
int pa_rio_writer_write(void* h, const char* data, size_t len);
int pa_rio_writer_close(void* h);
void* pa_rio_scanner_open(const char* path);
int pa_rio_scanner_next(void* h, const char** data, size_t* len);
void pa_rio_scanner_close(void* h);
void* pa_ts_open(const char* path, int write, int append);
int pa_ts_close(void* h);
int pa_ts_write_lod_tensor(void* h, int lod_level, const uint64_t* lod_flat, const int64_t* lod_lens, int dtype,
                           int ndims, const int64_t* dims, const void* data, size_t nbytes);
int pa_ts_read_header(void* h, int* lod_level, uint64_t* lod_flat, int64_t* lod_lens, int lod_levels_cap, int lod_cap, int* dtype,
                      int* ndims, int64_t* dims, int dims_cap, size_t* nbytes, int elem_size_by_dtype[32]);
int pa_ts_read_data(void* h, void* dst, size_t nbytes);
void* pa_bq_create(size_t capacity);
int pa_bq_push(void* h, const char* data, size_t len);
int pa_bq_pop(void* h, char** out, size_t* len, int timeout_ms);
void pa_bq_close(void* h);
void pa_bq_destroy(void* h);
void pa_rt_free(void* p);
typedef int (*pa_node_fn)(int node, void* user);
int pa_dag_run(int n, const int* indeg_in, const int* succ_off, const int* succ, int nthreads, pa_node_fn fn,
               void* user);
void pa_prof_enable(int on);
void* pa_opt_create(const unsigned char* config, int config_len, int dtype, void* param, int num_bytes,
                    const char* state, int state_len);
int pa_opt_release(void* h);
int pa_opt_update(void* h, int dtype, const void* grad, int num_bytes);
int pa_opt_get_weights(void* h, void** buf);
int pa_opt_get_state(void* h, const char** st);
void pa_prof_push(const char* name);
void pa_prof_pop();
long pa_prof_dump(const char* path);
}

#define CHECK(c)                                                          \
  do {                                                                    \
    if (!(c)) {                                                           \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                       \
    }                                                                     \
  } while (0)

static void test_buddy() {
  void* b = pa_buddy_create(-1, 1 << 20, 1);
  std::vector<void*> ps;
  for (int i = 0; i < 200; ++i) {
    size_t n = 64u << (i % 9);
    void* p = pa_buddy_alloc(b, n);
    CHECK(p != nullptr);
    std::memset(p, i & 0xff, n);  // writing the whole block must stay in bounds
    ps.push_back(p);
  }
  for (size_t i = 0; i < ps.size(); i += 2) CHECK(pa_buddy_free(b, ps[i]) == 0);
  for (size_t i = 1; i < ps.size(); i += 2) CHECK(pa_buddy_free(b, ps[i]) == 0);
  size_t used, reserved, peak, narenas;
  pa_buddy_stats(b, &used, &reserved, &peak, &narenas);
  CHECK(used == 0 && peak > 0);
  void* big = pa_buddy_alloc(b, 3u << 20);  // larger than one chunk
  CHECK(big != nullptr);
  std::memset(big, 1, 3u << 20);
  CHECK(pa_buddy_free(b, big) == 0);
  pa_buddy_destroy(b);
}

static void test_recordio(const std::string& dir) {
  for (int comp : {0, 2}) {
    std::string path = dir + "/t" + std::to_string(comp) + ".recordio";
    void* w = pa_rio_writer_open(path.c_str(), comp, 7);
    CHECK(w);
    for (int i = 0; i < 100; ++i) {
      std::string rec(i * 13 + 1, char('a' + i % 26));
      CHECK(pa_rio_writer_write(w, rec.data(), rec.size()) == 0);
    }
    CHECK(pa_rio_writer_close(w) == 0);
    void* s = pa_rio_scanner_open(path.c_str());
    CHECK(s);
    const char* d;
    size_t n;
    int i = 0;
    while (pa_rio_scanner_next(s, &d, &n) == 1) {
      CHECK(n == size_t(i * 13 + 1) && d[0] == char('a' + i % 26) && d[n - 1] == d[0]);
      ++i;
    }
    CHECK(i == 100);
    pa_rio_scanner_close(s);
  }
}

static void test_tensor_stream(const std::string& dir) {
  std::string path = dir + "/t.lodtensor";
  void* f = pa_ts_open(path.c_str(), 1, 0);
  uint64_t lod[] = {0, 2, 5};
  int64_t lens[] = {3};
  int64_t dims[] = {5, 4};
  std::vector<float> data(20);
  for (int i = 0; i < 20; ++i) data[i] = i * 0.5f;
  CHECK(pa_ts_write_lod_tensor(f, 1, lod, lens, /*FP32*/ 5, 2, dims, data.data(), data.size() * 4) == 0);
  pa_ts_close(f);
  f = pa_ts_open(path.c_str(), 0, 0);
  int lod_level, dtype, ndims;
  uint64_t lod2[8];
  int64_t lens2[4], dims2[8];
  size_t nbytes;
  int esz[32] = {0};
  esz[5] = 4;
  CHECK(pa_ts_read_header(f, &lod_level, lod2, lens2, 4, 8, &dtype, &ndims, dims2, 8, &nbytes, esz) == 1);
  CHECK(lod_level == 1 && lens2[0] == 3 && lod2[2] == 5 && ndims == 2 && dims2[1] == 4 && nbytes == 80);
  std::vector<float> back(20);
  CHECK(pa_ts_read_data(f, back.data(), nbytes) == 0);
  CHECK(std::memcmp(back.data(), data.data(), 80) == 0);
  pa_ts_close(f);
}

static void test_queue() {
  void* q = pa_bq_create(8);
  std::atomic<long> sum{0};
  std::vector<std::thread> th;
  for (int p = 0; p < 4; ++p)
    th.emplace_back([q, p] {
      for (int i = 0; i < 500; ++i) {
        long v = p * 1000 + i;
        CHECK(pa_bq_push(q, (const char*)&v, sizeof v) == 0);
      }
    });
  std::vector<std::thread> cons;
  for (int c = 0; c < 3; ++c)
    cons.emplace_back([q, &sum] {
      for (;;) {
        char* out;
        size_t n;
        int r = pa_bq_pop(q, &out, &n, 2000);
        if (r != 1) break;
        CHECK(n == sizeof(long));
        sum += *(long*)out;
        pa_rt_free(out);
      }
    });
  for (auto& t : th) t.join();
  pa_bq_close(q);
  for (auto& t : cons) t.join();
  long want = 0;
  for (int p = 0; p < 4; ++p)
    for (int i = 0; i < 500; ++i) want += p * 1000 + i;
  CHECK(sum == want);
  pa_bq_destroy(q);
}

struct DagCtx {
  std::atomic<int> order[6];
  std::atomic<int> clock{0};
  int fail_node;
};

static int dag_fn(int node, void* u) {
  DagCtx* c = (DagCtx*)u;
  c->order[node] = c->clock++;
  return node == c->fail_node ? 7 : 0;
}

static void test_dag() {
  // 0 -> {1,2} -> 3 -> {4,5}
  int indeg[6] = {0, 1, 1, 2, 1, 1};
  int off[7] = {0, 2, 3, 4, 6, 6, 6};
  int succ[6] = {1, 2, 3, 3, 4, 5};
  for (int rep = 0; rep < 50; ++rep) {
    DagCtx c;
    c.fail_node = -1;
    for (auto& o : c.order) o = -1;
    CHECK(pa_dag_run(6, indeg, off, succ, 4, dag_fn, &c) == 0);
    CHECK(c.order[0] < c.order[1] && c.order[0] < c.order[2] && c.order[3] > c.order[1] &&
          c.order[3] > c.order[2] && c.order[4] > c.order[3] && c.order[5] > c.order[3]);
  }
  DagCtx c;
  c.fail_node = 3;
  CHECK(pa_dag_run(6, indeg, off, succ, 4, dag_fn, &c) == 7);
}

static void test_profiler(const std::string& dir) {
  pa_prof_enable(1);
  std::vector<std::thread> th;
  for (int t = 0; t < 4; ++t)
    th.emplace_back([] {
      for (int i = 0; i < 100; ++i) {
        pa_prof_push("outer");
        pa_prof_push("inner");
        pa_prof_pop();
        pa_prof_pop();
      }
    });
  for (auto& t : th) t.join();
  long n = pa_prof_dump((dir + "/trace.json").c_str());
  CHECK(n >= 800);
  pa_prof_enable(0);
}

static void test_param_optimizer() {
  // OptimizerConfig{optimizer: Adam(4), adam{beta_1: 0.9}, lr_policy: Const, const_lr{learning_rate: 0.01}}
  std::vector<unsigned char> cfg = {0x08, 0x04, 0x32, 0x09, 0x09};
  const double b1 = 0.9, lr = 0.01;
  unsigned char d[8];
  std::memcpy(d, &b1, 8);
  cfg.insert(cfg.end(), d, d + 8);
  cfg.insert(cfg.end(), {0x58, 0x00, 0x62, 0x09, 0x09});
  std::memcpy(d, &lr, 8);
  cfg.insert(cfg.end(), d, d + 8);
  std::vector<float> w(1000, 1.0f), g(1000, 0.5f);
  void* o = pa_opt_create(cfg.data(), (int)cfg.size(), 4, w.data(), (int)(w.size() * 4), nullptr, 0);
  assert(o);
  for (int i = 0; i < 3; ++i) assert(pa_opt_update(o, 4, g.data(), (int)(g.size() * 4)) == 0);
  assert(pa_opt_update(o, 4, g.data(), 12) != 0);  // wrong size refused
  const char* st = nullptr;
  const int n = pa_opt_get_state(o, &st);
  std::string state(st, (size_t)n);
  void* o2 = pa_opt_create(cfg.data(), (int)cfg.size(), 4, nullptr, (int)(w.size() * 4), state.data(), n);
  assert(o2);
  assert(pa_opt_update(o, 4, g.data(), (int)(g.size() * 4)) == 0);
  assert(pa_opt_update(o2, 4, g.data(), (int)(g.size() * 4)) == 0);
  void *a = nullptr, *b = nullptr;
  assert(pa_opt_get_weights(o, &a) == 1000 && pa_opt_get_weights(o2, &b) == 1000);
  assert(std::memcmp(a, b, 4000) == 0);
  for (int cut = 0; cut < n; cut += 97)  // truncated states are refused, never read past the end
    if (void* o3 = pa_opt_create(cfg.data(), (int)cfg.size(), 4, nullptr, 4000, state.data(), cut)) pa_opt_release(o3);
  for (int cut = 0; cut < (int)cfg.size(); ++cut)
    if (void* o4 = pa_opt_create(cfg.data(), cut, 4, w.data(), 4000, nullptr, 0)) pa_opt_release(o4);
  pa_opt_release(o);
  pa_opt_release(o2);
}

int main(int argc, char** argv) {
  std::string dir = argc > 1 ? argv[1] : "/tmp";
  test_buddy();
  test_recordio(dir);
  test_tensor_stream(dir);
  test_queue();
  test_dag();
  test_profiler(dir);
  test_param_optimizer();
  std::printf("runtime selftest OK\n");
  return 0;
}
