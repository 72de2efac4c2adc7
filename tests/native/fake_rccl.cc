// Fake librccl for CPU tests of the framework's RCCL layer (csrc/runtime/rccl_comm.cc,
// parallel/rccl.py) with several ranks in one host: the subset of the NCCL C ABI that
// rccl_comm.cc resolves with dlsym, implemented over one POSIX shared-memory segment
// per clique.  "Device" buffers are host pointers, streams are ignored: a call has
// completed when it returns, except between ncclGroupStart/End, where calls are
// queued and run at the outermost GroupEnd (sends first, then receives, then the
// collectives in issue order -- NCCL's fused-group semantics as far as a test can
// observe them).  Test hooks:
//   fake_rccl_inject_async_error(comm, code): every rank's ncclCommGetAsyncError
//     reports `code` (a peer failure);
//   fake_rccl_log(buf, n): this process's "enqueue <op>" / "exec <op>" event log;
//   fake_rccl_aborted(comm): 1 once ncclCommAbort ran on it.
// Built by tests/test_rccl_fake_cpu.py with g++ (never shipped, never loaded unless
// PA_RCCL_LIBRARY names it).
#include <fcntl.h>
#include <sched.h>
#include <stdint.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <functional>
#include <random>
#include <string>
#include <vector>

namespace {

constexpr int MAXR = 8;
constexpr size_t SLOT = 2u << 20;  // per-rank collective staging bytes
constexpr int RING = 4;            // messages per (src, dst) mailbox
constexpr size_t MSG = 64u << 10;  // bytes per mailbox message

struct Mailbox {
  std::atomic<long> posted;
  std::atomic<long> taken;
  size_t len[RING];
  char data[RING][MSG];
};

struct Shared {
  std::atomic<int> joined;
  std::atomic<int> left;
  std::atomic<int> nranks;
  std::atomic<int> bar_count;
  std::atomic<int> bar_gen;
  std::atomic<int> async_err;
  char slot[MAXR][SLOT];
  Mailbox box[MAXR][MAXR];
};

struct Comm {
  Shared* sh;
  int rank, n;
  std::string name;
  bool aborted = false;
};

enum { ncclSuccess = 0, ncclUnhandledCudaError = 1, ncclSystemError = 2, ncclInternalError = 3,
       ncclInvalidArgument = 4, ncclInvalidUsage = 5, ncclRemoteError = 6 };

std::string g_log;
int g_depth = 0;
struct Pending {
  int kind;  // 0 send, 1 recv, 2 collective
  std::string what;
  std::function<int()> run;
};
std::vector<Pending> g_queue;

void log_ev(const char* ev, const std::string& what) {
  g_log += ev;
  g_log += ' ';
  g_log += what;
  g_log += '\n';
}

size_t esize(int dt) {
  switch (dt) {
    case 0: case 1: return 1;
    case 2: case 3: case 7: return 4;
    case 4: case 5: case 8: return 8;
    case 6: case 9: return 2;
  }
  return 0;
}

float bf2f(uint16_t v) {
  uint32_t u = (uint32_t)v << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
uint16_t f2bf(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}

double get(const char* p, int dt, size_t i) {
  switch (dt) {
    case 0: return ((const int8_t*)p)[i];
    case 1: return ((const uint8_t*)p)[i];
    case 2: return ((const int32_t*)p)[i];
    case 3: return ((const uint32_t*)p)[i];
    case 4: return (double)((const int64_t*)p)[i];
    case 5: return (double)((const uint64_t*)p)[i];
    case 7: return ((const float*)p)[i];
    case 8: return ((const double*)p)[i];
    case 9: return bf2f(((const uint16_t*)p)[i]);
  }
  return 0;
}
void put(char* p, int dt, size_t i, double v) {
  switch (dt) {
    case 0: ((int8_t*)p)[i] = (int8_t)v; break;
    case 1: ((uint8_t*)p)[i] = (uint8_t)v; break;
    case 2: ((int32_t*)p)[i] = (int32_t)v; break;
    case 3: ((uint32_t*)p)[i] = (uint32_t)v; break;
    case 4: ((int64_t*)p)[i] = (int64_t)v; break;
    case 5: ((uint64_t*)p)[i] = (uint64_t)v; break;
    case 7: ((float*)p)[i] = (float)v; break;
    case 8: ((double*)p)[i] = v; break;
    case 9: ((uint16_t*)p)[i] = f2bf((float)v); break;
  }
}

double combine(double a, double b, int op) {
  switch (op) {
    case 1: return a * b;
    case 2: return a > b ? a : b;
    case 3: return a < b ? a : b;
    default: return a + b;
  }
}

bool spin_until(const std::function<bool()>& ok, double timeout_s = 60.0) {
  const auto t0 = std::chrono::steady_clock::now();
  while (!ok()) {
    sched_yield();
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s) return false;
  }
  return true;
}

int barrier(Comm* c) {
  Shared* s = c->sh;
  const int gen = s->bar_gen.load();
  if (s->bar_count.fetch_add(1) + 1 == c->n) {
    s->bar_count.store(0);
    s->bar_gen.fetch_add(1);
    return ncclSuccess;
  }
  return spin_until([&] { return s->bar_gen.load() != gen; }) ? ncclSuccess : ncclSystemError;
}

int checked(Comm* c) {
  if (!c || !c->sh) return ncclInvalidArgument;
  if (c->aborted) return ncclInvalidUsage;
  return ncclSuccess;
}

// run now, or queue until the outermost GroupEnd
int submit(int kind, const std::string& what, std::function<int()> fn) {
  log_ev("enqueue", what);
  if (g_depth > 0) {
    g_queue.push_back({kind, what, std::move(fn)});
    return ncclSuccess;
  }
  log_ev("exec", what);
  return fn();
}

}  // namespace

extern "C" {

typedef struct { char internal[128]; } ncclUniqueId;

const char* ncclGetErrorString(int rc) {
  static const char* s[] = {"success", "unhandled device error", "system error", "internal error",
                            "invalid argument", "invalid usage", "remote error"};
  return rc >= 0 && rc <= 6 ? s[rc] : "unknown";
}

int ncclGetUniqueId(ncclUniqueId* id) {
  memset(id->internal, 0, 128);
  std::random_device rd;
  snprintf(id->internal, 128, "/pa_fake_rccl_%d_%08x%08x", (int)getpid(), rd(), rd());
  return ncclSuccess;
}

int ncclCommInitRank(void** out, int nranks, ncclUniqueId id, int rank) {
  if (nranks < 1 || nranks > MAXR || rank < 0 || rank >= nranks) return ncclInvalidArgument;
  const std::string name(id.internal);
  const int fd = shm_open(name.c_str(), O_CREAT | O_RDWR, 0600);
  if (fd < 0) return ncclSystemError;
  if (ftruncate(fd, sizeof(Shared)) != 0) {
    close(fd);
    return ncclSystemError;
  }
  void* p = mmap(nullptr, sizeof(Shared), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) return ncclSystemError;
  Comm* c = new Comm{(Shared*)p, rank, nranks, name};
  c->sh->nranks.store(nranks);
  c->sh->joined.fetch_add(1);
  // rendezvous: CommInitRank returns once every rank of the clique joined
  if (!spin_until([&] { return c->sh->joined.load() >= nranks; })) return ncclSystemError;
  *out = c;
  return ncclSuccess;
}

static int release(Comm* c) {
  if (c->sh->left.fetch_add(1) + 1 == c->n) shm_unlink(c->name.c_str());
  munmap(c->sh, sizeof(Shared));
  c->sh = nullptr;
  return ncclSuccess;
}

int ncclCommDestroy(void* comm) {
  Comm* c = (Comm*)comm;
  if (!c || !c->sh) return ncclInvalidArgument;
  return release(c);
}

int ncclCommAbort(void* comm) {
  Comm* c = (Comm*)comm;
  if (!c) return ncclInvalidArgument;
  c->aborted = true;
  log_ev("abort", std::to_string(c->rank));
  if (c->sh) release(c);  // the handle stays valid for fake_rccl_aborted
  return ncclSuccess;
}

int ncclCommGetAsyncError(void* comm, int* err) {
  Comm* c = (Comm*)comm;
  if (!c) return ncclInvalidArgument;
  *err = c->sh ? c->sh->async_err.load() : ncclRemoteError;
  return ncclSuccess;
}

int ncclGroupStart() {
  ++g_depth;
  return ncclSuccess;
}

int ncclGroupEnd() {
  if (g_depth <= 0) return ncclInvalidUsage;
  if (--g_depth > 0) return ncclSuccess;
  std::vector<Pending> q;
  q.swap(g_queue);
  int rc = ncclSuccess;
  for (int pass = 0; pass < 3 && rc == ncclSuccess; ++pass)
    for (auto& e : q)
      if (e.kind == pass && rc == ncclSuccess) {
        log_ev("exec", e.what);
        rc = e.run();
      }
  return rc;
}

int ncclAllReduce(const void* send, void* recv, size_t count, int dt, int op, void* comm, void*) {
  Comm* c = (Comm*)comm;
  if (int rc = checked(c)) return rc;
  const size_t es = esize(dt), bytes = count * es;
  if (!es || bytes > SLOT) return ncclInvalidArgument;
  return submit(2, "all_reduce", [=] {
    memcpy(c->sh->slot[c->rank], send, bytes);
    if (barrier(c)) return (int)ncclSystemError;
    std::vector<char> tmp(bytes);
    for (size_t i = 0; i < count; ++i) {
      double a = get(c->sh->slot[0], dt, i);
      for (int r = 1; r < c->n; ++r) a = combine(a, get(c->sh->slot[r], dt, i), op);
      if (op == 4) a /= c->n;
      put(tmp.data(), dt, i, a);
    }
    if (barrier(c)) return (int)ncclSystemError;
    memcpy(recv, tmp.data(), bytes);
    return (int)ncclSuccess;
  });
}

int ncclReduceScatter(const void* send, void* recv, size_t rcount, int dt, int op, void* comm, void*) {
  Comm* c = (Comm*)comm;
  if (int rc = checked(c)) return rc;
  const size_t es = esize(dt), bytes = rcount * es * c->n;
  if (!es || bytes > SLOT) return ncclInvalidArgument;
  return submit(2, "reduce_scatter", [=] {
    memcpy(c->sh->slot[c->rank], send, bytes);
    if (barrier(c)) return (int)ncclSystemError;
    std::vector<char> tmp(rcount * es);
    for (size_t i = 0; i < rcount; ++i) {
      const size_t j = c->rank * rcount + i;
      double a = get(c->sh->slot[0], dt, j);
      for (int r = 1; r < c->n; ++r) a = combine(a, get(c->sh->slot[r], dt, j), op);
      if (op == 4) a /= c->n;
      put(tmp.data(), dt, i, a);
    }
    if (barrier(c)) return (int)ncclSystemError;
    memcpy(recv, tmp.data(), tmp.size());
    return (int)ncclSuccess;
  });
}

int ncclAllGather(const void* send, void* recv, size_t scount, int dt, void* comm, void*) {
  Comm* c = (Comm*)comm;
  if (int rc = checked(c)) return rc;
  const size_t bytes = scount * esize(dt);
  if (!bytes || bytes > SLOT) return ncclInvalidArgument;
  return submit(2, "all_gather", [=] {
    memcpy(c->sh->slot[c->rank], send, bytes);
    if (barrier(c)) return (int)ncclSystemError;
    for (int r = 0; r < c->n; ++r) memcpy((char*)recv + r * bytes, c->sh->slot[r], bytes);
    return barrier(c) ? (int)ncclSystemError : (int)ncclSuccess;
  });
}

int ncclBroadcast(const void* send, void* recv, size_t count, int dt, int root, void* comm, void*) {
  Comm* c = (Comm*)comm;
  if (int rc = checked(c)) return rc;
  const size_t bytes = count * esize(dt);
  if (!bytes || bytes > SLOT || root < 0 || root >= c->n) return ncclInvalidArgument;
  return submit(2, "broadcast", [=] {
    if (c->rank == root) memcpy(c->sh->slot[root], send, bytes);
    if (barrier(c)) return (int)ncclSystemError;
    memcpy(recv, c->sh->slot[root], bytes);
    return barrier(c) ? (int)ncclSystemError : (int)ncclSuccess;
  });
}

int ncclSend(const void* buf, size_t count, int dt, int peer, void* comm, void*) {
  Comm* c = (Comm*)comm;
  if (int rc = checked(c)) return rc;
  const size_t bytes = count * esize(dt);
  if (bytes > MSG || peer < 0 || peer >= c->n) return ncclInvalidArgument;
  return submit(0, "send " + std::to_string(peer), [=] {
    Mailbox& m = c->sh->box[c->rank][peer];
    if (!spin_until([&] { return m.posted.load() - m.taken.load() < RING; })) return (int)ncclSystemError;
    const long k = m.posted.load() % RING;
    memcpy(m.data[k], buf, bytes);
    m.len[k] = bytes;
    m.posted.fetch_add(1);
    return (int)ncclSuccess;
  });
}

int ncclRecv(void* buf, size_t count, int dt, int peer, void* comm, void*) {
  Comm* c = (Comm*)comm;
  if (int rc = checked(c)) return rc;
  const size_t bytes = count * esize(dt);
  if (bytes > MSG || peer < 0 || peer >= c->n) return ncclInvalidArgument;
  return submit(1, "recv " + std::to_string(peer), [=] {
    Mailbox& m = c->sh->box[peer][c->rank];
    if (!spin_until([&] { return m.posted.load() > m.taken.load(); })) return (int)ncclSystemError;
    const long k = m.taken.load() % RING;
    if (m.len[k] != bytes) return (int)ncclInvalidUsage;  // size mismatch between the pair
    memcpy(buf, m.data[k], bytes);
    m.taken.fetch_add(1);
    return (int)ncclSuccess;
  });
}

// ---- test hooks
void fake_rccl_inject_async_error(void* comm, int code) {
  Comm* c = (Comm*)comm;
  if (c && c->sh) c->sh->async_err.store(code);
}

int fake_rccl_log(char* buf, int n) {
  const int m = (int)g_log.size() < n - 1 ? (int)g_log.size() : n - 1;
  memcpy(buf, g_log.data(), m);
  buf[m] = 0;
  return (int)g_log.size();
}

int fake_rccl_aborted(void* comm) { return comm && ((Comm*)comm)->aborted ? 1 : 0; }

}  // extern "C"
