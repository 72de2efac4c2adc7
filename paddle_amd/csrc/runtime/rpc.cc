// Parameter-server RPC transport (TCP).
//
// Reference: paddle/fluid/operators/distributed/ -- gRPC/bRPC RPCClient/RPCServer
// with SendVariable / GetVariable / PrefetchVariable / CheckpointNotify and
// server-side batch barriers (rpc_server.h:43-115, grpc_client.cc,
// request_handler_impl.cc:35-145, send_recv.proto.in:20-84).  This is a compact
// MI355X-host equivalent with no gRPC dependency:
//
//   frame  = u32 magic | u8 type | u32 name_len | u64 payload_len | name | payload
//   reply  = u32 magic | u8 status | u64 payload_len | payload
//
//   SEND(name, bytes)      -> queued for the server loop (pa_rpc_server_pop)
//   GET(name)              -> blocks while the store is not "ready" (sync mode: the
//                             optimisation of the round is still running), then
//                             returns the published bytes of `name`
//   PREFETCH(table, ids)   -> rows of a registered dense table (id-keyed)
//   SEND_BARRIER / FETCH_BARRIER / COMPLETE / CHECKPOINT(dir)
//
// Clients keep one persistent connection per endpoint (mutex-protected), so a
// trainer's per-step traffic is a handful of request/response round trips that
// ctypes issues with the GIL released (Python threads fan them out per pserver).
// The server accepts on its own thread and serves every connection on a
// dedicated thread; variable payloads are opaque (LoDTensor / SelectedRows
// streams produced by the framework's serialiser).
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "runtime.h"

namespace {

constexpr uint32_t kMagic = 0x50415250;  // "PARP"
enum : uint8_t { SEND = 1, GET = 2, PREFETCH = 3, SEND_BARRIER = 4, FETCH_BARRIER = 5, COMPLETE = 6, CHECKPOINT = 7 };

bool read_all(int fd, void* buf, size_t n) {
  char* p = static_cast<char*>(buf);
  while (n) {
    ssize_t r = ::recv(fd, p, n, 0);
    if (r <= 0) return false;
    p += r;
    n -= static_cast<size_t>(r);
  }
  return true;
}

bool write_all(int fd, const void* buf, size_t n) {
  const char* p = static_cast<const char*>(buf);
  while (n) {
    ssize_t r = ::send(fd, p, n, MSG_NOSIGNAL);
    if (r <= 0) return false;
    p += r;
    n -= static_cast<size_t>(r);
  }
  return true;
}

#pragma pack(push, 1)
constexpr uint32_t kMaxName = 4096;
constexpr uint64_t kDefaultMaxBody = 1ull << 32;  // 4 GiB (PADDLE_AMD_RPC_MAX_BODY overrides)

struct ReqHdr {
  uint32_t magic;
  uint8_t type;
  uint32_t name_len;
  uint64_t payload_len;
};
struct RepHdr {
  uint32_t magic;
  uint8_t status;
  uint64_t payload_len;
};
#pragma pack(pop)

// --------------------------------------------------------------------- server
struct Table {
  int64_t width = 0;
  std::unordered_map<int64_t, std::vector<float>> rows;
};

struct Server {
  int listen_fd = -1;
  int port = 0;
  int fanin = 1;
  std::atomic<bool> stop{false};
  std::thread acceptor;
  std::vector<std::thread> workers;
  std::vector<int> conn_fds;

  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::pair<std::string, std::string>> recv_q;  // (name, bytes)
  std::map<std::string, std::string> store;                // published vars for GET
  std::map<std::string, Table> tables;
  bool ready = false;
  int send_barrier = 0, fetch_barrier = 0, completed = 0;
  uint64_t fetch_round = 0;
  std::deque<std::string> checkpoints;

  // Frames come from the network: bound every length before allocating
  // (reference: the gRPC transport's FLAGS_rpc_max_message_size); a bad frame or
  // an allocation failure closes only that connection, never the server.
  uint64_t max_body = kDefaultMaxBody;

  void serve(int fd) {
    try {
      serve_loop(fd);
    } catch (...) {
    }
    ::close(fd);
  }

  void serve_loop(int fd) {
    std::string name, payload;
    for (;;) {
      ReqHdr h;
      if (!read_all(fd, &h, sizeof(h)) || h.magic != kMagic) break;
      if (h.name_len > kMaxName || h.payload_len > max_body) break;
      name.resize(h.name_len);
      payload.resize(h.payload_len);
      if ((h.name_len && !read_all(fd, &name[0], h.name_len)) ||
          (h.payload_len && !read_all(fd, &payload[0], h.payload_len)))
        break;
      std::string out;
      uint8_t status = 0;
      switch (h.type) {
        case SEND: {
          std::lock_guard<std::mutex> g(mu);
          recv_q.emplace_back(name, payload);
          cv.notify_all();
          break;
        }
        case GET: {
          std::unique_lock<std::mutex> g(mu);
          cv.wait(g, [&] { return ready || stop.load(); });
          auto it = store.find(name);
          if (it == store.end()) status = 2; else out = it->second;
          break;
        }
        case PREFETCH: {
          // not gated: a round's sparse-table rows are updated before its fetch
          // barrier releases the trainers, so a prefetch always sees them
          std::lock_guard<std::mutex> g(mu);
          auto it = tables.find(name);
          if (it == tables.end()) { status = 2; break; }
          const Table& t = it->second;
          size_t n = payload.size() / sizeof(int64_t);
          const int64_t* ids = reinterpret_cast<const int64_t*>(payload.data());
          out.resize(n * t.width * sizeof(float));
          float* dst = reinterpret_cast<float*>(&out[0]);
          for (size_t i = 0; i < n; ++i) {
            auto r = t.rows.find(ids[i]);
            if (r == t.rows.end()) std::memset(dst + i * t.width, 0, t.width * sizeof(float));
            else std::memcpy(dst + i * t.width, r->second.data(), t.width * sizeof(float));
          }
          break;
        }
        case SEND_BARRIER: {
          std::lock_guard<std::mutex> g(mu);
          ++send_barrier;
          cv.notify_all();
          break;
        }
        case COMPLETE: {
          // acknowledge first: the last COMPLETE lets the server loop exit and
          // stop() shuts every connection down
          RepHdr r{kMagic, 0, 0};
          bool ok = write_all(fd, &r, sizeof(r));
          {
            std::lock_guard<std::mutex> g(mu);
            ++completed;
            cv.notify_all();
          }
          if (!ok) break;
          continue;
        }
        case FETCH_BARRIER: {
          // hold the trainer until the server closes the round (GET gate shut),
          // so nobody can GET next round's parameters from this round's store
          std::unique_lock<std::mutex> g(mu);
          ++fetch_barrier;
          cv.notify_all();
          const uint64_t r = fetch_round;
          cv.wait(g, [&] { return fetch_round != r || stop.load() || completed >= fanin; });
          break;
        }
        case CHECKPOINT: {
          std::lock_guard<std::mutex> g(mu);
          checkpoints.push_back(payload);
          cv.notify_all();
          break;
        }
        default:
          status = 1;
      }
      RepHdr r{kMagic, status, out.size()};
      if (!write_all(fd, &r, sizeof(r)) || (!out.empty() && !write_all(fd, out.data(), out.size()))) break;
    }
  }

  void accept_loop() {
    while (!stop.load()) {
      sockaddr_in addr{};
      socklen_t len = sizeof(addr);
      int fd = ::accept(listen_fd, reinterpret_cast<sockaddr*>(&addr), &len);
      if (fd < 0) {
        if (stop.load()) break;
        continue;
      }
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      std::lock_guard<std::mutex> g(mu);
      conn_fds.push_back(fd);
      workers.emplace_back([this, fd] { serve(fd); });
    }
  }
};

// --------------------------------------------------------------------- client
struct Conn {
  int fd = -1;
  std::mutex mu;
};
std::mutex g_conns_mu;
std::unordered_map<std::string, std::shared_ptr<Conn>> g_conns;

int connect_to(const std::string& ep, int timeout_ms) {
  auto colon = ep.rfind(':');
  if (colon == std::string::npos) return -1;
  std::string host = ep.substr(0, colon), port = ep.substr(colon + 1);
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (getaddrinfo(host.c_str(), port.c_str(), &hints, &res) != 0) return -1;
  int fd = -1;
  // the pserver may still be starting: retry until the deadline
  for (int waited = 0; waited <= timeout_ms; waited += 100) {
    fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (::connect(fd, res->ai_addr, res->ai_addrlen) == 0) break;
    ::close(fd);
    fd = -1;
    std::this_thread::sleep_for(std::chrono::milliseconds(100));
  }
  freeaddrinfo(res);
  if (fd >= 0) {
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  }
  return fd;
}

std::shared_ptr<Conn> get_conn(const std::string& ep) {
  std::lock_guard<std::mutex> g(g_conns_mu);
  auto& c = g_conns[ep];
  if (!c) c = std::make_shared<Conn>();
  return c;
}

int call(const char* ep, uint8_t type, const char* name, const void* payload, size_t plen, char** out,
         size_t* out_len) {
  auto c = get_conn(ep);
  std::lock_guard<std::mutex> g(c->mu);
  if (c->fd < 0) c->fd = connect_to(ep, 120000);
  if (c->fd < 0) {
    pa_rt_set_error("rpc: cannot connect to %s", ep);
    return -1;
  }
  size_t nlen = name ? std::strlen(name) : 0;
  ReqHdr h{kMagic, type, static_cast<uint32_t>(nlen), plen};
  if (!write_all(c->fd, &h, sizeof(h)) || (nlen && !write_all(c->fd, name, nlen)) ||
      (plen && !write_all(c->fd, payload, plen))) {
    ::close(c->fd);
    c->fd = -1;
    pa_rt_set_error("rpc: send to %s failed", ep);
    return -1;
  }
  RepHdr r;
  if (!read_all(c->fd, &r, sizeof(r)) || r.magic != kMagic) {
    ::close(c->fd);
    c->fd = -1;
    pa_rt_set_error("rpc: bad reply from %s", ep);
    return -1;
  }
  char* buf = nullptr;
  if (r.payload_len) {
    buf = static_cast<char*>(std::malloc(r.payload_len));
    if (!read_all(c->fd, buf, r.payload_len)) {
      std::free(buf);
      ::close(c->fd);
      c->fd = -1;
      pa_rt_set_error("rpc: truncated reply from %s", ep);
      return -1;
    }
  }
  if (out) {
    *out = buf;
    *out_len = r.payload_len;
  } else {
    std::free(buf);
  }
  if (r.status) {
    pa_rt_set_error("rpc: %s on %s failed with status %d", name ? name : "", ep, int(r.status));
    return -2;
  }
  return 0;
}

}  // namespace

// ------------------------------------------------------------------ server C ABI
// host: address to bind (the pserver's configured endpoint); NULL or "" = all interfaces.
PA_RT_EXPORT void* pa_rpc_server_create(const char* host, int port, int fanin) {
  auto* s = new Server();
  s->fanin = fanin;
  if (const char* mb = std::getenv("PADDLE_AMD_RPC_MAX_BODY")) s->max_body = std::strtoull(mb, nullptr, 10);
  s->listen_fd = ::socket(AF_INET, SOCK_STREAM, 0);
  int one = 1;
  setsockopt(s->listen_fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_addr.s_addr = htonl(INADDR_ANY);
  if (host && *host && std::strcmp(host, "0.0.0.0") != 0) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    if (getaddrinfo(host, nullptr, &hints, &res) != 0 || !res) {
      pa_rt_set_error("rpc: cannot resolve bind address %s", host);
      ::close(s->listen_fd);
      delete s;
      return nullptr;
    }
    addr.sin_addr = reinterpret_cast<sockaddr_in*>(res->ai_addr)->sin_addr;
    freeaddrinfo(res);
  }
  addr.sin_port = htons(static_cast<uint16_t>(port));
  if (::bind(s->listen_fd, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0 || ::listen(s->listen_fd, 128)) {
    pa_rt_set_error("rpc: cannot listen on port %d", port);
    ::close(s->listen_fd);
    delete s;
    return nullptr;
  }
  socklen_t len = sizeof(addr);
  getsockname(s->listen_fd, reinterpret_cast<sockaddr*>(&addr), &len);
  s->port = ntohs(addr.sin_port);
  s->acceptor = std::thread([s] { s->accept_loop(); });
  return s;
}

PA_RT_EXPORT int pa_rpc_server_port(void* h) { return static_cast<Server*>(h)->port; }

// what: 1 = all trainers sent SEND_BARRIER (or all completed), 2 = all FETCH_BARRIER,
// 3 = at least one SEND queued (async mode) or all completed.  Returns 1 when every
// trainer has COMPLETEd (the loop should exit), 0 otherwise, -1 on timeout.
PA_RT_EXPORT int pa_rpc_server_wait(void* h, int what, int timeout_ms) {
  auto* s = static_cast<Server*>(h);
  std::unique_lock<std::mutex> g(s->mu);
  auto done = [&] {
    if (s->completed >= s->fanin) return true;
    if (what == 1) return s->send_barrier + s->completed >= s->fanin;
    if (what == 2) return s->fetch_barrier + s->completed >= s->fanin;
    return !s->recv_q.empty() || !s->checkpoints.empty();
  };
  if (timeout_ms < 0) s->cv.wait(g, done);
  else if (!s->cv.wait_for(g, std::chrono::milliseconds(timeout_ms), done)) return -1;
  return s->completed >= s->fanin ? 1 : 0;
}

// Pop one received variable: returns 1 and fills name/data (malloc'ed, free with
// pa_rpc_free) or 0 when the queue is empty.
PA_RT_EXPORT int pa_rpc_server_pop(void* h, char** name, char** data, size_t* len) {
  auto* s = static_cast<Server*>(h);
  std::lock_guard<std::mutex> g(s->mu);
  if (s->recv_q.empty()) return 0;
  auto& f = s->recv_q.front();
  *name = static_cast<char*>(std::malloc(f.first.size() + 1));
  std::memcpy(*name, f.first.c_str(), f.first.size() + 1);
  *data = static_cast<char*>(std::malloc(f.second.size() ? f.second.size() : 1));
  std::memcpy(*data, f.second.data(), f.second.size());
  *len = f.second.size();
  s->recv_q.pop_front();
  return 1;
}

PA_RT_EXPORT int pa_rpc_server_pop_checkpoint(void* h, char** dir) {
  auto* s = static_cast<Server*>(h);
  std::lock_guard<std::mutex> g(s->mu);
  if (s->checkpoints.empty()) return 0;
  auto& d = s->checkpoints.front();
  *dir = static_cast<char*>(std::malloc(d.size() + 1));
  std::memcpy(*dir, d.c_str(), d.size() + 1);
  s->checkpoints.pop_front();
  return 1;
}

PA_RT_EXPORT int pa_rpc_server_publish(void* h, const char* name, const char* data, size_t len) {
  auto* s = static_cast<Server*>(h);
  std::lock_guard<std::mutex> g(s->mu);
  s->store[name].assign(data, len);
  return 0;
}

PA_RT_EXPORT int pa_rpc_server_set_table(void* h, const char* name, const int64_t* ids, const float* rows,
                                         int64_t n, int64_t width) {
  auto* s = static_cast<Server*>(h);
  std::lock_guard<std::mutex> g(s->mu);
  Table& t = s->tables[name];
  t.width = width;
  for (int64_t i = 0; i < n; ++i) t.rows[ids[i]].assign(rows + i * width, rows + (i + 1) * width);
  return 0;
}

PA_RT_EXPORT int pa_rpc_server_set_ready(void* h, int ready) {
  auto* s = static_cast<Server*>(h);
  std::lock_guard<std::mutex> g(s->mu);
  s->ready = ready != 0;
  s->cv.notify_all();
  return 0;
}

PA_RT_EXPORT int pa_rpc_server_reset_barriers(void* h, int which) {
  auto* s = static_cast<Server*>(h);
  std::lock_guard<std::mutex> g(s->mu);
  if (which & 1) s->send_barrier = 0;
  if (which & 2) {
    s->fetch_barrier = 0;
    ++s->fetch_round;  // releases the trainers blocked in FETCH_BARRIER
    s->cv.notify_all();
  }
  return 0;
}

PA_RT_EXPORT int pa_rpc_server_stop(void* h) {
  auto* s = static_cast<Server*>(h);
  s->stop.store(true);
  {
    std::lock_guard<std::mutex> g(s->mu);
    s->ready = true;
    s->cv.notify_all();
    for (int fd : s->conn_fds) ::shutdown(fd, SHUT_RDWR);
  }
  ::shutdown(s->listen_fd, SHUT_RDWR);
  ::close(s->listen_fd);
  if (s->acceptor.joinable()) s->acceptor.join();
  for (auto& t : s->workers)
    if (t.joinable()) t.join();
  delete s;
  return 0;
}

// ------------------------------------------------------------------ client C ABI
PA_RT_EXPORT int pa_rpc_send(const char* ep, const char* name, const char* data, size_t len) {
  return call(ep, SEND, name, data, len, nullptr, nullptr);
}

PA_RT_EXPORT int pa_rpc_get(const char* ep, const char* name, char** out, size_t* out_len) {
  return call(ep, GET, name, nullptr, 0, out, out_len);
}

PA_RT_EXPORT int pa_rpc_prefetch(const char* ep, const char* table, const int64_t* ids, size_t n, char** out,
                                 size_t* out_len) {
  return call(ep, PREFETCH, table, ids, n * sizeof(int64_t), out, out_len);
}

PA_RT_EXPORT int pa_rpc_barrier(const char* ep, int kind) {
  uint8_t t = kind == 0 ? SEND_BARRIER : kind == 1 ? FETCH_BARRIER : COMPLETE;
  return call(ep, t, "", nullptr, 0, nullptr, nullptr);
}

PA_RT_EXPORT int pa_rpc_checkpoint_notify(const char* ep, const char* dir) {
  return call(ep, CHECKPOINT, "", dir, std::strlen(dir), nullptr, nullptr);
}

PA_RT_EXPORT void pa_rpc_free(void* p) { std::free(p); }

PA_RT_EXPORT int pa_rpc_close_all() {
  std::lock_guard<std::mutex> g(g_conns_mu);
  for (auto& kv : g_conns) {
    std::lock_guard<std::mutex> g2(kv.second->mu);
    if (kv.second->fd >= 0) ::close(kv.second->fd);
    kv.second->fd = -1;
  }
  return 0;
}
