// Framework-owned RCCL communicators (one per process group and device).
//
// Reference parity: platform/nccl_helper.h:49-123 (NCCLGroupGuard: a global mutex
// around ncclGroupStart/End; NCCLContextMap: one communicator + stream per place;
// InitRank with rank = trainer_id * ngpu + gpu_id) and operators/gen_nccl_id_op.cc:
// 54-110 (trainer 0 creates the ncclUniqueId and ships it to the other trainers).
//
// MI355X-first: one process per GPU, so a communicator is (group, device) -> one
// ncclComm_t; the unique id travels through the job's TCP key-value store (the
// Python side, parallel/rccl.py), and collectives are enqueued on the caller's HIP
// stream -- the framework's DeviceContext comm stream or torch's current stream --
// so they order with the producing kernels without host synchronisation.  librccl
// is loaded with dlopen (the process normally already holds it through torch; the
// same soname resolves to that copy), so this library has no link-time RCCL
// dependency and a missing RCCL is a clean error, not a load failure.
#include <dlfcn.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <string>

#include <hip/hip_runtime_api.h>

#include "runtime.h"

namespace {

typedef int ncclResult_t;
typedef void* ncclComm_t;
struct ncclUniqueId {
  char internal[128];
};

struct Rccl {
  void* h = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
  ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t*) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, int, int, ncclComm_t, void*) = nullptr;
  ncclResult_t (*ReduceScatter)(const void*, void*, size_t, int, int, ncclComm_t, void*) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, int, ncclComm_t, void*) = nullptr;
  ncclResult_t (*Broadcast)(const void*, void*, size_t, int, int, ncclComm_t, void*) = nullptr;
  ncclResult_t (*Send)(const void*, size_t, int, int, ncclComm_t, void*) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, int, int, ncclComm_t, void*) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
  std::string err;
};

Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    // PA_RCCL_LIBRARY: an explicit library with the same C ABI (the multi-rank CPU
    // tests load a shared-memory fake through it)
    const char* override_lib = getenv("PA_RCCL_LIBRARY");
    if (override_lib && *override_lib) {
      r.h = dlopen(override_lib, RTLD_NOW | RTLD_LOCAL);
    } else {
      const char* names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
      for (const char* n : names) {
        r.h = dlopen(n, RTLD_NOW | RTLD_GLOBAL);
        if (r.h) break;
      }
    }
    if (!r.h) {
      r.err = std::string("librccl not loadable: ") + dlerror();
      return;
    }
#define PA_SYM(field, name) r.field = reinterpret_cast<decltype(r.field)>(dlsym(r.h, name))
    PA_SYM(GetUniqueId, "ncclGetUniqueId");
    PA_SYM(CommInitRank, "ncclCommInitRank");
    PA_SYM(CommDestroy, "ncclCommDestroy");
    PA_SYM(CommAbort, "ncclCommAbort");
    PA_SYM(CommGetAsyncError, "ncclCommGetAsyncError");
    PA_SYM(AllReduce, "ncclAllReduce");
    PA_SYM(ReduceScatter, "ncclReduceScatter");
    PA_SYM(AllGather, "ncclAllGather");
    PA_SYM(Broadcast, "ncclBroadcast");
    PA_SYM(Send, "ncclSend");
    PA_SYM(Recv, "ncclRecv");
    PA_SYM(GroupStart, "ncclGroupStart");
    PA_SYM(GroupEnd, "ncclGroupEnd");
    PA_SYM(GetErrorString, "ncclGetErrorString");
#undef PA_SYM
    if (!r.GetUniqueId || !r.CommInitRank || !r.AllReduce || !r.GroupStart) r.err = "librccl is missing symbols";
  });
  return r;
}

// NCCLGroupGuard: ncclGroupStart/End are process-global; a mutex keeps two host
// threads from interleaving their groups (nccl_helper.h:49)
std::recursive_mutex& group_mutex() {
  static std::recursive_mutex m;
  return m;
}

thread_local std::string g_last_error;

int fail(const char* what, ncclResult_t rc) {
  Rccl& r = rccl();
  g_last_error = std::string(what) + ": " + (r.GetErrorString ? r.GetErrorString(rc) : "rccl error") + " (" +
                 std::to_string(rc) + ")";
  return rc ? rc : -1;
}

}  // namespace

extern "C" {

__attribute__((visibility("default"))) const char* pa_rccl_last_error() { return g_last_error.c_str(); }

__attribute__((visibility("default"))) int pa_rccl_available() { return rccl().err.empty() ? 1 : 0; }

// 128-byte unique id of a new communicator clique (rank 0 of the group calls this)
__attribute__((visibility("default"))) int pa_rccl_unique_id(char* out128) {
  Rccl& r = rccl();
  if (!r.err.empty()) {
    g_last_error = r.err;
    return -1;
  }
  ncclUniqueId id;
  ncclResult_t rc = r.GetUniqueId(&id);
  if (rc) return fail("ncclGetUniqueId", rc);
  memcpy(out128, id.internal, 128);
  return 0;
}

// collective: every rank of the group calls it with the same id
__attribute__((visibility("default"))) int pa_rccl_comm_init(const char* id128, int nranks, int rank, int device, void** comm) {
  Rccl& r = rccl();
  if (!r.err.empty()) {
    g_last_error = r.err;
    return -1;
  }
  // device < 0: host buffers (a CPU test against a fake library); no device to select
  if (device >= 0 && hipSetDevice(device) != hipSuccess) {
    g_last_error = "hipSetDevice failed";
    return -1;
  }
  ncclUniqueId id;
  memcpy(id.internal, id128, 128);
  ncclComm_t c = nullptr;
  ncclResult_t rc = r.CommInitRank(&c, nranks, id, rank);
  if (rc) return fail("ncclCommInitRank", rc);
  *comm = c;
  return 0;
}

__attribute__((visibility("default"))) int pa_rccl_comm_destroy(void* comm, int abort) {
  Rccl& r = rccl();
  if (!comm) return 0;
  ncclResult_t rc = abort && r.CommAbort ? r.CommAbort(comm) : r.CommDestroy(comm);
  return rc ? fail("ncclCommDestroy", rc) : 0;
}

// 0: healthy; else the communicator's asynchronous error (a peer died / timed out)
__attribute__((visibility("default"))) int pa_rccl_async_error(void* comm) {
  Rccl& r = rccl();
  ncclResult_t e = 0;
  if (!r.CommGetAsyncError) return 0;
  ncclResult_t rc = r.CommGetAsyncError(comm, &e);
  if (rc) return fail("ncclCommGetAsyncError", rc);
  return e ? fail("async error", e) : 0;
}

__attribute__((visibility("default"))) int pa_rccl_group_start() {
  group_mutex().lock();
  ncclResult_t rc = rccl().GroupStart();
  if (rc) {
    group_mutex().unlock();
    return fail("ncclGroupStart", rc);
  }
  return 0;
}

__attribute__((visibility("default"))) int pa_rccl_group_end() {
  ncclResult_t rc = rccl().GroupEnd();
  group_mutex().unlock();
  return rc ? fail("ncclGroupEnd", rc) : 0;
}

// dtype / op: the ncclDataType_t / ncclRedOp_t values of rccl.h
__attribute__((visibility("default"))) int pa_rccl_all_reduce(const void* send, void* recv, size_t count, int dtype, int op, void* comm,
                                 void* stream) {
  ncclResult_t rc = rccl().AllReduce(send, recv, count, dtype, op, comm, stream);
  return rc ? fail("ncclAllReduce", rc) : 0;
}

__attribute__((visibility("default"))) int pa_rccl_reduce_scatter(const void* send, void* recv, size_t recv_count, int dtype, int op, void* comm,
                                     void* stream) {
  ncclResult_t rc = rccl().ReduceScatter(send, recv, recv_count, dtype, op, comm, stream);
  return rc ? fail("ncclReduceScatter", rc) : 0;
}

__attribute__((visibility("default"))) int pa_rccl_all_gather(const void* send, void* recv, size_t send_count, int dtype, void* comm,
                                 void* stream) {
  ncclResult_t rc = rccl().AllGather(send, recv, send_count, dtype, comm, stream);
  return rc ? fail("ncclAllGather", rc) : 0;
}

__attribute__((visibility("default"))) int pa_rccl_broadcast(const void* send, void* recv, size_t count, int dtype, int root, void* comm,
                                void* stream) {
  ncclResult_t rc = rccl().Broadcast(send, recv, count, dtype, root, comm, stream);
  return rc ? fail("ncclBroadcast", rc) : 0;
}

__attribute__((visibility("default"))) int pa_rccl_send(const void* buf, size_t count, int dtype, int peer, void* comm, void* stream) {
  ncclResult_t rc = rccl().Send(buf, count, dtype, peer, comm, stream);
  return rc ? fail("ncclSend", rc) : 0;
}

__attribute__((visibility("default"))) int pa_rccl_recv(void* buf, size_t count, int dtype, int peer, void* comm, void* stream) {
  ncclResult_t rc = rccl().Recv(buf, count, dtype, peer, comm, stream);
  return rc ? fail("ncclRecv", rc) : 0;
}

// All-to-all with per-peer element counts and displacements (expert-parallel token
// exchange): one ncclSend + one ncclRecv per peer inside ONE group, so RCCL runs the
// whole exchange as a single fused launch over the xGMI links (no torch.distributed
// all_to_all_single, no host staging).  Zero-sized pairs are skipped.
__attribute__((visibility("default"))) int pa_rccl_all_to_all(const void* send, void* recv, const size_t* scount,
                                                              const size_t* sdispl, const size_t* rcount,
                                                              const size_t* rdispl, int nranks, int dtype,
                                                              size_t elem_bytes, void* comm, void* stream) {
  Rccl& r = rccl();
  if (!r.Send || !r.Recv) {
    g_last_error = "librccl has no point-to-point symbols";
    return -1;
  }
  std::lock_guard<std::recursive_mutex> lk(group_mutex());
  ncclResult_t rc = r.GroupStart();
  if (rc) return fail("ncclGroupStart", rc);
  ncclResult_t first = 0;
  for (int p = 0; p < nranks && !first; ++p) {
    if (scount[p]) first = r.Send((const char*)send + sdispl[p] * elem_bytes, scount[p], dtype, p, comm, stream);
    if (!first && rcount[p]) first = r.Recv((char*)recv + rdispl[p] * elem_bytes, rcount[p], dtype, p, comm, stream);
  }
  rc = r.GroupEnd();
  if (first) return fail("ncclSend/ncclRecv", first);
  return rc ? fail("ncclGroupEnd", rc) : 0;
}

}  // extern "C"
