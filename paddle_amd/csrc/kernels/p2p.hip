// Direct intra-node all-reduce over IPC-mapped peer buffers (xGMI on an 8-GPU
// MI355X node: every GPU reads / writes all 7 peers at once instead of one ring
// neighbour).  SURVEY.md §5.8; reference counterpart: platform/nccl_helper.h
// (NCCLContextMap) + the AllReduce op handle, which only ever call ncclAllReduce.
//
// Per rank: one staging buffer and one signal array, both allocated uncached
// (hipDeviceMallocUncached) so stores become visible to the peers' spinning
// loads without cache maintenance, exported with hipIpcGetMemHandle and mapped
// by every peer (parallel/direct.py).  Every signal is a vector (global) memory
// operation with system scope.
//
//   one-shot  (small messages): copy-in; barrier; out = sum over ranks of staging_r
//             (each rank reads every peer's whole buffer); barrier.
//   two-shot  (large): copy-in; barrier; rank r reduces chunk r of all stagings into
//             its own staging; barrier; every rank gathers chunk c from rank c;
//             barrier.  Per-rank traffic 2(P-1)/P of the message over P-1 links.
//
// Barriers spin a bounded number of times (then flag an error and exit), so a
// missing peer can never leave a wave running forever.  The reduce / gather
// kernels read that flag first: after a timed-out barrier they write NaN instead
// of summing a peer's stale or half-written staging data, so a lost peer shows up
// as a poisoned result (and parallel/direct.py raises on the flag), never as a
// silently wrong gradient.
#include <string.h>

#include "common.h"

namespace pa {
namespace {

constexpr int kMaxPeers = 8;

struct PeerArgs {
  const void* stage[kMaxPeers];  // staging buffer of rank p (mapped here)
  unsigned* sig[kMaxPeers];      // signal array of rank p (mapped here): sig[p][r] written by rank r
  int world, rank;
};

__global__ void p2p_barrier_kernel(PeerArgs a, unsigned epoch, long max_spins, int* err) {
  const int t = threadIdx.x;
  if (t >= a.world) return;
  // tell rank t that this rank reached `epoch`, then wait until rank t did too
  __hip_atomic_store(a.sig[t] + a.rank, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  unsigned* mine = a.sig[a.rank] + t;
  long spins = 0;
  while ((int)(__hip_atomic_load(mine, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
    if (++spins > max_spins) {
      __hip_atomic_store(err, 1 + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    __builtin_amdgcn_s_sleep(4);
  }
}

template <typename T>
__device__ __forceinline__ void ld8(const T* p, float (&o)[8]) {
  load8(p, o);
}

// out[i] = sum_r stage_r[i] over [begin, end) (elements; multiples of 8)
template <typename T>
__device__ __forceinline__ void poison8(T* p) {
  float nan8[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) nan8[j] = __builtin_nanf("");
  store8(p, nan8);
}

template <typename T>
__global__ __launch_bounds__(256) void p2p_reduce_kernel(PeerArgs a, T* __restrict__ out, long begin, long end,
                                                        const int* err) {
  const long n8 = (end - begin) / 8;
  const bool bad = err && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  for (long v = blockIdx.x * (long)blockDim.x + threadIdx.x; v < n8; v += (long)gridDim.x * blockDim.x) {
    const long i = begin + v * 8;
    if (bad) {
      poison8(out + i);
      continue;
    }
    float acc[8], x[8];
    ld8(static_cast<const T*>(a.stage[0]) + i, acc);
    for (int r = 1; r < a.world; ++r) {
      ld8(static_cast<const T*>(a.stage[r]) + i, x);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += x[j];
    }
    store8(out + i, acc);
  }
}

// out[i] = stage_{owner(i)}[i]: gather every rank's reduced chunk
template <typename T>
__global__ __launch_bounds__(256) void p2p_gather_kernel(PeerArgs a, T* __restrict__ out, long n, long chunk,
                                                        const int* err) {
  const long n8 = n / 8;
  const bool bad = err && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  for (long v = blockIdx.x * (long)blockDim.x + threadIdx.x; v < n8; v += (long)gridDim.x * blockDim.x) {
    const long i = v * 8;
    if (bad) {
      poison8(out + i);
      continue;
    }
    const int owner = (int)min((long)(a.world - 1), i / chunk);
    float x[8];
    ld8(static_cast<const T*>(a.stage[owner]) + i, x);
    store8(out + i, x);
  }
}

int blocks_for(long n8) {
  long b = (n8 + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 2048 ? 2048 : b));
}

PeerArgs make_args(const void* const* stage, unsigned* const* sig, int world, int rank) {
  PeerArgs a{};
  for (int p = 0; p < world && p < kMaxPeers; ++p) {
    a.stage[p] = stage[p];
    a.sig[p] = sig[p];
  }
  a.world = world;
  a.rank = rank;
  return a;
}
}  // namespace

}  // namespace pa

using namespace pa;

// ---------------------------------------------------------------- memory / IPC
PA_EXPORT int pa_p2p_alloc(void** p, size_t bytes) {
  return (int)hipExtMallocWithFlags(p, bytes, hipDeviceMallocUncached);
}
PA_EXPORT int pa_p2p_free(void* p) { return (int)hipFree(p); }
PA_EXPORT int pa_p2p_ipc_handle(void* p, void* out64) {
  hipIpcMemHandle_t h;
  hipError_t e = hipIpcGetMemHandle(&h, p);
  if (e == hipSuccess) memcpy(out64, &h, sizeof(h));
  return (int)e;
}
PA_EXPORT int pa_p2p_ipc_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }
PA_EXPORT int pa_p2p_ipc_open(const void* in64, void** p) {
  hipIpcMemHandle_t h;
  memcpy(&h, in64, sizeof(h));
  return (int)hipIpcOpenMemHandle(p, h, hipIpcMemLazyEnablePeerAccess);
}
PA_EXPORT int pa_p2p_ipc_close(void* p) { return (int)hipIpcCloseMemHandle(p); }

// ---------------------------------------------------------------- collectives
PA_EXPORT int pa_p2p_barrier(const void* const* stage, unsigned* const* sig, int world, int rank, unsigned epoch,
                             long max_spins, int* err, hipStream_t st) {
  if (world < 1 || world > kMaxPeers || rank < 0 || rank >= world) return -1;
  PeerArgs a = make_args(stage, sig, world, rank);
  hipLaunchKernelGGL(p2p_barrier_kernel, dim3(1), dim3(64), 0, st, a, epoch, max_spins, err);
  return (int)hipGetLastError();
}

// dtype: 0 fp32, 1 bf16.  [begin, end) in elements, multiples of 8.
// err: the barrier error flag (device int, may be null): set -> the output is NaN.
PA_EXPORT int pa_p2p_reduce(int dtype, const void* const* stage, unsigned* const* sig, int world, int rank,
                            void* out, long begin, long end, const int* err, hipStream_t st) {
  if (world < 1 || world > kMaxPeers || (begin % 8) || (end % 8) || end < begin) return -1;
  PeerArgs a = make_args(stage, sig, world, rank);
  const int g = blocks_for((end - begin) / 8);
  if (dtype == 0) hipLaunchKernelGGL(p2p_reduce_kernel<float>, dim3(g), dim3(256), 0, st, a, (float*)out, begin, end, err);
  else hipLaunchKernelGGL(p2p_reduce_kernel<u16>, dim3(g), dim3(256), 0, st, a, (u16*)out, begin, end, err);
  return (int)hipGetLastError();
}

PA_EXPORT int pa_p2p_gather(int dtype, const void* const* stage, unsigned* const* sig, int world, int rank, void* out,
                            long n, long chunk, const int* err, hipStream_t st) {
  if (world < 1 || world > kMaxPeers || (n % 8) || chunk <= 0 || (chunk % 8)) return -1;
  PeerArgs a = make_args(stage, sig, world, rank);
  const int g = blocks_for(n / 8);
  if (dtype == 0) hipLaunchKernelGGL(p2p_gather_kernel<float>, dim3(g), dim3(256), 0, st, a, (float*)out, n, chunk, err);
  else hipLaunchKernelGGL(p2p_gather_kernel<u16>, dim3(g), dim3(256), 0, st, a, (u16*)out, n, chunk, err);
  return (int)hipGetLastError();
}

PA_EXPORT int pa_p2p_zero(void* p, size_t bytes) { return (int)hipMemset(p, 0, bytes); }
PA_EXPORT int pa_p2p_copy(void* dst, const void* src, size_t bytes, hipStream_t st) {
  return (int)hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st);
}
