// MoE token dispatch / combine for gfx950 (bf16 activations, fp32 gate weights).
//
// Routing produces, for T tokens x k slots, the expert-sorted order of the kept
// slots: ``src[i]`` = token of sorted row i, and the inverse ``pos[t*k + j]`` =
// sorted row of slot (t, j) or -1 if the slot was dropped (capacity).  Every kernel
// below is a pure gather -- each output row has exactly one writer -- so there are
// no atomics and no sort-based index_put on the backward path:
//
//   dispatch    send[i]   = x[src[i]]
//   dispatch^T  dx[t]     = sum_j dsend[pos[t,j]]
//   combine     y[t]      = sum_j w[t,j] * ys[pos[t,j]]        (fp32 accumulate)
//   combine^T   dys[pos[t,j]] = w[t,j] * dy[t],  dw[t,j] = <dy[t], ys[pos[t,j]]>
//
// One wave per row, 16-B vectors per lane (8 bf16), H % 8 == 0.  Not in the
// reference (no MoE); replaces torch index_select / index_add_.
#include "common.h"

namespace pa {

constexpr int kMoeWaves = 4;

__global__ __launch_bounds__(64 * kMoeWaves) void moe_gather_kernel(const u16* __restrict__ x,
                                                                    const int* __restrict__ src,
                                                                    u16* __restrict__ out, long R, int H) {
  const long r = (long)blockIdx.x * kMoeWaves + (threadIdx.x >> 6);
  if (r >= R) return;
  const int lane = threadIdx.x & 63;
  const u16* xs = x + (long)src[r] * H;
  u16* o = out + r * H;
  for (int c = lane * 8; c < H; c += 512) *reinterpret_cast<u16x8*>(o + c) = *reinterpret_cast<const u16x8*>(xs + c);
}

// dx[t] = sum_j ds[pos[t*k+j]] (or, with w, y[t] = sum_j w[t*k+j] * ds[pos[...]])
__global__ __launch_bounds__(64 * kMoeWaves) void moe_reduce_kernel(const u16* __restrict__ ds,
                                                                    const int* __restrict__ pos,
                                                                    const float* __restrict__ w,
                                                                    u16* __restrict__ out, long T, int k, int H) {
  const long t = (long)blockIdx.x * kMoeWaves + (threadIdx.x >> 6);
  if (t >= T) return;
  const int lane = threadIdx.x & 63;
  for (int c = lane * 8; c < H; c += 512) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < k; ++j) {
      const int p = pos[t * k + j];
      if (p < 0) continue;
      const float s = w ? w[t * k + j] : 1.f;
      float v[8];
      load8(ds + (long)p * H + c, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += s * v[e];
    }
    store8(out + t * H + c, acc);
  }
}

__global__ __launch_bounds__(64 * kMoeWaves) void moe_combine_bwd_kernel(
    const u16* __restrict__ dy, const u16* __restrict__ ys, const int* __restrict__ pos,
    const float* __restrict__ w, u16* __restrict__ dys, float* __restrict__ dw, long T, int k, int H) {
  const long t = (long)blockIdx.x * kMoeWaves + (threadIdx.x >> 6);
  if (t >= T) return;
  const int lane = threadIdx.x & 63;
  const u16* g = dy + t * H;
  for (int j = 0; j < k; ++j) {
    const int p = pos[t * k + j];
    if (p < 0) {
      if (lane == 0) dw[t * k + j] = 0.f;
      continue;
    }
    const float s = w[t * k + j];
    float dot = 0.f;
    for (int c = lane * 8; c < H; c += 512) {
      float a[8], b[8], o[8];
      load8(g + c, a);
      load8(ys + (long)p * H + c, b);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        dot += a[e] * b[e];
        o[e] = s * a[e];
      }
      store8(dys + (long)p * H + c, o);
    }
    dot = wave_sum(dot);
    if (lane == 0) dw[t * k + j] = dot;
  }
}

}  // namespace pa

using namespace pa;

static inline int moe_grid(long rows) { return (int)((rows + kMoeWaves - 1) / kMoeWaves); }

PA_EXPORT int pa_moe_gather(const void* x, const int* src, void* out, long R, int H, hipStream_t st) {
  if (R <= 0) return 0;
  if (H % 8) return -1;
  hipLaunchKernelGGL(moe_gather_kernel, dim3(moe_grid(R)), dim3(64 * kMoeWaves), 0, st, (const u16*)x, src,
                     (u16*)out, R, H);
  PA_LAUNCH_CHECK();
}

// w == null: unweighted sum (dispatch backward); else the weighted combine
PA_EXPORT int pa_moe_reduce(const void* ds, const int* pos, const float* w, void* out, long T, int k, int H,
                            hipStream_t st) {
  if (T <= 0) return 0;
  if (H % 8) return -1;
  hipLaunchKernelGGL(moe_reduce_kernel, dim3(moe_grid(T)), dim3(64 * kMoeWaves), 0, st, (const u16*)ds, pos, w,
                     (u16*)out, T, k, H);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_moe_combine_bwd(const void* dy, const void* ys, const int* pos, const float* w, void* dys,
                                 float* dw, long T, int k, int H, hipStream_t st) {
  if (T <= 0) return 0;
  if (H % 8) return -1;
  hipLaunchKernelGGL(moe_combine_bwd_kernel, dim3(moe_grid(T)), dim3(64 * kMoeWaves), 0, st, (const u16*)dy,
                     (const u16*)ys, pos, w, (u16*)dys, dw, T, k, H);
  PA_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------
// Routing without a sort: the gate's expert per slot (flat_e [n = T*k]) -> the
// expert-sorted order of the kept slots: a stable counting sort over blocks of 1024
// slots, three launches.
//   count  block b: its slot counts per expert, cnt[b][e] (LDS integer atomics);
//   scan   one workgroup: per expert the running count over the blocks before b,
//          run[b][e], and the row offsets of the experts, off[e];
//   place  block b: a slot's rank inside its expert = run[b][e] + earlier lanes of
//          its wave with that expert (64 lane reads) + the counts of the earlier
//          waves of the block (the 16 waves take and advance an LDS base in turn),
//          so within an expert the order is slot order -- the stable argsort of
//          the torch path, exactly, with no dependence on atomic arrival order.
// mode 0: every slot kept, row = off[e] + rank               (outputs pos, src, e_sorted)
// mode 1: GShard capacity layout, row = e * cap + rank, dropped when rank >= cap
//         (pos, src [E * cap]; padding rows get token 0)
// mode 2: capacity drop with compact rows, row = offk[e] + rank, offk = scan of
//         min(count, cap)                                    (pos, src, e_sorted)
// counts[e] (int64) = kept slots of expert e in every mode.
namespace pa {

constexpr int kRouteT = 1024;

__global__ __launch_bounds__(kRouteT) void moe_route_count_kernel(const long* __restrict__ flat_e, long n, int E,
                                                                  int* __restrict__ cnt, int mode, long cap,
                                                                  int* __restrict__ src) {
  __shared__ int h[1024];
  const int tid = threadIdx.x;
  for (int e = tid; e < E; e += kRouteT) h[e] = 0;
  if (mode == 1)  // padding rows of the capacity layout read token 0
    for (long r = (long)blockIdx.x * kRouteT + tid; r < (long)E * cap; r += (long)gridDim.x * kRouteT) src[r] = 0;
  __syncthreads();
  const long i = (long)blockIdx.x * kRouteT + tid;
  if (i < n) {
    const long e = flat_e[i];
    if (e >= 0 && e < E) atomicAdd(&h[(int)e], 1);  // an out-of-range expert id is dropped, never indexed
  }
  __syncthreads();
  for (int e = tid; e < E; e += kRouteT) cnt[(long)blockIdx.x * E + e] = h[e];
}

__global__ __launch_bounds__(kRouteT) void moe_route_scan_kernel(const int* __restrict__ cnt, int nb, int E, int mode,
                                                                 long cap, int* __restrict__ run,
                                                                 int* __restrict__ off, long* __restrict__ counts) {
  __shared__ int sc[1024];
  const int e = threadIdx.x;
  int tot = 0;
  if (e < E)
    for (int b = 0; b < nb; ++b) {
      run[(long)b * E + e] = tot;
      tot += cnt[(long)b * E + e];
    }
  const int kept = e < E ? (mode == 0 ? tot : (tot < cap ? tot : (int)cap)) : 0;
  if (e < E) counts[e] = kept;
  // exclusive scan of kept over the experts (Hillis-Steele in LDS)
  sc[e] = kept;
  __syncthreads();
  for (int o = 1; o < kRouteT; o <<= 1) {
    const int v = e >= o ? sc[e - o] : 0;
    __syncthreads();
    sc[e] += v;
    __syncthreads();
  }
  if (e < E) off[e] = sc[e] - kept;
}

__global__ __launch_bounds__(kRouteT) void moe_route_place_kernel(const long* __restrict__ flat_e, long n, int E,
                                                                  int k, int mode, long cap,
                                                                  const int* __restrict__ run,
                                                                  const int* __restrict__ off, int* __restrict__ pos,
                                                                  int* __restrict__ src,
                                                                  long* __restrict__ e_sorted) {
  __shared__ int base[1024];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int e = tid; e < E; e += kRouteT) base[e] = run[(long)blockIdx.x * E + e];
  __syncthreads();
  const long i = (long)blockIdx.x * kRouteT + tid;
  const long ev = i < n ? flat_e[i] : -1;
  const int e = ev >= 0 && ev < E ? (int)ev : -1;
  int r = 0, c = 0;  // rank among / count of this wave's lanes with expert e
  for (int j = 0; j < 64; ++j) {
    const int ej = __shfl(e, j, 64);
    c += ej == e ? 1 : 0;
    r += (j < lane && ej == e) ? 1 : 0;
  }
  int rank = 0;
  for (int ww = 0; ww < kRouteT / 64; ++ww) {
    if (w == ww && e >= 0) {
      rank = base[e] + r;                  // every lane of the wave reads before ...
      if (r == c - 1) base[e] = rank + 1;  // ... the group's last lane advances the base
    }
    __syncthreads();
  }
  if (e >= 0) {
    const bool keep = mode == 0 || rank < cap;
    int row = -1;
    if (keep) {
      row = mode == 1 ? (int)(e * cap + rank) : off[e] + rank;
      src[row] = (int)(i / k);
      if (mode != 1) e_sorted[row] = e;
    }
    pos[i] = row;
  } else if (i < n) {
    pos[i] = -1;  // out-of-range expert id: the slot is dropped
  }
}

// frac_e = share of tokens whose first choice is e (idx [T, k] int64, column 0)
__global__ __launch_bounds__(1024) void moe_frac_kernel(const long* __restrict__ idx, long T, int k, int E,
                                                        float* __restrict__ frac) {
  __shared__ int cnt[1024];
  for (int e = threadIdx.x; e < E; e += 1024) cnt[e] = 0;
  __syncthreads();
  for (long t = threadIdx.x; t < T; t += 1024) atomicAdd(&cnt[(int)idx[t * k]], 1);
  __syncthreads();
  for (int e = threadIdx.x; e < E; e += 1024) frac[e] = (float)cnt[e] / (float)(T > 0 ? T : 1);
}

// Router backward (fp32), one wave per token: with valn = the top-k probabilities
// renormalised by s and the balance loss l = E * sum_e mean_t(p_te) frac_e
//   dv_j   = (dval_j - sum_i dval_i valn_i) / s     (renorm; else dval_j)
//   dp_te  = sum_j [idx_tj == e] dv_j + daux * E * frac_e / T
//   dlogit = p * (dp - <dp, p>)
// (the scatter_add + softmax backward of the torch formulation in one pass; k <= 64)
__global__ __launch_bounds__(256) void moe_gate_bwd_kernel(const float* __restrict__ probs,
                                                           const long* __restrict__ idx,
                                                           const float* __restrict__ valn,
                                                           const float* __restrict__ s,
                                                           const float* __restrict__ frac,
                                                           const float* __restrict__ dval,
                                                           const float* __restrict__ daux, long T, int E,
                                                           int k, int renorm, float* __restrict__ dlogits) {
  const long t = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= T) return;
  const int lane = threadIdx.x & 63;
  const float* p = probs + t * E;
  float dv = 0.f;
  if (dval) {
    dv = lane < k ? dval[t * k + lane] : 0.f;
    if (renorm) {
      const float dot = wave_sum(lane < k ? dv * valn[t * k + lane] : 0.f);
      dv = (dv - dot) / s[t];
    }
  }
  // the k (expert, dv) pairs of this token go through LDS: the expert loops below
  // are lane-divergent when E % 64 != 0, and a cross-lane read from a lane that has
  // left the loop returns nothing
  __shared__ int s_idx[4][64];
  __shared__ float s_dv[4][64];
  const int wv = threadIdx.x >> 6;
  s_idx[wv][lane] = lane < k ? (int)idx[t * k + lane] : -1;
  s_dv[wv][lane] = dv;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const float ga = daux ? daux[0] * (float)E / (float)T : 0.f;
  float part = 0.f;
  for (int e = lane; e < E; e += 64) {
    float dp = ga * frac[e];
    for (int j = 0; j < k; ++j)
      if (s_idx[wv][j] == e) dp += s_dv[wv][j];
    part += dp * p[e];
  }
  const float dot = wave_sum(part);
  for (int e = lane; e < E; e += 64) {
    float dp = ga * frac[e];
    for (int j = 0; j < k; ++j)
      if (s_idx[wv][j] == e) dp += s_dv[wv][j];
    dlogits[t * E + e] = p[e] * (dp - dot);
  }
}

}  // namespace pa

using namespace pa;

// ws: int workspace of pa_moe_route_ws(n, E) elements
PA_EXPORT long pa_moe_route_ws(long n, int E) {
  const long nb = (n + kRouteT - 1) / kRouteT;
  return 2 * nb * E + E;
}

PA_EXPORT int pa_moe_route(const long* flat_e, long n, int E, int k, int mode, long cap, int* pos, int* src,
                           long* e_sorted, long* counts, int* ws, hipStream_t st) {
  if (E <= 0 || E > 1024 || k <= 0 || mode < 0 || mode > 2 || (mode != 0 && cap < 0) || !ws) return -1;
  if (mode != 0 && (long)E * cap > 0x7fffffffL) return -1;
  if (mode != 1 && !e_sorted) return -1;
  if (n <= 0) return -1;
  const long nb = (n + kRouteT - 1) / kRouteT;
  if (nb > 0x7fffffffL / E) return -1;
  int* cnt = ws;
  int* run = ws + nb * E;
  int* off = run + nb * E;
  hipLaunchKernelGGL(moe_route_count_kernel, dim3((unsigned)nb), dim3(kRouteT), 0, st, flat_e, n, E, cnt, mode, cap,
                     src);
  hipLaunchKernelGGL(moe_route_scan_kernel, dim3(1), dim3(kRouteT), 0, st, (const int*)cnt, (int)nb, E, mode, cap,
                     run, off, counts);
  hipLaunchKernelGGL(moe_route_place_kernel, dim3((unsigned)nb), dim3(kRouteT), 0, st, flat_e, n, E, k, mode, cap,
                     (const int*)run, (const int*)off, pos, src, e_sorted);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_moe_frac(const long* idx, long T, int k, int E, float* frac, hipStream_t st) {
  if (E <= 0 || E > 1024 || k <= 0) return -1;
  hipLaunchKernelGGL(moe_frac_kernel, dim3(1), dim3(1024), 0, st, idx, T, k, E, frac);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_moe_gate_bwd(const float* probs, const long* idx, const float* valn, const float* s,
                              const float* frac, const float* dval, const float* daux, long T, int E, int k,
                              int renorm, float* dlogits, hipStream_t st) {
  if (k <= 0 || k > 64 || E <= 0) return -1;
  if (T <= 0) return 0;
  hipLaunchKernelGGL(moe_gate_bwd_kernel, dim3((unsigned)((T + 3) / 4)), dim3(256), 0, st, probs, idx, valn, s,
                     frac, dval, daux, T, E, k, renorm, dlogits);
  PA_LAUNCH_CHECK();
}
