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
