// Bandwidth-bound 2-D transpose of bf16 matrices (out[c][r] = in[r][c]), batched.
//
// Why it exists: hipBLASLt on gfx950 runs the K-contiguous "NT" GEMM form
// (C = A * B^T, both operands K-inner) at ~1.5 PF/s but the weight-gradient "TN"
// form (dW = X^T dY, reduction over tokens = the OUTER dim of both operands) at
// ~1.06-1.14 PF/s.  Re-laying X and dY out token-inner with this kernel costs one
// read + one write of each (~0.1-0.35 ms at LLaMA-7B shapes) and turns every dW
// into the fast form (see ops/fused.py _LinearFn).  torch's generic strided copy
// moves a transpose at ~1 TB/s; this one targets the HBM roofline.
//
// Layout: one 256-thread workgroup per 64x64 tile.  Global loads and stores are
// 16 B per lane with 8 consecutive lanes covering one 128-B row segment (fully
// coalesced both ways).  The LDS image is [64 rows][8 chunks of 16 B] with the
// chunk index XOR-swizzled by (row>>3)&7: the column gather in the store phase
// has the 8 lanes that share a column read rows 8 apart, which the swizzle puts
// on 8 different 16-B bank slots (conflict-free ds_read_u16, guide §2 / T2).
#include "common.h"

namespace pa {

template <typename T>
__global__ __launch_bounds__(256) void transpose64_kernel(const T* __restrict__ src, T* __restrict__ dst,
                                                          int R, int C, long ld_src, long ld_dst,
                                                          long bs_src, long bs_dst) {
  static_assert(sizeof(T) == 2, "16-bit elements");
  __shared__ __attribute__((aligned(16))) u16 tile[64 * 64];
  const int tid = threadIdx.x;
  const int c0 = blockIdx.x * 64, r0 = blockIdx.y * 64;
  const u16* s = reinterpret_cast<const u16*>(src) + (long)blockIdx.z * bs_src;
  u16* d = reinterpret_cast<u16*>(dst) + (long)blockIdx.z * bs_dst;
  const bool full = (r0 + 64 <= R) && (c0 + 64 <= C);
  // ---- load: 512 chunks of 8 elements, 2 per thread
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int i = tid + it * 256;
    const int r = i >> 3, ch = i & 7;
    const int gr = r0 + r, gc = c0 + ch * 8;
    u16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (full || (gr < R && gc < C)) v = *reinterpret_cast<const u16x8*>(s + (long)gr * ld_src + gc);
    const int pch = ch ^ ((r >> 3) & 7);
    *reinterpret_cast<u16x8*>(&tile[r * 64 + pch * 8]) = v;
  }
  __syncthreads();
  // ---- store: output row c (input column), 8 lanes x 16 B = the tile's 64 rows
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int i = tid + it * 256;
    const int c = i >> 3, rc = i & 7;  // rc: which 8-row group of the input
    const int ch = c >> 3, ce = c & 7;
    u16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int r = rc * 8 + j;
      v[j] = tile[r * 64 + ((ch ^ ((r >> 3) & 7)) * 8) + ce];
    }
    const int gc = c0 + c, gr = r0 + rc * 8;
    if (full || (gc < C && gr < R)) *reinterpret_cast<u16x8*>(d + (long)gc * ld_dst + gr) = v;
  }
}

// out[b][c][r] = in[b][r][c]; R, C multiples of 8; leading dims multiples of 8
PA_EXPORT int pa_transpose2d(int dtype, const void* src, void* dst, int R, int C, long ld_src, long ld_dst,
                             int batch, long bs_src, long bs_dst, hipStream_t st) {
  if (dtype != 1 && dtype != 2) return (int)hipErrorInvalidValue;  // bf16 / f16 bits only
  if ((R | C) & 7 || (ld_src | ld_dst) & 7) return (int)hipErrorInvalidValue;
  dim3 grid((C + 63) / 64, (R + 63) / 64, batch);
  hipLaunchKernelGGL(transpose64_kernel<u16>, grid, dim3(256), 0, st, (const u16*)src, (u16*)dst, R, C,
                     ld_src, ld_dst, bs_src, bs_dst);
  PA_LAUNCH_CHECK();
}

}  // namespace pa
