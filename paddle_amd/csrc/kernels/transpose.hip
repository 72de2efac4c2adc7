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
//
// transpose128_kernel (default since round 5, +0-15 % over the 64x64 kernel): a 128x128 tile per workgroup, 256-B
// row segments both ways (8 loads of 16 B in flight per lane), the store phase
// builds two output rows at once from ds_read_b32 pairs of adjacent input columns
// (8 LDS reads per 32 B stored instead of 16), and the tile order is grouped: GROUP
// consecutive workgroups walk GROUP row-tiles of one column-tile, so the blocks in
// flight write a few KB of contiguous output per output row instead of one 256-B
// piece per row at a 2^k stride (HBM channel camping at R = 16384).
#include <cstdlib>

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
__global__ __launch_bounds__(256) void transpose128_kernel(const u16* __restrict__ src, u16* __restrict__ dst,
                                                           int R, int C, long ld_src, long ld_dst, long bs_src,
                                                           long bs_dst, int ntx, int nty, int group) {
  // LDS image [128 rows][16 chunks of 16 B]; chunk index XOR (row >> 3): in the store
  // phase the 16 lanes of one output row read input rows 8 apart -> 16 distinct chunks
  __shared__ __attribute__((aligned(16))) u16 tile[128 * 128];
  const int tid = threadIdx.x;
  int tx, ty;
  {
    const int b = blockIdx.x;
    if (group > 0) {
      const int per = group * ntx, g = b / per, first = g * group;
      const int gsz = min(nty - first, group), w = b - g * per;
      ty = first + w % gsz;
      tx = w / gsz;
    } else {
      tx = b % ntx;
      ty = b / ntx;
    }
  }
  const int c0 = tx * 128, r0 = ty * 128;
  const u16* s = src + (long)blockIdx.y * bs_src;
  u16* d = dst + (long)blockIdx.y * bs_dst;
  const bool full = (r0 + 128 <= R) && (c0 + 128 <= C);
  u16x8 v[8];
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int i = tid + it * 256, r = i >> 4, ch = i & 15;
    const int gr = r0 + r, gc = c0 + ch * 8;
    v[it] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (full || (gr < R && gc < C)) v[it] = *reinterpret_cast<const u16x8*>(s + (long)gr * ld_src + gc);
  }
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int i = tid + it * 256, r = i >> 4, ch = i & 15;
    *reinterpret_cast<u16x8*>(&tile[r * 128 + ((ch ^ (r >> 3)) & 15) * 8]) = v[it];
  }
  __syncthreads();
  // ---- store: unit = (output row pair p: input columns 2p, 2p+1; 8-row group rc)
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int i = tid + it * 256, rc = i & 15, p = i >> 4;
    const int ch = p >> 2, w = p & 3;  // 16-B chunk of the input row, u32 word in it
    const int pos = ((ch ^ rc) & 15) * 8 + w * 2;
    u16x8 lo, hi;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const unsigned int pr = *reinterpret_cast<const unsigned int*>(&tile[(rc * 8 + j) * 128 + pos]);
      lo[j] = (u16)(pr & 0xffffu);
      hi[j] = (u16)(pr >> 16);
    }
    const int gr = r0 + rc * 8, gc = c0 + 2 * p;
    if (full || gr < R) {
      if (full || gc < C) *reinterpret_cast<u16x8*>(d + (long)gc * ld_dst + gr) = lo;
      if (full || gc + 1 < C) *reinterpret_cast<u16x8*>(d + (long)(gc + 1) * ld_dst + gr) = hi;
    }
  }
}

static int tr_mode() {
  static const int m = [] {
    const char* e = std::getenv("PA_TRANSPOSE");  // 0: 64x64 tiles (round 2-4 kernel)
    return e ? std::atoi(e) : 1;
  }();
  return m;
}

// tile-order group: measured (profiles/r5_transpose_ab.jsonl) 16 is best once the
// operands no longer fit the 256 MB MALL (>= 64 M elements: +8-15 % at 16384 x
// 12288 / 22016, 4096 x 32000), row-major is as good or better below that
static int tr_group(long elems) {
  static const int g = [] {
    const char* e = std::getenv("PA_TR_GROUP");
    return e ? std::atoi(e) : -1;
  }();
  return g >= 0 ? g : (elems >= (64l << 20) ? 16 : 0);
}

PA_EXPORT int pa_transpose2d(int dtype, const void* src, void* dst, int R, int C, long ld_src, long ld_dst,
                             int batch, long bs_src, long bs_dst, hipStream_t st) {
  if (dtype != 1 && dtype != 2) return (int)hipErrorInvalidValue;  // bf16 / f16 bits only
  if ((R | C) & 7 || (ld_src | ld_dst) & 7) return (int)hipErrorInvalidValue;
  if (tr_mode() == 1) {
    const int ntx = (C + 127) / 128, nty = (R + 127) / 128;
    dim3 grid(ntx * nty, batch);
    hipLaunchKernelGGL(transpose128_kernel, grid, dim3(256), 0, st, (const u16*)src, (u16*)dst, R, C, ld_src,
                       ld_dst, bs_src, bs_dst, ntx, nty, tr_group((long)R * C));
    PA_LAUNCH_CHECK();
  }
  dim3 grid((C + 63) / 64, (R + 63) / 64, batch);
  hipLaunchKernelGGL(transpose64_kernel<u16>, grid, dim3(256), 0, st, (const u16*)src, (u16*)dst, R, C,
                     ld_src, ld_dst, bs_src, bs_dst);
  PA_LAUNCH_CHECK();
}

}  // namespace pa
