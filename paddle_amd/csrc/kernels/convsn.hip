// Narrow-output implicit-GEMM convolution (NHWC bf16, Cout tile = 64) for the
// early ResNet stages, with the BatchNorm batch statistics of its output emitted
// from the epilogue.
//
// Why a second conv kernel: gemm.hip's 256x256 tile computes 256 output channels
// per tile; a 64- or 128-channel convolution (ResNet stages 1-2: 64/128 channels
// over 200k-800k output pixels) spends 75 % / 50 % of its MFMA work on zero
// columns.  Here a block owns 256 pixels x 64 channels, so every MFMA is useful,
// and the narrow B tile lets each wave keep ALL 64 columns: 16 ds_read_b128 feed
// 32 MFMAs per k-tile (0.5 reads per MFMA instead of the wide kernel's 0.75).
//
//  * 256 threads = 4 waves; wave w owns pixel rows 64w .. 64w+63 of the tile and
//    all 64 channels (4 x 4 tiles of v_mfma_f32_16x16x32_bf16, 64 fp32 acc/lane).
//  * Operands reach LDS by LDS-DMA (buffer_load_dwordx4 ... lds).  The A operand is
//    gathered straight from the NHWC activation (implicit im2col: a 64-wide k-tile
//    is one filter tap x 64 input channels, C % 64 == 0), with the zero-insertion
//    factor of a strided convolution's data gradient (same addressing as gemm.hip's
//    GA kernels).  Padding / edges / rows past M come back as zeros from the buffer
//    range check.
//  * 2 LDS stages of 40 KiB: two blocks are resident per CU, so one block's MFMA
//    cluster covers the other's barrier + DMA wait.  One barrier per k-tile: the
//    next k-tile's DMA goes out after this k-tile's fragments are in registers.
//  * Epilogue: bf16 store (+ bias) and, optionally, per-channel partial sums of the
//    ROUNDED outputs (shifted by `shift`, e.g. the running mean) and of their
//    squares: part[tile_m][0 / 1][c] -- the layout bn_finalize reduces, so the
//    BatchNorm that consumes this output skips its statistics pass over HBM.
//    STATS == 2 (data gradient of a BN output): the BN backward's sums instead,
//    sum g and sum g (x - mean) with g = the stored gradient under the ReLU mask
//    (common.h BnBwdSrc), taken after an accumulate-into so they cover the final sum.
//  * blockIdx -> tile is XCD-aware (contiguous tile ranges per XCD): neighbouring
//    pixel tiles share their 3x3 halo rows in the same L2.
//
// Reference behaviour: paddle/fluid/operators/conv_cudnn_op.cu.cc:43-171 (cuDNN
// forward / backward-data convolution) and batch_norm_op.cu.cc:53 (the statistics
// the BN forward computes).
#include "common.h"

namespace pa {
namespace convsn {

constexpr int BM = 256, BNC = 64, BK = 64, NT = 256;
constexpr int A_BYTES = BM * BK * 2;   // 32 KiB: 8 units of 32 rows x 128 B
constexpr int B_BYTES = BNC * BK * 2;  //  8 KiB: 2 units
constexpr int STAGE = A_BYTES + B_BYTES;
constexpr int LDS_BYTES = 2 * STAGE;   // 80 KiB -> 2 blocks per CU
constexpr unsigned OOB = 0xFFFFFFF0u;

struct Params {
  const u16* x;     // NHWC source [Nb, H, W, C]
  const u16* w;     // [Cout][KH * KW * C] (K-major rows)
  u16* y;           // [M, Cout]
  const u16* bias;  // [Cout] or null
  float* part;      // [tiles_m][2][Cout] or null
  const float* shift;  // [Cout] or null (0)
  int M, Cout, K;
  int H, W, C, OH, OW, KW, sy, sx, py, px, dy, dx, uy, ux;
  int tiles_m, tiles_n;
  int accumulate;  // y += result (bf16 read-modify-write; a gradient accumulated in place)
  BnBwdSrc bs;     // STATS == 2: BatchNorm backward statistics of y (a data gradient)
};

// Physical placement of piece q (1 KiB = 8 rows x 128 B) of an operand: rows
// 32 * (q >> 2) + 8 * (q & 3) + (lane >> 3); the lane's 16-B chunk is stored at
// position (lane & 7) and holds logical chunk (lane & 7) ^ ((row >> 1) & 7), the
// XOR swizzle under which frag() reads are bank-conflict free.
__device__ __forceinline__ void piece_coords(int q, int lane, int& row, int& kel) {
  row = 32 * (q >> 2) + 8 * (q & 3) + (lane >> 3);
  kel = 8 * ((lane & 7) ^ ((row >> 1) & 7));
}

// MFMA operand fragment: lane holds X[row 16 * i + (lane & 15) of unit u][k = 32 kk + 8 (lane >> 4) + e]
__device__ __forceinline__ bf16x8 frag(const char* opnd, int u, int i, int kk, int lane) {
  const int row = 16 * i + (lane & 15);
  const int ch = (4 * kk + (lane >> 4)) ^ ((row >> 1) & 7);
  return *reinterpret_cast<const bf16x8*>(opnd + u * 4096 + row * 128 + ch * 16);
}

// inclusive prefix sum inside each 16-lane DPP row: lane 16g + 15 ends with the row total
__device__ __forceinline__ float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x111, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x112, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x114, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x118, 0xf, 0xf, true));
  return v;
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

template <int STATS>
__global__ __launch_bounds__(NT, 2) void conv_sn_kernel(Params p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nwg = p.tiles_m * p.tiles_n;
  const int t = xcd_remap(blockIdx.x, nwg);
  const int tm = t / p.tiles_n, tn = t - tm * p.tiles_n;
  const int m0 = tm * BM, n0 = tn * BNC;

  const unsigned x_bytes = (unsigned)((long)(p.M / (p.OH * p.OW)) * p.H * p.W * p.C * 2);
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, 0, x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.w, 0, (unsigned)((long)p.Cout * p.K * 2), 0x00020000);

  // gather plan: wave w DMAs A pieces 8w .. 8w+7, B pieces 2w, 2w+1
  int nb[8], yx[8];
  const int hw = p.OH * p.OW;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    int row, kel;
    piece_coords(8 * wid + j, lane, row, kel);
    const int gm = m0 + row;
    if (gm < p.M) {
      const int n = gm / hw, r = gm - n * hw;
      const int oy = r / p.OW, ox = r - oy * p.OW;
      nb[j] = n * p.H * p.W * p.C + kel;
      yx[j] = ((oy * p.sy - p.py) << 16) | ((ox * p.sx - p.px) & 0xffff);
    } else {
      nb[j] = 0;
      yx[j] = (int)0x80008000u;
    }
  }
  unsigned boff[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    int row, kel;
    piece_coords(2 * wid + j, lane, row, kel);
    boff[j] = n0 + row < p.Cout ? (unsigned)(((long)(n0 + row) * p.K + kel) * 2) : OOB;
  }
  const int my = (1 << p.uy) - 1, mx = (1 << p.ux) - 1;
  auto issue = [&](int kt) {
    char* st = smem + (kt & 1) * STAGE;
    const int k0 = kt * BK;
    const int c0 = k0 % p.C, tap = k0 / p.C;  // wave-uniform: a k-tile is one tap
    const int kh = tap / p.KW, kw = tap - kh * p.KW;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int ny = (yx[j] >> 16) + kh * p.dy;
      const int nx = (int)(short)(yx[j] & 0xffff) + kw * p.dx;
      const int iy = ny >> p.uy, ix = nx >> p.ux;
      const bool ok = ((ny & my) | (nx & mx)) == 0 && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
      const unsigned vo = ok ? (unsigned)(nb[j] + (iy * p.W + ix) * p.C + c0) * 2u : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (__attribute__((address_space(3))) void*)(st + (8 * wid + j) * 1024),
                                               16, vo, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const unsigned vo = boff[j] != OOB ? boff[j] + (unsigned)(k0 * 2) : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsB, (__attribute__((address_space(3))) void*)(st + A_BYTES + (2 * wid + j) * 1024), 16, vo, 0, 0, 0);
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.K / BK;
  issue(0);
  for (int kt = 0; kt < nk; ++kt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of k-tile kt landed
    __builtin_amdgcn_s_barrier();                     // ... everyone's; everyone done reading kt-1
    __builtin_amdgcn_sched_barrier(0);
    const char* A_ = smem + (kt & 1) * STAGE;
    const char* B_ = A_ + A_BYTES;
    bf16x8 fa[4][2], fb[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) fa[i][kk] = frag(A_, 2 * wid + (i >> 1), i & 1, kk, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) fb[j][kk] = frag(B_, j >> 1, j & 1, kk, lane);
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 1 < nk) issue(kt + 1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j][kk], fa[i][kk], acc[i][j], 0, 0, 0);
  }

  // ---- epilogue: lane holds C[m = 64 wid + 16 i + (lane & 15)][n = 16 j + 4 (lane >> 4) + r]
  const int ml = lane & 15, g = lane >> 4;
  float bv[4][4], sh[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + 16 * j + 4 * g + r;
      bv[j][r] = (p.bias && n < p.Cout) ? bf2f(p.bias[n]) : 0.f;
      sh[j][r] = (STATS == 1 && p.shift && n < p.Cout) ? p.shift[n] : 0.f;
    }
  float msc[4][4], msf[4][4];
  if constexpr (STATS == 2) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + 16 * j + 4 * g + r;
        if (n < p.Cout) {
          bn_bwd_coef(p.bs, n, sh[j][r], msc[j][r], msf[j][r]);
        } else {
          sh[j][r] = msc[j][r] = msf[j][r] = 0.f;
        }
      }
  }
  float s1[4][4], s2[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) s1[j][r] = s2[j][r] = 0.f;
  // STATS == 2: every BN input / output chunk of the wave's rows is loaded before the
  // first store (the compiler cannot move loads across stores to y)
  u16x4 bxa[4][4], bya[4][4];
  if constexpr (STATS == 2) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = m0 + 64 * wid + 16 * i + ml;
        const int n = n0 + 16 * j + 4 * g;
        const bool ok = m < p.M && n < p.Cout;
        bxa[i][j] = ok ? *reinterpret_cast<const u16x4*>(p.bs.x + (long)m * p.Cout + n) : u16x4{0, 0, 0, 0};
        bya[i][j] = (ok && p.bs.y) ? *reinterpret_cast<const u16x4*>(p.bs.y + (long)m * p.Cout + n)
                                   : u16x4{0, 0, 0, 0};
      }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + 64 * wid + 16 * i + ml;
    const bool mok = m < p.M;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + 16 * j + 4 * g;
      const bool ok = mok && n < p.Cout;
      u16x4 old = {0, 0, 0, 0};
      if (p.accumulate && ok) old = *reinterpret_cast<const u16x4*>(p.y + (long)m * p.Cout + n);
      u16x4 o;
      u16x4 bx = {0, 0, 0, 0}, by = {0, 0, 0, 0};
      if constexpr (STATS == 2) {
        bx = bxa[i][j];
        by = bya[i][j];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        o[r] = f2bf(acc[i][j][r] + bv[j][r] + (p.accumulate ? bf2f(old[r]) : 0.f));
        if (STATS == 1) {
          const float d = mok ? bf2f(o[r]) - sh[j][r] : 0.f;
          s1[j][r] += d;
          s2[j][r] += d * d;
        } else if (STATS == 2) {
          const float xv = bf2f(bx[r]);
          const bool keep = !p.bs.relu || (p.bs.y ? bf2f(by[r]) > 0.f : fmaf(xv, msc[j][r], msf[j][r]) > 0.f);
          const float gv = (ok && keep) ? bf2f(o[r]) : 0.f;
          s1[j][r] += gv;
          s2[j][r] += gv * (xv - sh[j][r]);
        }
      }
      if (ok) *reinterpret_cast<u16x4*>(p.y + (long)m * p.Cout + n) = o;
    }
  }
  if constexpr (STATS != 0) {
    __syncthreads();  // every wave is done with the stage buffers
    float* red = reinterpret_cast<float*>(smem);  // [4 waves][64 channels][2]
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float a = row16_sum(s1[j][r]);
        const float b = row16_sum(s2[j][r]);
        if (ml == 15) {
          const int nl = 16 * j + 4 * g + r;
          red[(wid * 64 + nl) * 2] = a;
          red[(wid * 64 + nl) * 2 + 1] = b;
        }
      }
    __syncthreads();
    if (tid < 64 && n0 + tid < p.Cout) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        a += red[(w * 64 + tid) * 2];
        b += red[(w * 64 + tid) * 2 + 1];
      }
      p.part[((long)tm * 2) * p.Cout + n0 + tid] = a;
      p.part[((long)tm * 2 + 1) * p.Cout + n0 + tid] = b;
    }
  }
}

template <int STATS>
static int launch(const Params& p, hipStream_t st) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)conv_sn_kernel<STATS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       LDS_BYTES);
    if (e != hipSuccess) return (int)e;
    attr_set = true;
  }
  hipLaunchKernelGGL(conv_sn_kernel<STATS>, dim3(p.tiles_m * p.tiles_n), dim3(NT), LDS_BYTES, st, p);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------ weight gradient
// dW[co][(kh, kw, c)] = sum_m dY[m][co] X[pixel(m) + tap(kh, kw)][c] with the filter
// taps gathered from the NHWC activation (no im2col buffer).  Both operands have the
// reduction (output pixel m) as their outer dimension, so both are staged MN-major
// (64 k-rows x 128 B slabs, swizzled) and read with ds_read_b64_tr_b16.
//  * block tile: 64 output channels x 4 slabs of 64 K-columns; a K slab is one
//    (tap, 64-channel block), i.e. 128-B rows of the activation: each wave owns one
//    slab, so its gather tap is fixed for the whole block.
//  * the reduction over pixels is split across blocks (each block a contiguous range
//    of 64-pixel k-tiles); the partial tiles go to part[split][Cout][K] (fp32) and
//    pa_splitk_reduce sums them: deterministic, no atomics.
//  * pixel -> (image, oy, ox) is advanced incrementally per k-tile (no divisions in
//    the loop).
constexpr int WG_SLABS = 4;
constexpr int WG_STAGE = 8192 + WG_SLABS * 8192;  // dY slab + 4 X slabs = 40 KiB

struct WgParams {
  const u16* dy;  // [M][Cout]
  const u16* x;   // NHWC [Nb][H][W][C]
  float* part;    // [splits][Cout][K]
  int M, Cout, K, nslab;  // nslab = KH * KW * C / 64
  int H, W, C, OH, OW, KW, sy, sx, py, px, dly, dlx;
  int adv_oy, adv_ox;  // 64 pixels = adv_oy rows + adv_ox columns of the output grid
  int tiles_co, tiles_n, kt_per_split, nkt;
};

__device__ __forceinline__ int mn_swz(int k) { return 2 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1)); }

__device__ __forceinline__ unsigned lds_addr(const char* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

// MN-major fragment of 32-mn block u (slab u >> 1), 16-row half i, k-step kk:
// lane holds X[mn = 32 u + 16 i + (lane & 15)][k = 32 kk + 8 (lane >> 4) + e] (two
// transposing reads; the destinations are fenced by wait()).
struct FragT {
  i16x4 x, y;
  __device__ __forceinline__ void load(const char* opnd, int u, int i, int kk, int lane) {
    const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
    const int k0 = 32 * kk + 8 * g + q;
    const int ch = (4 * (u & 1) + 2 * i + (pp >> 1)) ^ mn_swz(k0);
    const unsigned a = lds_addr(opnd + (u >> 1) * 8192 + k0 * 128 + ch * 16 + 8 * (pp & 1));
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(x) : "v"(a));
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:512" : "=v"(y) : "v"(a));
  }
  __device__ __forceinline__ void wait() { asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(x), "+v"(y)); }
  __device__ __forceinline__ bf16x8 get() const {
    i16x8 v = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
};

__global__ __launch_bounds__(NT, 2) void conv_wgrad_sn_kernel(WgParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntile = p.tiles_co * p.tiles_n;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = bid / ntile, t = bid - split * ntile;
  const int tco = t / p.tiles_n, tn = t - tco * p.tiles_n;
  const int co0 = tco * 64;
  const int kt0 = split * p.kt_per_split;
  const int kt1 = min(p.nkt, kt0 + p.kt_per_split);
  if (kt0 >= kt1) return;  // block-uniform
  const int gs = WG_SLABS * tn + wid;  // this wave's K slab
  const bool slab_ok = gs < p.nslab;
  const int CB = p.C / 64;
  const int tap = slab_ok ? gs / CB : 0, cb = gs - (gs / CB) * CB;
  const int kh = tap / p.KW, kw = tap - (tap / p.KW) * p.KW;

  const __amdgpu_buffer_rsrc_t rsD =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.dy, 0, (unsigned)((long)p.M * p.Cout * 2), 0x00020000);
  const unsigned x_bytes = (unsigned)((long)(p.M / (p.OH * p.OW)) * p.H * p.W * p.C * 2);
  const __amdgpu_buffer_rsrc_t rsX = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, 0, x_bytes, 0x00020000);

  // per-lane gather state of the wave's 8 X pieces (rows 8j + (lane >> 3) of the k-tile)
  int gm[8], gn[8], goy[8], gox[8];
  const int hw = p.OH * p.OW;
  // 16-B chunk of a lane in piece j: logical chunk (lane & 7) ^ swz(k-row 8j + (lane >> 3));
  // the swizzle depends on bit 3 of the k-row, i.e. on the piece parity
  const int kx0 = 8 * ((lane & 7) ^ mn_swz(lane >> 3)), kx1 = 8 * ((lane & 7) ^ mn_swz(8 + (lane >> 3)));
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int m = kt0 * 64 + 8 * j + (lane >> 3);
    gm[j] = m;
    const int n = m / hw, r = m - n * hw;
    gn[j] = n;
    goy[j] = r / p.OW;
    gox[j] = r - goy[j] * p.OW;
  }
  // dY pieces 2w + jj: rows 8 (2w + jj) + (lane >> 3) (parity jj), chunk (lane & 7) ^ swz
  const int dyc0 = co0 + kx0, dyc1 = co0 + kx1;

  auto issue = [&](int kt) {
    char* st = smem + (kt & 1) * WG_STAGE;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int pc = 2 * wid + jj;
      const int m = kt * 64 + 8 * pc + (lane >> 3);
      const int dyc = jj ? dyc1 : dyc0;
      const unsigned vo = (dyc < p.Cout && m < p.M) ? (unsigned)(((long)m * p.Cout + dyc) * 2) : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsD, (__attribute__((address_space(3))) void*)(st + pc * 1024), 16, vo,
                                               0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int iy = goy[j] * p.sy - p.py + kh * p.dly;
      const int ix = gox[j] * p.sx - p.px + kw * p.dlx;
      const bool ok = slab_ok && gm[j] < p.M && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
      const unsigned vo = ok ? (unsigned)((((gn[j] * p.H + iy) * p.W + ix) * p.C + cb * 64 + ((j & 1) ? kx1 : kx0)) * 2)
                             : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsX, (__attribute__((address_space(3))) void*)(st + 8192 + wid * 8192 + j * 1024), 16, vo, 0, 0, 0);
    }
    // advance the gather state by 64 pixels
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      gm[j] += 64;
      gox[j] += p.adv_ox;
      goy[j] += p.adv_oy;
      if (gox[j] >= p.OW) {
        gox[j] -= p.OW;
        goy[j] += 1;
      }
      while (goy[j] >= p.OH) {
        goy[j] -= p.OH;
        gn[j] += 1;
      }
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue(kt0);
  for (int kt = kt0; kt < kt1; ++kt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const char* D_ = smem + (kt & 1) * WG_STAGE;
    const char* X_ = D_ + 8192 + wid * 8192;
    FragT fa[4][2], fb[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) fa[i][kk].load(D_, i >> 1, i & 1, kk, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) fb[j][kk].load(X_, j >> 1, j & 1, kk, lane);
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 1 < kt1) issue(kt + 1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        fa[i][kk].wait();
        fb[i][kk].wait();
      }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j][kk].get(), fa[i][kk].get(), acc[i][j], 0, 0, 0);
  }
  // lane holds dW[co = co0 + 16 i + (lane & 15)][kcol = 64 gs + 16 j + 4 (lane >> 4) + r]
  if (!slab_ok) return;
  float* out = p.part + (long)split * p.Cout * p.K;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int co = co0 + 16 * i + (lane & 15);
    if (co >= p.Cout) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int kc = 64 * gs + 16 * j + 4 * (lane >> 4);
      *reinterpret_cast<f32x4*>(out + (long)co * p.K + kc) = acc[i][j];
    }
  }
}

}  // namespace convsn
}  // namespace pa

using namespace pa;

PA_EXPORT int pa_splitk_reduce(const float* part, float* out, long n, int S, int accumulate, hipStream_t st);

// Same geometry arguments as pa_conv_gemm (uy / ux: log2 zero-insertion factors of a
// strided conv's data gradient).  part (nullable): per-channel partial statistics of
// the output, [tiles_m][2][Cout] with tiles_m = ceil(Nb*OH*OW / 256) (see
// pa_conv_sn_tiles); shift (nullable, fp32 [Cout]) is subtracted before summing.
PA_EXPORT int pa_conv_sn_acc(const void* src, const void* wt, void* out, const void* bias, int Nb, int H, int W,
                             int C, int OH, int OW, int Cout, int KH, int KW, int sy, int sx, int py, int px, int dy,
                             int dx, int uy, int ux, float* part, const float* shift, int accumulate, hipStream_t st);

PA_EXPORT int pa_conv_sn(const void* src, const void* wt, void* out, const void* bias, int Nb, int H, int W, int C,
                         int OH, int OW, int Cout, int KH, int KW, int sy, int sx, int py, int px, int dy, int dx,
                         int uy, int ux, float* part, const float* shift, hipStream_t st) {
  return pa_conv_sn_acc(src, wt, out, bias, Nb, H, W, C, OH, OW, Cout, KH, KW, sy, sx, py, px, dy, dx, uy, ux, part,
                        shift, 0, st);
}

// accumulate: out += conv (bf16 in place; no statistics with it)
PA_EXPORT int pa_conv_sn_acc(const void* src, const void* wt, void* out, const void* bias, int Nb, int H, int W,
                             int C, int OH, int OW, int Cout, int KH, int KW, int sy, int sx, int py, int px, int dy,
                             int dx, int uy, int ux, float* part, const float* shift, int accumulate, hipStream_t st) {
  const long M = (long)Nb * OH * OW;
  if (M <= 0 || Cout <= 0) return 0;
  if (C % 64 || Cout % 8 || M > 0x7fffffffL || (long)Nb * H * W * C >= 0x7fffffffL || H > 32767 || W > 32767 ||
      (long)Cout * KH * KW * C >= 0x7fffffffL)
    return -1;
  convsn::Params p{};
  p.x = (const u16*)src;
  p.w = (const u16*)wt;
  p.y = (u16*)out;
  p.bias = (const u16*)bias;
  p.part = part;
  p.shift = shift;
  p.M = (int)M;
  p.Cout = Cout;
  p.K = KH * KW * C;
  p.H = H; p.W = W; p.C = C; p.OH = OH; p.OW = OW; p.KW = KW;
  p.sy = sy; p.sx = sx; p.py = py; p.px = px; p.dy = dy; p.dx = dx; p.uy = uy; p.ux = ux;
  p.tiles_m = (int)((M + convsn::BM - 1) / convsn::BM);
  p.tiles_n = (Cout + convsn::BNC - 1) / convsn::BNC;
  p.accumulate = accumulate;
  if (accumulate && part) return -1;
  return part ? convsn::launch<1>(p, st) : convsn::launch<0>(p, st);
}

// Data gradient with the BatchNorm backward statistics of its (final, after an
// optional accumulate-into) values: part [tiles_m][2][Cout] of sum g, sum g (x - mean)
// (see BnBwdSrc); bx / by: BN input / output [M, Cout], by null = mask from bx.
PA_EXPORT int pa_conv_sn_bnbwd(const void* src, const void* wt, void* out, int Nb, int H, int W, int C, int OH, int OW,
                               int Cout, int KH, int KW, int sy, int sx, int py, int px, int dy, int dx, int uy, int ux,
                               int accumulate, float* part, const void* bx, const void* by, const float* mean,
                               const float* rstd, const void* w, const void* b, int wdt, int relu, hipStream_t st) {
  const long M = (long)Nb * OH * OW;
  if (M <= 0 || Cout <= 0 || !part || !bx || !mean || !rstd) return -1;
  if (C % 64 || Cout % 8 || M > 0x7fffffffL || (long)Nb * H * W * C >= 0x7fffffffL || H > 32767 || W > 32767 ||
      (long)Cout * KH * KW * C >= 0x7fffffffL)
    return -1;
  convsn::Params p{};
  p.x = (const u16*)src;
  p.w = (const u16*)wt;
  p.y = (u16*)out;
  p.part = part;
  p.M = (int)M;
  p.Cout = Cout;
  p.K = KH * KW * C;
  p.H = H; p.W = W; p.C = C; p.OH = OH; p.OW = OW; p.KW = KW;
  p.sy = sy; p.sx = sx; p.py = py; p.px = px; p.dy = dy; p.dx = dx; p.uy = uy; p.ux = ux;
  p.tiles_m = (int)((M + convsn::BM - 1) / convsn::BM);
  p.tiles_n = (Cout + convsn::BNC - 1) / convsn::BNC;
  p.accumulate = accumulate;
  p.bs = BnBwdSrc{(const u16*)bx, (const u16*)by, mean, rstd, w, b, wdt, relu};
  return convsn::launch<2>(p, st);
}

PA_EXPORT int pa_conv_sn_tiles(long M) { return (int)((M + convsn::BM - 1) / convsn::BM); }

// Weight gradient of an NHWC convolution (C % 64 == 0): dw [Cout][KH*KW*C] fp32
// (= or += with `accumulate`) from dY [Nb*OH*OW][Cout] and x; `ws`: workspace of
// pa_conv_wgrad_sn_ws floats (0 -> the kernel writes dw directly).
static void wgrad_plan(const convsn::WgParams& p0, int& splits, int& ktps) {
  const int tiles = p0.tiles_co * p0.tiles_n;
  int s = (1024 + tiles - 1) / tiles;          // ~4 resident waves of blocks over 256 CUs
  const int smax = (p0.nkt + 15) / 16;         // >= 16 k-tiles (1024 pixels) per block
  if (s > smax) s = smax;
  if (s < 1) s = 1;
  ktps = (p0.nkt + s - 1) / s;
  splits = (p0.nkt + ktps - 1) / ktps;
}

static int wgrad_setup(convsn::WgParams& p, const void* dyp, const void* x, int Nb, int H, int W, int C, int OH, int OW,
                       int Cout, int KH, int KW, int sy, int sx, int py, int px, int dly, int dlx) {
  const long M = (long)Nb * OH * OW;
  if (M <= 0 || C % 64 || Cout % 8 || M * Cout >= 0x7fffffffL || (long)Nb * H * W * C >= 0x7fffffffL) return -1;
  p = convsn::WgParams{};
  p.dy = (const u16*)dyp;
  p.x = (const u16*)x;
  p.M = (int)M;
  p.Cout = Cout;
  p.K = KH * KW * C;
  p.nslab = p.K / 64;
  p.H = H; p.W = W; p.C = C; p.OH = OH; p.OW = OW; p.KW = KW;
  p.sy = sy; p.sx = sx; p.py = py; p.px = px; p.dly = dly; p.dlx = dlx;
  p.adv_oy = 64 / OW;
  p.adv_ox = 64 % OW;
  p.tiles_co = (Cout + 63) / 64;
  p.tiles_n = (p.nslab + convsn::WG_SLABS - 1) / convsn::WG_SLABS;
  p.nkt = (int)((M + 63) / 64);
  return 0;
}

// sum of the split partials [S][Cout][(kh, kw, c)] written straight into the weight's
// own layout [Cout][C][KH][KW] and dtype (fp32 or bf16): no permute / cast pass after
__global__ void wgrad_reduce_kernel(const float* __restrict__ part, int S, int Cout, int C, int KH, int KW,
                                    void* __restrict__ out, int out_bf16, int accumulate) {
  // threads walk the partials in their own order (K-contiguous: every split's read is
  // coalesced); each sum is written once to its [co][c][kh][kw] slot
  const long K = (long)KH * KW * C, n = (long)Cout * K, taps = (long)KH * KW;
  for (long src = blockIdx.x * (long)blockDim.x + threadIdx.x; src < n; src += (long)gridDim.x * blockDim.x) {
    const long co = src / K, kk = src - co * K;
    const long c = kk % C, tap = kk / C;
    const long o = co * K + c * taps + tap;
    float a = 0.f;
    for (int sp = 0; sp < S; ++sp) a += part[(long)sp * n + src];
    if (out_bf16) {
      u16* y = (u16*)out;
      y[o] = f2bf(accumulate ? a + bf2f(y[o]) : a);
    } else {
      float* y = (float*)out;
      y[o] = accumulate ? a + y[o] : a;
    }
  }
}

PA_EXPORT long pa_conv_wgrad_sn_ws(int Nb, int H, int W, int C, int OH, int OW, int Cout, int KH, int KW) {
  convsn::WgParams p;
  if (wgrad_setup(p, nullptr, nullptr, Nb, H, W, C, OH, OW, Cout, KH, KW, 1, 1, 0, 0, 1, 1)) return -1;
  int splits, ktps;
  wgrad_plan(p, splits, ktps);
  return splits > 1 ? (long)splits * Cout * p.K : 0;
}

// workspace floats for pa_conv_wgrad_sn_w (always staged: the reduce writes the layout)
PA_EXPORT long pa_conv_wgrad_sn_ws2(int Nb, int H, int W, int C, int OH, int OW, int Cout, int KH, int KW) {
  convsn::WgParams p;
  if (wgrad_setup(p, nullptr, nullptr, Nb, H, W, C, OH, OW, Cout, KH, KW, 1, 1, 0, 0, 1, 1)) return -1;
  int splits, ktps;
  wgrad_plan(p, splits, ktps);
  return (long)splits * Cout * p.K;
}

// weight gradient in the PARAMETER's layout [Cout][C][KH][KW] and dtype (w_bf16);
// ws: pa_conv_wgrad_sn_ws2 floats
PA_EXPORT int pa_conv_wgrad_sn_w(const void* dyp, const void* x, void* dw, int w_bf16, float* ws, int Nb, int H,
                                 int W, int C, int OH, int OW, int Cout, int KH, int KW, int sy, int sx, int py,
                                 int px, int dly, int dlx, int accumulate, hipStream_t st) {
  convsn::WgParams p;
  if (wgrad_setup(p, dyp, x, Nb, H, W, C, OH, OW, Cout, KH, KW, sy, sx, py, px, dly, dlx)) return -1;
  if (!ws) return -2;
  int splits, ktps;
  wgrad_plan(p, splits, ktps);
  p.kt_per_split = ktps;
  p.part = ws;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)convsn::conv_wgrad_sn_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 2 * convsn::WG_STAGE);
    if (e != hipSuccess) return (int)e;
    attr_set = true;
  }
  hipLaunchKernelGGL(convsn::conv_wgrad_sn_kernel, dim3(p.tiles_co * p.tiles_n * splits), dim3(convsn::NT),
                     2 * convsn::WG_STAGE, st, p);
  const long n = (long)Cout * p.K;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(stream_grid(n, 256)), dim3(256), 0, st, ws, splits, Cout, C,
                     KH, KW, dw, w_bf16, accumulate);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_conv_wgrad_sn(const void* dyp, const void* x, float* dw, float* ws, int Nb, int H, int W, int C,
                               int OH, int OW, int Cout, int KH, int KW, int sy, int sx, int py, int px, int dly,
                               int dlx, int accumulate, hipStream_t st) {
  convsn::WgParams p;
  if (wgrad_setup(p, dyp, x, Nb, H, W, C, OH, OW, Cout, KH, KW, sy, sx, py, px, dly, dlx)) return -1;
  int splits, ktps;
  wgrad_plan(p, splits, ktps);
  if (splits > 1 && !ws) return -2;
  if (splits == 1 && accumulate && !ws) return -2;
  p.kt_per_split = ktps;
  p.part = (splits > 1 || accumulate) ? ws : dw;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)convsn::conv_wgrad_sn_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 2 * convsn::WG_STAGE);
    if (e != hipSuccess) return (int)e;
    attr_set = true;
  }
  const int grid = p.tiles_co * p.tiles_n * splits;
  hipLaunchKernelGGL(convsn::conv_wgrad_sn_kernel, dim3(grid), dim3(convsn::NT), 2 * convsn::WG_STAGE, st, p);
  if (p.part != dw) return pa_splitk_reduce(ws, dw, (long)Cout * p.K, splits, accumulate, st);
  PA_LAUNCH_CHECK();
}

