// Hand-written gfx950 bf16 GEMM on MFMA (v_mfma_f32_16x16x32_bf16), fp32 accumulate.
//
//   C[m, n] (=|+=) alpha * sum_k A(m, k) B(n, k)  (+ bias[n])
//
// Each operand is either K-contiguous ("K-major": X[mn * ld + k]) or MN-contiguous
// ("MN-major": X[k * ld + mn]), so one kernel family covers every linear-layer
// GEMM of a training step without transposed copies (Paddle weights are [in, out]):
//   forward   y  = x W      : A = x (K-major),   B = W (MN-major)
//   backward  dx = dy W^T   : A = dy (K-major),  B = W (K-major)
//   backward  dW = x^T dy   : A = x (MN-major),  B = dy (MN-major), fp32 += into main_grad
// Reference: paddle/fluid/operators/math/blas_impl.cu.h:27-200 (cuBLAS gemm /
// batched gemm behind mul_op / matmul_op / fc); here the library call is replaced.
//
// Design (MI355X-first; guide §5 "256² 8-phase template", re-derived):
//  * 256x256 block tile, BK = 64, 512 threads = 8 waves as 2 (M) x 4 (N); each wave
//    owns a 128 x 64 output (8 x 4 tiles of 16x16 = 128 fp32 accumulators/lane).
//  * Operands arrive in LDS by LDS-DMA (`buffer_load_dwordx4 ... lds`, 1 KiB per
//    wave-instruction); the buffer descriptor's range check zero-fills every edge
//    (M, N, K need only be multiples of 8), so there is no edge code in the loop.
//  * LDS holds 2 K-tile stages of 8 slabs (64 mn x 64 k, 8 KiB each), XOR-swizzled
//    for conflict-free reads: K-major slabs are read by ds_read_b128, MN-major slabs
//    by ds_read_b64_tr_b16 (hardware transpose); the swizzle is applied to the
//    per-lane SOURCE address because LDS-DMA writes lane-linearly, and every DMA
//    wave-instruction reads 8 full 128-B global lines in either layout.
//  * 4 phases per K-tile, one 64x32 quadrant (16 MFMA) per phase.  The two wave
//    groups (wr = 0/1, one wave of each per SIMD) run one barrier apart, so one
//    group's LDS reads + DMA issue overlap the other group's MFMA cluster.
//  * LDS regions are refilled as soon as their last reader has passed a barrier
//    (A rows 0-63 after phase 1, B after phase 2, A rows 64-127 after phase 3);
//    waits are counted `s_waitcnt vmcnt(N)` (never 0 in the loop) so each DMA has
//    ~4 phases of MFMA work to land under.
//  * blockIdx -> tile is XCD-aware (contiguous tile bands per XCD, bijective).
#include "common.h"

namespace pa {
namespace gemm {

constexpr int BM = 256, BN = 256, BKT = 64, NT = 512;
constexpr int UNIT = 4096;            // bytes: 32 (mn) x 64 (k) bf16
constexpr int OPND = 8 * UNIT;        // one operand of one stage (256 x 64 bf16)
constexpr int STAGE = 2 * OPND;       // A + B
constexpr int LDS_BYTES = STAGE + 128 * 528;  // 2 stages (128 KiB); C staging above stage 0
constexpr unsigned OOB = 0xFFFFFFF0u; // voffset beyond num_records -> DMA writes zeros

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

struct Params {
  const void* A;
  const void* B;
  void* C;
  const void* bias;  // [N], same dtype as C (bf16 or fp32); may be null
  int M, N, K;
  long lda, ldb, ldc;
  long sA, sB, sC;   // batch strides (elements)
  float alpha;
  int accumulate;    // C += result (beta = 1)
  int tiles_m, tiles_n;
  // split-K through the batch index: batch b reduces k in [b*K, min((b+1)*K, k_total))
  // (k_total = 0: batches are independent GEMMs of depth K)
  int k_total;
  int atomic;  // fp32 C only: C += tile with float atomics (split-K partials, no bias)
  // grouped (ragged) GEMM over batch = group: grp[0..G] are row offsets (device).
  //  grp_mode 1: group g owns rows [grp[g], grp[g+1]) of A (K-major) and of C; M is
  //              the total row count (sizes the grid), B advances by sB per group
  //  grp_mode 2: group g reduces over rows [grp[g], grp[g+1]) of A and B (both
  //              MN-major: dW of grouped experts); C advances by sC per group.
  //              Or both K-major (token-contiguous X^T / dY^T images, 64-aligned
  //              group columns): grp[] are column offsets; F8 additionally in fp8
  //              elements (multiples of 16), sa / sb per group (sas / sbs)
  const int* grp;
  int grp_mode;
  // F8 kernels: C = alpha * sa[row] * sb[col] * (A_q B_q^T); sa indexed by the
  // global row of A (grouped: the ragged row), sb by b * sbs + n
  const float* sa;
  const float* sb;
  int sbs;
  int sas;  // grp_mode 2 F8: sa advances by sas per group
  int ngrp;  // grp_mode 1: number of groups (M = total rows)
  const int* grp_tiles;  // grp_mode 1: per global tile row, group << 16 | row tile in group (-1: none)
  // implicit-GEMM convolution (GA kernels): A(m, k) gathered from an NHWC source
  // tensor: m = (n, oy, ox) over an OH x OW grid, k = (kh, kw, c) with Cc % 64 == 0.
  // Source pixel: ny = oy*sy - py + kh*dy; with a zero-insertion factor 2^uy
  // (dgrad of a stride-2^uy conv) only ny % 2^uy == 0 hits, at row ny >> uy.
  int H, W, Cc, OH, OW, KW, sy, sx, py, px, dy, dx, uy, ux;
  int stagger;  // persistent grids: block slot (bid / 8) % 8 idles slot * stagger * ~0.5 us first
  // GA (conv) kernels, bf16 out: per-channel BatchNorm statistics of the ROUNDED
  // output about `shift` (nullable) into part[tile_m][0 / 1][N] (sum, sum of squares)
  float* part;
  const float* shift;
  // GA conv kernels, bf16 out, bs.x != null: the BatchNorm BACKWARD statistics of the
  // stored gradient instead (sum g, sum g (x - mean); common.h BnBwdSrc), into part
  BnBwdSrc bs;
  // fused epilogues of the bf16 K x K kernels (EPI template parameter, pa_gemm_epi):
  //  1 SwiGLU forward: C = the [gate|up] tile with gate and up interleaved in blocks of
  //    16 columns (block b: gate cols 32b..32b+15, up 32b+16..32b+31); aux = h [M][N/2]
  //    = silu(gate) * up, computed from the stored (bf16-rounded) tile
  //  2 SwiGLU backward: the accumulator is da [M][N]; aux = gu [M][2N] in the layout of
  //    1; C = dgu [M][2N] (dgate, dup at gu's positions) -- da never reaches memory
  //  3 RoPE (neox, head dim 128): columns < rope_cols are rotated in 128-column heads
  //    by cos / sin [rope_S][64] at position row % rope_S (the packed QKV projection)
  void* aux;
  long ldaux;
  const float* cosT;
  const float* sinT;
  int rope_cols, rope_S;
};

// LDS image of one operand of one stage: 4 "slabs" of 64 mn x 64 k (8 KiB each);
// slab s covers mn 64s .. 64s+63 of the 256-wide tile.
//  * K-major slab: two 4-KiB units of 32 rows (mn) x 128 B (64 k);
//    16-B chunk' = chunk ^ ((row >> 1) & 7)   (conflict-free ds_read_b128)
//  * MN-major slab: 64 rows (k) x 128 B (64 mn);
//    chunk' = chunk ^ s(k), s(k) = 2*(((k>>1)&1) | (((k>>3)&1)<<1))  (conflict-free tr_b16)
// One LDS-DMA wave-instruction ("piece", 1 KiB) fills 8 rows of 128 B, i.e. full
// 128-B global lines in both layouts.  Regions (DMA'd as a unit): A_FIRST = slabs
// {0, 2} (rows 0-63 of each wave group), A_SEC = {1, 3}, B = all four slabs.
enum Region { A_FIRST = 0, A_SEC = 1, B_ALL = 2 };

__device__ __forceinline__ int mn_swz(int k) { return 2 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1)); }

// (mn, k) of the 16-B chunk this lane DMAs for piece pc (0..7) of slab sl.
template <bool KMAJ>
__device__ __forceinline__ void dma_coords(int sl, int pc, int lane, int& mn, int& k) {
  const int row = 8 * (pc & 3) + (lane >> 3);
  if (KMAJ) {
    const int ch = (lane & 7) ^ ((row >> 1) & 7);
    mn = 64 * sl + 32 * (pc >> 2) + row;
    k = 8 * ch;
  } else {
    const int kr = 8 * pc + (lane >> 3);
    const int ch = (lane & 7) ^ mn_swz(kr);
    mn = 64 * sl + 8 * ch;
    k = kr;
  }
}

// Pieces of a region issued by wave w: A regions have 16 pieces (2 per wave),
// B has 32 (4 per wave).  Returns the slab and the piece within it.
__device__ __forceinline__ void region_piece(int region, int wid, int j, int& sl, int& pc) {
  if (region == B_ALL) {
    const int q = 4 * wid + j;
    sl = q >> 3;
    pc = q & 7;
  } else {
    const int q = 2 * wid + j;
    sl = 2 * (q >> 3) + (region == A_SEC ? 1 : 0);
    pc = q & 7;
  }
}

// One wave's DMA plan for one region: byte offset of each piece at k-tile 0 (OOB
// when its mn row/col is outside the matrix) and, for K not a multiple of 64, the
// k coordinate within the tile for the per-lane range check of the last k-tile.
template <int NP, bool KFULL>
struct DmaLane {
  unsigned off[NP];
  int kk[KFULL ? 1 : NP];
};

template <bool KMAJ, int NP, bool KFULL>
__device__ __forceinline__ void dma_plan(DmaLane<NP, KFULL>& d, int region, int j0, int wid, int lane,
                                         int mn_tile0, int MN, long ld) {
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    int sl, pc, mn, k;
    region_piece(region, wid, j0 + j, sl, pc);
    dma_coords<KMAJ>(sl, pc, lane, mn, k);
    const int gmn = mn_tile0 + mn;
    if (!KFULL) d.kk[j] = k;
    d.off[j] = gmn >= MN ? OOB
                         : (KMAJ ? (unsigned)(((long)gmn * ld + k) * 2) : (unsigned)(((long)k * ld + gmn) * 2));
  }
}

// Issue this wave's pieces j0 .. j0+NP-1 of `region` for k-tile kt (kt >= nk: the
// whole wave writes zeros, no memory traffic).
template <bool KMAJ, int NP, bool KFULL>
__device__ __forceinline__ void dma_issue(const DmaLane<NP, KFULL>& d, __amdgpu_buffer_rsrc_t rs, char* stage_opnd,
                                          int region, int j0, int wid, int kt, int K, long ld) {
  const int k0 = kt * BKT;
  const unsigned kstep = KMAJ ? (unsigned)(k0 * 2) : (unsigned)((long)k0 * ld * 2);
  const bool kt_ok = k0 < K;  // wave-uniform
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    int sl, pc;
    region_piece(region, wid, j0 + j, sl, pc);
    bool ok = kt_ok && d.off[j] != OOB;
    if (!KFULL) ok = ok && (k0 + d.kk[j] < K);
    const unsigned vo = ok ? d.off[j] + kstep : OOB;
    char* dst = stage_opnd + sl * 8192 + pc * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)dst, 16, vo, 0, 0, 0);
  }
}

// Conv-gather plan of one A region for one wave: per piece the element offset of the
// image (plus this lane's 8-channel chunk) and the packed (ybase, xbase) of its
// output pixel (ybase = -32768 marks a row past M: every range check fails).
template <int NP>
struct GatherLane {
  int nb[NP];
  int yx[NP];
};

template <int NP>
__device__ __forceinline__ void gather_plan(GatherLane<NP>& d, int region, int wid, int lane, int m_tile0,
                                            const Params& p) {
  const int hw = p.OH * p.OW;
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    int sl, pc, mn, k;
    region_piece(region, wid, j, sl, pc);
    dma_coords<true>(sl, pc, lane, mn, k);
    const int gm = m_tile0 + mn;
    if (gm < p.M) {
      const int n = gm / hw, r = gm - n * hw;
      const int oy = r / p.OW, ox = r - oy * p.OW;
      d.nb[j] = n * p.H * p.W * p.Cc + k;
      d.yx[j] = ((oy * p.sy - p.py) << 16) | ((ox * p.sx - p.px) & 0xffff);
    } else {
      d.nb[j] = 0;
      d.yx[j] = (int)0x80008000u;
    }
  }
}

template <int NP>
__device__ __forceinline__ void gather_issue(const GatherLane<NP>& d, __amdgpu_buffer_rsrc_t rs, char* stage_opnd,
                                             int region, int wid, int kt, const Params& p) {
  const int k0 = kt * BKT;
  const bool kt_ok = k0 < p.K;
  // (kh, kw, c0) of this k-tile: wave-uniform scalars (a k-tile never crosses a tap, C % 64 == 0)
  const int c0 = k0 % p.Cc, tap = k0 / p.Cc;
  const int kh = tap / p.KW, kw = tap - kh * p.KW;
  const int my = (1 << p.uy) - 1, mx = (1 << p.ux) - 1;
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    int sl, pc;
    region_piece(region, wid, j, sl, pc);
    const int ny = (d.yx[j] >> 16) + kh * p.dy;
    const int nx = (int)(short)(d.yx[j] & 0xffff) + kw * p.dx;
    const int iy = ny >> p.uy, ix = nx >> p.ux;
    const bool ok = kt_ok && ((ny & my) | (nx & mx)) == 0 && (unsigned)iy < (unsigned)p.H &&
                    (unsigned)ix < (unsigned)p.W;
    const unsigned vo = ok ? (unsigned)(d.nb[j] + (iy * p.W + ix) * p.Cc + c0) * 2u : OOB;
    char* dst = stage_opnd + sl * 8192 + pc * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)dst, 16, vo, 0, 0, 0);
  }
}

// Fragment (16 mn x 32 k, MFMA operand layout: lane l holds X[mn = l&15][k = 8(l>>4) + j])
// of 32-mn block `u` (0..7), 16-row half i (0/1), k-step kk (0/1).
__device__ __forceinline__ bf16x8 frag_kmaj(const char* opnd, int u, int i, int kk, int lane) {
  const int row = 16 * i + (lane & 15);
  const int ch = (4 * kk + (lane >> 4)) ^ ((row >> 1) & 7);
  return *reinterpret_cast<const bf16x8*>(opnd + u * 4096 + row * 128 + ch * 16);
}

// MN-major fragments use the hardware transpose read.  It is issued by inline asm:
// hipcc cannot prove the ds_read_b64_tr_b16 builtin does not alias the in-flight
// LDS-DMA and puts an `s_waitcnt vmcnt(0)` in front of it, draining the whole
// prefetch pipeline every k-tile.  The asm destinations are then fenced by a
// wait statement that names them ("+v"), so nothing reads them before they land
// (guide §5.7 item 1, form ii).  LDS reads complete in order, so hipcc's own
// counted lgkmcnt waits for the K-major reads stay conservative-correct.
__device__ __forceinline__ unsigned lds_addr(const char* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

template <bool KMAJ>
struct Frag;

template <>
struct Frag<true> {
  bf16x8 v;
  __device__ __forceinline__ void load(const char* opnd, int u, int i, int kk, int lane) {
    v = frag_kmaj(opnd, u, i, kk, lane);
  }
  __device__ __forceinline__ void wait() {}
  __device__ __forceinline__ bf16x8 get() const { return v; }
};

template <>
struct Frag<false> {
  s16x4 x, y;
  __device__ __forceinline__ void load(const char* opnd, int u, int i, int kk, int lane) {
    const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
    const int k0 = 32 * kk + 8 * g + q;
    const int ch = (4 * (u & 1) + 2 * i + (p >> 1)) ^ mn_swz(k0);
    const unsigned a = lds_addr(opnd + (u >> 1) * 8192 + k0 * 128 + ch * 16 + 8 * (p & 1));
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(x) : "v"(a));
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:512" : "=v"(y) : "v"(a));
  }
  __device__ __forceinline__ void wait() { asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(x), "+v"(y)); }
  __device__ __forceinline__ bf16x8 get() const {
    i16x8 v = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
};

__device__ __forceinline__ void wait_vm4() { asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); }
__device__ __forceinline__ void wait_vm6() { asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); }
__device__ __forceinline__ void wait_vm8() { asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); }
__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// inclusive prefix sum inside each 16-lane DPP row: lane 16g + 15 ends with the row total
__device__ __forceinline__ float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x111, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x112, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x114, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x118, 0xf, 0xf, true));
  return v;
}

// Bijective XCD-aware remap: blocks that share an XCD (bid % 8) get a contiguous
// range of tile ids (guide §5 "XCD swizzle must be bijective").
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

#define WAIT_FRAGS(F, NI)                    \
  _Pragma("unroll") for (int i_ = 0; i_ < NI; ++i_) \
    _Pragma("unroll") for (int k_ = 0; k_ < 2; ++k_) F[i_][k_].wait();

// PF_IN_CLUSTER: schedule variant.  false = every fragment is read in a load
// section (phase 1 reads A rows 0-63 and B cols 0-31, phase 2 B cols 32-63, phase 3
// A rows 64-127); true = only B cols 0-31 are read in a load section, the rest are
// prefetched inside the preceding MFMA cluster (A double-buffered).  Measured
// (profiles/r2_gemm_v4_sched_ab.jsonl): the prefetch schedule wins ~5 % when both
// operands take transposed reads (24 tr_b16 in one phase-1 load section
// otherwise), and loses 2-5 % when an operand is K-major.
// One 64x32 quadrant of the non-prefetch schedule: 8 (i, j) accumulators over the
// two 32-k halves of the k-tile.  bf16: two v_mfma_f32_16x16x32_bf16 per (i, j),
// kk-outer so each accumulator has 7 independent MFMAs between its two updates.
// F8 (fp8 e4m3 operands, a "k unit" = 2 fp8 bytes): the two 16-B halves of a lane
// are one 32-byte operand of ONE block-scaled v_mfma_scale_f32_16x16x128_f8f6f4
// (unit E8M0 scales; the per-row / per-column fp32 scales are applied in the
// epilogue) -- the same cycles as the two bf16 MFMAs for twice the k.  A and B are
// both read by the K-major fragment loads, so the lane -> k permutation is common
// to both operands and the products pair up correctly.
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));

template <bool F8, class FA, class FB>
__device__ __forceinline__ void quad_mma(f32x4 (&acc)[8][4], const FA (&fa)[4][2], const FB (&fb)[2][2], int I0,
                                         int J0) {
  if constexpr (F8) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const i32x4 a0 = __builtin_bit_cast(i32x4, fa[i][0].get()), a1 = __builtin_bit_cast(i32x4, fa[i][1].get());
        const i32x4 b0 = __builtin_bit_cast(i32x4, fb[j][0].get()), b1 = __builtin_bit_cast(i32x4, fb[j][1].get());
        const i32x8 av = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
        const i32x8 bv = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
        acc[I0 + i][J0 + j] =
            __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bv, av, acc[I0 + i][J0 + j], 0, 0, 0, 127, 0, 127);
      }
  } else {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[I0 + i][J0 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j][kk].get(), fa[i][kk].get(), acc[I0 + i][J0 + j], 0, 0, 0);
  }
}

template <bool AK, bool BK, bool OUTF32, bool PF_IN_CLUSTER, bool KFULL, bool GA = false, bool F8 = false, int GM = 0,
          bool BNB = false, int EPI = 0>
__global__ __launch_bounds__(NT) void gemm_kernel(Params p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;

  long bz = blockIdx.y;
  int vb0 = blockIdx.x;  // this block's first tile (within its batch / group)
  if constexpr (GM == 1) {
    // grouped rows: flat tile v = (global tile row q, tile column) with q looked up in
    // the routing's tile table (grp_tiles[q] = group << 16 | tile row within it, -1
    // past the end), so the grid is sized from the total row count alone and the
    // host never needs the group sizes.  One tile per block.
    const int q = blockIdx.x / p.tiles_n;
    const int e = p.grp_tiles[q];
    if (e < 0) return;
    bz = e >> 16;
    vb0 = (e & 0xffff) * p.tiles_n + (blockIdx.x - q * p.tiles_n);  // row-major local tile
  }
  // per-group state (GM == 1 switches groups between persistent tiles)
  int Mb, Kb, tiles_m, nwg;
  long c_row0;
  __amdgpu_buffer_rsrc_t rsA, rsB;
  auto set_group = [&](long g) {
    Mb = p.M;  // rows of this batch / group
    Kb = p.k_total ? min(p.K, p.k_total - (int)g * p.K) : p.K;  // valid depth of this batch
    long a_off = g * p.sA, b_off = g * p.sB;
    c_row0 = 0;
    if constexpr (GM != 0) {  // grouped: this group's row range (see Params::grp)
      const int r0 = p.grp[g], r1 = p.grp[g + 1];
      if constexpr (GM == 1) {
        Mb = r1 - r0;
        a_off = (long)r0 * p.lda;
        c_row0 = r0;
      } else if constexpr (AK && BK) {
        // K-major operands (token-contiguous X^T / dY^T images): the group's k range
        // is a column range; fp8 counts k in units of 2 bytes
        constexpr int sh = F8 ? 1 : 0;
        Kb = (r1 - r0) >> sh;
        a_off = r0 >> sh;
        b_off = r0 >> sh;
      } else {
        Kb = r1 - r0;
        a_off = (long)r0 * p.lda;
        b_off = (long)r0 * p.ldb;
      }
    }
    tiles_m = (Mb + BM - 1) / BM;
    nwg = tiles_m * p.tiles_n;
    const char* Ab = (const char*)p.A + a_off * 2;
    const char* Bb = (const char*)p.B + b_off * 2;
    // descriptors over this batch's whole operand (host guarantees < 4 GiB)
    // (an empty group, Kb == 0, gets a zero-size range: every load returns 0)
    const unsigned a_bytes = GA ? (unsigned)((long)(p.M / (p.OH * p.OW)) * p.H * p.W * p.Cc * 2)
                           : Kb <= 0 ? 0u
                           : AK ? (unsigned)(((long)(Mb - 1) * p.lda + Kb) * 2)
                                : (unsigned)(((long)(Kb - 1) * p.lda + Mb) * 2);
    const unsigned b_bytes = Kb <= 0 ? 0u
                           : BK ? (unsigned)(((long)(p.N - 1) * p.ldb + Kb) * 2)
                                : (unsigned)(((long)(Kb - 1) * p.ldb + p.N) * 2);
    rsA = __builtin_amdgcn_make_buffer_rsrc((void*)Ab, 0, a_bytes, 0x00020000);
    rsB = __builtin_amdgcn_make_buffer_rsrc((void*)Bb, 0, b_bytes, 0x00020000);
  };
  set_group(bz);
  if (Mb <= 0 || vb0 >= nwg) return;  // wave-uniform: nothing for this block
  // start-time stagger (experiment knob, 0 = off): blocks of a persistent grid run
  // identical tile sequences in lockstep, so every CU's epilogue hits HBM at once;
  // offsetting their starts spreads those bursts
  if (p.stagger > 0) {
    const int slot = (blockIdx.x >> 3) & 7;
    for (int i = 0; i < slot * p.stagger; ++i) __builtin_amdgcn_s_sleep(16);
  }
  // ---- persistent tiles: virtual block vb = blockIdx.x + i * gridDim.x; XCD remap
  // (gridDim.x is a multiple of 8 or covers every tile, so a block keeps its XCD
  // group), then bands of 8 tile-rows for L2 reuse
  auto tile_of = [&](int vb, int& tm0, int& tn0) {
    if constexpr (GM == 1) {
      tm0 = (vb / p.tiles_n) * BM;
      tn0 = (vb % p.tiles_n) * BN;
      return;
    }
    const int t = xcd_remap(vb, nwg);
    constexpr int BAND = 8;
    const int band = t / (BAND * p.tiles_n);
    const int m_in_band = min(BAND, tiles_m - band * BAND);
    const int tin = t - band * BAND * p.tiles_n;
    tm0 = (band * BAND + tin % m_in_band) * BM;
    tn0 = (tin / m_in_band) * BN;
  };

  // ---- DMA plans: A_FIRST / A_SEC 2 pieces each, B 4 pieces per wave
  DmaLane<2, KFULL> daf, das;
  GatherLane<2> gaf, gas;
  DmaLane<4, KFULL> db;
  auto plan = [&](int mm0, int nn0) {
    if constexpr (GA) {
      gather_plan<2>(gaf, A_FIRST, wid, lane, mm0, p);
      gather_plan<2>(gas, A_SEC, wid, lane, mm0, p);
    } else {
      dma_plan<AK, 2, KFULL>(daf, A_FIRST, 0, wid, lane, mm0, Mb, p.lda);
      dma_plan<AK, 2, KFULL>(das, A_SEC, 0, wid, lane, mm0, Mb, p.lda);
    }
    dma_plan<BK, 4, KFULL>(db, B_ALL, 0, wid, lane, nn0, p.N, p.ldb);
  };

  const int nk = (Kb + BKT - 1) / BKT;
  auto sA = [&](int kt) { return smem + (kt & 1) * STAGE; };
  auto sB = [&](int kt) { return smem + (kt & 1) * STAGE + OPND; };
#define DMA_AF(kt)                                                        \
  do {                                                                    \
    if constexpr (GA)                                                     \
      gather_issue<2>(gaf, rsA, sA(kt), A_FIRST, wid, (kt), p);           \
    else                                                                  \
      dma_issue<AK, 2, KFULL>(daf, rsA, sA(kt), A_FIRST, 0, wid, (kt), Kb, p.lda); \
  } while (0)
#define DMA_AS(kt)                                                        \
  do {                                                                    \
    if constexpr (GA)                                                     \
      gather_issue<2>(gas, rsA, sA(kt), A_SEC, wid, (kt), p);             \
    else                                                                  \
      dma_issue<AK, 2, KFULL>(das, rsA, sA(kt), A_SEC, 0, wid, (kt), Kb, p.lda); \
  } while (0)
#define DMA_B(kt) dma_issue<BK, 4, KFULL>(db, rsB, sB(kt), B_ALL, 0, wid, (kt), Kb, p.ldb)

  // ---- DMA issue order (the counted waits depend on it):
  //   A_first(0) B(0) A_sec(0) A_first(1) B(1); the loop at k-tile t issues
  //   A_sec(t+1) in phase 2, A_first(t+2) in phase 3, B(t+2) in phase 4.  A tile's
  //   k-tile 0 is issued before the previous tile's epilogue, so its latency hides
  //   under the epilogue (which stages C in LDS above stage 0).
  int vb = vb0, m0, n0;
  tile_of(vb, m0, n0);
  plan(m0, n0);
  DMA_AF(0);
  DMA_B(0);
  DMA_AS(0);
  bool first = true;
  for (;;) {
  DMA_AF(1);
  DMA_B(1);
  if (first) {
    wait_vm8();  // A_first(0), B(0) landed
  } else {
    wait_vm6();  // k-tile 0 and the previous epilogue's memory ops retired
  }
  bar();

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (!PF_IN_CLUSTER) {
    if (wr == 1) bar();  // stagger: group 1 runs one barrier behind group 0

    Frag<AK> fa[4][2];
    Frag<BK> fb0[2][2], fb1[2][2];
    const int ua0 = 4 * wr, ub0 = 2 * wc;  // 32-mn blocks of this wave

    for (int kt = 0; kt < nk; ++kt) {
      const char* A_ = sA(kt);
      const char* B_ = sB(kt);
      // ---------------- phase 1: quadrant (rows 0-63, cols 0-31)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) fa[i][kk].load(A_, ua0 + (i >> 1), i & 1, kk, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) fb0[i][kk].load(B_, ub0, i, kk, lane);
      bar();
      WAIT_FRAGS(fa, 4);
      WAIT_FRAGS(fb0, 2);
      __builtin_amdgcn_s_setprio(1);
      if constexpr (F8) {
        quad_mma<true>(acc, fa, fb0, 0, 0);
      } else {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb0[j][kk].get(), fa[i][kk].get(), acc[i][j], 0, 0, 0);
      }
      __builtin_amdgcn_s_setprio(0);
      bar();
      // ---------------- phase 2: quadrant (rows 0-63, cols 32-63)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) fb1[i][kk].load(B_, ub0 + 1, i, kk, lane);
      wait_vm6();  // A_sec(kt) landed (read in phase 3)
      DMA_AS(kt + 1);
      bar();
      WAIT_FRAGS(fb1, 2);
      __builtin_amdgcn_s_setprio(1);
      if constexpr (F8) {
        quad_mma<true>(acc, fa, fb1, 0, 2);
      } else {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc[i][2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb1[j][kk].get(), fa[i][kk].get(), acc[i][2 + j], 0, 0, 0);
      }
      __builtin_amdgcn_s_setprio(0);
      bar();
      // ---------------- phase 3: quadrant (rows 64-127, cols 32-63)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) fa[i][kk].load(A_, ua0 + 2 + (i >> 1), i & 1, kk, lane);
      DMA_AF(kt + 2);
      bar();
      WAIT_FRAGS(fa, 4);
      __builtin_amdgcn_s_setprio(1);
      if constexpr (F8) {
        quad_mma<true>(acc, fa, fb1, 4, 2);
      } else {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc[4 + i][2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb1[j][kk].get(), fa[i][kk].get(), acc[4 + i][2 + j], 0, 0, 0);
      }
      __builtin_amdgcn_s_setprio(0);
      bar();
      // ---------------- phase 4: quadrant (rows 64-127, cols 0-31)
      wait_vm4();  // A_first(kt+1), B(kt+1) landed (read in the next phase 1)
      DMA_B(kt + 2);
      bar();
      __builtin_amdgcn_s_setprio(1);
      if constexpr (F8) {
        quad_mma<true>(acc, fa, fb0, 4, 0);
      } else {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb0[j][kk].get(), fa[i][kk].get(), acc[4 + i][j], 0, 0, 0);
      }
      __builtin_amdgcn_s_setprio(0);
      bar();
    }
  } else {

    // Fragment registers: fx = A rows 0-63 (A_first), fy = A rows 64-127 (A_sec),
    // fb0 / fb1 = B cols 0-31 / 32-63 of the wave.  Only fb0 is read in a load
    // section; fb1, fy and the next k-tile's fx are prefetched INSIDE the MFMA
    // clusters (one read per 2-4 MFMAs), into registers that cluster does not use.
    Frag<AK> fx[4][2], fy[4][2];
    Frag<BK> fb0[2][2], fb1[2][2];
    const int ua0 = 4 * wr, ub0 = 2 * wc;  // 32-mn blocks of this wave
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) fx[i][kk].load(sA(0), ua0 + (i >> 1), i & 1, kk, lane);
    if (wr == 1) bar();  // stagger: group 1 runs one barrier behind group 0

  // one 64x32 quadrant: 16 MFMAs (kk, i, j order); after MFMA q issue prefetch q/STEP
  #define QUAD(FA, FB, I0, J0, PF, STEP)                                                          \
    _Pragma("unroll") for (int q_ = 0; q_ < 16; ++q_) {                                          \
      const int kk_ = q_ >> 3, i_ = (q_ >> 1) & 3, j_ = q_ & 1;                                  \
      acc[I0 + i_][J0 + j_] =                                                                    \
          __builtin_amdgcn_mfma_f32_16x16x32_bf16(FB[j_][kk_].get(), FA[i_][kk_].get(), acc[I0 + i_][J0 + j_], 0, 0, 0); \
      if ((q_ % STEP) == STEP - 1) { PF(q_ / STEP); }                                            \
    }
  #define NOPF(x) \
    do {          \
    } while (0)

    for (int kt = 0; kt < nk; ++kt) {
      const char* A_ = sA(kt);
      const char* B_ = sB(kt);
      const char* An = sA(kt + 1);
      // ---------------- phase 1: quadrant (rows 0-63, cols 0-31); prefetch B cols 32-63
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) fb0[i][kk].load(B_, ub0, i, kk, lane);
      wait_vm6();  // A_sec(kt) landed (prefetched in phase 2)
      bar();
      WAIT_FRAGS(fx, 4);
      WAIT_FRAGS(fb0, 2);
      __builtin_amdgcn_s_setprio(1);
  #define PF1(f) fb1[(f) >> 1][(f) & 1].load(B_, ub0 + 1, (f) >> 1, (f) & 1, lane)
      QUAD(fx, fb0, 0, 0, PF1, 4)
  #undef PF1
      __builtin_amdgcn_s_setprio(0);
      bar();
      // ---------------- phase 2: quadrant (rows 0-63, cols 32-63); prefetch A rows 64-127
      DMA_AS(kt + 1);
      bar();
      WAIT_FRAGS(fb1, 2);
      __builtin_amdgcn_s_setprio(1);
  #define PF2(f) fy[(f) >> 1][(f) & 1].load(A_, ua0 + 2 + ((f) >> 2), ((f) >> 1) & 1, (f) & 1, lane)
      QUAD(fx, fb1, 0, 2, PF2, 2)
  #undef PF2
      __builtin_amdgcn_s_setprio(0);
      bar();
      // ---------------- phase 3: quadrant (rows 64-127, cols 32-63)
      wait_vm6();  // A_first(kt+1) landed (prefetched in phase 4)
      DMA_AF(kt + 2);
      bar();
      WAIT_FRAGS(fy, 4);
      __builtin_amdgcn_s_setprio(1);
      QUAD(fy, fb1, 4, 2, NOPF, 16)
      __builtin_amdgcn_s_setprio(0);
      bar();
      // ---------------- phase 4: quadrant (rows 64-127, cols 0-31); prefetch next A rows 0-63
      wait_vm4();  // B(kt+1) landed (read in the next phase 1)
      DMA_B(kt + 2);
      bar();
      __builtin_amdgcn_s_setprio(1);
  #define PF4(f) fx[(f) >> 1][(f) & 1].load(An, ua0 + ((f) >> 2), ((f) >> 1) & 1, (f) & 1, lane)
      QUAD(fy, fb0, 4, 0, PF4, 2)
  #undef PF4
      __builtin_amdgcn_s_setprio(0);
      bar();
    }
    WAIT_FRAGS(fx, 4);  // the last (unused) prefetch must land before LDS is reused
  #undef QUAD
  #undef NOPF
  }
  if (wr == 0) bar();  // match group 1's extra barrier
  wait_vm0();          // drain the zero-filling DMAs past the last k-tile (they write LDS)
  __builtin_amdgcn_s_barrier();  // every wave drained its DMAs: LDS is free

  // next tile's k-tile 0 (stage 0) goes out now and lands under this epilogue
  // the epilogue below writes THIS tile; the next tile may belong to another group
  const int eMb = Mb;
  const long erow0 = c_row0, ebz = bz;
  const int vb_next = vb + (int)gridDim.x;
  const bool has_next = GM != 1 && vb_next < nwg;
  int m0n = 0, n0n = 0;
  if (has_next) {
    tile_of(vb_next, m0n, n0n);
    plan(m0n, n0n);
    DMA_AF(0);
    DMA_B(0);
    DMA_AS(0);
  }

  // ---- epilogue, staged through LDS (above stage 0) so every global access is a
  // full-line 16-B vector (per-lane fragments would store 32 B per row and 16 rows
  // per instruction; the store tail is issue-bound, guide T21).  Lane holds
  // C[m = .. + (l&15)][n = .. + 4(l>>4) + r], r = 0..3.  bf16: 2 passes of 128 rows
  // (512 B + 16 B pad: conflict-free ds_write_b64), one per wave group; fp32: 4
  // passes of 64 rows (1024 + 16 B).
  {
  char* stg = smem + STAGE;
  const long cz = ebz * p.sC;
  constexpr int ROWB = OUTF32 ? 1040 : 528;
  const int ml = lane & 15;
  const int nl = 64 * wc + 4 * (lane >> 4);
  float bv[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[j][r] = 0.f;
  float sbv[4][4];
  if constexpr (F8) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + nl + 16 * j + r;
        sbv[j][r] = n < p.N ? p.sb[ebz * p.sbs + n] : 0.f;
      }
  }
  if (p.bias) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + nl + 16 * j;
      if (n < p.N) {
        if (OUTF32) {
          const f32x4 b4 = *reinterpret_cast<const f32x4*>((const float*)p.bias + n);
#pragma unroll
          for (int r = 0; r < 4; ++r) bv[j][r] = b4[r];
        } else {
          const u16x4 b4 = *reinterpret_cast<const u16x4*>((const u16*)p.bias + n);
#pragma unroll
          for (int r = 0; r < 4; ++r) bv[j][r] = bf2f(b4[r]);
        }
      }
    }
  }
  // pass ps stages m-tiles [PI*ps, PI*ps + PI) of BOTH wave groups, so each pass
  // retires a slice of every wave's accumulators (register pressure falls as it goes)
  constexpr int PASSES = OUTF32 ? 4 : 2;
  constexpr int PI = 8 / PASSES;           // 16-row m-tiles per group per pass
  constexpr int GR = 16 * PI;              // staged rows per group per pass
  constexpr int CPR = OUTF32 ? 64 : 32;  // 16-B chunks per 256-wide row
  constexpr int RPI = NT / CPR;          // rows per iteration
  constexpr int NIT = 2 * GR / RPI;      // store iterations per pass
  const bool acc_rd = p.accumulate && !(OUTF32 && p.atomic);
  // C descriptor based at this tile's first element (host: 256 rows of ldc fit in
  // 32-bit offsets).  Store iteration `it` of pass `ps` covers tile row
  // crow(it, ps) + tid / CPR (a compile-time row plus a lane row) and 16-B chunk
  // tid % CPR; its byte offset is c_base + crow * row_bytes, or OOB (load 0 /
  // store dropped) past M or N.  All scalars but c_base and the row test.
  constexpr int ESZ = OUTF32 ? 4 : 2;
  const __amdgpu_buffer_rsrc_t rsC = __builtin_amdgcn_make_buffer_rsrc(
      (char*)p.C + (cz + (erow0 + m0) * p.ldc + n0) * ESZ, 0, (int)OOB, 0x00020000);
  const unsigned row_bytes = (unsigned)p.ldc * ESZ;
  const int c_row = tid / CPR;
  const int rows_left = eMb - m0;  // rows of this tile inside M
  const bool c_colok = n0 + (tid % CPR) * (OUTF32 ? 4 : 8) < p.N;
  const unsigned c_base = (unsigned)c_row * row_bytes + (unsigned)((tid % CPR) * 16);
#define C_OFF(it, ps)                                                                          \
  ({                                                                                           \
    const int rr0_ = (it) * RPI;                                                           \
    const int crow_ = (rr0_ < GR ? rr0_ : 128 + rr0_ - GR) + GR * (ps);                    \
    (c_colok && c_row + crow_ < rows_left) ? c_base + (unsigned)crow_ * row_bytes : OOB;       \
  })
  // GA conv kernels with p.part: BatchNorm statistics of the stored (rounded) output,
  // accumulated from the staged 16-B chunks this thread stores (8 channels, fixed per
  // thread), then reduced over the 16 threads of a channel chunk through LDS
  const bool stats = GA && !OUTF32 && p.part != nullptr;
  const bool bstats = BNB && stats;  // BNB kernels: BN backward statistics (p.bs)
  float st1[8], st2[8], shc[8], msc[8], msf[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    st1[e] = st2[e] = 0.f;
    const int n = n0 + (tid % CPR) * 8 + e;
    shc[e] = msc[e] = msf[e] = 0.f;
    if (bstats && n < p.N)
      bn_bwd_coef(p.bs, n, shc[e], msc[e], msf[e]);
    else if (stats && p.shift && n < p.N)
      shc[e] = p.shift[n];
  }
  const long tile_off = (cz + (erow0 + m0) * p.ldc + n0) * 2;
  const __amdgpu_buffer_rsrc_t rsX = __builtin_amdgcn_make_buffer_rsrc(
      (char*)p.bs.x + (bstats ? tile_off : 0), 0, (int)OOB, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsY = __builtin_amdgcn_make_buffer_rsrc(
      (char*)p.bs.y + (bstats && p.bs.y ? tile_off : 0), 0, (int)OOB, 0x00020000);
#pragma unroll
  for (int ps = 0; ps < PASSES; ++ps) {
    // (a) fragments -> LDS (staged row = GR * wr + 16 * ii + ml)
#pragma unroll
    for (int ii = 0; ii < PI; ++ii)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = PI * ps + ii;
        char* dst = stg + (GR * wr + 16 * ii + ml) * ROWB + (nl + 16 * j) * (OUTF32 ? 4 : 2);
        if constexpr (F8) {
          const int m = m0 + 128 * wr + 16 * i + ml;
          const float sam = m < eMb ? p.alpha * p.sa[ebz * p.sas + erow0 + m] : 0.f;
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] *= sam * sbv[j][r];
        }
        if (OUTF32) {
          f32x4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = p.alpha * acc[i][j][r] + bv[j][r];
          *reinterpret_cast<f32x4*>(dst) = v;
        } else {
          uint2 w;
          w.x = pack2bf(p.alpha * acc[i][j][0] + bv[j][0], p.alpha * acc[i][j][1] + bv[j][1]);
          w.y = pack2bf(p.alpha * acc[i][j][2] + bv[j][2], p.alpha * acc[i][j][3] + bv[j][3]);
          *reinterpret_cast<uint2*>(dst) = w;
        }
      }
    __syncthreads();
    if (OUTF32 && p.atomic) {
      // split-K: one float per lane, 64 consecutive floats (256 B) per wave-instruction
      // (guide Guideline 12: atomic wave-instructions shaped as contiguous 256 B)
#pragma unroll 4
      for (int it = 0; it < 2 * GR * 256 / NT; ++it) {
        const int idx = it * NT + tid;
        const int rr = idx >> 8, cc = idx & 255;
        const int m = m0 + 128 * (rr / GR) + GR * ps + rr % GR;
        const int n = n0 + cc;
        const float v = *reinterpret_cast<const float*>(stg + rr * ROWB + cc * 4);
        if (m < eMb && n < p.N) atomicAdd((float*)p.C + cz + (erow0 + m) * p.ldc + n, v);
      }
      __syncthreads();
      continue;
    }
    // (b) LDS rows -> global, 16 B per lane, consecutive lanes along a row, in
    // halves of HB iterations.  C += : a half's old C values are loaded together
    // before its stores, so a pass costs two load round trips, not one per store
    // (vmcnt retires in issue order: a load issued after a store waits for it).
    // Loads and stores are buffer ops on the per-tile descriptor with masked lanes
    // sent out of range (load 0 / store dropped): uniform control flow, so hipcc
    // counts its vmcnt waits instead of falling back to vmcnt(0) at every store.
    constexpr int HB = (F8 || BNB || EPI == 3) ? 2 : NIT / 2;  // F8 / BNB / RoPE epilogues hold more per chunk
#pragma unroll 1
    for (int h = 0; h < (EPI == 2 ? 0 : NIT); h += HB) {
      u32x4 cold[HB];
      if (acc_rd) {
#pragma unroll
        for (int u = 0; u < HB; ++u) cold[u] = __builtin_amdgcn_raw_buffer_load_b128(rsC, C_OFF(h + u, ps), 0, 0);
      }
      u32x4 xo[HB], yo[HB];
      if constexpr (BNB && GA && !OUTF32) {
        if (bstats) {
#pragma unroll
          for (int u = 0; u < HB; ++u) {
            xo[u] = __builtin_amdgcn_raw_buffer_load_b128(rsX, C_OFF(h + u, ps), 0, 0);
            yo[u] = p.bs.y ? __builtin_amdgcn_raw_buffer_load_b128(rsY, C_OFF(h + u, ps), 0, 0) : u32x4{0, 0, 0, 0};
          }
        }
      }
#pragma unroll
      for (int u = 0; u < HB; ++u) {
        const int it = h + u;
        const int rr = it * RPI + tid / CPR, ch = tid % CPR;
        const f32x4 v = *reinterpret_cast<const f32x4*>(stg + rr * ROWB + ch * 16);
        u32x4 w = __builtin_bit_cast(u32x4, v);
        if constexpr (GA && !OUTF32) {
          if (stats && !bstats && C_OFF(it, ps) != OOB) {
            const u16x8 c = __builtin_bit_cast(u16x8, v);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float d = bf2f(c[e]) - shc[e];
              st1[e] += d;
              st2[e] += d * d;
            }
          }
        }
        if (acc_rd) {
          if constexpr (OUTF32) {
            w = __builtin_bit_cast(u32x4, v + __builtin_bit_cast(f32x4, cold[u]));
          } else {
            const u16x8 o = __builtin_bit_cast(u16x8, cold[u]);
            const u16x8 c = __builtin_bit_cast(u16x8, v);
            u16x8 r;
#pragma unroll
            for (int e = 0; e < 8; ++e) r[e] = f2bf(bf2f(c[e]) + bf2f(o[e]));
            w = __builtin_bit_cast(u32x4, r);
          }
        }
        if constexpr (EPI == 3) {
          // neox rotation of the q / k heads: this chunk (8 of a head's 128 columns)
          // and its partner 64 columns away, both staged in LDS
          const int gcol = n0 + ch * 8;
          if (gcol < p.rope_cols && C_OFF(it, ps) != OOB) {
            const u16x8 xs = __builtin_bit_cast(u16x8, v);
            const u16x8 xp = *reinterpret_cast<const u16x8*>(stg + rr * ROWB + (ch ^ 8) * 16);
            const int rr0_ = it * RPI;
            const int trow = (rr0_ < GR ? rr0_ : 128 + rr0_ - GR) + GR * ps + tid / CPR;
            const long pos = (erow0 + m0 + trow) % p.rope_S;
            const float* cp = p.cosT + pos * 64 + 8 * (ch & 7);
            const float* sp = p.sinT + pos * 64 + 8 * (ch & 7);
            const f32x4 c0 = *reinterpret_cast<const f32x4*>(cp), c1 = *reinterpret_cast<const f32x4*>(cp + 4);
            const f32x4 s0 = *reinterpret_cast<const f32x4*>(sp), s1 = *reinterpret_cast<const f32x4*>(sp + 4);
            const float sg = (ch & 8) ? 1.f : -1.f;
            u16x8 r;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float co = e < 4 ? c0[e] : c1[e - 4], si = e < 4 ? s0[e] : s1[e - 4];
              r[e] = f2bf(bf2f(xs[e]) * co + sg * bf2f(xp[e]) * si);
            }
            w = __builtin_bit_cast(u32x4, r);
          }
        }
        if constexpr (BNB && GA && !OUTF32) {
          if (bstats && C_OFF(it, ps) != OOB) {
            const u16x8 c = __builtin_bit_cast(u16x8, w);
            const u16x8 xb = __builtin_bit_cast(u16x8, xo[u]);
            const u16x8 yb = __builtin_bit_cast(u16x8, yo[u]);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float xv = bf2f(xb[e]);
              const bool keep = !p.bs.relu || (p.bs.y ? bf2f(yb[e]) > 0.f : fmaf(xv, msc[e], msf[e]) > 0.f);
              const float gv = keep ? bf2f(c[e]) : 0.f;
              st1[e] += gv;
              st2[e] += gv * (xv - shc[e]);
            }
          }
        }
        __builtin_amdgcn_raw_buffer_store_b128(w, rsC, C_OFF(it, ps), 0, 0);
      }
    }
    if constexpr (EPI == 1) {
      // (c) h = silu(gate) * up: 16 chunks of 8 h columns per staged row
      const __amdgpu_buffer_rsrc_t rsH = __builtin_amdgcn_make_buffer_rsrc(
          (char*)p.aux + ((erow0 + m0) * p.ldaux + n0 / 2) * 2, 0, (int)OOB, 0x00020000);
#pragma unroll 2
      for (int it = 0; it < 2 * GR * 16 / NT; ++it) {
        const int idx = it * NT + tid, rr = idx >> 4, k = idx & 15;
        const int trow = (rr < GR ? rr : 128 + rr - GR) + GR * ps;
        const int gch = 4 * (k >> 1) + (k & 1);
        const u16x8 g = *reinterpret_cast<const u16x8*>(stg + rr * ROWB + gch * 16);
        const u16x8 u = *reinterpret_cast<const u16x8*>(stg + rr * ROWB + (gch + 2) * 16);
        u16x8 r;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float gv = bf2f(g[e]);
          r[e] = f2bf(gv / (1.f + __expf(-gv)) * bf2f(u[e]));
        }
        const bool ok = trow < rows_left && n0 / 2 + 8 * k < p.N / 2;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, r), rsH,
                                               ok ? (unsigned)trow * (unsigned)p.ldaux * 2u + (unsigned)k * 16u : OOB,
                                               0, 0);
      }
    }
    if constexpr (EPI == 2) {
      // (c) SwiGLU backward from the staged da tile: for each 8-column da chunk k,
      // gate / up of the same columns sit at 32 (k >> 1) + 8 (k & 1) (+16) of the
      // 512-wide gu / dgu tile; four chunks per thread have their gu loads in flight
      const __amdgpu_buffer_rsrc_t rsG = __builtin_amdgcn_make_buffer_rsrc(
          (char*)p.aux + ((erow0 + m0) * p.ldaux + 2 * (long)n0) * 2, 0, (int)OOB, 0x00020000);
      const __amdgpu_buffer_rsrc_t rsD = __builtin_amdgcn_make_buffer_rsrc(
          (char*)p.C + (cz + (erow0 + m0) * p.ldc + 2 * (long)n0) * 2, 0, (int)OOB, 0x00020000);
#pragma unroll 1
      for (int h0 = 0; h0 < 2 * GR * 32 / NT; h0 += 4) {
        u32x4 gv[4], uv[4];
        unsigned og[4], od[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int idx = (h0 + u) * NT + tid, rr = idx >> 5, k = idx & 31;
          const int trow = (rr < GR ? rr : 128 + rr - GR) + GR * ps;
          const unsigned col = 32u * (unsigned)(k >> 1) + 8u * (unsigned)(k & 1);
          const bool ok = trow < rows_left && n0 + 8 * k < p.N;
          og[u] = ok ? (unsigned)trow * (unsigned)p.ldaux * 2u + col * 2u : OOB;
          od[u] = ok ? (unsigned)trow * (unsigned)p.ldc * 2u + col * 2u : OOB;
          gv[u] = __builtin_amdgcn_raw_buffer_load_b128(rsG, og[u], 0, 0);
          uv[u] = __builtin_amdgcn_raw_buffer_load_b128(rsG, ok ? og[u] + 32u : OOB, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int idx = (h0 + u) * NT + tid, rr = idx >> 5, k = idx & 31;
          const u16x8 d = *reinterpret_cast<const u16x8*>(stg + rr * ROWB + k * 16);
          const u16x8 g = __builtin_bit_cast(u16x8, gv[u]), up = __builtin_bit_cast(u16x8, uv[u]);
          u16x8 dg, du;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float gf = bf2f(g[e]), uf = bf2f(up[e]), df = bf2f(d[e]);
            const float sg = 1.f / (1.f + __expf(-gf));
            du[e] = f2bf(df * gf * sg);
            dg[e] = f2bf(df * uf * sg * (1.f + gf * (1.f - sg)));
          }
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, dg), rsD, od[u], 0, 0);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, du), rsD, od[u] == OOB ? OOB : od[u] + 32u, 0, 0);
        }
      }
    }
    __syncthreads();  // staging reads done (next pass / next tile's DMA into stage 1)
  }
  if (stats) {
    float* red = reinterpret_cast<float*>(stg);  // [NT / CPR row groups][256 columns][2]
    const int rg = tid / CPR, cb = (tid % CPR) * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[(rg * 256 + cb + e) * 2] = st1[e];
      red[(rg * 256 + cb + e) * 2 + 1] = st2[e];
    }
    __syncthreads();
    if (tid < 256 && n0 + tid < p.N) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int g = 0; g < NT / CPR; ++g) {
        a += red[(g * 256 + tid) * 2];
        b += red[(g * 256 + tid) * 2 + 1];
      }
      const long row = (long)(m0 / BM) * 2;
      p.part[row * p.N + n0 + tid] = a;
      p.part[(row + 1) * p.N + n0 + tid] = b;
    }
    __syncthreads();  // reduction reads done before the next tile's DMA into stage 1
  }
  }
#undef C_OFF
  if (!has_next) break;
  vb = vb_next;
  m0 = m0n;
  n0 = n0n;
  first = false;
  }  // persistent tile loop
#undef DMA_AF
#undef DMA_AS
#undef DMA_B
}

// ---------------------------------------------------------------------------------
// Weight-gradient GEMM with an MN-major operand, one wave per SIMD:
//   C (fp32, =|+=) alpha * sum_k A(m, k) B(n, k),  K % 64 == 0, no bias / batch.
// The two-wave kernel above owns a 128 x 64 output per wave; with an MN-major operand
// every 16 x 32 fragment costs two ds_read_b64_tr_b16, so its LDS-issue share doubles
// and the matrix pipe falls to ~60 % busy (profiles/r4_gemm_forms_pmc.md).  Here 256
// threads = 4 waves (2 M x 2 N) each own 128 x 128: 64 f32x4 accumulators (256
// registers, the AGPR half of the 512-entry file that one wave per SIMD has), and
// every fragment read feeds 8 MFMAs instead of 4-8, so a k32 step is 16 fragment
// loads under 64 MFMAs (1024 matrix cycles).  With no second wave on the SIMD to
// hide LDS latency, the next k32 step's fragments are read INSIDE the current
// step's MFMA stream (double-buffered registers).  Same LDS image, swizzles, LDS-DMA
// and XCD tile order as the kernel above; one barrier per 64-deep k-tile:
//   [step kk0 of tile t | reads kk1 of t] wait, barrier, DMA(t+2) into t's stage,
//   [step kk1 of t | reads kk0 of t+1]
// so each DMA lands under two k32 steps (2048 matrix cycles).
constexpr int NT1 = 256;

// Fragment registers of the one-wave kernel.  Every read is an asm ds_read with an
// IMMEDIATE offset from one of a few per-lane base addresses (the swizzle depends on
// the lane only), so no per-fragment address is ever materialised -- hipcc would
// otherwise hoist one loop-invariant address per fragment (64+ VGPRs) and spill.
//  K-major: base[kk] = slab row (l & 15), chunk (4 kk + (l >> 4)) ^ ((l & 15) >> 1);
//           fragment f (32-mn block f / 2, half f % 2) at + 4096 (f / 2) + 2048 (f % 2)
//  MN-major: base[c] (c = f % 4) = k row 8 (l >> 4) + ((l & 15) >> 2), chunk
//           (2 c ^ swz(k)) + ((l & 3) >> 1), + 8 (l & 1); + 8192 (f / 4) + 4096 kk
template <bool KMAJ>
struct F1w {
  bf16x8 v;
  s16x4 x, y;
  // off must fold to a constant (unrolled loops): it becomes the instruction's offset
  __device__ __forceinline__ void load(unsigned a, int off) {
    if constexpr (KMAJ) {
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(off));
    } else {
      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(x) : "v"(a), "i"(off));
      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(y) : "v"(a), "i"(off + 512));
    }
  }
  __device__ __forceinline__ void wait() {
    if constexpr (KMAJ) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v));
    else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(x), "+v"(y));
  }
  __device__ __forceinline__ bf16x8 get() const {
    if constexpr (KMAJ) {
      return v;
    } else {
      i16x8 t = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
      return __builtin_bit_cast(bf16x8, t);
    }
  }
};

// per-lane base addresses of one operand (stage 0) for this wave's 128-wide block
// starting at 32-mn block `u0` (a multiple of 4); [kk] for K-major, [c] for MN-major
template <bool KMAJ>
__device__ __forceinline__ void f1w_bases(unsigned (&b)[4], unsigned opnd, int u0, int lane) {
  if constexpr (KMAJ) {
    const int row = lane & 15;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = (4 * kk + (lane >> 4)) ^ ((row >> 1) & 7);
      b[kk] = opnd + (unsigned)(u0 * 4096 + row * 128 + ch * 16);
    }
    b[2] = b[3] = 0;
  } else {
    const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
    const int k0 = 8 * g + q;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int ch = ((2 * c) ^ mn_swz(k0)) + (pp >> 1);
      b[c] = opnd + (unsigned)((u0 >> 1) * 8192 + k0 * 128 + ch * 16 + 8 * (pp & 1));
    }
  }
}

// read fragment F (compile-time after unrolling) of k-half KK from bases b (+ stage)
#define F1W_LOAD(KMAJ, FR, b, F, KK)                                              \
  do {                                                                            \
    if constexpr (KMAJ)                                                           \
      FR.load(b[(KK)], 4096 * ((F) >> 1) + 2048 * ((F) & 1));            \
    else                                                                          \
      FR.load(b[(F) & 3], 8192 * ((F) >> 2) + 4096 * (KK));             \
  } while (0)

template <bool AK, bool BK>
__global__ __launch_bounds__(NT1) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm1w_kernel(Params p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const int M = p.M, N = p.N, K = p.K;
  const int tiles_m = p.tiles_m, nwg = tiles_m * p.tiles_n;
  // XCD-aware tile order, bands of 8 tile rows (as tile_of above)
  int m0, n0;
  {
    const int t = xcd_remap(blockIdx.x, nwg);
    constexpr int BAND = 8;
    const int band = t / (BAND * p.tiles_n);
    const int m_in_band = min(BAND, tiles_m - band * BAND);
    const int tin = t - band * BAND * p.tiles_n;
    m0 = (band * BAND + tin % m_in_band) * BM;
    n0 = (tin / m_in_band) * BN;
  }
  const unsigned a_bytes = AK ? (unsigned)(((long)(M - 1) * p.lda + K) * 2) : (unsigned)(((long)(K - 1) * p.lda + M) * 2);
  const unsigned b_bytes = BK ? (unsigned)(((long)(N - 1) * p.ldb + K) * 2) : (unsigned)(((long)(K - 1) * p.ldb + N) * 2);
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)p.A, 0, a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)p.B, 0, b_bytes, 0x00020000);
  // DMA plan: wave w fills slab w (64 mn x 64 k, 8 pieces of 1 KiB) of A and of B
  unsigned offA[8], offB[8];
#pragma unroll
  for (int pc = 0; pc < 8; ++pc) {
    int mn, k;
    dma_coords<AK>(wid, pc, lane, mn, k);
    int g = m0 + mn;
    offA[pc] = g >= M ? OOB : (AK ? (unsigned)(((long)g * p.lda + k) * 2) : (unsigned)(((long)k * p.lda + g) * 2));
    dma_coords<BK>(wid, pc, lane, mn, k);
    g = n0 + mn;
    offB[pc] = g >= N ? OOB : (BK ? (unsigned)(((long)g * p.ldb + k) * 2) : (unsigned)(((long)k * p.ldb + g) * 2));
  }
  const int nk = K / BKT;
  auto dma = [&](int kt) {
    char* st = smem + (kt & 1) * STAGE;
    const unsigned ka = AK ? (unsigned)(kt * BKT * 2) : (unsigned)((long)kt * BKT * p.lda * 2);
    const unsigned kb = BK ? (unsigned)(kt * BKT * 2) : (unsigned)((long)kt * BKT * p.ldb * 2);
#pragma unroll
    for (int pc = 0; pc < 8; ++pc)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (__attribute__((address_space(3))) void*)(st + wid * 8192 + pc * 1024),
                                               16, offA[pc] == OOB ? OOB : offA[pc] + ka, 0, 0, 0);
#pragma unroll
    for (int pc = 0; pc < 8; ++pc)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB,
                                               (__attribute__((address_space(3))) void*)(st + OPND + wid * 8192 + pc * 1024),
                                               16, offB[pc] == OOB ? OOB : offB[pc] + kb, 0, 0, 0);
  };

  // accumulators pinned to AGPRs for the whole tile (defined and read by asm with "a"
  // operands, as fa_bwd_split.hip): otherwise hipcc keeps them in VGPRs and spills
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      asm volatile("" : "=a"(acc[i][j]) : "0"(z));
    }
  // fragment f (0..7) of this wave: 32-mn block 4 w + f / 2, 16-row half f % 2
  F1w<AK> a0[8], a1[8];
  F1w<BK> b0[8], b1[8];
  unsigned baA[4], baB[4];
  const unsigned lds0 = lds_addr(smem);
  f1w_bases<AK>(baA, lds0, 4 * wr, lane);
  f1w_bases<BK>(baB, lds0 + OPND, 4 * wc, lane);

  dma(0);
  if (nk > 1) dma(1);
  if (nk > 1) {
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  } else {
    wait_vm0();
  }
  bar();
#pragma unroll
  for (int f = 0; f < 8; ++f) {
    F1W_LOAD(AK, a0[f], baA, f, 0);
    F1W_LOAD(BK, b0[f], baB, f, 0);
  }

  // one k32 step on (FA, FB): 16 groups of 4 MFMAs, with the 16 fragment reads of the
  // next step (bases NBA / NBB, k-half KK) spread over the first 12 groups
#define STEP1W(FA, FB, NA, NB, NBA, NBB, KK, DO)                                                     \
  _Pragma("unroll") for (int g_ = 0; g_ < 16; ++g_) {                                                 \
    const int i_ = g_ >> 1, j0_ = 4 * (g_ & 1);                                                       \
    /* the empty asm statements are ordered with the reads and pin each group of 4 */                  \
    /* MFMAs between them: the DAG scheduler places pure MFMAs anywhere otherwise */                   \
    asm volatile("" : "+a"(acc[i_][j0_]), "+a"(acc[i_][j0_ + 1]), "+a"(acc[i_][j0_ + 2]), "+a"(acc[i_][j0_ + 3])); \
    _Pragma("unroll") for (int j_ = j0_; j_ < j0_ + 4; ++j_)                                          \
      acc[i_][j_] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(FB[j_].get(), FA[i_].get(), acc[i_][j_], 0, 0, 0); \
    asm volatile("" : "+a"(acc[i_][j0_]), "+a"(acc[i_][j0_ + 1]), "+a"(acc[i_][j0_ + 2]), "+a"(acc[i_][j0_ + 3])); \
    /* read r goes out after group 3 r / 4: groups 12-15 (256 matrix cycles) cover */                  \
    /* the last read's latency before the next step waits for it */                                   \
    _Pragma("unroll") for (int r_ = 0; r_ < 16; ++r_) {                                               \
      if ((DO) && (3 * r_) / 4 == g_) {                                                               \
        if (r_ & 1)                                                                                   \
          F1W_LOAD(BK, NB[r_ >> 1], NBB, r_ >> 1, KK);                                                \
        else                                                                                          \
          F1W_LOAD(AK, NA[r_ >> 1], NBA, r_ >> 1, KK);                                                \
      }                                                                                               \
    }                                                                                                 \
  }

  for (int kt = 0; kt < nk; ++kt) {
    const unsigned so = (kt & 1) ? (unsigned)STAGE : 0u, sn = (unsigned)STAGE - so;
    unsigned cA[4], cB[4], nA[4], nB[4];  // this / the next stage's bases
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      cA[c] = baA[c] + so;
      cB[c] = baB[c] + so;
      nA[c] = baA[c] + sn;
      nB[c] = baB[c] + sn;
    }
    // ---- k32 step 0 of tile kt; reads of step 1 (same stage)
#pragma unroll
    for (int f = 0; f < 8; ++f) {
      a0[f].wait();
      b0[f].wait();
    }
    __builtin_amdgcn_s_setprio(1);
    STEP1W(a0, b0, a1, b1, cA, cB, 1, true)
    __builtin_amdgcn_s_setprio(0);
    // every wave's reads of stage kt done and DMA(kt+1) landed -> stage kt is free
#pragma unroll
    for (int f = 0; f < 8; ++f) {
      a1[f].wait();
      b1[f].wait();
    }
    wait_vm0();
    bar();
    if (kt + 2 < nk) dma(kt + 2);
    // ---- k32 step 1 of tile kt; reads of the next tile's step 0
    __builtin_amdgcn_s_setprio(1);
    // (the last tile reads the other stage too: stale, unused, and keeps the loop
    // body branch-free so the accumulators keep one register assignment)
    STEP1W(a1, b1, a0, b0, nA, nB, 0, true)
    __builtin_amdgcn_s_setprio(0);
  }
#pragma unroll
  for (int f = 0; f < 8; ++f) {
    a0[f].wait();
    b0[f].wait();
  }
#undef STEP1W
#undef F1W_LOAD

#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));
  // ---- epilogue: C (fp32) =|+= alpha * acc, straight from the registers.  Lane holds
  // C[m = 16 i + (l & 15)][n = 16 j + 4 (l >> 4) + r] of its 128 x 128; each 16-B
  // access is 4 consecutive n.  Per-tile descriptor, out-of-range lanes sent OOB.
  const __amdgpu_buffer_rsrc_t rsC =
      __builtin_amdgcn_make_buffer_rsrc((char*)p.C + ((long)m0 * p.ldc + n0) * 4, 0, (int)OOB, 0x00020000);
  const int ml = 128 * wr + (lane & 15), nl = 128 * wc + 4 * (lane >> 4);
  const unsigned rb = (unsigned)p.ldc * 4u;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = ml + 16 * i;
    unsigned off[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int n = nl + 16 * j;
      off[j] = (m0 + m < M && n0 + n < N) ? (unsigned)m * rb + (unsigned)n * 4u : OOB;
    }
    u32x4 old[8];
    if (p.accumulate) {
#pragma unroll
      for (int j = 0; j < 8; ++j) old[j] = __builtin_amdgcn_raw_buffer_load_b128(rsC, off[j], 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      f32x4 v = p.alpha * acc[i][j];
      if (p.accumulate) v += __builtin_bit_cast(f32x4, old[j]);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rsC, off[j], 0, 0);
    }
  }
}

// route fp32 weight-gradient GEMMs with an MN-major operand to gemm1w_kernel: OFF by
// default -- measured 0.75-0.85x of the two-wave kernel on every LLaMA dW shape
// (profiles/r6_gemm_dw_1wave_NEGATIVE.md); pa_gemm_set_dw1w(1) selects it
static int g_dw1w = 0;

template <bool AK, bool BK>
static int launch_1w(const Params& p0, hipStream_t st) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)gemm1w_kernel<AK, BK>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       2 * STAGE);
    if (e != hipSuccess) return (int)e;
    attr_set = true;
  }
  Params p = p0;
  p.tiles_m = (p.M + BM - 1) / BM;
  p.tiles_n = (p.N + BN - 1) / BN;
  hipLaunchKernelGGL((gemm1w_kernel<AK, BK>), dim3(p.tiles_m * p.tiles_n), dim3(NT1), 2 * STAGE, st, p);
  return (int)hipGetLastError();
}

static int g_sched = -1;     // -1: per-layout default; 0 / 1: force PF_IN_CLUSTER (A/B runs)
static int g_persistent = 1;  // 0: one tile per block (grid = tiles), for A/B runs
static int g_stagger = 1;     // start stagger units per block slot (profiles/r3_gemm_stagger_ab.jsonl: +0.7 % over the step GEMMs)

template <bool AK, bool BK, bool F32, bool PF, bool KFULL, bool GA = false, bool F8 = false, int GM = 0,
          bool BNB = false, int EPI = 0>
static int launch_v(const Params& p, int batch, hipStream_t st) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)gemm_kernel<AK, BK, F32, PF, KFULL, GA, F8, GM, BNB, EPI>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    if (e != hipSuccess) return (int)e;
    attr_set = true;
  }
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
    ncu = ncu / 8 * 8;  // keep gridDim.x a multiple of the XCD count
  }
  const int nwg = p.tiles_m * p.tiles_n;
  // persistent: one resident block per CU; grouped rows: one block per tile of the
  // flat schedule (tiles_m bounds the groups' tile rows), a single grid row
  const int grid = (GM == 1 || nwg < ncu || !g_persistent) ? nwg : ncu;
  Params pp = p;
  pp.stagger = grid == ncu ? g_stagger : 0;
  hipLaunchKernelGGL((gemm_kernel<AK, BK, F32, PF, KFULL, GA, F8, GM, BNB, EPI>), dim3(grid, GM == 1 ? 1 : batch), dim3(NT),
                     LDS_BYTES, st, pp);
  return (int)hipGetLastError();
}

// GM (grouped mode) is a template parameter so plain GEMMs carry no group state
// (registers): mode 1 needs a K-major A, mode 2 two MN-major operands.
template <bool AK, bool BK, bool F32, int GM>
static int launch_g(const Params& p, int batch, hipStream_t st) {
  if constexpr ((GM == 1 && !AK) || (GM == 2 && AK != BK)) {
    return -1;
  } else {
    const bool pf = g_sched == 1;  // measured: in-cluster prefetch loses on every form (profiles/r3_gemm_mn_forms.jsonl)
    if constexpr (GM != 2) {
      if (p.K % BKT == 0 && p.k_total % BKT == 0)  // every k-tile full: the k range check is wave-uniform
        return pf ? launch_v<AK, BK, F32, true, true, false, false, GM>(p, batch, st)
                  : launch_v<AK, BK, F32, false, true, false, false, GM>(p, batch, st);
    } else if constexpr (AK && BK) {
      // grouped-K over token images: every group's column range is a multiple of 64
      // (fp8.hip pa_group_image pads each expert to 64 tokens), so k-tiles are full
      if (p.K % BKT == 0) return launch_v<AK, BK, F32, false, true, false, false, GM>(p, batch, st);
    }
    return pf ? launch_v<AK, BK, F32, true, false, false, false, GM>(p, batch, st)
              : launch_v<AK, BK, F32, false, false, false, false, GM>(p, batch, st);
  }
}

template <bool AK, bool BK, bool F32>
static int launch(const Params& p0, int batch, hipStream_t st) {
  Params p = p0;
  p.tiles_m = (p.M + BM - 1) / BM;
  p.tiles_n = (p.N + BN - 1) / BN;
  if (p.grp_mode == 1) {
    // every group adds at most one partial tile row beyond total_rows / BM
    p.ngrp = batch;
    p.tiles_m = (p.M + BM - 1) / BM + batch;
    return launch_g<AK, BK, F32, 1>(p, batch, st);
  }
  if (p.grp_mode == 2) return launch_g<AK, BK, F32, 2>(p, batch, st);
  return launch_g<AK, BK, F32, 0>(p, batch, st);
}

template <bool F32, int GM>
static int launch_f8(const Params& p, int batch, hipStream_t st) {
  if constexpr (GM == 2) {
    // ragged k per group: the per-lane k range check of the partial-tile path
    return launch_v<true, true, F32, false, false, false, true, GM>(p, batch, st);
  } else {
    if (p.K % BKT == 0) return launch_v<true, true, F32, false, true, false, true, GM>(p, batch, st);
    return launch_v<true, true, F32, false, false, false, true, GM>(p, batch, st);
  }
}

// Tile table of a grouped-rows GEMM (grp_mode 1), built on the device from the row
// offsets grp[0..G]: tab[q] = g << 16 | j for the j-th 256-row tile of group g, in
// group order; -1 for the unused tail up to ntab = ceil(total / 256) + G entries.
// One block: each thread owns a contiguous chunk of groups; a block scan of the
// chunk totals gives every chunk its first tile row.
__global__ __launch_bounds__(1024) void group_tile_table_kernel(const int* __restrict__ grp, int G,
                                                                int* __restrict__ tab, int ntab) {
  __shared__ int part[1024];
  const int t = threadIdx.x;
  const int per = (G + 1023) / 1024;
  const int g0 = min(G, t * per), g1 = min(G, g0 + per);
  int sum = 0;
  for (int g = g0; g < g1; ++g) sum += (grp[g + 1] - grp[g] + BM - 1) / BM;
  part[t] = sum;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {  // inclusive Hillis-Steele scan
    const int v = t >= o ? part[t - o] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int q = part[t] - sum;  // first tile row of this chunk
  for (int g = g0; g < g1; ++g) {
    const int n = (grp[g + 1] - grp[g] + BM - 1) / BM;
    for (int j = 0; j < n && q < ntab; ++j) tab[q++] = (g << 16) | j;
  }
  for (int i = part[1023] + t; i < ntab; i += 1024) tab[i] = -1;
}

}  // namespace gemm
}  // namespace pa

using namespace pa;

// fp8 (OCP e4m3) GEMM, both operands K-major: C[m, n] (=|+=) alpha * sa[m] * sb[g*N + n]
//   * sum_k A[m, k] B[n, k].  K, lda, ldb, sB in fp8 elements (multiples of 16);
//   grp/grp_mode 1 as pa_gemm (ragged rows per group, B and sb advance per group).
PA_EXPORT int pa_gemm_f8(int out_f32, const void* A, const void* B, void* C, const float* sa, const float* sb,
                         int M, int N, int K, long lda, long ldb, long ldc, long sB, long sC, int batch, float alpha,
                         int accumulate, const int* grp, int grp_mode, hipStream_t st) {
  if (M <= 0 || N <= 0 || batch <= 0) return 0;
  if ((N & 7) || (K & 15) || (lda & 15) || (ldb & 15) || (sB & 15) || K <= 0 || !sa || !sb) return -1;
  gemm::Params p{};
  p.A = A; p.B = B; p.C = C;
  p.M = M; p.N = N; p.K = K / 2;  // k units of 2 fp8 bytes: the bf16 DMA / LDS machinery as is
  p.lda = lda / 2; p.ldb = ldb / 2; p.ldc = ldc;
  p.sB = sB / 2; p.sC = sC;
  p.alpha = alpha; p.accumulate = accumulate;
  p.grp = grp;
  p.grp_mode = grp ? grp_mode : 0;
  p.grp_tiles = grp && p.grp_mode == 1 ? grp + batch + 1 : nullptr;
  p.sa = sa; p.sb = sb;
  p.sbs = batch > 1 ? N : 0;
  p.sas = 0;
  p.tiles_m = (p.M + gemm::BM - 1) / gemm::BM + (p.grp_mode == 1 ? batch : 0);
  p.tiles_n = (p.N + gemm::BN - 1) / gemm::BN;
  p.ngrp = batch;
  if (p.grp_mode == 2) {
    // grouped dW: C[g] (M x N, stride sC) = sa[g] sb[g] (X_g^T dY_g), K = the padded
    // token extent (lda = ldb), group g's tokens [grp[g], grp[g+1]) in fp8 elements
    if (!out_f32) return -1;
    p.sas = M;
    p.sbs = N;
    return gemm::launch_f8<true, 2>(p, batch, st);
  }
  if (out_f32) return p.grp_mode ? gemm::launch_f8<true, 1>(p, batch, st) : gemm::launch_f8<true, 0>(p, batch, st);
  return p.grp_mode ? gemm::launch_f8<false, 1>(p, batch, st) : gemm::launch_f8<false, 0>(p, batch, st);
}

// grp: int[G + 1 + ceil(total_rows / 256) + G] -- the row offsets, then the tile
// table of a grouped-rows GEMM (grp_mode 1), filled here from the offsets.
PA_EXPORT int pa_group_tile_table(int* grp, int G, long total_rows, hipStream_t st) {
  if (G <= 0 || G >= 32768 || total_rows < 0) return -1;
  const int ntab = (int)((total_rows + gemm::BM - 1) / gemm::BM) + G;
  hipLaunchKernelGGL(gemm::group_tile_table_kernel, dim3(1), dim3(1024), 0, st, (const int*)grp, G, grp + G + 1,
                     ntab);
  return (int)hipGetLastError();
}

PA_EXPORT void pa_gemm_set_sched(int s) { gemm::g_sched = s; }
PA_EXPORT void pa_gemm_set_persistent(int s) { gemm::g_persistent = s; }
PA_EXPORT void pa_gemm_set_stagger(int s) { gemm::g_stagger = s; }
PA_EXPORT void pa_gemm_set_dw1w(int s) { gemm::g_dw1w = s; }

// Returns 0 on success, a hipError on launch failure, -1 for an unsupported shape
// (the caller checks shapes first: N a multiple of 8, K a multiple of 8 when an
// operand is K-major, M a multiple of 8 when A is M-major; 16-B aligned rows;
// every operand < 4 GiB).
//   a_kmaj: A is [M][lda] K-contiguous (else [K][lda] M-contiguous)
//   b_kmaj: B is [N][ldb] K-contiguous (else [K][ldb] N-contiguous)
//   out_f32: C is fp32 (else bf16); accumulate: C += alpha*AB (+bias)
//   grp (device int[batch + 1], + the tile table for mode 1: pa_group_tile_table)
//   + grp_mode: grouped / ragged GEMM (see Params)
//   k_total > 0: split-K, batch b covers k in [b*K, min((b+1)*K, k_total)) (sA/sB are
//   the k offsets of one split); atomic (fp32 C, sC = 0): every split adds its tile
//   into C with float atomics, otherwise the caller sums the per-batch outputs
static int gemm_entry(bool padded, int a_kmaj, int b_kmaj, int out_f32, const void* A, const void* B, void* C,
                      const void* bias, int M, int N, int K, long lda, long ldb, long ldc, long sA, long sB,
                      long sC, int batch, float alpha, int accumulate, int k_total, int atomic, const int* grp,
                      int grp_mode, hipStream_t st) {
  if (M <= 0 || N <= 0 || batch <= 0) return 0;
  // 16-B chunks: along K for a K-major operand, along M / N for an MN-major one,
  // along N for the output.  `padded` (pa_gemm_padded): the extents may be ragged
  // when the leading dimensions are 8-aligned -- a chunk that starts inside the
  // matrix is moved whole, so it reads / writes the row padding up to the next
  // multiple of 8 (see pa_gemm_padded for the caller's contract)
  if (padded) {
    auto r8 = [](long v) { return (v + 7) & ~7L; };
    if ((lda & 7) || (ldb & 7) || (ldc & 7) || ldc < r8(N)) return -1;
    if (lda < (a_kmaj ? r8(K) : r8(M)) || ldb < (b_kmaj ? r8(K) : r8(N))) return -1;
  } else if ((N & 7) || ((a_kmaj || b_kmaj) && (K & 7)) || (!a_kmaj && (M & 7))) {
    return -1;
  }
  gemm::Params p{};
  p.A = A; p.B = B; p.C = C; p.bias = bias;
  p.M = M; p.N = N; p.K = K;
  p.lda = lda; p.ldb = ldb; p.ldc = ldc;
  p.sA = sA; p.sB = sB; p.sC = sC;
  p.alpha = alpha; p.accumulate = accumulate; p.k_total = k_total;
  p.atomic = atomic && out_f32;
  p.grp = grp;
  p.grp_mode = grp ? grp_mode : 0;
  p.grp_tiles = grp ? grp + batch + 1 : nullptr;  // grp_mode 1: table after the offsets
  if (p.atomic && bias) return -1;
  if (K <= 0) return -1;
  if ((long)ldc * gemm::BM * (out_f32 ? 4 : 2) >= (long)gemm::OOB) return -1;  // per-tile C offsets are 32-bit
  // fp32 weight gradients with an MN-major operand: the one-wave-per-SIMD kernel
  if (gemm::g_dw1w && out_f32 && !(a_kmaj && b_kmaj) && !padded && !bias && batch == 1 && !grp && !k_total &&
      !p.atomic && K % gemm::BKT == 0) {
    if (a_kmaj) return gemm::launch_1w<true, false>(p, st);
    if (b_kmaj) return gemm::launch_1w<false, true>(p, st);
    return gemm::launch_1w<false, false>(p, st);
  }
#define PA_G(AK, BK, F)                                                \
  if (a_kmaj == AK && b_kmaj == BK && out_f32 == F) return gemm::launch<AK, BK, F>(p, batch, st);
  PA_G(1, 1, 0) PA_G(1, 0, 0) PA_G(0, 1, 0) PA_G(0, 0, 0)
  PA_G(1, 1, 1) PA_G(1, 0, 1) PA_G(0, 1, 1) PA_G(0, 0, 1)
#undef PA_G
  return -1;
}

PA_EXPORT int pa_gemm(int a_kmaj, int b_kmaj, int out_f32, const void* A, const void* B, void* C,
                      const void* bias, int M, int N, int K, long lda, long ldb, long ldc, long sA, long sB,
                      long sC, int batch, float alpha, int accumulate, int k_total, int atomic, const int* grp,
                      int grp_mode, hipStream_t st) {
  return gemm_entry(false, a_kmaj, b_kmaj, out_f32, A, B, C, bias, M, N, K, lda, ldb, ldc, sA, sB, sC, batch, alpha,
                    accumulate, k_total, atomic, grp, grp_mode, st);
}

// pa_gemm for ragged extents (a vocabulary that is not a multiple of 8: GPT's
// 50,257-wide tied LM head) on 8-aligned row buffers.  Contract: every row of A, B
// and C holds at least the extent rounded up to 8 elements (lda / ldb / ldc are
// multiples of 8); the padding of a K-major operand past K and of an MN-major A
// past M is ZERO (it enters the products); C columns N .. round8(N) are written
// (with zeros from out-of-range B rows) -- never C memory past the padded row.
// B rows past N (K-major B) and past K (MN-major B) are not read.
PA_EXPORT int pa_gemm_padded(int a_kmaj, int b_kmaj, int out_f32, const void* A, const void* B, void* C,
                             int M, int N, int K, long lda, long ldb, long ldc, int accumulate, hipStream_t st) {
  return gemm_entry(true, a_kmaj, b_kmaj, out_f32, A, B, C, nullptr, M, N, K, lda, ldb, ldc, 0, 0, 0, 1, 1.f,
                    accumulate, 0, 0, nullptr, 0, st);
}

// Fused-epilogue GEMMs, both operands K-major, bf16 C (see Params::aux):
//   epi 1: C [M][N] = A B^T (gate|up interleaved by 16), aux = h [M][N/2] (ldaux)
//   epi 2: aux = gu [M][2N] (ldaux), C = dgu [M][2N] (ldc) from da = A B^T
//   epi 3: C [M][N] = A B^T with columns < rope_cols rotated (neox, 128-col heads,
//          cos/sin [rope_S][64] fp32, position = row % rope_S)
// K must be a multiple of 64.  Returns -1 for shapes the fused epilogues do not cover.
PA_EXPORT int pa_gemm_epi(int epi, const void* A, const void* B, void* C, void* aux, long ldaux, int M, int N, int K,
                          long lda, long ldb, long ldc, const float* cosT, const float* sinT, int rope_cols,
                          int rope_S, hipStream_t st) {
  if (M <= 0 || N <= 0) return 0;
  if ((N & 7) || K <= 0 || (K % gemm::BKT) || (lda & 7) || (ldb & 7) || (ldc & 7)) return -1;
  gemm::Params p{};
  p.A = A; p.B = B; p.C = C;
  p.M = M; p.N = N; p.K = K;
  p.lda = lda; p.ldb = ldb; p.ldc = ldc;
  p.alpha = 1.f;
  p.aux = aux; p.ldaux = ldaux;
  p.cosT = cosT; p.sinT = sinT; p.rope_cols = rope_cols; p.rope_S = rope_S;
  p.tiles_m = (M + gemm::BM - 1) / gemm::BM;
  p.tiles_n = (N + gemm::BN - 1) / gemm::BN;
  const long out_w = epi == 2 ? 2L * N : N;
  if ((long)ldc * gemm::BM * 2 >= (long)gemm::OOB || ldc < out_w) return -1;
  if (epi == 1) {
    if ((N % 32) || !aux || (ldaux & 7) || ldaux < N / 2 || (long)ldaux * gemm::BM * 2 >= (long)gemm::OOB) return -1;
    return gemm::launch_v<true, true, false, false, true, false, false, 0, false, 1>(p, 1, st);
  }
  if (epi == 2) {
    if ((N % 16) || !aux || (ldaux & 7) || ldaux < 2L * N || (long)ldaux * gemm::BM * 2 >= (long)gemm::OOB) return -1;
    return gemm::launch_v<true, true, false, false, true, false, false, 0, false, 2>(p, 1, st);
  }
  if (epi == 3) {
    if (!cosT || !sinT || rope_S <= 0 || (rope_cols % 128) || rope_cols > N || (M % rope_S)) return -1;
    return gemm::launch_v<true, true, false, false, true, false, false, 0, false, 3>(p, 1, st);
  }
  return -1;
}

// Implicit-GEMM convolution, NHWC bf16 (forward, or dgrad with up = log2 stride):
//   out[(n, oy, ox)][co] = sum_{kh, kw, c} src[n, iy, ix, c] * wt[co][kh][kw][c]
// src: [N, H, W, C] (C % 64 == 0), wt: [Cout][KH*KW*C] K-major, out: [N*OH*OW][Cout]
// (ldc = Cout), bias [Cout] or null.  Returns -1 for shapes the kernel does not cover.
PA_EXPORT int pa_conv_gemm_acc(const void* src, const void* wt, void* out, const void* bias, int Nb, int H, int W,
                               int C, int OH, int OW, int Cout, int KH, int KW, int sy, int sx, int py, int px, int dy,
                               int dx, int uy, int ux, int accumulate, hipStream_t st);

PA_EXPORT int pa_conv_gemm(const void* src, const void* wt, void* out, const void* bias, int Nb, int H, int W, int C,
                           int OH, int OW, int Cout, int KH, int KW, int sy, int sx, int py, int px, int dy, int dx,
                           int uy, int ux, hipStream_t st) {
  return pa_conv_gemm_acc(src, wt, out, bias, Nb, H, W, C, OH, OW, Cout, KH, KW, sy, sx, py, px, dy, dx, uy, ux, 0,
                          st);
}

PA_EXPORT int pa_conv_gemm_stats(const void* src, const void* wt, void* out, const void* bias, int Nb, int H, int W,
                                 int C, int OH, int OW, int Cout, int KH, int KW, int sy, int sx, int py, int px,
                                 int dy, int dx, int uy, int ux, int accumulate, float* part, const float* shift,
                                 hipStream_t st);

// accumulate: out += conv (bf16 read-modify-write in the epilogue: a gradient summed in place)
PA_EXPORT int pa_conv_gemm_acc(const void* src, const void* wt, void* out, const void* bias, int Nb, int H, int W,
                               int C, int OH, int OW, int Cout, int KH, int KW, int sy, int sx, int py, int px, int dy,
                               int dx, int uy, int ux, int accumulate, hipStream_t st) {
  return pa_conv_gemm_stats(src, wt, out, bias, Nb, H, W, C, OH, OW, Cout, KH, KW, sy, sx, py, px, dy, dx, uy, ux,
                            accumulate, nullptr, nullptr, st);
}

PA_EXPORT int pa_conv_gemm_bnbwd(const void* src, const void* wt, void* out, const void* bias, int Nb, int H, int W,
                                 int C, int OH, int OW, int Cout, int KH, int KW, int sy, int sx, int py, int px,
                                 int dy, int dx, int uy, int ux, int accumulate, float* part, const float* shift,
                                 const void* bx, const void* by, const float* mean, const float* rstd, const void* w,
                                 const void* b, int wdt, int relu, hipStream_t st);

// part (nullable): BatchNorm statistics of the output, [ceil(M / 256)][2][Cout] about
// `shift` (nullable, fp32 [Cout]) -- the layout of pa_conv_sn's and bn_finalize's partials
PA_EXPORT int pa_conv_gemm_stats(const void* src, const void* wt, void* out, const void* bias, int Nb, int H, int W,
                                 int C, int OH, int OW, int Cout, int KH, int KW, int sy, int sx, int py, int px,
                                 int dy, int dx, int uy, int ux, int accumulate, float* part, const float* shift,
                                 hipStream_t st) {
  if (accumulate && part) return -1;
  return pa_conv_gemm_bnbwd(src, wt, out, bias, Nb, H, W, C, OH, OW, Cout, KH, KW, sy, sx, py, px, dy, dx, uy, ux,
                            accumulate, part, shift, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0, st);
}

// Data gradient with the BatchNorm backward statistics of its final values (after an
// optional accumulate-into): part [ceil(M / 256)][2][Cout] of sum g, sum g (x - mean)
// (common.h BnBwdSrc; bx null: forward statistics about `shift` as pa_conv_gemm_stats)
PA_EXPORT int pa_conv_gemm_bnbwd(const void* src, const void* wt, void* out, const void* bias, int Nb, int H, int W,
                                 int C, int OH, int OW, int Cout, int KH, int KW, int sy, int sx, int py, int px,
                                 int dy, int dx, int uy, int ux, int accumulate, float* part, const float* shift,
                                 const void* bx, const void* by, const float* mean, const float* rstd, const void* w,
                                 const void* b, int wdt, int relu, hipStream_t st) {
  if (bx && (!part || !mean || !rstd)) return -1;
  const long M = (long)Nb * OH * OW;
  if (M <= 0 || Cout <= 0) return 0;
  if (C % 64 || Cout % 8 || M > 0x7fffffffL || (long)Nb * H * W * C >= 0x7fffffffL || H > 32767 || W > 32767)
    return -1;
  gemm::Params p{};
  p.A = src; p.B = wt; p.C = out; p.bias = bias;
  p.M = (int)M; p.N = Cout; p.K = KH * KW * C;
  p.lda = C; p.ldb = p.K; p.ldc = Cout;
  p.alpha = 1.f;
  p.accumulate = accumulate;
  p.part = part;
  p.shift = shift;
  p.bs = BnBwdSrc{(const u16*)bx, (const u16*)by, mean, rstd, w, b, wdt, relu};
  p.H = H; p.W = W; p.Cc = C; p.OH = OH; p.OW = OW; p.KW = KW;
  p.sy = sy; p.sx = sx; p.py = py; p.px = px; p.dy = dy; p.dx = dx; p.uy = uy; p.ux = ux;
  p.tiles_m = (p.M + gemm::BM - 1) / gemm::BM;
  p.tiles_n = (p.N + gemm::BN - 1) / gemm::BN;
  if (bx) return gemm::launch_v<true, true, false, false, true, true, false, 0, true>(p, 1, st);
  return gemm::launch_v<true, true, false, false, true, true>(p, 1, st);
}

// Split-K epilogue: out[m, n] (bf16, row stride ldc) = sum_s part[s][m][n] (+ bias[n]).
// The GEMM of a shape with too few 256x256 tiles to fill the chip (e.g. T = 4096 tokens
// x 5120 outputs = 320 tiles on 256 CUs: two rounds for 1.25 rounds of work) runs as
// S k-slices into fp32 slabs; this pass sums them in a fixed order (deterministic).
namespace pa {
__global__ __launch_bounds__(256) void gemm_splitk_sum_kernel(const float* __restrict__ part, int S, long M, int N,
                                                            const void* __restrict__ bias, int bias_f32,
                                                            u16* __restrict__ out, long ldc) {
  const int nc = N / 8;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= M * nc) return;
  const long m = idx / nc;
  const int n0 = (int)(idx % nc) * 8;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < S; ++s) {
    float v[8];
    load8(part + ((long)s * M + m) * N + n0, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] += v[e];
  }
  if (bias) {
    float bv[8];
    if (bias_f32) load8((const float*)bias + n0, bv);
    else load8((const u16*)bias + n0, bv);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] += bv[e];
  }
  store8(out + m * ldc + n0, acc);
}
}  // namespace pa

PA_EXPORT int pa_gemm_splitk_sum(const float* part, int S, long M, int N, const void* bias, int bias_f32, void* out,
                               long ldc, hipStream_t st) {
  if (S <= 0 || M <= 0 || N <= 0 || (N % 8) || (ldc % 8)) return -1;
  const long n = M * (N / 8);
  hipLaunchKernelGGL(pa::gemm_splitk_sum_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, part, S, M, N,
                     bias, bias_f32, (u16*)out, ldc);
  PA_LAUNCH_CHECK();
}
