// Flash-attention backward as two MFMA kernels, no cross-workgroup dQ reduction
// (gfx950 / CDNA4, bf16 in, fp32 accumulate, D = 128).
//
// Semantics (the unfused reference: python/paddle/fluid/nets.py:332-460
// scaled_dot_product_attention -> matmul / softmax / matmul and their grads):
//   P = softmax(scale Q K^T + causal mask),  dV = P^T dO,  dP = dO V^T,
//   dS = P * (dP - rowsum(dO * O)),  dQ = scale dS K,  dK = scale dS^T Q.
// Optionally the inverse neox rotary (the backward of the rotary the forward applied
// to q / k) is applied to dQ / dK in the kernels' epilogues, and the results are
// written in bf16 straight into strided destinations (the packed dqkv gradient).
//
// Why two kernels (the round-3..5 fused kernels fa_bwd_kernel3 / kernel5 are kept in
// flash_attn.hip): a fused pass owns one key block and must SUM dQ over all key
// blocks of a query -- fp32 atomics (1.3 TB/s chip-wide) or per-key-block partial
// slabs plus a reduce pass -- and has to cross dS through LDS behind a workgroup
// barrier every query slice, which serialised the v5 kernel at 22-25 % MFMA busy.
// Here:
//   * fa_bwd_dq_kernel (query-stationary, the forward's structure): per wave 32
//     query rows; S^T = K Q^T and dP^T = V dO^T with the QUERY on the MFMA lane, so
//     P^T / dS^T accumulators are directly the B operand of dQ^T += K^T dS^T (K^T by
//     ds_read_b64_tr_b16 from the same LDS image the row reads use).  It also computes
//     delta = rowsum(dO * O) for its rows (no pre-pass) and publishes {lse*log2e,
//     delta} per row for the second kernel.  dQ is complete in registers at the end:
//     scale, inverse rotary, bf16 store.
//   * fa_bwd_dkdv_kernel (key-stationary): per wave 32 keys; S = Q K^T and dP = dO V^T
//     with the KEY on the lane, the accumulators initialised with -lse / -delta (row
//     constants as the initial accumulator: p = exp2(c S'), dS = p dP'), P / dS are
//     the B operands of dV^T += dO^T P and dK^T += Q^T dS.  Nothing crosses LDS
//     between waves except the staged Q / dO slices.  The GQA head group is summed in
//     registers (the slice loop runs over every query head of the kv head).
// The recomputation of S and dP in the dQ kernel costs 2 of the 7 GEMM units; in
// exchange no dQ partial ever leaves a workgroup, both kernels run two waves per SIMD
// (two workgroups per CU) and the separate pre-pass, dQ-reduce and dK-rotary passes
// are gone.
//
// Staging: Q / dO slices (dkdv) and K / V tiles (dq) reach LDS by LDS-DMA
// (buffer_load ... lds, 1 KiB per wave-instruction, no staging registers), one stage
// ahead, with the XOR swizzle applied on the SOURCE address (guide §5.4 rule 21).
// LDS reads of the compute phase are inline asm so hipcc does not put a vmcnt(0) in
// front of them for the in-flight DMA (the same reason as gemm.hip's Frag<false>);
// their results are fenced by lgkmcnt waits that name the registers.
#include <type_traits>

#include "common.h"

namespace pa {
namespace fab {

typedef __bf16 bf8v __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_vp;

constexpr int D = 128;
constexpr int KCH = D / 8;  // 16-B chunks per row
static int g_variant = 1;   // pa_fa_bwd_split_set_variant

struct Params {
  const u16 *q, *k, *v, *o, *dout;
  const float* lse;  // [B, Hq, Sq] natural log of the softmax denominators (forward)
  float* ld2;        // [B, Hq, Sq, 2] {-lse / scale, -delta} written by the dQ kernel
  u16 *dq, *dk, *dv;
  long q_bs, q_ss, q_hs, k_bs, k_ss, k_hs, v_bs, v_ss, v_hs, o_bs, o_ss, o_hs, do_bs, do_ss, do_hs;
  long dq_bs, dq_ss, dq_hs, dk_bs, dk_ss, dk_hs, dv_bs, dv_ss, dv_hs;
  const float *cosT, *sinT;  // [>= S, D/2] rotary tables (ROPE kernels only)
  int B, Sq, Sk, Hq, Hkv;
  float scale, scale_log2;
};

__device__ __forceinline__ f32x16 mfma32(bf8v a, bf8v b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ bf8v as_bf8(u16x8 v) { return __builtin_bit_cast(bf8v, v); }
__device__ __forceinline__ bf8v cat_tr(s4v lo, s4v hi) {
  typedef short s8v __attribute__((ext_vector_type(8)));
  s8v r = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf8v, r);
}
// 8 consecutive accumulator registers (k-slots of one 16-deep k-step) as a bf16 operand
__device__ __forceinline__ bf8v pack8(const f32x16& x, int base) {
  bf8v r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)x[base + j];
  return r;
}
__device__ __forceinline__ unsigned lds_addr(const char* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
// LDS reads as inline asm (see header); fenced by wait_lgkm(...) before use
__device__ __forceinline__ void rd128(u16x8& d, const char* p) {
  asm volatile("ds_read_b128 %0, %1" : "=v"(d) : "v"(lds_addr(p)));
}
__device__ __forceinline__ void rdtr(s4v& d, const char* p) {
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(d) : "v"(lds_addr(p)));
}
__device__ __forceinline__ void wait_lgkm(u16x8 (&a)[4]) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]));
}
__device__ __forceinline__ void wait_lgkm(s4v (&a)[8]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]));
}
__device__ __forceinline__ void wait_lgkm(s4v (&a)[16]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]),
                 "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]), "+v"(a[12]), "+v"(a[13]), "+v"(a[14]),
                 "+v"(a[15]));
}
__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// ---- LDS images (256-B rows of 16 chunks) ------------------------------------------
// dual image: row reads (b128, 16 consecutive rows) AND 4-row transposed reads are
// conflict-free (guide T10 layout (b)); same function as flash_attn.hip dual_off<128>
__device__ __forceinline__ int dual_sw(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ int dual_off(int row, int byte_in_row) {
  return row * 256 + ((((byte_in_row >> 4) ^ dual_sw(row)) << 4) | (byte_in_row & 15));
}
// row-read-only image: chunk XOR (row & 15) (16 distinct rows per b128 group)
__device__ __forceinline__ int rowimg_off(int row, int ch) { return row * 256 + ((ch ^ (row & 15)) << 4); }

// One LDS-DMA wave-instruction fills 4 rows (1 KiB) of an image: lane L writes the
// image bytes of row 4 * piece + (L >> 4), physical chunk L & 15, so it must LOAD the
// logical chunk that lands there.
template <bool DUAL>
__device__ __forceinline__ unsigned dma_src_off(int piece, int lane, long row_stride_elems) {
  const int row = 4 * piece + (lane >> 4), pc = lane & 15;
  const int ch = pc ^ (DUAL ? dual_sw(row) : (row & 15));
  return (unsigned)(row * row_stride_elems * 2 + ch * 16);
}
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, char* lds_piece, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_vp)lds_piece, 16, voff, 0, 0, 0);
}

// =====================================================================================
// dQ kernel: 4 waves x 32 query rows (128 rows of one (b, head)) per workgroup; key
// tiles of 32 (K dual image + V row image, 16 KiB, double-buffered).  The next tile
// is loaded into 16 registers under the current tile's MFMAs and written to the
// other stage after them (the forward kernel's staging, guide T14): one barrier per
// tile, and the LDS reads are plain loads the compiler counts and interleaves.
template <bool CAUSAL, bool ROPE>
__global__ __launch_bounds__(256, 2) void fa_bwd_dq_kernel(Params p) {
  constexpr int BM = 128, BN = 32, KS = D / 16, DB = D / 32;
  constexpr int TILE = BN * D * 2;  // 8 KiB
  constexpr int STG = 2 * TILE;     // K | V
  __shared__ __attribute__((aligned(1024))) char smem[2 * STG];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int h = blockIdx.x, b = blockIdx.y;
  const int mt = gridDim.z - 1 - blockIdx.z;  // causal: heaviest query blocks first
  const int kvh = h / (p.Hq / p.Hkv);
  const int q0 = mt * BM, qw = q0 + 32 * w, qrow = qw + r;
  const int offs = CAUSAL ? p.Sk - p.Sq : 0;
  const bool qok = qrow < p.Sq;

  // ---- this lane's query row: Q, dO (B operands), delta, lse
  const u16* qp = p.q + (long)b * p.q_bs + (long)h * p.q_hs + (long)qrow * p.q_ss;
  const u16* dop = p.dout + (long)b * p.do_bs + (long)h * p.do_hs + (long)qrow * p.do_ss;
  const u16* op = p.o + (long)b * p.o_bs + (long)h * p.o_hs + (long)qrow * p.o_ss;
  bf8v qf[KS], df[KS];
  float dsum = 0.f;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    u16x8 a = {0, 0, 0, 0, 0, 0, 0, 0}, d = a, o = a;
    if (qok) {
      a = *reinterpret_cast<const u16x8*>(qp + ks * 16 + hh * 8);
      d = *reinterpret_cast<const u16x8*>(dop + ks * 16 + hh * 8);
      o = *reinterpret_cast<const u16x8*>(op + ks * 16 + hh * 8);
    }
    qf[ks] = as_bf8(a);
    df[ks] = as_bf8(d);
#pragma unroll
    for (int j = 0; j < 8; ++j) dsum += bf2f(d[j]) * bf2f(o[j]);
  }
  const float delta = dsum + __shfl_xor(dsum, 32, 64);
  const long rowid = ((long)b * p.Hq + h) * p.Sq + qrow;
  // rows past Sq: lse2 = +inf makes every p = 0 (their dQ is never stored)
  const float lse2 = qok ? p.lse[rowid] * 1.44269504089f : INFINITY;
  // the dK / dV kernel's accumulator starts: S' = S - lse / scale, dP' = dP - delta
  if (qok && hh == 0) *reinterpret_cast<float2*>(p.ld2 + 2 * rowid) = make_float2(-lse2 / p.scale_log2, -delta);

  int kv_end = p.Sk;
  if (CAUSAL) kv_end = min(p.Sk, q0 + BM + offs);
  const int nt = kv_end > 0 ? (kv_end + BN - 1) / BN : 0;

  // ---- K / V tile staging: two 16-B chunks of K and two of V per thread
  const u16* kp = p.k + (long)b * p.k_bs + (long)kvh * p.k_hs;
  const u16* vp = p.v + (long)b * p.v_bs + (long)kvh * p.v_hs;
  const auto k_rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)kp, 0, (int)(unsigned)(((long)(p.Sk - 1) * p.k_ss + D) * 2), 0x00020000);
  const auto v_rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)vp, 0, (int)(unsigned)(((long)(p.Sk - 1) * p.v_ss + D) * 2), 0x00020000);
  // thread -> (row, chunk) of the tile; the second chunk is 16 rows further down
  // (dual_sw / row & 15 unchanged, so its LDS offset is +16 rows)
  const int srow = tid >> 4, sch = tid & 15;
  const unsigned koff = (unsigned)(srow * p.k_ss * 2 + sch * 16), voff = (unsigned)(srow * p.v_ss * 2 + sch * 16);
  const unsigned kstep16 = (unsigned)(16 * p.k_ss * 2), vstep16 = (unsigned)(16 * p.v_ss * 2);
  const int kls = dual_off(srow, sch * 16), vls = rowimg_off(srow, sch);
  u16x8 kst[2], vst[2];
  auto load_regs = [&](int t) {
    const unsigned kb = (unsigned)((long)t * BN * p.k_ss * 2) + koff, vb = (unsigned)((long)t * BN * p.v_ss * 2) + voff;
    // rows >= Sk fall outside the descriptor's range: zeros
    kst[0] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(k_rs, (int)kb, 0, 0));
    vst[0] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(v_rs, (int)vb, 0, 0));
    kst[1] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(k_rs, (int)(kb + kstep16), 0, 0));
    vst[1] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(v_rs, (int)(vb + vstep16), 0, 0));
  };
  auto store_lds = [&](int stage) {
    char* Ks = smem + stage * STG;
    char* Vs = Ks + TILE;
    *reinterpret_cast<u16x8*>(Ks + kls) = kst[0];
    *reinterpret_cast<u16x8*>(Ks + kls + 16 * 256) = kst[1];
    *reinterpret_cast<u16x8*>(Vs + vls) = vst[0];
    *reinterpret_cast<u16x8*>(Vs + vls + 16 * 256) = vst[1];
  };

  f32x16 dq[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) dq[i][e] = 0.f;

  if (nt > 0) {
    load_regs(0);
    store_lds(0);
  }
  __syncthreads();

  const int g = lane >> 4, gi = lane & 15, gq = gi >> 2, gp = gi & 3;
  for (int t = 0; t < nt; ++t) {
    if (t + 1 < nt) load_regs(t + 1);
    const char* Ks = smem + (t & 1) * STG;
    const char* Vs = Ks + TILE;
    const int kv0 = t * BN;
    const bool skip = CAUSAL && (kv0 > qw + 31 + offs);
    if (!skip) {
      // ---- S^T = K Q^T, dP'^T = V dO^T - delta (M = key, N = query, K = d)
      f32x16 s, dp;
#pragma unroll
      for (int e = 0; e < 16; ++e) { s[e] = 0.f; dp[e] = -delta; }
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const u16x8 kf = *reinterpret_cast<const u16x8*>(Ks + dual_off(r, (2 * ks + hh) * 16));
        s = mfma32(as_bf8(kf), qf[ks], s);
        const u16x8 vf = *reinterpret_cast<const u16x8*>(Vs + rowimg_off(r, 2 * ks + hh));
        dp = mfma32(as_bf8(vf), df[ks], dp);
      }
      // ---- P^T, dS^T (element e: key kv0 + (e & 3) + 8 (e >> 2) + 4 hh, query qrow)
      const bool need_mask = (kv0 + BN > p.Sk) || (CAUSAL && (kv0 + BN - 1 > qw + offs));
      if (need_mask) {
        int lim = p.Sk - kv0 - 4 * hh;
        if (CAUSAL) lim = min(lim, qrow + offs - kv0 - 4 * hh + 1);
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(s[e], p.scale_log2, -lse2));
          pv = ((e & 3) + 8 * (e >> 2) >= lim) ? 0.f : pv;
          dp[e] = pv * dp[e];
        }
      } else {
#pragma unroll
        for (int e = 0; e < 16; ++e) dp[e] = __builtin_amdgcn_exp2f(__builtin_fmaf(s[e], p.scale_log2, -lse2)) * dp[e];
      }
      // ---- dQ^T += K^T dS^T over 2 k-steps of 16 keys (A = K^T by transposed reads)
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const int rowb = 16 * st + 4 * (g >> 1) + gq;
        const bf8v dsf = pack8(dp, 8 * st);
#pragma unroll
        for (int db = 0; db < DB; ++db) {
          const int colb = (32 * db + 16 * (g & 1) + 4 * gp) * 2;
          const s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s4v*)(Ks + dual_off(rowb, colb)));
          const s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s4v*)(Ks + dual_off(rowb + 8, colb)));
          dq[db] = mfma32(cat_tr(lo, hi), dsf, dq[db]);
        }
      }
    }
    // stage (t+1)&1 was last read in iteration t-1, which every wave finished
    // before the barrier that closed it
    if (t + 1 < nt) store_lds((t + 1) & 1);
    __syncthreads();
  }

  // ---- epilogue: lane holds dQ^T[d = 32 db + (e & 3) + 8 (e >> 2) + 4 hh][qrow]
  if (!qok) return;
  u16* dst = p.dq + (long)b * p.dq_bs + (long)h * p.dq_hs + (long)qrow * p.dq_ss;
#pragma unroll
  for (int db = 0; db < DB; ++db)
#pragma unroll
    for (int e = 0; e < 16; ++e) dq[db][e] *= p.scale;
  if (ROPE) {
    // inverse neox rotation at position qrow: (lo, hi) = (lo c + hi s, hi c - lo s)
    const float* cr = p.cosT + (long)qrow * (D / 2);
    const float* sr = p.sinT + (long)qrow * (D / 2);
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int e4 = 0; e4 < 4; ++e4) {
        const int d = 32 * db + 8 * e4 + 4 * hh;
        const f32x4 co = *reinterpret_cast<const f32x4*>(cr + d);
        const f32x4 si = *reinterpret_cast<const f32x4*>(sr + d);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float lo = dq[db][4 * e4 + j], hi = dq[db + 2][4 * e4 + j];
          dq[db][4 * e4 + j] = lo * co[j] + hi * si[j];
          dq[db + 2][4 * e4 + j] = hi * co[j] - lo * si[j];
        }
      }
  }
#pragma unroll
  for (int db = 0; db < DB; ++db)
#pragma unroll
    for (int e4 = 0; e4 < 4; ++e4) {
      u16x4 o4;
#pragma unroll
      for (int j = 0; j < 4; ++j) o4[j] = f2bf(dq[db][4 * e4 + j]);
      *reinterpret_cast<u16x4*>(dst + 32 * db + 8 * e4 + 4 * hh) = o4;
    }
}

// =====================================================================================
// dK / dV kernel: 4 waves x 32 keys (128 keys of one (b, kv head)) per workgroup;
// query slices of 64 rows (Q, dO dual images + the two row constants, double-
// buffered), swept over every query head of the kv head's group.  V of the wave's
// keys stays in registers (B operand of dP); K rows sit in a wave-private LDS image.
// One wave per SIMD (dK / dV are 128 AGPRs): the next slice's Q / dO / row constants
// are loaded into registers under the current slice's 64 MFMAs and written to the
// other stage after them, one barrier per slice.  Every LDS address is a lane
// constant plus an immediate (the step loop is unrolled over the two stages), so the
// slice body issues no address arithmetic.
template <bool CAUSAL, bool ROPE, bool PIPE>
__global__ __launch_bounds__(256, 1) void fa_bwd_dkdv_kernel(Params p) {
  constexpr int BK = 128, BQ = 64, KS = D / 16, DB = D / 32;
  constexpr int KIMG = BK * D * 2;    // 32 KiB
  constexpr int QT = BQ * D * 2;      // 16 KiB
  constexpr int STG = 2 * QT + 512;   // Q | dO | -lse/scale x 64 | -delta x 64
  __shared__ __attribute__((aligned(1024))) char smem[KIMG + 2 * STG];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int kvh = blockIdx.x, b = blockIdx.y, kt = blockIdx.z;  // causal: early key blocks are heaviest
  const int ratio = p.Hq / p.Hkv;
  const int n0 = kt * BK, kw0 = n0 + 32 * w, mykey = kw0 + r;
  const int offs = CAUSAL ? p.Sk - p.Sq : 0;

  const u16* kp = p.k + (long)b * p.k_bs + (long)kvh * p.k_hs;
  const u16* vp = p.v + (long)b * p.v_bs + (long)kvh * p.v_hs;
  // V rows of this lane's key (B operand of dP = dO V^T): V[mykey][16 ks + 8 hh + j]
  bf8v vf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    u16x8 t = {0, 0, 0, 0, 0, 0, 0, 0};
    if (mykey < p.Sk) t = *reinterpret_cast<const u16x8*>(vp + (long)mykey * p.v_ss + ks * 16 + hh * 8);
    vf[ks] = as_bf8(t);
  }
  // K rows of this lane's key (B operand of S = Q K^T), register-resident in the PIPE
  // body: K[mykey][16 ks + 8 hh + j]
  bf8v kf[KS];
  if constexpr (PIPE) {
    const u16* kp_ = p.k + (long)b * p.k_bs + (long)kvh * p.k_hs;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      u16x8 t = {0, 0, 0, 0, 0, 0, 0, 0};
      if (mykey < p.Sk) t = *reinterpret_cast<const u16x8*>(kp_ + (long)mykey * p.k_ss + ks * 16 + hh * 8);
      kf[ks] = as_bf8(t);
    }
  }
  // K rows n0 .. n0 + 127 -> the row image (each wave reads back only its 32 rows)
  for (int idx = tid; idx < BK * KCH; idx += 256) {
    const int row = idx >> 4, ch = idx & 15;
    u16x8 t = {0, 0, 0, 0, 0, 0, 0, 0};
    if (n0 + row < p.Sk) t = *reinterpret_cast<const u16x8*>(kp + (long)(n0 + row) * p.k_ss + ch * 8);
    *reinterpret_cast<u16x8*>(smem + rowimg_off(row, ch)) = t;
  }

  int qstart = 0;
  if (CAUSAL) qstart = max(0, n0 - offs);
  qstart = (qstart / 32) * 32;
  const int nslice = qstart < p.Sq ? (p.Sq - qstart + BQ - 1) / BQ : 0;
  const int nsteps = nslice * ratio;  // step = (query head of the group, slice)

  // ---- staging: thread -> (row, chunk); chunks i = 0..3 are 16 rows apart (same swizzle)
  const int srow = tid >> 4, sch = tid & 15;
  const int sls = dual_off(srow, sch * 16);
  u16x8 qst[4], ost[4];
  float2 lst = make_float2(0.f, 0.f);
  auto load_regs = [&](int step) {
    const int hq = kvh * ratio + step / nslice;
    const int qt0 = qstart + (step % nslice) * BQ;
    const u16* qb = p.q + (long)b * p.q_bs + (long)hq * p.q_hs;
    const u16* ob = p.dout + (long)b * p.do_bs + (long)hq * p.do_hs;
    const auto q_rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)qb, 0, (int)(unsigned)(((long)(p.Sq - 1) * p.q_ss + D) * 2), 0x00020000);
    const auto o_rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)ob, 0, (int)(unsigned)(((long)(p.Sq - 1) * p.do_ss + D) * 2), 0x00020000);
    const unsigned qo = (unsigned)((qt0 + srow) * p.q_ss * 2 + sch * 16);
    const unsigned oo = (unsigned)((qt0 + srow) * p.do_ss * 2 + sch * 16);
    const unsigned qs16 = (unsigned)(16 * p.q_ss * 2), os16 = (unsigned)(16 * p.do_ss * 2);
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // rows >= Sq fall outside the descriptor's range: zeros
      qst[i] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(q_rs, (int)(qo + i * qs16), 0, 0));
      ost[i] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(o_rs, (int)(oo + i * os16), 0, 0));
    }
    if (tid < BQ) {
      typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
      const float* lb = p.ld2 + ((long)b * p.Hq + hq) * p.Sq * 2;
      const auto l_rs = __builtin_amdgcn_make_buffer_rsrc((void*)lb, 0, p.Sq * 8, 0x00020000);
      const u32x2 t = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(l_rs, (qt0 + tid) * 8, 0, 0));
      lst = make_float2(__uint_as_float(t[0]), __uint_as_float(t[1]));
    }
  };
  auto store_lds = [&](char* st) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      *reinterpret_cast<u16x8*>(st + sls + i * 4096) = qst[i];
      *reinterpret_cast<u16x8*>(st + QT + sls + i * 4096) = ost[i];
    }
    if (tid < BQ) {
      reinterpret_cast<float*>(st + 2 * QT)[tid] = lst.x;
      reinterpret_cast<float*>(st + 2 * QT)[BQ + tid] = lst.y;
    }
  };

  // ---- lane-constant LDS offsets (dual_sw / row & 15 depend on the row only through
  // row & 15: every c / st / stage variant is one of these plus an immediate)
  int a_off[KS], k_off[KS], t_off[DB][2];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    a_off[ks] = dual_off(r, (2 * ks + hh) * 16);
    k_off[ks] = rowimg_off(32 * w + r, 2 * ks + hh);
  }
  const int g = lane >> 4, gi = lane & 15, gq = gi >> 2, gp = gi & 3;
#pragma unroll
  for (int db = 0; db < DB; ++db)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf)
      t_off[db][hf] = dual_off(4 * (g >> 1) + gq + 8 * hf, (32 * db + 16 * (g & 1) + 4 * gp) * 2);
  const int l_off = (8 * 0 + 4 * hh) * 4;  // + 32 c + 8 e4 floats (immediates)

  // dK^T / dV^T live in AGPRs for the whole sweep: defined before the loop and read
  // after it by asm statements with "a" operands, so hipcc does not shuttle the
  // loop-carried accumulators through VGPRs around every MFMA (flash_attn.hip v5)
  f32x16 dk[DB], dv[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i) {
    f32x16 z;
#pragma unroll
    for (int e = 0; e < 16; ++e) z[e] = 0.f;
    asm volatile("" : "=a"(dk[i]) : "0"(z));
    asm volatile("" : "=a"(dv[i]) : "0"(z));
  }

  typedef __attribute__((address_space(3))) s4v lds_s4v;
  auto slice = [&](const char* Qs, int step) {
    const char* Os = Qs + QT;
    const char* L = Qs + 2 * QT;
    const int qt0 = qstart + (step % nslice) * BQ;
#pragma unroll
    for (int c = 0; c < 2; ++c) {  // two 32-query halves
      const int q32 = qt0 + 32 * c;
      // wave-uniform: keys kw0 .. kw0 + 31 vs queries q32 .. q32 + 31
      if ((CAUSAL && kw0 > q32 + 31 + offs) || q32 >= p.Sq) continue;
      // ---- accumulators start at the row constants: S' = Q K^T - lse / scale,
      // dP' = dO V^T - delta (element e: query q32 + 8 (e >> 2) + 4 hh + (e & 3))
      f32x16 sacc, dpacc;
#pragma unroll
      for (int e4 = 0; e4 < 4; ++e4) {
        const f32x4 a = *reinterpret_cast<const f32x4*>(L + l_off + (32 * c + 8 * e4) * 4);
        const f32x4 d4 = *reinterpret_cast<const f32x4*>(L + l_off + (BQ + 32 * c + 8 * e4) * 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          sacc[4 * e4 + j] = a[j];
          dpacc[4 * e4 + j] = d4[j];
        }
      }
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const u16x8 qa = *reinterpret_cast<const u16x8*>(Qs + a_off[ks] + c * 8192);
        const u16x8 kb = *reinterpret_cast<const u16x8*>(smem + k_off[ks]);
        sacc = mfma32(as_bf8(qa), as_bf8(kb), sacc);
        const u16x8 oa = *reinterpret_cast<const u16x8*>(Os + a_off[ks] + c * 8192);
        dpacc = mfma32(as_bf8(oa), vf[ks], dpacc);
      }
      // ---- P = exp2(scale log2e S'), dS = P dP' (scale folded into the dK epilogue)
      const bool need_mask = (CAUSAL && kw0 + 31 > q32 + offs) || q32 + 32 > p.Sq || kw0 + 32 > p.Sk;
      if (need_mask) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int q = q32 + 8 * (e >> 2) + 4 * hh + (e & 3);
          bool ok = q < p.Sq && mykey < p.Sk;
          if (CAUSAL) ok = ok && mykey <= q + offs;
          const float pv = ok ? __builtin_amdgcn_exp2f(sacc[e] * p.scale_log2) : 0.f;
          sacc[e] = pv;
          dpacc[e] = pv * dpacc[e];
        }
      } else {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const float pv = __builtin_amdgcn_exp2f(sacc[e] * p.scale_log2);
          sacc[e] = pv;
          dpacc[e] = pv * dpacc[e];
        }
      }
      // ---- dV^T += dO^T P, dK^T += Q^T dS (2 k-steps of 16 queries; A by transposed reads)
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const int rb = (32 * c + 16 * st) * 256;
        const bf8v pf = pack8(sacc, 8 * st);
        const bf8v sf = pack8(dpacc, 8 * st);
#pragma unroll
        for (int db = 0; db < DB; ++db) {
          const s4v o0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(Os + rb + t_off[db][0]));
          const s4v o1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(Os + rb + t_off[db][1]));
          dv[db] = mfma32(cat_tr(o0, o1), pf, dv[db]);
          const s4v q0_ = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(Qs + rb + t_off[db][0]));
          const s4v q1_ = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(Qs + rb + t_off[db][1]));
          dk[db] = mfma32(cat_tr(q0_, q1_), sf, dk[db]);
        }
      }
    }
  };

  // ---- software-pipelined slice (PIPE): both 32-query halves live at once, in program
  // order S/dP(0), S/dP(1), softmax(0), dK/dV(0), softmax(1), dK/dV(1) in ONE basic
  // block (the mask is a template constant, no branches), so the scheduler can put the
  // exp / mask / pack VALU of one half under the other half's independent MFMAs --
  // with one wave per SIMD nothing else hides them.
  // S / dP of one half: Q / dO rows in two groups of 4 k-steps, the second group's
  // reads in flight under the first group's MFMAs (fences that let VALU / SALU
  // through, so the other half's softmax can still fill the MFMA gaps)
  constexpr int FENCE = 0x0002 | 0x0004 | 0x0400;  // VALU, SALU, TRANS may cross
  auto sdp = [&](const char* Qs, int c, f32x16& sacc, f32x16& dpacc) {
    const char* Os = Qs + QT;
    const char* L = Qs + 2 * QT;
    u16x8 qa[KS], oa[KS];
#pragma unroll
    for (int ks = 0; ks < KS / 2; ++ks) {
      qa[ks] = *reinterpret_cast<const u16x8*>(Qs + a_off[ks] + c * 8192);
      oa[ks] = *reinterpret_cast<const u16x8*>(Os + a_off[ks] + c * 8192);
    }
#pragma unroll
    for (int e4 = 0; e4 < 4; ++e4) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(L + l_off + (32 * c + 8 * e4) * 4);
      const f32x4 d4 = *reinterpret_cast<const f32x4*>(L + l_off + (BQ + 32 * c + 8 * e4) * 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        sacc[4 * e4 + j] = a[j];
        dpacc[4 * e4 + j] = d4[j];
      }
    }
    __builtin_amdgcn_sched_barrier(FENCE);
#pragma unroll
    for (int ks = KS / 2; ks < KS; ++ks) {
      qa[ks] = *reinterpret_cast<const u16x8*>(Qs + a_off[ks] + c * 8192);
      oa[ks] = *reinterpret_cast<const u16x8*>(Os + a_off[ks] + c * 8192);
    }
    __builtin_amdgcn_sched_barrier(FENCE);
#pragma unroll
    for (int ks = 0; ks < KS / 2; ++ks) {
      sacc = mfma32(as_bf8(qa[ks]), kf[ks], sacc);
      dpacc = mfma32(as_bf8(oa[ks]), vf[ks], dpacc);
    }
    __builtin_amdgcn_sched_barrier(FENCE);
#pragma unroll
    for (int ks = KS / 2; ks < KS; ++ks) {
      sacc = mfma32(as_bf8(qa[ks]), kf[ks], sacc);
      dpacc = mfma32(as_bf8(oa[ks]), vf[ks], dpacc);
    }
  };
  // mask as data: element e is live iff lo <= 8 (e >> 2) + (e & 3) < hi (lane values)
  auto softmax = [&](f32x16& sacc, f32x16& dpacc, int lo, int hi, auto maskc) {
    constexpr bool MASK = decltype(maskc)::value;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      float pv = __builtin_amdgcn_exp2f(sacc[e] * p.scale_log2);
      if (MASK) {
        const int qe = 8 * (e >> 2) + (e & 3);
        pv = (qe >= lo && qe < hi) ? pv : 0.f;
      }
      sacc[e] = pv;
      dpacc[e] = pv * dpacc[e];
    }
  };
  // all 32 transposed reads of a half are issued before its first MFMA (a fence keeps
  // the scheduler from sinking each read next to its use, which exposed the LDS
  // latency once per MFMA)
  auto kvacc = [&](const char* Qs, int c, const f32x16& sacc, const f32x16& dpacc) {
    const char* Os = Qs + QT;
    s4v A[2][DB][4];
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int rb = (32 * c + 16 * st) * 256;
#pragma unroll
      for (int db = 0; db < DB; ++db) {
        A[st][db][0] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(Os + rb + t_off[db][0]));
        A[st][db][1] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(Os + rb + t_off[db][1]));
        A[st][db][2] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(Qs + rb + t_off[db][0]));
        A[st][db][3] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(Qs + rb + t_off[db][1]));
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const bf8v pf = pack8(sacc, 8 * st);
      const bf8v sf = pack8(dpacc, 8 * st);
#pragma unroll
      for (int db = 0; db < DB; ++db) {
        dv[db] = mfma32(cat_tr(A[st][db][0], A[st][db][1]), pf, dv[db]);
        dk[db] = mfma32(cat_tr(A[st][db][2], A[st][db][3]), sf, dk[db]);
      }
    }
  };
  auto slice_pipe = [&](const char* Qs, int step, int lo0, int hi0, int lo1, int hi1, auto maskc) {
    (void)step;
    f32x16 s0, d0, s1, d1;
    sdp(Qs, 0, s0, d0);
    sdp(Qs, 1, s1, d1);
    softmax(s0, d0, lo0, hi0, maskc);
    kvacc(Qs, 0, s0, d0);
    softmax(s1, d1, lo1, hi1, maskc);
    kvacc(Qs, 1, s1, d1);
  };
  // both halves active: the pipelined body (masked only where a half needs it)
  auto slice_any = [&](const char* Qs, int step) {
    const int qt0 = qstart + (step % nslice) * BQ;
    bool act = true, need = false;
    int lo[2], hi[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int q32 = qt0 + 32 * c;
      act = act && !((CAUSAL && kw0 > q32 + 31 + offs) || q32 >= p.Sq);
      need = need || (CAUSAL && kw0 + 31 > q32 + offs) || q32 + 32 > p.Sq || kw0 + 32 > p.Sk;
      // live: q < Sq, mykey < Sk, causal mykey <= q + offs, q = q32 + 4 hh + qe
      lo[c] = CAUSAL ? mykey - offs - q32 - 4 * hh : -1;
      hi[c] = p.Sq - q32 - 4 * hh;
      if (mykey >= p.Sk) hi[c] = -1;
    }
    if (!act) {
      slice(Qs, step);
    } else if (need) {
      slice_pipe(Qs, step, lo[0], hi[0], lo[1], hi[1], std::integral_constant<bool, true>());
    } else {
      slice_pipe(Qs, step, lo[0], hi[0], lo[1], hi[1], std::integral_constant<bool, false>());
    }
  };

  char* const st0 = smem + KIMG;
  char* const st1 = st0 + STG;
  if (nsteps > 0) {
    load_regs(0);
    store_lds(st0);
  }
  __syncthreads();
  for (int step = 0; step < nsteps; step += 2) {
    if (step + 1 < nsteps) load_regs(step + 1);
    if constexpr (PIPE) slice_any(st0, step);
    else slice(st0, step);
    if (step + 1 < nsteps) store_lds(st1);
    __syncthreads();
    if (step + 1 >= nsteps) break;
    if (step + 2 < nsteps) load_regs(step + 2);
    if constexpr (PIPE) slice_any(st1, step + 1);
    else slice(st1, step + 1);
    if (step + 2 < nsteps) store_lds(st0);
    __syncthreads();
  }

  // ---- epilogue: lane holds dK^T / dV^T [d = 32 db + (e & 3) + 8 (e >> 2) + 4 hh][mykey]
#pragma unroll
  for (int i = 0; i < DB; ++i) {
    asm volatile("" : "+a"(dk[i]));
    asm volatile("" : "+a"(dv[i]));
  }
  if (mykey >= p.Sk) return;
#pragma unroll
  for (int db = 0; db < DB; ++db)
#pragma unroll
    for (int e = 0; e < 16; ++e) dk[db][e] *= p.scale;
  if (ROPE) {
    const float* cr = p.cosT + (long)mykey * (D / 2);
    const float* sr = p.sinT + (long)mykey * (D / 2);
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int e4 = 0; e4 < 4; ++e4) {
        const int d = 32 * db + 8 * e4 + 4 * hh;
        const f32x4 co = *reinterpret_cast<const f32x4*>(cr + d);
        const f32x4 si = *reinterpret_cast<const f32x4*>(sr + d);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float lo = dk[db][4 * e4 + j], hi = dk[db + 2][4 * e4 + j];
          dk[db][4 * e4 + j] = lo * co[j] + hi * si[j];
          dk[db + 2][4 * e4 + j] = hi * co[j] - lo * si[j];
        }
      }
  }
  u16* dkp = p.dk + (long)b * p.dk_bs + (long)kvh * p.dk_hs + (long)mykey * p.dk_ss;
  u16* dvp = p.dv + (long)b * p.dv_bs + (long)kvh * p.dv_hs + (long)mykey * p.dv_ss;
#pragma unroll
  for (int db = 0; db < DB; ++db)
#pragma unroll
    for (int e4 = 0; e4 < 4; ++e4) {
      u16x4 a4, v4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a4[j] = f2bf(dk[db][4 * e4 + j]);
        v4[j] = f2bf(dv[db][4 * e4 + j]);
      }
      *reinterpret_cast<u16x4*>(dkp + 32 * db + 8 * e4 + 4 * hh) = a4;
      *reinterpret_cast<u16x4*>(dvp + 32 * db + 8 * e4 + 4 * hh) = v4;
    }
}

}  // namespace fab
}  // namespace pa

using namespace pa;

// A/B knob (benchmarks/fa_bwd_split_ab.py): bit 0 = the software-pipelined dK/dV slice
PA_EXPORT void pa_fa_bwd_split_set_variant(int v) { fab::g_variant = v; }

// Whether the split backward takes this problem (else the caller uses pa_flash_attn_bwd).
PA_EXPORT int pa_fa_bwd_split_ok(int B, int Sq, int Sk, int Hq, int Hkv, int D, const long* strides /*24*/) {
  if (D != 128 || Hkv <= 0 || Hq % Hkv || Sq <= 0 || Sk <= 0 || B <= 0) return 0;
  // 32-bit buffer offsets over one (b, head) and 16-B aligned rows
  const long lim = 1L << 31;
  const long rs[] = {strides[1], strides[4], strides[7], strides[13]};
  const long ss[] = {Sq, Sk, Sk, Sq};
  for (int i = 0; i < 4; ++i)
    if (rs[i] % 8 || (long)(ss[i] + 64) * rs[i] * 2 >= lim) return 0;
  for (int i = 0; i < 24; ++i)
    if (i % 3 != 0 && strides[i] % 8) return 0;  // row / head strides keep 16-B alignment
  return 1;
}

// strides (24): q, k, v, o, do, dq, dk, dv  x  (b, s, h).  dq is [B, Sq, Hq, D]-strided,
// dk / dv are per KV head ([B, Sk, Hkv, D]-strided).  ld2: [B, Hq, Sq, 2] fp32 scratch.
// cosT / sinT: [>= max(Sq, Sk), 64] fp32 or null (no rotary).
PA_EXPORT int pa_fa_bwd_split(const void* q, const void* k, const void* v, const void* o, const void* dout,
                              const float* lse, float* ld2, void* dq, void* dk, void* dv, const long* strides,
                              int B, int Sq, int Sk, int Hq, int Hkv, int D, float scale, int causal,
                              const float* cosT, const float* sinT, hipStream_t st) {
  if (!pa_fa_bwd_split_ok(B, Sq, Sk, Hq, Hkv, D, strides)) return (int)hipErrorInvalidValue;
  fab::Params p;
  p.q = (const u16*)q; p.k = (const u16*)k; p.v = (const u16*)v; p.o = (const u16*)o; p.dout = (const u16*)dout;
  p.lse = lse; p.ld2 = ld2; p.dq = (u16*)dq; p.dk = (u16*)dk; p.dv = (u16*)dv;
  long* f[] = {&p.q_bs, &p.q_ss, &p.q_hs, &p.k_bs, &p.k_ss, &p.k_hs, &p.v_bs, &p.v_ss, &p.v_hs,
               &p.o_bs, &p.o_ss, &p.o_hs, &p.do_bs, &p.do_ss, &p.do_hs, &p.dq_bs, &p.dq_ss, &p.dq_hs,
               &p.dk_bs, &p.dk_ss, &p.dk_hs, &p.dv_bs, &p.dv_ss, &p.dv_hs};
  for (int i = 0; i < 24; ++i) *f[i] = strides[i];
  p.cosT = cosT; p.sinT = sinT;
  p.B = B; p.Sq = Sq; p.Sk = Sk; p.Hq = Hq; p.Hkv = Hkv;
  p.scale = scale;
  p.scale_log2 = scale * 1.44269504089f;
  const bool rope = cosT != nullptr && sinT != nullptr;
  const dim3 gq(Hq, B, (Sq + 127) / 128), gk(Hkv, B, (Sk + 127) / 128);
#define PA_FAB_LAUNCH(C, R)                                                                  \
  hipLaunchKernelGGL((fab::fa_bwd_dq_kernel<C, R>), gq, dim3(256), 0, st, p);               \
  if ((fab::g_variant & 1) && C)                                                             \
    hipLaunchKernelGGL((fab::fa_bwd_dkdv_kernel<C, R, true>), gk, dim3(256), 0, st, p);     \
  else                                                                                       \
    hipLaunchKernelGGL((fab::fa_bwd_dkdv_kernel<C, R, false>), gk, dim3(256), 0, st, p);
  if (causal) {
    if (rope) { PA_FAB_LAUNCH(true, true) } else { PA_FAB_LAUNCH(true, false) }
  } else {
    if (rope) { PA_FAB_LAUNCH(false, true) } else { PA_FAB_LAUNCH(false, false) }
  }
#undef PA_FAB_LAUNCH
  PA_LAUNCH_CHECK();
}
