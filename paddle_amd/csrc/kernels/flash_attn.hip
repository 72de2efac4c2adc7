// Flash attention forward + backward for gfx950 (CDNA4), bf16 in / fp32 accumulate.
//
// The reference has no fused attention at all: nets.scaled_dot_product_attention
// (python/paddle/fluid/nets.py:332-460) materialises QK^T -> softmax -> PV as
// separate ops.  This is the north-star MI355X kernel.
//
// Forward (per workgroup: 4 waves x 32 query rows = 128 rows of one (b, head)):
//   * "swapped" QK^T: each wave computes S^T = K * Q^T with v_mfma_f32_32x32x16_bf16,
//     so a lane owns ONE query row (col = lane & 31) and the kv scores sit in its
//     registers: the online-softmax max/sum is lane-local + one xor-32 exchange.
//   * the S^T accumulator is fed straight back as the B operand of O^T += V^T P^T
//     (no LDS round trip for P); V^T fragments come from ds_read_b64_tr_b16
//     transposed LDS reads of a row-major V tile (T10).
//   * K tile XOR-swizzled at 16-B granularity (conflict-free ds_read_b128, T2);
//     V tile XOR-swizzled at 64-B granularity (conflict-free tr reads).
//   * next K/V tile prefetched into registers under the current tile's MFMAs and
//     written to LDS after the barrier (T14); the alpha rescale is a per-lane scalar.
//   * heaviest causal tiles are dispatched first (m-tile on grid.z, reversed), and
//     all m-tiles of one head land on the same XCD (head index on grid.x).
// Backward (per workgroup: 4 waves x 32 keys = 128 keys of one (b, head)):
//   * key on the MFMA lane for S and dP (their accumulators are the B operands of
//     dV^T += dO^T P and dK^T += Q^T dS), dK/dV accumulated in registers over all
//     query tiles, dS crosses LDS once (as dS^T) for dQ = dS K, which is reduced over
//     the workgroup's 128 keys on the MFMA before one f32 atomic add per element.
//   * Q/dO/K tiles use one LDS image for both row (b128) and transposed (tr_b16)
//     reads (guide T10 layout (b)).
#include "common.h"

namespace pa {

typedef __bf16 bf8v __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4v lds_s4v;

__device__ __forceinline__ f32x16 mfma32(bf8v a, bf8v b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ bf8v as_bf8(u16x8 v) { return __builtin_bit_cast(bf8v, v); }
__device__ __forceinline__ s4v tr_read(const char* lds_base, int byte_off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(lds_base + byte_off));
}
__device__ __forceinline__ bf8v cat_tr(s4v lo, s4v hi) {
  typedef short s8v __attribute__((ext_vector_type(8)));
  s8v r = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf8v, r);
}
__device__ __forceinline__ bf8v pack_p(const f32x16& x, int base) {
  bf8v r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)x[base + j];
  return r;
}

struct FwdParams {
  const u16 *q, *k, *v;
  u16* o;
  float* lse;  // [B, Hq, Sq]
  long q_bs, q_ss, q_hs, k_bs, k_ss, k_hs, v_bs, v_ss, v_hs, o_bs, o_ss, o_hs;
  int B, Sq, Sk, Hq, Hkv;
  float scale_log2;  // softmax_scale * log2(e)
};

// ---- LDS image helpers --------------------------------------------------------
// K (fwd): 16-B chunks XOR row (conflict-free b128 row reads of 16 distinct rows)
template <int D>
__device__ __forceinline__ int k_off(int row, int ch) {
  constexpr int KCH = D / 8;
  const int sw = (D == 128) ? (row & 15) : ((row >> 1) & (KCH - 1));
  return row * D * 2 + ((ch ^ sw) * 16);
}
// V (fwd): 64-B segments XOR row (conflict-free 4-row tr reads)
template <int D>
__device__ __forceinline__ int v_off_bytes(int row, int byte_in_row) {
  const int seg = byte_in_row >> 6;
  const int sw = (D == 128) ? (row & 3) : ((row >> 1) & 1);
  return row * D * 2 + (((seg ^ sw) << 6) | (byte_in_row & 63));
}
// dual-use image (bwd, D = 128 layout (b) of guide T10; generic for D = 64)
template <int D>
__device__ __forceinline__ int dual_off(int row, int byte_in_row) {
  constexpr int KCH = D / 8;
  const int ch = byte_in_row >> 4;
  int sw;
  if (D == 128) sw = ((row & 3) << 2) | ((row >> 2) & 3);
  else sw = ((row >> 1) & (KCH - 1));
  return row * D * 2 + (((ch ^ sw) << 4) | (byte_in_row & 15));
}

template <int D, bool CAUSAL>
__global__ __launch_bounds__(256, 2) void fa_fwd_kernel(FwdParams p) {
  constexpr int BM = 128, BN = 64;
  constexpr int KCH = D / 8;              // 16-B chunks per row
  constexpr int NCH = BN * KCH / 256;     // chunks per thread per tile
  constexpr int KS = D / 16;              // k-steps over head dim
  constexpr int DB = D / 32;              // 32-wide d blocks of O^T
  // two K|V stages: tile t+1 is stored into the other stage while tile t is
  // consumed, so one barrier per tile orders both the reads and the stores
  constexpr int STG = 2 * BN * D * 2;
  __shared__ __attribute__((aligned(16))) char smem[2 * STG];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int h = blockIdx.x, b = blockIdx.y;
  const int mt = gridDim.z - 1 - blockIdx.z;
  const int kvh = h / (p.Hq / p.Hkv);
  const long q0 = (long)mt * BM;
  const long qw = q0 + w * 32;
  const long qrow = qw + r;
  const long offs = CAUSAL ? (long)p.Sk - p.Sq : 0;

  const u16* qp = p.q + (long)b * p.q_bs + (long)h * p.q_hs;
  const u16* kp = p.k + (long)b * p.k_bs + (long)kvh * p.k_hs;
  const u16* vp = p.v + (long)b * p.v_bs + (long)kvh * p.v_hs;

  bf8v qf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    u16x8 t = {0, 0, 0, 0, 0, 0, 0, 0};
    if (qrow < p.Sq) t = *reinterpret_cast<const u16x8*>(qp + qrow * p.q_ss + ks * 16 + hh * 8);
    qf[ks] = as_bf8(t);
  }

  long kv_end = p.Sk;
  if (CAUSAL) kv_end = min((long)p.Sk, q0 + BM + offs);
  const int nt = kv_end > 0 ? (int)((kv_end + BN - 1) / BN) : 0;

  f32x16 oacc[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) oacc[i][e] = 0.f;
  float m = -1e30f, lsum = 0.f;

  u16x8 kst[NCH], vst[NCH];
  auto load_regs = [&](int t) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int idx = tid + 256 * i, row = idx / KCH, ch = idx % KCH;
      const long kr = (long)t * BN + row;
      if (kr < p.Sk) {
        kst[i] = *reinterpret_cast<const u16x8*>(kp + kr * p.k_ss + ch * 8);
        vst[i] = *reinterpret_cast<const u16x8*>(vp + kr * p.v_ss + ch * 8);
      } else {
        kst[i] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
        vst[i] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      }
    }
  };
  auto store_lds = [&](int stage) {
    char* Ks = smem + stage * STG;
    char* Vs = Ks + BN * D * 2;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int idx = tid + 256 * i, row = idx / KCH, ch = idx % KCH;
      *reinterpret_cast<u16x8*>(Ks + k_off<D>(row, ch)) = kst[i];
      *reinterpret_cast<u16x8*>(Vs + v_off_bytes<D>(row, ch * 16)) = vst[i];
    }
  };

  if (nt > 0) {
    load_regs(0);
    store_lds(0);
  }
  __syncthreads();

  // lane coordinates for the V^T transposed reads
  const int g = lane >> 4, gi = lane & 15, gq = gi >> 2, gp = gi & 3;

  for (int t = 0; t < nt; ++t) {
    if (t + 1 < nt) load_regs(t + 1);
    const char* Ks = smem + (t & 1) * STG;
    const char* Vs = Ks + BN * D * 2;
    const long kv0 = (long)t * BN;
    const bool skip = CAUSAL && (kv0 > qw + 31 + offs);
    if (!skip) {
      f32x16 s[2];
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int e = 0; e < 16; ++e) s[c][e] = 0.f;
      // the two key halves are independent accumulator chains: interleave them so
      // consecutive MFMAs never wait on each other's result
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const u16x8 kf = *reinterpret_cast<const u16x8*>(Ks + k_off<D>(32 * c + r, 2 * ks + hh));
          s[c] = mfma32(as_bf8(kf), qf[ks], s[c]);
        }
      }
      const bool need_mask = (kv0 + BN > p.Sk) || (CAUSAL && (kv0 + BN - 1 > qw + offs));
      // max over raw scores (scale > 0 commutes with max); the log2e*scale factor is
      // folded into one fma per element; raw v_exp_f32 (no denormal fix-up path)
      float tmax = -INFINITY;
      if (need_mask) {
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const long kv = kv0 + 32 * c + (e & 3) + 8 * (e >> 2) + 4 * hh;
            if (kv >= p.Sk || (CAUSAL && kv > qrow + offs)) s[c][e] = -INFINITY;
          }
      }
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int e = 0; e < 16; ++e) tmax = fmaxf(tmax, s[c][e]);
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64)) * p.scale_log2;
      // lazy rescaling: keep a stale running max unless some row's max grew by more
      // than 2^8 (exp2 values stay <= 256, safe in fp32 sums and bf16 P); the O
      // rescale then runs on a small fraction of tiles
      float alpha = 1.f;
      if (__any(tmax > m + 8.f)) {
        const float mnew = fmaxf(m, tmax);
        alpha = __builtin_amdgcn_exp2f(m - mnew);
        m = mnew;
      }
      const float mnew = m;
      float ps = 0.f;
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(s[c][e], p.scale_log2, -mnew));
          s[c][e] = pv;
          ps += pv;
        }
      lsum = lsum * alpha + ps;
      if (__any(alpha != 1.f)) {
#pragma unroll
        for (int i = 0; i < DB; ++i)
#pragma unroll
          for (int e = 0; e < 16; ++e) oacc[i][e] *= alpha;
      }
      // O^T += V^T P^T over 4 k-steps of 16 kv
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        const int c = st >> 1, half = st & 1;
        const bf8v pf = pack_p(s[c], 8 * half);
        const int rowb = 32 * c + 16 * half + 4 * (g >> 1) + gq;
#pragma unroll
        for (int db = 0; db < DB; ++db) {
          const int colb = (32 * db + 16 * (g & 1) + 4 * gp) * 2;
          const s4v lo = tr_read(Vs, v_off_bytes<D>(rowb, colb));
          const s4v hi = tr_read(Vs, v_off_bytes<D>(rowb + 8, colb));
          oacc[db] = mfma32(cat_tr(lo, hi), pf, oacc[db]);
        }
      }
    }
    // stage (t+1)&1 was last read in iteration t-1, which every wave finished
    // before the barrier that closed it
    if (t + 1 < nt) store_lds((t + 1) & 1);
    __syncthreads();
  }

  const float ltot = lsum + __shfl_xor(lsum, 32, 64);
  const float inv = ltot > 0.f ? 1.f / ltot : 0.f;
  if (qrow < p.Sq) {
    u16* op = p.o + (long)b * p.o_bs + (long)h * p.o_hs + qrow * p.o_ss;
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int e4 = 0; e4 < 4; ++e4) {
        const int d = 32 * db + 8 * e4 + 4 * hh;
        u16x4 o4;
#pragma unroll
        for (int j = 0; j < 4; ++j) o4[j] = f2bf(oacc[db][4 * e4 + j] * inv);
        *reinterpret_cast<u16x4*>(op + d) = o4;
      }
    if (hh == 0)
      p.lse[((long)b * p.Hq + h) * p.Sq + qrow] =
          ltot > 0.f ? (m + __log2f(ltot)) * 0.69314718056f : -INFINITY;
  }
}

template <int D, bool CAUSAL>
__global__ __launch_bounds__(256, 2) void fa_fwd_kernel2(FwdParams p) {
  constexpr int BM = 128, BN = 64;
  constexpr int KCH = D / 8;              // 16-B chunks per row
  constexpr int NCH = BN * KCH / 256;     // chunks per thread per tile
  constexpr int KS = D / 16;              // k-steps over head dim
  constexpr int DB = D / 32;              // 32-wide d blocks of O^T
  // two K|V stages: tile t+1 is stored into the other stage while tile t is
  // consumed, so one barrier per tile orders both the reads and the stores
  constexpr int STG = 2 * BN * D * 2;
  __shared__ __attribute__((aligned(16))) char smem[2 * STG];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int h = blockIdx.x, b = blockIdx.y;
  const int mt = gridDim.z - 1 - blockIdx.z;
  const int kvh = h / (p.Hq / p.Hkv);
  const int q0 = mt * BM;
  const int qw = q0 + w * 32;
  const int qrow = qw + r;
  const int offs = CAUSAL ? p.Sk - p.Sq : 0;

  const u16* qp = p.q + (long)b * p.q_bs + (long)h * p.q_hs;
  const u16* kp = p.k + (long)b * p.k_bs + (long)kvh * p.k_hs;
  const u16* vp = p.v + (long)b * p.v_bs + (long)kvh * p.v_hs;

  bf8v qf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    u16x8 t = {0, 0, 0, 0, 0, 0, 0, 0};
    if (qrow < p.Sq) t = *reinterpret_cast<const u16x8*>(qp + (long)qrow * p.q_ss + ks * 16 + hh * 8);
    qf[ks] = as_bf8(t);
  }

  int kv_end = p.Sk;
  if (CAUSAL) kv_end = min(p.Sk, q0 + BM + offs);
  const int nt = kv_end > 0 ? (kv_end + BN - 1) / BN : 0;

  f32x16 oacc[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) oacc[i][e] = 0.f;
  float m = -1e30f, lsum = 0.f;

  u16x8 kst[NCH], vst[NCH];
  // per-chunk element offsets within one tile (32-bit); the tile base pointers advance
  // by BN rows per tile, so the loop does no 64-bit address arithmetic per chunk
  int krow[NCH], koff[NCH], voff[NCH];
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int idx = tid + 256 * i, row = idx / KCH, ch = idx % KCH;
    krow[i] = row;
    koff[i] = row * (int)p.k_ss + ch * 8;
    voff[i] = row * (int)p.v_ss + ch * 8;
  }
  auto load_regs = [&](int t) {
    const u16* kt = kp + (long)t * BN * p.k_ss;
    const u16* vt = vp + (long)t * BN * p.v_ss;
    const int rows_left = p.Sk - t * BN;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      if (krow[i] < rows_left) {
        kst[i] = *reinterpret_cast<const u16x8*>(kt + koff[i]);
        vst[i] = *reinterpret_cast<const u16x8*>(vt + voff[i]);
      } else {
        kst[i] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
        vst[i] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      }
    }
  };
  auto store_lds = [&](int stage) {
    char* Ks = smem + stage * STG;
    char* Vs = Ks + BN * D * 2;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int idx = tid + 256 * i, row = idx / KCH, ch = idx % KCH;
      *reinterpret_cast<u16x8*>(Ks + k_off<D>(row, ch)) = kst[i];
      *reinterpret_cast<u16x8*>(Vs + v_off_bytes<D>(row, ch * 16)) = vst[i];
    }
  };

  if (nt > 0) {
    load_regs(0);
    store_lds(0);
  }
  __syncthreads();

  // lane coordinates for the V^T transposed reads
  const int g = lane >> 4, gi = lane & 15, gq = gi >> 2, gp = gi & 3;

  for (int t = 0; t < nt; ++t) {
    if (t + 1 < nt) load_regs(t + 1);
    const char* Ks = smem + (t & 1) * STG;
    const char* Vs = Ks + BN * D * 2;
    const int kv0 = t * BN;
    const bool skip = CAUSAL && (kv0 > qw + 31 + offs);
    if (!skip) {
      f32x16 s[2];
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int e = 0; e < 16; ++e) s[c][e] = 0.f;
      // the two key halves are independent accumulator chains: interleave them so
      // consecutive MFMAs never wait on each other's result
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const u16x8 kf = *reinterpret_cast<const u16x8*>(Ks + k_off<D>(32 * c + r, 2 * ks + hh));
          s[c] = mfma32(as_bf8(kf), qf[ks], s[c]);
        }
      }
      const bool need_mask = (kv0 + BN > p.Sk) || (CAUSAL && (kv0 + BN - 1 > qw + offs));
      // max over raw scores (scale > 0 commutes with max); the log2e*scale factor is
      // folded into one fma per element; raw v_exp_f32 (no denormal fix-up path)
      float tmax = -INFINITY;
      if (need_mask) {
        // element (c, e) is key kv0 + 4 hh + k(c, e), k = 32c + (e & 3) + 8 (e >> 2):
        // valid while k < lim (lane constant per tile)
        int lim = p.Sk - kv0 - 4 * hh;
        if (CAUSAL) lim = min(lim, qrow + offs - kv0 - 4 * hh + 1);
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int e = 0; e < 16; ++e)
            if (32 * c + (e & 3) + 8 * (e >> 2) >= lim) s[c][e] = -INFINITY;
      }
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int e = 0; e < 16; ++e) tmax = fmaxf(tmax, s[c][e]);
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64)) * p.scale_log2;
      // lazy rescaling: keep a stale running max unless some row's max grew by more
      // than 2^8 (exp2 values stay <= 256, safe in fp32 sums and bf16 P); the O
      // rescale then runs on a small fraction of tiles
      float alpha = 1.f;
      if (__any(tmax > m + 8.f)) {
        const float mnew = fmaxf(m, tmax);
        alpha = __builtin_amdgcn_exp2f(m - mnew);
        m = mnew;
      }
      const float mnew = m;
      float ps = 0.f;
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(s[c][e], p.scale_log2, -mnew));
          s[c][e] = pv;
          ps += pv;
        }
      lsum = lsum * alpha + ps;
      if (__any(alpha != 1.f)) {
#pragma unroll
        for (int i = 0; i < DB; ++i)
#pragma unroll
          for (int e = 0; e < 16; ++e) oacc[i][e] *= alpha;
      }
      // O^T += V^T P^T over 4 k-steps of 16 kv
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        const int c = st >> 1, half = st & 1;
        const bf8v pf = pack_p(s[c], 8 * half);
        const int rowb = 32 * c + 16 * half + 4 * (g >> 1) + gq;
#pragma unroll
        for (int db = 0; db < DB; ++db) {
          const int colb = (32 * db + 16 * (g & 1) + 4 * gp) * 2;
          const s4v lo = tr_read(Vs, v_off_bytes<D>(rowb, colb));
          const s4v hi = tr_read(Vs, v_off_bytes<D>(rowb + 8, colb));
          oacc[db] = mfma32(cat_tr(lo, hi), pf, oacc[db]);
        }
      }
    }
    // stage (t+1)&1 was last read in iteration t-1, which every wave finished
    // before the barrier that closed it
    if (t + 1 < nt) store_lds((t + 1) & 1);
    __syncthreads();
  }

  const float ltot = lsum + __shfl_xor(lsum, 32, 64);
  const float inv = ltot > 0.f ? 1.f / ltot : 0.f;
  if (qrow < p.Sq) {
    u16* op = p.o + (long)b * p.o_bs + (long)h * p.o_hs + (long)qrow * p.o_ss;
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int e4 = 0; e4 < 4; ++e4) {
        const int d = 32 * db + 8 * e4 + 4 * hh;
        u16x4 o4;
#pragma unroll
        for (int j = 0; j < 4; ++j) o4[j] = f2bf(oacc[db][4 * e4 + j] * inv);
        *reinterpret_cast<u16x4*>(op + d) = o4;
      }
    if (hh == 0)
      p.lse[((long)b * p.Hq + h) * p.Sq + qrow] =
          ltot > 0.f ? (m + __log2f(ltot)) * 0.69314718056f : -INFINITY;
  }
}

// ------------------------------------------------------------------ backward
struct BwdParams {
  const u16 *q, *k, *v, *o, *dout;
  const float* lse;  // [B, Hq, Sq]
  float* delta;      // [B, Hq, Sq]
  float* dq_acc;     // [B, Sq, Hq, D] fp32
  float* dq_part;    // v4: per-key-block dQ partials [nkb, B, Hq, Sq, D] bf16 bits (or null)
  u16 *dk, *dv;      // [B, Sk, Hq, D] (expanded per q-head for GQA)
  long q_bs, q_ss, q_hs, k_bs, k_ss, k_hs, v_bs, v_ss, v_hs, o_bs, o_ss, o_hs, do_bs, do_ss, do_hs;
  long dk_bs, dk_ss, dk_hs;
  int B, Sq, Sk, Hq, Hkv;
  float scale;       // softmax scale
  float scale_log2;  // scale * log2(e)
};

// delta[b,h,q] = sum_d dO * O ; 16 lanes per row (8 elems each for D=128)
template <int D>
__global__ void fa_bwd_pre_kernel(BwdParams p) {
  constexpr int LPR = D / 8;  // lanes per row
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long row = gid / LPR;  // over B*Hq*Sq, ordered (b, h, q)
  const int c = (int)(gid % LPR);
  const long total = (long)p.B * p.Hq * p.Sq;
  float s = 0.f;
  if (row < total) {
    const long q = row % p.Sq;
    const long bh = row / p.Sq;
    const int h = (int)(bh % p.Hq), b = (int)(bh / p.Hq);
    float a[8], d[8];
    load8(p.o + (long)b * p.o_bs + q * p.o_ss + (long)h * p.o_hs + c * 8, a);
    load8(p.dout + (long)b * p.do_bs + q * p.do_ss + (long)h * p.do_hs + c * 8, d);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += a[j] * d[j];
  }
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (row < total && c == 0) p.delta[row] = s;
  // fused zero-init of this row's fp32 dQ accumulator ([B, Sq, Hq, D])
  if (row < total && p.dq_acc != nullptr) {  // null: v4 (the reduce writes every element)
    const long q = row % p.Sq;
    const long bh = row / p.Sq;
    const int h = (int)(bh % p.Hq), b = (int)(bh / p.Hq);
    float* dq = p.dq_acc + (((long)b * p.Sq + q) * p.Hq + h) * D + c * 8;
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    *reinterpret_cast<f32x4*>(dq) = z;
    *reinterpret_cast<f32x4*>(dq + 4) = z;
  }
}

template <int D, bool CAUSAL>
__global__ __launch_bounds__(256, 1) void fa_bwd_kernel(BwdParams p) {
  constexpr int BK = 128, BQ = 32;
  constexpr int KS = D / 16, DB = D / 32;
  constexpr int KCH = D / 8;
  // LDS: K [BK][D] dual image | Q [BQ][D] | dO [BQ][D] | dS^T [BK][BQ] | lse2, delta [BQ]
  constexpr int K_BYTES = BK * D * 2, Q_BYTES = BQ * D * 2, DS_BYTES = BK * BQ * 2;
  __shared__ __attribute__((aligned(16))) char smem[K_BYTES + 2 * Q_BYTES + DS_BYTES + 2 * BQ * 4];
  char* Ks = smem;
  char* Qs = Ks + K_BYTES;
  char* Os = Qs + Q_BYTES;
  char* DSs = Os + Q_BYTES;
  float* L2s = (float*)(DSs + DS_BYTES);
  float* DLs = L2s + BQ;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int h = blockIdx.x, b = blockIdx.y;
  const int kt = blockIdx.z;  // causal: early key tiles carry the most query tiles -> dispatch first
  const int kvh = h / (p.Hq / p.Hkv);
  const long n0 = (long)kt * BK;
  const long offs = CAUSAL ? (long)p.Sk - p.Sq : 0;

  const u16* qp = p.q + (long)b * p.q_bs + (long)h * p.q_hs;
  const u16* dop = p.dout + (long)b * p.do_bs + (long)h * p.do_hs;
  const u16* kp = p.k + (long)b * p.k_bs + (long)kvh * p.k_hs;
  const u16* vp = p.v + (long)b * p.v_bs + (long)kvh * p.v_hs;
  const float* lsep = p.lse + ((long)b * p.Hq + h) * p.Sq;
  const float* dlp = p.delta + ((long)b * p.Hq + h) * p.Sq;
  float* dqp = p.dq_acc + (long)b * p.Sq * p.Hq * D + (long)h * D;  // row stride Hq*D

  // K tile -> LDS (dual image)
  for (int idx = tid; idx < BK * KCH; idx += 256) {
    const int row = idx / KCH, ch = idx % KCH;
    const long kr = n0 + row;
    u16x8 t = {0, 0, 0, 0, 0, 0, 0, 0};
    if (kr < p.Sk) t = *reinterpret_cast<const u16x8*>(kp + kr * p.k_ss + ch * 8);
    *reinterpret_cast<u16x8*>(Ks + dual_off<D>(row, ch * 16)) = t;
  }
  // V fragments (B operand of dP = dO V^T): lane holds V[kv = 32w + r][16ks + 8hh + j]
  bf8v vf[KS];
  const long mykv = n0 + 32 * w + r;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    u16x8 t = {0, 0, 0, 0, 0, 0, 0, 0};
    if (mykv < p.Sk) t = *reinterpret_cast<const u16x8*>(vp + mykv * p.v_ss + ks * 16 + hh * 8);
    vf[ks] = as_bf8(t);
  }

  f32x16 dk[DB], dv[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) { dk[i][e] = 0.f; dv[i][e] = 0.f; }

  long qstart = 0;
  if (CAUSAL) qstart = max(0L, n0 - offs);
  qstart = (qstart / BQ) * BQ;
  const int g = lane >> 4, gi = lane & 15, gq = gi >> 2, gp = gi & 3;
  const int wkv = 32 * w;  // this wave's key offset inside the tile

  for (long qt0 = qstart; qt0 < p.Sq; qt0 += BQ) {
    // stage Q, dO tiles + row constants
    for (int idx = tid; idx < BQ * KCH; idx += 256) {
      const int row = idx / KCH, ch = idx % KCH;
      const long qr = qt0 + row;
      u16x8 a = {0, 0, 0, 0, 0, 0, 0, 0}, d = a;
      if (qr < p.Sq) {
        a = *reinterpret_cast<const u16x8*>(qp + qr * p.q_ss + ch * 8);
        d = *reinterpret_cast<const u16x8*>(dop + qr * p.do_ss + ch * 8);
      }
      *reinterpret_cast<u16x8*>(Qs + dual_off<D>(row, ch * 16)) = a;
      *reinterpret_cast<u16x8*>(Os + dual_off<D>(row, ch * 16)) = d;
    }
    if (tid < BQ) {
      const long qr = qt0 + tid;
      L2s[tid] = qr < p.Sq ? lsep[qr] * 1.44269504089f : 0.f;
      DLs[tid] = qr < p.Sq ? dlp[qr] : 0.f;
    }
    __syncthreads();

    const bool wave_active = !(CAUSAL && (n0 + wkv > qt0 + BQ - 1 + offs)) && (n0 + wkv < p.Sk);
    f32x16 sacc, dpacc;
    if (wave_active) {
#pragma unroll
      for (int e = 0; e < 16; ++e) { sacc[e] = 0.f; dpacc[e] = 0.f; }
      // S = Q K^T (A = Q rows, B = K rows of this wave's keys), dP = dO V^T
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const u16x8 qa = *reinterpret_cast<const u16x8*>(Qs + dual_off<D>(r, (2 * ks + hh) * 16));
        const u16x8 kb = *reinterpret_cast<const u16x8*>(Ks + dual_off<D>(wkv + r, (2 * ks + hh) * 16));
        sacc = mfma32(as_bf8(qa), as_bf8(kb), sacc);
        const u16x8 oa = *reinterpret_cast<const u16x8*>(Os + dual_off<D>(r, (2 * ks + hh) * 16));
        dpacc = mfma32(as_bf8(oa), vf[ks], dpacc);
      }
      // P and dS; rows (queries) in registers, key on the lane
      const long kv = mykv;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int qi = (e & 3) + 8 * (e >> 2) + 4 * hh;
        const long q = qt0 + qi;
        float pv = exp2f(sacc[e] * p.scale_log2 - L2s[qi]);
        if (q >= p.Sq || kv >= p.Sk || (CAUSAL && kv > q + offs)) pv = 0.f;
        sacc[e] = pv;
        dpacc[e] = pv * (dpacc[e] - DLs[qi]) * p.scale;
      }
      // dV^T += dO^T P ; dK^T += Q^T dS   (sum over the 32 queries: 2 k-steps)
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const bf8v pf = pack_p(sacc, 8 * st);
        const bf8v sf = pack_p(dpacc, 8 * st);
        const int rowb = 16 * st + 4 * (g >> 1) + gq;
#pragma unroll
        for (int db = 0; db < DB; ++db) {
          const int colb = (32 * db + 16 * (g & 1) + 4 * gp) * 2;
          const bf8v oa = cat_tr(tr_read(Os, dual_off<D>(rowb, colb)), tr_read(Os, dual_off<D>(rowb + 8, colb)));
          dv[db] = mfma32(oa, pf, dv[db]);
          const bf8v qa = cat_tr(tr_read(Qs, dual_off<D>(rowb, colb)), tr_read(Qs, dual_off<D>(rowb + 8, colb)));
          dk[db] = mfma32(qa, sf, dk[db]);
        }
      }
      // dS^T -> LDS: [key][query] with 64-B rows; lane writes 4 consecutive queries
#pragma unroll
      for (int e4 = 0; e4 < 4; ++e4) {
        u16x4 v4;
#pragma unroll
        for (int j = 0; j < 4; ++j) v4[j] = f2bf(dpacc[4 * e4 + j]);
        *reinterpret_cast<u16x4*>(DSs + (wkv + r) * (BQ * 2) + (8 * e4 + 4 * hh) * 2) = v4;
      }
    } else {
#pragma unroll
      for (int e4 = 0; e4 < 4; ++e4)
        *reinterpret_cast<u16x4*>(DSs + (wkv + r) * (BQ * 2) + (8 * e4 + 4 * hh) * 2) = u16x4{0, 0, 0, 0};
    }
    __syncthreads();
    // dQ[q, d-block db] = sum over the tile's 128 keys dS[q, kv] K[kv, d]; wave w owns
    // d-blocks w, w + 4, ... (DB = 2 / 4 / 8 for D = 64 / 128 / 256)
    for (int db = w; db < DB; db += 4) {
      f32x16 dq;
#pragma unroll
      for (int e = 0; e < 16; ++e) dq[e] = 0.f;
      const int kend = CAUSAL ? (int)min((long)BK, max(0L, qt0 + BQ + offs - n0)) : BK;
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        if (ks * 16 < kend) {
          // A = dS[q = r][kv = 16ks + 8hh + j] from dS^T via transposed reads
          const int arow = 16 * ks + 8 * hh + gq;  // kv rows for this lane's group
          const int acol = (16 * (g & 1) + 4 * gp) * 2;
          const bf8v af = cat_tr(tr_read(DSs, arow * (BQ * 2) + acol),
                                 tr_read(DSs, (arow + 4) * (BQ * 2) + acol));
          // B = K[kv = 16ks + 8hh + j][d = 32db + r]
          const int brow = 16 * ks + 8 * hh + gq;
          const int bcol = (32 * db + 16 * (g & 1) + 4 * gp) * 2;
          const bf8v bfk = cat_tr(tr_read(Ks, dual_off<D>(brow, bcol)), tr_read(Ks, dual_off<D>(brow + 4, bcol)));
          dq = mfma32(af, bfk, dq);
        }
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int qi = (e & 3) + 8 * (e >> 2) + 4 * hh;
        const long q = qt0 + qi;
        if (q < p.Sq) atomicAdd(dqp + q * ((long)p.Hq * D) + 32 * db + r, dq[e]);
      }
    }
    __syncthreads();
  }

  // write dK, dV (per q-head layout [B, Sk, Hq, D])
  if (mykv < p.Sk) {
    u16* dkp = p.dk + (long)b * p.dk_bs + mykv * p.dk_ss + (long)h * p.dk_hs;
    u16* dvp = p.dv + (long)b * p.dk_bs + mykv * p.dk_ss + (long)h * p.dk_hs;
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int e4 = 0; e4 < 4; ++e4) {
        const int d = 32 * db + 8 * e4 + 4 * hh;
        u16x4 a4, b4;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          a4[j] = f2bf(dk[db][4 * e4 + j]);
          b4[j] = f2bf(dv[db][4 * e4 + j]);
        }
        *reinterpret_cast<u16x4*>(dkp + d) = a4;
        *reinterpret_cast<u16x4*>(dvp + d) = b4;
      }
  }
}

// LDS-only workgroup barrier: waits for this wave's LDS traffic, not for its
// outstanding global loads / fire-and-forget dQ atomics (which __syncthreads'
// release fence would drain with vmcnt(0)).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Pipelined backward: same math and per-wave ownership as fa_bwd_kernel, but
//   * the next query tile (Q, dO, lse, delta) is prefetched into registers while the
//     current one is on the MFMAs, and written into the other half of a
//     double-buffered LDS stage -> ONE barrier per query tile;
//   * this wave's K rows are also kept in registers (B operand of S), so the S GEMM
//     reads only Q from LDS;
//   * NOATOMIC is a measurement probe (plain stores instead of dQ atomics).
template <int D, bool CAUSAL, bool NOATOMIC>
__global__ __launch_bounds__(256, 1) void fa_bwd_kernel2(BwdParams p) {
  constexpr int BK = 128, BQ = 32;
  constexpr int KS = D / 16, DB = D / 32;
  constexpr int KCH = D / 8;
  constexpr int NQ = BQ * KCH / 256;  // 16-B chunks per thread per Q (and dO) tile
  constexpr int K_BYTES = BK * D * 2, Q_BYTES = BQ * D * 2, DS_BYTES = BK * BQ * 2;
  constexpr int STAGE = 2 * Q_BYTES + DS_BYTES + 2 * BQ * 4;
  __shared__ __attribute__((aligned(16))) char smem[K_BYTES + 2 * STAGE];
  char* Ks = smem;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 31, hh = lane >> 5;
  const int h = blockIdx.x, b = blockIdx.y;
  const int kt = blockIdx.z;
  const int kvh = h / (p.Hq / p.Hkv);
  const long n0 = (long)kt * BK;
  const long offs = CAUSAL ? (long)p.Sk - p.Sq : 0;

  const u16* qp = p.q + (long)b * p.q_bs + (long)h * p.q_hs;
  const u16* dop = p.dout + (long)b * p.do_bs + (long)h * p.do_hs;
  const u16* kp = p.k + (long)b * p.k_bs + (long)kvh * p.k_hs;
  const u16* vp = p.v + (long)b * p.v_bs + (long)kvh * p.v_hs;
  const float* lsep = p.lse + ((long)b * p.Hq + h) * p.Sq;
  const float* dlp = p.delta + ((long)b * p.Hq + h) * p.Sq;
  float* dqp = p.dq_acc + (long)b * p.Sq * p.Hq * D + (long)h * D;

  long qstart = 0;
  if (CAUSAL) qstart = max(0L, n0 - offs);
  qstart = (qstart / BQ) * BQ;

  // Buffer descriptors (wave-uniform, 32-bit offsets): no 64-bit per-lane pointers live
  // across the loop, and the hardware range check zero-fills / drops the rows >= Sq of
  // a ragged last query tile (host guarantees every extent fits in 32 bits).
  const auto q_rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)qp, 0, (int)(unsigned)(((long)(p.Sq - 1) * p.q_ss + D) * 2), 0x00020000);
  const auto do_rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)dop, 0, (int)(unsigned)(((long)(p.Sq - 1) * p.do_ss + D) * 2), 0x00020000);
  const auto lse_rs = __builtin_amdgcn_make_buffer_rsrc((void*)lsep, 0, p.Sq * 4, 0x00020000);
  const auto dl_rs = __builtin_amdgcn_make_buffer_rsrc((void*)dlp, 0, p.Sq * 4, 0x00020000);
  const long dq_rstride = (long)p.Hq * D;
  const auto dq_rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)dqp, 0, (int)(unsigned)(((long)(p.Sq - 1) * dq_rstride + D) * 4), 0x00020000);
  unsigned qoff[NQ], ooff[NQ];
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const int idx = tid + 256 * i, row = idx / KCH, ch = idx % KCH;
    qoff[i] = (unsigned)(row * p.q_ss * 2 + ch * 16);
    ooff[i] = (unsigned)(row * p.do_ss * 2 + ch * 16);
  }

  u16x8 qst[NQ], ost[NQ];
  float lst = 0.f, dst = 0.f;
  auto load_regs = [&](long qt0) {
    const unsigned qb = (unsigned)(qt0 * p.q_ss * 2), ob = (unsigned)(qt0 * p.do_ss * 2);
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
      qst[i] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(q_rs, (int)(qb + qoff[i]), 0, 0));
      ost[i] = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(do_rs, (int)(ob + ooff[i]), 0, 0));
    }
    const int lo = (int)(qt0 + (tid & (BQ - 1))) * 4;
    // (raw values: scaling here would make the issuing code wait on the prefetch)
    lst = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(lse_rs, lo, 0, 0));
    dst = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(dl_rs, lo, 0, 0));
  };
  auto store_lds = [&](int buf) {
    char* st = smem + K_BYTES + buf * STAGE;
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
      const int idx = tid + 256 * i, row = idx / KCH, ch = idx % KCH;
      *reinterpret_cast<u16x8*>(st + dual_off<D>(row, ch * 16)) = qst[i];
      *reinterpret_cast<u16x8*>(st + Q_BYTES + dual_off<D>(row, ch * 16)) = ost[i];
    }
    if (tid < BQ) {
      float* l2 = (float*)(st + 2 * Q_BYTES + DS_BYTES);
      l2[tid] = lst * 1.44269504089f;
      l2[BQ + tid] = dst;
    }
  };

  load_regs(qstart);
  // K tile -> LDS (dual image, read transposed by the dQ GEMM)
  for (int idx = tid; idx < BK * KCH; idx += 256) {
    const int row = idx / KCH, ch = idx % KCH;
    const long kr = n0 + row;
    u16x8 t = {0, 0, 0, 0, 0, 0, 0, 0};
    if (kr < p.Sk) t = *reinterpret_cast<const u16x8*>(kp + kr * p.k_ss + ch * 8);
    *reinterpret_cast<u16x8*>(Ks + dual_off<D>(row, ch * 16)) = t;
  }
  // this wave's K and V rows as MFMA B operands: lane holds X[kv = 32w + r][16ks + 8hh + j]
  bf8v vf[KS], kf[KS];
  const long mykv = n0 + 32 * w + r;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    u16x8 t = {0, 0, 0, 0, 0, 0, 0, 0}, u = t;
    if (mykv < p.Sk) {
      t = *reinterpret_cast<const u16x8*>(vp + mykv * p.v_ss + ks * 16 + hh * 8);
      u = *reinterpret_cast<const u16x8*>(kp + mykv * p.k_ss + ks * 16 + hh * 8);
    }
    vf[ks] = as_bf8(t);
    kf[ks] = as_bf8(u);
  }
  store_lds(0);
  lds_barrier();

  f32x16 dk[DB], dv[DB];
#pragma unroll
  for (int i = 0; i < DB; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) { dk[i][e] = 0.f; dv[i][e] = 0.f; }

  const int g = lane >> 4, gi = lane & 15, gq = gi >> 2, gp = gi & 3;
  const int wkv = 32 * w;
  // dQ of query tile t is flushed (atomics) at the start of iteration t + 1, so a whole
  // compute phase separates the atomics from the reuse of their source registers
  // (otherwise the next MFMA waits on vmcnt(0) for every atomic in flight).
  f32x16 dq_prev;
#pragma unroll
  for (int e = 0; e < 16; ++e) dq_prev[e] = 0.f;
  auto flush_dq = [&](long qt_prev) {
    // rows >= Sq fall outside dq_rs and are dropped by the range check
    const unsigned base = (unsigned)(((qt_prev + 4 * hh) * dq_rstride + 32 * w + r) * 4);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int voff = (int)(base + (unsigned)(((e & 3) + 8 * (e >> 2)) * dq_rstride * 4));
      if (NOATOMIC) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(dq_prev[e]), dq_rs, voff, 0, 0);
      else __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(dq_prev[e], dq_rs, voff, 0, 0);
    }
  };
  int buf = 0;
  for (long qt0 = qstart; qt0 < p.Sq; qt0 += BQ, buf ^= 1) {
    // unconditional prefetch: past the end the range check returns zeros
    load_regs(qt0 + BQ);
    __builtin_amdgcn_sched_barrier(0);
    if (w < DB && qt0 > qstart) flush_dq(qt0 - BQ);
    char* Qs = smem + K_BYTES + buf * STAGE;
    char* Os = Qs + Q_BYTES;
    char* DSs = Os + Q_BYTES;
    const float* L2s = (const float*)(DSs + DS_BYTES);
    const float* DLs = L2s + BQ;

    // Branch-free body (uniform control flow keeps dK/dV/dQ accumulators in place):
    // fully masked waves on the causal diagonal just accumulate zeros.
    f32x16 sacc, dpacc;
#pragma unroll
    for (int e = 0; e < 16; ++e) { sacc[e] = 0.f; dpacc[e] = 0.f; }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const u16x8 qa = *reinterpret_cast<const u16x8*>(Qs + dual_off<D>(r, (2 * ks + hh) * 16));
      sacc = mfma32(as_bf8(qa), kf[ks], sacc);
      const u16x8 oa = *reinterpret_cast<const u16x8*>(Os + dual_off<D>(r, (2 * ks + hh) * 16));
      dpacc = mfma32(as_bf8(oa), vf[ks], dpacc);
    }
    {
      // element e holds query qb + c_e (c_e = (e&3) + 8(e>>2)); valid iff lo <= c_e < hi
      const int qb = (int)qt0 + 4 * hh;
      const int lo = CAUSAL ? (int)(mykv - qb - offs) : 0;
      const int hi = mykv < p.Sk ? p.Sq - qb : -1;
      const unsigned span = hi > lo ? (unsigned)(hi - lo) : 0u;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int c = (e & 3) + 8 * (e >> 2);
        const int qi = c + 4 * hh;
        float pv = __builtin_amdgcn_exp2f(sacc[e] * p.scale_log2 - L2s[qi]);
        pv = ((unsigned)(c - lo) < span) ? pv : 0.f;
        sacc[e] = pv;
        dpacc[e] = pv * (dpacc[e] - DLs[qi]) * p.scale;
      }
    }
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const bf8v pf = pack_p(sacc, 8 * st);
      const bf8v sf = pack_p(dpacc, 8 * st);
      const int rowb = 16 * st + 4 * (g >> 1) + gq;
#pragma unroll
      for (int db = 0; db < DB; ++db) {
        const int colb = (32 * db + 16 * (g & 1) + 4 * gp) * 2;
        const bf8v oa = cat_tr(tr_read(Os, dual_off<D>(rowb, colb)), tr_read(Os, dual_off<D>(rowb + 8, colb)));
        dv[db] = mfma32(oa, pf, dv[db]);
        const bf8v qa = cat_tr(tr_read(Qs, dual_off<D>(rowb, colb)), tr_read(Qs, dual_off<D>(rowb + 8, colb)));
        dk[db] = mfma32(qa, sf, dk[db]);
      }
    }
#pragma unroll
    for (int e4 = 0; e4 < 4; ++e4) {
      u16x4 v4;
#pragma unroll
      for (int j = 0; j < 4; ++j) v4[j] = f2bf(dpacc[4 * e4 + j]);
      *reinterpret_cast<u16x4*>(DSs + (wkv + r) * (BQ * 2) + (8 * e4 + 4 * hh) * 2) = v4;
    }
    // the other stage's Q/dO/lse/delta were last read before the previous barrier
    store_lds(buf ^ 1);
    // keep the flushed dQ registers allocated across the compute phase (see flush_dq)
#pragma unroll
    for (int e = 0; e < 16; ++e) asm volatile("" ::"v"(dq_prev[e]));
    lds_barrier();
    if (w < DB) {
      f32x16 dq;
#pragma unroll
      for (int e = 0; e < 16; ++e) dq[e] = 0.f;
      // the K-image swizzle only uses row bits 0..3, so the 16-row k-step offsets are
      // plain immediates on two per-lane base addresses
      const int arow0 = 8 * hh + gq;
      const int acol = (16 * (g & 1) + 4 * gp) * 2;
      const int bcol = (32 * w + 16 * (g & 1) + 4 * gp) * 2;
      const char* kb0 = Ks + dual_off<D>(arow0, bcol);
      const char* kb1 = Ks + dual_off<D>(arow0 + 4, bcol);
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        const int arow = 16 * ks + arow0;
        const bf8v af = cat_tr(tr_read(DSs, arow * (BQ * 2) + acol),
                               tr_read(DSs, (arow + 4) * (BQ * 2) + acol));
        const bf8v bfk = cat_tr(tr_read(kb0, ks * 16 * D * 2), tr_read(kb1, ks * 16 * D * 2));
        dq = mfma32(af, bfk, dq);
      }
      dq_prev = dq;
    }
  }
  if (w < DB && qstart < p.Sq) {
    const long last = qstart + ((p.Sq - 1 - qstart) / BQ) * BQ;
    flush_dq(last);
  }

  if (mykv < p.Sk) {
    u16* dkp = p.dk + (long)b * p.dk_bs + mykv * p.dk_ss + (long)h * p.dk_hs;
    u16* dvp = p.dv + (long)b * p.dk_bs + mykv * p.dk_ss + (long)h * p.dk_hs;
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int e4 = 0; e4 < 4; ++e4) {
        const int d = 32 * db + 8 * e4 + 4 * hh;
        u16x4 a4, b4;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          a4[j] = f2bf(dk[db][4 * e4 + j]);
          b4[j] = f2bf(dv[db][4 * e4 + j]);
        }
        *reinterpret_cast<u16x4*>(dkp + d) = a4;
        *reinterpret_cast<u16x4*>(dvp + d) = b4;
      }
  }
}

// ---------------------------------------------------------------------------------
// Backward v3: 8 waves x 16 keys (128 keys per workgroup), MFMA 16x16x32, TWO waves
// per SIMD.  v2 (fa_bwd_kernel2) keeps 32 keys x D=128 dK/dV accumulators per wave
// (128 regs) plus K/V operand registers -> 365 VGPR+AGPR, one wave per SIMD, and its
// per-tile chain (S/dP MFMAs -> exp -> dV/dK -> dS -> barrier -> dQ -> atomics) runs
// with nothing to overlap it (~13 % MFMA busy).  Here a wave owns 16 keys:
//   * S = Q K^T and dP = dO V^T with queries on the MFMA rows and the wave's keys on
//     the lanes: Q/dO rows are b128 LDS reads, K/V^T fragments stay in 32 registers;
//   * the S/dP accumulators (q = 16qt + 4g + i on registers, key on lane) ARE the A
//     operands of dV = P^T dO and dK = dS^T Q once the 32-query k-slots are permuted
//     (slot (g, j) <-> q = 4g + j for j < 4, 16 + 4g + j - 4 otherwise); the dO / Q
//     B fragments come from two ds_read_b64_tr_b16 of the same permuted rows;
//   * dS goes to LDS as [key][q] (two ds_write_b64 per lane) and dQ (32 q x 16 d per
//     wave) reads it back transposed, K from the dual-use image; fp32 atomics on dQ
//     are deferred by one tile as in v2.
// Accumulators: dK/dV 64 regs, S/dP 16, dQ 2x8 -> fits 256 VGPRs (2 waves / SIMD).
typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));
__device__ __forceinline__ f32x4 mfma16(bf16x8v a, bf16x8v b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <bool CAUSAL, bool PARTIAL>
__global__ __launch_bounds__(512, 2) void fa_bwd_kernel3(BwdParams p) {
  constexpr int D = 128, BK = 128, BQ = 32;
  constexpr int KCH = D / 8;                     // 16-B chunks per 128-d row
  constexpr int K_BYTES = BK * D * 2;            // 32 KB  K image (dual layout)
  constexpr int Q_BYTES = BQ * D * 2;            // 8 KB
  constexpr int DS_BYTES = BK * BQ * 2;          // 8 KB   dS^T [key][q]
  constexpr int STAGE = 2 * Q_BYTES + DS_BYTES + 2 * BQ * 4;
  // K and V images (dual layout): K feeds S (row reads) and dQ (transposed reads),
  // V feeds dP; keeping the wave's K/V fragments in LDS instead of 32 registers is
  // what lets the two prefetch register sets fit in 256 VGPRs.
  __shared__ __attribute__((aligned(16))) char smem[2 * K_BYTES + 2 * STAGE];
  char* Ks = smem;
  char* Vs = smem + K_BYTES;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int li = lane & 15, g = lane >> 4;       // MFMA16 lane row / lane group
  const int gq = li >> 2, gp = li & 3;           // tr-read block row / column quad
  const int h = blockIdx.x, b = blockIdx.y, kt = blockIdx.z;
  const int kvh = h / (p.Hq / p.Hkv);
  const long n0 = (long)kt * BK;
  const long offs = CAUSAL ? (long)p.Sk - p.Sq : 0;

  const u16* qp = p.q + (long)b * p.q_bs + (long)h * p.q_hs;
  const u16* dop = p.dout + (long)b * p.do_bs + (long)h * p.do_hs;
  const u16* kp = p.k + (long)b * p.k_bs + (long)kvh * p.k_hs;
  const u16* vp = p.v + (long)b * p.v_bs + (long)kvh * p.v_hs;
  const float* lsep = p.lse + ((long)b * p.Hq + h) * p.Sq;
  const float* dlp = p.delta + ((long)b * p.Hq + h) * p.Sq;
  float* dqp = p.dq_acc + (long)b * p.Sq * p.Hq * D + (long)h * D;

  long qstart = 0;
  if (CAUSAL) qstart = max(0L, n0 - offs);
  qstart = (qstart / BQ) * BQ;

  const auto q_rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)qp, 0, (int)(unsigned)(((long)(p.Sq - 1) * p.q_ss + D) * 2), 0x00020000);
  const auto do_rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)dop, 0, (int)(unsigned)(((long)(p.Sq - 1) * p.do_ss + D) * 2), 0x00020000);
  const auto lse_rs = __builtin_amdgcn_make_buffer_rsrc((void*)lsep, 0, p.Sq * 4, 0x00020000);
  const auto dl_rs = __builtin_amdgcn_make_buffer_rsrc((void*)dlp, 0, p.Sq * 4, 0x00020000);
  const long dq_rstride = (long)p.Hq * D;
  const auto dq_rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)dqp, 0, (int)(unsigned)(((long)(p.Sq - 1) * dq_rstride + D) * 4), 0x00020000);

  // one 16-B chunk of Q and of dO per thread per tile (32 rows x 16 chunks = 512)
  const int srow = tid / KCH, sch = tid % KCH;
  const unsigned qoff = (unsigned)(srow * p.q_ss * 2 + sch * 16);
  const unsigned ooff = (unsigned)(srow * p.do_ss * 2 + sch * 16);
  // Two prefetch register sets (A/B): tile t+2 is loaded while tile t computes, so
  // the vmcnt wait before staging a tile only drains VM ops issued >= 2 tiles ago --
  // the dQ flush (memory-side atomics / stores, ~3k cycles in vmcnt under load) of
  // the previous tile no longer sits in front of the prefetch it must wait for.
  struct Pf {
    u16x8 q, o;
    float l, d;
  };
  Pf pa_, pb_;
  auto load_regs = [&](Pf& r, long qt0) {
    r.q = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                        q_rs, (int)((unsigned)(qt0 * p.q_ss * 2) + qoff), 0, 0));
    r.o = __builtin_bit_cast(u16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                        do_rs, (int)((unsigned)(qt0 * p.do_ss * 2) + ooff), 0, 0));
    const int lo = (int)(qt0 + (tid & (BQ - 1))) * 4;
    r.l = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(lse_rs, lo, 0, 0));
    r.d = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(dl_rs, lo, 0, 0));
  };
  auto store_lds = [&](const Pf& r, int buf) {
    char* st = smem + 2 * K_BYTES + buf * STAGE;
    *reinterpret_cast<u16x8*>(st + dual_off<D>(srow, sch * 16)) = r.q;
    *reinterpret_cast<u16x8*>(st + Q_BYTES + dual_off<D>(srow, sch * 16)) = r.o;
    // every thread writes its (tid & 31) slot (16 identical writers per slot): no
    // branch, so hipcc's vmcnt accounting for the prefetch stays static
    float* l2 = (float*)(st + 2 * Q_BYTES + DS_BYTES);
    l2[tid & (BQ - 1)] = r.l * 1.44269504089f;
    l2[BQ + (tid & (BQ - 1))] = r.d;
  };

  load_regs(pa_, qstart);
  load_regs(pb_, qstart + BQ);
  for (int idx = tid; idx < BK * KCH; idx += 512) {
    const int row = idx / KCH, ch = idx % KCH;
    const long kr = n0 + row;
    u16x8 t = {0, 0, 0, 0, 0, 0, 0, 0}, u = t;
    if (kr < p.Sk) {
      t = *reinterpret_cast<const u16x8*>(kp + kr * p.k_ss + ch * 8);
      u = *reinterpret_cast<const u16x8*>(vp + kr * p.v_ss + ch * 8);
    }
    *reinterpret_cast<u16x8*>(Ks + dual_off<D>(row, ch * 16)) = t;
    *reinterpret_cast<u16x8*>(Vs + dual_off<D>(row, ch * 16)) = u;
  }
  const long mykey = n0 + 16 * w + li;
  store_lds(pa_, 0);
  lds_barrier();

  f32x4 dk[8], dv[8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) { dk[i][e] = 0.f; dv[i][e] = 0.f; }
  // dQ element (qt, i): row q = 16qt + 4g + i, column d = 16w + li.
  // PARTIAL (v4): plain stores of this key block's partial into its own [Sq][D] slab
  // (HBM store rate, ~6 TB/s) instead of fp32 atomics (~1.3 TB/s chip-wide, which
  // bound v2/v3: 16 KB of adds per 128x32 tile); fa_bwd_dq_reduce sums the slabs.
  // slabs are bf16: each partial is an fp32 sum over 128 keys rounded once; the
  // reduce adds <= Sk/128 of them in fp32 (halves the slab store + reduce traffic)
  const auto part_rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(PARTIAL ? (u16*)p.dq_part + (((long)kt * p.B + b) * p.Hq + h) * (long)p.Sq * D : nullptr), 0,
      PARTIAL ? p.Sq * D * 2 : 0, 0x00020000);
  auto flush_dq = [&](long qt_prev, const f32x4 (&dq_prev)[2]) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const long q = qt_prev + 16 * t + 4 * g + i;
        if (PARTIAL) {
          const int poff = (int)(unsigned)((q * D + 16 * w + li) * 2);
          // (__builtin_bit_cast of an ext_vector element miscompiles to element 0 on this
          // toolchain: go through a scalar)
          const float v = dq_prev[t][i];
          __builtin_amdgcn_raw_buffer_store_b16(f2bf(v), part_rs, poff, 0, 0);
        } else {
          const int voff = (int)(unsigned)((q * dq_rstride + 16 * w + li) * 4);
          __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(dq_prev[t][i], dq_rs, voff, 0, 0);
        }
      }
  };

  // one query tile: compute on stage `buf`, prefetch tile +2 into `ld`, stage tile +1 from `st`
  auto body = [&](long qt0, int buf, Pf& ld, const Pf& stg) {
    load_regs(ld, qt0 + 2 * BQ);
    __builtin_amdgcn_sched_barrier(0);
    char* Qs = smem + 2 * K_BYTES + buf * STAGE;
    char* Os = Qs + Q_BYTES;
    char* DSs = Os + Q_BYTES;
    const float* L2s = (const float*)(DSs + DS_BYTES);
    const float* DLs = L2s + BQ;

    // ---- S = Q K^T, dP = dO V^T  (lanes: keys).  Tile t row m holds query
    // 8(m>>2) + 4t + (m&3), so lane group g's accumulator rows are queries 8g .. 8g+7
    // (t-major): the P / dS operands are then in natural k order and the dO / Q
    // transposed reads of the two groups of a 32-lane half sit 8 rows apart
    // (conflict-free on the dual image, guide T10) instead of stacked (2-way).
    f32x4 sacc[2], dpacc[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) { sacc[t][e] = 0.f; dpacc[t][e] = 0.f; }
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int r = 8 * (li >> 2) + 4 * t + (li & 3), cb = (4 * ks + g) * 16;
        // B fragments: lane holds X[key = 16w + li][32ks + 8g + j] (row read of K / V)
        const bf16x8v kfr = __builtin_bit_cast(bf16x8v, *reinterpret_cast<const u16x8*>(Ks + dual_off<D>(16 * w + li, cb)));
        const bf16x8v vfr = __builtin_bit_cast(bf16x8v, *reinterpret_cast<const u16x8*>(Vs + dual_off<D>(16 * w + li, cb)));
        const u16x8 qa = *reinterpret_cast<const u16x8*>(Qs + dual_off<D>(r, cb));
        sacc[t] = mfma16(__builtin_bit_cast(bf16x8v, qa), kfr, sacc[t]);
        const u16x8 oa = *reinterpret_cast<const u16x8*>(Os + dual_off<D>(r, cb));
        dpacc[t] = mfma16(__builtin_bit_cast(bf16x8v, oa), vfr, dpacc[t]);
      }
    // ---- P, dS (element (t, i): query qt0 + 8g + 4t + i, key mykey)
    bf16x8v pa, da;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const f32x4 l2 = *reinterpret_cast<const f32x4*>(L2s + 8 * g + 4 * t);
      const f32x4 dl = *reinterpret_cast<const f32x4*>(DLs + 8 * g + 4 * t);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const long q = qt0 + 8 * g + 4 * t + i;
        float pv = __builtin_amdgcn_exp2f(sacc[t][i] * p.scale_log2 - l2[i]);
        bool ok = q < p.Sq && mykey < p.Sk;
        if (CAUSAL) ok = ok && (mykey <= q + offs);
        pv = ok ? pv : 0.f;
        const float ds = pv * (dpacc[t][i] - dl[i]) * p.scale;
        pa[4 * t + i] = (__bf16)pv;
        da[4 * t + i] = (__bf16)ds;
      }
    }
    // ---- dV += P^T dO, dK += dS^T Q  (k-slot (g, j) <-> query 8g + j)
#pragma unroll
    for (int db = 0; db < 8; ++db) {
      const int colb = (16 * db + 4 * gp) * 2;
      const bf8v ob = cat_tr(tr_read(Os, dual_off<D>(8 * g + gq, colb)),
                             tr_read(Os, dual_off<D>(8 * g + 4 + gq, colb)));
      dv[db] = mfma16(pa, ob, dv[db]);
      const bf8v qb = cat_tr(tr_read(Qs, dual_off<D>(8 * g + gq, colb)),
                             tr_read(Qs, dual_off<D>(8 * g + 4 + gq, colb)));
      dk[db] = mfma16(da, qb, dk[db]);
    }
    // ---- dS^T -> LDS [key][q]: this lane's 4 consecutive queries per tile t
    // dS^T image [key][q] (64-B rows): queries 8g..8g+7 of this lane's key in one
    // 16-B store; the q column is XOR-ed with 16 on odd 8-key groups so the dQ
    // transposed reads of the two groups in a 32-lane half hit disjoint banks.
    // (bit-cast the whole vector: per-element __bf16 -> u16 casts miscompile)
    *reinterpret_cast<u16x8*>(DSs + (16 * w + li) * (BQ * 2) + ((8 * g) ^ (((li >> 3) & 1) << 4)) * 2) =
        __builtin_bit_cast(u16x8, da);
    store_lds(stg, buf ^ 1);
    lds_barrier();
    // ---- dQ[32 q x 16 d (cols 16w..)] = dS[q][keys] K[keys][d]
    f32x4 dq[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) dq[t][e] = 0.f;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int kr = 32 * ks + 8 * g + gq;
      const int kcol = (16 * w + 4 * gp) * 2;
      const bf8v kb = cat_tr(tr_read(Ks, dual_off<D>(kr, kcol)), tr_read(Ks, dual_off<D>(kr + 4, kcol)));
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int acol = ((16 * t + 4 * gp) ^ ((g & 1) << 4)) * 2;   // key group (kr >> 3) & 1 == g & 1
        const bf8v af = cat_tr(tr_read(DSs, kr * (BQ * 2) + acol), tr_read(DSs, (kr + 4) * (BQ * 2) + acol));
        dq[t] = mfma16(af, kb, dq[t]);
      }
    }
    // flushed right away: the prefetch waited on next is 2 tiles old, so these
    // memory-side atomics / stores stay in flight instead of being drained by it
    flush_dq(qt0, dq);
  };
  for (long qt0 = qstart; qt0 < p.Sq;) {
    body(qt0, 0, pa_, pb_);
    qt0 += BQ;
    if (qt0 >= p.Sq) break;
    body(qt0, 1, pb_, pa_);
    qt0 += BQ;
  }
  // ---- dK / dV: element (db, i) = key 16w + 4g + i, d = 16db + li
  u16* dkp = p.dk + (long)b * p.dk_bs + (long)h * p.dk_hs;
  u16* dvp = p.dv + (long)b * p.dk_bs + (long)h * p.dk_hs;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const long key = n0 + 16 * w + 4 * g + i;
    if (key < p.Sk) {
#pragma unroll
      for (int db = 0; db < 8; ++db) {
        dkp[key * p.dk_ss + 16 * db + li] = f2bf(dk[db][i]);
        dvp[key * p.dk_ss + 16 * db + li] = f2bf(dv[db][i]);
      }
    }
  }
}

// ---------------------------------------------------------------------------------
// Backward v5: 4 waves x 32 keys = 128 keys of one (b, head) per workgroup, ONE wave
// per SIMD, MFMA 32x32x16 throughout (v3 uses 16x16x32 on 16 keys / wave and is
// bound by LDS operand reads: a 32x32x16 MFMA reads a quarter of the operand bytes
// per multiply-add).  Per wave, for the whole sweep over 32-row query slices:
// dK^T, dV^T of its 32 keys (128 accumulator registers) and its V rows (registers).
//   S  = Q K^T and dP = dO V^T with the key on the lane (B operand = K / V rows of the
//        wave's keys; A = Q / dO rows of the slice).  The accumulators start at
//        -lse/scale and -delta, so p = exp2(scale_log2 * S) and dS = p * dP * scale
//        need no further row constants;
//   dV^T += dO^T P and dK^T += Q^T dS take P / dS straight from those accumulators as
//        B operands (register j of k-step st is query slot 16 st + 8 hh + j, which is
//        row 16 st + 8 (j >> 2) + 4 hh + (j & 3): the dO^T / Q^T A operands are two
//        4-row transposed reads of the same rows);
//   dS^T goes to LDS ([key][q], XOR-swizzled 8-B slots) and, after the slice's one
//        barrier, wave w computes dQ^T for head dims 32w..32w+31 over the block's 128
//        keys (A = K^T and B = dS^T, both transposed reads) and stores the bf16
//        partial of this key block (summed per query by fa_dq_reduce_rope).
// Every LDS operand is read two k-steps ahead of its MFMAs (three register sets,
// sched barriers stop the compiler from hoisting all reads of the unrolled loops).
// Q / dO / lse / delta of slice t+1 are loaded into registers during slice t and
// written into the other LDS stage before the barrier; dS^T is double-buffered, so
// one barrier per slice orders everything.  D = 128, Sk % 128 == 0, Sq % 32 == 0.
__device__ __forceinline__ int ds_off(int key, int q) {
  // [128 keys][32 q] bf16, 64-B rows; 8-B slot XOR-swizzled by key so the per-key
  // b64 stores of 16 consecutive keys hit distinct banks
  return key * 64 + ((((q >> 2) ^ ((key >> 1) & 7)) << 3) | ((q & 3) << 1));
}

template <bool CAUSAL>
__global__ __launch_bounds__(256, 1) void fa_bwd_kernel5(BwdParams p) {
  constexpr int D = 128, BK = 128, BQ = 32;
  constexpr int K_BYTES = BK * D * 2;            // 32 KB  K image (dual layout)
  constexpr int V_BYTES = BK * D * 2;            // 32 KB  V image (row reads only, same swizzle)
  constexpr int Q_BYTES = BQ * D * 2;            // 8 KB
  constexpr int STAGE = 2 * Q_BYTES + 2 * BQ * 4;
  constexpr int DSB = BK * BQ * 2;               // 8 KB  dS^T [key][q]
  __shared__ __attribute__((aligned(16))) char smem[K_BYTES + V_BYTES + 2 * STAGE + 2 * DSB];
  char* Ks = smem;
  char* Vs = smem + K_BYTES;
  char* stage0 = Vs + V_BYTES;
  char* dsbuf0 = stage0 + 2 * STAGE;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int G = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;  // transposed-read lane roles
  const int h = blockIdx.x, b = blockIdx.y, kb = blockIdx.z;
  const int kvh = h / (p.Hq / p.Hkv);
  const int n0 = kb * BK;
  const int offs = CAUSAL ? p.Sk - p.Sq : 0;
  const int key_w0 = n0 + 32 * w;
  const int mykey = key_w0 + l32;

  const u16* qp = p.q + (long)b * p.q_bs + (long)h * p.q_hs;
  const u16* dop = p.dout + (long)b * p.do_bs + (long)h * p.do_hs;
  const u16* kp = p.k + (long)b * p.k_bs + (long)kvh * p.k_hs;
  const u16* vp = p.v + (long)b * p.v_bs + (long)kvh * p.v_hs;
  const float* lsep = p.lse + ((long)b * p.Hq + h) * p.Sq;
  const float* dlp = p.delta + ((long)b * p.Hq + h) * p.Sq;
  u16* part = (u16*)p.dq_part + (((long)kb * p.B + b) * p.Hq + h) * (long)p.Sq * D;

  int qstart = 0;
  if (CAUSAL) qstart = max(0, n0 - offs);
  qstart = (qstart / BQ) * BQ;

  // ---- K and V images (dual layout) for the whole sweep
  for (int idx = tid; idx < BK * (D / 8); idx += 256) {
    const int row = idx >> 4, ch = idx & 15;
    const int o = dual_off<D>(row, ch * 16);
    *reinterpret_cast<u16x8*>(Ks + o) = *reinterpret_cast<const u16x8*>(kp + (long)(n0 + row) * p.k_ss + ch * 8);
    *reinterpret_cast<u16x8*>(Vs + o) = *reinterpret_cast<const u16x8*>(vp + (long)(n0 + row) * p.v_ss + ch * 8);
  }

  // ---- lane-constant LDS offsets.  dual_off's XOR depends on the row only through
  // row & 15, so every k-step / d-block / key-step variant below is one of these plus
  // a compile-time constant (an instruction immediate), not a fresh computation.
  const int dsw = ((l32 & 3) << 2) | ((l32 >> 2) & 3);     // swizzle of rows l32 and 32w + l32
  int s_off[8];                                            // chunk (2 ks + hh) of a row read
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) s_off[ks] = ((2 * ks + hh) ^ dsw) << 4;
  const int q_row = l32 * 256, k_row = (32 * w + l32) * 256;
  // transposed reads of the slice (dO^T / Q^T): rows 4(G>>1) + qq (+8) (+16 s2 = +4096)
  int t_off[4][2];
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const int r = 4 * (G >> 1) + qq + 8 * hf;
      t_off[db][hf] = dual_off<D>(r, (32 * db + 16 * (G & 1) + 4 * pp) * 2);
    }
  // dQ: K^T rows 8(G>>1) + qq (+4) (+16 ks = +4096 ks); dS^T rows likewise (+1024 ks)
  const int kr0 = 8 * (G >> 1) + qq;
  const int kcolb = (32 * w + 16 * (G & 1) + 4 * pp) * 2;
  const int qcol = 16 * (G & 1) + 4 * pp;
  const int kt_off0 = dual_off<D>(kr0, kcolb), kt_off1 = dual_off<D>(kr0 + 4, kcolb);
  const int ds_off0 = ds_off(kr0, qcol), ds_off1 = ds_off(kr0 + 4, qcol);

  // ---- slice prefetch: 2 Q chunks + 2 dO chunks per thread, lse / delta by 32 threads
  const int srow = tid >> 3, sch = (tid & 7) * 2;   // 32 rows x 16 chunks = 512 = 2 / thread
  const int st_off0 = dual_off<D>(srow, sch * 16), st_off1 = dual_off<D>(srow, sch * 16 + 16);
  struct Pf {
    u16x8 q0, q1, o0, o1;
    float l, d;
  };
  auto load_regs = [&](Pf& r, int qt0) {
    const u16* qr = qp + (long)(qt0 + srow) * p.q_ss + sch * 8;
    const u16* orow = dop + (long)(qt0 + srow) * p.do_ss + sch * 8;
    r.q0 = *reinterpret_cast<const u16x8*>(qr);
    r.q1 = *reinterpret_cast<const u16x8*>(qr + 8);
    r.o0 = *reinterpret_cast<const u16x8*>(orow);
    r.o1 = *reinterpret_cast<const u16x8*>(orow + 8);
    const int qi = qt0 + (tid & 31);
    r.l = lsep[qi];
    r.d = dlp[qi];
  };
  const float inv_scale = 1.f / p.scale;
  auto store_lds = [&](const Pf& r, char* st) {
    *reinterpret_cast<u16x8*>(st + st_off0) = r.q0;
    *reinterpret_cast<u16x8*>(st + st_off1) = r.q1;
    *reinterpret_cast<u16x8*>(st + Q_BYTES + st_off0) = r.o0;
    *reinterpret_cast<u16x8*>(st + Q_BYTES + st_off1) = r.o1;
    float* lc = (float*)(st + 2 * Q_BYTES);
    if (tid < 32) {
      lc[tid] = -r.l * inv_scale;  // S accumulator start: p = exp2(scale_log2 * (S - lse / scale))
      lc[BQ + tid] = -r.d;         // dP accumulator start: dS = p * (dP - delta) * scale
    }
  };

  // dK^T / dV^T live in AGPRs for the whole sweep: their definition before the loop
  // and their read after it are asm statements with AGPR ("a") operands, so hipcc
  // allocates the loop-carried values there instead of shuttling them through VGPRs
  // around each MFMA (the MFMAs themselves stay builtins: hipcc places their hazard
  // wait states, which it does not do for MFMAs written in inline asm)
  f32x16 dk[4], dv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f32x16 z;
#pragma unroll
    for (int e = 0; e < 16; ++e) z[e] = 0.f;
    asm volatile("" : "=a"(dk[i]) : "0"(z));
    asm volatile("" : "=a"(dv[i]) : "0"(z));
  }

  const int nslices = (p.Sq - qstart) / BQ;
  Pf pf;
  if (nslices > 0) {
    load_regs(pf, qstart);
    store_lds(pf, stage0);
  }
  lds_barrier();

  for (int t = 0; t < nslices; ++t) {
    const int q0 = qstart + t * BQ;
    char* st = stage0 + (t & 1) * STAGE;
    char* dsb = dsbuf0 + (t & 1) * DSB;
    const char* Qs = st;
    const char* Os = st + Q_BYTES;
    const float* lc = (const float*)(st + 2 * Q_BYTES);
    const bool more = t + 1 < nslices;
    if (more) load_regs(pf, q0 + BQ);

    const bool wave_masked = CAUSAL && (q0 + BQ - 1 + offs < key_w0);
    const bool wave_diag = CAUSAL && !(key_w0 + 31 <= q0 + offs);
    if (!wave_masked) {
      // ---- S, dP (accumulators start at the row constants)
      f32x16 sacc, dpacc;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x4 l4 = *reinterpret_cast<const f32x4*>(lc + 8 * i + 4 * hh);
        const f32x4 d4 = *reinterpret_cast<const f32x4*>(lc + BQ + 8 * i + 4 * hh);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          sacc[4 * i + j] = l4[j];
          dpacc[4 * i + j] = d4[j];
        }
      }
      bf8v sq[3], so[3], sk[3], sv[3];
      auto sload = [&](int j, int ks) {
        sq[j] = as_bf8(*reinterpret_cast<const u16x8*>(Qs + q_row + s_off[ks]));
        so[j] = as_bf8(*reinterpret_cast<const u16x8*>(Os + q_row + s_off[ks]));
        sk[j] = as_bf8(*reinterpret_cast<const u16x8*>(Ks + k_row + s_off[ks]));
        sv[j] = as_bf8(*reinterpret_cast<const u16x8*>(Vs + k_row + s_off[ks]));
      };
      sload(0, 0);
      sload(1, 1);
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        if (ks + 2 < 8) sload((ks + 2) % 3, ks + 2);
        sacc = mfma32(sq[ks % 3], sk[ks % 3], sacc);
        dpacc = mfma32(so[ks % 3], sv[ks % 3], dpacc);
        __builtin_amdgcn_sched_barrier(0);
      }
      // ---- P, dS as bf16 B operands: register r <-> query 8 (r >> 2) + 4 hh + (r & 3)
      bf8v pB[2], dB[2];
      const int lim = mykey - offs - q0 - 4 * hh;  // masked when 8 (r>>2) + (r&3) < lim
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float pv = __builtin_amdgcn_exp2f(sacc[r] * p.scale_log2);
        if (wave_diag) pv = (8 * (r >> 2) + (r & 3)) >= lim ? pv : 0.f;
        pB[r >> 3][r & 7] = (__bf16)pv;
        dB[r >> 3][r & 7] = (__bf16)(pv * dpacc[r] * p.scale);
      }
      // ---- dV^T += dO^T P, dK^T += Q^T dS: 8 (d block, k-step) pairs
      bf8v to[3], tq[3];
      auto tload = [&](int j, int it) {
        const int db = it >> 1, s2 = it & 1;
        to[j] = cat_tr(tr_read(Os, t_off[db][0] + 4096 * s2), tr_read(Os, t_off[db][1] + 4096 * s2));
        tq[j] = cat_tr(tr_read(Qs, t_off[db][0] + 4096 * s2), tr_read(Qs, t_off[db][1] + 4096 * s2));
      };
      tload(0, 0);
      tload(1, 1);
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        if (it + 2 < 8) tload((it + 2) % 3, it + 2);
        dv[it >> 1] = mfma32(to[it % 3], pB[it & 1], dv[it >> 1]);
        dk[it >> 1] = mfma32(tq[it % 3], dB[it & 1], dk[it >> 1]);
        __builtin_amdgcn_sched_barrier(0);
      }
      // ---- dS^T -> LDS [key][q]: 4 consecutive queries per 8-B store
      const int key = 32 * w + l32;
      const u16x8 lo = __builtin_bit_cast(u16x8, dB[0]), hi = __builtin_bit_cast(u16x8, dB[1]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const u16x8& src = i < 2 ? lo : hi;
        const int o = 4 * (i & 1);
        const u16x4 v4 = {src[o], src[o + 1], src[o + 2], src[o + 3]};
        *reinterpret_cast<u16x4*>(dsb + ds_off(key, 8 * i + 4 * hh)) = v4;
      }
    } else {
      const u16x4 z = {0, 0, 0, 0};
#pragma unroll
      for (int i = 0; i < 4; ++i) *reinterpret_cast<u16x4*>(dsb + ds_off(32 * w + l32, 8 * i + 4 * hh)) = z;
    }
    if (more) store_lds(pf, stage0 + ((t + 1) & 1) * STAGE);
    lds_barrier();
    // ---- dQ^T[d = 32w + m][q = n] = sum over the block's 128 keys of K[key][d] dS^T[key][q]
    f32x16 dq;
#pragma unroll
    for (int e = 0; e < 16; ++e) dq[e] = 0.f;
    bf8v qk[3], qs_[3];
    auto qload = [&](int j, int ks) {
      qk[j] = cat_tr(tr_read(Ks, kt_off0 + 4096 * ks), tr_read(Ks, kt_off1 + 4096 * ks));
      qs_[j] = cat_tr(tr_read(dsb, ds_off0 + 1024 * ks), tr_read(dsb, ds_off1 + 1024 * ks));
    };
    qload(0, 0);
    qload(1, 1);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      if (ks + 2 < 8) qload((ks + 2) % 3, ks + 2);
      dq = mfma32(qk[ks % 3], qs_[ks % 3], dq);
      __builtin_amdgcn_sched_barrier(0);
    }
    // lane: q = q0 + l32; d = 32w + 8i + 4hh + 0..3 -> bf16 partial of this key block
    u16* prow = part + (long)(q0 + l32) * D + 32 * w + 4 * hh;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const u16x4 v4 = {f2bf(dq[4 * i]), f2bf(dq[4 * i + 1]), f2bf(dq[4 * i + 2]), f2bf(dq[4 * i + 3])};
      *reinterpret_cast<u16x4*>(prow + 8 * i) = v4;
    }
  }
  // ---- dK / dV: element (db, r) = key mykey, d = 32db + 8(r>>2) + 4hh + (r&3)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    asm volatile("" : "+a"(dk[i]));
    asm volatile("" : "+a"(dv[i]));
  }
  u16* dkp = p.dk + (long)b * p.dk_bs + (long)h * p.dk_hs + (long)mykey * p.dk_ss;
  u16* dvp = p.dv + (long)b * p.dk_bs + (long)h * p.dk_hs + (long)mykey * p.dk_ss;
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int d = 32 * db + 8 * i + 4 * hh;
      const u16x4 k4 = {f2bf(dk[db][4 * i]), f2bf(dk[db][4 * i + 1]), f2bf(dk[db][4 * i + 2]), f2bf(dk[db][4 * i + 3])};
      const u16x4 v4 = {f2bf(dv[db][4 * i]), f2bf(dv[db][4 * i + 1]), f2bf(dv[db][4 * i + 2]), f2bf(dv[db][4 * i + 3])};
      *reinterpret_cast<u16x4*>(dkp + d) = k4;
      *reinterpret_cast<u16x4*>(dvp + d) = v4;
    }
}

// dq_acc[b, q, h, :] = sum of the key-block partials that cover query q (v4).  The
// causal kernel for key block kb starts at query floor(max(0, 128kb - offs) / 32) * 32
// and writes every query from there (masked ones as zeros), so exactly those blocks
// are summed.  One thread per 4 consecutive d (16-B loads/stores).
template <int D, bool CAUSAL>
__global__ __launch_bounds__(256) void fa_bwd_dq_reduce(BwdParams p, int nkb, int kblk) {
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)p.B * p.Hq * p.Sq * (D / 4);
  if (gid >= total) return;
  const int d4 = (int)(gid % (D / 4));
  const long r = gid / (D / 4);           // (b, h, q)
  const long q = r % p.Sq;
  const long bh = r / p.Sq;
  const int h = (int)(bh % p.Hq), b = (int)(bh / p.Hq);
  const long offs = CAUSAL ? (long)p.Sk - p.Sq : 0;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const long slab = (long)p.B * p.Hq * p.Sq * D;
  const u16* src = (const u16*)p.dq_part + ((long)b * p.Hq + h) * p.Sq * D + q * D + 4 * d4;
  for (int kb = 0; kb < nkb; ++kb) {
    if (CAUSAL) {
      long qs = (long)kblk * kb - offs;
      qs = qs > 0 ? (qs / 32) * 32 : 0;
      if (qs > q) break;
    }
    const u16x4 v = *reinterpret_cast<const u16x4*>(src + kb * slab);
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] += bf2f(v[k]);
  }
  *reinterpret_cast<f32x4*>(p.dq_acc + (((long)b * p.Sq + q) * p.Hq + h) * D + 4 * d4) = acc;
}

// v4 dQ epilogue fused with the inverse (neox) rotary and the bf16 cast, writing the
// dq slot of the packed dqkv gradient directly: the slabs are read once and the
// fp32 [B, Sq, Hq, D] accumulator is never materialised (D = 128; position = q).
// Thread = 4 consecutive d of the low half plus the same 4 of the high half.
template <bool CAUSAL>
__global__ __launch_bounds__(256) void fa_dq_reduce_rope(const float* __restrict__ part, int nkb, int B,
                                                         int Sq, int Sk, int Hq, u16* __restrict__ out,
                                                         long out_ts, const float* __restrict__ cosT,
                                                         const float* __restrict__ sinT, int kblk) {
  constexpr int D = 128, HALF = 64;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)B * Hq * Sq * (HALF / 4);
  if (gid >= total) return;
  const int c = (int)(gid & 15);
  const long r = gid >> 4;  // (b, h, q)
  const long q = r % Sq;
  const long bh = r / Sq;
  const int h = (int)(bh % Hq), b = (int)(bh / Hq);
  const long offs = CAUSAL ? (long)Sk - Sq : 0;
  const long slab = (long)B * Hq * Sq * D;
  const u16* src = (const u16*)part + (bh * Sq + q) * D + 4 * c;
  f32x4 lo = {0.f, 0.f, 0.f, 0.f}, hi = {0.f, 0.f, 0.f, 0.f};
  for (int kb = 0; kb < nkb; ++kb) {
    if (CAUSAL) {
      long qs = (long)kblk * kb - offs;
      qs = qs > 0 ? (qs / 32) * 32 : 0;
      if (qs > q) break;
    }
    const u16x4 vl = *reinterpret_cast<const u16x4*>(src + kb * slab);
    const u16x4 vh = *reinterpret_cast<const u16x4*>(src + kb * slab + HALF);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      lo[k] += bf2f(vl[k]);
      hi[k] += bf2f(vh[k]);
    }
  }
  const f32x4 co = *reinterpret_cast<const f32x4*>(cosT + q * HALF + 4 * c);
  const f32x4 si = *reinterpret_cast<const f32x4*>(sinT + q * HALF + 4 * c);
  u16x4 ol, oh;
#pragma unroll
  for (int j = 0; j < 4; ++j) {  // inverse rotation: sin -> -sin
    ol[j] = f2bf(lo[j] * co[j] + hi[j] * si[j]);
    oh[j] = f2bf(hi[j] * co[j] - lo[j] * si[j]);
  }
  u16* dst = out + ((long)b * Sq + q) * out_ts + (long)h * D + 4 * c;
  *reinterpret_cast<u16x4*>(dst) = ol;
  *reinterpret_cast<u16x4*>(dst + HALF) = oh;
}

// 0 = fa_bwd_kernel, 1 = pipelined, 2 = probe without dQ atomics (wrong dQ),
// 3 = 8-wave MFMA16 (D = 128), 4 = v3 with per-key-block dQ partials + reduce (needs dq_part),
// 5 = 4 waves x 32 keys, MFMA 32x32x16 + partials (D = 128, causal, Sk % 128, Sq % 32; else v4)
// default: v4 (causal D = 128: 1.50 ms + 0.46 ms reduce vs v2 2.18 ms at B8 H32 S2048);
// other shapes fall back to v2 in the launcher
static int g_fa_bwd_variant = 4;

}  // namespace pa

using namespace pa;

PA_EXPORT int pa_fa_bwd_set_variant(int v) {
  g_fa_bwd_variant = v;
  return 0;
}

PA_EXPORT int pa_fa_bwd_get_variant() { return g_fa_bwd_variant; }

// forward: 1 = fa_fwd_kernel, 2 = fa_fwd_kernel2 (32-bit positions / offsets, lane-
// constant mask limit: fewer VALU per MFMA)
static int g_fa_fwd_variant = 2;
PA_EXPORT int pa_fa_fwd_set_variant(int v) {
  g_fa_fwd_variant = v;
  return 0;
}

static bool fa_v5_ok(int Sq, int Sk, int D, int causal) {
  return g_fa_bwd_variant == 5 && D == 128 && causal && Sk % 128 == 0 && Sq % 32 == 0 && Sq > 0;
}

// key rows per dQ partial slab of the partial-slab path (0: that path is off)
PA_EXPORT int pa_fa_bwd_part_kblk(int Sq, int Sk, int D, int causal) {
  if (fa_v5_ok(Sq, Sk, D, causal)) return 128;
  if ((g_fa_bwd_variant == 4 || g_fa_bwd_variant == 5) && D == 128 && causal) return 128;
  return 0;
}

PA_EXPORT int pa_flash_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse,
                                const long* strides /*12: q b,s,h k b,s,h v b,s,h o b,s,h*/,
                                int B, int Sq, int Sk, int Hq, int Hkv, int D, float scale,
                                int causal, hipStream_t st) {
  if (Hq % Hkv) return (int)hipErrorInvalidValue;
  FwdParams p;
  p.q = (const u16*)q; p.k = (const u16*)k; p.v = (const u16*)v; p.o = (u16*)o; p.lse = lse;
  p.q_bs = strides[0]; p.q_ss = strides[1]; p.q_hs = strides[2];
  p.k_bs = strides[3]; p.k_ss = strides[4]; p.k_hs = strides[5];
  p.v_bs = strides[6]; p.v_ss = strides[7]; p.v_hs = strides[8];
  p.o_bs = strides[9]; p.o_ss = strides[10]; p.o_hs = strides[11];
  p.B = B; p.Sq = Sq; p.Sk = Sk; p.Hq = Hq; p.Hkv = Hkv;
  p.scale_log2 = scale * 1.44269504089f;
  dim3 grid(Hq, B, (Sq + 127) / 128);
  const bool v2ok = g_fa_fwd_variant == 2 && (long)Sk * strides[4] < (1L << 31) && (long)Sk * strides[7] < (1L << 31);
  if (D == 128 && v2ok) {
    if (causal) hipLaunchKernelGGL((fa_fwd_kernel2<128, true>), grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((fa_fwd_kernel2<128, false>), grid, dim3(256), 0, st, p);
  } else if (D == 128) {
    if (causal) hipLaunchKernelGGL((fa_fwd_kernel<128, true>), grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((fa_fwd_kernel<128, false>), grid, dim3(256), 0, st, p);
  } else if (D == 64) {
    if (causal) hipLaunchKernelGGL((fa_fwd_kernel<64, true>), grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((fa_fwd_kernel<64, false>), grid, dim3(256), 0, st, p);
  } else if (D == 256) {
    if (causal) hipLaunchKernelGGL((fa_fwd_kernel<256, true>), grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((fa_fwd_kernel<256, false>), grid, dim3(256), 0, st, p);
  } else {
    return (int)hipErrorInvalidValue;
  }
  PA_LAUNCH_CHECK();
}

// dq_acc ([B, Sq, Hq, D] fp32) is zeroed by the pre-pass; dk/dv share strides
// strides[15..17] and are indexed by the q-head (GQA callers reduce head groups).
PA_EXPORT int pa_flash_attn_bwd(const void* q, const void* k, const void* v, const void* o,
                                const void* dout, const float* lse, float* delta, float* dq_acc,
                                void* dk, void* dv, const long* strides /*18: q k v o do dk(b,s,h)*/, int B, int Sq,
                                int Sk, int Hq, int Hkv, int D, float scale, int causal, float* dq_part,
                                hipStream_t st) {
  if (Hq % Hkv) return (int)hipErrorInvalidValue;
  BwdParams p;
  p.q = (const u16*)q; p.k = (const u16*)k; p.v = (const u16*)v; p.o = (const u16*)o;
  p.dout = (const u16*)dout; p.lse = lse; p.delta = delta; p.dq_acc = dq_acc; p.dq_part = dq_part;
  p.dk = (u16*)dk; p.dv = (u16*)dv;
  p.q_bs = strides[0]; p.q_ss = strides[1]; p.q_hs = strides[2];
  p.k_bs = strides[3]; p.k_ss = strides[4]; p.k_hs = strides[5];
  p.v_bs = strides[6]; p.v_ss = strides[7]; p.v_hs = strides[8];
  p.o_bs = strides[9]; p.o_ss = strides[10]; p.o_hs = strides[11];
  p.do_bs = strides[12]; p.do_ss = strides[13]; p.do_hs = strides[14];
  p.dk_bs = strides[15]; p.dk_ss = strides[16]; p.dk_hs = strides[17];
  p.B = B; p.Sq = Sq; p.Sk = Sk; p.Hq = Hq; p.Hkv = Hkv;
  p.scale = scale;
  p.scale_log2 = scale * 1.44269504089f;
  // the pipelined kernel addresses Q/dO/dQ of one (b, head) with 32-bit buffer offsets
  const long lim = 1L << 31;
  const bool fits32 = (long)Sq * strides[1] * 2 < lim && (long)Sq * strides[13] * 2 < lim &&
                      (long)Sq * Hq * D * 4 < lim;
  int variant = fits32 ? g_fa_bwd_variant : 0;
  if (variant == 5 && !(fa_v5_ok(Sq, Sk, D, causal) && dq_part != nullptr)) variant = 4;
  if (variant == 4 && (D != 128 || dq_part == nullptr || !causal)) variant = 1;
  if (variant != 4 && dq_acc == nullptr) return (int)hipErrorInvalidValue;
  const long rows = (long)B * Hq * Sq;
  const int lpr = D / 8;
  const long pre_threads = rows * lpr;
  BwdParams pp = p;
  if (variant >= 4) pp.dq_acc = nullptr;  // partial slabs: no accumulator to zero
  if (D == 128) hipLaunchKernelGGL(fa_bwd_pre_kernel<128>, dim3((pre_threads + 255) / 256), dim3(256), 0, st, pp);
  else if (D == 64) hipLaunchKernelGGL(fa_bwd_pre_kernel<64>, dim3((pre_threads + 255) / 256), dim3(256), 0, st, pp);
  else if (D == 256) hipLaunchKernelGGL(fa_bwd_pre_kernel<256>, dim3((pre_threads + 255) / 256), dim3(256), 0, st, pp);
  else return (int)hipErrorInvalidValue;
  dim3 grid(Hq, B, (Sk + 127) / 128);
  if (variant == 5) {
    const int nkb = Sk / 128;
    hipLaunchKernelGGL(fa_bwd_kernel5<true>, dim3(Hq, B, nkb), dim3(256), 0, st, p);
    if (dq_acc == nullptr) {
      PA_LAUNCH_CHECK();
    }
    const long n = (long)B * Hq * Sq * (D / 4);
    hipLaunchKernelGGL((fa_bwd_dq_reduce<128, true>), dim3((n + 255) / 256), dim3(256), 0, st, p, nkb, 128);
    PA_LAUNCH_CHECK();
  }
  if (D == 128 && (variant == 3 || variant == 4)) {
    const int nkb = (Sk + 127) / 128;
    dim3 g3(Hq, B, nkb);
    if (variant == 4) {
      if (causal) hipLaunchKernelGGL((fa_bwd_kernel3<true, true>), g3, dim3(512), 0, st, p);
      else hipLaunchKernelGGL((fa_bwd_kernel3<false, true>), g3, dim3(512), 0, st, p);
      // dq_acc == nullptr: the caller runs the fused reduce (pa_fa_dq_reduce_rope)
      if (dq_acc == nullptr) {
        PA_LAUNCH_CHECK();
      }
      const long n = (long)B * Hq * Sq * (D / 4);
      if (causal) hipLaunchKernelGGL((fa_bwd_dq_reduce<128, true>), dim3((n + 255) / 256), dim3(256), 0, st, p, nkb, 128);
      else hipLaunchKernelGGL((fa_bwd_dq_reduce<128, false>), dim3((n + 255) / 256), dim3(256), 0, st, p, nkb, 128);
    } else {
      if (causal) hipLaunchKernelGGL((fa_bwd_kernel3<true, false>), g3, dim3(512), 0, st, p);
      else hipLaunchKernelGGL((fa_bwd_kernel3<false, false>), g3, dim3(512), 0, st, p);
    }
    PA_LAUNCH_CHECK();
  }
#define PA_FA_BWD_LAUNCH(DD, CC)                                                                    \
  switch (variant) {                                                                      \
    case 0: hipLaunchKernelGGL((fa_bwd_kernel<DD, CC>), grid, dim3(256), 0, st, p); break;         \
    case 2: hipLaunchKernelGGL((fa_bwd_kernel2<DD, CC, true>), grid, dim3(256), 0, st, p); break;  \
    default: hipLaunchKernelGGL((fa_bwd_kernel2<DD, CC, false>), grid, dim3(256), 0, st, p); break; \
  }
  if (D == 128) {
    if (causal) { PA_FA_BWD_LAUNCH(128, true) } else { PA_FA_BWD_LAUNCH(128, false) }
  } else if (D == 256) {
    if (causal) hipLaunchKernelGGL((fa_bwd_kernel<256, true>), grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((fa_bwd_kernel<256, false>), grid, dim3(256), 0, st, p);
  } else {
    if (causal) { PA_FA_BWD_LAUNCH(64, true) } else { PA_FA_BWD_LAUNCH(64, false) }
  }
#undef PA_FA_BWD_LAUNCH
  PA_LAUNCH_CHECK();
}

// Fused v4 dQ epilogue: sum the per-key-block slabs, inverse-rotate (neox, position
// = query index) and store bf16 into ``out`` rows of stride ``out_ts`` elements
// (the dq columns of the packed dqkv gradient).  D = 128.
PA_EXPORT int pa_fa_dq_reduce_rope(const float* part, int nkb, int B, int Sq, int Sk, int Hq, int causal,
                                   void* out, long out_ts, const float* cosT, const float* sinT, int kblk,
                                   hipStream_t st) {
  if (kblk != 128 && kblk != 256) return (int)hipErrorInvalidValue;
  const long n = (long)B * Hq * Sq * 16;
  const dim3 g((unsigned)((n + 255) / 256));
  if (causal)
    hipLaunchKernelGGL(fa_dq_reduce_rope<true>, g, dim3(256), 0, st, part, nkb, B, Sq, Sk, Hq, (u16*)out,
                       out_ts, cosT, sinT, kblk);
  else
    hipLaunchKernelGGL(fa_dq_reduce_rope<false>, g, dim3(256), 0, st, part, nkb, B, Sq, Sk, Hq, (u16*)out,
                       out_ts, cosT, sinT, kblk);
  PA_LAUNCH_CHECK();
}

// GQA backward fold: the backward kernels write dK / dV per QUERY head
// ([B, S, Hq, D] contiguous); the kv head kh receives the sum over its `ratio` query
// heads, stored into a strided destination (the packed dqkv's k / v slot, rows
// `dst_ss` elements apart).  grid.y = 0: dK, 1: dV.  fp32 sums, one bf16 rounding.
namespace pa {
__global__ __launch_bounds__(256) void fa_gqa_fold_kernel(const u16* __restrict__ dk_e, const u16* __restrict__ dv_e,
                                                          u16* __restrict__ dk, u16* __restrict__ dv, long rows,
                                                          int Hq, int Hk, int D, long dst_ss) {
  const int ratio = Hq / Hk, nc = D / 8;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= rows * Hk * nc) return;
  const int c = (int)(idx % nc);
  const int kh = (int)((idx / nc) % Hk);
  const long row = idx / nc / Hk;
  const u16* src = blockIdx.y ? dv_e : dk_e;
  u16* dst = blockIdx.y ? dv : dk;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int r = 0; r < ratio; ++r) {
    float v[8];
    load8(src + ((row * Hq + (long)kh * ratio + r) * D + 8 * c), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] += v[e];
  }
  store8(dst + row * dst_ss + (long)kh * D + 8 * c, acc);
}
}  // namespace pa

PA_EXPORT int pa_fa_gqa_fold(const void* dk_e, const void* dv_e, void* dk, void* dv, long rows, int Hq, int Hk,
                             int D, long dst_ss, hipStream_t st) {
  if (Hk <= 0 || Hq % Hk || D % 8 || dst_ss % 8 || rows <= 0) return -1;
  const long n = rows * Hk * (D / 8);
  hipLaunchKernelGGL(pa::fa_gqa_fold_kernel, dim3((unsigned)((n + 255) / 256), 2), dim3(256), 0, st,
                     (const u16*)dk_e, (const u16*)dv_e, (u16*)dk, (u16*)dv, rows, Hq, Hk, D, dst_ss);
  PA_LAUNCH_CHECK();
}
