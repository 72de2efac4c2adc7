// Channel-first (NCHW / NCDHW) convolution, transposed convolution and pooling on
// gfx950 for the Fluid operators (conv2d / conv3d / conv2d_transpose /
// conv3d_transpose / pool2d / pool3d / max_pool{2,3}d_with_index / unpool / maxout).
// The NHWC bf16 training path of the models lives in gemm.hip / conv_aux.hip; this
// file serves the reference's channel-first, usually fp32, Fluid programs.
//
// * sgemm: exact-fp32 GEMM on v_mfma_f32_32x32x2f32 (128x128x16 tiles, 4 waves of
//   64x64), fully strided operands, two batch dimensions on blockIdx.z (image x
//   group), an inner "k-batch" that sums several strided GEMMs in registers (weight
//   gradients over a chunk of images), row bias, alpha/beta, or float-atomic
//   accumulation for split reductions.
// * vol2col / col2vol: the 3-D lowering (2-D = depth 1) of math/vol2col.cu and
//   math/im2col.cu (CFO layout: rows (c, kd, kh, kw), columns (od, oh, ow));
//   col2vol gathers per input element over the kernel taps (no atomics).
// * pooling: max / avg (exclusive or not, ceil-mode output sizes computed by the
//   caller) with the int32 in-plane argmax of KernelMaxPool{2,3}dWithIdx; the
//   backward gathers over the windows that cover an input element (max: through
//   the argmax, i.e. the first maximum as in KernelMaxPool2DGrad).
// * unpool (max) scatter / gather, maxout (first maximum gets the gradient).
//
// Reference behaviour: operators/math/{vol2col,im2col,pooling,maxouting,
// unpooling}.cu, conv_cudnn_op.cu.cc, conv_transpose_cudnn_op.cu.cc, pool_op.cc
// (output size), pool_with_index_op.cc.
#include "common.h"

#include <type_traits>

namespace pa {
namespace {

inline int grid_for(long n, int block = 256) {
  long g = (n + block - 1) / block;
  return (int)(g < 1 ? 1 : (g > 16384 ? 16384 : g));
}

#define GRID_STRIDE(i, n) for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < (n); i += (long)gridDim.x * blockDim.x)

// ================================================================ fp32 MFMA GEMM
struct SgemmArgs {
  const float* A;
  const float* B;
  float* C;
  const float* bias_m;  // [M] (+ z2 * bsBias2) or null
  long bsBias2;
  long M, N, K;
  long sam, sak;  // A(m, k) = A[m * sam + k * sak]
  long sbk, sbn;  // B(k, n) = B[k * sbk + n * sbn]
  long ldc;
  int Z2;                   // blockIdx.z = z1 * Z2 + z2
  long bsA1, bsB1, bsC1;    // strides of z1
  long bsA2, bsB2, bsC2;    // strides of z2
  int kb;                   // inner k-batch: sum over kb GEMMs ...
  long kbA, kbB;            // ... whose operands are offset by these strides
  float alpha, beta;
  int atomic;               // C += alpha * AB with float atomics (beta / bias ignored)
  long ksplit;              // > 0: k-slices of this length (split-K, atomic)
  // implicit-GEMM B operand (2-D conv gather, CONVB kernels): image [C][H][W] at B
  int cH, cW, cOW, ckh, ckw, csh, csw, cph, cpw, cdh, cdw;
  int kbsplit;              // > 0: k-batch ranges of this many members (split over the k-batch, atomic)
  int nks;                  // split mode: z1 = kbatch_slice * nks + k_slice
};

constexpr int SBM = 128, SBN = 128, SBK = 32, SPAD = 4;
// LDS tiles are [mn][k] with rows of SBK + KPAD floats (144 B): the 16 lanes of a
// ds_read_b128 phase hit 16 distinct 4-bank groups
constexpr int KPAD = 4;
// 16-B k-group swizzle by row: k -> k ^ (((row >> 2) & 7) << 2).  The transposed
// (mn-contiguous operand) stores write 4 rows per lane; without it those rows,
// 4 apart, hit one 16-bank slice (8-way conflicts).  Reads stay whole 16-B groups.
__device__ __forceinline__ int ksw(int row, int k) { return k ^ (((row >> 2) & 7) << 2); }

// One k-tile of an operand, staged global -> registers -> LDS ([SBK][128 + SPAD],
// k-major).  KF: the operand's k index is the contiguous one (A row-major / B
// column-major); VEC: 16-B aligned float4 loads along the contiguous dimension.
// Each of the 256 threads owns 16 elements = 4 float4.
template <bool KF, bool VEC>
struct TileLoader {
  float r[16];
  __device__ __forceinline__ void load(const float* __restrict__ P, long s_mn, long s_k, long mn0, long k0, long MN,
                                       long K, int tid) {
    if (!VEC) {
      // scalar path: element e = j * 256 + tid, consecutive lanes on the contiguous
      // (or, when neither is, the k) dimension -> every wave load is one dense run
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int e = j * 256 + tid;
        int mn, kk;
        if (KF) { mn = e >> 5; kk = e & 31; } else { kk = e >> 7; mn = e & 127; }
        const long gm = mn0 + mn, gk = k0 + kk;
        r[j] = (gm < MN && gk < K) ? P[gm * s_mn + gk * s_k] : 0.f;
      }
      return;
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int q = v * 256 + tid;  // float4 slot within the 128 x 32 tile
      int mn, kk;
      if (KF) { mn = q >> 3; kk = (q & 7) * 4; } else { kk = q >> 5; mn = (q & 31) * 4; }
      const long gm = mn0 + mn, gk = k0 + kk;
      if (KF ? (gm < MN && gk + 3 < K) : (gk < K && gm + 3 < MN)) {
        const f32x4 t = *reinterpret_cast<const f32x4*>(P + gm * s_mn + gk * s_k);
        r[4 * v] = t[0]; r[4 * v + 1] = t[1]; r[4 * v + 2] = t[2]; r[4 * v + 3] = t[3];
        continue;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const long m = KF ? gm : gm + e, k = KF ? gk + e : gk;
        r[4 * v + e] = (m < MN && k < K) ? P[m * s_mn + k * s_k] : 0.f;
      }
    }
  }
  __device__ __forceinline__ void store(float (*S)[SBK + KPAD], int tid) const {
    if (!VEC) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int e = j * 256 + tid;
        if (KF) S[e >> 5][ksw(e >> 5, e & 31)] = r[j];
        else S[e & 127][ksw(e & 127, e >> 7)] = r[j];
      }
      return;
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int q = v * 256 + tid;
      if (KF) {
        const int mn = q >> 3, kk = (q & 7) * 4;
        *reinterpret_cast<f32x4*>(&S[mn][ksw(mn, kk)]) = f32x4{r[4 * v], r[4 * v + 1], r[4 * v + 2], r[4 * v + 3]};
      } else {
        const int kk = q >> 5, mn = (q & 31) * 4;
#pragma unroll
        for (int e = 0; e < 4; ++e) S[mn + e][ksw(mn + e, kk)] = r[4 * v + e];
      }
    }
  }
};

// Implicit im2col B operand of a 2-D convolution: B(k = (c, kh, kw), n = (oh, ow))
// (forward, KF = false) or B(k = (oh, ow), n = (c, kh, kw)) (weight gradient,
// KF = true), gathered from the image with zero padding -- no column buffer.  The
// element -> (k, n) map is the scalar TileLoader's, so one index of each pair is
// fixed per thread and decomposed once per tile.
template <bool KF>
struct ConvGather {
  float r[16];
  __device__ __forceinline__ float at(const float* __restrict__ P, const SgemmArgs& g, long ck, long s) const {
    const int KT = g.ckh * g.ckw;
    const int c = (int)(ck / KT), t = (int)(ck - (long)c * KT);
    const int kh = t / g.ckw, kw = t - kh * g.ckw;
    const int oh = (int)(s / g.cOW), ow = (int)(s - (long)oh * g.cOW);
    const int ih = oh * g.csh - g.cph + kh * g.cdh, iw = ow * g.csw - g.cpw + kw * g.cdw;
    return (ih >= 0 && ih < g.cH && iw >= 0 && iw < g.cW) ? P[((long)c * g.cH + ih) * g.cW + iw] : 0.f;
  }
  __device__ __forceinline__ void load(const float* __restrict__ P, const SgemmArgs& g, long mn0, long k0, long MN,
                                       long K, int tid) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int e = j * 256 + tid;
      int mn, kk;
      if (KF) { mn = e >> 5; kk = e & 31; } else { kk = e >> 7; mn = e & 127; }
      const long gm = mn0 + mn, gk = k0 + kk;
      r[j] = (gm < MN && gk < K) ? (KF ? at(P, g, gm, gk) : at(P, g, gk, gm)) : 0.f;
    }
  }
  __device__ __forceinline__ void store(float (*S)[SBK + KPAD], int tid) const {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int e = j * 256 + tid;
      if (KF) S[e >> 5][ksw(e >> 5, e & 31)] = r[j];
      else S[e & 127][ksw(e & 127, e >> 7)] = r[j];
    }
  }
};

// 128 x 128 output tile, 4 waves of 64 x 64 (2 x 2 v_mfma_f32_32x32x2f32), k-tiles
// of 32 double-buffered in LDS with the next tile's global loads issued before the
// current tile's MFMAs (one barrier per k-tile).
template <bool AK, bool BK_, bool VEC, bool CONVB>
__global__ __launch_bounds__(256) void sgemm_kernel(SgemmArgs g) {
  __shared__ __attribute__((aligned(16))) float As[2][SBM][SBK + KPAD];
  __shared__ __attribute__((aligned(16))) float Bs[2][SBN][SBK + KPAD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long z1 = blockIdx.z / g.Z2, z2 = blockIdx.z % g.Z2;
  const float* A0 = g.A + z1 * g.bsA1 + z2 * g.bsA2;
  const float* B0 = g.B + z1 * g.bsB1 + z2 * g.bsB2;
  float* C = g.C + z1 * g.bsC1 + z2 * g.bsC2;
  const float* bias = g.bias_m ? g.bias_m + z2 * g.bsBias2 : nullptr;
  const long m0 = (long)blockIdx.y * SBM, n0 = (long)blockIdx.x * SBN;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  long K = g.K, kbase = 0;
  int b_lo = 0, b_hi = g.kb;
  if (g.ksplit > 0 || g.kbsplit > 0) {  // split mode: z1 -> (k-batch slice, k slice)
    const long zk = z1 % g.nks, zb = z1 / g.nks;
    if (g.ksplit > 0) {
      const long kb0 = zk * g.ksplit;
      A0 += kb0 * g.sak;
      if (CONVB) kbase = kb0;  // gathered B: the k slice starts at kb0
      else B0 += kb0 * g.sbk;
      K = min(g.ksplit, g.K - kb0);
    }
    if (g.kbsplit > 0) {
      b_lo = (int)(zb * g.kbsplit);
      b_hi = min(g.kb, b_lo + g.kbsplit);
    }
  }
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  TileLoader<AK, VEC> la;
  typename std::conditional<CONVB, ConvGather<BK_>, TileLoader<BK_, VEC>>::type lb;
  const long ktiles = (K + SBK - 1) / SBK;
  const long total = ktiles * (b_hi - b_lo);
  if (total <= 0) return;  // empty split slice (uniform per workgroup: no barrier skipped by part of it)
  A0 += b_lo * g.kbA;
  B0 += b_lo * g.kbB;
  // B(k, n) = B[k * sbk + n * sbn]: as an "MN x K" operand its mn stride is sbn
  la.load(A0, g.sam, g.sak, m0, 0, g.M, K, tid);
  if constexpr (CONVB) lb.load(B0, g, n0, kbase, g.N, kbase + K, tid);
  else lb.load(B0, g.sbn, g.sbk, n0, 0, g.N, K, tid);
  la.store(As[0], tid);
  lb.store(Bs[0], tid);
  __syncthreads();
  for (long t = 0; t < total; ++t) {
    const int cur = (int)(t & 1);
    const bool more = t + 1 < total;
    if (more) {
      const long tn = t + 1;
      const long b = tn / ktiles, k0 = (tn % ktiles) * SBK;
      la.load(A0 + b * g.kbA, g.sam, g.sak, m0, k0, g.M, K, tid);
      if constexpr (CONVB) lb.load(B0 + b * g.kbB, g, n0, kbase + k0, g.N, kbase + K, tid);
      else lb.load(B0 + b * g.kbB, g.sbn, g.sbk, n0, k0, g.N, K, tid);
    }
    // k permuted inside the tile: lanes 0-31 feed k = j, lanes 32-63 k = 16 + j for
    // MFMA step j (the reduction order is free), so every lane reads 4 consecutive k
    // of its row with one ds_read_b128 per operand block
    const int kh = (lane >> 5) * 16, rl = lane & 31;
#pragma unroll
    for (int j0 = 0; j0 < 16; j0 += 4) {
      const int ka = kh + j0;
      const f32x4 a0 = *reinterpret_cast<const f32x4*>(&As[cur][wm + rl][ksw(wm + rl, ka)]);
      const f32x4 a1 = *reinterpret_cast<const f32x4*>(&As[cur][wm + 32 + rl][ksw(wm + 32 + rl, ka)]);
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(&Bs[cur][wn + rl][ksw(wn + rl, ka)]);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(&Bs[cur][wn + 32 + rl][ksw(wn + 32 + rl, ka)]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[e], b0[e], acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[e], b1[e], acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[e], b0[e], acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[e], b1[e], acc[1][1], 0, 0, 0);
      }
    }
    if (more) {
      la.store(As[cur ^ 1], tid);
      lb.store(Bs[cur ^ 1], tid);
    }
    __syncthreads();
  }
  // 32x32 accumulator map: column = lane & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const long n = n0 + wn + 32 * j + (lane & 31);
      if (n >= g.N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long m = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m >= g.M) continue;
        float* c = C + m * g.ldc + n;
        if (g.atomic) {
          atomicAdd(c, g.alpha * acc[i][j][r]);
        } else {
          float v = g.alpha * acc[i][j][r] + (bias ? bias[m] : 0.f);
          if (g.beta != 0.f) v += g.beta * *c;
          *c = v;
        }
      }
    }
}

// ================================================================ vol2col / col2vol
struct Geo {
  int C, D, H, W;        // input (image) dims
  int OD, OH, OW;        // column dims
  int kd, kh, kw;
  int sd, sh, sw;
  int pd, ph, pw;
  int dd, dh, dw;
};

// col[n][(c, kd, kh, kw)][(od, oh, ow)] for nb images
template <typename T>
__global__ void vol2col_kernel(const T* __restrict__ x, T* __restrict__ col, Geo g, int nb) {
  const long S = (long)g.OD * g.OH * g.OW;
  const int KT = g.kd * g.kh * g.kw;
  const long rows = (long)g.C * KT;
  const long total = (long)nb * rows * S;
  const long img = (long)g.C * g.D * g.H * g.W;
  GRID_STRIDE(i, total) {
    const long s = i % S;
    const long r = (i / S) % rows;
    const long n = i / (S * rows);
    const int ow = (int)(s % g.OW), oh = (int)((s / g.OW) % g.OH), od = (int)(s / ((long)g.OW * g.OH));
    const int tap = (int)(r % KT), c = (int)(r / KT);
    const int tw = tap % g.kw, th = (tap / g.kw) % g.kh, td = tap / (g.kw * g.kh);
    const int d = od * g.sd - g.pd + td * g.dd, h = oh * g.sh - g.ph + th * g.dh, w = ow * g.sw - g.pw + tw * g.dw;
    T v = (T)0;
    if (d >= 0 && d < g.D && h >= 0 && h < g.H && w >= 0 && w < g.W)
      v = x[n * img + (((long)c * g.D + d) * g.H + h) * g.W + w];
    col[i] = v;
  }
}

// x[n][c][d][h][w] (+)= sum over taps of col at the output position that read it
__global__ void col2vol_kernel(const float* __restrict__ col, float* __restrict__ x, Geo g, int nb, int accumulate) {
  const long S = (long)g.OD * g.OH * g.OW;
  const int KT = g.kd * g.kh * g.kw;
  const long plane = (long)g.D * g.H * g.W;
  const long total = (long)nb * g.C * plane;
  GRID_STRIDE(i, total) {
    const int w = (int)(i % g.W), h = (int)((i / g.W) % g.H), d = (int)((i / ((long)g.W * g.H)) % g.D);
    const long nc = i / plane;  // n * C + c
    const float* cb = col + nc * KT * S;  // rows (c, taps) of image n start at (n * C + c) * KT
    float acc = 0.f;
    for (int td = 0; td < g.kd; ++td) {
      const int zd = d + g.pd - td * g.dd;
      if (zd < 0 || zd % g.sd) continue;
      const int od = zd / g.sd;
      if (od >= g.OD) continue;
      for (int th = 0; th < g.kh; ++th) {
        const int zh = h + g.ph - th * g.dh;
        if (zh < 0 || zh % g.sh) continue;
        const int oh = zh / g.sh;
        if (oh >= g.OH) continue;
        for (int tw = 0; tw < g.kw; ++tw) {
          const int zw = w + g.pw - tw * g.dw;
          if (zw < 0 || zw % g.sw) continue;
          const int ow = zw / g.sw;
          if (ow >= g.OW) continue;
          const int tap = (td * g.kh + th) * g.kw + tw;
          acc += cb[(long)tap * S + ((long)od * g.OH + oh) * g.OW + ow];
        }
      }
    }
    x[i] = accumulate ? x[i] + acc : acc;
  }
}

// per-channel sum of y[n][c][s] (bias gradient): one workgroup per channel
__global__ __launch_bounds__(256) void chan_sum_kernel(const float* __restrict__ y, float* __restrict__ out, int N,
                                                       int C, long S, int accumulate) {
  __shared__ float red[4];
  const int c = blockIdx.x;
  float acc = 0.f;
  for (int n = 0; n < N; ++n) {
    const float* p = y + ((long)n * C + c) * S;
    for (long s = threadIdx.x; s < S; s += 256) acc += p[s];
  }
  acc = block_sum<256>(acc, red);
  if (threadIdx.x == 0) out[c] = accumulate ? out[c] + acc : acc;
}

// ================================================================ pooling (NC[D]HW)
struct PoolGeo {
  long NC;
  int D, H, W, OD, OH, OW;
  int kd, kh, kw, sd, sh, sw, pd, ph, pw;
};

// type 0 max (writes the in-plane argmax when mask != null), 1 avg
template <typename T>
__global__ void pool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int* __restrict__ mask, PoolGeo g,
                                int type, int exclusive) {
  const long OS = (long)g.OD * g.OH * g.OW;
  const long IS = (long)g.D * g.H * g.W;
  GRID_STRIDE(i, g.NC * OS) {
    const long nc = i / OS;
    const int ow = (int)(i % g.OW), oh = (int)((i / g.OW) % g.OH), od = (int)((i / ((long)g.OW * g.OH)) % g.OD);
    int d0 = od * g.sd - g.pd, h0 = oh * g.sh - g.ph, w0 = ow * g.sw - g.pw;
    const int d1 = min(d0 + g.kd, g.D), h1 = min(h0 + g.kh, g.H), w1 = min(w0 + g.kw, g.W);
    d0 = max(d0, 0);
    h0 = max(h0, 0);
    w0 = max(w0, 0);
    const T* p = x + nc * IS;
    if (type == 0) {
      float best = -3.402823466e+38f;
      int arg = -1;
      for (int d = d0; d < d1; ++d)
        for (int h = h0; h < h1; ++h)
          for (int w = w0; w < w1; ++w) {
            const int idx = (d * g.H + h) * g.W + w;
            const float v = IO<T>::ld(p, idx);
            if (v > best) { best = v; arg = idx; }
          }
      IO<T>::st(y, i, best);
      if (mask) mask[i] = arg;
    } else {
      float s = 0.f;
      for (int d = d0; d < d1; ++d)
        for (int h = h0; h < h1; ++h)
          for (int w = w0; w < w1; ++w) s += IO<T>::ld(p, (d * g.H + h) * g.W + w);
      const int cnt = exclusive ? (d1 - d0) * (h1 - h0) * (w1 - w0) : g.kd * g.kh * g.kw;
      IO<T>::st(y, i, cnt > 0 ? s / (float)cnt : 0.f);
    }
  }
}

// output range [lo, hi] whose windows (start o * s - p, length k) cover input i
__device__ __forceinline__ void cover(int i, int k, int s, int p, int O, int& lo, int& hi) {
  const int t = i + p - k + 1;
  lo = t <= 0 ? 0 : (t + s - 1) / s;
  hi = min((i + p) / s, O - 1);
}

template <typename T>
__global__ void pool_bwd_kernel(const T* __restrict__ dy, const int* __restrict__ mask, T* __restrict__ dx, PoolGeo g,
                                int type, int exclusive) {
  const long OS = (long)g.OD * g.OH * g.OW;
  const long IS = (long)g.D * g.H * g.W;
  GRID_STRIDE(i, g.NC * IS) {
    const long nc = i / IS;
    const int idx = (int)(i % IS);
    const int w = idx % g.W, h = (idx / g.W) % g.H, d = idx / (g.W * g.H);
    int dl, dh_, hl, hh, wl, wh;
    cover(d, g.kd, g.sd, g.pd, g.OD, dl, dh_);
    cover(h, g.kh, g.sh, g.ph, g.OH, hl, hh);
    cover(w, g.kw, g.sw, g.pw, g.OW, wl, wh);
    const T* gy = dy + nc * OS;
    float acc = 0.f;
    for (int od = dl; od <= dh_; ++od)
      for (int oh = hl; oh <= hh; ++oh)
        for (int ow = wl; ow <= wh; ++ow) {
          const long o = ((long)od * g.OH + oh) * g.OW + ow;
          if (type == 0) {
            if (mask[nc * OS + o] == idx) acc += IO<T>::ld(gy, o);
          } else {
            int cnt = g.kd * g.kh * g.kw;
            if (exclusive) {
              const int d0 = od * g.sd - g.pd, h0 = oh * g.sh - g.ph, w0 = ow * g.sw - g.pw;
              cnt = (min(d0 + g.kd, g.D) - max(d0, 0)) * (min(h0 + g.kh, g.H) - max(h0, 0)) *
                    (min(w0 + g.kw, g.W) - max(w0, 0));
            }
            acc += IO<T>::ld(gy, o) / (float)cnt;
          }
        }
    IO<T>::st(dx, i, acc);
  }
}

// ================================================================ unpool / maxout
// unpool (max): out[nc][mask[nc][i]] = x[nc][i]; out zero-filled by the caller
template <typename T>
__global__ void unpool_fwd_kernel(const T* __restrict__ x, const int* __restrict__ mask, T* __restrict__ out, long NC,
                                  long IS, long OS, int* __restrict__ bad) {
  GRID_STRIDE(i, NC * IS) {
    const long nc = i / IS;
    const int m = mask[i];
    if (m < 0 || m >= OS) { *bad = 1; continue; }
    out[nc * OS + m] = x[i];
  }
}

template <typename T>
__global__ void unpool_bwd_kernel(const T* __restrict__ dout, const int* __restrict__ mask, T* __restrict__ dx, long NC,
                                  long IS, long OS) {
  GRID_STRIDE(i, NC * IS) {
    const long nc = i / IS;
    const int m = mask[i];
    dx[i] = (m >= 0 && m < OS) ? dout[nc * OS + m] : (T)0;
  }
}

// maxout: y[n][c][s] = max_g x[n][c * groups + g][s]  (math/maxouting.cu)
template <typename T>
__global__ void maxout_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int N, int Co, int groups, long S) {
  GRID_STRIDE(i, (long)N * Co * S) {
    const long s = i % S;
    const long nc = i / S;  // n * Co + c
    const T* p = x + nc * groups * S + s;
    float best = IO<T>::ld(p, 0);
    for (int q = 1; q < groups; ++q) best = fmaxf(best, IO<T>::ld(p, (long)q * S));
    IO<T>::st(y, i, best);
  }
}

template <typename T>
__global__ void maxout_bwd_kernel(const T* __restrict__ x, const T* __restrict__ y, const T* __restrict__ dy,
                                  T* __restrict__ dx, int N, int Co, int groups, long S) {
  GRID_STRIDE(i, (long)N * Co * S) {
    const long s = i % S;
    const long nc = i / S;
    const float out = IO<T>::ld(y, i), g = IO<T>::ld(dy, i);
    const long base = nc * groups * S + s;
    bool done = false;
    for (int q = 0; q < groups; ++q) {
      const bool hit = !done && IO<T>::ld(x, base + (long)q * S) == out;
      IO<T>::st(dx, base + (long)q * S, hit ? g : 0.f);
      done = done || hit;
    }
  }
}


// ================================================================ batch norm (NC[D]HW)
// Per-channel reductions over (n, s) split into G slices per channel (grid C x G);
// the statistics pass sums (x - shift) and (x - shift)^2 with shift = the channel's
// first element (cancellation-safe without Welford), the backward pass sums dy and
// dy * xhat.  Reference: batch_norm_op.cc (biased batch variance for the running
// average, SavedVariance = 1 / sqrt(var + eps)), batch_norm_op.cu.cc.
template <typename T>
__global__ __launch_bounds__(256) void bn_partial_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                         const T* __restrict__ y, const float* __restrict__ mean,
                                                         const float* __restrict__ rstd, float* __restrict__ part,
                                                         int N, int C, long S, int G, int relu) {
  __shared__ float red[4];
  const int c = blockIdx.x, gi = blockIdx.y;
  const long M = (long)N * S;
  const long chunk = (M + G - 1) / G;
  const long lo = gi * chunk, hi = min(M, lo + chunk);
  float a = 0.f, b = 0.f;
  if (!dy) {
    const float shift = IO<T>::ld(x, (long)c * S);
    for (long i = lo + threadIdx.x; i < hi; i += 256) {
      const long n = i / S, sidx = i % S;
      const float v = IO<T>::ld(x, ((long)n * C + c) * S + sidx) - shift;
      a += v;
      b += v * v;
    }
  } else {
    const float mu = mean[c], rs = rstd[c];
    for (long i = lo + threadIdx.x; i < hi; i += 256) {
      const long n = i / S, sidx = i % S;
      const long off = ((long)n * C + c) * S + sidx;
      float g = IO<T>::ld(dy, off);
      if (relu && IO<T>::ld(y, off) <= 0.f) g = 0.f;
      a += g;
      b += g * (IO<T>::ld(x, off) - mu) * rs;
    }
  }
  a = block_sum<256>(a, red);
  __syncthreads();
  b = block_sum<256>(b, red);
  if (threadIdx.x == 0) {
    part[((long)c * G + gi) * 2] = a;
    part[((long)c * G + gi) * 2 + 1] = b;
  }
}

// mode 0: training statistics -> mean, rstd, running averages (momentum)
// mode 1: backward sums -> dbias (o0), dscale (o1)
// mode 2: inference -> mean = running mean, rstd from the running variance
template <typename T>
__global__ void bn_finalize_kernel(const T* __restrict__ x, const float* __restrict__ part, int C, int G, long M,
                                   float eps, float momentum, int mode, const float* __restrict__ run_mean,
                                   const float* __restrict__ run_var, float* __restrict__ o0, float* __restrict__ o1,
                                   float* __restrict__ mean_out, float* __restrict__ var_out, long S,
                                   int unbiased) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  if (mode == 2) {
    o0[c] = run_mean[c];
    o1[c] = rsqrtf(run_var[c] + eps);
    return;
  }
  double a = 0.0, b = 0.0;
  for (int g = 0; g < G; ++g) {
    a += part[((long)c * G + g) * 2];
    b += part[((long)c * G + g) * 2 + 1];
  }
  if (mode == 1) {
    o0[c] = (float)a;
    o1[c] = (float)b;
    return;
  }
  const double shift = IO<T>::ld(x, (long)c * S);
  const double m1 = a / (double)M;
  double var = b / (double)M - m1 * m1;
  if (var < 0.0) var = 0.0;
  const float mean = (float)(shift + m1);
  o0[c] = mean;
  o1[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (mean_out) mean_out[c] = run_mean[c] * momentum + mean * (1.f - momentum);
  const double rv = (unbiased && M > 1) ? var * (double)M / (double)(M - 1) : var;
  if (var_out) var_out[c] = run_var[c] * momentum + (float)rv * (1.f - momentum);
}

// forward: y = (x - mean) * rstd * scale + bias (+ relu)
// backward: dx = scale * rstd * (g - dbias / M - xhat * dscale / M), g = dy masked by relu
template <typename T>
__global__ void bn_apply_kernel(const T* __restrict__ x, const T* __restrict__ dy, const T* __restrict__ y,
                                T* __restrict__ out, const float* __restrict__ mean, const float* __restrict__ rstd,
                                const float* __restrict__ scale, const float* __restrict__ bias,
                                const float* __restrict__ dbias, const float* __restrict__ dscale, int C, long S,
                                long total, long M, int relu) {
  GRID_STRIDE(i, total) {
    const int c = (int)((i / S) % C);
    const float xh = (IO<T>::ld(x, i) - mean[c]) * rstd[c];
    const float sc = scale ? scale[c] : 1.f;
    if (!dy) {
      float v = xh * sc + (bias ? bias[c] : 0.f);
      if (relu && v < 0.f) v = 0.f;
      IO<T>::st(out, i, v);
    } else {
      float g = IO<T>::ld(dy, i);
      if (relu && IO<T>::ld(y, i) <= 0.f) g = 0.f;
      const float inv = 1.f / (float)M;
      IO<T>::st(out, i, sc * rstd[c] * (g - dbias[c] * inv - xh * dscale[c] * inv));
    }
  }
}

}  // namespace

// Deterministic split-K: the k slices write fp32 partial slabs into a per-device
// workspace and one pass sums them in slice order (no float atomics, so the result
// does not depend on the order in which workgroups finish).  On for every call while
// pa_sgemm_set_deterministic(1) (FLAGS_cudnn_deterministic, the MoE router).
static int g_sgemm_det = 0;
static float* g_sgemm_ws[64];
static size_t g_sgemm_ws_cap[64];

__global__ __launch_bounds__(256) void sgemm_slab_sum_kernel(const float* __restrict__ ws, float* __restrict__ C,
                                                             long mn, int ns, float beta_c) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < mn; i += (long)gridDim.x * 256) {
    float s = 0.f;
    for (int z = 0; z < ns; ++z) s += ws[(long)z * mn + i];
    C[i] = beta_c != 0.f ? C[i] + s : s;
  }
}

static float* sgemm_ws(size_t floats) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (g_sgemm_ws_cap[dev] < floats) {
    if (g_sgemm_ws[dev]) hipFree(g_sgemm_ws[dev]);  // synchronises the device
    g_sgemm_ws[dev] = nullptr;
    g_sgemm_ws_cap[dev] = 0;
    if (hipMalloc(&g_sgemm_ws[dev], floats * sizeof(float)) != hipSuccess) return nullptr;
    g_sgemm_ws_cap[dev] = floats;
  }
  return g_sgemm_ws[dev];
}

PA_EXPORT void pa_sgemm_set_deterministic(int d) { g_sgemm_det = d; }
PA_EXPORT int pa_sgemm_get_deterministic() { return g_sgemm_det; }

// ================================================================ C ABI
PA_EXPORT int pa_sgemm(const float* A, long sam, long sak, const float* B, long sbk, long sbn, float* C, long ldc,
                       long M, long N, long K, int Z1, int Z2, long bsA1, long bsB1, long bsC1, long bsA2, long bsB2,
                       long bsC2, int kb, long kbA, long kbB, const float* bias_m, long bsBias2, float alpha, float beta,
                       int atomic, const int* conv, hipStream_t st) {
  if (M <= 0 || N <= 0) return 0;
  if (Z1 < 1 || Z2 < 1 || kb < 1 || (long)Z1 * Z2 > 65535) return (int)hipErrorInvalidValue;
  const long gy = (M + SBM - 1) / SBM, gx = (N + SBN - 1) / SBN;
  if (gy > 65535 || gx > 2147483647L) return (int)hipErrorInvalidValue;
  SgemmArgs g;
  g.A = A; g.B = B; g.C = C; g.bias_m = bias_m; g.bsBias2 = bsBias2;
  g.M = M; g.N = N; g.K = K;
  g.sam = sam; g.sak = sak; g.sbk = sbk; g.sbn = sbn; g.ldc = ldc;
  g.Z2 = Z2;
  g.bsA1 = bsA1; g.bsB1 = bsB1; g.bsC1 = bsC1;
  g.bsA2 = bsA2; g.bsB2 = bsB2; g.bsC2 = bsC2;
  g.kb = kb; g.kbA = kbA; g.kbB = kbB;
  g.alpha = alpha; g.beta = beta; g.atomic = atomic; g.ksplit = 0;
  g.kbsplit = 0;
  g.nks = 1;
  int det_ns = 0;
  float* det_C = nullptr;
  // split for under-filled problems (few output tiles, deep reduction): the k-batch
  // and / or K are cut into slices on z1, accumulated with float atomics (C zeroed
  // here unless the caller already accumulates atomically)
  const long tiles = gx * gy * Z2;
  const bool can_zero = beta == 0.f && !bias_m && ldc == N && Z2 == 1;
  if (Z1 == 1 && tiles < 192 && (kb > 1 || K >= 256) && (atomic || can_zero)) {
    const long target = (384 + tiles - 1) / tiles;
    long nb = 1, kbs = kb;
    if (kb > 1) {
      nb = target < kb ? target : kb;
      kbs = (kb + nb - 1) / nb;
      nb = (kb + kbs - 1) / kbs;
    }
    long nk = 1, ks = K;
    const long rem = (target + nb - 1) / nb;
    if (rem >= 2 && K >= 256) {
      nk = rem;
      if (nk > K / 128) nk = K / 128;
      if (nk > 64) nk = 64;
      if (nk < 1) nk = 1;
      ks = (K + nk - 1) / nk;
      ks = (ks + SBK - 1) / SBK * SBK;
      nk = (K + ks - 1) / ks;
    }
    float* ws = (g_sgemm_det && !atomic && nb * nk >= 2 && nb * nk * Z2 <= 65535)
                    ? sgemm_ws((size_t)(nb * nk) * M * N) : nullptr;
    if (ws) {
      // deterministic: one slab per split, then an ordered sum into C (after launch)
      det_C = C;
      det_ns = (int)(nb * nk);
      g.C = ws;
      g.atomic = 0;
      g.ksplit = nk > 1 ? ks : 0;
      g.kbsplit = nb > 1 ? (int)kbs : 0;
      g.nks = (int)nk;
      g.bsA1 = g.bsB1 = 0;
      g.bsC1 = M * N;
      Z1 = det_ns;
    } else
    if (nb * nk >= 2 && nb * nk * Z2 <= 65535) {
      if (!atomic && hipMemsetAsync(C, 0, sizeof(float) * M * N, st) != hipSuccess) return (int)hipGetLastError();
      g.atomic = 1;
      g.ksplit = nk > 1 ? ks : 0;
      g.kbsplit = nb > 1 ? (int)kbs : 0;
      g.nks = (int)nk;
      g.bsA1 = g.bsB1 = g.bsC1 = 0;
      Z1 = (int)(nb * nk);
    }
  }
  const dim3 grid((unsigned)gx, (unsigned)gy, (unsigned)(Z1 * Z2));
  g.Z2 = Z2;
#define SG_DONE()                                                                                        \
  do {                                                                                                   \
    if (det_ns) {                                                                                        \
      const hipError_t e_ = hipGetLastError();                                                           \
      if (e_ != hipSuccess) return (int)e_;                                                              \
      const long mn_ = M * N;                                                                            \
      hipLaunchKernelGGL(sgemm_slab_sum_kernel, dim3((unsigned)std::min<long>((mn_ + 255) / 256, 4096)),  \
                         dim3(256), 0, st, g.C, det_C, mn_, det_ns, 0.f);                                \
    }                                                                                                    \
    PA_LAUNCH_CHECK();                                                                                   \
  } while (0)
  const bool ak = sak == 1, bk = sbk == 1;
  // float4 path: 16-B aligned bases and every non-contiguous stride a multiple of 4
  auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  auto m4 = [](long v) { return (v & 3) == 0; };
  if (conv) {  // implicit-GEMM B: conv = {H, W, OW, kh, kw, sh, sw, ph, pw, dh, dw}
    g.cH = conv[0]; g.cW = conv[1]; g.cOW = conv[2]; g.ckh = conv[3]; g.ckw = conv[4];
    g.csh = conv[5]; g.csw = conv[6]; g.cph = conv[7]; g.cpw = conv[8]; g.cdh = conv[9]; g.cdw = conv[10];
    const bool va = al(A) && m4(ak ? sam : sak) && m4(bsA1) && m4(bsA2) && m4(kbA) && (ak ? sak == 1 : sam == 1);
    if (!ak) return (int)hipErrorInvalidValue;  // the conv forms use a k-contiguous A
    if (va) {
      if (bk) hipLaunchKernelGGL((sgemm_kernel<true, true, true, true>), grid, dim3(256), 0, st, g);
      else hipLaunchKernelGGL((sgemm_kernel<true, false, true, true>), grid, dim3(256), 0, st, g);
    } else {
      if (bk) hipLaunchKernelGGL((sgemm_kernel<true, true, false, true>), grid, dim3(256), 0, st, g);
      else hipLaunchKernelGGL((sgemm_kernel<true, false, false, true>), grid, dim3(256), 0, st, g);
    }
    SG_DONE();
  }
  const bool vec = al(A) && al(B) && m4(ak ? sam : sak) && m4(bk ? sbn : sbk) && m4(bsA1) && m4(bsA2) && m4(bsB1) &&
                   m4(bsB2) && m4(kbA) && m4(kbB) && (ak ? sak == 1 : sam == 1) && (bk ? sbk == 1 : sbn == 1);
#define SG(AKv, BKv, V) hipLaunchKernelGGL((sgemm_kernel<AKv, BKv, V, false>), grid, dim3(256), 0, st, g)
  if (vec) {
    if (ak && bk) SG(true, true, true);
    else if (ak) SG(true, false, true);
    else if (bk) SG(false, true, true);
    else SG(false, false, true);
  } else {
    if (ak && bk) SG(true, true, false);
    else if (ak) SG(true, false, false);
    else if (bk) SG(false, true, false);
    else SG(false, false, false);
  }
#undef SG
  SG_DONE();
#undef SG_DONE
}

static Geo make_geo(const int* v) {
  // v: C, D, H, W, OD, OH, OW, kd, kh, kw, sd, sh, sw, pd, ph, pw, dd, dh, dw
  Geo g;
  g.C = v[0]; g.D = v[1]; g.H = v[2]; g.W = v[3];
  g.OD = v[4]; g.OH = v[5]; g.OW = v[6];
  g.kd = v[7]; g.kh = v[8]; g.kw = v[9];
  g.sd = v[10]; g.sh = v[11]; g.sw = v[12];
  g.pd = v[13]; g.ph = v[14]; g.pw = v[15];
  g.dd = v[16]; g.dh = v[17]; g.dw = v[18];
  return g;
}

static bool geo_ok(const Geo& g) {
  return g.C > 0 && g.D > 0 && g.H > 0 && g.W > 0 && g.OD > 0 && g.OH > 0 && g.OW > 0 && g.kd > 0 && g.kh > 0 &&
         g.kw > 0 && g.sd > 0 && g.sh > 0 && g.sw > 0 && g.dd > 0 && g.dh > 0 && g.dw > 0 && g.pd >= 0 && g.ph >= 0 &&
         g.pw >= 0;
}

PA_EXPORT int pa_vol2col(int dt, const void* x, void* col, const int* geo, int nb, hipStream_t st) {
  const Geo g = make_geo(geo);
  if (!geo_ok(g) || nb <= 0) return (int)hipErrorInvalidValue;
  const long total = (long)nb * g.C * g.kd * g.kh * g.kw * g.OD * g.OH * g.OW;
  if (dt == 1)
    hipLaunchKernelGGL(vol2col_kernel<u16>, dim3(grid_for(total)), dim3(256), 0, st, (const u16*)x, (u16*)col, g, nb);
  else
    hipLaunchKernelGGL(vol2col_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, (const float*)x, (float*)col,
                       g, nb);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_col2vol(const float* col, float* x, const int* geo, int nb, int accumulate, hipStream_t st) {
  const Geo g = make_geo(geo);
  if (!geo_ok(g) || nb <= 0) return (int)hipErrorInvalidValue;
  const long total = (long)nb * g.C * g.D * g.H * g.W;
  hipLaunchKernelGGL(col2vol_kernel, dim3(grid_for(total)), dim3(256), 0, st, col, x, g, nb, accumulate);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_chan_sum(const float* y, float* out, int N, int C, long S, int accumulate, hipStream_t st) {
  if (C <= 0 || N <= 0) return 0;
  hipLaunchKernelGGL(chan_sum_kernel, dim3((unsigned)C), dim3(256), 0, st, y, out, N, C, S, accumulate);
  PA_LAUNCH_CHECK();
}

static PoolGeo make_pool(long NC, const int* v) {
  // v: D, H, W, OD, OH, OW, kd, kh, kw, sd, sh, sw, pd, ph, pw
  PoolGeo g;
  g.NC = NC;
  g.D = v[0]; g.H = v[1]; g.W = v[2];
  g.OD = v[3]; g.OH = v[4]; g.OW = v[5];
  g.kd = v[6]; g.kh = v[7]; g.kw = v[8];
  g.sd = v[9]; g.sh = v[10]; g.sw = v[11];
  g.pd = v[12]; g.ph = v[13]; g.pw = v[14];
  return g;
}

static bool pool_ok(const PoolGeo& g) {
  return g.NC > 0 && g.D > 0 && g.H > 0 && g.W > 0 && g.OD > 0 && g.OH > 0 && g.OW > 0 && g.kd > 0 && g.kh > 0 &&
         g.kw > 0 && g.sd > 0 && g.sh > 0 && g.sw > 0 && g.pd >= 0 && g.ph >= 0 && g.pw >= 0;
}

PA_EXPORT int pa_pool_fwd(int dt, const void* x, void* y, int* mask, long NC, const int* geo, int type, int exclusive,
                          hipStream_t st) {
  const PoolGeo g = make_pool(NC, geo);
  if (!pool_ok(g)) return (int)hipErrorInvalidValue;
  const long total = NC * g.OD * g.OH * g.OW;
  if (dt == 1)
    hipLaunchKernelGGL(pool_fwd_kernel<u16>, dim3(grid_for(total)), dim3(256), 0, st, (const u16*)x, (u16*)y, mask, g,
                       type, exclusive);
  else
    hipLaunchKernelGGL(pool_fwd_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, (const float*)x, (float*)y,
                       mask, g, type, exclusive);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_pool_bwd(int dt, const void* dy, const int* mask, void* dx, long NC, const int* geo, int type,
                          int exclusive, hipStream_t st) {
  const PoolGeo g = make_pool(NC, geo);
  if (!pool_ok(g) || (type == 0 && !mask)) return (int)hipErrorInvalidValue;
  const long total = NC * g.D * g.H * g.W;
  if (dt == 1)
    hipLaunchKernelGGL(pool_bwd_kernel<u16>, dim3(grid_for(total)), dim3(256), 0, st, (const u16*)dy, mask, (u16*)dx,
                       g, type, exclusive);
  else
    hipLaunchKernelGGL(pool_bwd_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, (const float*)dy, mask,
                       (float*)dx, g, type, exclusive);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_unpool(int dt, int backward, const void* src, const int* mask, void* dst, long NC, long IS, long OS,
                        int* bad, hipStream_t st) {
  const long total = NC * IS;
  if (total <= 0) return 0;
  if (!backward) {
    if (dt == 1)
      hipLaunchKernelGGL(unpool_fwd_kernel<u16>, dim3(grid_for(total)), dim3(256), 0, st, (const u16*)src, mask,
                         (u16*)dst, NC, IS, OS, bad);
    else
      hipLaunchKernelGGL(unpool_fwd_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, (const float*)src, mask,
                         (float*)dst, NC, IS, OS, bad);
  } else {
    if (dt == 1)
      hipLaunchKernelGGL(unpool_bwd_kernel<u16>, dim3(grid_for(total)), dim3(256), 0, st, (const u16*)src, mask,
                         (u16*)dst, NC, IS, OS);
    else
      hipLaunchKernelGGL(unpool_bwd_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, (const float*)src, mask,
                         (float*)dst, NC, IS, OS);
  }
  PA_LAUNCH_CHECK();
}


static int bn_groups(int C, long M) {
  long g = 2048 / (C > 0 ? C : 1);
  const long cap = (M + 2047) / 2048;
  if (g > cap) g = cap;
  if (g > 1024) g = 1024;
  return (int)(g < 1 ? 1 : g);
}

PA_EXPORT int pa_bn_nchw_groups(int C, long M) { return bn_groups(C, M); }

// Training forward: stats (mean, rstd, running outputs) + normalised output.
// part holds C * G * 2 floats (G = pa_bn_nchw_groups(C, N * S)).
PA_EXPORT int pa_bn_nchw_fwd(int dt, const void* x, void* y, const float* scale, const float* bias,
                             const float* run_mean, const float* run_var, float* mean_out, float* var_out,
                             float* mean, float* rstd, float* part, int N, int C, long S, float eps, float momentum,
                             int training, int relu, int unbiased, hipStream_t st) {
  const long M = (long)N * S, total = M * C;
  if (C <= 0 || M <= 0) return 0;
  const int G = bn_groups(C, M);
#define BN_FWD(T)                                                                                                 \
  if (training)                                                                                                   \
    hipLaunchKernelGGL(bn_partial_kernel<T>, dim3((unsigned)C, (unsigned)G), dim3(256), 0, st, (const T*)x,       \
                       (const T*)nullptr, (const T*)nullptr, (const float*)nullptr, (const float*)nullptr, part, N, C, \
                       S, G, 0);                                                                                  \
  hipLaunchKernelGGL(bn_finalize_kernel<T>, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, st, (const T*)x, part, C, \
                     G, M, eps, momentum, training ? 0 : 2, run_mean, run_var, mean, rstd, training ? mean_out : nullptr, \
                     training ? var_out : nullptr, S, unbiased);                                                  \
  hipLaunchKernelGGL(bn_apply_kernel<T>, dim3(grid_for(total)), dim3(256), 0, st, (const T*)x, (const T*)nullptr,   \
                     (const T*)nullptr, (T*)y, mean, rstd, scale, bias, (const float*)nullptr, (const float*)nullptr, C, \
                     S, total, M, relu);
  if (dt == 1) {
    BN_FWD(u16)
  } else {
    BN_FWD(float)
  }
#undef BN_FWD
  PA_LAUNCH_CHECK();
}

// Backward: dscale, dbias (fp32, [C]) and dx.  y is the forward output (relu mask).
PA_EXPORT int pa_bn_nchw_bwd(int dt, const void* x, const void* dy, const void* y, const float* mean,
                             const float* rstd, const float* scale, float* dscale, float* dbias, void* dx, float* part,
                             int N, int C, long S, int relu, hipStream_t st) {
  const long M = (long)N * S, total = M * C;
  if (C <= 0 || M <= 0) return 0;
  const int G = bn_groups(C, M);
#define BN_BWD(T)                                                                                                  \
  hipLaunchKernelGGL(bn_partial_kernel<T>, dim3((unsigned)C, (unsigned)G), dim3(256), 0, st, (const T*)x,           \
                     (const T*)dy, (const T*)y, mean, rstd, part, N, C, S, G, relu);                                \
  hipLaunchKernelGGL(bn_finalize_kernel<T>, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, st, (const T*)x, part, C, \
                     G, M, 0.f, 0.f, 1, (const float*)nullptr, (const float*)nullptr, dbias, dscale, (float*)nullptr, \
                     (float*)nullptr, S, 0);                                                                        \
  if (dx)                                                                                                          \
    hipLaunchKernelGGL(bn_apply_kernel<T>, dim3(grid_for(total)), dim3(256), 0, st, (const T*)x, (const T*)dy,      \
                       (const T*)y, (T*)dx, mean, rstd, scale, (const float*)nullptr, dbias, dscale, C, S, total, M, relu);
  if (dt == 1) {
    BN_BWD(u16)
  } else {
    BN_BWD(float)
  }
#undef BN_BWD
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_maxout(int dt, const void* x, const void* y, const void* dy, void* out, int N, int Co, int groups,
                        long S, hipStream_t st) {
  const long total = (long)N * Co * S;
  if (total <= 0 || groups < 1) return 0;
  if (!dy) {
    if (dt == 1)
      hipLaunchKernelGGL(maxout_fwd_kernel<u16>, dim3(grid_for(total)), dim3(256), 0, st, (const u16*)x, (u16*)out, N,
                         Co, groups, S);
    else
      hipLaunchKernelGGL(maxout_fwd_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, (const float*)x,
                         (float*)out, N, Co, groups, S);
  } else {
    if (dt == 1)
      hipLaunchKernelGGL(maxout_bwd_kernel<u16>, dim3(grid_for(total)), dim3(256), 0, st, (const u16*)x, (const u16*)y,
                         (const u16*)dy, (u16*)out, N, Co, groups, S);
    else
      hipLaunchKernelGGL(maxout_bwd_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, (const float*)x,
                         (const float*)y, (const float*)dy, (float*)out, N, Co, groups, S);
  }
  PA_LAUNCH_CHECK();
}

}  // namespace pa
