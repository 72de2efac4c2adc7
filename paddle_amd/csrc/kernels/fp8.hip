// fp8 (OCP e4m3fn) quantisation for the fp8 GEMM (gemm.hip pa_gemm_f8): both
// operands are consumed K-major, with fp32 scales applied in the GEMM epilogue.
//
//   quant_rows:   q[r, :] = x[r, :] / s[r],  s[r] = amax_k |x[r, k]| / 448
//                 (activations per token; weights used K-major as stored)
//   quant_cols_t: qt[g, n, :] = w[g, :, n] / s[g, n],  s[g, n] = amax_k |w[g, k, n]| / 448
//                 (Paddle [in, out] weights -> K-major [out, in] per output channel)
//
// f32 -> e4m3 by v_cvt_pk_fp8_f32 (gfx950: OCP encoding, round-to-nearest-even;
// inputs pre-clamped to +-448 so nothing saturates to NaN).
#include "common.h"

namespace pa {

constexpr float kE4M3Max = 448.f;

__device__ __forceinline__ uint32_t cvt4_fp8(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return (uint32_t)w;
}

__device__ __forceinline__ float clamp448(float v) { return fminf(fmaxf(v, -kE4M3Max), kE4M3Max); }

// one wave per row; K % 16 == 0; 16 elements (2 x 16 B in, 16 B out) per lane-step
__global__ __launch_bounds__(256) void quant_rows_kernel(const u16* __restrict__ x, long ldx, uint8_t* __restrict__ q,
                                                         long ldq, float* __restrict__ scale, long R, int K) {
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const int lane = threadIdx.x & 63;
  const u16* xr = x + r * ldx;
  float amax = 0.f;
  for (int c = lane * 16; c < K; c += 1024) {
    float a[8], b[8];
    load8(xr + c, a);
    load8(xr + c + 8, b);
#pragma unroll
    for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fmaxf(fabsf(a[e]), fabsf(b[e])));
  }
  amax = wave_max(amax);
  const float s = amax > 0.f ? amax / kE4M3Max : 1.f;
  const float inv = 1.f / s;
  if (lane == 0) scale[r] = s;
  uint8_t* qr = q + r * ldq;
  for (int c = lane * 16; c < K; c += 1024) {
    float a[8], b[8];
    load8(xr + c, a);
    load8(xr + c + 8, b);
    uint4 o;
    o.x = cvt4_fp8(clamp448(a[0] * inv), clamp448(a[1] * inv), clamp448(a[2] * inv), clamp448(a[3] * inv));
    o.y = cvt4_fp8(clamp448(a[4] * inv), clamp448(a[5] * inv), clamp448(a[6] * inv), clamp448(a[7] * inv));
    o.z = cvt4_fp8(clamp448(b[0] * inv), clamp448(b[1] * inv), clamp448(b[2] * inv), clamp448(b[3] * inv));
    o.w = cvt4_fp8(clamp448(b[4] * inv), clamp448(b[5] * inv), clamp448(b[6] * inv), clamp448(b[7] * inv));
    *reinterpret_cast<uint4*>(qr + c) = o;
  }
}

// single-pass variant for K <= 1024 * NCH: the row stays in registers between the
// amax reduction and the quantised store (one HBM read instead of two)
template <int NCH>
__global__ __launch_bounds__(256) void quant_rows_reg_kernel(const u16* __restrict__ x, long ldx,
                                                             uint8_t* __restrict__ q, long ldq,
                                                             float* __restrict__ scale, long R, int K) {
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const int lane = threadIdx.x & 63;
  const u16* xr = x + r * ldx;
  u16x8 v[NCH][2];
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = lane * 16 + i * 1024;
    if (c < K) {
      v[i][0] = *reinterpret_cast<const u16x8*>(xr + c);
      v[i][1] = *reinterpret_cast<const u16x8*>(xr + c + 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fmaxf(fabsf(bf2f(v[i][0][e])), fabsf(bf2f(v[i][1][e]))));
    }
  }
  amax = wave_max(amax);
  const float s = amax > 0.f ? amax / kE4M3Max : 1.f;
  const float inv = 1.f / s;
  if (lane == 0) scale[r] = s;
  uint8_t* qr = q + r * ldq;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = lane * 16 + i * 1024;
    if (c < K) {
      float f[16];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        f[e] = clamp448(bf2f(v[i][0][e]) * inv);
        f[8 + e] = clamp448(bf2f(v[i][1][e]) * inv);
      }
      uint4 o;
      o.x = cvt4_fp8(f[0], f[1], f[2], f[3]);
      o.y = cvt4_fp8(f[4], f[5], f[6], f[7]);
      o.z = cvt4_fp8(f[8], f[9], f[10], f[11]);
      o.w = cvt4_fp8(f[12], f[13], f[14], f[15]);
      *reinterpret_cast<uint4*>(qr + c) = o;
    }
  }
}

// column amax of w[g] ([Kd, N] row-major): block = (g, 64 columns); 256 threads =
// 8 column chunks (8 bf16 = 16 B) x 32 row lanes, reduced through LDS.
__global__ __launch_bounds__(256) void col_amax_kernel(const u16* __restrict__ w, float* __restrict__ scale, int Kd,
                                                       int N) {
  __shared__ float red[32][65];
  const int g = blockIdx.y, n0 = blockIdx.x * 64;
  const int ch = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const u16* wg = w + (long)g * Kd * N;
  float m[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int n = n0 + ch * 8;
  if (n < N) {
    for (int k = rl; k < Kd; k += 32) {
      float v[8];
      load8(wg + (long)k * N + n, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) m[e] = fmaxf(m[e], fabsf(v[e]));
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[rl][ch * 8 + e] = m[e];
  __syncthreads();
  if (threadIdx.x < 64) {
    float a = 0.f;
    for (int i = 0; i < 32; ++i) a = fmaxf(a, red[i][threadIdx.x]);
    const int nn = n0 + threadIdx.x;
    if (nn < N) scale[(long)g * N + nn] = a > 0.f ? a / kE4M3Max : 1.f;
  }
}

// transpose-quantise a 64 (k) x 64 (n) tile of w[g] into qt[g] ([N, Kd] row-major)
__global__ __launch_bounds__(256) void quant_cols_t_kernel(const u16* __restrict__ w, const float* __restrict__ scale,
                                                           uint8_t* __restrict__ qt, int Kd, int N) {
  __shared__ float tile[64][65];
  const int g = blockIdx.z, k0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  const u16* wg = w + (long)g * Kd * N;
  // load: 64 rows x 8 chunks of 8 columns -> 512 chunk loads, 2 per thread
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int idx = it * 256 + threadIdx.x, r = idx >> 3, c = (idx & 7) * 8;
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (k0 + r < Kd && n0 + c < N) load8(wg + (long)(k0 + r) * N + n0 + c, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) tile[r][c + e] = v[e];
  }
  __syncthreads();
  // store: 64 n-rows x 4 chunks of 16 k -> 256 stores of 16 B, one per thread
  const int nr = threadIdx.x >> 2, kc = (threadIdx.x & 3) * 16;
  const int n = n0 + nr;
  if (n >= N || k0 + kc >= Kd) return;
  const float inv = 1.f / scale[(long)g * N + n];
  float f[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) f[e] = clamp448(tile[kc + e][nr] * inv);
  uint4 o;
  o.x = cvt4_fp8(f[0], f[1], f[2], f[3]);
  o.y = cvt4_fp8(f[4], f[5], f[6], f[7]);
  o.z = cvt4_fp8(f[8], f[9], f[10], f[11]);
  o.w = cvt4_fp8(f[12], f[13], f[14], f[15]);
  *reinterpret_cast<uint4*>(qt + (long)g * N * Kd + (long)n * Kd + k0 + kc) = o;
}

}  // namespace pa

using namespace pa;

PA_EXPORT int pa_quant_rows_f8(const void* x, long ldx, void* q, long ldq, float* scale, long R, int K,
                               hipStream_t st) {
  if (R <= 0) return 0;
  if (K % 16 || ldx % 8 || ldq % 16) return -1;
  const dim3 grid((unsigned)((R + 3) / 4));
  const int nch = (K + 1023) / 1024;
#define PA_QR(N)                                                                                                 \
  if (nch == N) {                                                                                                \
    hipLaunchKernelGGL(quant_rows_reg_kernel<N>, grid, dim3(256), 0, st, (const u16*)x, ldx, (uint8_t*)q, ldq, \
                       scale, R, K);                                                                             \
    PA_LAUNCH_CHECK();                                                                                           \
  }
  PA_QR(1) PA_QR(2) PA_QR(3) PA_QR(4) PA_QR(5) PA_QR(6) PA_QR(7) PA_QR(8)
#undef PA_QR
  hipLaunchKernelGGL(quant_rows_kernel, grid, dim3(256), 0, st, (const u16*)x, ldx, (uint8_t*)q, ldq, scale, R, K);
  PA_LAUNCH_CHECK();
}

// w: [G, Kd, N] bf16 -> qt: [G, N, Kd] e4m3, scale: [G, N]
PA_EXPORT int pa_quant_cols_t_f8(const void* w, void* qt, float* scale, int G, int Kd, int N, hipStream_t st) {
  if (G <= 0) return 0;
  if (N % 8 || Kd % 16) return -1;
  hipLaunchKernelGGL(col_amax_kernel, dim3((N + 63) / 64, G), dim3(256), 0, st, (const u16*)w, scale, Kd, N);
  hipLaunchKernelGGL(quant_cols_t_kernel, dim3((N + 63) / 64, (Kd + 63) / 64, G), dim3(256), 0, st, (const u16*)w,
                     (const float*)scale, (uint8_t*)qt, Kd, N);
  PA_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------
// Grouped expert dW images (gemm.hip grp_mode 2 with K-major operands): dW_g =
// X_g^T dY_g needs both operands K-major over the TOKENS, i.e. the expert-sorted rows
// transposed.  Each expert's tokens -- gathered over up to 8 micro-batches, whose
// rows [offs_j[g], offs_j[g+1]) are concatenated in micro-batch order -- are placed
// at a 64-aligned column poffs[g] of the transposed image q [C][ldq] (zero-filled up
// to the next multiple of 64), so every K-major 16-B load of the GEMM is aligned and
// the padding adds 0.  One GEMM then reduces an expert over all micro-batches of a
// step (one fp32 main_grad write instead of a read-modify-write per micro-batch).
// fp8 images: s[g, c] = amax over the expert's tokens / 448, q = x / s (e4m3);
// bf16 images: a plain transposed copy.
namespace pa {

constexpr int kGT = 64;  // tokens per tile (and the padding granule)
constexpr int kMaxMb = 8;

struct MbSrc {
  const u16* x[kMaxMb];
  long ldx[kMaxMb];
  const int* offs[kMaxMb];
  int n;
};

// cum[j * G + g] = tokens of expert g in micro-batches < j (j = 0..n); poffs [G+1]
__global__ void group_cat_offsets_kernel(MbSrc src, int G, int* __restrict__ cum, int* __restrict__ poffs) {
  if (threadIdx.x != 0) return;
  int acc = 0;
  for (int g = 0; g < G; ++g) {
    int c = 0;
    for (int j = 0; j < src.n; ++j) {
      cum[j * G + g] = c;
      c += src.offs[j][g + 1] - src.offs[j][g];
    }
    cum[src.n * G + g] = c;
    poffs[g] = acc;
    acc += (c + kGT - 1) / kGT * kGT;
  }
  poffs[G] = acc;
}

// group of padded token column pt (binary search over poffs); -1 past the end
__device__ __forceinline__ int group_of(const int* __restrict__ poffs, int G, long pt) {
  if (pt >= poffs[G]) return -1;
  int lo = 0, hi = G - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (poffs[mid] <= pt) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// source row of token t of expert g (t < total): micro-batch j and its row
__device__ __forceinline__ const u16* token_row(const MbSrc& src, const int* __restrict__ cum, int G, int g, int t) {
  int j = 0;
  while (j + 1 < src.n && t >= cum[(j + 1) * G + g]) ++j;
  const long r = src.offs[j][g] + (t - cum[j * G + g]);
  return src.x[j] + r * src.ldx[j];
}

// amax[g, c] = max |x[token, c]| over the expert's tokens (amax zero-filled by the
// host); grid (token tiles of the padded extent, C / 64), 256 threads: 8 channels
// per thread
__global__ __launch_bounds__(256) void group_amax_kernel(MbSrc src, const int* __restrict__ cum,
                                                         const int* __restrict__ poffs, int G, int C,
                                                         float* __restrict__ amax) {
  const long pt = (long)blockIdx.x * kGT;
  const int g = group_of(poffs, G, pt);
  if (g < 0) return;  // block-uniform
  const int t0 = (int)(pt - poffs[g]), tot = cum[src.n * G + g];
  const int c0 = blockIdx.y * 64;
  const int tc = threadIdx.x & 7, tr = threadIdx.x >> 3;  // 8 channel chunks x 32 rows
  float m[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int i = tr; i < kGT; i += 32) {
    const int t = t0 + i;
    if (t < tot) {
      const u16x8 v = *reinterpret_cast<const u16x8*>(token_row(src, cum, G, g, t) + c0 + 8 * tc);
#pragma unroll
      for (int e = 0; e < 8; ++e) m[e] = fmaxf(m[e], fabsf(bf2f(v[e])));
    }
  }
  __shared__ float red[32][65];
#pragma unroll
  for (int e = 0; e < 8; ++e) red[tr][8 * tc + e] = m[e];
  __syncthreads();
  if (threadIdx.x < 64) {
    float v = 0.f;
    for (int i = 0; i < 32; ++i) v = fmaxf(v, red[i][threadIdx.x]);
    // non-negative floats order like their bit patterns: integer max is float max
    atomicMax(reinterpret_cast<int*>(amax) + (long)g * C + c0 + threadIdx.x, __float_as_int(v));
  }
}

// q[c, poffs[g] + t] = x[token t of g, c] (/ s[g, c] for fp8) for the expert's
// tokens, 0 in its padding; fp8: s[g, c] written alongside.  grid as above.
template <bool QUANT>
__global__ __launch_bounds__(256) void group_image_kernel(MbSrc src, const int* __restrict__ cum,
                                                          const int* __restrict__ poffs, int G, int C,
                                                          const float* __restrict__ amax, void* __restrict__ qv,
                                                          long ldq, float* __restrict__ scale) {
  const long pt = (long)blockIdx.x * kGT;
  const int g = group_of(poffs, G, pt);
  if (g < 0) return;
  const int t0 = (int)(pt - poffs[g]), tot = cum[src.n * G + g];
  const int c0 = blockIdx.y * 64;
  __shared__ u16 tile[kGT][64 + 8];  // [token][channel], rows padded against bank conflicts
  {
    const int tc = threadIdx.x & 7, tr = threadIdx.x >> 3;
    for (int i = tr; i < kGT; i += 32) {
      const int t = t0 + i;
      u16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
      if (t < tot) v = *reinterpret_cast<const u16x8*>(token_row(src, cum, G, g, t) + c0 + 8 * tc);
#pragma unroll
      for (int e = 0; e < 8; ++e) tile[i][8 * tc + e] = v[e];
    }
  }
  __syncthreads();
  const int c = threadIdx.x >> 2, j0 = (threadIdx.x & 3) * 16;  // one channel, 16 tokens
  if constexpr (QUANT) {
    const float am = amax[(long)g * C + c0 + c];
    const float sc = am > 0.f ? am / kE4M3Max : 1.f;
    const float inv = 1.f / sc;
    if ((threadIdx.x & 3) == 0) scale[(long)g * C + c0 + c] = sc;
    float f[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) f[e] = clamp448(bf2f(tile[j0 + e][c]) * inv);
    uint4 o;
    o.x = cvt4_fp8(f[0], f[1], f[2], f[3]);
    o.y = cvt4_fp8(f[4], f[5], f[6], f[7]);
    o.z = cvt4_fp8(f[8], f[9], f[10], f[11]);
    o.w = cvt4_fp8(f[12], f[13], f[14], f[15]);
    *reinterpret_cast<uint4*>((uint8_t*)qv + (long)(c0 + c) * ldq + pt + j0) = o;
  } else {
    u16x8 a, b;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      a[e] = tile[j0 + e][c];
      b[e] = tile[j0 + 8 + e][c];
    }
    u16* d = (u16*)qv + (long)(c0 + c) * ldq + pt + j0;
    *reinterpret_cast<u16x8*>(d) = a;
    *reinterpret_cast<u16x8*>(d + 8) = b;
  }
}

static int mb_src(MbSrc& s, int n, const void* const* xs, const long* ldx, const int* const* offs) {
  if (n <= 0 || n > kMaxMb) return -1;
  s.n = n;
  for (int j = 0; j < n; ++j) {
    if (!xs[j] || !offs[j] || (ldx[j] % 8)) return -1;
    s.x[j] = (const u16*)xs[j];
    s.ldx[j] = ldx[j];
    s.offs[j] = offs[j];
  }
  return 0;
}

}  // namespace pa

// Offsets of the concatenated grouped image: offs[j] (device int [G+1], expert row
// offsets of micro-batch j, j < n <= 8) -> cum [(n+1) * G] (ws) and poffs [G+1].
// Only the offset pointers of xs-less callers are read (xs may be null here).
PA_EXPORT int pa_group_cat_offsets(int n, const int* const* offs, int G, int* cum, int* poffs, hipStream_t st) {
  if (G <= 0 || n <= 0 || n > pa::kMaxMb) return -1;
  pa::MbSrc s{};
  s.n = n;
  for (int j = 0; j < n; ++j) s.offs[j] = offs[j];
  hipLaunchKernelGGL(pa::group_cat_offsets_kernel, dim3(1), dim3(64), 0, st, s, G, cum, poffs);
  PA_LAUNCH_CHECK();
}

// Transposed image of the concatenated expert rows: xs[j] [R_j, C] bf16 (row stride
// ldx[j]), C % 64 == 0 -> q [C][ldq] (quant: e4m3 + scale [G][C], amax [G][C] fp32
// workspace; else bf16), ldq >= sum R_j + 64 G and a multiple of 64, columns past
// poffs[G] untouched.  cum / poffs from pa_group_cat_offsets.
PA_EXPORT int pa_group_image(int quant, int n, const void* const* xs, const long* ldx, const int* const* offs,
                             const int* cum, const int* poffs, int G, long R, int C, float* amax, void* q, long ldq,
                             float* scale, hipStream_t st) {
  pa::MbSrc s{};
  if (pa::mb_src(s, n, xs, ldx, offs)) return -1;
  if (G <= 0 || C <= 0 || (C % 64) || (ldq % 64) || ldq < R + 64L * G) return -1;
  const long tiles = (R + 64L * G + pa::kGT - 1) / pa::kGT;
  if (tiles > 0x7fffffffL || C / 64 > 65535) return -1;
  dim3 grid((unsigned)tiles, C / 64);
  if (quant) {
    if (!amax || !scale) return -1;
    hipError_t e = hipMemsetAsync(amax, 0, sizeof(float) * (size_t)G * C, st);
    if (e != hipSuccess) return (int)e;
    // experts without tokens get no tile: their scales stay 0 (the GEMM's 0 * s stays 0)
    e = hipMemsetAsync(scale, 0, sizeof(float) * (size_t)G * C, st);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(pa::group_amax_kernel, grid, dim3(256), 0, st, s, cum, poffs, G, C, amax);
    hipLaunchKernelGGL(pa::group_image_kernel<true>, grid, dim3(256), 0, st, s, cum, poffs, G, C, (const float*)amax,
                       q, ldq, scale);
  } else {
    hipLaunchKernelGGL(pa::group_image_kernel<false>, grid, dim3(256), 0, st, s, cum, poffs, G, C, nullptr, q, ldq,
                       nullptr);
  }
  PA_LAUNCH_CHECK();
}
