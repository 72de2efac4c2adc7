// Sequence / detection / metric kernels of the op library (SURVEY §2.8 "misc" rows):
//
//   CTC loss + gradient  (warp-ctc replacement; reference operators/warpctc_op.h,
//                        which calls the bundled warp-ctc GPU library)
//   roi_pool fwd / bwd   (operators/roi_pool_op.cu: GPUROIPoolForward / Backward)
//   edit_distance        (operators/edit_distance_op.cu)
//   ctc_align            (operators/ctc_align_op.cu)
//   mean_iou histogram   (operators/mean_iou_op.cu)
//   fake_quantize_*      (operators/fake_quantize_op.cu: FindAbsMaxFunctor + ClipAndFakeQuant)
//   isfinite             (operators/isfinite_op.h)
//   sequence pad / unpad / scale (operators/math/sequence_padding.cu, sequence_scale.cu)
//
// CTC: one workgroup per (sequence, direction) computes the log-space alpha (even
// blocks) or beta (odd blocks) lattice for the blank-extended label of length
// S = 2L + 1, keeping the previous time step in LDS and every step in a global
// workspace; a second kernel (one workgroup per time row) turns alpha + beta into the
// softmax-fused logits gradient  y_tk - exp(lse_{s: l'(s)=k}(a_ts + b_ts) - logp_tk + loss).
#include "common.h"

namespace pa {
namespace {

constexpr int kCtcThreads = 256;
constexpr int kCtcMaxS = 8192;  // 2 * 4095 labels + 1

__device__ __forceinline__ float lse2(float a, float b) {
  const float m = fmaxf(a, b);
  if (m == -INFINITY) return -INFINITY;
  return m + logf(expf(a - m) + expf(b - m));
}

// per-row log-sum-exp of the logits (one wave per row)
__global__ __launch_bounds__(256) void row_lse_kernel(const float* __restrict__ x, float* __restrict__ lse, long rows,
                                                      int C) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = x + row * C;
  float m = -INFINITY;
  for (int c = lane; c < C; c += 64) m = fmaxf(m, xr[c]);
  m = wave_max(m);
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += expf(xr[c] - m);
  s = wave_sum(s);
  if (lane == 0) lse[row] = m + logf(s);
}

__device__ __forceinline__ int ext_label(const int* lab, int s, int blank) { return (s & 1) ? lab[s >> 1] : blank; }

// blockIdx.x = 2 * n + dir (dir 0: alpha, 1: beta).  ws layout [Ttot, Smax].
__global__ __launch_bounds__(kCtcThreads) void ctc_lattice_kernel(const float* __restrict__ x,
                                                                  const float* __restrict__ lse,
                                                                  const int* __restrict__ xoff,
                                                                  const int* __restrict__ labels,
                                                                  const int* __restrict__ loff, int C, int Smax,
                                                                  int blank, float* __restrict__ alpha,
                                                                  float* __restrict__ beta) {
  __shared__ float buf[2][kCtcMaxS];
  const int n = blockIdx.x >> 1, dir = blockIdx.x & 1;
  const int t0 = xoff[n], T = xoff[n + 1] - t0;
  const int* lab = labels + loff[n];
  const int L = loff[n + 1] - loff[n];
  const int S = 2 * L + 1;
  if (T <= 0) return;
  float* ws = (dir == 0 ? alpha : beta) + (long)t0 * Smax;
  auto logp = [&](int t, int s) {
    const int k = ext_label(lab, s, blank);
    return x[(long)(t0 + t) * C + k] - lse[t0 + t];
  };
  int cur = 0;
  // first step
  const int tf = dir == 0 ? 0 : T - 1;
  for (int s = threadIdx.x; s < S; s += kCtcThreads) {
    const bool start = dir == 0 ? (s < 2) : (s >= S - 2);
    const float v = start ? logp(tf, s) : -INFINITY;
    buf[cur][s] = v;
    ws[(long)tf * Smax + s] = v;
  }
  __syncthreads();
  for (int step = 1; step < T; ++step) {
    const int t = dir == 0 ? step : T - 1 - step;
    const int nxt = cur ^ 1;
    for (int s = threadIdx.x; s < S; s += kCtcThreads) {
      float v;
      if (dir == 0) {
        v = buf[cur][s];
        if (s >= 1) v = lse2(v, buf[cur][s - 1]);
        if (s >= 2 && (s & 1) && lab[s >> 1] != lab[(s >> 1) - 1]) v = lse2(v, buf[cur][s - 2]);
      } else {
        v = buf[cur][s];
        if (s + 1 < S) v = lse2(v, buf[cur][s + 1]);
        if (s + 2 < S && (s & 1) && lab[s >> 1] != lab[(s >> 1) + 1]) v = lse2(v, buf[cur][s + 2]);
      }
      v = v == -INFINITY ? v : v + logp(t, s);
      buf[nxt][s] = v;
      ws[(long)t * Smax + s] = v;
    }
    __syncthreads();
    cur = nxt;
  }
}

// loss[n] = -log p(l | x_n); zero_infinity: an impossible alignment gives loss 0
__global__ void ctc_loss_kernel(const float* __restrict__ alpha, const int* __restrict__ xoff,
                                const int* __restrict__ loff, int N, int Smax, float* __restrict__ loss) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const int T = xoff[n + 1] - xoff[n];
  const int S = 2 * (loff[n + 1] - loff[n]) + 1;
  if (T <= 0) {
    loss[n] = 0.f;
    return;
  }
  const float* a = alpha + (long)(xoff[n] + T - 1) * Smax;
  const float lp = S >= 2 ? lse2(a[S - 1], a[S - 2]) : a[S - 1];
  loss[n] = lp == -INFINITY ? 0.f : -lp;
}

__device__ __forceinline__ int seq_of_row(const int* xoff, int N, int row) {
  int lo = 0, hi = N;  // largest n with xoff[n] <= row
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (xoff[mid] <= row) lo = mid; else hi = mid;
  }
  return lo;
}

// one workgroup per time row
__global__ __launch_bounds__(256) void ctc_grad_kernel(const float* __restrict__ x, const float* __restrict__ lse,
                                                       const float* __restrict__ alpha, const float* __restrict__ beta,
                                                       const int* __restrict__ xoff, const int* __restrict__ labels,
                                                       const int* __restrict__ loff, const float* __restrict__ loss,
                                                       int N, int C, int Smax, int blank, float* __restrict__ grad) {
  __shared__ float red[4];
  const int row = blockIdx.x;
  const int n = seq_of_row(xoff, N, row);
  const int T = xoff[n + 1] - xoff[n];
  const int L = loff[n + 1] - loff[n];
  const int S = 2 * L + 1;
  const int* lab = labels + loff[n];
  const float* a = alpha + (long)row * Smax;
  const float* b = beta + (long)row * Smax;
  const float* xr = x + (long)row * C;
  float* g = grad + (long)row * C;
  // an impossible alignment (alpha at the end all -inf) has a zero gradient
  const float* aend = alpha + (long)(xoff[n] + T - 1) * Smax;
  const float lp = S >= 2 ? lse2(aend[S - 1], aend[S - 2]) : aend[S - 1];
  const float ls = lse[row];
  if (lp == -INFINITY) {
    for (int c = threadIdx.x; c < C; c += 256) g[c] = 0.f;
    return;
  }
  (void)loss;
  for (int c = threadIdx.x; c < C; c += 256) g[c] = expf(xr[c] - ls);
  __syncthreads();  // workgroup fence: the softmax row is in L2 before the atomics below
  const float lpb = xr[blank] - ls;
  float bsum = 0.f;
  for (int s = threadIdx.x; s < S; s += 256) {
    const float ab = a[s] + b[s];
    if (ab == -INFINITY) continue;
    if (s & 1) {
      const int k = lab[s >> 1];
      atomicAdd(g + k, -expf(ab - (xr[k] - ls) - lp));
    } else {
      bsum += expf(ab - lpb - lp);
    }
  }
  bsum = block_sum<256>(bsum, red);
  if (threadIdx.x == 0) atomicAdd(g + blank, -bsum);
}

// ---------------------------------------------------------------- roi pool
__global__ __launch_bounds__(256) void roi_pool_fwd_kernel(const float* __restrict__ x, const float* __restrict__ rois,
                                                           const int* __restrict__ bid, int R, int C, int H, int W,
                                                           int PH, int PW, float scale, float* __restrict__ out,
                                                           long long* __restrict__ argmax) {
  const long total = (long)R * C * PH * PW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int pw = (int)(i % PW), ph = (int)((i / PW) % PH), c = (int)((i / PW / PH) % C);
    const int r = (int)(i / PW / PH / C);
    const float* ro = rois + (long)r * 4;
    const int sw = (int)roundf(ro[0] * scale), sh = (int)roundf(ro[1] * scale);
    const int ew = (int)roundf(ro[2] * scale), eh = (int)roundf(ro[3] * scale);
    const int rw = max(ew - sw + 1, 1), rh = max(eh - sh + 1, 1);
    int hs = (int)floor((double)ph * rh / PH), ws = (int)floor((double)pw * rw / PW);
    int he = (int)ceil((double)(ph + 1) * rh / PH), we = (int)ceil((double)(pw + 1) * rw / PW);
    hs = min(max(hs + sh, 0), H);
    he = min(max(he + sh, 0), H);
    ws = min(max(ws + sw, 0), W);
    we = min(max(we + sw, 0), W);
    const bool empty = he <= hs || we <= ws;
    float m = empty ? 0.f : -3.402823466e38f;
    int mi = -1;
    const float* xp = x + ((long)bid[r] * C + c) * H * W;
    for (int h = hs; h < he; ++h)
      for (int w = ws; w < we; ++w) {
        const float v = xp[h * W + w];
        if (v > m) {
          m = v;
          mi = h * W + w;
        }
      }
    out[i] = m;
    argmax[i] = mi;
  }
}

__global__ __launch_bounds__(256) void roi_pool_bwd_kernel(const float* __restrict__ dy,
                                                           const long long* __restrict__ argmax,
                                                           const int* __restrict__ bid, int R, int C, int H, int W,
                                                           int PH, int PW, float* __restrict__ dx) {
  const long total = (long)R * C * PH * PW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long long am = argmax[i];
    if (am < 0) continue;
    const int c = (int)((i / PW / PH) % C), r = (int)(i / PW / PH / C);
    atomicAdd(dx + ((long)bid[r] * C + c) * H * W + am, dy[i]);
  }
}

// ---------------------------------------------------------------- edit distance
// one lane per (hyp, ref) pair; two DP rows of the reference length in `ws`
__global__ void edit_distance_kernel(const long long* __restrict__ hyp, const int* __restrict__ hoff,
                                     const long long* __restrict__ ref, const int* __restrict__ roff, int N, int wsw,
                                     int* __restrict__ ws, int normalized, float* __restrict__ out) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const long long* a = hyp + hoff[n];
  const long long* b = ref + roff[n];
  const int la = hoff[n + 1] - hoff[n], lb = roff[n + 1] - roff[n];
  int* prev = ws + (long)n * 2 * wsw;
  int* cur = prev + wsw;
  for (int j = 0; j <= lb; ++j) prev[j] = j;
  for (int i = 1; i <= la; ++i) {
    cur[0] = i;
    const long long ai = a[i - 1];
    for (int j = 1; j <= lb; ++j) {
      const int sub = prev[j - 1] + (ai != b[j - 1]);
      cur[j] = min(min(prev[j] + 1, cur[j - 1] + 1), sub);
    }
    int* t = prev;
    prev = cur;
    cur = t;
  }
  float d = (float)prev[lb];
  if (normalized) d /= (float)max(lb, 1);
  out[n] = d;
}

// ---------------------------------------------------------------- ctc align
// one lane per sequence: drop blanks (and repeats when merge) into out[off[n]..]
__global__ void ctc_align_kernel(const long long* __restrict__ in, const int* __restrict__ off, int N, int blank,
                                 int merge, long long* __restrict__ out, int* __restrict__ counts) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  int k = off[n];
  long long prev = -1;
  bool has_prev = false;
  for (int t = off[n]; t < off[n + 1]; ++t) {
    const long long v = in[t];
    if (v != blank && !(merge && has_prev && v == prev)) out[k++] = v;
    prev = v;
    has_prev = true;
  }
  counts[n] = k - off[n];
}

// ---------------------------------------------------------------- mean iou
template <typename I>
__global__ void iou_hist_kernel(const I* __restrict__ pred, const I* __restrict__ lab, long n, int C,
                                int* __restrict__ correct, int* __restrict__ wrong) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long p = (long)pred[i], l = (long)lab[i];
    if (p < 0 || p >= C || l < 0 || l >= C) continue;
    if (p == l) {
      atomicAdd(correct + p, 1);
    } else {
      atomicAdd(wrong + p, 1);
      atomicAdd(wrong + l, 1);
    }
  }
}

// ---------------------------------------------------------------- fake quant
// |x| max as the bit pattern of a non-negative float (monotone as unsigned)
__global__ __launch_bounds__(256) void absmax_kernel(const float* __restrict__ x, long n,
                                                     unsigned* __restrict__ out) {
  __shared__ float red[4];
  float m = 0.f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    m = fmaxf(m, fabsf(x[i]));
  m = block_max<256>(m, red);
  if (threadIdx.x == 0) atomicMax(out, __float_as_uint(m));
}

// scale = max(absmax, in_scale?) (or in_scale when use_in); out = round(clip(x) / s * bins)
__global__ __launch_bounds__(256) void fake_quant_kernel(const float* __restrict__ x, long n,
                                                         const unsigned* __restrict__ amax,
                                                         const float* __restrict__ in_scale, int use_in, int clip,
                                                         float bins, float* __restrict__ out,
                                                         float* __restrict__ scale_out) {
  float s = use_in ? in_scale[0] : __uint_as_float(amax[0]);
  if (!use_in && in_scale) s = fmaxf(s, in_scale[0]);
  const float inv = 1.f / fmaxf(s, 1e-30f);
  if (blockIdx.x == 0 && threadIdx.x == 0) scale_out[0] = s;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float v = x[i];
    if (clip) v = fminf(fmaxf(v, -s), s);
    out[i] = rintf(v * inv * bins);
  }
}

// ---------------------------------------------------------------- isfinite
template <typename T>
__global__ __launch_bounds__(256) void isfinite_kernel(const T* __restrict__ x, long n, int* __restrict__ bad) {
  int any = 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    any |= !isfinite(IO<T>::ld(x, i));
  if (__any(any) && (threadIdx.x & 63) == 0) atomicOr(bad, 1);
}

// ---------------------------------------------------------------- sequence pad / unpad / scale
template <typename T>
__global__ __launch_bounds__(256) void seq_pad_kernel(const T* __restrict__ x, const int* __restrict__ off, int N,
                                                      int maxlen, long D, const T* __restrict__ padv, int padw,
                                                      T* __restrict__ out) {
  const long total = (long)N * maxlen * D;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long d = i % D;
    const int t = (int)((i / D) % maxlen), n = (int)(i / D / maxlen);
    const int len = off[n + 1] - off[n];
    out[i] = t < len ? x[(long)(off[n] + t) * D + d] : padv[padw == 1 ? 0 : d];
  }
}

template <typename T>
__global__ __launch_bounds__(256) void seq_unpad_kernel(const T* __restrict__ p, const int* __restrict__ off, int N,
                                                        int maxlen, long D, long rows, T* __restrict__ out) {
  const long total = rows * D;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long d = i % D;
    const int row = (int)(i / D);
    const int n = seq_of_row(off, N, row);
    out[i] = p[((long)n * maxlen + (row - off[n])) * D + d];
  }
}

template <typename T>
__global__ __launch_bounds__(256) void seq_scale_kernel(T* __restrict__ x, const int* __restrict__ off, int N, long D,
                                                        long rows, const float* __restrict__ sc) {
  const long total = rows * D;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int n = seq_of_row(off, N, (int)(i / D));
    IO<T>::st(x, i, IO<T>::ld(x, i) * sc[n]);
  }
}

}  // namespace
}  // namespace pa

using namespace pa;

// CTC: logits f32 [Ttot, C]; xoff / loff int32 [N + 1] (device); labels int32 packed;
// workspaces lse [Ttot], alpha / beta [Ttot * Smax] with Smax >= 2 * max L + 1 <= 8192.
PA_EXPORT int pa_ctc_loss(const float* x, const int* xoff, const int* labels, const int* loff, int N, int Ttot, int C,
                          int Smax, int blank, float* lse, float* alpha, float* beta, float* loss, float* grad,
                          hipStream_t st) {
  if (N <= 0 || Ttot < 0 || C <= 0 || Smax < 1 || Smax > kCtcMaxS || blank < 0 || blank >= C) return -1;
  if (Ttot > 0) {
    hipLaunchKernelGGL(row_lse_kernel, dim3((Ttot + 3) / 4), dim3(256), 0, st, x, lse, (long)Ttot, C);
    hipLaunchKernelGGL(ctc_lattice_kernel, dim3(2 * N), dim3(kCtcThreads), 0, st, x, lse, xoff, labels, loff, C, Smax,
                       blank, alpha, beta);
  }
  hipLaunchKernelGGL(ctc_loss_kernel, dim3((N + 255) / 256), dim3(256), 0, st, alpha, xoff, loff, N, Smax, loss);
  if (grad && Ttot > 0)
    hipLaunchKernelGGL(ctc_grad_kernel, dim3(Ttot), dim3(256), 0, st, x, lse, alpha, beta, xoff, labels, loff, loss,
                       N, C, Smax, blank, grad);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_roi_pool_fwd(const float* x, const float* rois, const int* bid, int R, int C, int H, int W, int PH,
                              int PW, float scale, float* out, long long* argmax, hipStream_t st) {
  if (R < 0 || C <= 0 || PH <= 0 || PW <= 0) return -1;
  if (R == 0) return 0;
  hipLaunchKernelGGL(roi_pool_fwd_kernel, dim3(stream_grid((long)R * C * PH * PW, 256)), dim3(256), 0, st, x, rois,
                     bid, R, C, H, W, PH, PW, scale, out, argmax);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_roi_pool_bwd(const float* dy, const long long* argmax, const int* bid, int R, int C, int H, int W,
                              int PH, int PW, float* dx, hipStream_t st) {
  if (R < 0 || C <= 0 || PH <= 0 || PW <= 0) return -1;
  if (R == 0) return 0;
  hipLaunchKernelGGL(roi_pool_bwd_kernel, dim3(stream_grid((long)R * C * PH * PW, 256)), dim3(256), 0, st, dy, argmax,
                     bid, R, C, H, W, PH, PW, dx);
  PA_LAUNCH_CHECK();
}

// ws: int32 [N * 2 * wsw], wsw >= max ref length + 1
PA_EXPORT int pa_edit_distance(const long long* hyp, const int* hoff, const long long* ref, const int* roff, int N,
                               int wsw, int* ws, int normalized, float* out, hipStream_t st) {
  if (N <= 0 || wsw < 1) return -1;
  hipLaunchKernelGGL(edit_distance_kernel, dim3((N + 63) / 64), dim3(64), 0, st, hyp, hoff, ref, roff, N, wsw, ws,
                     normalized, out);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_ctc_align(const long long* in, const int* off, int N, int blank, int merge, long long* out,
                           int* counts, hipStream_t st) {
  if (N <= 0) return -1;
  hipLaunchKernelGGL(ctc_align_kernel, dim3((N + 63) / 64), dim3(64), 0, st, in, off, N, blank, merge, out, counts);
  PA_LAUNCH_CHECK();
}

// correct / wrong: int32 [C], zeroed; idx64: predictions / labels are int64 (else int32)
PA_EXPORT int pa_mean_iou_hist(const void* pred, const void* lab, long n, int C, int idx64, int* correct, int* wrong,
                               hipStream_t st) {
  if (C <= 0 || n < 0) return -1;
  if (n == 0) return 0;
  const dim3 g(stream_grid(n, 256));
  if (idx64)
    hipLaunchKernelGGL(iou_hist_kernel<long long>, g, dim3(256), 0, st, (const long long*)pred, (const long long*)lab,
                       n, C, correct, wrong);
  else
    hipLaunchKernelGGL(iou_hist_kernel<int>, g, dim3(256), 0, st, (const int*)pred, (const int*)lab, n, C, correct,
                       wrong);
  PA_LAUNCH_CHECK();
}

// amax: one zeroed uint32 of workspace; in_scale may be null; use_in: take in_scale as
// the scale (is_test); clip: clamp x to [-s, s] first (range_abs_max)
PA_EXPORT int pa_fake_quant(const float* x, long n, int bit_length, const float* in_scale, int use_in, int clip,
                            unsigned* amax, float* out, float* scale_out, hipStream_t st) {
  if (n < 0 || bit_length < 2 || bit_length > 16 || (use_in && !in_scale)) return -1;
  const dim3 g(stream_grid(n > 0 ? n : 1, 256));
  if (!use_in && n > 0) hipLaunchKernelGGL(absmax_kernel, g, dim3(256), 0, st, x, n, amax);
  const float bins = (float)((1 << (bit_length - 1)) - 1);
  hipLaunchKernelGGL(fake_quant_kernel, g, dim3(256), 0, st, x, n, amax, in_scale, use_in, clip, bins, out,
                     scale_out);
  PA_LAUNCH_CHECK();
}

// bad: one zeroed int32; set to 1 when any element is inf / nan.  dtype 0 f32, 1 bf16
PA_EXPORT int pa_isfinite(const void* x, long n, int dtype, int* bad, hipStream_t st) {
  if (n < 0) return -1;
  if (n == 0) return 0;
  const dim3 g(stream_grid(n, 256));
  if (dtype == 0)
    hipLaunchKernelGGL(isfinite_kernel<float>, g, dim3(256), 0, st, (const float*)x, n, bad);
  else if (dtype == 1)
    hipLaunchKernelGGL(isfinite_kernel<u16>, g, dim3(256), 0, st, (const u16*)x, n, bad);
  else
    return -1;
  PA_LAUNCH_CHECK();
}

// padded [N, maxlen, D]; pad value: padw == 1 (scalar) or D elements.  elem: 4 or 2 bytes
PA_EXPORT int pa_seq_pad(const void* x, const int* off, int N, int maxlen, long D, const void* padv, int padw,
                         int elem, void* out, hipStream_t st) {
  if (N <= 0 || maxlen < 0 || D <= 0) return -1;
  if (maxlen == 0) return 0;
  const dim3 g(stream_grid((long)N * maxlen * D, 256));
  if (elem == 4)
    hipLaunchKernelGGL(seq_pad_kernel<float>, g, dim3(256), 0, st, (const float*)x, off, N, maxlen, D,
                       (const float*)padv, padw, (float*)out);
  else if (elem == 2)
    hipLaunchKernelGGL(seq_pad_kernel<u16>, g, dim3(256), 0, st, (const u16*)x, off, N, maxlen, D, (const u16*)padv,
                       padw, (u16*)out);
  else
    return -1;
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_seq_unpad(const void* p, const int* off, int N, int maxlen, long D, long rows, int elem, void* out,
                           hipStream_t st) {
  if (N <= 0 || D <= 0 || rows < 0) return -1;
  if (rows == 0) return 0;
  const dim3 g(stream_grid(rows * D, 256));
  if (elem == 4)
    hipLaunchKernelGGL(seq_unpad_kernel<float>, g, dim3(256), 0, st, (const float*)p, off, N, maxlen, D, rows,
                       (float*)out);
  else if (elem == 2)
    hipLaunchKernelGGL(seq_unpad_kernel<u16>, g, dim3(256), 0, st, (const u16*)p, off, N, maxlen, D, rows,
                       (u16*)out);
  else
    return -1;
  PA_LAUNCH_CHECK();
}

// in place: x[row, :] *= sc[seq(row)]; dtype 0 f32, 1 bf16
PA_EXPORT int pa_seq_scale(void* x, const int* off, int N, long D, long rows, const float* sc, int dtype,
                           hipStream_t st) {
  if (N <= 0 || D <= 0 || rows < 0) return -1;
  if (rows == 0) return 0;
  const dim3 g(stream_grid(rows * D, 256));
  if (dtype == 0)
    hipLaunchKernelGGL(seq_scale_kernel<float>, g, dim3(256), 0, st, (float*)x, off, N, D, rows, sc);
  else if (dtype == 1)
    hipLaunchKernelGGL(seq_scale_kernel<u16>, g, dim3(256), 0, st, (u16*)x, off, N, D, rows, sc);
  else
    return -1;
  PA_LAUNCH_CHECK();
}
