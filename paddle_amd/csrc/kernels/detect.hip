// Detection kernels (reference operators/detection/: iou_similarity_op.h,
// box_coder_op.cu, multiclass_nms_op.cc's NMSFast on the host there).
//
//   iou     : [Na, Nb] Jaccard matrix, +1 pixel convention when not normalized
//   box_coder encode_center_size [N, M, 4] / decode_center_size [N, M, 4]
//   nms     : one workgroup per (image, class) over that pair's score-sorted top-K
//             candidates (K <= 512): the K x K suppression bitmask (IoU > thr, j > i)
//             is built in LDS by all lanes, then a greedy scan walks i in order and
//             ORs kept rows into a removed-set held in LDS.  keep[pair, k] = 1 / 0.
#include "common.h"

namespace pa {
namespace {

constexpr int kNmsMaxK = 512;
constexpr int kNmsWords = kNmsMaxK / 64;

__device__ __forceinline__ float iou4(const float* a, const float* b, float one) {
  const float aw = a[2] - a[0] + one, ah = a[3] - a[1] + one;
  const float bw = b[2] - b[0] + one, bh = b[3] - b[1] + one;
  const float iw = fmaxf(fminf(a[2], b[2]) - fmaxf(a[0], b[0]) + one, 0.f);
  const float ih = fmaxf(fminf(a[3], b[3]) - fmaxf(a[1], b[1]) + one, 0.f);
  const float inter = iw * ih;
  return inter / fmaxf(aw * ah + bw * bh - inter, 1e-10f);
}

__global__ __launch_bounds__(256) void iou_kernel(const float* __restrict__ a, const float* __restrict__ b, int na,
                                                  int nb, float one, float* __restrict__ out) {
  const long total = (long)na * nb;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x)
    out[i] = iou4(a + (i / nb) * 4, b + (i % nb) * 4, one);
}

// encode: tgt [N, 4] against priors [M, 4] -> out [N, M, 4]
__global__ __launch_bounds__(256) void box_encode_kernel(const float* __restrict__ prior, const float* __restrict__ var,
                                                         const float* __restrict__ tgt, int N, int M, float one,
                                                         float* __restrict__ out) {
  const long total = (long)N * M;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int n = (int)(i / M), m = (int)(i % M);
    const float* p = prior + m * 4;
    const float* t = tgt + (long)n * 4;
    const float pw = p[2] - p[0] + one, ph = p[3] - p[1] + one;
    const float pcx = (p[0] + p[2]) * 0.5f, pcy = (p[1] + p[3]) * 0.5f;
    const float tw = t[2] - t[0] + one, th = t[3] - t[1] + one;
    const float tcx = (t[0] + t[2]) * 0.5f, tcy = (t[1] + t[3]) * 0.5f;
    float o[4] = {(tcx - pcx) / pw, (tcy - pcy) / ph, logf(fabsf(tw / pw)), logf(fabsf(th / ph))};
    if (var)
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] /= var[m * 4 + k];
#pragma unroll
    for (int k = 0; k < 4; ++k) out[i * 4 + k] = o[k];
  }
}

// decode: deltas [N, M, 4] against priors [M, 4] -> boxes [N, M, 4]
__global__ __launch_bounds__(256) void box_decode_kernel(const float* __restrict__ prior, const float* __restrict__ var,
                                                         const float* __restrict__ d, int N, int M, float one,
                                                         float* __restrict__ out) {
  const long total = (long)N * M;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int m = (int)(i % M);
    const float* p = prior + m * 4;
    const float pw = p[2] - p[0] + one, ph = p[3] - p[1] + one;
    const float pcx = (p[0] + p[2]) * 0.5f, pcy = (p[1] + p[3]) * 0.5f;
    float v[4] = {1.f, 1.f, 1.f, 1.f};
    if (var)
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = var[m * 4 + k];
    const float* di = d + i * 4;
    const float cx = v[0] * di[0] * pw + pcx, cy = v[1] * di[1] * ph + pcy;
    const float w = expf(v[2] * di[2]) * pw, h = expf(v[3] * di[3]) * ph;
    out[i * 4 + 0] = cx - w * 0.5f;
    out[i * 4 + 1] = cy - h * 0.5f;
    out[i * 4 + 2] = cx + w * 0.5f - one;
    out[i * 4 + 3] = cy + h * 0.5f - one;
  }
}

// boxes [N, Mb, 4]; order [P, K] int32 (candidate box index within the image, score-
// sorted), count [P] valid candidates; pair p -> image p / C.
__global__ __launch_bounds__(256) void nms_kernel(const float* __restrict__ boxes, const int* __restrict__ order,
                                                  const int* __restrict__ count, int C, int Mb, int K, float thr,
                                                  float one, unsigned char* __restrict__ keep) {
  __shared__ unsigned long long mask[kNmsMaxK][kNmsWords];
  __shared__ unsigned long long removed[kNmsWords];
  __shared__ float bx[kNmsMaxK][4];
  const int p = blockIdx.x;
  const int n = min(count[p], K);
  const int img = p / C;
  const int* ord = order + (long)p * K;
  const float* bb = boxes + (long)img * Mb * 4;
  const int words = (n + 63) / 64;
  for (int i = threadIdx.x; i < n; i += 256)
#pragma unroll
    for (int k = 0; k < 4; ++k) bx[i][k] = bb[(long)ord[i] * 4 + k];
  if (threadIdx.x < kNmsWords) removed[threadIdx.x] = 0ull;
  __syncthreads();
  // suppression bitmask: one lane per (row i, 64-column word w)
  for (int t = threadIdx.x; t < n * words; t += 256) {
    const int i = t / words, w = t % words;
    unsigned long long bits = 0ull;
    const int j0 = w * 64;
    for (int b = 0; b < 64; ++b) {
      const int j = j0 + b;
      if (j > i && j < n && iou4(bx[i], bx[j], one) > thr) bits |= 1ull << b;
    }
    mask[i][w] = bits;
  }
  __syncthreads();
  // greedy scan: lane w owns removed word w; every lane reads the decision bit
  for (int i = 0; i < n; ++i) {
    const bool alive = !((removed[i >> 6] >> (i & 63)) & 1ull);
    __syncthreads();
    if (alive && threadIdx.x < words) removed[threadIdx.x] |= mask[i][threadIdx.x];
    if (threadIdx.x == 0) keep[(long)p * K + i] = alive ? 1 : 0;
    __syncthreads();
  }
  for (int i = n + threadIdx.x; i < K; i += 256) keep[(long)p * K + i] = 0;
}

}  // namespace
}  // namespace pa

using namespace pa;

PA_EXPORT int pa_iou_matrix(const float* a, const float* b, int na, int nb, int normalized, float* out,
                            hipStream_t st) {
  if (na < 0 || nb < 0) return -1;
  if ((long)na * nb == 0) return 0;
  hipLaunchKernelGGL(iou_kernel, dim3(stream_grid((long)na * nb, 256)), dim3(256), 0, st, a, b, na, nb,
                     normalized ? 0.f : 1.f, out);
  PA_LAUNCH_CHECK();
}

// encode: t [N, 4]; decode: t [N, M, 4]; var [M, 4] or null
PA_EXPORT int pa_box_coder(int decode, const float* prior, const float* var, const float* t, int N, int M,
                           int normalized, float* out, hipStream_t st) {
  if (N < 0 || M < 0) return -1;
  if ((long)N * M == 0) return 0;
  const dim3 g(stream_grid((long)N * M, 256));
  const float one = normalized ? 0.f : 1.f;
  if (decode)
    hipLaunchKernelGGL(box_decode_kernel, g, dim3(256), 0, st, prior, var, t, N, M, one, out);
  else
    hipLaunchKernelGGL(box_encode_kernel, g, dim3(256), 0, st, prior, var, t, N, M, one, out);
  PA_LAUNCH_CHECK();
}

// P = images * C pairs; K <= 512
PA_EXPORT int pa_nms_bitmask(const float* boxes, const int* order, const int* count, int P, int C, int Mb, int K,
                             float thr, int normalized, unsigned char* keep, hipStream_t st) {
  if (P <= 0 || C <= 0 || K <= 0 || K > kNmsMaxK || Mb <= 0) return -1;
  hipLaunchKernelGGL(nms_kernel, dim3(P), dim3(256), 0, st, boxes, order, count, C, Mb, K, thr,
                     normalized ? 0.f : 1.f, keep);
  PA_LAUNCH_CHECK();
}

// ---------------------------------------------------------------- box generators / target assignment
// prior_box (prior_box_op.cu GenPriorBox): boxes [H, W, P, 4] from the per-prior
// (w, h) list; anchor_generator (anchor_generator_op.cu GenAnchors) in pixels;
// polygon_box_transform (PolygonBoxTransformKernel); target_assign
// (target_assign_op.h / NegTargetAssignKernel).
namespace pa {
namespace {

__global__ void prior_box_kernel(const float* __restrict__ bw, const float* __restrict__ bh, float* __restrict__ boxes,
                                 float* __restrict__ vars, int H, int W, int P, float IW, float IH, float sw, float sh,
                                 float off, int clip, float v0, float v1, float v2, float v3) {
  const long total = (long)H * W * P;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int p = (int)(i % P), w = (int)((i / P) % W), h = (int)(i / ((long)P * W));
    const float cx = (w + off) * sw, cy = (h + off) * sh;
    float b[4] = {(cx - bw[p] * 0.5f) / IW, (cy - bh[p] * 0.5f) / IH, (cx + bw[p] * 0.5f) / IW,
                  (cy + bh[p] * 0.5f) / IH};
    for (int j = 0; j < 4; ++j) {
      float v = b[j];
      if (clip) v = fminf(fmaxf(v, 0.f), 1.f);
      boxes[i * 4 + j] = v;
    }
    vars[i * 4] = v0;
    vars[i * 4 + 1] = v1;
    vars[i * 4 + 2] = v2;
    vars[i * 4 + 3] = v3;
  }
}

__global__ void anchor_kernel(const float* __restrict__ aw, const float* __restrict__ ah, float* __restrict__ anchors,
                              float* __restrict__ vars, int H, int W, int A, float sw, float sh, float off, float v0,
                              float v1, float v2, float v3) {
  const long total = (long)H * W * A;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int a = (int)(i % A), w = (int)((i / A) % W), h = (int)(i / ((long)A * W));
    const float xc = w * sw + off * (sw - 1.f), yc = h * sh + off * (sh - 1.f);
    anchors[i * 4] = xc - 0.5f * (aw[a] - 1.f);
    anchors[i * 4 + 1] = yc - 0.5f * (ah[a] - 1.f);
    anchors[i * 4 + 2] = xc + 0.5f * (aw[a] - 1.f);
    anchors[i * 4 + 3] = yc + 0.5f * (ah[a] - 1.f);
    vars[i * 4] = v0;
    vars[i * 4 + 1] = v1;
    vars[i * 4 + 2] = v2;
    vars[i * 4 + 3] = v3;
  }
}

__global__ void polygon_kernel(const float* __restrict__ x, float* __restrict__ y, long NC, int C, int H, int W) {
  const long total = NC * H * W;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int w = (int)(i % W), h = (int)((i / W) % H), c = (int)((i / ((long)W * H)) % C);
    y[i] = (c % 2 == 0 ? (float)w : (float)h) - x[i];
  }
}

// out[b][p][:] = x[xoff[b] + m][p % Pw][:] for m = match[b][p] >= 0, else mismatch
__global__ void target_assign_kernel(const float* __restrict__ x, const int* __restrict__ xoff,
                                     const long* __restrict__ match, float* __restrict__ out, float* __restrict__ wt,
                                     int N, int P, int Pw, int K, float mismatch) {
  const long total = (long)N * P * K;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int k = (int)(i % K);
    const long bp = i / K;
    const int p = (int)(bp % P), b = (int)(bp / P);
    const long m = match[bp];
    if (m >= 0) {
      out[i] = x[(((long)xoff[b] + m) * Pw + (Pw > 1 ? p % Pw : 0)) * K + k];
      if (k == 0) wt[bp] = 1.f;
    } else {
      out[i] = mismatch;
      if (k == 0) wt[bp] = 0.f;
    }
  }
}

__global__ void neg_assign_kernel(const long* __restrict__ neg, const int* __restrict__ neg_img,
                                  float* __restrict__ out, float* __restrict__ wt, long nneg, int P, int K,
                                  float mismatch) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < nneg * K; i += (long)gridDim.x * blockDim.x) {
    const long e = i / K;
    const int k = (int)(i % K);
    const long bp = (long)neg_img[e] * P + neg[e];
    out[bp * K + k] = mismatch;
    if (k == 0) wt[bp] = 1.f;
  }
}

}  // namespace
}  // namespace pa

using namespace pa;

PA_EXPORT int pa_prior_box(const float* bw, const float* bh, float* boxes, float* vars, int H, int W, int P, float IW,
                           float IH, float sw, float sh, float off, int clip, const float* v, hipStream_t st) {
  const long total = (long)H * W * P;
  if (total <= 0) return 0;
  hipLaunchKernelGGL(prior_box_kernel, dim3(stream_grid(total, 256)), dim3(256), 0, st, bw, bh, boxes, vars, H, W, P,
                     IW, IH, sw, sh, off, clip, v[0], v[1], v[2], v[3]);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_anchor_generator(const float* aw, const float* ah, float* anchors, float* vars, int H, int W, int A,
                                  float sw, float sh, float off, const float* v, hipStream_t st) {
  const long total = (long)H * W * A;
  if (total <= 0) return 0;
  hipLaunchKernelGGL(anchor_kernel, dim3(stream_grid(total, 256)), dim3(256), 0, st, aw, ah, anchors, vars, H, W, A,
                     sw, sh, off, v[0], v[1], v[2], v[3]);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_polygon_box_transform(const float* x, float* y, long NC, int C, int H, int W, hipStream_t st) {
  if (NC * H * W <= 0) return 0;
  hipLaunchKernelGGL(polygon_kernel, dim3(stream_grid(NC * H * W, 256)), dim3(256), 0, st, x, y, NC, C, H, W);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_target_assign(const float* x, const int* xoff, const long* match, const long* neg,
                               const int* neg_img, float* out, float* wt, int N, int P, int Pw, int K, long nneg,
                               float mismatch, hipStream_t st) {
  if ((long)N * P * K > 0)
    hipLaunchKernelGGL(target_assign_kernel, dim3(stream_grid((long)N * P * K, 256)), dim3(256), 0, st, x, xoff, match,
                       out, wt, N, P, Pw, K, mismatch);
  if (nneg > 0)
    hipLaunchKernelGGL(neg_assign_kernel, dim3(stream_grid(nneg * K, 256)), dim3(256), 0, st, neg, neg_img, out, wt,
                       nneg, P, K, mismatch);
  PA_LAUNCH_CHECK();
}
