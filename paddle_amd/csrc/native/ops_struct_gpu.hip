// gfx950 device kernels of linear_chain_crf / linear_chain_crf_grad / crf_decoding
// (semantics: ops_struct.cc).  One workgroup per sequence: lane j owns tag j and the
// time recursion runs in the workgroup, the previous step's log-alpha (or beta)
// row staged in LDS -- the reference's LinearChainCRF forward / backward
// (linear_chain_crf_op.h:54-190) and Viterbi (crf_decoding_op.h) per sequence.
// Transition gradients from all sequences meet in fp32 atomics on the (D + 2) x D
// matrix.
#include <hip/hip_runtime.h>
#include <math.h>

#include <vector>

#include "device_util.h"

namespace pa {
namespace {

__device__ float block_max(float v, float* red) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = red[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); ++i) r = fmaxf(r, red[i]);
  return r;
}
__device__ float block_sum(float v, float* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) r += red[i];
  return r;
}

// log-space forward recursion of sequence s into alpha[s0 .. s0 + L) (rows of [T, D]);
// returns log Z (every thread)
__device__ float crf_alpha(const float* __restrict__ em, const float* __restrict__ tr, int s0, int L, int D,
                           float* __restrict__ alpha, float* prev, float* red) {
  const float* T = tr + 2 * D;
  for (int j = threadIdx.x; j < D; j += blockDim.x) {
    const float a = tr[j] + em[(int64_t)s0 * D + j];
    alpha[(int64_t)s0 * D + j] = a;
    prev[j] = a;
  }
  __syncthreads();
  for (int t = 1; t < L; ++t) {
    float nv[4];
    int c = 0;
    for (int j = threadIdx.x; j < D; j += blockDim.x, ++c) {
      float m = -INFINITY;
      for (int i = 0; i < D; ++i) m = fmaxf(m, prev[i] + T[i * D + j]);
      float sum = 0.f;
      for (int i = 0; i < D; ++i) sum += expf(prev[i] + T[i * D + j] - m);
      nv[c] = m + logf(sum) + em[(int64_t)(s0 + t) * D + j];
    }
    __syncthreads();
    c = 0;
    for (int j = threadIdx.x; j < D; j += blockDim.x, ++c) {
      prev[j] = nv[c];
      alpha[(int64_t)(s0 + t) * D + j] = nv[c];
    }
    __syncthreads();
  }
  float m = -INFINITY;
  for (int j = threadIdx.x; j < D; j += blockDim.x) m = fmaxf(m, prev[j] + tr[D + j]);
  m = block_max(m, red);
  float sum = 0.f;
  for (int j = threadIdx.x; j < D; j += blockDim.x) sum += expf(prev[j] + tr[D + j] - m);
  sum = block_sum(sum, red);
  return m + logf(sum);
}

__device__ float crf_score(const float* em, const float* tr, const long long* y, int s0, int L, int D) {
  const float* T = tr + 2 * D;
  float sc = tr[y[s0]] + em[(int64_t)s0 * D + y[s0]];
  for (int t = 1; t < L; ++t) sc += T[y[s0 + t - 1] * D + y[s0 + t]] + em[(int64_t)(s0 + t) * D + y[s0 + t]];
  return sc + tr[D + y[s0 + L - 1]];
}

__global__ void crf_fwd_kernel(const float* __restrict__ em, const float* __restrict__ tr,
                               const long long* __restrict__ y, const int* __restrict__ off, int D,
                               float* __restrict__ alpha, float* __restrict__ nll) {
  extern __shared__ float sm[];
  float* prev = sm;
  float* red = sm + D;
  const int s = blockIdx.x, s0 = off[s], L = off[s + 1] - s0;
  if (L <= 0) {
    if (threadIdx.x == 0) nll[s] = 0.f;
    return;
  }
  const float logz = crf_alpha(em, tr, s0, L, D, alpha, prev, red);
  if (threadIdx.x == 0) nll[s] = logz - crf_score(em, tr, y, s0, L, D);
}

// backward recursion + marginal-minus-indicator gradients of sequence s
__global__ void crf_bwd_kernel(const float* __restrict__ em, const float* __restrict__ tr,
                               const long long* __restrict__ y, const int* __restrict__ off, int D,
                               const float* __restrict__ g, float* __restrict__ alpha, float* __restrict__ beta,
                               float* __restrict__ dem, float* __restrict__ dtr) {
  extern __shared__ float sm[];
  float* prev = sm;
  float* red = sm + D;
  const int s = blockIdx.x, s0 = off[s], L = off[s + 1] - s0;
  if (L <= 0) return;
  const float gs = g ? g[s] : 1.f;
  const float logz = crf_alpha(em, tr, s0, L, D, alpha, prev, red);
  const float* T = tr + 2 * D;
  for (int j = threadIdx.x; j < D; j += blockDim.x) {
    beta[(int64_t)(s0 + L - 1) * D + j] = tr[D + j];
    prev[j] = tr[D + j] + em[(int64_t)(s0 + L - 1) * D + j];  // beta + emission of step t + 1
  }
  __syncthreads();
  for (int t = L - 2; t >= 0; --t) {
    float nv[4];
    int c = 0;
    for (int i = threadIdx.x; i < D; i += blockDim.x, ++c) {
      float m = -INFINITY;
      for (int j = 0; j < D; ++j) m = fmaxf(m, T[i * D + j] + prev[j]);
      float sum = 0.f;
      for (int j = 0; j < D; ++j) sum += expf(T[i * D + j] + prev[j] - m);
      nv[c] = m + logf(sum);
    }
    __syncthreads();
    c = 0;
    for (int i = threadIdx.x; i < D; i += blockDim.x, ++c) {
      beta[(int64_t)(s0 + t) * D + i] = nv[c];
      prev[i] = nv[c] + em[(int64_t)(s0 + t) * D + i];
    }
    __syncthreads();
  }
  // emission gradients, start / end rows
  for (int t = 0; t < L; ++t)
    for (int j = threadIdx.x; j < D; j += blockDim.x) {
      const int64_t o = (int64_t)(s0 + t) * D + j;
      const float mg = expf(alpha[o] + beta[o] - logz);
      const float ind = y[s0 + t] == j ? 1.f : 0.f;
      dem[o] = gs * (mg - ind);
      if (t == 0) atomicAdd(dtr + j, gs * (mg - ind));
      if (t == L - 1) atomicAdd(dtr + D + j, gs * (mg - (y[s0 + L - 1] == j ? 1.f : 0.f)));
    }
  // pair marginals: dT[i][j] += gs * sum_t p(y_{t-1} = i, y_t = j) - count(i -> j)
  for (int j = threadIdx.x; j < D; j += blockDim.x)
    for (int i = 0; i < D; ++i) {
      float acc = 0.f;
      for (int t = 1; t < L; ++t)
        acc += expf(alpha[(int64_t)(s0 + t - 1) * D + i] + T[i * D + j] + em[(int64_t)(s0 + t) * D + j] +
                    beta[(int64_t)(s0 + t) * D + j] - logz);
      atomicAdd(dtr + (2 + i) * D + j, gs * acc);
    }
  if (threadIdx.x == 0)
    for (int t = 1; t < L; ++t) atomicAdd(dtr + (2 + y[s0 + t - 1]) * D + y[s0 + t], -gs);
}

// Viterbi of sequence s (first maximum on ties, as the host kernel)
__global__ void crf_viterbi_kernel(const float* __restrict__ em, const float* __restrict__ tr,
                                   const int* __restrict__ off, int D, int* __restrict__ back,
                                   const long long* __restrict__ label, long long* __restrict__ path) {
  extern __shared__ float sm[];
  float* score = sm;
  const int s = blockIdx.x, s0 = off[s], L = off[s + 1] - s0;
  if (L <= 0) return;
  const float* T = tr + 2 * D;
  for (int j = threadIdx.x; j < D; j += blockDim.x) score[j] = tr[j] + em[(int64_t)s0 * D + j];
  __syncthreads();
  for (int t = 1; t < L; ++t) {
    float nv[4];
    int c = 0;
    for (int j = threadIdx.x; j < D; j += blockDim.x, ++c) {
      float best = score[0] + T[j];
      int arg = 0;
      for (int i = 1; i < D; ++i) {
        const float v = score[i] + T[i * D + j];
        if (v > best) {
          best = v;
          arg = i;
        }
      }
      nv[c] = best + em[(int64_t)(s0 + t) * D + j];
      back[(int64_t)(s0 + t) * D + j] = arg;
    }
    __syncthreads();
    c = 0;
    for (int j = threadIdx.x; j < D; j += blockDim.x, ++c) score[j] = nv[c];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    int best = 0;
    for (int j = 1; j < D; ++j)
      if (score[j] + tr[D + j] > score[best] + tr[D + best]) best = j;
    for (int t = L - 1; t >= 0; --t) {
      path[s0 + t] = label ? (label[s0 + t] == best ? 1 : 0) : best;
      if (t > 0) best = back[(int64_t)(s0 + t) * D + best];
    }
  }
}

const int* upload_off(const OpRun& r, const Tensor& x, const char* tag, int64_t* nseq) {
  std::vector<int> h;
  if (!x.lod.empty())
    for (size_t v : x.lod.back()) h.push_back((int)v);
  else
    h = {0, (int)x.dims[0]};
  *nseq = (int64_t)h.size() - 1;
  return (const int*)device_upload(r, tag, h.data(), h.size() * sizeof(int));
}

const long long* labels64(const Tensor& t) {
  if (t.dtype != DT::INT64 || t.device < 0) throw Decline{};
  return t.data<long long>();
}

constexpr int kThreads = 256;
constexpr int kMaxTags = 4 * kThreads;  // nv[4] per thread

void k_linear_chain_crf(const OpRun& r) {
  Tensor& emt = r.in("Emission");
  Tensor& trt = r.in("Transition");
  const int64_t T = emt.dims[0], D = emt.dims[1];
  if (D > kMaxTags || trt.dims[0] != D + 2) throw Decline{};
  const float *em = dev_f32(emt), *tr = dev_f32(trt);
  const long long* y = labels64(r.in("Label"));
  int64_t N;
  const int* off = upload_off(r, emt, "@crf_off@", &N);
  const int dev = dev_id(r);
  hipStream_t s = dev_stream(r);
  float* nll = r.out("LogLikelihood")->alloc<float>({N, 1}, dev);
  float* alpha = r.out("Alpha") ? r.out("Alpha")->alloc<float>({T, D}, dev) : device_workspace(r, "@crf_a@", T * D);
  if (N > 0)
    hipLaunchKernelGGL(crf_fwd_kernel, dim3((unsigned)N), dim3(kThreads), (D + 16) * sizeof(float), s, em, tr, y, off,
                       (int)D, alpha, nll);
  // EmissionExps / TransitionExps: intermediates no kernel of this executor reads
  if (Tensor* ee = r.out("EmissionExps")) PA_HIPCHK(hipMemsetAsync(ee->alloc<float>({T, D}, dev), 0, T * D * 4, s));
  if (Tensor* te = r.out("TransitionExps"))
    PA_HIPCHK(hipMemsetAsync(te->alloc<float>(trt.dims, dev), 0, trt.numel() * 4, s));
  PA_HIPCHK(hipGetLastError());
}

void k_linear_chain_crf_grad(const OpRun& r) {
  Tensor& emt = r.in("Emission");
  Tensor& trt = r.in("Transition");
  Tensor* g = r.in_opt("LogLikelihood@GRAD");
  const int64_t T = emt.dims[0], D = emt.dims[1];
  if (D > kMaxTags) throw Decline{};
  const float *em = dev_f32(emt), *tr = dev_f32(trt);
  const float* gp = g ? dev_f32(*g) : nullptr;
  const long long* y = labels64(r.in("Label"));
  int64_t N;
  const int* off = upload_off(r, emt, "@crfg_off@", &N);
  const int dev = dev_id(r);
  hipStream_t s = dev_stream(r);
  Tensor* de = r.out("Emission@GRAD");
  float* dem = de ? de->alloc<float>(emt.dims, dev) : device_workspace(r, "@crf_dem@", T * D);
  if (de) de->lod = emt.lod;
  Tensor* dt = r.out("Transition@GRAD");
  float* dtr = dt ? dt->alloc<float>(trt.dims, dev) : device_workspace(r, "@crf_dtr@", trt.numel());
  PA_HIPCHK(hipMemsetAsync(dem, 0, sizeof(float) * T * D, s));
  PA_HIPCHK(hipMemsetAsync(dtr, 0, sizeof(float) * trt.numel(), s));
  float* alpha = device_workspace(r, "@crfg_a@", T * D);
  float* beta = device_workspace(r, "@crfg_b@", T * D);
  if (N > 0)
    hipLaunchKernelGGL(crf_bwd_kernel, dim3((unsigned)N), dim3(kThreads), (D + 16) * sizeof(float), s, em, tr, y,
                       off, (int)D, gp, alpha, beta, dem, dtr);
  PA_HIPCHK(hipGetLastError());
}

void k_crf_decoding(const OpRun& r) {
  Tensor& emt = r.in("Emission");
  Tensor& trt = r.in("Transition");
  Tensor* lab = r.in_opt("Label");
  const int64_t T = emt.dims[0], D = emt.dims[1];
  if (D > kMaxTags) throw Decline{};
  const float *em = dev_f32(emt), *tr = dev_f32(trt);
  const long long* lp = lab ? labels64(*lab) : nullptr;
  int64_t N;
  const int* off = upload_off(r, emt, "@crfd_off@", &N);
  const int dev = dev_id(r);
  hipStream_t s = dev_stream(r);
  Tensor* out = r.out("ViterbiPath");
  long long* path = reinterpret_cast<long long*>(out->alloc<int64_t>({T, 1}, dev));
  PA_HIPCHK(hipMemsetAsync(path, 0, sizeof(long long) * T, s));
  int* back = reinterpret_cast<int*>(device_workspace(r, "@crfd_back@", T * D));
  if (N > 0)
    hipLaunchKernelGGL(crf_viterbi_kernel, dim3((unsigned)N), dim3(kThreads), D * sizeof(float), s, em, tr, off,
                       (int)D, back, lp, path);
  out->lod = emt.lod;
  PA_HIPCHK(hipGetLastError());
}

}  // namespace

PA_DEVICE_KERNEL(linear_chain_crf, k_linear_chain_crf);
PA_DEVICE_KERNEL(linear_chain_crf_grad, k_linear_chain_crf_grad);
PA_DEVICE_KERNEL(crf_decoding, k_crf_decoding);

}  // namespace pa
