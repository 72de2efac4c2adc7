// gfx950 device kernels of the native executor (fp32 inference / training ops on
// HBM-resident tensors).  Ops without a device kernel here run through the
// executor's host fallback (inputs copied to host, outputs back to HBM).
//
// GEMM (mul / fc / matmul / conv2d's im2col product) runs on the exact-f32 matrix
// cores: v_mfma_f32_32x32x2_f32 over a 128x128x32 LDS-tiled block of 4 wave64s
// (each wave a 64x64 quadrant = 2x2 MFMA tiles), operands addressed through
// (row, k) strides so transposed layouts need no copy; bias / relu / beta fused in
// the epilogue.  gfx950 has no xf32 path, so f32 MFMA is bit-for-bit an f32 FMA
// chain (cdna_hip_programming.md, "FP32-input MFMA").
#include <hip/hip_runtime.h>
#include <math.h>
#include <string.h>

#include <algorithm>

#include "framework.h"

namespace pa {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

#define HIPCHK(x)                                                                  \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) ::pa::fail("%s failed: %s", #x, hipGetErrorString(e_)); \
  } while (0)

inline hipStream_t S(const OpRun& r) { return (hipStream_t)r.ctx.stream; }
inline int D(const OpRun& r) { return r.ctx.device; }

int grid_for(int64_t n, int block = 256) {
  int64_t g = (n + block - 1) / block;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, 256 * 16));
}

using Dims = std::vector<int64_t>;
int64_t prod(const Dims& d, size_t b = 0, size_t e = (size_t)-1) {
  int64_t n = 1;
  for (size_t i = b; i < std::min(e, d.size()); ++i) n *= d[i];
  return n;
}

float* f32(Tensor& t) {
  PA_CHECK(t.dtype == DT::FP32, "expected float32 tensor, got %s", dt_name(t.dtype));
  PA_CHECK(t.device >= 0, "expected a device tensor");
  return t.data<float>();
}

// =============================================================== f32 MFMA GEMM
struct GemmArgs {
  const float* A;
  const float* B;
  float* C;
  const float* bias;  // [N] or null
  int64_t M, N, K;
  int64_t sam, sak;  // A(m, k) = A[m*sam + k*sak]
  int64_t sbk, sbn;  // B(k, n) = B[k*sbk + n*sbn]
  int64_t ldc;
  int64_t bsA, bsB, bsC;  // batch strides
  float alpha, beta;
  int relu;
};

constexpr int BM = 128, BN = 128, BK = 32, LPAD = 4;

__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmArgs g) {
  __shared__ float As[BK][BM + LPAD];
  __shared__ float Bs[BK][BN + LPAD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t bz = blockIdx.z;
  const float* A = g.A + bz * g.bsA;
  const float* B = g.B + bz * g.bsB;
  float* C = g.C + bz * g.bsC;
  const int64_t m0 = (int64_t)blockIdx.y * BM, n0 = (int64_t)blockIdx.x * BN;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  f32x16 acc[2][2];
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j)
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  // loaders: A tile 128 x 32; when A is k-contiguous (sak == 1) a thread walks k
  const bool a_k_fast = g.sak == 1, b_n_fast = g.sbn == 1;
  for (int64_t k0 = 0; k0 < g.K; k0 += BK) {
    for (int e = tid; e < BM * BK; e += 256) {
      int mm, kk;
      if (a_k_fast) { mm = e / BK; kk = e % BK; } else { kk = e / BM; mm = e % BM; }
      const int64_t m = m0 + mm, k = k0 + kk;
      As[kk][mm] = (m < g.M && k < g.K) ? A[m * g.sam + k * g.sak] : 0.f;
    }
    for (int e = tid; e < BN * BK; e += 256) {
      int nn, kk;
      if (b_n_fast) { kk = e / BN; nn = e % BN; } else { nn = e / BK; kk = e % BK; }
      const int64_t n = n0 + nn, k = k0 + kk;
      Bs[kk][nn] = (n < g.N && k < g.K) ? B[k * g.sbk + n * g.sbn] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      const int k = kk + (lane >> 5);
      const float a0 = As[k][wm + (lane & 31)], a1 = As[k][wm + 32 + (lane & 31)];
      const float b0 = Bs[k][wn + (lane & 31)], b1 = Bs[k][wn + 32 + (lane & 31)];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    __syncthreads();
  }
  // C/D map of 32x32: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j) {
      const int64_t n = n0 + wn + 32 * j + (lane & 31);
      if (n >= g.N) continue;
      const float bv = g.bias ? g.bias[n] : 0.f;
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m >= g.M) continue;
        float v = g.alpha * acc[i][j][r] + bv;
        if (g.beta != 0.f) v += g.beta * C[m * g.ldc + n];
        if (g.relu) v = v > 0.f ? v : 0.f;
        C[m * g.ldc + n] = v;
      }
    }
}

void gemm(hipStream_t s, bool ta, bool tb, int64_t M, int64_t N, int64_t K, float alpha, const float* A,
          int64_t lda, const float* B, int64_t ldb, float beta, float* C, int64_t ldc, const float* bias = nullptr,
          bool relu = false, int64_t batch = 1, int64_t bsA = 0, int64_t bsB = 0, int64_t bsC = 0) {
  if (M <= 0 || N <= 0) return;
  GemmArgs g;
  g.A = A; g.B = B; g.C = C; g.bias = bias;
  g.M = M; g.N = N; g.K = K;
  g.sam = ta ? 1 : lda; g.sak = ta ? lda : 1;
  g.sbk = tb ? 1 : ldb; g.sbn = tb ? ldb : 1;
  g.ldc = ldc; g.bsA = bsA; g.bsB = bsB; g.bsC = bsC;
  g.alpha = alpha; g.beta = beta; g.relu = relu ? 1 : 0;
  PA_CHECK(batch <= 65535, "gemm: batch %lld too large", (long long)batch);
  dim3 grid((unsigned)((N + BN - 1) / BN), (unsigned)((M + BM - 1) / BM), (unsigned)batch);
  PA_CHECK(grid.y <= 65535u, "gemm: M too large for the grid");
  hipLaunchKernelGGL(gemm_f32_kernel, grid, dim3(256), 0, s, g);
  HIPCHK(hipGetLastError());
}

// =============================================================== elementwise
constexpr int kMaxR = 6;
struct BcArgs {
  int R;
  int64_t out[kMaxR], sx[kMaxR], sy[kMaxR];
  int64_t n;
};

enum BinOp { B_ADD, B_SUB, B_MUL, B_DIV, B_MAX, B_MIN, B_POW };

__device__ inline float bin(int op, float a, float b) {
  switch (op) {
    case B_ADD: return a + b;
    case B_SUB: return a - b;
    case B_MUL: return a * b;
    case B_DIV: return a / b;
    case B_MAX: return a > b ? a : b;
    case B_MIN: return a < b ? a : b;
    default: return powf(a, b);
  }
}

__global__ void binary_kernel(BcArgs b, int op, const float* __restrict__ x, const float* __restrict__ y,
                              float* __restrict__ o) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < b.n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t rem = i, ox = 0, oy = 0;
    for (int d = b.R - 1; d >= 0; --d) {
      const int64_t k = rem % b.out[d];
      rem /= b.out[d];
      ox += k * b.sx[d];
      oy += k * b.sy[d];
    }
    o[i] = bin(op, x[ox], y[oy]);
  }
}

// x [pre, n, post] (op) y [n]: the common bias / per-channel case, no index math per dim
__global__ void binary_pnp_kernel(int op, const float* __restrict__ x, const float* __restrict__ y,
                                  float* __restrict__ o, int64_t total, int64_t n, int64_t post) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x)
    o[i] = bin(op, x[i], y[(i / post) % n]);
}

bool make_bc(const Dims& x, const Dims& y, int64_t axis, BcArgs* b, int64_t* pre, int64_t* n, int64_t* post) {
  const int64_t xr = (int64_t)x.size();
  if ((int64_t)y.size() > xr || xr > kMaxR) return false;
  if (axis < 0) axis = xr - (int64_t)y.size();
  Dims yf((size_t)xr, 1);
  for (size_t i = 0; i < y.size(); ++i) yf[(size_t)axis + i] = y[i];
  b->R = (int)xr;
  int64_t s1 = 1, s2 = 1;
  for (int64_t i = xr - 1; i >= 0; --i) {
    PA_CHECK(x[(size_t)i] == yf[(size_t)i] || yf[(size_t)i] == 1, "elementwise: Y does not broadcast to X");
    b->out[i] = x[(size_t)i];
    b->sx[i] = s1;
    b->sy[i] = yf[(size_t)i] == 1 ? 0 : s2;
    s1 *= x[(size_t)i];
    s2 *= yf[(size_t)i];
  }
  b->n = s1;
  // contiguous-block form: y's non-1 dims form one run [a, e) equal to x's
  int64_t a = -1, e = -1;
  for (int64_t i = 0; i < xr; ++i)
    if (yf[(size_t)i] != 1) {
      if (a < 0) a = i;
      e = i + 1;
    }
  bool run = true;
  for (int64_t i = a; a >= 0 && i < e; ++i) run &= yf[(size_t)i] == x[(size_t)i];
  if (a < 0) { a = xr; e = xr; }
  *pre = prod(x, 0, (size_t)a);
  *n = prod(x, (size_t)a, (size_t)e);
  *post = prod(x, (size_t)e);
  return run;
}

template <int OP> void k_binary(const OpRun& r) {
  Tensor x = r.in("X");
  Tensor y = r.in("Y");
  BcArgs b;
  int64_t pre, n, post;
  const bool pnp = make_bc(x.dims, y.dims, r.op.GetInt("axis", -1), &b, &pre, &n, &post);
  PA_CHECK(b.R <= kMaxR, "elementwise: rank");
  Tensor* o = r.out("Out");
  LoD lod = x.lod;
  Dims d = x.dims;
  float* op = o->alloc<float>(d, D(r));
  o->lod = lod;
  if (b.n == 0) return;
  if (pnp)
    hipLaunchKernelGGL(binary_pnp_kernel, dim3(grid_for(b.n)), dim3(256), 0, S(r), OP, f32(x), f32(y), op, b.n,
                       n, post);
  else
    hipLaunchKernelGGL(binary_kernel, dim3(grid_for(b.n)), dim3(256), 0, S(r), b, OP, f32(x), f32(y), op);
}

enum UnOp { U_RELU, U_SIGMOID, U_TANH, U_EXP, U_LOG, U_SQRT, U_ABS, U_SQUARE, U_SCALE, U_LEAKY, U_GELU,
            U_RELU6, U_SOFTPLUS, U_SWISH, U_HSIG, U_ELU, U_RECIP };

__device__ inline float un(int op, float v, float p0, float p1) {
  switch (op) {
    case U_RELU: return v > 0.f ? v : 0.f;
    case U_SIGMOID: return 1.f / (1.f + __expf(-v));
    case U_TANH: return tanhf(v);
    case U_EXP: return __expf(v);
    case U_LOG: return __logf(v);
    case U_SQRT: return sqrtf(v);
    case U_ABS: return fabsf(v);
    case U_SQUARE: return v * v;
    case U_SCALE: return v * p0 + p1;
    case U_LEAKY: return v > 0.f ? v : v * p0;
    case U_GELU: return 0.5f * v * (1.f + erff(v * 0.70710678f));
    case U_RELU6: return fminf(fmaxf(v, 0.f), p0);
    case U_SOFTPLUS: return v > 20.f ? v : log1pf(__expf(v));
    case U_SWISH: return v / (1.f + __expf(-p0 * v));
    case U_HSIG: return fminf(1.f, fmaxf(0.f, v * p0 + p1));
    case U_ELU: return v > 0.f ? v : p0 * (__expf(v) - 1.f);
    default: return 1.f / v;
  }
}

__global__ void unary_kernel(int op, float p0, float p1, const float* __restrict__ x, float* __restrict__ o,
                             int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    o[i] = un(op, x[i], p0, p1);
}

void launch_unary(const OpRun& r, Tensor& x, Tensor* o, int op, float p0, float p1) {
  Tensor xs = x;
  LoD lod = x.lod;
  Dims d = x.dims;
  float* op_ = o->alloc<float>(d, D(r));
  o->lod = lod;
  if (xs.numel())
    hipLaunchKernelGGL(unary_kernel, dim3(grid_for(xs.numel())), dim3(256), 0, S(r), op, p0, p1, f32(xs), op_,
                       xs.numel());
}

template <int OP> void k_unary(const OpRun& r) {
  float p0 = 0.f, p1 = 0.f;
  switch (OP) {
    case U_LEAKY: p0 = r.op.GetFloat("alpha", 0.02f); break;
    case U_RELU6: p0 = r.op.GetFloat("threshold", 6.f); break;
    case U_SWISH: p0 = r.op.GetFloat("beta", 1.f); break;
    case U_HSIG: p0 = r.op.GetFloat("slope", 0.2f); p1 = r.op.GetFloat("offset", 0.5f); break;
    case U_ELU: p0 = r.op.GetFloat("alpha", 1.f); break;
    default: break;
  }
  launch_unary(r, r.in("X"), r.out("Out"), OP, p0, p1);
}

void k_scale(const OpRun& r) {
  const float s = r.op.GetFloat("scale", 1.f), b = r.op.GetFloat("bias", 0.f);
  const bool after = r.op.GetBool("bias_after_scale", true);
  launch_unary(r, r.in("X"), r.out("Out"), U_SCALE, s, after ? b : b * s);
}

void k_dropout(const OpRun& r) {
  PA_CHECK(r.ctx.is_test || r.op.GetBool("is_test"), "dropout: device kernel is inference-only");
  const float p = r.op.GetFloat("dropout_prob", 0.5f);
  const bool upscale = r.op.GetString("dropout_implementation", "downgrade_in_infer") == "upscale_in_train";
  launch_unary(r, r.in("X"), r.out("Out"), U_SCALE, upscale ? 1.f : 1.f - p, 0.f);
}

// =============================================================== GEMM ops
void k_mul(const OpRun& r) {
  Tensor x = r.in("X");
  Tensor y = r.in("Y");
  const size_t xnc = (size_t)r.op.GetInt("x_num_col_dims", 1), ync = (size_t)r.op.GetInt("y_num_col_dims", 1);
  const int64_t M = prod(x.dims, 0, xnc), K = prod(x.dims, xnc), N = prod(y.dims, ync);
  PA_CHECK(prod(y.dims, 0, ync) == K, "mul: X %s and Y %s do not match", x.shape_str().c_str(),
           y.shape_str().c_str());
  Dims od(x.dims.begin(), x.dims.begin() + xnc);
  od.insert(od.end(), y.dims.begin() + ync, y.dims.end());
  Tensor* o = r.out("Out");
  float* c = o->alloc<float>(od, D(r));
  o->lod = x.lod;
  gemm(S(r), false, false, M, N, K, 1.f, f32(x), K, f32(y), N, 0.f, c, N);
}

void k_fc(const OpRun& r) {
  Tensor x = r.in("Input");
  Tensor w = r.in("W");
  Tensor* b = r.in_opt("Bias");
  const size_t nc = (size_t)r.op.GetInt("in_num_col_dims", 1);
  const int64_t M = prod(x.dims, 0, nc), K = prod(x.dims, nc), N = w.dims[1];
  Dims od(x.dims.begin(), x.dims.begin() + nc);
  od.push_back(N);
  Tensor* o = r.out("Out");
  float* c = o->alloc<float>(od, D(r));
  o->lod = x.lod;
  gemm(S(r), false, false, M, N, K, 1.f, f32(x), K, f32(w), N, 0.f, c, N, b ? f32(*b) : nullptr,
       r.op.GetString("activation_type") == "relu");
}

void k_matmul(const OpRun& r) {
  Tensor x = r.in("X");
  Tensor y = r.in("Y");
  const bool tx = r.op.GetBool("transpose_X"), ty = r.op.GetBool("transpose_Y");
  const float alpha = r.op.GetFloat("alpha", 1.f);
  Dims xd = x.dims, yd = y.dims;
  const bool xv = xd.size() == 1, yv = yd.size() == 1;
  if (xv) xd = tx ? Dims{xd[0], 1} : Dims{1, xd[0]};
  if (yv) yd = ty ? Dims{1, yd[0]} : Dims{yd[0], 1};
  const int64_t xr = xd[xd.size() - 2], xc = xd.back(), yr = yd[yd.size() - 2], yc = yd.back();
  const int64_t M = tx ? xc : xr, K = tx ? xr : xc, N = ty ? yr : yc;
  PA_CHECK((ty ? yc : yr) == K, "matmul: inner dims differ");
  const int64_t bx = prod(xd, 0, xd.size() - 2), by = prod(yd, 0, yd.size() - 2);
  PA_CHECK(bx == by || bx == 1 || by == 1, "matmul: batch dims differ");
  Dims od = xd.size() >= yd.size() ? Dims(xd.begin(), xd.end() - 2) : Dims(yd.begin(), yd.end() - 2);
  if (bx == 1 && by > 1) od.assign(yd.begin(), yd.end() - 2);
  if (!xv) od.push_back(M);
  if (!yv) od.push_back(N);
  if (od.empty()) od.push_back(1);
  Tensor* o = r.out("Out");
  float* c = o->alloc<float>(od, D(r));
  gemm(S(r), tx, ty, M, N, K, alpha, f32(x), tx ? M : K, f32(y), ty ? K : N, 0.f, c, N, nullptr, false,
       std::max(bx, by), bx == 1 ? 0 : M * K, by == 1 ? 0 : K * N, M * N);
}

// =============================================================== conv2d (im2col + MFMA GEMM)
__global__ void im2col_kernel(const float* __restrict__ x, float* __restrict__ col, int C, int H, int W, int kh,
                              int kw, int sh, int sw, int ph, int pw, int dh, int dw, int OH, int OW) {
  const int64_t total = (int64_t)C * kh * kw * OH * OW;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int ow = (int)(i % OW);
    int64_t t = i / OW;
    const int oh = (int)(t % OH);
    t /= OH;
    const int j = (int)(t % kw);
    t /= kw;
    const int ii = (int)(t % kh);
    const int c = (int)(t / kh);
    const int ih = oh * sh - ph + ii * dh, iw = ow * sw - pw + j * dw;
    col[i] = (ih >= 0 && ih < H && iw >= 0 && iw < W) ? x[((int64_t)c * H + ih) * W + iw] : 0.f;
  }
}

void k_conv2d(const OpRun& r) {
  Tensor x = r.in("Input");
  Tensor w = r.in("Filter");
  auto st = r.op.GetInts("strides"), pd = r.op.GetInts("paddings"), dl = r.op.GetInts("dilations");
  if (st.empty()) st = {1, 1};
  if (pd.empty()) pd = {0, 0};
  if (dl.empty()) dl = {1, 1};
  const int64_t g = std::max<int64_t>(1, r.op.GetInt("groups", 1));
  const int64_t N = x.dims[0], C = x.dims[1], H = x.dims[2], W = x.dims[3];
  const int64_t OC = w.dims[0], kh = w.dims[2], kw = w.dims[3];
  PA_CHECK(w.dims[1] * g == C, "conv2d: filter / input channel mismatch");
  const int64_t OH = (H + 2 * pd[0] - (dl[0] * (kh - 1) + 1)) / st[0] + 1;
  const int64_t OW = (W + 2 * pd[1] - (dl[1] * (kw - 1) + 1)) / st[1] + 1;
  Tensor* o = r.out("Output");
  float* op = o->alloc<float>({N, OC, OH, OW}, D(r));
  const int64_t Cg = C / g, OCg = OC / g, Kc = Cg * kh * kw, P = OH * OW;
  Variable* cv = r.scope.Var("@conv_col@");  // im2col workspace kept across ops / runs
  float* col = cv->tensor.alloc<float>({Kc, P}, D(r));
  const float* xp = f32(x);
  const float* wp = f32(w);
  for (int64_t n = 0; n < N; ++n)
    for (int64_t gi = 0; gi < g; ++gi) {
      hipLaunchKernelGGL(im2col_kernel, dim3(grid_for(Kc * P)), dim3(256), 0, S(r), xp + (n * C + gi * Cg) * H * W,
                         col, (int)Cg, (int)H, (int)W, (int)kh, (int)kw, (int)st[0], (int)st[1], (int)pd[0],
                         (int)pd[1], (int)dl[0], (int)dl[1], (int)OH, (int)OW);
      gemm(S(r), false, false, OCg, P, Kc, 1.f, wp + gi * OCg * Kc, Kc, col, P, 0.f, op + (n * OC + gi * OCg) * P,
           P);
    }
}

// =============================================================== pooling / batch norm
__global__ void pool2d_kernel(const float* __restrict__ x, float* __restrict__ o, int64_t NC, int H, int W, int OH,
                              int OW, int kh, int kw, int sh, int sw, int ph, int pw, int is_max, int excl) {
  const int64_t total = NC * OH * OW;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int ow = (int)(i % OW), oh = (int)((i / OW) % OH);
    const int64_t nc = i / ((int64_t)OW * OH);
    const int h0 = oh * sh - ph, w0 = ow * sw - pw;
    const int h1 = min(h0 + kh, H), w1 = min(w0 + kw, W), hs = max(h0, 0), ws = max(w0, 0);
    const float* xi = x + nc * H * W;
    float acc = is_max ? -INFINITY : 0.f;
    for (int h = hs; h < h1; ++h)
      for (int w = ws; w < w1; ++w) acc = is_max ? fmaxf(acc, xi[h * W + w]) : acc + xi[h * W + w];
    if (!is_max) acc /= (float)max(1, excl ? (h1 - hs) * (w1 - ws) : kh * kw);
    o[i] = acc;
  }
}

void k_pool2d(const OpRun& r) {
  Tensor x = r.in("X");
  const bool is_max = r.op.GetString("pooling_type", "max") == "max";
  auto ks = r.op.GetInts("ksize"), st = r.op.GetInts("strides"), pd = r.op.GetInts("paddings");
  if (st.empty()) st = {1, 1};
  if (pd.empty()) pd = {0, 0};
  const int64_t N = x.dims[0], C = x.dims[1], H = x.dims[2], W = x.dims[3];
  if (r.op.GetBool("global_pooling")) {
    ks = {H, W};
    pd = {0, 0};
  }
  const bool ceil = r.op.GetBool("ceil_mode"), excl = r.op.GetBool("exclusive", true);
  auto osz = [&](int64_t in, int64_t k, int64_t p, int64_t s) {
    return ceil ? (in - k + 2 * p + s - 1) / s + 1 : (in - k + 2 * p) / s + 1;
  };
  const int64_t OH = osz(H, ks[0], pd[0], st[0]), OW = osz(W, ks[1], pd[1], st[1]);
  float* o = r.out("Out")->alloc<float>({N, C, OH, OW}, D(r));
  hipLaunchKernelGGL(pool2d_kernel, dim3(grid_for(N * C * OH * OW)), dim3(256), 0, S(r), f32(x), o, N * C, (int)H,
                     (int)W, (int)OH, (int)OW, (int)ks[0], (int)ks[1], (int)st[0], (int)st[1], (int)pd[0],
                     (int)pd[1], is_max ? 1 : 0, excl ? 1 : 0);
}

__global__ void bn_infer_kernel(const float* __restrict__ x, float* __restrict__ y, const float* __restrict__ sc,
                                const float* __restrict__ bi, const float* __restrict__ mean,
                                const float* __restrict__ var, float eps, int64_t total, int64_t C, int64_t HW,
                                int nhwc) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = nhwc ? i % C : (i / HW) % C;
    const float a = sc[c] * rsqrtf(var[c] + eps);
    y[i] = (x[i] - mean[c]) * a + bi[c];
  }
}

void k_batch_norm(const OpRun& r) {
  PA_CHECK(r.ctx.is_test || r.op.GetBool("is_test") || r.op.GetBool("use_global_stats"),
           "batch_norm: device kernel is inference-only");
  Tensor x = r.in("X");
  const bool nhwc = r.op.GetString("data_layout", "NCHW") == "NHWC";
  const int64_t N = x.dims[0], C = nhwc ? x.dims.back() : x.dims[1], HW = x.numel() / (N * C);
  Dims d = x.dims;
  float* y = r.out("Y")->alloc<float>(d, D(r));
  hipLaunchKernelGGL(bn_infer_kernel, dim3(grid_for(x.numel())), dim3(256), 0, S(r), f32(x), y, f32(r.in("Scale")),
                     f32(r.in("Bias")), f32(r.in("Mean")), f32(r.in("Variance")), r.op.GetFloat("epsilon", 1e-5f),
                     x.numel(), C, HW, nhwc ? 1 : 0);
}

// =============================================================== softmax (one wave per row)
__global__ void softmax_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t rows, int64_t n) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = x + row * n;
  float* yr = y + row * n;
  float m = -INFINITY;
  for (int64_t j = lane; j < n; j += 64) m = fmaxf(m, xr[j]);
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  float s = 0.f;
  for (int64_t j = lane; j < n; j += 64) s += __expf(xr[j] - m);
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  const float inv = 1.f / s;
  for (int64_t j = lane; j < n; j += 64) yr[j] = __expf(xr[j] - m) * inv;
}

void k_softmax(const OpRun& r) {
  Tensor x = r.in("X");
  int64_t axis = r.op.GetInt("axis", -1);
  if (axis < 0) axis += (int64_t)x.dims.size();
  PA_CHECK(axis == (int64_t)x.dims.size() - 1, "softmax: last axis only");
  const int64_t n = x.dims.back(), rows = x.numel() / n;
  Tensor* o = r.out("Out");
  Dims d = x.dims;
  float* y = o->alloc<float>(d, D(r));
  o->lod = x.lod;
  hipLaunchKernelGGL(softmax_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, S(r), f32(x), y, rows, n);
}

// =============================================================== reductions over [pre, R, post]
__global__ void reduce_kernel(const float* __restrict__ x, float* __restrict__ o, int64_t pre, int64_t R,
                              int64_t post, int kind) {
  const int64_t total = pre * post;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t a = i / post, c = i % post;
    const float* p = x + a * R * post + c;
    float acc = kind == 2 ? -INFINITY : kind == 3 ? INFINITY : 0.f;
    for (int64_t k = 0; k < R; ++k) {
      const float v = p[k * post];
      acc = kind == 2 ? fmaxf(acc, v) : kind == 3 ? fminf(acc, v) : acc + v;
    }
    o[i] = kind == 1 ? acc / (float)R : acc;
  }
}

template <int KIND> void k_reduce(const OpRun& r) {  // 0 sum 1 mean 2 max 3 min
  Tensor x = r.in("X");
  const int64_t R = (int64_t)x.dims.size();
  std::vector<bool> red((size_t)R, r.op.GetBool("reduce_all"));
  for (int64_t a : r.op.GetInts("dim")) red[(size_t)(a < 0 ? a + R : a)] = true;
  int64_t a = -1, e = -1;
  for (int64_t i = 0; i < R; ++i)
    if (red[(size_t)i]) {
      if (a < 0) a = i;
      e = i + 1;
    }
  for (int64_t i = a; i < e; ++i) PA_CHECK(red[(size_t)i], "reduce: non-contiguous reduced dims on device");
  Dims od, kd;
  for (int64_t i = 0; i < R; ++i) {
    if (!red[(size_t)i]) od.push_back(x.dims[(size_t)i]);
    kd.push_back(red[(size_t)i] ? 1 : x.dims[(size_t)i]);
  }
  Dims outd = r.op.GetBool("keep_dim") ? kd : (od.empty() ? Dims{1} : od);
  float* o = r.out("Out")->alloc<float>(outd, D(r));
  const int64_t pre = prod(x.dims, 0, (size_t)a), RR = prod(x.dims, (size_t)a, (size_t)e), post = prod(x.dims, (size_t)e);
  hipLaunchKernelGGL(reduce_kernel, dim3(grid_for(pre * post)), dim3(256), 0, S(r), f32(x), o, pre, RR, post, KIND);
}

void k_mean(const OpRun& r) {
  Tensor x = r.in("X");
  float* o = r.out("Out")->alloc<float>({1}, D(r));
  hipLaunchKernelGGL(reduce_kernel, dim3(1), dim3(64), 0, S(r), f32(x), o, (int64_t)1, x.numel(), (int64_t)1, 1);
}

// =============================================================== data movement
__global__ void gather_rows_kernel(const float* __restrict__ w, const int64_t* __restrict__ ids,
                                   float* __restrict__ o, int64_t n, int64_t D, int64_t V, int64_t pad) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n * D; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / D, id = ids[row];
    o[i] = (id == pad || id < 0 || id >= V) ? 0.f : w[id * D + (i % D)];
  }
}

void k_lookup_table(const OpRun& r) {
  Tensor w = r.in("W");
  Tensor ids = r.in("Ids");
  PA_CHECK(ids.dtype == DT::INT64, "lookup_table: int64 ids expected on device");
  const int64_t V = w.dims[0], Dm = w.dims[1], n = ids.numel();
  Dims od = ids.dims;
  if (od.size() > 1 && od.back() == 1) od.back() = Dm;
  else od.push_back(Dm);
  Tensor* o = r.out("Out");
  float* op = o->alloc<float>(od, D(r));
  o->lod = ids.lod;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(grid_for(n * Dm)), dim3(256), 0, S(r), f32(w), ids.data<int64_t>(), op,
                     n, Dm, V, (int64_t)r.op.GetInt("padding_idx", -1));
}

void k_concat(const OpRun& r) {
  auto xs = r.ins("X");
  std::vector<Tensor> keep;
  for (auto* t : xs) keep.push_back(*t);
  int64_t axis = r.op.GetInt("axis", 0);
  if (axis < 0) axis += (int64_t)keep[0].dims.size();
  Dims od = keep[0].dims;
  od[(size_t)axis] = 0;
  for (auto& t : keep) od[(size_t)axis] += t.dims[(size_t)axis];
  const int64_t pre = prod(od, 0, (size_t)axis), post = prod(od, (size_t)axis + 1);
  const size_t es = dt_size(keep[0].dtype);
  char* o = (char*)r.out("Out")->alloc(keep[0].dtype, od, D(r));
  int64_t off = 0;
  for (auto& t : keep) {
    const int64_t w = t.dims[(size_t)axis] * post;
    if (w && pre)
      HIPCHK(hipMemcpy2DAsync(o + off * es, (size_t)(od[(size_t)axis] * post) * es, t.raw(), (size_t)w * es,
                              (size_t)w * es, (size_t)pre, hipMemcpyDeviceToDevice, S(r)));
    off += w;
  }
}

void k_split(const OpRun& r) {
  Tensor x = r.in("X");
  int64_t axis = r.op.GetInt("axis", 0);
  if (axis < 0) axis += (int64_t)x.dims.size();
  auto& outs = r.op.Outputs("Out");
  std::vector<int64_t> sec = r.op.GetInts("sections");
  const int64_t num = r.op.GetInt("num", 0);
  if (sec.empty()) sec.assign(outs.size(), x.dims[(size_t)axis] / (num ? num : (int64_t)outs.size()));
  const int64_t pre = prod(x.dims, 0, (size_t)axis), post = prod(x.dims, (size_t)axis + 1);
  const size_t es = dt_size(x.dtype);
  int64_t off = 0;
  for (size_t i = 0; i < outs.size(); ++i) {
    Dims od = x.dims;
    od[(size_t)axis] = sec[i];
    char* o = (char*)r.out("Out", i)->alloc(x.dtype, od, D(r));
    const int64_t w = sec[i] * post;
    if (w && pre)
      HIPCHK(hipMemcpy2DAsync(o, (size_t)w * es, (const char*)x.raw() + off * es,
                              (size_t)(x.dims[(size_t)axis] * post) * es, (size_t)w * es, (size_t)pre,
                              hipMemcpyDeviceToDevice, S(r)));
    off += w;
  }
}

struct PermArgs {
  int R;
  int64_t od[kMaxR], src_stride[kMaxR];  // src stride of each OUTPUT dim
  int64_t n;
};

__global__ void permute_kernel(PermArgs p, const float* __restrict__ x, float* __restrict__ o) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < p.n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t rem = i, off = 0;
    for (int d = p.R - 1; d >= 0; --d) {
      off += (rem % p.od[d]) * p.src_stride[d];
      rem /= p.od[d];
    }
    o[i] = x[off];
  }
}

void k_transpose(const OpRun& r) {
  Tensor x = r.in("X");
  auto perm = r.op.GetInts("axis");
  const size_t R = x.dims.size();
  PA_CHECK(R <= (size_t)kMaxR && x.dtype == DT::FP32, "transpose: rank / dtype unsupported on device");
  PermArgs p;
  p.R = (int)R;
  Dims sx(R), od(R);
  int64_t s = 1;
  for (size_t i = R; i-- > 0;) {
    sx[i] = s;
    s *= x.dims[i];
  }
  for (size_t i = 0; i < R; ++i) {
    od[i] = x.dims[(size_t)perm[i]];
    p.od[i] = od[i];
    p.src_stride[i] = sx[(size_t)perm[i]];
  }
  p.n = x.numel();
  float* o = r.out("Out")->alloc<float>(od, D(r));
  if (Tensor* xs = r.out("XShape")) {
    Dims d{0};
    d.insert(d.end(), x.dims.begin(), x.dims.end());
    xs->dims = d;
  }
  if (p.n) hipLaunchKernelGGL(permute_kernel, dim3(grid_for(p.n)), dim3(256), 0, S(r), p, f32(x), o);
}

__global__ void fill_kernel(float* o, int64_t n, float v) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) o[i] = v;
}

__global__ void accumulate_kernel(float* o, const float* x, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) o[i] += x[i];
}

void k_fill_constant(const OpRun& r) {
  const DT dt = (DT)r.op.GetInt("dtype", (int)DT::FP32);
  PA_CHECK(dt == DT::FP32, "fill_constant: float32 only on device");
  Tensor* o = r.out("Out");
  float* p = o->alloc<float>(r.op.GetInts("shape"), D(r));
  hipLaunchKernelGGL(fill_kernel, dim3(grid_for(o->numel())), dim3(256), 0, S(r), p, o->numel(),
                     r.op.GetFloat("value"));
}

void k_sum(const OpRun& r) {
  auto xs = r.ins("X");
  std::vector<Tensor> keep;
  for (auto* t : xs) keep.push_back(*t);
  Dims d = keep[0].dims;
  Tensor* o = r.out("Out");
  float* op = o->alloc<float>(d, D(r));
  const int64_t n = prod(d);
  HIPCHK(hipMemcpyAsync(op, f32(keep[0]), n * 4, hipMemcpyDeviceToDevice, S(r)));
  for (size_t i = 1; i < keep.size(); ++i)
    hipLaunchKernelGGL(accumulate_kernel, dim3(grid_for(n)), dim3(256), 0, S(r), op, f32(keep[i]), n);
}

}  // namespace

PA_DEVICE_KERNEL(mul, k_mul);
PA_DEVICE_KERNEL(fc, k_fc);
PA_DEVICE_KERNEL(matmul, k_matmul);
PA_DEVICE_KERNEL(conv2d, k_conv2d);
PA_DEVICE_KERNEL(depthwise_conv2d, k_conv2d);
PA_DEVICE_KERNEL(pool2d, k_pool2d);
PA_DEVICE_KERNEL(batch_norm, k_batch_norm);
PA_DEVICE_KERNEL(softmax, k_softmax);
PA_DEVICE_KERNEL(elementwise_add, k_binary<B_ADD>);
PA_DEVICE_KERNEL(elementwise_sub, k_binary<B_SUB>);
PA_DEVICE_KERNEL(elementwise_mul, k_binary<B_MUL>);
PA_DEVICE_KERNEL(elementwise_div, k_binary<B_DIV>);
PA_DEVICE_KERNEL(elementwise_max, k_binary<B_MAX>);
PA_DEVICE_KERNEL(elementwise_min, k_binary<B_MIN>);
PA_DEVICE_KERNEL(elementwise_pow, k_binary<B_POW>);
PA_DEVICE_KERNEL(relu, k_unary<U_RELU>);
PA_DEVICE_KERNEL(sigmoid, k_unary<U_SIGMOID>);
PA_DEVICE_KERNEL(tanh, k_unary<U_TANH>);
PA_DEVICE_KERNEL(exp, k_unary<U_EXP>);
PA_DEVICE_KERNEL(log, k_unary<U_LOG>);
PA_DEVICE_KERNEL(sqrt, k_unary<U_SQRT>);
PA_DEVICE_KERNEL(abs, k_unary<U_ABS>);
PA_DEVICE_KERNEL(square, k_unary<U_SQUARE>);
PA_DEVICE_KERNEL(leaky_relu, k_unary<U_LEAKY>);
PA_DEVICE_KERNEL(gelu, k_unary<U_GELU>);
PA_DEVICE_KERNEL(relu6, k_unary<U_RELU6>);
PA_DEVICE_KERNEL(softplus, k_unary<U_SOFTPLUS>);
PA_DEVICE_KERNEL(swish, k_unary<U_SWISH>);
PA_DEVICE_KERNEL(hard_sigmoid, k_unary<U_HSIG>);
PA_DEVICE_KERNEL(elu, k_unary<U_ELU>);
PA_DEVICE_KERNEL(reciprocal, k_unary<U_RECIP>);
PA_DEVICE_KERNEL(scale, k_scale);
PA_DEVICE_KERNEL(dropout, k_dropout);
PA_DEVICE_KERNEL(reduce_sum, k_reduce<0>);
PA_DEVICE_KERNEL(reduce_mean, k_reduce<1>);
PA_DEVICE_KERNEL(reduce_max, k_reduce<2>);
PA_DEVICE_KERNEL(reduce_min, k_reduce<3>);
PA_DEVICE_KERNEL(mean, k_mean);
PA_DEVICE_KERNEL(lookup_table, k_lookup_table);
PA_DEVICE_KERNEL(concat, k_concat);
PA_DEVICE_KERNEL(split, k_split);
PA_DEVICE_KERNEL(transpose, k_transpose);
PA_DEVICE_KERNEL(transpose2, k_transpose);
PA_DEVICE_KERNEL(fill_constant, k_fill_constant);
PA_DEVICE_KERNEL(sum, k_sum);

void link_device_kernels() {}

// GEMM entry for tests / benchmarks (C ABI below)
void device_sgemm(void* stream, bool ta, bool tb, int64_t M, int64_t N, int64_t K, float alpha, const float* A,
                  int64_t lda, const float* B, int64_t ldb, float beta, float* C, int64_t ldc) {
  gemm((hipStream_t)stream, ta, tb, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc);
}

}  // namespace pa

extern "C" __attribute__((visibility("default"))) int pa_nat_device_sgemm(void* stream, int ta, int tb, int64_t M,
                                                                         int64_t N, int64_t K, float alpha,
                                                                         const float* A, int64_t lda, const float* B,
                                                                         int64_t ldb, float beta, float* C,
                                                                         int64_t ldc) {
  try {
    pa::device_sgemm(stream, ta != 0, tb != 0, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc);
    return 0;
  } catch (...) {
    return -1;
  }
}
