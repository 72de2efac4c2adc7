// gfx950 device kernels of the native executor (fp32 inference AND training ops on
// HBM-resident tensors).
//
// The heavy lifting runs on the shared kernel library (kernel_lib.h,
// libpaddle_amd_kernels.so): GEMM (mul / fc / matmul and their grads) and the
// conv2d products on pa_sgemm (exact-fp32 MFMA, strided / batched / split-K),
// im2col / col2im on pa_vol2col / pa_col2vol, pooling on pa_pool_*, batch norm on
// pa_bn_nchw_*, activations on pa_act_*, softmax / cross-entropy on the
// softmax_ce / nnmisc kernels and the optimizer updates on pa_adamw / pa_momentum /
// pa_sgd -- the same launchers, with the same call shapes, the Python Fluid
// operators use (ops/convnd.py, ops/blas.py, operators/*), so the two engines train
// along the same trajectory.  Only thin glue lives here: broadcast elementwise,
// reductions, gathers / concat / split / transpose and fills.
//
// A device kernel may decline an op configuration it does not cover (throw
// pa::Decline before touching any output); the executor then runs the host
// kernel on host copies and counts the fallback (Executor::host_fallbacks).
//
// Reference: framework/executor.cc:125-353 (op loop), operators/{mul,conv,pool,
// batch_norm,softmax,cross_entropy,activation,elementwise,sgd,momentum,adam}_op.*
#include <hip/hip_runtime.h>
#include <math.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <string>

#include "framework.h"
#include "kernel_lib.h"

namespace pa {
namespace {

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

float* f32(const Tensor& t) {
  PA_CHECK(t.dtype == DT::FP32, "expected float32 tensor, got %s", dt_name(t.dtype));
  PA_CHECK(t.device >= 0, "expected a device tensor");
  return t.data<float>();
}

// Output `slot` with dims `d`.  When the output variable IS the input tensor `in`
// (in-place op: ParamOut == Param, Out == X) its buffer is kept as is.
float* out_f32(const OpRun& r, const std::string& slot, const Dims& d, const Tensor* in = nullptr, size_t i = 0) {
  Tensor* o = r.out(slot, i);
  if (!o) return nullptr;
  if (in && o == in) {
    PA_CHECK(o->dims == d || o->numel() == prod(d), "%s: in-place output shape mismatch", slot.c_str());
    return f32(*o);
  }
  return o->alloc<float>(d, D(r));
}

// scope-held device workspace (kept across ops / runs: steady-state steps reuse it)
float* workspace(const OpRun& r, const char* name, int64_t n) {
  // held by the root scope: ops inside per-step scopes (while / while_grad) reuse one
  // buffer instead of allocating (and hipFree-syncing) one per step
  Variable* v = r.scope.Root().Var(name);
  if (v->tensor.initialized() && v->tensor.device == D(r) && v->tensor.numel() >= n) return f32(v->tensor);
  return v->tensor.alloc<float>({std::max<int64_t>(n, 1)}, D(r));
}

void copy_d2d(const OpRun& r, void* dst, const void* src, size_t bytes) {
  if (bytes && dst != src) HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, S(r)));
}

// =============================================================== GEMM (pa_sgemm)
// C[M,N] (+batch) = alpha op(A) op(B) + beta C, row-major, transposes as strides.
void gemm(hipStream_t s, bool ta, bool tb, int64_t M, int64_t N, int64_t K, float alpha, const float* A,
          int64_t lda, const float* B, int64_t ldb, float beta, float* C, int64_t ldc, int64_t batch = 1,
          int64_t bsA = 0, int64_t bsB = 0, int64_t bsC = 0) {
  if (M <= 0 || N <= 0) return;
  PA_CHECK(batch >= 1 && batch <= 65535, "gemm: batch %lld out of range", (long long)batch);
  PA_KL(pa_sgemm(A, ta ? 1 : lda, ta ? lda : 1, B, tb ? 1 : ldb, tb ? ldb : 1, C, ldc, M, N, K, 1, (int)batch, 0, 0,
                 0, bsA, bsB, bsC, 1, 0, 0, nullptr, 0, alpha, beta, 0, nullptr, s));
}

__global__ void bias_rows_kernel(float* __restrict__ c, const float* __restrict__ b, int64_t M, int64_t N) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < M * N; i += (int64_t)gridDim.x * blockDim.x)
    c[i] = b[i % N];
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
  Dims yt = y;  // trailing singular dims of Y are trimmed (elementwise_op_function.h)
  while (yt.size() > 1 && yt.back() == 1 && x != y) yt.pop_back();
  if ((int64_t)yt.size() > xr || xr > kMaxR) return false;
  if (axis < 0) axis = xr - (int64_t)yt.size();
  Dims yf((size_t)xr, 1);
  for (size_t i = 0; i < yt.size(); ++i) yf[(size_t)axis + i] = yt[i];
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
  if ((x.dtype == DT::INT64 || x.dtype == DT::INT32) && OP != B_POW) return elementwise_int_any(r, (int)OP);
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

__global__ void scale_kernel(const float* __restrict__ x, float* __restrict__ o, int64_t n, float s, float b) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    o[i] = x[i] * s + b;
}

void launch_scale(const OpRun& r, const Tensor& x, float* o, float s, float b) {
  if (x.numel())
    hipLaunchKernelGGL(scale_kernel, dim3(grid_for(x.numel())), dim3(256), 0, S(r), f32(x), o, x.numel(), s, b);
}

// elementwise_{add,sub}_grad: dX = dOut, dY = (+/-) dOut summed over Y's broadcast
// dims ([pre, n, post] -> [n] on pa_chan_sum); other layouts decline to the host
template <int SIGN> void k_ew_grad(const OpRun& r) {
  Tensor& x = r.in("X");
  Tensor& y = r.in("Y");
  Tensor& g = r.in("Out@GRAD");
  BcArgs b;
  int64_t pre, n, post;
  if (!make_bc(x.dims, y.dims, r.op.GetInt("axis", -1), &b, &pre, &n, &post)) throw Decline();
  const Dims xd = x.dims, yd = y.dims;
  const LoD lod = x.lod;
  if (Tensor* dx = r.out("X@GRAD")) {
    float* p = dx->alloc<float>(xd, D(r));
    dx->lod = lod;
    copy_d2d(r, p, f32(g), g.nbytes());
  }
  if (Tensor* dy = r.out("Y@GRAD")) {
    float* p = dy->alloc<float>(yd, D(r));
    if (pre * post == 1)
      copy_d2d(r, p, f32(g), g.nbytes());
    else
      PA_KL(pa_chan_sum(f32(g), p, (int)pre, (int)n, post, 0, S(r)));
    if (SIGN < 0) launch_scale(r, *dy, p, -1.f, 0.f);
  }
}

// =============================================================== activations (pa_act_*)
struct ActSpec {
  int id;
  const char* a_attr;
  float a_def;
  const char* b_attr;
  float b_def;
};

template <int ID> ActSpec act_spec() {
  switch (ID) {
    case act::SOFTSHRINK: return {ID, "lambda", 0.5f, nullptr, 0.f};
    case act::BRELU: return {ID, "t_min", 0.f, "t_max", 24.f};
    case act::LEAKY_RELU: return {ID, "alpha", 0.02f, nullptr, 0.f};
    case act::SOFT_RELU: return {ID, "threshold", 40.f, nullptr, 0.f};
    case act::ELU: return {ID, "alpha", 1.f, nullptr, 0.f};
    case act::RELU6: return {ID, "threshold", 6.f, nullptr, 0.f};
    case act::POW: return {ID, "factor", 1.f, nullptr, 0.f};
    case act::STANH: return {ID, "scale_a", 2.f / 3.f, "scale_b", 1.7159f};
    case act::HARD_SHRINK: return {ID, "threshold", 0.5f, nullptr, 0.f};
    case act::THRESHOLDED_RELU: return {ID, "threshold", 1.f, nullptr, 0.f};
    case act::HARD_SIGMOID: return {ID, "slope", 0.2f, "offset", 0.5f};
    case act::SWISH: return {ID, "beta", 1.f, nullptr, 0.f};
    default: return {ID, nullptr, 0.f, nullptr, 0.f};
  }
}

template <int ID> void k_act(const OpRun& r) {
  const ActSpec sp = act_spec<ID>();
  const float a = sp.a_attr ? r.op.GetFloat(sp.a_attr, sp.a_def) : 0.f;
  const float b = sp.b_attr ? r.op.GetFloat(sp.b_attr, sp.b_def) : 0.f;
  Tensor& x = r.in("X");
  const LoD lod = x.lod;
  float* o = out_f32(r, "Out", x.dims, &x);
  r.out("Out")->lod = lod;
  PA_KL(pa_act_fwd(ID, 0, f32(x), o, x.numel(), a, b, S(r)));
}

// <act>_grad: X, Out, Out@GRAD -> X@GRAD (whichever of X / Out the derivative reads)
template <int ID> void k_act_grad(const OpRun& r) {
  const ActSpec sp = act_spec<ID>();
  const float a = sp.a_attr ? r.op.GetFloat(sp.a_attr, sp.a_def) : 0.f;
  const float b = sp.b_attr ? r.op.GetFloat(sp.b_attr, sp.b_def) : 0.f;
  Tensor& g = r.in("Out@GRAD");
  Tensor* x = r.in_opt("X");
  Tensor* y = r.in_opt("Out");
  const Dims d = g.dims;
  const LoD lod = x ? x->lod : g.lod;
  Tensor* dx = r.out("X@GRAD");
  if (!dx) return;
  float* p = dx->alloc<float>(d, D(r));
  dx->lod = lod;
  PA_KL(pa_act_bwd(ID, 0, x ? f32(*x) : nullptr, y ? f32(*y) : nullptr, f32(g), p, g.numel(), a, b, S(r)));
}

void k_scale(const OpRun& r) {
  const float s = r.op.GetFloat("scale", 1.f), b = r.op.GetFloat("bias", 0.f);
  const bool after = r.op.GetBool("bias_after_scale", true);
  Tensor& x = r.in("X");
  const LoD lod = x.lod;
  float* o = out_f32(r, "Out", x.dims, &x);
  r.out("Out")->lod = lod;
  launch_scale(r, x, o, s, after ? b : b * s);
}

// scale's gradient (the auto-VJP grad op of the Python library): dX = scale * dOut
void k_scale_grad(const OpRun& r) {
  Tensor g = r.in("Out@GRAD");
  Tensor* dx = r.out("X@GRAD");
  if (!dx) return;
  const LoD lod = g.lod;
  float* o = out_f32(r, "X@GRAD", g.dims, &g);
  dx->lod = lod;
  launch_scale(r, g, o, r.op.GetFloat("scale", 1.f), 0.f);
}

void k_dropout(const OpRun& r) {
  if (!(r.ctx.is_test || r.op.GetBool("is_test"))) throw Decline();  // training masks: host RNG
  const float p = r.op.GetFloat("dropout_prob", 0.5f);
  const bool upscale = r.op.GetString("dropout_implementation", "downgrade_in_infer") == "upscale_in_train";
  Tensor& x = r.in("X");
  const LoD lod = x.lod;
  float* o = out_f32(r, "Out", x.dims, &x);
  r.out("Out")->lod = lod;
  launch_scale(r, x, o, upscale ? 1.f : 1.f - p, 0.f);
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

// mul_grad (mul_op.h MulGradKernel): dX = dOut Y^T, dY = X^T dOut
void k_mul_grad(const OpRun& r) {
  Tensor x = r.in("X");
  Tensor y = r.in("Y");
  Tensor g = r.in("Out@GRAD");
  const size_t xnc = (size_t)r.op.GetInt("x_num_col_dims", 1), ync = (size_t)r.op.GetInt("y_num_col_dims", 1);
  const int64_t M = prod(x.dims, 0, xnc), K = prod(x.dims, xnc), N = prod(y.dims, ync);
  PA_CHECK(g.numel() == M * N, "mul_grad: Out@GRAD %s does not match", g.shape_str().c_str());
  if (Tensor* dx = r.out("X@GRAD")) {
    float* p = dx->alloc<float>(x.dims, D(r));
    dx->lod = x.lod;
    gemm(S(r), false, true, M, K, N, 1.f, f32(g), N, f32(y), N, 0.f, p, K);
  }
  if (Tensor* dy = r.out("Y@GRAD")) {
    float* p = dy->alloc<float>(y.dims, D(r));
    gemm(S(r), true, false, K, N, M, 1.f, f32(x), K, f32(g), N, 0.f, p, N);
  }
}

// fc (fc_op.cc): the bias pre-broadcast into C, the GEMM accumulates (beta = 1), relu in place
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
  if (b && M * N)
    hipLaunchKernelGGL(bias_rows_kernel, dim3(grid_for(M * N)), dim3(256), 0, S(r), c, f32(*b), M, N);
  gemm(S(r), false, false, M, N, K, 1.f, f32(x), K, f32(w), N, b ? 1.f : 0.f, c, N);
  const std::string act = r.op.GetString("activation_type");
  int code = -1;
  if (act == "relu") code = act::RELU;
  else if (act == "tanh") code = act::TANH;
  else if (act == "sigmoid") code = act::SIGMOID;
  else if (act == "gelu") code = act::GELU;
  else if (!act.empty()) fail("fc: activation %s not supported on the device", act.c_str());
  if (code >= 0) PA_KL(pa_act_fwd(code, 0, c, c, M * N, 0.f, 0.f, S(r)));
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
  gemm(S(r), tx, ty, M, N, K, alpha, f32(x), tx ? M : K, f32(y), ty ? K : N, 0.f, c, N, std::max(bx, by),
       bx == 1 ? 0 : M * K, by == 1 ? 0 : K * N, M * N);
}

// =============================================================== conv2d (ops/convnd.py call shapes)
constexpr int64_t kColBudget = int64_t(1) << 28;  // floats per column chunk (1 GiB)

struct Conv {
  int64_t N, C, H, W, OC, kh, kw, OH, OW, G, Cg, OCg, CgK, S;
  bool pointwise;
  int geo[19];  // vol2col geometry: C, D, H, W, OD, OH, OW, kd, kh, kw, sd, sh, sw, pd, ph, pw, dd, dh, dw
  int64_t chunk() const {
    int64_t nb = std::max<int64_t>(1, std::min<int64_t>(N, kColBudget / std::max<int64_t>(C * kh * kw * S, 1)));
    return std::max<int64_t>(1, std::min<int64_t>(nb, 65535 / std::max<int64_t>(G, 1)));
  }
};

Conv conv_of(const OpRun& r, const Dims& xd, const Dims& wd) {
  auto st = r.op.GetInts("strides"), pd = r.op.GetInts("paddings"), dl = r.op.GetInts("dilations");
  if (st.empty()) st = {1, 1};
  if (pd.empty()) pd = {0, 0};
  if (dl.empty()) dl = {1, 1};
  PA_CHECK(xd.size() == 4 && wd.size() == 4 && st.size() >= 2 && pd.size() >= 2 && dl.size() >= 2,
           "conv2d: NCHW input and 2-D attributes expected");
  Conv c;
  c.G = std::max<int64_t>(1, r.op.GetInt("groups", 1));
  c.N = xd[0]; c.C = xd[1]; c.H = xd[2]; c.W = xd[3];
  c.OC = wd[0]; c.kh = wd[2]; c.kw = wd[3];
  PA_CHECK(wd[1] * c.G == c.C && c.OC % c.G == 0, "conv2d: filter / input channel mismatch");
  c.OH = (c.H + 2 * pd[0] - (dl[0] * (c.kh - 1) + 1)) / st[0] + 1;
  c.OW = (c.W + 2 * pd[1] - (dl[1] * (c.kw - 1) + 1)) / st[1] + 1;
  PA_CHECK(c.OH > 0 && c.OW > 0, "conv2d: empty output");
  c.Cg = c.C / c.G; c.OCg = c.OC / c.G; c.CgK = c.Cg * c.kh * c.kw; c.S = c.OH * c.OW;
  c.pointwise = c.kh == 1 && c.kw == 1 && st[0] == 1 && st[1] == 1 && pd[0] == 0 && pd[1] == 0;
  const int64_t g[19] = {c.C, 1, c.H, c.W, 1, c.OH, c.OW, 1, c.kh, c.kw, 1, st[0], st[1], 0, pd[0], pd[1],
                         1, dl[0], dl[1]};
  for (int i = 0; i < 19; ++i) c.geo[i] = (int)g[i];
  return c;
}

void sg(const OpRun& r, const float* A, long sam, long sak, const float* B, long sbk, long sbn, float* C, long ldc,
        long M, long N, long K, int Z1, int Z2, long a1, long b1, long c1, long a2, long b2, long c2, int kb = 1,
        long kbA = 0, long kbB = 0, const float* bias = nullptr, long bsb = 0, int atomic = 0) {
  PA_CHECK((int64_t)Z1 * Z2 <= 65535, "conv: batch x groups too large");
  PA_KL(pa_sgemm(A, sam, sak, B, sbk, sbn, C, ldc, M, N, K, Z1, Z2, a1, b1, c1, a2, b2, c2, kb, kbA, kbB, bias, bsb,
                 1.f, 0.f, atomic, nullptr, S(r)));
}

void k_conv2d(const OpRun& r) {
  Tensor x = r.in("Input");
  Tensor w = r.in("Filter");
  Tensor* b = r.in_opt("Bias");
  const Conv c = conv_of(r, x.dims, w.dims);
  float* y = r.out("Output")->alloc<float>({c.N, c.OC, c.OH, c.OW}, D(r));
  const float* xp = f32(x);
  const float* wp = f32(w);
  const float* bp = b ? f32(*b) : nullptr;
  if (c.pointwise) {
    sg(r, wp, c.CgK, 1, xp, c.S, 1, y, c.S, c.OCg, c.S, c.CgK, (int)c.N, (int)c.G, 0, c.C * c.S, c.OC * c.S,
       c.OCg * c.CgK, c.CgK * c.S, c.OCg * c.S, 1, 0, 0, bp, c.OCg);
    return;
  }
  const int64_t nb = c.chunk(), rows = c.C * c.kh * c.kw;
  float* col = workspace(r, "@conv_col@", nb * rows * c.S);
  for (int64_t n0 = 0; n0 < c.N; n0 += nb) {
    const int m = (int)std::min(nb, c.N - n0);
    PA_KL(pa_vol2col(0, xp + n0 * c.C * c.H * c.W, col, c.geo, m, S(r)));
    sg(r, wp, c.CgK, 1, col, c.S, 1, y + n0 * c.OC * c.S, c.S, c.OCg, c.S, c.CgK, m, (int)c.G, 0, rows * c.S,
       c.OC * c.S, c.OCg * c.CgK, c.CgK * c.S, c.OCg * c.S, 1, 0, 0, bp, c.OCg);
  }
}

// conv2d_grad (conv_op.h GemmConvGradKernel): dX = col2im(W^T dY), dW = sum_img dY col(X)^T
// (images on the GEMM's k-batch, float-atomic split), dBias = per-channel sums of dY
void k_conv2d_grad(const OpRun& r) {
  Tensor x = r.in("Input");
  Tensor w = r.in("Filter");
  Tensor dy = r.in("Output@GRAD");
  const Conv c = conv_of(r, x.dims, w.dims);
  PA_CHECK(dy.numel() == c.N * c.OC * c.S, "conv2d_grad: Output@GRAD %s does not match", dy.shape_str().c_str());
  const float* xp = f32(x);
  const float* wp = f32(w);
  const float* gp = f32(dy);
  const int64_t nb = c.chunk(), rows = c.C * c.kh * c.kw;
  Tensor* dxt = r.out("Input@GRAD");
  Tensor* dwt = r.out("Filter@GRAD");
  Tensor* dbt = r.out("Bias@GRAD");
  float* col = (dxt || dwt) && !c.pointwise ? workspace(r, "@conv_col@", nb * rows * c.S) : nullptr;
  if (dxt) {
    float* dx = dxt->alloc<float>(x.dims, D(r));
    if (c.pointwise) {
      sg(r, wp, 1, c.CgK, gp, c.S, 1, dx, c.S, c.CgK, c.S, c.OCg, (int)c.N, (int)c.G, 0, c.OC * c.S, c.C * c.S,
         c.OCg * c.CgK, c.OCg * c.S, c.CgK * c.S);
    } else {
      for (int64_t n0 = 0; n0 < c.N; n0 += nb) {
        const int m = (int)std::min(nb, c.N - n0);
        sg(r, wp, 1, c.CgK, gp + n0 * c.OC * c.S, c.S, 1, col, c.S, c.CgK, c.S, c.OCg, m, (int)c.G, 0, c.OC * c.S,
           rows * c.S, c.OCg * c.CgK, c.OCg * c.S, c.CgK * c.S);
        PA_KL(pa_col2vol(col, dx + n0 * c.C * c.H * c.W, c.geo, m, 0, S(r)));
      }
    }
  }
  if (dwt) {
    float* dw = dwt->alloc<float>(w.dims, D(r));
    HIPCHK(hipMemsetAsync(dw, 0, sizeof(float) * w.numel(), S(r)));
    for (int64_t n0 = 0; n0 < c.N; n0 += nb) {
      const int m = (int)std::min(nb, c.N - n0);
      const float* cp = xp + n0 * c.C * c.H * c.W;
      if (!c.pointwise) {
        PA_KL(pa_vol2col(0, cp, col, c.geo, m, S(r)));
        cp = col;
      }
      sg(r, gp + n0 * c.OC * c.S, c.S, 1, cp, 1, c.S, dw, c.CgK, c.OCg, c.CgK, c.S, 1, (int)c.G, 0, 0, 0,
         c.OCg * c.S, c.CgK * c.S, c.OCg * c.CgK, m, c.OC * c.S, rows * c.S, nullptr, 0, 1);
    }
  }
  if (dbt) PA_KL(pa_chan_sum(gp, dbt->alloc<float>({c.OC}, D(r)), (int)c.N, (int)c.OC, c.S, 0, S(r)));
}

// =============================================================== pooling (pa_pool_*)
struct Pool {
  int64_t N, C, H, W, OH, OW;
  int type, exclusive;
  int geo[15];  // D, H, W, OD, OH, OW, kd, kh, kw, sd, sh, sw, pd, ph, pw
};

Pool pool_of(const OpRun& r, const Dims& xd) {
  PA_CHECK(xd.size() == 4, "pool2d: NCHW input expected");
  auto ks = r.op.GetInts("ksize"), st = r.op.GetInts("strides"), pd = r.op.GetInts("paddings");
  if (st.empty()) st = {1, 1};
  if (pd.empty()) pd = {0, 0};
  Pool p;
  p.N = xd[0]; p.C = xd[1]; p.H = xd[2]; p.W = xd[3];
  if (r.op.GetBool("global_pooling")) {
    ks = {p.H, p.W};
    pd = {0, 0};
  }
  PA_CHECK(ks.size() >= 2 && st.size() >= 2 && pd.size() >= 2, "pool2d: 2-D attributes expected");
  const bool ceil = r.op.GetBool("ceil_mode");
  auto osz = [&](int64_t in, int64_t k, int64_t pp, int64_t s) {
    return ceil ? (in - k + 2 * pp + s - 1) / s + 1 : (in - k + 2 * pp) / s + 1;
  };
  p.OH = osz(p.H, ks[0], pd[0], st[0]);
  p.OW = osz(p.W, ks[1], pd[1], st[1]);
  p.type = r.op.GetString("pooling_type", "max") == "max" ? 0 : 1;
  p.exclusive = r.op.GetBool("exclusive", true) ? 1 : 0;
  const int64_t g[15] = {1, p.H, p.W, 1, p.OH, p.OW, 1, ks[0], ks[1], 1, st[0], st[1], 0, pd[0], pd[1]};
  for (int i = 0; i < 15; ++i) p.geo[i] = (int)g[i];
  return p;
}

// max pooling keeps its in-plane argmax next to Out (var "<Out>@MASK") for the grad op
int* pool_mask(const OpRun& r, const std::string& out_name, const Pool& p) {
  Variable* v = r.scope.Var(out_name + "@MASK");
  return static_cast<int*>(v->tensor.alloc(DT::INT32, {p.N, p.C, p.OH, p.OW}, D(r)));
}

void k_pool2d(const OpRun& r) {
  Tensor x = r.in("X");
  const Pool p = pool_of(r, x.dims);
  float* o = r.out("Out")->alloc<float>({p.N, p.C, p.OH, p.OW}, D(r));
  int* mask = p.type == 0 ? pool_mask(r, r.op.Output("Out"), p) : nullptr;
  PA_KL(pa_pool_fwd(0, f32(x), o, mask, p.N * p.C, p.geo, p.type, p.exclusive, S(r)));
}

void k_pool2d_grad(const OpRun& r) {
  Tensor x = r.in("X");
  Tensor dy = r.in("Out@GRAD");
  const Pool p = pool_of(r, x.dims);
  Tensor* dx = r.out("X@GRAD");
  if (!dx) return;
  const int* mask = nullptr;
  if (p.type == 0) {
    Variable* mv = r.scope.Find(r.op.Input("Out") + "@MASK");
    if (mv && mv->tensor.initialized() && mv->tensor.device == D(r) && mv->tensor.numel() == dy.numel()) {
      mask = mv->tensor.data<int>();
    } else {  // forward ran elsewhere (host fallback / another executor): rebuild the argmax
      int* m = pool_mask(r, r.op.Input("Out"), p);
      float* tmp = workspace(r, "@pool_tmp@", dy.numel());
      PA_KL(pa_pool_fwd(0, f32(x), tmp, m, p.N * p.C, p.geo, 0, p.exclusive, S(r)));
      mask = m;
    }
  }
  float* dxp = dx->alloc<float>(x.dims, D(r));
  PA_KL(pa_pool_bwd(0, f32(dy), mask, dxp, p.N * p.C, p.geo, p.type, p.exclusive, S(r)));
}

// =============================================================== batch norm (pa_bn_nchw_*)
__global__ void bn_infer_nhwc_kernel(const float* __restrict__ x, float* __restrict__ y, const float* __restrict__ sc,
                                     const float* __restrict__ bi, const float* __restrict__ mean,
                                     const float* __restrict__ var, float eps, int64_t total, int64_t C) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = i % C;
    y[i] = (x[i] - mean[c]) * (sc[c] * rsqrtf(var[c] + eps)) + bi[c];
  }
}

// the output buffer of `out_slot`: the input's buffer when the op updates in place
float* io_slot(const OpRun& r, const char* in_slot, const char* out_slot, int64_t n) {
  Tensor& in = r.in(in_slot);
  if (r.op.Output(out_slot) == r.op.Input(in_slot) || r.op.Output(out_slot).empty()) return f32(in);
  return r.out(out_slot)->alloc<float>({n}, D(r));
}

void k_batch_norm(const OpRun& r) {
  Tensor& x = r.in("X");
  const bool test = r.ctx.is_test || r.op.GetBool("is_test") || r.op.GetBool("use_global_stats");
  const float eps = r.op.GetFloat("epsilon", 1e-5f), mom = r.op.GetFloat("momentum", 0.9f);
  const int relu = r.op.GetBool("fuse_with_relu") ? 1 : 0;
  const Dims xd = x.dims;
  if (r.op.GetString("data_layout", "NCHW") == "NHWC") {
    if (!test || relu) throw Decline();
    const int64_t C = xd.back();
    float* y = r.out("Y")->alloc<float>(xd, D(r));
    hipLaunchKernelGGL(bn_infer_nhwc_kernel, dim3(grid_for(x.numel())), dim3(256), 0, S(r), f32(x), y,
                       f32(r.in("Scale")), f32(r.in("Bias")), f32(r.in("Mean")), f32(r.in("Variance")), eps,
                       x.numel(), C);
    return;
  }
  PA_CHECK(xd.size() >= 2, "batch_norm: rank");
  const int64_t N = xd[0], C = xd[1], Sp = x.numel() / std::max<int64_t>(N * C, 1);
  const float* xp = f32(x);
  float* mean_out = test ? nullptr : io_slot(r, "Mean", "MeanOut", C);
  float* var_out = test ? nullptr : io_slot(r, "Variance", "VarianceOut", C);
  Tensor* sm = r.out("SavedMean");
  Tensor* sv = r.out("SavedVariance");
  float* mean = sm ? sm->alloc<float>({C}, D(r)) : workspace(r, "@bn_mean@", C);
  float* rstd = sv ? sv->alloc<float>({C}, D(r)) : workspace(r, "@bn_rstd@", C);
  float* part = workspace(r, "@bn_part@", C * (int64_t)pa_bn_nchw_groups((int)C, N * Sp) * 2);
  float* y = r.out("Y")->alloc<float>(xd, D(r));
  PA_KL(pa_bn_nchw_fwd(0, xp, y, f32(r.in("Scale")), f32(r.in("Bias")), f32(r.in("Mean")), f32(r.in("Variance")),
                       mean_out, var_out, mean, rstd, part, (int)N, (int)C, Sp, eps, mom, test ? 0 : 1, relu, 0,
                       S(r)));
}

// batch_norm_grad (batch_norm_op.cc BatchNormGradKernel) from SavedMean / SavedVariance (= 1/std)
void k_batch_norm_grad(const OpRun& r) {
  if (r.op.GetString("data_layout", "NCHW") == "NHWC") throw Decline();
  Tensor& x = r.in("X");
  Tensor& dy = r.in("Y@GRAD");
  const int relu = r.op.GetBool("fuse_with_relu") ? 1 : 0;
  Tensor* y = r.in_opt("Y");
  if (relu && !y) throw Decline();
  const Dims xd = x.dims;
  const int64_t N = xd[0], C = xd[1], Sp = x.numel() / std::max<int64_t>(N * C, 1);
  Tensor* ds = r.out("Scale@GRAD");
  Tensor* db = r.out("Bias@GRAD");
  float* dscale = ds ? ds->alloc<float>(r.in("Scale").dims, D(r)) : workspace(r, "@bn_dscale@", C);
  float* dbias = db ? db->alloc<float>(r.in("Bias").dims, D(r)) : workspace(r, "@bn_dbias@", C);
  Tensor* dxt = r.out("X@GRAD");
  float* dx = dxt ? dxt->alloc<float>(xd, D(r)) : nullptr;
  float* part = workspace(r, "@bn_part@", C * (int64_t)pa_bn_nchw_groups((int)C, N * Sp) * 2);
  PA_KL(pa_bn_nchw_bwd(0, f32(x), f32(dy), y ? f32(*y) : nullptr, f32(r.in("SavedMean")),
                       f32(r.in("SavedVariance")), f32(r.in("Scale")), dscale, dbias, dx, part, (int)N, (int)C, Sp,
                       relu, S(r)));
}

// =============================================================== softmax / cross entropy
int64_t last_axis_rows(const OpRun& r, const Tensor& x, int64_t* n) {
  int64_t axis = r.op.GetInt("axis", -1);
  if (axis < 0) axis += (int64_t)x.dims.size();
  if (axis != (int64_t)x.dims.size() - 1) throw Decline();
  *n = x.dims.back();
  return *n ? x.numel() / *n : 0;
}

void k_softmax(const OpRun& r) {
  Tensor& x = r.in("X");
  int64_t n;
  const int64_t rows = last_axis_rows(r, x, &n);
  const LoD lod = x.lod;
  float* y = out_f32(r, "Out", x.dims, &x);
  r.out("Out")->lod = lod;
  PA_KL(pa_softmax_fwd(0, f32(x), y, rows, (int)n, 0, S(r)));
}

void k_softmax_grad(const OpRun& r) {
  Tensor& y = r.in("Out");
  Tensor& g = r.in("Out@GRAD");
  int64_t n;
  const int64_t rows = last_axis_rows(r, y, &n);
  Tensor* dx = r.out("X@GRAD");
  if (!dx) return;
  PA_KL(pa_softmax_bwd(0, f32(y), f32(g), dx->alloc<float>(y.dims, D(r)), rows, (int)n, 0, S(r)));
}

const long* hard_labels(const Tensor& l, int64_t rows) {
  if (l.dtype != DT::INT64 || l.numel() != rows) throw Decline();
  return l.data<long>();
}

void k_cross_entropy(const OpRun& r) {
  Tensor& x = r.in("X");
  Tensor& l = r.in("Label");
  const int64_t n = x.dims.back(), rows = n ? x.numel() / n : 0;
  const bool soft = r.op.GetBool("soft_label");
  const long* lab = soft ? nullptr : hard_labels(l, rows);
  if (soft && (l.dtype != DT::FP32 || l.numel() != x.numel())) throw Decline();
  Dims od(x.dims.begin(), x.dims.end() - 1);
  od.push_back(1);
  const LoD lod = x.lod;
  float* y = r.out("Y")->alloc<float>(od, D(r));
  r.out("Y")->lod = lod;
  PA_KL(pa_cross_entropy(0, 0, f32(x), lab, soft ? f32(l) : nullptr, nullptr, y, rows, (int)n,
                         r.op.GetInt("ignore_index", -100), S(r)));
}

void k_cross_entropy_grad(const OpRun& r) {
  Tensor& x = r.in("X");
  Tensor& l = r.in("Label");
  Tensor& g = r.in("Y@GRAD");
  const int64_t n = x.dims.back(), rows = n ? x.numel() / n : 0;
  const bool soft = r.op.GetBool("soft_label");
  const long* lab = soft ? nullptr : hard_labels(l, rows);
  if (soft && (l.dtype != DT::FP32 || l.numel() != x.numel())) throw Decline();
  Tensor* dx = r.out("X@GRAD");
  if (!dx) return;
  PA_KL(pa_cross_entropy(0, 1, f32(x), lab, soft ? f32(l) : nullptr, f32(g), dx->alloc<float>(x.dims, D(r)), rows,
                         (int)n, r.op.GetInt("ignore_index", -100), S(r)));
}

void k_softmax_ce(const OpRun& r) {
  Tensor& x = r.in("Logits");
  Tensor& l = r.in("Label");
  int64_t n;
  const int64_t rows = last_axis_rows(r, x, &n);
  const bool soft = r.op.GetBool("soft_label");
  const long* lab = soft ? nullptr : hard_labels(l, rows);
  if (soft && (l.dtype != DT::FP32 || l.numel() != x.numel())) throw Decline();
  Dims od(x.dims.begin(), x.dims.end() - 1);
  od.push_back(1);
  const Dims xd = x.dims;
  float* prob = r.out("Softmax")->alloc<float>(xd, D(r));
  float* loss = r.out("Loss")->alloc<float>(od, D(r));
  PA_KL(pa_softmax_ce_prob_fwd(0, f32(x), lab, soft ? f32(l) : nullptr, prob, loss, rows, (int)n,
                               r.op.GetInt("ignore_index", -100), S(r)));
}

void k_softmax_ce_grad(const OpRun& r) {
  Tensor& p = r.in("Softmax");
  Tensor& l = r.in("Label");
  Tensor& g = r.in("Loss@GRAD");
  int64_t n;
  const int64_t rows = last_axis_rows(r, p, &n);
  const bool soft = r.op.GetBool("soft_label");
  const long* lab = soft ? nullptr : hard_labels(l, rows);
  if (soft && (l.dtype != DT::FP32 || l.numel() != p.numel())) throw Decline();
  Tensor* dx = r.out("Logits@GRAD");
  if (!dx) return;
  PA_KL(pa_softmax_ce_prob_bwd(0, f32(p), lab, soft ? f32(l) : nullptr, f32(g), dx->alloc<float>(p.dims, D(r)), rows,
                               (int)n, r.op.GetInt("ignore_index", -100), S(r)));
}

// =============================================================== reductions over [pre, R, post]
__global__ void reduce_kernel(const float* __restrict__ x, float* __restrict__ o, int64_t pre, int64_t R,
                              int64_t post, int kind) {
  const int64_t total = pre * post;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t a = i / post, c = i % post;
    const float* p = x + a * R * post + c;
    float acc = kind == 2 ? -INFINITY : kind == 3 ? INFINITY : kind == 4 ? 1.f : 0.f;
    for (int64_t k = 0; k < R; ++k) {
      const float v = p[k * post];
      acc = kind == 2 ? fmaxf(acc, v) : kind == 3 ? fminf(acc, v) : kind == 4 ? acc * v : acc + v;
    }
    o[i] = kind == 1 ? acc / (float)R : acc;
  }
}

template <int KIND> void k_reduce(const OpRun& r) {  // 0 sum 1 mean 2 max 3 min 4 prod
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
  for (int64_t i = a; i < e; ++i)
    if (!red[(size_t)i]) throw Decline();  // non-contiguous reduced dims: host
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

// mean: one 1024-thread block, fixed-order tree (deterministic)
__global__ __launch_bounds__(1024) void mean_kernel(const float* __restrict__ x, float* __restrict__ o, int64_t n) {
  __shared__ float red[16];
  float s = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += 1024) s += x[i];
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x < 64) {
    s = threadIdx.x < 16 ? red[threadIdx.x] : 0.f;
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    if (threadIdx.x == 0) o[0] = s / (float)n;
  }
}

void k_mean(const OpRun& r) {
  Tensor x = r.in("X");
  float* o = r.out("Out")->alloc<float>({1}, D(r));
  hipLaunchKernelGGL(mean_kernel, dim3(1), dim3(1024), 0, S(r), f32(x), o, x.numel());
}

__global__ void mean_grad_kernel(const float* __restrict__ g, float* __restrict__ dx, int64_t n) {
  const float v = g[0] / (float)n;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dx[i] = v;
}

void k_mean_grad(const OpRun& r) {
  Tensor& x = r.in("X");
  Tensor& g = r.in("Out@GRAD");
  Tensor* dx = r.out("X@GRAD");
  if (!dx) return;
  const Dims d = x.dims;
  const LoD lod = x.lod;
  float* p = dx->alloc<float>(d, D(r));
  dx->lod = lod;
  if (dx->numel())
    hipLaunchKernelGGL(mean_grad_kernel, dim3(grid_for(dx->numel())), dim3(256), 0, S(r), f32(g), p, dx->numel());
}

// =============================================================== optimizers (in place when Out == In)
int64_t opt_n(const OpRun& r) {
  Tensor& p = r.in("Param");
  Tensor& g = r.in("Grad");
  if (g.dtype != DT::FP32 || g.numel() != p.numel()) throw Decline();  // e.g. SelectedRows grads: host
  return p.numel();
}

// the update target of `in_slot` -> `out_slot`: in place, or a copy of the input
float* opt_target(const OpRun& r, const char* in_slot, const char* out_slot) {
  Tensor& in = r.in(in_slot);
  if (r.op.Output(out_slot) == r.op.Input(in_slot)) return f32(in);
  const Dims d = in.dims;
  const float* src = f32(in);
  float* dst = r.out(out_slot)->alloc<float>(d, D(r));
  copy_d2d(r, dst, src, sizeof(float) * prod(d));
  return dst;
}

void k_sgd(const OpRun& r) {
  if (selected_rows_sgd(r)) return;
  const int64_t n = opt_n(r);
  float* p = opt_target(r, "Param", "ParamOut");
  PA_KL(pa_sgd(0, p, f32(r.in("Grad")), f32(r.in("LearningRate")), n, S(r)));
}

void k_momentum(const OpRun& r) {
  const int64_t n = opt_n(r);
  float* p = opt_target(r, "Param", "ParamOut");
  float* v = opt_target(r, "Velocity", "VelocityOut");
  PA_KL(pa_momentum(0, p, f32(r.in("Grad")), v, n, 0.f, f32(r.in("LearningRate")), r.op.GetFloat("mu", 0.9f),
                    r.op.GetBool("use_nesterov") ? 1 : 0, 0.f, 1.f, S(r)));
}

// adam_op.h: lr_t = lr sqrt(1 - beta2^t) / (1 - beta1^t), p -= lr_t m / (sqrt(v) + eps)
void k_adam(const OpRun& r) {
  if (selected_rows_adam(r)) return;
  const int64_t n = opt_n(r);
  float* p = opt_target(r, "Param", "ParamOut");
  float* m1 = opt_target(r, "Moment1", "Moment1Out");
  float* m2 = opt_target(r, "Moment2", "Moment2Out");
  PA_KL(pa_adamw(0, -1, p, f32(r.in("Grad")), m1, m2, nullptr, n, 0.f, f32(r.in("LearningRate")),
                 r.op.GetFloat("beta1", 0.9f), r.op.GetFloat("beta2", 0.999f), r.op.GetFloat("epsilon", 1e-8f), 0.f,
                 0.f, 0.f, f32(r.in("Beta1Pow")), f32(r.in("Beta2Pow")), n, 1.f, nullptr, 1, S(r)));
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

// fill_constant_op.cc: force_cpu pins the tensor to the host (loop counters and
// bounds the executor reads every iteration); anything else fills HBM
void k_fill_constant(const OpRun& r) {
  const DT dt = (DT)r.op.GetInt("dtype", (int)DT::FP32);
  const double v = r.op.Has("str_value") && !r.op.GetString("str_value").empty()
                       ? atof(r.op.GetString("str_value").c_str())
                       : (double)r.op.GetFloat("value");
  Tensor* o = r.out("Out");
  if (r.op.GetBool("force_cpu", false)) {
    o->alloc(dt, r.op.GetInts("shape"), -1);
    const int64_t n = o->numel();
    switch (dt) {
      case DT::FP32: std::fill_n(o->data<float>(), n, (float)v); break;
      case DT::FP64: std::fill_n(o->data<double>(), n, v); break;
      case DT::INT64: std::fill_n(o->data<int64_t>(), n, (int64_t)v); break;
      case DT::INT32: std::fill_n(o->data<int32_t>(), n, (int32_t)v); break;
      case DT::BOOL: case DT::UINT8: std::fill_n(o->data<uint8_t>(), n, (uint8_t)v); break;
      default: throw Decline();
    }
    return;
  }
  switch (dt) {
    case DT::FP32: case DT::FP64: case DT::INT64: case DT::INT32: case DT::BOOL: case DT::UINT8: break;
    default: throw Decline();
  }
  o->alloc(dt, r.op.GetInts("shape"), D(r));
  device_fill(r.ctx.stream, o->raw(), dt, o->numel(), v);
}

void k_fill_zeros_like(const OpRun& r) {  // any dtype: all-zero bytes
  Tensor& x = r.in("X");
  const Dims d = x.dims;
  const DT dt = x.dtype;
  Tensor* o = r.out("Out");
  void* p = o->alloc(dt, d, D(r));
  if (o->nbytes()) HIPCHK(hipMemsetAsync(p, 0, o->nbytes(), S(r)));
}

void k_sum(const OpRun& r) {
  if (selected_rows_sum(r)) return;
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


namespace {
// ---------------------------------------------------------------- sequence (LoD) ops
// sequence_pool / sequence_softmax over the last LoD level on the shared kernel
// library (math/sequence_pooling.cu, sequence_softmax_op.cu); the level's offsets are
// uploaded to a per-op device scratch through a pinned staging buffer (upload_host).
int seq_pool_type(const std::string& pt) {
  static const char* names[] = {"SUM", "AVERAGE", "SQRT", "MAX", "LAST", "FIRST"};
  for (int i = 0; i < 6; ++i)
    if (pt == names[i]) return i;
  return -1;
}

// Host -> device upload of a small host array into the op's device scratch `name`.
// The source is first copied into a PINNED staging buffer owned by (device, name)
// and kept alive until the copy has executed: hipMemcpyAsync from pageable memory
// does not promise to have consumed the source when it returns, and a caller's
// std::vector dies with the op.  Before the staging buffer is rewritten the event
// recorded after its previous copy is waited for.  Not capturable into a HIP graph
// (event sync, pinned allocation): the native executor runs these ops eagerly.
struct PinnedSlot {
  void* host = nullptr;
  size_t cap = 0;
  hipEvent_t ev = nullptr;
};

void* upload_host(const OpRun& r, const char* name, const void* src, size_t bytes) {
  static std::mutex mu;
  static std::map<std::string, PinnedSlot> slots;
  void* d = workspace(r, name, (int64_t)(bytes + 3) / 4);
  if (bytes == 0) return d;
  std::lock_guard<std::mutex> lk(mu);
  PinnedSlot& sl = slots[std::string(name) + "@" + std::to_string(D(r))];
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  HIPCHK(hipStreamIsCapturing(S(r), &cs));
  if (cs != hipStreamCaptureStatusNone) {
    // inside a HIP graph capture the copy's source must stay valid for every replay:
    // a dedicated pinned buffer, never reused or freed (the slot's event is not touched)
    static std::vector<void*> graph_bufs;
    void* h = nullptr;
    HIPCHK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
    memcpy(h, src, bytes);
    HIPCHK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, S(r)));
    graph_bufs.push_back(h);
    return d;
  }
  if (sl.ev) {
    if (hipEventSynchronize(sl.ev) != hipSuccess) {
      // an event that cannot be waited on (recorded into a since-abandoned capture):
      // retire the slot -- its buffer may still be referenced, so it is not freed
      (void)hipGetLastError();
      sl.ev = nullptr;
      sl.host = nullptr;
      sl.cap = 0;
    }
  }
  if (!sl.ev) HIPCHK(hipEventCreateWithFlags(&sl.ev, hipEventDisableTiming));
  if (sl.cap < bytes) {
    if (sl.host) HIPCHK(hipHostFree(sl.host));
    sl.cap = std::max(bytes, (size_t)4096);
    HIPCHK(hipHostMalloc(&sl.host, sl.cap, hipHostMallocDefault));
  }
  memcpy(sl.host, src, bytes);
  HIPCHK(hipMemcpyAsync(d, sl.host, bytes, hipMemcpyHostToDevice, S(r)));
  HIPCHK(hipEventRecord(sl.ev, S(r)));
  return d;
}

template <class T>
T* upload_offsets(const OpRun& r, const char* name, const std::vector<size_t>& off) {
  std::vector<T> h(off.begin(), off.end());
  return reinterpret_cast<T*>(upload_host(r, name, h.data(), h.size() * sizeof(T)));
}

void k_sequence_pool(const OpRun& r) {
  Tensor x = r.in("X");
  const int type = seq_pool_type(r.op.GetString("pooltype", "AVERAGE"));
  if (x.dtype != DT::FP32 || x.dims.empty() || type < 0) throw Decline();
  // no LoD: one sequence of all rows (the Python op library's _last_level)
  const std::vector<size_t> off = x.lod.empty() ? std::vector<size_t>{0, (size_t)x.dims[0]} : x.lod.back();
  const int64_t n = (int64_t)off.size() - 1, Dm = x.dims[0] ? x.numel() / x.dims[0] : 0;
  Dims od = x.dims;
  od[0] = n;
  float* y = out_f32(r, "Out", od);
  Tensor* mt = r.out("MaxIndex");
  int* mi = mt ? static_cast<int*>(mt->alloc(DT::INT32, od, D(r))) : reinterpret_cast<int*>(workspace(r, "@sp_mi@", n * Dm));
  if (mt) HIPCHK(hipMemsetAsync(mi, 0, sizeof(int) * n * Dm, S(r)));
  if (n > 0 && Dm > 0) PA_KL(pa_seq_pool(0, f32(x), upload_offsets<int>(r, "@sp_off@", off), y, mi, (int)n, (int)Dm, type, 0.f, S(r)));
  if (!x.lod.empty()) r.out("Out")->lod.assign(x.lod.begin(), x.lod.end() - 1);
}

void k_sequence_pool_grad(const OpRun& r) {
  Tensor x = r.in("X");
  Tensor g = r.in("Out@GRAD");
  const int type = seq_pool_type(r.op.GetString("pooltype", "AVERAGE"));
  if (x.dtype != DT::FP32 || g.dtype != DT::FP32 || x.dims.empty() || type < 0) throw Decline();
  Tensor* mt = r.in_opt("MaxIndex");
  if (type == 3 && (!mt || mt->dtype != DT::INT32 || mt->device != D(r))) throw Decline();
  const std::vector<size_t> off = x.lod.empty() ? std::vector<size_t>{0, (size_t)x.dims[0]} : x.lod.back();
  const int64_t n = (int64_t)off.size() - 1, Dm = x.dims[0] ? x.numel() / x.dims[0] : 0;
  float* dx = out_f32(r, "X@GRAD", x.dims);
  r.out("X@GRAD")->lod = x.lod;
  HIPCHK(hipMemsetAsync(dx, 0, sizeof(float) * x.numel(), S(r)));
  if (n > 0 && Dm > 0)
    PA_KL(pa_seq_pool_grad(0, f32(g), upload_offsets<int>(r, "@spg_off@", off), type == 3 ? mt->data<int>() : nullptr,
                           dx, (int)n, (int)Dm, type, S(r)));
}

void k_sequence_softmax(const OpRun& r) {
  Tensor x = r.in("X");
  if (x.dtype != DT::FP32 || x.lod.empty()) throw Decline();
  const auto& off = x.lod.back();
  float* y = out_f32(r, "Out", x.dims);
  r.out("Out")->lod = x.lod;
  const long n = (long)off.size() - 1;
  if (n > 0) PA_KL(pa_seq_softmax_fwd(0, f32(x), upload_offsets<long>(r, "@ss_off@", off), y, n, S(r)));
}

void k_sequence_softmax_grad(const OpRun& r) {
  Tensor y = r.in("Out");
  Tensor g = r.in("Out@GRAD");
  Tensor* xl = r.in_opt("X");
  const LoD lod = !y.lod.empty() ? y.lod : (xl ? xl->lod : LoD{});
  if (y.dtype != DT::FP32 || g.dtype != DT::FP32 || lod.empty()) throw Decline();
  const auto& off = lod.back();
  float* dx = out_f32(r, "X@GRAD", y.dims);
  r.out("X@GRAD")->lod = lod;
  const long n = (long)off.size() - 1;
  if (n > 0) PA_KL(pa_seq_softmax_bwd(0, f32(y), f32(g), upload_offsets<long>(r, "@ssg_off@", off), dx, n, S(r)));
}

// sequence_expand: the row map (sequence_expand_rows, host) uploaded once per op, then
// a row gather forward and a row scatter-add (the embedding backward) for X@GRAD
int64_t* upload_rows(const OpRun& r, const char* name, const std::vector<int64_t>& rows) {
  return reinterpret_cast<int64_t*>(upload_host(r, name, rows.data(), rows.size() * sizeof(int64_t)));
}

template <bool AS>
std::vector<int64_t> expand_rows(const OpRun& r, LoD* ol) {
  return AS ? sequence_expand_as_rows(r.in("X"), r.in("Y"), ol)
            : sequence_expand_rows(r.in("X"), r.in("Y"), r.op.GetInt("ref_level", -1), ol);
}

template <bool AS>
void k_sequence_expand(const OpRun& r) {
  Tensor x = r.in("X");
  if (x.dtype != DT::FP32 || x.dims.empty()) throw Decline();
  LoD ol;
  const auto rows = expand_rows<AS>(r, &ol);
  const int64_t n = (int64_t)rows.size(), Dm = x.dims[0] ? x.numel() / x.dims[0] : 0;
  Dims od = x.dims;
  od[0] = n;
  float* y = out_f32(r, "Out", od);
  r.out("Out")->lod = ol;
  if (n > 0 && Dm > 0)
    hipLaunchKernelGGL(gather_rows_kernel, dim3(grid_for(n * Dm)), dim3(256), 0, S(r), f32(x),
                       upload_rows(r, "@se_rows@", rows), y, n, Dm, x.dims[0], (int64_t)-1);
}

template <bool AS>
void k_sequence_expand_grad(const OpRun& r) {
  Tensor x = r.in("X");
  Tensor g = r.in("Out@GRAD");
  if (x.dtype != DT::FP32 || g.dtype != DT::FP32 || x.dims.empty()) throw Decline();
  LoD ol;
  const auto rows = expand_rows<AS>(r, &ol);
  const int64_t n = (int64_t)rows.size(), Dm = x.dims[0] ? x.numel() / x.dims[0] : 0;
  PA_CHECK(g.numel() == n * Dm, "sequence_expand_grad: Out@GRAD has %lld elements, expected %lld",
           (long long)g.numel(), (long long)(n * Dm));
  float* dx = out_f32(r, "X@GRAD", x.dims);
  r.out("X@GRAD")->lod = x.lod;
  HIPCHK(hipMemsetAsync(dx, 0, sizeof(float) * x.numel(), S(r)));
  if (n > 0 && Dm > 0)
    PA_KL(pa_embedding_bwd(0, reinterpret_cast<const long*>(upload_rows(r, "@seg_rows@", rows)), f32(g), dx, n,
                           (int)Dm, -1, S(r)));
  if (r.out("Y@GRAD")) {  // Y only shapes the expansion
    Tensor yt = r.in("Y");
    float* dy = out_f32(r, "Y@GRAD", yt.dims);
    r.out("Y@GRAD")->lod = yt.lod;
    HIPCHK(hipMemsetAsync(dy, 0, sizeof(float) * yt.numel(), S(r)));
  }
}

// sequence_concat: each input's rows scattered to their output rows (forward) and
// gathered back from Out@GRAD (backward), one launch per input over the host row map
__global__ void scatter_rows_kernel(const float* __restrict__ x, const int64_t* __restrict__ dst,
                                    float* __restrict__ o, int64_t n, int64_t D) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n * D; i += (int64_t)gridDim.x * blockDim.x)
    o[dst[i / D] * D + (i % D)] = x[i];
}

int64_t row_width(const Tensor& t) { return t.dims.empty() || t.dims[0] == 0 ? 0 : t.numel() / t.dims[0]; }

void k_sequence_concat(const OpRun& r) {
  if (r.op.GetInt("axis", 0) != 0 || r.op.GetInt("level", 0) != 0) throw Decline();
  auto xs = r.ins("X");
  for (Tensor* x : xs)
    if (x->dtype != DT::FP32 || x->dims.empty() || row_width(*x) != row_width(*xs[0])) throw Decline();
  LoD ol;
  const auto dst = sequence_concat_rows(xs, &ol);
  const int64_t Dm = row_width(*xs[0]);
  Dims od = xs[0]->dims;
  od[0] = (int64_t)ol.back().back();
  float* y = out_f32(r, "Out", od);
  r.out("Out")->lod = ol;
  for (size_t k = 0; k < xs.size(); ++k) {
    const int64_t n = (int64_t)dst[k].size();
    if (n == 0 || Dm == 0) continue;
    const std::string ws = "@sc_rows" + std::to_string(k) + "@";
    hipLaunchKernelGGL(scatter_rows_kernel, dim3(grid_for(n * Dm)), dim3(256), 0, S(r), f32(*xs[k]),
                       upload_rows(r, ws.c_str(), dst[k]), y, n, Dm);
  }
}

void k_sequence_concat_grad(const OpRun& r) {
  if (r.op.GetInt("axis", 0) != 0 || r.op.GetInt("level", 0) != 0) throw Decline();
  auto xs = r.ins("X");
  Tensor g = r.in("Out@GRAD");
  if (g.dtype != DT::FP32) throw Decline();
  for (Tensor* x : xs)
    if (x->dtype != DT::FP32 || x->dims.empty()) throw Decline();
  LoD ol;
  const auto dst = sequence_concat_rows(xs, &ol);
  for (size_t k = 0; k < xs.size(); ++k) {
    Tensor* dxt = r.out("X@GRAD", k);
    if (!dxt) continue;
    const int64_t n = (int64_t)dst[k].size(), Dm = row_width(*xs[k]);
    float* dx = static_cast<float*>(dxt->alloc(DT::FP32, xs[k]->dims, D(r)));
    dxt->lod = xs[k]->lod;
    if (n == 0 || Dm == 0) continue;
    const std::string ws = "@scg_rows" + std::to_string(k) + "@";
    hipLaunchKernelGGL(gather_rows_kernel, dim3(grid_for(n * Dm)), dim3(256), 0, S(r), f32(g),
                       upload_rows(r, ws.c_str(), dst[k]), dx, n, Dm, (int64_t)ol.back().back(), (int64_t)-1);
  }
}
}  // namespace

PA_DEVICE_KERNEL(mul, k_mul);
PA_DEVICE_KERNEL(mul_grad, k_mul_grad);
PA_DEVICE_KERNEL(fc, k_fc);
PA_DEVICE_KERNEL(matmul, k_matmul);
PA_DEVICE_KERNEL(conv2d, k_conv2d);
PA_DEVICE_KERNEL(depthwise_conv2d, k_conv2d);
PA_DEVICE_KERNEL(conv2d_grad, k_conv2d_grad);
PA_DEVICE_KERNEL(depthwise_conv2d_grad, k_conv2d_grad);
PA_DEVICE_KERNEL(pool2d, k_pool2d);
PA_DEVICE_KERNEL(pool2d_grad, k_pool2d_grad);
PA_DEVICE_KERNEL(batch_norm, k_batch_norm);
PA_DEVICE_KERNEL(batch_norm_grad, k_batch_norm_grad);
PA_DEVICE_KERNEL(softmax, k_softmax);
PA_DEVICE_KERNEL(softmax_grad, k_softmax_grad);
PA_DEVICE_KERNEL(cross_entropy, k_cross_entropy);
PA_DEVICE_KERNEL(cross_entropy_grad, k_cross_entropy_grad);
PA_DEVICE_KERNEL(softmax_with_cross_entropy, k_softmax_ce);
PA_DEVICE_KERNEL(softmax_with_cross_entropy_grad, k_softmax_ce_grad);
PA_DEVICE_KERNEL(elementwise_add, k_binary<B_ADD>);
PA_DEVICE_KERNEL(elementwise_sub, k_binary<B_SUB>);
PA_DEVICE_KERNEL(elementwise_mul, k_binary<B_MUL>);
PA_DEVICE_KERNEL(elementwise_div, k_binary<B_DIV>);
PA_DEVICE_KERNEL(elementwise_max, k_binary<B_MAX>);
PA_DEVICE_KERNEL(elementwise_min, k_binary<B_MIN>);
PA_DEVICE_KERNEL(elementwise_pow, k_binary<B_POW>);
PA_DEVICE_KERNEL(elementwise_add_grad, k_ew_grad<1>);
PA_DEVICE_KERNEL(elementwise_sub_grad, k_ew_grad<-1>);
#define PA_ACT(name, ID)                       \
  PA_DEVICE_KERNEL(name, k_act<act::ID>);      \
  PA_DEVICE_KERNEL(name##_grad, k_act_grad<act::ID>)
PA_ACT(relu, RELU);
PA_ACT(sigmoid, SIGMOID);
PA_ACT(logsigmoid, LOGSIGMOID);
PA_ACT(exp, EXP);
PA_ACT(tanh, TANH);
PA_ACT(tanh_shrink, TANH_SHRINK);
PA_ACT(softshrink, SOFTSHRINK);
PA_ACT(sqrt, SQRT);
PA_ACT(rsqrt, RSQRT);
PA_ACT(abs, ABS);
PA_ACT(ceil, CEIL);
PA_ACT(floor, FLOOR);
PA_ACT(cos, COS);
PA_ACT(sin, SIN);
PA_ACT(round, ROUND);
PA_ACT(reciprocal, RECIPROCAL);
PA_ACT(log, LOG);
PA_ACT(square, SQUARE);
PA_ACT(softplus, SOFTPLUS);
PA_ACT(softsign, SOFTSIGN);
PA_ACT(brelu, BRELU);
PA_ACT(leaky_relu, LEAKY_RELU);
PA_ACT(soft_relu, SOFT_RELU);
PA_ACT(elu, ELU);
PA_ACT(relu6, RELU6);
PA_ACT(pow, POW);
PA_ACT(stanh, STANH);
PA_ACT(hard_shrink, HARD_SHRINK);
PA_ACT(thresholded_relu, THRESHOLDED_RELU);
PA_ACT(hard_sigmoid, HARD_SIGMOID);
PA_ACT(swish, SWISH);
PA_ACT(gelu, GELU);
PA_ACT(silu, SILU);
#undef PA_ACT
PA_DEVICE_KERNEL(scale, k_scale);
PA_DEVICE_KERNEL(scale_grad, k_scale_grad);
PA_DEVICE_KERNEL(dropout, k_dropout);
PA_DEVICE_KERNEL(reduce_sum, k_reduce<0>);
PA_DEVICE_KERNEL(reduce_mean, k_reduce<1>);
PA_DEVICE_KERNEL(reduce_max, k_reduce<2>);
PA_DEVICE_KERNEL(reduce_min, k_reduce<3>);
PA_DEVICE_KERNEL(reduce_prod, k_reduce<4>);
PA_DEVICE_KERNEL(mean, k_mean);
PA_DEVICE_KERNEL(mean_grad, k_mean_grad);
PA_DEVICE_KERNEL(sgd, k_sgd);
PA_DEVICE_KERNEL(momentum, k_momentum);
PA_DEVICE_KERNEL(adam, k_adam);
PA_DEVICE_KERNEL(lookup_table, k_lookup_table);
PA_DEVICE_KERNEL(concat, k_concat);
PA_DEVICE_KERNEL(split, k_split);
PA_DEVICE_KERNEL(transpose, k_transpose);
PA_DEVICE_KERNEL(transpose2, k_transpose);
PA_DEVICE_KERNEL(fill_constant, k_fill_constant);
PA_DEVICE_KERNEL(fill_zeros_like, k_fill_zeros_like);
PA_DEVICE_KERNEL(sum, k_sum);

// =============================================================== transformer / metric ops
// layer_norm_op.cu on the shared norm kernel (norm.hip): Y plus per-row Mean and
// Variance (the grad op's inputs); rows of H % 8 != 0 or H > 8192 decline to the
// Python kernel
__global__ void rstd_to_var_kernel(const float* __restrict__ rstd, float* __restrict__ var, int64_t n, float eps) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    var[i] = 1.f / (rstd[i] * rstd[i]) - eps;
}
__global__ void var_to_rstd_kernel(const float* __restrict__ var, float* __restrict__ rstd, int64_t n, float eps) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    rstd[i] = rsqrtf(var[i] + eps);
}

// the fused norm kernel's shapes; others run the one-source row kernels
bool ln_rows(const OpRun& r, const Tensor& x, int64_t& rows, int64_t& H) {
  const size_t ax = (size_t)r.op.GetInt("begin_norm_axis", 1);
  rows = prod(x.dims, 0, ax);
  H = prod(x.dims, ax);
  if (x.dtype != DT::FP32 || rows <= 0) throw Decline();
  return H % 8 == 0 && H <= 8192;
}

void k_layer_norm(const OpRun& r) {
  Tensor x = r.in("X");
  int64_t rows, H;
  if (!ln_rows(r, x, rows, H)) return layer_norm_any(r);
  Tensor* sc = r.in_opt("Scale");
  Tensor* bi = r.in_opt("Bias");
  if ((sc && sc->dtype != DT::FP32) || (bi && bi->dtype != DT::FP32)) throw Decline();
  const float eps = r.op.GetFloat("epsilon", 1e-5f);
  const void* w = sc ? (const void*)f32(*sc) : nullptr;
  const void* b = bi ? (const void*)f32(*bi) : nullptr;
  float* y = out_f32(r, "Y", x.dims);
  r.out("Y")->lod = x.lod;
  float* rstd = workspace(r, "@ln_rstd@", rows);
  float* mean = r.out("Mean") ? out_f32(r, "Mean", {rows}) : workspace(r, "@ln_mean@", rows);
  PA_KL(pa_norm_fwd(0, 0, f32(x), nullptr, w, b, y, nullptr, mean, rstd, rows, (int)H, eps, S(r)));
  if (r.out("Variance"))
    hipLaunchKernelGGL(rstd_to_var_kernel, dim3(grid_for(rows)), dim3(256), 0, S(r), rstd,
                       out_f32(r, "Variance", {rows}), rows, eps);
}

void k_layer_norm_grad(const OpRun& r) {
  Tensor x = r.in("X");
  int64_t rows, H;
  if (!ln_rows(r, x, rows, H)) return layer_norm_grad_any(r);
  Tensor dy = r.in("Y@GRAD");
  Tensor mean = r.in("Mean");
  Tensor var = r.in("Variance");
  Tensor* sc = r.in_opt("Scale");
  if (dy.dtype != DT::FP32 || (sc && sc->dtype != DT::FP32)) throw Decline();
  const float eps = r.op.GetFloat("epsilon", 1e-5f);
  float* rstd = workspace(r, "@ln_rstd@", rows);
  hipLaunchKernelGGL(var_to_rstd_kernel, dim3(grid_for(rows)), dim3(256), 0, S(r), f32(var), rstd, rows, eps);
  const int64_t parts = std::min<int64_t>(1024, (rows + 3) / 4);  // the kernel's block cap (norm.hip)
  float* ws = workspace(r, "@ln_ws@", 2 * parts * H);
  float* dx = r.out("X@GRAD") ? out_f32(r, "X@GRAD", x.dims) : workspace(r, "@ln_dx@", rows * H);
  float* dw = (sc && r.out("Scale@GRAD")) ? out_f32(r, "Scale@GRAD", sc->dims) : workspace(r, "@ln_dw@", H);
  float* db = r.out("Bias@GRAD") ? out_f32(r, "Bias@GRAD", {H}) : workspace(r, "@ln_db@", H);
  PA_KL(pa_norm_bwd(0, 0, f32(dy), f32(x), sc ? (const void*)f32(*sc) : nullptr, f32(mean), rstd, nullptr, dx, dw,
                    db, ws, rows, (int)H, S(r)));
}

// lookup_table_grad (dense W@GRAD): zero + scatter-add of the output rows
void k_lookup_table_grad(const OpRun& r) {
  if (r.op.GetBool("is_sparse")) return lookup_table_grad_sparse(r);  // SelectedRows W@GRAD
  Tensor w = r.in("W");
  Tensor ids = r.in("Ids");
  Tensor dout = r.in("Out@GRAD");
  if (ids.dtype != DT::INT64 || dout.dtype != DT::FP32 || w.dims.size() != 2) throw Decline();
  const int64_t V = w.dims[0], Dm = w.dims[1], n = ids.numel();
  float* dw = out_f32(r, "W@GRAD", w.dims);
  HIPCHK(hipMemsetAsync(dw, 0, sizeof(float) * V * Dm, S(r)));
  if (n) PA_KL(pa_embedding_bwd(0, ids.data<int64_t>(), f32(dout), dw, n, (int)Dm, r.op.GetInt("padding_idx", -1),
                                S(r)));
}

// top_k (last axis, k <= 64): values + int64 indices
void k_top_k(const OpRun& r) {
  Tensor x = r.in("X");
  if (x.dtype != DT::FP32 || x.dims.empty()) throw Decline();
  const int k = r.op.GetInt("k", 1);
  const int64_t n = x.dims.back(), rows = x.numel() / std::max<int64_t>(n, 1);
  if (k <= 0 || k > 64 || k > n) throw Decline();
  Dims od = x.dims;
  od.back() = k;
  float* vals = out_f32(r, "Out", od);
  Tensor* it = r.out("Indices");
  int64_t* idx = static_cast<int64_t*>(it->alloc(DT::INT64, od, D(r)));
  r.out("Out")->lod = x.lod;
  it->lod = x.lod;
  PA_KL(pa_topk(0, f32(x), vals, (long*)idx, rows, (int)n, k, S(r)));
}

// accuracy (accuracy_op.cu): top-k indices vs label -> Accuracy (f32), Correct / Total (int32)
void k_accuracy(const OpRun& r) {
  Tensor ind = r.in("Indices");
  Tensor lab = r.in("Label");
  if (ind.dtype != DT::INT64 || lab.dtype != DT::INT64 || ind.dims.size() != 2) throw Decline();
  const int64_t rows = ind.dims[0];
  const int k = (int)ind.dims[1];
  float* acc = out_f32(r, "Accuracy", {1});
  int* correct = static_cast<int*>(r.out("Correct")->alloc(DT::INT32, {1}, D(r)));
  int* total = static_cast<int*>(r.out("Total")->alloc(DT::INT32, {1}, D(r)));
  PA_KL(pa_accuracy(ind.data<int64_t>(), lab.data<int64_t>(), rows, k, correct, acc, total, S(r)));
}

// dropout_grad with the native Philox mask (uint8): dX = dOut * mask * scale
void k_dropout_grad(const OpRun& r) {
  Tensor m = r.in("Mask");
  Tensor d = r.in("Out@GRAD");
  if (d.dtype != DT::FP32 || (m.dtype != DT::UINT8 && m.dtype != DT::BOOL)) throw Decline();
  const float p = r.op.GetFloat("dropout_prob", 0.5f);
  const bool upscale = r.op.GetString("dropout_implementation", "downgrade_in_infer") == "upscale_in_train";
  const float scale = (upscale && p < 1.f) ? 1.f / (1.f - p) : 1.f;
  float* dx = out_f32(r, "X@GRAD", d.dims);
  r.out("X@GRAD")->lod = d.lod;
  PA_KL(pa_mask_mul(0, f32(d), m.raw(), dx, d.numel(), scale, S(r)));
}

PA_DEVICE_KERNEL(layer_norm, k_layer_norm);
PA_DEVICE_KERNEL(layer_norm_grad, k_layer_norm_grad);
PA_DEVICE_KERNEL(lookup_table_grad, k_lookup_table_grad);
PA_DEVICE_KERNEL(top_k, k_top_k);
PA_DEVICE_KERNEL(accuracy, k_accuracy);
PA_DEVICE_KERNEL(dropout_grad, k_dropout_grad);
PA_DEVICE_KERNEL(sequence_pool, k_sequence_pool);
PA_DEVICE_KERNEL(sequence_pool_grad, k_sequence_pool_grad);
PA_DEVICE_KERNEL(sequence_softmax, k_sequence_softmax);
PA_DEVICE_KERNEL(sequence_softmax_grad, k_sequence_softmax_grad);
PA_DEVICE_KERNEL(sequence_expand, k_sequence_expand<false>);
PA_DEVICE_KERNEL(sequence_expand_grad, k_sequence_expand_grad<false>);
PA_DEVICE_KERNEL(sequence_expand_as, k_sequence_expand<true>);
PA_DEVICE_KERNEL(sequence_expand_as_grad, k_sequence_expand_grad<true>);
PA_DEVICE_KERNEL(sequence_concat, k_sequence_concat);
PA_DEVICE_KERNEL(sequence_concat_grad, k_sequence_concat_grad);

// =============================================================== ops that had only host kernels
// (every one of these used to copy its inputs to the host, sync
// twice and copy back on a HIP place)
namespace {
// elementwise_{mul,div}_grad over the [pre, n, post] broadcast of Y (the bias /
// per-channel layout): dX in one pass, dY as the per-element partial reduced by
// pa_chan_sum.  MUL: dX = g y, dY = sum g x.  DIV: dX = g / y, dY = -sum g x / y^2.
template <bool DIV>
__global__ void ew_muldiv_grad_kernel(const float* __restrict__ g, const float* __restrict__ x,
                                      const float* __restrict__ y, float* __restrict__ dx,
                                      float* __restrict__ part, int64_t total, int64_t n, int64_t post) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const float yv = y[(i / post) % n], gv = g[i];
    if (dx) dx[i] = DIV ? gv / yv : gv * yv;
    if (part) part[i] = DIV ? -gv * x[i] / (yv * yv) : gv * x[i];
  }
}

template <bool DIV> void k_ew_muldiv_grad(const OpRun& r) {
  Tensor x = r.in("X");
  Tensor y = r.in("Y");
  Tensor g = r.in("Out@GRAD");
  if (x.dtype != DT::FP32 || y.dtype != DT::FP32 || g.dtype != DT::FP32 || g.numel() != x.numel()) throw Decline();
  BcArgs b;
  int64_t pre, n, post;
  if (!make_bc(x.dims, y.dims, r.op.GetInt("axis", -1), &b, &pre, &n, &post)) throw Decline();
  const int64_t total = x.numel();
  Tensor* dxt = r.out("X@GRAD");
  Tensor* dyt = r.out("Y@GRAD");
  float* dx = nullptr;
  if (dxt) {
    dx = dxt->alloc<float>(x.dims, D(r));
    dxt->lod = x.lod;
  }
  float* dy = dyt ? dyt->alloc<float>(y.dims, D(r)) : nullptr;
  float* part = nullptr;
  if (dy) part = (pre * post == 1) ? dy : workspace(r, "@ew_grad_part@", total);
  if (total)
    hipLaunchKernelGGL(ew_muldiv_grad_kernel<DIV>, dim3(grid_for(total)), dim3(256), 0, S(r), f32(g), f32(x),
                       f32(y), dx, part, total, n, post);
  if (dy && pre * post != 1) PA_KL(pa_chan_sum(part, dy, (int)pre, (int)n, post, 0, S(r)));
}

template <class T>
__global__ void increment_kernel(const T* __restrict__ x, T* __restrict__ o, T step) {
  o[0] = x[0] + step;
}

void k_increment(const OpRun& r) {
  Tensor x = r.in("X");
  const float step = r.op.GetFloat("step", 1.f);
  Tensor* o = r.out("Out");
  void* op = o->alloc(x.dtype, {1}, D(r));
  switch (x.dtype) {
    case DT::INT64:
      hipLaunchKernelGGL(increment_kernel<int64_t>, dim3(1), dim3(1), 0, S(r), x.data<int64_t>(), (int64_t*)op,
                         (int64_t)step);
      break;
    case DT::INT32:
      hipLaunchKernelGGL(increment_kernel<int32_t>, dim3(1), dim3(1), 0, S(r), x.data<int32_t>(), (int32_t*)op,
                         (int32_t)step);
      break;
    case DT::FP32:
      hipLaunchKernelGGL(increment_kernel<float>, dim3(1), dim3(1), 0, S(r), x.data<float>(), (float*)op, step);
      break;
    default: throw Decline();
  }
}

enum CmpOp { C_LT, C_LE, C_GT, C_GE, C_EQ, C_NE, C_AND, C_OR, C_XOR, C_NOT };

template <class T>
__global__ void compare_kernel(int op, const T* __restrict__ x, const T* __restrict__ y, uint8_t* __restrict__ o,
                               int64_t n, int64_t ny) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const T a = x[i], b = y ? y[i % ny] : T(0);
    bool v;
    switch (op) {
      case C_LT: v = a < b; break;
      case C_LE: v = a <= b; break;
      case C_GT: v = a > b; break;
      case C_GE: v = a >= b; break;
      case C_EQ: v = a == b; break;
      case C_NE: v = a != b; break;
      case C_AND: v = (a != T(0)) && (b != T(0)); break;
      case C_OR: v = (a != T(0)) || (b != T(0)); break;
      case C_XOR: v = (a != T(0)) != (b != T(0)); break;
      default: v = a == T(0); break;
    }
    o[i] = v ? 1 : 0;
  }
}

// compare_op.cc / logical_op.cc on HBM: X, Y of one dtype, Y a trailing block of X
template <int OP> void k_compare(const OpRun& r) {
  Tensor x = r.in("X");
  Tensor* yp = r.in_opt("Y");
  Tensor y = yp ? *yp : Tensor();
  if (yp && (y.dtype != x.dtype || y.device != x.device)) throw Decline();
  const int64_t n = x.numel(), ny = yp ? y.numel() : 1;
  if (yp && (ny == 0 || n % ny)) throw Decline();
  Tensor* o = r.out("Out");
  uint8_t* op = static_cast<uint8_t*>(o->alloc(DT::BOOL, x.dims, D(r)));
  o->lod = x.lod;
  if (!n) return;
  const dim3 g(grid_for(n)), bl(256);
  switch (x.dtype) {
    case DT::FP32:
      hipLaunchKernelGGL(compare_kernel<float>, g, bl, 0, S(r), OP, x.data<float>(), yp ? y.data<float>() : nullptr,
                         op, n, ny);
      break;
    case DT::INT64:
      hipLaunchKernelGGL(compare_kernel<int64_t>, g, bl, 0, S(r), OP, x.data<int64_t>(),
                         yp ? y.data<int64_t>() : nullptr, op, n, ny);
      break;
    case DT::INT32:
      hipLaunchKernelGGL(compare_kernel<int32_t>, g, bl, 0, S(r), OP, x.data<int32_t>(),
                         yp ? y.data<int32_t>() : nullptr, op, n, ny);
      break;
    case DT::BOOL: case DT::UINT8:
      hipLaunchKernelGGL(compare_kernel<uint8_t>, g, bl, 0, S(r), OP, x.data<uint8_t>(),
                         yp ? y.data<uint8_t>() : nullptr, op, n, ny);
      break;
    default: throw Decline();
  }
}

void k_assign(const OpRun& r) {
  Tensor x = r.in("X");
  Tensor* o = r.out("Out");
  if (o->raw() == x.raw() && o->raw()) return;  // assign onto itself
  void* p = o->alloc(x.dtype, x.dims, D(r));
  o->lod = x.lod;
  copy_d2d(r, p, x.raw(), x.nbytes());
}

// cast_op.cc: any of fp32 / fp64 / int64 / int32 / bool / uint8 / bf16 / fp16 to any
__device__ inline double cast_load(const void* p, int dt, int64_t i) {
  switch (dt) {
    case (int)DT::FP32: return ((const float*)p)[i];
    case (int)DT::FP64: return ((const double*)p)[i];
    case (int)DT::INT64: return (double)((const int64_t*)p)[i];
    case (int)DT::INT32: return ((const int32_t*)p)[i];
    case (int)DT::BF16: return __uint_as_float((uint32_t)((const uint16_t*)p)[i] << 16);
    case (int)DT::FP16: return (float)((const _Float16*)p)[i];
    default: return ((const uint8_t*)p)[i];
  }
}

__device__ inline void cast_store(void* p, int dt, int64_t i, double v) {
  switch (dt) {
    case (int)DT::FP32: ((float*)p)[i] = (float)v; break;
    case (int)DT::FP64: ((double*)p)[i] = v; break;
    case (int)DT::INT64: ((int64_t*)p)[i] = (int64_t)v; break;
    case (int)DT::INT32: ((int32_t*)p)[i] = (int32_t)v; break;
    case (int)DT::BF16: {
      const float f = (float)v;
      const uint32_t u = __float_as_uint(f);
      ((uint16_t*)p)[i] = (u & 0x7fffffffu) > 0x7f800000u ? (uint16_t)((u >> 16) | 0x40)
                                                           : (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
      break;
    }
    case (int)DT::FP16: ((_Float16*)p)[i] = (_Float16)(float)v; break;
    case (int)DT::BOOL: ((uint8_t*)p)[i] = v != 0.0; break;
    default: ((uint8_t*)p)[i] = (uint8_t)v; break;
  }
}

__global__ void cast_kernel(const void* __restrict__ x, int xdt, void* __restrict__ o, int odt, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    cast_store(o, odt, i, cast_load(x, xdt, i));
}

bool cast_dt_ok(DT t) {
  switch (t) {
    case DT::FP32: case DT::FP64: case DT::INT64: case DT::INT32: case DT::BOOL: case DT::UINT8: case DT::BF16:
    case DT::FP16: return true;
    default: return false;
  }
}

void k_cast(const OpRun& r) {
  Tensor x = r.in("X");
  const DT out = (DT)r.op.GetInt("out_dtype", (int)DT::FP32);
  if (!cast_dt_ok(x.dtype) || !cast_dt_ok(out)) throw Decline();
  Tensor* o = r.out("Out");
  Tensor keep = x;  // Out may alias X
  Tensor res;
  res.alloc(out, x.dims, D(r));
  if (x.numel())
    hipLaunchKernelGGL(cast_kernel, dim3(grid_for(x.numel())), dim3(256), 0, S(r), keep.raw(), (int)x.dtype,
                       res.raw(), (int)out, x.numel());
  res.lod = x.lod;
  *o = res;
}

// uniform_random / gaussian_random: counter-based (splitmix64 of seed ^ index), the
// seed is the op's `seed` attr or one draw of the executor's generator per run
__device__ inline uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__device__ inline float u01(uint64_t s, int64_t i) {
  return ((mix64(s ^ (uint64_t)i * 0xd1342543de82ef95ull) >> 40) + 0.5f) * (1.f / 16777216.f);
}

template <bool GAUSS>
__global__ void random_kernel(float* __restrict__ o, int64_t n, uint64_t seed, float a, float b) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (GAUSS) {
      const float u1 = u01(seed, 2 * i), u2 = u01(seed, 2 * i + 1);
      o[i] = a + b * sqrtf(-2.f * logf(u1)) * cosf(6.283185307f * u2);
    } else {
      o[i] = a + (b - a) * u01(seed, i);
    }
  }
}

template <bool GAUSS> void k_random(const OpRun& r) {
  const DT dt = (DT)r.op.GetInt("dtype", (int)DT::FP32);
  if (dt != DT::FP32) throw Decline();
  Tensor* o = r.out("Out");
  Dims shape = r.op.GetInts("shape");
  if (r.op.type.find("batch_size_like") != std::string::npos) {  // batch_size_like.h
    const Tensor& in = r.in("Input");
    const size_t oi = (size_t)r.op.GetInt("output_dim_idx", 0), ii = (size_t)r.op.GetInt("input_dim_idx", 0);
    PA_CHECK(oi < shape.size() && ii < in.dims.size(), "%s: dim index out of range", r.op.type.c_str());
    shape[oi] = in.dims[ii];
  }
  float* p = o->alloc<float>(shape, D(r));
  const int64_t s = r.op.GetInt("seed");
  const uint64_t seed = s ? (uint64_t)s : r.ctx.rng();
  const float a = GAUSS ? r.op.GetFloat("mean", 0.f) : r.op.GetFloat("min", -1.f);
  const float b = GAUSS ? r.op.GetFloat("std", 1.f) : r.op.GetFloat("max", 1.f);
  if (o->numel())
    hipLaunchKernelGGL(random_kernel<GAUSS>, dim3(grid_for(o->numel())), dim3(256), 0, S(r), p, o->numel(), seed, a,
                       b);
}
// arg_max_op.cc over [pre, n, post] (axis attr): int64 index of the first maximum
__global__ void arg_max_kernel(const float* __restrict__ x, int64_t* __restrict__ o, int64_t pre, int64_t n,
                               int64_t post) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < pre * post; i += (int64_t)gridDim.x * blockDim.x) {
    const float* p = x + (i / post) * n * post + i % post;
    float best = p[0];
    int64_t bi = 0;
    for (int64_t k = 1; k < n; ++k)
      if (p[k * post] > best) {
        best = p[k * post];
        bi = k;
      }
    o[i] = bi;
  }
}

void k_arg_max(const OpRun& r) {
  Tensor x = r.in("X");
  if (x.dtype != DT::FP32 || x.dims.empty()) throw Decline();
  int64_t axis = r.op.GetInt("axis", -1);
  if (axis < 0) axis += (int64_t)x.dims.size();
  const int64_t pre = prod(x.dims, 0, (size_t)axis), n = x.dims[(size_t)axis], post = prod(x.dims, (size_t)axis + 1);
  Dims od;
  for (size_t i = 0; i < x.dims.size(); ++i)
    if ((int64_t)i != axis) od.push_back(x.dims[i]);
  if (od.empty()) od.push_back(1);
  Tensor* o = r.out("Out");
  int64_t* op = static_cast<int64_t*>(o->alloc(DT::INT64, od, D(r)));
  if (pre * post && n)
    hipLaunchKernelGGL(arg_max_kernel, dim3(grid_for(pre * post)), dim3(256), 0, S(r), f32(x), op, pre, n, post);
}

// shape_op.cc: the dims of Input as an int32 tensor on the executor's place
void k_shape(const OpRun& r) {
  const Dims d = r.in("Input").dims;
  std::vector<int32_t> h(d.begin(), d.end());
  Tensor* o = r.out("Out");
  void* p = o->alloc(DT::INT32, {(int64_t)h.size()}, D(r));
  copy_d2d(r, p, upload_host(r, "@shape@", h.data(), h.size() * 4), h.size() * 4);
}
}  // namespace

PA_DEVICE_KERNEL(arg_max, k_arg_max);
PA_DEVICE_KERNEL(shape, k_shape);
PA_DEVICE_KERNEL(elementwise_mul_grad, k_ew_muldiv_grad<false>);
PA_DEVICE_KERNEL(elementwise_div_grad, k_ew_muldiv_grad<true>);
PA_DEVICE_KERNEL(increment, k_increment);
PA_DEVICE_KERNEL(less_than, k_compare<C_LT>);
PA_DEVICE_KERNEL(less_equal, k_compare<C_LE>);
PA_DEVICE_KERNEL(greater_than, k_compare<C_GT>);
PA_DEVICE_KERNEL(greater_equal, k_compare<C_GE>);
PA_DEVICE_KERNEL(equal, k_compare<C_EQ>);
PA_DEVICE_KERNEL(not_equal, k_compare<C_NE>);
PA_DEVICE_KERNEL(logical_and, k_compare<C_AND>);
PA_DEVICE_KERNEL(logical_or, k_compare<C_OR>);
PA_DEVICE_KERNEL(logical_xor, k_compare<C_XOR>);
PA_DEVICE_KERNEL(logical_not, k_compare<C_NOT>);
PA_DEVICE_KERNEL(assign, k_assign);
PA_DEVICE_KERNEL(cast, k_cast);
PA_DEVICE_KERNEL(uniform_random, k_random<false>);
PA_DEVICE_KERNEL(gaussian_random, k_random<true>);
PA_DEVICE_KERNEL(uniform_random_batch_size_like, k_random<false>);
PA_DEVICE_KERNEL(gaussian_random_batch_size_like, k_random<true>);

// =============================================================== row movement for ops_control.cc
namespace {
__global__ void gather_words_kernel(const uint32_t* __restrict__ src, const int64_t* __restrict__ rows,
                                    uint32_t* __restrict__ dst, int64_t n, int64_t w) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n * w; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[rows[i / w] * w + i % w];
}
__global__ void gather_bytes_kernel(const uint8_t* __restrict__ src, const int64_t* __restrict__ rows,
                                    uint8_t* __restrict__ dst, int64_t n, int64_t w) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n * w; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[rows[i / w] * w + i % w];
}
__global__ void scatter_words_kernel(const uint32_t* __restrict__ src, const int64_t* __restrict__ rows,
                                     uint32_t* __restrict__ dst, int64_t n, int64_t w) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n * w; i += (int64_t)gridDim.x * blockDim.x)
    dst[rows[i / w] * w + i % w] = src[i];
}
__global__ void scatter_add_f32_kernel(const float* __restrict__ src, const int64_t* __restrict__ rows,
                                       float* __restrict__ dst, int64_t n, int64_t w) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n * w; i += (int64_t)gridDim.x * blockDim.x)
    atomicAdd(dst + rows[i / w] * w + i % w, src[i]);
}
template <class T>
__global__ void fill_typed_kernel(T* o, int64_t n, T v) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) o[i] = v;
}
}  // namespace

void device_gather_rows(const OpRun& r, const void* src, int64_t row_bytes, const std::vector<int64_t>& rows,
                        void* dst) {
  const int64_t n = (int64_t)rows.size();
  if (n == 0 || row_bytes == 0) return;
  const int64_t* d = upload_rows(r, "@cf_gather_rows@", rows);
  if (row_bytes % 4 == 0)
    hipLaunchKernelGGL(gather_words_kernel, dim3(grid_for(n * row_bytes / 4)), dim3(256), 0, S(r),
                       (const uint32_t*)src, d, (uint32_t*)dst, n, row_bytes / 4);
  else
    hipLaunchKernelGGL(gather_bytes_kernel, dim3(grid_for(n * row_bytes)), dim3(256), 0, S(r), (const uint8_t*)src,
                       d, (uint8_t*)dst, n, row_bytes);
}

void device_scatter_rows(const OpRun& r, const void* src, int64_t row_bytes, const std::vector<int64_t>& rows,
                         void* dst, bool add) {
  const int64_t n = (int64_t)rows.size();
  if (n == 0 || row_bytes == 0) return;
  PA_CHECK(row_bytes % 4 == 0, "device_scatter_rows: row of %lld bytes", (long long)row_bytes);
  const int64_t* d = upload_rows(r, "@cf_scatter_rows@", rows);
  const int64_t w = row_bytes / 4;
  if (add)
    hipLaunchKernelGGL(scatter_add_f32_kernel, dim3(grid_for(n * w)), dim3(256), 0, S(r), (const float*)src, d,
                       (float*)dst, n, w);
  else
    hipLaunchKernelGGL(scatter_words_kernel, dim3(grid_for(n * w)), dim3(256), 0, S(r), (const uint32_t*)src, d,
                       (uint32_t*)dst, n, w);
}

void device_copy2d(const OpRun& r, void* dst, size_t dpitch, const void* src, size_t spitch, size_t width,
                   size_t height) {
  if (width && height)
    HIPCHK(hipMemcpy2DAsync(dst, dpitch, src, spitch, width, height, hipMemcpyDeviceToDevice, S(r)));
}

namespace {
__global__ void sgd_rows_kernel(float* __restrict__ p, const float* __restrict__ v, const int64_t* __restrict__ rows,
                                const float* __restrict__ lr, int64_t n, int64_t w) {
  const float l = lr[0];
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n * w; i += (int64_t)gridDim.x * blockDim.x)
    atomicAdd(p + rows[i / w] * w + i % w, -l * v[i]);
}
// rows are unique: one thread per element, no atomics
__global__ void adam_rows_kernel(float* __restrict__ p, float* __restrict__ m1, float* __restrict__ m2,
                                 const float* __restrict__ g, const int64_t* __restrict__ rows,
                                 const float* __restrict__ lr, const float* __restrict__ b1p,
                                 const float* __restrict__ b2p, int64_t n, int64_t w, float b1, float b2, float eps) {
  const float lr_t = lr[0] * sqrtf(1.f - b2p[0]) / (1.f - b1p[0]);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n * w; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = rows[i / w] * w + i % w;
    const float gv = g[i];
    const float a = b1 * m1[e] + (1.f - b1) * gv;
    const float b = b2 * m2[e] + (1.f - b2) * gv * gv;
    m1[e] = a;
    m2[e] = b;
    p[e] -= lr_t * a / (sqrtf(b) + eps);
  }
}
}  // namespace

void device_sgd_rows(const OpRun& r, float* p, const float* v, const std::vector<int64_t>& rows, int64_t w,
                     const float* lr) {
  const int64_t n = (int64_t)rows.size();
  if (!n || !w) return;
  hipLaunchKernelGGL(sgd_rows_kernel, dim3(grid_for(n * w)), dim3(256), 0, S(r), p, v,
                     upload_rows(r, "@sgd_rows@", rows), lr, n, w);
}

void device_adam_rows(const OpRun& r, float* p, float* m1, float* m2, const float* g,
                      const std::vector<int64_t>& rows, int64_t w, const float* lr, const float* b1p,
                      const float* b2p, float b1, float b2, float eps) {
  const int64_t n = (int64_t)rows.size();
  if (!n || !w) return;
  hipLaunchKernelGGL(adam_rows_kernel, dim3(grid_for(n * w)), dim3(256), 0, S(r), p, m1, m2, g,
                     upload_rows(r, "@adam_rows@", rows), lr, b1p, b2p, n, w, b1, b2, eps);
}

void device_add_f32(void* stream, float* acc, const float* x, int64_t n) {
  if (n) hipLaunchKernelGGL(accumulate_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, acc, x, n);
}

void device_fill(void* stream, void* dst, DT dt, int64_t n, double v) {
  if (n <= 0) return;
  hipStream_t s = (hipStream_t)stream;
  const dim3 g(grid_for(n)), b(256);
  switch (dt) {
    case DT::FP32: hipLaunchKernelGGL(fill_typed_kernel<float>, g, b, 0, s, (float*)dst, n, (float)v); break;
    case DT::FP64: hipLaunchKernelGGL(fill_typed_kernel<double>, g, b, 0, s, (double*)dst, n, v); break;
    case DT::INT64: hipLaunchKernelGGL(fill_typed_kernel<int64_t>, g, b, 0, s, (int64_t*)dst, n, (int64_t)v); break;
    case DT::INT32: hipLaunchKernelGGL(fill_typed_kernel<int32_t>, g, b, 0, s, (int32_t*)dst, n, (int32_t)v); break;
    case DT::BOOL: case DT::UINT8: case DT::INT8:
      hipLaunchKernelGGL(fill_typed_kernel<uint8_t>, g, b, 0, s, (uint8_t*)dst, n, (uint8_t)v);
      break;
    default: fail("device_fill: dtype %s", dt_name(dt));
  }
}

void link_device_kernels() {}

// helpers for the device kernels of other translation units (device_util.h)
void* device_upload(const OpRun& r, const char* name, const void* src, size_t bytes) {
  return upload_host(r, name, src, bytes);
}
float* device_workspace(const OpRun& r, const char* name, int64_t n) { return workspace(r, name, n); }

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
