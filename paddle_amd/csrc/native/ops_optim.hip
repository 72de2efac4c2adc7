// Dense elementwise optimizer updates of the native executor, host AND device:
// adagrad, decayed_adagrad, adadelta, rmsprop (plain / centered), adamax, ftrl.
//
// Semantics: operators/{adagrad,decayed_adagrad,adadelta,rmsprop,adamax,ftrl}_op.h
// of the reference (the Python kernels of operators/optimizer_ops.py compute the
// same expressions, in the same order, so the engines train along one trajectory).
// One __host__ __device__ update per element serves both places: the host kernel
// runs it over the worker pool, the device kernel as a grid-stride HIP kernel with
// the learning rate (and beta powers) read from device memory -- no host sync.
// Outputs may alias their inputs (ParamOut == Param): every update reads an
// element's inputs before writing its outputs.  SelectedRows gradients decline.
#include <hip/hip_runtime.h>
#include <math.h>

#include <string.h>

#include <string>

#include "device_util.h"

namespace pa {
namespace {

enum OptKind { O_ADAGRAD, O_DECAYED_ADAGRAD, O_ADADELTA, O_RMSPROP, O_ADAMAX, O_FTRL };

struct OptArgs {
  int kind;
  int64_t n;
  float* p;
  const float* g;
  float *s0, *s1, *s2;   // state buffers (meaning per kind)
  const float* lr;       // [1] (null for adadelta)
  const float* b1pow;    // adamax
  float a0, a1, a2, a3;  // attributes (meaning per kind)
  int centered;
};

__host__ __device__ __forceinline__ void opt_update(const OptArgs& A, int64_t i) {
  const float g = A.g[i];
  const float lr = A.lr ? A.lr[0] : 0.f;
  switch (A.kind) {
    case O_ADAGRAD: {  // s0 = moment; a0 = eps
      const float m2 = A.s0[i] + g * g;
      A.s0[i] = m2;
      A.p[i] = A.p[i] - lr * g / (sqrtf(m2) + A.a0);
      break;
    }
    case O_DECAYED_ADAGRAD: {  // s0 = moment; a0 = decay, a1 = eps
      const float m2 = A.a0 * A.s0[i] + (1.f - A.a0) * g * g;
      A.s0[i] = m2;
      A.p[i] = A.p[i] - lr * g / (sqrtf(m2) + A.a1);
      break;
    }
    case O_ADADELTA: {  // s0 = avg sq grad, s1 = avg sq update; a0 = rho, a1 = eps
      const float ag2 = A.a0 * A.s0[i] + (1.f - A.a0) * g * g;
      const float upd = -sqrtf((A.s1[i] + A.a1) / (ag2 + A.a1)) * g;
      A.s0[i] = ag2;
      A.s1[i] = A.a0 * A.s1[i] + (1.f - A.a0) * upd * upd;
      A.p[i] = A.p[i] + upd;
      break;
    }
    case O_RMSPROP: {  // s0 = mean square, s1 = moment, s2 = mean grad; a0 = eps, a1 = decay, a2 = momentum
      const float ms2 = A.a1 * A.s0[i] + (1.f - A.a1) * g * g;
      float mom2;
      if (A.centered) {
        const float mg2 = A.a1 * A.s2[i] + (1.f - A.a1) * g;
        mom2 = A.a2 * A.s1[i] + lr * g / sqrtf(ms2 - mg2 * mg2 + A.a0);
        A.s2[i] = mg2;
      } else {
        mom2 = A.a2 * A.s1[i] + lr * g / sqrtf(ms2 + A.a0);
      }
      A.s0[i] = ms2;
      A.s1[i] = mom2;
      A.p[i] = A.p[i] - mom2;
      break;
    }
    case O_ADAMAX: {  // s0 = moment, s1 = inf norm; a0 = beta1, a1 = beta2, a2 = eps
      const float m2 = A.a0 * A.s0[i] + (1.f - A.a0) * g;
      const float u2 = fmaxf(A.a1 * A.s1[i] + A.a2, fabsf(g));
      A.s0[i] = m2;
      A.s1[i] = u2;
      A.p[i] = A.p[i] - lr / (1.f - A.b1pow[0]) * m2 / u2;
      break;
    }
    case O_FTRL: {  // s0 = squared accum, s1 = linear accum; a0 = l1, a1 = l2, a2 = lr_power
      const float sq = A.s0[i], p = A.p[i];
      const float nsq = sq + g * g;
      float sigma, y;
      if (A.a2 == -0.5f) {
        sigma = (sqrtf(nsq) - sqrtf(sq)) / lr;
        y = sqrtf(nsq) / lr + 2.f * A.a1;
      } else {
        sigma = (powf(nsq, -A.a2) - powf(sq, -A.a2)) / lr;
        y = powf(nsq, -A.a2) / lr + 2.f * A.a1;
      }
      const float nlin = A.s1[i] + g - sigma * p;
      const float pre = fminf(fmaxf(nlin, -A.a0), A.a0) - nlin;
      A.p[i] = fabsf(nlin) > A.a0 ? pre / y : 0.f;
      A.s0[i] = nsq;
      A.s1[i] = nlin;
      break;
    }
  }
}

__global__ void opt_kernel(OptArgs A) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < A.n; i += (int64_t)gridDim.x * blockDim.x)
    opt_update(A, i);
}

// Output `out` of the op bound to the state `in`: in place when they alias, else the
// output is allocated on `in`'s place and initialised from it.
float* state_out(const OpRun& r, const char* in_slot, const char* out_slot) {
  Tensor& in = r.in(in_slot);
  if (in.dtype != DT::FP32) throw Decline{};
  Tensor* o = r.out(out_slot);
  if (!o) throw Decline{};
  if (o == &in || o->raw() == in.raw()) return in.data<float>();
  const Tensor src = in;  // (the output may re-point the variable that held `in`)
  o->alloc(DT::FP32, src.dims, src.device);
  if (src.nbytes()) {
    if (src.device < 0) memcpy(o->raw(), src.raw(), src.nbytes());
    else device_copy(o->raw(), src.device, src.raw(), src.device, src.nbytes(), r.ctx.stream);
  }
  return o->data<float>();
}

template <bool DEVICE>
void run_opt(const OpRun& r, int kind) {
  Variable* gv = r.in_var("Grad");
  if (gv->kind != VK_LOD_TENSOR) throw Decline{};  // SelectedRows: the embedder's kernel
  Tensor& g = gv->tensor;
  Tensor& p = r.in("Param");
  if (g.dtype != DT::FP32 || p.dtype != DT::FP32 || g.numel() != p.numel()) throw Decline{};
  if (DEVICE != (p.device >= 0) || g.device != p.device) throw Decline{};
  OptArgs A{};
  A.kind = kind;
  A.n = p.numel();
  A.g = g.data<float>();
  A.p = state_out(r, "Param", "ParamOut");
  const OpDesc& op = r.op;
  if (kind != O_ADADELTA) {
    Tensor& lr = r.in("LearningRate");
    if (lr.dtype != DT::FP32 || lr.device != p.device) throw Decline{};
    A.lr = lr.data<float>();
  }
  switch (kind) {
    case O_ADAGRAD:
      A.s0 = state_out(r, "Moment", "MomentOut");
      A.a0 = op.GetFloat("epsilon", 1e-6f);
      break;
    case O_DECAYED_ADAGRAD:
      A.s0 = state_out(r, "Moment", "MomentOut");
      A.a0 = op.GetFloat("decay", 0.95f);
      A.a1 = op.GetFloat("epsilon", 1e-6f);
      break;
    case O_ADADELTA:
      A.s0 = state_out(r, "AvgSquaredGrad", "AvgSquaredGradOut");
      A.s1 = state_out(r, "AvgSquaredUpdate", "AvgSquaredUpdateOut");
      A.a0 = op.GetFloat("rho", 0.95f);
      A.a1 = op.GetFloat("epsilon", 1e-6f);
      break;
    case O_RMSPROP:
      A.s0 = state_out(r, "MeanSquare", "MeanSquareOut");
      A.s1 = state_out(r, "Moment", "MomentOut");
      A.centered = op.GetBool("centered", false);
      if (A.centered) A.s2 = state_out(r, "MeanGrad", "MeanGradOut");
      A.a0 = op.GetFloat("epsilon", 1e-10f);
      A.a1 = op.GetFloat("decay", 0.9f);
      A.a2 = op.GetFloat("momentum", 0.f);
      break;
    case O_ADAMAX: {
      A.s0 = state_out(r, "Moment", "MomentOut");
      A.s1 = state_out(r, "InfNorm", "InfNormOut");
      Tensor& bp = r.in("Beta1Pow");
      if (bp.dtype != DT::FP32) throw Decline{};
      if (DEVICE && bp.device != p.device) throw Decline{};
      A.b1pow = bp.data<float>();
      A.a0 = op.GetFloat("beta1", 0.9f);
      A.a1 = op.GetFloat("beta2", 0.999f);
      A.a2 = op.GetFloat("epsilon", 1e-8f);
      break;
    }
    case O_FTRL:
      A.s0 = state_out(r, "SquaredAccumulator", "SquaredAccumOut");
      A.s1 = state_out(r, "LinearAccumulator", "LinearAccumOut");
      A.a0 = op.GetFloat("l1", 0.f);
      A.a1 = op.GetFloat("l2", 0.f);
      A.a2 = op.GetFloat("lr_power", -0.5f);
      break;
  }
  if (A.n == 0) return;
  if (DEVICE) {
    hipLaunchKernelGGL(opt_kernel, dim3(dev_grid(A.n)), dim3(256), 0, dev_stream(r), A);
    PA_HIPCHK(hipGetLastError());
  } else {
    parallel_for(A.n, 4096, [&](int64_t a, int64_t b) {
      for (int64_t i = a; i < b; ++i) opt_update(A, i);
    });
  }
}

template <int KIND>
void k_host(const OpRun& r) { run_opt<false>(r, KIND); }
template <int KIND>
void k_dev(const OpRun& r) { run_opt<true>(r, KIND); }

}  // namespace

#define PA_OPT_KERNEL(name, KIND)              \
  PA_HOST_KERNEL(name, k_host<KIND>);          \
  PA_DEVICE_KERNEL(name, k_dev<KIND>)
PA_OPT_KERNEL(adagrad, O_ADAGRAD);
PA_OPT_KERNEL(decayed_adagrad, O_DECAYED_ADAGRAD);
PA_OPT_KERNEL(adadelta, O_ADADELTA);
PA_OPT_KERNEL(rmsprop, O_RMSPROP);
PA_OPT_KERNEL(adamax, O_ADAMAX);
PA_OPT_KERNEL(ftrl, O_FTRL);
#undef PA_OPT_KERNEL

void link_optim_kernels() {}

}  // namespace pa
