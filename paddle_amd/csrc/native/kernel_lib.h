// C ABI of the gfx950 kernel library (libpaddle_amd_kernels.so, csrc/kernels/*.hip)
// that the native executor's device kernels call.  The executor has no GEMM, conv,
// pooling, norm, softmax / loss or optimizer kernels of its own: the Python Fluid
// operators and the C++ executor run the SAME launchers, so fixes and tuning land
// once (libpaddle_amd_native.so links the kernel library, rpath $ORIGIN).
//
// Every launcher returns 0 or a hipError_t / -1 on bad arguments; call through
// PA_KL() so a failure raises pa::Error naming the launcher.
#pragma once

#include <hip/hip_runtime.h>

extern "C" {
// convnd.hip: strided / batched exact-fp32 MFMA GEMM (+ k-batch, row bias, split-K)
int pa_sgemm(const float* A, long sam, long sak, const float* B, long sbk, long sbn, float* C, long ldc, long M,
             long N, long K, int Z1, int Z2, long bsA1, long bsB1, long bsC1, long bsA2, long bsB2, long bsC2, int kb,
             long kbA, long kbB, const float* bias_m, long bsBias2, float alpha, float beta, int atomic,
             const int* conv, hipStream_t st);
// geo: C, D, H, W, OD, OH, OW, kd, kh, kw, sd, sh, sw, pd, ph, pw, dd, dh, dw (host array)
int pa_vol2col(int dt, const void* x, void* col, const int* geo, int nb, hipStream_t st);
int pa_col2vol(const float* col, float* x, const int* geo, int nb, int accumulate, hipStream_t st);
int pa_chan_sum(const float* y, float* out, int N, int C, long S, int accumulate, hipStream_t st);
// pool geo: D, H, W, OD, OH, OW, kd, kh, kw, sd, sh, sw, pd, ph, pw; type 0 max (mask) / 1 avg
int pa_pool_fwd(int dt, const void* x, void* y, int* mask, long NC, const int* geo, int type, int exclusive,
                hipStream_t st);
int pa_pool_bwd(int dt, const void* dy, const int* mask, void* dx, long NC, const int* geo, int type, int exclusive,
                hipStream_t st);
int pa_bn_nchw_groups(int C, long M);
int pa_bn_nchw_fwd(int dt, const void* x, void* y, const float* scale, const float* bias, const float* run_mean,
                   const float* run_var, float* mean_out, float* var_out, float* mean, float* rstd, float* part, int N,
                   int C, long S, float eps, float momentum, int training, int relu, int unbiased, hipStream_t st);
int pa_bn_nchw_bwd(int dt, const void* x, const void* dy, const void* y, const float* mean, const float* rstd,
                   const float* scale, float* dscale, float* dbias, void* dx, float* part, int N, int C, long S,
                   int relu, hipStream_t st);
// fluid_ops.hip: activation table (enum Act) and softmax + cross-entropy on probabilities
int pa_act_fwd(int op, int dtype, const void* x, void* y, long n, float a, float b, hipStream_t st);
int pa_act_bwd(int op, int dtype, const void* x, const void* y, const void* dy, void* dx, long n, float a, float b,
               hipStream_t st);
int pa_softmax_ce_prob_fwd(int dtype, const void* x, const long* label, const void* soft, void* prob, void* loss,
                           long N, int V, long ignore_index, hipStream_t st);
int pa_softmax_ce_prob_bwd(int dtype, const void* prob, const long* label, const void* soft, const void* dloss,
                           void* dx, long N, int V, long ignore_index, hipStream_t st);
// softmax_ce.hip
int pa_softmax_fwd(int dtype, const void* x, void* y, long N, int V, int log_softmax, hipStream_t st);
int pa_softmax_bwd(int dtype, const void* y, const void* dy, void* dx, long N, int V, int log_softmax,
                   hipStream_t st);
// nnmisc.hip: cross_entropy on probabilities (hard or soft labels)
int pa_cross_entropy(int dt, int backward, const void* x, const long* label, const void* soft, const void* dy,
                     void* out, long rows, int D, long ignore, hipStream_t st);
// optimizer.hip / oplib.hip (lr, beta pows read from device memory)
int pa_adamw(int gdtype, int pdtype, float* p, const void* g, float* m, float* v, void* pout, long n, float lr,
             const float* lr_ptr, float b1, float b2, float eps, float wd, float bc1, float bc2, const float* b1pow,
             const float* b2pow, long decay_end, float gscale, const float* gscale_ptr, int lr_t_eps,
             hipStream_t st);
int pa_momentum(int gdtype, float* p, const void* g, float* vel, long n, float lr, const float* lr_ptr, float mu,
                int nesterov, float wd, float gscale, hipStream_t st);
int pa_sgd(int dt, void* p, const void* g, const float* lr, long n, hipStream_t st);
// norm.hip: LayerNorm / RMSNorm rows (H % 8 == 0, H <= 8192); ws: 2 * min(512, ceil(N/4)) * H floats
int pa_norm_fwd(int dtype, int rms, const void* x, const void* res, const void* w, const void* b, void* y,
                void* hout, float* mean, float* rstd, long N, int H, float eps, hipStream_t st);
int pa_norm_bwd(int dtype, int rms, const void* dy, const void* h, const void* w, const float* mean,
                const float* rstd, const void* dres, void* dx, void* dw, void* db, float* ws, long N, int H,
                hipStream_t st);
// elementwise.hip / oplib.hip / misc.hip
int pa_embedding_bwd(int dtype, const long* ids, const void* dout, float* dW, long N, int H, long padding_idx,
                     hipStream_t st);
int pa_topk(int dt, const void* x, void* vals, long* idx, long rows, int n, int k, hipStream_t st);
int pa_accuracy(const long* ind, const long* lab, long rows, int k, int* correct, float* acc, int* total,
                hipStream_t st);
int pa_mask_mul(int dt, const void* d, const void* mask, void* out, long n, float scale, hipStream_t st);
int pa_seq_pool(int dt, const void* x, const int* off, void* out, int* maxi, int nseq, int D, int type, float pad,
                hipStream_t st);
int pa_seq_pool_grad(int dt, const void* dout, const int* off, const int* maxi, void* dx, int nseq, int D, int type,
                     hipStream_t st);
int pa_seq_softmax_fwd(int dtype, const void* x, const long* off, void* y, long nseq, hipStream_t st);
int pa_seq_softmax_bwd(int dtype, const void* y, const void* dy, const long* off, void* dx, long nseq, hipStream_t st);
}

// activation ids of fluid_ops.hip enum Act
namespace pa {
namespace act {
enum {
  RELU = 0, SIGMOID, LOGSIGMOID, EXP, TANH, TANH_SHRINK, SOFTSHRINK, SQRT, RSQRT, ABS, CEIL, FLOOR, COS, SIN,
  ROUND, RECIPROCAL, LOG, SQUARE, SOFTPLUS, SOFTSIGN, BRELU, LEAKY_RELU, SOFT_RELU, ELU, RELU6, POW, STANH,
  HARD_SHRINK, THRESHOLDED_RELU, HARD_SIGMOID, SWISH, GELU, SILU
};
}  // namespace act
}  // namespace pa

#define PA_KL(call)                                                       \
  do {                                                                    \
    const int rc_ = (call);                                               \
    if (rc_ != 0) ::pa::fail("%s failed (code %d)", #call, rc_);          \
  } while (0)
