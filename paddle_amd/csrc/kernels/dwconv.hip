// Depthwise 2-D convolution, NHWC bf16 (reference operators/math/depthwise_conv.cu:
// KernelDepthwiseConv / ...InputGrad / ...FilterGrad, NCHW fp32 there).
//
// groups == C, Cout = C * mult (channel multiplier): output channel co reads input
// channel co / mult.  Every lane handles 8 consecutive output channels (16-B loads
// and stores on the NHWC channel axis); fp32 accumulation.
//   fwd   : y[n, oy, ox, co]  = sum_{ky,kx} x[n, iy, ix, co / mult] * w[co, ky, kx]
//   dgrad : dx[n, iy, ix, c]  = sum_{m, ky, kx : iy = oy*s - p + ky*d} dy[n, oy, ox, c*mult + m] * w[.]
//   wgrad : dw[co, ky, kx]    = sum_{n, oy, ox} dy[n, oy, ox, co] * x[n, iy, ix, co / mult]
//           (block-level partial sums over a slice of the positions, fp32 atomics)
#include "common.h"

namespace pa {
namespace {

struct DwArgs {
  int N, H, W, C, OH, OW, Cout, mult, KH, KW, sy, sx, py, px, dy_, dx_;
};

__device__ __forceinline__ float wld(const u16* w, long i) { return bf2f(w[i]); }

// w layout: [KH * KW, Cout] (the [Cout, 1, KH, KW] Paddle / torch weight transposed on
// the host, so the 8 channels of a lane are one 16-B load)
__global__ __launch_bounds__(256) void dw_fwd_kernel(DwArgs a, const u16* __restrict__ x, const u16* __restrict__ w,
                                                     const u16* __restrict__ bias, u16* __restrict__ y) {
  const int CG = a.Cout / 8;
  const long total = (long)a.N * a.OH * a.OW * CG;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int cg = (int)(i % CG);
    long t = i / CG;
    const int ox = (int)(t % a.OW);
    t /= a.OW;
    const int oy = (int)(t % a.OH);
    const int n = (int)(t / a.OH);
    const int co0 = cg * 8;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = bias ? bf2f(bias[co0 + j]) : 0.f;
    for (int ky = 0; ky < a.KH; ++ky) {
      const int iy = oy * a.sy - a.py + ky * a.dy_;
      if (iy < 0 || iy >= a.H) continue;
      for (int kx = 0; kx < a.KW; ++kx) {
        const int ix = ox * a.sx - a.px + kx * a.dx_;
        if (ix < 0 || ix >= a.W) continue;
        const u16* xp = x + (((long)n * a.H + iy) * a.W + ix) * a.C;
        float wv[8];
        load8(w + (long)(ky * a.KW + kx) * a.Cout + co0, wv);
        if (a.mult == 1) {
          float xv[8];
          load8(xp + co0, xv);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += xv[j] * wv[j];
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += bf2f(xp[(co0 + j) / a.mult]) * wv[j];
        }
      }
    }
    store8(y + (((long)n * a.OH + oy) * a.OW + ox) * a.Cout + co0, acc);
  }
}

// dx: one lane per 8 input channels of one input pixel
__global__ __launch_bounds__(256) void dw_dgrad_kernel(DwArgs a, const u16* __restrict__ dy, const u16* __restrict__ w,
                                                       u16* __restrict__ dx) {
  const int CG = a.C / 8;
  const long total = (long)a.N * a.H * a.W * CG;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int cg = (int)(i % CG);
    long t = i / CG;
    const int ix = (int)(t % a.W);
    t /= a.W;
    const int iy = (int)(t % a.H);
    const int n = (int)(t / a.H);
    const int c0 = cg * 8;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int ky = 0; ky < a.KH; ++ky) {
      const int ty = iy + a.py - ky * a.dy_;
      if (ty < 0 || ty % a.sy) continue;
      const int oy = ty / a.sy;
      if (oy >= a.OH) continue;
      for (int kx = 0; kx < a.KW; ++kx) {
        const int tx = ix + a.px - kx * a.dx_;
        if (tx < 0 || tx % a.sx) continue;
        const int ox = tx / a.sx;
        if (ox >= a.OW) continue;
        const u16* gp = dy + (((long)n * a.OH + oy) * a.OW + ox) * a.Cout;
        const u16* wp = w + (long)(ky * a.KW + kx) * a.Cout;
        if (a.mult == 1) {
          float g[8], wv[8];
          load8(gp + c0, g);
          load8(wp + c0, wv);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += g[j] * wv[j];
        } else {
          for (int m = 0; m < a.mult; ++m) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const int co = (c0 + j) * a.mult + m;
              acc[j] += bf2f(gp[co]) * wld(wp, co);
            }
          }
        }
      }
    }
    store8(dx + (((long)n * a.H + iy) * a.W + ix) * a.C + c0, acc);
  }
}

// dw (fp32, zeroed, [KH * KW, Cout]): grid (KH*KW, channel-group blocks, position
// slices).  A block's 256 lanes are (position lane r, channel group cg) with
// cgn = min(CG, 256) groups per block and 256 / cgn positions per pass, so small C
// (MobileNet's first layers: C = 32 -> 4 groups) still keeps every lane busy.
__global__ __launch_bounds__(256) void dw_wgrad_kernel(DwArgs a, const u16* __restrict__ dy, const u16* __restrict__ x,
                                                       float* __restrict__ dw, long slice, int cgn) {
  const int tap = blockIdx.x;
  const int ky = tap / a.KW, kx = tap % a.KW;
  const int CG = a.Cout / 8;
  const int rows = 256 / cgn;
  const int r = threadIdx.x / cgn;
  const int cg = blockIdx.y * cgn + threadIdx.x % cgn;
  const long P = (long)a.N * a.OH * a.OW;
  const long p0 = (long)blockIdx.z * slice, p1 = min(P, p0 + slice);
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (r < rows && cg < CG) {
    const int co0 = cg * 8;
    for (long pos = p0 + r; pos < p1; pos += rows) {
      const int ox = (int)(pos % a.OW);
      long t = pos / a.OW;
      const int oy = (int)(t % a.OH);
      const int n = (int)(t / a.OH);
      const int iy = oy * a.sy - a.py + ky * a.dy_, ix = ox * a.sx - a.px + kx * a.dx_;
      if (iy < 0 || iy >= a.H || ix < 0 || ix >= a.W) continue;
      float g[8];
      load8(dy + pos * a.Cout + co0, g);
      const u16* xp = x + (((long)n * a.H + iy) * a.W + ix) * a.C;
      if (a.mult == 1) {
        float xv[8];
        load8(xp + co0, xv);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += g[j] * xv[j];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += g[j] * bf2f(xp[(co0 + j) / a.mult]);
      }
    }
  }
  __shared__ float red[256][9];
#pragma unroll
  for (int j = 0; j < 8; ++j) red[threadIdx.x][j] = acc[j];
  __syncthreads();
  // lanes 0..cgn-1 fold the position rows, 8 channels each
  if (threadIdx.x < cgn && cg < CG) {
    float s8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int rr = 0; rr < rows; ++rr)
#pragma unroll
      for (int j = 0; j < 8; ++j) s8[j] += red[rr * cgn + threadIdx.x][j];
    float* o = dw + (long)tap * a.Cout + cg * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) atomicAdd(o + j, s8[j]);
  }
}

DwArgs make(int N, int H, int W, int C, int Cout, int KH, int KW, int sy, int sx, int py, int px, int dy, int dx) {
  DwArgs a;
  a.N = N; a.H = H; a.W = W; a.C = C; a.Cout = Cout; a.mult = Cout / C;
  a.KH = KH; a.KW = KW; a.sy = sy; a.sx = sx; a.py = py; a.px = px; a.dy_ = dy; a.dx_ = dx;
  a.OH = (H + 2 * py - dy * (KH - 1) - 1) / sy + 1;
  a.OW = (W + 2 * px - dx * (KW - 1) - 1) / sx + 1;
  return a;
}

int grid_for(long n) {
  long g = (n + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}
}  // namespace
}  // namespace pa

using namespace pa;

// shapes: C % 8 == 0, Cout % C == 0 (checked here: a malformed call returns -1)
PA_EXPORT int pa_dwconv_fwd(const void* x, const void* w, const void* bias, void* y, int N, int H, int W, int C,
                            int Cout, int KH, int KW, int sy, int sx, int py, int px, int dy, int dx, hipStream_t st) {
  if (C % 8 || Cout % C || Cout % 8 || sy < 1 || sx < 1 || dy < 1 || dx < 1) return -1;
  DwArgs a = make(N, H, W, C, Cout, KH, KW, sy, sx, py, px, dy, dx);
  if (a.OH <= 0 || a.OW <= 0) return -1;
  hipLaunchKernelGGL(dw_fwd_kernel, dim3(grid_for((long)N * a.OH * a.OW * (Cout / 8))), dim3(256), 0, st, a,
                     (const u16*)x, (const u16*)w, (const u16*)bias, (u16*)y);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_dwconv_dgrad(const void* dy_, const void* w, void* dx_, int N, int H, int W, int C, int Cout, int KH,
                              int KW, int sy, int sx, int py, int px, int dy, int dx, hipStream_t st) {
  if (C % 8 || Cout % C || sy < 1 || sx < 1 || dy < 1 || dx < 1) return -1;
  DwArgs a = make(N, H, W, C, Cout, KH, KW, sy, sx, py, px, dy, dx);
  hipLaunchKernelGGL(dw_dgrad_kernel, dim3(grid_for((long)N * H * W * (C / 8))), dim3(256), 0, st, a,
                     (const u16*)dy_, (const u16*)w, (u16*)dx_);
  PA_LAUNCH_CHECK();
}

PA_EXPORT int pa_dwconv_wgrad(const void* dy_, const void* x, float* dw, int N, int H, int W, int C, int Cout, int KH,
                              int KW, int sy, int sx, int py, int px, int dy, int dx, hipStream_t st) {
  if (C % 8 || Cout % C || Cout % 8 || sy < 1 || sx < 1 || dy < 1 || dx < 1) return -1;
  DwArgs a = make(N, H, W, C, Cout, KH, KW, sy, sx, py, px, dy, dx);
  const long P = (long)N * a.OH * a.OW;
  const int CG = Cout / 8;
  const int cgn = CG < 256 ? CG : 256;
  const int cgb = (CG + cgn - 1) / cgn;
  // enough position slices to put ~8 blocks on every CU
  long slices = (2048 + (long)KH * KW * cgb - 1) / ((long)KH * KW * cgb);
  if (slices < 1) slices = 1;
  if (slices > P) slices = P;
  const long slice = (P + slices - 1) / slices;
  dim3 g((unsigned)(KH * KW), (unsigned)cgb, (unsigned)((P + slice - 1) / slice));
  hipLaunchKernelGGL(dw_wgrad_kernel, g, dim3(256), 0, st, a, (const u16*)dy_, (const u16*)x, dw, slice, cgn);
  PA_LAUNCH_CHECK();
}
