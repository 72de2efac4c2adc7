// Layout operators of the native executor, host AND device: slice / slice_grad,
// stack / stack_grad, unstack / unstack_grad, transpose_grad, expand, and the
// view-only gradients of squeeze / unsqueeze / flatten (+ their "2" variants).
//
// Semantics: reference operators/slice_op.{cc,h} (starts / ends clamped to the
// axis, negatives counted from the end; the gradient pads Out@GRAD back with
// zeros), stack_op.h (Y[pre, i, post] = X_i[pre, post]), unstack_op.h,
// transpose_op.h (the gradient is the inverse permutation), expand_op.h (tile by
// expand_times), squeeze_op.cc / unsqueeze_op.cc / flatten_op.cc (grads reshape
// Out@GRAD to X's dims).  All data movement is one strided-region copy: an up to
// 8-D box read with the source's strides (0 for a broadcast dim) and written with
// the destination's, run over the worker pool on the host and as a grid-stride
// HIP kernel on the op's stream on a device place -- the multi-axis slice of a
// StaticRNN step is one launch, not a chain of 2-D copies.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <string>

#include "device_util.h"

namespace pa {
namespace {

using Dims = std::vector<int64_t>;
constexpr int kMaxBox = 8;

int64_t prodd(const Dims& d, size_t b = 0, size_t e = (size_t)-1) {
  int64_t n = 1;
  for (size_t i = b; i < d.size() && i < e; ++i) n *= d[i];
  return n;
}

Dims contiguous_strides(const Dims& d) {
  Dims s(d.size());
  int64_t acc = 1;
  for (size_t i = d.size(); i-- > 0;) {
    s[i] = acc;
    acc *= d[i];
  }
  return s;
}

// dst[off_d + sum i_k * ds_k] = src[off_s + sum i_k * ss_k] over the box `n`
struct Box {
  int R;
  int64_t n[kMaxBox], ss[kMaxBox], ds[kMaxBox];
  int64_t off_s, off_d, total;
};

template <class T>
__host__ __device__ __forceinline__ void box_one(const Box& b, const T* __restrict__ s, T* __restrict__ d, int64_t i) {
  int64_t so = b.off_s, dof = b.off_d;
  for (int k = b.R - 1; k >= 0; --k) {
    const int64_t q = i % b.n[k];
    i /= b.n[k];
    so += q * b.ss[k];
    dof += q * b.ds[k];
  }
  d[dof] = s[so];
}

template <class T>
__global__ void box_kernel(Box b, const T* __restrict__ s, T* __restrict__ d) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < b.total; i += (int64_t)gridDim.x * blockDim.x)
    box_one<T>(b, s, d, i);
}

// merge adjacent dims that are contiguous in BOTH source and destination, so the
// common "row block" copy runs with one or two index divisions per element
Box make_box(Dims n, Dims ss, Dims ds, int64_t off_s, int64_t off_d) {
  Dims mn, ms, md;
  for (size_t k = 0; k < n.size(); ++k) {
    if (n[k] == 1) continue;
    if (!mn.empty() && ms.back() == ss[k] * n[k] && md.back() == ds[k] * n[k]) {
      mn.back() *= n[k];
      ms.back() = ss[k];
      md.back() = ds[k];
      continue;
    }
    mn.push_back(n[k]);
    ms.push_back(ss[k]);
    md.push_back(ds[k]);
  }
  if (mn.empty()) {
    mn = {1};
    ms = {0};
    md = {0};
  }
  PA_CHECK(mn.size() <= (size_t)kMaxBox, "layout op: more than %d non-mergeable dims", kMaxBox);
  Box b{};
  b.R = (int)mn.size();
  b.total = 1;
  for (int k = 0; k < b.R; ++k) {
    b.n[k] = mn[(size_t)k];
    b.ss[k] = ms[(size_t)k];
    b.ds[k] = md[(size_t)k];
    b.total *= b.n[k];
  }
  b.off_s = off_s;
  b.off_d = off_d;
  for (size_t k = 0; k < n.size(); ++k)
    if (n[k] == 0) b.total = 0;
  return b;
}

template <class T>
void run_box_t(const OpRun& r, const Box& b, const void* s, void* d, bool dev) {
  if (dev) {
    hipLaunchKernelGGL(box_kernel<T>, dim3(dev_grid(b.total)), dim3(256), 0, dev_stream(r), b, (const T*)s, (T*)d);
    PA_HIPCHK(hipGetLastError());
  } else {
    parallel_for(b.total, 16384, [&](int64_t a, int64_t e) {
      for (int64_t i = a; i < e; ++i) box_one<T>(b, (const T*)s, (T*)d, i);
    });
  }
}

void run_box(const OpRun& r, const Box& b, DT dt, const void* s, void* d, bool dev) {
  if (b.total == 0) return;
  switch (dt_size(dt)) {
    case 1: run_box_t<uint8_t>(r, b, s, d, dev); break;
    case 2: run_box_t<uint16_t>(r, b, s, d, dev); break;
    case 4: run_box_t<uint32_t>(r, b, s, d, dev); break;
    case 8: run_box_t<uint64_t>(r, b, s, d, dev); break;
    default: fail("layout op: unsupported element size %zu", dt_size(dt));
  }
}

void zero_fill(const OpRun& r, Tensor* t) {
  if (!t->numel()) return;
  if (t->device >= 0) device_fill(r.ctx.stream, t->raw(), t->dtype, t->numel(), 0.0);
  else memset(t->raw(), 0, t->nbytes());
}

// ------------------------------------------------------------------ slice
struct SliceBox {
  Dims out, begin;
};

SliceBox slice_region(const OpRun& r, const Dims& in) {
  SliceBox s{in, Dims(in.size(), 0)};
  const auto axes = r.op.GetInts("axes"), starts = r.op.GetInts("starts"), ends = r.op.GetInts("ends");
  PA_CHECK(axes.size() == starts.size() && axes.size() == ends.size(), "slice: axes / starts / ends differ in length");
  for (size_t i = 0; i < axes.size(); ++i) {
    int64_t a = axes[i] < 0 ? axes[i] + (int64_t)in.size() : axes[i];
    PA_CHECK(a >= 0 && a < (int64_t)in.size(), "slice: axis %lld out of range", (long long)axes[i]);
    const int64_t n = in[(size_t)a];
    int64_t b = starts[i] < 0 ? starts[i] + n : std::min(starts[i], n);
    int64_t e = ends[i] < 0 ? ends[i] + n : std::min(ends[i], n);
    b = std::max<int64_t>(b, 0);
    e = std::max<int64_t>(e, 0);
    s.begin[(size_t)a] = b;
    s.out[(size_t)a] = std::max<int64_t>(e - b, 0);
  }
  return s;
}

void k_slice(const OpRun& r) {
  const Tensor x = r.in("Input");
  const bool dev = x.device >= 0;
  const SliceBox s = slice_region(r, x.dims);
  const Dims xs = contiguous_strides(x.dims);
  int64_t off = 0;
  for (size_t k = 0; k < xs.size(); ++k) off += s.begin[k] * xs[k];
  Tensor* o = r.out("Out");
  Tensor out;
  out.alloc(x.dtype, s.out, x.device);
  run_box(r, make_box(s.out, xs, contiguous_strides(s.out), off, 0), x.dtype, x.raw(), out.raw(), dev);
  *o = std::move(out);
}

void k_slice_grad(const OpRun& r) {
  const Tensor x = r.in("Input");
  const Tensor g = r.in("Out@GRAD");
  const SliceBox s = slice_region(r, x.dims);
  PA_CHECK(s.out == g.dims, "slice_grad: Out@GRAD does not have the slice's shape");
  Tensor dx;
  dx.alloc(g.dtype, x.dims, g.device);
  dx.lod = x.lod;
  zero_fill(r, &dx);
  const Dims xs = contiguous_strides(x.dims);
  int64_t off = 0;
  for (size_t k = 0; k < xs.size(); ++k) off += s.begin[k] * xs[k];
  run_box(r, make_box(s.out, contiguous_strides(s.out), xs, 0, off), g.dtype, g.raw(), dx.raw(), g.device >= 0);
  *r.out("Input@GRAD") = std::move(dx);
}

// ------------------------------------------------------------------ stack / unstack
int64_t norm_axis(int64_t a, int64_t rank) { return a < 0 ? a + rank : a; }

// Y[p, i, q] <-> X_i[p, q] with p over dims[:axis] and q over dims[axis:]
void stack_copy(const OpRun& r, const Tensor& part, void* whole, int64_t axis, int64_t count, int64_t i,
                bool to_whole) {
  const int64_t pre = prodd(part.dims, 0, (size_t)axis), post = prodd(part.dims, (size_t)axis);
  const Dims n{pre, post};
  const Dims sp{post, 1}, sw{count * post, 1};
  const bool dev = part.device >= 0;
  if (to_whole) run_box(r, make_box(n, sp, sw, 0, i * post), part.dtype, part.raw(), whole, dev);
  else run_box(r, make_box(n, sw, sp, i * post, 0), part.dtype, whole, const_cast<void*>(part.raw()), dev);
}

void k_stack(const OpRun& r) {
  auto xs = r.ins("X");
  PA_CHECK(!xs.empty(), "stack: no inputs");
  std::vector<Tensor> keep;
  for (Tensor* t : xs) keep.push_back(*t);
  const int64_t R = (int64_t)keep[0].dims.size();
  const int64_t axis = norm_axis(r.op.GetInt("axis", 0), R + 1);
  PA_CHECK(axis >= 0 && axis <= R, "stack: axis out of range");
  for (auto& t : keep)
    PA_CHECK(t.dims == keep[0].dims && t.dtype == keep[0].dtype && t.device == keep[0].device,
             "stack: inputs differ in shape, dtype or place");
  Dims od = keep[0].dims;
  od.insert(od.begin() + axis, (int64_t)keep.size());
  Tensor y;
  y.alloc(keep[0].dtype, od, keep[0].device);
  for (size_t i = 0; i < keep.size(); ++i)
    stack_copy(r, keep[i], y.raw(), axis, (int64_t)keep.size(), (int64_t)i, true);
  *r.out("Y") = std::move(y);
}

// pieces of `whole` along `axis` into the outputs `slot` (stack_grad's X@GRAD,
// unstack's Y); a missing output is skipped
void unstack_into(const OpRun& r, const Tensor& whole, int64_t axis, const char* slot) {
  const size_t n = r.op.Outputs(slot).size();
  PA_CHECK((int64_t)n == whole.dims[(size_t)axis], "%s: %zu outputs for an axis of %lld", r.op.type.c_str(), n,
           (long long)whole.dims[(size_t)axis]);
  Dims pd = whole.dims;
  pd.erase(pd.begin() + axis);
  for (size_t i = 0; i < n; ++i) {
    Variable* v = r.out_var(slot, i);
    if (!v) continue;
    Tensor t;
    t.alloc(whole.dtype, pd, whole.device);
    stack_copy(r, t, const_cast<void*>(whole.raw()), axis, (int64_t)n, (int64_t)i, false);
    v->kind = VK_LOD_TENSOR;
    v->tensor = std::move(t);
  }
}

void k_stack_grad(const OpRun& r) {
  const Tensor g = r.in("Y@GRAD");
  unstack_into(r, g, norm_axis(r.op.GetInt("axis", 0), (int64_t)g.dims.size()), "X@GRAD");
}

void k_unstack(const OpRun& r) {
  const Tensor x = r.in("X");
  unstack_into(r, x, norm_axis(r.op.GetInt("axis", 0), (int64_t)x.dims.size()), "Y");
}

void k_unstack_grad(const OpRun& r) {  // stack of Y@GRAD (absent pieces are zeros)
  const Tensor x = r.in("X");
  const int64_t axis = norm_axis(r.op.GetInt("axis", 0), (int64_t)x.dims.size());
  Tensor dx;
  dx.alloc(x.dtype, x.dims, x.device);
  const size_t n = r.op.Inputs("Y@GRAD").size();
  bool all = n == (size_t)x.dims[(size_t)axis];
  for (size_t i = 0; i < n && all; ++i) all = r.in_opt("Y@GRAD", i) != nullptr;
  if (!all) zero_fill(r, &dx);
  for (size_t i = 0; i < n; ++i)
    if (Tensor* gi = r.in_opt("Y@GRAD", i)) {
      const Tensor part = *gi;
      stack_copy(r, part, dx.raw(), axis, x.dims[(size_t)axis], (int64_t)i, true);
    }
  *r.out("X@GRAD") = std::move(dx);
}

// ------------------------------------------------------------------ transpose_grad
void k_transpose_grad(const OpRun& r) {
  const Tensor g = r.in("Out@GRAD");
  const auto perm = r.op.GetInts("axis");
  PA_CHECK(perm.size() == g.dims.size(), "transpose_grad: axis does not match Out@GRAD's rank");
  // dX[perm[k] index] = dOut[k index]: read dOut contiguously, write dX with permuted strides
  Dims xd(g.dims.size());
  for (size_t k = 0; k < perm.size(); ++k) xd[(size_t)perm[k]] = g.dims[k];
  const Dims xs = contiguous_strides(xd);
  Dims ds(perm.size());
  for (size_t k = 0; k < perm.size(); ++k) ds[k] = xs[(size_t)perm[k]];
  Tensor dx;
  dx.alloc(g.dtype, xd, g.device);
  run_box(r, make_box(g.dims, contiguous_strides(g.dims), ds, 0, 0), g.dtype, g.raw(), dx.raw(), g.device >= 0);
  *r.out("X@GRAD") = std::move(dx);
}

// ------------------------------------------------------------------ expand (tile)
void k_expand(const OpRun& r) {
  const Tensor x = r.in("X");
  const auto reps = r.op.GetInts("expand_times");
  PA_CHECK(reps.size() == x.dims.size(), "expand: expand_times must match X's rank");
  // out viewed as [reps_0, d_0, reps_1, d_1, ...]; the repeat dims read with stride 0
  Dims n, ss, od;
  const Dims xs = contiguous_strides(x.dims);
  for (size_t k = 0; k < x.dims.size(); ++k) {
    n.push_back(reps[k]);
    ss.push_back(0);
    n.push_back(x.dims[k]);
    ss.push_back(xs[k]);
    od.push_back(reps[k] * x.dims[k]);
  }
  Tensor o;
  o.alloc(x.dtype, od, x.device);
  run_box(r, make_box(n, ss, contiguous_strides(n), 0, 0), x.dtype, x.raw(), o.raw(), x.device >= 0);
  *r.out("Out") = std::move(o);
}

// expand_grad: dX[c] = sum over every tile t of dOut[t * d + c]
struct TileSum {
  int R;
  int64_t d[kMaxBox], reps[kMaxBox], gs[kMaxBox];
  int64_t n, ntiles;
};

__host__ __device__ __forceinline__ float tile_sum_one(const TileSum& a, const float* __restrict__ g, int64_t i) {
  int64_t c[kMaxBox];
  for (int k = a.R - 1; k >= 0; --k) {
    c[k] = i % a.d[k];
    i /= a.d[k];
  }
  float acc = 0.f;
  for (int64_t t = 0; t < a.ntiles; ++t) {
    int64_t rem = t, off = 0;
    for (int k = a.R - 1; k >= 0; --k) {
      const int64_t rk = rem % a.reps[k];
      rem /= a.reps[k];
      off += (rk * a.d[k] + c[k]) * a.gs[k];
    }
    acc += g[off];
  }
  return acc;
}

__global__ void tile_sum_kernel(TileSum a, const float* __restrict__ g, float* __restrict__ dx) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x)
    dx[i] = tile_sum_one(a, g, i);
}

void k_expand_grad(const OpRun& r) {
  const Tensor x = r.in("X");
  const Tensor g = r.in("Out@GRAD");
  const auto reps = r.op.GetInts("expand_times");
  if (g.dtype != DT::FP32) throw Decline{};
  PA_CHECK(reps.size() == x.dims.size() && x.dims.size() <= (size_t)kMaxBox, "expand_grad: bad expand_times");
  TileSum a{};
  a.R = (int)x.dims.size();
  a.n = x.numel();
  a.ntiles = 1;
  const Dims gs = contiguous_strides(g.dims);
  for (int k = 0; k < a.R; ++k) {
    a.d[k] = x.dims[(size_t)k];
    a.reps[k] = reps[(size_t)k];
    a.gs[k] = gs[(size_t)k];
    a.ntiles *= reps[(size_t)k];
    PA_CHECK(g.dims[(size_t)k] == a.d[k] * a.reps[k], "expand_grad: Out@GRAD shape mismatch");
  }
  Tensor dx;
  dx.alloc(DT::FP32, x.dims, g.device);
  dx.lod = x.lod;
  if (a.n) {
    if (g.device >= 0) {
      hipLaunchKernelGGL(tile_sum_kernel, dim3(dev_grid(a.n)), dim3(256), 0, dev_stream(r), a, g.data<float>(),
                         dx.data<float>());
      PA_HIPCHK(hipGetLastError());
    } else {
      const float* gp = g.data<float>();
      float* dp = dx.data<float>();
      parallel_for(a.n, 1024, [&](int64_t b, int64_t e) {
        for (int64_t i = b; i < e; ++i) dp[i] = tile_sum_one(a, gp, i);
      });
    }
  }
  *r.out("X@GRAD") = std::move(dx);
}

// ------------------------------------------------------------------ view-only grads
// squeeze / unsqueeze / flatten gradients: Out@GRAD's buffer with X's dims
void k_view_grad(const OpRun& r) {
  Tensor g = r.in("Out@GRAD");
  Dims d;
  if (Tensor* x = r.in_opt("X")) d = x->dims;
  else if (Tensor* xs = r.in_opt("XShape")) d.assign(xs->dims.begin() + 1, xs->dims.end());
  else fail("%s: needs X or XShape", r.op.type.c_str());
  PA_CHECK(prodd(d) == g.numel(), "%s: Out@GRAD holds %lld elements, X %lld", r.op.type.c_str(),
           (long long)g.numel(), (long long)prodd(d));
  Tensor* dx = r.out("X@GRAD");
  *dx = g;
  dx->dims = d;
  if (Tensor* x = r.in_opt("X")) dx->lod = x->lod;
}

}  // namespace

#define PA_ANY_KERNEL(name, fn) \
  PA_HOST_KERNEL(name, fn);     \
  PA_DEVICE_KERNEL(name, fn)
PA_ANY_KERNEL(slice, k_slice);
PA_ANY_KERNEL(slice_grad, k_slice_grad);
PA_ANY_KERNEL(stack, k_stack);
PA_ANY_KERNEL(stack_grad, k_stack_grad);
PA_ANY_KERNEL(unstack, k_unstack);
PA_ANY_KERNEL(unstack_grad, k_unstack_grad);
PA_ANY_KERNEL(transpose_grad, k_transpose_grad);
PA_ANY_KERNEL(transpose2_grad, k_transpose_grad);
PA_ANY_KERNEL(expand, k_expand);
PA_ANY_KERNEL(expand_grad, k_expand_grad);
PA_ANY_KERNEL(squeeze_grad, k_view_grad);
PA_ANY_KERNEL(squeeze2_grad, k_view_grad);
PA_ANY_KERNEL(unsqueeze_grad, k_view_grad);
PA_ANY_KERNEL(unsqueeze2_grad, k_view_grad);
PA_ANY_KERNEL(flatten_grad, k_view_grad);
PA_ANY_KERNEL(flatten2_grad, k_view_grad);
#undef PA_ANY_KERNEL

void link_tensor_kernels() {}

}  // namespace pa
