// Place-agnostic kernels of the LoD row-map sequence operators and their gradients:
// sequence_slice, sequence_pad, sequence_unpad, sequence_erase, sequence_mask,
// sequence_enumerate, sequence_conv.
//
// Semantics: reference operators/sequence_{slice,pad,unpad,erase,mask,enumerate,
// conv}_op.h (sequence_conv: math/context_project.h); the Python kernels of
// operators/sequence_ops.py compute the same functions.  Each op is a row map built
// on the host from LoD metadata (and, where the reference reads them on the host
// too, the small Offset / Length / id inputs); the rows themselves move on the
// tensor's own place -- memcpy on the host, the gather / scatter kernels of
// ops_gpu.hip on HBM -- and the sequence_conv product runs on sgemm / pa_sgemm.
// Gradients scatter(-add) the output gradient rows back along the same map.
#include <string.h>

#include <algorithm>
#include <vector>

#include "framework.h"

namespace pa {

void device_sgemm(void* stream, bool ta, bool tb, int64_t M, int64_t N, int64_t K, float alpha, const float* A,
                  int64_t lda, const float* B, int64_t ldb, float beta, float* C, int64_t ldc);

namespace {

using Dims = std::vector<int64_t>;

int64_t rows_of(const Tensor& t) { return t.dims.empty() ? 0 : t.dims[0]; }
int64_t row_bytes(const Tensor& t) {
  const int64_t n = rows_of(t);
  return n ? (int64_t)t.nbytes() / n : 0;
}

Tensor host_view(const OpRun& r, const Tensor& t) {
  if (t.device < 0) return t;
  Tensor h = t.to(-1, r.ctx.stream);
  device_stream_sync(r.ctx.stream);
  return h;
}

std::vector<int64_t> ints_of(const OpRun& r, const Tensor& t) {
  const Tensor h = host_view(r, t);
  std::vector<int64_t> v((size_t)h.numel());
  switch (h.dtype) {
    case DT::INT64: memcpy(v.data(), h.raw(), v.size() * 8); break;
    case DT::INT32: for (size_t i = 0; i < v.size(); ++i) v[i] = h.data<int32_t>()[i]; break;
    case DT::FP32: for (size_t i = 0; i < v.size(); ++i) v[i] = (int64_t)h.data<float>()[i]; break;
    default: fail("%s: integer input expected, got %s", r.op.type.c_str(), dt_name(h.dtype));
  }
  return v;
}

const std::vector<size_t>& last_level(const Tensor& x, const char* op) {
  PA_CHECK(!x.lod.empty(), "%s: the input has no LoD", op);
  return x.lod.back();
}

// dst row i <- src row rows[i]
void gather(const OpRun& r, const Tensor& src, const std::vector<int64_t>& rows, void* dst) {
  const int64_t rb = row_bytes(src);
  if (src.device < 0) {
    for (size_t i = 0; i < rows.size(); ++i)
      memcpy((char*)dst + i * rb, (const char*)src.raw() + rows[i] * rb, (size_t)rb);
  } else {
    device_gather_rows(r, src.raw(), rb, rows, dst);
  }
}

// dst row rows[i] (+)= src row i
void scatter(const OpRun& r, const Tensor& src, const std::vector<int64_t>& rows, void* dst, bool add) {
  const int64_t rb = row_bytes(src);
  if (src.device < 0) {
    if (add) {
      const int64_t w = rb / 4;
      for (size_t i = 0; i < rows.size(); ++i)
        for (int64_t j = 0; j < w; ++j) ((float*)dst)[rows[i] * w + j] += src.data<float>()[i * w + j];
    } else {
      for (size_t i = 0; i < rows.size(); ++i)
        memcpy((char*)dst + rows[i] * rb, (const char*)src.raw() + i * rb, (size_t)rb);
    }
  } else {
    device_scatter_rows(r, src.raw(), rb, rows, dst, add);
  }
}

void zero(const OpRun& r, Tensor* t) {
  if (t->device < 0) memset(t->raw(), 0, t->nbytes());
  else device_fill(r.ctx.stream, t->raw(), t->dtype, t->numel(), 0.0);
}

// an output with a host vector's values, on `dev`
template <class T>
void put(const OpRun& r, Tensor* o, DT dt, const Dims& dims, const std::vector<T>& v, int dev) {
  o->alloc(dt, dims, dev);
  if (v.empty()) return;
  if (dev < 0) {
    memcpy(o->raw(), v.data(), v.size() * sizeof(T));
  } else {
    device_copy(o->raw(), dev, v.data(), -1, v.size() * sizeof(T), r.ctx.stream);
    device_stream_sync(r.ctx.stream);  // `v` dies with the op
  }
}

// ---------------------------------------------------------------- sequence_slice
std::vector<int64_t> slice_rows(const OpRun& r, const Tensor& x, std::vector<size_t>* new_off) {
  const auto& off = last_level(x, "sequence_slice");
  const std::vector<int64_t> so = ints_of(r, r.in("Offset")), sl = ints_of(r, r.in("Length"));
  const size_t n = off.size() - 1;
  PA_CHECK(so.size() == n && sl.size() == n, "sequence_slice: one Offset / Length per sequence");
  std::vector<int64_t> rows;
  new_off->assign(1, 0);
  for (size_t i = 0; i < n; ++i) {
    PA_CHECK(so[i] >= 0 && sl[i] >= 0 && (int64_t)off[i] + so[i] + sl[i] <= (int64_t)off[i + 1],
             "sequence_slice: slice %zu out of its sequence", i);
    for (int64_t t = 0; t < sl[i]; ++t) rows.push_back((int64_t)off[i] + so[i] + t);
    new_off->push_back(rows.size());
  }
  return rows;
}

void k_sequence_slice(const OpRun& r) {
  Tensor& x = r.in("X");
  std::vector<size_t> no;
  const auto rows = slice_rows(r, x, &no);
  Dims d = x.dims;
  d[0] = (int64_t)rows.size();
  Tensor* o = r.out("Out");
  const Tensor xs = x;
  o->alloc(xs.dtype, d, xs.device);
  gather(r, xs, rows, o->raw());
  LoD lod(xs.lod.begin(), xs.lod.end() - 1);
  lod.push_back(no);
  o->lod = lod;
}

void k_sequence_slice_grad(const OpRun& r) {
  Tensor& x = r.in("X");
  Tensor& g = r.in("Out@GRAD");
  std::vector<size_t> no;
  const auto rows = slice_rows(r, x, &no);
  Tensor* dx = r.out("X@GRAD");
  dx->alloc(g.dtype, x.dims, g.device);
  zero(r, dx);
  scatter(r, g, rows, dx->raw(), false);
  dx->lod = x.lod;
}

// ---------------------------------------------------------------- sequence_pad / unpad
void k_sequence_pad(const OpRun& r) {
  Tensor& x = r.in("X");
  Tensor& pv = r.in("PadValue");
  const auto& off = last_level(x, "sequence_pad");
  const int64_t n = (int64_t)off.size() - 1;
  std::vector<int64_t> lens((size_t)n);
  int64_t L = 0;
  for (int64_t i = 0; i < n; ++i) L = std::max(L, lens[(size_t)i] = (int64_t)(off[(size_t)i + 1] - off[(size_t)i]));
  const int64_t pl = r.op.GetInt("padded_length", -1);
  if (pl != -1) {
    PA_CHECK(pl >= L, "sequence_pad: padded_length %lld < longest sequence %lld", (long long)pl, (long long)L);
    L = pl;
  }
  Dims d{n, L};
  d.insert(d.end(), x.dims.begin() + 1, x.dims.end());
  const Tensor xs = x;
  Tensor* o = r.out("Out");
  o->alloc(xs.dtype, d, xs.device);
  const int64_t w = rows_of(xs) ? xs.numel() / rows_of(xs) : 1;
  // fill every slot with the pad value (one scalar, or one row broadcast)
  std::vector<int64_t> all((size_t)(n * L), 0);
  if (pv.numel() == 1) {
    const Tensor ph = host_view(r, pv);
    PA_CHECK(ph.dtype == xs.dtype || ph.dtype == DT::FP32, "sequence_pad: PadValue dtype");
    const double v = ph.dtype == DT::FP32 ? ph.data<float>()[0] : ph.dtype == DT::INT64 ? (double)ph.data<int64_t>()[0]
                                                                                         : 0.0;
    if (xs.device < 0) {
      if (xs.dtype == DT::FP32) std::fill_n(o->data<float>(), o->numel(), (float)v);
      else if (xs.dtype == DT::INT64) std::fill_n(o->data<int64_t>(), o->numel(), (int64_t)v);
      else fail("sequence_pad: dtype %s", dt_name(xs.dtype));
    } else {
      device_fill(r.ctx.stream, o->raw(), xs.dtype, o->numel(), v);
    }
  } else {
    PA_CHECK(pv.numel() == w && pv.dtype == xs.dtype, "sequence_pad: PadValue must be a scalar or one row");
    Tensor pr = pv;
    pr.dims = {1, w};
    if (pr.device != xs.device) pr = pr.to(xs.device, r.ctx.stream);
    gather(r, pr, all, o->raw());
  }
  std::vector<int64_t> dst;
  for (int64_t i = 0; i < n; ++i)
    for (int64_t t = 0; t < lens[(size_t)i]; ++t) dst.push_back(i * L + t);
  scatter(r, xs, dst, o->raw(), false);
  if (Tensor* lt = r.out("Length")) put(r, lt, DT::INT64, {n}, lens, xs.device);
}

void k_sequence_pad_grad(const OpRun& r) {
  Tensor& x = r.in("X");
  Tensor& g = r.in("Out@GRAD");
  const auto& off = last_level(x, "sequence_pad_grad");
  const int64_t n = (int64_t)off.size() - 1, L = g.dims.size() > 1 ? g.dims[1] : 0;
  std::vector<int64_t> src;
  for (int64_t i = 0; i < n; ++i)
    for (int64_t t = 0; t < (int64_t)(off[(size_t)i + 1] - off[(size_t)i]); ++t) src.push_back(i * L + t);
  Tensor gr = g;
  gr.dims = x.dims;
  gr.dims[0] = n * L;
  Tensor* dx = r.out("X@GRAD");
  dx->alloc(g.dtype, x.dims, g.device);
  gather(r, gr, src, dx->raw());
  dx->lod = x.lod;
}

std::vector<int64_t> unpad_rows(const OpRun& r, const Tensor& x, std::vector<size_t>* off) {
  const std::vector<int64_t> lens = ints_of(r, r.in("Length"));
  const int64_t L = x.dims.size() > 1 ? x.dims[1] : 0;
  std::vector<int64_t> rows;
  off->assign(1, 0);
  for (size_t i = 0; i < lens.size(); ++i) {
    PA_CHECK(lens[i] >= 0 && lens[i] <= L, "sequence_unpad: Length %lld out of [0, %lld]", (long long)lens[i],
             (long long)L);
    for (int64_t t = 0; t < lens[i]; ++t) rows.push_back((int64_t)i * L + t);
    off->push_back(rows.size());
  }
  return rows;
}

void k_sequence_unpad(const OpRun& r) {
  Tensor& x = r.in("X");
  std::vector<size_t> off;
  const auto rows = unpad_rows(r, x, &off);
  Tensor xr = x;
  xr.dims.erase(xr.dims.begin());
  xr.dims[0] = x.dims[0] * x.dims[1];
  Dims d = xr.dims;
  d[0] = (int64_t)rows.size();
  Tensor* o = r.out("Out");
  o->alloc(xr.dtype, d, xr.device);
  gather(r, xr, rows, o->raw());
  o->lod = {off};
}

void k_sequence_unpad_grad(const OpRun& r) {
  Tensor& x = r.in("X");
  Tensor& g = r.in("Out@GRAD");
  std::vector<size_t> off;
  const auto rows = unpad_rows(r, x, &off);
  Tensor* dx = r.out("X@GRAD");
  dx->alloc(g.dtype, x.dims, g.device);
  zero(r, dx);
  scatter(r, g, rows, dx->raw(), false);
}

// ---------------------------------------------------------------- id-valued ops (no grad)
void k_sequence_erase(const OpRun& r) {
  Tensor& x = r.in("X");
  const auto& off = last_level(x, "sequence_erase");
  const std::vector<int64_t> v = ints_of(r, x);
  const std::vector<int64_t> toks = r.op.GetInts("tokens");
  std::vector<int64_t> rows;
  std::vector<size_t> no{0};
  for (size_t s = 0; s + 1 < off.size(); ++s) {
    for (size_t i = off[s]; i < off[s + 1]; ++i)
      if (std::find(toks.begin(), toks.end(), v[i]) == toks.end()) rows.push_back((int64_t)i);
    no.push_back(rows.size());
  }
  const Tensor xs = x;
  Dims d = xs.dims;
  d[0] = (int64_t)rows.size();
  Tensor* o = r.out("Out");
  o->alloc(xs.dtype, d, xs.device);
  gather(r, xs, rows, o->raw());
  o->lod = {no};
}

void k_sequence_mask(const OpRun& r) {
  Tensor& x = r.in("X");
  const std::vector<int64_t> v = ints_of(r, x);
  int64_t ml = r.op.GetInt("maxlen", -1);
  if (ml < 0) ml = v.empty() ? 0 : *std::max_element(v.begin(), v.end());
  const DT dt = (DT)r.op.GetInt("out_dtype", (int)DT::INT64);
  Dims d = x.dims;
  d.push_back(ml);
  const size_t n = v.size() * (size_t)ml;
  Tensor* o = r.out("Y");
  switch (dt) {
    case DT::INT64: {
      std::vector<int64_t> m(n);
      for (size_t i = 0; i < v.size(); ++i)
        for (int64_t j = 0; j < ml; ++j) m[i * ml + j] = j < v[i];
      put(r, o, dt, d, m, x.device);
      break;
    }
    case DT::INT32: {
      std::vector<int32_t> m(n);
      for (size_t i = 0; i < v.size(); ++i)
        for (int64_t j = 0; j < ml; ++j) m[i * ml + j] = j < v[i];
      put(r, o, dt, d, m, x.device);
      break;
    }
    case DT::FP32: {
      std::vector<float> m(n);
      for (size_t i = 0; i < v.size(); ++i)
        for (int64_t j = 0; j < ml; ++j) m[i * ml + j] = j < v[i] ? 1.f : 0.f;
      put(r, o, dt, d, m, x.device);
      break;
    }
    case DT::BOOL: case DT::UINT8: {
      std::vector<uint8_t> m(n);
      for (size_t i = 0; i < v.size(); ++i)
        for (int64_t j = 0; j < ml; ++j) m[i * ml + j] = j < v[i];
      put(r, o, dt, d, m, x.device);
      break;
    }
    default: fail("sequence_mask: out_dtype %s", dt_name(dt));
  }
}

void k_sequence_enumerate(const OpRun& r) {
  Tensor& x = r.in("X");
  const auto& off = last_level(x, "sequence_enumerate");
  const std::vector<int64_t> v = ints_of(r, x);
  const int64_t w = r.op.GetInt("win_size", 2), pv = r.op.GetInt("pad_value", 0);
  std::vector<int64_t> o(v.size() * (size_t)w, pv);
  for (size_t s = 0; s + 1 < off.size(); ++s)
    for (size_t i = off[s]; i < off[s + 1]; ++i)
      for (int64_t k = 0; k < w; ++k)
        if (i + (size_t)k < off[s + 1]) o[i * (size_t)w + (size_t)k] = v[i + (size_t)k];
  Tensor* out = r.out("Out");
  if (x.dtype == DT::INT64) {
    put(r, out, DT::INT64, {(int64_t)v.size(), w}, o, x.device);
  } else {
    std::vector<int32_t> o32(o.begin(), o.end());
    put(r, out, DT::INT32, {(int64_t)v.size(), w}, o32, x.device);
  }
  out->lod = x.lod;
}

// ---------------------------------------------------------------- sequence_conv
// context projection row map over the table [X; PaddingData; zero row]
std::vector<int64_t> context_rows(const std::vector<size_t>& off, int64_t T, int64_t cl, int64_t cs, int64_t up_pad,
                                  bool has_pad, int64_t zero_row) {
  std::vector<int64_t> idx((size_t)(T * cl));
  for (size_t sq = 0; sq + 1 < off.size(); ++sq) {
    const int64_t s = (int64_t)off[sq], e = (int64_t)off[sq + 1];
    for (int64_t row = s; row < e; ++row)
      for (int64_t k = 0; k < cl; ++k) {
        const int64_t src = row + cs + k;
        int64_t v = (src >= s && src < e) ? src : zero_row;
        if (has_pad && src < s) v = T + up_pad + (src - s);
        if (has_pad && src >= e) v = T + up_pad + (src - e);
        idx[(size_t)(row * cl + k)] = v;
      }
  }
  return idx;
}

struct ConvCtx {
  int64_t T, Dm, cl, cs, up_pad, npad;
  bool has_pad;
  std::vector<int64_t> idx;
};

ConvCtx conv_ctx(const OpRun& r, const Tensor& x) {
  ConvCtx c;
  c.T = x.dims[0];
  c.Dm = x.dims.size() > 1 ? x.dims[1] : 1;
  c.cl = r.op.GetInt("contextLength", 3);
  c.cs = r.op.GetInt("contextStart", 0);
  PA_CHECK(r.op.GetInt("contextStride", 1) == 1, "sequence_conv: contextStride must be 1");
  c.up_pad = std::max<int64_t>(0, -c.cs);
  Tensor* pad = r.in_opt("PaddingData");
  c.has_pad = r.op.GetBool("paddingTrainable", false) && pad != nullptr;
  c.npad = c.has_pad ? pad->dims[0] : 0;
  c.idx = context_rows(last_level(x, "sequence_conv"), c.T, c.cl, c.cs, c.up_pad, c.has_pad, c.T + c.npad);
  return c;
}

// table [X; PaddingData; zero row] on x's place
Tensor conv_table(const OpRun& r, const Tensor& x, const ConvCtx& c) {
  Tensor tab;
  tab.alloc(DT::FP32, {c.T + c.npad + 1, c.Dm}, x.device);
  const size_t rb = (size_t)c.Dm * 4;
  if (x.device < 0) {
    memcpy(tab.raw(), x.raw(), c.T * rb);
    if (c.has_pad) memcpy((char*)tab.raw() + c.T * rb, r.in("PaddingData").raw(), c.npad * rb);
    memset((char*)tab.raw() + (c.T + c.npad) * rb, 0, rb);
  } else {
    device_copy(tab.raw(), x.device, x.raw(), x.device, c.T * rb, r.ctx.stream);
    if (c.has_pad)
      device_copy((char*)tab.raw() + c.T * rb, x.device, r.in("PaddingData").raw(), x.device, c.npad * rb,
                  r.ctx.stream);
    device_fill(r.ctx.stream, (char*)tab.raw() + (c.T + c.npad) * rb, DT::FP32, c.Dm, 0.0);
  }
  return tab;
}

void mm(const OpRun& r, int dev, bool ta, bool tb, int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
        const float* B, int64_t ldb, float beta, float* C, int64_t ldc) {
  if (dev < 0) sgemm(ta, tb, M, N, K, 1.f, A, lda, B, ldb, beta, C, ldc);
  else device_sgemm(r.ctx.stream, ta, tb, M, N, K, 1.f, A, lda, B, ldb, beta, C, ldc);
}

void k_sequence_conv(const OpRun& r) {
  Tensor& x = r.in("X");
  Tensor& w = r.in("Filter");
  if (x.dtype != DT::FP32 || w.dtype != DT::FP32 || w.device != x.device) throw Decline{};
  const ConvCtx c = conv_ctx(r, x);
  const Tensor tab = conv_table(r, x, c);
  Tensor cols;
  cols.alloc(DT::FP32, {c.T * c.cl, c.Dm}, x.device);
  gather(r, tab, c.idx, cols.raw());
  const int64_t N = w.dims[1];
  Tensor* o = r.out("Out");
  const LoD lod = x.lod;
  float* op = o->alloc<float>({c.T, N}, x.device);
  mm(r, x.device, false, false, c.T, N, c.cl * c.Dm, cols.data<float>(), c.cl * c.Dm, w.data<float>(), N, 0.f, op, N);
  o->lod = lod;
  if (x.device >= 0) device_stream_sync(r.ctx.stream);  // the local table / cols die here
}

void k_sequence_conv_grad(const OpRun& r) {
  Tensor& x = r.in("X");
  Tensor& w = r.in("Filter");
  Tensor& g = r.in("Out@GRAD");
  if (x.dtype != DT::FP32 || g.dtype != DT::FP32) throw Decline{};
  const ConvCtx c = conv_ctx(r, x);
  const int64_t N = w.dims[1], K = c.cl * c.Dm;
  const int dev = x.device;
  if (Tensor* dw = r.out("Filter@GRAD")) {
    const Tensor tab = conv_table(r, x, c);
    Tensor cols;
    cols.alloc(DT::FP32, {c.T * c.cl, c.Dm}, dev);
    gather(r, tab, c.idx, cols.raw());
    mm(r, dev, true, false, K, N, c.T, cols.data<float>(), K, g.data<float>(), N, 0.f,
       dw->alloc<float>(w.dims, dev), N);
    if (dev >= 0) device_stream_sync(r.ctx.stream);
  }
  Tensor* dx = r.out("X@GRAD");
  Tensor* dpad = c.has_pad ? r.out("PaddingData@GRAD") : nullptr;
  if (dx || dpad) {
    // dcols = dOut W^T, scattered (added) back into [dX; dPad; sink]
    Tensor dcols, dtab;
    dcols.alloc(DT::FP32, {c.T * c.cl, c.Dm}, dev);
    mm(r, dev, false, true, c.T, K, N, g.data<float>(), N, w.data<float>(), N, 0.f, dcols.data<float>(), K);
    dtab.alloc(DT::FP32, {c.T + c.npad + 1, c.Dm}, dev);
    zero(r, &dtab);
    scatter(r, dcols, c.idx, dtab.raw(), true);
    const size_t rb = (size_t)c.Dm * 4;
    if (dx) {
      dx->alloc(DT::FP32, x.dims, dev);
      if (dev < 0) memcpy(dx->raw(), dtab.raw(), c.T * rb);
      else device_copy(dx->raw(), dev, dtab.raw(), dev, c.T * rb, r.ctx.stream);
      dx->lod = x.lod;
    }
    if (dpad) {
      Tensor& pd = r.in("PaddingData");
      dpad->alloc(DT::FP32, pd.dims, dev);
      if (dev < 0) memcpy(dpad->raw(), (char*)dtab.raw() + c.T * rb, c.npad * rb);
      else device_copy(dpad->raw(), dev, (char*)dtab.raw() + c.T * rb, dev, c.npad * rb, r.ctx.stream);
    }
    if (dev >= 0) device_stream_sync(r.ctx.stream);
  }
}

// cast_grad (cast_op.cc CastOpGradMaker): X@GRAD = cast(Out@GRAD, in_dtype) -- the
// registered cast kernel of the same place, run on a re-wired op description
template <bool DEVICE>
void k_cast_grad(const OpRun& r) {
  OpDesc op;
  op.type = "cast";
  op.inputs = {{"X", {r.op.Input("Out@GRAD")}}};
  op.outputs = {{"Out", {r.op.Output("X@GRAD")}}};
  Attr a;
  a.name = "out_dtype";
  a.type = A_INT;
  a.i = r.op.GetInt("in_dtype", (int)DT::FP32);
  op.attrs["out_dtype"] = a;
  Attr b = a;
  b.name = "in_dtype";
  b.i = r.op.GetInt("out_dtype", (int)DT::FP32);
  op.attrs["in_dtype"] = b;
  const Kernel* k = find_kernel("cast", DEVICE);
  if (!k) throw Decline{};
  (*k)(OpRun{op, r.scope, r.ctx});
}

}  // namespace

PA_HOST_KERNEL(cast_grad, k_cast_grad<false>);
PA_DEVICE_KERNEL(cast_grad, k_cast_grad<true>);

#define PA_ANY_KERNEL(name, fn) \
  PA_HOST_KERNEL(name, fn);     \
  PA_DEVICE_KERNEL(name, fn)
PA_ANY_KERNEL(sequence_slice, k_sequence_slice);
PA_ANY_KERNEL(sequence_slice_grad, k_sequence_slice_grad);
PA_ANY_KERNEL(sequence_pad, k_sequence_pad);
PA_ANY_KERNEL(sequence_pad_grad, k_sequence_pad_grad);
PA_ANY_KERNEL(sequence_unpad, k_sequence_unpad);
PA_ANY_KERNEL(sequence_unpad_grad, k_sequence_unpad_grad);
PA_ANY_KERNEL(sequence_erase, k_sequence_erase);
PA_ANY_KERNEL(sequence_mask, k_sequence_mask);
PA_ANY_KERNEL(sequence_enumerate, k_sequence_enumerate);
PA_ANY_KERNEL(sequence_conv, k_sequence_conv);
PA_ANY_KERNEL(sequence_conv_grad, k_sequence_conv_grad);
#undef PA_ANY_KERNEL

void link_seq_kernels() {}

}  // namespace pa
