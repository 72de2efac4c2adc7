// Place-agnostic kernels of the native executor for the non-tensor variable kinds:
// LoDTensorArray (tensor_array_read_write_op.cc, lod_tensor_to_array_op.cc,
// array_to_lod_tensor_op.cc, shrink_rnn_memory_op.cc), LoDRankTable
// (lod_rank_table_op.cc, max_sequence_len_op.cc, reorder_lod_tensor_by_rank_op.cc)
// and SelectedRows (lookup_table_op.cu:118 sparse W@GRAD, sum_op.h, sgd_op.h,
// adam_op.h SparseAdamFunctor), plus the gradients DynamicRNN training needs.
//
// Every kernel here is registered for the host AND the device: the row maps are
// computed on the host from LoD / rank-table metadata, and the rows themselves move
// on the tensor's own place (memcpy on the host, the gather / scatter kernels of
// ops_gpu.hip on HBM) -- a DynamicRNN step on a HIP place never round-trips through
// host memory.  Loop indices (`I`) are the host-pinned counters of the reference
// (fill_constant force_cpu); a device-resident index is read back once.
//
// Semantics match the Python op library (operators/io_ops.py,
// operators/control_flow_grad.py) so the two engines train along one trajectory.
#include <string.h>

#include <algorithm>
#include <cmath>
#include <map>

#include "framework.h"

namespace pa {
namespace {

using Dims = std::vector<int64_t>;

int64_t row_count(const Tensor& t) { return t.dims.empty() ? 0 : t.dims[0]; }
int64_t row_bytes(const Tensor& t) {
  const int64_t n = row_count(t);
  return n ? (int64_t)t.nbytes() / n : 0;
}

int64_t read_index(const OpRun& r, const char* slot = "I") {
  Tensor& t = r.in(slot);
  PA_CHECK(t.numel() >= 1, "%s: index %s is empty", r.op.type.c_str(), slot);
  Tensor h = t.device >= 0 ? t.to(-1, r.ctx.stream) : t;
  if (t.device >= 0) device_stream_sync(r.ctx.stream);
  switch (h.dtype) {
    case DT::INT64: return h.data<int64_t>()[0];
    case DT::INT32: return h.data<int32_t>()[0];
    case DT::FP32: return (int64_t)h.data<float>()[0];
    case DT::FP64: return (int64_t)h.data<double>()[0];
    default: fail("%s: index dtype %s", r.op.type.c_str(), dt_name(h.dtype));
  }
}

// a private copy of `src` on its own place
Tensor clone(const OpRun& r, const Tensor& src) {
  Tensor t;
  t.alloc(src.dtype, src.dims, src.device);
  t.lod = src.lod;
  if (src.nbytes()) device_copy(t.raw(), src.device, src.raw(), src.device, src.nbytes(), r.ctx.stream);
  return t;
}

Tensor zeros_like(const OpRun& r, const Tensor& src) {
  Tensor t;
  t.alloc(src.dtype, src.dims, src.device);
  t.lod = src.lod;
  if (t.device >= 0) device_fill(r.ctx.stream, t.raw(), t.dtype, t.numel(), 0.0);
  else if (t.nbytes()) memset(t.raw(), 0, t.nbytes());
  return t;
}

// dst rows = src rows[rows[i]] (dst allocated by the caller with rows.size() rows)
void gather(const OpRun& r, const Tensor& src, const std::vector<int64_t>& rows, Tensor& dst) {
  const int64_t rb = row_bytes(src);
  for (int64_t v : rows) PA_CHECK(v >= 0 && v < row_count(src), "%s: row %lld out of range", r.op.type.c_str(), (long long)v);
  if (src.device >= 0) {
    device_gather_rows(r, src.raw(), rb, rows, dst.raw());
    return;
  }
  for (size_t i = 0; i < rows.size(); ++i)
    memcpy((char*)dst.raw() + i * rb, (const char*)src.raw() + rows[i] * rb, (size_t)rb);
}

// dst rows[rows[i]] = (or += for fp32 `add`) src row i
void scatter(const OpRun& r, const Tensor& src, const std::vector<int64_t>& rows, Tensor& dst, bool add) {
  const int64_t rb = row_bytes(dst);
  PA_CHECK(rows.empty() || row_bytes(src) == rb, "%s: row widths differ", r.op.type.c_str());
  for (int64_t v : rows) PA_CHECK(v >= 0 && v < row_count(dst), "%s: row %lld out of range", r.op.type.c_str(), (long long)v);
  if (dst.device >= 0) {
    device_scatter_rows(r, src.raw(), rb, rows, dst.raw(), add);
    return;
  }
  if (add) {
    PA_CHECK(dst.dtype == DT::FP32 && src.dtype == DT::FP32, "%s: accumulation needs float32", r.op.type.c_str());
    const int64_t w = rb / 4;
    for (size_t i = 0; i < rows.size(); ++i) {
      float* d = dst.data<float>() + rows[i] * w;
      const float* s = src.data<float>() + i * w;
      for (int64_t j = 0; j < w; ++j) d[j] += s[j];
    }
    return;
  }
  for (size_t i = 0; i < rows.size(); ++i)
    memcpy((char*)dst.raw() + rows[i] * rb, (const char*)src.raw() + i * rb, (size_t)rb);
}

Tensor& set_out(const OpRun& r, const char* slot, Tensor t) {
  Variable* v = r.out_var(slot);
  PA_CHECK(v != nullptr, "%s: output %s missing", r.op.type.c_str(), slot);
  v->kind = VK_LOD_TENSOR;
  v->tensor = std::move(t);
  return v->tensor;
}

Tensor host_scalar_i64(int64_t v) {
  Tensor t;
  t.alloc<int64_t>({1}, -1)[0] = v;
  return t;
}

const Variable& rank_table(const OpRun& r) {
  Variable* v = r.in_var("RankTable");
  PA_CHECK(v->kind == VK_LOD_RANK_TABLE, "%s: RankTable is not a rank table", r.op.type.c_str());
  return *v;
}

// the finest LoD level of x, or one sequence per row
std::vector<size_t> last_level(const Tensor& x) {
  if (!x.lod.empty()) return x.lod.back();
  std::vector<size_t> l((size_t)row_count(x) + 1);
  for (size_t i = 0; i < l.size(); ++i) l[i] = i;
  return l;
}

// ---------------------------------------------------------------- tensor arrays
void k_write_to_array(const OpRun& r) {
  const int64_t i = read_index(r);
  PA_CHECK(i >= 0, "write_to_array: negative index");
  Tensor x = r.in("X");
  Variable* out = r.out_var("Out");
  out->kind = VK_LOD_TENSOR_ARRAY;
  if ((int64_t)out->list.size() <= i) out->list.resize((size_t)i + 1);
  out->list[(size_t)i] = clone(r, x);
}

void k_read_from_array(const OpRun& r) {
  const int64_t i = read_index(r);
  Variable* a = r.in_var("X");
  PA_CHECK(i >= 0 && i < (int64_t)a->list.size() && a->list[(size_t)i].initialized(),
           "read_from_array: slot %lld of %s is empty", (long long)i, r.op.Input("X").c_str());
  set_out(r, "Out", clone(r, a->list[(size_t)i]));
}

void k_lod_array_length(const OpRun& r) {
  set_out(r, "Out", host_scalar_i64((int64_t)r.in_var("X")->list.size()));
}

void k_lod_rank_table(const OpRun& r) {
  Tensor x = r.in("X");
  const size_t level = (size_t)r.op.GetInt("level", 0);
  std::vector<size_t> lvl;
  if (x.lod.empty()) {
    lvl = last_level(x);
  } else {
    PA_CHECK(level < x.lod.size(), "lod_rank_table: level %zu of a %zu-level LoD", level, x.lod.size());
    lvl = x.lod[level];
  }
  Variable* out = r.out_var("Out");
  out->kind = VK_LOD_RANK_TABLE;
  out->rank.clear();
  for (size_t i = 0; i + 1 < lvl.size(); ++i) out->rank.push_back({(int64_t)i, (int64_t)(lvl[i + 1] - lvl[i])});
  std::stable_sort(out->rank.begin(), out->rank.end(),
                   [](const RankItem& a, const RankItem& b) { return a.length > b.length; });
  out->rank_coarse_lod.assign(x.lod.begin(), x.lod.begin() + std::min(level, x.lod.size()));
}

void k_max_sequence_len(const OpRun& r) {
  const Variable& t = rank_table(r);
  set_out(r, "Out", host_scalar_i64(t.rank.empty() ? 0 : t.rank[0].length));
}

// rows of X at time step t of every sequence still alive, in rank order
std::vector<int64_t> step_rows(const std::vector<RankItem>& items, const std::vector<size_t>& lvl, int64_t t) {
  std::vector<int64_t> rows;
  for (auto& it : items)
    if (it.length > t) rows.push_back((int64_t)lvl[(size_t)it.index] + t);
  return rows;
}

void k_lod_tensor_to_array(const OpRun& r) {
  Tensor x = r.in("X");
  const Variable& tab = rank_table(r);
  const auto lvl = last_level(x);
  const int64_t maxlen = tab.rank.empty() ? 0 : tab.rank[0].length;
  std::vector<Tensor> arr((size_t)maxlen);
  for (int64_t t = 0; t < maxlen; ++t) {
    const auto rows = step_rows(tab.rank, lvl, t);
    Dims d = x.dims;
    d[0] = (int64_t)rows.size();
    arr[(size_t)t].alloc(x.dtype, d, x.device);
    gather(r, x, rows, arr[(size_t)t]);
  }
  Variable* out = r.out_var("Out");
  out->kind = VK_LOD_TENSOR_ARRAY;
  out->list = std::move(arr);
}

// output offsets of the sequences in their ORIGINAL order (array_to_lod_tensor)
std::vector<size_t> seq_offsets(const std::vector<RankItem>& items) {
  std::vector<int64_t> len(items.size(), 0);
  for (auto& it : items) len[(size_t)it.index] = it.length;
  std::vector<size_t> off{0};
  for (int64_t l : len) off.push_back(off.back() + (size_t)l);
  return off;
}

void k_array_to_lod_tensor(const OpRun& r) {
  Variable* a = r.in_var("X");
  const Variable& tab = rank_table(r);
  const auto off = seq_offsets(tab.rank);
  PA_CHECK(!a->list.empty() && a->list[0].initialized(), "array_to_lod_tensor: empty array");
  const Tensor& first = a->list[0];
  Dims d = first.dims;
  d[0] = (int64_t)off.back();
  Tensor out;
  out.alloc(first.dtype, d, first.device);
  for (size_t t = 0; t < a->list.size(); ++t) {
    std::vector<int64_t> dst;
    for (auto& it : tab.rank)
      if (it.length > (int64_t)t) dst.push_back((int64_t)off[(size_t)it.index] + (int64_t)t);
    if (dst.empty()) continue;
    PA_CHECK(a->list[t].initialized() && row_count(a->list[t]) == (int64_t)dst.size(),
             "array_to_lod_tensor: step %zu holds %lld rows, %zu sequences are alive", t,
             (long long)row_count(a->list[t]), dst.size());
    scatter(r, a->list[t], dst, out, false);
  }
  out.lod = LoD{off};
  set_out(r, "Out", std::move(out));
}

void k_shrink_rnn_memory(const OpRun& r) {
  const int64_t i = read_index(r);
  const Variable& tab = rank_table(r);
  Tensor x = r.in("X");
  int64_t alive = 0;
  for (auto& it : tab.rank) alive += it.length > i;
  alive = std::min(alive, row_count(x));
  std::vector<int64_t> rows((size_t)alive);
  for (int64_t k = 0; k < alive; ++k) rows[(size_t)k] = k;
  Dims d = x.dims;
  d[0] = alive;
  Tensor out;
  out.alloc(x.dtype, d, x.device);
  gather(r, x, rows, out);
  set_out(r, "Out", std::move(out));
}

// reorder_lod_tensor_by_rank: the X rows of each ranked item, in rank order
std::vector<int64_t> rank_rows(const Tensor& x, const std::vector<RankItem>& items, std::vector<size_t>* off) {
  std::vector<int64_t> rows;
  off->assign(1, 0);
  if (x.lod.empty()) {
    for (auto& it : items) rows.push_back(it.index);
    return rows;
  }
  const auto& lvl = x.lod[0];
  for (auto& it : items) {
    for (size_t k = lvl[(size_t)it.index]; k < lvl[(size_t)it.index + 1]; ++k) rows.push_back((int64_t)k);
    off->push_back(off->back() + lvl[(size_t)it.index + 1] - lvl[(size_t)it.index]);
  }
  return rows;
}

void k_reorder_lod_tensor_by_rank(const OpRun& r) {
  Tensor x = r.in("X");
  const Variable& tab = rank_table(r);
  std::vector<size_t> off;
  const auto rows = rank_rows(x, tab.rank, &off);
  Dims d = x.dims;
  d[0] = (int64_t)rows.size();
  Tensor out;
  out.alloc(x.dtype, d, x.device);
  gather(r, x, rows, out);
  if (!x.lod.empty()) out.lod = LoD{off};
  set_out(r, "Out", std::move(out));
}

// ---------------------------------------------------------------- their gradients
void add_into(const OpRun& r, Tensor& acc, const Tensor& g) {
  PA_CHECK(acc.dtype == DT::FP32 && g.dtype == DT::FP32 && acc.numel() == g.numel(), "%s: cannot accumulate",
           r.op.type.c_str());
  if (acc.device >= 0) {
    device_add_f32(r.ctx.stream, acc.data<float>(), g.data<float>(), g.numel());
  } else {
    for (int64_t i = 0; i < g.numel(); ++i) acc.data<float>()[i] += g.data<float>()[i];
  }
}

void k_read_from_array_grad(const OpRun& r) {
  const int64_t i = read_index(r);
  Variable* out = r.out_var("X@GRAD");
  if (!out) return;
  if (out->kind != VK_LOD_TENSOR_ARRAY) {
    out->kind = VK_LOD_TENSOR_ARRAY;
    out->list.clear();
  }
  if ((int64_t)out->list.size() <= i) out->list.resize((size_t)i + 1);
  Tensor* g = r.in_opt("Out@GRAD");
  if (!g) return;
  Tensor& cur = out->list[(size_t)i];
  if (cur.initialized() && cur.dims == g->dims) {
    Tensor sum = clone(r, cur);  // a fresh buffer: the slot may share storage with a reader
    add_into(r, sum, *g);
    sum.lod = g->lod;
    cur = sum;
  } else {
    cur = clone(r, *g);
  }
}

void k_write_to_array_grad(const OpRun& r) {
  const int64_t i = read_index(r);
  Tensor x = r.in("X");
  const Tensor* g = nullptr;
  const auto& gn = r.op.Inputs("Out@GRAD");
  if (!gn.empty())
    if (Variable* a = r.scope.Find(gn[0]))
      if (a->kind == VK_LOD_TENSOR_ARRAY && i < (int64_t)a->list.size() && a->list[(size_t)i].initialized())
        g = &a->list[(size_t)i];
  Tensor out = g ? clone(r, *g) : zeros_like(r, x);
  out.lod = x.lod;
  set_out(r, "X@GRAD", std::move(out));
}

void k_lod_tensor_to_array_grad(const OpRun& r) {
  Tensor x = r.in("X");
  const Variable& tab = rank_table(r);
  const auto lvl = last_level(x);
  Tensor gx = zeros_like(r, x);
  const auto& gn = r.op.Inputs("Out@GRAD");
  if (!gn.empty())
    if (Variable* a = r.scope.Find(gn[0]))
      if (a->kind == VK_LOD_TENSOR_ARRAY)
        for (size_t t = 0; t < a->list.size(); ++t) {
          if (!a->list[t].initialized()) continue;
          scatter(r, a->list[t], step_rows(tab.rank, lvl, (int64_t)t), gx, true);
        }
  gx.lod = x.lod;
  set_out(r, "X@GRAD", std::move(gx));
}

void k_array_to_lod_tensor_grad(const OpRun& r) {
  Tensor g = r.in("Out@GRAD");
  const Variable& tab = rank_table(r);
  const auto off = seq_offsets(tab.rank);
  const int64_t maxlen = tab.rank.empty() ? 0 : tab.rank[0].length;
  std::vector<Tensor> arr((size_t)maxlen);
  for (int64_t t = 0; t < maxlen; ++t) {
    std::vector<int64_t> rows;
    for (auto& it : tab.rank)
      if (it.length > t) rows.push_back((int64_t)off[(size_t)it.index] + t);
    Dims d = g.dims;
    d[0] = (int64_t)rows.size();
    arr[(size_t)t].alloc(g.dtype, d, g.device);
    gather(r, g, rows, arr[(size_t)t]);
  }
  Variable* out = r.out_var("X@GRAD");
  if (!out) return;
  out->kind = VK_LOD_TENSOR_ARRAY;
  out->list = std::move(arr);
}

void k_shrink_rnn_memory_grad(const OpRun& r) {
  Tensor x = r.in("X");
  Tensor gx = zeros_like(r, x);
  if (Tensor* g = r.in_opt("Out@GRAD")) {
    PA_CHECK(row_count(*g) <= row_count(x) && row_bytes(*g) == row_bytes(gx), "shrink_rnn_memory_grad: shapes");
    if (g->nbytes()) device_copy(gx.raw(), gx.device, g->raw(), g->device, g->nbytes(), r.ctx.stream);
  }
  gx.lod = x.lod;
  set_out(r, "X@GRAD", std::move(gx));
}

void k_reorder_lod_tensor_by_rank_grad(const OpRun& r) {
  Tensor x = r.in("X");
  Tensor g = r.in("Out@GRAD");
  const Variable& tab = rank_table(r);
  std::vector<size_t> off;
  const auto rows = rank_rows(x, tab.rank, &off);
  Tensor gx = zeros_like(r, x);
  scatter(r, g, rows, gx, false);
  gx.lod = x.lod;
  set_out(r, "X@GRAD", std::move(gx));
}

// ---------------------------------------------------------------- misc ops of the RNN programs
// fill_constant_batch_size_like_op.cc: shape[output_dim_idx] = Input.dims[input_dim_idx]
void k_fill_constant_batch_size_like(const OpRun& r) {
  Tensor in = r.in("Input");
  Dims shape = r.op.GetInts("shape");
  const size_t oi = (size_t)r.op.GetInt("output_dim_idx", 0), ii = (size_t)r.op.GetInt("input_dim_idx", 0);
  PA_CHECK(oi < shape.size() && ii < in.dims.size(), "fill_constant_batch_size_like: dim index out of range");
  shape[oi] = in.dims[ii];
  const DT dt = (DT)r.op.GetInt("dtype", (int)DT::FP32);
  const double v = (double)r.op.GetFloat("value");
  const int dev = r.op.GetBool("force_cpu", false) ? -1 : r.ctx.device;
  Tensor out;
  out.alloc(dt, shape, dev);
  if (dev >= 0) {
    device_fill(r.ctx.stream, out.raw(), dt, out.numel(), v);
  } else {
    const int64_t n = out.numel();
    switch (dt) {
      case DT::FP32: std::fill_n(out.data<float>(), n, (float)v); break;
      case DT::FP64: std::fill_n(out.data<double>(), n, v); break;
      case DT::INT64: std::fill_n(out.data<int64_t>(), n, (int64_t)v); break;
      case DT::INT32: std::fill_n(out.data<int32_t>(), n, (int32_t)v); break;
      case DT::BOOL: case DT::UINT8: std::fill_n(out.data<uint8_t>(), n, (uint8_t)v); break;
      default: fail("fill_constant_batch_size_like: dtype %s", dt_name(dt));
    }
  }
  set_out(r, "Out", std::move(out));
}

// sum's gradient: every X@GRAD[i] is a copy of Out@GRAD
void k_sum_grad(const OpRun& r) {
  Tensor g = r.in("Out@GRAD");
  const auto& xs = r.op.Inputs("X");
  for (size_t i = 0; i < r.op.Outputs("X@GRAD").size(); ++i) {
    Variable* v = r.out_var("X@GRAD", i);
    if (!v) continue;
    Tensor t = clone(r, g);
    if (i < xs.size())
      if (Variable* x = r.scope.Find(xs[i]))
        if (x->tensor.initialized()) {
          PA_CHECK(x->tensor.numel() == g.numel(), "sum_grad: X[%zu] and Out@GRAD differ in size", i);
          t.dims = x->tensor.dims;
          t.lod = x->tensor.lod;
        }
    v->kind = VK_LOD_TENSOR;
    v->tensor = std::move(t);
  }
}

// assign's gradient: X@GRAD is a copy of Out@GRAD
void k_assign_grad(const OpRun& r) {
  Tensor g = r.in("Out@GRAD");
  if (r.out_var("X@GRAD")) set_out(r, "X@GRAD", clone(r, g));
}

// concat's gradient: Out@GRAD split along `axis` into the shapes of X
void k_concat_grad(const OpRun& r) {
  Tensor g = r.in("Out@GRAD");
  auto xs = r.ins("X");
  std::vector<Tensor> keep;
  for (auto* t : xs) keep.push_back(*t);
  int64_t axis = r.op.GetInt("axis", 0);
  if (axis < 0) axis += (int64_t)g.dims.size();
  const int64_t pre = [&] { int64_t n = 1; for (int64_t i = 0; i < axis; ++i) n *= g.dims[(size_t)i]; return n; }();
  int64_t post = 1;
  for (size_t i = (size_t)axis + 1; i < g.dims.size(); ++i) post *= g.dims[i];
  const size_t es = dt_size(g.dtype);
  const int64_t gw = g.dims[(size_t)axis] * post;
  int64_t off = 0;
  for (size_t k = 0; k < keep.size(); ++k) {
    const int64_t w = keep[k].dims[(size_t)axis] * post;
    Variable* v = r.out_var("X@GRAD", k);
    if (v) {
      Tensor t;
      t.alloc(g.dtype, keep[k].dims, g.device);
      t.lod = keep[k].lod;
      // pre rows of w elements each, strided gw in Out@GRAD: gather as rows of w
      if (pre && w) {
        if (g.device >= 0) {
          device_copy2d(r, t.raw(), (size_t)(w * es), (const char*)g.raw() + off * es, (size_t)(gw * es),
                        (size_t)(w * es), (size_t)pre);
        } else {
          for (int64_t p = 0; p < pre; ++p)
            memcpy((char*)t.raw() + p * w * es, (const char*)g.raw() + (p * gw + off) * es, (size_t)(w * es));
        }
      }
      v->kind = VK_LOD_TENSOR;
      v->tensor = std::move(t);
    }
    off += w;
  }
}

// ---------------------------------------------------------------- SelectedRows
bool is_sr(const Variable* v) { return v && v->kind == VK_SELECTED_ROWS; }

}  // namespace

void lookup_table_grad_sparse(const OpRun& r) {
  Tensor w = r.in("W");
  Tensor ids = r.in("Ids");
  Tensor g = r.in("Out@GRAD");
  PA_CHECK(w.dims.size() == 2, "lookup_table_grad: W must be 2-D");
  Tensor hid = ids.device >= 0 ? ids.to(-1, r.ctx.stream) : ids;
  if (ids.device >= 0) device_stream_sync(r.ctx.stream);
  std::vector<int64_t> rows((size_t)hid.numel());
  if (hid.dtype == DT::INT64) memcpy(rows.data(), hid.raw(), rows.size() * 8);
  else if (hid.dtype == DT::INT32)
    for (size_t i = 0; i < rows.size(); ++i) rows[i] = hid.data<int32_t>()[i];
  else fail("lookup_table_grad: ids dtype %s", dt_name(hid.dtype));
  const int64_t D = w.dims[1], pad = r.op.GetInt("padding_idx", -1);
  PA_CHECK(g.numel() == (int64_t)rows.size() * D, "lookup_table_grad: Out@GRAD has %lld elements, expected %lld",
           (long long)g.numel(), (long long)rows.size() * D);
  Tensor val = clone(r, g);
  val.dims = {(int64_t)rows.size(), D};
  val.lod.clear();
  if (pad != -1)
    for (size_t i = 0; i < rows.size(); ++i)
      if (rows[i] == pad) {
        if (val.device >= 0) device_fill(r.ctx.stream, val.data<float>() + i * D, DT::FP32, D, 0.0);
        else std::fill_n(val.data<float>() + i * D, D, 0.f);
      }
  Variable* out = r.out_var("W@GRAD");
  out->kind = VK_SELECTED_ROWS;
  out->rows = std::move(rows);
  out->height = w.dims[0];
  out->tensor = std::move(val);
}

// sum_op.h: SelectedRows-only inputs concatenate into a SelectedRows; a mix with
// dense tensors densifies the SelectedRows into the dense sum
bool selected_rows_sum(const OpRun& r) {
  const auto& names = r.op.Inputs("X");
  bool any = false;
  for (auto& n : names) any |= is_sr(r.scope.Find(n));
  if (!any) return false;
  std::vector<const Variable*> vs;
  for (auto& n : names) vs.push_back(r.var(n));
  bool all = true;
  for (auto* v : vs) all &= is_sr(v) || !v->tensor.initialized();
  Variable* out = r.out_var("Out");
  if (all) {
    std::vector<int64_t> rows;
    int64_t height = 0, total = 0, width = 0;
    const Tensor* proto = nullptr;
    for (auto* v : vs) {
      if (!is_sr(v)) continue;
      rows.insert(rows.end(), v->rows.begin(), v->rows.end());
      height = v->height;
      total += row_count(v->tensor);
      width = row_count(v->tensor) ? v->tensor.numel() / row_count(v->tensor) : width;
      proto = &v->tensor;
    }
    PA_CHECK(proto != nullptr, "sum: no SelectedRows input holds a value");
    Tensor val;
    val.alloc(proto->dtype, {total, width}, proto->device);
    int64_t at = 0;
    for (auto* v : vs) {
      if (!is_sr(v) || !v->tensor.nbytes()) continue;
      device_copy((char*)val.raw() + at, val.device, v->tensor.raw(), v->tensor.device, v->tensor.nbytes(),
                  r.ctx.stream);
      at += (int64_t)v->tensor.nbytes();
    }
    out->kind = VK_SELECTED_ROWS;
    out->rows = std::move(rows);
    out->height = height;
    out->tensor = std::move(val);
    return true;
  }
  const Tensor* dense = nullptr;
  for (auto* v : vs)
    if (!is_sr(v) && v->tensor.initialized()) dense = &v->tensor;
  Tensor acc = zeros_like(r, *dense);
  for (auto* v : vs) {
    if (is_sr(v)) {
      Tensor src = v->tensor;
      scatter(r, src, v->rows, acc, true);
    } else if (v->tensor.initialized()) {
      add_into(r, acc, v->tensor);
    }
  }
  out->kind = VK_LOD_TENSOR;
  out->rows.clear();
  out->tensor = std::move(acc);
  return true;
}

// sgd_op.h SelectedRows branch: Param[rows[i]] -= lr * value[i] (duplicates add up)
bool selected_rows_sgd(const OpRun& r) {
  Variable* gv = r.in_var("Grad");
  if (!is_sr(gv)) return false;
  Tensor& p = r.in("Param");
  Tensor* po = r.out("ParamOut");
  PA_CHECK(po && po->raw() == p.raw(), "sgd: a SelectedRows update must be in place (ParamOut == Param)");
  const Tensor& val = gv->tensor;
  const int64_t w = row_count(p) ? p.numel() / row_count(p) : 0;
  PA_CHECK(val.numel() == (int64_t)gv->rows.size() * w, "sgd: SelectedRows value does not match Param rows");
  const Tensor& lr = r.in("LearningRate");
  if (p.device >= 0) {
    device_sgd_rows(r, p.data<float>(), val.data<float>(), gv->rows, w, lr.data<float>());
    return true;
  }
  const float l = lr.data<float>()[0];
  for (size_t i = 0; i < gv->rows.size(); ++i) {
    PA_CHECK(gv->rows[i] >= 0 && gv->rows[i] < row_count(p), "sgd: row %lld out of range", (long long)gv->rows[i]);
    float* d = p.data<float>() + gv->rows[i] * w;
    const float* s = val.data<float>() + i * w;
    for (int64_t j = 0; j < w; ++j) d[j] -= l * s[j];
  }
  return true;
}

// adam_op.h SparseAdamFunctor (the Python engine's semantics): duplicate rows are
// merged, then only the touched rows of Param / Moment1 / Moment2 update
bool selected_rows_adam(const OpRun& r) {
  Variable* gv = r.in_var("Grad");
  if (!is_sr(gv)) return false;
  Tensor& p = r.in("Param");
  Tensor& m1 = r.in("Moment1");
  Tensor& m2 = r.in("Moment2");
  PA_CHECK(r.out("ParamOut")->raw() == p.raw() && r.out("Moment1Out")->raw() == m1.raw() &&
               r.out("Moment2Out")->raw() == m2.raw(),
           "adam: a SelectedRows update must be in place");
  const int64_t w = row_count(p) ? p.numel() / row_count(p) : 0;
  std::vector<int64_t> uniq = gv->rows;
  std::sort(uniq.begin(), uniq.end());
  uniq.erase(std::unique(uniq.begin(), uniq.end()), uniq.end());
  std::vector<int64_t> inv(gv->rows.size());
  for (size_t i = 0; i < inv.size(); ++i)
    inv[i] = std::lower_bound(uniq.begin(), uniq.end(), gv->rows[i]) - uniq.begin();
  for (int64_t u : uniq) PA_CHECK(u >= 0 && u < row_count(p), "adam: row %lld out of range", (long long)u);
  Tensor merged;
  merged.alloc(DT::FP32, {(int64_t)uniq.size(), w}, p.device);
  if (merged.device >= 0) device_fill(r.ctx.stream, merged.raw(), DT::FP32, merged.numel(), 0.0);
  else std::fill_n(merged.data<float>(), merged.numel(), 0.f);
  Tensor val = gv->tensor;
  val.dims = {(int64_t)gv->rows.size(), w};
  scatter(r, val, inv, merged, true);
  const float b1 = r.op.GetFloat("beta1", 0.9f), b2 = r.op.GetFloat("beta2", 0.999f),
              eps = r.op.GetFloat("epsilon", 1e-8f);
  const Tensor& lr = r.in("LearningRate");
  const Tensor& b1p = r.in("Beta1Pow");
  const Tensor& b2p = r.in("Beta2Pow");
  if (p.device >= 0) {
    device_adam_rows(r, p.data<float>(), m1.data<float>(), m2.data<float>(), merged.data<float>(), uniq, w,
                     lr.data<float>(), b1p.data<float>(), b2p.data<float>(), b1, b2, eps);
    return true;
  }
  const float l = lr.data<float>()[0], bp1 = b1p.data<float>()[0], bp2 = b2p.data<float>()[0];
  const float lr_t = l * sqrtf(1.f - bp2) / (1.f - bp1);
  for (size_t k = 0; k < uniq.size(); ++k)
    for (int64_t j = 0; j < w; ++j) {
      const int64_t e = uniq[k] * w + j;
      const float g = merged.data<float>()[k * w + j];
      float& a = m1.data<float>()[e];
      float& b = m2.data<float>()[e];
      a = b1 * a + (1.f - b1) * g;
      b = b2 * b + (1.f - b2) * g * g;
      p.data<float>()[e] -= lr_t * a / (sqrtf(b) + eps);
    }
  return true;
}

#define PA_ANY_KERNEL(name, fn)   \
  PA_HOST_KERNEL(name, fn);       \
  PA_DEVICE_KERNEL(name, fn)
PA_ANY_KERNEL(write_to_array, k_write_to_array);
PA_ANY_KERNEL(read_from_array, k_read_from_array);
PA_ANY_KERNEL(lod_array_length, k_lod_array_length);
PA_ANY_KERNEL(lod_rank_table, k_lod_rank_table);
PA_ANY_KERNEL(max_sequence_len, k_max_sequence_len);
PA_ANY_KERNEL(lod_tensor_to_array, k_lod_tensor_to_array);
PA_ANY_KERNEL(array_to_lod_tensor, k_array_to_lod_tensor);
PA_ANY_KERNEL(shrink_rnn_memory, k_shrink_rnn_memory);
PA_ANY_KERNEL(reorder_lod_tensor_by_rank, k_reorder_lod_tensor_by_rank);
PA_ANY_KERNEL(read_from_array_grad, k_read_from_array_grad);
PA_ANY_KERNEL(write_to_array_grad, k_write_to_array_grad);
PA_ANY_KERNEL(lod_tensor_to_array_grad, k_lod_tensor_to_array_grad);
PA_ANY_KERNEL(array_to_lod_tensor_grad, k_array_to_lod_tensor_grad);
PA_ANY_KERNEL(shrink_rnn_memory_grad, k_shrink_rnn_memory_grad);
PA_ANY_KERNEL(reorder_lod_tensor_by_rank_grad, k_reorder_lod_tensor_by_rank_grad);
PA_ANY_KERNEL(fill_constant_batch_size_like, k_fill_constant_batch_size_like);
PA_ANY_KERNEL(sum_grad, k_sum_grad);
PA_ANY_KERNEL(assign_grad, k_assign_grad);
PA_ANY_KERNEL(concat_grad, k_concat_grad);
#undef PA_ANY_KERNEL

void link_control_kernels() {}

}  // namespace pa
