// Place-agnostic kernels of the decoding-side LoD operators: beam_search,
// beam_search_decode, lod_reset, is_empty.
//
// Semantics (reference operators/beam_search_op.cc:27-260, beam_search_decode_op.h,
// lod_reset_op.h, is_empty_op.cc; the Python kernels of operators/structured_ops.py
// compute the same selections):
//   * beam_search: for every source sentence (LoD level `level` of `ids`, in
//     absolute row offsets) the beam_size best (score, prefix, id) candidates over
//     all of its prefixes' top-k candidates; a prefix that already emitted end_id
//     carries (end_id, its score) forward; a source whose every branch ended is
//     pruned (no rows).  Outputs carry the 2-level LoD [sources, prefixes].
//   * beam_search_decode: backtrack the per-step (ids, scores) arrays into whole
//     sentences per source, best final score first.
// Like the reference, which registers these kernels for the CPU only, the
// selection is a short integer algorithm over a few KB: on a HIP place the inputs
// are read back (one stream sync) and the results uploaded on the same stream, the
// same pattern as the LoDRankTable kernels of ops_control.cc.
#include <string.h>

#include <algorithm>
#include <vector>

#include "framework.h"

namespace pa {
namespace {

Tensor host_copy(const OpRun& r, const Tensor& t) {
  if (t.device < 0) return t;
  Tensor h = t.to(-1, r.ctx.stream);
  device_stream_sync(r.ctx.stream);
  return h;
}

std::vector<int64_t> as_i64(const Tensor& h) {
  std::vector<int64_t> v((size_t)h.numel());
  if (h.dtype == DT::INT64) memcpy(v.data(), h.raw(), v.size() * 8);
  else if (h.dtype == DT::INT32)
    for (size_t i = 0; i < v.size(); ++i) v[i] = h.data<int32_t>()[i];
  else fail("expected an integer id tensor, got %s", dt_name(h.dtype));
  return v;
}

std::vector<float> as_f32(const Tensor& h) {
  std::vector<float> v((size_t)h.numel());
  if (h.dtype == DT::FP32) memcpy(v.data(), h.raw(), v.size() * 4);
  else if (h.dtype == DT::FP64)
    for (size_t i = 0; i < v.size(); ++i) v[i] = (float)h.data<double>()[i];
  else fail("expected a float score tensor, got %s", dt_name(h.dtype));
  return v;
}

// a [n, 1] tensor of `vals` on `dev` (uploaded through a host tensor)
template <class T>
void put_column(const OpRun& r, Tensor* out, DT dt, const std::vector<T>& vals, int dev, bool column = true) {
  Tensor h;
  const int64_t n = (int64_t)vals.size();
  h.alloc(dt, column ? std::vector<int64_t>{n, 1} : std::vector<int64_t>{n}, -1);
  if (n) memcpy(h.raw(), vals.data(), sizeof(T) * (size_t)n);
  if (dev < 0) {
    *out = h;
    return;
  }
  out->alloc(dt, h.dims, dev);
  if (n) device_copy(out->raw(), dev, h.raw(), -1, h.nbytes(), r.ctx.stream);
  device_stream_sync(r.ctx.stream);  // `h` dies with this op
}

void k_beam_search(const OpRun& r) {
  Tensor& ids_t = r.in("ids");
  const int dev = ids_t.device;
  const std::vector<int64_t> pre_ids = as_i64(host_copy(r, r.in("pre_ids")));
  Tensor* ps = r.in_opt("pre_scores");
  std::vector<float> pre_scores = ps ? as_f32(host_copy(r, *ps)) : std::vector<float>(pre_ids.size(), 0.f);
  const std::vector<int64_t> ids = as_i64(host_copy(r, ids_t));
  const std::vector<float> scores = as_f32(host_copy(r, r.in("scores")));
  const int64_t level = r.op.GetInt("level", 0), beam = r.op.GetInt("beam_size", 1), end = r.op.GetInt("end_id", 0);
  const int64_t P = (int64_t)pre_ids.size();
  PA_CHECK(P > 0 && (int64_t)ids.size() % P == 0, "beam_search: ids rows must match pre_ids");
  const int64_t K = (int64_t)ids.size() / P;
  // absolute row offsets of the source level (framework::ToAbsOffset)
  std::vector<size_t> high;
  if (!ids_t.lod.empty()) {
    LoD abs = ids_t.lod;
    for (int64_t lv = (int64_t)abs.size() - 2; lv >= 0; --lv)
      for (auto& x : abs[(size_t)lv]) x = abs[(size_t)lv + 1][x];
    PA_CHECK(level < (int64_t)abs.size(), "beam_search: level %lld out of the LoD", (long long)level);
    high = abs[(size_t)level];
  } else {
    high = {0, (size_t)P};
  }
  struct Cand {
    float score;
    int64_t off, id;
  };
  std::vector<std::vector<std::pair<int64_t, float>>> per_prefix((size_t)P);
  for (size_t s = 0; s + 1 < high.size(); ++s) {
    std::vector<Cand> items;
    for (int64_t off = (int64_t)high[s]; off < (int64_t)high[s + 1]; ++off) {
      if (pre_ids[(size_t)off] == end) {
        items.push_back({pre_scores[(size_t)off], off, end});
      } else {
        for (int64_t d = 0; d < K; ++d) items.push_back({scores[(size_t)(off * K + d)], off, ids[(size_t)(off * K + d)]});
      }
    }
    std::stable_sort(items.begin(), items.end(), [](const Cand& a, const Cand& b) { return a.score > b.score; });
    for (int64_t k = 0; k < std::min<int64_t>(beam, (int64_t)items.size()); ++k)
      per_prefix[(size_t)items[(size_t)k].off].push_back({items[(size_t)k].id, items[(size_t)k].score});
    bool all_end = true;
    for (int64_t off = (int64_t)high[s]; off < (int64_t)high[s + 1] && all_end; ++off) {
      if (pre_ids[(size_t)off] != end) all_end = false;
      for (auto& c : per_prefix[(size_t)off])
        if (c.first != end) all_end = false;
    }
    if (all_end)
      for (int64_t off = (int64_t)high[s]; off < (int64_t)high[s + 1]; ++off) per_prefix[(size_t)off].clear();
  }
  std::vector<int64_t> out_ids;
  std::vector<float> out_sc;
  std::vector<size_t> low{0};
  for (auto& lst : per_prefix) {
    std::stable_sort(lst.begin(), lst.end(), [](const auto& a, const auto& b) { return a.second > b.second; });
    for (auto& c : lst) {
      out_ids.push_back(c.first);
      out_sc.push_back(c.second);
    }
    low.push_back(out_ids.size());
  }
  Tensor* oi = r.out("selected_ids");
  Tensor* os = r.out("selected_scores");
  put_column(r, oi, DT::INT64, out_ids, dev);
  put_column(r, os, DT::FP32, out_sc, dev);
  oi->lod = {high, low};
  os->lod = {high, low};
}

void k_beam_search_decode(const OpRun& r) {
  Variable* iv = r.in_var("Ids");
  Variable* sv = r.in_var("Scores");
  PA_CHECK(iv->kind == VK_LOD_TENSOR_ARRAY && sv->kind == VK_LOD_TENSOR_ARRAY, "beam_search_decode: arrays expected");
  const int64_t end = r.op.GetInt("end_id", 0);
  const size_t steps = iv->list.size();
  PA_CHECK(steps > 0 && sv->list.size() == steps, "beam_search_decode: empty or mismatched step arrays");
  const int dev = iv->list[0].device;
  PA_CHECK(iv->list[0].lod.size() >= 2, "beam_search_decode: step ids need a 2-level LoD");
  const size_t src_num = iv->list[0].lod[0].size() - 1;
  struct Sent {
    std::vector<int64_t> w;
    std::vector<float> s;
  };
  std::vector<std::vector<Sent>> sents(src_num);
  std::vector<std::vector<size_t>> prefix(src_num);
  for (int64_t t = (int64_t)steps - 1; t >= 0; --t) {
    const Tensor& it = iv->list[(size_t)t];
    const std::vector<int64_t> ids = as_i64(host_copy(r, it));
    const std::vector<float> scs = as_f32(host_copy(r, sv->list[(size_t)t]));
    const auto& src_lod = it.lod[0];
    const auto& sent_lod = it.lod[1];
    for (size_t s = 0; s < src_num; ++s) {
      const size_t ps = src_lod[s], pe = src_lod[s + 1];
      if (prefix[s].empty()) {
        for (size_t p = ps; p < pe; ++p)
          for (size_t c = sent_lod[p]; c < sent_lod[p + 1]; ++c) {
            prefix[s].push_back(p);
            sents[s].push_back(Sent{{ids[c]}, {scs[c]}});
          }
      } else {
        for (size_t k = 0; k < prefix[s].size(); ++k) {
          const size_t c = prefix[s][k];
          Sent& st = sents[s][k];
          if (ids[c] != end || st.w.empty()) {
            st.w.push_back(ids[c]);
            st.s.push_back(scs[c]);
          }
          size_t p = ps;
          while (sent_lod[p + 1] <= c) ++p;
          prefix[s][k] = p;
        }
      }
    }
  }
  std::vector<int64_t> out_ids;
  std::vector<float> out_sc;
  std::vector<size_t> src_off{0}, sent_off{0};
  for (size_t s = 0; s < src_num; ++s) {
    std::vector<Sent> ordered = sents[s];
    std::stable_sort(ordered.begin(), ordered.end(), [](const Sent& a, const Sent& b) { return a.s[0] > b.s[0]; });
    for (auto& st : ordered) {
      out_ids.insert(out_ids.end(), st.w.rbegin(), st.w.rend());
      out_sc.insert(out_sc.end(), st.s.rbegin(), st.s.rend());
      sent_off.push_back(out_ids.size());
    }
    src_off.push_back(src_off.back() + ordered.size());
  }
  Tensor* oi = r.out("SentenceIds");
  Tensor* os = r.out("SentenceScores");
  put_column(r, oi, DT::INT64, out_ids, dev, false);
  put_column(r, os, DT::FP32, out_sc, dev, false);
  oi->lod = {src_off, sent_off};
  os->lod = {src_off, sent_off};
}

// lod_reset_op.h: Out shares X's data with the LoD of Y (or Y's values, or target_lod)
void k_lod_reset(const OpRun& r) {
  Tensor& x = r.in("X");
  LoD lod;
  if (Tensor* y = r.in_opt("Y")) {
    if (!y->lod.empty()) {
      lod = y->lod;
    } else {
      const std::vector<int64_t> v = as_i64(host_copy(r, *y));
      lod = {std::vector<size_t>(v.begin(), v.end())};
    }
  } else {
    const auto t = r.op.GetInts("target_lod");
    lod = {std::vector<size_t>(t.begin(), t.end())};
  }
  Tensor* o = r.out("Out");
  if (o != &x) o->share(x);
  o->lod = lod;
}

// is_empty_op.cc: a host bool [1]
void k_is_empty(const OpRun& r) {
  Tensor* o = r.out("Out");
  o->alloc(DT::BOOL, {1}, -1);
  *o->data<uint8_t>() = r.in("X").numel() == 0 ? 1 : 0;
}

}  // namespace

#define PA_ANY_KERNEL(name, fn) \
  PA_HOST_KERNEL(name, fn);     \
  PA_DEVICE_KERNEL(name, fn)
PA_ANY_KERNEL(beam_search, k_beam_search);
PA_ANY_KERNEL(beam_search_decode, k_beam_search_decode);
PA_ANY_KERNEL(lod_reset, k_lod_reset);
PA_ANY_KERNEL(is_empty, k_is_empty);
#undef PA_ANY_KERNEL

void link_beam_kernels() {}

}  // namespace pa
