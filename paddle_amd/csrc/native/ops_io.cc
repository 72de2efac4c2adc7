// save / load / save_combine / load_combine on the C++ executor (host and device).
//
// Semantics: reference operators/save_op.cc, load_op.cc, save_combine_op.cc,
// load_combine_op.cc -- the LoDTensor stream format of framework/lod_tensor.cc
// (SerializeToStream: u32 version, LoD levels, then the TensorDesc-prefixed data),
// written / read by read_lod_tensor / write_lod_tensor (core.cc), the same bytes
// the Python op library's framework/serialization.py produces.  save_as_fp16 /
// load_as_fp16 convert floating tensors to fp16 on the way.  A device tensor is
// staged through the host (the file IS on the host), then uploaded on the op's
// stream: no host-kernel fallback.
#include <errno.h>
#include <math.h>
#include <string.h>
#include <sys/stat.h>

#include <string>

#include "framework.h"

namespace pa {
namespace {

void ensure_dir(const std::string& path) {
  const size_t p = path.find_last_of('/');
  if (p == std::string::npos || p == 0) return;
  std::string acc;
  const std::string dir = path.substr(0, p);
  for (size_t i = 0; i <= dir.size(); ++i) {
    if (i == dir.size() || dir[i] == '/') {
      if (!acc.empty() && mkdir(acc.c_str(), 0755) != 0 && errno != EEXIST)
        fail("save: cannot create directory %s", acc.c_str());
    }
    if (i < dir.size()) acc.push_back(dir[i]);
  }
}

uint16_t f32_to_f16(float f) {
  uint32_t x;
  memcpy(&x, &f, 4);
  const uint32_t sign = (x >> 16) & 0x8000;
  int32_t exp = (int32_t)((x >> 23) & 0xff) - 127 + 15;
  uint32_t mant = x & 0x7fffff;
  if (((x >> 23) & 0xff) == 0xff) return (uint16_t)(sign | 0x7c00 | (mant ? 0x200 : 0));  // inf / nan
  if (exp >= 31) return (uint16_t)(sign | 0x7c00);
  if (exp <= 0) {
    if (exp < -10) return (uint16_t)sign;
    mant |= 0x800000;
    const uint32_t shift = (uint32_t)(14 - exp);
    uint32_t h = mant >> shift;
    const uint32_t rem = mant & ((1u << shift) - 1), half = 1u << (shift - 1);
    if (rem > half || (rem == half && (h & 1))) ++h;
    return (uint16_t)(sign | h);
  }
  uint32_t h = ((uint32_t)exp << 10) | (mant >> 13);
  const uint32_t rem = mant & 0x1fff;
  if (rem > 0x1000 || (rem == 0x1000 && (h & 1))) ++h;  // round to nearest even (may carry into exp)
  return (uint16_t)(sign | h);
}

Tensor to_host(const OpRun& r, const Tensor& t) {
  if (t.device < 0) return t;
  Tensor h = t.to(-1, r.ctx.stream);
  device_stream_sync(r.ctx.stream);
  return h;
}

Tensor as_fp16(const Tensor& h) {
  if (h.dtype != DT::FP32) return h;
  Tensor o;
  o.alloc(DT::FP16, h.dims, -1);
  o.lod = h.lod;
  for (int64_t i = 0; i < h.numel(); ++i) o.data<uint16_t>()[i] = f32_to_f16(h.data<float>()[i]);
  return o;
}

FILE* open_for_write(const OpRun& r) {
  const std::string path = r.op.GetString("file_path");
  PA_CHECK(!path.empty(), "%s: empty file_path", r.op.type.c_str());
  struct stat st;
  PA_CHECK(r.op.GetBool("overwrite", true) || stat(path.c_str(), &st) != 0,
           "%s: %s exists; set overwrite=True", r.op.type.c_str(), path.c_str());
  ensure_dir(path);
  FILE* f = fopen(path.c_str(), "wb");
  PA_CHECK(f != nullptr, "%s: cannot open %s for writing", r.op.type.c_str(), path.c_str());
  return f;
}

void store(const OpRun& r, Tensor* out, const Tensor& h) {
  const int dev = r.ctx.device;
  Tensor t = r.op.GetBool("load_as_fp16", false) ? as_fp16(h) : h;
  if (dev < 0) {
    *out = t;
    return;
  }
  *out = t.to(dev, r.ctx.stream);
  device_stream_sync(r.ctx.stream);  // the host staging tensor dies with the op
}

void k_save(const OpRun& r) {
  Tensor h = to_host(r, r.in("X"));
  if (r.op.GetBool("save_as_fp16", false)) h = as_fp16(h);
  FILE* f = open_for_write(r);
  write_lod_tensor(f, h);
  fclose(f);
}

void k_save_combine(const OpRun& r) {
  std::vector<Tensor> hs;
  for (Tensor* t : r.ins("X")) {
    Tensor h = to_host(r, *t);
    if (r.op.GetBool("save_as_fp16", false)) h = as_fp16(h);
    hs.push_back(h);
  }
  FILE* f = open_for_write(r);
  for (const Tensor& h : hs) write_lod_tensor(f, h);
  fclose(f);
}

FILE* open_for_read(const OpRun& r) {
  const std::string path = r.op.GetString("file_path");
  FILE* f = fopen(path.c_str(), "rb");
  PA_CHECK(f != nullptr, "%s: cannot open %s", r.op.type.c_str(), path.c_str());
  return f;
}

void k_load(const OpRun& r) {
  FILE* f = open_for_read(r);
  Tensor h;
  const bool ok = read_lod_tensor(f, &h);
  fclose(f);
  PA_CHECK(ok, "load: %s holds no tensor", r.op.GetString("file_path").c_str());
  store(r, r.out("Out"), h);
}

void k_load_combine(const OpRun& r) {
  FILE* f = open_for_read(r);
  const size_t n = r.op.Outputs("Out").size();
  for (size_t i = 0; i < n; ++i) {
    Tensor h;
    const bool ok = read_lod_tensor(f, &h);
    if (!ok) {
      fclose(f);
      fail("load_combine: %s ends after %zu of %zu tensors", r.op.GetString("file_path").c_str(), i, n);
    }
    store(r, r.out("Out", i), h);
  }
  fclose(f);
}

}  // namespace

#define PA_ANY_KERNEL(name, fn) \
  PA_HOST_KERNEL(name, fn);     \
  PA_DEVICE_KERNEL(name, fn)
PA_ANY_KERNEL(save, k_save);
PA_ANY_KERNEL(save_combine, k_save_combine);
PA_ANY_KERNEL(load, k_load);
PA_ANY_KERNEL(load_combine, k_load_combine);
#undef PA_ANY_KERNEL

void link_io_kernels() {}

}  // namespace pa
