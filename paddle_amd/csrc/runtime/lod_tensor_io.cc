// LoDTensor stream serialisation in C++ (reference: framework/lod_tensor.cc:251-304,
// tensor_util.cc TensorToStream).  Used for large checkpoints: streams host
// buffers straight to the file (no intermediate Python bytes objects).
//
//   LoDTensor := u32 0 | u64 lod_level | lod_level x (u64 nbytes | u64[])  | Tensor
//   Tensor    := u32 0 | i32 desc_size | TensorDesc proto | raw data
//   TensorDesc proto: field 1 varint data_type, field 2 repeated int64 dims
//   (proto2, unpacked: one (tag 0x10, varint) per dim).
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "runtime.h"

namespace {
void put_varint(std::string& s, uint64_t v) {
  while (v >= 0x80) {
    s.push_back((char)(v | 0x80));
    v >>= 7;
  }
  s.push_back((char)v);
}

bool get_varint(const unsigned char*& p, const unsigned char* end, uint64_t& v) {
  v = 0;
  int shift = 0;
  while (p < end && shift < 64) {
    uint8_t b = *p++;
    v |= (uint64_t)(b & 0x7f) << shift;
    if (!(b & 0x80)) return true;
    shift += 7;
  }
  return false;
}
}  // namespace

PA_RT_EXPORT void* pa_ts_open(const char* path, int write, int append) {
  FILE* f = fopen(path, write ? (append ? "ab" : "wb") : "rb");
  if (!f) pa_rt_set_error("cannot open %s", path);
  return f;
}

PA_RT_EXPORT int pa_ts_close(void* h) { return fclose((FILE*)h); }

// lod: lod_level arrays given as one flat u64 array + per-level lengths.
PA_RT_EXPORT int pa_ts_write_lod_tensor(void* h, int lod_level, const uint64_t* lod_flat,
                                        const int64_t* lod_lens, int dtype, int ndims,
                                        const int64_t* dims, const void* data, size_t nbytes) {
  FILE* f = (FILE*)h;
  uint32_t ver = 0;
  uint64_t ll = (uint64_t)lod_level;
  fwrite(&ver, 4, 1, f);
  fwrite(&ll, 8, 1, f);
  const uint64_t* p = lod_flat;
  for (int i = 0; i < lod_level; ++i) {
    uint64_t nb = (uint64_t)lod_lens[i] * 8;
    fwrite(&nb, 8, 1, f);
    fwrite(p, 8, (size_t)lod_lens[i], f);
    p += lod_lens[i];
  }
  std::string desc;
  desc.push_back(0x08);
  put_varint(desc, (uint64_t)dtype);
  for (int i = 0; i < ndims; ++i) {
    desc.push_back(0x10);
    put_varint(desc, (uint64_t)dims[i]);
  }
  int32_t dsz = (int32_t)desc.size();
  fwrite(&ver, 4, 1, f);
  fwrite(&dsz, 4, 1, f);
  fwrite(desc.data(), 1, desc.size(), f);
  // stream in 64 MB pieces (reference copies GPU tensors out in 64 MB chunks)
  const char* d = (const char*)data;
  size_t left = nbytes;
  while (left) {
    size_t n = left < (64u << 20) ? left : (64u << 20);
    if (fwrite(d, 1, n, f) != n) {
      pa_rt_set_error("short write");
      return -1;
    }
    d += n;
    left -= n;
  }
  return 0;
}

// Reads the header of the next LoDTensor.  Caller passes capacity-bounded arrays:
// lod_lens holds lod_levels_cap levels, lod_flat lod_cap offsets, dims dims_cap
// dims.  Every length read from the file is validated against those capacities
// and against sane limits before it is used (a checkpoint is untrusted input);
// nothing throws across the C ABI.  Returns the data byte count via *nbytes; the
// payload is then read with pa_ts_read_data.  Returns 1 = ok, 0 = EOF, -1 = error.
static constexpr int32_t kMaxDescBytes = 1 << 16;  // a TensorDesc is a few dozen bytes

PA_RT_EXPORT int pa_ts_read_header(void* h, int* lod_level, uint64_t* lod_flat, int64_t* lod_lens,
                                   int lod_levels_cap, int lod_cap, int* dtype, int* ndims,
                                   int64_t* dims, int dims_cap, size_t* nbytes,
                                   int elem_size_by_dtype[32]) {
  try {
    FILE* f = (FILE*)h;
    uint32_t ver;
    size_t got = fread(&ver, 1, 4, f);
    if (got == 0) return 0;  // clean end of stream
    if (got != 4) {
      pa_rt_set_error("truncated tensor header");
      return -1;
    }
    uint64_t ll;
    if (fread(&ll, 8, 1, f) != 1) return -1;
    if (ll > (uint64_t)lod_levels_cap) {
      pa_rt_set_error("lod_level %llu exceeds capacity %d", (unsigned long long)ll, lod_levels_cap);
      return -1;
    }
    *lod_level = (int)ll;
    uint64_t* p = lod_flat;
    int64_t used = 0;
    for (uint64_t i = 0; i < ll; ++i) {
      uint64_t nb;
      if (fread(&nb, 8, 1, f) != 1) return -1;
      if (nb % 8 != 0 || nb / 8 > (uint64_t)lod_cap) {
        pa_rt_set_error("bad lod level byte count %llu", (unsigned long long)nb);
        return -1;
      }
      int64_t n = (int64_t)(nb / 8);
      if (used + n > lod_cap) {
        pa_rt_set_error("lod capacity exceeded");
        return -1;
      }
      if (fread(p, 8, (size_t)n, f) != (size_t)n) return -1;
      lod_lens[i] = n;
      p += n;
      used += n;
    }
    int32_t dsz;
    if (fread(&ver, 4, 1, f) != 1 || fread(&dsz, 4, 1, f) != 1) return -1;
    if (dsz < 0 || dsz > kMaxDescBytes) {
      pa_rt_set_error("bad TensorDesc size %d", dsz);
      return -1;
    }
    std::vector<unsigned char> desc((size_t)dsz);
    if (fread(desc.data(), 1, desc.size(), f) != desc.size()) return -1;
    const unsigned char* q = desc.data();
    const unsigned char* end = q + desc.size();
    int nd = 0;
    *dtype = 5;
    auto push_dim = [&](uint64_t v) {
      if (nd >= dims_cap) {
        pa_rt_set_error("tensor rank exceeds capacity %d", dims_cap);
        return false;
      }
      if (v > ((uint64_t)1 << 48)) {
        pa_rt_set_error("implausible dim %llu", (unsigned long long)v);
        return false;
      }
      dims[nd++] = (int64_t)v;
      return true;
    };
    while (q < end) {
      uint64_t tag, v;
      if (!get_varint(q, end, tag)) return -1;
      if ((tag >> 3) == 1) {
        if (!get_varint(q, end, v)) return -1;
        *dtype = (int)v;
      } else if ((tag >> 3) == 2 && (tag & 7) == 0) {
        if (!get_varint(q, end, v) || !push_dim(v)) return -1;
      } else if ((tag >> 3) == 2 && (tag & 7) == 2) {  // packed
        uint64_t len;
        if (!get_varint(q, end, len)) return -1;
        if (len > (uint64_t)(end - q)) {
          pa_rt_set_error("packed dims run past the TensorDesc");
          return -1;
        }
        const unsigned char* pe = q + len;
        while (q < pe) {
          if (!get_varint(q, pe, v) || !push_dim(v)) return -1;
        }
      } else {
        pa_rt_set_error("unexpected TensorDesc field");
        return -1;
      }
    }
    *ndims = nd;
    int es = (*dtype >= 0 && *dtype < 32) ? elem_size_by_dtype[*dtype] : 0;
    if (es <= 0) {
      pa_rt_set_error("unknown dtype %d", *dtype);
      return -1;
    }
    unsigned __int128 total = (unsigned __int128)es;
    for (int i = 0; i < nd; ++i) {
      total *= (uint64_t)dims[i];
      if (total > ((unsigned __int128)1 << 46)) {  // 64 TiB: no real tensor is this large
        pa_rt_set_error("tensor byte count overflows");
        return -1;
      }
    }
    *nbytes = (size_t)total;
    return 1;
  } catch (...) {
    pa_rt_set_error("exception while reading tensor header");
    return -1;
  }
}

PA_RT_EXPORT int pa_ts_read_data(void* h, void* dst, size_t nbytes) {
  return fread(dst, 1, nbytes, (FILE*)h) == nbytes ? 0 : -1;
}
