// RecordIO chunked record files (reference: paddle/fluid/recordio/{header,chunk,writer,
// scanner}.cc).  On-disk layout per chunk:
//   u32 magic 0x01020304 | u32 num_records | u32 crc32(payload) | u32 compressor |
//   u32 payload_size | payload
// payload (after decompression) = num_records x (u32 len | bytes).
// Compressors: 0 none, 2 zlib/gzip.  (1 = snappy is not available in this
// image; writers asked for it emit zlib and record compressor 2.)
#include <stdarg.h>
#include <stdio.h>
#include <string.h>
#include <zlib.h>

#include <mutex>
#include <string>
#include <vector>

#include "runtime.h"

static thread_local std::string g_err;

PA_RT_EXPORT const char* pa_rt_last_error() { return g_err.c_str(); }

void pa_rt_set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
}

namespace {
constexpr uint32_t kMagic = 0x01020304;

struct Writer {
  FILE* f = nullptr;
  uint32_t compressor = 0;
  uint32_t max_records = 1000;
  std::vector<std::string> records;
  size_t bytes = 0;
};

bool flush_chunk(Writer* w) {
  if (w->records.empty()) return true;
  std::string raw;
  raw.reserve(w->bytes + 4 * w->records.size());
  for (auto& r : w->records) {
    uint32_t n = (uint32_t)r.size();
    raw.append((const char*)&n, 4);
    raw.append(r);
  }
  std::string payload;
  if (w->compressor == 2) {
    uLongf cap = compressBound(raw.size());
    payload.resize(cap);
    if (compress2((Bytef*)&payload[0], &cap, (const Bytef*)raw.data(), raw.size(), Z_DEFAULT_COMPRESSION) != Z_OK) {
      pa_rt_set_error("zlib compress failed");
      return false;
    }
    payload.resize(cap);
  } else {
    payload.swap(raw);
  }
  uint32_t crc = (uint32_t)crc32(0, (const Bytef*)payload.data(), (uInt)payload.size());
  uint32_t hdr[5] = {kMagic, (uint32_t)w->records.size(), crc, w->compressor, (uint32_t)payload.size()};
  if (fwrite(hdr, 4, 5, w->f) != 5 || fwrite(payload.data(), 1, payload.size(), w->f) != payload.size()) {
    pa_rt_set_error("short write");
    return false;
  }
  w->records.clear();
  w->bytes = 0;
  return true;
}

struct Scanner {
  FILE* f = nullptr;
  std::string chunk;  // decompressed payload of the current chunk
  size_t pos = 0;
  uint32_t left = 0;
  std::string cur;
};

bool load_chunk(Scanner* s) {
  uint32_t hdr[5];
  size_t got = fread(hdr, 4, 5, s->f);
  if (got == 0) return false;
  if (got != 5 || hdr[0] != kMagic) {
    pa_rt_set_error("bad recordio chunk header");
    return false;
  }
  std::string payload(hdr[4], '\0');
  if (fread(&payload[0], 1, hdr[4], s->f) != hdr[4]) {
    pa_rt_set_error("truncated recordio chunk");
    return false;
  }
  uint32_t crc = (uint32_t)crc32(0, (const Bytef*)payload.data(), (uInt)payload.size());
  if (crc != hdr[2]) {
    pa_rt_set_error("recordio checksum mismatch");
    return false;
  }
  if (hdr[3] == 2) {
    // unknown raw size: grow until it fits
    uLongf cap = payload.size() * 4 + 1024;
    for (int i = 0; i < 16; ++i) {
      s->chunk.resize(cap);
      uLongf n = cap;
      int rc = uncompress((Bytef*)&s->chunk[0], &n, (const Bytef*)payload.data(), payload.size());
      if (rc == Z_OK) {
        s->chunk.resize(n);
        break;
      }
      if (rc != Z_BUF_ERROR) {
        pa_rt_set_error("zlib uncompress failed");
        return false;
      }
      cap *= 4;
    }
  } else if (hdr[3] == 0) {
    s->chunk.swap(payload);
  } else {
    pa_rt_set_error("unsupported recordio compressor %u", hdr[3]);
    return false;
  }
  s->pos = 0;
  s->left = hdr[1];
  return true;
}
}  // namespace

PA_RT_EXPORT void* pa_rio_writer_open(const char* path, int compressor, int max_records) {
  Writer* w = new Writer();
  w->f = fopen(path, "wb");
  if (!w->f) {
    pa_rt_set_error("cannot open %s", path);
    delete w;
    return nullptr;
  }
  w->compressor = compressor == 0 ? 0 : 2;
  w->max_records = max_records > 0 ? max_records : 1000;
  return w;
}

PA_RT_EXPORT int pa_rio_writer_write(void* h, const char* data, size_t len) {
  Writer* w = (Writer*)h;
  w->records.emplace_back(data, len);
  w->bytes += len;
  if (w->records.size() >= w->max_records) return flush_chunk(w) ? 0 : -1;
  return 0;
}

PA_RT_EXPORT int pa_rio_writer_close(void* h) {
  Writer* w = (Writer*)h;
  bool ok = flush_chunk(w);
  fclose(w->f);
  delete w;
  return ok ? 0 : -1;
}

PA_RT_EXPORT void* pa_rio_scanner_open(const char* path) {
  Scanner* s = new Scanner();
  s->f = fopen(path, "rb");
  if (!s->f) {
    pa_rt_set_error("cannot open %s", path);
    delete s;
    return nullptr;
  }
  return s;
}

// Returns 1 and sets *data/*len on a record, 0 at EOF, -1 on error.  The buffer
// is owned by the scanner and valid until the next call.
PA_RT_EXPORT int pa_rio_scanner_next(void* h, const char** data, size_t* len) {
  Scanner* s = (Scanner*)h;
  while (s->left == 0) {
    g_err.clear();
    if (!load_chunk(s)) return g_err.empty() ? 0 : -1;
  }
  uint32_t n;
  memcpy(&n, s->chunk.data() + s->pos, 4);
  s->pos += 4;
  *data = s->chunk.data() + s->pos;
  *len = n;
  s->pos += n;
  s->left--;
  return 1;
}

PA_RT_EXPORT void pa_rio_scanner_close(void* h) {
  Scanner* s = (Scanner*)h;
  if (s->f) fclose(s->f);
  delete s;
}
