// The legacy C-API function set (reference paddle/legacy/capi: Main.cpp, Matrix.cpp,
// Vector.cpp, Arguments.cpp, gradient_machine.cpp) over the native predictor of this
// library (api.cc: pa_nat_create / pa_nat_run / pa_nat_output / pa_nat_clone).  See
// paddle_capi.h for the model formats and the slot <-> feed-target mapping.
#include "paddle_capi.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <memory>
#include <string>
#include <vector>

extern "C" {
void* pa_nat_create(const char* model_dir, const char* prog_file, const char* param_file, int use_gpu, int device,
                    int ir_optim);
void* pa_nat_clone(void* h);
void pa_nat_destroy(void* h);
int pa_nat_run(void* h, int n, const int* dtypes, const int* ndims, const int64_t* dims, const void* const* data,
               const int64_t* lod, const int* lod_len);
int pa_nat_output(void* h, int i, int* dtype, int* ndim, int64_t* dims, int dims_cap, const void** data,
                  size_t* nbytes);
const char* pa_nat_last_error();
}

namespace {

bool g_use_gpu = false;
int g_gpu_id = 0;

using FBuf = std::shared_ptr<std::vector<float>>;
using IBuf = std::shared_ptr<std::vector<int>>;

struct Mat {
  FBuf buf;
  uint64_t h = 0, w = 0;
};
struct IVec {
  IBuf buf;
};
struct Slot {
  FBuf val;
  uint64_t h = 0, w = 0;
  IBuf ids;
  IBuf seq[2];
  uint64_t fh = 0, fw = 0;
};
struct Args {
  std::vector<Slot> slots;
};
struct Machine {
  void* pred = nullptr;
  std::string tmp;   // private directory holding the program (and merged parameters)
  std::string prog;  // program file inside tmp
  ~Machine() {
    if (pred) pa_nat_destroy(pred);
    if (!tmp.empty()) {
      unlink((tmp + "/__model__").c_str());
      unlink((tmp + "/params").c_str());
      rmdir(tmp.c_str());
    }
  }
};

bool write_file(const std::string& path, const void* data, size_t n) {
  FILE* f = fopen(path.c_str(), "wb");
  if (!f) return false;
  const bool ok = fwrite(data, 1, n, f) == n;
  return fclose(f) == 0 && ok;
}

Machine* new_machine(const void* prog, size_t n) {
  auto m = std::make_unique<Machine>();
  char tmpl[] = "/tmp/paddle_capi_XXXXXX";
  if (!mkdtemp(tmpl)) return nullptr;
  m->tmp = tmpl;
  m->prog = m->tmp + "/__model__";
  if (!write_file(m->prog, prog, n)) return nullptr;
  return m.release();
}

}  // namespace

extern "C" {

PD_API const char* paddle_error_string(paddle_error err) {
  switch (err) {
    case kPD_NO_ERROR: return "no error";
    case kPD_NULLPTR: return "null pointer";
    case kPD_OUT_OF_RANGE: return "out of range";
    case kPD_PROTOBUF_ERROR: return "protobuf / model error";
    case kPD_NOT_SUPPORTED: return "not supported";
    default: return "undefined error";
  }
}

PD_API paddle_error paddle_init(int argc, char** argv) {
  for (int i = 0; i < argc; ++i) {
    if (!argv || !argv[i]) continue;
    const char* a = argv[i];
    if (!strncmp(a, "--use_gpu=", 10)) g_use_gpu = !strcmp(a + 10, "true") || !strcmp(a + 10, "1") ||
                                                   !strcmp(a + 10, "True");
    else if (!strncmp(a, "--gpu_id=", 9)) g_gpu_id = atoi(a + 9);
  }
  return kPD_NO_ERROR;
}

PD_API paddle_error paddle_init_thread() { return kPD_NO_ERROR; }

// ------------------------------------------------------------------ matrix
PD_API paddle_matrix paddle_matrix_create(uint64_t height, uint64_t width, bool useGpu) {
  (void)useGpu;  // host buffers; the predictor moves them to the device it runs on
  auto* m = new Mat();
  m->h = height;
  m->w = width;
  m->buf = std::make_shared<std::vector<float>>(height * width, 0.f);
  return m;
}

PD_API paddle_matrix paddle_matrix_create_none() { return new Mat(); }

PD_API paddle_matrix paddle_matrix_create_sparse(uint64_t, uint64_t, uint64_t, bool, bool) { return nullptr; }

PD_API paddle_error paddle_matrix_destroy(paddle_matrix mat) {
  if (!mat) return kPD_NULLPTR;
  delete static_cast<Mat*>(mat);
  return kPD_NO_ERROR;
}

PD_API paddle_error paddle_matrix_set_row(paddle_matrix mat, uint64_t rowID, paddle_real* rowArray) {
  auto* m = static_cast<Mat*>(mat);
  if (!m || !rowArray || !m->buf) return kPD_NULLPTR;
  if (rowID >= m->h) return kPD_OUT_OF_RANGE;
  memcpy(m->buf->data() + rowID * m->w, rowArray, m->w * sizeof(float));
  return kPD_NO_ERROR;
}

PD_API paddle_error paddle_matrix_set_value(paddle_matrix mat, paddle_real* value) {
  auto* m = static_cast<Mat*>(mat);
  if (!m || !value || !m->buf) return kPD_NULLPTR;
  memcpy(m->buf->data(), value, m->h * m->w * sizeof(float));
  return kPD_NO_ERROR;
}

PD_API paddle_error paddle_matrix_get_row(paddle_matrix mat, uint64_t rowID, paddle_real** rawRowBuffer) {
  auto* m = static_cast<Mat*>(mat);
  if (!m || !rawRowBuffer || !m->buf) return kPD_NULLPTR;
  if (rowID >= m->h) return kPD_OUT_OF_RANGE;
  *rawRowBuffer = m->buf->data() + rowID * m->w;
  return kPD_NO_ERROR;
}

PD_API paddle_error paddle_matrix_get_value(paddle_matrix mat, paddle_real* result) {
  auto* m = static_cast<Mat*>(mat);
  if (!m || !result || !m->buf) return kPD_NULLPTR;
  memcpy(result, m->buf->data(), m->h * m->w * sizeof(float));
  return kPD_NO_ERROR;
}

PD_API paddle_error paddle_matrix_get_shape(paddle_matrix mat, uint64_t* height, uint64_t* width) {
  auto* m = static_cast<Mat*>(mat);
  if (!m || !height || !width) return kPD_NULLPTR;
  *height = m->h;
  *width = m->w;
  return kPD_NO_ERROR;
}

PD_API paddle_error paddle_matrix_sparse_copy_from(paddle_matrix, int*, uint64_t, int*, uint64_t, float*, uint64_t) {
  return kPD_NOT_SUPPORTED;  // sparse input matrices: feed ids + sequence positions instead
}

// ------------------------------------------------------------------ ivector
PD_API paddle_ivector paddle_ivector_create_none() {
  auto* v = new IVec();
  v->buf = std::make_shared<std::vector<int>>();
  return v;
}

PD_API paddle_ivector paddle_ivector_create(int* array, uint64_t size, bool copy, bool useGPU) {
  (void)copy;  // always a private copy: later writes to `array` are not seen
  (void)useGPU;
  if (!array && size) return nullptr;
  auto* v = new IVec();
  v->buf = std::make_shared<std::vector<int>>(array, array + size);
  return v;
}

PD_API paddle_error paddle_ivector_destroy(paddle_ivector ivec) {
  if (!ivec) return kPD_NULLPTR;
  delete static_cast<IVec*>(ivec);
  return kPD_NO_ERROR;
}

PD_API paddle_error paddle_ivector_get(paddle_ivector ivec, int** buffer) {
  auto* v = static_cast<IVec*>(ivec);
  if (!v || !buffer || !v->buf) return kPD_NULLPTR;
  *buffer = v->buf->data();
  return kPD_NO_ERROR;
}

PD_API paddle_error paddle_ivector_resize(paddle_ivector ivec, uint64_t size) {
  auto* v = static_cast<IVec*>(ivec);
  if (!v || !v->buf) return kPD_NULLPTR;
  v->buf->resize(size);
  return kPD_NO_ERROR;
}

PD_API paddle_error paddle_ivector_get_size(paddle_ivector ivec, uint64_t* size) {
  auto* v = static_cast<IVec*>(ivec);
  if (!v || !size || !v->buf) return kPD_NULLPTR;
  *size = v->buf->size();
  return kPD_NO_ERROR;
}

// ------------------------------------------------------------------ arguments
PD_API paddle_arguments paddle_arguments_create_none() { return new Args(); }

PD_API paddle_error paddle_arguments_destroy(paddle_arguments args) {
  if (!args) return kPD_NULLPTR;
  delete static_cast<Args*>(args);
  return kPD_NO_ERROR;
}

PD_API paddle_error paddle_arguments_get_size(paddle_arguments args, uint64_t* size) {
  auto* a = static_cast<Args*>(args);
  if (!a || !size) return kPD_NULLPTR;
  *size = a->slots.size();
  return kPD_NO_ERROR;
}

PD_API paddle_error paddle_arguments_resize(paddle_arguments args, uint64_t size) {
  auto* a = static_cast<Args*>(args);
  if (!a) return kPD_NULLPTR;
  a->slots.resize(size);
  return kPD_NO_ERROR;
}

#define PD_SLOT(args, ID)                                  \
  auto* a_ = static_cast<Args*>(args);                     \
  if (!a_) return kPD_NULLPTR;                             \
  if (ID >= a_->slots.size()) return kPD_OUT_OF_RANGE;     \
  Slot& s = a_->slots[ID]

PD_API paddle_error paddle_arguments_set_value(paddle_arguments args, uint64_t ID, paddle_matrix mat) {
  auto* m = static_cast<Mat*>(mat);
  if (!m) return kPD_NULLPTR;
  PD_SLOT(args, ID);
  s.val = m->buf;  // shared, as the reference's Argument::value
  s.h = m->h;
  s.w = m->w;
  return kPD_NO_ERROR;
}

PD_API paddle_error paddle_arguments_get_value(paddle_arguments args, uint64_t ID, paddle_matrix mat) {
  auto* m = static_cast<Mat*>(mat);
  if (!m) return kPD_NULLPTR;
  PD_SLOT(args, ID);
  if (!s.val) return kPD_NULLPTR;
  m->buf = s.val;
  m->h = s.h;
  m->w = s.w;
  return kPD_NO_ERROR;
}

PD_API paddle_error paddle_arguments_get_prob(paddle_arguments args, uint64_t ID, paddle_matrix mat) {
  return paddle_arguments_get_value(args, ID, mat);
}

PD_API paddle_error paddle_arguments_get_ids(paddle_arguments args, uint64_t ID, paddle_ivector ids) {
  auto* v = static_cast<IVec*>(ids);
  if (!v) return kPD_NULLPTR;
  PD_SLOT(args, ID);
  if (!s.ids) return kPD_NULLPTR;
  v->buf = s.ids;
  return kPD_NO_ERROR;
}

PD_API paddle_error paddle_arguments_set_ids(paddle_arguments args, uint64_t ID, paddle_ivector ids) {
  auto* v = static_cast<IVec*>(ids);
  if (!v) return kPD_NULLPTR;
  PD_SLOT(args, ID);
  s.ids = v->buf;
  return kPD_NO_ERROR;
}

PD_API paddle_error paddle_arguments_set_frame_shape(paddle_arguments args, uint64_t ID, uint64_t frameHeight,
                                                     uint64_t frameWidth) {
  PD_SLOT(args, ID);
  s.fh = frameHeight;
  s.fw = frameWidth;
  return kPD_NO_ERROR;
}

PD_API paddle_error paddle_arguments_set_sequence_start_pos(paddle_arguments args, uint64_t ID, uint32_t nestedLevel,
                                                            paddle_ivector seqPos) {
  auto* v = static_cast<IVec*>(seqPos);
  if (!v) return kPD_NULLPTR;
  if (nestedLevel > 1) return kPD_OUT_OF_RANGE;
  PD_SLOT(args, ID);
  s.seq[nestedLevel] = v->buf;
  return kPD_NO_ERROR;
}

PD_API paddle_error paddle_arguments_get_sequence_start_pos(paddle_arguments args, uint64_t ID, uint32_t nestedLevel,
                                                            paddle_ivector seqPos) {
  auto* v = static_cast<IVec*>(seqPos);
  if (!v) return kPD_NULLPTR;
  if (nestedLevel > 1) return kPD_OUT_OF_RANGE;
  PD_SLOT(args, ID);
  if (!s.seq[nestedLevel]) return kPD_NULLPTR;
  v->buf = s.seq[nestedLevel];
  return kPD_NO_ERROR;
}

// ------------------------------------------------------------------ gradient machine
PD_API paddle_error paddle_gradient_machine_create_for_inference(paddle_gradient_machine* machine,
                                                                 void* modelConfigProtobuf, int size) {
  if (!machine || !modelConfigProtobuf || size <= 0) return kPD_NULLPTR;
  Machine* m = new_machine(modelConfigProtobuf, (size_t)size);
  if (!m) return kPD_UNDEFINED_ERROR;
  *machine = m;
  return kPD_NO_ERROR;
}

PD_API paddle_error paddle_gradient_machine_load_parameter_from_disk(paddle_gradient_machine machine,
                                                                     const char* path) {
  auto* m = static_cast<Machine*>(machine);
  if (!m || !path) return kPD_NULLPTR;
  // a directory of per-variable files, or one combined parameter file
  const bool is_dir = access((std::string(path) + "/.").c_str(), F_OK) == 0;
  void* p = is_dir ? pa_nat_create(path, m->prog.c_str(), "", g_use_gpu, g_gpu_id, 0)
                   : pa_nat_create(m->tmp.c_str(), m->prog.c_str(), path, g_use_gpu, g_gpu_id, 0);
  if (!p) {
    fprintf(stderr, "paddle_capi: %s\n", pa_nat_last_error());
    return kPD_PROTOBUF_ERROR;
  }
  if (m->pred) pa_nat_destroy(m->pred);
  m->pred = p;
  return kPD_NO_ERROR;
}

PD_API paddle_error paddle_gradient_machine_create_for_inference_with_parameters(paddle_gradient_machine* machine,
                                                                                 void* mergedModel, uint64_t size) {
  if (!machine || !mergedModel) return kPD_NULLPTR;
  const char* b = static_cast<const char*>(mergedModel);
  uint64_t plen = 0, qlen = 0;
  if (size < 24 || memcmp(b, "PAMERGE1", 8) != 0) return kPD_PROTOBUF_ERROR;
  memcpy(&plen, b + 8, 8);
  if (plen > size - 24) return kPD_PROTOBUF_ERROR;
  memcpy(&qlen, b + 16 + plen, 8);
  if (qlen > size - 24 - plen) return kPD_PROTOBUF_ERROR;
  Machine* m = new_machine(b + 16, plen);
  if (!m) return kPD_UNDEFINED_ERROR;
  const std::string params = m->tmp + "/params";
  if (!write_file(params, b + 24 + plen, qlen)) {
    delete m;
    return kPD_UNDEFINED_ERROR;
  }
  const paddle_error e = paddle_gradient_machine_load_parameter_from_disk(m, params.c_str());
  if (e != kPD_NO_ERROR) {
    delete m;
    return e;
  }
  *machine = m;
  return kPD_NO_ERROR;
}

PD_API paddle_error paddle_gradient_machine_forward(paddle_gradient_machine machine, paddle_arguments inArgs,
                                                    paddle_arguments outArgs, bool isTrain) {
  auto* m = static_cast<Machine*>(machine);
  auto* in = static_cast<Args*>(inArgs);
  auto* out = static_cast<Args*>(outArgs);
  if (!m || !in || !out) return kPD_NULLPTR;
  if (isTrain) return kPD_NOT_SUPPORTED;  // inference machines
  if (!m->pred) return kPD_NULLPTR;       // parameters were never loaded
  const int n = (int)in->slots.size();
  std::vector<int> dtypes(n), ndims(n), lod_len(n, 0);
  std::vector<int64_t> dims, lod;
  std::vector<const void*> data(n);
  std::vector<std::vector<int64_t>> ids64(n);
  for (int i = 0; i < n; ++i) {
    const Slot& s = in->slots[i];
    if (s.val) {
      dtypes[i] = 0;  // FLOAT32
      if (s.fh && s.fw && s.w == s.fh * s.fw) {  // image-shaped input: [h, 1, fh, fw]... as NCHW with C = 1
        ndims[i] = 4;
        dims.insert(dims.end(), {(int64_t)s.h, 1, (int64_t)s.fh, (int64_t)s.fw});
      } else {
        ndims[i] = 2;
        dims.insert(dims.end(), {(int64_t)s.h, (int64_t)s.w});
      }
      data[i] = s.val->data();
    } else if (s.ids) {
      dtypes[i] = 1;  // INT64 ids [n, 1]
      ids64[i].assign(s.ids->begin(), s.ids->end());
      ndims[i] = 2;
      dims.insert(dims.end(), {(int64_t)ids64[i].size(), 1});
      data[i] = ids64[i].data();
    } else {
      return kPD_NULLPTR;
    }
    if (s.seq[0]) {
      lod_len[i] = (int)s.seq[0]->size();
      lod.insert(lod.end(), s.seq[0]->begin(), s.seq[0]->end());
    }
  }
  const int nout = pa_nat_run(m->pred, n, dtypes.data(), ndims.data(), dims.data(), data.data(), lod.data(),
                              lod_len.data());
  if (nout < 0) {
    fprintf(stderr, "paddle_capi: %s\n", pa_nat_last_error());
    return kPD_UNDEFINED_ERROR;
  }
  out->slots.assign((size_t)nout, Slot());
  for (int i = 0; i < nout; ++i) {
    int dt = 0, nd = 0;
    int64_t od[16];
    const void* p = nullptr;
    size_t nb = 0;
    if (pa_nat_output(m->pred, i, &dt, &nd, od, 16, &p, &nb) != 0) return kPD_OUT_OF_RANGE;
    Slot& s = out->slots[(size_t)i];
    const int64_t rows = nd ? od[0] : 1;
    if (dt == 0) {
      s.val = std::make_shared<std::vector<float>>(nb / 4);
      memcpy(s.val->data(), p, nb);
      s.h = (uint64_t)rows;
      s.w = rows ? (uint64_t)(nb / 4) / (uint64_t)rows : 0;
    } else {  // integer outputs (e.g. argmax ids) come back as ids
      s.ids = std::make_shared<std::vector<int>>();
      if (dt == 1)
        for (size_t k = 0; k < nb / 8; ++k) s.ids->push_back((int)static_cast<const int64_t*>(p)[k]);
      else
        s.ids->assign(static_cast<const int*>(p), static_cast<const int*>(p) + nb / 4);
    }
  }
  return kPD_NO_ERROR;
}

PD_API paddle_error paddle_gradient_machine_create_shared_param(paddle_gradient_machine origin,
                                                                void* modelConfigProtobuf, int size,
                                                                paddle_gradient_machine* slave) {
  auto* o = static_cast<Machine*>(origin);
  if (!o || !slave || !o->pred) return kPD_NULLPTR;
  (void)modelConfigProtobuf;
  (void)size;  // the clone runs the origin's program on its parameters (api Clone)
  auto* m = new Machine();
  m->pred = pa_nat_clone(o->pred);
  *slave = m;
  return kPD_NO_ERROR;
}

PD_API paddle_error paddle_gradient_machine_randomize_param(paddle_gradient_machine machine) {
  return machine ? kPD_NOT_SUPPORTED : kPD_NULLPTR;  // inference machines load trained parameters
}

PD_API paddle_error paddle_gradient_machine_destroy(paddle_gradient_machine machine) {
  if (!machine) return kPD_NULLPTR;
  delete static_cast<Machine*>(machine);
  return kPD_NO_ERROR;
}

PD_API paddle_error paddle_gradient_machine_get_layer_output(paddle_gradient_machine machine, const char* layerName,
                                                             paddle_arguments args) {
  (void)layerName;
  (void)args;
  return machine ? kPD_NOT_SUPPORTED : kPD_NULLPTR;  // only the program's fetch targets are outputs
}

PD_API paddle_error paddle_gradient_machine_release_layer_output(paddle_gradient_machine machine) {
  return machine ? kPD_NO_ERROR : kPD_NULLPTR;
}

}  // extern "C"
