// Public C++ inference API of paddle_amd (libpaddle_amd_native.so).
//
// Same surface as the reference's paddle/fluid/inference/api/paddle_inference_api.h
// (PaddleBuf / PaddleTensor / PaddlePredictor / NativeConfig /
// CreatePaddlePredictor), so C++ serving code written against it compiles here.
// The predictor is the native C++ executor (framework.h): it decodes the saved
// ``__model__`` ProgramDesc, loads the LoDTensor parameter files, and runs the
// block on host kernels or -- with ``use_gpu`` -- on gfx950 HIP kernels with the
// parameters resident in HBM.  No Python interpreter is involved.
#pragma once

#include <cassert>
#include <memory>
#include <string>
#include <vector>

namespace paddle {

enum PaddleDType {
  FLOAT32,
  INT64,
  INT32,  // extension
};

class PaddleBuf {
 public:
  PaddleBuf() = default;
  PaddleBuf(PaddleBuf&& other);
  explicit PaddleBuf(const PaddleBuf&);  // deep copy
  PaddleBuf& operator=(const PaddleBuf&);
  PaddleBuf& operator=(PaddleBuf&&);
  // does not own `data`
  PaddleBuf(void* data, size_t length) : data_(data), length_(length), memory_owned_{false} {}
  // owns a fresh buffer of `length` bytes
  explicit PaddleBuf(size_t length) : data_(new char[length]), length_(length), memory_owned_(true) {}
  void Resize(size_t length);
  void Reset(void* data, size_t length);
  bool empty() const { return length_ == 0; }
  void* data() const { return data_; }
  size_t length() const { return length_; }
  ~PaddleBuf() { Free(); }

 private:
  void Free();
  void* data_{nullptr};
  size_t length_{0};
  bool memory_owned_{true};
};

struct PaddleTensor {
  PaddleTensor() = default;
  std::string name;
  std::vector<int> shape;
  PaddleBuf data;
  PaddleDType dtype{FLOAT32};
  std::vector<std::vector<size_t>> lod;  // Tensor + LoD = LoDTensor
};

enum class PaddleEngineKind {
  kNative = 0,
  kAnakin,
  kAutoMixedTensorRT,
  kAnalysis,
};

class PaddlePredictor {
 public:
  struct Config;
  PaddlePredictor() = default;
  PaddlePredictor(const PaddlePredictor&) = delete;
  PaddlePredictor& operator=(const PaddlePredictor&) = delete;

  // Runs the model on `inputs`; fills `output_data` with the fetch targets in
  // fetch order (owned buffers).  Returns false (with the reason on stderr and in
  // LastError()) on failure.
  virtual bool Run(const std::vector<PaddleTensor>& inputs, std::vector<PaddleTensor>* output_data,
                   int batch_size = -1) = 0;
  // A predictor sharing this one's parameters; each clone may run on its own
  // thread concurrently with the others.
  virtual std::unique_ptr<PaddlePredictor> Clone() = 0;
  virtual ~PaddlePredictor() = default;

  struct Config {
    std::string model_dir;
  };
};

struct NativeConfig : public PaddlePredictor::Config {
  bool use_gpu{false};
  int device{0};
  float fraction_of_gpu_memory{-1.f};
  bool specify_input_name{false};
  std::string prog_file;
  std::string param_file;
};

// kAnalysis: the same predictor after the inference IR passes that the native
// executor applies itself (fc fusion of mul + elementwise_add).
struct AnalysisConfig : public NativeConfig {
  bool enable_ir_optim{true};
};

template <typename ConfigT, PaddleEngineKind engine = PaddleEngineKind::kNative>
std::unique_ptr<PaddlePredictor> CreatePaddlePredictor(const ConfigT& config);

int PaddleDtypeSize(PaddleDType dtype);
const std::string& LastError();

}  // namespace paddle
