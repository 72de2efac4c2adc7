// Native C++ executor core: ProgramDesc (decoded from the wire format of the
// reference's framework.proto), tensors, scopes, the op-kernel registry and the
// block executor.  No Python, no torch: a C++ program links libpaddle_amd_native.so
// and runs saved programs (inference models, the training demo) directly.
//
// Reference parity: framework/{program_desc,block_desc,op_desc,var_desc}.h (desc
// objects), framework/{tensor,lod_tensor,scope,variable}.h, framework/executor.cc:125
// (Executor::Run: create block vars, run ops in order), op_registry.h (kernel lookup
// by op type + place).
//
// MI355X-first: tensors carry a device id (-1 = host); device tensors live in HBM
// (hipMalloc) and device kernels run on one HIP stream per executor context
// (ops_gpu.hip).  Host kernels run on a persistent worker pool (parallel_for).
#pragma once

#include <stdint.h>

#include <atomic>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace pa {

// ---------------------------------------------------------------- errors
struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};
[[noreturn]] void fail(const char* fmt, ...);
// Thrown by a device kernel (before it touches any output) for a configuration it
// does not cover; the executor runs the op's host kernel instead.
struct Decline {};
#define PA_CHECK(cond, ...) \
  do {                      \
    if (!(cond)) ::pa::fail(__VA_ARGS__); \
  } while (0)

// ---------------------------------------------------------------- dtypes
// VarType.Type values of framework.proto
enum class DT : int {
  BOOL = 0, INT16 = 1, INT32 = 2, INT64 = 3, FP16 = 4, FP32 = 5, FP64 = 6,
  UINT8 = 20, INT8 = 21, BF16 = 22,
};
size_t dt_size(DT t);
const char* dt_name(DT t);

// ---------------------------------------------------------------- program desc
enum AttrType { A_INT = 0, A_FLOAT, A_STRING, A_INTS, A_FLOATS, A_STRINGS, A_BOOLEAN, A_BOOLEANS,
                A_BLOCK, A_LONG, A_BLOCKS };

struct Attr {
  std::string name;
  int type = A_INT;
  int64_t i = 0;  // INT / LONG / BOOLEAN / BLOCK
  float f = 0.f;
  std::string s;
  std::vector<int64_t> ints;  // INTS / BOOLEANS / BLOCKS
  std::vector<float> floats;
  std::vector<std::string> strings;
};

// VarType.Type values that are not tensors
enum VarKind { VK_LOD_TENSOR = 7, VK_SELECTED_ROWS = 8, VK_FEED_MINIBATCH = 9, VK_FETCH_LIST = 10,
               VK_STEP_SCOPES = 11, VK_LOD_RANK_TABLE = 12, VK_LOD_TENSOR_ARRAY = 13, VK_READER = 15,
               VK_RAW = 17 };

struct VarDesc {
  std::string name;
  int type = VK_LOD_TENSOR;
  DT dtype = DT::FP32;
  std::vector<int64_t> dims;
  int lod_level = 0;
  bool persistable = false;
};

struct OpDesc {
  std::string type;
  std::vector<std::pair<std::string, std::vector<std::string>>> inputs, outputs;
  std::map<std::string, Attr> attrs;

  const std::vector<std::string>& Inputs(const std::string& slot) const;
  const std::vector<std::string>& Outputs(const std::string& slot) const;
  std::string Input(const std::string& slot) const;   // first argument or ""
  std::string Output(const std::string& slot) const;  // first argument or ""
  bool Has(const std::string& a) const { return attrs.count(a) != 0; }
  int64_t GetInt(const std::string& a, int64_t def = 0) const;
  float GetFloat(const std::string& a, float def = 0.f) const;
  bool GetBool(const std::string& a, bool def = false) const;
  std::string GetString(const std::string& a, const std::string& def = "") const;
  std::vector<int64_t> GetInts(const std::string& a) const;
  std::vector<float> GetFloats(const std::string& a) const;
};

struct BlockDesc {
  int idx = 0, parent_idx = -1, forward_block_idx = -1;
  std::vector<VarDesc> vars;
  std::vector<OpDesc> ops;
  const VarDesc* FindVar(const std::string& n) const;
};

struct ProgramDesc {
  std::vector<BlockDesc> blocks;
  // Decodes a serialized ProgramDesc (proto2 wire format); throws pa::Error on
  // malformed input (the file is untrusted: every length is bounds-checked).
  static ProgramDesc Parse(const std::string& bytes);
  static ProgramDesc Load(const std::string& path);
  const BlockDesc& Block(int i) const { return blocks.at(i); }
};

// ---------------------------------------------------------------- tensors
struct Buffer {
  void* ptr = nullptr;
  size_t bytes = 0;
  int device = -1;
  bool owned = true;  // false: memory lent by the embedder (e.g. a torch tensor), never freed here
  Buffer(size_t n, int dev);
  Buffer(void* p, size_t n, int dev) : ptr(p), bytes(n), device(dev), owned(false) {}
  ~Buffer();
  Buffer(const Buffer&) = delete;
  Buffer& operator=(const Buffer&) = delete;
};

using LoD = std::vector<std::vector<size_t>>;

struct Tensor {
  DT dtype = DT::FP32;
  std::vector<int64_t> dims;
  LoD lod;
  std::shared_ptr<Buffer> buf;
  int device = -1;

  int64_t numel() const;
  size_t nbytes() const { return (size_t)numel() * dt_size(dtype); }
  bool initialized() const { return buf != nullptr; }
  void* raw() const { return buf ? buf->ptr : nullptr; }
  template <class T> T* data() const { return static_cast<T*>(raw()); }
  // (Re)allocates when the existing buffer is too small or on another device;
  // keeps the buffer otherwise (steady-state runs reuse their memory).
  void* alloc(DT t, const std::vector<int64_t>& d, int dev);
  template <class T> T* alloc(const std::vector<int64_t>& d, int dev);
  void share(const Tensor& o) { *this = o; }  // same buffer, own dims/lod copies
  Tensor to(int dev, void* stream = nullptr) const;
  std::string shape_str() const;
};

// ---------------------------------------------------------------- variables / scopes
class Scope;

// lod_rank_table.h: one entry per sequence of the ranked LoD level, longest first
// (stable for equal lengths)
struct RankItem {
  int64_t index, length;
};

struct Variable {
  int kind = VK_LOD_TENSOR;
  Tensor tensor;             // LOD_TENSOR; SELECTED_ROWS: the value rows [rows.size(), ...]
  std::vector<Tensor> list;  // FEED_MINIBATCH / FETCH_LIST / LOD_TENSOR_ARRAY
  // SELECTED_ROWS (selected_rows.h): row indices into a [height, ...] dense table
  std::vector<int64_t> rows;
  int64_t height = 0;
  // LOD_RANK_TABLE: the ranked items and the LoD levels above the ranked one
  std::vector<RankItem> rank;
  LoD rank_coarse_lod;
  // STEP_SCOPES: the per-iteration child scopes of `steps_owner` a training `while`
  // keeps for its while_grad (while_op.cc kStepScopes); dropped when the loop reruns
  std::vector<Scope*> steps;
  Scope* steps_owner = nullptr;
};

class Scope {
 public:
  explicit Scope(const Scope* parent = nullptr) : parent_(parent) {}
  Variable* Var(const std::string& name);           // find or create locally
  Variable* Find(const std::string& name) const;    // walks up the parents
  Variable* FindLocal(const std::string& name) const;
  Scope& NewScope();
  void DropKid(Scope* kid);  // frees a child scope created by NewScope()
  void Erase(const std::string& name);
  std::vector<std::string> LocalNames() const;
  const Scope* parent() const { return parent_; }
  Scope& Root();  // the outermost ancestor (per-device workspaces live there)

 private:
  const Scope* parent_;
  std::unordered_map<std::string, std::unique_ptr<Variable>> vars_;
  std::vector<std::unique_ptr<Scope>> kids_;
  mutable std::mutex mu_;
};

// ---------------------------------------------------------------- execution context
struct ThreadPool;
ThreadPool& host_pool();
// Runs fn(begin, end) over [0, n) split across the host workers (serial when
// n < grain).
void parallel_for(int64_t n, int64_t grain, const std::function<void(int64_t, int64_t)>& fn);

struct ExecContext {
  int device = -1;        // -1 host, else HIP device id
  void* stream = nullptr;  // hipStream_t of the device kernels
  std::mt19937_64 rng{0x5eed};
  bool is_test = false;   // inference predictor: force is_test semantics
};

struct OpRun {
  const OpDesc& op;
  Scope& scope;
  ExecContext& ctx;
  Tensor& in(const std::string& slot, size_t i = 0) const;
  Tensor* in_opt(const std::string& slot, size_t i = 0) const;  // null if absent/uninitialised
  std::vector<Tensor*> ins(const std::string& slot) const;
  Tensor* out(const std::string& slot, size_t i = 0) const;      // null if the slot is empty
  Variable* var(const std::string& name) const;
  Variable* in_var(const std::string& slot, size_t i = 0) const;   // must exist
  Variable* out_var(const std::string& slot, size_t i = 0) const;  // found or created; null if empty
};

using Kernel = std::function<void(const OpRun&)>;
// device < 0: host kernel; device >= 0: HIP kernel
void register_kernel(const std::string& type, bool device, Kernel k);
const Kernel* find_kernel(const std::string& type, bool device);
std::vector<std::string> registered_ops(bool device);

struct KernelRegistrar {
  KernelRegistrar(const char* type, bool device, Kernel k) { register_kernel(type, device, std::move(k)); }
};
#define PA_HOST_KERNEL(name, fn) static ::pa::KernelRegistrar _pa_hk_##name(#name, false, fn)
#define PA_DEVICE_KERNEL(name, fn) static ::pa::KernelRegistrar _pa_dk_##name(#name, true, fn)

// forces the static registrars of every kernel translation unit to be linked
void link_host_kernels();
void link_device_kernels();
void link_control_kernels();
void link_rnn_kernels();
void link_struct_kernels();
void link_beam_kernels();
void link_optim_kernels();
void link_seq_kernels();
void link_io_kernels();
void link_tensor_kernels();
void link_rnn_unit_kernels();
void link_conv3d_kernels();
void link_loss_kernels();
void link_misc_kernels();
void link_more_kernels();
void link_extra_kernels();

// one-source kernels of ops_extra.hip that other kernel files fall back to
void layer_norm_any(const OpRun& r);
void layer_norm_grad_any(const OpRun& r);
void elementwise_int_any(const OpRun& r, int op);  // 0 add 1 sub 2 mul 3 div 4 max 5 min

// ---------------------------------------------------------------- executor
class Executor {
 public:
  explicit Executor(int device = -1);
  ~Executor();
  // Executor::Run of the reference: creates the block's variables (persistables in
  // `scope`, temporaries in `local` when given, else in `scope`) and runs the ops.
  void Run(const ProgramDesc& prog, Scope* scope, int block_id = 0, Scope* local = nullptr);
  void RunBlock(const ProgramDesc& prog, const BlockDesc& block, Scope* scope);
  ExecContext& context() { return ctx_; }
  void Sync();  // waits for the device stream
  // per-op wall time accumulation (the reference's kCPU profiler in the demo)
  bool profile = false;
  std::map<std::string, std::pair<int64_t, double>> op_time_ms;  // type -> (calls, ms)
  // device executors: ops that ran on host copies (no device kernel, or it declined)
  std::map<std::string, int64_t> host_fallbacks;
  // FLAGS_strict_native: a device-place op that would run on host copies is an error
  bool strict_native = false;
  // Per-op fallback for op types with no C++ kernel (the embedder's registered
  // kernel, e.g. the Python op library behind fluid.Executor(engine="native")):
  // called with the op, the scope it runs in, and its (block, op) position.
  // Unset: such an op is an error (the reference's "kernel not found" enforce).
  std::function<void(const OpDesc&, Scope&, int, int)> fallback;
  std::map<std::string, int64_t> embedder_fallbacks;  // op type -> calls through `fallback`
  // Runs device kernels on an embedder-owned stream (e.g. torch's current stream,
  // so embedder kernels and ours are ordered without host syncs); null restores
  // the executor's own stream.
  void SetStream(void* stream);
  // sub-block control flow (framework/executor.cc + operators/while_op.cc,
  // conditional_block_op.cc): forward execution of `while` / `conditional_block`
  void RunWhile(const ProgramDesc& prog, const OpDesc& op, Scope* scope);
  void RunConditionalBlock(const ProgramDesc& prog, const OpDesc& op, Scope* scope);
  // while_op.cc WhileGradOp: the grad block once per kept step scope, last step first
  void RunWhileGrad(const ProgramDesc& prog, const OpDesc& op, Scope* scope);
  void RunConditionalBlockGrad(const ProgramDesc& prog, const OpDesc& op, Scope* scope);
  // recurrent_op.cc RecurrentOp / RecurrentGradOp (StaticRNN): one kept step scope
  // per time step, states linked step to step
  void RunRecurrent(const ProgramDesc& prog, const OpDesc& op, Scope* scope);
  void RunRecurrentGrad(const ProgramDesc& prog, const OpDesc& op, Scope* scope);

 private:
  bool ReadBool(const Tensor& t);
  ExecContext ctx_;
  void* own_stream_ = nullptr;
};

// ---------------------------------------------------------------- tensor IO
// LoDTensor stream (framework/lod_tensor.cc SerializeToStream): one tensor per
// call; returns false at a clean end of stream.
bool read_lod_tensor(FILE* f, Tensor* t);
void write_lod_tensor(FILE* f, const Tensor& t);
void load_persistables(const ProgramDesc& prog, Scope* scope, const std::string& dir,
                       const std::string& combined_file, int device, void* stream);

// sequence_expand (sequence_expand_op.h): the X row each output row copies.  X's
// sequence i (its level-1 LoD, or row i when X has none) repeats len(Y's ref_level
// sequence i) times; *out_lod receives the expanded level-1 LoD when X has one.
std::vector<int64_t> sequence_expand_rows(const Tensor& x, const Tensor& y, int ref_level, LoD* out_lod);
// sequence_expand_as (sequence_expand_as_op.h): row i of X repeated len(Y's sequence i)
// times; *out_lod = Y's level-1 LoD.
std::vector<int64_t> sequence_expand_as_rows(const Tensor& x, const Tensor& y, LoD* out_lod);
// sequence_concat (sequence_concat_op.h): output sequence i = sequence i of every input
// in turn.  Returns, per input, the output row of each of its rows; *out_lod = the
// concatenated level-1 LoD.
std::vector<std::vector<int64_t>> sequence_concat_rows(const std::vector<Tensor*>& xs, LoD* out_lod);

// ---------------------------------------------------------------- host math
// C[M,N] = alpha * op(A) op(B) + beta * C, row-major, fp32, multithreaded.
void sgemm(bool ta, bool tb, int64_t M, int64_t N, int64_t K, float alpha, const float* A, int64_t lda,
           const float* B, int64_t ldb, float beta, float* C, int64_t ldc);

// device helpers (ops_gpu.hip; no-ops that fail when built without HIP devices)
void* device_alloc(size_t n, int dev);
void device_free(void* p, int dev);
void device_copy(void* dst, int dst_dev, const void* src, int src_dev, size_t n, void* stream);
void* device_stream_create(int dev);
void device_stream_destroy(void* s);
void device_stream_sync(void* s);
void device_synchronize(int dev);
int device_count();

// Device row movement / arithmetic behind the place-agnostic kernels of
// ops_control.cc (tensor arrays, rank tables, SelectedRows): the row maps are built
// on the host from LoD metadata and uploaded through the op's pinned staging buffer.
// Row sizes are in bytes; `add` scatters accumulate fp32 rows (duplicates allowed).
void device_gather_rows(const OpRun& r, const void* src, int64_t row_bytes, const std::vector<int64_t>& rows,
                        void* dst);
void device_scatter_rows(const OpRun& r, const void* src, int64_t row_bytes, const std::vector<int64_t>& rows,
                         void* dst, bool add);
void device_add_f32(void* stream, float* acc, const float* x, int64_t n);
void device_copy2d(const OpRun& r, void* dst, size_t dpitch, const void* src, size_t spitch, size_t width,
                   size_t height);
// sparse optimizer rows on HBM: Param[rows[i]] -= lr * V[i] (atomic: duplicates add)
void device_sgd_rows(const OpRun& r, float* p, const float* v, const std::vector<int64_t>& rows, int64_t w,
                     const float* lr);
// Adam on the (unique) rows of Param / Moment1 / Moment2 with the merged gradient g
void device_adam_rows(const OpRun& r, float* p, float* m1, float* m2, const float* g,
                      const std::vector<int64_t>& rows, int64_t w, const float* lr, const float* b1p,
                      const float* b2p, float b1, float b2, float eps);
void device_fill(void* stream, void* dst, DT dt, int64_t n, double v);

// SelectedRows-aware paths of sum / sgd / adam (ops_control.cc): true when the op's
// gradient / inputs were SelectedRows and the op has been run
bool selected_rows_sum(const OpRun& r);
bool selected_rows_sgd(const OpRun& r);
bool selected_rows_adam(const OpRun& r);
// lookup_table_grad with is_sparse: W@GRAD = SelectedRows{Ids, Out@GRAD rows}
void lookup_table_grad_sparse(const OpRun& r);

}  // namespace pa
