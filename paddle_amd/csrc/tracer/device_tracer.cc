// In-process kernel activity tracer on rocprofiler-sdk (the MI355X counterpart of
// the reference's CUPTI DeviceTracer: paddle/fluid/platform/device_tracer.cc:98-121
// buffers CUPTI kernel activity records; device_tracer.h:45-92 the interface).
//
// This library is a rocprofiler-sdk *tool*: it exports rocprofiler_configure and
// also registers itself with rocprofiler_force_configure from pa_tracer_register(),
// which must run before the HIP runtime initialises (the Python side loads it at
// import time when FLAGS_device_tracer / PADDLE_AMD_DEVICE_TRACER is set).
//
//  * context `sym_ctx` (always on): code-object callback tracing of device kernel
//    symbol registration -> kernel_id -> demangled-later name table, so kernels
//    loaded before a tracing window still get names;
//  * context `act_ctx` (started / stopped by pa_tracer_enable / pa_tracer_disable):
//    buffered KERNEL_DISPATCH tracing -> {kernel_id, GPU ordinal, queue, start_ns,
//    end_ns, correlation, external correlation (the framework range id pushed by
//    pa_tracer_push_range), grid, workgroup, LDS, scratch} appended to a vector;
//  * timestamps are rocprofiler's (the same clock as pa_tracer_now_ns), so host
//    ranges stamped with pa_tracer_now_ns land on the kernels' time axis.
#include <rocprofiler-sdk/registration.h>
#include <rocprofiler-sdk/rocprofiler.h>

#include <cstdint>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#define PA_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

struct KernelRec {
  uint64_t kernel_id, start_ns, end_ns, corr, ext;
  uint64_t queue;
  int32_t device;
  uint32_t grid[3], wg[3];
  uint32_t lds, scratch;
};

struct State {
  std::mutex mu;
  std::vector<KernelRec> recs;
  std::unordered_map<uint64_t, std::string> names;  // kernel_id -> symbol
  std::unordered_map<uint64_t, int32_t> gpu_of;     // agent handle -> GPU ordinal
  rocprofiler_context_id_t sym_ctx{0}, act_ctx{0};
  rocprofiler_buffer_id_t buf{0};
  rocprofiler_client_id_t* client = nullptr;
  bool configured = false;  // tool_init ran and both contexts are valid
  bool active = false;
  uint64_t dropped = 0;
  int last_error = 0;
};

State& st() {
  static State* s = new State();  // never destroyed: rocprofiler may call back at exit
  return *s;
}

void on_code_object(rocprofiler_callback_tracing_record_t rec, rocprofiler_user_data_t*, void*) {
  if (rec.kind != ROCPROFILER_CALLBACK_TRACING_CODE_OBJECT ||
      rec.operation != ROCPROFILER_CODE_OBJECT_DEVICE_KERNEL_SYMBOL_REGISTER ||
      rec.phase != ROCPROFILER_CALLBACK_PHASE_LOAD)
    return;
  auto* d = static_cast<rocprofiler_callback_tracing_code_object_kernel_symbol_register_data_t*>(rec.payload);
  std::string nm = d->kernel_name ? d->kernel_name : "";
  // strip the ".kd" descriptor suffix the loader reports
  if (nm.size() > 3 && nm.compare(nm.size() - 3, 3, ".kd") == 0) nm.resize(nm.size() - 3);
  std::lock_guard<std::mutex> g(st().mu);
  st().names[d->kernel_id] = std::move(nm);
}

void on_buffer(rocprofiler_context_id_t, rocprofiler_buffer_id_t, rocprofiler_record_header_t** hdrs, size_t n,
               void*, uint64_t drop_count) {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  s.dropped += drop_count;
  for (size_t i = 0; i < n; ++i) {
    const rocprofiler_record_header_t* h = hdrs[i];
    if (h->category != ROCPROFILER_BUFFER_CATEGORY_TRACING || h->kind != ROCPROFILER_BUFFER_TRACING_KERNEL_DISPATCH)
      continue;
    auto* r = static_cast<const rocprofiler_buffer_tracing_kernel_dispatch_record_t*>(h->payload);
    const rocprofiler_kernel_dispatch_info_t& di = r->dispatch_info;
    KernelRec k{};
    k.kernel_id = di.kernel_id;
    k.start_ns = r->start_timestamp;
    k.end_ns = r->end_timestamp;
    k.corr = r->correlation_id.internal;
    k.ext = r->correlation_id.external.value;
    k.queue = di.queue_id.handle;
    auto it = s.gpu_of.find(di.agent_id.handle);
    k.device = it == s.gpu_of.end() ? -1 : it->second;
    k.grid[0] = di.grid_size.x; k.grid[1] = di.grid_size.y; k.grid[2] = di.grid_size.z;
    k.wg[0] = di.workgroup_size.x; k.wg[1] = di.workgroup_size.y; k.wg[2] = di.workgroup_size.z;
    k.lds = di.group_segment_size;
    k.scratch = di.private_segment_size;
    s.recs.push_back(k);
  }
}

rocprofiler_status_t on_agents(rocprofiler_agent_version_t, const void** agents, size_t n, void*) {
  State& s = st();
  for (size_t i = 0; i < n; ++i) {
    auto* a = static_cast<const rocprofiler_agent_v0_t*>(agents[i]);
    if (a->type == ROCPROFILER_AGENT_TYPE_GPU) s.gpu_of[a->id.handle] = a->logical_node_type_id;
  }
  return ROCPROFILER_STATUS_SUCCESS;
}

#define PA_RP(call)                                      \
  do {                                                   \
    rocprofiler_status_t rc_ = (call);                   \
    if (rc_ != ROCPROFILER_STATUS_SUCCESS) {             \
      st().last_error = (int)rc_;                        \
      return -1;                                         \
    }                                                    \
  } while (0)

int tool_init(rocprofiler_client_finalize_t, void*) {
  State& s = st();
  PA_RP(rocprofiler_query_available_agents(ROCPROFILER_AGENT_INFO_VERSION_0, on_agents, sizeof(rocprofiler_agent_v0_t),
                                           nullptr));
  PA_RP(rocprofiler_create_context(&s.sym_ctx));
  rocprofiler_tracing_operation_t ops[] = {ROCPROFILER_CODE_OBJECT_DEVICE_KERNEL_SYMBOL_REGISTER};
  PA_RP(rocprofiler_configure_callback_tracing_service(s.sym_ctx, ROCPROFILER_CALLBACK_TRACING_CODE_OBJECT, ops, 1,
                                                       on_code_object, nullptr));
  PA_RP(rocprofiler_create_context(&s.act_ctx));
  constexpr size_t kBuf = 1 << 20;  // 1 MiB of records; flushed at 7/8
  PA_RP(rocprofiler_create_buffer(s.act_ctx, kBuf, kBuf - kBuf / 8, ROCPROFILER_BUFFER_POLICY_LOSSLESS, on_buffer,
                                  nullptr, &s.buf));
  PA_RP(rocprofiler_configure_buffer_tracing_service(s.act_ctx, ROCPROFILER_BUFFER_TRACING_KERNEL_DISPATCH, nullptr, 0,
                                                     s.buf));
  rocprofiler_callback_thread_t th{};
  PA_RP(rocprofiler_create_callback_thread(&th));
  PA_RP(rocprofiler_assign_callback_thread(s.buf, th));
  int ok = 0;
  PA_RP(rocprofiler_context_is_valid(s.sym_ctx, &ok));
  if (!ok) return -1;
  PA_RP(rocprofiler_context_is_valid(s.act_ctx, &ok));
  if (!ok) return -1;
  PA_RP(rocprofiler_start_context(s.sym_ctx));
  s.configured = true;
  return 0;
}

void tool_fini(void*) {
  State& s = st();
  if (s.configured) {
    if (s.active) rocprofiler_stop_context(s.act_ctx);
    rocprofiler_flush_buffer(s.buf);
  }
  s.configured = false;
  s.active = false;
}

}  // namespace

extern "C" __attribute__((visibility("default"))) rocprofiler_tool_configure_result_t* rocprofiler_configure(
    uint32_t, const char*, uint32_t, rocprofiler_client_id_t* id) {
  if (st().client != nullptr) return nullptr;  // configured once (env discovery or force_configure)
  id->name = "paddle_amd.device_tracer";
  st().client = id;
  static rocprofiler_tool_configure_result_t cfg{sizeof(rocprofiler_tool_configure_result_t), &tool_init, &tool_fini,
                                                 nullptr};
  return &cfg;
}

// 0: registered (or already configured by discovery); -2: rocprofiler is already
// initialised without this tool (the HIP runtime started first); other: the status.
PA_EXPORT int pa_tracer_register() {
  int inited = 0;
  if (rocprofiler_is_initialized(&inited) == ROCPROFILER_STATUS_SUCCESS && inited) return st().client ? 0 : -2;
  rocprofiler_status_t rc = rocprofiler_force_configure(&rocprofiler_configure);
  if (rc == ROCPROFILER_STATUS_SUCCESS) return 0;
  return st().client ? 0 : (int)rc;
}

PA_EXPORT int pa_tracer_available() { return st().configured ? 1 : 0; }
PA_EXPORT int pa_tracer_last_error() { return st().last_error; }

PA_EXPORT int pa_tracer_enable() {
  State& s = st();
  if (!s.configured) return -1;
  if (s.active) return 0;
  if (rocprofiler_start_context(s.act_ctx) != ROCPROFILER_STATUS_SUCCESS) return -1;
  s.active = true;
  return 0;
}

// Stops recording and flushes every buffered record into the host vector (the
// caller synchronises the device first so the window's kernels have completed).
PA_EXPORT int pa_tracer_disable() {
  State& s = st();
  if (!s.configured) return -1;
  if (s.active) {
    rocprofiler_stop_context(s.act_ctx);
    s.active = false;
  }
  return rocprofiler_flush_buffer(s.buf) == ROCPROFILER_STATUS_SUCCESS ? 0 : -1;
}

PA_EXPORT int pa_tracer_flush() {
  State& s = st();
  if (!s.configured) return -1;
  return rocprofiler_flush_buffer(s.buf) == ROCPROFILER_STATUS_SUCCESS ? 0 : -1;
}

PA_EXPORT uint64_t pa_tracer_now_ns() {
  rocprofiler_timestamp_t t = 0;
  rocprofiler_get_timestamp(&t);
  return t;
}

// Framework range correlation: kernels dispatched by this thread while a range
// is pushed carry its id as their external correlation id.
PA_EXPORT int pa_tracer_push_range(uint64_t id) {
  State& s = st();
  if (!s.configured) return -1;
  rocprofiler_thread_id_t tid = 0;
  rocprofiler_get_thread_id(&tid);
  rocprofiler_user_data_t u{};
  u.value = id;
  return rocprofiler_push_external_correlation_id(s.act_ctx, tid, u) == ROCPROFILER_STATUS_SUCCESS ? 0 : -1;
}

PA_EXPORT int pa_tracer_pop_range() {
  State& s = st();
  if (!s.configured) return -1;
  rocprofiler_thread_id_t tid = 0;
  rocprofiler_get_thread_id(&tid);
  rocprofiler_user_data_t u{};
  return rocprofiler_pop_external_correlation_id(s.act_ctx, tid, &u) == ROCPROFILER_STATUS_SUCCESS ? 0 : -1;
}

PA_EXPORT long pa_tracer_count() {
  std::lock_guard<std::mutex> g(st().mu);
  return (long)st().recs.size();
}

PA_EXPORT uint64_t pa_tracer_dropped() { return st().dropped; }

PA_EXPORT void pa_tracer_clear() {
  std::lock_guard<std::mutex> g(st().mu);
  st().recs.clear();
  st().dropped = 0;
}

// Record i: u64 out[8] = {kernel_id, start_ns, end_ns, correlation, external
// correlation, queue, lds bytes, scratch bytes}; i32 out2[7] = {device, grid xyz,
// workgroup xyz}; the kernel symbol (mangled) into name[0..cap).  Returns the
// symbol's full length, or -1 past the end.
PA_EXPORT int pa_tracer_get(long i, uint64_t* out, int32_t* out2, char* name, int cap) {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  if (i < 0 || i >= (long)s.recs.size()) return -1;
  const KernelRec& k = s.recs[i];
  out[0] = k.kernel_id; out[1] = k.start_ns; out[2] = k.end_ns; out[3] = k.corr;
  out[4] = k.ext; out[5] = k.queue; out[6] = k.lds; out[7] = k.scratch;
  out2[0] = k.device;
  for (int d = 0; d < 3; ++d) {
    out2[1 + d] = (int32_t)k.grid[d];
    out2[4 + d] = (int32_t)k.wg[d];
  }
  auto it = s.names.find(k.kernel_id);
  const std::string nm = it == s.names.end() ? std::string("kernel_") + std::to_string(k.kernel_id) : it->second;
  if (name && cap > 0) {
    const int n = (int)nm.size() < cap - 1 ? (int)nm.size() : cap - 1;
    std::memcpy(name, nm.data(), n);
    name[n] = 0;
  }
  return (int)nm.size();
}
