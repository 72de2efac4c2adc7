// paddle_amd native runtime: C ABI shared by all runtime components.
//
// The reference implements its runtime in C++ (RecordIO, LoDTensor stream IO,
// buddy allocator, thread pool / blocking queue, SSA graph executor, profiler:
// SURVEY §2.1 #9, #20, #27-31); these are the MI355X-native equivalents, bound to
// Python with ctypes (paddle_amd/runtime.py).
#pragma once
#include <stddef.h>
#include <stdint.h>

#define PA_RT_EXPORT extern "C" __attribute__((visibility("default")))

// ---- errors: every call returns 0 on success; pa_rt_last_error() explains failures
PA_RT_EXPORT const char* pa_rt_last_error();
void pa_rt_set_error(const char* fmt, ...);
