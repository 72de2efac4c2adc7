// Shared pieces of the LoD recurrent kernels (ops_rnn.cc host, ops_rnn_gpu.hip device):
// activation ids (math/detail/activation_functions.h order), and the
// LoDTensor2Batch step schedule (math/sequence2batch.cc).
#pragma once

#include <math.h>
#include <stdint.h>

#include <vector>

#include "framework.h"

namespace pa {
namespace rnn {

enum { ACT_IDENTITY = 0, ACT_SIGMOID = 1, ACT_TANH = 2, ACT_RELU = 3 };

// string ("sigmoid", ...) or int attribute -> ACT_*
int act_id(const OpDesc& op, const char* name, int def);

#if defined(__HIPCC__)
#define PA_RNN_HD __host__ __device__ __forceinline__
#else
#define PA_RNN_HD inline
#endif

PA_RNN_HD float act(int a, float x) {
  switch (a) {
    case ACT_SIGMOID: return 1.f / (1.f + expf(-x));
    case ACT_TANH: return tanhf(x);
    case ACT_RELU: return x > 0.f ? x : 0.f;
    default: return x;
  }
}
// derivative expressed through the activation's OUTPUT y
PA_RNN_HD float dact(int a, float y) {
  switch (a) {
    case ACT_SIGMOID: return y * (1.f - y);
    case ACT_TANH: return 1.f - y * y;
    case ACT_RELU: return y > 0.f ? 1.f : 0.f;
    default: return 1.f;
  }
}

// Time-step schedule of a LoD batch: sequences longest first (stable); step t covers
// the rows [step_begin[t], step_begin[t+1]) of (rows, seq, prev): the LoD row processed,
// its sequence, and the row of the same sequence at step t - 1 (-1 at t = 0).
struct SeqBatch {
  std::vector<int64_t> order;       // sequences, longest first
  std::vector<int64_t> step_begin;  // size L + 1
  std::vector<int64_t> rows, seq, prev;
};
SeqBatch make_batch(const std::vector<size_t>& off, bool reverse);

}  // namespace rnn
}  // namespace pa
