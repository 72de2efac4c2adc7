// Shared pieces of the structured-prediction kernels (ops_struct.cc host,
// ops_struct_gpu.hip device): the CRF forward / backward recursions and Viterbi.
#pragma once

#include <stdint.h>

#include <vector>

namespace pa {
namespace crf {

// Log-space forward (alpha [L, D]) and, when beta != null, backward (beta [L, D])
// recursions of one sequence; *nll = log Z - score(y).  tr = [D + 2, D] (start, end, T).
void forward_backward(const float* em, const float* tr, const int64_t* y, int64_t L, int64_t D, double* alpha,
                      double* beta, double* nll);
// Viterbi path of one sequence (first maximum on ties) into path[0 .. L).
void viterbi(const float* em, const float* tr, int64_t L, int64_t D, std::vector<float>& score,
             std::vector<float>& nxt, std::vector<int32_t>& back, int64_t* path);

}  // namespace crf
}  // namespace pa
