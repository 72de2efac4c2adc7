// Host fp32 GEMM for the native executor's CPU kernels (mul / matmul / fc / conv
// im2col).  Row-major C[M,N] = alpha * op(A) * op(B) + beta * C.
//
// Transposed operands are first copied into row-major panels; the product runs
// as a 4x16 register-blocked micro-kernel (GCC vector extensions -> AVX2/FMA with
// the build's -mavx2 -mfma) over 256-deep K slices, parallel over 64x256 output
// tiles on the host worker pool.
#include <string.h>

#include <vector>

#include "framework.h"

namespace pa {
namespace {
typedef float v8 __attribute__((vector_size(32), aligned(4)));

constexpr int64_t kMB = 64, kNB = 256, kKB = 256;

inline v8 ld(const float* p) {
  v8 v;
  memcpy(&v, p, sizeof(v));
  return v;
}
inline void st(float* p, v8 v) { memcpy(p, &v, sizeof(v)); }

// C[i0:i1, j0:j1] += A[i, k0:k1] * B[k0:k1, j] (A, B row-major, unit column stride)
void tile(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc, int64_t i0,
          int64_t i1, int64_t j0, int64_t j1, int64_t k0, int64_t k1) {
  int64_t i = i0;
  for (; i + 4 <= i1; i += 4) {
    int64_t j = j0;
    for (; j + 16 <= j1; j += 16) {
      v8 c00 = ld(C + (i + 0) * ldc + j), c01 = ld(C + (i + 0) * ldc + j + 8);
      v8 c10 = ld(C + (i + 1) * ldc + j), c11 = ld(C + (i + 1) * ldc + j + 8);
      v8 c20 = ld(C + (i + 2) * ldc + j), c21 = ld(C + (i + 2) * ldc + j + 8);
      v8 c30 = ld(C + (i + 3) * ldc + j), c31 = ld(C + (i + 3) * ldc + j + 8);
      const float* a0 = A + (i + 0) * lda;
      const float* a1 = A + (i + 1) * lda;
      const float* a2 = A + (i + 2) * lda;
      const float* a3 = A + (i + 3) * lda;
      for (int64_t k = k0; k < k1; ++k) {
        const v8 b0 = ld(B + k * ldb + j), b1 = ld(B + k * ldb + j + 8);
        c00 += a0[k] * b0; c01 += a0[k] * b1;
        c10 += a1[k] * b0; c11 += a1[k] * b1;
        c20 += a2[k] * b0; c21 += a2[k] * b1;
        c30 += a3[k] * b0; c31 += a3[k] * b1;
      }
      st(C + (i + 0) * ldc + j, c00); st(C + (i + 0) * ldc + j + 8, c01);
      st(C + (i + 1) * ldc + j, c10); st(C + (i + 1) * ldc + j + 8, c11);
      st(C + (i + 2) * ldc + j, c20); st(C + (i + 2) * ldc + j + 8, c21);
      st(C + (i + 3) * ldc + j, c30); st(C + (i + 3) * ldc + j + 8, c31);
    }
    for (; j < j1; ++j)
      for (int r = 0; r < 4; ++r) {
        float s = C[(i + r) * ldc + j];
        for (int64_t k = k0; k < k1; ++k) s += A[(i + r) * lda + k] * B[k * ldb + j];
        C[(i + r) * ldc + j] = s;
      }
  }
  for (; i < i1; ++i) {
    float* c = C + i * ldc;
    const float* a = A + i * lda;
    for (int64_t k = k0; k < k1; ++k) {
      const float av = a[k];
      const float* b = B + k * ldb;
      for (int64_t j = j0; j < j1; ++j) c[j] += av * b[j];
    }
  }
}

void transpose_copy(const float* src, int64_t rows, int64_t cols, int64_t ld, std::vector<float>& dst) {
  // src is [rows, cols] with leading dim ld; dst = src^T as [cols, rows]
  dst.resize((size_t)rows * cols);
  float* d = dst.data();
  parallel_for(cols, 64, [&](int64_t c0, int64_t c1) {
    for (int64_t c = c0; c < c1; ++c)
      for (int64_t r = 0; r < rows; ++r) d[c * rows + r] = src[r * ld + c];
  });
}
}  // namespace

void sgemm(bool ta, bool tb, int64_t M, int64_t N, int64_t K, float alpha, const float* A, int64_t lda,
           const float* B, int64_t ldb, float beta, float* C, int64_t ldc) {
  if (M <= 0 || N <= 0) return;
  std::vector<float> at, bt;
  if (ta) {  // A stored [K, M]
    transpose_copy(A, K, M, lda, at);
    A = at.data();
    lda = K;
  }
  if (tb) {  // B stored [N, K]
    transpose_copy(B, N, K, ldb, bt);
    B = bt.data();
    ldb = N;
  }
  const bool scale_after = alpha != 1.f;
  // beta pass
  parallel_for(M, 16, [&](int64_t r0, int64_t r1) {
    for (int64_t i = r0; i < r1; ++i) {
      float* c = C + i * ldc;
      if (beta == 0.f) memset(c, 0, sizeof(float) * N);
      else if (beta != 1.f)
        for (int64_t j = 0; j < N; ++j) c[j] *= beta;
    }
  });
  if (K <= 0) return;
  std::vector<float> acc;
  float* out = C;
  int64_t ldo = ldc;
  if (scale_after || beta != 0.f) {
    if (scale_after) {  // accumulate alpha*AB separately, then add into C
      acc.assign((size_t)M * N, 0.f);
      out = acc.data();
      ldo = N;
    }
  }
  const int64_t tm = (M + kMB - 1) / kMB, tn = (N + kNB - 1) / kNB;
  parallel_for(tm * tn, 1, [&](int64_t t0, int64_t t1) {
    for (int64_t t = t0; t < t1; ++t) {
      const int64_t i0 = (t / tn) * kMB, j0 = (t % tn) * kNB;
      const int64_t i1 = std::min(M, i0 + kMB), j1 = std::min(N, j0 + kNB);
      for (int64_t k0 = 0; k0 < K; k0 += kKB)
        tile(A, lda, B, ldb, out, ldo, i0, i1, j0, j1, k0, std::min(K, k0 + kKB));
    }
  });
  if (scale_after) {
    parallel_for(M, 16, [&](int64_t r0, int64_t r1) {
      for (int64_t i = r0; i < r1; ++i)
        for (int64_t j = 0; j < N; ++j) C[i * ldc + j] += alpha * acc[(size_t)i * N + j];
    });
  }
}

}  // namespace pa
