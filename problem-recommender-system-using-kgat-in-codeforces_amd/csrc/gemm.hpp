// The hand-written fp32 MFMA GEMM of gemm.hip (see there for the tiling).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kgat {

// C[m, n] (+)= op(A)[m, k] . op(B)[k, n], row-major; ta: A stored [k, m]; tb: B stored [n, k];
// batch z uses A + z*sA, B + z*sB, C + z*sC.  Returns a kgat status.
int gemm_f32(bool ta, bool tb, int64_t M, int64_t N, int64_t K, const float* A, int64_t lda, int64_t sA,
             const float* B, int64_t ldb, int64_t sB, float* C, int64_t ldc, int64_t sC, int64_t batch,
             bool accumulate, hipStream_t st);

// Two products on the same tile coordinates in one launch (gemm.hip's dual_gemm_kernel):
// C1 = op(A1) op(B1), C2 = op(A2) op(B2), each with gemm_f32's bits.  a_um: (A1, A2) = (X, S)
// and the products take (X + S, X * S) (not transposed A only); b_um: the same for (B1, B2)
// (row-major [K, N] B only).  dxs: C1 <- du + dm * S, C2 <- du + dm * X (C1 = du, C2 = dm; the
// bi-interaction backward; X / S [M, N]).  cs1 / cs2 (ta only): column sums of op(A1) / op(A2).
struct DualGemm {
  bool ta = false, tb = false, a_um = false, b_um = false, dxs = false;
  int64_t M = 0, N = 0, K = 0, batch = 1;
  const float* A1 = nullptr;
  const float* A2 = nullptr;
  int64_t lda1 = 0, lda2 = 0, sA1 = 0, sA2 = 0;
  const float* B1 = nullptr;
  const float* B2 = nullptr;
  int64_t ldb1 = 0, ldb2 = 0, sB1 = 0, sB2 = 0;
  float* C1 = nullptr;
  float* C2 = nullptr;
  int64_t ldc1 = 0, ldc2 = 0, sC1 = 0, sC2 = 0;
  float* cs1 = nullptr;
  float* cs2 = nullptr;
  int64_t ldcs = 0, sCS1 = 0, sCS2 = 0;
  const float* X = nullptr;
  const float* S = nullptr;
  int64_t ldx = 0, lds = 0;
  // row lists (nullable, -1 = a zero row): arows -- A's stored row of each of its M rows (not
  // transposed A); brows -- B's stored row of each of its K rows (row-major B; batch z reads
  // brows + z * sBrows); erows -- the dXd / dS epilogue's row of X / S for each output row
  const int32_t* arows = nullptr;
  const int32_t* brows = nullptr;
  int64_t sBrows = 0;
  const int32_t* erows = nullptr;
};
int dual_gemm_f32(const DualGemm& d, hipStream_t st);

}  // namespace kgat
