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

// The same with ta = true, plus the column sums of op(A) over k: cs[z*sCS + m*ldcs] =
// sum_k A_z[k][m] (written by the blocks of output tile column 0; per-thread partial sums
// over fixed k residues combined in a fixed order -- deterministic).  cs may be null.
int gemm_f32_tn_colsum(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda, int64_t sA, const float* B,
                       int64_t ldb, int64_t sB, float* C, int64_t ldc, int64_t sC, float* cs, int64_t ldcs,
                       int64_t sCS, int64_t batch, hipStream_t st);

}  // namespace kgat
