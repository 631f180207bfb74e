// Hand-written fp32 MFMA GEMM for gfx950 -- the plain contractions of the wide layers
// (d = 128 / 256 at C4 / C5): the bi-interaction's W1 / W2 products and their backward
// (src/model/KGAT/aggregator.py:57-65), the weight gradients' split-K slabs, and the edge
// scorer's T . W_r, W_v, W_o products (src/model/KGAT/model.py:263-316).  Replaces the
// vendor sgemm: no library GEMM runs on the hot path.
//
//   C[m, n] (+)= sum_k op(A)[m, k] * op(B)[k, n]      (row-major, fp32 in / fp32 out)
//   op(A) = A [M, K] (lda)  or, TA, A^T with A stored [K, M]
//   op(B) = B [K, N] (ldb)  or, TB, B^T with B stored [N, K]
//   batched: blockIdx.z selects A + z*sA, B + z*sB, C + z*sC.
//
// Tiling: a 256-thread block (4 waves, 2 x 2) owns a 128 x 128 tile of C; each wave a
// 64 x 64 quarter as 2 x 2 tiles of v_mfma_f32_32x32x2_f32 (16 accumulators per tile,
// 64 per lane).  K advances in 16-deep stages through two LDS buffers (register-staged:
// the next stage's global loads are in flight while the current one is multiplied).
// MFMA step s (s = 0..7) of a stage multiplies k = 8h + s of half h = lane >> 5, so a
// stage sums k in a fixed order: results are deterministic and exact fp32 fma chains
// (the MFMA rounds once per product), not bit-equal to a library sgemm.
// LDS layout per operand, by its global layout:
//  * k-contiguous (A, or B^T): [row][k], row pitch 20 floats -- lane l reads its 8
//    k-values of row (l & 31) with two ds_read_b128; with the 80-byte pitch the 16 lanes
//    of a b128 phase hit 16 distinct 4-bank groups (conflict-free);
//  * k-major (A^T, or B: the weight-gradient GEMMs' operands): [k][row], pitch 132 floats --
//    the global float4 (4 rows of one k) is stored whole (one ds_write_b128, where a
//    [row][k] image needs four conflicting ds_write_b32), and step s's operand is one
//    ds_read_b32 per lane: 32 consecutive rows of k = s (lanes 0-31) and of k = 8 + s
//    (lanes 32-63, 8 pitches = 1056 floats away: the other 32 banks).
#include <cstdlib>

#include "common.hpp"
#include "gemm.hpp"

namespace kgat {

namespace {

constexpr int kBM = 128, kBN = 128;
constexpr int kPitchT = kBM + 4;  // LDS k-row pitch in floats ([k][row])
constexpr int kThreads = 256;
// k-depth of a stage (one barrier per stage); the launches use 16 (32 gives the same k order: stage kt,
// sub-stage u, step s takes k = 32 kt + 16 u + 8 h + s)
template <int BK>
struct Tile {
  static constexpr int kPitch = BK + 4;  // LDS row pitch in floats ([row][k]): conflict-free b128 reads
  static constexpr int kStageFloats = kBM * kPitch > BK * kPitchT ? kBM * kPitch : BK * kPitchT;
  static constexpr int kPer = BK / 8;    // float4 per thread per operand stage
};

typedef float floatx16 __attribute__((ext_vector_type(16)));

struct GemmArgs {
  const float* A;
  const float* B;
  float* C;
  int64_t lda, ldb, ldc;
  int64_t sA, sB, sC;
  int64_t M, N, K;
  int accumulate;
  float* cs;  // TA only: column sums of op(A) over k (nullable)
  int64_t ldcs, sCS;
};

// One operand stage: 128 rows x BK k as 32 BK float4 (BK/8 per thread), and where they go in LDS.
// KCONTIG: the operand's k index is its contiguous dimension (A not transposed / B transposed).
template <bool KCONTIG, int BK>
struct Stage {
  static constexpr int P = Tile<BK>::kPitch;
  static constexpr int Q = Tile<BK>::kPer;
  float4 v[Q];

  // idx (nullable): the operand's stored-row index of each logical row -- its m / n row when the
  // k index is contiguous, its k row otherwise (a row list; -1 = a zero row)
  __device__ __forceinline__ void load(const float* __restrict__ Pm, int64_t ld, int64_t rows, int64_t K, int64_t r0,
                                       int64_t k0, int t, const int32_t* __restrict__ ridx = nullptr) {
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int idx = t + q * kThreads;
      if (KCONTIG) {  // P[r][k]: BK/4 float4 per row
        const int64_t r = r0 + idx / (BK / 4), k = k0 + (idx % (BK / 4)) * 4;
        const int64_t rr = (ridx != nullptr && r < rows) ? static_cast<int64_t>(ridx[r]) : r;
        v[q] = (r < rows && k < K && rr >= 0) ? *reinterpret_cast<const float4*>(Pm + rr * ld + k)
                                               : make_float4(0.f, 0.f, 0.f, 0.f);
      } else {        // P[k][r]: 32 float4 per k-row
        const int64_t k = k0 + (idx >> 5), r = r0 + (idx & 31) * 4;
        const int64_t kk = (ridx != nullptr && k < K) ? static_cast<int64_t>(ridx[k]) : k;
        v[q] = (k < K && r < rows && kk >= 0) ? *reinterpret_cast<const float4*>(Pm + kk * ld + r)
                                               : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  }

  __device__ __forceinline__ void store(float* __restrict__ lds, int t) const {
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int idx = t + q * kThreads;
      if (KCONTIG) {
        *reinterpret_cast<float4*>(lds + (idx / (BK / 4)) * P + (idx % (BK / 4)) * 4) = v[q];
      } else {  // [k][row]: the 4 rows of one k stay together
        *reinterpret_cast<float4*>(lds + (idx >> 5) * kPitchT + (idx & 31) * 4) = v[q];
      }
    }
  }

  // The 8 k-values (k = 16 u + 8h + s, s = 0..7) of sub-stage u of tile row `row` (0..127) for
  // this lane's half h.
  __device__ __forceinline__ static void read(const float* __restrict__ lds, int row, int h, int u, float (&out)[8]) {
    if (KCONTIG) {
      const float4 a = *reinterpret_cast<const float4*>(lds + row * P + 16 * u + 8 * h);
      const float4 b = *reinterpret_cast<const float4*>(lds + row * P + 16 * u + 8 * h + 4);
      out[0] = a.x, out[1] = a.y, out[2] = a.z, out[3] = a.w;
      out[4] = b.x, out[5] = b.y, out[6] = b.z, out[7] = b.w;
    } else {
#pragma unroll
      for (int s = 0; s < 8; ++s) out[s] = lds[(16 * u + 8 * h + s) * kPitchT + row];
    }
  }
};

// csum += the float4s of a (k-major, !KCONTIG) stage this thread loaded (k = (t >> 5) + 8 q: the
// same k order for any BK)
template <bool KC, int BK>
__device__ __forceinline__ void add_stage(float4& csum, const Stage<KC, BK>& st) {
#pragma unroll
  for (int q = 0; q < Tile<BK>::kPer; ++q) {
    csum.x += st.v[q].x;
    csum.y += st.v[q].y;
    csum.z += st.v[q].z;
    csum.w += st.v[q].w;
  }
}

template <bool TA, bool TB, int BK>
__global__ __launch_bounds__(kThreads, 2) void gemm_kernel(GemmArgs g) {
  __shared__ float lds[2][2][Tile<BK>::kStageFloats];  // [buffer][A | B][operand image]
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int tiles_n = static_cast<int>((g.N + kBN - 1) / kBN);
  const int64_t m0 = static_cast<int64_t>(blockIdx.x / tiles_n) * kBM;
  const int64_t n0 = static_cast<int64_t>(blockIdx.x % tiles_n) * kBN;
  const float* __restrict__ A = g.A + blockIdx.z * g.sA;
  const float* __restrict__ B = g.B + blockIdx.z * g.sB;
  float* __restrict__ C = g.C + blockIdx.z * g.sC;

  Stage<!TA, BK> sa;
  Stage<TB, BK> sb;
  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;

  const int nk = static_cast<int>((g.K + BK - 1) / BK);
  // TA column sums: this thread's float4 of A^T rows k = (t >> 5) + 8 q (q = 0, 1) of every
  // stage covers columns m0 + 4 (t & 31) .. + 3; summed over its k residues here, combined
  // over the 8 residue threads in order at the end
  const bool do_cs = TA && g.cs != nullptr && n0 == 0;
  float4 csum = make_float4(0.f, 0.f, 0.f, 0.f);
  sa.load(A, g.lda, g.M, g.K, m0, 0, t);
  sb.load(B, g.ldb, g.N, g.K, n0, 0, t);
  sa.store(lds[0][0], t);
  sb.store(lds[0][1], t);
  if (do_cs) add_stage(csum, sa);
  __syncthreads();
  const int wm = (w >> 1) * 64, wn = (w & 1) * 64;
  const int r = lane & 31, h = lane >> 5;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      sa.load(A, g.lda, g.M, g.K, m0, static_cast<int64_t>(kt + 1) * BK, t);
      sb.load(B, g.ldb, g.N, g.K, n0, static_cast<int64_t>(kt + 1) * BK, t);
    }
#pragma unroll
    for (int u = 0; u < BK / 16; ++u) {
      float fa[2][8], fb[2][8];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        Stage<!TA, BK>::read(lds[cur][0], wm + 32 * i + r, h, u, fa[i]);
        Stage<TB, BK>::read(lds[cur][1], wn + 32 * i + r, h, u, fb[i]);
      }
#pragma unroll
      for (int s = 0; s < 8; ++s) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][s], fb[j][s], acc[i][j], 0, 0, 0);
        }
      }
    }
    if (kt + 1 < nk) {
      sa.store(lds[cur ^ 1][0], t);
      sb.store(lds[cur ^ 1][1], t);
      if (do_cs) add_stage(csum, sa);
    }
    __syncthreads();
  }
  if (do_cs) {
    __shared__ float4 cpart[kThreads];
    cpart[t] = csum;
    __syncthreads();
    if (t < 32) {
      float4 s = cpart[t];
      for (int j = 1; j < 8; ++j) {
        const float4 o = cpart[t + 32 * j];
        s.x += o.x;
        s.y += o.y;
        s.z += o.z;
        s.w += o.w;
      }
      float* cs = g.cs + blockIdx.z * g.sCS;
      const float v[4] = {s.x, s.y, s.z, s.w};
      for (int i = 0; i < 4; ++i)
        if (m0 + 4 * t + i < g.M) cs[(m0 + 4 * t + i) * g.ldcs] = v[i];
    }
  }
  // C/D layout of 32x32: col = lane & 31, row = (q & 3) + 8 (q >> 2) + 4 (lane >> 5)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t col = n0 + wn + 32 * j + r;
      if (col >= g.N) continue;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int64_t row = m0 + wm + 32 * i + (q & 3) + 8 * (q >> 2) + 4 * h;
        if (row < g.M) {
          float* c = C + row * g.ldc + col;
          *c = g.accumulate ? *c + acc[i][j][q] : acc[i][j][q];
        }
      }
    }
}

// ---------------------------------------------------------------------------------------------
// Dual GEMM: two products on the same tile coordinates in one launch,
//   C1 = op(A1) . op(B1),   C2 = op(A2) . op(B2),
// each with gemm_kernel's tiling, stage order and MFMA order (so each product has exactly the
// single kernel's bits).  An operand pair is either two matrices (kSep) or the bi-interaction's
// (X + S, X * S) formed from one load of X and S (kUM: no U / M array in HBM).  Epilogues:
// kStore writes C1, C2; kDXS is the bi-interaction backward's dXd = du + dm * S, dS = du + dm * X
// (C1 = du, C2 = dm; X, S read at the output element), written to C1 / C2.
enum DualOp { kSep = 0, kUM = 1 };
enum DualEpi { kStore = 0, kDXS = 1 };

struct DualArgs {
  const float* A1;
  const float* A2;
  int64_t lda1, lda2, sA1, sA2;
  const float* B1;
  const float* B2;
  int64_t ldb1, ldb2, sB1, sB2;
  float* C1;
  float* C2;
  int64_t ldc1, ldc2, sC1, sC2;
  int64_t M, N, K;
  float* cs1;  // TA only: column sums of op(A1) / op(A2) over k (nullable)
  float* cs2;
  int64_t ldcs, sCS1, sCS2;
  const float* X;  // kDXS
  const float* S;
  int64_t ldx, lds;
  const int32_t* arows;  // nullable row lists (-1 = zero row): A's m rows, B's k rows (+ z * sBrows),
  const int32_t* brows;  // the dXd / dS epilogue's X / S rows
  int64_t sBrows;
  const int32_t* erows;
};

// Two stages of one operand pair; kUM turns the loaded (X, S) into (X + S, X * S).
template <bool KC, int OP, int BK>
struct StagePair {
  Stage<KC, BK> a, b;

  __device__ __forceinline__ void load(const float* __restrict__ P1, int64_t ld1, const float* __restrict__ P2,
                                       int64_t ld2, int64_t rows, int64_t K, int64_t r0, int64_t k0, int t,
                                       const int32_t* __restrict__ ridx = nullptr) {
    a.load(P1, ld1, rows, K, r0, k0, t, ridx);
    b.load(P2, ld2, rows, K, r0, k0, t, ridx);
    if (OP == kUM) {
#pragma unroll
      for (int q = 0; q < Tile<BK>::kPer; ++q) {
        const float4 x = a.v[q], s = b.v[q];
        a.v[q] = make_float4(x.x + s.x, x.y + s.y, x.z + s.z, x.w + s.w);
        b.v[q] = make_float4(x.x * s.x, x.y * s.y, x.z * s.z, x.w * s.w);
      }
    }
  }
  __device__ __forceinline__ void store(float* __restrict__ l1, float* __restrict__ l2, int t) const {
    a.store(l1, t);
    b.store(l2, t);
  }
};

template <bool TA, bool TB, int AOP, int BOP, int EPI, int BK>
__global__ __launch_bounds__(kThreads, 2) void dual_gemm_kernel(DualArgs g) {
  __shared__ float lds[2][4][Tile<BK>::kStageFloats];  // [buffer][A1 | A2 | B1 | B2][operand image]
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int tiles_n = static_cast<int>((g.N + kBN - 1) / kBN);
  const int64_t m0 = static_cast<int64_t>(blockIdx.x / tiles_n) * kBM;
  const int64_t n0 = static_cast<int64_t>(blockIdx.x % tiles_n) * kBN;
  const int64_t z = blockIdx.z;
  const float* __restrict__ A1 = g.A1 + z * g.sA1;
  const float* __restrict__ A2 = g.A2 + z * g.sA2;
  const float* __restrict__ B1 = g.B1 + z * g.sB1;
  const float* __restrict__ B2 = g.B2 + z * g.sB2;

  StagePair<!TA, AOP, BK> sa;
  StagePair<TB, BOP, BK> sb;
  floatx16 acc1[2][2], acc2[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc1[i][j][q] = acc2[i][j][q] = 0.f;

  const int nk = static_cast<int>((g.K + BK - 1) / BK);
  const bool do_cs = TA && g.cs1 != nullptr && n0 == 0;
  float4 cs1 = make_float4(0.f, 0.f, 0.f, 0.f), cs2 = cs1;
  const int32_t* __restrict__ brows = g.brows != nullptr ? g.brows + z * g.sBrows : nullptr;
  sa.load(A1, g.lda1, A2, g.lda2, g.M, g.K, m0, 0, t, g.arows);
  sb.load(B1, g.ldb1, B2, g.ldb2, g.N, g.K, n0, 0, t, brows);
  sa.store(lds[0][0], lds[0][1], t);
  sb.store(lds[0][2], lds[0][3], t);
  if (do_cs) {
    add_stage(cs1, sa.a);
    add_stage(cs2, sa.b);
  }
  __syncthreads();
  const int wm = (w >> 1) * 64, wn = (w & 1) * 64;
  const int r = lane & 31, h = lane >> 5;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      sa.load(A1, g.lda1, A2, g.lda2, g.M, g.K, m0, static_cast<int64_t>(kt + 1) * BK, t, g.arows);
      sb.load(B1, g.ldb1, B2, g.ldb2, g.N, g.K, n0, static_cast<int64_t>(kt + 1) * BK, t, brows);
    }
#pragma unroll
    for (int up = 0; up < 2 * (BK / 16); ++up) {  // sub-stage u of product p: 8 k-values per tile row, MFMAs
      const int u = up >> 1, p = up & 1;
      float fa[2][8], fb[2][8];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        Stage<!TA, BK>::read(lds[cur][p], wm + 32 * i + r, h, u, fa[i]);
        Stage<TB, BK>::read(lds[cur][2 + p], wn + 32 * i + r, h, u, fb[i]);
      }
#pragma unroll
      for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            if (p == 0) acc1[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][s], fb[j][s], acc1[i][j], 0, 0, 0);
            else acc2[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][s], fb[j][s], acc2[i][j], 0, 0, 0);
          }
    }
    if (kt + 1 < nk) {
      sa.store(lds[cur ^ 1][0], lds[cur ^ 1][1], t);
      sb.store(lds[cur ^ 1][2], lds[cur ^ 1][3], t);
      if (do_cs) {
        add_stage(cs1, sa.a);
        add_stage(cs2, sa.b);
      }
    }
    __syncthreads();
  }
  if (do_cs) {
    // the operand images are free after the last barrier: the column-sum partials go there (an
    // array of their own would push the block past 80 KB of LDS, one block per CU)
    float4(*cpart)[kThreads] = reinterpret_cast<float4(*)[kThreads]>(&lds[0][0][0]);
    cpart[0][t] = cs1;
    cpart[1][t] = cs2;
    __syncthreads();
    if (t < 64) {
      const int which = t >> 5, tt = t & 31;
      float4 s = cpart[which][tt];
      for (int j = 1; j < 8; ++j) {
        const float4 o = cpart[which][tt + 32 * j];
        s.x += o.x;
        s.y += o.y;
        s.z += o.z;
        s.w += o.w;
      }
      float* cs = which == 0 ? g.cs1 + z * g.sCS1 : g.cs2 + z * g.sCS2;
      const float v[4] = {s.x, s.y, s.z, s.w};
      for (int i = 0; i < 4; ++i)
        if (m0 + 4 * tt + i < g.M) cs[(m0 + 4 * tt + i) * g.ldcs] = v[i];
    }
  }
  float* __restrict__ C1 = g.C1 + z * g.sC1;
  float* __restrict__ C2 = g.C2 + z * g.sC2;
  const float* __restrict__ Xe = g.X;
  const float* __restrict__ Se = g.S;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t col = n0 + wn + 32 * j + r;
      if (col >= g.N) continue;
      float sv[16], xv[16];
      if (EPI == kDXS) {
        // the tile's S / X elements all in flight before its first store (a store between two
        // loads would make each load wait for the previous one's round trip)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int64_t row = m0 + wm + 32 * i + (q & 3) + 8 * (q >> 2) + 4 * h;
          const int64_t er = (g.erows != nullptr && row < g.M) ? static_cast<int64_t>(g.erows[row]) : row;
          const bool ok = row < g.M && er >= 0;
          sv[q] = ok ? Se[er * g.lds + col] : 0.f;
          xv[q] = ok ? Xe[er * g.ldx + col] : 0.f;
        }
      }
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int64_t row = m0 + wm + 32 * i + (q & 3) + 8 * (q >> 2) + 4 * h;
        if (row >= g.M) continue;
        if (EPI == kDXS) {
          const float du = acc1[i][j][q], dm = acc2[i][j][q];
          C1[row * g.ldc1 + col] = fmaf(dm, sv[q], du);
          C2[row * g.ldc2 + col] = fmaf(dm, xv[q], du);
        } else {
          C1[row * g.ldc1 + col] = acc1[i][j][q];
          C2[row * g.ldc2 + col] = acc2[i][j][q];
        }
      }
    }
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

int dual_gemm_f32(const DualGemm& d, hipStream_t st) {
  const int64_t M = d.M, N = d.N, K = d.K;
  if (M < 0 || N < 0 || K < 0 || d.batch < 0) return KGAT_ERR_INVALID;
  if (M == 0 || N == 0 || d.batch == 0) return KGAT_OK;
  if (!d.A1 || !d.A2 || !d.B1 || !d.B2 || !d.C1 || !d.C2 || K == 0) return KGAT_ERR_INVALID;
  if ((d.lda1 | d.lda2 | d.ldb1 | d.ldb2 | d.sA1 | d.sA2 | d.sB1 | d.sB2) & 3) return KGAT_ERR_INVALID;
  if (!aligned16(d.A1) || !aligned16(d.A2) || !aligned16(d.B1) || !aligned16(d.B2)) return KGAT_ERR_INVALID;
  if ((d.ta ? M : K) & 3 || (d.tb ? K : N) & 3) return KGAT_ERR_INVALID;
  if (d.lda1 < (d.ta ? M : K) || d.lda2 < (d.ta ? M : K) || d.ldb1 < (d.tb ? K : N) || d.ldb2 < (d.tb ? K : N) ||
      d.ldc1 < N || d.ldc2 < N)
    return KGAT_ERR_INVALID;
  if (d.dxs && (!d.X || !d.S || d.ldx < N || d.lds < N || d.batch != 1)) return KGAT_ERR_INVALID;
  if ((d.arows && d.ta) || (d.brows && d.tb) || (d.erows && !d.dxs)) return KGAT_ERR_INVALID;  // row lists
  if (d.a_um && d.ta) return KGAT_ERR_INVALID;  // (X+S, X*S) pairs: row-major k-contiguous A only
  if (d.b_um && d.tb) return KGAT_ERR_INVALID;  // ... and row-major [K, N] B only
  if ((d.cs1 != nullptr) != (d.cs2 != nullptr) || (d.cs1 && !d.ta)) return KGAT_ERR_INVALID;
  const int64_t tiles = ((M + kBM - 1) / kBM) * ((N + kBN - 1) / kBN);
  if (tiles > 0x7fffffff || d.batch > 65535) return KGAT_ERR_INVALID;
  DualArgs g{d.A1, d.A2, d.lda1, d.lda2, d.sA1, d.sA2, d.B1, d.B2, d.ldb1, d.ldb2, d.sB1, d.sB2,
             d.C1, d.C2, d.ldc1, d.ldc2, d.sC1, d.sC2, M, N, K, d.cs1, d.cs2, d.ldcs, d.sCS1, d.sCS2,
             d.X, d.S, d.ldx, d.lds, d.arows, d.brows, d.sBrows, d.erows};
  const dim3 grid(static_cast<unsigned>(tiles), 1, static_cast<unsigned>(d.batch));
  // the three forms the bi-interaction uses: forward (UM x W^T), backward du/dm + dXd/dS
  // epilogue (dA.W), weight gradients (dA^T x UM, split-K batches, column sums)
// 16-deep stages: the four operand images of two 16-deep buffers are 80 KB, so two blocks (two waves
// per SIMD, <= 256 registers each) share a CU; 32-deep stages would leave one
#define KGAT_DUAL_LAUNCH(TA_, TB_, AOP_, BOP_, EPI_) \
  hipLaunchKernelGGL((dual_gemm_kernel<TA_, TB_, AOP_, BOP_, EPI_, 16>), grid, dim3(kThreads), 0, st, g)
  if (!d.ta && d.tb && d.a_um && !d.b_um && !d.dxs)
    KGAT_DUAL_LAUNCH(false, true, kUM, kSep, kStore);
  else if (!d.ta && !d.tb && !d.a_um && !d.b_um && d.dxs)
    KGAT_DUAL_LAUNCH(false, false, kSep, kSep, kDXS);
  else if (d.ta && !d.tb && !d.a_um && d.b_um && !d.dxs)
    KGAT_DUAL_LAUNCH(true, false, kSep, kUM, kStore);
  else if (!d.ta && d.tb && !d.a_um && !d.b_um && !d.dxs)
    KGAT_DUAL_LAUNCH(false, true, kSep, kSep, kStore);
  else
    return KGAT_ERR_UNSUPPORTED_DIM;
#undef KGAT_DUAL_LAUNCH
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

int gemm_f32(bool ta, bool tb, int64_t M, int64_t N, int64_t K, const float* A, int64_t lda, int64_t sA,
             const float* B, int64_t ldb, int64_t sB, float* C, int64_t ldc, int64_t sC, int64_t batch,
             bool accumulate, hipStream_t st) {
  if (M < 0 || N < 0 || K < 0 || batch < 0 || !A || !B || !C) return KGAT_ERR_INVALID;
  if (M == 0 || N == 0 || batch == 0) return KGAT_OK;
  // float4 loads: leading dimensions, batch strides and bases 16-byte aligned; the contiguous
  // dimension of each operand a multiple of 4 (k for A / B^T, m for A^T, n for B)
  if ((lda | ldb | sA | sB) & 3 || !aligned16(A) || !aligned16(B)) return KGAT_ERR_INVALID;
  if ((ta ? M : K) & 3 || (tb ? K : N) & 3) return KGAT_ERR_INVALID;
  if (lda < (ta ? M : K) || ldb < (tb ? K : N) || ldc < N) return KGAT_ERR_INVALID;
  if (K == 0) {
    if (accumulate) return KGAT_OK;
    for (int64_t z = 0; z < batch; ++z)
      if (hipError_t e = hipMemset2DAsync(C + z * sC, ldc * sizeof(float), 0, N * sizeof(float), M, st);
          e != hipSuccess)
        return static_cast<int>(e);
    return KGAT_OK;
  }
  const int64_t tiles = ((M + kBM - 1) / kBM) * ((N + kBN - 1) / kBN);
  if (tiles > 0x7fffffff || batch > 65535) return KGAT_ERR_INVALID;
  GemmArgs g{A, B, C, lda, ldb, ldc, sA, sB, sC, M, N, K, accumulate ? 1 : 0, nullptr, 0, 0};
  const dim3 grid(static_cast<unsigned>(tiles), 1, static_cast<unsigned>(batch));
// 16-deep stages (32 measured no faster, same bits: the k order is fixed by the tile)
#define KGAT_GEMM_LAUNCH(TA_, TB_) hipLaunchKernelGGL((gemm_kernel<TA_, TB_, 16>), grid, dim3(kThreads), 0, st, g)
  if (ta) {
    if (tb) KGAT_GEMM_LAUNCH(true, true);
    else KGAT_GEMM_LAUNCH(true, false);
  } else {
    if (tb) KGAT_GEMM_LAUNCH(false, true);
    else KGAT_GEMM_LAUNCH(false, false);
  }
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

}  // namespace kgat

extern "C" int kgat_gemm_f32(int32_t trans_a, int32_t trans_b, int64_t m, int64_t n, int64_t k, const float* A,
                             int64_t lda, int64_t stride_a, const float* B, int64_t ldb, int64_t stride_b, float* C,
                             int64_t ldc, int64_t stride_c, int64_t batch, int32_t accumulate, void* stream) {
  return kgat::gemm_f32(trans_a != 0, trans_b != 0, m, n, k, A, lda, stride_a, B, ldb, stride_b, C, ldc, stride_c,
                        batch, accumulate != 0, reinterpret_cast<hipStream_t>(stream));
}
