// a1 -- attentive-propagation SpMM over a CSR graph: Y = A . X (+ Y).
//
// Replaces torch.matmul(sparse attentive_matrix, ego) at
// src/model/KGAT/aggregator.py:54 (and its autograd A^T . G when called with
// the transposed CSR).  HBM-bound gather: per edge 4 B col + 4 B val + 4*d B
// of the source row.
//
// Layout of the work:
//  * a row of d floats is read as d/4 float4 lanes ("a group"); a wave holds
//    64/(d/4) groups, each owning one destination row at a time, so a wave
//    keeps up to 64/(d/4) gathered rows x unroll in flight;
//  * every group walks its row's edges in chunks of d/4: the group's lanes
//    load the chunk's (col, val) pairs cooperatively (one coalesced load
//    each), then broadcast them with ds_bpermute while the float4 row loads
//    are issued 4 at a time;
//  * rows with degree > long_threshold (power-law hubs: popular problems)
//    would serialise one group for thousands of edges, so they are cut into
//    seg_len-edge segments handled by whole waves (blocks scheduled first),
//    written as partial sums and reduced in segment order by a fix-up pass.
//    Every output is therefore produced in a fixed order: deterministic.
#include "common.hpp"

namespace kgat {

template <int D>
struct SpmmShape {
  static constexpr int kLanes = D / 4;            // float4 lanes per row
  static constexpr int kGroups = kWave / kLanes;  // rows in flight per wave
  static constexpr int kRowsPerGroup = 4;
  static constexpr int kRowsPerWave = kGroups * kRowsPerGroup;
  static constexpr int kRowsPerBlock = kRowsPerWave * 4;  // 256-thread blocks
};

__device__ __forceinline__ void fma4(float v, const float4& x, float4& acc) {
  acc.x = fmaf(v, x.x, acc.x);
  acc.y = fmaf(v, x.y, acc.y);
  acc.z = fmaf(v, x.z, acc.z);
  acc.w = fmaf(v, x.w, acc.w);
}

// Accumulate edges [beg, end) of one row into acc.  All lanes of the group
// (base .. base+kLanes-1) run this with identical bounds (group-uniform).
template <int D>
__device__ __forceinline__ void gather_edges(const kgat_csr& A, const float4* __restrict__ X4, int64_t ldx4,
                                             int64_t beg, int64_t end, int base, int gl, float4& acc) {
  constexpr int L = SpmmShape<D>::kLanes;
  for (int64_t cb = beg; cb < end; cb += L) {
    const int n = static_cast<int>(end - cb < L ? end - cb : L);
    int mc = 0;
    float mv = 0.f;
    if (gl < n) {
      mc = A.col[cb + gl];
      mv = A.val[cb + gl];
    }
    int j = 0;
    for (; j + 4 <= n; j += 4) {
      const int c0 = __shfl(mc, base + j), c1 = __shfl(mc, base + j + 1);
      const int c2 = __shfl(mc, base + j + 2), c3 = __shfl(mc, base + j + 3);
      const float v0 = __shfl(mv, base + j), v1 = __shfl(mv, base + j + 1);
      const float v2 = __shfl(mv, base + j + 2), v3 = __shfl(mv, base + j + 3);
      const float4 x0 = X4[static_cast<int64_t>(c0) * ldx4 + gl];
      const float4 x1 = X4[static_cast<int64_t>(c1) * ldx4 + gl];
      const float4 x2 = X4[static_cast<int64_t>(c2) * ldx4 + gl];
      const float4 x3 = X4[static_cast<int64_t>(c3) * ldx4 + gl];
      fma4(v0, x0, acc);
      fma4(v1, x1, acc);
      fma4(v2, x2, acc);
      fma4(v3, x3, acc);
    }
    for (; j < n; ++j) {
      const int c = __shfl(mc, base + j);
      const float v = __shfl(mv, base + j);
      fma4(v, X4[static_cast<int64_t>(c) * ldx4 + gl], acc);
    }
  }
}

template <int D, bool ACC>
__global__ __launch_bounds__(256) void spmm_main_kernel(kgat_csr A, const float* __restrict__ X, int64_t ldx,
                                                        float* __restrict__ Y, int64_t ldy,
                                                        float* __restrict__ part, int seg_blocks) {
  using S = SpmmShape<D>;
  constexpr int L = S::kLanes;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int g = lane / L, gl = lane % L, base = g * L;
  const float4* X4 = reinterpret_cast<const float4*>(X);
  const int64_t ldx4 = ldx / 4;

  if (static_cast<int>(blockIdx.x) < seg_blocks) {
    // ---- long-row segment: the whole wave, groups take interleaved sub-chunks
    const int s = blockIdx.x * 4 + wave;
    if (s >= A.n_seg) return;
    const int row = A.seg_row[s];
    const int64_t beg = A.seg_beg[s];
    const int64_t row_end = A.rowptr[row + 1];
    const int64_t end = beg + A.seg_len < row_end ? beg + A.seg_len : row_end;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    // group g handles edges [beg + g*L + k*64, ... + L) for k = 0, 1, ...
    for (int64_t cb = beg + g * L; cb < end; cb += kWave) {
      const int64_t ce = cb + L < end ? cb + L : end;
      gather_edges<D>(A, X4, ldx4, cb, ce, base, gl, acc);
    }
#pragma unroll
    for (int o = L; o < kWave; o <<= 1) {
      acc.x += __shfl_xor(acc.x, o);
      acc.y += __shfl_xor(acc.y, o);
      acc.z += __shfl_xor(acc.z, o);
      acc.w += __shfl_xor(acc.w, o);
    }
    if (g == 0) reinterpret_cast<float4*>(part)[static_cast<int64_t>(s) * L + gl] = acc;
    return;
  }

  // ---- short rows: one group per row
  const int64_t w = static_cast<int64_t>(blockIdx.x - seg_blocks) * 4 + wave;
  const int64_t r_begin = w * S::kRowsPerWave;
  int64_t r_end = r_begin + S::kRowsPerWave;
  if (r_end > A.n_rows) r_end = A.n_rows;
  for (int64_t r = r_begin + g; r < r_end; r += S::kGroups) {
    const int64_t beg = A.rowptr[r], end = A.rowptr[r + 1];
    if (end - beg > A.long_threshold) continue;  // produced by the fix-up pass
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    gather_edges<D>(A, X4, ldx4, beg, end, base, gl, acc);
    float4* y = reinterpret_cast<float4*>(Y + r * ldy) + gl;
    if (ACC) {
      const float4 o = *y;
      acc.x += o.x;
      acc.y += o.y;
      acc.z += o.z;
      acc.w += o.w;
    }
    *y = acc;
  }
}

// Sum the segment partials of each long row in segment order.
template <int D, bool ACC>
__global__ __launch_bounds__(256) void spmm_fixup_kernel(kgat_csr A, const float* __restrict__ part,
                                                         float* __restrict__ Y, int64_t ldy) {
  constexpr int L = D / 4;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (wave >= A.n_long || lane >= L) return;
  const int row = A.long_rows[wave];
  const float4* P = reinterpret_cast<const float4*>(part);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int s = A.long_seg_off[wave]; s < A.long_seg_off[wave + 1]; ++s) {
    const float4 p = P[static_cast<int64_t>(s) * L + lane];
    acc.x += p.x;
    acc.y += p.y;
    acc.z += p.z;
    acc.w += p.w;
  }
  float4* y = reinterpret_cast<float4*>(Y + static_cast<int64_t>(row) * ldy) + lane;
  if (ACC) {
    const float4 o = *y;
    acc.x = o.x + acc.x;
    acc.y = o.y + acc.y;
    acc.z = o.z + acc.z;
    acc.w = o.w + acc.w;
  }
  *y = acc;
}

template <int D>
static int launch_spmm(const kgat_csr& A, const float* X, int64_t ldx, float* Y, int64_t ldy, bool acc,
                       float* ws, hipStream_t st) {
  using S = SpmmShape<D>;
  const int seg_blocks = (A.n_seg + 3) / 4;
  const int64_t row_blocks = (A.n_rows + S::kRowsPerBlock - 1) / S::kRowsPerBlock;
  const int64_t grid = seg_blocks + row_blocks;
  if (grid > 0x7fffffff) return KGAT_ERR_INVALID;
  if (acc)
    hipLaunchKernelGGL((spmm_main_kernel<D, true>), dim3(grid), dim3(256), 0, st, A, X, ldx, Y, ldy, ws,
                       seg_blocks);
  else
    hipLaunchKernelGGL((spmm_main_kernel<D, false>), dim3(grid), dim3(256), 0, st, A, X, ldx, Y, ldy, ws,
                       seg_blocks);
  KGAT_LAUNCH_CHECK();
  if (A.n_long > 0) {
    const int fb = (A.n_long + 3) / 4;
    if (acc)
      hipLaunchKernelGGL((spmm_fixup_kernel<D, true>), dim3(fb), dim3(256), 0, st, A, ws, Y, ldy);
    else
      hipLaunchKernelGGL((spmm_fixup_kernel<D, false>), dim3(fb), dim3(256), 0, st, A, ws, Y, ldy);
    KGAT_LAUNCH_CHECK();
  }
  return KGAT_OK;
}

}  // namespace kgat

extern "C" int kgat_spmm_csr_f32(const kgat_csr* A, const float* X, int64_t ldx, float* Y, int64_t ldy,
                                 int32_t d, int32_t accumulate, float* workspace, int64_t workspace_floats,
                                 void* stream) {
  if (!A || !X || !Y || A->n_rows < 0 || ldx < d || ldy < d || (ldx & 3) || (ldy & 3)) return KGAT_ERR_INVALID;
  if ((reinterpret_cast<uintptr_t>(X) & 15) || (reinterpret_cast<uintptr_t>(Y) & 15)) return KGAT_ERR_INVALID;
  if (A->n_rows == 0) return KGAT_OK;
  if (A->n_seg > 0 && (workspace == nullptr || workspace_floats < static_cast<int64_t>(A->n_seg) * d))
    return KGAT_ERR_WORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const bool acc = accumulate != 0;
  switch (d) {
    case 16: return kgat::launch_spmm<16>(*A, X, ldx, Y, ldy, acc, workspace, st);
    case 32: return kgat::launch_spmm<32>(*A, X, ldx, Y, ldy, acc, workspace, st);
    case 64: return kgat::launch_spmm<64>(*A, X, ldx, Y, ldy, acc, workspace, st);
    case 128: return kgat::launch_spmm<128>(*A, X, ldx, Y, ldy, acc, workspace, st);
    case 256: return kgat::launch_spmm<256>(*A, X, ldx, Y, ldy, acc, workspace, st);
    default: return KGAT_ERR_UNSUPPORTED_DIM;
  }
}
