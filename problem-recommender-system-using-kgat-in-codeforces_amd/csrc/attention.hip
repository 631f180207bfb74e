// a6/a7 -- knowledge-aware attention refresh (src/model/KGAT/model.py:263-366,
// src/model/KGAT/multi_head_attention.py:35-58).
//
// Edge scorer, per edge e = (h, t, r):
//   t' = e_t W_r                      (TransR projection, W_r = trans[r], d x d)
//   v  = W_v t' + b_v                 (MHA value path; the query/key path is dead:
//                                      softmax over a size-1 key axis is exactly 1)
//   v  = v * drop(1.0) per head       (train mode: MHA attention dropout)
//   o  = LayerNorm(W_o v + b_o)       (eps 1e-5, affine)
//   logit_e = sum_j tanh(o_j) / (log1p(deg_h) + log1p(deg_t))   (per-relation degrees)
// Edges are processed in 16-edge tiles of ONE relation (a relation-sorted
// permutation built once per graph), one tile per wave: the three d x d
// contractions are fp32 MFMA (v_mfma_f32_16x16x4_f32) chains, the tile is
// re-laid from accumulator layout to operand layout through a per-wave LDS
// scratch, and LayerNorm / tanh / sum are fused epilogues.
//
// Neighbour softmax: A[h, :] = softmax over the stored entries of row h
// (torch.sparse.softmax(dim=1), model.py:364), one wave per CSR row.
#include <cmath>

#include "common.hpp"

namespace kgat {

constexpr float kLnEps = 1e-5f;  // nn.LayerNorm default

struct EdgeScoreArgs {
  const float* emb;
  int64_t ld_emb;
  int64_t n_nodes;
  const float* trans;  // [R][D][D]
  const float* Wv;     // [D][D] (nn.Linear: out x in)
  const float* bv;
  const float* Wo;
  const float* bo;
  const float* ln_w;
  const float* ln_b;
  const int32_t* tails;        // [E] edge order
  const float* edge_weight;    // [E]
  const int32_t* rel_perm;     // [E] relation-sorted edge ids
  const int32_t* tile_rel;     // [T]
  const int32_t* tile_beg;     // [T + 1] into rel_perm
  int32_t n_tiles;
  float p;
  uint64_t seed;
  const int32_t* out_pos;      // [E] edge -> output position (nullable: edge order)
  float* logits;
};

template <int D>
__device__ __forceinline__ void load_a(const float* __restrict__ P, int64_t ld, int64_t row, int q,
                                       float (&out)[D / 4]) {
  constexpr int KQ = D / 4;
  if (row >= 0) {
    const float4* p = reinterpret_cast<const float4*>(P + row * ld + q * KQ);
#pragma unroll
    for (int t = 0; t < KQ / 4; ++t) {
      const float4 v = p[t];
      out[4 * t] = v.x;
      out[4 * t + 1] = v.y;
      out[4 * t + 2] = v.z;
      out[4 * t + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int t = 0; t < KQ; ++t) out[t] = 0.f;
  }
}

// C-layout accumulators -> LDS tile [16][D+4] -> A-operand layout registers.
template <int D>
__device__ __forceinline__ void relayout(float* tile, const floatx4 (&acc)[D / 16], int q, int c,
                                         float (&out)[D / 4]) {
  constexpr int TLD = D + 4, KQ = D / 4;
#pragma unroll
  for (int cb = 0; cb < D / 16; ++cb)
#pragma unroll
    for (int i = 0; i < 4; ++i) tile[(q * 4 + i) * TLD + cb * 16 + c] = acc[cb][i];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const float* src = tile + c * TLD + q * KQ;
#pragma unroll
  for (int t = 0; t < KQ; t += 4) {
    const float4 v = *reinterpret_cast<const float4*>(src + t);
    out[t] = v.x;
    out[t + 1] = v.y;
    out[t + 2] = v.z;
    out[t + 3] = v.w;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// acc[cb] = A . W^T for nn.Linear weight W [D out][D in] (row stride wld),
// A in operand layout (k = q*KQ + step).
template <int D>
__device__ __forceinline__ void linear_t(const float (&a)[D / 4], const float* W, int wld, int q, int c,
                                         floatx4 (&acc)[D / 16]) {
  constexpr int KQ = D / 4;
#pragma unroll
  for (int cb = 0; cb < D / 16; ++cb) {
    __builtin_amdgcn_sched_barrier(0);
    floatx4 s = {0.f, 0.f, 0.f, 0.f};
    const float* w = W + (cb * 16 + c) * wld + q * KQ;
#pragma unroll
    for (int t = 0; t < KQ; t += 4) {
      const float4 x = *reinterpret_cast<const float4*>(w + t);
      s = mfma16x4(a[t], x.x, s);
      s = mfma16x4(a[t + 1], x.y, s);
      s = mfma16x4(a[t + 2], x.z, s);
      s = mfma16x4(a[t + 3], x.w, s);
    }
    acc[cb] = s;
  }
}

template <int D, bool WLDS>
__global__ __launch_bounds__(256) void edge_score_kernel(EdgeScoreArgs a) {
  constexpr int KQ = D / 4, NCB = D / 16, WLD = D + 4, TLD = D + 4;
  constexpr int kDepth = D / 8;  // 8 heads (multi_head_attention.py:6)
  constexpr int kWFloats = WLDS ? 2 * D * WLD : 0;
  __shared__ __attribute__((aligned(16))) float smem[kWFloats + 4 * 16 * TLD];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, q = lane >> 4, c = lane & 15;
  const float* wv = a.Wv;
  const float* wo = a.Wo;
  int wld = D;
  if constexpr (WLDS) {
    for (int i = threadIdx.x; i < D * D / 4; i += 256) {
      const int j = (i * 4) / D, k = (i * 4) % D;
      *reinterpret_cast<float4*>(smem + j * WLD + k) = reinterpret_cast<const float4*>(a.Wv)[i];
      *reinterpret_cast<float4*>(smem + D * WLD + j * WLD + k) = reinterpret_cast<const float4*>(a.Wo)[i];
    }
    __syncthreads();
    wv = smem;
    wo = smem + D * WLD;
    wld = WLD;
  }
  float* tile = smem + kWFloats + wave * 16 * TLD;
  float bv[NCB], bo[NCB], lw[NCB], lb[NCB];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) {
    bv[cb] = a.bv[cb * 16 + c];
    bo[cb] = a.bo[cb * 16 + c];
    lw[cb] = a.ln_w[cb * 16 + c];
    lb[cb] = a.ln_b[cb * 16 + c];
  }
  const float scale = a.p > 0.f ? 1.f / (1.f - a.p) : 1.f;
  for (int tl = blockIdx.x * 4 + wave; tl < a.n_tiles; tl += gridDim.x * 4) {
    const int beg = a.tile_beg[tl], cnt = a.tile_beg[tl + 1] - beg;
    const int64_t r = a.tile_rel[tl];
    const int ea = c < cnt ? a.rel_perm[beg + c] : -1;  // A-operand row edge
    float x[KQ];
    load_a<D>(a.emb, a.ld_emb, ea >= 0 ? static_cast<int64_t>(a.tails[ea]) : -1, q, x);
    // t' = e_t W_r : B[k][j] = W_r[k][j], k = q*KQ + step
    floatx4 acc[NCB];
    const float* Wr = a.trans + r * D * D;
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) {
      __builtin_amdgcn_sched_barrier(0);
      floatx4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < KQ; ++t) s = mfma16x4(x[t], Wr[(q * KQ + t) * D + cb * 16 + c], s);
      acc[cb] = s;
    }
    relayout<D>(tile, acc, q, c, x);
    // v = W_v t' + b_v, with the per-(edge, head) attention dropout of train mode
    linear_t<D>(x, wv, wld, q, c, acc);
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = acc[cb][i] + bv[cb];
        if (a.p > 0.f) {
          const int er = q * 4 + i;
          const int64_t e = er < cnt ? a.rel_perm[beg + er] : 0;
          const int head = (cb * 16 + c) / kDepth;
          v = dropout_keep(a.seed, static_cast<uint64_t>(e) * 8 + head, a.p) ? v * scale : 0.f;
        }
        acc[cb][i] = v;
      }
    relayout<D>(tile, acc, q, c, x);
    // o = W_o v + b_o, then LayerNorm and sum tanh
    linear_t<D>(x, wo, wld, q, c, acc);
    float mean[4], var[4], tsum[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float s = 0.f;
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        acc[cb][i] += bo[cb];
        s += acc[cb][i];
      }
      mean[i] = sum16(s) / static_cast<float>(D);
      float v2 = 0.f;
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        const float dlt = acc[cb][i] - mean[i];
        v2 = fmaf(dlt, dlt, v2);
      }
      var[i] = sum16(v2) / static_cast<float>(D);
      const float rstd = 1.f / sqrtf(var[i] + kLnEps);
      float ts = 0.f;
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) ts += tanhf((acc[cb][i] - mean[i]) * rstd * lw[cb] + lb[cb]);
      tsum[i] = sum16(ts);
    }
    if (c == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int er = q * 4 + i;
        if (er < cnt) {
          const int e = a.rel_perm[beg + er];
          a.logits[a.out_pos ? a.out_pos[e] : e] = tsum[i] * a.edge_weight[e];
        }
      }
    }
  }
}

// slot logit = sum of the logits of the edges stored at that CSR slot
// (duplicate (h, t) pairs across relations are summed before the softmax);
// edges of slot s are order[ptr[s] .. ptr[s+1]).
__global__ __launch_bounds__(256) void slot_sum_kernel(const int64_t* __restrict__ ptr, const int32_t* __restrict__ order,
                                                       int64_t nnz, const float* __restrict__ elog,
                                                       float* __restrict__ slog) {
  const int64_t s = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (s >= nnz) return;
  float v = 0.f;
  for (int64_t e = ptr[s]; e < ptr[s + 1]; ++e) v += elog[order[e]];
  slog[s] = v;
}

// val[slot] = softmax over the stored entries of each row (model.py:355-366, torch.sparse.softmax).
// Rows of <= 256 entries (all but the hubs) take a 4-lane group each, 16 rows per wave in flight: a row of
// <= 32 entries is read once into 8 registers per lane (max, exp-sum, write from registers), a longer one
// in max / exp-sum / write passes of 32-entry chunks (the later passes re-read it from L1/L2).  Lane j of
// the group holds entries j, j + 4, ...; the lane partials reduce in a fixed butterfly (deterministic, and
// the same bits wherever the row sits).  Longer rows: the segment plan below.
constexpr int kSoftmaxShort = 256;

__device__ __forceinline__ void short_row_softmax(const int64_t* __restrict__ rowptr, int64_t row, int j,
                                                  const float* __restrict__ logit, float* __restrict__ val) {
  const int64_t beg = rowptr[row], end = rowptr[row + 1];
  const int64_t len = end - beg;
  if (len == 0 || len > kSoftmaxShort) return;  // (group-uniform) long rows: the segment kernels
  if (len <= 32) {
    float x[8];
    float m = -INFINITY;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int64_t e = beg + j + 4 * k;
      x[k] = e < end ? logit[e] : -INFINITY;
      m = fmaxf(m, x[k]);
    }
    m = fmaxf(m, __shfl_xor(m, 1));
    m = fmaxf(m, __shfl_xor(m, 2));
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      x[k] = beg + j + 4 * k < end ? expf(x[k] - m) : 0.f;
      s += x[k];
    }
    s += __shfl_xor(s, 1);
    s += __shfl_xor(s, 2);
    const float inv = 1.f / s;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int64_t e = beg + j + 4 * k;
      if (e < end) val[e] = x[k] * inv;
    }
    return;
  }
  float m = -INFINITY;
  for (int64_t e = beg + j; e < end; e += 4) m = fmaxf(m, logit[e]);
  m = fmaxf(m, __shfl_xor(m, 1));
  m = fmaxf(m, __shfl_xor(m, 2));
  float s = 0.f;
  for (int64_t e = beg + j; e < end; e += 4) s += expf(logit[e] - m);
  s += __shfl_xor(s, 1);
  s += __shfl_xor(s, 2);
  const float inv = 1.f / s;
  for (int64_t e = beg + j; e < end; e += 4) val[e] = expf(logit[e] - m) * inv;
}

__global__ __launch_bounds__(256) void row_softmax_kernel(const int64_t* __restrict__ rowptr, int64_t n_rows,
                                                          const float* __restrict__ logit, float* __restrict__ val) {
  const int64_t row = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 2;
  if (row >= n_rows) return;  // whole 4-lane groups leave together
  short_row_softmax(rowptr, row, threadIdx.x & 3, logit, val);
}

// Long rows, cut into the CSR's long-row plan segments (one wave each, <= kSoftmaxSeg entries, 8 per lane
// in registers).  Pass 1 (with the short rows, segment waves first): each segment's max m_s and
// s_s = sum exp(x - m_s) -> stat[2s], stat[2s + 1].  Pass 2: every segment wave of a row combines the
// row's segment stats in segment order -- M = max m_s, S = sum_s s_s exp(m_s - M), lane-strided partials
// then a fixed butterfly, the same bits in every wave of the row -- and writes its own entries
// exp(x - M) / S.  A hub row of 10^5 entries runs on ~200 waves instead of one block's three serial passes.
constexpr int kSoftmaxSeg = 512;

__global__ __launch_bounds__(256) void row_softmax_stats_kernel(kgat_csr A, const float* __restrict__ logit,
                                                                float* __restrict__ val, float* __restrict__ stat,
                                                                int seg_blocks) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (static_cast<int>(blockIdx.x) >= seg_blocks) {  // short rows (row_softmax_kernel's body)
    const int64_t row = (static_cast<int64_t>(blockIdx.x - seg_blocks) * blockDim.x + threadIdx.x) >> 2;
    if (row < A.n_rows) short_row_softmax(A.rowptr, row, threadIdx.x & 3, logit, val);
    return;
  }
  const int sg = blockIdx.x * 4 + wave;
  if (sg >= A.n_seg) return;
  const int64_t row = A.seg_row[sg];
  const int64_t beg = A.seg_beg[sg], row_end = A.rowptr[row + 1];
  const int64_t end = beg + kSoftmaxSeg < row_end ? beg + kSoftmaxSeg : row_end;
  float x[kSoftmaxSeg / 64];
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < kSoftmaxSeg / 64; ++k) {
    const int64_t e = beg + lane + 64 * k;
    x[k] = e < end ? logit[e] : -INFINITY;
    m = fmaxf(m, x[k]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < kSoftmaxSeg / 64; ++k) s += beg + lane + 64 * k < end ? expf(x[k] - m) : 0.f;
  s = wave_sum(s);
  if (lane == 0) {
    stat[2 * static_cast<int64_t>(sg)] = m;
    stat[2 * static_cast<int64_t>(sg) + 1] = s;
  }
}

__global__ __launch_bounds__(256) void row_softmax_seg_write_kernel(kgat_csr A, const float* __restrict__ logit,
                                                                    const float* __restrict__ stat,
                                                                    float* __restrict__ val) {
  const int sg = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (sg >= A.n_seg) return;
  const int64_t row = A.seg_row[sg];
  const int64_t rbeg = A.rowptr[row], rend = A.rowptr[row + 1];
  const int64_t beg = A.seg_beg[sg];
  const int s0 = sg - static_cast<int>((beg - rbeg) / kSoftmaxSeg);  // the row's first segment
  const int ns = static_cast<int>((rend - rbeg + kSoftmaxSeg - 1) / kSoftmaxSeg);
  float M = -INFINITY;
  for (int i = lane; i < ns; i += 64) M = fmaxf(M, stat[2 * static_cast<int64_t>(s0 + i)]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) M = fmaxf(M, __shfl_xor(M, o));
  float S = 0.f;
  for (int i = lane; i < ns; i += 64) {
    const int64_t k = 2 * static_cast<int64_t>(s0 + i);
    S += stat[k + 1] * expf(stat[k] - M);
  }
  S = wave_sum(S);
  const float inv = 1.f / S;
  const int64_t end = beg + kSoftmaxSeg < rend ? beg + kSoftmaxSeg : rend;
#pragma unroll
  for (int k = 0; k < kSoftmaxSeg / 64; ++k) {
    const int64_t e = beg + lane + 64 * k;
    if (e < end) val[e] = expf(logit[e] - M) * inv;
  }
}

// Rows longer than kSoftmaxShort found by a scan of all rows (callers without a
// long-row list): one wave per row.
__global__ __launch_bounds__(256) void row_softmax_scan_long_kernel(const int64_t* __restrict__ rowptr, int64_t n_rows,
                                                                    const float* __restrict__ logit,
                                                                    float* __restrict__ val) {
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n_rows) return;
  const int64_t beg = rowptr[row], end = rowptr[row + 1];
  if (end - beg <= kSoftmaxShort) return;
  float m = -INFINITY;
  for (int64_t e = beg + lane; e < end; e += 64) m = fmaxf(m, logit[e]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  float s = 0.f;
  for (int64_t e = beg + lane; e < end; e += 64) s += expf(logit[e] - m);
  const float inv = 1.f / wave_sum(s);
  for (int64_t e = beg + lane; e < end; e += 64) val[e] = expf(logit[e] - m) * inv;
}

// Rows longer than kSoftmaxShort: one 256-thread block per row, block
// reductions in a fixed order.
__global__ __launch_bounds__(256) void row_softmax_long_kernel(const int64_t* __restrict__ rowptr,
                                                               const int32_t* __restrict__ long_rows,
                                                               const float* __restrict__ logit,
                                                               float* __restrict__ val) {
  __shared__ float red[4];
  const int64_t row = long_rows[blockIdx.x];
  const int64_t beg = rowptr[row], end = rowptr[row + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float m = -INFINITY;
  for (int64_t e = beg + threadIdx.x; e < end; e += 256) m = fmaxf(m, logit[e]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if (lane == 0) red[wave] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float s = 0.f;
  for (int64_t e = beg + threadIdx.x; e < end; e += 256) s += expf(logit[e] - m);
  s = wave_sum(s);
  if (lane == 0) red[wave] = s;
  __syncthreads();
  const float inv = 1.f / (((red[0] + red[1]) + red[2]) + red[3]);
  for (int64_t e = beg + threadIdx.x; e < end; e += 256) val[e] = expf(logit[e] - m) * inv;
}

template <int D>
static int launch_scores(const EdgeScoreArgs& a, hipStream_t st) {
  constexpr bool wlds = D <= 64;
  const int grid = blocks_for(a.n_tiles, 4, kCUs * 8);
  hipLaunchKernelGGL((edge_score_kernel<D, wlds>), dim3(grid), dim3(256), 0, st, a);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

}  // namespace kgat

extern "C" int64_t kgat_row_softmax_work_floats(const kgat_csr* A) { return A ? 2 * static_cast<int64_t>(A->n_seg) + 2 : -1; }

extern "C" int kgat_row_softmax_plan_f32(const kgat_csr* A, const float* slot_logits, float* val, float* work,
                                         int64_t work_floats, void* stream) {
  if (!A || !slot_logits || !val || A->n_rows < 0) return KGAT_ERR_INVALID;
  if (A->n_seg > 0 && (A->seg_len != kgat::kSoftmaxSeg || A->long_threshold != kgat::kSoftmaxShort))
    return KGAT_ERR_INVALID;  // the plan's cut must be the softmax's
  if (A->n_rows == 0) return KGAT_OK;
  if (!work || work_floats < kgat_row_softmax_work_floats(A)) return KGAT_ERR_WORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int seg_blocks = (A->n_seg + 3) / 4;
  const int64_t grid = seg_blocks + (A->n_rows * 4 + 255) / 256;
  if (grid > 0x7fffffff) return KGAT_ERR_INVALID;
  hipLaunchKernelGGL(kgat::row_softmax_stats_kernel, dim3(grid), dim3(256), 0, st, *A, slot_logits, val, work,
                     seg_blocks);
  KGAT_LAUNCH_CHECK();
  if (A->n_seg > 0) {
    hipLaunchKernelGGL(kgat::row_softmax_seg_write_kernel, dim3(seg_blocks), dim3(256), 0, st, *A, slot_logits, work,
                       val);
    KGAT_LAUNCH_CHECK();
  }
  return KGAT_OK;
}

extern "C" int kgat_row_softmax_ex_f32(const int64_t* rowptr, int64_t n_rows, const int32_t* long_rows,
                                       int32_t n_long, const float* slot_logits, float* val, void* stream) {
  if (!rowptr || !slot_logits || !val || n_rows < 0 || n_long < 0 || (n_long > 0 && !long_rows))
    return KGAT_ERR_INVALID;
  if (n_rows == 0) return KGAT_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(kgat::row_softmax_kernel, dim3((n_rows * 4 + 255) / 256), dim3(256), 0, st, rowptr, n_rows,
                     slot_logits, val);
  KGAT_LAUNCH_CHECK();
  if (long_rows == nullptr) {
    hipLaunchKernelGGL(kgat::row_softmax_scan_long_kernel, dim3((n_rows + 3) / 4), dim3(256), 0, st, rowptr, n_rows,
                       slot_logits, val);
    KGAT_LAUNCH_CHECK();
  } else if (n_long > 0) {
    hipLaunchKernelGGL(kgat::row_softmax_long_kernel, dim3(n_long), dim3(256), 0, st, rowptr, long_rows, slot_logits,
                       val);
    KGAT_LAUNCH_CHECK();
  }
  return KGAT_OK;
}

extern "C" int kgat_edge_logits_f32(const float* emb, int64_t ld_emb, int64_t n_nodes, const float* trans, int32_t d,
                                    const float* Wv, const float* bv, const float* Wo, const float* bo,
                                    const float* ln_w, const float* ln_b, const int32_t* tails,
                                    const float* edge_weight, const int32_t* rel_perm, const int32_t* tile_rel,
                                    const int32_t* tile_beg, int32_t n_tiles, float dropout_p, uint64_t seed,
                                    const int32_t* out_pos, float* logits, void* stream) {
  if (!emb || !trans || !Wv || !bv || !Wo || !bo || !ln_w || !ln_b || !tails || !edge_weight || !rel_perm ||
      !tile_rel || !tile_beg || !logits || n_tiles < 0 || ld_emb < d || (ld_emb & 3) || n_nodes < 0)
    return KGAT_ERR_INVALID;
  if (!(dropout_p >= 0.f && dropout_p < 1.f)) return KGAT_ERR_INVALID;
  if (n_tiles == 0) return KGAT_OK;
  const kgat::EdgeScoreArgs a{emb, ld_emb, n_nodes, trans, Wv, bv, Wo, bo, ln_w, ln_b, tails, edge_weight,
                              rel_perm, tile_rel, tile_beg, n_tiles, dropout_p, seed, out_pos, logits};
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  switch (d) {
    case 16: return kgat::launch_scores<16>(a, st);
    case 32: return kgat::launch_scores<32>(a, st);
    case 64: return kgat::launch_scores<64>(a, st);
    case 128: return kgat::launch_scores<128>(a, st);
    default: return KGAT_ERR_UNSUPPORTED_DIM;
  }
}

extern "C" int kgat_slot_sum_f32(const int64_t* slot_edge_ptr, const int32_t* edge_order, int64_t nnz,
                                 const float* edge_logits, float* slot_logits, void* stream) {
  if (!slot_edge_ptr || !edge_order || !edge_logits || !slot_logits || nnz < 0) return KGAT_ERR_INVALID;
  if (nnz == 0) return KGAT_OK;
  hipLaunchKernelGGL(kgat::slot_sum_kernel, dim3((nnz + 255) / 256), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), slot_edge_ptr, edge_order, nnz, edge_logits, slot_logits);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int kgat_row_softmax_f32(const int64_t* rowptr, int64_t n_rows, const float* slot_logits, float* val,
                                    void* stream) {
  return kgat_row_softmax_ex_f32(rowptr, n_rows, nullptr, 0, slot_logits, val, stream);
}
