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
// permutation built once per graph), one tile per wave (two from d = 64): the three d x d
// contractions are fp32 MFMA (v_mfma_f32_16x16x4_f32) chains computed
// transposed, so each product's accumulators are the next one's operand (no
// relayout); dropout, LayerNorm, tanh and the sum are fused epilogues.
//
// Neighbour softmax: A[h, :] = softmax over the stored entries of row h
// (torch.sparse.softmax(dim=1), model.py:364): rows by length class (4-lane
// groups, 16-lane groups, 512-entry segments of hub rows).
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

// tanh from one v_exp_f32 and one v_rcp_f32, branch-free: tanh|x| = (1 - e^{-2|x|}) / (1 + e^{-2|x|}),
// absolute error ~3e-7 (the logit sums 64 of them).  libm's tanhf is ~25 VALU with branches, 64 per lane
// per tile -- as much issue time as the tile's MFMA chain.
__device__ __forceinline__ float tanh_fast(float x) {
  const float t = __expf(-2.f * fabsf(x));
  return copysignf(__fdividef(1.f - t, 1.f + t), x);
}

// The scorer computes every contraction transposed (features x edges): out^T = W . in^T, the weights
// the MFMA A operand and the tile's edges its B operand.  The accumulator layout of one product
// (lane (q, c): features mb*16 + q*4 + i of edge c) is then the B-operand layout of the next with the
// contraction index taken in the permuted order k = kb*16 + q*4 + i -- the chain needs no LDS relayout,
// and each lane's A operand for 4 consecutive MFMAs is one float4 of a weight row.  Per lane: one edge,
// 16 of its features; LayerNorm and the tanh sum reduce over the 4 lanes c + 16 q.
//   t'^T = W_r^T e_t^T : A[m][kk] = W_r[q*KQ + t][mb*16 + c], B = e_t[c][q*KQ + t] (load_a's layout)
//   v^T  = W_v t'^T     : A = W_v[mb*16 + c][kb*16 + q*4 + i], B = t'^T from the accumulators
//   o^T  = W_o v^T
template <int D, bool WLDS, int NW, int P>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(D <= 64 ? 4 : 1))) void edge_score_t_kernel(EdgeScoreArgs a) {
  constexpr int KQ = D / 4, NB = D / 16, WLD = D + 4;
  constexpr int kDepth = D / 8;  // 8 heads (multi_head_attention.py:6)
  constexpr int kWFloats = WLDS ? 2 * D * WLD : 0;
  __shared__ __attribute__((aligned(16))) float smem[kWFloats + 4 * D];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, q = lane >> 4, c = lane & 15;
  const float* wv = a.Wv;
  const float* wo = a.Wo;
  int wld = D;
  if constexpr (WLDS) {
    for (int i = threadIdx.x; i < D * D / 4; i += 64 * NW) {
      const int j = (i * 4) / D, k = (i * 4) % D;
      *reinterpret_cast<float4*>(smem + j * WLD + k) = reinterpret_cast<const float4*>(a.Wv)[i];
      *reinterpret_cast<float4*>(smem + D * WLD + j * WLD + k) = reinterpret_cast<const float4*>(a.Wo)[i];
    }
    wv = smem;
    wo = smem + D * WLD;
    wld = WLD;
  }
  float* cst = smem + kWFloats;  // b_v, b_o, LayerNorm weight, bias
  for (int i = threadIdx.x; i < D; i += 64 * NW) {
    cst[i] = a.bv[i];
    cst[D + i] = a.bo[i];
    cst[2 * D + i] = a.ln_w[i];
    cst[3 * D + i] = a.ln_b[i];
  }
  __syncthreads();
  const float scale = a.p > 0.f ? 1.f / (1.f - a.p) : 1.f;
  // P consecutive tiles per wave (relation-sorted, so nearly always one relation): every weight value loaded
  // feeds P MFMA chains, one per tile; each tile's chains are the P = 1 chains, so the same bits.
  const int n_groups = (a.n_tiles + P - 1) / P;
  for (int tg = blockIdx.x * NW + wave; tg < n_groups; tg += gridDim.x * NW) {
    int ec[P];
    int64_t r[P];
    uint64_t keep[P];
    float x[P][KQ];
#pragma unroll
    for (int j = 0; j < P; ++j) {
      const int tl = tg * P + j;
      const bool live = tl < a.n_tiles;  // wave-uniform
      const int beg = live ? a.tile_beg[tl] : 0, cnt = live ? a.tile_beg[tl + 1] - beg : 0;
      r[j] = live ? a.tile_rel[tl] : r[0];
      ec[j] = c < cnt ? a.rel_perm[beg + c] : -1;  // this lane's edge of tile j
      load_a<D>(a.emb, a.ld_emb, ec[j] >= 0 ? static_cast<int64_t>(a.tails[ec[j]]) : -1, q, x[j]);
      uint64_t keep_lo = ~0ull, keep_hi = ~0ull;  // train-mode dropout bits, pair = edge * 8 + head
      if (a.p > 0.f) {
        const int er = lane >> 3, head = lane & 7;
        const int64_t e0 = er < cnt ? a.rel_perm[beg + er] : 0;
        const int64_t e1 = er + 8 < cnt ? a.rel_perm[beg + er + 8] : 0;
        keep_lo = __ballot(dropout_keep(a.seed, static_cast<uint64_t>(e0) * 8 + head, a.p));
        keep_hi = __ballot(dropout_keep(a.seed, static_cast<uint64_t>(e1) * 8 + head, a.p));
      }
      keep[j] = (c < 8 ? keep_lo : keep_hi) >> ((c & 7) * 8);  // this edge's 8 head bits
    }
    floatx4 acc[P][NB];
    bool one_rel = true;
#pragma unroll
    for (int j = 1; j < P; ++j) one_rel = one_rel && r[j] == r[0];
    // t'^T = W_r^T e_t^T.  A relation boundary inside the group (rare: at most one group per relation)
    // takes one pass per tile, each keeping the chains of the tiles of its relation.
    const int npass = one_rel ? 1 : P;  // wave-uniform
#pragma unroll 1
    for (int ps = 0; ps < npass; ++ps) {
      const int64_t rp = r[ps];
      const float* Wr = a.trans + rp * D * D;
#pragma unroll
      for (int mb = 0; mb < NB; ++mb) {
        __builtin_amdgcn_sched_barrier(0);  // one column block's W_r loads in flight at a time
        floatx4 s[P];
#pragma unroll
        for (int j = 0; j < P; ++j) s[j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < KQ; ++t) {
          const float w = Wr[(q * KQ + t) * D + mb * 16 + c];
#pragma unroll
          for (int j = 0; j < P; ++j) s[j] = mfma16x4(w, x[j][t], s[j]);
        }
#pragma unroll
        for (int j = 0; j < P; ++j)
          if (ps == 0 || r[j] == rp) acc[j][mb] = s[j];
      }
    }
    // v^T = W_v t'^T + b_v, dropped per (edge, head)
    floatx4 acc2[P][NB];
#pragma unroll
    for (int mb = 0; mb < NB; ++mb) {
      if (mb % 2 == 0) __builtin_amdgcn_sched_barrier(0);  // two column blocks' chains interleave
      floatx4 s[P];
#pragma unroll
      for (int j = 0; j < P; ++j) s[j] = floatx4{0.f, 0.f, 0.f, 0.f};
      const float* w = wv + (mb * 16 + c) * wld + q * 4;
#pragma unroll
      for (int kb = 0; kb < NB; ++kb) {
        const float4 wk = *reinterpret_cast<const float4*>(w + kb * 16);
#pragma unroll
        for (int j = 0; j < P; ++j) {
          s[j] = mfma16x4(wk.x, acc[j][kb][0], s[j]);
          s[j] = mfma16x4(wk.y, acc[j][kb][1], s[j]);
          s[j] = mfma16x4(wk.z, acc[j][kb][2], s[j]);
          s[j] = mfma16x4(wk.w, acc[j][kb][3], s[j]);
        }
      }
      const float4 b = *reinterpret_cast<const float4*>(cst + mb * 16 + q * 4);
      const float bb[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
      for (int j = 0; j < P; ++j) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float v = s[j][i] + bb[i];
          const int head = (mb * 16 + q * 4 + i) / kDepth;
          s[j][i] = (keep[j] >> head) & 1 ? (a.p > 0.f ? v * scale : v) : 0.f;
        }
        acc2[j][mb] = s[j];
      }
    }
    // o^T = W_o v^T + b_o, then LayerNorm over the features and the tanh sum
    float sum[P];
#pragma unroll
    for (int j = 0; j < P; ++j) sum[j] = 0.f;
#pragma unroll
    for (int mb = 0; mb < NB; ++mb) {
      if (mb % 2 == 0) __builtin_amdgcn_sched_barrier(0);  // two column blocks' chains interleave
      floatx4 s[P];
#pragma unroll
      for (int j = 0; j < P; ++j) s[j] = floatx4{0.f, 0.f, 0.f, 0.f};
      const float* w = wo + (mb * 16 + c) * wld + q * 4;
#pragma unroll
      for (int kb = 0; kb < NB; ++kb) {
        const float4 wk = *reinterpret_cast<const float4*>(w + kb * 16);
#pragma unroll
        for (int j = 0; j < P; ++j) {
          s[j] = mfma16x4(wk.x, acc2[j][kb][0], s[j]);
          s[j] = mfma16x4(wk.y, acc2[j][kb][1], s[j]);
          s[j] = mfma16x4(wk.z, acc2[j][kb][2], s[j]);
          s[j] = mfma16x4(wk.w, acc2[j][kb][3], s[j]);
        }
      }
      const float4 b = *reinterpret_cast<const float4*>(cst + D + mb * 16 + q * 4);
#pragma unroll
      for (int j = 0; j < P; ++j) {
        s[j][0] += b.x;
        s[j][1] += b.y;
        s[j][2] += b.z;
        s[j][3] += b.w;
        sum[j] += (s[j][0] + s[j][1]) + (s[j][2] + s[j][3]);
        acc[j][mb] = s[j];
      }
    }
#pragma unroll
    for (int j = 0; j < P; ++j) {
      float sm = sum[j];
      sm += __shfl_xor(sm, 16);
      sm += __shfl_xor(sm, 32);
      const float mean = sm / static_cast<float>(D);
      float v2 = 0.f;
#pragma unroll
      for (int mb = 0; mb < NB; ++mb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float dl = acc[j][mb][i] - mean;
          v2 = fmaf(dl, dl, v2);
        }
      v2 += __shfl_xor(v2, 16);
      v2 += __shfl_xor(v2, 32);
      const float rstd = 1.f / sqrtf(v2 / static_cast<float>(D) + kLnEps);
      float ts = 0.f;
#pragma unroll
      for (int mb = 0; mb < NB; ++mb) {
        const float4 lw = *reinterpret_cast<const float4*>(cst + 2 * D + mb * 16 + q * 4);
        const float4 lb = *reinterpret_cast<const float4*>(cst + 3 * D + mb * 16 + q * 4);
        ts += tanh_fast((acc[j][mb][0] - mean) * rstd * lw.x + lb.x);
        ts += tanh_fast((acc[j][mb][1] - mean) * rstd * lw.y + lb.y);
        ts += tanh_fast((acc[j][mb][2] - mean) * rstd * lw.z + lb.z);
        ts += tanh_fast((acc[j][mb][3] - mean) * rstd * lw.w + lb.w);
      }
      ts += __shfl_xor(ts, 16);
      ts += __shfl_xor(ts, 32);
      if (q == 0 && ec[j] >= 0) a.logits[a.out_pos ? a.out_pos[ec[j]] : ec[j]] = ts * a.edge_weight[ec[j]];
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
// A wave takes 16 consecutive rows.  Rows of <= 32 entries: a 4-lane group each, read once into 8
// registers per lane (max, exp-sum, write from registers) -- 16 rows in flight per wave.  Rows of
// 33..256 entries (half of a power-law CKG's entries): a 16-lane group each, 4 rows per round, 16 entries
// per lane in registers (one read round instead of a 4-lane group's 8-64 serial ones).  Lane partials reduce in a fixed butterfly relative
// to the row's first entry: deterministic, and the same bits wherever the row sits.  Longer rows: the
// segment plan below.
constexpr int kSoftmaxShort = 256;

__device__ __forceinline__ void wave_lds_sync() {
  // orders this wave's LDS writes before its later LDS reads of other lanes' data
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// softmax of one 16-lane group's row held in y[16] (entry gl + 16 k), written to val
__device__ __forceinline__ void group16_softmax(float (&y)[16], int64_t b, int64_t e1, int gl, float* __restrict__ val) {
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < 16; ++k) m = fmaxf(m, y[k]);
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    y[k] = b + gl + 16 * k < e1 ? __expf(y[k] - m) : 0.f;
    s += y[k];
  }
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o);
  const float inv = 1.f / s;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int64_t e = b + gl + 16 * k;
    if (e < e1) val[e] = y[k] * inv;
  }
}

__device__ __forceinline__ int64_t shfl64(int64_t v, int src) {
  const int lo = __shfl(static_cast<int>(v & 0xffffffff), src);
  const int hi = __shfl(static_cast<int>(v >> 32), src);
  return (static_cast<int64_t>(hi) << 32) | static_cast<uint32_t>(lo);
}

// The k-th (k = this lane's 16-lane group) set bit of med, or -1; med loses its first 4 set bits.
__device__ __forceinline__ int take_group_row(unsigned long long& med, int g) {
  int src = -1;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int f = med ? __ffsll(static_cast<long long>(med)) - 1 : -1;
    if (k == g) src = f;
    if (med) med &= med - 1;
  }
  return src;
}

// softmax of one 4-lane group's row held in x[S] (entry j + 4 k), written to val
template <int S>
__device__ __forceinline__ void group4_softmax(float (&x)[S], int64_t beg, int64_t end, int j, float* __restrict__ val) {
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < S; ++k) m = fmaxf(m, x[k]);
  m = fmaxf(m, __shfl_xor(m, 1));
  m = fmaxf(m, __shfl_xor(m, 2));
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < S; ++k) {
    x[k] = beg + j + 4 * k < end ? __expf(x[k] - m) : 0.f;
    s += x[k];
  }
  s += __shfl_xor(s, 1);
  s += __shfl_xor(s, 2);
  const float inv = 1.f / s;
#pragma unroll
  for (int k = 0; k < S; ++k) {
    const int64_t e = beg + j + 4 * k;
    if (e < end) val[e] = x[k] * inv;
  }
}

// A wave takes kSoftmaxRG x 16 rows: 4-lane group g4 the rows row0 + g4 + 16 t (t < kSoftmaxRG), all their
// row pointers, then all their entries, in flight together before the first reduction.
constexpr int kSoftmaxRG = 2;

template <int R = kSoftmaxRG>
__device__ __forceinline__ void wave_rows_softmax(const int64_t* __restrict__ rowptr, int64_t n_rows, int64_t row0,
                                                  int lane, const float* __restrict__ logit, float* __restrict__ val) {
  const int j = lane & 3, g = lane >> 4, gl = lane & 15, g4 = lane >> 2;
  int64_t beg[R], end[R];
#pragma unroll
  for (int t = 0; t < R; ++t) {
    const int64_t row = row0 + g4 + 16 * t;
    beg[t] = end[t] = 0;
    if (row < n_rows) {
      beg[t] = rowptr[row];
      end[t] = rowptr[row + 1];
    }
  }
  float x[R][8];
#pragma unroll
  for (int t = 0; t < R; ++t) {
    const int64_t len = end[t] - beg[t];
    const int slots = len <= 8 ? 2 : 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int64_t e = beg[t] + j + 4 * k;
      x[t][k] = len <= 32 && k < slots && e < end[t] ? logit[e] : -INFINITY;
    }
  }
#pragma unroll
  for (int t = 0; t < R; ++t) {
    const int64_t len = end[t] - beg[t];
    if (len > 0 && len <= 8) {  // (group-uniform) two entries per lane
      float x2[2] = {x[t][0], x[t][1]};
      group4_softmax<2>(x2, beg[t], end[t], j, val);
    } else if (len > 8 && len <= 32) {
      group4_softmax<8>(x[t], beg[t], end[t], j, val);
    }
  }
  // rows of 33..256 entries: up to 4 per round, one per 16-lane group; lane 4 g4 + t reports row t of its group
  bool is_med = false;
  int64_t pb = 0, pe = 0;
#pragma unroll
  for (int t = 0; t < R; ++t)
    if (j == t) {
      const int64_t len = end[t] - beg[t];
      is_med = len > 32 && len <= kSoftmaxShort;
      pb = beg[t];
      pe = end[t];
    }
  unsigned long long med = __ballot(is_med);
  while (med) {
    const int src = take_group_row(med, g);
    // (every lane takes part in the shuffles: a source lane may sit in a group with no row this round)
    const int64_t b2 = shfl64(pb, src < 0 ? 0 : src), e2_src = shfl64(pe, src < 0 ? 0 : src);
    const int64_t e2 = src < 0 ? b2 : e2_src;
    if (src >= 0) {
      float y[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int64_t e = b2 + gl + 16 * k;
        y[k] = e < e2 ? logit[e] : -INFINITY;
      }
      group16_softmax(y, b2, e2, gl, val);
    }
  }
}

__global__ __launch_bounds__(256) void row_softmax_kernel(const int64_t* __restrict__ rowptr, int64_t n_rows,
                                                          const float* __restrict__ logit, float* __restrict__ val) {
  const int64_t row0 = (static_cast<int64_t>(blockIdx.x) * blockDim.x + (threadIdx.x & ~63)) / 4 * kSoftmaxRG;
  if (row0 >= n_rows) return;  // (wave-uniform)
  wave_rows_softmax(rowptr, n_rows, row0, threadIdx.x & 63, logit, val);
}

// Long rows, cut into the CSR's long-row plan segments (one wave each, <= kSoftmaxSeg entries, 8 per lane
// in registers).  Pass 1 (with the short rows, segment waves first): each segment's max m_s and
// s_s = sum exp(x - m_s) -> stat[2s], stat[2s + 1].  Pass 2: every segment wave of a row combines the
// row's segment stats in segment order -- M = max m_s, S = sum_s s_s exp(m_s - M), lane-strided partials
// then a fixed butterfly, the same bits in every wave of the row -- and writes its own entries
// exp(x - M) / S.  A hub row of 10^5 entries runs on ~200 waves instead of one block's three serial passes.
constexpr int kSoftmaxSeg = 512;

template <int RG>
__global__ __launch_bounds__(256) void row_softmax_stats_kernel(kgat_csr A, const float* __restrict__ logit,
                                                                float* __restrict__ val, float* __restrict__ stat,
                                                                int seg_blocks) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (static_cast<int>(blockIdx.x) >= seg_blocks) {  // rows of <= 256 entries, 16 RG per wave
    const int64_t row0 = (static_cast<int64_t>(blockIdx.x - seg_blocks) * blockDim.x + (threadIdx.x & ~63)) / 4 * RG;
    if (row0 < A.n_rows) wave_rows_softmax<RG>(A.rowptr, A.n_rows, row0, lane, logit, val);
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
  for (int k = 0; k < kSoftmaxSeg / 64; ++k) s += beg + lane + 64 * k < end ? __expf(x[k] - m) : 0.f;
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
  const int64_t beg = A.seg_beg[sg];
  const int64_t rbeg = A.rowptr[row], rend = A.rowptr[row + 1];
  const int s0 = sg - static_cast<int>((beg - rbeg) / kSoftmaxSeg);  // the row's first segment
  const int ns = static_cast<int>((rend - rbeg + kSoftmaxSeg - 1) / kSoftmaxSeg);
  const int64_t end = beg + kSoftmaxSeg < rend ? beg + kSoftmaxSeg : rend;
  // this segment's entries and the row's first 64 segment stats in one round trip
  float x[kSoftmaxSeg / 64];
#pragma unroll
  for (int k = 0; k < kSoftmaxSeg / 64; ++k) {
    const int64_t e = beg + lane + 64 * k;
    x[k] = e < end ? logit[e] : 0.f;
  }
  const float m0 = lane < ns ? stat[2 * static_cast<int64_t>(s0 + lane)] : -INFINITY;
  const float z0 = lane < ns ? stat[2 * static_cast<int64_t>(s0 + lane) + 1] : 0.f;
  float M = m0;
  for (int i = lane + 64; i < ns; i += 64) M = fmaxf(M, stat[2 * static_cast<int64_t>(s0 + i)]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) M = fmaxf(M, __shfl_xor(M, o));
  float S = lane < ns ? z0 * __expf(m0 - M) : 0.f;
  for (int i = lane + 64; i < ns; i += 64) {
    const int64_t k = 2 * static_cast<int64_t>(s0 + i);
    S += stat[k + 1] * __expf(stat[k] - M);
  }
  S = wave_sum(S);
  const float inv = 1.f / S;
#pragma unroll
  for (int k = 0; k < kSoftmaxSeg / 64; ++k) {
    const int64_t e = beg + lane + 64 * k;
    if (e < end) val[e] = __expf(x[k] - M) * inv;
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
  for (int64_t e = beg + lane; e < end; e += 64) s += __expf(logit[e] - m);
  const float inv = 1.f / wave_sum(s);
  for (int64_t e = beg + lane; e < end; e += 64) val[e] = __expf(logit[e] - m) * inv;
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
  for (int64_t e = beg + threadIdx.x; e < end; e += 256) s += __expf(logit[e] - m);
  s = wave_sum(s);
  if (lane == 0) red[wave] = s;
  __syncthreads();
  const float inv = 1.f / (((red[0] + red[1]) + red[2]) + red[3]);
  for (int64_t e = beg + threadIdx.x; e < end; e += 256) val[e] = __expf(logit[e] - m) * inv;
}

template <int D>
static int launch_scores(const EdgeScoreArgs& a, hipStream_t st) {
  constexpr bool wlds = D <= 64;
  // two tiles per wave from d = 64 (every weight load feeds two chains; tools/score_ab.py on the C2 graph, bit
  // for bit: d = 128 25.5 -> 21.0 ms, 0.49 -> 0.60 of the fp32 MFMA peak; d = 64 5.56 -> 5.40 ms; four tiles
  // at d = 64 5.45 ms, 2 waves / SIMD)
  constexpr int P = D >= 64 ? 2 : 1;
  const int grid = blocks_for((a.n_tiles + P - 1) / P, 4, kCUs * 8);
  // (4 waves per block: 8-wave blocks at 6 waves / SIMD measured 6.14 vs 6.05 ms at C2 -- not occupancy-bound)
  hipLaunchKernelGGL((edge_score_t_kernel<D, wlds, 4, P>), dim3(grid), dim3(256), 0, st, a);
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
  // 16 x kSoftmaxRG short rows per wave (RG = 4, all 64 rows' loads in flight: 48.9 vs 43.8 us at C2,
  // profiles/r06_softmax_ab.md)
  const int64_t grid = seg_blocks + (A->n_rows * 4 / kgat::kSoftmaxRG + 255) / 256;
  if (grid > 0x7fffffff) return KGAT_ERR_INVALID;
  hipLaunchKernelGGL(kgat::row_softmax_stats_kernel<kgat::kSoftmaxRG>, dim3(grid), dim3(256), 0, st, *A, slot_logits,
                     val, work, seg_blocks);
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
  hipLaunchKernelGGL(kgat::row_softmax_kernel, dim3((n_rows * 4 / kgat::kSoftmaxRG + 255) / 256), dim3(256), 0, st,
                     rowptr, n_rows,
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
