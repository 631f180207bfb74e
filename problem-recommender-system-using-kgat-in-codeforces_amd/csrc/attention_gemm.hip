// a6 for the wide embeddings of C5 (d > 128, e.g. 256): the edge scorer of
// attention.hip (src/model/KGAT/model.py:263-316, multi_head_attention.py:35-58)
// as GEMMs over relation-sorted edge chunks plus fused HIP epilogues.
// At d = 256 three d x d matrices no longer fit a CU's LDS beside a tile, so:
//   per chunk of the relation-sorted edge order (rel_perm):
//     T  = emb[tail]                      (gather_edge_rows_kernel)
//     T' = T W_r   per relation segment   (gemm_f32, gemm.hip)
//     V  = T' W_v^T, + b_v, per-(edge, head) attention dropout  (gemm_f32, bias_drop_kernel)
//     O  = V W_o^T                        (gemm_f32)
//     logit = sum tanh(LayerNorm(O + b_o)) * degree weight      (ln_logit_kernel)
// Same arithmetic, dropout keys (edge * 8 + head) and output placement
// (out_pos or edge order) as kgat_edge_logits_f32.
#include <cmath>

#include "common.hpp"
#include "gemm.hpp"

namespace kgat {

__global__ __launch_bounds__(256) void gather_edge_rows_kernel(const float* __restrict__ emb, int64_t ld,
                                                               const int32_t* __restrict__ tails,
                                                               const int32_t* __restrict__ perm, int64_t pos0,
                                                               int64_t n, int d, float* __restrict__ T) {
  const int64_t row = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 4;
  const int lane = threadIdx.x & 15;
  if (row >= n) return;
  const int64_t t = tails[perm[pos0 + row]];
  for (int c = lane * 4; c < d; c += 64)
    *reinterpret_cast<float4*>(T + row * d + c) = *reinterpret_cast<const float4*>(emb + t * ld + c);
}

__global__ __launch_bounds__(256) void bias_drop_kernel(float* __restrict__ V, const float* __restrict__ bv,
                                                        const int32_t* __restrict__ perm, int64_t pos0, int64_t n,
                                                        int d, float p, uint64_t seed) {
  const int64_t total = n * d;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const int depth = d / 8;  // 8 heads (multi_head_attention.py:6)
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int64_t r = i / d;
    const int c = static_cast<int>(i % d);
    float v = V[i] + bv[c];
    if (p > 0.f) {
      const uint64_t e = static_cast<uint64_t>(perm[pos0 + r]);
      v = dropout_keep(seed, e * 8 + c / depth, p) ? v * scale : 0.f;
    }
    V[i] = v;
  }
}

// one wave per edge
__global__ __launch_bounds__(256) void ln_logit_kernel(const float* __restrict__ O, const float* __restrict__ bo,
                                                       const float* __restrict__ ln_w, const float* __restrict__ ln_b,
                                                       const float* __restrict__ weight,
                                                       const int32_t* __restrict__ perm, int64_t pos0, int64_t n,
                                                       int d, const int32_t* __restrict__ out_pos,
                                                       float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t r = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  float o[16];
  float s = 0.f;
  int k = 0;
  for (int c = lane; c < d; c += 64, ++k) {
    o[k] = O[r * d + c] + bo[c];
    s += o[k];
  }
  const float mean = wave_sum(s) / static_cast<float>(d);
  float v2 = 0.f;
  k = 0;
  for (int c = lane; c < d; c += 64, ++k) {
    const float dl = o[k] - mean;
    v2 = fmaf(dl, dl, v2);
  }
  const float rstd = 1.f / sqrtf(wave_sum(v2) / static_cast<float>(d) + 1e-5f);
  float ts = 0.f;
  k = 0;
  for (int c = lane; c < d; c += 64, ++k) ts += tanhf((o[k] - mean) * rstd * ln_w[c] + ln_b[c]);
  ts = wave_sum(ts);
  if (lane == 0) {
    const int32_t e = perm[pos0 + r];
    out[out_pos ? out_pos[e] : e] = ts * weight[e];
  }
}

}  // namespace kgat

extern "C" int64_t kgat_edge_logits_gemm_work_floats(int64_t chunk_edges, int32_t d) {
  if (chunk_edges < 16 || d < 16 || d % 16 || d > 1024) return -1;
  return 2 * chunk_edges * static_cast<int64_t>(d);
}

extern "C" int kgat_edge_logits_gemm_f32(const float* emb, int64_t ld_emb, int64_t n_nodes, const float* trans,
                                         int32_t d, const float* Wv, const float* bv, const float* Wo, const float* bo,
                                         const float* ln_w, const float* ln_b, const int32_t* tails,
                                         const float* edge_weight, const int32_t* rel_perm, int64_t n_edges,
                                         const int32_t* seg_rel, const int64_t* seg_beg, int32_t n_seg,
                                         float dropout_p, uint64_t seed, const int32_t* out_pos, float* out,
                                         float* work, int64_t work_floats, void* stream) {
  if (!emb || !trans || !Wv || !bv || !Wo || !bo || !ln_w || !ln_b || !tails || !edge_weight || !rel_perm || !out ||
      !seg_rel || !seg_beg || n_edges < 0 || n_seg < 0 || d < 16 || d % 16 || d > 1024 || ld_emb < d ||
      (ld_emb & 3) || !(dropout_p >= 0.f && dropout_p < 1.f))
    return KGAT_ERR_INVALID;
  (void)n_nodes;
  if (n_edges == 0) return KGAT_OK;
  if (!work || work_floats < 2 * 16 * static_cast<int64_t>(d)) return KGAT_ERR_WORKSPACE;
  const int64_t chunk = work_floats / (2 * static_cast<int64_t>(d));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  float* T = work;                // gathered tails, later O
  float* P = work + chunk * d;    // T W_r, later V
  float* V = T;
  int sg = 0;
  for (int64_t c0 = 0; c0 < n_edges; c0 += chunk) {
    const int64_t c1 = c0 + chunk < n_edges ? c0 + chunk : n_edges;
    const int64_t rows = c1 - c0;
    hipLaunchKernelGGL(kgat::gather_edge_rows_kernel, dim3(kgat::blocks_for(rows, 16, 1 << 30)), dim3(256), 0, st, emb,
                       ld_emb, tails, rel_perm, c0, rows, d, T);
    KGAT_LAUNCH_CHECK();
    // T' = T W_r over each relation segment overlapping [c0, c1)
    while (sg < n_seg && seg_beg[sg + 1] <= c0) ++sg;
    for (int s = sg; s < n_seg && seg_beg[s] < c1; ++s) {
      const int64_t a = seg_beg[s] > c0 ? seg_beg[s] : c0;
      const int64_t b = seg_beg[s + 1] < c1 ? seg_beg[s + 1] : c1;
      if (b <= a) continue;
      const float* Wr = trans + static_cast<int64_t>(seg_rel[s]) * d * d;
      if (int e = kgat::gemm_f32(false, false, b - a, d, d, T + (a - c0) * d, d, 0, Wr, d, 0, P + (a - c0) * d, d, 0,
                                 1, false, st))
        return e;
    }
    // V = T' W_v^T (+ b_v, dropout) into T's buffer
    if (int e = kgat::gemm_f32(false, true, rows, d, d, P, d, 0, Wv, d, 0, V, d, 0, 1, false, st)) return e;
    hipLaunchKernelGGL(kgat::bias_drop_kernel, dim3(kgat::blocks_for(rows * d, 256, kgat::kCUs * 8)), dim3(256), 0, st,
                       V, bv, rel_perm, c0, rows, d, dropout_p, seed);
    KGAT_LAUNCH_CHECK();
    // O = V W_o^T into P's buffer
    if (int e = kgat::gemm_f32(false, true, rows, d, d, V, d, 0, Wo, d, 0, P, d, 0, 1, false, st)) return e;
    hipLaunchKernelGGL(kgat::ln_logit_kernel, dim3((rows + 3) / 4), dim3(256), 0, st, P, bo, ln_w, ln_b, edge_weight,
                       rel_perm, c0, rows, d, out_pos, out);
    KGAT_LAUNCH_CHECK();
  }
  return KGAT_OK;
}
