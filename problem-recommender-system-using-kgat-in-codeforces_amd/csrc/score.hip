// a8 -- CF scores (src/model/KGAT/model.py:368-391):
//   S[u, i] = < all[users[u]], all[items[i]] >   over the concatenated width
// of the propagated tables [X0 | H1 | ... | HL] (never concatenated here).
// Item ids index the table raw, as model.py:389-390 does.
//
// fp32 MFMA GEMM with the row gather fused into the operand loads: a wave
// computes a 16 (users) x 64 (items) tile; lane l loads the contiguous k-range
// (l>>4)*W/4 .. of user row (l&15) (A operand) and of item row (l&15) of each
// 16-item block (B operand) straight from the gathered rows, table by table.
#include "common.hpp"

namespace kgat {

__global__ __launch_bounds__(256) void score_kernel(kgat_tables T, const int64_t* __restrict__ users, int n_users,
                                                    const int64_t* __restrict__ items, int n_items,
                                                    float* __restrict__ S, int64_t lds) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, q = lane >> 4, c = lane & 15;
  const int u0 = blockIdx.y * 16;
  const int i0 = (blockIdx.x * 4 + wave) * 64;
  if (i0 >= n_items) return;
  const int ua = u0 + c;
  const int64_t urow = ua < n_users ? users[ua] : -1;
  int64_t irow[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    const int it = i0 + cb * 16 + c;
    irow[cb] = it < n_items ? items[it] : -1;
  }
  floatx4 acc[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) acc[cb] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int t = 0; t < T.count; ++t) {
    const int kq = T.width[t] / 4;  // contiguous k values per lane
    const float* base = T.ptr[t];
    const int64_t ld = T.ld[t];
    for (int k0 = 0; k0 < kq; k0 += 4) {
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
      if (urow >= 0) a = *reinterpret_cast<const float4*>(base + urow * ld + q * kq + k0);
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        float4 b = make_float4(0.f, 0.f, 0.f, 0.f);
        if (irow[cb] >= 0) b = *reinterpret_cast<const float4*>(base + irow[cb] * ld + q * kq + k0);
        acc[cb] = mfma16x4(a.x, b.x, acc[cb]);
        acc[cb] = mfma16x4(a.y, b.y, acc[cb]);
        acc[cb] = mfma16x4(a.z, b.z, acc[cb]);
        acc[cb] = mfma16x4(a.w, b.w, acc[cb]);
      }
    }
  }
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    const int it = i0 + cb * 16 + c;
    if (it >= n_items) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int u = u0 + q * 4 + i;
      if (u < n_users) S[static_cast<int64_t>(u) * lds + it] = acc[cb][i];
    }
  }
}

}  // namespace kgat

extern "C" int kgat_score_f32(const kgat_tables* T, const int64_t* users, int32_t n_users, const int64_t* items,
                              int32_t n_items, float* scores, int64_t ld_scores, void* stream) {
  if (!T || !users || !items || !scores || n_users < 0 || n_items < 0 || ld_scores < n_items) return KGAT_ERR_INVALID;
  if (T->count < 1 || T->count > KGAT_MAX_TABLES) return KGAT_ERR_INVALID;
  for (int i = 0; i < T->count; ++i)
    if (!T->ptr[i] || T->width[i] % 16 != 0 || T->ld[i] % 4 != 0 ||
        (reinterpret_cast<uintptr_t>(T->ptr[i]) & 15))
      return KGAT_ERR_INVALID;
  if (n_users == 0 || n_items == 0) return KGAT_OK;
  dim3 grid((n_items + 255) / 256, (n_users + 15) / 16);
  hipLaunchKernelGGL(kgat::score_kernel, grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream), *T, users, n_users,
                     items, n_items, scores, ld_scores);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}
