// a3/a4 -- CF BPR loss over gathered rows of the propagated tables
// (src/model/KGAT/model.py:165-202):
//   pos_b = <u_b, p_b>, neg_b = <u_b, n_b> over the concatenated width D,
//   L = mean_b softplus(neg_b - pos_b) + reg * (l2(U) + l2(P) + l2(N)),
//   l2(X) = mean_b sum_j X_bj^2 / 2.
// Item ids index the user+entity table raw (not offset by user_num), exactly
// as model.py:189-191 does.  The tables are never concatenated: each layer's
// output stays its own buffer and the gather walks the table list.
#include "common.hpp"

namespace kgat {

__device__ __forceinline__ float row_val(const kgat_tables& T, int t, int64_t id, int j) {
  return T.ptr[t][id * T.ld[t] + j];
}

// One block: waves stride over samples; per-sample terms are reduced in a
// fixed order, so the scalar loss is deterministic.
__global__ __launch_bounds__(256) void bpr_fwd_kernel(kgat_tables T, const int64_t* __restrict__ users,
                                                      const int64_t* __restrict__ pos,
                                                      const int64_t* __restrict__ neg, int batch, float reg,
                                                      float* __restrict__ loss, float* __restrict__ coef) {
  __shared__ float part[4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float acc = 0.f;
  for (int b = wave; b < batch; b += 4) {
    const int64_t u = users[b], p = pos[b], n = neg[b];
    float sp = 0.f, sn = 0.f, qu = 0.f, qp = 0.f, qn = 0.f;
    for (int t = 0; t < T.count; ++t) {
      for (int j = lane; j < T.width[t]; j += 64) {
        const float xu = row_val(T, t, u, j), xp = row_val(T, t, p, j), xn = row_val(T, t, n, j);
        sp = fmaf(xu, xp, sp);
        sn = fmaf(xu, xn, sn);
        qu = fmaf(xu, xu, qu);
        qp = fmaf(xp, xp, qp);
        qn = fmaf(xn, xn, qn);
      }
    }
    sp = wave_sum(sp);
    sn = wave_sum(sn);
    qu = wave_sum(qu);
    qp = wave_sum(qp);
    qn = wave_sum(qn);
    const float x = sp - sn;
    // -logsigmoid(x) = softplus(-x), computed stably
    const float nls = fmaxf(-x, 0.f) + log1pf(expf(-fabsf(x)));
    const float sig = 1.f / (1.f + expf(-x));
    if (lane == 0) coef[b] = sig - 1.f;
    acc += nls + reg * 0.5f * (qu + qp + qn);
  }
  if (lane == 0) part[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) *loss = (part[0] + part[1] + part[2] + part[3]) / static_cast<float>(batch);
}

// Gradient rows of table t scattered into dst.  One wave per slot k of the
// concatenated id list [users | pos | neg]; a slot whose id already occurred
// at an earlier slot returns, otherwise it sums every slot with the same id
// in slot order and adds the sum once: deterministic, no atomics.
__global__ __launch_bounds__(256) void bpr_bwd_kernel(kgat_tables T, int t, const int64_t* __restrict__ users,
                                                      const int64_t* __restrict__ pos,
                                                      const int64_t* __restrict__ neg, int batch, float reg,
                                                      const float* __restrict__ coef,
                                                      const float* __restrict__ grad_out, float* __restrict__ dst,
                                                      int64_t lddst) {
  const int slots = 3 * batch;
  const int k = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (k >= slots) return;
  auto id_of = [&](int s) -> int64_t { return s < batch ? users[s] : (s < 2 * batch ? pos[s - batch] : neg[s - 2 * batch]); };
  const int64_t id = id_of(k);
  // earlier occurrence?
  bool dup = false;
  for (int s0 = 0; s0 < k && !dup; s0 += 64) {
    const int s = s0 + lane;
    const bool hit = s < k && id_of(s) == id;
    dup = __any(hit);
  }
  if (dup) return;
  const float scale = grad_out[0] / static_cast<float>(batch);
  const float* tab = T.ptr[t];
  const int64_t ld = T.ld[t];
  const int w = T.width[t];
  constexpr int kCols = 4;  // widths up to 256 columns: lane owns columns lane + 64*c
  float g[kCols] = {0.f, 0.f, 0.f, 0.f};
  for (int s0 = k; s0 < slots; s0 += 64) {
    // ballot with every lane active, before any column-dependent branch
    unsigned long long mask = __ballot(s0 + lane < slots && id_of(s0 + lane) == id);
    while (mask) {  // matching slots in increasing order (wave-uniform)
      const int bit = __ffsll(static_cast<long long>(mask)) - 1;
      mask &= mask - 1;
      const int s = s0 + bit;
      const int b = s % batch;
      const float c = coef[b];
      const int64_t iu = users[b] * ld, ip = pos[b] * ld, in = neg[b] * ld;
#pragma unroll
      for (int cc = 0; cc < kCols; ++cc) {
        const int j = lane + 64 * cc;
        if (j < w) {
          const float xu = tab[iu + j];
          float v;
          if (s < batch) v = c * (tab[ip + j] - tab[in + j]) + reg * xu;
          else if (s < 2 * batch) v = c * xu + reg * tab[ip + j];
          else v = -c * xu + reg * tab[in + j];
          g[cc] = fmaf(v, scale, g[cc]);
        }
      }
    }
  }
#pragma unroll
  for (int cc = 0; cc < kCols; ++cc) {
    const int j = lane + 64 * cc;
    if (j < w) dst[id * lddst + j] += g[cc];
  }
}

}  // namespace kgat

static int check_tables(const kgat_tables* T) {
  if (!T || T->count < 1 || T->count > KGAT_MAX_TABLES) return KGAT_ERR_INVALID;
  for (int i = 0; i < T->count; ++i)
    if (!T->ptr[i] || T->width[i] <= 0 || T->ld[i] < T->width[i]) return KGAT_ERR_INVALID;
  return KGAT_OK;
}

extern "C" int kgat_bpr_fwd_f32(const kgat_tables* T, const int64_t* users, const int64_t* pos, const int64_t* neg,
                                int32_t batch, float reg, float* loss, float* coef, void* stream) {
  if (int e = check_tables(T)) return e;
  if (!users || !pos || !neg || !loss || !coef || batch <= 0) return KGAT_ERR_INVALID;
  hipLaunchKernelGGL(kgat::bpr_fwd_kernel, dim3(1), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), *T, users,
                     pos, neg, batch, reg, loss, coef);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int kgat_bpr_bwd_f32(const kgat_tables* T, int32_t table, const int64_t* users, const int64_t* pos,
                                const int64_t* neg, int32_t batch, float reg, const float* coef,
                                const float* grad_out, float* dst, int64_t lddst, void* stream) {
  if (int e = check_tables(T)) return e;
  if (table < 0 || table >= T->count || !users || !pos || !neg || !coef || !grad_out || !dst || batch <= 0 ||
      lddst < T->width[table] || T->width[table] > 256)
    return KGAT_ERR_INVALID;
  const int blocks = (3 * batch + 3) / 4;
  hipLaunchKernelGGL(kgat::bpr_bwd_kernel, dim3(blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), *T,
                     table, users, pos, neg, batch, reg, coef, grad_out, dst, lddst);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}
