// a5 -- TransR KG loss forward/backward (src/model/KGAT/model.py:204-261):
//   h' = e_h W_r, t+' = e_t+ W_r, t-' = e_t- W_r    (W_r = trans[r], d x k, row vector times W)
//   s+ = |h' + e_r - t+'|^2, s- = |h' + e_r - t-'|^2
//   L = mean_b softplus(s+ - s-) + reg * (l2(h') + l2(e_r) + l2(t+') + l2(t-'))
// with l2(V) = mean_b sum_j V_bj^2 / 2.
//
// Forward: one wave per sample; lanes own output columns j of the projections
// (W_r rows are read coalesced, the gathered embedding row is broadcast).  It
// also keeps, per sample, the gradients w.r.t. the projected vectors and the
// table rows (unscaled by the upstream gradient) in a caller workspace.
// Backward: the table-row gradients are scattered with duplicate ids summed
// in slot order (no atomics), and d trans[r] / d rel_emb[r] are reduced per
// relation over the samples in batch order -- both deterministic.
#include "common.hpp"

namespace kgat {

struct TransrWork {  // offsets (floats) into the workspace
  int64_t term, gproj, grow;
  __host__ __device__ static TransrWork at(int batch, int d, int k) {
    TransrWork w;
    w.term = 0;
    w.gproj = batch;                                   // [batch][4][k]: g_h', g_t+', g_t-', g_er
    w.grow = w.gproj + static_cast<int64_t>(batch) * 4 * k;  // [batch][3][d]: d e_h, d e_t+, d e_t-
    return w;
  }
  __host__ __device__ static int64_t size(int batch, int d, int k) {
    return at(batch, d, k).grow + static_cast<int64_t>(batch) * 3 * d;
  }
};

constexpr int kMaxCols = 4;  // k, d <= 256 = 4 columns per lane

__global__ __launch_bounds__(256) void transr_fwd_kernel(const float* __restrict__ emb, int64_t lde,
                                                         const float* __restrict__ rel_emb,
                                                         const float* __restrict__ trans, int d, int k,
                                                         const int64_t* __restrict__ heads,
                                                         const int64_t* __restrict__ rels,
                                                         const int64_t* __restrict__ pos,
                                                         const int64_t* __restrict__ neg, int batch, float reg,
                                                         float* __restrict__ work) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= batch) return;
  const TransrWork off = TransrWork::at(batch, d, k);
  const int64_t r = rels[b];
  const float* W = trans + r * static_cast<int64_t>(d) * k;
  const float* eh = emb + heads[b] * lde;
  const float* ep = emb + pos[b] * lde;
  const float* en = emb + neg[b] * lde;
  float h[kMaxCols], tp[kMaxCols], tn[kMaxCols], er[kMaxCols];
#pragma unroll
  for (int cc = 0; cc < kMaxCols; ++cc) h[cc] = tp[cc] = tn[cc] = er[cc] = 0.f;
  for (int i = 0; i < d; ++i) {
    const float xh = eh[i], xp = ep[i], xn = en[i];
#pragma unroll
    for (int cc = 0; cc < kMaxCols; ++cc) {
      const int j = lane + 64 * cc;
      if (j < k) {
        const float w = W[static_cast<int64_t>(i) * k + j];
        h[cc] = fmaf(xh, w, h[cc]);
        tp[cc] = fmaf(xp, w, tp[cc]);
        tn[cc] = fmaf(xn, w, tn[cc]);
      }
    }
  }
  float sp = 0.f, sn = 0.f, q = 0.f;
#pragma unroll
  for (int cc = 0; cc < kMaxCols; ++cc) {
    const int j = lane + 64 * cc;
    if (j < k) {
      er[cc] = rel_emb[r * k + j];
      const float dp = h[cc] + er[cc] - tp[cc], dn = h[cc] + er[cc] - tn[cc];
      sp = fmaf(dp, dp, sp);
      sn = fmaf(dn, dn, sn);
      q += h[cc] * h[cc] + er[cc] * er[cc] + tp[cc] * tp[cc] + tn[cc] * tn[cc];
    }
  }
  sp = wave_sum(sp);
  sn = wave_sum(sn);
  q = wave_sum(q);
  const float x = sn - sp;  // loss = softplus(-x)
  const float c = 1.f / (1.f + expf(-x)) - 1.f;
  if (lane == 0) work[off.term + b] = fmaxf(-x, 0.f) + log1pf(expf(-fabsf(x))) + reg * 0.5f * q;
  // gradients w.r.t. the projected vectors (per sample, before the 1/B and upstream scale)
  float* gp = work + off.gproj + static_cast<int64_t>(b) * 4 * k;
  float g3[3][kMaxCols];  // g_h', g_t+', g_t-' held by lane j (column j + 64*cc)
#pragma unroll
  for (int cc = 0; cc < kMaxCols; ++cc) {
    const int j = lane + 64 * cc;
    g3[0][cc] = g3[1][cc] = g3[2][cc] = 0.f;
    if (j < k) {
      const float dp = h[cc] + er[cc] - tp[cc], dn = h[cc] + er[cc] - tn[cc];
      const float g_common = 2.f * c * (dn - dp);
      g3[0][cc] = g_common + reg * h[cc];
      g3[1][cc] = 2.f * c * dp + reg * tp[cc];
      g3[2][cc] = -2.f * c * dn + reg * tn[cc];
      gp[j] = g3[0][cc];
      gp[k + j] = g3[1][cc];
      gp[2 * k + j] = g3[2][cc];
      gp[3 * k + j] = g_common + reg * er[cc];
    }
  }
  // table-row gradients d e = W g' (lane i owns row i of W; g'[j] is broadcast
  // from lane j % 64 with a shuffle)
  float* gr = work + off.grow + static_cast<int64_t>(b) * 3 * d;
#pragma unroll
  for (int ic = 0; ic < kMaxCols; ++ic) {
    const int i = lane + 64 * ic;
    if (ic * 64 >= d) break;  // wave-uniform
    float acc[3] = {0.f, 0.f, 0.f};
    const float* wr = W + static_cast<int64_t>(i < d ? i : 0) * k;
#pragma unroll
    for (int cc = 0; cc < kMaxCols; ++cc) {
      if (cc * 64 >= k) break;  // wave-uniform
      for (int jj = 0; jj < 64 && cc * 64 + jj < k; ++jj) {
        const float w = wr[cc * 64 + jj];
#pragma unroll
        for (int v = 0; v < 3; ++v) acc[v] = fmaf(w, __shfl(g3[v][cc], jj), acc[v]);
      }
    }
    if (i < d) {
#pragma unroll
      for (int v = 0; v < 3; ++v) gr[v * d + i] = acc[v];
    }
  }
}

__global__ __launch_bounds__(256) void transr_loss_kernel(const float* __restrict__ term, int batch,
                                                          float* __restrict__ loss) {
  __shared__ float red[256];
  float s = 0.f;
  for (int b = threadIdx.x; b < batch; b += 256) s += term[b];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (static_cast<int>(threadIdx.x) < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) *loss = red[0] / static_cast<float>(batch);
}

// d_emb[id] += scale * sum of the table-row gradients of every slot with that
// id, slots = [heads | pos | neg]; first occurrence owns the row (no atomics).
__global__ __launch_bounds__(256) void transr_scatter_kernel(const int64_t* __restrict__ heads,
                                                             const int64_t* __restrict__ pos,
                                                             const int64_t* __restrict__ neg, int batch, int d,
                                                             const float* __restrict__ grow,
                                                             const float* __restrict__ grad_out,
                                                             float* __restrict__ dst, int64_t lddst) {
  const int slots = 3 * batch;
  const int s0k = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (s0k >= slots) return;
  auto id_of = [&](int s) -> int64_t { return s < batch ? heads[s] : (s < 2 * batch ? pos[s - batch] : neg[s - 2 * batch]); };
  const int64_t id = id_of(s0k);
  bool dup = false;
  for (int s0 = 0; s0 < s0k && !dup; s0 += 64) dup = __any(s0 + lane < s0k && id_of(s0 + lane) == id);
  if (dup) return;
  const float scale = grad_out[0] / static_cast<float>(batch);
  float g[kMaxCols] = {0.f, 0.f, 0.f, 0.f};
  for (int s0 = s0k; s0 < slots; s0 += 64) {
    unsigned long long mask = __ballot(s0 + lane < slots && id_of(s0 + lane) == id);
    while (mask) {
      const int bit = __ffsll(static_cast<long long>(mask)) - 1;
      mask &= mask - 1;
      const int s = s0 + bit;
      const int b = s % batch, v = s / batch;  // v: 0 head, 1 pos, 2 neg
      const float* src = grow + (static_cast<int64_t>(b) * 3 + v) * d;
#pragma unroll
      for (int cc = 0; cc < kMaxCols; ++cc) {
        const int j = lane + 64 * cc;
        if (j < d) g[cc] = fmaf(src[j], scale, g[cc]);
      }
    }
  }
#pragma unroll
  for (int cc = 0; cc < kMaxCols; ++cc) {
    const int j = lane + 64 * cc;
    if (j < d) dst[id * lddst + j] += g[cc];
  }
}

// Per relation r (blockIdx.x) and a 4096-entry slice of trans[r]
// (blockIdx.y): d trans[r][i][j] = scale * sum over samples of relation r, in
// batch order, of e_h[i] g_h'[j] + e_t+[i] g_t+'[j] + e_t-[i] g_t-'[j];
// slice 0 also produces d rel_emb[r] = scale * sum g_er.
// The block lists relation r's samples first (256 relation ids per pass,
// ballot + wave counts -> batch order), then stages kWgradStage of them at a
// time in LDS -- the three table rows and the four projected gradients, every
// load of the stage in flight at once -- so the per-sample accumulation reads
// LDS instead of waiting on a chain of dependent global loads per sample (the
// former sample-serial loop was latency-bound: 1.6 ms per call at B = 512).
// Per entry the samples are summed in batch order with the same fma chain.
constexpr int kWgradStage = 8;

__global__ __launch_bounds__(256) void transr_wgrad_kernel(const float* __restrict__ emb, int64_t lde, int d, int k,
                                                           const int64_t* __restrict__ heads,
                                                           const int64_t* __restrict__ rels,
                                                           const int64_t* __restrict__ pos,
                                                           const int64_t* __restrict__ neg, int batch,
                                                           const float* __restrict__ gproj,
                                                           const float* __restrict__ grad_out,
                                                           float* __restrict__ d_rel, float* __restrict__ d_trans) {
  constexpr int kPer = 16;
  extern __shared__ __attribute__((aligned(16))) float stage[];  // [kWgradStage][3d + 4k]
  __shared__ int s_ids[256];
  __shared__ int s_wcnt[4];
  const int r = blockIdx.x;
  const int tid = static_cast<int>(threadIdx.x), lane = tid & 63, wv = tid >> 6;
  const int64_t dk = static_cast<int64_t>(d) * k;
  const int64_t e0 = static_cast<int64_t>(blockIdx.y) * 256 * kPer;
  const float scale = grad_out[0] / static_cast<float>(batch);
  const int row_w = 3 * d + 4 * k;
  float acc[kPer];
  int ei[kPer], ej[kPer];
#pragma unroll
  for (int t = 0; t < kPer; ++t) {
    acc[t] = 0.f;
    const int64_t e = e0 + static_cast<int64_t>(t) * 256 + tid;
    ei[t] = e < dk ? static_cast<int>(e / k) : -1;
    ej[t] = e < dk ? static_cast<int>(e % k) : 0;
  }
  float racc = 0.f;
  for (int w0 = 0; w0 < batch; w0 += 256) {
    const int b = w0 + tid;
    const bool hit = b < batch && rels[b] == r;
    const uint64_t m = __ballot(hit);
    if (lane == 0) s_wcnt[wv] = __popcll(m);
    __syncthreads();
    int base = 0;
    for (int w = 0; w < wv; ++w) base += s_wcnt[w];
    const int total = s_wcnt[0] + s_wcnt[1] + s_wcnt[2] + s_wcnt[3];
    if (hit) s_ids[base + __popcll(m & ((1ull << lane) - 1ull))] = b;
    __syncthreads();
    for (int c0 = 0; c0 < total; c0 += kWgradStage) {
      const int cnt = min(kWgradStage, total - c0);
      for (int x = tid; x < cnt * row_w; x += 256) {
        const int s = x / row_w, o = x - s * row_w;
        const int bb = s_ids[c0 + s];
        float v;
        if (o < 3 * d) {
          const int which = o / d, i = o - which * d;
          const int64_t id = which == 0 ? heads[bb] : (which == 1 ? pos[bb] : neg[bb]);
          v = emb[id * lde + i];
        } else {
          v = gproj[static_cast<int64_t>(bb) * 4 * k + (o - 3 * d)];
        }
        stage[x] = v;
      }
      __syncthreads();
      for (int s = 0; s < cnt; ++s) {
        const float* eh = stage + s * row_w;
        const float* ep = eh + d;
        const float* en = ep + d;
        const float* g = en + d;
#pragma unroll
        for (int t = 0; t < kPer; ++t) {
          if (ei[t] >= 0) {
            const int i = ei[t], j = ej[t];
            float v = eh[i] * g[j];
            v = fmaf(ep[i], g[k + j], v);
            v = fmaf(en[i], g[2 * k + j], v);
            acc[t] += v;
          }
        }
        if (blockIdx.y == 0 && tid < k) racc += g[3 * k + tid];
      }
      __syncthreads();  // the stage is read before the next one overwrites it
    }
    __syncthreads();  // s_ids / s_wcnt are read before the next window rewrites them
  }
#pragma unroll
  for (int t = 0; t < kPer; ++t) {
    const int64_t e = e0 + static_cast<int64_t>(t) * 256 + threadIdx.x;
    if (e < dk) d_trans[static_cast<int64_t>(r) * dk + e] = acc[t] * scale;
  }
  if (blockIdx.y == 0 && static_cast<int>(threadIdx.x) < k) d_rel[static_cast<int64_t>(r) * k + threadIdx.x] = racc * scale;
}

}  // namespace kgat

extern "C" int64_t kgat_transr_work_floats(int32_t batch, int32_t d, int32_t k) {
  return kgat::TransrWork::size(batch, d, k);
}

extern "C" int kgat_transr_fwd_f32(const float* emb, int64_t ld_emb, const float* rel_emb, const float* trans,
                                   int32_t d, int32_t k, const int64_t* heads, const int64_t* rels,
                                   const int64_t* pos, const int64_t* neg, int32_t batch, float reg, float* loss,
                                   float* work, void* stream) {
  if (!emb || !rel_emb || !trans || !heads || !rels || !pos || !neg || !loss || !work || batch <= 0) return KGAT_ERR_INVALID;
  if (d <= 0 || k <= 0 || d > 256 || k > 256 || ld_emb < d) return KGAT_ERR_INVALID;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(kgat::transr_fwd_kernel, dim3((batch + 3) / 4), dim3(256), 0, st, emb, ld_emb, rel_emb, trans, d,
                     k, heads, rels, pos, neg, batch, reg, work);
  KGAT_LAUNCH_CHECK();
  hipLaunchKernelGGL(kgat::transr_loss_kernel, dim3(1), dim3(256), 0, st, work, batch, loss);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int kgat_transr_bwd_f32(const float* emb, int64_t ld_emb, int32_t d, int32_t k, const int64_t* heads,
                                   const int64_t* rels, const int64_t* pos, const int64_t* neg, int32_t batch,
                                   int32_t n_rel, const float* work, const float* grad_out, float* d_emb,
                                   int64_t ld_demb, float* d_rel, float* d_trans, void* stream) {
  if (!emb || !heads || !rels || !pos || !neg || !work || !grad_out || !d_emb || !d_rel || !d_trans || batch <= 0 ||
      n_rel <= 0)
    return KGAT_ERR_INVALID;
  if (d <= 0 || k <= 0 || d > 256 || k > 256 || ld_emb < d || ld_demb < d) return KGAT_ERR_INVALID;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const kgat::TransrWork off = kgat::TransrWork::at(batch, d, k);
  hipLaunchKernelGGL(kgat::transr_scatter_kernel, dim3((3 * batch + 3) / 4), dim3(256), 0, st, heads, pos, neg, batch,
                     d, work + off.grow, grad_out, d_emb, ld_demb);
  KGAT_LAUNCH_CHECK();
  const int64_t dk = static_cast<int64_t>(d) * k;
  const int ys = static_cast<int>((dk + 4095) / 4096);
  const size_t smem = sizeof(float) * kgat::kWgradStage * (3 * static_cast<size_t>(d) + 4 * static_cast<size_t>(k));
  hipLaunchKernelGGL(kgat::transr_wgrad_kernel, dim3(n_rel, ys), dim3(256), smem, st, emb, ld_emb, d, k, heads, rels, pos,
                     neg, batch, work + off.gproj, grad_out, d_rel, d_trans);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}
