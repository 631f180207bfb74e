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
#include <cstdlib>

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
  // the three gathered rows in registers (lane l holds element l + 64*ic), broadcast by
  // shuffles in the loop below: no dependent global load per step of i
  float rh[kMaxCols], rp[kMaxCols], rn[kMaxCols];
#pragma unroll
  for (int ic = 0; ic < kMaxCols; ++ic) {
    const int i = lane + 64 * ic;
    rh[ic] = i < d ? eh[i] : 0.f;
    rp[ic] = i < d ? ep[i] : 0.f;
    rn[ic] = i < d ? en[i] : 0.f;
  }
  // rows of W_r in groups of kRowGroup: the group's loads are issued before its fmas, so a
  // wave has kRowGroup * kMaxCols loads in flight instead of one dependent step per row
  constexpr int kRowGroup = 8;
  auto bcast = [&](const float (&v)[kMaxCols], int i) {
    const int ic = i >> 6;
    return __shfl(ic == 0 ? v[0] : ic == 1 ? v[1] : ic == 2 ? v[2] : v[3], i & 63);
  };
  auto rows = [&](int i0, int cnt) {
    float w[kRowGroup][kMaxCols];
#pragma unroll
    for (int u = 0; u < kRowGroup; ++u)
#pragma unroll
      for (int cc = 0; cc < kMaxCols; ++cc) {
        const int j = lane + 64 * cc;
        w[u][cc] = (u < cnt && j < k) ? W[static_cast<int64_t>(i0 + u) * k + j] : 0.f;
      }
#pragma unroll
    for (int u = 0; u < kRowGroup; ++u) {
      if (u >= cnt) break;  // wave-uniform
      const float xh = bcast(rh, i0 + u), xp = bcast(rp, i0 + u), xn = bcast(rn, i0 + u);
#pragma unroll
      for (int cc = 0; cc < kMaxCols; ++cc) {
        if (lane + 64 * cc < k) {
          h[cc] = fmaf(xh, w[u][cc], h[cc]);
          tp[cc] = fmaf(xp, w[u][cc], tp[cc]);
          tn[cc] = fmaf(xn, w[u][cc], tn[cc]);
        }
      }
    }
  };
  for (int i0 = 0; i0 < d; i0 += kRowGroup) rows(i0, min(kRowGroup, d - i0));
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
      const int jn = min(64, k - cc * 64);
      for (int j0 = 0; j0 < jn; j0 += kRowGroup) {  // kRowGroup loads of the row in flight
        float w[kRowGroup];
#pragma unroll
        for (int u = 0; u < kRowGroup; ++u) w[u] = j0 + u < jn ? wr[cc * 64 + j0 + u] : 0.f;
#pragma unroll
        for (int u = 0; u < kRowGroup; ++u) {
          if (j0 + u >= jn) break;  // wave-uniform
#pragma unroll
          for (int v = 0; v < 3; ++v) acc[v] = fmaf(w[u], __shfl(g3[v][cc], j0 + u), acc[v]);
        }
      }
    }
    if (i < d) {
#pragma unroll
      for (int v = 0; v < 3; ++v) gr[v * d + i] = acc[v];
    }
  }
}

// The same forward on the fp32 MFMA (v_mfma_f32_16x16x4_f32), one block per (relation r,
// 16-sample chunk z of r's samples in batch order): the chunk's 3 x 16 gathered rows
// (head / pos / neg) form one 48 x D operand in LDS and W_r is read ONCE per chunk
// (the per-sample kernel re-reads all d x k of W_r for every sample: 256 KB per sample
// at d = k = 256) for both products of the chunk:
//   P  = X W_r          [48, K]   (h', t+', t-' rows)
//   GR = G W_r^T        [48, D]   (d e_h, d e_t+, d e_t- from g_h', g_t+', g_t-')
// Wave w owns the output column tiles w, w+4, ... of both products.  K order of the sums:
// the first product walks k = 0..D-1 in steps of 4 (lane group q takes k0 + q); the
// second takes the contiguous ranges q*K/4 + s, so its operands load as float4.
constexpr int kTrChunk = 16;

template <int D, int K>
__global__ __launch_bounds__(256) void transr_fwd_mfma_kernel(const float* __restrict__ emb, int64_t lde,
                                                              const float* __restrict__ rel_emb,
                                                              const float* __restrict__ trans,
                                                              const int64_t* __restrict__ heads,
                                                              const int64_t* __restrict__ rels,
                                                              const int64_t* __restrict__ pos,
                                                              const int64_t* __restrict__ neg, int batch, float reg,
                                                              float* __restrict__ work) {
  constexpr int XP = D + 4, GP = K + 4;  // LDS row pitches (floats)
  constexpr int NTP = (K / 16 + 3) / 4;  // column tiles per wave, first product
  constexpr int NTG = (D / 16 + 3) / 4;  // column tiles per wave, second product
  __shared__ __attribute__((aligned(16))) float xs[3 * kTrChunk * XP];
  __shared__ __attribute__((aligned(16))) float gs[3 * kTrChunk * GP];
  __shared__ int s_ids[kTrChunk];
  __shared__ int s_wcnt[4];
  __shared__ int s_seen;
  const int r = blockIdx.x, z = blockIdx.y;
  const int tid = static_cast<int>(threadIdx.x), lane = tid & 63, wv = tid >> 6;
  const int q = lane >> 4, c = lane & 15;
  // relation r's samples in batch order; this block takes list positions [z*16, z*16 + 16)
  if (tid == 0) s_seen = 0;
  __syncthreads();
  const int lo = z * kTrChunk;
  for (int w0 = 0; w0 < batch; w0 += 256) {
    const int b = w0 + tid;
    const bool hit = b < batch && rels[b] == r;
    const uint64_t m = __ballot(hit);
    if (lane == 0) s_wcnt[wv] = __popcll(m);
    __syncthreads();
    int base = s_seen;
    for (int w = 0; w < wv; ++w) base += s_wcnt[w];
    const int li = base + __popcll(m & ((1ull << lane) - 1ull));
    if (hit && li >= lo && li < lo + kTrChunk) s_ids[li - lo] = b;
    __syncthreads();
    if (tid == 0) s_seen += s_wcnt[0] + s_wcnt[1] + s_wcnt[2] + s_wcnt[3];
    __syncthreads();
  }
  const int cnt = min(kTrChunk, s_seen - lo);
  if (cnt <= 0) return;  // block-uniform
  const TransrWork off = TransrWork::at(batch, D, K);
  // stage the 48 gathered rows (row v*16 + s: v = head / pos / neg of sample s; zeros past cnt)
  for (int i = tid; i < 3 * kTrChunk * (D / 4); i += 256) {
    const int row = i / (D / 4), c4 = i % (D / 4), v = row / kTrChunk, s = row % kTrChunk;
    float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
    if (s < cnt) {
      const int b = s_ids[s];
      const int64_t id = v == 0 ? heads[b] : (v == 1 ? pos[b] : neg[b]);
      x = *reinterpret_cast<const float4*>(emb + id * lde + c4 * 4);
    }
    *reinterpret_cast<float4*>(xs + row * XP + c4 * 4) = x;
  }
  __syncthreads();
  const float* W = trans + static_cast<int64_t>(r) * D * K;
  // ---- P = X W_r  (lane (q, c): A = X[mt*16 + c][k0 + q], B = W[k0 + q][nt*16 + c])
  floatx4 acc[3][NTP];
#pragma unroll
  for (int mt = 0; mt < 3; ++mt)
#pragma unroll
    for (int j = 0; j < NTP; ++j) acc[mt][j] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int k0 = 0; k0 < D; k0 += 4) {
    float bw[NTP];
#pragma unroll
    for (int j = 0; j < NTP; ++j) {
      const int nt = wv + 4 * j;
      bw[j] = nt < K / 16 ? W[static_cast<int64_t>(k0 + q) * K + nt * 16 + c] : 0.f;
    }
#pragma unroll
    for (int mt = 0; mt < 3; ++mt) {
      const float a = xs[(mt * kTrChunk + c) * XP + k0 + q];
#pragma unroll
      for (int j = 0; j < NTP; ++j)
        if (wv + 4 * j < K / 16) acc[mt][j] = mfma16x4(a, bw[j], acc[mt][j]);
    }
  }
  // P rows into LDS (C layout: lane (q, c) element i = row q*4 + i, column nt*16 + c)
#pragma unroll
  for (int mt = 0; mt < 3; ++mt)
#pragma unroll
    for (int j = 0; j < NTP; ++j) {
      const int nt = wv + 4 * j;
      if (nt >= K / 16) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i) gs[(mt * kTrChunk + q * 4 + i) * GP + nt * 16 + c] = acc[mt][j][i];
    }
  __syncthreads();
  // ---- per sample (wave w: samples w, w+4, ...): scores, loss term, the projected gradients
  //      (gproj, for the weight gradient) and G = (g_h', g_t+', g_t-') rows over P in LDS
  constexpr int KC = (K + 63) / 64;
  for (int s = wv; s < cnt; s += 4) {
    const int b = s_ids[s];
    float h[KC], tp[KC], tn[KC], er[KC];
    float sp = 0.f, sn = 0.f, qq = 0.f;
#pragma unroll
    for (int cc = 0; cc < KC; ++cc) {
      const int j = lane + 64 * cc;
      h[cc] = tp[cc] = tn[cc] = er[cc] = 0.f;
      if (j < K) {
        h[cc] = gs[s * GP + j];
        tp[cc] = gs[(kTrChunk + s) * GP + j];
        tn[cc] = gs[(2 * kTrChunk + s) * GP + j];
        er[cc] = rel_emb[static_cast<int64_t>(r) * K + j];
        const float dp = h[cc] + er[cc] - tp[cc], dn = h[cc] + er[cc] - tn[cc];
        sp = fmaf(dp, dp, sp);
        sn = fmaf(dn, dn, sn);
        qq += h[cc] * h[cc] + er[cc] * er[cc] + tp[cc] * tp[cc] + tn[cc] * tn[cc];
      }
    }
    sp = wave_sum(sp);
    sn = wave_sum(sn);
    qq = wave_sum(qq);
    const float x = sn - sp;  // loss = softplus(-x)
    const float cf = 1.f / (1.f + expf(-x)) - 1.f;
    if (lane == 0) work[off.term + b] = fmaxf(-x, 0.f) + log1pf(expf(-fabsf(x))) + reg * 0.5f * qq;
    float* gp = work + off.gproj + static_cast<int64_t>(b) * 4 * K;
#pragma unroll
    for (int cc = 0; cc < KC; ++cc) {
      const int j = lane + 64 * cc;
      if (j < K) {
        const float dp = h[cc] + er[cc] - tp[cc], dn = h[cc] + er[cc] - tn[cc];
        const float g_common = 2.f * cf * (dn - dp);
        const float g0 = g_common + reg * h[cc];
        const float g1 = 2.f * cf * dp + reg * tp[cc];
        const float g2 = -2.f * cf * dn + reg * tn[cc];
        gp[j] = g0;
        gp[K + j] = g1;
        gp[2 * K + j] = g2;
        gp[3 * K + j] = g_common + reg * er[cc];
        gs[s * GP + j] = g0;
        gs[(kTrChunk + s) * GP + j] = g1;
        gs[(2 * kTrChunk + s) * GP + j] = g2;
      }
    }
  }
  // rows of absent samples stay zero: their X rows were staged as zeros, so their P rows are 0
  __syncthreads();
  // ---- GR = G W_r^T  (lane (q, c): A = G[mt*16 + c][q*K/4 + s], B = W[nt*16 + c][q*K/4 + s])
  floatx4 ag[3][NTG];
#pragma unroll
  for (int mt = 0; mt < 3; ++mt)
#pragma unroll
    for (int j = 0; j < NTG; ++j) ag[mt][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  constexpr int KQ = K / 4;
#pragma unroll 1
  for (int s0 = 0; s0 < KQ; s0 += 4) {
    float4 bw[NTG];
#pragma unroll
    for (int j = 0; j < NTG; ++j) {
      const int nt = wv + 4 * j;
      bw[j] = nt < D / 16 ? *reinterpret_cast<const float4*>(W + static_cast<int64_t>(nt * 16 + c) * K + q * KQ + s0)
                          : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float4 av[3];
#pragma unroll
    for (int mt = 0; mt < 3; ++mt) av[mt] = *reinterpret_cast<const float4*>(gs + (mt * kTrChunk + c) * GP + q * KQ + s0);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int mt = 0; mt < 3; ++mt)
#pragma unroll
        for (int j = 0; j < NTG; ++j)
          if (wv + 4 * j < D / 16) ag[mt][j] = mfma16x4(av[mt][t], bw[j][t], ag[mt][j]);
  }
  float* gr = work + off.grow;
#pragma unroll
  for (int mt = 0; mt < 3; ++mt)
#pragma unroll
    for (int j = 0; j < NTG; ++j) {
      const int nt = wv + 4 * j;
      if (nt >= D / 16) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int s = q * 4 + i;
        if (s < cnt) gr[(static_cast<int64_t>(s_ids[s]) * 3 + mt) * D + nt * 16 + c] = ag[mt][j][i];
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
// With row_map the row is d_emb[row_map[id]] (a compact gradient, kgat_frontier_build's
// numbering; -1 skipped).
__global__ __launch_bounds__(256) void transr_scatter_kernel(const int64_t* __restrict__ heads,
                                                             const int64_t* __restrict__ pos,
                                                             const int64_t* __restrict__ neg, int batch, int d,
                                                             const float* __restrict__ grow,
                                                             const float* __restrict__ grad_out,
                                                             float* __restrict__ dst, int64_t lddst,
                                                             const int32_t* __restrict__ row_map) {
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
  const int64_t row = row_map ? static_cast<int64_t>(row_map[id]) : id;
  if (row < 0) return;
#pragma unroll
  for (int cc = 0; cc < kMaxCols; ++cc) {
    const int j = lane + 64 * cc;
    if (j < d) dst[row * lddst + j] += g[cc];
  }
}

// Per relation r (blockIdx.x) and a slice of 16 * (256 / k) rows of trans[r]
// (blockIdx.y; thread: column j = tid % k, 16 consecutive rows): d trans[r][i][j] = scale * sum over samples of relation r, in
// batch order, of e_h[i] g_h'[j] + e_t+[i] g_t+'[j] + e_t-[i] g_t-'[j];
// slice 0 also produces d rel_emb[r] = scale * sum g_er.
// The block lists relation r's samples first (256 relation ids per pass,
// ballot + wave counts -> batch order), then stages wgrad_stage(d, k) of them at a
// time in LDS -- the three table rows and the four projected gradients, every
// load of the stage in flight at once -- so the per-sample accumulation reads
// LDS instead of waiting on a chain of dependent global loads per sample (the
// former sample-serial loop was latency-bound: 1.6 ms per call at B = 512).
// Per entry the samples are summed in batch order with the same fma chain.
constexpr int kWgradChunk = 32;          // samples of one relation per block (list positions)
constexpr int kWgradStageMax = 32;       // samples staged per round (at most)
constexpr int kWgradLdsFloats = 14336;   // 56 KB of staged rows per block
__host__ __device__ inline int wgrad_stage(int d, int k) {
  const int n = kWgradLdsFloats / (3 * d + 4 * k);
  return n < 1 ? 1 : (n > kWgradStageMax ? kWgradStageMax : n);
}

__global__ __launch_bounds__(256) void transr_wgrad_kernel(const float* __restrict__ emb, int64_t lde, int d, int k,
                                                           const int64_t* __restrict__ heads,
                                                           const int64_t* __restrict__ rels,
                                                           const int64_t* __restrict__ pos,
                                                           const int64_t* __restrict__ neg, int batch,
                                                           const float* __restrict__ gproj,
                                                           float* __restrict__ part, int* __restrict__ counts,
                                                           int n_chunk) {
  constexpr int kPer = 16;
  extern __shared__ __attribute__((aligned(16))) float stage[];  // [wgrad_stage(d, k)][3d + 4k]
  __shared__ int s_ids[kWgradChunk];
  __shared__ int s_seen;
  __shared__ int s_wcnt[4];
  __shared__ int64_t s_row[3 * kWgradStageMax];
  const int r = blockIdx.x;
  const int tid = static_cast<int>(threadIdx.x), lane = tid & 63, wv = tid >> 6;
  const int64_t dk = static_cast<int64_t>(d) * k;
  const int row_w = 3 * d + 4 * k;
  const int stage_n = wgrad_stage(d, k);
  // this thread's entries: column j = tid % k, rows [i0, i0 + kPer) of the block's row slice
  const int nrb = 256 / k;                       // row blocks per slice (k <= 256)
  const bool active = tid < nrb * k;
  const int j = active ? tid % k : 0;
  const int i0 = blockIdx.y * nrb * kPer + (active ? tid / k : 0) * kPer;
  const bool vec = (d % 4 == 0) && (k % 4 == 0);  // 16-byte aligned staged rows
  float acc[kPer];
#pragma unroll
  for (int t = 0; t < kPer; ++t) acc[t] = 0.f;
  float racc = 0.f;
  // relation r's samples in batch order; this block takes list positions [z*C, (z+1)*C)
  const int z = blockIdx.z, lo = z * kWgradChunk;
  if (tid == 0) s_seen = 0;
  __syncthreads();
  for (int w0 = 0; w0 < batch; w0 += 256) {
    const int b = w0 + tid;
    const bool hit = b < batch && rels[b] == r;
    const uint64_t m = __ballot(hit);
    if (lane == 0) s_wcnt[wv] = __popcll(m);
    __syncthreads();
    int base = s_seen;
    for (int w = 0; w < wv; ++w) base += s_wcnt[w];
    const int li = base + __popcll(m & ((1ull << lane) - 1ull));
    if (hit && li >= lo && li < lo + kWgradChunk) s_ids[li - lo] = b;
    __syncthreads();
    if (tid == 0) s_seen += s_wcnt[0] + s_wcnt[1] + s_wcnt[2] + s_wcnt[3];
    __syncthreads();
  }
  const int n_r = s_seen;
  if (z == 0 && blockIdx.y == 0 && tid == 0) counts[r] = n_r;
  const int total = min(kWgradChunk, n_r - lo);
  if (total <= 0) return;  // block-uniform: this chunk holds no sample
  {
    for (int c0 = 0; c0 < total; c0 += stage_n) {
      const int cnt = min(stage_n, total - c0);
      if (tid < 3 * cnt) {  // the stage's table-row offsets: one dependent load, once
        const int s = tid / 3, which = tid - 3 * s;
        const int bb = s_ids[c0 + s];
        s_row[tid] = (which == 0 ? heads[bb] : (which == 1 ? pos[bb] : neg[bb])) * lde;
      }
      __syncthreads();
      // kUnroll independent loads in flight per thread and pass
      constexpr int kUnroll = 8;
      for (int x0 = 0; x0 < cnt * row_w; x0 += 256 * kUnroll) {
        float v[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
          const int x = x0 + u * 256 + tid;
          v[u] = 0.f;
          if (x < cnt * row_w) {
            const int s = x / row_w, o = x - s * row_w;
            if (o < 3 * d) {
              const int which = o / d;
              v[u] = emb[s_row[3 * s + which] + (o - which * d)];
            } else {
              v[u] = gproj[static_cast<int64_t>(s_ids[c0 + s]) * 4 * k + (o - 3 * d)];
            }
          }
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
          const int x = x0 + u * 256 + tid;
          if (x < cnt * row_w) stage[x] = v[u];
        }
      }
      __syncthreads();
      for (int s = 0; s < cnt; ++s) {
        const float* eh = stage + s * row_w;
        const float* ep = eh + d;
        const float* en = ep + d;
        const float* g = en + d;
        if (blockIdx.y == 0 && tid < k) racc += g[3 * k + tid];
        if (!active || i0 >= d) continue;  // this thread's rows lie past d
        const float gh = g[j], gpp = g[k + j], gn = g[2 * k + j];
        float xh[kPer], xp[kPer], xn[kPer];
        if (vec) {
#pragma unroll
          for (int t = 0; t < kPer; t += 4) {
            const float4 a = *reinterpret_cast<const float4*>(eh + i0 + t);
            const float4 b = *reinterpret_cast<const float4*>(ep + i0 + t);
            const float4 c = *reinterpret_cast<const float4*>(en + i0 + t);
            xh[t] = a.x; xh[t + 1] = a.y; xh[t + 2] = a.z; xh[t + 3] = a.w;
            xp[t] = b.x; xp[t + 1] = b.y; xp[t + 2] = b.z; xp[t + 3] = b.w;
            xn[t] = c.x; xn[t + 1] = c.y; xn[t + 2] = c.z; xn[t + 3] = c.w;
          }
        } else {
#pragma unroll
          for (int t = 0; t < kPer; ++t) {
            const int i = i0 + t < d ? i0 + t : 0;
            xh[t] = eh[i];
            xp[t] = ep[i];
            xn[t] = en[i];
          }
        }
#pragma unroll
        for (int t = 0; t < kPer; ++t) {
          float v = xh[t] * gh;
          v = fmaf(xp[t], gpp, v);
          v = fmaf(xn[t], gn, v);
          acc[t] += v;
        }
      }
      __syncthreads();  // the stage is read before the next one overwrites it
    }
  }
  // this chunk's partial sums: part[(r * n_chunk + z)] = [trans rows (d*k) | rel (k)]
  float* pz = part + (static_cast<int64_t>(r) * n_chunk + z) * (dk + k);
  if (active) {
#pragma unroll
    for (int t = 0; t < kPer; ++t)
      if (i0 + t < d) pz[static_cast<int64_t>(i0 + t) * k + j] = acc[t];
  }
  if (blockIdx.y == 0 && tid < k) pz[dk + tid] = racc;
}

// d trans[r] / d rel_emb[r] = scale * (sum of relation r's chunk partials in chunk order)
__global__ __launch_bounds__(256) void transr_wgrad_reduce_kernel(const float* __restrict__ part,
                                                                  const int* __restrict__ counts, int n_rel, int d,
                                                                  int k, int n_chunk, int batch,
                                                                  const float* __restrict__ grad_out,
                                                                  float* __restrict__ d_rel,
                                                                  float* __restrict__ d_trans) {
  const int64_t dk = static_cast<int64_t>(d) * k, w = dk + k;
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (idx >= n_rel * w) return;
  const int r = static_cast<int>(idx / w);
  const int64_t e = idx - r * w;
  const int nz = (counts[r] + kWgradChunk - 1) / kWgradChunk;
  float s = 0.f;
  for (int z = 0; z < nz; ++z) s += part[(static_cast<int64_t>(r) * n_chunk + z) * w + e];
  const float v = s * (grad_out[0] / static_cast<float>(batch));
  if (e < dk) d_trans[r * dk + e] = v;
  else d_rel[static_cast<int64_t>(r) * k + (e - dk)] = v;
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

template <int D>
static bool launch_fwd_mfma_d(int k, int n_rel, const float* emb, int64_t ld_emb, const float* rel_emb,
                              const float* trans, const int64_t* heads, const int64_t* rels, const int64_t* pos,
                              const int64_t* neg, int batch, float reg, float* work, hipStream_t st) {
  const dim3 grid(n_rel, (batch + kgat::kTrChunk - 1) / kgat::kTrChunk);
#define KGAT_TR_K(KK)                                                                                              \
  case KK:                                                                                                         \
    hipLaunchKernelGGL((kgat::transr_fwd_mfma_kernel<D, KK>), grid, dim3(256), 0, st, emb, ld_emb, rel_emb, trans, \
                       heads, rels, pos, neg, batch, reg, work);                                                   \
    return true;
  switch (k) {
    KGAT_TR_K(64)
    KGAT_TR_K(128)
    KGAT_TR_K(256)
    default: return false;
  }
#undef KGAT_TR_K
}

extern "C" int kgat_transr_fwd_ex_f32(const float* emb, int64_t ld_emb, const float* rel_emb, const float* trans,
                                      int32_t d, int32_t k, int32_t n_rel, const int64_t* heads, const int64_t* rels,
                                      const int64_t* pos, const int64_t* neg, int32_t batch, float reg, float* loss,
                                      float* work, void* stream) {
  if (!emb || !rel_emb || !trans || !heads || !rels || !pos || !neg || !loss || !work || batch <= 0 || n_rel <= 0)
    return KGAT_ERR_INVALID;
  if (d <= 0 || k <= 0 || d > 256 || k > 256 || ld_emb < d) return KGAT_ERR_INVALID;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // the chunked MFMA form where W_r is big enough for its re-reads to dominate (d >= 128); the
  // per-sample kernel otherwise (and for shapes without an instantiation)
  bool done = false;
  if (d >= 128 && (ld_emb & 3) == 0 && (reinterpret_cast<uintptr_t>(emb) & 15) == 0 &&
      (reinterpret_cast<uintptr_t>(trans) & 15) == 0 && n_rel <= 65535 * 64 && (batch + 15) / 16 <= 65535) {
    if (d == 128) done = launch_fwd_mfma_d<128>(k, n_rel, emb, ld_emb, rel_emb, trans, heads, rels, pos, neg, batch, reg, work, st);
    else if (d == 256) done = launch_fwd_mfma_d<256>(k, n_rel, emb, ld_emb, rel_emb, trans, heads, rels, pos, neg, batch, reg, work, st);
  }
  if (!done)
    hipLaunchKernelGGL(kgat::transr_fwd_kernel, dim3((batch + 3) / 4), dim3(256), 0, st, emb, ld_emb, rel_emb, trans, d,
                       k, heads, rels, pos, neg, batch, reg, work);
  KGAT_LAUNCH_CHECK();
  hipLaunchKernelGGL(kgat::transr_loss_kernel, dim3(1), dim3(256), 0, st, work, batch, loss);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int64_t kgat_transr_bwd_workspace_floats(int32_t batch, int32_t d, int32_t k, int32_t n_rel) {
  if (batch <= 0 || d <= 0 || k <= 0 || n_rel <= 0) return -1;
  const int64_t n_chunk = (batch + kgat::kWgradChunk - 1) / kgat::kWgradChunk;
  return static_cast<int64_t>(n_rel) * n_chunk * (static_cast<int64_t>(d) * k + k) + n_rel;  // partials + counts
}

extern "C" int kgat_transr_bwd_f32(const float* emb, int64_t ld_emb, int32_t d, int32_t k, const int64_t* heads,
                                   const int64_t* rels, const int64_t* pos, const int64_t* neg, int32_t batch,
                                   int32_t n_rel, const float* work, const float* grad_out, float* d_emb,
                                   int64_t ld_demb, float* d_rel, float* d_trans, float* workspace,
                                   int64_t workspace_floats, void* stream) {
  return kgat_transr_bwd_ex_f32(emb, ld_emb, d, k, heads, rels, pos, neg, batch, n_rel, work, grad_out, d_emb,
                                ld_demb, nullptr, d_rel, d_trans, workspace, workspace_floats, stream);
}

extern "C" int kgat_transr_bwd_ex_f32(const float* emb, int64_t ld_emb, int32_t d, int32_t k, const int64_t* heads,
                                      const int64_t* rels, const int64_t* pos, const int64_t* neg, int32_t batch,
                                      int32_t n_rel, const float* work, const float* grad_out, float* d_emb,
                                      int64_t ld_demb, const int32_t* row_map, float* d_rel, float* d_trans,
                                      float* workspace, int64_t workspace_floats, void* stream) {
  if (!emb || !heads || !rels || !pos || !neg || !work || !grad_out || !d_emb || !d_rel || !d_trans || batch <= 0 ||
      n_rel <= 0)
    return KGAT_ERR_INVALID;
  if (d <= 0 || k <= 0 || d > 256 || k > 256 || ld_emb < d || ld_demb < d) return KGAT_ERR_INVALID;
  if (!workspace || workspace_floats < kgat_transr_bwd_workspace_floats(batch, d, k, n_rel)) return KGAT_ERR_WORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const kgat::TransrWork off = kgat::TransrWork::at(batch, d, k);
  hipLaunchKernelGGL(kgat::transr_scatter_kernel, dim3((3 * batch + 3) / 4), dim3(256), 0, st, heads, pos, neg, batch,
                     d, work + off.grow, grad_out, d_emb, ld_demb, row_map);
  KGAT_LAUNCH_CHECK();
  const int n_chunk = (batch + kgat::kWgradChunk - 1) / kgat::kWgradChunk;
  const int64_t w = static_cast<int64_t>(d) * k + k;
  float* part = workspace;
  int* counts = reinterpret_cast<int*>(workspace + static_cast<int64_t>(n_rel) * n_chunk * w);
  const int ys = (d + (256 / k) * 16 - 1) / ((256 / k) * 16);  // row slices of 16 rows per thread
  const size_t smem = sizeof(float) * kgat::wgrad_stage(d, k) * (3 * static_cast<size_t>(d) + 4 * static_cast<size_t>(k));
  hipLaunchKernelGGL(kgat::transr_wgrad_kernel, dim3(n_rel, ys, n_chunk), dim3(256), smem, st, emb, ld_emb, d, k, heads,
                     rels, pos, neg, batch, work + off.gproj, part, counts, n_chunk);
  KGAT_LAUNCH_CHECK();
  const int64_t total = static_cast<int64_t>(n_rel) * w;
  hipLaunchKernelGGL(kgat::transr_wgrad_reduce_kernel, dim3(static_cast<unsigned>((total + 255) / 256)), dim3(256), 0,
                     st, part, counts, n_rel, d, k, n_chunk, batch, grad_out, d_rel, d_trans);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}
