// a10/a11 -- NFM (src/model/NFM/model.py:73-129, hidden_layer.py:31-35):
//   z  = 0.5 * ((x V)^2 - (x^2)(V^2))                    bi-interaction pooling
//   h  = Dropout(ReLU(W_l h + b_l)) for each hidden layer
//   y  = W_out h + (x w + b)                              deep + wide heads
//   L  = -mean log(1e-10 + sigmoid(y_pos - y_neg)) + lambda |W_out|^2 / 2
// x is a sparse feature batch (CSR here; the reference feeds COO, ~5 nnz/row:
// user one-hot + item one-hot + its KG tails).  One wave per row: lanes own
// embedding / hidden columns (lane + 64*c), the pooling is an embedding-bag
// gather of the row's feature vectors, each MLP layer a lane-parallel matvec
// with the input broadcast by shuffles.  Weight gradients are reduced over
// rows in row order and the feature gradients (dV, dw) are scattered with
// duplicate feature ids summed in entry order: deterministic, no atomics.
#include <cmath>

#include "common.hpp"

namespace kgat {

constexpr int kNfmMaxLayers = 4;
constexpr int kNfmCols = 4;  // dims <= 256

struct NfmNet {
  const float* V;       // [F][d]
  int64_t ldv;
  const float* w_lin;   // [F]
  const float* b_lin;   // [1]
  const float* W[kNfmMaxLayers];
  const float* b[kNfmMaxLayers];
  int dims[kNfmMaxLayers + 1];  // dims[0] = d, dims[l+1] = out of layer l
  int n_layers;
  const float* W_out;   // [dims[L]]
  float p;
  uint64_t seed;
};

__device__ __forceinline__ float vget(const float (&v)[kNfmCols], int i) {
  // value of column i held by lane i % 64 in slot i / 64 (wave-uniform i)
  float r = 0.f;
#pragma unroll
  for (int cc = 0; cc < kNfmCols; ++cc)
    if (i / 64 == cc) r = __shfl(v[cc], i % 64);
  return r;
}

__device__ __forceinline__ bool nfm_keep(const NfmNet& N, int layer, int64_t row, int o) {
  return dropout_keep(N.seed + 0x51ed270b7ull * static_cast<uint64_t>(layer + 1),
                      static_cast<uint64_t>(row) * 4096 + o, N.p);
}

// act layout per row: [ s (d) | z (d) | pre_0 (dims[1]) | ... | pre_{L-1} ]
__device__ __forceinline__ int64_t act_width(const NfmNet& N) {
  int64_t w = 2 * N.dims[0];
  for (int l = 0; l < N.n_layers; ++l) w += N.dims[l + 1];
  return w;
}

__global__ __launch_bounds__(256) void nfm_fwd_kernel(NfmNet N, const int64_t* __restrict__ rowptr,
                                                      const int64_t* __restrict__ col, const float* __restrict__ val,
                                                      int64_t rows, float* __restrict__ act, float* __restrict__ y) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const int d = N.dims[0];
  const int64_t beg = rowptr[r], end = rowptr[r + 1];
  float s[kNfmCols] = {0.f, 0.f, 0.f, 0.f}, q[kNfmCols] = {0.f, 0.f, 0.f, 0.f};
  float wide = 0.f;
  for (int64_t e = beg; e < end; ++e) {
    const int64_t c = col[e];
    const float x = val[e];
    const float* v = N.V + c * N.ldv;
#pragma unroll
    for (int cc = 0; cc < kNfmCols; ++cc) {
      const int j = lane + 64 * cc;
      if (j < d) {
        const float t = x * v[j];
        s[cc] += t;
        q[cc] = fmaf(t, t, q[cc]);
      }
    }
    if (lane == 0) wide = fmaf(x, N.w_lin[c], wide);
  }
  float h[kNfmCols];
  float* ar = act ? act + r * act_width(N) : nullptr;
#pragma unroll
  for (int cc = 0; cc < kNfmCols; ++cc) {
    const int j = lane + 64 * cc;
    h[cc] = 0.5f * (s[cc] * s[cc] - q[cc]);
    if (ar && j < d) {
      ar[j] = s[cc];
      ar[d + j] = h[cc];
    }
  }
  int64_t off = 2 * d;
  const float scale = N.p > 0.f ? 1.f / (1.f - N.p) : 1.f;
  for (int l = 0; l < N.n_layers; ++l) {
    const int din = N.dims[l], dout = N.dims[l + 1];
    const float* W = N.W[l];
    float nh[kNfmCols] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int cc = 0; cc < kNfmCols; ++cc) {
      const int o = lane + 64 * cc;
      float acc = 0.f;
      for (int i = 0; i < din; ++i) {
        const float hi = vget(h, i);
        if (o < dout) acc = fmaf(W[static_cast<int64_t>(o) * din + i], hi, acc);
      }
      if (o < dout) {
        const float pre = acc + N.b[l][o];
        if (ar) ar[off + o] = pre;
        float a = fmaxf(pre, 0.f);
        if (N.p > 0.f) a = nfm_keep(N, l, r, o) ? a * scale : 0.f;
        nh[cc] = a;
      }
    }
#pragma unroll
    for (int cc = 0; cc < kNfmCols; ++cc) h[cc] = nh[cc];
    off += dout;
  }
  const int dl = N.dims[N.n_layers];
  float deep = 0.f;
#pragma unroll
  for (int cc = 0; cc < kNfmCols; ++cc) {
    const int j = lane + 64 * cc;
    if (j < dl) deep = fmaf(N.W_out[j], h[cc], deep);
  }
  deep = wave_sum(deep);
  if (lane == 0) y[r] = (wide + N.b_lin[0]) + deep;
}

// loss over B pairs (rows b and B+b); dy[row] = dL/dy (before the upstream scale)
__global__ __launch_bounds__(256) void nfm_loss_kernel(const float* __restrict__ y, int batch, const float* __restrict__ W_out,
                                                       int dl, float lam, float* __restrict__ loss,
                                                       float* __restrict__ dy) {
  __shared__ float red[256];
  float acc = 0.f;
  for (int b = threadIdx.x; b < batch; b += 256) {
    const float dlt = y[b] - y[batch + b];
    const float sg = 1.f / (1.f + expf(-dlt));
    acc += -logf(1e-10f + sg);
    const float g = -(sg * (1.f - sg)) / (1e-10f + sg) / static_cast<float>(batch);
    dy[b] = g;
    dy[batch + b] = -g;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (static_cast<int>(threadIdx.x) < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    float w2 = 0.f;
    for (int j = 0; j < dl; ++j) w2 = fmaf(W_out[j], W_out[j], w2);
    *loss = red[0] / static_cast<float>(batch) + lam * (sqrtf(w2) * sqrtf(w2)) / 2.f;
  }
}

// Per row: push g = gout * dy[row] back through the MLP; keeps dpre per layer
// and dz in the workspace ([rows][sum dims[1..L]] and [rows][d]).
__global__ __launch_bounds__(256) void nfm_bwd_kernel(NfmNet N, const float* __restrict__ act, int64_t rows,
                                                      const float* __restrict__ dy, const float* __restrict__ gout,
                                                      float* __restrict__ dpre_ws, float* __restrict__ dz_ws) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const int L = N.n_layers;
  const float g = gout[0] * dy[r];
  const float* ar = act + r * act_width(N);
  int64_t hsum = 0;
  for (int l = 0; l < L; ++l) hsum += N.dims[l + 1];
  float* dpr = dpre_ws + r * hsum;
  const float scale = N.p > 0.f ? 1.f / (1.f - N.p) : 1.f;
  float dh[kNfmCols];
  const int dl = N.dims[L];
#pragma unroll
  for (int cc = 0; cc < kNfmCols; ++cc) {
    const int j = lane + 64 * cc;
    dh[cc] = j < dl ? g * N.W_out[j] : 0.f;
  }
  // offsets of pre_l inside act and of dpre_l inside the workspace row
  int64_t pre_off[kNfmMaxLayers], dp_off[kNfmMaxLayers];
  int64_t o1 = 2 * N.dims[0], o2 = 0;
  for (int l = 0; l < L; ++l) {
    pre_off[l] = o1;
    dp_off[l] = o2;
    o1 += N.dims[l + 1];
    o2 += N.dims[l + 1];
  }
  for (int l = L - 1; l >= 0; --l) {
    const int din = N.dims[l], dout = N.dims[l + 1];
    float dp[kNfmCols];
#pragma unroll
    for (int cc = 0; cc < kNfmCols; ++cc) {
      const int o = lane + 64 * cc;
      dp[cc] = 0.f;
      if (o < dout) {
        const float pre = ar[pre_off[l] + o];
        float v = pre > 0.f ? dh[cc] : 0.f;
        if (N.p > 0.f) v = nfm_keep(N, l, r, o) ? v * scale : 0.f;
        dp[cc] = v;
        dpr[dp_off[l] + o] = v;
      }
    }
    const float* W = N.W[l];
#pragma unroll
    for (int cc = 0; cc < kNfmCols; ++cc) {
      const int i = lane + 64 * cc;
      float acc = 0.f;
      for (int o = 0; o < dout; ++o) {
        const float dpo = vget(dp, o);
        if (i < din) acc = fmaf(W[static_cast<int64_t>(o) * din + i], dpo, acc);
      }
      dh[cc] = i < din ? acc : 0.f;
    }
  }
  const int d = N.dims[0];
#pragma unroll
  for (int cc = 0; cc < kNfmCols; ++cc) {
    const int j = lane + 64 * cc;
    if (j < d) dz_ws[r * d + j] = dh[cc];
  }
}

// Input of layer l for row r, column i (recomputed from the saved act).
__device__ __forceinline__ float nfm_hin(const NfmNet& N, const float* ar, int l, int64_t r, int i,
                                         const int64_t* pre_off, float scale) {
  if (l == 0) return ar[N.dims[0] + i];
  const float pre = ar[pre_off[l - 1] + i];
  float a = fmaxf(pre, 0.f);
  if (N.p > 0.f) a = nfm_keep(N, l - 1, r, i) ? a * scale : 0.f;
  return a;
}

// Layer l < L: dW_l[o][i] = sum_r dpre_l[r][o] * hin_l[r][i], db_l[o] = sum_r dpre_l[r][o];
// l == L (output head): dW_out[j] = sum_r g_r h_L[r][j] + lam W_out[j], db_lin = sum_r g_r.
// Rows are summed in row order (deterministic); one thread per output element.
__global__ __launch_bounds__(256) void nfm_wgrad_kernel(NfmNet N, int l, const float* __restrict__ act, int64_t rows,
                                                        const float* __restrict__ dy, const float* __restrict__ gout,
                                                        const float* __restrict__ dpre_ws, float lam,
                                                        float* __restrict__ dWl, float* __restrict__ dbl,
                                                        float* __restrict__ dW_out, float* __restrict__ db_lin) {
  const int L = N.n_layers;
  int64_t pre_off[kNfmMaxLayers], dp_off[kNfmMaxLayers];
  int64_t o1 = 2 * N.dims[0], o2 = 0;
  for (int k = 0; k < L; ++k) {
    pre_off[k] = o1;
    dp_off[k] = o2;
    o1 += N.dims[k + 1];
    o2 += N.dims[k + 1];
  }
  const int64_t aw = o1, hsum = o2;
  const float scale = N.p > 0.f ? 1.f / (1.f - N.p) : 1.f;
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (l < L) {
    const int din = N.dims[l], dout = N.dims[l + 1];
    if (t < dout * din) {
      const int o = t / din, i = t % din;
      float acc = 0.f;
      for (int64_t r = 0; r < rows; ++r)
        acc = fmaf(dpre_ws[r * hsum + dp_off[l] + o], nfm_hin(N, act + r * aw, l, r, i, pre_off, scale), acc);
      dWl[t] = acc;
    } else if (t < dout * din + dout) {
      const int o = t - dout * din;
      float acc = 0.f;
      for (int64_t r = 0; r < rows; ++r) acc += dpre_ws[r * hsum + dp_off[l] + o];
      dbl[o] = acc;
    }
  } else {
    const int dl = N.dims[L];
    const float go = gout[0];
    if (t < dl) {
      float acc = 0.f;
      for (int64_t r = 0; r < rows; ++r) acc = fmaf(go * dy[r], nfm_hin(N, act + r * aw, L, r, t, pre_off, scale), acc);
      dW_out[t] = acc + go * lam * N.W_out[t];
    } else if (t == dl) {
      float acc = 0.f;
      for (int64_t r = 0; r < rows; ++r) acc += go * dy[r];
      db_lin[0] = acc;
    }
  }
}

// Feature gradients: entry k (row rk, feature ck, value xk) contributes
//   dV[ck]  += xk * (s_rk - xk V[ck]) * dz_rk        d z / d V through the pooling
//   dw[ck]  += xk * g_rk                               the wide head
// One wave per entry; the first entry of each feature id owns the feature row
// and sums every entry of that id in entry order.  dV / dw are zero-filled.
__global__ __launch_bounds__(256) void nfm_feat_kernel(NfmNet N, const int64_t* __restrict__ erow,
                                                       const int64_t* __restrict__ col, const float* __restrict__ val,
                                                       int64_t nnz, const float* __restrict__ act,
                                                       const float* __restrict__ dz_ws, const float* __restrict__ dy,
                                                       const float* __restrict__ gout, float* __restrict__ dV,
                                                       int64_t lddv, float* __restrict__ dw) {
  const int64_t k = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (k >= nnz) return;
  const int64_t c = col[k];
  bool dup = false;
  for (int64_t s0 = 0; s0 < k && !dup; s0 += 64) dup = __any(s0 + lane < k && col[s0 + lane] == c);
  if (dup) return;
  const int d = N.dims[0];
  int64_t aw = 2 * d;
  for (int l = 0; l < N.n_layers; ++l) aw += N.dims[l + 1];
  const float go = gout[0];
  const float* vc = N.V + c * N.ldv;
  float g[kNfmCols] = {0.f, 0.f, 0.f, 0.f};
  float gw = 0.f;
  for (int64_t s0 = k; s0 < nnz; s0 += 64) {
    unsigned long long mask = __ballot(s0 + lane < nnz && col[s0 + lane] == c);
    while (mask) {
      const int bit = __ffsll(static_cast<long long>(mask)) - 1;
      mask &= mask - 1;
      const int64_t e = s0 + bit;
      const int64_t r = erow[e];
      const float x = val[e];
      const float* sr = act + r * aw;
      const float* dzr = dz_ws + r * d;
#pragma unroll
      for (int cc = 0; cc < kNfmCols; ++cc) {
        const int j = lane + 64 * cc;
        if (j < d) g[cc] = fmaf(x * (sr[j] - x * vc[j]), dzr[j], g[cc]);
      }
      gw = fmaf(x, go * dy[r], gw);
    }
  }
#pragma unroll
  for (int cc = 0; cc < kNfmCols; ++cc) {
    const int j = lane + 64 * cc;
    if (j < d) dV[c * lddv + j] += g[cc];
  }
  if (lane == 0) dw[c] += gw;
}

__global__ __launch_bounds__(256) void rowptr_kernel(const int64_t* __restrict__ rows_sorted, int64_t nnz,
                                                     int64_t n_rows, int64_t* __restrict__ rowptr) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (r > n_rows) return;
  int64_t lo = 0, hi = nnz;  // first index with rows_sorted[idx] >= r
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (rows_sorted[mid] < r) lo = mid + 1;
    else hi = mid;
  }
  rowptr[r] = lo;
}

static int check_net(const NfmNet& N) {
  if (!N.V || !N.w_lin || !N.b_lin || !N.W_out || N.n_layers < 0 || N.n_layers > kNfmMaxLayers) return KGAT_ERR_INVALID;
  for (int l = 0; l <= N.n_layers; ++l)
    if (N.dims[l] <= 0 || N.dims[l] > 64 * kNfmCols) return KGAT_ERR_UNSUPPORTED_DIM;
  for (int l = 0; l < N.n_layers; ++l)
    if (!N.W[l] || !N.b[l]) return KGAT_ERR_INVALID;
  if (!(N.p >= 0.f && N.p < 1.f)) return KGAT_ERR_INVALID;
  return KGAT_OK;
}

}  // namespace kgat

extern "C" int kgat_coo_rowptr(const int64_t* rows_sorted, int64_t nnz, int64_t n_rows, int64_t* rowptr,
                               void* stream) {
  if (!rows_sorted && nnz > 0) return KGAT_ERR_INVALID;
  if (!rowptr || n_rows < 0) return KGAT_ERR_INVALID;
  hipLaunchKernelGGL(kgat::rowptr_kernel, dim3((n_rows + 256) / 256), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), rows_sorted, nnz, n_rows, rowptr);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int64_t kgat_nfm_act_floats(const kgat_nfm* net, int64_t rows) {
  int64_t w = 2 * net->dims[0];
  for (int l = 0; l < net->n_layers; ++l) w += net->dims[l + 1];
  return rows * w;
}

static kgat::NfmNet to_net(const kgat_nfm* n) {
  kgat::NfmNet N{};
  N.V = n->V;
  N.ldv = n->ld_v;
  N.w_lin = n->w_lin;
  N.b_lin = n->b_lin;
  N.n_layers = n->n_layers;
  for (int l = 0; l < kgat::kNfmMaxLayers; ++l) {
    N.W[l] = l < n->n_layers ? n->W[l] : nullptr;
    N.b[l] = l < n->n_layers ? n->b[l] : nullptr;
  }
  for (int l = 0; l <= kgat::kNfmMaxLayers; ++l) N.dims[l] = l <= n->n_layers ? n->dims[l] : 0;
  N.W_out = n->W_out;
  N.p = n->dropout_p;
  N.seed = n->seed;
  return N;
}

extern "C" int kgat_nfm_fwd_f32(const kgat_nfm* net, const int64_t* rowptr, const int64_t* col, const float* val,
                                int64_t rows, float* act, float* y, void* stream) {
  if (!net || !rowptr || !y || rows < 0) return KGAT_ERR_INVALID;
  const kgat::NfmNet N = to_net(net);
  if (int e = kgat::check_net(N)) return e;
  if (rows == 0) return KGAT_OK;
  hipLaunchKernelGGL(kgat::nfm_fwd_kernel, dim3((rows + 3) / 4), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), N,
                     rowptr, col, val, rows, act, y);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int kgat_nfm_loss_f32(const kgat_nfm* net, const float* y, int32_t batch, float lam, float* loss, float* dy,
                                 void* stream) {
  if (!net || !y || !loss || !dy || batch <= 0) return KGAT_ERR_INVALID;
  hipLaunchKernelGGL(kgat::nfm_loss_kernel, dim3(1), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), y, batch,
                     net->W_out, net->dims[net->n_layers], lam, loss, dy);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int64_t kgat_nfm_bwd_workspace(const kgat_nfm* net, int64_t rows) {
  int64_t h = 0;
  for (int l = 0; l < net->n_layers; ++l) h += net->dims[l + 1];
  return rows * (h + net->dims[0]);
}

extern "C" int kgat_nfm_bwd_f32(const kgat_nfm* net, const int64_t* erow, const int64_t* col, const float* val,
                                int64_t nnz, int64_t rows, const float* act, const float* dy, const float* grad_out,
                                float lam, float* dV, int64_t ld_dv, float* dw_lin, float* db_lin, float* const* dW,
                                float* const* db, float* dW_out, float* workspace, int64_t workspace_floats,
                                void* stream) {
  if (!net || !act || !dy || !grad_out || !dV || !dw_lin || !db_lin || !dW_out || !workspace || rows < 0 || nnz < 0)
    return KGAT_ERR_INVALID;
  const kgat::NfmNet N = to_net(net);
  if (int e = kgat::check_net(N)) return e;
  if (N.n_layers > 0 && (!dW || !db)) return KGAT_ERR_INVALID;
  if (workspace_floats < kgat_nfm_bwd_workspace(net, rows)) return KGAT_ERR_WORKSPACE;
  if (rows == 0) return KGAT_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int64_t hsum = 0;
  for (int l = 0; l < N.n_layers; ++l) hsum += N.dims[l + 1];
  float* dpre = workspace;
  float* dz = workspace + rows * hsum;
  hipLaunchKernelGGL(kgat::nfm_bwd_kernel, dim3((rows + 3) / 4), dim3(256), 0, st, N, act, rows, dy, grad_out, dpre, dz);
  KGAT_LAUNCH_CHECK();
  for (int l = 0; l <= N.n_layers; ++l) {  // one launch per layer + the output head
    const int w = l < N.n_layers ? N.dims[l] * N.dims[l + 1] + N.dims[l + 1] : N.dims[N.n_layers] + 1;
    float* wl = l < N.n_layers ? dW[l] : nullptr;
    float* bl = l < N.n_layers ? db[l] : nullptr;
    hipLaunchKernelGGL(kgat::nfm_wgrad_kernel, dim3((w + 255) / 256), dim3(256), 0, st, N, l, act, rows, dy, grad_out,
                       dpre, lam, wl, bl, dW_out, db_lin);
    KGAT_LAUNCH_CHECK();
  }
  if (nnz > 0) {
    hipLaunchKernelGGL(kgat::nfm_feat_kernel, dim3((nnz + 3) / 4), dim3(256), 0, st, N, erow, col, val, nnz, act, dz, dy,
                       grad_out, dV, ld_dv, dw_lin);
    KGAT_LAUNCH_CHECK();
  }
  return KGAT_OK;
}
