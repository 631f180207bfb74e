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

#include <hipcub/hipcub.hpp>

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

__device__ __forceinline__ void wave_lds_sync() {
  // orders this wave's LDS writes before its later LDS reads of other lanes' data
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// LDS plan of the forward (offsets / pitches in floats).  With `wlds` the hidden
// weights sit in LDS zero-padded to [round16(dout)][round16(din) + 4] (+4: the 16
// rows a B fragment reads land 4 banks apart) with round16(dout) biases; then one
// 16 x P activation tile per wave.
struct NfmLds {
  int w_off[kNfmMaxLayers], w_pitch[kNfmMaxLayers], b_off[kNfmMaxLayers];
  int tile_off, P, total;
  bool wlds;
};

// Forward over tiles of 16 rows, one tile per wave.
//  pooling: 16-lane groups each pool one row; the row pointers of all 16 rows
//           and the first 16 entries of the group's 4 rows are loaded up front,
//           then 4 entries' embedding rows at a time; lane cl of a group owns
//           columns cl + 16k; z goes to the wave's LDS tile (zero-padded to a
//           multiple of 16 columns), s and z to act;
//  layers:  pre[16][dout] = h[16][din] W^T on v_mfma_f32_16x16x4_f32 -- lane l
//           feeds A = h[l&15][k] and B = W[n][k] for k = k0 + 4(l>>4) + j, four
//           MFMAs per 16-wide k step; bias, act store, ReLU and dropout fused on
//           the accumulators, which overwrite the tile once the layer is done;
//  head:    y = (x w + b) + W_out . h_L, a 16-lane reduction per row.
// NC: dims <= 16 NC (column slots per pooling lane and output blocks per layer).
// One hidden layer on a wave's 16-row tile: pre = h W^T + b (NB output blocks of 16,
// blocks past dout read clamped weights and are dropped), act store, ReLU,
// dropout; the result overwrites the tile.
template <int NB, bool WLDS>
__device__ __forceinline__ void nfm_layer(const NfmNet& N, const NfmLds& plan, const float* smem, float* tile, int l,
                                          int64_t off, int64_t row0, int64_t rows, float* __restrict__ act, int64_t aw,
                                          float scale) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, cl = lane & 15;
  const int P = plan.P;
  const int din = N.dims[l], dout = N.dims[l + 1];
  const int kpad = (din + 15) & ~15;
  const int nblk = (dout + 15) >> 4;
  floatx4 acc[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) acc[nb] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int wp = WLDS ? plan.w_pitch[l] : 0;
  // global weights (too large for LDS): 16-byte fragment loads where the rows allow them
  const bool w4 = !WLDS && (din & 3) == 0 && (reinterpret_cast<uintptr_t>(N.W[l]) & 15) == 0;
  const float* wlds = WLDS ? smem + plan.w_off[l] + cl * wp + 4 * g : nullptr;
  const float* a_row = tile + cl * P + 4 * g;
  if (!WLDS && w4 && (din & 15) == 0 && (dout & 15) == 0) {
    // global weights whose 16-wide blocks are whole: every fragment is one unconditional 16-byte load
    // (no per-fragment branches), and the next k-step's fragments are in flight while this step's
    // MFMAs run -- an L2 round trip per k-step otherwise stalls the wave (8 k-steps per 128-wide layer)
    // one per-lane base; the blocks' offsets are wave-uniform
    const float* wb = N.W[l] + static_cast<int64_t>(cl) * din + 4 * g;
    const int64_t bstride = static_cast<int64_t>(16) * din;
    float4 bn[NB];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) bn[nb] = *reinterpret_cast<const float4*>(wb + (nb < nblk ? nb : nblk - 1) * bstride);
    for (int k0 = 0; k0 < kpad; k0 += 16) {
      const float4 a4 = *reinterpret_cast<const float4*>(a_row + k0);
      float4 b4[NB];
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) b4[nb] = bn[nb];
      if (k0 + 16 < kpad) {
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
          bn[nb] = *reinterpret_cast<const float4*>(wb + (nb < nblk ? nb : nblk - 1) * bstride + k0 + 16);
      }
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        acc[nb] = mfma16x4(a4.x, b4[nb].x, acc[nb]);
        acc[nb] = mfma16x4(a4.y, b4[nb].y, acc[nb]);
        acc[nb] = mfma16x4(a4.z, b4[nb].z, acc[nb]);
        acc[nb] = mfma16x4(a4.w, b4[nb].w, acc[nb]);
      }
    }
  } else {
    for (int k0 = 0; k0 < kpad; k0 += 16) {  // one A fragment feeds NB interleaved MFMA chains
      const float4 a4 = *reinterpret_cast<const float4*>(a_row + k0);
      float4 b4[NB];
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {  // every B fragment of the step read before the first MFMA
        const int nbc = nb < nblk ? nb : nblk - 1;
        if (WLDS) {
          b4[nb] = *reinterpret_cast<const float4*>(wlds + nbc * 16 * wp + k0);
        } else {
          const int n = nbc * 16 + cl, kk = k0 + 4 * g;
          const float* wr = N.W[l] + static_cast<int64_t>(n < dout ? n : 0) * din;
          if (w4 && n < dout && kk + 3 < din) {
            b4[nb] = *reinterpret_cast<const float4*>(wr + kk);  // one 16-byte load (L1 / L2 resident weights)
          } else {
            b4[nb].x = (n < dout && kk < din) ? wr[kk] : 0.f;
            b4[nb].y = (n < dout && kk + 1 < din) ? wr[kk + 1] : 0.f;
            b4[nb].z = (n < dout && kk + 2 < din) ? wr[kk + 2] : 0.f;
            b4[nb].w = (n < dout && kk + 3 < din) ? wr[kk + 3] : 0.f;
          }
        }
      }
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        acc[nb] = mfma16x4(a4.x, b4[nb].x, acc[nb]);
        acc[nb] = mfma16x4(a4.y, b4[nb].y, acc[nb]);
        acc[nb] = mfma16x4(a4.z, b4[nb].z, acc[nb]);
        acc[nb] = mfma16x4(a4.w, b4[nb].w, acc[nb]);
      }
    }
  }
  wave_lds_sync();  // every lane has read the layer input
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    if (nb < nblk) {
      const int n = nb * 16 + cl;
      const float bias = WLDS ? smem[plan.b_off[l] + n] : (n < dout ? N.b[l][n] : 0.f);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = g * 4 + i;
        const int64_t r = row0 + m;
        const float pre = acc[nb][i] + bias;
        if (act && r < rows && n < dout) act[r * aw + off + n] = pre;
        float h = fmaxf(pre, 0.f);
        if (N.p > 0.f) h = nfm_keep(N, l, r, n) ? h * scale : 0.f;
        tile[m * P + n] = n < dout ? h : 0.f;
      }
    }
  }
  wave_lds_sync();
}

// Column j of pooling slot k of lane cl: V4 (d % 4 == 0, 16-byte aligned rows) -- each lane loads float4s,
// slots 4f..4f+3 = columns 4 cl + 64 f + t; otherwise one float per slot, columns cl + 16 k.
template <bool V4>
__device__ __forceinline__ int pool_col(int cl, int k) {
  return V4 ? 4 * cl + 64 * (k >> 2) + (k & 3) : cl + 16 * k;
}

template <int NC, bool WLDS, bool V4>
__device__ __forceinline__ void nfm_fwd_tile(const NfmNet& N, const NfmLds& plan, const float* smem, float* tile,
                                             int64_t row0, const int64_t* __restrict__ rowptr,
                                             const int64_t* __restrict__ col, const float* __restrict__ val,
                                             int64_t rows, float* __restrict__ act, float* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, cl = lane & 15;
  const int P = plan.P;
  const int d = N.dims[0];
  const int dpad = (d + 15) & ~15;
  const int64_t aw = act_width(N);
  // row pointers of the wave's 16 rows (lanes 0..16); rows past the end are empty
  int rp = 0;  // entry offsets fit 32 bits (a batch holds < 2^31 entries)
  if (lane <= 16) rp = static_cast<int>(rowptr[row0 + lane < rows ? row0 + lane : rows]);
  int colk[NC];
  float colm[NC];
#pragma unroll
  for (int k = 0; k < NC; ++k) {  // this lane's pooling columns, clamped to the row (exact x*v*1 when inside)
    const int j = pool_col<V4>(cl, k);
    colk[k] = j < d ? j : d - 1;
    colm[k] = j < d ? 1.f : 0.f;
  }
  // round rr pools row rr*4 + g; lane cl holds entry beg + cl (past the end: x = 0),
  // and the next round's entries are loaded while this round's rows are fetched
  int nbeg = __shfl(rp, g), nend = __shfl(rp, g + 1);
  int nce = nend > nbeg ? static_cast<int>(col[nbeg + (cl < nend - nbeg ? cl : 0)]) : 0;
  float nxe = cl < nend - nbeg ? val[nbeg + cl] : 0.f;
#pragma unroll 1
  for (int rr = 0; rr < 4; ++rr) {
    const int m = rr * 4 + g;
    const int64_t r = row0 + m;
    const int beg = nbeg, end = nend;
    const int ce = nce;
    const float xe = nxe;
    if (rr < 3) {
      nbeg = __shfl(rp, m + 4);
      nend = __shfl(rp, m + 5);
      nce = nend > nbeg ? static_cast<int>(col[nbeg + (cl < nend - nbeg ? cl : 0)]) : 0;
      nxe = cl < nend - nbeg ? val[nbeg + cl] : 0.f;
    }
    float s[NC], q[NC];
#pragma unroll
    for (int k = 0; k < NC; ++k) s[k] = q[k] = 0.f;
    float wd = 0.f;
    for (int e0 = beg; e0 < end; e0 += 16) {
      const int cnt = end - e0 < 16 ? end - e0 : 16;
      int c_l = ce;
      float x_l = xe;
      if (e0 != beg) {  // rows of more than 16 entries
        c_l = static_cast<int>(col[e0 + (cl < cnt ? cl : 0)]);
        x_l = cl < cnt ? val[e0 + cl] : 0.f;
      }
      wd = fmaf(x_l, N.w_lin[c_l], wd);
      constexpr int EB = NC <= 4 ? 8 : 4;     // entries whose loads are in flight together
      for (int k0 = 0; k0 < cnt; k0 += EB) {  // summed in entry order
        float xb[EB], vb[EB][NC];
#pragma unroll
        for (int u = 0; u < EB; ++u) {
          const int src = g * 16 + (k0 + u < 16 ? k0 + u : 15);
          const uint32_t c = static_cast<uint32_t>(__shfl(c_l, src));
          xb[u] = k0 + u < 16 ? __shfl(x_l, src) : 0.f;
          const float* v = N.V + static_cast<uint64_t>(c) * static_cast<uint32_t>(N.ldv);
          if constexpr (V4) {
#pragma unroll
            for (int f = 0; f < NC / 4; ++f) {  // one 16-byte load per 4 columns (the row's bytes in 1/4 the loads)
              const int c4 = 4 * cl + 64 * f;
              const float4 x4 = c4 < d ? *reinterpret_cast<const float4*>(v + c4) : make_float4(0.f, 0.f, 0.f, 0.f);
              vb[u][4 * f] = x4.x;
              vb[u][4 * f + 1] = x4.y;
              vb[u][4 * f + 2] = x4.z;
              vb[u][4 * f + 3] = x4.w;
            }
          } else {
#pragma unroll
            for (int k = 0; k < NC; ++k) vb[u][k] = v[colk[k]];  // unconditional: columns clamped, masked below
          }
        }
#pragma unroll
        for (int u = 0; u < EB; ++u)
#pragma unroll
          for (int k = 0; k < NC; ++k) {
            const float t = xb[u] * vb[u][k] * colm[k];
            s[k] += t;
            q[k] = fmaf(t, t, q[k]);
          }
      }
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) wd += __shfl_xor(wd, o);
    if (cl == 0) tile[m * P + P - 1] = wd;  // the wide head waits in the tile's last pad column
    float* ar = act && r < rows ? act + r * aw : nullptr;
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const int j = pool_col<V4>(cl, k);
      if (j < dpad) {
        const float z = j < d ? 0.5f * (s[k] * s[k] - q[k]) : 0.f;
        tile[m * P + j] = z;
        if (ar && j < d) {
          ar[j] = s[k];
          ar[d + j] = z;
        }
      }
    }
  }
  wave_lds_sync();
  int64_t off = 2 * d;
  const float scale = N.p > 0.f ? 1.f / (1.f - N.p) : 1.f;
  for (int l = 0; l < N.n_layers; ++l) {
    const int nblk = (N.dims[l + 1] + 15) >> 4;  // output blocks: a compile-time count per instance
    if (nblk <= 1) nfm_layer<1, WLDS>(N, plan, smem, tile, l, off, row0, rows, act, aw, scale);
    else if (nblk <= 2) nfm_layer<2, WLDS>(N, plan, smem, tile, l, off, row0, rows, act, aw, scale);
    else if (nblk <= 4 || NC < 8) nfm_layer<(NC < 4 ? NC : 4), WLDS>(N, plan, smem, tile, l, off, row0, rows, act, aw, scale);
    else if (nblk <= 8 || NC < 16) nfm_layer<(NC < 8 ? NC : 8), WLDS>(N, plan, smem, tile, l, off, row0, rows, act, aw, scale);
    else nfm_layer<NC, WLDS>(N, plan, smem, tile, l, off, row0, rows, act, aw, scale);
    off += N.dims[l + 1];
  }
  const int dl = N.dims[N.n_layers];
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int m = rr * 4 + g;
    float deep = 0.f;
    for (int j = cl; j < dl; j += 16) deep = fmaf(N.W_out[j], tile[m * P + j], deep);
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) deep += __shfl_xor(deep, o);
    const int64_t r = row0 + m;
    if (cl == 0 && r < rows) y[r] = (tile[m * P + P - 1] + N.b_lin[0]) + deep;
  }
  wave_lds_sync();  // the tile is free for the wave's next rows
}

template <int NC, bool WLDS, bool V4>
__global__ __launch_bounds__(256, NC <= 4 ? 3 : NC <= 8 ? 2 : 1) void nfm_fwd_kernel(NfmNet N, NfmLds plan, const int64_t* __restrict__ rowptr,
                                                      const int64_t* __restrict__ col, const float* __restrict__ val,
                                                      int64_t rows, float* __restrict__ act, float* __restrict__ y) {
  extern __shared__ float smem[];
  const int wv = threadIdx.x >> 6;
  if (WLDS) {  // stage the hidden layers once per block (8 loads in flight per thread)
    for (int l = 0; l < N.n_layers; ++l) {
      const int din = N.dims[l], dout = N.dims[l + 1], pitch = plan.w_pitch[l];
      const int npad = (dout + 15) & ~15;
      const int total = npad * pitch;
      for (int t0 = threadIdx.x; t0 < total; t0 += 256 * 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int t = t0 + u * 256;
          const int n = t / pitch, k = t - n * pitch;
          v[u] = (t < total && n < dout && k < din) ? N.W[l][static_cast<int64_t>(n) * din + k] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (t0 + u * 256 < total) smem[plan.w_off[l] + t0 + u * 256] = v[u];
      }
      for (int t = threadIdx.x; t < npad; t += 256) smem[plan.b_off[l] + t] = t < dout ? N.b[l][t] : 0.f;
    }
    __syncthreads();
  }
  float* tile = smem + plan.tile_off + wv * 16 * plan.P;
  // persistent: the block walks 64-row groups (the staged weights serve them all)
  for (int64_t grp = blockIdx.x; grp * 64 < rows; grp += gridDim.x) {
    const int64_t row0 = grp * 64 + wv * 16;
    if (row0 < rows) nfm_fwd_tile<NC, WLDS, V4>(N, plan, smem, tile, row0, rowptr, col, val, rows, act, y);
  }
}


// Inference forward (PREDICT / eval: no dropout, no saved activations) for feature widths that are
// multiples of 16 up to 128: every MLP layer computed transposed, pre^T = W h^T with the weights the MFMA A
// operand and the tile's 16 rows its B operand, so a layer's accumulators (lane (q, c): features
// mb*16 + q*4 + i of row c) are the next layer's operand -- no LDS tile between layers -- and each lane's A
// operand of 4 consecutive MFMAs is one float4 of a weight row (all layers staged in LDS once per block).
// Pooling produces that layout directly: the four lanes c + 16 q of a row each read a quarter of every entry's
// feature row (float4 at kb*16 + q*4), 16 rows per wave at once; per feature the entries are summed in entry
// order (s and sum of squares: the training kernel's z bits).
constexpr int kNfmTB = 8;  // 16-wide feature blocks (widths <= 128)

struct NfmTPlan {
  int w_off[kNfmMaxLayers], pitch[kNfmMaxLayers], b_off[kNfmMaxLayers];
  int wout_off, total;
};

__global__ __launch_bounds__(1024) void nfm_fwd_t_kernel(NfmNet N, NfmTPlan plan, const int64_t* __restrict__ rowptr,
                                                         const int64_t* __restrict__ col,
                                                         const float* __restrict__ val, int64_t rows,
                                                         float* __restrict__ y) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  for (int l = 0; l < N.n_layers; ++l) {
    const int din = N.dims[l], dout = N.dims[l + 1];
    for (int t = threadIdx.x; t < din * dout; t += 1024) {
      const int n = t / din, k = t - n * din;
      smem[plan.w_off[l] + n * plan.pitch[l] + k] = N.W[l][t];
    }
    for (int t = threadIdx.x; t < dout; t += 1024) smem[plan.b_off[l] + t] = N.b[l][t];
  }
  for (int t = threadIdx.x; t < N.dims[N.n_layers]; t += 1024) smem[plan.wout_off + t] = N.W_out[t];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, q = lane >> 4, c = lane & 15;
  const int nb0 = N.dims[0] >> 4;
  const int64_t ntiles = (rows + 15) / 16;
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * 16 + wave; t < ntiles; t += static_cast<int64_t>(gridDim.x) * 16) {
    const int64_t r = t * 16 + c;
    float h[kNfmTB][4];
    float wd = 0.f;
    {
      float sq[kNfmTB][4];
#pragma unroll
      for (int kb = 0; kb < kNfmTB; ++kb)
#pragma unroll
        for (int i = 0; i < 4; ++i) h[kb][i] = sq[kb][i] = 0.f;
      if (r < rows) {
        const int64_t beg = rowptr[r], end = rowptr[r + 1];
        int64_t cn = beg < end ? col[beg] : 0;  // the next entry's id and value load under this one's row
        float xn = beg < end ? val[beg] : 0.f;
        for (int64_t e = beg; e < end; ++e) {
          const int64_t ce = cn;
          const float xe = xn;
          if (e + 1 < end) {
            cn = col[e + 1];
            xn = val[e + 1];
          }
          const float* v = N.V + ce * N.ldv + q * 4;
#pragma unroll
          for (int kb = 0; kb < kNfmTB; ++kb) {
            if (kb < nb0) {
              const float4 f = *reinterpret_cast<const float4*>(v + kb * 16);
              const float tv[4] = {xe * f.x, xe * f.y, xe * f.z, xe * f.w};
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                h[kb][i] += tv[i];
                sq[kb][i] = fmaf(tv[i], tv[i], sq[kb][i]);
              }
            }
          }
          wd = fmaf(xe, N.w_lin[ce], wd);  // the wide head, entries in order (every lane of the row alike)
        }
      }
#pragma unroll
      for (int kb = 0; kb < kNfmTB; ++kb)
#pragma unroll
        for (int i = 0; i < 4; ++i) h[kb][i] = 0.5f * (h[kb][i] * h[kb][i] - sq[kb][i]);
    }
    for (int l = 0; l < N.n_layers; ++l) {
      const int nbi = N.dims[l] >> 4, nbo = N.dims[l + 1] >> 4, pitch = plan.pitch[l];
      const float* W = smem + plan.w_off[l] + c * pitch + q * 4;
      const float* bs = smem + plan.b_off[l] + q * 4;
      float o[kNfmTB][4];
#pragma unroll
      for (int mb = 0; mb < kNfmTB; ++mb) {
        o[mb][0] = o[mb][1] = o[mb][2] = o[mb][3] = 0.f;
        if (mb < nbo) {  // (wave-uniform)
          floatx4 acc = {0.f, 0.f, 0.f, 0.f};
          const float* w = W + mb * 16 * pitch;
#pragma unroll
          for (int kb = 0; kb < kNfmTB; ++kb) {
            if (kb < nbi) {
              const float4 wk = *reinterpret_cast<const float4*>(w + kb * 16);
              acc = mfma16x4(wk.x, h[kb][0], acc);
              acc = mfma16x4(wk.y, h[kb][1], acc);
              acc = mfma16x4(wk.z, h[kb][2], acc);
              acc = mfma16x4(wk.w, h[kb][3], acc);
            }
          }
          const float4 b = *reinterpret_cast<const float4*>(bs + mb * 16);
          o[mb][0] = fmaxf(acc[0] + b.x, 0.f);
          o[mb][1] = fmaxf(acc[1] + b.y, 0.f);
          o[mb][2] = fmaxf(acc[2] + b.z, 0.f);
          o[mb][3] = fmaxf(acc[3] + b.w, 0.f);
        }
      }
#pragma unroll
      for (int mb = 0; mb < kNfmTB; ++mb)
#pragma unroll
        for (int i = 0; i < 4; ++i) h[mb][i] = o[mb][i];
    }
    const int nbl = N.dims[N.n_layers] >> 4;
    float deep = 0.f;
#pragma unroll
    for (int mb = 0; mb < kNfmTB; ++mb) {
      if (mb < nbl) {
        const float4 wo = *reinterpret_cast<const float4*>(smem + plan.wout_off + mb * 16 + q * 4);
        deep = fmaf(wo.x, h[mb][0], deep);
        deep = fmaf(wo.y, h[mb][1], deep);
        deep = fmaf(wo.z, h[mb][2], deep);
        deep = fmaf(wo.w, h[mb][3], deep);
      }
    }
    deep += __shfl_xor(deep, 16);
    deep += __shfl_xor(deep, 32);
    if (q == 0 && r < rows) y[r] = (wd + N.b_lin[0]) + deep;
  }
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
// Split over 64-row chunks (blockIdx.y): one thread per output element sums its chunk's rows
// in row order into part[chunk][t]; nfm_wgrad_reduce_kernel then adds the chunks in chunk
// order -- deterministic, and every CU has work at training batch sizes.
constexpr int kNfmRowChunk = 64;

__global__ __launch_bounds__(256) void nfm_wgrad_kernel(NfmNet N, int l, const float* __restrict__ act, int64_t rows,
                                                        const float* __restrict__ dy, const float* __restrict__ gout,
                                                        const float* __restrict__ dpre_ws, int w,
                                                        float* __restrict__ part) {
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
  if (t >= w) return;
  const int64_t r0 = static_cast<int64_t>(blockIdx.y) * kNfmRowChunk;
  const int64_t r1 = r0 + kNfmRowChunk < rows ? r0 + kNfmRowChunk : rows;
  float acc = 0.f;
  if (l < L) {
    const int din = N.dims[l], dout = N.dims[l + 1];
    if (t < dout * din) {
      const int o = t / din, i = t % din;
      for (int64_t r = r0; r < r1; ++r)
        acc = fmaf(dpre_ws[r * hsum + dp_off[l] + o], nfm_hin(N, act + r * aw, l, r, i, pre_off, scale), acc);
    } else {
      const int o = t - dout * din;
      for (int64_t r = r0; r < r1; ++r) acc += dpre_ws[r * hsum + dp_off[l] + o];
    }
  } else {
    const int dl = N.dims[L];
    const float go = gout[0];
    if (t < dl) {
      for (int64_t r = r0; r < r1; ++r) acc = fmaf(go * dy[r], nfm_hin(N, act + r * aw, L, r, t, pre_off, scale), acc);
    } else {
      for (int64_t r = r0; r < r1; ++r) acc += go * dy[r];
    }
  }
  part[static_cast<int64_t>(blockIdx.y) * w + t] = acc;
}

__global__ __launch_bounds__(256) void nfm_wgrad_reduce_kernel(NfmNet N, int l, const float* __restrict__ part,
                                                               int nchunks, int w, const float* __restrict__ gout,
                                                               float lam, float* __restrict__ dWl,
                                                               float* __restrict__ dbl, float* __restrict__ dW_out,
                                                               float* __restrict__ db_lin) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= w) return;
  float acc = 0.f;
  for (int k = 0; k < nchunks; ++k) acc += part[static_cast<int64_t>(k) * w + t];
  const int L = N.n_layers;
  if (l < L) {
    const int n_w = N.dims[l] * N.dims[l + 1];
    if (t < n_w) dWl[t] = acc;
    else dbl[t - n_w] = acc;
  } else {
    const int dl = N.dims[L];
    if (t < dl) dW_out[t] = acc + gout[0] * lam * N.W_out[t];
    else db_lin[0] = acc;
  }
}

// Feature gradients: entry k (row rk, feature ck, value xk) contributes
//   dV[ck]  += xk * (s_rk - xk V[ck]) * dz_rk        d z / d V through the pooling
//   dw[ck]  += xk * g_rk                               the wide head
// The entries are radix-sorted by feature id (stable: entry order kept within a
// feature), and every run of equal ids is summed in entry order by exactly one
// writer of its feature row -- deterministic, no atomics.  dV / dw are zero-filled.
__global__ __launch_bounds__(256) void nfm_feat_keys_kernel(const int64_t* __restrict__ col, int64_t nnz,
                                                            uint32_t* __restrict__ keys, uint32_t* __restrict__ idx) {
  const int64_t k = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (k >= nnz) return;
  keys[k] = static_cast<uint32_t>(col[k]);
  idx[k] = static_cast<uint32_t>(k);
}

// The sorted entries are cut into chunks of kFeatChunk; one wave per chunk walks
// its runs ("pieces") in order, four entries' rows loaded at a time.  A piece
// that is a whole run writes dV / dw itself; a piece of a run that crosses a
// chunk edge leaves its partial sum in slot 0 (piece at the chunk start) or 1
// (piece at the end) of its chunk, and nfm_feat_join_kernel has the chunk where
// the run starts add those partials in chunk order.
constexpr int kFeatChunk = 16;

__global__ __launch_bounds__(256) void nfm_feat_piece_kernel(
    NfmNet N, const uint32_t* __restrict__ skey, const uint32_t* __restrict__ sidx, const int64_t* __restrict__ erow,
    const float* __restrict__ val, int64_t nnz, const float* __restrict__ act, const float* __restrict__ dz_ws,
    const float* __restrict__ dy, const float* __restrict__ gout, float* __restrict__ dV, int64_t lddv,
    float* __restrict__ dw, float* __restrict__ slots) {
  const int64_t c = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int64_t base = c * kFeatChunk;
  if (base >= nnz) return;
  const int cnt = nnz - base < kFeatChunk ? static_cast<int>(nnz - base) : kFeatChunk;
  const int d = N.dims[0];
  const int64_t aw = act_width(N);
  const float go = gout[0];
  uint32_t key_l = 0;
  int64_t r_l = 0;
  float x_l = 0.f;
  if (lane < cnt) {
    key_l = skey[base + lane];
    const int64_t e = sidx[base + lane];
    r_l = erow[e];
    x_l = val[e];
  }
  const float gy_l = lane < cnt ? go * dy[r_l] : 0.f;
  const bool prev_same = base > 0 && skey[base - 1] == __shfl(key_l, 0);
  const bool next_same = base + cnt < nnz && skey[base + cnt] == __shfl(key_l, cnt - 1);
  const int64_t slot_w = d + 1;
  float g[kNfmCols] = {0.f, 0.f, 0.f, 0.f}, vcur[kNfmCols] = {0.f, 0.f, 0.f, 0.f};
  float gw = 0.f;
  int ps = 0;
  for (int j0 = 0; j0 < cnt; j0 += 4) {
    float sr[4][kNfmCols], dz[4][kNfmCols], vv[4][kNfmCols];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = j0 + u < cnt ? j0 + u : cnt - 1;
      const int64_t r = __shfl(r_l, j);
      const uint32_t k = __shfl(key_l, j);
#pragma unroll
      for (int cc = 0; cc < kNfmCols; ++cc) {
        const int col = lane + 64 * cc;
        const bool in = col < d;
        sr[u][cc] = in ? act[r * aw + col] : 0.f;
        dz[u][cc] = in ? dz_ws[r * d + col] : 0.f;
        vv[u][cc] = in ? N.V[static_cast<int64_t>(k) * N.ldv + col] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = j0 + u;
      if (j >= cnt) break;
      const uint32_t k = __shfl(key_l, j);
      if (j == ps) {
#pragma unroll
        for (int cc = 0; cc < kNfmCols; ++cc) vcur[cc] = vv[u][cc];
      }
      const float x = __shfl(x_l, j);
#pragma unroll
      for (int cc = 0; cc < kNfmCols; ++cc) g[cc] = fmaf(x * (sr[u][cc] - x * vcur[cc]), dz[u][cc], g[cc]);
      gw = fmaf(x, __shfl(gy_l, j), gw);
      const bool last = j == cnt - 1 || __shfl(key_l, j + 1 < cnt ? j + 1 : j) != k;
      if (last) {
        const bool cont_prev = ps == 0 && prev_same;
        const bool cont_next = j == cnt - 1 && next_same;
        float* dst;
        if (!cont_prev && !cont_next) {  // a whole run: this wave owns feature k
          dst = dV + static_cast<int64_t>(k) * lddv;
#pragma unroll
          for (int cc = 0; cc < kNfmCols; ++cc)
            if (lane + 64 * cc < d) dst[lane + 64 * cc] += g[cc];
          if (lane == 0) dw[k] += gw;
        } else {
          dst = slots + (c * 2 + (ps == 0 ? 0 : 1)) * slot_w;
#pragma unroll
          for (int cc = 0; cc < kNfmCols; ++cc)
            if (lane + 64 * cc < d) dst[lane + 64 * cc] = g[cc];
          if (lane == 0) dst[d] = gw;
        }
#pragma unroll
        for (int cc = 0; cc < kNfmCols; ++cc) g[cc] = 0.f;
        gw = 0.f;
        ps = j + 1;
      }
    }
  }
}

__global__ __launch_bounds__(256) void nfm_feat_join_kernel(const uint32_t* __restrict__ skey, int64_t nnz, int d,
                                                            const float* __restrict__ slots, float* __restrict__ dV,
                                                            int64_t lddv, float* __restrict__ dw) {
  const int64_t c = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int64_t base = c * kFeatChunk, cend = base + kFeatChunk;
  if (cend >= nnz) return;
  const uint32_t k = skey[cend - 1];
  if (skey[cend] != k) return;                              // no run crosses this chunk's end
  const bool piece_at_start = skey[base] == k;
  if (piece_at_start && base > 0 && skey[base - 1] == k) return;  // the run started in an earlier chunk
  const int64_t slot_w = d + 1;
  float acc[kNfmCols];
  const float* src = slots + (c * 2 + (piece_at_start ? 0 : 1)) * slot_w;
#pragma unroll
  for (int cc = 0; cc < kNfmCols; ++cc) acc[cc] = lane + 64 * cc < d ? src[lane + 64 * cc] : 0.f;
  float aw = src[d];
  const int64_t nch = (nnz + kFeatChunk - 1) / kFeatChunk;
  bool more = true;
  for (int64_t c2 = c + 1; more; c2 += 8) {  // later chunks: the run's piece sits at their start
    float v[8][kNfmCols], vw[8];              // 8 chunks' loads in flight, added in chunk order
    bool cont[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t cu = c2 + u;
      const bool ok = cu < nch;
      const float* p = slots + (ok ? cu : c2) * 2 * slot_w;
#pragma unroll
      for (int cc = 0; cc < kNfmCols; ++cc) v[u][cc] = lane + 64 * cc < d ? p[lane + 64 * cc] : 0.f;
      vw[u] = p[d];
      const int64_t e2 = (cu + 1) * kFeatChunk;
      cont[u] = ok && e2 < nnz && skey[e2 - 1] == k && skey[e2] == k;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (!more) break;
#pragma unroll
      for (int cc = 0; cc < kNfmCols; ++cc) acc[cc] += v[u][cc];
      aw += vw[u];
      more = cont[u];
    }
  }
#pragma unroll
  for (int cc = 0; cc < kNfmCols; ++cc)
    if (lane + 64 * cc < d) dV[static_cast<int64_t>(k) * lddv + lane + 64 * cc] += acc[cc];
  if (lane == 0) dw[k] += aw;
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
  int dmax = 16;
  for (int l = 0; l <= N.n_layers; ++l) dmax = N.dims[l] > dmax ? N.dims[l] : dmax;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // inference (no dropout, nothing saved) at widths that are multiples of 16 up to 128: the transposed-MLP
  // kernel with every layer's weights in LDS
  bool t_ok = act == nullptr && N.p == 0.f && N.n_layers >= 1 && (N.ldv & 3) == 0 &&
              (reinterpret_cast<uintptr_t>(N.V) & 15) == 0;
  for (int l = 0; l <= N.n_layers && t_ok; ++l) t_ok = N.dims[l] % 16 == 0 && N.dims[l] <= 16 * kgat::kNfmTB;
  if (t_ok) {
    kgat::NfmTPlan tp{};
    int to = 0;
    for (int l = 0; l < N.n_layers; ++l) {
      tp.w_off[l] = to;
      tp.pitch[l] = N.dims[l] + 4;  // rows 4 banks apart for the float4 A-operand reads
      to += N.dims[l + 1] * tp.pitch[l];
      tp.b_off[l] = to;
      to += N.dims[l + 1];
    }
    tp.wout_off = to;
    to += N.dims[N.n_layers];
    tp.total = to;
    const size_t tlds = sizeof(float) * static_cast<size_t>(to);
    if (tlds <= 150 * 1024) {
      const void* fn = reinterpret_cast<const void*>(kgat::nfm_fwd_t_kernel);
      if (tlds > 65536) {
        const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(tlds));
        if (e != hipSuccess) return static_cast<int>(e);
      }
      int per_cu = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 1024, tlds) != hipSuccess || per_cu < 1) per_cu = 1;
      const int64_t tiles = (rows + 15) / 16;
      const int64_t cap = static_cast<int64_t>(per_cu) * kgat::kCUs;
      const int64_t need = (tiles + 15) / 16;
      hipLaunchKernelGGL(kgat::nfm_fwd_t_kernel, dim3(static_cast<unsigned>(need < cap ? need : cap)), dim3(1024), tlds,
                         st, N, tp, rowptr, col, val, rows, y);
      KGAT_LAUNCH_CHECK();
      return KGAT_OK;
    }
  }
  kgat::NfmLds plan{};
  plan.P = ((dmax + 15) & ~15) + 4;  // tile pitch: rows 4 banks apart
  int o = 0;
  for (int l = 0; l < N.n_layers; ++l) {
    plan.w_off[l] = o;
    plan.w_pitch[l] = ((N.dims[l] + 15) & ~15) + 4;
    o += ((N.dims[l + 1] + 15) & ~15) * plan.w_pitch[l];
    plan.b_off[l] = o;
    o += (N.dims[l + 1] + 15) & ~15;
  }
  plan.wlds = o <= 12288;  // <= 48 KB of weights: 2-3 blocks per CU beside the tiles
  plan.tile_off = plan.wlds ? o : 0;
  plan.total = plan.tile_off + 4 * 16 * plan.P;
  const size_t lds = sizeof(float) * static_cast<size_t>(plan.total);
  const int nc = dmax <= 64 ? 4 : dmax <= 128 ? 8 : 16;
  // float4 pooling loads where the feature rows allow them (bit-identical: per column the same sums)
  const bool v4 = (N.dims[0] & 3) == 0 && (N.ldv & 3) == 0 && (reinterpret_cast<uintptr_t>(N.V) & 15) == 0;
  using Fn = void (*)(kgat::NfmNet, kgat::NfmLds, const int64_t*, const int64_t*, const float*, int64_t, float*, float*);
#define KGAT_NFM_FN(NCV, W) (v4 ? kgat::nfm_fwd_kernel<NCV, W, true> : kgat::nfm_fwd_kernel<NCV, W, false>)
  Fn fn = nc == 4    ? (plan.wlds ? KGAT_NFM_FN(4, true) : KGAT_NFM_FN(4, false))
          : nc == 8  ? (plan.wlds ? KGAT_NFM_FN(8, true) : KGAT_NFM_FN(8, false))
                     : (plan.wlds ? KGAT_NFM_FN(16, true) : KGAT_NFM_FN(16, false));
#undef KGAT_NFM_FN
  if (lds > 65536) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    if (e != hipSuccess) return static_cast<int>(e);
  }
  int per_cu = 0;  // persistent grid: as many blocks as fit at once
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(fn), 256, lds) != hipSuccess ||
      per_cu < 1)
    per_cu = 1;
  const int64_t groups = (rows + 63) / 64;
  const int64_t cap = static_cast<int64_t>(per_cu) * kgat::kCUs;
  const dim3 grid(static_cast<unsigned>(groups < cap ? groups : cap));
  hipLaunchKernelGGL(fn, grid, dim3(256), lds, st, N, plan, rowptr, col, val, rows, act, y);
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

static int64_t nfm_wgrad_width(const kgat_nfm* net) {
  int64_t w = net->dims[net->n_layers] + 1;
  for (int l = 0; l < net->n_layers; ++l) {
    const int64_t wl = static_cast<int64_t>(net->dims[l]) * net->dims[l + 1] + net->dims[l + 1];
    if (wl > w) w = wl;
  }
  return w;
}

// workspace: dpre [rows][sum dims[1..L]] | dz [rows][d] | weight-gradient chunk
// partials | run-piece partials [2 per 16 sorted entries][d + 1] | the feature sort: keys/idx in and out (4 nnz uint32) | radix-sort scratch
struct NfmBwdWs {
  int64_t dpre, dz, part, slots, sort, scratch, total;  // offsets in floats
  size_t scratch_bytes;
};

static int nfm_bwd_ws(const kgat_nfm* net, int64_t rows, int64_t nnz, NfmBwdWs* w) {
  int64_t h = 0;
  for (int l = 0; l < net->n_layers; ++l) h += net->dims[l + 1];
  const int64_t chunks = (rows + kgat::kNfmRowChunk - 1) / kgat::kNfmRowChunk;
  w->dpre = 0;
  w->dz = rows * h;
  w->part = w->dz + rows * net->dims[0];
  w->slots = w->part + chunks * nfm_wgrad_width(net);
  w->sort = w->slots + 2 * ((nnz + kgat::kFeatChunk - 1) / kgat::kFeatChunk) * (net->dims[0] + 1);
  w->scratch_bytes = 0;
  if (nnz > 0) {
    const hipError_t e = hipcub::DeviceRadixSort::SortPairs(
        nullptr, w->scratch_bytes, static_cast<const uint32_t*>(nullptr), static_cast<uint32_t*>(nullptr),
        static_cast<const uint32_t*>(nullptr), static_cast<uint32_t*>(nullptr), static_cast<int>(nnz), 0, 32);
    if (e != hipSuccess) return static_cast<int>(e);
  }
  w->scratch = (w->sort + 4 * nnz + 63) & ~static_cast<int64_t>(63);  // 256-byte aligned
  w->total = w->scratch + static_cast<int64_t>((w->scratch_bytes + 3) / 4);
  return KGAT_OK;
}

extern "C" int64_t kgat_nfm_bwd_workspace(const kgat_nfm* net, int64_t rows, int64_t nnz) {
  if (!net || rows < 0 || nnz < 0 || nnz > INT32_MAX) return -1;
  NfmBwdWs w;
  if (nfm_bwd_ws(net, rows, nnz, &w) != KGAT_OK) return -1;
  return w.total;
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
  if (nnz > INT32_MAX || (nnz > 0 && (!erow || !col || !val))) return KGAT_ERR_INVALID;
  NfmBwdWs ws;
  if (int e = nfm_bwd_ws(net, rows, nnz, &ws)) return e;
  if (workspace_floats < ws.total) return KGAT_ERR_WORKSPACE;
  if (rows == 0) return KGAT_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  float* dpre = workspace + ws.dpre;
  float* dz = workspace + ws.dz;
  float* part = workspace + ws.part;
  const int nchunks = static_cast<int>((rows + kgat::kNfmRowChunk - 1) / kgat::kNfmRowChunk);
  hipLaunchKernelGGL(kgat::nfm_bwd_kernel, dim3((rows + 3) / 4), dim3(256), 0, st, N, act, rows, dy, grad_out, dpre, dz);
  KGAT_LAUNCH_CHECK();
  for (int l = 0; l <= N.n_layers; ++l) {  // per layer + the output head: chunk partials, then their ordered sum
    const int w = l < N.n_layers ? N.dims[l] * N.dims[l + 1] + N.dims[l + 1] : N.dims[N.n_layers] + 1;
    float* wl = l < N.n_layers ? dW[l] : nullptr;
    float* bl = l < N.n_layers ? db[l] : nullptr;
    hipLaunchKernelGGL(kgat::nfm_wgrad_kernel, dim3((w + 255) / 256, nchunks), dim3(256), 0, st, N, l, act, rows, dy,
                       grad_out, dpre, w, part);
    KGAT_LAUNCH_CHECK();
    hipLaunchKernelGGL(kgat::nfm_wgrad_reduce_kernel, dim3((w + 255) / 256), dim3(256), 0, st, N, l, part, nchunks, w,
                       grad_out, lam, wl, bl, dW_out, db_lin);
    KGAT_LAUNCH_CHECK();
  }
  if (nnz > 0) {
    uint32_t* keys = reinterpret_cast<uint32_t*>(workspace + ws.sort);
    uint32_t* idx = keys + nnz;
    uint32_t* skey = idx + nnz;
    uint32_t* sidx = skey + nnz;
    hipLaunchKernelGGL(kgat::nfm_feat_keys_kernel, dim3((nnz + 255) / 256), dim3(256), 0, st, col, nnz, keys, idx);
    KGAT_LAUNCH_CHECK();
    size_t bytes = ws.scratch_bytes;
    const hipError_t e = hipcub::DeviceRadixSort::SortPairs(workspace + ws.scratch, bytes, keys, skey, idx, sidx,
                                                            static_cast<int>(nnz), 0, 32, st);
    if (e != hipSuccess) return static_cast<int>(e);
    const int64_t fchunks = (nnz + kgat::kFeatChunk - 1) / kgat::kFeatChunk;
    float* slots = workspace + ws.slots;
    hipLaunchKernelGGL(kgat::nfm_feat_piece_kernel, dim3((fchunks + 3) / 4), dim3(256), 0, st, N, skey, sidx, erow, val,
                       nnz, act, dz, dy, grad_out, dV, ld_dv, dw_lin, slots);
    KGAT_LAUNCH_CHECK();
    hipLaunchKernelGGL(kgat::nfm_feat_join_kernel, dim3((fchunks + 3) / 4), dim3(256), 0, st, skey, nnz, N.dims[0],
                       slots, dV, ld_dv, dw_lin);
    KGAT_LAUNCH_CHECK();
  }
  return KGAT_OK;
}
