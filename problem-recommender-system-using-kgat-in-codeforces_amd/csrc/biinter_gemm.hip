// a2 for the wide layers of C4/C5 (d_in or d_out of 256): the bi-interaction as
// two GEMMs plus fused HIP epilogues (src/model/KGAT/aggregator.py:57-65).
//
// At these widths the layer is MFMA-bound (4*d_in*d_out flop per row against
// 4*(2*d_in + d_out) bytes) and a whole row of both products no longer fits a
// wave's registers, so the contractions run as the hand-written fp32 MFMA GEMM of
// gemm.hip (deterministic k order) and everything around them is fused here:
//   forward:  U = X+S, M = X*S                                   (um_kernel)
//             P1 = U W1^T, P2 = M W2^T                           (gemm_f32)
//             H = normalize(dropout(LReLU(P1+b1) + LReLU(P2+b2))) (epi_fwd_kernel,
//             keeps P+b and the row norm as the backward's state)
//   backward: dA, dB from H, dH, the norm, the signs of P+b       (epi_bwd_kernel)
//             du = dA W1, dm = dB W2                             (gemm_f32, into dXd / dS)
//             dXd = du + dm*S, dS = du + dm*X                    (dxs_kernel, in place)
//             dW = dA^T U, dB^T M; db = column sums              (gemm_f32 split-K slabs)
// Dropout draws are the fused kernels' (one 64-bit hash per node, 16-column
// group of 4 blocks), so both paths drop the same elements.
#include <cstdlib>
#include <utility>

#include "common.hpp"
#include "gemm.hpp"

namespace kgat {

__device__ __forceinline__ bool gemm_keep(uint64_t seed, int64_t node, int col, int dout, uint32_t thr) {
  const int groups = (dout / 16 + 3) / 4;
  const int cb = col >> 4;
  const uint64_t h = mix_hash64(seed, (static_cast<uint64_t>(node) * groups + (cb >> 2)) * 16 + (col & 15));
  return static_cast<uint32_t>((h >> (16 * (cb & 3))) & 0xFFFFu) >= thr;
}

__device__ __forceinline__ uint32_t gemm_threshold(float p) {
  const float t = p * 65536.f + 0.5f;
  return t >= 65536.f ? 65536u : static_cast<uint32_t>(t);
}

// [dW | db] = sum over row chunks of the slabs [nb][dout][d_in + 4], in chunk order, in two
// levels: pass 1 (blockIdx.y = group g of kSlabGroups) sums the slabs of group g's contiguous
// range in order into part[g]; pass 2 sums the groups in order.  (One thread per output
// element walking ~1k slabs left 65 blocks latency-bound: 140 us per call at C4.)
constexpr int kSlabGroups = 16;

__global__ __launch_bounds__(256) void wslab_part_kernel(const float* __restrict__ slabs, int nb, int din, int dout,
                                                         float* __restrict__ part) {
  const int w = din + 4;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= dout * (din + 1)) return;
  const int o = i / (din + 1), k = i % (din + 1);
  const int per = (nb + kSlabGroups - 1) / kSlabGroups;
  const int b0 = blockIdx.y * per, b1 = min(nb, b0 + per);
  const float* p = slabs + o * w + k;
  const int64_t sw = static_cast<int64_t>(dout) * w;
  float acc = 0.f;
  int b = b0;
  for (; b + 4 <= b1; b += 4) {  // four loads in flight, added in order
    const float v0 = p[b * sw], v1 = p[(b + 1) * sw], v2 = p[(b + 2) * sw], v3 = p[(b + 3) * sw];
    acc += v0;
    acc += v1;
    acc += v2;
    acc += v3;
  }
  for (; b < b1; ++b) acc += p[b * sw];
  part[static_cast<int64_t>(blockIdx.y) * dout * (din + 1) + i] = acc;
}

__global__ __launch_bounds__(256) void wslab_reduce_kernel(const float* __restrict__ part, int din, int dout,
                                                           float* __restrict__ dW, float* __restrict__ db) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int tot = dout * (din + 1);
  if (i >= tot) return;
  float acc = 0.f;
  for (int g = 0; g < kSlabGroups; ++g) acc += part[static_cast<int64_t>(g) * tot + i];
  const int o = i / (din + 1), k = i % (din + 1);
  if (k < din) dW[o * din + k] = acc;
  else db[o] = acc;
}

// one wave per row; P1/P2 [n, dout] in, P+b written to P1o/P2o (the backward's sign source; in place
// when they are P1/P2).  rows (nullable): row r is node rows[r] (-1: padding, nothing written) --
// its H row, norm, state rows and dropout draws are that node's, as in the whole-table call.
__global__ __launch_bounds__(256) void epi_fwd_kernel(float* __restrict__ P1, float* __restrict__ P2,
                                                      const float* __restrict__ b1, const float* __restrict__ b2,
                                                      float* __restrict__ H, int64_t ldh, float* __restrict__ norm,
                                                      int64_t n, int dout, float p, uint64_t seed,
                                                      const int32_t* __restrict__ rows = nullptr,
                                                      float* __restrict__ P1o = nullptr,
                                                      float* __restrict__ P2o = nullptr) {
  const int lane = threadIdx.x & 63;
  const int64_t r = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  const int64_t node = rows != nullptr ? static_cast<int64_t>(rows[r]) : r;
  if (node < 0) return;
  if (P1o == nullptr) P1o = P1;
  if (P2o == nullptr) P2o = P2;
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const uint32_t thr = gemm_threshold(p);
  float v[16];
  float sq = 0.f;
  int cnt = 0;
  for (int c = lane; c < dout; c += 64, ++cnt) {
    const float pa = P1[r * dout + c] + b1[c], pb = P2[r * dout + c] + b2[c];
    P1o[node * dout + c] = pa;
    P2o[node * dout + c] = pb;
    float g = lrelu(pa) + lrelu(pb);
    if (p > 0.f) g = gemm_keep(seed, node, c, dout, thr) ? g * scale : 0.f;
    v[cnt] = g;
    sq = fmaf(g, g, sq);
  }
  const float nrm = sqrtf(wave_sum(sq));
  const float inv = 1.f / fmaxf(nrm, kNormEps);
  cnt = 0;
  for (int c = lane; c < dout; c += 64, ++cnt) H[node * ldh + c] = v[cnt] * inv;
  if (lane == 0) norm[node] = nrm >= kNormEps ? nrm : -kNormEps;
}

// one wave per row: dA, dB written over the P+b state
__global__ __launch_bounds__(256) void epi_bwd_kernel(float* __restrict__ P1, float* __restrict__ P2,
                                                      const float* __restrict__ H, int64_t ldh,
                                                      const float* __restrict__ norm, const float* __restrict__ dH,
                                                      int64_t lddh, int64_t n, int dout, float p, uint64_t seed,
                                                      const int32_t* __restrict__ key_rows) {
  const int lane = threadIdx.x & 63;
  const int64_t r = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const uint32_t thr = gemm_threshold(p);
  const int64_t key = key_rows ? static_cast<int64_t>(key_rows[r]) : r;
  float dot = 0.f;
  for (int c = lane; c < dout; c += 64) dot = fmaf(H[r * ldh + c], dH[r * lddh + c], dot);
  dot = wave_sum(dot);
  const float nr = norm[r];
  const bool clamped = nr < 0.f;
  const float inv = clamped ? 1.f / kNormEps : 1.f / nr;
  const float proj = clamped ? 0.f : dot;
  for (int c = lane; c < dout; c += 64) {
    float dg = (dH[r * lddh + c] - H[r * ldh + c] * proj) * inv;
    if (p > 0.f) dg = (key >= 0 && gemm_keep(seed, key, c, dout, thr)) ? dg * scale : 0.f;
    if (key < 0) dg = 0.f;
    const float pa = P1[r * dout + c], pb = P2[r * dout + c];
    P1[r * dout + c] = pa > 0.f ? dg : dg * kLeakySlope;
    P2[r * dout + c] = pb > 0.f ? dg : dg * kLeakySlope;
  }
}

// one wave per output row r of a row list (the hop rows of a layer's backward): node = rows[r]
// (-1: padding, zero gradient); H, dH, the pre-activation state and the norm read at the node's
// own row of the whole-table arrays, dA / dB written compactly at r -- epi_bwd_kernel's arithmetic
// on gathered rows, without the gathers.  bits (nullable): the fused forward's sign/keep words
// instead of the pre-activations (P1 / P2 unused).
__global__ __launch_bounds__(256) void epi_bwd_rows_kernel(float* __restrict__ dA, float* __restrict__ dB,
                                                           const float* __restrict__ P1, const float* __restrict__ P2,
                                                           const uint64_t* __restrict__ mask,
                                                           const float* __restrict__ H, int64_t ldh,
                                                           const float* __restrict__ norm,
                                                           const float* __restrict__ dH, int64_t lddh,
                                                           const int32_t* __restrict__ rows, int64_t m, int dout,
                                                           float p, uint64_t seed) {
  const int lane = threadIdx.x & 63;
  const int64_t r = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (r >= m) return;
  const int64_t node = rows[r];
  if (node < 0) {
    for (int c = lane; c < dout; c += 64) dA[r * dout + c] = dB[r * dout + c] = 0.f;
    return;
  }
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const uint32_t thr = gemm_threshold(p);
  float dot = 0.f;
  for (int c = lane; c < dout; c += 64) dot = fmaf(H[node * ldh + c], dH[node * lddh + c], dot);
  dot = wave_sum(dot);
  const float nr = norm[node];
  const bool clamped = nr < 0.f;
  const float inv = clamped ? 1.f / kNormEps : 1.f / nr;
  const float proj = clamped ? 0.f : dot;
  const int ng = (dout / 16 + 3) / 4;
  const int64_t st = node >> 4;
  const int q = static_cast<int>(node & 15) >> 2, i = static_cast<int>(node & 3);
  for (int c = lane; c < dout; c += 64) {
    float dg = (dH[node * lddh + c] - H[node * ldh + c] * proj) * inv;
    if (mask != nullptr) {
      const int cb = c >> 4;
      const uint64_t w = mask[(st * ng + (cb >> 2)) * 64 + q * 16 + (c & 15)];
      const uint32_t bits = static_cast<uint32_t>(w >> (((cb & 3) * 4 + i) * 3)) & 7u;
      dg = (bits & 4u) ? dg * scale : 0.f;
      dA[r * dout + c] = (bits & 1u) ? dg : dg * kLeakySlope;
      dB[r * dout + c] = (bits & 2u) ? dg : dg * kLeakySlope;
    } else {
      if (p > 0.f) dg = gemm_keep(seed, node, c, dout, thr) ? dg * scale : 0.f;
      const float pa = P1[node * dout + c], pb = P2[node * dout + c];
      dA[r * dout + c] = pa > 0.f ? dg : dg * kLeakySlope;
      dB[r * dout + c] = pb > 0.f ? dg : dg * kLeakySlope;
    }
  }
}

// one wave per row: dA, dB from H, dH and the fused forward's saved state (row
// norm + per-element pre_sum > 0 / pre_mul > 0 / keep bits, kgat_biinter_fwd_f32's
// mask_out layout, indexed by node = key) instead of the pre-activations
__global__ __launch_bounds__(256) void epi_bwd_bits_kernel(float* __restrict__ dA, float* __restrict__ dB,
                                                           const float* __restrict__ H, int64_t ldh,
                                                           const float* __restrict__ norm,
                                                           const uint64_t* __restrict__ mask,
                                                           const float* __restrict__ dH, int64_t lddh, int64_t n,
                                                           int dout, float p, const int32_t* __restrict__ key_rows) {
  const int lane = threadIdx.x & 63;
  const int64_t r = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  const int64_t key = key_rows ? static_cast<int64_t>(key_rows[r]) : r;
  if (key < 0) {  // padding row: zero gradient
    for (int c = lane; c < dout; c += 64) dA[r * dout + c] = dB[r * dout + c] = 0.f;
    return;
  }
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  float dot = 0.f;
  for (int c = lane; c < dout; c += 64) dot = fmaf(H[r * ldh + c], dH[r * lddh + c], dot);
  dot = wave_sum(dot);
  const float nr = norm[key];
  const bool clamped = nr < 0.f;
  const float inv = clamped ? 1.f / kNormEps : 1.f / nr;
  const float proj = clamped ? 0.f : dot;
  const int ng = (dout / 16 + 3) / 4;
  const int64_t st = key >> 4;
  const int q = static_cast<int>(key & 15) >> 2, i = static_cast<int>(key & 3);
  for (int c = lane; c < dout; c += 64) {
    const int cb = c >> 4;
    const uint64_t w = mask[(st * ng + (cb >> 2)) * 64 + q * 16 + (c & 15)];
    const uint32_t bits = static_cast<uint32_t>(w >> (((cb & 3) * 4 + i) * 3)) & 7u;
    float dg = (dH[r * lddh + c] - H[r * ldh + c] * proj) * inv;
    dg = (bits & 4u) ? dg * scale : 0.f;
    dA[r * dout + c] = (bits & 1u) ? dg : dg * kLeakySlope;
    dB[r * dout + c] = (bits & 2u) ? dg : dg * kLeakySlope;
  }
}

// Rows per split-K chunk of the weight-gradient GEMMs.  dW is one or two 128 x 128 output tiles,
// so the chunks are the GEMM's only parallelism: about 1k chunks (>= 4 blocks per CU, so two
// stay resident per CU and hide each other's barriers), 512 .. 65536 rows each, a multiple of
// 256.  A function of n only: the same n always sums in the same order.  (Fixed 65536-row
// chunks left ~150 blocks of 4096 k-steps each at C4: 5 ms per call.)
inline int64_t gemm_chunk(int64_t n) {
  int64_t c = (n + 1023) / 1024;
  c = (c + 255) / 256 * 256;
  return c < 512 ? 512 : (c > 65536 ? 65536 : c);
}
inline int64_t wslab_count(int64_t n) { return (n + gemm_chunk(n) - 1) / gemm_chunk(n); }

#define KGAT_GEMM(call)                \
  do {                                 \
    if (int e_ = (call)) return e_;    \
  } while (0)

// The two products of each direction run in one dual-GEMM launch (gemm.hip's dual_gemm_kernel: the
// (X+S, X*S) operands formed at load, dXd / dS formed in the du / dm epilogue -- no U / M arrays, no
// um / dxs passes).  Every entry point requires row strides that are multiples of 4 floats (the dual
// kernel's float4 operand loads), so there is no separate-launch path.

}  // namespace kgat

namespace kgat {

static int zero_wgrads(float* dW1, float* db1, float* dW2, float* db2, int32_t d_in, int32_t d_out, hipStream_t st) {
  for (auto [ptr, count] : {std::pair<float*, size_t>{dW1, size_t(d_in) * d_out}, {dW2, size_t(d_in) * d_out},
                            {db1, size_t(d_out)}, {db2, size_t(d_out)}})
    if (hipError_t e = hipMemsetAsync(ptr, 0, sizeof(float) * count, st); e != hipSuccess) return static_cast<int>(e);
  return KGAT_OK;
}

// du = dA W1, dm = dB W2 (into dXd / dS), dXd = du + dm*S, dS = du + dm*X, dW1 = dA^T (X+S), dW2 = dB^T (X*S),
// db = colsum dA / dB (split-K over row chunks, slabs summed in chunk order); the slabs live in work.
static int bwd_gemm_tail(const float* X, int64_t ldx, const float* S, int64_t lds, const float* W1, const float* W2,
                         const float* dA, const float* dB, float* dXd, int64_t lddxd, float* dS, int64_t ldds,
                         float* dW1, float* db1, float* dW2, float* db2, int64_t n, int32_t d_in, int32_t d_out,
                         float* work, hipStream_t st, const int32_t* rows = nullptr, int phases = 3) {
  // rows: row r of dA / dB / dXd / dS is row rows[r] of X / S (-1: zero).
  // phases: bit 1 the dXd / dS GEMM, bit 2 the weight gradients (work keeps what the second needs)
  const int ldu = d_in + 4;
  const int64_t nb = wslab_count(n);
  float* slab1 = work;
  float* slab2 = slab1 + nb * d_out * static_cast<int64_t>(ldu);
  float* part = slab2 + nb * d_out * static_cast<int64_t>(ldu);  // [kSlabGroups][d_out][d_in + 1]
  if (phases & 1) {
    // du = dA W1, dm = dB W2, then dXd = du + dm*S, dS = du + dm*X in the epilogue: one launch
    DualGemm g;
    g.dxs = true;
    g.M = n, g.N = d_in, g.K = d_out;
    g.A1 = dA, g.A2 = dB, g.lda1 = g.lda2 = d_out;
    g.B1 = W1, g.B2 = W2, g.ldb1 = g.ldb2 = d_in;
    g.C1 = dXd, g.C2 = dS, g.ldc1 = lddxd, g.ldc2 = ldds;
    g.X = X, g.S = S, g.ldx = ldx, g.lds = lds;
    g.erows = rows;
    KGAT_GEMM(dual_gemm_f32(g, st));
  }
  if (!(phases & 2)) return KGAT_OK;
  // [dW | db] = [dA^T U | colsum dA], split over row chunks (deterministic: chunk slabs summed in
  // order): slab_b[d_out, 0:d_in] = dA_b[chunk, d_out]^T . U_b[chunk, d_in], slab_b[:, d_in] = the
  // chunk's column sums of dA, produced by the same GEMM from its A tiles.  [dW1 | db1], [dW2 | db2]
  // chunk slabs in one launch per batch shape: dA^T (X+S), dB^T (X*S), the operands formed from X and S
  // at load, the column sums from the dA / dB tiles
  const int64_t chunk = gemm_chunk(n);
  const int64_t full = n / chunk, rest = n - full * chunk;
  const int64_t sl_stride = static_cast<int64_t>(ldu) * d_out;
  DualGemm g;
  g.ta = true, g.b_um = true;
  g.M = d_out, g.N = d_in;
  g.lda1 = g.lda2 = d_out, g.ldb1 = ldx, g.ldb2 = lds;
  g.ldc1 = g.ldc2 = ldu, g.ldcs = ldu;
  for (int pt = 0; pt < 2; ++pt) {
    const int64_t nbat = pt == 0 ? full : (rest > 0 ? 1 : 0);
    if (nbat == 0) continue;
    const int64_t r0 = pt == 0 ? 0 : full * chunk;
    g.K = pt == 0 ? chunk : rest, g.batch = nbat;
    g.A1 = dA + r0 * d_out, g.A2 = dB + r0 * d_out, g.sA1 = g.sA2 = chunk * d_out;
    if (rows != nullptr) {  // X / S rows through the list: the chunk offsets move the list
      g.B1 = X, g.B2 = S, g.sB1 = g.sB2 = 0;
      g.brows = rows + r0, g.sBrows = chunk;
    } else {
      g.B1 = X + r0 * ldx, g.B2 = S + r0 * lds, g.sB1 = chunk * ldx, g.sB2 = chunk * lds;
    }
    g.C1 = slab1 + (pt == 0 ? 0 : full) * sl_stride, g.C2 = slab2 + (pt == 0 ? 0 : full) * sl_stride;
    g.sC1 = g.sC2 = sl_stride;
    g.cs1 = g.C1 + d_in, g.cs2 = g.C2 + d_in, g.sCS1 = g.sCS2 = sl_stride;
    KGAT_GEMM(dual_gemm_f32(g, st));
  }
  for (int mat = 0; mat < 2; ++mat) {
    float* sl = mat == 0 ? slab1 : slab2;
    const int eblocks = (d_out * (d_in + 1) + 255) / 256;
    hipLaunchKernelGGL(wslab_part_kernel, dim3(eblocks, kSlabGroups), dim3(256), 0, st, sl, static_cast<int>(nb), d_in,
                       d_out, part);
    KGAT_LAUNCH_CHECK();
    hipLaunchKernelGGL(wslab_reduce_kernel, dim3(eblocks), dim3(256), 0, st, part, d_in, d_out, mat == 0 ? dW1 : dW2,
                       mat == 0 ? db1 : db2);
    KGAT_LAUNCH_CHECK();
  }
  return KGAT_OK;
}

}  // namespace kgat

static bool gemm_dims_ok(int32_t din, int32_t dout) {
  return din >= 16 && dout >= 16 && din % 16 == 0 && dout % 16 == 0 && din <= 1024 && dout <= 1024;
}

extern "C" int64_t kgat_biinter_gemm_state_floats(int64_t n_rows, int32_t d_in, int32_t d_out) {
  if (n_rows < 0 || !gemm_dims_ok(d_in, d_out)) return -1;
  return n_rows * 2 * static_cast<int64_t>(d_out) + n_rows;
}

extern "C" int64_t kgat_biinter_gemm_work_floats(int64_t n_rows, int32_t d_in, int32_t d_out) {
  if (n_rows < 0 || !gemm_dims_ok(d_in, d_out)) return -1;
  // two sets of split-K slabs [chunks][d_out][d_in + 4] + the two-level reduction's group sums
  return 2 * kgat::wslab_count(n_rows) * d_out * static_cast<int64_t>(d_in + 4) +
         kgat::kSlabGroups * static_cast<int64_t>(d_out) * (d_in + 1) + 4;
}

extern "C" int kgat_biinter_fwd_gemm_f32(const float* X, int64_t ldx, const float* S, int64_t lds, const float* W1,
                                         const float* b1, const float* W2, const float* b2, float* H, int64_t ldh,
                                         int64_t n, int32_t d_in, int32_t d_out, float dropout_p, uint64_t seed,
                                         float* state, float* work, int64_t work_floats, void* stream) {
  if (!X || !S || !W1 || !b1 || !W2 || !b2 || !H || !state || n < 0 || !gemm_dims_ok(d_in, d_out))
    return KGAT_ERR_INVALID;
  if (ldx < d_in || lds < d_in || ldh < d_out || (ldx & 3) || (lds & 3) || !(dropout_p >= 0.f && dropout_p < 1.f))
    return KGAT_ERR_INVALID;
  if (n == 0) return KGAT_OK;
  if (!work || work_floats < kgat_biinter_gemm_work_floats(n, d_in, d_out)) return KGAT_ERR_WORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  float* P1 = state;
  float* P2 = state + n * d_out;
  float* norm = state + 2 * n * d_out;
  // P1 = (X+S) W1^T, P2 = (X*S) W2^T in one launch, the operands formed at load
  kgat::DualGemm g;
  g.tb = true, g.a_um = true;
  g.M = n, g.N = d_out, g.K = d_in;
  g.A1 = X, g.A2 = S, g.lda1 = ldx, g.lda2 = lds;
  g.B1 = W1, g.B2 = W2, g.ldb1 = g.ldb2 = d_in;
  g.C1 = P1, g.C2 = P2, g.ldc1 = g.ldc2 = d_out;
  KGAT_GEMM(kgat::dual_gemm_f32(g, st));
  hipLaunchKernelGGL(kgat::epi_fwd_kernel, dim3((n + 3) / 4), dim3(256), 0, st, P1, P2, b1, b2, H, ldh, norm, n, d_out,
                     dropout_p, seed);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int64_t kgat_biinter_gemm_rows_work_floats(int64_t m, int32_t d_in, int32_t d_out) {
  const int64_t w = kgat_biinter_gemm_work_floats(m, d_in, d_out);
  return w < 0 ? -1 : w + 2 * m * static_cast<int64_t>(d_out);  // + the compact P1, P2
}

extern "C" int kgat_biinter_fwd_gemm_rows_f32(const float* X, int64_t ldx, const float* S, int64_t lds,
                                              const int32_t* rows, int64_t m, const float* W1, const float* b1,
                                              const float* W2, const float* b2, float* H, int64_t ldh, int64_t n,
                                              int32_t d_in, int32_t d_out, float dropout_p, uint64_t seed,
                                              float* state, float* work, int64_t work_floats, void* stream) {
  if (!X || !S || !rows || !W1 || !b1 || !W2 || !b2 || !H || !state || n < 0 || m < 0 || !gemm_dims_ok(d_in, d_out))
    return KGAT_ERR_INVALID;
  if (ldx < d_in || lds < d_in || ldh < d_out || (ldx & 3) || (lds & 3) || !(dropout_p >= 0.f && dropout_p < 1.f))
    return KGAT_ERR_INVALID;
  if (m == 0) return KGAT_OK;
  if (!work || work_floats < kgat_biinter_gemm_rows_work_floats(m, d_in, d_out)) return KGAT_ERR_WORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  float* P1 = work + kgat_biinter_gemm_work_floats(m, d_in, d_out);
  float* P2 = P1 + m * d_out;
  // P1 = (X+S) W1^T, P2 = (X*S) W2^T on the listed rows, X / S read through the list at load
  kgat::DualGemm g;
  g.tb = true, g.a_um = true;
  g.M = m, g.N = d_out, g.K = d_in;
  g.A1 = X, g.A2 = S, g.lda1 = ldx, g.lda2 = lds, g.arows = rows;
  g.B1 = W1, g.B2 = W2, g.ldb1 = g.ldb2 = d_in;
  g.C1 = P1, g.C2 = P2, g.ldc1 = g.ldc2 = d_out;
  KGAT_GEMM(kgat::dual_gemm_f32(g, st));
  hipLaunchKernelGGL(kgat::epi_fwd_kernel, dim3((m + 3) / 4), dim3(256), 0, st, P1, P2, b1, b2, H, ldh,
                     state + 2 * n * d_out, m, d_out, dropout_p, seed, rows, state, state + n * d_out);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int kgat_biinter_bwd_gemm_f32(const float* X, int64_t ldx, const float* S, int64_t lds, const float* H,
                                         int64_t ldh, float* state, const float* dH, int64_t lddh, const float* W1,
                                         const float* W2, float* dXd, int64_t lddxd, float* dS, int64_t ldds,
                                         float* dW1, float* db1, float* dW2, float* db2, int64_t n, int32_t d_in,
                                         int32_t d_out, float dropout_p, uint64_t seed, const int32_t* key_rows,
                                         float* work, int64_t work_floats, void* stream) {
  if (!X || !S || !H || !state || !dH || !W1 || !W2 || !dXd || !dS || !dW1 || !db1 || !dW2 || !db2 || n < 0 ||
      !gemm_dims_ok(d_in, d_out))
    return KGAT_ERR_INVALID;
  if (ldx < d_in || lds < d_in || ldh < d_out || lddh < d_out || lddxd < d_in || ldds < d_in || (ldx & 3) ||
      (lds & 3) || !(dropout_p >= 0.f && dropout_p < 1.f))
    return KGAT_ERR_INVALID;
  if (!work || work_floats < kgat_biinter_gemm_work_floats(n, d_in, d_out)) return KGAT_ERR_WORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (n == 0) return kgat::zero_wgrads(dW1, db1, dW2, db2, d_in, d_out, st);
  float* dA = state;
  float* dB = state + n * d_out;
  const float* norm = state + 2 * n * d_out;
  hipLaunchKernelGGL(kgat::epi_bwd_kernel, dim3((n + 3) / 4), dim3(256), 0, st, dA, dB, H, ldh, norm, dH, lddh, n,
                     d_out, dropout_p, seed, key_rows);
  KGAT_LAUNCH_CHECK();
  return kgat::bwd_gemm_tail(X, ldx, S, lds, W1, W2, dA, dB, dXd, lddxd, dS, ldds, dW1, db1, dW2, db2, n, d_in,
                             d_out, work, st);
}

extern "C" int kgat_biinter_bwd_gemm_rows_f32(const float* X, int64_t ldx, const float* S, int64_t lds,
                                              const float* H, int64_t ldh, const float* state, const float* norm,
                                              const uint64_t* mask, const float* dH, int64_t lddh,
                                              const int32_t* rows, int64_t m, const float* W1, const float* W2,
                                              float* dXd, int64_t lddxd, float* dS, int64_t ldds, float* dW1,
                                              float* db1, float* dW2, float* db2, int64_t n, int32_t d_in,
                                              int32_t d_out, float dropout_p, uint64_t seed, float* work,
                                              int64_t work_floats, void* stream) {
  return kgat_biinter_bwd_gemm_rows_ex_f32(X, ldx, S, lds, H, ldh, state, norm, mask, dH, lddh, rows, m, W1, W2, dXd,
                                           lddxd, dS, ldds, dW1, db1, dW2, db2, n, d_in, d_out, dropout_p, seed, work,
                                           work_floats, 3, stream);
}

extern "C" int kgat_biinter_bwd_gemm_rows_ex_f32(const float* X, int64_t ldx, const float* S, int64_t lds,
                                                 const float* H, int64_t ldh, const float* state, const float* norm,
                                                 const uint64_t* mask, const float* dH, int64_t lddh,
                                                 const int32_t* rows, int64_t m, const float* W1, const float* W2,
                                                 float* dXd, int64_t lddxd, float* dS, int64_t ldds, float* dW1,
                                                 float* db1, float* dW2, float* db2, int64_t n, int32_t d_in,
                                                 int32_t d_out, float dropout_p, uint64_t seed, float* work,
                                                 int64_t work_floats, int32_t phases, void* stream) {
  if (phases < 1 || phases > 3) return KGAT_ERR_INVALID;
  // state: the GEMM forward's [P1 + b1 | P2 + b2 | norm] over all n rows (mask null), or null with
  // norm + mask: the fused forward's saved state (the "bits" kind, d_out <= 128)
  if (!X || !S || !H || !dH || !rows || !W1 || !W2 || !dXd || !dS || !dW1 || !db1 || !dW2 || !db2 || n < 0 || m < 0 ||
      !gemm_dims_ok(d_in, d_out))
    return KGAT_ERR_INVALID;
  if ((state == nullptr) == (mask == nullptr) || (mask != nullptr && (norm == nullptr || d_out > 128)))
    return KGAT_ERR_INVALID;
  if (ldx < d_in || lds < d_in || ldh < d_out || lddh < d_out || lddxd < d_in || ldds < d_in || (ldx & 3) ||
      (lds & 3) || !(dropout_p >= 0.f && dropout_p < 1.f))
    return KGAT_ERR_INVALID;
  if (!work || work_floats < kgat_biinter_bwd_gemm_rows_work_floats(m, d_in, d_out)) return KGAT_ERR_WORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (m == 0) return kgat::zero_wgrads(dW1, db1, dW2, db2, d_in, d_out, st);
  float* dA = work + kgat_biinter_gemm_work_floats(m, d_in, d_out);
  float* dB = dA + m * d_out;
  // X / S rows gathered once, compactly: the GEMMs then read contiguous tiles (read through the list
  // inside the GEMMs -- the dXd / dS epilogue and the k-major weight-gradient loads -- they ran 0.5 ms
  // slower at 300k rows than this copy costs); H, dH and the state are read through the list
  float* Xc = dB + m * d_out;
  float* Sc = Xc + m * static_cast<int64_t>(d_in);
  if (phases & 1) {
    if (int e = kgat_gather_rows_f32(X, ldx, rows, m, d_in, Xc, d_in, stream)) return e;
    if (int e = kgat_gather_rows_f32(S, lds, rows, m, d_in, Sc, d_in, stream)) return e;
    const float* P1 = state;
    const float* P2 = state != nullptr ? state + n * d_out : nullptr;
    const float* nrm = state != nullptr ? state + 2 * n * d_out : norm;
    hipLaunchKernelGGL(kgat::epi_bwd_rows_kernel, dim3((m + 3) / 4), dim3(256), 0, st, dA, dB, P1, P2, mask, H, ldh,
                       nrm, dH, lddh, rows, m, d_out, dropout_p, seed);
    KGAT_LAUNCH_CHECK();
  }
  return kgat::bwd_gemm_tail(Xc, d_in, Sc, d_in, W1, W2, dA, dB, dXd, lddxd, dS, ldds, dW1, db1, dW2, db2, m, d_in,
                             d_out, work, st, nullptr, phases);
}

extern "C" int64_t kgat_biinter_bwd_gemm_rows_work_floats(int64_t m, int32_t d_in, int32_t d_out) {
  const int64_t w = kgat_biinter_gemm_bits_work_floats(m, d_in, d_out);
  return w < 0 ? -1 : w + 2 * m * static_cast<int64_t>(d_in);  // + the gathered X, S rows
}

extern "C" int64_t kgat_biinter_gemm_bits_work_floats(int64_t n_rows, int32_t d_in, int32_t d_out) {
  const int64_t w = kgat_biinter_gemm_work_floats(n_rows, d_in, d_out);
  return w < 0 ? -1 : w + 2 * n_rows * static_cast<int64_t>(d_out);  // + dA, dB
}

extern "C" int kgat_biinter_bwd_gemm_bits_f32(const float* X, int64_t ldx, const float* S, int64_t lds, const float* H,
                                              int64_t ldh, const float* norm, const uint64_t* mask, const float* dH,
                                              int64_t lddh, const float* W1, const float* W2, float* dXd,
                                              int64_t lddxd, float* dS, int64_t ldds, float* dW1, float* db1,
                                              float* dW2, float* db2, int64_t n, int32_t d_in, int32_t d_out,
                                              float dropout_p, const int32_t* key_rows, float* work,
                                              int64_t work_floats, void* stream) {
  if (!X || !S || !H || !norm || !mask || !dH || !W1 || !W2 || !dXd || !dS || !dW1 || !db1 || !dW2 || !db2 || n < 0 ||
      !gemm_dims_ok(d_in, d_out) || d_out > 128)
    return KGAT_ERR_INVALID;
  if (ldx < d_in || lds < d_in || ldh < d_out || lddh < d_out || lddxd < d_in || ldds < d_in || (ldx & 3) ||
      (lds & 3) || !(dropout_p >= 0.f && dropout_p < 1.f))
    return KGAT_ERR_INVALID;
  if (!work || work_floats < kgat_biinter_gemm_bits_work_floats(n, d_in, d_out)) return KGAT_ERR_WORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (n == 0) return kgat::zero_wgrads(dW1, db1, dW2, db2, d_in, d_out, st);
  float* dA = work + kgat_biinter_gemm_work_floats(n, d_in, d_out);
  float* dB = dA + n * d_out;
  hipLaunchKernelGGL(kgat::epi_bwd_bits_kernel, dim3((n + 3) / 4), dim3(256), 0, st, dA, dB, H, ldh, norm, mask, dH,
                     lddh, n, d_out, dropout_p, key_rows);
  KGAT_LAUNCH_CHECK();
  return kgat::bwd_gemm_tail(X, ldx, S, lds, W1, W2, dA, dB, dXd, lddxd, dS, ldds, dW1, db1, dW2, db2, n, d_in,
                             d_out, work, st);
}
