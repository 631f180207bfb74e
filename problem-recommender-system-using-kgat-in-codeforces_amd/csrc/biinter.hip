// a2 -- fused bi-interaction aggregator (src/model/KGAT/aggregator.py:57-65):
//   H = normalize(dropout(LReLU(W1 (X+S) + b1) + LReLU(W2 (X*S) + b2)))
// and its backward.  The two d_in x d_out contractions run on the fp32 MFMA
// (v_mfma_f32_16x16x4_f32, exact fp32 fma chains); everything else (bias,
// LeakyReLU, dropout, row L2 norm) is fused into the MFMA epilogue, so X and
// S are read once and H written once.
//
// Operand layout (both kernels): a wave owns a 16-row sub-tile.  For the
// X.W^T products lane l holds row (l & 15) and the contiguous k-range
// [(l>>4)*K/4, (l>>4+1)*K/4) of its row, so A-operand loads are float4 row
// reads and the k-order of the MFMA chain is (q*K/4 + step) -- any order of a
// sum is a valid fp32 schedule.  W is staged once per block in LDS with a
// 4-float pad per row.
#include "common.hpp"
#include "spmm_core.hpp"

namespace kgat {

template <int DIN, int DOUT>
struct BiShape {
  static constexpr int KQ = DIN / 4;     // k values per lane (A operand, K = DIN)
  static constexpr int KO = DOUT / 4;    // k values per lane (A operand, K = DOUT)
  static constexpr int NCB = DOUT / 16;  // 16-wide output column blocks
  static constexpr int NIB = DIN / 16;   // 16-wide input column blocks
  static constexpr int WLD = DIN + 4;    // padded LDS row of W (floats)
  static constexpr int ILD = DIN + 4;    // padded LDS row of an X/S tile
  static constexpr int OLD = DOUT + 4;   // padded LDS row of a dA/dB tile
};

// Load this lane's A-operand slice of a 16-row sub-tile (zeros past n, or
// for a negative source row).
template <int K>
__device__ __forceinline__ void load_rows(const float* __restrict__ P, int64_t ld, int64_t row, int64_t n, int q,
                                          float (&out)[K / 4]) {
  constexpr int KQ = K / 4;
  if (row >= 0 && row < n) {
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

// a1 = U . W1^T, a2 = M . W2^T for ONE 16-wide output column block cb (the
// epilogue of each block runs before the next block's MFMAs, so only one
// block's accumulators are live).  w rows are wld floats apart (LDS copy in the
// forward, LDS or global in the backward).
template <int DIN>
__device__ __forceinline__ void bi_block(const float (&u)[DIN / 4], const float (&m)[DIN / 4], const float* w1s,
                                         const float* w2s, int wld, int q, int c, int cb, floatx4& a1, floatx4& a2) {
  constexpr int KQ = DIN / 4;
  a1 = floatx4{0.f, 0.f, 0.f, 0.f};
  a2 = floatx4{0.f, 0.f, 0.f, 0.f};
  const float* r1 = w1s + (cb * 16 + c) * wld + q * KQ;
  const float* r2 = w2s + (cb * 16 + c) * wld + q * KQ;
#pragma unroll
  for (int t = 0; t < KQ; t += 4) {
    const float4 x1 = *reinterpret_cast<const float4*>(r1 + t);
    const float4 x2 = *reinterpret_cast<const float4*>(r2 + t);
    a1 = mfma16x4(u[t], x1.x, a1);
    a2 = mfma16x4(m[t], x2.x, a2);
    a1 = mfma16x4(u[t + 1], x1.y, a1);
    a2 = mfma16x4(m[t + 1], x2.y, a2);
    a1 = mfma16x4(u[t + 2], x1.z, a1);
    a2 = mfma16x4(m[t + 2], x2.z, a2);
    a1 = mfma16x4(u[t + 3], x1.w, a1);
    a2 = mfma16x4(m[t + 3], x2.w, a2);
  }
}

// Dropout draws of the bi-interaction output.  One 64-bit hash per (node,
// lane column c, group of four 16-wide column blocks) yields four 16-bit
// uniforms, one per column block: element (node, cb*16 + c) is kept iff its
// draw >= round(p * 65536).  Shared by the forward and the recomputing backward.
__device__ __forceinline__ uint32_t bi_drop_threshold(float p) {
  const float t = p * 65536.f + 0.5f;
  return t >= 65536.f ? 65536u : static_cast<uint32_t>(t);
}
template <int DOUT>
__device__ __forceinline__ uint64_t bi_drop_hash(uint64_t seed, int64_t node, int group, int c) {
  constexpr int kGroups = (DOUT / 16 + 3) / 4;
  return mix_hash64(seed, (static_cast<uint64_t>(node) * kGroups + group) * 16 + c);
}
__device__ __forceinline__ bool bi_drop_keep(uint64_t h, int cb, uint32_t thr) {
  return static_cast<uint32_t>((h >> (16 * (cb & 3))) & 0xFFFFu) >= thr;
}

template <int DIN, int DOUT>
__device__ __forceinline__ void stage_weights(float* w1s, float* w2s, const float* __restrict__ W1,
                                              const float* __restrict__ W2) {
  using B = BiShape<DIN, DOUT>;
  for (int i = threadIdx.x; i < DOUT * DIN / 4; i += blockDim.x) {
    const int j = (i * 4) / DIN, k = (i * 4) % DIN;
    *reinterpret_cast<float4*>(w1s + j * B::WLD + k) = reinterpret_cast<const float4*>(W1)[i];
    *reinterpret_cast<float4*>(w2s + j * B::WLD + k) = reinterpret_cast<const float4*>(W2)[i];
  }
}

// The forward epilogue of one 16-row sub-tile st: u = X+S and m = X*S in the
// A-operand layout (lane (q, c): row c, k in [q*KQ, (q+1)*KQ)), W staged in
// LDS.  Writes H, the row norms and the per-lane state word.  Shared by
// the whole-table and the tile-list forward, so both produce the same bits.
// The forward epilogue of one 16-row sub-tile st: u = X+S and m = X*S in the
// A-operand layout (lane (q, c): row c, k in [q*KQ, (q+1)*KQ)), W staged in
// LDS.  Writes H, the row norms and the per-lane state word.  Shared by
// the whole-table and the tile-list forward, so both produce the same bits.
template <int DIN, int DOUT, bool SB = true>
__device__ __forceinline__ void bi_fwd_subtile(const float (&u)[DIN / 4], const float (&m)[DIN / 4], int64_t st,
                                               int lane, const float* w1s, const float* w2s,
                                               const float (&bias1)[DOUT / 16], const float (&bias2)[DOUT / 16],
                                               float p, float scale, uint32_t thr, uint64_t seed,
                                               float* __restrict__ H, int64_t ldh, int64_t n,
                                               float* __restrict__ norm_out, uint64_t* __restrict__ mask_out,
                                               int64_t node0 = 0) {
  using B = BiShape<DIN, DOUT>;
  const int q = lane >> 4, c = lane & 15;
  const int64_t r0 = st * 16;
  float g[B::NCB][4];
  float sq[4] = {0.f, 0.f, 0.f, 0.f};
  constexpr int NG = (B::NCB + 3) / 4;
  uint64_t word[NG];  // saved state, word g: 3 bits per (cb in [4g, 4g+4), i) -- pre_sum > 0, pre_mul > 0, kept
#pragma unroll
  for (int gi = 0; gi < NG; ++gi) word[gi] = 0;
  uint64_t dh_[4][NG];
  if (p > 0.f) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int gi = 0; gi < NG; ++gi) dh_[i][gi] = bi_drop_hash<DOUT>(seed, node0 + r0 + q * 4 + i, gi, c);
  }
#pragma unroll
  for (int cb = 0; cb < B::NCB; ++cb) {
    floatx4 acc1, acc2;
    if (SB) __builtin_amdgcn_sched_barrier(0);  // keep one column block's W reads/accumulators live at a time
    bi_block<DIN>(u, m, w1s, w2s, B::WLD, q, c, cb, acc1, acc2);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float pa = acc1[i] + bias1[cb], pb = acc2[i] + bias2[cb];
      float v = lrelu(pa) + lrelu(pb);
      bool keep = true;
      if (p > 0.f) {
        keep = bi_drop_keep(dh_[i][cb / 4], cb, thr);
        v = keep ? v * scale : 0.f;
      }
      word[cb / 4] |= static_cast<uint64_t>((pa > 0.f) | ((pb > 0.f) << 1) | (keep << 2)) << (((cb & 3) * 4 + i) * 3);
      g[cb][i] = v;
      sq[i] = fmaf(v, v, sq[i]);
    }
  }
  if (mask_out != nullptr) {
#pragma unroll
    for (int gi = 0; gi < NG; ++gi) mask_out[(st * NG + gi) * 64 + lane] = word[gi];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float nrm = sqrtf(sum16(sq[i]));
    const float inv = 1.f / fmaxf(nrm, kNormEps);
    const int64_t row = r0 + q * 4 + i;
    if (row < n) {
      float* h = H + row * ldh + c;
#pragma unroll
      for (int cb = 0; cb < B::NCB; ++cb) __builtin_nontemporal_store(g[cb][i] * inv, h + cb * 16);
      // saved norm; negative = the clamp was active (F.normalize's eps)
      if (norm_out != nullptr && c == 0) norm_out[row] = nrm >= kNormEps ? nrm : -kNormEps;
    }
  }
}

// bi_fwd_subtile for a row list: the lane's rows are those of 4-row quad `quad` (rows 4*quad + i; -1 = none,
// nothing written) and its state word is the one the whole-table launch writes for that quad (there: quad
// st*4 + q), so row-list launches fill the same layout.  The whole-table launch keeps its own copy above (a
// shared form with the quad index arithmetic measured ~10 us slower per C2 launch of it).
template <int DIN, int DOUT>
__device__ __forceinline__ void bi_fwd_quad(const float (&u)[DIN / 4], const float (&m)[DIN / 4], int64_t quad,
                                            int lane, const float* w1s, const float* w2s,
                                            const float (&bias1)[DOUT / 16], const float (&bias2)[DOUT / 16],
                                            float p, float scale, uint32_t thr, uint64_t seed,
                                            float* __restrict__ H, int64_t ldh, int64_t n,
                                            float* __restrict__ norm_out, uint64_t* __restrict__ mask_out,
                                            int64_t node0) {
  using B = BiShape<DIN, DOUT>;
  const int q = lane >> 4, c = lane & 15;
  const int64_t qb = quad * 4;  // first row of this lane's quad
  float g[B::NCB][4];
  float sq[4] = {0.f, 0.f, 0.f, 0.f};
  constexpr int NG = (B::NCB + 3) / 4;
  uint64_t word[NG];  // saved state, word g: 3 bits per (cb in [4g, 4g+4), i) -- pre_sum > 0, pre_mul > 0, kept
#pragma unroll
  for (int gi = 0; gi < NG; ++gi) word[gi] = 0;
  uint64_t dh_[4][NG];
  if (p > 0.f) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int gi = 0; gi < NG; ++gi) dh_[i][gi] = bi_drop_hash<DOUT>(seed, node0 + qb + i, gi, c);
  }
#pragma unroll
  for (int cb = 0; cb < B::NCB; ++cb) {
    floatx4 acc1, acc2;
    __builtin_amdgcn_sched_barrier(0);  // keep one column block's W reads/accumulators live at a time
    bi_block<DIN>(u, m, w1s, w2s, B::WLD, q, c, cb, acc1, acc2);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float pa = acc1[i] + bias1[cb], pb = acc2[i] + bias2[cb];
      float v = lrelu(pa) + lrelu(pb);
      bool keep = true;
      if (p > 0.f) {
        keep = bi_drop_keep(dh_[i][cb / 4], cb, thr);
        v = keep ? v * scale : 0.f;
      }
      word[cb / 4] |= static_cast<uint64_t>((pa > 0.f) | ((pb > 0.f) << 1) | (keep << 2)) << (((cb & 3) * 4 + i) * 3);
      g[cb][i] = v;
      sq[i] = fmaf(v, v, sq[i]);
    }
  }
  if (mask_out != nullptr && quad >= 0) {
#pragma unroll
    for (int gi = 0; gi < NG; ++gi) mask_out[((quad >> 2) * NG + gi) * 64 + (quad & 3) * 16 + c] = word[gi];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float nrm = sqrtf(sum16(sq[i]));
    const float inv = 1.f / fmaxf(nrm, kNormEps);
    const int64_t row = qb + i;
    if (quad >= 0 && row < n) {
      float* h = H + row * ldh + c;
#pragma unroll
      for (int cb = 0; cb < B::NCB; ++cb) __builtin_nontemporal_store(g[cb][i] * inv, h + cb * 16);
      // saved norm; negative = the clamp was active (F.normalize's eps)
      if (norm_out != nullptr && c == 0) norm_out[row] = nrm >= kNormEps ? nrm : -kNormEps;
    }
  }
}

// Waves per block of the standalone forward: 4, or 8 where the two staged W
// copies leave room for one block per CU only (128 -> 128: 135 KB of LDS), so
// that one block still puts two waves on every SIMD.
template <int DIN, int DOUT>
struct BiFwdWaves {
  static constexpr int k = 2 * DOUT * (DIN + 4) * 4 > 80 * 1024 ? 8 : 4;
};

template <int DIN, int DOUT, bool PF, int MINW, int NWV = 4>
__global__ __launch_bounds__(64 * NWV, MINW) void biinter_fwd_kernel(const float* __restrict__ X, int64_t ldx,
                                                          const float* __restrict__ S, int64_t lds,
                                                          const float* __restrict__ W1, const float* __restrict__ b1,
                                                          const float* __restrict__ W2, const float* __restrict__ b2,
                                                          float* __restrict__ H, int64_t ldh, int64_t n, float p,
                                                          uint64_t seed, float* __restrict__ norm_out,
                                                          uint64_t* __restrict__ mask_out, int64_t node0) {
  using B = BiShape<DIN, DOUT>;
  __shared__ __attribute__((aligned(16))) float smem[2 * DOUT * B::WLD];
  float* w1s = smem;
  float* w2s = smem + DOUT * B::WLD;
  stage_weights<DIN, DOUT>(w1s, w2s, W1, W2);
  __syncthreads();

  const int lane = threadIdx.x & 63, q = lane >> 4, c = lane & 15;
  float bias1[B::NCB], bias2[B::NCB];
#pragma unroll
  for (int cb = 0; cb < B::NCB; ++cb) {
    bias1[cb] = b1[cb * 16 + c];
    bias2[cb] = b2[cb * 16 + c];
  }
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const uint32_t thr = bi_drop_threshold(p);
  const int64_t nsub = (n + 15) / 16;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * NWV;
  int64_t k = static_cast<int64_t>(blockIdx.x) * NWV + (threadIdx.x >> 6);
  // PF: the next sub-tile's rows are loaded while the current one computes
  float nx[B::KQ], ns[B::KQ];
  if (PF) {
    load_rows<DIN>(X, ldx, k * 16 + c, n, q, nx);
    load_rows<DIN>(S, lds, k * 16 + c, n, q, ns);
  }
  for (; k < nsub; k += stride) {
    const int64_t st = k;
    if (!PF) {
      load_rows<DIN>(X, ldx, st * 16 + c, n, q, nx);
      load_rows<DIN>(S, lds, st * 16 + c, n, q, ns);
    }
    float u[B::KQ], m[B::KQ];
#pragma unroll
    for (int t = 0; t < B::KQ; ++t) {
      u[t] = nx[t] + ns[t];
      m[t] = nx[t] * ns[t];
    }
    if (PF && k + stride < nsub) {
      load_rows<DIN>(X, ldx, (k + stride) * 16 + c, n, q, nx);
      load_rows<DIN>(S, lds, (k + stride) * 16 + c, n, q, ns);
    }
    bi_fwd_subtile<DIN, DOUT>(u, m, st, lane, w1s, w2s, bias1, bias2, p, scale, thr, seed, H, ldh, n, norm_out,
                              mask_out, node0);
  }
}

// The row-set forward (kgat_biinter_fwd_tiles_f32): the 16-row sub-tiles holding a member of the node set
// row_bits (a hop set's bitmap: a tile's 16 bits are one half-word), with the whole-table launch's per-tile
// arithmetic (bi_fwd_subtile), so the same bits.  A block owns a chunk of 4 * NWV consecutive tiles: every
// wave reads the chunk's half-words (one coalesced load) and ballots them, a chunk with no member returns
// before staging W, and the waves take the member tiles round-robin -- no grid-stride walk of dependent
// bitmap loads over the whole table.
template <int DIN, int DOUT, int NWV>
__global__ __launch_bounds__(64 * NWV, 2) void biinter_fwd_set_kernel(const float* __restrict__ X, int64_t ldx,
                                                                      const float* __restrict__ S, int64_t lds,
                                                                      const float* __restrict__ W1,
                                                                      const float* __restrict__ b1,
                                                                      const float* __restrict__ W2,
                                                                      const float* __restrict__ b2,
                                                                      float* __restrict__ H, int64_t ldh, int64_t n,
                                                                      float p, uint64_t seed,
                                                                      float* __restrict__ norm_out,
                                                                      uint64_t* __restrict__ mask_out,
                                                                      const uint32_t* __restrict__ row_bits) {
  using B = BiShape<DIN, DOUT>;
  constexpr int kTiles = 4 * NWV;  // <= 64: one ballot
  static_assert(kTiles <= 64, "one ballot per chunk");
  __shared__ __attribute__((aligned(16))) float smem[2 * DOUT * B::WLD];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c = lane & 15;
  const int64_t nsub = (n + 15) / 16;
  const int64_t t0 = static_cast<int64_t>(blockIdx.x) * kTiles;
  uint32_t hw = 0;
  if (lane < kTiles && t0 + lane < nsub) hw = (row_bits[(t0 + lane) >> 1] >> (((t0 + lane) & 1) * 16)) & 0xffffu;
  const uint64_t members = __ballot(hw != 0);  // the same in every wave of the block
  if (members == 0) return;                    // block-uniform
  float* w1s = smem;
  float* w2s = smem + DOUT * B::WLD;
  stage_weights<DIN, DOUT>(w1s, w2s, W1, W2);
  __syncthreads();
  const int q = lane >> 4;
  float bias1[B::NCB], bias2[B::NCB];
#pragma unroll
  for (int cb = 0; cb < B::NCB; ++cb) {
    bias1[cb] = b1[cb * 16 + c];
    bias2[cb] = b2[cb * 16 + c];
  }
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const uint32_t thr = bi_drop_threshold(p);
  int k = 0;
  for (uint64_t mm = members; mm != 0; mm &= mm - 1, ++k) {
    if (k % NWV != wave) continue;  // wave-uniform
    const int64_t st = t0 + __ffsll(static_cast<long long>(mm)) - 1;
    float nx[B::KQ], ns[B::KQ], u[B::KQ], m[B::KQ];
    load_rows<DIN>(X, ldx, st * 16 + c, n, q, nx);
    load_rows<DIN>(S, lds, st * 16 + c, n, q, ns);
#pragma unroll
    for (int t = 0; t < B::KQ; ++t) {
      u[t] = nx[t] + ns[t];
      m[t] = nx[t] * ns[t];
    }
    bi_fwd_subtile<DIN, DOUT>(u, m, st, lane, w1s, w2s, bias1, bias2, p, scale, thr, seed, H, ldh, n, norm_out,
                              mask_out, 0);
  }
}

// The row-list forward (kgat_biinter_fwd_list_f32): the rows of a listed node set (rows[0 .. *count), -1 =
// padding; a sorted list, e.g. a hop set, computes each quad once) in 16-row sub-tiles of four 4-row quads --
// the quads of the list, not every 16-row tile holding a member: a 15.6k-row hop set spreads over several
// thousand tiles.  Per quad row the whole-table arithmetic (bi_fwd_quad; the A operand's row c is row c & 3 of
// the sub-tile's quad c >> 2), so the same bits in H, the norms and the state words.  A block takes windows of
// 4 * NWV list entries (<= NWV sub-tiles, one per wave); a quad belongs to the window of its first entry.
template <int DIN, int DOUT, int NWV>
__global__ __launch_bounds__(64 * NWV, 2) void biinter_fwd_list_kernel(const float* __restrict__ X, int64_t ldx,
                                                                       const float* __restrict__ S, int64_t lds,
                                                                       const float* __restrict__ W1,
                                                                       const float* __restrict__ b1,
                                                                       const float* __restrict__ W2,
                                                                       const float* __restrict__ b2,
                                                                       float* __restrict__ H, int64_t ldh, int64_t n,
                                                                       float p, uint64_t seed,
                                                                       float* __restrict__ norm_out,
                                                                       uint64_t* __restrict__ mask_out,
                                                                       const int32_t* __restrict__ rows,
                                                                       const int32_t* __restrict__ count,
                                                                       int64_t cap) {
  using B = BiShape<DIN, DOUT>;
  constexpr int kWin = 4 * NWV;  // list entries per window: at most kWin quads, NWV sub-tiles
  static_assert(kWin <= 64, "one wave builds a window");
  __shared__ __attribute__((aligned(16))) float smem[2 * DOUT * B::WLD];
  __shared__ int32_t s_quad[kWin];
  __shared__ int32_t s_nq;
  const int64_t c0 = *count;
  const int64_t cnt = c0 < 0 ? 0 : (c0 > cap ? cap : c0);  // never past the list
  const int64_t n_win = (cnt + kWin - 1) / kWin;
  if (static_cast<int64_t>(blockIdx.x) >= n_win) return;  // block-uniform
  float* w1s = smem;
  float* w2s = smem + DOUT * B::WLD;
  stage_weights<DIN, DOUT>(w1s, w2s, W1, W2);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, q = lane >> 4, c = lane & 15;
  float bias1[B::NCB], bias2[B::NCB];
#pragma unroll
  for (int cb = 0; cb < B::NCB; ++cb) {
    bias1[cb] = b1[cb * 16 + c];
    bias2[cb] = b2[cb * 16 + c];
  }
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const uint32_t thr = bi_drop_threshold(p);
  auto quad_of = [&](int64_t pos) -> int32_t {
    const int32_t r = pos >= 0 && pos < cnt ? rows[pos] : -1;
    return r >= 0 && r < n ? (r >> 2) : -1;
  };
  for (int64_t win = blockIdx.x; win < n_win; win += gridDim.x) {
    const int64_t pos0 = win * kWin;
    if (wave == 0) {
      const int32_t Q = lane < kWin ? quad_of(pos0 + lane) : -1;
      int32_t prev = __shfl_up(Q, 1);
      if (lane == 0) prev = quad_of(pos0 - 1);
      const bool head = Q >= 0 && Q != prev;
      const uint64_t hm = __ballot(head);
      if (head) s_quad[__popcll(hm & ((uint64_t{1} << lane) - 1))] = Q;
      if (lane == 0) s_nq = __popcll(hm);
    }
    __syncthreads();  // (the first round: W staged too)
    const int nq = s_nq;
    if (4 * wave < nq) {  // wave-uniform
      int32_t qd[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) qd[j] = 4 * wave + j < nq ? s_quad[4 * wave + j] : -1;
      const int32_t qa = (c >> 2) == 0 ? qd[0] : (c >> 2) == 1 ? qd[1] : (c >> 2) == 2 ? qd[2] : qd[3];
      const int32_t qc = q == 0 ? qd[0] : q == 1 ? qd[1] : q == 2 ? qd[2] : qd[3];
      const int64_t arow = qa >= 0 ? static_cast<int64_t>(qa) * 4 + (c & 3) : -1;
      float nx[B::KQ], ns[B::KQ], u[B::KQ], m[B::KQ];
      load_rows<DIN>(X, ldx, arow, n, q, nx);
      load_rows<DIN>(S, lds, arow, n, q, ns);
#pragma unroll
      for (int t = 0; t < B::KQ; ++t) {
        u[t] = nx[t] + ns[t];
        m[t] = nx[t] * ns[t];
      }
      bi_fwd_quad<DIN, DOUT>(u, m, qc, lane, w1s, w2s, bias1, bias2, p, scale, thr, seed, H, ldh, n, norm_out,
                             mask_out, 0);
    }
    __syncthreads();  // the window's quads are read before the next window writes them
  }
}

// Backward.  Phase A (per wave, own 16 rows): recompute the forward, push dH
// through normalize / dropout / LeakyReLU to dA = dL/d(pre_sum) and
// dB = dL/d(pre_mul); du = dA.W1, dm = dB.W2 on MFMA; write
//   dXd = du + dm * S      dS = du + dm * X.
// Phase B (block, 64 rows): dW1 += dA^T (X+S), dW2 += dB^T (X*S) with K = rows
// on MFMA, accumulated in registers across the grid-stride loop and written
// as one slab per block; db1/db2 are column sums of dA/dB.  A second kernel
// sums the slabs in block order (deterministic).
// W1/W2 are read through L1/L2 in the backward (16-64 KB, every wave re-reads
// them), so the LDS holds only the 64-row X/S/dA/dB tiles.
template <int DIN, int DOUT, bool WLDS>
struct BwdLds {
  using B = BiShape<DIN, DOUT>;
  static constexpr int kX = 64 * B::ILD;
  static constexpr int kO = 64 * B::OLD;
  static constexpr int kTiles = 2 * kX + 2 * kO;  // floats
  static constexpr int kW = 2 * DOUT * B::WLD;
  // stage W in LDS too (when asked and everything fits the 160 KiB of one CU)
  static constexpr bool kWInLds = WLDS && (kTiles + kW) * 4 <= 160 * 1024;
  static constexpr int kTotal = kTiles + (kWInLds ? kW : 0);
};

// One wave's 16-row slice of a tile, loaded one tile ahead (software pipelining:
// the next tile's HBM reads are in flight while the current tile computes).
template <int DIN, int DOUT>
struct BwdRegs {
  float xs[DIN / 4], ss[DIN / 4];
  float dh[DOUT / 16][4];
};

template <int DIN, int DOUT>
__device__ __forceinline__ void load_bwd_tile(BwdRegs<DIN, DOUT>& R, int64_t r0, int64_t n,
                                              const int32_t* __restrict__ rows, int64_t n_src,
                                              const float* __restrict__ X, int64_t ldx, const float* __restrict__ S,
                                              int64_t lds, const float* __restrict__ dH, int64_t lddh, int q,
                                              int c) {
  int64_t src = r0 + c < n ? r0 + c : -1;
  if (rows != nullptr && src >= 0) src = rows[src];
  load_rows<DIN>(X, ldx, src, n_src, q, R.xs);
  load_rows<DIN>(S, lds, src, n_src, q, R.ss);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t row = r0 + q * 4 + i;
#pragma unroll
    for (int cb = 0; cb < DOUT / 16; ++cb) R.dh[cb][i] = row < n ? dH[row * lddh + cb * 16 + c] : 0.f;
  }
}

template <int DIN, int DOUT, bool WLDS>
__global__ __launch_bounds__(256, 2) void biinter_bwd_kernel(
    const float* __restrict__ X, int64_t ldx, const float* __restrict__ S, int64_t lds,
    const float* __restrict__ dH, int64_t lddh, const float* __restrict__ W1, const float* __restrict__ b1,
    const float* __restrict__ W2, const float* __restrict__ b2, float* __restrict__ dXd, int64_t lddxd,
    float* __restrict__ dS, int64_t ldds, float* __restrict__ slab, int64_t n, float p, uint64_t seed,
    const int32_t* __restrict__ rows, int64_t n_src) {
  using B = BiShape<DIN, DOUT>;
  using Lds = BwdLds<DIN, DOUT, WLDS>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* tx = smem;             // [64][ILD] X tile
  float* ts = tx + Lds::kX;     // [64][ILD] S tile
  float* tda = ts + Lds::kX;    // [64][OLD] dA tile
  float* tdb = tda + Lds::kO;   // [64][OLD] dB tile
  const float* w1p = W1;
  const float* w2p = W2;
  int wld = DIN;
  if constexpr (Lds::kWInLds) {
    float* w1s = smem + Lds::kTiles;
    float* w2s = w1s + DOUT * B::WLD;
    stage_weights<DIN, DOUT>(w1s, w2s, W1, W2);
    __syncthreads();
    w1p = w1s;
    w2p = w2s;
    wld = B::WLD;
  }

  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63, q = lane >> 4, c = lane & 15;
  float bias1[B::NCB], bias2[B::NCB];
#pragma unroll
  for (int cb = 0; cb < B::NCB; ++cb) {
    bias1[cb] = b1[cb * 16 + c];
    bias2[cb] = b2[cb * 16 + c];
  }
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const uint32_t thr = bi_drop_threshold(p);

  // phase-B ownership: output 16x16 blocks of [dW1 | dW2], block id
  // ob = o-block, ib = i-block, mat; wave w takes ids w, w+4, ...
  constexpr int kBlocks = 2 * B::NCB * B::NIB;
  constexpr int kMine = (kBlocks + 3) / 4;
  floatx4 dw[kMine];
#pragma unroll
  for (int k = 0; k < kMine; ++k) dw[k] = floatx4{0.f, 0.f, 0.f, 0.f};
  float dbias = 0.f, dbias2 = 0.f;  // column sums owned by waves 0 (dA) / 1 (dB)

  const int64_t ntile = (n + 63) / 64;
  BwdRegs<DIN, DOUT> nxt;
  if (static_cast<int64_t>(blockIdx.x) < ntile)
    load_bwd_tile<DIN, DOUT>(nxt, static_cast<int64_t>(blockIdx.x) * 64 + wave * 16, n, rows, n_src, X, ldx, S, lds,
                             dH, lddh, q, c);
  for (int64_t tile = blockIdx.x; tile < ntile; tile += gridDim.x) {
    const int64_t r0 = tile * 64 + wave * 16;
    // ---------------- phase A
    // compact row i reads source row rows[i] (frontier mode) or i
    float xs[B::KQ], ss[B::KQ], u[B::KQ], m[B::KQ], dh[B::NCB][4];
#pragma unroll
    for (int t = 0; t < B::KQ; ++t) {
      xs[t] = nxt.xs[t];
      ss[t] = nxt.ss[t];
    }
#pragma unroll
    for (int cb = 0; cb < B::NCB; ++cb)
#pragma unroll
      for (int i = 0; i < 4; ++i) dh[cb][i] = nxt.dh[cb][i];
    if (tile + gridDim.x < ntile)
      load_bwd_tile<DIN, DOUT>(nxt, (tile + gridDim.x) * 64 + wave * 16, n, rows, n_src, X, ldx, S, lds, dH, lddh,
                               q, c);
    {
      float* px = tx + (wave * 16 + c) * B::ILD + q * B::KQ;
      float* ps = ts + (wave * 16 + c) * B::ILD + q * B::KQ;
#pragma unroll
      for (int t = 0; t < B::KQ; t += 4) {
        *reinterpret_cast<float4*>(px + t) = make_float4(xs[t], xs[t + 1], xs[t + 2], xs[t + 3]);
        *reinterpret_cast<float4*>(ps + t) = make_float4(ss[t], ss[t + 1], ss[t + 2], ss[t + 3]);
      }
    }
#pragma unroll
    for (int t = 0; t < B::KQ; ++t) {
      u[t] = xs[t] + ss[t];
      m[t] = xs[t] * ss[t];
    }
    float gd[B::NCB][4];
    uint64_t pos_a = 0, pos_b = 0;  // bit (cb*4+i): pre-activation > 0 (LeakyReLU slope select)
    float sq[4] = {0.f, 0.f, 0.f, 0.f}, dt[4] = {0.f, 0.f, 0.f, 0.f};
    // node id of each C-layout row: the dropout mask is keyed by the node, as in the forward
    int64_t node[4];
    constexpr int NG = (B::NCB + 3) / 4;
    uint64_t hsh[4][NG];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t row = r0 + q * 4 + i;
      node[i] = (rows != nullptr && row < n) ? static_cast<int64_t>(rows[row]) : row;
      if (p > 0.f) {
#pragma unroll
        for (int gi = 0; gi < NG; ++gi) hsh[i][gi] = bi_drop_hash<DOUT>(seed, node[i], gi, c);
      }
    }
#pragma unroll
    for (int cb = 0; cb < B::NCB; ++cb) {
      floatx4 a1, a2;
      __builtin_amdgcn_sched_barrier(0);
      bi_block<DIN>(u, m, w1p, w2p, wld, q, c, cb, a1, a2);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float pa = a1[i] + bias1[cb], pb = a2[i] + bias2[cb];
        pos_a |= static_cast<uint64_t>(pa > 0.f) << (cb * 4 + i);
        pos_b |= static_cast<uint64_t>(pb > 0.f) << (cb * 4 + i);
        float v = lrelu(pa) + lrelu(pb);
        if (p > 0.f) v = bi_drop_keep(hsh[i][cb / 4], cb, thr) ? v * scale : 0.f;
        gd[cb][i] = v;
        sq[i] = fmaf(v, v, sq[i]);
        dt[i] = fmaf(v, dh[cb][i], dt[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float nrm = sqrtf(sum16(sq[i]));
      const float dot = sum16(dt[i]);
      const bool pass = nrm >= kNormEps;
      const float inv = pass ? 1.f / nrm : 1.f / kNormEps;
      const float coef = pass ? dot / (nrm * nrm) : 0.f;
#pragma unroll
      for (int cb = 0; cb < B::NCB; ++cb) {
        // d(g/den): dh/den - g (dh.g)/den^3 while the clamp is inactive
        float dg = (dh[cb][i] - gd[cb][i] * coef) * inv;
        if (p > 0.f) dg = bi_drop_keep(hsh[i][cb / 4], cb, thr) ? dg * scale : 0.f;
        const float da = dg * (((pos_a >> (cb * 4 + i)) & 1) ? 1.f : kLeakySlope);
        const float db = dg * (((pos_b >> (cb * 4 + i)) & 1) ? 1.f : kLeakySlope);
        tda[(wave * 16 + q * 4 + i) * B::OLD + cb * 16 + c] = da;
        tdb[(wave * 16 + q * 4 + i) * B::OLD + cb * 16 + c] = db;
      }
    }
    __syncthreads();

    // du = dA . W1, dm = dB . W2 over K = DOUT (k = q*KO + step)
    {
      float dar[B::KO], dbr[B::KO];
      const float* pa = tda + (wave * 16 + c) * B::OLD + q * B::KO;
      const float* pb = tdb + (wave * 16 + c) * B::OLD + q * B::KO;
#pragma unroll
      for (int t = 0; t < B::KO; t += 4) {
        const float4 va = *reinterpret_cast<const float4*>(pa + t);
        const float4 vb = *reinterpret_cast<const float4*>(pb + t);
        dar[t] = va.x; dar[t + 1] = va.y; dar[t + 2] = va.z; dar[t + 3] = va.w;
        dbr[t] = vb.x; dbr[t + 1] = vb.y; dbr[t + 2] = vb.z; dbr[t + 3] = vb.w;
      }
#pragma unroll 1
      for (int ib = 0; ib < B::NIB; ++ib) {
        __builtin_amdgcn_sched_barrier(0);
        floatx4 du = {0.f, 0.f, 0.f, 0.f}, dm = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < B::KO; ++t) {
          const int k = q * B::KO + t;
          du = mfma16x4(dar[t], w1p[k * wld + ib * 16 + c], du);
          dm = mfma16x4(dbr[t], w2p[k * wld + ib * 16 + c], dm);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int lr = wave * 16 + q * 4 + i;
          const int64_t row = r0 + q * 4 + i;
          const float xv = tx[lr * B::ILD + ib * 16 + c];
          const float sv = ts[lr * B::ILD + ib * 16 + c];
          if (row < n) {
            dXd[row * lddxd + ib * 16 + c] = fmaf(dm[i], sv, du[i]);
            dS[row * ldds + ib * 16 + c] = fmaf(dm[i], xv, du[i]);
          }
        }
      }
    }

    // ---------------- phase B: weight gradients over the 64-row tile
#pragma unroll
    for (int k = 0; k < kMine; ++k) {
      const int id = wave + 4 * k;
      __builtin_amdgcn_sched_barrier(0);
      if (id < kBlocks) {
        const int mat = id / (B::NCB * B::NIB);
        const int rem = id % (B::NCB * B::NIB);
        const int ob = rem / B::NIB, ib = rem % B::NIB;
        const float* tg = mat == 0 ? tda : tdb;
        floatx4 acc = dw[k];
#pragma unroll 4
        for (int s = 0; s < 16; ++s) {
          const int r = 4 * s + q;  // K slot (l>>4) of step s
          const float a = tg[r * B::OLD + ob * 16 + c];
          const float xv = tx[r * B::ILD + ib * 16 + c];
          const float sv = ts[r * B::ILD + ib * 16 + c];
          acc = mfma16x4(a, mat == 0 ? xv + sv : xv * sv, acc);
        }
        dw[k] = acc;
      }
    }
    if (wave < 2) {
      const float* tg = wave == 0 ? tda : tdb;
      for (int j = lane; j < DOUT; j += 64) {
        float s = 0.f;
        for (int r = 0; r < 64; ++r) s += tg[r * B::OLD + j];
        if (j == lane) dbias += s; else dbias2 += s;
      }
    }
    __syncthreads();
  }

  // ---------------- slab write: [dW1 | dW2 | db1 | db2] per block
  constexpr int kSlab = 2 * DOUT * DIN + 2 * DOUT;
  float* out = slab + static_cast<int64_t>(blockIdx.x) * kSlab;
#pragma unroll
  for (int k = 0; k < kMine; ++k) {
    const int id = wave + 4 * k;
    if (id < kBlocks) {
      const int mat = id / (B::NCB * B::NIB);
      const int rem = id % (B::NCB * B::NIB);
      const int ob = rem / B::NIB, ib = rem % B::NIB;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        out[mat * DOUT * DIN + (ob * 16 + q * 4 + i) * DIN + ib * 16 + c] = dw[k][i];
    }
  }
  if (wave < 2) {
    float* ob = out + 2 * DOUT * DIN + wave * DOUT;
    if (lane < DOUT) ob[lane] = dbias;
    if (lane + 64 < DOUT) ob[lane + 64] = dbias2;
  }
}

// Backward from the forward's saved state (norm + per-lane mask words).
// Nothing of the forward is recomputed: with h = H (the saved output) and
// n = the saved norm,
//   dG = keep * scale * (dH - h (h . dH)) / n       (dH / eps when clamped)
//   dA = dG * LReLU'(pre_sum), dB = dG * LReLU'(pre_mul)   (from the sign bits)
//   du = dA . W1, dm = dB . W2  ->  dXd = du + dm*S, dS = du + dm*X
//   dW1 += dA^T (X+S), dW2 += dB^T (X*S), db1/db2 += column sums.
// Every operand is kept in the MFMA C-layout (lane (c, q), element i = row
// q*4+i, column blk*16+c).  That layout IS the A/B operand layout of the
// K = rows product (step s takes element s), so the weight gradients are
// accumulated straight from registers; only dA/dB take an LDS transpose for
// the K = DOUT product.  Each wave works alone (no block barrier in the loop)
// and keeps all 2*DIN*DOUT weight-gradient accumulators in registers (<= 128
// per lane, one wave per SIMD).  The next sub-tile's rows (X, S, H, dH, norms,
// mask words) stream into a per-wave LDS image by LDS-DMA (global_load_lds)
// while the current one computes: no prefetch registers, no per-element
// address arithmetic.  The DMA image is lane-linear, so the row chunks are
// XOR-swizzled on the SOURCE address (chunk ^ 4*((row>>2)&3)), which makes
// the C-layout ds_read_b32 of 4 rows x 16 columns bank-conflict-free.
template <int DIN, int DOUT>
struct SavedBwd {
  using B = BiShape<DIN, DOUT>;
  // W row pitch in LDS chosen so the 4 lane groups (k = q*KO + t) hit 4
  // different 16-bank groups
  static constexpr int wpitch() {
    for (int pad = 0; pad < 64; ++pad)
      if ((B::KO * (DIN + pad)) % 64 == 16) return DIN + pad;
    return DIN + 1;
  }
  static constexpr int WLDB = wpitch();
  static constexpr int OLD = DOUT + 4;
  // per-wave LDS (floats): DMA image [X | S | H | dH | norm(64) | mask(16x16 u64)], dA/dB transpose
  static constexpr int kX = 16 * DIN, kH = 16 * DOUT;
  static constexpr int kNorm = 2 * kX + 2 * kH;
  static constexpr int kMask = kNorm + 64;
  static constexpr int kImg = kMask + 512;
  static constexpr int kT = 2 * 16 * OLD;
  static constexpr int kWave = kImg + kT;
  static constexpr int kTotal = 2 * DOUT * WLDB + 4 * kWave;
  static constexpr bool kOk = DOUT <= 64 && 2 * DIN * DOUT <= 128 * 64 && kTotal * 4 <= 160 * 1024;
};

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;

__device__ __forceinline__ void dma16(const void* src, float* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)lds_wave_base, 16, 0, 0);
}
__device__ __forceinline__ void dma4(const void* src, float* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)lds_wave_base, 4, 0, 0);
}

// chunk swizzle of a D-float row (D/4 16-byte chunks)
template <int D>
__device__ __forceinline__ int chunk_swz(int row) {
  return ((((row >> 2) & 3) << 2)) & (D / 4 - 1);
}

// DMA 16 rows of a row-major [*, D] array into img[16][D] (swizzled chunks).
// node_of(row) gives the source row (negative = none: row 0 is read and the
// consumer zeroes it).
template <int D, typename NodeOf>
__device__ __forceinline__ void dma_rows(float* img, const float* __restrict__ base, int64_t ld, int lane,
                                         NodeOf node_of) {
  constexpr int CH = D / 4;     // chunks per row
  constexpr int RPI = 64 / CH;  // rows per wave instruction
#pragma unroll
  for (int k = 0; k < 16 / RPI; ++k) {
    const int row = k * RPI + lane / CH;
    const int pos = lane % CH;
    const int64_t node = node_of(row);
    const int64_t src = (node >= 0 ? node : 0) * ld + ((pos ^ chunk_swz<D>(row)) << 2);
    dma16(base + src, img + k * RPI * D);
  }
}

// element (row, col) of a swizzled image
template <int D>
__device__ __forceinline__ float img_at(const float* img, int row, int col) {
  return img[row * D + ((((col >> 2) ^ chunk_swz<D>(row))) << 2) + (col & 3)];
}

template <int DIN, int DOUT, bool FRONTIER>
__global__ __launch_bounds__(256, 1) void biinter_bwd_saved_kernel(
    const float* __restrict__ X, int64_t ldx, const float* __restrict__ S, int64_t lds, const float* __restrict__ H,
    int64_t ldh, const float* __restrict__ norm, const uint64_t* __restrict__ mask, const float* __restrict__ dH,
    int64_t lddh, const float* __restrict__ W1, const float* __restrict__ W2, float* __restrict__ dXd,
    int64_t lddxd, float* __restrict__ dS, int64_t ldds, float* __restrict__ slab, int64_t n, float p,
    const int32_t* __restrict__ rows, int64_t n_src, const int32_t* __restrict__ n_dev, int dh_by_node,
    const float* __restrict__ G, int64_t ldg, const int32_t* __restrict__ gidx, int32_t* __restrict__ gmap) {
  using B = BiShape<DIN, DOUT>;
  using F = SavedBwd<DIN, DOUT>;
  // hop mode: the row count is produced on the device (kgat_hop_compact); n is its bound
  if (n_dev != nullptr) {
    const int64_t nd = *n_dev;
    n = nd < n ? nd : n;
  }
  constexpr int NCB = B::NCB, NIB = B::NIB, KO = B::KO;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* w1s = smem;
  float* w2s = smem + DOUT * F::WLDB;
  for (int i = threadIdx.x; i < DOUT * DIN; i += blockDim.x) {
    const int j = i / DIN, k = i % DIN;
    w1s[j * F::WLDB + k] = W1[i];
    w2s[j * F::WLDB + k] = W2[i];
  }
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // scalar: DMA bases live in SGPRs
  const int lane = threadIdx.x & 63, q = lane >> 4, c = lane & 15;
  float* img = smem + 2 * DOUT * F::WLDB + wave * F::kWave;
  float* ix = img;
  float* is = img + F::kX;
  float* ih = img + 2 * F::kX;
  float* ig = img + 2 * F::kX + F::kH;
  float* inorm = img + F::kNorm;
  const uint64_t* imask = reinterpret_cast<const uint64_t*>(img + F::kMask);
  float* tda = img + F::kImg;
  float* tdb = tda + 16 * F::OLD;
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;

  floatx4 dw1[NCB][NIB], dw2[NCB][NIB];
#pragma unroll
  for (int ob = 0; ob < NCB; ++ob)
#pragma unroll
    for (int ib = 0; ib < NIB; ++ib) {
      dw1[ob][ib] = floatx4{0.f, 0.f, 0.f, 0.f};
      dw2[ob][ib] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
  float gb1[NCB], gb2[NCB];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) gb1[cb] = gb2[cb] = 0.f;

  const int64_t nsub = (n + 15) / 16;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 4;
  int64_t st = static_cast<int64_t>(blockIdx.x) * 4 + wave;

  // frontier mode with G: the G row of each of this lane's 4 rows (gidx, by row position: -1 = none), loaded
  // with the sub-tile's DMA; the G rows themselves are loaded once it has landed, under the tile's math
  int32_t gnext[4] = {-1, -1, -1, -1};
  int32_t ndnext = -1;  // frontier mode: the node of row (lane & 15) of the sub-tile in flight
  // issue the DMA of sub-tile t into this wave's image
  auto issue = [&](int64_t t) {
    const int64_t r0 = t * 16;
    if constexpr (FRONTIER) {
      if (gidx != nullptr) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int64_t cr = r0 + q * 4 + i;
          gnext[i] = cr < n ? gidx[cr] : -1;
        }
      }
    }
    const int64_t lim = n - r0;  // rows of this sub-tile that exist
    int32_t nd = -1;             // frontier mode: node of row (lane & 15)
    if constexpr (FRONTIER) {
      const int64_t r = r0 + (lane & 15);
      nd = r < n ? rows[r] : -1;
      if (nd >= n_src) nd = -1;
      ndnext = nd;
    }
    auto node_of = [&](int row) -> int64_t {
      if constexpr (FRONTIER) return __shfl(nd, row);
      return row < lim ? r0 + row : -1;
    };
    auto crow_of = [&](int row) -> int64_t { return row < lim ? r0 + row : -1; };
    auto dh_of = [&](int row) -> int64_t { return dh_by_node ? node_of(row) : crow_of(row); };
    dma_rows<DIN>(ix, X, ldx, lane, node_of);
    dma_rows<DIN>(is, S, lds, lane, node_of);
    dma_rows<DOUT>(ih, H, ldh, lane, node_of);
    dma_rows<DOUT>(ig, dH, lddh, lane, dh_of);
    {
      const int64_t nn = node_of(lane & 15);
      dma4(norm + (nn >= 0 ? nn : 0), inorm);
    }
    // mask image [row][c] (u64): the forward's lane (c, (node>>2)&3) of sub-tile node>>4
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int row = k * 8 + (lane >> 3);
      const int64_t nn = node_of(row);
      const int64_t w = nn >= 0 ? (nn >> 4) * 64 + ((nn >> 2) & 3) * 16 + (lane & 7) * 2 : 0;
      dma16(mask + w, const_cast<float*>(reinterpret_cast<const float*>(imask)) + k * 256);
    }
  };

  __syncthreads();  // W staged
  if (st < nsub) issue(st);
  for (; st < nsub; st += stride) {
    const int64_t r0 = st * 16;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this sub-tile's DMA (and its G row indices) has landed
    const int32_t ndcur = ndnext;
    int32_t grow[4] = {-1, -1, -1, -1};
    float gv[NIB][4];
    if constexpr (FRONTIER) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        grow[i] = gnext[i];
#pragma unroll
        for (int ib = 0; ib < NIB; ++ib)
          gv[ib][i] = grow[i] >= 0 ? G[static_cast<int64_t>(grow[i]) * ldg + ib * 16 + c] : 0.f;
      }
    }
    int32_t gnode[4] = {0, 0, 0, 0};
    float x[NIB][4], sv[NIB][4], da[NCB][4], db[NCB][4];
    {
      float h[NCB][4], dh[NCB][4], nrm[4];
      uint64_t mw[4];
      int32_t node[4];
      bool okr[4], inr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = q * 4 + i;
        const int64_t cr = r0 + row;
        inr[i] = cr < n;
        int64_t nn = cr;
        if constexpr (FRONTIER) {
          const int32_t v = __shfl(ndcur, row);  // issue()'s load of rows[cr] (-1 past n or n_src)
          nn = inr[i] ? v : -1;
        }
        okr[i] = inr[i] && nn >= 0 && nn < n_src;
        node[i] = okr[i] ? static_cast<int32_t>(nn) : 0;
        gnode[i] = node[i];
#pragma unroll
        for (int ib = 0; ib < NIB; ++ib) {
          x[ib][i] = img_at<DIN>(ix, row, ib * 16 + c);
          sv[ib][i] = img_at<DIN>(is, row, ib * 16 + c);
        }
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) {
          h[cb][i] = img_at<DOUT>(ih, row, cb * 16 + c);
          dh[cb][i] = img_at<DOUT>(ig, row, cb * 16 + c);
        }
        nrm[i] = inorm[row];
        mw[i] = imask[row * 16 + c];
      }
      const bool partial = FRONTIER || r0 + 16 > n;
      if (partial) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
          for (int ib = 0; ib < NIB; ++ib) {
            x[ib][i] = okr[i] ? x[ib][i] : 0.f;
            sv[ib][i] = okr[i] ? sv[ib][i] : 0.f;
          }
#pragma unroll
          for (int cb = 0; cb < NCB; ++cb) {
            h[cb][i] = okr[i] ? h[cb][i] : 0.f;
            dh[cb][i] = inr[i] ? dh[cb][i] : 0.f;
          }
          nrm[i] = okr[i] ? nrm[i] : 1.f;
          mw[i] = okr[i] ? mw[i] : 0ull;
        }
      }
      // the image is in registers: stream the next sub-tile into it
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (st + stride < nsub) issue(st + stride);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float dot = 0.f;
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) dot = fmaf(h[cb][i], dh[cb][i], dot);
        dot = sum16(dot);
        const bool clamped = nrm[i] < 0.f;
        const float inv = clamped ? 1.f / kNormEps : 1.f / nrm[i];
        const float proj = clamped ? 0.f : dot;
        const int sh = (node[i] & 3) * 3;
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) {
          const uint32_t bits = static_cast<uint32_t>(mw[i] >> (cb * 12 + sh)) & 7u;
          float dg = (dh[cb][i] - h[cb][i] * proj) * inv;
          dg = (bits & 4u) ? dg * scale : 0.f;
          da[cb][i] = (bits & 1u) ? dg : dg * kLeakySlope;
          db[cb][i] = (bits & 2u) ? dg : dg * kLeakySlope;
          gb1[cb] += da[cb][i];
          gb2[cb] += db[cb][i];
          tda[(q * 4 + i) * F::OLD + cb * 16 + c] = da[cb][i];
          tdb[(q * 4 + i) * F::OLD + cb * 16 + c] = db[cb][i];
        }
      }
    }
    __builtin_amdgcn_wave_barrier();  // LDS ops of one wave complete in order

    // du = dA . W1, dm = dB . W2 over K = DOUT (k = q*KO + step)
    {
      const bool full = r0 + 16 <= n;
      float* pxd[4];
      float* psd[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t row = r0 + q * 4 + i;
        pxd[i] = dXd + row * lddxd + c;
        psd[i] = dS + row * ldds + c;
      }
      float dar[KO], dbr[KO];
      const float* pa = tda + c * F::OLD + q * KO;
      const float* pb = tdb + c * F::OLD + q * KO;
#pragma unroll
      for (int t = 0; t < KO; t += 4) {
        const float4 va = *reinterpret_cast<const float4*>(pa + t);
        const float4 vb = *reinterpret_cast<const float4*>(pb + t);
        dar[t] = va.x; dar[t + 1] = va.y; dar[t + 2] = va.z; dar[t + 3] = va.w;
        dbr[t] = vb.x; dbr[t + 1] = vb.y; dbr[t + 2] = vb.z; dbr[t + 3] = vb.w;
      }
#pragma unroll
      for (int ib = 0; ib < NIB; ++ib) {
        floatx4 du = {0.f, 0.f, 0.f, 0.f}, dm = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < KO; ++t) {
          const int k = q * KO + t;
          du = mfma16x4(dar[t], w1s[k * F::WLDB + ib * 16 + c], du);
          dm = mfma16x4(dbr[t], w2s[k * F::WLDB + ib * 16 + c], dm);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (full || q * 4 + i < n - r0) {
            float vx = fmaf(dm[i], sv[ib][i], du[i]);
            if (FRONTIER && grow[i] >= 0) vx = vx + gv[ib][i];  // kgat_bpr_bwd_f32's dst += g, folded
            pxd[i][ib * 16] = vx;
            psd[i][ib * 16] = fmaf(dm[i], x[ib][i], du[i]);
          }
        }
      }
      if constexpr (FRONTIER) {
        // the batch-row map entries this tile consumed go back to -1 (kgat_frontier_reset folded in): each
        // node is in one tile only, and the store depends on the loaded entry
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (c == 0 && grow[i] >= 0 && gmap != nullptr) gmap[gnode[i]] = -1;
      }
    }
    __builtin_amdgcn_wave_barrier();

    // weight gradients, K = the 16 rows (step s = C-layout element s)
#pragma unroll
    for (int ib = 0; ib < NIB; ++ib) {
      float u[4], m[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        u[i] = x[ib][i] + sv[ib][i];
        m[i] = x[ib][i] * sv[ib][i];
      }
#pragma unroll
      for (int ob = 0; ob < NCB; ++ob)
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          dw1[ob][ib] = mfma16x4(da[ob][s4], u[s4], dw1[ob][ib]);
          dw2[ob][ib] = mfma16x4(db[ob][s4], m[s4], dw2[ob][ib]);
        }
    }
  }

  // one slab per block: [dW1 | dW2 | db1 | db2] = ((wave 0 + wave 1) + wave 2) + wave 3, the four waves'
  // partials added through LDS (the staging images are free once every wave has left the loop) -- a quarter of
  // the slab bytes written here and read by slab_reduce_kernel (C2's layer-0 hop backward: 34 -> 8.5 MB)
  constexpr int kSlab = 2 * DOUT * DIN + 2 * DOUT;
  static_assert(4 * kSlab <= F::kTotal, "the four wave slabs must fit the staging LDS");
  __syncthreads();  // every wave is done with its image (no DMA in flight past the last sub-tile)
  float* ws = smem + wave * kSlab;
#pragma unroll
  for (int ob = 0; ob < NCB; ++ob)
#pragma unroll
    for (int ib = 0; ib < NIB; ++ib)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        ws[(ob * 16 + q * 4 + i) * DIN + ib * 16 + c] = dw1[ob][ib][i];
        ws[DOUT * DIN + (ob * 16 + q * 4 + i) * DIN + ib * 16 + c] = dw2[ob][ib][i];
      }
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) {
    float a = gb1[cb], b = gb2[cb];
    a += __shfl_xor(a, 16);
    a += __shfl_xor(a, 32);
    b += __shfl_xor(b, 16);
    b += __shfl_xor(b, 32);
    if (q == 0) {
      ws[2 * DOUT * DIN + cb * 16 + c] = a;
      ws[2 * DOUT * DIN + DOUT + cb * 16 + c] = b;
    }
  }
  __syncthreads();
  float* out = slab + static_cast<int64_t>(blockIdx.x) * kSlab;
  for (int j = threadIdx.x; j < kSlab; j += 256)
    out[j] = ((smem[j] + smem[kSlab + j]) + smem[2 * kSlab + j]) + smem[3 * kSlab + j];
}

// Sum the per-block slabs: one 1024-thread block per 64 outputs, 16 waves
// split the slabs (wave w takes slabs w, w+16, ...), then add the 16 wave
// partials in wave order -- deterministic.
__global__ __launch_bounds__(1024) void slab_reduce_kernel(const float* __restrict__ slab, int nslab, int width,
                                                           float* __restrict__ dW1, float* __restrict__ dW2,
                                                           float* __restrict__ db1, float* __restrict__ db2,
                                                           int din, int dout) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (i < width) {
#pragma unroll 8
    for (int b = wave; b < nslab; b += 16) s += slab[static_cast<int64_t>(b) * width + i];
  }
  red[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && i < width) {
    float t = red[0][lane];
    for (int w = 1; w < 16; ++w) t += red[w][lane];
    const int wsz = din * dout;
    if (i < wsz) dW1[i] = t;
    else if (i < 2 * wsz) dW2[i - wsz] = t;
    else if (i < 2 * wsz + dout) db1[i - 2 * wsz] = t;
    else db2[i - 2 * wsz - dout] = t;
  }
}

// The backward stages W1/W2 in LDS when they fit beside the tiles (measured at 64x64 on MI355X:
// 1.05 ms vs 1.66 ms reading W through L1/L2, whose extra registers spill).
template <int DIN, int DOUT>
static int bwd_grid(int64_t n) {
  const int lds = BwdLds<DIN, DOUT, true>::kTotal * 4;
  int per_cu = (160 * 1024) / lds;
  if (per_cu < 1) per_cu = 1;
  if (per_cu > 4) per_cu = 4;
  return blocks_for(n, 64, kCUs * per_cu);
}

template <int DIN, int DOUT, bool WLDS>
static int launch_bwd_kernel(int grid, const float* X, int64_t ldx, const float* S, int64_t lds, const float* dH,
                             int64_t lddh, const float* W1, const float* b1, const float* W2, const float* b2,
                             float* dXd, int64_t lddxd, float* dS, int64_t ldds, float* ws, int64_t n, float p,
                             uint64_t seed, const int32_t* rows, int64_t n_src, hipStream_t st) {
  const size_t lds_bytes = BwdLds<DIN, DOUT, WLDS>::kTotal * sizeof(float);
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&biinter_bwd_kernel<DIN, DOUT, WLDS>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds_bytes));
    if (e != hipSuccess) return static_cast<int>(e);
    attr_set = true;
  }
  hipLaunchKernelGGL((biinter_bwd_kernel<DIN, DOUT, WLDS>), dim3(grid), dim3(256), lds_bytes, st, X, ldx, S, lds, dH,
                     lddh, W1, b1, W2, b2, dXd, lddxd, dS, ldds, ws, n, p, seed, rows, n_src);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

template <int DIN, int DOUT>
static int launch_fwd(const float* X, int64_t ldx, const float* S, int64_t lds, const float* W1, const float* b1,
                      const float* W2, const float* b2, float* H, int64_t ldh, int64_t n, float p, uint64_t seed,
                      float* norm, uint64_t* mask, int64_t node0, hipStream_t st) {
  // no prefetch, 2 waves/SIMD minimum (measured at C2, 64->64: the prefetch's 172 VGPRs allow 2 waves per SIMD,
  // without it 132; a one-round grid, 4 waves/SIMD and the prefetch at 3 / 4 waves/SIMD measured no faster,
  // DESIGN.md §5)
  constexpr int NWV = BiFwdWaves<DIN, DOUT>::k;
  const int grid = blocks_for(n, 16 * NWV, kCUs * 8 * 4 / NWV);
  hipLaunchKernelGGL((biinter_fwd_kernel<DIN, DOUT, false, 2, NWV>), dim3(grid), dim3(64 * NWV), 0, st, X, ldx, S,
                     lds, W1, b1, W2, b2, H, ldh, n, p, seed, norm, mask, node0);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

template <int DIN, int DOUT>
static int launch_fwd_tiles(const float* X, int64_t ldx, const float* S, int64_t lds, const float* W1,
                            const float* b1, const float* W2, const float* b2, float* H, int64_t ldh, int64_t n,
                            float p, uint64_t seed, float* norm, uint64_t* mask, const uint32_t* row_bits,
                            hipStream_t st) {
  constexpr int NWV = BiFwdWaves<DIN, DOUT>::k;
  // one block per chunk of 4 * NWV tiles (probe at C2, rocprof kernel time, bit-identical: a 15.6k-row hop set
  // 89.6 -> 79.7 us at 64 -> 64, the ~720 batch rows 20.8 -> 13.5 us, against the grid-stride walk over every
  // tile's bitmap word; tools/tiles_probe_prof.sh)
  const int64_t grid = ((n + 15) / 16 + 4 * NWV - 1) / (4 * NWV);
  if (grid > 0x7fffffff) return KGAT_ERR_INVALID;
  hipLaunchKernelGGL((biinter_fwd_set_kernel<DIN, DOUT, NWV>), dim3(grid), dim3(64 * NWV), 0, st, X, ldx, S, lds, W1,
                     b1, W2, b2, H, ldh, n, p, seed, norm, mask, row_bits);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

template <int DIN, int DOUT>
static int launch_fwd_list(const float* X, int64_t ldx, const float* S, int64_t lds, const float* W1,
                           const float* b1, const float* W2, const float* b2, float* H, int64_t ldh, int64_t n,
                           float p, uint64_t seed, float* norm, uint64_t* mask, const int32_t* rows,
                           const int32_t* count, int64_t cap, hipStream_t st) {
  constexpr int NWV = BiFwdWaves<DIN, DOUT>::k;
  // one round of blocks (W staged once per block), windows strided over them; blocks past the set's windows
  // return after reading the count
  const int grid = blocks_for(cap, 4 * NWV, kCUs * 4 * 4 / NWV);
  hipLaunchKernelGGL((biinter_fwd_list_kernel<DIN, DOUT, NWV>), dim3(grid), dim3(64 * NWV), 0, st, X, ldx, S, lds, W1,
                     b1, W2, b2, H, ldh, n, p, seed, norm, mask, rows, count, cap);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

template <int DIN, int DOUT>
static int saved_grid(int64_t n) {
  return blocks_for(n, 64, kCUs);
}

// Workspace floats: slabs of whichever backward variant the shape can take.
template <int DIN, int DOUT>
static int64_t bwd_workspace(int64_t n) {
  const int64_t width = 2LL * DIN * DOUT + 2LL * DOUT;
  int64_t slabs = bwd_grid<DIN, DOUT>(n);
  if constexpr (SavedBwd<DIN, DOUT>::kOk) {
    const int64_t sl = saved_grid<DIN, DOUT>(n);
    if (sl > slabs) slabs = sl;
  }
  return slabs * width;
}

template <int DIN, int DOUT>
static int launch_saved(const float* X, int64_t ldx, const float* S, int64_t lds, const float* H, int64_t ldh,
                        const float* norm, const uint64_t* mask, const float* dH, int64_t lddh, const float* W1,
                        const float* W2, float* dXd, int64_t lddxd, float* dS, int64_t ldds, int64_t n, float p,
                        const int32_t* rows, int64_t n_src, float* ws, int64_t ws_floats, int* nslab,
                        hipStream_t st, const int32_t* n_dev = nullptr, int dh_by_node = 0,
                        const float* G = nullptr, int64_t ldg = 0, const int32_t* gidx = nullptr,
                        int32_t* gmap = nullptr) {
  using F = SavedBwd<DIN, DOUT>;
  const int width = 2 * DOUT * DIN + 2 * DOUT;
  const int grid = saved_grid<DIN, DOUT>(n);
  *nslab = grid;  // one slab per block (the four waves' partials summed in the kernel)
  if (ws == nullptr || ws_floats < static_cast<int64_t>(*nslab) * width) return KGAT_ERR_WORKSPACE;
  const size_t lds_bytes = F::kTotal * sizeof(float);
  static bool attr_set = false;
  if (!attr_set) {
    for (const void* fn : {reinterpret_cast<const void*>(&biinter_bwd_saved_kernel<DIN, DOUT, false>),
                           reinterpret_cast<const void*>(&biinter_bwd_saved_kernel<DIN, DOUT, true>)}) {
      hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds_bytes));
      if (e != hipSuccess) return static_cast<int>(e);
    }
    attr_set = true;
  }
  if (rows != nullptr)
    hipLaunchKernelGGL((biinter_bwd_saved_kernel<DIN, DOUT, true>), dim3(grid), dim3(256), lds_bytes, st, X, ldx, S,
                       lds, H, ldh, norm, mask, dH, lddh, W1, W2, dXd, lddxd, dS, ldds, ws, n, p, rows, n_src,
                       n_dev, dh_by_node, G, ldg, gidx, gmap);
  else
    hipLaunchKernelGGL((biinter_bwd_saved_kernel<DIN, DOUT, false>), dim3(grid), dim3(256), lds_bytes, st, X, ldx, S,
                       lds, H, ldh, norm, mask, dH, lddh, W1, W2, dXd, lddxd, dS, ldds, ws, n, p, rows, n_src,
                       nullptr, 0, nullptr, 0, nullptr, nullptr);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

// Hop-chain backward: rows / count from kgat_hop_compact (count on the device,
// n_max its bound), dH indexed by node, dXd / dS compact.  Saved state only.
template <int DIN, int DOUT>
static int launch_hop(const float* X, int64_t ldx, const float* S, int64_t lds, const float* H, int64_t ldh,
                      const float* norm, const uint64_t* mask, const float* dH, int64_t lddh, const float* W1,
                      const float* W2, float* dXd, int64_t lddxd, float* dS, int64_t ldds, float* dW1, float* db1,
                      float* dW2, float* db2, int64_t n_max, float p, const int32_t* rows, const int32_t* n_dev,
                      int64_t src_rows, int dh_by_node, float* ws, int64_t ws_floats, hipStream_t st,
                      const float* G = nullptr, int64_t ldg = 0, const int32_t* gidx = nullptr,
                      int32_t* gmap = nullptr) {
  if constexpr (!SavedBwd<DIN, DOUT>::kOk) {
    return KGAT_ERR_UNSUPPORTED_DIM;
  } else {
    const int width = 2 * DOUT * DIN + 2 * DOUT;
    int nslab = 0;
    if (int e = launch_saved<DIN, DOUT>(X, ldx, S, lds, H, ldh, norm, mask, dH, lddh, W1, W2, dXd, lddxd, dS, ldds,
                                        n_max, p, rows, src_rows, ws, ws_floats, &nslab, st, n_dev, dh_by_node, G,
                                        ldg, gidx, gmap))
      return e;
    hipLaunchKernelGGL(slab_reduce_kernel, dim3((width + 63) / 64), dim3(1024), 0, st, ws, nslab, width, dW1, dW2,
                       db1, db2, DIN, DOUT);
    KGAT_LAUNCH_CHECK();
    return KGAT_OK;
  }
}

template <int DIN, int DOUT>
static int launch_bwd(const float* X, int64_t ldx, const float* S, int64_t lds, const float* H, int64_t ldh,
                      const float* norm, const uint64_t* mask, const float* dH, int64_t lddh, const float* W1,
                      const float* b1, const float* W2, const float* b2, float* dXd, int64_t lddxd, float* dS,
                      int64_t ldds, float* dW1, float* db1, float* dW2, float* db2, int64_t n, float p, uint64_t seed,
                      const int32_t* rows, int64_t src_rows, float* ws, int64_t ws_floats, hipStream_t st) {
  const int width = 2 * DOUT * DIN + 2 * DOUT;
  const int64_t n_src = rows ? src_rows : n;
  int nslab = 0;
  bool saved = false;
  if constexpr (SavedBwd<DIN, DOUT>::kOk) {
    if (H != nullptr && norm != nullptr && mask != nullptr) {
      saved = true;
      if (int e = launch_saved<DIN, DOUT>(X, ldx, S, lds, H, ldh, norm, mask, dH, lddh, W1, W2, dXd, lddxd, dS, ldds,
                                          n, p, rows, n_src, ws, ws_floats, &nslab, st))
        return e;
    }
  }
  if (!saved) {
    const int grid = bwd_grid<DIN, DOUT>(n);
    nslab = grid;
    if (ws == nullptr || ws_floats < static_cast<int64_t>(grid) * width) return KGAT_ERR_WORKSPACE;
    if (int e = launch_bwd_kernel<DIN, DOUT, true>(grid, X, ldx, S, lds, dH, lddh, W1, b1, W2, b2, dXd, lddxd, dS,
                                                   ldds, ws, n, p, seed, rows, n_src, st))
      return e;
  }
  hipLaunchKernelGGL(slab_reduce_kernel, dim3((width + 63) / 64), dim3(1024), 0, st, ws, nslab, width, dW1, dW2,
                     db1, db2, DIN, DOUT);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

}  // namespace kgat

#define KGAT_BI_DISPATCH(CALL)                                  \
  switch (d_in * 1000 + d_out) {                                \
    case 16016: return CALL(16, 16);                            \
    case 32016: return CALL(32, 16);                            \
    case 32032: return CALL(32, 32);                            \
    case 64016: return CALL(64, 16);                            \
    case 64032: return CALL(64, 32);                            \
    case 64064: return CALL(64, 64);                            \
    case 128032: return CALL(128, 32);                          \
    case 128064: return CALL(128, 64);                          \
    case 128128: return CALL(128, 128);                         \
    case 32064: return CALL(32, 64);                            \
    case 16032: return CALL(16, 32);                            \
    case 64128: return CALL(64, 128);                           \
    default: return KGAT_ERR_UNSUPPORTED_DIM;                   \
  }

static bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

extern "C" int kgat_biinter_fwd_rows_f32(const float* X, int64_t ldx, const float* S, int64_t lds, const float* W1,
                                         const float* b1, const float* W2, const float* b2, float* H, int64_t ldh,
                                         int64_t n_rows, int64_t node0, int32_t d_in, int32_t d_out, float dropout_p,
                                         uint64_t seed, float* norm_out, uint64_t* mask_out, void* stream) {
  if (!X || !S || !W1 || !b1 || !W2 || !b2 || !H || n_rows < 0 || node0 < 0 || (node0 & 15)) return KGAT_ERR_INVALID;
  if (!aligned16(X) || !aligned16(S) || !aligned16(W1) || !aligned16(W2) || (ldx & 3) || (lds & 3))
    return KGAT_ERR_INVALID;
  if (ldx < d_in || lds < d_in || ldh < d_out || !(dropout_p >= 0.f && dropout_p < 1.f)) return KGAT_ERR_INVALID;
  if ((norm_out == nullptr) != (mask_out == nullptr) || (mask_out != nullptr && d_out > 128)) return KGAT_ERR_INVALID;
  if (mask_out != nullptr && d_out > 64 && node0 != 0) return KGAT_ERR_INVALID;  // multi-word state: whole tables
  if (n_rows == 0) return KGAT_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define KGAT_FWD_CALL(a, b) kgat::launch_fwd<a, b>(X, ldx, S, lds, W1, b1, W2, b2, H, ldh, n_rows, dropout_p, seed, \
                                                  norm_out, mask_out, node0, st)
  KGAT_BI_DISPATCH(KGAT_FWD_CALL)
#undef KGAT_FWD_CALL
}

extern "C" int kgat_biinter_fwd_tiles_f32(const float* X, int64_t ldx, const float* S, int64_t lds,
                                          const float* W1, const float* b1, const float* W2, const float* b2,
                                          float* H, int64_t ldh, int64_t n_rows, const uint32_t* row_bits,
                                          int32_t d_in, int32_t d_out,
                                          float dropout_p, uint64_t seed, float* norm_out, uint64_t* mask_out,
                                          void* stream) {
  if (!X || !S || !W1 || !b1 || !W2 || !b2 || !H || !row_bits || n_rows < 0) return KGAT_ERR_INVALID;
  if (!aligned16(X) || !aligned16(S) || !aligned16(W1) || !aligned16(W2) || (ldx & 3) || (lds & 3))
    return KGAT_ERR_INVALID;
  if (ldx < d_in || lds < d_in || ldh < d_out || !(dropout_p >= 0.f && dropout_p < 1.f)) return KGAT_ERR_INVALID;
  if ((norm_out == nullptr) != (mask_out == nullptr) || (mask_out != nullptr && d_out > 128)) return KGAT_ERR_INVALID;
  if (n_rows == 0) return KGAT_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define KGAT_FWDT_CALL(a, b) kgat::launch_fwd_tiles<a, b>(X, ldx, S, lds, W1, b1, W2, b2, H, ldh, n_rows, dropout_p, \
                                                         seed, norm_out, mask_out, row_bits, st)
  KGAT_BI_DISPATCH(KGAT_FWDT_CALL)
#undef KGAT_FWDT_CALL
}

extern "C" int kgat_biinter_fwd_list_f32(const float* X, int64_t ldx, const float* S, int64_t lds,
                                         const float* W1, const float* b1, const float* W2, const float* b2,
                                         float* H, int64_t ldh, int64_t n_rows, const int32_t* rows,
                                         const int32_t* count, int64_t cap, int32_t d_in, int32_t d_out,
                                         float dropout_p, uint64_t seed, float* norm_out, uint64_t* mask_out,
                                         void* stream) {
  if (!X || !S || !W1 || !b1 || !W2 || !b2 || !H || !rows || !count || n_rows < 0 || cap < 0) return KGAT_ERR_INVALID;
  if (!aligned16(X) || !aligned16(S) || !aligned16(W1) || !aligned16(W2) || (ldx & 3) || (lds & 3))
    return KGAT_ERR_INVALID;
  if (ldx < d_in || lds < d_in || ldh < d_out || !(dropout_p >= 0.f && dropout_p < 1.f)) return KGAT_ERR_INVALID;
  if ((norm_out == nullptr) != (mask_out == nullptr) || (mask_out != nullptr && d_out > 128)) return KGAT_ERR_INVALID;
  if (n_rows == 0 || cap == 0) return KGAT_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define KGAT_FWDL_CALL(a, b) kgat::launch_fwd_list<a, b>(X, ldx, S, lds, W1, b1, W2, b2, H, ldh, n_rows, dropout_p, \
                                                        seed, norm_out, mask_out, rows, count, cap, st)
  KGAT_BI_DISPATCH(KGAT_FWDL_CALL)
#undef KGAT_FWDL_CALL
}

extern "C" int kgat_biinter_fwd_f32(const float* X, int64_t ldx, const float* S, int64_t lds, const float* W1,
                                    const float* b1, const float* W2, const float* b2, float* H, int64_t ldh,
                                    int64_t n_rows, int32_t d_in, int32_t d_out, float dropout_p, uint64_t seed,
                                    float* norm_out, uint64_t* mask_out, void* stream) {
  return kgat_biinter_fwd_rows_f32(X, ldx, S, lds, W1, b1, W2, b2, H, ldh, n_rows, 0, d_in, d_out, dropout_p, seed,
                                   norm_out, mask_out, stream);
}

extern "C" int64_t kgat_biinter_bwd_workspace(int64_t n_rows, int32_t d_in, int32_t d_out) {
  if (n_rows < 0) return -1;
#define KGAT_WS_CALL(a, b) kgat::bwd_workspace<a, b>(n_rows)
  switch (d_in * 1000 + d_out) {
    case 16016: return KGAT_WS_CALL(16, 16);
    case 32016: return KGAT_WS_CALL(32, 16);
    case 32032: return KGAT_WS_CALL(32, 32);
    case 64016: return KGAT_WS_CALL(64, 16);
    case 64032: return KGAT_WS_CALL(64, 32);
    case 64064: return KGAT_WS_CALL(64, 64);
    case 128032: return KGAT_WS_CALL(128, 32);
    case 128064: return KGAT_WS_CALL(128, 64);
    case 128128: return KGAT_WS_CALL(128, 128);
    case 32064: return KGAT_WS_CALL(32, 64);
    case 16032: return KGAT_WS_CALL(16, 32);
    case 64128: return KGAT_WS_CALL(64, 128);
    default: return -1;
  }
#undef KGAT_WS_CALL
}

extern "C" int kgat_biinter_bwd_f32(const float* X, int64_t ldx, const float* S, int64_t lds, const float* H,
                                    int64_t ldh, const float* norm, const uint64_t* mask, const float* dH,
                                    int64_t lddh, const float* W1, const float* b1, const float* W2, const float* b2,
                                    float* dXd, int64_t lddxd, float* dS, int64_t ldds, float* dW1, float* db1,
                                    float* dW2, float* db2, int64_t n_rows, int32_t d_in, int32_t d_out,
                                    float dropout_p, uint64_t seed, const int32_t* rows, int64_t src_rows,
                                    float* workspace, int64_t workspace_floats, void* stream) {
  if (!X || !S || !dH || !W1 || !b1 || !W2 || !b2 || !dXd || !dS || !dW1 || !db1 || !dW2 || !db2 || n_rows < 0)
    return KGAT_ERR_INVALID;
  if (!aligned16(X) || !aligned16(S) || !aligned16(W1) || !aligned16(W2) || (ldx & 3) || (lds & 3))
    return KGAT_ERR_INVALID;
  if (ldx < d_in || lds < d_in || lddh < d_out || lddxd < d_in || ldds < d_in) return KGAT_ERR_INVALID;
  if (!(dropout_p >= 0.f && dropout_p < 1.f)) return KGAT_ERR_INVALID;
  const int n_state = (H != nullptr) + (norm != nullptr) + (mask != nullptr);
  if (n_state != 0 && (n_state != 3 || ldh < d_out)) return KGAT_ERR_INVALID;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define KGAT_BWD_CALL(a, b)                                                                                   \
  kgat::launch_bwd<a, b>(X, ldx, S, lds, H, ldh, norm, mask, dH, lddh, W1, b1, W2, b2, dXd, lddxd, dS, ldds, dW1, db1, dW2, db2, \
                         n_rows, dropout_p, seed, rows, src_rows, workspace, workspace_floats, st)
  KGAT_BI_DISPATCH(KGAT_BWD_CALL)
#undef KGAT_BWD_CALL
}

extern "C" int kgat_biinter_bwd_hop_ex_f32(const float* X, int64_t ldx, const float* S, int64_t lds, const float* H,
                                           int64_t ldh, const float* norm, const uint64_t* mask, const float* dH,
                                           int64_t lddh, const float* W1, const float* W2, float* dXd, int64_t lddxd,
                                           float* dS, int64_t ldds, float* dW1, float* db1, float* dW2, float* db2,
                                           const int32_t* rows, const int32_t* count, int64_t n_max, int64_t src_rows,
                                           int32_t dh_compact, int32_t d_in, int32_t d_out, float dropout_p,
                                           const float* G, int64_t ldg, const int32_t* gidx, int32_t* gmap,
                                           float* workspace,
                                           int64_t workspace_floats, void* stream) {
  if (!X || !S || !H || !norm || !mask || !dH || !W1 || !W2 || !dXd || !dS || !dW1 || !db1 || !dW2 || !db2 ||
      !rows || !count || n_max < 0 || src_rows < 0)
    return KGAT_ERR_INVALID;
  if (!aligned16(X) || !aligned16(S) || !aligned16(W1) || !aligned16(W2) || (ldx & 3) || (lds & 3))
    return KGAT_ERR_INVALID;
  if (ldx < d_in || lds < d_in || lddh < d_out || lddxd < d_in || ldds < d_in || ldh < d_out) return KGAT_ERR_INVALID;
  if (!(dropout_p >= 0.f && dropout_p < 1.f)) return KGAT_ERR_INVALID;
  if ((G == nullptr) != (gidx == nullptr) || (G != nullptr && ldg < d_in)) return KGAT_ERR_INVALID;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define KGAT_HOP_CALL(a, b)                                                                                       \
  kgat::launch_hop<a, b>(X, ldx, S, lds, H, ldh, norm, mask, dH, lddh, W1, W2, dXd, lddxd, dS, ldds, dW1, db1, dW2, \
                         db2, n_max, dropout_p, rows, count, src_rows, dh_compact ? 0 : 1, workspace, workspace_floats, \
                         st, G, ldg, gidx, gmap)
  KGAT_BI_DISPATCH(KGAT_HOP_CALL)
#undef KGAT_HOP_CALL
}

extern "C" int kgat_biinter_bwd_hop_f32(const float* X, int64_t ldx, const float* S, int64_t lds, const float* H,
                                        int64_t ldh, const float* norm, const uint64_t* mask, const float* dH,
                                        int64_t lddh, const float* W1, const float* W2, float* dXd, int64_t lddxd,
                                        float* dS, int64_t ldds, float* dW1, float* db1, float* dW2, float* db2,
                                        const int32_t* rows, const int32_t* count, int64_t n_max, int64_t src_rows,
                                        int32_t dh_compact, int32_t d_in, int32_t d_out, float dropout_p,
                                        float* workspace, int64_t workspace_floats, void* stream) {
  return kgat_biinter_bwd_hop_ex_f32(X, ldx, S, lds, H, ldh, norm, mask, dH, lddh, W1, W2, dXd, lddxd, dS, ldds, dW1,
                                     db1, dW2, db2, rows, count, n_max, src_rows, dh_compact, d_in, d_out, dropout_p,
                                     nullptr, 0, nullptr, nullptr, workspace, workspace_floats, stream);
}
