// Shared device helpers for the gfx950 KGAT kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kgat_hip.h"

#define KGAT_LAUNCH_CHECK()                          \
  do {                                               \
    hipError_t e_ = hipGetLastError();               \
    if (e_ != hipSuccess) return static_cast<int>(e_); \
  } while (0)

namespace kgat {

constexpr int kWave = 64;           // CDNA wavefront
constexpr int kCUs = 256;           // MI355X compute units
constexpr float kLeakySlope = 0.01f;  // nn.LeakyReLU() default (aggregator.py:23)
constexpr float kNormEps = 1e-12f;    // F.normalize default (aggregator.py:65)

typedef float floatx4 __attribute__((ext_vector_type(4)));

// D[16x16] += A[16x4] . B[4x16], exact fp32 fma chain (v_mfma_f32_16x16x4_f32).
// Lane l supplies A[l&15][l>>4] and B[l>>4][l&15]; lane l receives
// D[(l>>4)*4 + i][l&15] in element i.
__device__ __forceinline__ floatx4 mfma16x4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float lrelu(float x) { return x > 0.f ? x : x * kLeakySlope; }
__device__ __forceinline__ float lrelu_grad(float x) { return x > 0.f ? 1.f : kLeakySlope; }

// Counter-based dropout mask: a splitmix64 finaliser of (seed, element index).
// Regenerated bit-identically by every backward kernel, so no mask is stored.
__device__ __forceinline__ uint32_t mix_hash(uint64_t seed, uint64_t idx) {
  uint64_t z = seed + (idx + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return static_cast<uint32_t>(z >> 32);
}
__device__ __forceinline__ uint64_t mix_hash64(uint64_t seed, uint64_t idx) {
  uint64_t z = seed + (idx + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ bool dropout_keep(uint64_t seed, uint64_t idx, float p) {
  return static_cast<float>(mix_hash(seed, idx) >> 8) * (1.0f / 16777216.0f) >= p;
}

// v + (v of lane lane' in the same DPP row), lane' given by the DPP control CTRL.
template <int CTRL>
__device__ __forceinline__ float dpp_add(float v) {
  return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// Sum over the 16 lanes that share (lane >> 4): a butterfly inside the DPP row (no LDS-path
// ds_bpermute): quad_perm [1,0,3,2] (lane ^ 1), quad_perm [2,3,0,1] (lane ^ 2), row_half_mirror
// (lane 7 - i: the other quad), row_mirror (lane 15 - i: the other half).  Each level adds the
// same two partial sums as the xor butterfly (lane ^ 1, ^ 2, ^ 4, ^ 8), so every lane gets the same
// bits as it.  All 16 lanes of the row must be active.
__device__ __forceinline__ float sum16(float v) {
  v = dpp_add<0xB1>(v);
  v = dpp_add<0x4E>(v);
  v = dpp_add<0x141>(v);
  v = dpp_add<0x140>(v);
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// One torch.optim.Adam element update (model.py:404-419), same operation order as
// torch's single/multi-tensor paths:
//   m = m + (1-b1)(g - m)       (lerp, weight < 0.5 branch)
//   v = v*b2 + ((1-b2) g) g     (mul_ then addcmul_)
//   p = p + (-step_size) * (m / (sqrt(v)/bc2_sqrt + eps))
// each operation rounded on its own (no FMA contraction), so every kernel that
// calls it -- the Adam passes and the fused table update -- produces the same bits.
__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float w1, float b2, float w2,
                                          float step_size, float bc2s, float eps) {
#pragma clang fp contract(off)
  m = m + w1 * (g - m);
  v = v * b2 + (w2 * g) * g;
  p = p + (-step_size) * (m / (sqrtf(v) / bc2s + eps));
}

// Lazy table Adam (a table's Adam on the rows a step touches only).  The dense step moves every row
// each step -- rows with a zero gradient too, which still decays their moments and moves p.  Here a
// row keeps the number of the last step applied to it (last[row]); the steps it skipped are replayed
// in order, with their own step size and bias correction (kept on the device, entry s % cap of the
// history) and the same adam_elem(g = 0) arithmetic, when it is next read or updated, and for every
// row at a flush.  Each element's sequence of operations is the dense step's: the same bits.
struct LazyHist {
  float* sz;
  float* bc;
  int32_t* skip;
  int32_t cap;
};

__device__ __forceinline__ void lazy_replay(float& p, float& m, float& v, int32_t from, int32_t to, const LazyHist& h,
                                            float w1, float b2, float w2, float eps) {
  for (int32_t s = from + 1; s <= to; ++s) {
    const int32_t j = s % h.cap;
    if (h.skip[j] != 0) continue;
    adam_elem(p, 0.f, m, v, w1, b2, w2, h.sz[j], h.bc[j], eps);
  }
}

// The history of the last kHistLds steps staged in LDS by a block before its replays: a replay of k
// steps then costs k LDS reads instead of k dependent global-load round trips (a stale row's replay
// loop was latency-bound); older steps still come from the global ring.
constexpr int kHistLds = 256;
struct LazyHistLds {
  float sz[kHistLds];
  float bc[kHistLds];
  int32_t skip[kHistLds];
};

// Stage steps [lo, to] (lo = max(1, to - kHistLds + 1)) of the ring into L; every thread of the block
// calls it (it ends with a barrier).  Returns lo.
__device__ __forceinline__ int32_t stage_hist(LazyHistLds& L, const LazyHist& h, int32_t to) {
  const int32_t lo = to - kHistLds + 1 > 1 ? to - kHistLds + 1 : 1;
  for (int i = threadIdx.x; i < kHistLds; i += blockDim.x) {
    const int32_t s = lo + i;
    if (s <= to) {
      const int32_t j = s % h.cap;
      L.sz[i] = h.sz[j];
      L.bc[i] = h.bc[j];
      L.skip[i] = h.skip[j];
    }
  }
  __syncthreads();
  return lo;
}

// lazy_replay with steps >= lo read from the staged copy (same values, same order: same bits).
__device__ __forceinline__ void lazy_replay_lds(float& p, float& m, float& v, int32_t from, int32_t to,
                                                const LazyHist& h, const LazyHistLds& L, int32_t lo, float w1,
                                                float b2, float w2, float eps) {
  for (int32_t s = from + 1; s <= to; ++s) {
    float sz, bc;
    int32_t sk;
    if (s >= lo) {
      sz = L.sz[s - lo];
      bc = L.bc[s - lo];
      sk = L.skip[s - lo];
    } else {
      const int32_t j = s % h.cap;
      sz = h.sz[j];
      bc = h.bc[j];
      sk = h.skip[j];
    }
    if (sk != 0) continue;
    adam_elem(p, 0.f, m, v, w1, b2, w2, sz, bc, eps);
  }
}

inline int blocks_for(int64_t work, int per_block, int cap) {
  int64_t b = (work + per_block - 1) / per_block;
  if (b < 1) b = 1;
  return static_cast<int>(b < cap ? b : cap);
}

}  // namespace kgat
