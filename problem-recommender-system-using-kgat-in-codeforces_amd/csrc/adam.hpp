// The multi-tensor Adam step (a9, model.py:393-419) shared by kgat_adam_multi_*_f32 (misc.hip) and the
// fused table update's fix-up launch (spmm.hip: the small tensors' step in the same launch pair).
#pragma once

#include <stdint.h>

#include "common.hpp"

namespace kgat {

// A captured optimiser step's scalars on the device (a HIP graph replays the same kernel arguments every
// step): t = *t + add (the captured update's first Adam launch applies *t + 1 and hands the number on
// through out; the second reads it there and writes it back to t), step size and sqrt(1 - beta2^t) =
// sz[t] / bc[t] -- tables the host filled with FusedAdam's own expressions, so the same floats the
// by-value launches get.  t == nullptr: the by-value arguments.
struct StepSched {
  const int32_t* t;
  const float* sz;
  const float* bc;
  int32_t add = 0;         // the step applied is *t + add
  int32_t* out = nullptr;  // nullable: block 0 / thread 0 writes that step number there (the next launch's t)
};

// The step a scheduled launch applies; its number handed on to the next launch of the captured update.
__device__ __forceinline__ int32_t sched_step(const StepSched& s) {
  const int32_t t = *s.t + s.add;
  if (s.out != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *s.out = t;
  return t;
}

// Every tensor of one optimiser step in ONE launch: the tensor table travels in
// the kernel arguments; block b works on chunk b of the concatenated float4
// index space (tensor chosen by a scan of <= 16 chunk offsets).
struct AdamTable {
  kgat_adam_tensor t[KGAT_ADAM_MAX_TENSORS];
  int64_t chunk_off[KGAT_ADAM_MAX_TENSORS + 1];  // first chunk of tensor i
  int32_t count;
};

constexpr int kAdamChunk = 256 * 4 * 4;  // floats per block-iteration: 256 threads x float4 x 4

template <int V>
__device__ __forceinline__ float4 ld4(const float* p) {
  if constexpr (V == 2) {
    const floatx4 v = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(p));
    return make_float4(v[0], v[1], v[2], v[3]);
  }
  return *reinterpret_cast<const float4*>(p);
}
template <int V>
__device__ __forceinline__ void st4(float* p, float4 v) {
  if constexpr (V == 2) __builtin_nontemporal_store(floatx4{v.x, v.y, v.z, v.w}, reinterpret_cast<floatx4*>(p));
  else *reinterpret_cast<float4*>(p) = v;
}

// V = 0: per float4 load -> update -> store; V >= 1: a chunk's 16 float4 loads issued first
// (all four arrays, four float4 per lane), then the updates, then the stores; V = 2 with
// non-temporal loads/stores (every byte is touched once per step).
// Blocks [block, ...) stepping by nblocks over the concatenated float4 chunks of T (a launch's blocks, or
// the extra blocks of another launch).  ts: the scheduled step (sched.t != nullptr).
template <int V>
__device__ __forceinline__ void adam_multi_chunks(const AdamTable& T, float b1, float b2, float eps,
                                                  const StepSched& sched, int32_t ts, int64_t block, int64_t nblocks) {
  const float w1 = 1.f - b1, w2 = 1.f - b2;
  const int64_t total = T.chunk_off[T.count];
  for (int64_t c = block; c < total; c += nblocks) {
    int i = 0;
    while (i + 1 < T.count && T.chunk_off[i + 1] <= c) ++i;
    const kgat_adam_tensor& a = T.t[i];
    const int64_t base = (c - T.chunk_off[i]) * kAdamChunk;
    const float step_size = sched.t != nullptr ? sched.sz[ts] : a.step_size;
    const float bc2s = sched.t != nullptr ? sched.bc[ts] : a.bc2_sqrt;
    if (V >= 1 && base + kAdamChunk <= a.n) {
      float4 pp[4], mm[4], vv[4], gg[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t e = base + (static_cast<int64_t>(u) * 256 + threadIdx.x) * 4;
        pp[u] = ld4<V>(a.p + e);
        mm[u] = ld4<V>(a.m + e);
        vv[u] = ld4<V>(a.v + e);
        gg[u] = ld4<V>(a.g + e);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float* P = &pp[u].x;
        float* Mv = &mm[u].x;
        float* Vv = &vv[u].x;
        const float* G = &gg[u].x;
#pragma unroll
        for (int k = 0; k < 4; ++k) adam_elem(P[k], G[k], Mv[k], Vv[k], w1, b2, w2, step_size, bc2s, eps);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t e = base + (static_cast<int64_t>(u) * 256 + threadIdx.x) * 4;
        st4<V>(a.p + e, pp[u]);
        st4<V>(a.m + e, mm[u]);
        st4<V>(a.v + e, vv[u]);
      }
      continue;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t e = base + (static_cast<int64_t>(u) * 256 + threadIdx.x) * 4;
      if (e + 4 <= a.n) {
        float4 pp = *reinterpret_cast<float4*>(a.p + e), mm = *reinterpret_cast<float4*>(a.m + e);
        float4 vv = *reinterpret_cast<float4*>(a.v + e);
        const float4 gg = *reinterpret_cast<const float4*>(a.g + e);
        float* P = &pp.x;
        float* Mv = &mm.x;
        float* V_ = &vv.x;
        const float* G = &gg.x;
#pragma unroll
        for (int k = 0; k < 4; ++k) adam_elem(P[k], G[k], Mv[k], V_[k], w1, b2, w2, step_size, bc2s, eps);
        *reinterpret_cast<float4*>(a.p + e) = pp;
        *reinterpret_cast<float4*>(a.m + e) = mm;
        *reinterpret_cast<float4*>(a.v + e) = vv;
      } else {
        for (int64_t k = e; k < a.n && k < e + 4; ++k) {
          float pp = a.p[k], mm = a.m[k], vv = a.v[k];
          adam_elem(pp, a.g[k], mm, vv, w1, b2, w2, step_size, bc2s, eps);
          a.p[k] = pp;
          a.m[k] = mm;
          a.v[k] = vv;
        }
      }
    }
  }
}

// Host: the launch table of <= KGAT_ADAM_MAX_TENSORS tensors (16-byte aligned arrays), KGAT_OK or an error.
inline int adam_table(const kgat_adam_tensor* tensors, int32_t count, AdamTable& T) {
  if (!tensors || count < 1 || count > KGAT_ADAM_MAX_TENSORS) return KGAT_ERR_INVALID;
  T.count = count;
  int64_t off = 0;
  for (int i = 0; i < count; ++i) {
    const kgat_adam_tensor& a = tensors[i];
    if (!a.p || !a.g || !a.m || !a.v || a.n < 0) return KGAT_ERR_INVALID;
    if ((reinterpret_cast<uintptr_t>(a.p) | reinterpret_cast<uintptr_t>(a.g) | reinterpret_cast<uintptr_t>(a.m) |
         reinterpret_cast<uintptr_t>(a.v)) & 15)
      return KGAT_ERR_INVALID;
    T.t[i] = a;
    T.chunk_off[i] = off;
    off += (a.n + kAdamChunk - 1) / kAdamChunk;
  }
  T.chunk_off[count] = off;
  return KGAT_OK;
}

// Blocks of a launch over T's chunks.
inline int adam_grid(const AdamTable& T) {
  const int64_t off = T.chunk_off[T.count];
  return static_cast<int>(off < kCUs * 8 ? off : kCUs * 8);
}

}  // namespace kgat
