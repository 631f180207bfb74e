// Shared pieces of the CSR gather (a1, src/model/KGAT/aggregator.py:54): the
// row-per-group edge walk used by spmm.hip and by the fused propagation +
// bi-interaction forward in biinter.hip.
#pragma once

#include "common.hpp"

namespace kgat {

enum SpmmMode { kOverwrite = 0, kAccumulate = 1, kMasked = 2, kMaskedRows = 3, kMaskedAdam = 4, kRows = 5 };

// kRows: the dense product A . X on the rows of an output set only (out_rows / out_bits /
// out_count; -1 entries of out_rows are padding), each written at its own row of Y -- the
// forward of a layer whose output is needed on a hop set only (kgat_spmm_csr_rows_f32).
// Per row the same edges in the same order as kOverwrite (same bits).

// kMaskedAdam: the masked product's row is the gradient of a table row and is
// consumed on the spot by its Adam step (p, m, v rows of the same index), so
// the dense gradient is never written nor read back.  A short row's p / m / v
// loads go out before its gather (76 VGPRs, 6 waves/SIMD): with the hits
// compacted in LDS that measured ~2 % faster (round 4; in round 2, with the
// per-pick lane search, it was not).
struct SpmmAdam {
  float* p;
  float* m;
  float* v;
  int64_t ld;  // row stride of p, m, v (floats)
  float step_size, b1, b2, bc2s, eps;
  const int32_t* skip;  // nullable: *skip != 0 -> the launch leaves p / m / v untouched (bad step ids)
};

struct SpmmIo {
  const float* X;         // source rows (dense) or compact source rows (masked)
  int64_t ldx;
  float* Y;
  int64_t ldy;
  float* part;            // [n_seg][D] long-row segment partials
  const int32_t* src_map; // masked: node -> compact row or -1
  const float* Yc;        // masked: compact init rows (nullable)
  int64_t ldyc;
  int32_t* row_hit;       // masked: set to 1 for every output row that gathered an edge or has a Yc row (nullable)
  int64_t row0;           // masked: global row of local row 0 (Yc lookup of a row-block view)
  const uint32_t* src_bits;  // masked: bit c set <=> src_map[c] >= 0 (nullable: test src_map directly)
  const uint64_t* src_rank;  // masked, ascending compact order: word c/32 = (#members before it) << 32 | its bits
  // kMaskedRows: only the rows of an output set are produced, compactly (row out_rows[k] -> Y row k);
  // kRows: the same set, each row written at its own index
  const uint32_t* out_bits;  // bit r set <=> r in the set
  const int32_t* out_map;    // r -> k or -1
  const int32_t* out_rows;   // k -> r, ascending
  const int32_t* out_count;  // device: the set's size
  SpmmAdam adam;             // kMaskedAdam only
  // masked modes (not kMaskedAdam): compact rows added after the Yc term through the same src_map row --
  // the BPR loss's direct gradient of the batch rows (kgat_bpr_bwd_multi_f32), folded into the product's
  // store instead of a kgat_bpr_bwd_f32 launch after it (same bits: (Yc + sum) + g either way)
  const float* Gc = nullptr;
  int64_t ldgc = 0;
  int32_t* out_src = nullptr;  // kMaskedRows (nullable): out_src[k] = src_map[out_rows[k]] -- which output rows
                               // have a compact source row (the batch rows' BPR terms, kgat_biinter_bwd_hop_ex_f32)
};

__device__ __forceinline__ bool bit_of(const uint32_t* bits, int64_t i) {
  return ((bits[i >> 5] >> (i & 31)) & 1u) != 0;
}

template <int D>
struct SpmmShape {
  static constexpr int kLanes = D / 4;            // float4 lanes per row
  static constexpr int kGroups = kWave / kLanes;  // rows in flight per wave
  static constexpr int kRowsPerGroup = 4;
  static constexpr int kRowsPerWave = kGroups * kRowsPerGroup;
  static constexpr int kRowsPerBlock = kRowsPerWave * 4;  // 256-thread blocks
};

__device__ __forceinline__ void fma4(float v, const float4& x, float4& acc) {
  acc.x = fmaf(v, x.x, acc.x);
  acc.y = fmaf(v, x.y, acc.y);
  acc.z = fmaf(v, x.z, acc.z);
  acc.w = fmaf(v, x.w, acc.w);
}

// float4 offset of row c (a node id or compact row: 0 <= c < 2^31) of a source with ld4 float4 per row:
// one 32 x 32 -> 64-bit multiply-add instead of a signed 64-bit product
__device__ __forceinline__ uint64_t row_off(int c, uint32_t ld4) {
  return static_cast<uint64_t>(static_cast<uint32_t>(c)) * ld4;
}

__device__ __forceinline__ void add4(float4& a, const float4& b) {
  a.x += b.x;
  a.y += b.y;
  a.z += b.z;
  a.w += b.w;
}

// Wave-scope LDS ordering: this wave's LDS writes land before its later reads of other lanes' slots.
__device__ __forceinline__ void wave_lds_order() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Accumulate edges [beg, end) of one row into acc.  All lanes of the group
// (base .. base+kLanes-1) run this with identical bounds (group-uniform).
// MASKED: hb is the group's kLanes-entry LDS slot array (the chunk's hits compacted there).
template <int D, bool MASKED, int U = 4, int UM = 4>
__device__ __forceinline__ void gather_edges(const kgat_csr& A, const SpmmIo& io, int64_t beg, int64_t end, int base,
                                             int gl, float4& acc, bool& any, int2* hb = nullptr) {
  constexpr int L = SpmmShape<D>::kLanes;
  const float4* X4 = reinterpret_cast<const float4*>(io.X);
  const uint32_t ldx4u = static_cast<uint32_t>(io.ldx / 4);
  for (int64_t cb = beg; cb < end; cb += L) {
    const int n = static_cast<int>(end - cb < L ? end - cb : L);
    int mc = 0;
    float mv = 0.f;
    if (MASKED) {
      // membership first: a bit of the source set (its rank word gives the compact row
      // too, with one 8-byte load), then the gathers of the edges that hit; skipped
      // edges add an exact 0, so the gathered ones keep the dense order
      bool in = false;
      if (gl < n) {
        mc = A.col[cb + gl];
        mv = A.val[cb + gl];
        if (io.src_rank != nullptr) {
          const uint64_t w = io.src_rank[mc >> 5];
          const uint32_t b = static_cast<uint32_t>(mc & 31);
          in = ((w >> b) & 1u) != 0;
          mc = static_cast<int>(w >> 32) + __popc(static_cast<uint32_t>(w) & ((1u << b) - 1u));
        } else {
          in = io.src_bits != nullptr ? ((io.src_bits[mc >> 5] >> (mc & 31)) & 1u) != 0 : io.src_map[mc] >= 0;
        }
      }
      // the group's hit bits in a 32-bit word where they fit (the group's lanes are L <= 32 bits of the ballot)
      using HitT = typename std::conditional<(L <= 32), uint32_t, uint64_t>::type;
      constexpr HitT kMask = L >= 32 ? static_cast<HitT>(~HitT{0}) : static_cast<HitT>((HitT{1} << L) - 1);
      const HitT hit = static_cast<HitT>(__ballot(in) >> base) & kMask;
      if (hit == 0) continue;
      any = true;
      if (in && io.src_rank == nullptr) mc = io.src_map[mc];
      // the hits compacted into the group's LDS slots in edge order (slot = hits on lower lanes), then
      // read back UM at a time with a broadcast read each -- no per-pick lane search and shuffles.  A
      // pick past the last hit adds fma(0, 0, acc) = acc + 0 = acc exactly (acc starts at +0 and an
      // exact-zero sum rounds to +0, so acc is never -0): the same bits as skipping it.
      int nh;
      if constexpr (L <= 32) {
        nh = __popc(hit);
        if (in) hb[__popc(hit & ((1u << gl) - 1u))] = make_int2(mc, __float_as_int(mv));
      } else {
        nh = __popcll(hit);
        if (in) hb[__popcll(hit & ((uint64_t{1} << gl) - 1))] = make_int2(mc, __float_as_int(mv));
      }
      wave_lds_order();
      for (int k0 = 0; k0 < nh; k0 += UM) {
        float4 xs[UM];
        float vs[UM];
#pragma unroll
        for (int k = 0; k < UM; ++k) {
          const bool ok = k0 + k < nh;
          const int2 e = hb[ok ? k0 + k : 0];
          vs[k] = ok ? __int_as_float(e.y) : 0.f;
          xs[k] = ok ? X4[row_off(e.x, ldx4u) + gl] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int k = 0; k < UM; ++k) fma4(vs[k], xs[k], acc);
      }
      wave_lds_order();  // every lane of the group has read the slots before the next chunk writes them
      continue;
    }
    if (gl < n) {
      mc = A.col[cb + gl];
      mv = A.val[cb + gl];
    }
    int j = 0;
    for (; j + U <= n; j += U) {
      // U source rows in flight, added in edge order
      float4 xs[U];
      float vs[U];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const int ck = __shfl(mc, base + j + k);
        vs[k] = __shfl(mv, base + j + k);
        xs[k] = X4[row_off(ck, ldx4u) + gl];
      }
#pragma unroll
      for (int k = 0; k < U; ++k) fma4(vs[k], xs[k], acc);
    }
    if (U > 8 && j + 8 <= n) {
      float4 xs[8];
      float vs[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int ck = __shfl(mc, base + j + k);
        vs[k] = __shfl(mv, base + j + k);
        xs[k] = X4[row_off(ck, ldx4u) + gl];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) fma4(vs[k], xs[k], acc);
      j += 8;
    }
    if (U > 4 && j + 4 <= n) {
      float4 xs[4];
      float vs[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int ck = __shfl(mc, base + j + k);
        vs[k] = __shfl(mv, base + j + k);
        xs[k] = X4[row_off(ck, ldx4u) + gl];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) fma4(vs[k], xs[k], acc);
      j += 4;
    }
    for (; j < n; ++j) {
      const int c = __shfl(mc, base + j);
      const float v = __shfl(mv, base + j);
      fma4(v, X4[row_off(c, ldx4u) + gl], acc);
    }
  }
}

}  // namespace kgat
