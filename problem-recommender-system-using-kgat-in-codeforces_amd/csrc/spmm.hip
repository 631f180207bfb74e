// a1 -- attentive-propagation SpMM over a CSR graph: Y = A . X (+ Y).
//
// Replaces torch.matmul(sparse attentive_matrix, ego) at
// src/model/KGAT/aggregator.py:54 (and its autograd A^T . G when called with
// the transposed CSR).  HBM-bound gather: per edge 4 B col + 4 B val + 4*d B
// of the source row.
//
// Layout of the work:
//  * a row of d floats is read as d/4 float4 lanes ("a group"); a wave holds
//    64/(d/4) groups, each owning one destination row at a time, so a wave
//    keeps up to 64/(d/4) gathered rows x unroll in flight;
//  * every group walks its row's edges in chunks of d/4: the group's lanes
//    load the chunk's (col, val) pairs cooperatively (one coalesced load
//    each), then broadcast them with ds_bpermute while the float4 row loads
//    are issued 4 at a time;
//  * rows with degree > long_threshold (power-law hubs: popular problems)
//    would serialise one group for thousands of edges, so they are cut into
//    seg_len-edge segments handled by whole waves (blocks scheduled first),
//    written as partial sums and reduced by a fix-up pass (one block per long
//    row).  Every output is produced in a fixed order: deterministic.
//
// Masked mode (the frontier backward of the last layer): the source rows are
// a compact buffer Xc indexed through src_map[node] (-1 = row is zero), so
// only edges into the frontier gather anything; the output is initialised
// from a compact Yc through the same map.  Skipped edges contribute exactly
// 0, so the result equals the dense product with zero rows.
#include "common.hpp"
#include "adam.hpp"
#include "spmm_core.hpp"

#include <hipcub/hipcub.hpp>

#include <algorithm>

namespace kgat {

// The p / m / v float4s of one table row segment (lane gl) for kMaskedAdam: every
// byte is touched once per step, so non-temporal (keeps the gathered rows cached).
struct AdamRow {
  floatx4 p, m, v;
};

__device__ __forceinline__ AdamRow adam_row_load(const SpmmAdam& a, int64_t row, int gl) {
  const int64_t o = row * a.ld + 4 * gl;
  return AdamRow{__builtin_nontemporal_load(reinterpret_cast<const floatx4*>(a.p + o)),
                 __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(a.m + o)),
                 __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(a.v + o))};
}

// Adam on one row segment with gradient g (misc.hip's adam_multi arithmetic, same bits).
__device__ __forceinline__ void adam_row_step(const SpmmAdam& a, int64_t row, int gl, float4 g, AdamRow r) {
  const float w1 = 1.f - a.b1, w2 = 1.f - a.b2;
  const float gg[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float pk = r.p[k], mk = r.m[k], vk = r.v[k];
    adam_elem(pk, gg[k], mk, vk, w1, a.b2, w2, a.step_size, a.bc2s, a.eps);
    r.p[k] = pk;
    r.m[k] = mk;
    r.v[k] = vk;
  }
  const int64_t o = row * a.ld + 4 * gl;
  __builtin_nontemporal_store(r.p, reinterpret_cast<floatx4*>(a.p + o));
  __builtin_nontemporal_store(r.m, reinterpret_cast<floatx4*>(a.m + o));
  __builtin_nontemporal_store(r.v, reinterpret_cast<floatx4*>(a.v + o));
}

// Final write of one output row segment (lane gl) in the five modes: row is
// the (global-id) row of A, out the row of Y it lands in (row, or its position
// in the output set for kMaskedRows).  kMaskedAdam writes no Y: the row is the
// gradient of table row `row` and goes straight into its Adam step.
template <int MODE>
__device__ __forceinline__ void store_row(const SpmmIo& io, int64_t row, int64_t out, int gl, float4 acc,
                                          bool any = false) {
  if (MODE == kMasked || MODE == kMaskedRows || MODE == kMaskedAdam) {
    if (io.Yc != nullptr || io.Gc != nullptr || (MODE == kMaskedRows && io.out_src != nullptr)) {
      const int m = io.src_map[io.row0 + row];
      if (m >= 0) {
        if (io.Yc != nullptr) {
          const float4 o = reinterpret_cast<const float4*>(io.Yc + static_cast<int64_t>(m) * io.ldyc)[gl];
          acc = make_float4(o.x + acc.x, o.y + acc.y, o.z + acc.z, o.w + acc.w);
        }
        if (MODE != kMaskedAdam && io.Gc != nullptr) {
          const float4 o = reinterpret_cast<const float4*>(io.Gc + static_cast<int64_t>(m) * io.ldgc)[gl];
          acc = make_float4(acc.x + o.x, acc.y + o.y, acc.z + o.z, acc.w + o.w);
        }
        any = true;
      }
      if (MODE == kMaskedRows && io.out_src != nullptr && gl == 0) io.out_src[out] = m;
    }
    if (MODE == kMasked && io.row_hit != nullptr && any && gl == 0) io.row_hit[row] = 1;
  }
  if (MODE == kMaskedAdam) {
    adam_row_step(io.adam, row, gl, acc, adam_row_load(io.adam, row, gl));
    return;
  }
  float4* y = reinterpret_cast<float4*>(io.Y + out * io.ldy) + gl;
  if (MODE == kAccumulate) {
    const float4 o = *y;
    acc = make_float4(o.x + acc.x, o.y + acc.y, o.z + acc.z, o.w + acc.w);
  }
  if (MODE == kOverwrite) {  // the dense product's output is written once: non-temporal, so the gathered table keeps the
                    // caches (C2 forward 0.555 -> 0.550 ms, full step 2.040 -> 2.025 ms, two interleaved A/B pairs)
    const floatx4 v = {acc.x, acc.y, acc.z, acc.w};
    __builtin_nontemporal_store(v, reinterpret_cast<floatx4*>(y));
    return;
  }
  *y = acc;
}

// Source rows in flight per lane group in the row-set forward (kRows); 4, 8 and 16 measured
// alike, the sum stays in edge order for any value.
constexpr int kRowsUnroll = 4;

// One long-row segment s (the whole wave; groups take interleaved sub-chunks) -> its partial sum in
// io.part, reduced by the fix-up pass.
template <int D, int MODE>
__device__ __forceinline__ void long_segment(const kgat_csr& A, const SpmmIo& io, int s, int g, int gl, int base,
                                             int2* hb) {
  constexpr int L = SpmmShape<D>::kLanes;
  constexpr bool MASKED = MODE == kMasked || MODE == kMaskedRows || MODE == kMaskedAdam;
  if (A.seg_order != nullptr) s = A.seg_order[s];  // launch slot -> segment (kgat_csr_seg_order)
  if (s >= A.n_seg) return;
  const int row = A.seg_row[s];
  if ((MODE == kMaskedRows || MODE == kRows) && !bit_of(io.out_bits, row)) return;  // not an output row
  const int64_t beg = A.seg_beg[s];
  const int64_t row_end = A.rowptr[row + 1];
  const int64_t nxt = s + 1 < A.n_seg ? A.seg_beg[s + 1] : row_end;  // segments tile each long row in order
  const int64_t end = nxt < row_end ? nxt : row_end;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  bool any = false;
  // group g handles edges [beg + g*L + k*64, ... + L) for k = 0, 1, ...
  for (int64_t cb = beg + g * L; cb < end; cb += kWave) {
    const int64_t ce = cb + L < end ? cb + L : end;
    gather_edges<D, MASKED>(A, io, cb, ce, base, gl, acc, any, hb);
  }
  // a long row is flagged by any of its segments that gathered (row_hit was zeroed)
  if (MODE == kMasked && io.row_hit != nullptr && any && gl == 0) io.row_hit[row] = 1;
#pragma unroll
  for (int o = L; o < kWave; o <<= 1) {
    acc.x += __shfl_xor(acc.x, o);
    acc.y += __shfl_xor(acc.y, o);
    acc.z += __shfl_xor(acc.z, o);
    acc.w += __shfl_xor(acc.w, o);
  }
  if (g == 0) reinterpret_cast<float4*>(io.part)[static_cast<int64_t>(s) * L + gl] = acc;
}

template <int D, int MODE>
__global__ __launch_bounds__(256) void spmm_main_kernel(kgat_csr A, SpmmIo io, int seg_blocks) {
  using S = SpmmShape<D>;
  constexpr int L = S::kLanes;
  constexpr bool MASKED = MODE == kMasked || MODE == kMaskedRows || MODE == kMaskedAdam;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int g = lane / L, gl = lane % L, base = g * L;
  if ((MODE == kMaskedAdam) && io.adam.skip != nullptr && *io.adam.skip != 0) return;
  __shared__ int2 hitbuf[4][kWave];  // masked modes: each lane group's compacted hits (gather_edges)
  int2* hb = hitbuf[wave] + base;

  if (static_cast<int>(blockIdx.x) < seg_blocks) {
    long_segment<D, MODE>(A, io, blockIdx.x * 4 + wave, g, gl, base, hb);
    return;
  }

  if (MODE == kMaskedRows || MODE == kRows) {
    // ---- short rows of the output set: one group per row, groups stride over the list one row
    // at a time (a set of ~10^4 rows keeps every group of the grid busy instead of a few waves
    // walking kRowsPerWave rows each; each row is still summed by one group in edge order)
    const int64_t cnt = *io.out_count;
    const int64_t stride = static_cast<int64_t>(gridDim.x - seg_blocks) * 4 * S::kGroups;
    {
      for (int64_t k = (static_cast<int64_t>(blockIdx.x - seg_blocks) * 4 + wave) * S::kGroups + g; k < cnt;
           k += stride) {
        const int64_t r = io.out_rows[k];
        if (MODE == kRows && r < 0) continue;  // padding of a frontier list
        const int64_t beg = A.rowptr[r], end = A.rowptr[r + 1];
        if (end - beg > A.long_threshold) continue;  // produced by the fix-up pass
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        bool any = false;
        gather_edges<D, MODE == kMaskedRows, MODE == kRows ? kRowsUnroll : 4>(A, io, beg, end, base, gl, acc, any,
                                                                              hb);
        store_row<MODE>(io, r, MODE == kRows ? r : k, gl, acc, any);
      }
    }
    return;
  }

  // ---- short rows: one group per row
  const int64_t w = static_cast<int64_t>(blockIdx.x - seg_blocks) * 4 + wave;
  const int64_t r_begin = w * S::kRowsPerWave;
  int64_t r_end = r_begin + S::kRowsPerWave;
  if (r_end > A.n_rows) r_end = A.n_rows;
  for (int64_t r = r_begin + g; r < r_end; r += S::kGroups) {
    const int64_t beg = A.rowptr[r], end = A.rowptr[r + 1];
    if (end - beg > A.long_threshold) continue;  // produced by the fix-up pass
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    bool any = false;
    if (MODE == kMaskedAdam) {
      // the row's p / m / v and its Yc row index are loaded before the gather (independent of it), so
      // their round trips overlap the gather chain instead of following it (76 VGPRs, 6 waves / SIMD:
      // table update 0.431 / 0.421 -> 0.421 / 0.417 ms in an interleaved A/B, tools/gpu_r04_ab.sh)
      const AdamRow pre = adam_row_load(io.adam, r, gl);
      const int ym = io.Yc != nullptr ? io.src_map[io.row0 + r] : -1;
      gather_edges<D, MASKED>(A, io, beg, end, base, gl, acc, any, hb);
      if (ym >= 0) {
        const float4 o = reinterpret_cast<const float4*>(io.Yc + static_cast<int64_t>(ym) * io.ldyc)[gl];
        acc = make_float4(o.x + acc.x, o.y + acc.y, o.z + acc.z, o.w + acc.w);
      }
      adam_row_step(io.adam, r, gl, acc, pre);
      continue;
    }
    gather_edges<D, MASKED>(A, io, beg, end, base, gl, acc, any, hb);
    store_row<MODE>(io, r, r, gl, acc, any);
  }
}

// Sum the segment partials of each long row.  One 256-thread block per long
// row: G = 256/(D/4) groups stride over the row's segments, then the group
// partials are added in group order through LDS -- a fixed order, so the
// result is deterministic, and a 196-segment hub row takes 13 steps, not 196.
template <int D, int MODE>
__device__ __forceinline__ void fixup_row(const kgat_csr& A, const SpmmIo& io, int lr) {
  constexpr int L = D / 4;
  constexpr int G = 256 / L;
  __shared__ float4 red[G][L];
  const int g = threadIdx.x / L, gl = threadIdx.x % L;
  const int row = A.long_rows[lr];
  if ((MODE == kMaskedRows || MODE == kRows) && !bit_of(io.out_bits, row)) return;  // block-uniform
  const float4* P = reinterpret_cast<const float4*>(io.part);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  const int s_end = A.long_seg_off[lr + 1];
  for (int s = A.long_seg_off[lr] + g; s < s_end; s += G) add4(acc, P[static_cast<int64_t>(s) * L + gl]);
  red[g][gl] = acc;
  __syncthreads();
  if (threadIdx.x < L) {
    float4 t = red[0][gl];
    for (int k = 1; k < G; ++k) add4(t, red[k][gl]);
    store_row<MODE>(io, row, MODE == kMaskedRows ? io.out_map[row] : row, gl, t);
  }
}

template <int D, int MODE>
__global__ __launch_bounds__(256) void spmm_fixup_kernel(kgat_csr A, SpmmIo io) {
  if ((MODE == kMaskedAdam) && io.adam.skip != nullptr && *io.adam.skip != 0) return;
  fixup_row<D, MODE>(A, io, blockIdx.x);
}

// The fused table update's fix-up launch carrying the step's other tensors (the aggregator weights): blocks
// [0, n_long) sum the long rows' partials into their Adam step, the rest run adam_multi_kernel<2>'s
// chunks of T (independent parameters; the same arithmetic and skip flag) -- one launch fewer per step.
template <int D>
__global__ __launch_bounds__(256) void spmm_fixup_adam_kernel(kgat_csr A, SpmmIo io, AdamTable T) {
  if (io.adam.skip != nullptr && *io.adam.skip != 0) return;
  if (static_cast<int64_t>(blockIdx.x) < A.n_long) {
    fixup_row<D, kMaskedAdam>(A, io, blockIdx.x);
    return;
  }
  adam_multi_chunks<2>(T, io.adam.b1, io.adam.b2, io.adam.eps, StepSched{nullptr, nullptr, nullptr},
                       0, blockIdx.x - A.n_long, gridDim.x - A.n_long);
}

template <int D, int MODE>
static int launch_mode(const kgat_csr& A, const SpmmIo& io, hipStream_t st) {
  using S = SpmmShape<D>;
  const int seg_blocks = (A.n_seg + 3) / 4;
  int64_t row_blocks = (A.n_rows + S::kRowsPerBlock - 1) / S::kRowsPerBlock;
  if ((MODE == kMaskedRows || MODE == kRows) && row_blocks > 2048) row_blocks = 2048;  // waves stride over the set (size on device)
  const int64_t grid = seg_blocks + row_blocks;
  if (grid > 0x7fffffff) return KGAT_ERR_INVALID;
  hipLaunchKernelGGL((spmm_main_kernel<D, MODE>), dim3(grid), dim3(256), 0, st, A, io, seg_blocks);
  KGAT_LAUNCH_CHECK();
  if (A.n_long > 0) {
    hipLaunchKernelGGL((spmm_fixup_kernel<D, MODE>), dim3(A.n_long), dim3(256), 0, st, A, io);
    KGAT_LAUNCH_CHECK();
  }
  return KGAT_OK;
}

template <int D>
static int launch_adam_multi(const kgat_csr& A, const SpmmIo& io, const AdamTable& T, hipStream_t st) {
  using S = SpmmShape<D>;
  const int seg_blocks = (A.n_seg + 3) / 4;
  const int64_t grid = seg_blocks + (A.n_rows + S::kRowsPerBlock - 1) / S::kRowsPerBlock;
  if (grid > 0x7fffffff) return KGAT_ERR_INVALID;
  hipLaunchKernelGGL((spmm_main_kernel<D, kMaskedAdam>), dim3(grid), dim3(256), 0, st, A, io, seg_blocks);
  KGAT_LAUNCH_CHECK();
  const int64_t fix = static_cast<int64_t>(A.n_long) + adam_grid(T);
  if (fix > 0) {
    hipLaunchKernelGGL((spmm_fixup_adam_kernel<D>), dim3(fix), dim3(256), 0, st, A, io, T);
    KGAT_LAUNCH_CHECK();
  }
  return KGAT_OK;
}

template <int MODE>
static int dispatch(const kgat_csr& A, const SpmmIo& io, int d, hipStream_t st) {
  switch (d) {
    case 16: return launch_mode<16, MODE>(A, io, st);
    case 32: return launch_mode<32, MODE>(A, io, st);
    case 64: return launch_mode<64, MODE>(A, io, st);
    case 128: return launch_mode<128, MODE>(A, io, st);
    case 256: return launch_mode<256, MODE>(A, io, st);
    default: return KGAT_ERR_UNSUPPORTED_DIM;
  }
}

static bool misaligned(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) != 0; }

// The first hop of the backward chain, structurally: bits0 marks the frontier
// rows F (rows[0..n) of kgat_frontier_build, -1 padded), bits1 marks F and
// every column of A's rows F -- exactly the rows the A^T product over F can
// reach (A^T[j, i] != 0 <=> A[i, j] != 0).  One block per frontier slot.
__global__ __launch_bounds__(256) void frontier_mark_kernel(kgat_csr A, const int32_t* __restrict__ rows,
                                                            uint32_t* __restrict__ bits0,
                                                            uint32_t* __restrict__ bits1) {
  const int32_t i = rows[blockIdx.x];
  if (i < 0) return;
  if (threadIdx.x == 0) {
    atomicOr(&bits0[i >> 5], 1u << (i & 31));
    atomicOr(&bits1[i >> 5], 1u << (i & 31));
  }
  for (int64_t e = A.rowptr[i] + threadIdx.x; e < A.rowptr[i + 1]; e += blockDim.x) {
    const int32_t j = A.col[e];
    const uint32_t b = 1u << (j & 31);
    // test before set (see cf_begin_kernel); a relaxed atomic load: the word is being OR-ed by other threads
    if ((__hip_atomic_load(&bits1[j >> 5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & b) == 0u)
      atomicOr(&bits1[j >> 5], b);
  }
}

// hit[r] = 1 for every row r of A that is itself in the set (bit row0 + r of bits) or has an edge
// into it (bit col): the next row set of the frontier chain, computed by the rows that pull from it
// (the row-sharded forward marks its rows of the first hop F + N(F) from its rows of A^T).  hit is
// zeroed by the caller; lanes only ever store 1.  Blocks [0, seg_blocks): one long-row segment per
// wave (64 lanes over <= seg_len edges); the rest: 16-lane groups, one short row each.
__global__ __launch_bounds__(256) void csr_mark_rows_kernel(kgat_csr A, const uint32_t* __restrict__ bits,
                                                            int64_t row0, int32_t* __restrict__ hit,
                                                            int seg_blocks) {
  if (static_cast<int>(blockIdx.x) < seg_blocks) {
    const int s = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (s >= A.n_seg) return;
    const int row = A.seg_row[s];
    const int64_t beg = A.seg_beg[s];
    const int64_t row_end = A.rowptr[row + 1];
    const int64_t nxt = s + 1 < A.n_seg ? A.seg_beg[s + 1] : row_end;
    const int64_t end = nxt < row_end ? nxt : row_end;
    for (int64_t e = beg + (threadIdx.x & 63); e < end; e += 64)
      if (bit_of(bits, A.col[e])) {
        hit[row] = 1;
        break;
      }
    return;
  }
  const int64_t r = (static_cast<int64_t>(blockIdx.x - seg_blocks) * 256 + threadIdx.x) >> 4;
  const int lane = threadIdx.x & 15;
  if (r >= A.n_rows) return;
  const int64_t beg = A.rowptr[r], end = A.rowptr[r + 1];
  if (lane == 0 && bit_of(bits, row0 + r)) hit[r] = 1;
  if (end - beg > A.long_threshold) return;  // the segment waves scan it
  for (int64_t e = beg + lane; e < end; e += 16)
    if (bit_of(bits, A.col[e])) {
      hit[r] = 1;
      break;
    }
}

// The set in a bitmap listed in one launch: node_map[i] = position of i among the members (ascending
// node order) or -1, rows[pos] = i, *count (and *count_host), rank words (kgat_map_rank's layout).
// Positions come from a single-pass scan of the word popcounts: each block takes kListWords words and a
// ticket (launch order, so every block it waits for is already running), publishes its popcount total
// as an 8-byte {tag | status | value} granule (one write-through agent-scope store, polled with
// agent-scope loads: self-contained, no fence), and looks back over its predecessors' granules for its
// prefix (decoupled look-back).  The tag is the launch's epoch + 1, so the granules of earlier launches
// never match and nothing is reset between launches; the last block to finish zeroes the ticket and
// advances the epoch.  state: uint32 [4] {ticket, done, epoch, -} + uint64 [blocks] granules, zero
// before the first launch (kgat_frontier_hop_work_bytes), never shared by concurrent launches.
constexpr int kListWords = 256;  // bitmap words (8192 nodes) per block

__device__ __forceinline__ uint64_t lb_granule(uint32_t tag, uint32_t status, int32_t v) {
  return (static_cast<uint64_t>(tag) << 34) | (static_cast<uint64_t>(status) << 32) | static_cast<uint32_t>(v);
}

__global__ __launch_bounds__(256) void bits_list_kernel(const uint32_t* __restrict__ bits, int64_t n, int64_t words,
                                                        int32_t* __restrict__ node_map, int32_t* __restrict__ rows,
                                                        int32_t* __restrict__ count, int32_t* __restrict__ count_host,
                                                        uint64_t* __restrict__ rank, uint32_t* __restrict__ state) {
  __shared__ uint32_t s_w[kListWords];
  __shared__ int32_t s_off[kListWords];
  __shared__ int32_t s_wsum[4];
  __shared__ int32_t s_blk, s_prefix;
  __shared__ uint32_t s_tag;
  uint64_t* granule = reinterpret_cast<uint64_t*>(state + 4);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) {
    s_blk = static_cast<int32_t>(__hip_atomic_fetch_add(&state[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    s_tag = (__hip_atomic_load(&state[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 0x3FFFFFFFu) + 1u;
  }
  __syncthreads();
  const int blk = s_blk;
  const uint32_t tag = s_tag;
  const int64_t w = static_cast<int64_t>(blk) * kListWords + tid;
  const uint32_t bw = w < words ? bits[w] : 0u;
  const int c = __popc(bw);
  int incl = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(incl, o);
    if (lane >= o) incl += v;
  }
  if (lane == 63) s_wsum[wave] = incl;
  s_w[tid] = bw;
  __syncthreads();
  int base = 0, agg = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (k < wave) base += s_wsum[k];
    agg += s_wsum[k];
  }
  if (wave == 0) {
    // look-back by the whole wave: lane i reads predecessor p_hi - i, 64 granules per round
    int32_t prefix = 0;
    if (lane == 0)
      __hip_atomic_store(&granule[blk], lb_granule(tag, blk == 0 ? 2u : 1u, agg), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    for (int p_hi = blk - 1; p_hi >= 0; p_hi -= 64) {
      const int p = p_hi - lane;
      uint64_t g = p >= 0 ? __hip_atomic_load(&granule[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                          : lb_granule(tag, 2u, 0);
      while (__any(static_cast<uint32_t>(g >> 34) != tag)) {
        __builtin_amdgcn_s_sleep(1);
        if (static_cast<uint32_t>(g >> 34) != tag)
          g = __hip_atomic_load(&granule[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      const uint64_t incl_lanes = __ballot(((g >> 32) & 3u) == 2u);
      const int lim = incl_lanes ? __ffsll(static_cast<long long>(incl_lanes)) - 1 : 63;
      int32_t v = lane <= lim ? static_cast<int32_t>(static_cast<uint32_t>(g)) : 0;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
      prefix += v;
      if (incl_lanes) break;
    }
    if (lane == 0) {
      if (blk > 0)
        __hip_atomic_store(&granule[blk], lb_granule(tag, 2u, prefix + agg), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      s_prefix = prefix;
      if (blk == static_cast<int>(gridDim.x) - 1) {
        *count = prefix + agg;
        // pinned host mirror (no copy launch), stored through to memory: the host reads it without an event
        if (count_host != nullptr)
          __hip_atomic_store(count_host, prefix + agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
  __syncthreads();
  const int32_t off = s_prefix + base + incl - c;
  s_off[tid] = off;
  if (rank != nullptr && w < words) rank[w] = (static_cast<uint64_t>(static_cast<uint32_t>(off)) << 32) | bw;
  __syncthreads();
  const int64_t node0 = static_cast<int64_t>(blk) * kListWords * 32;
  for (int q = tid; q < kListWords * 8; q += 256) {
    const int64_t nd = node0 + 4LL * q;
    if (nd >= n) break;
    const int wl = q >> 3, sh = (q & 7) * 4;
    const uint32_t wv = s_w[wl];
    int32_t pos = s_off[wl] + __popc(wv & ((1u << sh) - 1u));
    int32_t m[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool in = ((wv >> (sh + j)) & 1u) != 0;
      m[j] = in ? pos : -1;
      if (in) rows[pos++] = static_cast<int32_t>(nd + j);
    }
    if (nd + 4 <= n) {
      *reinterpret_cast<int4*>(node_map + nd) = make_int4(m[0], m[1], m[2], m[3]);
    } else {
      for (int j = 0; j < 4 && nd + j < n; ++j) node_map[nd + j] = m[j];
    }
  }
  __syncthreads();
  if (tid == 0 &&
      __hip_atomic_fetch_add(&state[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
    __hip_atomic_store(&state[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&state[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&state[2], tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

static int launch_bits_list(const uint32_t* bits, int64_t n, int32_t* node_map, int32_t* rows, int32_t* count,
                            int32_t* count_host, uint64_t* rank, void* work, hipStream_t st) {
  const int64_t words = (n + 31) / 32;
  const int64_t blocks = (words + kListWords - 1) / kListWords;
  if (blocks > 0x7fffffff) return KGAT_ERR_INVALID;
  hipLaunchKernelGGL(bits_list_kernel, dim3(blocks), dim3(256), 0, st, bits, n, words, node_map, rows, count,
                     count_host, rank, static_cast<uint32_t*>(work));
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

__global__ __launch_bounds__(256) void clear2_kernel(uint32_t* __restrict__ a, uint32_t* __restrict__ b, int64_t words) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < words) {
    a[i] = 0u;
    b[i] = 0u;
  }
}

// Frontier bitmap from a node map: bit i of the (64-bit) word i/64 = map[i] >= 0.
__global__ __launch_bounds__(256) void map_bits_kernel(const int32_t* __restrict__ node_map, int64_t n,
                                                       uint64_t* __restrict__ bits) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t b = __ballot(i < n && node_map[i] >= 0);
  if ((threadIdx.x & 63) == 0 && i < n) bits[i >> 6] = b;
}

// Rank words of a set given by an ascending-order node map (position = rank):
// word w = (position of its first member) << 32 | membership bits of nodes
// 32w .. 32w+31, so one 8-byte load answers both "in the set?" and "which
// compact row?" (position = hi + popcount of the lower member bits).
__global__ __launch_bounds__(256) void map_rank_kernel(const int32_t* __restrict__ node_map, int64_t n,
                                                       uint64_t* __restrict__ rank) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int32_t m = i < n ? node_map[i] : -1;
  const uint64_t b = __ballot(m >= 0);
  const int lane = threadIdx.x & 63;
  const uint32_t lo = static_cast<uint32_t>(b), hi = static_cast<uint32_t>(b >> 32);
  const int32_t p_lo = __shfl(m, lo ? __ffs(lo) - 1 : 0);
  const int32_t p_hi = __shfl(m, hi ? 32 + __ffs(hi) - 1 : 32);
  if (lane == 0 && i < n) {
    rank[i >> 5] = (static_cast<uint64_t>(lo ? static_cast<uint32_t>(p_lo) : 0u) << 32) | lo;
    if (i + 32 < n) rank[(i >> 5) + 1] = (static_cast<uint64_t>(hi ? static_cast<uint32_t>(p_hi) : 0u) << 32) | hi;
  }
}

// Hop set from the masked product's row flags: pos = exclusive scan of hit
// (already in node_map); a flagged node keeps its position and is listed in
// rows[pos], an unflagged one gets -1.  Thread i alone rewrites node_map[i],
// so the last thread can read its own scan value for the count first.
__global__ __launch_bounds__(256) void hop_finish_kernel(const int32_t* __restrict__ hit, int64_t n,
                                                         int32_t* __restrict__ node_map, int32_t* __restrict__ rows,
                                                         int32_t* __restrict__ count, int32_t* __restrict__ count_host) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t pos = node_map[i];
  const bool h = hit[i] != 0;
  if (i == n - 1) {
    *count = pos + (h ? 1 : 0);
    if (count_host != nullptr)
      __hip_atomic_store(count_host, pos + (h ? 1 : 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (h) {
    rows[pos] = static_cast<int32_t>(i);
  } else {
    node_map[i] = -1;
  }
}

// Union of G row lists (list g = lists[g*cap .. g*cap + counts[g])): bit of every listed row.
__global__ __launch_bounds__(256) void lists_mark_kernel(const int32_t* __restrict__ lists,
                                                         const int32_t* __restrict__ counts, int32_t cap,
                                                         int64_t total, int64_t n, uint32_t* __restrict__ bits) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int64_t g = i / cap;
  if (i - g * cap >= counts[g]) return;  // (a count past cap reads nothing beyond list g: i - g * cap < cap)
  const int32_t r = lists[i];
  if (r >= 0 && r < n) atomicOr(&bits[r >> 5], 1u << (r & 31));
}

// out[k] = scale * (sum over g = 0..G-1 of vals[g*cap + pos_g(rows[k])]), pos_g = position of
// rows[k] in list g (ascending; binary search by lane g), lists without the row skipped.
// One wave per union row, w/4 lanes of float4; the sum runs in list order on every replica
// alike, so every rank merging the same all-gathered lists gets the same bits.
__global__ __launch_bounds__(256) void lists_merge_kernel(const int32_t* __restrict__ lists,
                                                          const int32_t* __restrict__ counts, int32_t G,
                                                          int32_t cap, const float* __restrict__ vals, int64_t ldv,
                                                          int32_t w, const int32_t* __restrict__ rows,
                                                          const int32_t* __restrict__ count, int64_t max_rows,
                                                          float* __restrict__ out, int64_t ldo, float scale) {
  __shared__ int32_t spos[4][64];  // per wave: the row's position in each list (-1: absent)
  const int lane = threadIdx.x & 63;
  int32_t* wpos = spos[threadIdx.x >> 6];
  const int64_t waves = static_cast<int64_t>(gridDim.x) * (blockDim.x >> 6);
  const int64_t nrows = min(static_cast<int64_t>(*count), max_rows);
  for (int64_t k = static_cast<int64_t>(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6); k < nrows;
       k += waves) {
    const int32_t node = rows[k];
    int32_t pos = -1;
    if (lane < G) {  // lane g: lower bound of node in list g
      const int32_t* lg = lists + static_cast<int64_t>(lane) * cap;
      const int32_t cnt = min(max(counts[lane], 0), cap);  // a corrupt gathered count stays inside list g
      int32_t lo = 0, hi = cnt;
      while (lo < hi) {
        const int32_t mid = (lo + hi) >> 1;
        if (lg[mid] < node) lo = mid + 1; else hi = mid;
      }
      if (lo < cnt && lg[lo] == node) pos = lo;
    }
    wpos[lane] = pos;
    __builtin_amdgcn_wave_barrier();
    for (int c = lane * 4; c < w; c += 256) {
      floatx4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int g = 0; g < G; ++g) {
        const int32_t p = wpos[g];
        if (p < 0) continue;
        const floatx4 v = *reinterpret_cast<const floatx4*>(vals + (static_cast<int64_t>(g) * cap + p) * ldv + c);
        acc += v;
      }
      *reinterpret_cast<floatx4*>(out + k * ldo + c) = acc * scale;
    }
    __builtin_amdgcn_wave_barrier();  // wpos is rewritten for the wave's next row
  }
}

}  // namespace kgat

extern "C" int kgat_spmm_csr_f32(const kgat_csr* A, const float* X, int64_t ldx, float* Y, int64_t ldy,
                                 int32_t d, int32_t accumulate, float* workspace, int64_t workspace_floats,
                                 void* stream) {
  using namespace kgat;
  if (!A || !X || !Y || A->n_rows < 0 || ldx < d || ldy < d || (ldx & 3) || (ldy & 3)) return KGAT_ERR_INVALID;
  if (misaligned(X) || misaligned(Y)) return KGAT_ERR_INVALID;
  if (A->n_rows == 0) return KGAT_OK;
  if (A->n_seg > 0 && (workspace == nullptr || workspace_floats < static_cast<int64_t>(A->n_seg) * d))
    return KGAT_ERR_WORKSPACE;
  const SpmmIo io{X, ldx, Y, ldy, workspace, nullptr, nullptr, 0, nullptr, 0, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  return accumulate ? dispatch<kAccumulate>(*A, io, d, st) : dispatch<kOverwrite>(*A, io, d, st);
}

extern "C" int kgat_spmm_csr_masked_ex_f32(const kgat_csr* A, const int32_t* src_map, const float* Xc, int64_t ldxc,
                                           const float* Yc_init, int64_t ldyc, int64_t yc_row0, float* Y, int64_t ldy,
                                           int32_t d, int32_t* row_hit, const uint32_t* src_bits,
                                           const uint64_t* src_rank, int64_t n_src, float* workspace,
                                           int64_t workspace_floats, void* stream) {
  using namespace kgat;
  if (!A || !src_map || !Xc || !Y || A->n_rows < 0 || ldxc < d || ldy < d || (ldxc & 3) || (ldy & 3) || yc_row0 < 0)
    return KGAT_ERR_INVALID;
  if (misaligned(Xc) || misaligned(Y) || (Yc_init && (misaligned(Yc_init) || ldyc < d || (ldyc & 3))))
    return KGAT_ERR_INVALID;
  if (A->n_rows == 0) return KGAT_OK;
  if (A->n_seg > 0 && (workspace == nullptr || workspace_floats < static_cast<int64_t>(A->n_seg) * d))
    return KGAT_ERR_WORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (row_hit != nullptr &&
      hipMemsetAsync(row_hit, 0, static_cast<size_t>(A->n_rows) * sizeof(int32_t), st) != hipSuccess)
    return KGAT_ERR_INVALID;
  const SpmmIo io{Xc, ldxc, Y, ldy, workspace, src_map, Yc_init, ldyc, row_hit, yc_row0, src_bits, src_rank, nullptr, nullptr, nullptr, nullptr};
  (void)n_src;  // reserved: source-set size (an LDS-staged variant measured slower)
  return dispatch<kMasked>(*A, io, d, st);
}

extern "C" int kgat_spmm_csr_masked_f32(const kgat_csr* A, const int32_t* src_map, const float* Xc, int64_t ldxc,
                                        const float* Yc_init, int64_t ldyc, float* Y, int64_t ldy, int32_t d,
                                        float* workspace, int64_t workspace_floats, void* stream) {
  return kgat_spmm_csr_masked_ex_f32(A, src_map, Xc, ldxc, Yc_init, ldyc, 0, Y, ldy, d, nullptr, nullptr, nullptr, 0,
                                     workspace, workspace_floats, stream);
}

extern "C" int kgat_spmm_csr_masked_adam_f32(const kgat_csr* A, const int32_t* src_map, const float* Xc,
                                             int64_t ldxc, const float* Yc_init, int64_t ldyc,
                                             const uint64_t* src_rank, float* p, float* m, float* v, int64_t ldp,
                                             int32_t d, float step_size, float beta1, float beta2, float bc2_sqrt,
                                             float eps, float* workspace, int64_t workspace_floats, void* stream) {
  return kgat_spmm_csr_masked_adam_ex_f32(A, src_map, Xc, ldxc, Yc_init, ldyc, src_rank, p, m, v, ldp, d, step_size,
                                          beta1, beta2, bc2_sqrt, eps, nullptr, workspace, workspace_floats, stream);
}

extern "C" int kgat_spmm_csr_masked_adam_ex_f32(const kgat_csr* A, const int32_t* src_map, const float* Xc,
                                                int64_t ldxc, const float* Yc_init, int64_t ldyc,
                                                const uint64_t* src_rank, float* p, float* m, float* v, int64_t ldp,
                                                int32_t d, float step_size, float beta1, float beta2, float bc2_sqrt,
                                                float eps, const int32_t* skip, float* workspace,
                                                int64_t workspace_floats, void* stream) {
  return kgat_spmm_csr_masked_adam_block_f32(A, src_map, Xc, ldxc, Yc_init, ldyc, 0, src_rank, p, m, v, ldp, d,
                                             step_size, beta1, beta2, bc2_sqrt, eps, skip, workspace,
                                             workspace_floats, stream);
}

extern "C" int kgat_spmm_csr_masked_adam_multi_f32(const kgat_csr* A, const int32_t* src_map, const float* Xc,
                                                   int64_t ldxc, const float* Yc_init, int64_t ldyc,
                                                   const uint64_t* src_rank, float* p, float* m, float* v, int64_t ldp,
                                                   int32_t d, float step_size, float beta1, float beta2,
                                                   float bc2_sqrt, float eps, const int32_t* skip, float* workspace,
                                                   int64_t workspace_floats, const kgat_adam_tensor* extra,
                                                   int32_t n_extra, void* stream) {
  using namespace kgat;
  if (n_extra == 0)
    return kgat_spmm_csr_masked_adam_ex_f32(A, src_map, Xc, ldxc, Yc_init, ldyc, src_rank, p, m, v, ldp, d,
                                            step_size, beta1, beta2, bc2_sqrt, eps, skip, workspace,
                                            workspace_floats, stream);
  AdamTable T{};
  if (int e = adam_table(extra, n_extra, T)) return e;
  if (!A || !src_map || !Xc || !p || !m || !v || A->n_rows <= 0 || ldxc < d || ldp < d || (ldxc & 3) || (ldp & 3))
    return KGAT_ERR_INVALID;
  if (misaligned(Xc) || misaligned(p) || misaligned(m) || misaligned(v) ||
      (Yc_init && (misaligned(Yc_init) || ldyc < d || (ldyc & 3))))
    return KGAT_ERR_INVALID;
  if (src_rank != nullptr && (reinterpret_cast<uintptr_t>(src_rank) & 7)) return KGAT_ERR_INVALID;
  if (A->n_seg > 0 && (workspace == nullptr || workspace_floats < static_cast<int64_t>(A->n_seg) * d))
    return KGAT_ERR_WORKSPACE;
  SpmmIo io{Xc, ldxc, nullptr, 0, workspace, src_map, Yc_init, ldyc, nullptr, 0, nullptr, src_rank,
            nullptr, nullptr, nullptr, nullptr};
  io.adam = SpmmAdam{p, m, v, ldp, step_size, beta1, beta2, bc2_sqrt, eps, skip};
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  switch (d) {
    case 16: return launch_adam_multi<16>(*A, io, T, st);
    case 32: return launch_adam_multi<32>(*A, io, T, st);
    case 64: return launch_adam_multi<64>(*A, io, T, st);
    case 128: return launch_adam_multi<128>(*A, io, T, st);
    case 256: return launch_adam_multi<256>(*A, io, T, st);
    default: return KGAT_ERR_UNSUPPORTED_DIM;
  }
}

extern "C" int kgat_spmm_csr_masked_adam_block_f32(const kgat_csr* A, const int32_t* src_map, const float* Xc,
                                                   int64_t ldxc, const float* Yc_init, int64_t ldyc, int64_t yc_row0,
                                                   const uint64_t* src_rank, float* p, float* m, float* v, int64_t ldp,
                                                   int32_t d, float step_size, float beta1, float beta2,
                                                   float bc2_sqrt, float eps, const int32_t* skip, float* workspace,
                                                   int64_t workspace_floats, void* stream) {
  using namespace kgat;
  if (yc_row0 < 0) return KGAT_ERR_INVALID;
  if (!A || !src_map || !Xc || !p || !m || !v || A->n_rows < 0 || ldxc < d || ldp < d || (ldxc & 3) || (ldp & 3))
    return KGAT_ERR_INVALID;
  if (misaligned(Xc) || misaligned(p) || misaligned(m) || misaligned(v) ||
      (Yc_init && (misaligned(Yc_init) || ldyc < d || (ldyc & 3))))
    return KGAT_ERR_INVALID;
  if (src_rank != nullptr && (reinterpret_cast<uintptr_t>(src_rank) & 7)) return KGAT_ERR_INVALID;
  if (A->n_rows == 0) return KGAT_OK;
  if (A->n_seg > 0 && (workspace == nullptr || workspace_floats < static_cast<int64_t>(A->n_seg) * d))
    return KGAT_ERR_WORKSPACE;
  SpmmIo io{Xc, ldxc, nullptr, 0, workspace, src_map, Yc_init, ldyc, nullptr, yc_row0, nullptr, src_rank,
            nullptr, nullptr, nullptr, nullptr};
  io.adam = SpmmAdam{p, m, v, ldp, step_size, beta1, beta2, bc2_sqrt, eps, skip};
  return dispatch<kMaskedAdam>(*A, io, d, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int64_t kgat_hop_compact_work_bytes(int64_t n) {
  if (n < 0 || n > INT32_MAX) return -1;
  size_t bytes = 0;
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, static_cast<const int32_t*>(nullptr),
                                       static_cast<int32_t*>(nullptr), static_cast<int>(n)) != hipSuccess)
    return -1;
  return static_cast<int64_t>(bytes > 0 ? bytes : 1);
}

extern "C" int kgat_hop_compact(const int32_t* hit, int64_t n, int32_t* node_map, int32_t* rows, int32_t* count,
                                int32_t* count_host, void* work, int64_t work_bytes, void* stream) {
  if (!hit || !node_map || !rows || !count || n < 0 || n > INT32_MAX) return KGAT_ERR_INVALID;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (n == 0) {
    if (count_host != nullptr) *count_host = 0;
    return hipMemsetAsync(count, 0, sizeof(int32_t), st) == hipSuccess ? KGAT_OK : KGAT_ERR_INVALID;
  }
  const int64_t need = kgat_hop_compact_work_bytes(n);
  if (need < 0 || !work || work_bytes < need) return KGAT_ERR_WORKSPACE;
  size_t bytes = static_cast<size_t>(need);
  const hipError_t e = hipcub::DeviceScan::ExclusiveSum(work, bytes, hit, node_map, static_cast<int>(n), st);
  if (e != hipSuccess) return static_cast<int>(e);
  hipLaunchKernelGGL(kgat::hop_finish_kernel, dim3((n + 255) / 256), dim3(256), 0, st, hit, n, node_map, rows, count,
                     count_host);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int kgat_map_bits(const int32_t* node_map, int64_t n, uint32_t* bits, void* stream) {
  if (!node_map || !bits || n < 0) return KGAT_ERR_INVALID;
  if (reinterpret_cast<uintptr_t>(bits) & 7) return KGAT_ERR_INVALID;
  if (n == 0) return KGAT_OK;
  hipLaunchKernelGGL(kgat::map_bits_kernel, dim3((n + 255) / 256), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     node_map, n, reinterpret_cast<uint64_t*>(bits));
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

// Scratch of kgat_frontier_hop / kgat_rows_union: bits_list_kernel's scan state (zero before the
// first call, left reusable by every call).
extern "C" int64_t kgat_frontier_hop_work_bytes(int64_t n) {
  if (n < 0 || n > INT32_MAX) return -1;
  const int64_t words = (n + 31) / 32;
  return 16 + 8 * ((words + kgat::kListWords - 1) / kgat::kListWords + 1);
}

extern "C" int kgat_frontier_hop_ex(const kgat_csr* A, const int32_t* rows0, int32_t n0, uint32_t* bits0,
                                    uint32_t* bits1, int32_t* node_map, int32_t* hop_rows, int32_t* hop_count,
                                    int32_t* hop_count_host, uint64_t* hop_rank, void* work, int64_t work_bytes,
                                    int32_t flags, void* stream) {
  if (!A || !rows0 || !bits0 || !bits1 || !node_map || !hop_rows || !hop_count || n0 < 0 || A->n_rows < 0 ||
      (flags & ~KGAT_HOP_PRECLEARED))
    return KGAT_ERR_INVALID;
  const int64_t n = A->n_rows;
  const int64_t need = kgat_frontier_hop_work_bytes(n);
  if (need < 0 || !work || work_bytes < need || (reinterpret_cast<uintptr_t>(work) & 7)) return KGAT_ERR_WORKSPACE;
  if (hop_rank != nullptr && (reinterpret_cast<uintptr_t>(hop_rank) & 7)) return KGAT_ERR_INVALID;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t words = (n + 31) / 32;
  if (n == 0) return hipMemsetAsync(hop_count, 0, 4, st) == hipSuccess ? KGAT_OK : KGAT_ERR_INVALID;
  if (!(flags & KGAT_HOP_PRECLEARED)) {
    hipLaunchKernelGGL(kgat::clear2_kernel, dim3((words + 255) / 256), dim3(256), 0, st, bits0, bits1, words);
    KGAT_LAUNCH_CHECK();
  }
  if (n0 > 0) {
    hipLaunchKernelGGL(kgat::frontier_mark_kernel, dim3(n0), dim3(256), 0, st, *A, rows0, bits0, bits1);
    KGAT_LAUNCH_CHECK();
  }
  return kgat::launch_bits_list(bits1, n, node_map, hop_rows, hop_count, hop_count_host, hop_rank, work, st);
}

extern "C" int kgat_frontier_hop(const kgat_csr* A, const int32_t* rows0, int32_t n0, uint32_t* bits0,
                                 uint32_t* bits1, int32_t* node_map, int32_t* hop_rows, int32_t* hop_count,
                                 int32_t* hop_count_host, uint64_t* hop_rank, void* work, int64_t work_bytes,
                                 void* stream) {
  return kgat_frontier_hop_ex(A, rows0, n0, bits0, bits1, node_map, hop_rows, hop_count, hop_count_host, hop_rank,
                              work, work_bytes, 0, stream);
}

extern "C" int kgat_spmm_csr_masked_rows_ex_f32(const kgat_csr* A, const int32_t* src_map, const uint32_t* src_bits,
                                                const float* Xc, int64_t ldxc, const float* Yc_init, int64_t ldyc,
                                                const float* Gc, int64_t ldgc, const uint32_t* out_bits,
                                                const int32_t* out_map, const int32_t* out_rows,
                                                const int32_t* out_count, float* Y, int64_t ldy, int32_t* out_src,
                                                int32_t d, float* workspace, int64_t workspace_floats, void* stream) {
  using namespace kgat;
  if (!A || !src_map || !Xc || !Y || !out_bits || !out_map || !out_rows || !out_count || A->n_rows < 0 || ldxc < d ||
      ldy < d || (ldxc & 3) || (ldy & 3))
    return KGAT_ERR_INVALID;
  if (misaligned(Xc) || misaligned(Y) || (Yc_init && (misaligned(Yc_init) || ldyc < d || (ldyc & 3))) ||
      (Gc && (misaligned(Gc) || ldgc < d || (ldgc & 3))))
    return KGAT_ERR_INVALID;
  if (A->n_rows == 0) return KGAT_OK;
  if (A->n_seg > 0 && (workspace == nullptr || workspace_floats < static_cast<int64_t>(A->n_seg) * d))
    return KGAT_ERR_WORKSPACE;
  SpmmIo io{Xc, ldxc, Y, ldy, workspace, src_map, Yc_init, ldyc, nullptr, 0, src_bits, nullptr,
            out_bits, out_map, out_rows, out_count};
  io.Gc = Gc;
  io.ldgc = ldgc;
  io.out_src = out_src;
  return dispatch<kMaskedRows>(*A, io, d, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int kgat_spmm_csr_masked_rows_f32(const kgat_csr* A, const int32_t* src_map, const uint32_t* src_bits,
                                             const float* Xc, int64_t ldxc, const float* Yc_init, int64_t ldyc,
                                             const uint32_t* out_bits, const int32_t* out_map, const int32_t* out_rows,
                                             const int32_t* out_count, float* Y, int64_t ldy, int32_t d,
                                             float* workspace, int64_t workspace_floats, void* stream) {
  return kgat_spmm_csr_masked_rows_ex_f32(A, src_map, src_bits, Xc, ldxc, Yc_init, ldyc, nullptr, 0, out_bits, out_map,
                                          out_rows, out_count, Y, ldy, nullptr, d, workspace, workspace_floats, stream);
}

extern "C" int kgat_spmm_csr_rows_f32(const kgat_csr* A, const float* X, int64_t ldx, const uint32_t* out_bits,
                                      const int32_t* out_rows, const int32_t* out_count, float* Y, int64_t ldy,
                                      int32_t d, float* workspace, int64_t workspace_floats, void* stream) {
  using namespace kgat;
  if (!A || !X || !Y || !out_bits || !out_rows || !out_count || A->n_rows < 0 || ldx < d || ldy < d || (ldx & 3) ||
      (ldy & 3))
    return KGAT_ERR_INVALID;
  if (misaligned(X) || misaligned(Y)) return KGAT_ERR_INVALID;
  if (A->n_rows == 0) return KGAT_OK;
  if (A->n_seg > 0 && (workspace == nullptr || workspace_floats < static_cast<int64_t>(A->n_seg) * d))
    return KGAT_ERR_WORKSPACE;
  const SpmmIo io{X, ldx, Y, ldy, workspace, nullptr, nullptr, 0, nullptr, 0, nullptr, nullptr,
                  out_bits, nullptr, out_rows, out_count};
  return dispatch<kRows>(*A, io, d, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int kgat_csr_mark_rows(const kgat_csr* A, const uint32_t* bits, int64_t n_bits, int64_t row0,
                                  int32_t* hit, void* stream) {
  if (!A || !bits || !hit || A->n_rows < 0 || row0 < 0 || n_bits < row0 + A->n_rows) return KGAT_ERR_INVALID;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (A->n_rows == 0) return KGAT_OK;
  if (hipMemsetAsync(hit, 0, static_cast<size_t>(A->n_rows) * sizeof(int32_t), st) != hipSuccess)
    return KGAT_ERR_INVALID;
  const int seg_blocks = (A->n_seg + 3) / 4;
  const int64_t grid = seg_blocks + (A->n_rows + 15) / 16;
  if (grid > 0x7fffffff) return KGAT_ERR_INVALID;
  hipLaunchKernelGGL(kgat::csr_mark_rows_kernel, dim3(grid), dim3(256), 0, st, *A, bits, row0, hit, seg_blocks);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int kgat_map_rank(const int32_t* node_map, int64_t n, uint64_t* rank, void* stream) {
  if (!node_map || !rank || n < 0) return KGAT_ERR_INVALID;
  if (reinterpret_cast<uintptr_t>(rank) & 7) return KGAT_ERR_INVALID;
  if (n == 0) return KGAT_OK;
  hipLaunchKernelGGL(kgat::map_rank_kernel, dim3((n + 255) / 256), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     node_map, n, rank);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

// Union of the G replicas' hop sets (data-parallel exchange of the compact
// table gradient, replicas.ShardedGradSync): the bitmap of every listed row,
// then kgat_frontier_hop's popcount scan and finish (sorted rows, node map,
// count, rank words).  work: kgat_frontier_hop_work_bytes(n) bytes.
extern "C" int kgat_rows_union(const int32_t* lists, const int32_t* counts, int32_t G, int32_t cap, int64_t n,
                               uint32_t* bits, int32_t* node_map, int32_t* rows, int32_t* count, uint64_t* rank,
                               void* work, int64_t work_bytes, void* stream) {
  if (!counts || !bits || !node_map || !rows || !count || G < 1 || cap < 0 || n < 0) return KGAT_ERR_INVALID;
  if (cap > 0 && !lists) return KGAT_ERR_INVALID;
  if (rank != nullptr && (reinterpret_cast<uintptr_t>(rank) & 7)) return KGAT_ERR_INVALID;
  const int64_t need = kgat_frontier_hop_work_bytes(n);
  if (need < 0 || !work || work_bytes < need || (reinterpret_cast<uintptr_t>(work) & 7)) return KGAT_ERR_WORKSPACE;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (n == 0) return hipMemsetAsync(count, 0, 4, st) == hipSuccess ? KGAT_OK : KGAT_ERR_INVALID;
  const int64_t words = (n + 31) / 32;
  if (hipMemsetAsync(bits, 0, 4 * words, st) != hipSuccess) return KGAT_ERR_INVALID;
  const int64_t total = static_cast<int64_t>(G) * cap;
  if (total > 0) {
    hipLaunchKernelGGL(kgat::lists_mark_kernel, dim3((total + 255) / 256), dim3(256), 0, st, lists, counts, cap,
                       total, n, bits);
    KGAT_LAUNCH_CHECK();
  }
  return kgat::launch_bits_list(bits, n, node_map, rows, count, nullptr, rank, work, st);
}

extern "C" int kgat_rows_merge_f32(const int32_t* lists, const int32_t* counts, int32_t G, int32_t cap,
                                   const float* vals, int64_t ldv, int32_t w, const int32_t* rows,
                                   const int32_t* count, int64_t max_rows, float* out, int64_t ldo, float scale,
                                   void* stream) {
  if (!counts || !rows || !count || !out || G < 1 || G > 64 || cap < 0 || w < 0 || max_rows < 0)
    return KGAT_ERR_INVALID;
  if ((w & 3) || (ldo & 3) || ldo < w || kgat::misaligned(out)) return KGAT_ERR_INVALID;
  if (cap > 0 && (!lists || !vals || (ldv & 3) || ldv < w || kgat::misaligned(vals))) return KGAT_ERR_INVALID;
  if (max_rows == 0 || w == 0) return KGAT_OK;
  const int64_t blocks = std::min<int64_t>((max_rows + 3) / 4, 8192);
  hipLaunchKernelGGL(kgat::lists_merge_kernel, dim3(blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     lists, counts, G, cap, vals, ldv, w, rows, count, max_rows, out, ldo, scale);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}
