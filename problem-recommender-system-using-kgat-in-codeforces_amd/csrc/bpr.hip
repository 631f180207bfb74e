// a3/a4 -- CF BPR loss over gathered rows of the propagated tables
// (src/model/KGAT/model.py:165-202):
//   pos_b = <u_b, p_b>, neg_b = <u_b, n_b> over the concatenated width D,
//   L = mean_b softplus(neg_b - pos_b) + reg * (l2(U) + l2(P) + l2(N)),
//   l2(X) = mean_b sum_j X_bj^2 / 2.
// Item ids index the user+entity table raw (not offset by user_num), exactly
// as model.py:189-191 does.  The tables are never concatenated: each layer's
// output stays its own buffer and the gather walks the table list.
#include "common.hpp"

namespace kgat {

__device__ __forceinline__ float row_val(const kgat_tables& T, int t, int64_t id, int j) {
  return T.ptr[t][id * T.ld[t] + j];
}

// One wave per sample: the per-sample loss term goes to term[b] and
// coef[b] = sigmoid(pos_b - neg_b) - 1 is kept for the backward; the loss is
// sum(term) / batch in index order (deterministic) -- by a second single-block
// kernel, or (ticket != nullptr) by the block that finishes last: every block
// publishes its terms with write-through (sc1) stores, drains them and takes a
// ticket (agent-scope atomic add); the block whose add returns gridDim.x - 1
// sums term[] with sc1 loads and leaves the ticket 0 again.
__device__ __forceinline__ void bpr_loss_sum(const float* __restrict__ term, int batch, float* __restrict__ loss,
                                             float* red, bool coherent) {
  float s = 0.f;
  for (int b = threadIdx.x; b < batch; b += 256)
    s += coherent ? __uint_as_float(__hip_atomic_load(reinterpret_cast<const uint32_t*>(term + b), __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT))
                  : term[b];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (static_cast<int>(threadIdx.x) < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) *loss = red[0] / static_cast<float>(batch);
}

__global__ __launch_bounds__(256) void bpr_fwd_kernel(kgat_tables T, const int64_t* __restrict__ users,
                                                      const int64_t* __restrict__ pos,
                                                      const int64_t* __restrict__ neg, int batch, float reg,
                                                      float* __restrict__ coef, float* __restrict__ term,
                                                      uint32_t* __restrict__ ticket, float* __restrict__ loss) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b < batch) {
    const int64_t u = users[b], p = pos[b], n = neg[b];
    float sp = 0.f, sn = 0.f, qu = 0.f, qp = 0.f, qn = 0.f;
    for (int t = 0; t < T.count; ++t) {
      for (int j = lane; j < T.width[t]; j += 64) {
        const float xu = row_val(T, t, u, j), xp = row_val(T, t, p, j), xn = row_val(T, t, n, j);
        sp = fmaf(xu, xp, sp);
        sn = fmaf(xu, xn, sn);
        qu = fmaf(xu, xu, qu);
        qp = fmaf(xp, xp, qp);
        qn = fmaf(xn, xn, qn);
      }
    }
    sp = wave_sum(sp);
    sn = wave_sum(sn);
    qu = wave_sum(qu);
    qp = wave_sum(qp);
    qn = wave_sum(qn);
    const float x = sp - sn;
    // -logsigmoid(x) = softplus(-x), computed stably
    const float nls = fmaxf(-x, 0.f) + log1pf(expf(-fabsf(x)));
    if (lane == 0) {
      coef[b] = 1.f / (1.f + expf(-x)) - 1.f;
      const float tv = nls + reg * 0.5f * (qu + qp + qn);
      if (ticket != nullptr)
        __hip_atomic_store(reinterpret_cast<uint32_t*>(term + b), __float_as_uint(tv), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      else
        term[b] = tv;
    }
  }
  if (ticket == nullptr) return;  // grid-uniform
  __shared__ float red[256];
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's term store has completed
  __syncthreads();
  // acq_rel: releases this block's term stores to every XCD's L2 before its arrival counts, and the last
  // arrival acquires every other block's before the sum reads them (the memory model, not the s_waitcnt)
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;  // block-uniform
  bpr_loss_sum(term, batch, loss, red, true);
  if (threadIdx.x == 0) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(256) void bpr_sum_kernel(const float* __restrict__ term, int batch,
                                                      float* __restrict__ loss) {
  __shared__ float red[256];
  bpr_loss_sum(term, batch, loss, red, false);
}

// Unique ids of the batch [users | pos | neg] in first-occurrence order:
// rows[0..count) = ids, node_map[id] = its position, rows[count..3B) = -1.
// node_map must hold -1 for every node on entry (kgat_frontier_reset restores
// it).  O(slots): the first slot of every id is elected in an LDS hash table, a
// block scan numbers the winners in slot order, and the winners write
// node_map[id] = position.  One 1024-thread block; thread tid owns the
// contiguous slots [tid*kSlotsPer, tid*kSlotsPer + kSlotsPer).
constexpr int kBatchSlots = 4096;
constexpr int kSlotsPer = kBatchSlots / 1024;

// The distinct ids are found in an LDS hash table (open addressing, 2 * kBatchSlots entries: the id
// claims an entry with a CAS, then the smallest slot holding it wins an atomicMin), so node_map sees
// plain stores only -- one global round trip instead of three (global atomicMin, agent-scope reload,
// store).  Ids are node ids < 2^31.
constexpr int kHashSize = 2 * kBatchSlots;

__device__ __forceinline__ void number_batch(const int64_t (&ids)[kSlotsPer], int slots,
                                             int32_t* __restrict__ node_map, int32_t* __restrict__ rows,
                                             int32_t* __restrict__ count) {
  __shared__ int32_t wsum[16];
  __shared__ int32_t hkey[kHashSize];
  __shared__ int32_t hslot[kHashSize];
  const int tid = threadIdx.x;
  for (int i = tid; i < kHashSize; i += 1024) {
    hkey[i] = -1;
    hslot[i] = 0x7fffffff;
  }
  __syncthreads();
  int hpos[kSlotsPer];
#pragma unroll
  for (int j = 0; j < kSlotsPer; ++j) {
    const int k = tid * kSlotsPer + j;
    hpos[j] = -1;
    if (k < slots) {
      const int32_t id = static_cast<int32_t>(ids[j]);
      uint32_t h = (static_cast<uint32_t>(id) * 0x9E3779B1u) >> 19;  // 13 bits = kHashSize
      while (true) {
        const int32_t prev = atomicCAS(&hkey[h], -1, id);
        if (prev == -1 || prev == id) break;
        h = (h + 1) & (kHashSize - 1);
      }
      atomicMin(&hslot[h], k);
      hpos[j] = static_cast<int>(h);
    }
  }
  __syncthreads();
  int first[kSlotsPer];
  int local = 0;
#pragma unroll
  for (int j = 0; j < kSlotsPer; ++j) {
    const int k = tid * kSlotsPer + j;
    first[j] = k < slots && hslot[hpos[j]] == k;
    local += first[j];
  }
  // block exclusive scan of the per-thread counts (slot order = thread order)
  const int lane = tid & 63, wave = tid >> 6;
  int incl = local;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(incl, o);
    if (lane >= o) incl += v;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  int base = 0;
  for (int w = 0; w < wave; ++w) base += wsum[w];
  int total = 0;
  for (int w = 0; w < 16; ++w) total += wsum[w];
  int p = base + incl - local;
#pragma unroll
  for (int j = 0; j < kSlotsPer; ++j) {
    const int k = tid * kSlotsPer + j;
    if (k < slots && first[j]) {
      rows[p] = static_cast<int32_t>(ids[j]);
      node_map[ids[j]] = p;
      ++p;
    }
  }
  for (int k = total + tid; k < slots; k += 1024) rows[k] = -1;
  if (tid == 0) *count = total;
}

__device__ __forceinline__ int64_t batch_id(const int64_t* users, const int64_t* pos, const int64_t* neg, int batch,
                                            int k) {
  return k < batch ? users[k] : (k < 2 * batch ? pos[k - batch] : neg[k - 2 * batch]);
}

__global__ __launch_bounds__(1024) void frontier_build_kernel(const int64_t* __restrict__ users,
                                                              const int64_t* __restrict__ pos,
                                                              const int64_t* __restrict__ neg, int batch,
                                                              int32_t* __restrict__ node_map,
                                                              int32_t* __restrict__ rows,
                                                              int32_t* __restrict__ count) {
  const int slots = 3 * batch;
  int64_t ids[kSlotsPer];
#pragma unroll
  for (int j = 0; j < kSlotsPer; ++j) {
    const int k = threadIdx.x * kSlotsPer + j;
    ids[j] = k < slots ? batch_id(users, pos, neg, batch, k) : -1;
  }
  number_batch(ids, slots, node_map, rows, count);
}

// The prologue of a TRAIN_CF step in one block: the id check of kgat_ids_check_ex (an id outside
// [0, bound) becomes 0 in out and sets *bad / *bad_dev), the batch numbering of kgat_frontier_build
// on the checked ids, and the zeroing of the two hop bitmaps kgat_frontier_hop marks next
// (clr0 / clr1, clr_words uint32 each; nullable).  tag > 0: bad[1] receives the tag once the check is done,
// from thread 0, stored through to memory after bad[0] = 1 when an id was bad (a release store then) -- the
// host learns the check is done from the tag itself, with no event record behind the launch.
// mark0 / mark1 (nullable, zero on entry, not the cleared pair): blocks 1.. mark the batch's first hop
// there as kgat_frontier_hop's frontier_mark_kernel does -- mark0 the batch rows, mark1 those rows and
// every column of their rows of A -- from the checked ids directly (four slots per block, 256 threads
// each; a repeated id marks the same bits again), beside block 0's numbering.
__global__ __launch_bounds__(1024) void cf_begin_kernel(const int64_t* __restrict__ users,
                                                        const int64_t* __restrict__ pos,
                                                        const int64_t* __restrict__ neg, int batch, int64_t bound,
                                                        int64_t* __restrict__ out, int32_t* __restrict__ bad,
                                                        int32_t* __restrict__ bad_dev, int32_t* __restrict__ node_map,
                                                        int32_t* __restrict__ rows, int32_t* __restrict__ count,
                                                        uint32_t* __restrict__ clr0, uint32_t* __restrict__ clr1,
                                                        int64_t clr_words, int32_t tag, kgat_csr A,
                                                        uint32_t* __restrict__ mark0, uint32_t* __restrict__ mark1) {
  const int slots = 3 * batch;
  if (blockIdx.x > 0) {
    const int k = (blockIdx.x - 1) * 4 + (threadIdx.x >> 8);
    const int t = threadIdx.x & 255;
    if (k >= slots) return;
    const int64_t v = batch_id(users, pos, neg, batch, k);
    const int32_t i = v >= 0 && v < bound ? static_cast<int32_t>(v) : 0;  // block 0's substitution
    if (t == 0) {
      atomicOr(&mark0[i >> 5], 1u << (i & 31));
      atomicOr(&mark1[i >> 5], 1u << (i & 31));
    }
    // test before set: on dense graphs (C3: rows of thousands of entries over a 16k-node bitmap) most bits are
    // already set by another slot, and the atomics of 768 slots on a few hundred words serialised (291 us)
    for (int64_t e = A.rowptr[i] + t; e < A.rowptr[i + 1]; e += 256) {
      const int32_t j = A.col[e];
      const uint32_t b = 1u << (j & 31);
      if ((__hip_atomic_load(&mark1[j >> 5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & b) == 0u)
        atomicOr(&mark1[j >> 5], b);
    }
    return;
  }
  int64_t ids[kSlotsPer];
  bool flag = false;
#pragma unroll
  for (int j = 0; j < kSlotsPer; ++j) {
    const int k = threadIdx.x * kSlotsPer + j;
    ids[j] = -1;
    if (k < slots) {
      const int64_t v = batch_id(users, pos, neg, batch, k);
      const bool ok = v >= 0 && v < bound;
      ids[j] = ok ? v : 0;
      out[k] = ids[j];
      flag |= !ok;
    }
  }
  if (flag) {  // every writer stores 1 (bad may be host-mapped pinned memory)
    if (tag == 0) *bad = 1;
    if (bad_dev != nullptr) *bad_dev = 1;
  }
  if (tag > 0) {
    const int any = __syncthreads_or(flag ? 1 : 0);
    if (threadIdx.x == 0) {
      if (any) {  // rare: the flag, then the tag ordered behind it
        __hip_atomic_store(bad, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(bad + 1, tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      } else {
        __hip_atomic_store(bad + 1, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
  if (clr0 != nullptr) {
    // 16-byte stores where the bitmaps allow them (torch allocations are 16-byte aligned)
    const int64_t q = clr_words / 4;
    for (int64_t i = threadIdx.x; i < q; i += 1024) {
      reinterpret_cast<uint4*>(clr0)[i] = make_uint4(0u, 0u, 0u, 0u);
      reinterpret_cast<uint4*>(clr1)[i] = make_uint4(0u, 0u, 0u, 0u);
    }
    for (int64_t i = 4 * q + threadIdx.x; i < clr_words; i += 1024) {
      clr0[i] = 0u;
      clr1[i] = 0u;
    }
  }
  number_batch(ids, slots, node_map, rows, count);
}

__global__ __launch_bounds__(256) void frontier_reset_kernel(const int32_t* __restrict__ rows, int n,
                                                             int32_t* __restrict__ node_map) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n && rows[i] >= 0) node_map[rows[i]] = -1;
}

// Gradient rows of table t scattered into dst.  One wave per slot k of the
// concatenated id list [users | pos | neg]; a slot whose id already occurred
// at an earlier slot returns, otherwise it sums every slot with the same id
// in slot order and adds the sum once: deterministic, no atomics.
__global__ __launch_bounds__(256) void bpr_bwd_kernel(kgat_tables T, int t, const int64_t* __restrict__ users,
                                                      const int64_t* __restrict__ pos,
                                                      const int64_t* __restrict__ neg, int batch, float reg,
                                                      const float* __restrict__ coef,
                                                      const float* __restrict__ grad_out, float* __restrict__ dst,
                                                      int64_t lddst, const int32_t* __restrict__ row_map) {
  const int slots = 3 * batch;
  const int k = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (k >= slots) return;
  auto id_of = [&](int s) -> int64_t { return s < batch ? users[s] : (s < 2 * batch ? pos[s - batch] : neg[s - 2 * batch]); };
  const int64_t id = id_of(k);
  // earlier occurrence?
  bool dup = false;
  for (int s0 = 0; s0 < k && !dup; s0 += 64) {
    const int s = s0 + lane;
    const bool hit = s < k && id_of(s) == id;
    dup = __any(hit);
  }
  if (dup) return;
  const int64_t drow = row_map ? static_cast<int64_t>(row_map[id]) : id;
  if (drow < 0) return;  // row_map -1: a row this caller does not own (row-sharded mode); wave-uniform
  const float scale = grad_out[0] / static_cast<float>(batch);
  const float* tab = T.ptr[t];
  const int64_t ld = T.ld[t];
  const int w = T.width[t];
  constexpr int kCols = 4;  // widths up to 256 columns: lane owns columns lane + 64*c
  float g[kCols] = {0.f, 0.f, 0.f, 0.f};
  for (int s0 = k; s0 < slots; s0 += 64) {
    // ballot with every lane active, before any column-dependent branch
    unsigned long long mask = __ballot(s0 + lane < slots && id_of(s0 + lane) == id);
    while (mask) {  // matching slots in increasing order (wave-uniform)
      const int bit = __ffsll(static_cast<long long>(mask)) - 1;
      mask &= mask - 1;
      const int s = s0 + bit;
      const int b = s % batch;
      const float c = coef[b];
      const int64_t iu = users[b] * ld, ip = pos[b] * ld, in = neg[b] * ld;
#pragma unroll
      for (int cc = 0; cc < kCols; ++cc) {
        const int j = lane + 64 * cc;
        if (j < w) {
          const float xu = tab[iu + j];
          float v;
          if (s < batch) v = c * (tab[ip + j] - tab[in + j]) + reg * xu;
          else if (s < 2 * batch) v = c * xu + reg * tab[ip + j];
          else v = -c * xu + reg * tab[in + j];
          g[cc] = fmaf(v, scale, g[cc]);
        }
      }
    }
  }
#pragma unroll
  for (int cc = 0; cc < kCols; ++cc) {
    const int j = lane + 64 * cc;
    if (j < w) dst[drow * lddst + j] += g[cc];
  }
}

// kgat_bpr_bwd_f32 for tables t0 .. T.count - 1 in one launch, each WRITTEN into its own compact
// buffer D.ptr[t] (ld D.ld[t]; tables with D.ptr[t] null skipped) at the row's frontier position: one
// wave per (frontier row p = blockIdx.x * 4 + wave, table t0 + blockIdx.y) -- rows[p] is the id, every
// slot holding it is summed in slot order with kgat_bpr_bwd_f32's fma into zeros (g starts at +0, so g
// is never -0: 0 + g = g, the same bits).  Rows [*count, 3 * batch) are zeroed (the list's padding).
__global__ __launch_bounds__(256) void bpr_bwd_multi_kernel(kgat_tables T, int t0, const int64_t* __restrict__ users,
                                                            const int64_t* __restrict__ pos,
                                                            const int64_t* __restrict__ neg, int batch, float reg,
                                                            const float* __restrict__ coef,
                                                            const float* __restrict__ grad_out, kgat_tables D,
                                                            const int32_t* __restrict__ rows,
                                                            const int32_t* __restrict__ count) {
  const int slots = 3 * batch;
  const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int t = t0 + static_cast<int>(blockIdx.y);
  const int lane = threadIdx.x & 63;
  float* dst = const_cast<float*>(D.ptr[t]);
  if (p >= slots || dst == nullptr) return;
  const int w = T.width[t];
  const int64_t ldd = D.ld[t];
  if (p >= *count) {
    for (int j = lane; j < w; j += 64) dst[static_cast<int64_t>(p) * ldd + j] = 0.f;
    return;
  }
  auto id_of = [&](int s) -> int64_t { return s < batch ? users[s] : (s < 2 * batch ? pos[s - batch] : neg[s - 2 * batch]); };
  const int64_t id = rows[p];
  const float scale = grad_out[0] / static_cast<float>(batch);
  const float* tab = T.ptr[t];
  const int64_t ld = T.ld[t];
  float g[4] = {0.f, 0.f, 0.f, 0.f};
  for (int s0 = 0; s0 < slots; s0 += 64) {
    unsigned long long mask = __ballot(s0 + lane < slots && id_of(s0 + lane) == id);
    while (mask) {  // matching slots in increasing order (wave-uniform)
      const int bit = __ffsll(static_cast<long long>(mask)) - 1;
      mask &= mask - 1;
      const int s = s0 + bit;
      const int b = s % batch;
      const float c = coef[b];
      const int64_t iu = users[b] * ld, ip = pos[b] * ld, in = neg[b] * ld;
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) {
        const int j = lane + 64 * cc;
        if (j < w) {
          const float xu = tab[iu + j];
          float v;
          if (s < batch) v = c * (tab[ip + j] - tab[in + j]) + reg * xu;
          else if (s < 2 * batch) v = c * xu + reg * tab[ip + j];
          else v = -c * xu + reg * tab[in + j];
          g[cc] = fmaf(v, scale, g[cc]);
        }
      }
    }
  }
#pragma unroll
  for (int cc = 0; cc < 4; ++cc) {
    const int j = lane + 64 * cc;
    if (j < w) dst[static_cast<int64_t>(p) * ldd + j] = g[cc];
  }
}

}  // namespace kgat

static int check_tables(const kgat_tables* T) {
  if (!T || T->count < 1 || T->count > KGAT_MAX_TABLES) return KGAT_ERR_INVALID;
  for (int i = 0; i < T->count; ++i)
    if (!T->ptr[i] || T->width[i] <= 0 || T->ld[i] < T->width[i]) return KGAT_ERR_INVALID;
  return KGAT_OK;
}

extern "C" int kgat_bpr_fwd_ex_f32(const kgat_tables* T, const int64_t* users, const int64_t* pos, const int64_t* neg,
                                   int32_t batch, float reg, float* loss, float* coef, uint32_t* ticket, void* stream) {
  if (int e = check_tables(T)) return e;
  if (!users || !pos || !neg || !loss || !coef || batch <= 0) return KGAT_ERR_INVALID;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(kgat::bpr_fwd_kernel, dim3((batch + 3) / 4), dim3(256), 0, st, *T, users, pos, neg, batch, reg,
                     coef, coef + batch, ticket, loss);
  KGAT_LAUNCH_CHECK();
  if (ticket == nullptr) {
    hipLaunchKernelGGL(kgat::bpr_sum_kernel, dim3(1), dim3(256), 0, st, coef + batch, batch, loss);
    KGAT_LAUNCH_CHECK();
  }
  return KGAT_OK;
}

extern "C" int kgat_bpr_fwd_f32(const kgat_tables* T, const int64_t* users, const int64_t* pos, const int64_t* neg,
                                int32_t batch, float reg, float* loss, float* coef, void* stream) {
  return kgat_bpr_fwd_ex_f32(T, users, pos, neg, batch, reg, loss, coef, nullptr, stream);
}

extern "C" int kgat_bpr_bwd_f32(const kgat_tables* T, int32_t table, const int64_t* users, const int64_t* pos,
                                const int64_t* neg, int32_t batch, float reg, const float* coef,
                                const float* grad_out, float* dst, int64_t lddst, const int32_t* row_map,
                                void* stream) {
  if (int e = check_tables(T)) return e;
  if (table < 0 || table >= T->count || !users || !pos || !neg || !coef || !grad_out || !dst || batch <= 0 ||
      lddst < T->width[table] || T->width[table] > 256)
    return KGAT_ERR_INVALID;
  const int blocks = (3 * batch + 3) / 4;
  hipLaunchKernelGGL(kgat::bpr_bwd_kernel, dim3(blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), *T,
                     table, users, pos, neg, batch, reg, coef, grad_out, dst, lddst, row_map);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int kgat_frontier_build(const int64_t* users, const int64_t* pos, const int64_t* neg, int32_t batch,
                                   int32_t* node_map, int32_t* rows, int32_t* count, void* stream) {
  if (!users || !pos || !neg || !node_map || !rows || !count || batch <= 0 || 3 * batch > kgat::kBatchSlots)
    return KGAT_ERR_INVALID;
  hipLaunchKernelGGL(kgat::frontier_build_kernel, dim3(1), dim3(1024), 0, reinterpret_cast<hipStream_t>(stream), users,
                     pos, neg, batch, node_map, rows, count);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int kgat_frontier_reset(const int32_t* rows, int32_t n, int32_t* node_map, void* stream) {
  if (!rows || !node_map || n < 0) return KGAT_ERR_INVALID;
  if (n == 0) return KGAT_OK;
  hipLaunchKernelGGL(kgat::frontier_reset_kernel, dim3((n + 255) / 256), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), rows, n, node_map);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int kgat_bpr_bwd_multi_f32(const kgat_tables* T, int32_t t0, const int64_t* users, const int64_t* pos,
                                      const int64_t* neg, int32_t batch, float reg, const float* coef,
                                      const float* grad_out, const kgat_tables* D, const int32_t* rows,
                                      const int32_t* count, void* stream) {
  if (int e = check_tables(T)) return e;
  if (!D || D->count != T->count || t0 < 0 || t0 >= T->count || !users || !pos || !neg || !coef || !grad_out ||
      !rows || !count || batch <= 0)
    return KGAT_ERR_INVALID;
  for (int t = t0; t < T->count; ++t)
    if (D->ptr[t] != nullptr && (D->ld[t] < T->width[t] || T->width[t] > 256)) return KGAT_ERR_INVALID;
  const int blocks = (3 * batch + 3) / 4;
  hipLaunchKernelGGL(kgat::bpr_bwd_multi_kernel, dim3(blocks, T->count - t0), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), *T, t0, users, pos, neg, batch, reg, coef, grad_out, *D,
                     rows, count);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int kgat_cf_begin_ex(const int64_t* users, const int64_t* pos, const int64_t* neg, int32_t batch,
                                int64_t bound, int64_t* ids_out, int32_t* bad, int32_t* bad_dev, int32_t* node_map,
                                int32_t* rows, int32_t* count, uint32_t* clear0, uint32_t* clear1,
                                int64_t clear_words, const kgat_csr* A, uint32_t* mark0, uint32_t* mark1, int32_t tag,
                                void* stream) {
  if (!users || !pos || !neg || !ids_out || !bad || !node_map || !rows || !count || batch <= 0 ||
      3 * batch > kgat::kBatchSlots || bound <= 0 || clear_words < 0 || ((clear0 == nullptr) != (clear1 == nullptr)) ||
      tag < 0 || tag >= (1 << 29) || ((mark0 == nullptr) != (mark1 == nullptr)))
    return KGAT_ERR_INVALID;
  if (mark0 != nullptr && (!A || !A->rowptr || !A->col || A->n_rows < bound || mark0 == clear0 || mark0 == clear1 ||
                           mark1 == clear0 || mark1 == clear1 || mark0 == mark1))
    return KGAT_ERR_INVALID;
  if (clear0 != nullptr && ((reinterpret_cast<uintptr_t>(clear0) | reinterpret_cast<uintptr_t>(clear1)) & 15))
    return KGAT_ERR_INVALID;
  kgat_csr a{};
  if (mark0 != nullptr) a = *A;
  const int grid = mark0 != nullptr ? 1 + (3 * batch + 3) / 4 : 1;
  hipLaunchKernelGGL(kgat::cf_begin_kernel, dim3(grid), dim3(1024), 0, reinterpret_cast<hipStream_t>(stream), users,
                     pos, neg, batch, bound, ids_out, bad, bad_dev, node_map, rows, count, clear0, clear1, clear_words,
                     tag, a, mark0, mark1);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int kgat_cf_begin(const int64_t* users, const int64_t* pos, const int64_t* neg, int32_t batch,
                             int64_t bound, int64_t* ids_out, int32_t* bad, int32_t* bad_dev, int32_t* node_map,
                             int32_t* rows, int32_t* count, uint32_t* clear0, uint32_t* clear1, int64_t clear_words,
                             void* stream) {
  return kgat_cf_begin_ex(users, pos, neg, batch, bound, ids_out, bad, bad_dev, node_map, rows, count, clear0, clear1,
                          clear_words, nullptr, nullptr, nullptr, 0, stream);
}
