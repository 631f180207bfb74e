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
// coef[b] = sigmoid(pos_b - neg_b) - 1 is kept for the backward; a second
// single-block kernel sums term[] in index order (deterministic).
__global__ __launch_bounds__(256) void bpr_fwd_kernel(kgat_tables T, const int64_t* __restrict__ users,
                                                      const int64_t* __restrict__ pos,
                                                      const int64_t* __restrict__ neg, int batch, float reg,
                                                      float* __restrict__ coef, float* __restrict__ term) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= batch) return;
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
    term[b] = nls + reg * 0.5f * (qu + qp + qn);
  }
}

__global__ __launch_bounds__(256) void bpr_sum_kernel(const float* __restrict__ term, int batch,
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

// Unique ids of the batch [users | pos | neg] in first-occurrence order:
// rows[0..count) = ids, node_map[id] = its position, rows[count..3B) = -1.
// node_map must hold -1 for every node on entry (kgat_frontier_reset restores
// it).  O(slots): an atomicMin of (slot - slots - 1) < -1 into node_map[id]
// elects the first slot of every id, a block scan numbers the winners in slot
// order, and the winners overwrite node_map[id] with their position.
__global__ __launch_bounds__(1024) void frontier_build_kernel(const int64_t* __restrict__ users,
                                                              const int64_t* __restrict__ pos,
                                                              const int64_t* __restrict__ neg, int batch,
                                                              int32_t* __restrict__ node_map,
                                                              int32_t* __restrict__ rows,
                                                              int32_t* __restrict__ count) {
  constexpr int kMax = 4096;
  constexpr int kPer = kMax / 1024;
  __shared__ int32_t wsum[16];
  const int slots = 3 * batch;
  const int tid = threadIdx.x;
  // thread tid owns the contiguous slots [tid*kPer, tid*kPer + kPer)
  int64_t ids[kPer];
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int k = tid * kPer + j;
    ids[j] = k < slots ? (k < batch ? users[k] : (k < 2 * batch ? pos[k - batch] : neg[k - 2 * batch])) : -1;
    if (k < slots) atomicMin(&node_map[ids[j]], k - slots - 1);
  }
  __syncthreads();
  __threadfence_block();
  int first[kPer];
  int local = 0;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int k = tid * kPer + j;
    first[j] = 0;
    if (k < slots) first[j] = __hip_atomic_load(&node_map[ids[j]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                              k - slots - 1;
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
  for (int j = 0; j < kPer; ++j) {
    const int k = tid * kPer + j;
    if (k < slots && first[j]) {
      rows[p] = static_cast<int32_t>(ids[j]);
      node_map[ids[j]] = p;
      ++p;
    }
  }
  for (int k = total + tid; k < slots; k += 1024) rows[k] = -1;
  if (tid == 0) *count = total;
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

}  // namespace kgat

static int check_tables(const kgat_tables* T) {
  if (!T || T->count < 1 || T->count > KGAT_MAX_TABLES) return KGAT_ERR_INVALID;
  for (int i = 0; i < T->count; ++i)
    if (!T->ptr[i] || T->width[i] <= 0 || T->ld[i] < T->width[i]) return KGAT_ERR_INVALID;
  return KGAT_OK;
}

extern "C" int kgat_bpr_fwd_f32(const kgat_tables* T, const int64_t* users, const int64_t* pos, const int64_t* neg,
                                int32_t batch, float reg, float* loss, float* coef, void* stream) {
  if (int e = check_tables(T)) return e;
  if (!users || !pos || !neg || !loss || !coef || batch <= 0) return KGAT_ERR_INVALID;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(kgat::bpr_fwd_kernel, dim3((batch + 3) / 4), dim3(256), 0, st, *T, users, pos, neg, batch, reg,
                     coef, coef + batch);
  KGAT_LAUNCH_CHECK();
  hipLaunchKernelGGL(kgat::bpr_sum_kernel, dim3(1), dim3(256), 0, st, coef + batch, batch, loss);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
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
  if (!users || !pos || !neg || !node_map || !rows || !count || batch <= 0 || 3 * batch > 4096)
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
