// a8 / §8(f)1 -- ranking for evaluation and recommendation
// (src/model/KGAT/main.py:70-130 and 576-605, src/utils/metrics_calculator.py:84-131).
//
//   kgat_mask_rows_f32     scores[r, idx] = value for a per-row index list (the
//                          reference's `cf_scores[idx][train_items] = -inf`)
//   kgat_topk_f32          per row, the k largest scores in descending order;
//                          equal scores are ordered by ascending column
//   kgat_rank_metrics_f32  precision / recall / nDCG @k from the top-k columns
//                          and each row's (sorted, unique) test items
//
// Top-k is a block-per-row radix select on order-preserving uint32 keys
// (4 passes of 8 bits, LDS histograms), then one pass that collects the
// strictly-greater keys and the lowest-index ties of the k-th key, and a
// bitonic sort of the <= 1024 survivors in LDS.  Deterministic.
#include "common.hpp"

namespace kgat {

constexpr int kTopkThreads = 1024;
constexpr int kTopkMax = 1024;

__device__ __forceinline__ uint32_t order_key(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float key_value(uint32_t k) {
  const uint32_t b = (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k;
  return __uint_as_float(b);
}

__global__ void mask_rows_kernel(float* __restrict__ S, int64_t ld, int32_t rows, const int64_t* __restrict__ rowptr,
                                 const int32_t* __restrict__ idx, int32_t cols, float value) {
  const int r = blockIdx.x;
  if (r >= rows) return;
  for (int64_t e = rowptr[r] + threadIdx.x; e < rowptr[r + 1]; e += blockDim.x) {
    const int32_t j = idx[e];
    if (j >= 0 && j < cols) S[r * ld + j] = value;
  }
}

// block-wide exclusive prefix of one flag per thread (in thread order); returns
// this thread's rank, writes the block total
__device__ __forceinline__ int block_rank(bool flag, int* wsum, int& total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t bal = __ballot(flag);
  const int in_wave = __popcll(bal & ((1ull << lane) - 1ull));
  if (lane == 0) wsum[wave] = __popcll(bal);
  __syncthreads();
  int before = 0;
  total = 0;
  for (int w = 0; w < kTopkThreads / 64; ++w) {
    const int c = wsum[w];
    if (w < wave) before += c;
    total += c;
  }
  __syncthreads();
  return before + in_wave;
}

__global__ __launch_bounds__(kTopkThreads) void topk_kernel(const float* __restrict__ S, int64_t ld, int32_t cols,
                                                            int32_t k, int32_t* __restrict__ out_idx,
                                                            float* __restrict__ out_val) {
  __shared__ int hist[256];
  __shared__ int wsum[kTopkThreads / 64];
  __shared__ uint32_t ck[kTopkMax];
  __shared__ int32_t ci[kTopkMax];
  __shared__ uint32_t s_prefix, s_mask;
  __shared__ int s_need, s_ngt;
  const int r = blockIdx.x;
  const float* row = S + static_cast<int64_t>(r) * ld;
  const int tid = threadIdx.x;

  // ---- radix select of the k-th largest key
  if (tid == 0) {
    s_prefix = 0;
    s_mask = 0;
    s_need = k;  // rank still to find within the current prefix
  }
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    if (tid < 256) hist[tid] = 0;
    __syncthreads();
    const uint32_t prefix = s_prefix, mask = s_mask;
    for (int j = tid; j < cols; j += kTopkThreads) {
      const uint32_t key = order_key(row[j]);
      if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255], 1);
    }
    __syncthreads();
    if (tid == 0) {
      int need = s_need, d = 255;
      for (; d > 0; --d) {
        if (hist[d] >= need) break;
        need -= hist[d];
      }
      s_need = need;
      s_prefix = prefix | (static_cast<uint32_t>(d) << shift);
      s_mask = mask | (255u << shift);
    }
    __syncthreads();
  }
  const uint32_t kth = s_prefix;
  const int take_eq = s_need;  // ties of the k-th key to take (lowest columns first)
  if (tid == 0) s_ngt = 0;
  __syncthreads();

  // ---- collect: every key > kth, and the first take_eq columns with key == kth
  int eq_seen = 0;
  for (int base = 0; base < cols; base += kTopkThreads) {
    const int j = base + tid;
    uint32_t key = 0;
    if (j < cols) key = order_key(row[j]);
    const bool gt = j < cols && key > kth;
    const bool eq = j < cols && key == kth;
    if (gt) {
      const int pos = atomicAdd(&s_ngt, 1);  // order fixed by the sort below
      ck[pos] = key;
      ci[pos] = j;
    }
    int total;
    const int rank = block_rank(eq, wsum, total);
    if (eq && eq_seen + rank < take_eq) {
      const int pos = (k - take_eq) + eq_seen + rank;
      ck[pos] = key;
      ci[pos] = j;
    }
    eq_seen += total;
  }
  __syncthreads();

  // ---- bitonic sort of the k survivors: key descending, column ascending
  int P = 1;
  while (P < k) P <<= 1;
  for (int i = tid; i < P; i += kTopkThreads)
    if (i >= k) {
      ck[i] = 0u;
      ci[i] = 0x7FFFFFFF;
    }
  __syncthreads();
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < P; i += kTopkThreads) {
        const int jx = i ^ stride;
        if (jx > i) {
          const bool desc = (i & size) == 0;
          const uint32_t ka = ck[i], kb = ck[jx];
          const int32_t ia = ci[i], ib = ci[jx];
          // "a before b" in the final order
          const bool a_first = ka > kb || (ka == kb && ia < ib);
          if (a_first != desc) {
            ck[i] = kb;
            ck[jx] = ka;
            ci[i] = ib;
            ci[jx] = ia;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < k; i += kTopkThreads) {
    out_idx[static_cast<int64_t>(r) * k + i] = ci[i];
    if (out_val != nullptr) out_val[static_cast<int64_t>(r) * k + i] = key_value(ck[i]);
  }
}

struct KList {
  int32_t k[16];
  int32_t n;
};

// one wave per row: hits at ranks 0..kmax-1 by binary search in the row's test items
__global__ void rank_metrics_kernel(const int32_t* __restrict__ topk, int32_t rows, int32_t kmax,
                                    const int64_t* __restrict__ test_rowptr, const int32_t* __restrict__ test_idx,
                                    KList ks, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int64_t beg = test_rowptr[r], end = test_rowptr[r + 1];
  const double npos = static_cast<double>(end - beg);
  double hits_acc[16], dcg_acc[16];
  for (int t = 0; t < ks.n; ++t) hits_acc[t] = dcg_acc[t] = 0.0;
  for (int j0 = 0; j0 < kmax; j0 += 64) {
    const int j = j0 + lane;
    bool hit = false;
    if (j < kmax) {
      const int32_t item = topk[static_cast<int64_t>(r) * kmax + j];
      int64_t lo = beg, hi = end;
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (test_idx[mid] < item) lo = mid + 1;
        else hi = mid;
      }
      hit = lo < end && test_idx[lo] == item;
    }
    const double g = hit ? 1.0 / log2(static_cast<double>(j + 2)) : 0.0;
    for (int t = 0; t < ks.n; ++t) {
      const bool in = j < ks.k[t];
      double h = (hit && in) ? 1.0 : 0.0, d = in ? g : 0.0;
      for (int o = 32; o > 0; o >>= 1) {
        h += __shfl_xor(h, o);
        d += __shfl_xor(d, o);
      }
      hits_acc[t] += h;
      dcg_acc[t] += d;
    }
  }
  if (lane == 0) {
    for (int t = 0; t < ks.n; ++t) {
      const int k = ks.k[t];
      double idcg = 0.0;
      const int m = npos < k ? static_cast<int>(npos) : k;
      for (int j = 0; j < m; ++j) idcg += 1.0 / log2(static_cast<double>(j + 2));
      float* o = out + static_cast<int64_t>(t) * 3 * rows;
      o[r] = static_cast<float>(hits_acc[t] / k);                       // precision
      o[rows + r] = static_cast<float>(hits_acc[t] / npos);             // recall (0/0 = nan, as numpy)
      o[2 * rows + r] = static_cast<float>(idcg > 0.0 ? dcg_acc[t] / idcg : 0.0);  // ndcg
    }
  }
}

}  // namespace kgat

extern "C" int kgat_mask_rows_f32(float* scores, int64_t ld, int32_t rows, int32_t cols, const int64_t* rowptr,
                                  const int32_t* idx, float value, void* stream) {
  if (!scores || !rowptr || rows < 0 || cols < 0 || ld < cols) return KGAT_ERR_INVALID;
  if (rows == 0) return KGAT_OK;
  if (idx == nullptr) return KGAT_ERR_INVALID;
  hipLaunchKernelGGL(kgat::mask_rows_kernel, dim3(rows), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), scores,
                     ld, rows, rowptr, idx, cols, value);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int kgat_topk_f32(const float* scores, int64_t ld, int32_t rows, int32_t cols, int32_t k, int32_t* out_idx,
                             float* out_val, void* stream) {
  if (!scores || !out_idx || rows < 0 || cols < 1 || ld < cols) return KGAT_ERR_INVALID;
  if (k < 1 || k > cols || k > kgat::kTopkMax) return KGAT_ERR_INVALID;
  if (rows == 0) return KGAT_OK;
  hipLaunchKernelGGL(kgat::topk_kernel, dim3(rows), dim3(kgat::kTopkThreads), 0,
                     reinterpret_cast<hipStream_t>(stream), scores, ld, cols, k, out_idx, out_val);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int kgat_rank_metrics_f32(const int32_t* topk_idx, int32_t rows, int32_t kmax, const int64_t* test_rowptr,
                                     const int32_t* test_idx, const int32_t* k_list, int32_t n_k, float* out,
                                     void* stream) {
  if (!topk_idx || !test_rowptr || !out || !k_list || rows < 0 || kmax < 1 || n_k < 1 || n_k > 16)
    return KGAT_ERR_INVALID;
  kgat::KList ks{};
  ks.n = n_k;
  for (int t = 0; t < n_k; ++t) {
    if (k_list[t] < 1 || k_list[t] > kmax) return KGAT_ERR_INVALID;
    ks.k[t] = k_list[t];
  }
  if (rows == 0) return KGAT_OK;
  const int per_block = 4;
  hipLaunchKernelGGL(kgat::rank_metrics_kernel, dim3((rows + per_block - 1) / per_block), dim3(64 * per_block), 0,
                     reinterpret_cast<hipStream_t>(stream), topk_idx, rows, kmax, test_rowptr, test_idx, ks, out);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}
