// a9 fused Adam, small device utilities, and the host-side CSR plan builder.
#include <cmath>

#include <cstdlib>

#include <algorithm>
#include <vector>

#include "adam.hpp"
#include "common.hpp"

namespace kgat {

// torch.optim.Adam step for one tensor (model.py:404-419): adam_elem (common.hpp)
// per element.  HBM-bound: 28 B per parameter (read p g m v, write p m v).
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                   float step_size, float b1, float b2, float bc2s, float eps) {
  const float w1 = 1.f - b1, w2 = 1.f - b2;
  const int64_t n4 = n / 4;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  float4* p4 = reinterpret_cast<float4*>(p);
  float4* m4 = reinterpret_cast<float4*>(m);
  float4* v4 = reinterpret_cast<float4*>(v);
  const float4* g4 = reinterpret_cast<const float4*>(g);
  auto upd = [&](float& pp, float gg, float& mm, float& vv) {
    adam_elem(pp, gg, mm, vv, w1, b2, w2, step_size, bc2s, eps);
  };
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pp = p4[i], mm = m4[i], vv = v4[i];
    const float4 gg = g4[i];
    upd(pp.x, gg.x, mm.x, vv.x);
    upd(pp.y, gg.y, mm.y, vv.y);
    upd(pp.z, gg.z, mm.z, vv.z);
    upd(pp.w, gg.w, mm.w, vv.w);
    p4[i] = pp;
    m4[i] = mm;
    v4[i] = vv;
  }
  for (int64_t i = n4 * 4 + static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride)
    upd(p[i], g[i], m[i], v[i]);
}

__global__ __launch_bounds__(256) void gather_kernel(const float* __restrict__ src, const int32_t* __restrict__ idx,
                                                     int64_t n, float* __restrict__ dst) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride)
    dst[i] = src[idx[i]];
}

// ids of up to KGAT_IDS_MAX arrays, concatenated into out; out-of-range ids become 0 and set *bad = 1
// (and *bad_dev = 1 when given: the optimiser kernels' skip flag)
struct IdBounds {
  int64_t b[KGAT_IDS_MAX];
};

__global__ __launch_bounds__(256) void ids_check_kernel(kgat_ids ids, int64_t total, IdBounds bounds,
                                                        int64_t* __restrict__ out, int32_t* __restrict__ bad,
                                                        int32_t* __restrict__ bad_dev) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  bool flag = false;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += stride) {
    int k = 0;
    int64_t off = i;
    while (k + 1 < ids.count && off >= ids.n[k]) off -= ids.n[k++];
    const int64_t v = ids.ptr[k][off];
    const bool ok = v >= 0 && v < bounds.b[k];
    out[i] = ok ? v : 0;
    flag |= !ok;
  }
  if (flag) {  // every writer stores 1: no atomic needed (bad may be host-mapped pinned memory)
    *bad = 1;
    if (bad_dev != nullptr) *bad_dev = 1;
  }
}

// node_map[ids[i]] = i (distinct ids; ids[i] < 0 skipped)
__global__ __launch_bounds__(256) void map_build_kernel(const int32_t* __restrict__ ids, int64_t n,
                                                        int32_t* __restrict__ node_map) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride)
    if (ids[i] >= 0) node_map[ids[i]] = static_cast<int32_t>(i);
}

// kgat_map_build over ids that came from another process (a row-sharded peer's gathered hop rows): an
// id outside [-1, n_nodes) is not mapped -- it is set to -1 in place, so kgat_frontier_reset skips it
// too -- and raises the host flag (pinned, host-mapped; plain store) and the device skip flag.
__global__ __launch_bounds__(256) void map_build_checked_kernel(int32_t* __restrict__ ids, int64_t n,
                                                                int32_t* __restrict__ node_map, int64_t n_nodes,
                                                                int32_t* bad_host, int32_t* bad_dev) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  bool flag = false;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int32_t x = ids[i];
    if (x >= 0 && x < n_nodes) {
      node_map[x] = static_cast<int32_t>(i);
    } else if (x != -1) {
      ids[i] = -1;
      flag = true;
    }
  }
  if (flag) {  // every writer stores 1 (as ids_check_kernel): no atomic needed
    if (bad_host != nullptr) *bad_host = 1;
    if (bad_dev != nullptr) *bad_dev = 1;
  }
}

// ids outside [-1, bound) become -1 in place and raise the flags (a gathered row list from other
// processes, checked before anything indexes with it)
__global__ __launch_bounds__(256) void ids_sanitize_kernel(int32_t* __restrict__ ids, int64_t n, int64_t bound,
                                                           int32_t* bad_host, int32_t* bad_dev) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  bool flag = false;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int32_t x = ids[i];
    if (x < -1 || x >= bound) {
      ids[i] = -1;
      flag = true;
    }
  }
  if (flag) {  // every writer stores 1 (as ids_check_kernel)
    if (bad_host != nullptr) *bad_host = 1;
    if (bad_dev != nullptr) *bad_dev = 1;
  }
}

// out[i] = a[i] < 0 ? -1 : (b ? b[a[i]] : a[i]) + offset  (b[.] < 0 stays -1)
__global__ __launch_bounds__(256) void map_compose_kernel(const int32_t* __restrict__ a, int64_t n,
                                                          const int32_t* __restrict__ b, int32_t offset,
                                                          int32_t* __restrict__ out) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int32_t x = a[i];
    const int32_t y = x < 0 ? -1 : (b != nullptr ? b[x] : x);
    out[i] = y < 0 ? -1 : y + offset;
  }
}

__global__ __launch_bounds__(256) void fill_kernel(float* __restrict__ dst, int64_t n, float value) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = value;
}

}  // namespace kgat

extern "C" const char* kgat_strerror(int status) {
  switch (status) {
    case KGAT_OK: return "ok";
    case KGAT_ERR_INVALID: return "kgat: invalid argument (null pointer, bad size, or misaligned buffer)";
    case KGAT_ERR_UNSUPPORTED_DIM: return "kgat: feature width not supported by the compiled kernels";
    case KGAT_ERR_WORKSPACE: return "kgat: workspace too small";
    case KGAT_ERR_COMM_UNAVAILABLE: return "kgat: no loadable RCCL library (kgat_comm_load)";
    default:
      if (status >= KGAT_ERR_COMM_BASE && status < KGAT_ERR_COMM_BASE + 100) return kgat_comm_error_string(status);
      return hipGetErrorString(static_cast<hipError_t>(status));
  }
}

extern "C" int kgat_version(void) { return 1; }

namespace kgat {

// V = 0: per float4 load -> update -> store; V >= 1: a chunk's 16 float4 loads issued first
// (all four arrays, four float4 per lane), then the updates, then the stores; V = 2 with
// non-temporal loads/stores (every byte is touched once per step).
template <int V>
__global__ __launch_bounds__(256) void adam_multi_kernel(AdamTable T, float b1, float b2, float eps,
                                                         const int32_t* __restrict__ skip, StepSched sched) {
  // a captured step (kgat_adam_multi_sched_f32): every tensor's step size and bias correction are step t's
  // entries of the host-computed schedule, t read on the device (and handed on before a skip returns)
  const int32_t ts = sched.t != nullptr ? sched_step(sched) : 0;
  if (skip != nullptr && *skip != 0) return;  // the step's ids were out of range: no parameter moves
  adam_multi_chunks<V>(T, b1, b2, eps, sched, ts, blockIdx.x, gridDim.x);
}

// The table's Adam step whose gradient is nonzero on a few rows only (the KG step: TransR reads
// <= 3B rows, model.py:204-261): row r's gradient is Gc[row_map[r]] (compact, kgat_transr_bwd_ex_f32
// with the same map) or exactly 0 -- the bits the dense step gets from its zero-filled [N, d]
// gradient, without writing it, reading it back or zeroing it (24 B per parameter + 4 B per row
// instead of 28 + 4 + the scatter).  adam_multi_kernel<2>'s access pattern (four float4 of each
// array in flight per thread, non-temporal).
__global__ __launch_bounds__(256) void adam_rows_kernel(float* __restrict__ p, float* __restrict__ m,
                                                        float* __restrict__ v, int64_t n4, int d4,
                                                        const int32_t* __restrict__ row_map,
                                                        const float* __restrict__ Gc, int64_t ldg, float step_size,
                                                        float b1, float b2, float bc2s, float eps,
                                                        const int32_t* __restrict__ skip) {
  if (skip != nullptr && *skip != 0) return;
  const float w1 = 1.f - b1, w2 = 1.f - b2;
  const int64_t chunks = (n4 + 1023) / 1024;
  for (int64_t c = blockIdx.x; c < chunks; c += gridDim.x) {
    float4 pp[4], mm[4], vv[4], gg[4];
    int64_t e4[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      e4[u] = c * 1024 + u * 256 + threadIdx.x;
      if (e4[u] < n4) {
        pp[u] = ld4<2>(p + 4 * e4[u]);
        mm[u] = ld4<2>(m + 4 * e4[u]);
        vv[u] = ld4<2>(v + 4 * e4[u]);
        const int32_t mi = row_map[e4[u] / d4];
        gg[u] = mi >= 0 ? *reinterpret_cast<const float4*>(Gc + mi * ldg + 4 * (e4[u] % d4))
                        : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (e4[u] >= n4) continue;
      float* P = &pp[u].x;
      float* Mv = &mm[u].x;
      float* Vv = &vv[u].x;
      const float* G = &gg[u].x;
#pragma unroll
      for (int k = 0; k < 4; ++k) adam_elem(P[k], G[k], Mv[k], Vv[k], w1, b2, w2, step_size, bc2s, eps);
      st4<2>(p + 4 * e4[u], pp[u]);
      st4<2>(m + 4 * e4[u], mm[u]);
      st4<2>(v + 4 * e4[u], vv[u]);
    }
  }
}

}  // namespace kgat

extern "C" int kgat_adam_multi_f32(const kgat_adam_tensor* tensors, int32_t count, float beta1, float beta2,
                                   float eps, void* stream) {
  return kgat_adam_multi_ex_f32(tensors, count, beta1, beta2, eps, nullptr, stream);
}

extern "C" int kgat_adam_multi_ex_f32(const kgat_adam_tensor* tensors, int32_t count, float beta1, float beta2,
                                      float eps, const int32_t* skip, void* stream) {
  return kgat_adam_multi_sched_f32(tensors, count, beta1, beta2, eps, skip, nullptr, nullptr, nullptr, 0, nullptr,
                                   stream);
}

extern "C" int kgat_adam_multi_sched_f32(const kgat_adam_tensor* tensors, int32_t count, float beta1, float beta2,
                                         float eps, const int32_t* skip, const int32_t* t_dev, const float* sched_sz,
                                         const float* sched_bc, int32_t t_add, int32_t* t_out, void* stream) {
  if (!tensors || count < 1 || count > KGAT_ADAM_MAX_TENSORS) return KGAT_ERR_INVALID;
  if (t_dev != nullptr && (!sched_sz || !sched_bc)) return KGAT_ERR_INVALID;
  const kgat::StepSched sched{t_dev, sched_sz, sched_bc, t_add, t_out};
  kgat::AdamTable T{};
  if (int e = kgat::adam_table(tensors, count, T)) return e;
  const int64_t off = T.chunk_off[count];
  if (off == 0) return KGAT_OK;
  const int grid = kgat::adam_grid(T);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // the <2> access pattern: C2 table (64M parameters) 314 us vs 346 us for <0> / <1> on the same box
  hipLaunchKernelGGL(kgat::adam_multi_kernel<2>, dim3(grid), dim3(256), 0, st, T, beta1, beta2, eps, skip, sched);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int kgat_adam_rows_f32(float* p, float* m, float* v, int64_t n_rows, int32_t d, const int32_t* row_map,
                                  const float* Gc, int64_t ldg, float step_size, float beta1, float beta2,
                                  float bc2_sqrt, float eps, const int32_t* skip, void* stream) {
  if (!p || !m || !v || !row_map || !Gc || n_rows < 0 || d < 4 || (d & 3) || ldg < d || (ldg & 3)) return KGAT_ERR_INVALID;
  if ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(m) | reinterpret_cast<uintptr_t>(v) |
       reinterpret_cast<uintptr_t>(Gc)) & 15)
    return KGAT_ERR_INVALID;
  const int64_t n4 = n_rows * (d / 4);
  if (n4 == 0) return KGAT_OK;
  const int64_t chunks = (n4 + 1023) / 1024;
  const int grid = static_cast<int>(chunks < kgat::kCUs * 8 ? chunks : kgat::kCUs * 8);
  hipLaunchKernelGGL(kgat::adam_rows_kernel, dim3(grid), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), p, m, v,
                     n4, d / 4, row_map, Gc, ldg, step_size, beta1, beta2, bc2_sqrt, eps, skip);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

namespace kgat {

// Lazy table Adam of the KG phase (common.hpp's LazyHist / lazy_replay): the batch rows only.  A
// row's elements are threads of one block (256 % d == 0).
// rows (nullable = every row): bring the listed rows up to step t (replay only).
__global__ __launch_bounds__(256) void adam_lazy_catchup_kernel(float* __restrict__ p, float* __restrict__ m,
                                                                float* __restrict__ v, int d,
                                                                const int32_t* __restrict__ rows, int64_t n_list,
                                                                int32_t* __restrict__ last, int32_t t, LazyHist h,
                                                                float b1, float b2, float eps, StepSched sched) {
  if (sched.t != nullptr) t = *sched.t;
  __shared__ LazyHistLds hl;
  const int32_t lo = stage_hist(hl, h, t);
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  const int64_t k = i / d;
  const int c = static_cast<int>(i % d);
  const int64_t r = k < n_list ? (rows != nullptr ? static_cast<int64_t>(rows[k]) : k) : -1;
  const int32_t from = r >= 0 ? last[r] : t;
  if (from < t) {
    const int64_t o = r * d + c;
    float pp = p[o], mm = m[o], vv = v[o];
    lazy_replay_lds(pp, mm, vv, from, t, h, hl, lo, 1.f - b1, b2, 1.f - b2, eps);
    p[o] = pp;
    m[o] = mm;
    v[o] = vv;
  }
  __syncthreads();  // every thread of the row has read last[r]
  if (c == 0 && r >= 0 && from < t) last[r] = t;
}

// Step t on the listed rows (rows[k] with the compact gradient Gc[k]): the skipped steps first,
// then step t itself; step t's scalars and skip flag go into the history for the other rows.
__global__ __launch_bounds__(256) void adam_lazy_rows_kernel(float* __restrict__ p, float* __restrict__ m,
                                                             float* __restrict__ v, int d,
                                                             const int32_t* __restrict__ rows, int64_t n_list,
                                                             const float* __restrict__ Gc, int64_t ldg,
                                                             int32_t* __restrict__ last, int32_t t, LazyHist h,
                                                             float step_size, float b1, float b2, float bc2s,
                                                             float eps, const int32_t* __restrict__ skip,
                                                             StepSched sched, int32_t* __restrict__ row_map) {
  if (sched.t != nullptr) {
    t = sched_step(sched);
    step_size = sched.sz[t];
    bc2s = sched.bc[t];
  }
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  const bool skipped = skip != nullptr && *skip != 0;
  if (i == 0) {
    const int32_t j = t % h.cap;
    h.sz[j] = step_size;
    h.bc[j] = bc2s;
    h.skip[j] = skipped ? 1 : 0;
  }
  const int64_t k = i / d;
  const int c = static_cast<int>(i % d);
  const int64_t r = k < n_list ? static_cast<int64_t>(rows[k]) : -1;
  const int32_t from = r >= 0 ? last[r] : t;
  if (r >= 0 && !skipped) {
    const float w1 = 1.f - b1, w2 = 1.f - b2;
    const int64_t o = r * d + c;
    float pp = p[o], mm = m[o], vv = v[o];
    lazy_replay(pp, mm, vv, from, t - 1, h, w1, b2, w2, eps);
    adam_elem(pp, Gc[k * ldg + c], mm, vv, w1, b2, w2, step_size, bc2s, eps);
    p[o] = pp;
    m[o] = mm;
    v[o] = vv;
  }
  __syncthreads();
  if (c == 0 && r >= 0 && !skipped) last[r] = t;
  // the batch rows' map entries back to -1 (the captured update's frontier_reset, folded in: nothing
  // after this kernel reads the map in the step; a skipped step resets it too)
  if (row_map != nullptr && c == 0 && r >= 0) row_map[r] = -1;
}

}  // namespace kgat

static bool lazy_args_ok(const float* p, const float* m, const float* v, int32_t d, const int32_t* last,
                         const float* hsz, const float* hbc, const int32_t* hskip, int32_t cap) {
  return p && m && v && last && hsz && hbc && hskip && cap > 0 && d > 0 && d <= 256 && (256 % d) == 0;
}

static int lazy_catchup(float* p, float* m, float* v, int64_t n_rows, int32_t d, const int32_t* rows, int64_t n_list,
                        int32_t* last, int32_t t, const int32_t* t_dev, float* hist_sz, float* hist_bc,
                        int32_t* hist_skip, int32_t cap, float beta1, float beta2, float eps, void* stream) {
  if (!lazy_args_ok(p, m, v, d, last, hist_sz, hist_bc, hist_skip, cap) || n_rows < 0 || n_list < 0 || t < 0)
    return KGAT_ERR_INVALID;
  const int64_t n = rows != nullptr ? n_list : n_rows;
  if (n == 0) return KGAT_OK;
  const int64_t blocks = (n * d + 255) / 256;
  if (blocks > 0x7fffffff) return KGAT_ERR_INVALID;
  hipLaunchKernelGGL(kgat::adam_lazy_catchup_kernel, dim3(blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     p, m, v, d, rows, n, last, t, kgat::LazyHist{hist_sz, hist_bc, hist_skip, cap}, beta1, beta2,
                     eps, kgat::StepSched{t_dev, nullptr, nullptr});
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int kgat_adam_lazy_catchup_f32(float* p, float* m, float* v, int64_t n_rows, int32_t d,
                                          const int32_t* rows, int64_t n_list, int32_t* last, int32_t t,
                                          float* hist_sz, float* hist_bc, int32_t* hist_skip, int32_t cap,
                                          float beta1, float beta2, float eps, void* stream) {
  return lazy_catchup(p, m, v, n_rows, d, rows, n_list, last, t, nullptr, hist_sz, hist_bc, hist_skip, cap, beta1,
                      beta2, eps, stream);
}

extern "C" int kgat_adam_lazy_catchup_sched_f32(float* p, float* m, float* v, int64_t n_rows, int32_t d,
                                                const int32_t* rows, int64_t n_list, int32_t* last,
                                                const int32_t* t_dev, float* hist_sz, float* hist_bc,
                                                int32_t* hist_skip, int32_t cap, float beta1, float beta2, float eps,
                                                void* stream) {
  if (!t_dev) return KGAT_ERR_INVALID;
  return lazy_catchup(p, m, v, n_rows, d, rows, n_list, last, 0, t_dev, hist_sz, hist_bc, hist_skip, cap, beta1,
                      beta2, eps, stream);
}

static int lazy_rows(float* p, float* m, float* v, int32_t d, const int32_t* rows, int64_t n_list, const float* Gc,
                     int64_t ldg, int32_t* last, int32_t t, float* hist_sz, float* hist_bc, int32_t* hist_skip,
                     int32_t cap, float step_size, float beta1, float beta2, float bc2_sqrt, float eps,
                     const int32_t* skip, kgat::StepSched sched, void* stream, int32_t* row_map = nullptr) {
  if (!lazy_args_ok(p, m, v, d, last, hist_sz, hist_bc, hist_skip, cap) || !rows || !Gc || n_list < 0 || ldg < d ||
      (sched.t == nullptr && t < 1))
    return KGAT_ERR_INVALID;
  const int64_t blocks = (std::max<int64_t>(n_list, 1) * d + 255) / 256;  // >= 1 block: the history entry
  hipLaunchKernelGGL(kgat::adam_lazy_rows_kernel, dim3(blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     p, m, v, d, rows, n_list, Gc, ldg, last, t, kgat::LazyHist{hist_sz, hist_bc, hist_skip, cap},
                     step_size, beta1, beta2, bc2_sqrt, eps, skip, sched, row_map);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int kgat_adam_lazy_rows_f32(float* p, float* m, float* v, int32_t d, const int32_t* rows, int64_t n_list,
                                       const float* Gc, int64_t ldg, int32_t* last, int32_t t, float* hist_sz,
                                       float* hist_bc, int32_t* hist_skip, int32_t cap, float step_size,
                                       float beta1, float beta2, float bc2_sqrt, float eps, const int32_t* skip,
                                       void* stream) {
  return lazy_rows(p, m, v, d, rows, n_list, Gc, ldg, last, t, hist_sz, hist_bc, hist_skip, cap, step_size, beta1,
                   beta2, bc2_sqrt, eps, skip, kgat::StepSched{nullptr, nullptr, nullptr}, stream);
}

extern "C" int kgat_adam_lazy_rows_sched_f32(float* p, float* m, float* v, int32_t d, const int32_t* rows,
                                             int64_t n_list, const float* Gc, int64_t ldg, int32_t* last,
                                             float* hist_sz, float* hist_bc, int32_t* hist_skip, int32_t cap,
                                             const int32_t* t_dev, const float* sched_sz, const float* sched_bc,
                                             float beta1, float beta2, float eps, const int32_t* skip, int32_t* row_map,
                                             int32_t t_add, int32_t* t_out, void* stream) {
  if (!t_dev || !sched_sz || !sched_bc) return KGAT_ERR_INVALID;
  return lazy_rows(p, m, v, d, rows, n_list, Gc, ldg, last, 0, hist_sz, hist_bc, hist_skip, cap, 0.f, beta1, beta2,
                   0.f, eps, skip, kgat::StepSched{t_dev, sched_sz, sched_bc, t_add, t_out}, stream, row_map);
}


extern "C" int kgat_adam_f32(float* p, const float* g, float* m, float* v, int64_t n, float step_size, float beta1,
                             float beta2, float bc2_sqrt, float eps, void* stream) {
  if (!p || !g || !m || !v || n < 0) return KGAT_ERR_INVALID;
  if ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(m) |
       reinterpret_cast<uintptr_t>(v)) & 15)
    return KGAT_ERR_INVALID;
  if (n == 0) return KGAT_OK;
  const int grid = kgat::blocks_for(n / 4 + 1, 256, kgat::kCUs * 8);
  hipLaunchKernelGGL(kgat::adam_kernel, dim3(grid), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), p, g, m, v,
                     n, step_size, beta1, beta2, bc2_sqrt, eps);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

namespace kgat {

// Row movers for the row-sharded mode: one 16-lane group per row, float4 per lane.
__global__ __launch_bounds__(256) void gather_rows_kernel(const float* __restrict__ src, int64_t lds,
                                                          const int32_t* __restrict__ rows, int64_t n, int d,
                                                          float* __restrict__ dst, int64_t ldd) {
  const int64_t g = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 4;
  const int lane = threadIdx.x & 15;
  if (g >= n) return;
  const int32_t r = rows[g];
  for (int c = lane * 4; c < d; c += 64) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r >= 0) v = *reinterpret_cast<const float4*>(src + r * lds + c);
    *reinterpret_cast<float4*>(dst + g * ldd + c) = v;
  }
}

__global__ __launch_bounds__(256) void scatter_rows_kernel(float* __restrict__ dst, int64_t ldd,
                                                           const int32_t* __restrict__ rows, int64_t n, int d,
                                                           const float* __restrict__ src, int64_t lds,
                                                           int accumulate) {
  const int64_t g = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 4;
  const int lane = threadIdx.x & 15;
  if (g >= n) return;
  const int32_t r = rows[g];
  if (r < 0) return;
  for (int c = lane * 4; c < d; c += 64) {
    float4 v = *reinterpret_cast<const float4*>(src + g * lds + c);
    float4* o = reinterpret_cast<float4*>(dst + r * ldd + c);
    if (accumulate) {
      const float4 w = *o;
      v = make_float4(w.x + v.x, w.y + v.y, w.z + v.z, w.w + v.w);
    }
    *o = v;
  }
}

__global__ __launch_bounds__(256) void add_kernel(float* __restrict__ y, const float* __restrict__ x, int64_t n) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) y[i] += x[i];
}

}  // namespace kgat

static bool rows_args_ok(const void* a, int64_t lda, const void* b, int64_t ldb, int d) {
  return a && b && d > 0 && (d & 3) == 0 && lda >= d && ldb >= d && (lda & 3) == 0 && (ldb & 3) == 0 &&
         (reinterpret_cast<uintptr_t>(a) & 15) == 0 && (reinterpret_cast<uintptr_t>(b) & 15) == 0;
}

extern "C" int kgat_gather_rows_f32(const float* src, int64_t lds, const int32_t* rows, int64_t n, int32_t d,
                                    float* dst, int64_t ldd, void* stream) {
  if (!rows || n < 0 || !rows_args_ok(src, lds, dst, ldd, d)) return KGAT_ERR_INVALID;
  if (n == 0) return KGAT_OK;
  hipLaunchKernelGGL(kgat::gather_rows_kernel, dim3(kgat::blocks_for(n, 16, 1 << 30)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), src, lds, rows, n, d, dst, ldd);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int kgat_scatter_rows_f32(float* dst, int64_t ldd, const int32_t* rows, int64_t n, int32_t d,
                                     const float* src, int64_t lds, int32_t accumulate, void* stream) {
  if (!rows || n < 0 || !rows_args_ok(dst, ldd, src, lds, d)) return KGAT_ERR_INVALID;
  if (n == 0) return KGAT_OK;
  hipLaunchKernelGGL(kgat::scatter_rows_kernel, dim3(kgat::blocks_for(n, 16, 1 << 30)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), dst, ldd, rows, n, d, src, lds, accumulate);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int kgat_add_f32(float* y, const float* x, int64_t n, void* stream) {
  if (!y || !x || n < 0) return KGAT_ERR_INVALID;
  if (n == 0) return KGAT_OK;
  hipLaunchKernelGGL(kgat::add_kernel, dim3(kgat::blocks_for(n, 256, kgat::kCUs * 8)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), y, x, n);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int kgat_gather_f32(const float* src, const int32_t* idx, int64_t n, float* dst, void* stream) {
  if (!src || !idx || !dst || n < 0) return KGAT_ERR_INVALID;
  if (n == 0) return KGAT_OK;
  hipLaunchKernelGGL(kgat::gather_kernel, dim3(kgat::blocks_for(n, 256, kgat::kCUs * 8)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), src, idx, n, dst);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int kgat_ids_check(const kgat_ids* ids, int64_t bound, int64_t* out, int32_t* bad, void* stream) {
  return kgat_ids_check_ex(ids, bound, out, bad, nullptr, stream);
}

extern "C" int kgat_ids_check_ex(const kgat_ids* ids, int64_t bound, int64_t* out, int32_t* bad, int32_t* bad_dev,
                                 void* stream) {
  if (!ids || ids->count < 1 || ids->count > KGAT_IDS_MAX) return KGAT_ERR_INVALID;
  int64_t b[KGAT_IDS_MAX];
  for (int k = 0; k < ids->count; ++k) b[k] = bound;
  return kgat_ids_check_multi(ids, b, out, bad, bad_dev, stream);
}

extern "C" int kgat_ids_check_multi(const kgat_ids* ids, const int64_t* bounds, int64_t* out, int32_t* bad,
                                    int32_t* bad_dev, void* stream) {
  if (!ids || !bounds || !out || !bad || ids->count < 1 || ids->count > KGAT_IDS_MAX) return KGAT_ERR_INVALID;
  kgat::IdBounds bb{};
  int64_t total = 0;
  for (int k = 0; k < ids->count; ++k) {
    if (ids->n[k] < 0 || (ids->n[k] && !ids->ptr[k]) || bounds[k] < 0) return KGAT_ERR_INVALID;
    total += ids->n[k];
    bb.b[k] = bounds[k];
  }
  if (total == 0) return KGAT_OK;
  hipLaunchKernelGGL(kgat::ids_check_kernel, dim3(kgat::blocks_for(total, 256, kgat::kCUs * 4)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), *ids, total, bb, out, bad, bad_dev);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int kgat_map_build(const int32_t* ids, int64_t n, int32_t* node_map, void* stream) {
  if (!node_map || n < 0 || (n && !ids) || n > INT32_MAX) return KGAT_ERR_INVALID;
  if (n == 0) return KGAT_OK;
  hipLaunchKernelGGL(kgat::map_build_kernel, dim3(kgat::blocks_for(n, 256, kgat::kCUs * 4)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), ids, n, node_map);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int kgat_map_build_checked(int32_t* ids, int64_t n, int32_t* node_map, int64_t n_nodes, int32_t* bad_host,
                                      int32_t* bad_dev, void* stream) {
  if (!node_map || n < 0 || (n && !ids) || n > INT32_MAX || n_nodes < 0 || n_nodes > INT32_MAX)
    return KGAT_ERR_INVALID;
  if (n == 0) return KGAT_OK;
  hipLaunchKernelGGL(kgat::map_build_checked_kernel, dim3(kgat::blocks_for(n, 256, kgat::kCUs * 4)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), ids, n, node_map, n_nodes, bad_host, bad_dev);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int kgat_ids_sanitize_i32(int32_t* ids, int64_t n, int64_t bound, int32_t* bad_host, int32_t* bad_dev,
                                     void* stream) {
  if (n < 0 || (n && !ids) || bound < 0) return KGAT_ERR_INVALID;
  if (n == 0) return KGAT_OK;
  hipLaunchKernelGGL(kgat::ids_sanitize_kernel, dim3(kgat::blocks_for(n, 256, kgat::kCUs * 4)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), ids, n, bound, bad_host, bad_dev);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int kgat_map_compose(const int32_t* a, int64_t n, const int32_t* b, int32_t offset, int32_t* out,
                                void* stream) {
  if (n < 0 || (n && (!a || !out))) return KGAT_ERR_INVALID;
  if (n == 0) return KGAT_OK;
  hipLaunchKernelGGL(kgat::map_compose_kernel, dim3(kgat::blocks_for(n, 256, kgat::kCUs * 4)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), a, n, b, offset, out);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

extern "C" int kgat_fill_f32(float* dst, int64_t n, float value, void* stream) {
  if (!dst || n < 0) return KGAT_ERR_INVALID;
  if (n == 0) return KGAT_OK;
  hipLaunchKernelGGL(kgat::fill_kernel, dim3(kgat::blocks_for(n, 256, kgat::kCUs * 8)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), dst, n, value);
  KGAT_LAUNCH_CHECK();
  return KGAT_OK;
}

// Host: rows with degree > long_threshold become long rows cut into
// ceil(deg / seg_len) segments (see spmm.hip).
extern "C" int kgat_csr_plan(const int64_t* rowptr, int64_t n_rows, int32_t long_threshold, int32_t seg_len,
                             int32_t* n_long, int32_t* n_seg, int32_t* long_rows, int32_t* long_seg_off,
                             int32_t* seg_row, int64_t* seg_beg) {
  if (!rowptr || n_rows < 0 || long_threshold < 1 || seg_len < 1 || !n_long || !n_seg) return KGAT_ERR_INVALID;
  int64_t nl = 0, ns = 0;
  for (int64_t r = 0; r < n_rows; ++r) {
    const int64_t deg = rowptr[r + 1] - rowptr[r];
    if (deg > long_threshold) {
      const int64_t k = (deg + seg_len - 1) / seg_len;
      if (long_rows) {
        long_rows[nl] = static_cast<int32_t>(r);
        long_seg_off[nl] = static_cast<int32_t>(ns);
        for (int64_t j = 0; j < k; ++j) {
          seg_row[ns + j] = static_cast<int32_t>(r);
          seg_beg[ns + j] = rowptr[r] + j * seg_len;
        }
      }
      ++nl;
      ns += k;
    }
  }
  if (long_rows) long_seg_off[nl] = static_cast<int32_t>(ns);
  if (nl > 0x7fffffff || ns > 0x7fffffff) return KGAT_ERR_INVALID;
  *n_long = static_cast<int32_t>(nl);
  *n_seg = static_cast<int32_t>(ns);
  return KGAT_OK;
}

// Host: the SpMM's long-row plan with column-aware cuts.  A long row (degree > long_threshold) is
// cut where a segment reaches seg_len entries, or where its column crosses a multiple of col_block
// once the segment holds min_piece entries: a hub row's segments then each gather from one
// col_block-row slice of the source table (with kgat_csr_seg_order, one XCD's L2 serves a few
// slices instead of the whole table).  A pure function of each row's entries, so a row view's plan
// matches the full matrix's row by row.  Pass null outputs to only count.
extern "C" int kgat_csr_plan_cols(const int64_t* rowptr, const int32_t* col, int64_t n_rows, int32_t long_threshold,
                                  int32_t seg_len, int32_t col_block, int32_t min_piece, int32_t* n_long,
                                  int32_t* n_seg, int32_t* long_rows, int32_t* long_seg_off, int32_t* seg_row,
                                  int64_t* seg_beg) {
  if (!rowptr || n_rows < 0 || long_threshold < 1 || seg_len < 1 || col_block < 1 || min_piece < 1 || !n_long ||
      !n_seg || (n_rows > 0 && !col))
    return KGAT_ERR_INVALID;
  int64_t nl = 0, ns = 0;
  for (int64_t r = 0; r < n_rows; ++r) {
    const int64_t a = rowptr[r], b = rowptr[r + 1];
    if (b - a <= long_threshold) continue;
    if (long_rows) {
      long_rows[nl] = static_cast<int32_t>(r);
      long_seg_off[nl] = static_cast<int32_t>(ns);
    }
    int64_t s = a;
    for (int64_t i = a + 1; i < b; ++i) {
      if (i - s >= seg_len || (col[i] / col_block != col[i - 1] / col_block && i - s >= min_piece)) {
        if (seg_row) {
          seg_row[ns] = static_cast<int32_t>(r);
          seg_beg[ns] = s;
        }
        ++ns;
        s = i;
      }
    }
    if (seg_row) {
      seg_row[ns] = static_cast<int32_t>(r);
      seg_beg[ns] = s;
    }
    ++ns;
    ++nl;
  }
  if (long_rows) long_seg_off[nl] = static_cast<int32_t>(ns);
  if (nl > 0x7fffffff || ns > 0x7fffffff) return KGAT_ERR_INVALID;
  *n_long = static_cast<int32_t>(nl);
  *n_seg = static_cast<int32_t>(ns);
  return KGAT_OK;
}

// Host: the SpMM's launch order of the long-row segments (kgat_csr::seg_order).  Segments sorted
// by their first column (stable), then dealt so that the long-row blocks sharing an XCD (blocks
// b, b + 8, ... -- round-robin dispatch) take one contiguous run of the sorted list: each XCD's
// L2 then holds the source rows of one eighth of the column range instead of all of it (the hub
// rows of a user -> item graph all gather the same user table).
extern "C" int kgat_csr_seg_order(const int32_t* col, const int64_t* seg_beg, int32_t n_seg, int32_t* order) {
  if (n_seg < 0 || (n_seg > 0 && (!col || !seg_beg || !order))) return KGAT_ERR_INVALID;
  constexpr int kXcds = 8;
  std::vector<int32_t> by_col(n_seg);
  for (int32_t s = 0; s < n_seg; ++s) by_col[s] = s;
  std::stable_sort(by_col.begin(), by_col.end(),
                   [&](int32_t a, int32_t b) { return col[seg_beg[a]] < col[seg_beg[b]]; });
  const int64_t nb = (static_cast<int64_t>(n_seg) + 3) / 4;
  int64_t start[kXcds + 1] = {0};
  for (int x = 0; x < kXcds; ++x) start[x + 1] = start[x] + (nb > x ? (nb - x + kXcds - 1) / kXcds : 0);
  for (int64_t b = 0; b < nb; ++b) {
    const int64_t vb = start[b % kXcds] + b / kXcds;
    for (int w = 0; w < 4; ++w) {
      const int64_t pos = vb * 4 + w;
      order[b * 4 + w] = pos < n_seg ? by_col[pos] : n_seg;
    }
  }
  return KGAT_OK;
}
