// In-kernel phase timeline of the bi-interaction forward (64 -> 64, the C2 layer-0 shape): the
// product kernel's sub-tile loop (biinter_fwd_kernel<64, 64, false, 2, 4>, same helpers, same
// grid) with s_memtime stamps around its two phases -- (a) issue the sub-tile's X / S row loads and
// form U, M (waits for the loads), (b) the MFMA products + epilogue + H / state stores issued -- so
// the per-wave cycles of each phase and the waves' lifetime can be compared with the kernel time.
// Measurement tool (not product code): builds against csrc/biinter.hip directly.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -I<pkg>/csrc tools/biinter_stamps.hip -o tools/biinter_stamps
#include "biinter.hip"

#include <cstdio>
#include <vector>

namespace kgat {

__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

template <int DIN, int DOUT, bool SB>
__global__ __launch_bounds__(256, 2) void fwd_stamp_kernel(const float* __restrict__ X, int64_t ldx,
                                                           const float* __restrict__ S, int64_t lds,
                                                           const float* __restrict__ W1, const float* __restrict__ b1,
                                                           const float* __restrict__ W2, const float* __restrict__ b2,
                                                           float* __restrict__ H, int64_t ldh, int64_t n, float p,
                                                           uint64_t seed, float* __restrict__ norm_out,
                                                           uint64_t* __restrict__ mask_out,
                                                           unsigned long long* __restrict__ stamps) {
  using B = BiShape<DIN, DOUT>;
  constexpr int NWV = 4;
  __shared__ __attribute__((aligned(16))) float smem[2 * DOUT * B::WLD];
  float* w1s = smem;
  float* w2s = smem + DOUT * B::WLD;
  const unsigned long long t_start = stamp();
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
  unsigned long long t_load = 0, t_comp = 0, count = 0;
  for (int64_t st = static_cast<int64_t>(blockIdx.x) * NWV + (threadIdx.x >> 6); st < nsub; st += stride) {
    const unsigned long long t0 = stamp();
    float nx[B::KQ], ns[B::KQ];
    load_rows<DIN>(X, ldx, st * 16 + c, n, q, nx);
    load_rows<DIN>(S, lds, st * 16 + c, n, q, ns);
    float u[B::KQ], m[B::KQ];
#pragma unroll
    for (int t = 0; t < B::KQ; ++t) {
      u[t] = nx[t] + ns[t];
      m[t] = nx[t] * ns[t];
    }
#pragma unroll
    for (int t = 0; t < B::KQ; ++t) asm volatile("" ::"v"(u[t]), "v"(m[t]));  // formed before the stamp
    const unsigned long long t1 = stamp();
    bi_fwd_subtile<DIN, DOUT, SB>(u, m, st, lane, w1s, w2s, bias1, bias2, p, scale, thr, seed, H, ldh, n, norm_out,
                                  mask_out, 0);
    const unsigned long long t2 = stamp();
    t_load += t1 - t0;
    t_comp += t2 - t1;
    ++count;
  }
  const unsigned long long t_end = stamp();
  if (lane == 0) {
    const int64_t gw = static_cast<int64_t>(blockIdx.x) * NWV + (threadIdx.x >> 6);
    stamps[gw * 5 + 0] = t_load;
    stamps[gw * 5 + 1] = t_comp;
    stamps[gw * 5 + 2] = count;
    stamps[gw * 5 + 3] = t_end - t_start;
    stamps[gw * 5 + 4] = t_start;
  }
}

}  // namespace kgat

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main() {
  const int64_t n = 1000000;
  const int din = 64, dout = 64;
  std::vector<float> hx(n * din);
  uint64_t s = 88172645463325252ull;
  for (auto& v : hx) {
    s ^= s << 13, s ^= s >> 7, s ^= s << 17;
    v = static_cast<float>(static_cast<int64_t>(s % 2000001) - 1000000) * 1e-6f;
  }
  std::vector<float> hw(dout * din);
  for (auto& v : hw) {
    s ^= s << 13, s ^= s >> 7, s ^= s << 17;
    v = static_cast<float>(static_cast<int64_t>(s % 2001) - 1000) * 1e-4f;
  }
  float *X, *S, *W1, *W2, *b, *H, *norm;
  uint64_t* mask;
  unsigned long long* stamps;
  CK(hipMalloc(&X, n * din * 4));
  CK(hipMalloc(&S, n * din * 4));
  CK(hipMalloc(&W1, dout * din * 4));
  CK(hipMalloc(&W2, dout * din * 4));
  CK(hipMalloc(&b, dout * 4));
  CK(hipMalloc(&H, n * dout * 4));
  CK(hipMalloc(&norm, n * 4));
  CK(hipMalloc(&mask, (n + 15) / 16 * 64 * 8));
  CK(hipMemcpy(X, hx.data(), n * din * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(S, hx.data(), n * din * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(W1, hw.data(), dout * din * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(W2, hw.data(), dout * din * 4, hipMemcpyHostToDevice));
  CK(hipMemset(b, 0, dout * 4));
  // the product launch's grid (launch_fwd, default variant): blocks_for(n, 64, kCUs * 8)
  const int grid = kgat::blocks_for(n, 64, kgat::kCUs * 8);
  const int waves = grid * 4;
  CK(hipMalloc(&stamps, static_cast<size_t>(waves) * 5 * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int sb = 1; sb >= 0; --sb) {
  float ms_prod = 0.f, ms_stamp = 0.f;
  for (int rep = 0; rep < 12; ++rep) {
    CK(hipEventRecord(e0));
    if (kgat_biinter_fwd_f32(X, din, S, din, W1, b, W2, b, H, dout, n, din, dout, 0.1f, 7, norm, mask, nullptr) != 0)
      return 1;
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float t;
    CK(hipEventElapsedTime(&t, e0, e1));
    if (rep >= 2) ms_prod += t / 10;
    CK(hipEventRecord(e0));
    if (sb)
      hipLaunchKernelGGL((kgat::fwd_stamp_kernel<64, 64, true>), dim3(grid), dim3(256), 0, nullptr, X, (int64_t)din, S,
                         (int64_t)din, W1, b, W2, b, H, (int64_t)dout, n, 0.1f, (uint64_t)7, norm, mask, stamps);
    else
      hipLaunchKernelGGL((kgat::fwd_stamp_kernel<64, 64, false>), dim3(grid), dim3(256), 0, nullptr, X, (int64_t)din,
                         S, (int64_t)din, W1, b, W2, b, H, (int64_t)dout, n, 0.1f, (uint64_t)7, norm, mask, stamps);
    CK(hipGetLastError());
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&t, e0, e1));
    if (rep >= 2) ms_stamp += t / 10;
  }
  std::vector<unsigned long long> hs(static_cast<size_t>(waves) * 5);
  CK(hipMemcpy(hs.data(), stamps, hs.size() * 8, hipMemcpyDeviceToHost));
  double load = 0, comp = 0, cnt = 0, life = 0;
  unsigned long long tmin = ~0ull, tmax = 0;
  for (int w = 0; w < waves; ++w) {
    load += hs[w * 5 + 0];
    comp += hs[w * 5 + 1];
    cnt += hs[w * 5 + 2];
    life += hs[w * 5 + 3];
    tmin = std::min(tmin, hs[w * 5 + 4]);
    tmax = std::max(tmax, hs[w * 5 + 4] + hs[w * 5 + 3]);
  }
  printf("{\"kernel\": \"biinter_fwd<64,64> 1M rows\", \"sched_barrier_per_column_block\": %d, \"product_us\": %.1f, "
         "\"stamped_us\": %.1f, \"waves\": %d, \"subtiles_per_wave\": %.2f, \"load_phase_cycles_per_subtile\": %.0f, "
         "\"compute_phase_cycles_per_subtile\": %.0f, \"wave_lifetime_cycles\": %.0f, \"span_cycles\": %llu}\n",
         sb, ms_prod * 1e3, ms_stamp * 1e3, waves, cnt / waves, load / cnt, comp / cnt, life / waves, tmax - tmin);
  }
  return 0;
}
