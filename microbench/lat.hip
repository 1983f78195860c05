// Microbenchmark: dependent latencies of the primitives a 64x64 Cholesky critical path is built from
// (gfx950, one wave unless noted), in s_memtime ticks and, via s_memrealtime (100 MHz), in ns.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 microbench/lat.hip -o microbench/lat
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <utility>

typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double readlane_d(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}


template <int L>
__device__ __forceinline__ double dpp_bcast(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0x150 + L, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x150 + L, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
template <int... Q>
__device__ __forceinline__ double dpp16(double v, double acc, std::integer_sequence<int, Q...>) {
  ((acc = fma(dpp_bcast<Q>(v), 1.0000001, acc)), ...);
  return acc;
}
__device__ __forceinline__ double rl16(double v, double acc) {
  for (int q = 0; q < 16; ++q) acc = fma(readlane_d(v, q), 1.0000001, acc);
  return acc;
}
constexpr int IT = 256;

__global__ void k_lat(double* out, long long* res, double x) {
  __shared__ double sh[1024];
  const int lane = threadIdx.x & 63;
  double v = x + lane * 1e-3;
  long long t0, t1, r0, r1;
  int slot = 0;
#define MEASURE(body)                                         \
  __syncthreads();                                           \
  t0 = __builtin_amdgcn_s_memtime();                         \
  r0 = __builtin_amdgcn_s_memrealtime();                     \
  for (int i = 0; i < IT; ++i) { body; }                     \
  t1 = __builtin_amdgcn_s_memtime();                         \
  r1 = __builtin_amdgcn_s_memrealtime();                     \
  if (threadIdx.x == 0) { res[2 * slot] = t1 - t0; res[2 * slot + 1] = r1 - r0; }  \
  ++slot;
  // 0: dependent v_fma_f64
  MEASURE(v = fma(v, 1.0000001, 1e-9));
  // 1: dependent rsq_f64
  MEASURE(v = __builtin_amdgcn_rsq(v + 1.0));
  // 2: rsq + 2 Newton steps (the pivot chain)
  MEASURE({
    double p = v + 1.0;
    double y = __builtin_amdgcn_rsq(p);
    const double h = 0.5 * p;
    y = y * (1.5 - h * y * y);
    y = y * (1.5 - h * y * y);
    v = y;
  });
  // 3: readlane f64 -> use (broadcast chain)
  MEASURE(v = readlane_d(v, i & 63) * 1.0000001);
  // 4: shfl (ds_bpermute) chain
  MEASURE(v = __shfl(v, (lane + 1) & 63, 64) * 1.0000001);
  // 5: LDS write -> read chain (same wave)
  MEASURE({
    sh[lane] = v;
    __builtin_amdgcn_s_waitcnt(0xc07f);
    v = sh[(lane + 1) & 63] * 1.0000001;
  });
  // 6: dependent MFMA f64 16x16x4 chain
  d4 acc = {v, v, v, v};
  MEASURE(acc = __builtin_amdgcn_mfma_f64_16x16x4f64(v, 1.0000001, acc, 0, 0, 0));
  // 7: 4 independent MFMA chains interleaved (throughput per MFMA)
  d4 a1 = acc, a2 = acc, a3 = acc;
  MEASURE({
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(v, 1.0000001, acc, 0, 0, 0);
    a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(v, 1.0000001, a1, 0, 0, 0);
    a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(v, 1.0000001, a2, 0, 0, 0);
    a3 = __builtin_amdgcn_mfma_f64_16x16x4f64(v, 1.0000001, a3, 0, 0, 0);
  });
  // 8: s_barrier (all waves of the block)
  MEASURE(__syncthreads());
  // 9: v_div-free reciprocal via rcp + 2 NR
  MEASURE({
    double y = __builtin_amdgcn_rcp(v + 2.0);
    const double p = v + 2.0;
    y = y * (2.0 - p * y);
    y = y * (2.0 - p * y);
    v = y;
  });
  // 10: DPP row broadcast style: __shfl_xor 1 chain
  MEASURE(v = __shfl_xor(v, 1, 64) * 1.0000001);
  // 11: DPP row_newbcast (lane 1 of each row of 16) f64 chain
  MEASURE({
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0x151, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x151, 0xf, 0xf, false);
    v = __longlong_as_double(((long long)hi << 32) | (unsigned)lo) * 1.0000001;
  });
  // 12: permlane32_swap f64 chain
  MEASURE({
    const long long b = __double_as_longlong(v);
    auto r0 = __builtin_amdgcn_permlane32_swap((int)b, (int)b, false, false);
    auto r1 = __builtin_amdgcn_permlane32_swap((int)(b >> 32), (int)(b >> 32), false, false);
    v = __longlong_as_double(((long long)r1[0] << 32) | (unsigned)r0[0]) * 1.0000001;
  });
  // 13: 16 independent readlane_d (throughput per readlane_d)
  double acc16 = 0.0;
  MEASURE({ acc16 = rl16(v, acc16); v = v + acc16 * 1e-30; });
  // 14: 16 independent DPP newbcast f64 (throughput)
  MEASURE({ acc16 = dpp16(v, acc16, std::make_integer_sequence<int, 16>{}); v = v + acc16 * 1e-30; });
  out[threadIdx.x] = v + acc[0] + a1[1] + a2[2] + a3[3] + acc16;
}

int main() {
  double* o;
  long long* r;
  (void)hipMalloc(&o, 1 << 16);
  (void)hipMalloc(&r, 1024);
  const char* names[] = {"fma_f64 dep", "rsq_f64 dep", "rsq+2NR", "readlane f64+mul", "shfl(bpermute)+mul",
                         "lds st->ld+mul", "mfma_f64_16x16x4 dep", "mfma x4 indep (per 4)", "s_barrier",
                         "rcp+2NR", "shfl_xor1+mul", "dpp newbcast f64+mul", "permlane32_swap f64+mul", "16x readlane_d+fma (per 16)", "16x dpp bcast f64+fma (per 16)"};
  for (int wpb : {1, 4}) {
    for (int rep = 0; rep < 2; ++rep) k_lat<<<1, 64 * wpb>>>(o, r, 0.5);
    (void)hipDeviceSynchronize();
    long long h[64];
    (void)hipMemcpy(h, r, sizeof(h), hipMemcpyDeviceToHost);
    printf("waves/block = %d\n", wpb);
    for (int s = 0; s < 15; ++s)
      printf("  %-26s %8.1f ticks  %7.2f ns per op\n", names[s], (double)h[2 * s] / IT, 10.0 * h[2 * s + 1] / IT);
  }
  return 0;
}
