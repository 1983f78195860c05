// Microbenchmark: issue cost per instruction (one wave, many independent chains) of the broadcast
// primitives available to a lane-per-row / lane-per-column dense factorization on gfx950.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 microbench/tput.hip -o microbench/tput
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int IT = 64;
constexpr int CH = 16;

__device__ __forceinline__ double dpp_bcast(double v, int) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0x153, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0x153, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__global__ void k_tput(double* out, long long* res, double x) {
  __shared__ double sh[256];
  const int lane = threadIdx.x & 63;
  double a[CH];
_Pragma("unroll")
  for (int i = 0; i < CH; ++i) a[i] = x + lane + i;
  sh[lane] = x * lane;
  __syncthreads();
  long long t0, t1;
  int slot = 0;
#define MEASURE(body)                                                  \
  t0 = __builtin_amdgcn_s_memtime();                                   \
  for (int it = 0; it < IT; ++it) { body; }                            \
  t1 = __builtin_amdgcn_s_memtime();                                   \
  if (threadIdx.x == 0) res[slot] = t1 - t0;                           \
  ++slot;
  // 0: independent v_fma_f64 (VGPR operands)
  MEASURE(_Pragma("unroll")
      for (int i = 0; i < CH; ++i) a[i] = fma(a[i], 1.0000001, a[(i + 1) % CH]));
  // 1: v_readlane_b32 pairs feeding fma (SGPR operand)
  MEASURE(_Pragma("unroll")
      for (int i = 0; i < CH; ++i) {
        const long long b = __double_as_longlong(a[(i + 3) % CH]);
        const int lo = __builtin_amdgcn_readlane((int)b, i);
        const int hi = __builtin_amdgcn_readlane((int)(b >> 32), i);
        a[i] = fma(a[i], __longlong_as_double(((long long)hi << 32) | (unsigned)lo), 1e-9);
      });
  // 2: DPP row_newbcast pairs feeding fma
  MEASURE(_Pragma("unroll")
      for (int i = 0; i < CH; ++i) a[i] = fma(a[i], dpp_bcast(a[(i + 3) % CH], i), 1e-9));
  // 3: LDS broadcast ds_read_b128 (same address in all lanes) feeding 2 fma
  MEASURE(_Pragma("unroll")
      for (int i = 0; i < CH; i += 2) {
        typedef double v2 __attribute__((ext_vector_type(2)));
        const v2 l = *reinterpret_cast<const v2*>(&sh[(2 * i + it) & 127]);
        a[i] = fma(a[i], l[0], 1e-9);
        a[i + 1] = fma(a[i + 1], l[1], 1e-9);
      });
  // 4: v_mul_f64 independent
  MEASURE(_Pragma("unroll")
      for (int i = 0; i < CH; ++i) a[i] = a[i] * a[(i + 5) % CH]);
  double s = 0;
_Pragma("unroll")
  for (int i = 0; i < CH; ++i) s += a[i];
  out[threadIdx.x] = s;
}

int main() {
  double* o;
  long long* r;
  (void)hipMalloc(&o, 1 << 16);
  (void)hipMalloc(&r, 1024);
  const char* names[] = {"fma_f64 indep", "readlane pair + fma", "dpp newbcast pair + fma", "ds_read_b128 bcast + 2 fma",
                         "mul_f64 indep"};
  const double per[] = {CH, CH, CH, CH / 2, CH};
  for (int wpb : {1, 4, 8}) {
    for (int rep = 0; rep < 2; ++rep) k_tput<<<1, 64 * wpb>>>(o, r, 0.5);
    (void)hipDeviceSynchronize();
    long long h[8];
    (void)hipMemcpy(h, r, sizeof(h), hipMemcpyDeviceToHost);
    printf("waves/block = %d\n", wpb);
    for (int s = 0; s < 5; ++s) printf("  %-28s %7.2f cycles per unit\n", names[s], (double)h[s] / (IT * per[s]));
  }
  return 0;
}
