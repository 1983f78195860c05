// Microbenchmark: FP64 VALU v_fma_f64 issue rate and dependent latency on gfx950 (cycles via s_memtime).
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int CH>
__global__ void k_fma(double* out, unsigned long long* cyc, int iters, double x) {
  double a[CH];
  for (int i = 0; i < CH; ++i) a[i] = x + threadIdx.x + i;
  const double b = 1.0000001, c = 1e-9;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
      for (int i = 0; i < CH; ++i) a[i] = fma(a[i], b, c);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
  for (int i = 0; i < CH; ++i) s += a[i];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int CH>
void run(int waves_per_block) {
  double* o;
  unsigned long long* c;
  (void)hipMalloc(&o, 1 << 16);
  (void)hipMalloc(&c, 8);
  const int iters = 1000;
  k_fma<CH><<<1, 64 * waves_per_block>>>(o, c, iters, 1.0);
  k_fma<CH><<<1, 64 * waves_per_block>>>(o, c, iters, 1.0);
  unsigned long long h;
  (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
  const double n = (double)iters * 16 * CH;
  printf("chains=%2d waves/block=%d: %.2f cycles per v_fma_f64 (per wave)\n", CH, waves_per_block, h / n);
}

int main() {
  run<1>(1);
  run<2>(1);
  run<4>(1);
  run<8>(1);
  run<16>(1);
  run<8>(4);
  run<8>(8);
  return 0;
}
