// Microbenchmark: sustained v_mfma_f64_16x16x4_f64 throughput on one MI355X (register-only loop, 16
// independent accumulators per wave), to calibrate the FP64 MFMA roofline used by bench.py.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void k_peak(double* out, int iters, double seed) {
  d4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = d4{0, 0, 0, 0};
  double a = seed + threadIdx.x, b = seed * 0.5 + threadIdx.x;
  for (int it = 0; it < iters; it += 16) {
#pragma unroll
    for (int i = 0; i < NACC * 16; ++i) acc[i % NACC] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i % NACC], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 12345.678) out[threadIdx.x] = s;
}

template <int NACC>
void run(int wgs, int threads, int iters) {
  double* out;
  (void)hipMalloc(&out, 4096);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  k_peak<NACC><<<wgs, threads>>>(out, iters, 1.0);
  (void)hipEventRecord(e0);
  k_peak<NACC><<<wgs, threads>>>(out, iters, 1.0);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double flops = 2.0 * 16 * 16 * 4 * (double)NACC * iters * wgs * (threads / 64);
  printf("nacc=%d wgs=%d threads=%d: %.3f ms  %.2f TFLOP/s\n", NACC, wgs, threads, ms, flops / ms / 1e9);
  (void)hipFree(out);
}

int main() {
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  int clk = 0;
  (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
  printf("CUs=%d clock=%d kHz\n", ncu, clk);
  run<16>(ncu, 256, 20000);
  run<16>(2 * ncu, 256, 20000);
  run<8>(2 * ncu, 256, 40000);
  run<4>(2 * ncu, 256, 80000);
  run<16>(4 * ncu, 256, 10000);
  return 0;
}
