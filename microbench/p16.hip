// Microbenchmark: the 16-column lane-per-row elimination of potrf64.hpp in isolation (one wave, matrix in
// registers, many repetitions), with variants that remove one ingredient at a time to attribute the cost.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 microbench/p16.hip -o microbench/p16
#include <hip/hip_runtime.h>
#include <stdio.h>

__device__ __forceinline__ double rcp_nr(double p) {
  double y = __builtin_amdgcn_rcp(p);
  y = y * (2.0 - p * y);
  y = y * (2.0 - p * y);
  return y;
}
__device__ __forceinline__ double readlane_d(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// V: 0 full, 1 no readlanes for lc (uniform constant), 2 no rcp chain, 3 no fmacs, 4 readlane to VGPR copy
template <int V>
__device__ __forceinline__ void p16(double (&a)[16], int r) {
  double piv = readlane_d(a[0], 0);
  double rinv = rcp_nr(piv);
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    double lc[16];
#pragma unroll
    for (int c = j + 1; c < 16; ++c) lc[c] = (V == 1) ? 0.25 + c : readlane_d(a[j], c);
    const double rj = rinv;
    if (j + 1 < 16) {
      const double dn = readlane_d(a[j + 1], j + 1);
      piv = fma(-(lc[j + 1] * rj), lc[j + 1], dn);
      rinv = (V == 2) ? piv : rcp_nr(piv);
    }
    const double t = a[j] * rj;
    if (V != 3) {
#pragma unroll
      for (int c = j + 1; c < 16; ++c) a[c] = fma(-t, lc[c], a[c]);
    } else {
      a[j + 1 < 16 ? j + 1 : 15] += t;
    }
  }
}

template <int V>
__global__ void k_p16(double* out, long long* res, double x, int reps) {
  const int lane = threadIdx.x & 63, r = lane & 15;
  double a[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) a[c] = (c == r) ? 16.0 + x : 0.01 * (c + r);
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < reps; ++i) {
    p16<V>(a, r);
#pragma unroll
    for (int c = 0; c < 16; ++c) a[c] = (c == r) ? 16.0 + a[c] * 1e-9 : a[c] * 1e-3;  // keep it well-posed
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
#pragma unroll
  for (int c = 0; c < 16; ++c) s += a[c];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) res[V] = t1 - t0;
}

int main() {
  double* o;
  long long* r;
  (void)hipMalloc(&o, 1 << 16);
  (void)hipMalloc(&r, 1024);
  const int reps = 100;
  for (int k = 0; k < 2; ++k) {
    k_p16<0><<<1, 64>>>(o, r, 0.5, reps);
    k_p16<1><<<1, 64>>>(o, r, 0.5, reps);
    k_p16<2><<<1, 64>>>(o, r, 0.5, reps);
    k_p16<3><<<1, 64>>>(o, r, 0.5, reps);
  }
  (void)hipDeviceSynchronize();
  long long h[8];
  (void)hipMemcpy(h, r, sizeof(h), hipMemcpyDeviceToHost);
  const char* names[] = {"full", "no lc readlanes", "no rcp chain", "no fmac updates"};
  for (int v = 0; v < 4; ++v) printf("  %-18s %8.1f cycles per 16-column sweep\n", names[v], (double)h[v] / reps);
  return 0;
}
