// Microbenchmark: 16x16 Cholesky in one wave with the identity border (lanes 16-31) and a rhs row (lanes
// 32-47) eliminated by the same column operations (lanes = rows of three bordered systems), cycles via
// s_memtime.  Validates the base case of the tall dataflow POTRF before building it.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

__device__ __forceinline__ double rsqrt_nr(double p) {
  double y = __builtin_amdgcn_rsq(p);
  const double h = 0.5 * p;
  y = y * (1.5 - h * y * y);
  y = y * (1.5 - h * y * y);
  return y;
}
__device__ __forceinline__ double readlane_d(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__global__ void k16(const double* A, const double* b, double* out, unsigned long long* cyc) {
  const int lane = threadIdx.x, sys = lane >> 4, r = lane & 15;
  double v[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const double a = A[r * 16 + c];
    v[c] = sys == 0 ? (c <= r ? a : 0.0) : sys == 1 ? (c == r ? 1.0 : 0.0) : sys == 2 ? b[c] : 0.0;
  }
  __syncthreads();
  unsigned long long t0;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0) :: "memory");
#pragma unroll
  for (int c = 0; c < 16; ++c) asm volatile("" : "+v"(v[c]) : "s"(t0));  // the work depends on the first stamp
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const double piv = readlane_d(v[j], j);
    const double rl = rsqrt_nr(piv);
    v[j] *= rl;
#pragma unroll
    for (int c = j + 1; c < 16; ++c) v[c] = fma(-v[j], readlane_d(v[j], c), v[c]);
  }
#pragma unroll
  for (int c = 0; c < 16; ++c) asm volatile("" : "+v"(v[c]));  // results complete before the second stamp
  unsigned long long t1;
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1) :: "memory");
#pragma unroll
  for (int c = 0; c < 16; ++c) out[lane * 16 + c] = v[c];
  if (lane == 0) *cyc = t1 - t0;
}

int main() {
  double hA[256], hb[16], B[256];
  srand(3);
  for (int i = 0; i < 256; ++i) B[i] = (double)rand() / RAND_MAX - 0.5;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double s = 0;
      for (int k = 0; k < 16; ++k) s += B[i * 16 + k] * B[j * 16 + k];
      hA[i * 16 + j] = s + (i == j ? 1.0 : 0.0);
    }
  for (int i = 0; i < 16; ++i) hb[i] = i + 1.0;
  double *dA, *db, *dout;
  unsigned long long* dc;
  (void)hipMalloc(&dA, sizeof(hA));
  (void)hipMalloc(&db, sizeof(hb));
  (void)hipMalloc(&dout, 64 * 16 * 8);
  (void)hipMalloc(&dc, 8);
  (void)hipMemcpy(dA, hA, sizeof(hA), hipMemcpyHostToDevice);
  (void)hipMemcpy(db, hb, sizeof(hb), hipMemcpyHostToDevice);
  k16<<<1, 64>>>(dA, db, dout, dc);
  k16<<<1, 64>>>(dA, db, dout, dc);
  double o[64 * 16];
  unsigned long long c;
  (void)hipMemcpy(o, dout, sizeof(o), hipMemcpyDeviceToHost);
  (void)hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
  double e1 = 0, e2 = 0, e3 = 0;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j <= i; ++j) {
      double s = 0;
      for (int k = 0; k <= j; ++k) s += o[i * 16 + k] * o[j * 16 + k];
      e1 = fmax(e1, fabs(s - hA[i * 16 + j]));
    }
  for (int i = 0; i < 16; ++i)  // lanes 16..31: row r = W[r][c] = Linv[c][r]; check (L Linv)[i][j]
    for (int j = 0; j < 16; ++j) {
      double s = 0;
      for (int k = 0; k <= i; ++k) s += o[i * 16 + k] * o[(16 + j) * 16 + k];
      e2 = fmax(e2, fabs(s - (i == j ? 1.0 : 0.0)));
    }
  for (int i = 0; i < 16; ++i) {
    double s = 0;
    for (int k = 0; k <= i; ++k) s += o[i * 16 + k] * o[32 * 16 + k];
    e3 = fmax(e3, fabs(s - hb[i]));
  }
  printf("potrf16: %llu cycles; err LL'=%.2e  L Linv=%.2e  Lw=%.2e\n", c, e1, e2, e3);
  return 0;
}
