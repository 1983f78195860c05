// mfma_f64_semantics.hip — how v_mfma_f64_16x16x4f64 rounds its 4-term dot products: each output element of one
// MFMA is compared with (a) a chain of IEEE fmas in k order 0..3 on top of the accumulator, (b) the reverse order,
// (c) the exactly rounded value (long-double-free: two-sum based).  Inputs are built to cancel.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

typedef double d4f __attribute__((ext_vector_type(4)));

// one wave: A 16x4, B 4x16, C 16x16 -> D
__global__ void k_mfma(const double* A, const double* B, const double* C, double* D) {
  const int lane = threadIdx.x;
  const double a = A[(lane & 15) * 4 + (lane >> 4)];
  const double b = B[(lane >> 4) * 16 + (lane & 15)];
  d4f c;
  for (int r = 0; r < 4; ++r) c[r] = C[((lane >> 4) + 4 * r) * 16 + (lane & 15)];
  d4f d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[((lane >> 4) + 4 * r) * 16 + (lane & 15)] = d[r];
}

static double two_sum_exact(const double* v, int n) {  // Shewchuk-style exact sum rounded once (small n)
  double p[64];
  int m = 0;
  for (int i = 0; i < n; ++i) {
    double x = v[i];
    int k = 0;
    for (int j = 0; j < m; ++j) {
      double y = p[j], s = x + y, bb = s - x, e = (x - (s - bb)) + (y - bb);
      if (e != 0.0) p[k++] = e;
      x = s;
    }
    p[k++] = x;
    m = k;
  }
  double s = 0.0;
  for (int j = 0; j < m; ++j) s += p[j];
  return s;
}

int main() {
  const int trials = 2000;
  double *A, *B, *C, *D;
  hipMallocManaged(&A, 64 * 8);
  hipMallocManaged(&B, 64 * 8);
  hipMallocManaged(&C, 256 * 8);
  hipMallocManaged(&D, 256 * 8);
  srand(7);
  long same_fwd = 0, same_rev = 0, same_exact = 0, total = 0, worse = 0;
  double maxrel_fwd = 0.0;
  for (int t = 0; t < trials; ++t) {
    for (int i = 0; i < 64; ++i) {
      A[i] = ldexp((double)rand() / RAND_MAX - 0.5, (rand() % 60) - 30);
      B[i] = ldexp((double)rand() / RAND_MAX - 0.5, (rand() % 60) - 30);
    }
    for (int i = 0; i < 256; ++i) C[i] = ldexp((double)rand() / RAND_MAX - 0.5, (rand() % 60) - 30);
    k_mfma<<<1, 64>>>(A, B, C, D);
    hipDeviceSynchronize();
    for (int r = 0; r < 16; ++r)
      for (int c = 0; c < 16; ++c) {
        double f = C[r * 16 + c], g = C[r * 16 + c];
        for (int k = 0; k < 4; ++k) f = fma(A[r * 4 + k], B[k * 16 + c], f);
        for (int k = 3; k >= 0; --k) g = fma(A[r * 4 + k], B[k * 16 + c], g);
        // exact: products split into exact pairs
        double terms[9];
        terms[0] = C[r * 16 + c];
        for (int k = 0; k < 4; ++k) {
          const double pr = A[r * 4 + k] * B[k * 16 + c];
          terms[1 + 2 * k] = pr;
          terms[2 + 2 * k] = fma(A[r * 4 + k], B[k * 16 + c], -pr);
        }
        const double ex = two_sum_exact(terms, 9);
        const double d = D[r * 16 + c];
        ++total;
        same_fwd += (d == f);
        same_rev += (d == g);
        same_exact += (d == ex);
        if (fabs(d - ex) > fabs(f - ex)) ++worse;
        if (ex != 0.0) maxrel_fwd = fmax(maxrel_fwd, fabs(d - f) / fabs(ex));
      }
  }
  printf("mfma_f64_16x16x4: %ld outputs; equal to fma chain k=0..3: %ld, k=3..0: %ld, exactly rounded: %ld; "
         "farther from exact than the k=0..3 chain: %ld; max |mfma - chain| / |exact| = %.3e\n",
         total, same_fwd, same_rev, same_exact, worse, maxrel_fwd);
  return 0;
}
