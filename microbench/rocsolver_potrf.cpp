// The vendor baseline for the engine's Cholesky: rocSOLVER dpotrf (lower) on the C3-sized SPD matrix (n = 4096), the
// same factorization k_chol_dataflow performs (without its fused forward solve and L^-1 blocks).  Times 10 calls with
// HIP events after 2 warm-up calls, restoring the matrix from a device copy before each call (the copy is timed
// separately and subtracted).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 microbench/rocsolver_potrf.cpp -o microbench/rocsolver_potrf \
//         -L/opt/rocm/lib -lrocsolver -lrocblas
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CK(x)                                                             \
  do {                                                                    \
    auto e_ = (x);                                                        \
    if ((int)e_ != 0) {                                                   \
      fprintf(stderr, "%s:%d: %s -> %d\n", __FILE__, __LINE__, #x, (int)e_); \
      return 1;                                                           \
    }                                                                     \
  } while (0)

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4096, k = n;
  std::vector<double> hB((size_t)n * k);
  srand(7);
  for (auto& v : hB) v = (double)rand() / RAND_MAX - 0.5;
  double *B, *A, *A0;
  int* info;
  CK(hipMalloc(&B, hB.size() * 8));
  CK(hipMalloc(&A, (size_t)n * n * 8));
  CK(hipMalloc(&A0, (size_t)n * n * 8));
  CK(hipMalloc(&info, sizeof(int)));
  CK(hipMemcpy(B, hB.data(), hB.size() * 8, hipMemcpyHostToDevice));
  rocblas_handle h;
  CK(rocblas_create_handle(&h));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  CK(rocblas_set_stream(h, s));
  // A0 = B B^T / k + I (SPD, well conditioned like the equilibrated Q)
  const double alpha = 1.0 / k, beta = 0.0;
  CK(rocblas_dsyrk(h, rocblas_fill_lower, rocblas_operation_none, n, k, &alpha, B, n, &beta, A0, n));
  std::vector<double> hA((size_t)n * n);
  CK(hipMemcpy(hA.data(), A0, hA.size() * 8, hipMemcpyDeviceToHost));
  for (int i = 0; i < n; ++i) hA[(size_t)i * n + i] += 1.0;
  CK(hipMemcpy(A0, hA.data(), hA.size() * 8, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float ms_copy = 0, ms_all = 0;
  const int reps = 10;
  for (int r = 0; r < 2; ++r) {
    CK(hipMemcpyAsync(A, A0, (size_t)n * n * 8, hipMemcpyDeviceToDevice, s));
    CK(rocsolver_dpotrf(h, rocblas_fill_lower, n, A, n, info));
  }
  CK(hipStreamSynchronize(s));
  CK(hipEventRecord(e0, s));
  for (int r = 0; r < reps; ++r) CK(hipMemcpyAsync(A, A0, (size_t)n * n * 8, hipMemcpyDeviceToDevice, s));
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms_copy, e0, e1));
  CK(hipEventRecord(e0, s));
  for (int r = 0; r < reps; ++r) {
    CK(hipMemcpyAsync(A, A0, (size_t)n * n * 8, hipMemcpyDeviceToDevice, s));
    CK(rocsolver_dpotrf(h, rocblas_fill_lower, n, A, n, info));
  }
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms_all, e0, e1));
  int hinfo = -1;
  CK(hipMemcpy(&hinfo, info, sizeof(int), hipMemcpyDeviceToHost));
  const double ms = (ms_all - ms_copy) / reps;
  printf("rocsolver_dpotrf lower n=%d: %.3f ms per factorization (%.2f TF/s, n^3/3 flops), info=%d\n", n, ms,
         (double)n * n * n / 3.0 / (ms * 1e-3) / 1e12, hinfo);
  return hinfo == 0 ? 0 : 2;
}
