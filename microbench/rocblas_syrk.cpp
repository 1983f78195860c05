// The vendor baseline for the engine's assembly: rocBLAS dsyrk C = A A^T (lower) with n = 4096, k = 8192 -- the
// flop count of H = A' diag(w) A at C3 without the weights (k_syrk_direct also scales by w and adds t P).  Times 10
// calls with HIP events after 2 warm-up calls.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 microbench/rocblas_syrk.cpp -o microbench/rocblas_syrk \
//         -L/opt/rocm/lib -lrocblas
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    auto e_ = (x);                                                            \
    if ((int)e_ != 0) {                                                       \
      fprintf(stderr, "%s:%d: %s -> %d\n", __FILE__, __LINE__, #x, (int)e_); \
      return 1;                                                               \
    }                                                                         \
  } while (0)

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4096, k = argc > 2 ? atoi(argv[2]) : 8192;
  std::vector<double> hA((size_t)n * k);
  srand(7);
  for (auto& v : hA) v = (double)rand() / RAND_MAX - 0.5;
  double *A, *C;
  CK(hipMalloc(&A, hA.size() * 8));
  CK(hipMalloc(&C, (size_t)n * n * 8));
  CK(hipMemcpy(A, hA.data(), hA.size() * 8, hipMemcpyHostToDevice));
  rocblas_handle h;
  CK(rocblas_create_handle(&h));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  CK(rocblas_set_stream(h, s));
  const double alpha = 1.0, beta = 0.0;
  for (int r = 0; r < 2; ++r)
    CK(rocblas_dsyrk(h, rocblas_fill_lower, rocblas_operation_none, n, k, &alpha, A, n, &beta, C, n));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 10;
  CK(hipEventRecord(e0, s));
  for (int r = 0; r < reps; ++r)
    CK(rocblas_dsyrk(h, rocblas_fill_lower, rocblas_operation_none, n, k, &alpha, A, n, &beta, C, n));
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms_all = 0;
  CK(hipEventElapsedTime(&ms_all, e0, e1));
  const double ms = ms_all / reps, fl = (double)k * n * (n + 1);
  printf("rocblas_dsyrk lower n=%d k=%d: %.3f ms per call (%.1f TF/s on k n (n+1) flops)\n", n, k, ms,
         fl / (ms * 1e-3) / 1e12);
  return 0;
}
