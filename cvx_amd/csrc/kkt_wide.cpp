// kkt_wide.cpp — library calls of KKTSystem.solveWithCholFactor (KKTSystem.scala:99-167) for equality blocks wider
// than the dataflow factorization's fused forward solve (p + 1 > MAX_RHS right-hand sides).
//
// The reference solves the n x (p+1) right-hand side [B' | Dq] with two LAPACK dtrtrs calls (MatrixUtils.
// triangularSolve, MatrixUtils.scala:362-376: L then L'), forms R = B H^-1 B' with a GEMM, and factors the p x p
// Schur complement S = (R + R')/2 with Breeze cholesky (LAPACK dpotrf).  With many right-hand sides these are plain
// dense BLAS-3 / LAPACK calls on the factor the engine already holds, so they go to rocBLAS dtrsm / dgemm / dgemv and
// rocSOLVER dpotrf / dpotrs on the context's stream (one persistent handle per context).
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include "kernels.hpp"

namespace cvxg {

int lib_handle_create(hipStream_t s, void** out) {
  rocblas_handle h = nullptr;
  if (rocblas_create_handle(&h) != rocblas_status_success) return -1;
  rocblas_set_stream(h, s);
  rocblas_set_pointer_mode(h, rocblas_pointer_mode_host);
  *out = h;
  return 0;
}

void lib_handle_destroy(void* h) {
  if (h) rocblas_destroy_handle(static_cast<rocblas_handle>(h));
}

// Y (column-major n x k, leading dimension ldy) <- L'^-1 L^-1 Y, where L is the engine's factor: row-major lower with
// leading dimension ldl, i.e. the column-major UPPER triangle U = L' (the other triangle is ignored).
int lib_llt_solve(void* hp, int n, int k, const double* L, int ldl, double* Y, int ldy) {
  rocblas_handle h = static_cast<rocblas_handle>(hp);
  const double one = 1.0;
  // L Y1 = Y  <=>  U' Y1 = Y
  if (rocblas_dtrsm(h, rocblas_side_left, rocblas_fill_upper, rocblas_operation_transpose, rocblas_diagonal_non_unit, n,
                    k, &one, L, ldl, Y, ldy) != rocblas_status_success)
    return -2;
  // L' X = Y1  <=>  U X = Y1
  if (rocblas_dtrsm(h, rocblas_side_left, rocblas_fill_upper, rocblas_operation_none, rocblas_diagonal_non_unit, n, k,
                    &one, L, ldl, Y, ldy) != rocblas_status_success)
    return -3;
  return 0;
}

// C = alpha op(A) op(B) + beta C (column-major)
int lib_gemm_h(void* hp, bool ta, bool tb, int m, int n, int k, double alpha, const double* A, int lda, const double* B,
               int ldb, double beta, double* C, int ldc) {
  rocblas_handle h = static_cast<rocblas_handle>(hp);
  const rocblas_operation oa = ta ? rocblas_operation_transpose : rocblas_operation_none;
  const rocblas_operation ob = tb ? rocblas_operation_transpose : rocblas_operation_none;
  return rocblas_dgemm(h, oa, ob, m, n, k, &alpha, A, lda, B, ldb, &beta, C, ldc) == rocblas_status_success ? 0 : -2;
}

// y = alpha A x + beta y (column-major A of rows x cols)
int lib_gemv_h(void* hp, int rows, int cols, double alpha, const double* A, int lda, const double* x, double beta,
               double* y) {
  rocblas_handle h = static_cast<rocblas_handle>(hp);
  return rocblas_dgemv(h, rocblas_operation_none, rows, cols, &alpha, A, lda, x, 1, &beta, y, 1) ==
                 rocblas_status_success
             ? 0
             : -2;
}

// S (p x p column-major, lower used) <- its Cholesky factor K (LAPACK dpotrf 'L'); *dinfo (device int) receives
// dpotrf's info (> 0: not positive definite, Breeze's NotConvergedException).
int lib_potrf(void* hp, int p, double* S, int lds, int* dinfo) {
  rocblas_handle h = static_cast<rocblas_handle>(hp);
  if (rocsolver_dpotrf(h, rocblas_fill_lower, p, S, lds, dinfo) != rocblas_status_success) return -2;
  return 0;
}

// z <- (K K')^-1 z with the dpotrf factor K (LAPACK dpotrs: forward then back substitution, KKTSystem.scala:143-144)
int lib_potrs(void* hp, int p, const double* K, int ldk, double* z) {
  rocblas_handle h = static_cast<rocblas_handle>(hp);
  return rocsolver_dpotrs(h, rocblas_fill_lower, p, 1, const_cast<double*>(K), ldk, z, p) == rocblas_status_success
             ? 0
             : -2;
}

}  // namespace cvxg
