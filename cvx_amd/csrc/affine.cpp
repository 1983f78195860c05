// affine.cpp — library calls of the affine re-parametrisation x = z0 + F u (setup only, never per Newton step).
//
// Reference: MatrixUtils.solveUnderdetermined (MatrixUtils.scala:536-550: Breeze qr(A.t) = LAPACK dgeqrf + dorgqr
// with the full Q) behind SolutionSpace (SolutionSpace.scala:20-33), and the data transforms that
// BarrierSolver.affineTransformed (BarrierSolver.scala:209-232) implies: F'PF, A F, F'(a + P z0).  These are plain
// dense GEMM / GEMV / QR calls run once per problem, so they go to rocBLAS / rocSOLVER on the device; the Newton
// iterations of the transformed problem then run on this engine's own kernels in dimension F.cols.
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include "kernels.hpp"

namespace cvxg {

namespace {
struct Handle {
  rocblas_handle h = nullptr;
  explicit Handle(hipStream_t s) {
    if (rocblas_create_handle(&h) == rocblas_status_success) {
      rocblas_set_stream(h, s);
      rocblas_set_pointer_mode(h, rocblas_pointer_mode_host);
    } else {
      h = nullptr;
    }
  }
  ~Handle() {
    if (h) rocblas_destroy_handle(h);
  }
};
inline rocblas_operation op(bool t) { return t ? rocblas_operation_transpose : rocblas_operation_none; }
}  // namespace

// M: n x n column-major (ld n), the first p columns hold A'.  On return M holds the full Q of A' = QR and
// Rcols (device, n x p, ld n) the first p columns after dgeqrf (R in their upper triangle).
int lib_qr_full(hipStream_t s, double* M, int n, int p, double* tau, double* Rcols) {
  Handle H(s);
  if (!H.h) return -1;
  if (rocsolver_dgeqrf(H.h, n, p, M, n, tau) != rocblas_status_success) return -2;
  if (hipMemcpyAsync(Rcols, M, sizeof(double) * (size_t)n * p, hipMemcpyDeviceToDevice, s) != hipSuccess) return -3;
  if (rocsolver_dorgqr(H.h, n, n, p, M, n, tau) != rocblas_status_success) return -4;
  return hipStreamSynchronize(s) == hipSuccess ? 0 : -5;
}

// C = op(A) op(B) (column-major, alpha 1, beta 0).
int lib_gemm(hipStream_t s, bool ta, bool tb, int m, int n, int k, const double* A, int lda, const double* B, int ldb,
             double* C, int ldc) {
  Handle H(s);
  if (!H.h) return -1;
  const double one = 1.0, zero = 0.0;
  if (rocblas_dgemm(H.h, op(ta), op(tb), m, n, k, &one, A, lda, B, ldb, &zero, C, ldc) != rocblas_status_success)
    return -2;
  return 0;
}

// y = alpha op(A) x + beta y (column-major A of rows x cols).
int lib_gemv(hipStream_t s, bool ta, int rows, int cols, double alpha, const double* A, int lda, const double* x,
             double beta, double* y) {
  Handle H(s);
  if (!H.h) return -1;
  if (rocblas_dgemv(H.h, op(ta), rows, cols, &alpha, A, lda, x, 1, &beta, y, 1) != rocblas_status_success) return -2;
  return 0;
}

// Host result of u . v (synchronous).
int lib_dot(hipStream_t s, int n, const double* u, const double* v, double* out) {
  Handle H(s);
  if (!H.h) return -1;
  if (rocblas_ddot(H.h, n, u, 1, v, 1, out) != rocblas_status_success) return -2;
  return hipStreamSynchronize(s) == hipSuccess ? 0 : -3;
}

}  // namespace cvxg
