// symsolve.cpp — the failure-only fallbacks MatrixUtils.symSolve / KKTSystem.kktSymSolve on the device.
//
// Reference: MatrixUtils.scala:734-751 (symSolve: eigSym, then diagonalizationSolve :603-706) and
// KKTSystem.scala:283-310 (kktSymSolve: symSolve on the KKT matrix [H A'; A 0] with rhs (-g, r)).
// The symmetric eigen-decomposition is rocSOLVER's dsyevd on the device (a library call: this path runs
// only after both Cholesky attempts failed); the projections, the solvability test and the residual test
// are this engine's kernels.
//
// diagonalizationSolve quirk reproduced (MatrixUtils.scala:666-699): the regularization loop's `relError`
// is a fresh val inside the loop body, so the loop condition and the final test read the outer, unchanged
// relError: once the plain eigen solution misses the tolerance the reference always ends in
// UnsolvableSystemException.  The loop itself only logs, so it is not run here.
#include <hip/hip_runtime.h>
#include <math.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include "kernels.hpp"

namespace cvxg {

// M (row-major n2 x n2, leading dimension ldm, zero padded to ldm x ldm) is overwritten by its eigenvectors
// (row j of the row-major view = eigenvector j); d receives the eigenvalues.  Returns rocSOLVER's info.
int sym_eig(hipStream_t s, double* M, int n2, int ldm, double* d, double* e_work, int* dinfo) {
  rocblas_handle h = nullptr;
  if (rocblas_create_handle(&h) != rocblas_status_success) return -1;
  rocblas_set_stream(h, s);
  const rocblas_status st =
      rocsolver_dsyevd(h, rocblas_evect_original, rocblas_fill_lower, n2, M, ldm, d, e_work, dinfo);
  (void)hipStreamSynchronize(s);
  rocblas_destroy_handle(h);
  if (st != rocblas_status_success) return -2;
  int info = 0;
  (void)hipMemcpy(&info, dinfo, sizeof(int), hipMemcpyDeviceToHost);
  return info;
}

}  // namespace cvxg
