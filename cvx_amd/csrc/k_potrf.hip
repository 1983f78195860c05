// k_potrf.hip — per-block launch of the 64x64 diagonal-block Cholesky (potrf64.hpp), used by the
// kernel-per-step blocked factorization (cvxg.cpp factor_attempt, CVXG_CHOL=blocked).
#include "potrf64.hpp"

namespace cvxg {

__global__ __launch_bounds__(256) void k_potrf_blocked(double* __restrict__ L, int ld, int k, double* __restrict__ rhs,
                                                       int nrhs, double* __restrict__ Linv, DevCtrl* ctrl) {
  if (ctrl->chol_info != 0) return;
  __shared__ __attribute__((aligned(16))) Potrf64Smem sm;
  potrf64<PlainMem>(L, ld, k, rhs, nrhs, Linv, ctrl, sm);
}

void launch_potrf_diag(hipStream_t s, double* L, int ld, int k, double* rhs, int nrhs, double* Linv, DevCtrl* ctrl) {
  k_potrf_blocked<<<1, 256, 0, s>>>(L, ld, k, rhs, nrhs, Linv, ctrl);
}

}  // namespace cvxg
