// k_chol.hip — blocked right-looking Cholesky (row-major lower L, NB = 64) with the forward
// substitution fused in, plus the diagonal-block inverses and the backward-substitution steps.
//
// Reference: MatrixUtils.regularizedCholesky -> Breeze cholesky -> LAPACK dpotrf('L')
// (MatrixUtils.scala:452-461), then forwardSolve(L, d*b) / backSolve(L', w) (MatrixUtils.scala:383-430,
// 491-493).  The right-hand sides ride along as extra rows of the factorisation (the bordered-matrix
// form of forward substitution), so w = L^-1 (d*b) is ready when the last pivot is taken.
#include <math.h>

#include "kernels.hpp"

namespace cvxg {

// ------------------------------------------------------------------------------------------------
// Diagonal block factorisation: 256 threads as 16x16, thread (tr,tc) owns rows tr+16a, cols tc+16b in
// registers.  Step j: owners of column j publish it to LDS, everybody updates its trailing entries
// a_rc -= a_rj a_cj / a_jj.  Non-positive or NaN pivot -> ctrl->chol_info = global index + 1 (dpotrf info).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_potrf_diag(double* __restrict__ L, int ld, int k, double* __restrict__ rhs,
                                                    int nrhs, DevCtrl* ctrl) {
  if (ctrl->chol_info != 0) return;
  __shared__ double col[2][NB];
  __shared__ double rh[MAX_RHS][NB];
  const int tr = threadIdx.x >> 4, tc = threadIdx.x & 15;
  const int base = k * NB;
  double e[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int r = tr + 16 * a, c = tc + 16 * b;
      e[a][b] = (c <= r) ? L[(size_t)(base + r) * ld + base + c] : 0.0;
    }
  for (int t = threadIdx.x; t < nrhs * NB; t += 256) rh[t / NB][t % NB] = rhs[(size_t)(base + t % NB) * nrhs + t / NB];
  __syncthreads();

#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int buf = j & 1;
    if (tc == (j & 15)) {
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const int r = tr + 16 * a;
        if (r >= j) col[buf][r] = e[a][j >> 4];
      }
    }
    __syncthreads();
    const double piv = col[buf][j];
    if (!(piv > 0.0)) {  // dpotrf info > 0 -> NotConvergedException (uniform across the block)
      if (threadIdx.x == 0) atomicCAS(&ctrl->chol_info, 0, base + j + 1);
      return;
    }
    const double ljj = sqrt(piv);
    const double rl = 1.0 / ljj;
    const double ipiv = 1.0 / piv;
    if (tc == (j & 15)) {
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const int r = tr + 16 * a;
        if (r >= j) L[(size_t)(base + r) * ld + base + j] = (r == j) ? ljj : col[buf][r] * rl;
      }
    }
    if (threadIdx.x == 0) atomic_min_pos(&ctrl->min_diag, ljj);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int r = tr + 16 * a, c = tc + 16 * b;
        if (c > j && c <= r) e[a][b] -= col[buf][r] * (col[buf][c] * ipiv);
      }
    for (int t = threadIdx.x; t < nrhs * NB; t += 256) {
      const int rho = t / NB, c = t % NB;
      if (c > j) rh[rho][c] -= rh[rho][j] * (col[buf][c] * ipiv);
      else if (c == j) rhs[(size_t)(base + j) * nrhs + rho] = rh[rho][j] * rl;  // w_j
    }
  }
}

void launch_potrf_diag(hipStream_t s, double* L, int ld, int k, double* rhs, int nrhs, DevCtrl* ctrl) {
  k_potrf_diag<<<1, 256, 0, s>>>(L, ld, k, rhs, nrhs, ctrl);
}

// ------------------------------------------------------------------------------------------------
// Panel TRSM: L[i, kb] = A[i, kb] L_kk^-T for rows i below the diagonal block; one thread per row, the
// 64-entry row in registers (fully unrolled), L_kk broadcast from LDS.  The fused forward substitution
// then updates rhs[i] -= L[i, kb] . w_kb.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_trsm_panel(double* __restrict__ L, int ld, int np, int k,
                                                    double* __restrict__ rhs, int nrhs, const DevCtrl* ctrl) {
  if (ctrl->chol_info != 0) return;
  __shared__ double lkk[NB][NB + 1];
  __shared__ double rinv[NB];
  __shared__ double wk[MAX_RHS][NB];
  const int base = k * NB;
  for (int t = threadIdx.x; t < NB * NB; t += 256) {
    const int r = t / NB, c = t % NB;
    lkk[r][c] = (c <= r) ? L[(size_t)(base + r) * ld + base + c] : 0.0;
  }
  for (int t = threadIdx.x; t < nrhs * NB; t += 256) wk[t / NB][t % NB] = rhs[(size_t)(base + t % NB) * nrhs + t / NB];
  __syncthreads();
  if (threadIdx.x < NB) rinv[threadIdx.x] = 1.0 / lkk[threadIdx.x][threadIdx.x];
  __syncthreads();
  const int i = base + NB + blockIdx.x * 256 + threadIdx.x;
  if (i >= np) return;
  double x[NB];
  double* row = L + (size_t)i * ld + base;
#pragma unroll
  for (int c = 0; c < NB; c += 2) {
    const double2 v = *reinterpret_cast<const double2*>(row + c);
    x[c] = v.x;
    x[c + 1] = v.y;
  }
#pragma unroll
  for (int c = 0; c < NB; ++c) {
    double s = x[c];
#pragma unroll
    for (int j = 0; j < c; ++j) s -= x[j] * lkk[c][j];
    x[c] = s * rinv[c];
  }
#pragma unroll
  for (int c = 0; c < NB; c += 2) {
    double2 v;
    v.x = x[c];
    v.y = x[c + 1];
    *reinterpret_cast<double2*>(row + c) = v;
  }
  for (int rho = 0; rho < nrhs; ++rho) {
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < NB; ++c) s = fma(x[c], wk[rho][c], s);
    rhs[(size_t)i * nrhs + rho] -= s;
  }
}

void launch_trsm_panel(hipStream_t s, double* L, int ld, int np, int k, double* rhs, int nrhs, const DevCtrl* ctrl) {
  const int rows = np - (k + 1) * NB;
  if (rows <= 0) return;
  k_trsm_panel<<<(rows + 255) / 256, 256, 0, s>>>(L, ld, np, k, rhs, nrhs, ctrl);
}

// ------------------------------------------------------------------------------------------------
// Inverses of the diagonal blocks (for the backward substitution): thread c solves L_kk y = e_c.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_trtri_diag(const double* __restrict__ L, int ld, double* __restrict__ Linv,
                                                   const DevCtrl* ctrl) {
  if (ctrl->chol_info != 0) return;
  __shared__ double lkk[NB][NB + 1];
  const int base = blockIdx.x * NB;
  for (int t = threadIdx.x; t < NB * NB; t += 64) {
    const int r = t / NB, c = t % NB;
    lkk[r][c] = (c <= r) ? L[(size_t)(base + r) * ld + base + c] : 0.0;
  }
  __syncthreads();
  const int c = threadIdx.x;
  double y[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    double s = (i == c) ? 1.0 : 0.0;
#pragma unroll
    for (int j = 0; j < i; ++j) s -= lkk[i][j] * y[j];
    y[i] = s / lkk[i][i];
  }
  double* out = Linv + (size_t)blockIdx.x * NB * NB;
#pragma unroll
  for (int i = 0; i < NB; ++i) out[i * NB + c] = y[i];
}

void launch_trtri_diag(hipStream_t s, const double* L, int ld, int nblk, double* Linv, const DevCtrl* ctrl) {
  k_trtri_diag<<<nblk, 64, 0, s>>>(L, ld, Linv, ctrl);
}

// ------------------------------------------------------------------------------------------------
// Backward substitution L' u = w, block step k (k = nblk-1 .. 0):
//   u_k = Linv_kk' v_k  (every workgroup, redundantly),  workgroup b < k: v_b -= L[kb, bb]' u_k.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_bwd_step(const double* __restrict__ L, int ld,
                                                  const double* __restrict__ Linv, int k, double* __restrict__ rhs,
                                                  double* __restrict__ out, int nrhs, const DevCtrl* ctrl) {
  if (ctrl->chol_info != 0) return;
  __shared__ double v[MAX_RHS][NB];
  __shared__ double u[MAX_RHS][NB];
  __shared__ double part[4][MAX_RHS][NB];
  const int base = k * NB;
  const int g = threadIdx.x >> 6, c = threadIdx.x & 63;
  for (int t = threadIdx.x; t < nrhs * NB; t += 256) v[t / NB][t % NB] = rhs[(size_t)(base + t % NB) * nrhs + t / NB];
  __syncthreads();
  const double* li = Linv + (size_t)k * NB * NB;
  for (int rho = 0; rho < nrhs; ++rho) {
    double s = 0.0;
    for (int r = g * 16; r < g * 16 + 16; ++r) s = fma(li[r * NB + c], v[rho][r], s);
    part[g][rho][c] = s;
  }
  __syncthreads();
  if (g == 0) {
    for (int rho = 0; rho < nrhs; ++rho) {
      const double s = ((part[0][rho][c] + part[1][rho][c]) + part[2][rho][c]) + part[3][rho][c];
      u[rho][c] = s;
      if (blockIdx.x == 0) out[(size_t)(base + c) * nrhs + rho] = s;
    }
  }
  __syncthreads();
  if (k == 0) return;
  const int b = blockIdx.x;  // < k
  const double* tile = L + (size_t)base * ld + b * NB;  // rows kb, cols bb
  for (int rho = 0; rho < nrhs; ++rho) {
    double s = 0.0;
    for (int r = g * 16; r < g * 16 + 16; ++r) s = fma(tile[(size_t)r * ld + c], u[rho][r], s);
    part[g][rho][c] = s;
  }
  __syncthreads();
  if (g == 0) {
    for (int rho = 0; rho < nrhs; ++rho) {
      const double s = ((part[0][rho][c] + part[1][rho][c]) + part[2][rho][c]) + part[3][rho][c];
      rhs[(size_t)(b * NB + c) * nrhs + rho] -= s;
    }
  }
}

void launch_bwd_step(hipStream_t s, const double* L, int ld, const double* Linv, int k, double* rhs, double* out,
                     int nrhs, const DevCtrl* ctrl) {
  k_bwd_step<<<k > 0 ? k : 1, 256, 0, s>>>(L, ld, Linv, k, rhs, out, nrhs, ctrl);
}

}  // namespace cvxg
