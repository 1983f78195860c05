// k_chol.hip — blocked right-looking Cholesky (row-major lower L, NB = 64) with the forward
// substitution fused in, and the backward-substitution steps.
//
// Reference: MatrixUtils.regularizedCholesky -> Breeze cholesky -> LAPACK dpotrf('L')
// (MatrixUtils.scala:452-461), then forwardSolve(L, d*b) / backSolve(L', w) (MatrixUtils.scala:383-430,
// 491-493).  The right-hand sides and the 64 unit vectors ride along as extra rows of each diagonal-block
// elimination (bordered form): the same sweep that produces L_kk yields w_k = L_kk^-1 b_k and
// L_kk^-1, so the panel TRSM and the backward substitution are products with L_kk^-1 instead of
// sequential substitutions.
#include <math.h>

#include "kernels.hpp"

namespace cvxg {

// ------------------------------------------------------------------------------------------------
// Diagonal block factorisation: 256 threads as 16x16, thread (tr,tc) owns rows tr+16a, cols tc+16b of
// the block (e) and of the identity border (ee) in registers.  Step j: owners of column j publish it,
// everybody updates its trailing entries a_rc -= a_rj a_cj / a_jj (one barrier per step).  Results are
// collected in LDS and written once at the end.  Non-positive or NaN pivot -> ctrl->chol_info =
// global index + 1 (dpotrf info > 0).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_potrf_diag(double* __restrict__ L, int ld, int k, double* __restrict__ rhs,
                                                    int nrhs, double* __restrict__ Linv, DevCtrl* ctrl) {
  if (ctrl->chol_info != 0) return;
  __shared__ double col[2][NB];
  __shared__ double colE[2][NB];
  __shared__ double lfin[NB][NB + 1];
  __shared__ double linv[NB][NB + 1];
  __shared__ double rh[MAX_RHS][NB];
  __shared__ double wfin[MAX_RHS][NB];
  const int tid = threadIdx.x;
  const int tr = tid >> 4, tc = tid & 15;
  const int base = k * NB;
  double e[4][4], ee[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int r = tr + 16 * a, c = tc + 16 * b;
      e[a][b] = (c <= r) ? L[(size_t)(base + r) * ld + base + c] : 0.0;
      ee[a][b] = (c == r) ? 1.0 : 0.0;
    }
  for (int t = tid; t < nrhs * NB; t += 256) rh[t / NB][t % NB] = rhs[(size_t)(base + t % NB) * nrhs + t / NB];
  for (int t = tid; t < NB * (NB + 1); t += 256) {
    (&lfin[0][0])[t] = 0.0;
    (&linv[0][0])[t] = 0.0;
  }
  double mind = __builtin_inf();
  __syncthreads();

#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int buf = j & 1;
    if (tc == (j & 15)) {
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const int r = tr + 16 * a;
        col[buf][r] = (r >= j) ? e[a][j >> 4] : 0.0;
        colE[buf][r] = ee[a][j >> 4];
      }
    }
    __syncthreads();
    const double piv = col[buf][j];
    if (!(piv > 0.0)) {  // dpotrf info > 0 -> NotConvergedException (uniform across the block)
      if (tid == 0) atomicCAS(&ctrl->chol_info, 0, base + j + 1);
      return;
    }
    const double ljj = sqrt(piv);
    const double rl = 1.0 / ljj;
    const double ipiv = 1.0 / piv;
    if (tc == (j & 15)) {
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const int r = tr + 16 * a;
        if (r >= j) lfin[r][j] = (r == j) ? ljj : col[buf][r] * rl;
        linv[j][r] = colE[buf][r] * rl;  // Linv[j][r] = (L^-1 e_r)_j
      }
    }
    mind = fmin(mind, ljj);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int r = tr + 16 * a, c = tc + 16 * b;
        if (c > j) {
          const double f = col[buf][c] * ipiv;
          if (c <= r) e[a][b] -= col[buf][r] * f;
          ee[a][b] -= colE[buf][r] * f;
        }
      }
    for (int t = tid; t < nrhs * NB; t += 256) {
      const int rho = t / NB, c = t % NB;
      if (c > j) rh[rho][c] -= rh[rho][j] * (col[buf][c] * ipiv);
      else if (c == j) wfin[rho][j] = rh[rho][j] * rl;  // w_j
    }
  }
  __syncthreads();
  for (int t = tid; t < NB * NB; t += 256) {
    const int r = t / NB, c = t % NB;
    if (c <= r) L[(size_t)(base + r) * ld + base + c] = lfin[r][c];
    Linv[(size_t)k * NB * NB + t] = linv[r][c];
  }
  for (int t = tid; t < nrhs * NB; t += 256) rhs[(size_t)(base + t % NB) * nrhs + t / NB] = wfin[t / NB][t % NB];
  if (tid == 0) atomic_min_pos(&ctrl->min_diag, mind);
}

void launch_potrf_diag(hipStream_t s, double* L, int ld, int k, double* rhs, int nrhs, double* Linv, DevCtrl* ctrl) {
  k_potrf_diag<<<1, 256, 0, s>>>(L, ld, k, rhs, nrhs, Linv, ctrl);
}

// ------------------------------------------------------------------------------------------------
// Panel TRSM as a product with L_kk^-1:  L[i, kb] = A[i, kb] L_kk^-T, i.e. x_c = sum_{j<=c} a_j Linv[c][j].
// Four threads per row (each owns the outputs c = q + 4u), the row in registers, Linv broadcast from
// LDS.  Fused forward substitution: rhs[i] -= L[i, kb] . w_kb (shuffle-reduced over the 4 threads).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_trsm_panel(double* __restrict__ L, int ld, int np, int k,
                                                    double* __restrict__ rhs, int nrhs,
                                                    const double* __restrict__ Linv, const DevCtrl* ctrl) {
  if (ctrl->chol_info != 0) return;
  __shared__ double li[NB][NB + 1];
  __shared__ double wk[MAX_RHS][NB];
  const int base = k * NB;
  const double* lsrc = Linv + (size_t)k * NB * NB;
  for (int t = threadIdx.x; t < NB * NB; t += 256) li[t / NB][t % NB] = lsrc[t];
  for (int t = threadIdx.x; t < nrhs * NB; t += 256) wk[t / NB][t % NB] = rhs[(size_t)(base + t % NB) * nrhs + t / NB];
  __syncthreads();
  const int q = threadIdx.x & 3;
  const int i = base + NB + blockIdx.x * 64 + (threadIdx.x >> 2);
  const bool valid = i < np;
  const int ir = valid ? i : np - 1;
  double a[NB];
  double* row = L + (size_t)ir * ld + base;
#pragma unroll
  for (int c = 0; c < NB; c += 2) {
    typedef double d2 __attribute__((ext_vector_type(2)));
    const d2 v = *reinterpret_cast<const d2*>(row + c);
    a[c] = v[0];
    a[c + 1] = v[1];
  }
  double x[NB / 4];
#pragma unroll
  for (int u = 0; u < NB / 4; ++u) {
    const int c = q + 4 * u;
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int j = 0; j < NB; j += 2) {  // Linv[c][j] = 0 for j > c
      s0 = fma(a[j], li[c][j], s0);
      s1 = fma(a[j + 1], li[c][j + 1], s1);
    }
    x[u] = s0 + s1;
  }
  if (valid) {
#pragma unroll
    for (int u = 0; u < NB / 4; ++u) row[q + 4 * u] = x[u];
  }
  for (int rho = 0; rho < nrhs; ++rho) {
    double s = 0.0;
#pragma unroll
    for (int u = 0; u < NB / 4; ++u) s = fma(x[u], wk[rho][q + 4 * u], s);
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    if (valid && q == 0) rhs[(size_t)i * nrhs + rho] -= s;
  }
}

void launch_trsm_panel(hipStream_t s, double* L, int ld, int np, int k, double* rhs, int nrhs, const double* Linv,
                       const DevCtrl* ctrl) {
  const int rows = np - (k + 1) * NB;
  if (rows <= 0) return;
  k_trsm_panel<<<(rows + 63) / 64, 256, 0, s>>>(L, ld, np, k, rhs, nrhs, Linv, ctrl);
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
