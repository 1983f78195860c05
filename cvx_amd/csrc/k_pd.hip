// k_pd.hip — device pieces of the primal-dual interior-point iteration (PrimalDualSolver.scala:162-240, 311-374)
// that are not already barrier-path kernels: the KKT-matrix weights, the right-hand side, the symmetric
// Ruiz scaling of SymmetricLinearSystem, delta lambda with the step bound s0, and the batched residual-norm
// line-search trials.  Everything is O(m) or O(n^2) elementwise; the GEMVs and the SYRK are shared kernels.
#include "kernels.hpp"

namespace cvxg {

// rhs1 (PrimalDualSolver.scala:162-176) = -grad f + sum_i a_i / (t f_i) = -(t grad f + sum_i a_i / d_i) / t,
// i.e. minus the barrier gradient y (BarrierSolver.scala:291-301) over t; 0 on the padding.
__global__ void k_pd_rhs(const double* __restrict__ y, double t, int n, int np, double* __restrict__ rhs) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < np) rhs[j] = (j < n) ? -(y[j] / t) : 0.0;
}
void launch_pd_rhs(hipStream_t s, const double* y, double t, int n, int np, double* rhs) {
  k_pd_rhs<<<(np + 255) / 256, 256, 0, s>>>(y, t, n, np, rhs);
}

// kktMatrix_noEqs weights (:226-238): hpd += -(G G') (l_i / f_i) = G G' (l_i / d_i), d_i = -f_i; 0 on padded rows
__global__ void k_pd_weights(const double* __restrict__ lam, const double* __restrict__ d, int m, int mp,
                             double* __restrict__ w) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < mp) w[i] = (i < m) ? lam[i] / d[i] : 0.0;
}
void launch_pd_weights(hipStream_t s, const double* lam, const double* d, int m, int mp, double* w) {
  k_pd_weights<<<(mp + 255) / 256, 256, 0, s>>>(lam, d, m, mp, w);
}

// Q = (d d') o H over the whole np x np matrix (SymmetricLinearSystem.scala:20-22 via MatrixUtils.scala:267)
__global__ void k_scale_sym(double* __restrict__ H, int ld, int np, const double* __restrict__ d) {
  const int i = blockIdx.y, j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= np) return;
  H[(size_t)i * ld + j] = (d[i] * d[j]) * H[(size_t)i * ld + j];
}
void launch_scale_sym(hipStream_t s, double* H, int ld, int np, const double* d) {
  k_scale_sym<<<dim3((np + 255) / 256, np), 256, 0, s>>>(H, ld, np, d);
}

// y = -(d o r): the rhs s = d :* r of the equilibrated system (SymmetricLinearSystem.scala:23) in the
// "minus gradient" convention of the shared choleskySolve pipeline (it solves H x = -y).
__global__ void k_neg_scaled(const double* __restrict__ d, const double* __restrict__ r, int np, double* __restrict__ y) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < np) y[j] = -(d[j] * r[j]);
}
void launch_neg_scaled(hipStream_t s, const double* d, const double* r, int np, double* y) {
  k_neg_scaled<<<(np + 255) / 256, 256, 0, s>>>(d, r, np, y);
}

// deltaLambda (:184-209): h = g - ub = c - ub, r_cent = -l h - 1/t, dl = (-l (A dx) + r_cent) / h; also the
// central residual at (x, lambda) (for |r_t|, :343) and the step bound s0 = min(1, -l_i/dl_i over dl_i < 0)
// (:331-338; a min, so the reference's sequential loop order does not matter).  Padded rows: dl = rc = 0.
__global__ void k_pd_dlambda(const double* __restrict__ c, const double* __restrict__ ub,
                             const double* __restrict__ lam, const double* __restrict__ e, double t, int m, int mp,
                             double* __restrict__ dlam, double* __restrict__ rc, DevCtrl* ctrl) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= mp) return;
  if (i >= m) {
    dlam[i] = 0.0;
    rc[i] = 0.0;
    return;
  }
  const double h = c[i] - ub[i];
  const double l = lam[i];
  const double r = -l * h - 1.0 / t;
  const double dl = (-l * e[i] + r) / h;
  dlam[i] = dl;
  rc[i] = r;
  if (dl < 0.0) {
    const double q = -l / dl;
    if (q < 1.0) atomic_min_pos(&ctrl->pd_s0, q);
  }
}
void launch_pd_dlambda(hipStream_t s, const double* c, const double* ub, const double* lam, const double* e, double t,
                       int m, int mp, double* dlam, double* rc, DevCtrl* ctrl) {
  k_pd_dlambda<<<(mp + 255) / 256, 256, 0, s>>>(c, ub, lam, e, t, m, mp, dlam, rc, ctrl);
}

// lambda_0 = -1/h(x_0) (ConstraintSet.lambda, ConstraintSet.scala:116-120) = 1/d = invd bit for bit (ub - c = -(c - ub)
// and 1/(-h) = -(1/h) exactly); 0 on the padded rows.
__global__ void k_pd_lambda0(const double* __restrict__ invd, int m, int mp, double* __restrict__ lam) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < mp) lam[i] = (i < m) ? invd[i] : 0.0;
}
void launch_pd_lambda0(hipStream_t s, const double* invd, int m, int mp, double* lam) {
  k_pd_lambda0<<<(mp + 255) / 256, 256, 0, s>>>(invd, m, mp, lam);
}
__global__ void k_pd_reset_s0(DevCtrl* ctrl) { ctrl->pd_s0 = (unsigned long long)__double_as_longlong(1.0); }
void launch_pd_reset_s0(hipStream_t s, DevCtrl* ctrl) { k_pd_reset_s0<<<1, 1, 0, s>>>(ctrl); }

// out = (a0 + Pv) + sum_c part[c]  (a0, Pv nullable): grad f + A' v, the dual residual (:63-71)
__global__ void k_pd_finalize(const double* __restrict__ a0, const double* __restrict__ Pv,
                              const double* __restrict__ part, int nchunks, int cols, double* __restrict__ out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= cols) return;
  const double g = (a0 ? a0[j] : 0.0) + (Pv ? Pv[j] : 0.0);
  double s = 0.0;
  for (int c = 0; c < nchunks; ++c) s += part[(size_t)c * cols + j];
  out[j] = g + s;
}
void launch_pd_finalize(hipStream_t s, const double* a0, const double* Pv, const double* part, int nchunks, int cols,
                        double* out) {
  k_pd_finalize<<<(cols + 255) / 256, 256, 0, s>>>(a0, Pv, part, nchunks, cols, out);
}

// Line-search trials (:344-368) along s_k = s_base beta^k (repeated products): per trial, over the constraint
// rows, the number failing g_i(x + s dx) (1 + 3e-16) < ub_i (Constraint.scala:23) and the sum of squares of the
// central residual -(l + s dl)(g - ub) - 1/t; g(x + s dx) = c + s (G dx) (+ s^2 dx'P dx / 2 for a QuadraticConstraint
// row, f != NULL).  Per-block partials, [block][trial][2] as doubles, summed in a fixed order by k_sum_chunks.
__global__ __launch_bounds__(256) void k_pd_trials_rows(const double* __restrict__ c, const double* __restrict__ e,
                                                        const double* __restrict__ ub, const double* __restrict__ lam,
                                                        const double* __restrict__ dlam, int m, double sbase,
                                                        double beta, double t, double* __restrict__ part,
                                                        const double* __restrict__ f) {
  __shared__ double scent[4][LS_TRIALS];
  __shared__ int sviol[4][LS_TRIALS];
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const bool valid = i < m;
  const double ci = valid ? c[i] : 0.0, ei = valid ? e[i] : 0.0, ubi = valid ? ub[i] : 1.0;
  const double li = valid ? lam[i] : 0.0, dli = valid ? dlam[i] : 0.0;
  const double fi = (valid && f) ? f[i] : 0.0;
  double s = sbase;
  for (int k = 0; k < LS_TRIALS; ++k) {
    const double g = f ? (ci + s * ei) + (s * s * fi) / 2 : ci + s * ei;
    const bool viol = valid && !(g * (1 + 3e-16) < ubi);
    const double r = -(li + s * dli) * (g - ubi) - 1.0 / t;
    const double sc = wave_sum(valid ? r * r : 0.0);
    const unsigned long long bv = __ballot(viol);
    if (lane == 0) {
      scent[wid][k] = sc;
      sviol[wid][k] = __popcll(bv);
    }
    s *= beta;
  }
  __syncthreads();
  if (threadIdx.x < LS_TRIALS) {
    const int k = threadIdx.x;
    part[((size_t)blockIdx.x * LS_TRIALS + k) * 2 + 0] = ((scent[0][k] + scent[1][k]) + scent[2][k]) + scent[3][k];
    part[((size_t)blockIdx.x * LS_TRIALS + k) * 2 + 1] = (double)(sviol[0][k] + sviol[1][k] + sviol[2][k] + sviol[3][k]);
  }
}
// ... and over the variables, the dual residual grad f(x_s) + Dg(x_s)' l_s = R0 + s R1 (+ s^2 R2 with
// QuadraticConstraint rows, whose gradients a + P x_s move with the step).  With the KL primal objective (x != NULL)
// grad f(x_s) is evaluated afresh per trial, (1 + log(x_j + dx_j s)) + log n (Dist_KL.scala:228-229), and R0 / R1
// carry only the constraint terms; a trial outside the domain gives NaN, which no acceptance test passes.
__global__ __launch_bounds__(256) void k_pd_trials_cols(const double* __restrict__ R0, const double* __restrict__ R1,
                                                        int n, double sbase, double beta, double* __restrict__ part,
                                                        const double* __restrict__ R2, const double* __restrict__ x,
                                                        const double* __restrict__ dx, double nd) {
  __shared__ double sd[4][LS_TRIALS];
  const int j = blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const bool valid = j < n;
  const double r0 = valid ? R0[j] : 0.0, r1 = valid ? R1[j] : 0.0, r2 = (valid && R2) ? R2[j] : 0.0;
  const double xj = (valid && x) ? x[j] : 1.0, dxj = (valid && x) ? dx[j] : 0.0;
  const double logn = x ? log(nd) : 0.0;  // (as k_klp_eval forms it)
  double s = sbase;
  for (int k = 0; k < LS_TRIALS; ++k) {
    double v = R2 ? (r0 + s * r1) + (s * s) * r2 : r0 + s * r1;
    if (x && valid) v = ((1.0 + log(xj + dxj * s)) + logn) + v;
    const double sv = wave_sum(v * v);
    if (lane == 0) sd[wid][k] = sv;
    s *= beta;
  }
  __syncthreads();
  if (threadIdx.x < LS_TRIALS) {
    const int k = threadIdx.x;
    part[(size_t)blockIdx.x * LS_TRIALS + k] = ((sd[0][k] + sd[1][k]) + sd[2][k]) + sd[3][k];
  }
}
int pd_row_blocks(int m) { return m > 0 ? (m + 255) / 256 : 1; }
// out[0 .. 2 LS_TRIALS): (central sum of squares, violations) per trial; out[2 LS_TRIALS ..): dual sum of squares;
// with equality rows (p > 0, solve_withEQs :531-534) out[3 LS_TRIALS ..): the primal residual |A x_s - b|^2 =
// |(A x - b) + s (A dx)|^2 per trial, the column kernel over the p rows.
void launch_pd_trials(hipStream_t s, const double* c, const double* e, const double* ub, const double* lam,
                      const double* dlam, int m, const double* R0, const double* R1, int n, double sbase, double beta,
                      double t, double* part_rows, double* part_cols, double* out, const double* f, const double* R2,
                      const double* rp, const double* adx, int p, double* part_eq, const double* klx,
                      const double* kldx, double klp_n) {
  const int br = pd_row_blocks(m), bc = (n + 255) / 256;
  k_pd_trials_rows<<<br, 256, 0, s>>>(c, e, ub, lam, dlam, m, sbase, beta, t, part_rows, f);
  k_pd_trials_cols<<<bc, 256, 0, s>>>(R0, R1, n, sbase, beta, part_cols, R2, klx, kldx, klp_n);
  launch_sum_chunks(s, part_rows, br, 2 * LS_TRIALS, out);
  launch_sum_chunks(s, part_cols, bc, LS_TRIALS, out + 2 * LS_TRIALS);
  if (p > 0) {
    const int be = (p + 255) / 256;
    k_pd_trials_cols<<<be, 256, 0, s>>>(rp, adx, p, sbase, beta, part_eq, nullptr, nullptr, nullptr, 1.0);
    launch_sum_chunks(s, part_eq, be, LS_TRIALS, out + 3 * LS_TRIALS);
  }
}

// The central residual r_cent = -l (c - ub) - 1/t at (x, lambda) (:97-106; k_pd_dlambda's expression), 0 on padded
// rows: the state's |r_t| after a step (solve_withEQs :606).
__global__ void k_pd_central(const double* __restrict__ c, const double* __restrict__ ub,
                             const double* __restrict__ lam, double t, int m, int mp, double* __restrict__ rc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= mp) return;
  rc[i] = (i < m) ? -lam[i] * (c[i] - ub[i]) - 1.0 / t : 0.0;
}
void launch_pd_central(hipStream_t s, const double* c, const double* ub, const double* lam, double t, int m, int mp,
                       double* rc) {
  k_pd_central<<<(mp + 255) / 256, 256, 0, s>>>(c, ub, lam, t, m, mp, rc);
}

}  // namespace cvxg
