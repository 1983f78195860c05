// kernels.hpp — host-side launch wrappers for the HIP kernels of the barrier engine.
#pragma once
#include <assert.h>
#include <hip/hip_runtime.h>

#include "common.hpp"

namespace cvxg {

struct TileList {
  const int* ij;  // device array of packed (I<<16 | J), J <= I
  int count;
};

// ---- GEMV-like streaming kernels (k_vec.hip) -----------------------------------------------------
// Constraint evaluation at x: c = r + A x, d = ub - c, invd = 1/d, w = 1/(d*d), logd = log d and
// the infeasible / not-strict counters in ctrl (LinearConstraint.scala:22-24, BarrierSolver.scala:283-312,
// Constraint.scala:23).
void launch_constraint_eval(hipStream_t s, const double* A, int ld, int mp, int n_cols, const double* x,
                            const double* r, const double* ub, double* c, double* d, double* invd,
                            double* w, double* logd, DevCtrl* ctrl, const double* extra = nullptr,
                            double* cabs = nullptr);
// y = M v (row-major, one wave per row); rows, cols multiples of 128 / any.
void launch_rowdot(hipStream_t s, const double* M, int ld, int rows, int cols, const double* v, double* y);
// y = M v + add, the add fused into the row sweep (bitwise the rowdot followed by launch_axpy(y, add, 1.0))
void launch_rowdot_add(hipStream_t s, const double* M, int ld, int rows, int cols, const double* v,
                       const double* add, double* y);
// y = M v and yabs = |M| |v| in the same sweep; max_wg > 0 bounds the grid (the waves loop over the row pairs,
// bitwise the same sums): beside the assembly SYRK it then holds few CU slots
void launch_rowdot_abs(hipStream_t s, const double* M, int ld, int rows, int cols, const double* v, double* y,
                       double* yabs, int max_wg = 0);
// y = H v + add from the lower triangle of a symmetric H (diagonal 64 x 64 tiles whole); S: nbn x (nbn 64) partials
void launch_symv_lower_add(hipStream_t s, const double* H, int ld, int n, const double* v, const double* add,
                           double* y, double* S);
// the strictly upper triangle of H from its lower triangle
void launch_mirror_lower(hipStream_t s, double* H, int ld, int n);
void launch_ls_setup_eval(hipStream_t st, const double* A, int ld, int mp, int cols, const double* s, const double* x1,
                          double* e, double* eabs, const double* r, const double* ub, double* c, double* d,
                          double* invd, double* w, double* logd, double* cabs, DevCtrl* ctrl);
void launch_spec_prep(hipStream_t st, const double* dx, const double* x, int n, double* s, double* x1, DevCtrl* ctrl);
void launch_ctrl_take_spec(hipStream_t st, DevCtrl* ctrl);
// part[chunk][j] = sum_{i in chunk} M[i][j] v[i]  (chunks of COLDOT_ROWS rows; rows % 64 == 0)
int coldot_chunks(int rows);
void launch_coldot_partials(hipStream_t s, const double* M, int ld, int rows, int cols, const double* v,
                            double* part);
// y_j = t*(a0_j + Px_j) + sum_chunks part[chunk][j]   (gradientBarrierFunction, BarrierSolver.scala:291-301)
void launch_gradient_finalize(hipStream_t s, const double* a0, const double* Px, const double* part,
                              int nchunks, int n_cols, const DevCtrl* ctrl, double* y);
// single-block deterministic sums into ctrl->sc[slot]
void launch_dot(hipStream_t s, const double* u, const double* v, int n, DevCtrl* ctrl, int slot);
void launch_sum(hipStream_t s, const double* u, int n, DevCtrl* ctrl, int slot);
// Up to DOTS_MAX independent single-block reductions in one launch (one block each), every one in exactly
// the order of its single-launch form (bit-identical results):
//   DOT  sum_i u_i v_i   (v NULL: u_i u_i)       = launch_dot
//   SUM  sum_i u_i                                = launch_sum
//   ABS  sum_i |u_i| |v_i| (v NULL: sum_i |u_i|)  -- the error scales of the certified line search
constexpr int DOTS_MAX = 8;
enum DotKind : int { DOT_FMA = 0, DOT_SUM = 1, DOT_ABS = 2 };
struct DotBatch {
  const double* u[DOTS_MAX];
  const double* v[DOTS_MAX];
  int n[DOTS_MAX];
  int slot[DOTS_MAX];
  int kind[DOTS_MAX];
  int count;
  void add(int k, const double* uu, const double* vv, int len, int sl) {
    assert(count < DOTS_MAX && "DotBatch full: launch it and start a new batch");
    u[count] = uu, v[count] = vv, n[count] = len, slot[count] = sl, kind[count] = k, ++count;
  }
  bool full() const { return count >= DOTS_MAX; }
};
void launch_dots(hipStream_t s, const DotBatch& a, DevCtrl* ctrl);
// out = u + v*alpha (alpha read from device scalar pointer or host value)
void launch_axpy(hipStream_t s, const double* u, const double* v, double alpha, int n, double* out);
void launch_scale_vec(hipStream_t s, const double* u, const double* d, int n, double* out);  // out = d*u

// ---- Ruiz equilibration + Q formation ------------------------------------------------------------
// d0 (and d1 when given) = 1, rho[0] = 1, rho[1..] = 0, work[0..nwork) = 0 (k_ruiz_loop's counters and flags)
void launch_ruiz_init(hipStream_t s, double* d0, int np, DevCtrl* ctrl, double* d1 = nullptr, int* work = nullptr,
                      size_t nwork = 0);
// The same sweep from the lower triangle only (64 x 64 tiles -> partials S[nbn][nbn*64] -> fixed-order row sums).
void launch_ruiz_sweep_tri(hipStream_t s, const double* H, int ld, int n, int np, const double* dcur, double* dnext,
                           double* S, DevCtrl* ctrl, int k);
void launch_ruiz_final(hipStream_t s, const double* d0, const double* d1, int np, double* dfin, DevCtrl* ctrl, int k1,
                       const int* abortw = nullptr /* k_ruiz_loop's abort word: set -> ruiz_sweeps = -2 */);
// Every sweep in one persistent launch of nwg workgroups (k_ruiz.hip), then dfin and ruiz_sweeps: the same d, rho
// and sweep count as launch_ruiz_sweep_tri for k = 0 .. RUIZ_MAX-1 + launch_ruiz_final.  gbuf =
// ruiz_loop_doubles(nbn) doubles of data-tagged granules, work = ruiz_loop_work_ints(nbn) ints; gen: nonzero, new
// per launch on the same buffers.  Only while ruiz_loop_fits(nbn).
size_t ruiz_loop_work_ints(int nbn);
size_t ruiz_loop_doubles(int nbn);
bool ruiz_loop_fits(int nbn);
void launch_ruiz_loop(hipStream_t s, const double* H, int ld, int n, int np, double* gbuf, int* work, double* dfin,
                      DevCtrl* ctrl, int nwg, unsigned long long gen, unsigned long long* trace = nullptr);
// L[i][j] = d_i d_j H_ij (+reg on the diagonal), lower triangle; padded diagonal = 1.
void launch_form_q(hipStream_t s, const double* H, double* L, int ld, int n, int np, const double* d,
                   const DevCtrl* ctrl);
void launch_add_diag(hipStream_t s, double* H, int ld, int n, double v);
void launch_copy_diag(hipStream_t s, const double* H, int ld, int n, double* out);
void launch_set_diag(hipStream_t s, double* H, int ld, int n, const double* diag);

// sparse constraint rows: H[p][q] (+ mirror) += sum over the rows i of entry t of coef_e * w[i] (fixed order)
void launch_sparse_hess(hipStream_t s, const int* ptr, const int* pq, const int* row, const double* coef,
                        const double* w, int T, double* H, int ld);
void launch_gather_w(hipStream_t s, const double* w, const int* idx, int nd, int ndp, double* wd);

// ---- QuadraticConstraint rows (k_quad.hip) ------------------------------------------------------------
void launch_quad_xpx(hipStream_t s, const double* qPx, const double* x, const int* qrows, int nq, int np,
                     double* extra);
void launch_quad_grad(hipStream_t s, const double* qPx, const double* invd, const int* qrows, int nq, int np,
                      double* y);
void launch_quad_rows(hipStream_t s, const double* A, const double* qPx, const int* qrows, const int* qslot, int nq,
                      int np, double* As);
void launch_quad_hess(hipStream_t s, const double* Pq, const double* invd, const int* qrows, int nq, int np,
                      double* H);
void launch_quad_ls(hipStream_t s, const double* qPx, const double* qPs, const double* sdir, const int* qrows, int nq,
                    int np, double* e, double* f);
// out[row_k] (+)= scale * |v|.M_k (M: the stacked |P_k| v products of k_rowdot_abs)
void launch_quad_absdot(hipStream_t s, const double* M, const double* v, const int* qrows, int nq, int np, double scale,
                        int accumulate, double* out);

// ---- primal-dual iteration pieces (k_pd.hip) ---------------------------------------------------------
void launch_pd_rhs(hipStream_t s, const double* y, double t, int n, int np, double* rhs);
void launch_pd_weights(hipStream_t s, const double* lam, const double* d, int m, int mp, double* w);
void launch_scale_sym(hipStream_t s, double* H, int ld, int np, const double* d);
void launch_neg_scaled(hipStream_t s, const double* d, const double* r, int np, double* y);
void launch_pd_dlambda(hipStream_t s, const double* c, const double* ub, const double* lam, const double* e, double t,
                       int m, int mp, double* dlam, double* rc, DevCtrl* ctrl);
void launch_pd_finalize(hipStream_t s, const double* a0, const double* Pv, const double* part, int nchunks, int cols,
                        double* out);
int pd_row_blocks(int m);
void launch_pd_lambda0(hipStream_t s, const double* invd, int m, int mp, double* lam);
void launch_pd_reset_s0(hipStream_t s, DevCtrl* ctrl);
// f (QuadraticConstraint rows: dx'P dx per row, 0 on linear rows) and R2 (the s^2 term of the dual residual) may be
// NULL when every constraint is linear.
void launch_pd_trials(hipStream_t s, const double* c, const double* e, const double* ub, const double* lam,
                      const double* dlam, int m, const double* R0, const double* R1, int n, double sbase, double beta,
                      double t, double* part_rows, double* part_cols, double* out, const double* f = nullptr,
                      const double* R2 = nullptr, const double* rp = nullptr, const double* adx = nullptr, int p = 0,
                      double* part_eq = nullptr, const double* klx = nullptr, const double* kldx = nullptr,
                      double klp_n = 0.0);
void launch_pd_central(hipStream_t s, const double* c, const double* ub, const double* lam, double t, int m, int mp,
                       double* rc);

// ---- MFMA SYRK (k_syrk.hip) -----------------------------------------------------------------------
// H = t*P + A' diag(w) A over the lower tile list; split-K when nsplit > 1 (partials + ordered reduce).
// Pd (optional, with P NULL): a diagonal objective Hessian, H_jj += t Pd_j (the KL primal objective's diag(1/x)).
// mirror: every lower entry is also stored at its upper position; false: only those of the diagonal tiles (H stays
// lower-only elsewhere, for consumers that read the lower triangle and whole diagonal tiles).
void launch_syrk_assemble(hipStream_t s, const double* A, int lda, const double* w, int mp, const double* P,
                          const DevCtrl* ctrl, double* H, int ldh, TileList tiles, int nsplit, double* partials,
                          const double* Pd = nullptr, bool mirror = true);

// ---- Cholesky (k_chol.hip) ------------------------------------------------------------------------
// k_dataflow.hip: the whole factorization (potrf + trsm + updates + fused forward solve) as one persistent
// launch over the 64x64 tile DAG in the host-built task order (build_chol_schedule in cvxg.cpp)
size_t chol_dataflow_work_ints(int nblk);
// Linv buffer of the dataflow Cholesky: the nblk diagonal-block inverses L_kk^-1 (64 x 64 each)
__host__ __device__ constexpr size_t chol_dataflow_linv_doubles(int nblk) { return (size_t)nblk * NB * NB; }
void launch_chol_dataflow(hipStream_t s, double* L, int ld, double* rhs, int nrhs, double* Linv, DevCtrl* ctrl,
                          int* work, int nblk, const unsigned* tasks, int ntasks, int nwg,
                          unsigned long long* trace /* nullable: per task {claim, ready, done, wg} (100 MHz) */,
                          bool zero_work = true /* false: launch_factor_prep zeroed it */,
                          const double* Hq = nullptr /* non-null: factor Q = (d d') o H + reg I (k_form_q's entries),
                                                        formed as each tile is first read; L is then output only */,
                          const double* dq = nullptr, int nq = 0,
                          bool ruiz_gate = false /* true: every workgroup leaves at once when ctrl->ruiz_sweeps < 0
                                                    (a short Ruiz lookahead, cvxg.cpp: factor_attempt) */,
                          double early_min = 0.0 /* > 0: stop (abort word, min_diag and small_piv set) at the first
                                                    16-column block whose min diag(L) <= early_min */);
// (the chain workgroups apply panel b-2 to block row b themselves: UPDATE(b,b,b-2), UPDATE(b,b-1,b-2) are not in
// `tasks`, which chol_schedule builds accordingly)
// the whole backward substitution in one launch (flags[nblk], published as flags[b] = gen)
size_t bwd_work_ints(int nblk);  // flag words + the data-tagged u granules of k_bwd_dataflow
// Optional epilogue (nrhs = 1): dx = d :* u; with s, also s = dx and x1 = x + s (the speculative line search's
// direction and trial point), and sctrl's speculative evaluation counters reset.
struct BwdEpilogue {
  const double* d = nullptr;
  double* dx = nullptr;
  double* s = nullptr;
  const double* x = nullptr;
  double* x1 = nullptr;  // x1 = x + s t1: the speculative next point (t1: the step the line search is expected to take)
  double t1 = 1.0;
  DevCtrl* sctrl = nullptr;
};
// The second factorization of a speculative pair (regularized_cholesky_spec): used instead of L / Linv / rhs when
// ctrl->spec_sel is set (its failure word is ctrl->chol_info2).
struct BwdAlt {
  const double* L = nullptr;
  const double* Linv = nullptr;
  const double* rhs = nullptr;
};
void launch_bwd_dataflow(hipStream_t s, const double* L, int ld, const double* Linv, const double* rhs, double* out,
                         int nrhs, int nblk, int* flags, int gen, const DevCtrl* ctrl, BwdEpilogue epi = {},
                         BwdAlt alt = {});
// ctrl2 of the speculative second attempt: its factor prep (reg, chol fields) and the main control block's Ruiz
// verdict (the dataflow launch's gate)
void launch_spec_prep2(hipStream_t s, DevCtrl* ctrl2, const DevCtrl* ctrl, double reg);
// after both attempts: ctrl->spec_sel (first attempt discarded) and the second attempt's chol fields into ctrl
void launch_spec_select(hipStream_t s, DevCtrl* ctrl, const DevCtrl* ctrl2);

// ---- line search ----------------------------------------------------------------------------------
// For trials k in [0, LS_TRIALS): t_k = tbase*beta^k; g_i = c_i + t_k e_i; per-block partials of
// (#violations of g*(1+3e-16)<ub, #(ub-g<=0), sum log(ub-g)).
// With cabs / eabs (|r| + |a|.|x|, |a|.|s|) the trials also report sure / ambiguous violation counts and the log-sum
// error bound (certified decisions, see k_vec.hip); part_aux: 2 doubles per (block, trial).
// fabsq (certified mode, QuadraticConstraint rows): |s|'|P||s| per row (0 on linear rows), the t^2 term of the band.
void launch_ls_trials(hipStream_t s, const double* c, const double* e, const double* ub, int m, double tbase,
                      double beta, double* part_log, int* part_cnt, const double* f, const double* cabs,
                      const double* eabs, double gamma, double* part_aux, const double* fabsq = nullptr);
void launch_ls_finalize(hipStream_t s, const double* part_log, const int* part_cnt, const double* part_aux,
                        int nblocks, double* out_log, int* out_cnt);
int ls_blocks(int m);
// KL dual objective (Dist_KL.scala:146-170): y = R exp(-v) (masked padding); trial sums of R exp(-(v + t_k u))
void launch_kl_eval(hipStream_t s, const double* v, int nout, int noutp, double R, double* y);
// out[k] = the trial sums, out[LS_TRIALS + k] = their error scales (vabs / uabs NULL: zeros)
int ls_kl_blocks(int nout);
void launch_ls_kl(hipStream_t s, const double* v, const double* u, int nout, double R, double tbase, double beta,
                  double* part, double* out, const double* vabs, const double* uabs, double gamma);

// KL primal objective (Dist_KL.scala:223-239): lx = log(n x), g0 = gradient, hd = diag of the Hessian, ab = error
// scale of the value terms (each output may be NULL but lx)
void launch_klp_eval(hipStream_t s, const double* x, int n, int np, double nd, double* lx, double* g0, double* hd,
                     double* ab);
// per trial k: out[k] = sum_j xt log(n xt), out[LS_TRIALS + k] = its error scale, xt = x + s t_k
int ls_klp_blocks(int n);
void launch_ls_klp(hipStream_t s, const double* x, const double* sdir, int n, double nd, double tbase, double beta,
                   double* part, double* out);

// ---- KKT equality block (k_kkt.hip) ------------------------------------------------------------------
// L Z = Y (transposed = false) or L' X = Y (true) in place for nchunk * 16 right-hand-side columns (row-major, leading
// dimension ldy), one dataflow launch; gran: trsm_many_granule_doubles(nblk, nchunk) doubles of hand-off granules
// (zeroed once; gen increases per launch)
size_t trsm_many_granule_doubles(int nblk, int nchunk);
void launch_trsm_many(hipStream_t s, bool transposed, const double* L, int ld, const double* Linv, double* Y, int ldy,
                      int nblk, int nchunk, double* gran, int gen, DevCtrl* ctrl);
// R = B X (B row-major p x ldb, X row-major np x ldx with p + 1 columns), S = (R + R')/2 (lower, rows >= p: identity
// padding up to ps) and z = -(b + R[:, p]) (zero-padded to ps); part: schur_partial_doubles(np, p) doubles
size_t schur_partial_doubles(int np, int p);
void launch_schur_form(hipStream_t s, const double* B, int ldb, const double* X, int ldx, int p, int np, double* part,
                       const double* bvec, int ps, int lds, double* S, double* z);
// w = S^-1 z for p <= 64 (S row-major p x p, lower); a non-positive pivot sets ctrl->chol_info = -1
void launch_schur_small(hipStream_t s, const double* S, int p, const double* z, double* w, DevCtrl* ctrl);
// y = -(X[:, p] + X[:, :p] w)
void launch_kkt_v(hipStream_t s, const double* X, int ldx, int p, int np, const double* w, double* y);

// ---- symSolve / kktSymSolve fallback (symsolve.cpp, k_vec.hip) ----------------------------------------
int sym_eig(hipStream_t s, double* M, int n2, int ldm, double* d, double* e_work, int* dinfo);
// affine.cpp: rocSOLVER / rocBLAS calls of the affine re-parametrisation (setup only)
int lib_qr_full(hipStream_t s, double* M, int n, int p, double* tau, double* Rcols);
int lib_gemm(hipStream_t s, bool ta, bool tb, int m, int n, int k, const double* A, int lda, const double* B, int ldb,
             double* C, int ldc);
int lib_gemv(hipStream_t s, bool ta, int rows, int cols, double alpha, const double* A, int lda, const double* x,
             double beta, double* y);
int lib_dot(hipStream_t s, int n, const double* u, const double* v, double* out);
void launch_eig_coeffs(hipStream_t s, const double* dots, const double* d, int n2, int npad, double* a, double* z);
void launch_sum_chunks(hipStream_t s, const double* part, int nchunks, int cols, double* out);
void launch_kkt_matrix(hipStream_t s, const double* H, int ldh, const double* Aeq, int lda, int n, int p, int ld,
                       double* K);

}  // namespace cvxg

namespace cvxg {
void launch_ctrl_set(hipStream_t s, DevCtrl* ctrl, int which, double v);
void launch_ctrl_reset_eval(hipStream_t s, DevCtrl* ctrl);
void launch_ctrl_reset_chol(hipStream_t s, DevCtrl* ctrl);
// one launch before a factorization attempt: ctrl->reg = reg, the chol fields reset, the dataflow work words zeroed
void launch_factor_prep(hipStream_t s, DevCtrl* ctrl, double reg, int* work, size_t nwork);
// copy two device ranges (multiples of 8 bytes; bytes1 may be 0) into coherent host memory (device-side addresses),
// then *flag = seq (system scope)
void launch_publish(hipStream_t s, const void* s0, void* d0, size_t bytes0, const void* s1, void* d1, size_t bytes1,
                    unsigned* flag, unsigned seq);
void launch_scaled_col(hipStream_t s, const double* d, const double* v, double sgn, int n, int np, int nrhs, int col,
                       double* rhs);
void launch_kkt_prep(hipStream_t s, const double* Aeq, int ld, int p, int n, int np, const double* d, double* B,
                     double* rhs, int nrhs);
void launch_axpy_strided(hipStream_t s, const double* u, const double* v, int vs, int vc, double alpha, int n,
                         double* out);
void launch_scale_strided(hipStream_t s, const double* d, const double* v, int vs, int vc, int n, double* out);
void launch_add_ata(hipStream_t s, double* H, int ld, const double* Aeq, int p, int n);
void launch_q_minus_atb(hipStream_t s, const double* q, const double* Aeq, int ld, int p, const double* b, int n,
                        double* z);
void launch_btw_plus(hipStream_t s, const double* B, int ld, int p, const double* w, const double* u, int n,
                     double* y);
}  // namespace cvxg
