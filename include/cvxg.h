/*
 * cvxg.h — C-ABI of the MI355X dense barrier Newton-step engine (drop-in boundary).
 *
 * Plain pointers, sizes and status codes; no torch or HIP types.  Every entry point below names the
 * reference interface (spyqqqdia/cvx, Scala 2.11 + Breeze 0.10) it replaces; INTEGRATION.md shows the
 * JNI binding a maintainer adds on the Scala side (GpuBarrierSolver).
 *
 * Ownership: the caller owns every host array and the engine only reads / writes it during the call
 * (never retained).  The context owns all device buffers.  One context per GPU, not thread-safe; calls
 * are synchronous on return.  Matrices are dense FP64 with an explicit leading dimension; `row_major`
 * selects the layout (Breeze DenseMatrix is column-major, so a JVM caller passes row_major = 0, or 1
 * for a transposed view).
 */
#ifndef CVXG_H
#define CVXG_H

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes: the JNI shim maps them back to the reference's exceptions so its fallback chains
 *  keep working. */
#define CVXG_OK 0
#define CVXG_E_NOT_PD 1          /* breeze NotConvergedException from cholesky (dpotrf info>0), MatrixUtils.scala:456 */
#define CVXG_E_LINSOLVE_TOL 2    /* LinSolveException, MatrixUtils.scala:507 / KKTSystem.scala:164 */
#define CVXG_E_INFEASIBLE_X 3    /* IllegalArgumentException "x not strictly feasible", BarrierSolver.scala:285 */
#define CVXG_E_LINESEARCH 4      /* NotConvergedException from line search, UnconstrainedSolver.scala:94,109 */
#define CVXG_E_UNSOLVABLE 5      /* UnsolvableSystemException, MatrixUtils.scala:631,698 */
#define CVXG_E_DIM 6             /* assert dimension mismatch */
#define CVXG_E_HIP 7             /* HIP runtime / device error */
#define CVXG_E_ARG 8             /* invalid argument or call order */
#define CVXG_E_UNSUPPORTED 9     /* configuration outside this build (e.g. n > 65472) */

/* Equality rows whose KKT right-hand sides can ride the factorization's fused forward solve (small problems).  Wider
 * equality blocks (any p < n) take the same KKTSystem.solveWithCholFactor sequence on the engine's own kernels
 * (k_kkt.hip): the p + 1 right-hand sides by two many-column triangular solves on the factor, and the p x p Schur
 * complement by a one-wave dpotf2-order factorization (p <= 64) or the dataflow Cholesky (p > 64).  rocBLAS /
 * rocSOLVER are not on any per-step path. */
#define CVXG_MAX_EQ 8

typedef struct cvxg_ctx cvxg_ctx;

/* Mirrors SolverParams (SolverParams.scala:24-46). */
typedef struct cvxg_params {
  int maxIter;        /* 1000 */
  double alpha;       /* 0.04  line-search descent factor */
  double beta;        /* 0.8   line-search backtrack factor */
  double tolSolver;   /* 1e-8  gap / decrement / gradient tolerance */
  double tolEqSolve;  /* 1e-1  relative residual tolerance of the KKT solve */
  double tolFeas;     /* 1e-7 */
  double delta;       /* 1e-6 */
} cvxg_params;

/* One inner Newton iteration (UnconstrainedSolver.scala:47-134 / EqualityConstrainedSolver.scala:61-110). */
typedef struct cvxg_step_info {
  double t;                 /* barrier parameter */
  double f;                 /* barrier value at x (BarrierSolver.scala:280-289) */
  double norm_grad;         /* |grad| at x */
  double q;                 /* dx . grad */
  double newton_decrement;  /* -q/2 */
  double hnorm;             /* sqrt(-q) = |dx|_H */
  double trust_radius;      /* frozen at iteration 0 (rho = 1+1/4 == 1) */
  double step;              /* accepted backtracking factor t = beta^k (0 if no step was taken) */
  double rel_err;           /* relativeSize(H dx + grad, -grad, tolEqSolve) of the accepted solve */
  double min_diag;          /* min diag(L) of the accepted Cholesky factor */
  double norm_grad_new;     /* |grad| at the new x */
  double equality_gap;      /* |b - A x| at the new x (p > 0) */
  int backtracks_c;         /* halvings until x + t s in C */
  int backtracks_armijo;    /* further halvings for sufficient decrease */
  int fallback;             /* 0 choleskySolve(H), 1 choleskySolve(H+1e-9 I) / solvePD(H+A'A), 2 symSolve / kktSymSolve */
  int ruiz_sweeps;          /* Ruiz iterations executed */
  int regularized;          /* regularizedCholesky used Q + 1e-10 I */
  int took_step;            /* 1 if x moved */
  int done;                 /* 1 if the centering loop terminates after this iteration */
  int iter;                 /* inner iteration index */
  int ls_fresh;             /* line-search feasibility trials evaluated fresh (margin inside the rounding band) */
  int ls_ties;              /* Armijo decisions inside the rounding band of the barrier value (rounding noise) */
  int small_pivot;          /* regularized: the 1-based row where the first attempt chol(Q) stopped -- its first
                               non-positive pivot, or the first row of the 16-column block whose min diag(L) <= 1e-7
                               (MatrixUtils.scala:456-460); 0 = not regularized */
} cvxg_step_info;

/* UnconstrainedSolver / EqualityConstrainedSolver result (Solution.scala:32-43). */
typedef struct cvxg_centering_info {
  int iter;
  int maxed_out;
  double newton_decrement;
  double norm_grad;
  double equality_gap;
} cvxg_centering_info;

/* BarrierSolver.solve result (BarrierSolver.scala:113-116, 173-176). */
typedef struct cvxg_solution {
  double duality_gap;
  double equality_gap;
  double newton_decrement;
  double norm_grad;
  double objective;         /* objF.valueAt(x) at the returned x */
  int iter;                 /* inner iterations of the LAST centering (reference semantics) */
  int maxed_out;
  int outer_iters;          /* t-loop passes */
  int newton_steps;         /* total inner Newton iterations (instrumentation the reference lacks) */
} cvxg_solution;

/* ---- context ------------------------------------------------------------------------------------ */

/* Allocate a context on HIP device `device` for n variables, m linear inequalities, p < n equalities (CVXG_E_DIM
 * otherwise, as EqualityConstraint asserts).  n <= 65472 (1023 Cholesky blocks of 64; CVXG_E_UNSUPPORTED above). */
int cvxg_create(int device, int n, int m, int p, cvxg_ctx** out);
void cvxg_destroy(cvxg_ctx* ctx);
const char* cvxg_last_error(const cvxg_ctx* ctx);  /* NULL: the last error of a context-free call (this thread) */
/* Library version / build string (for logs). */
const char* cvxg_version(void);

/* ---- packing of the reference's callback objects ------------------------------- */

/* QuadraticObjectiveFunction(dim, r, a, P) (QuadraticObjectiveFunction.scala:7-33); P == NULL gives
 * LinearObjectiveFunction(dim, r, a) (LinearObjectiveFunction.scala:7-21).  P must be symmetric. */
int cvxg_set_objective(cvxg_ctx* ctx, const double* P, int ldP, const double* a, double r);

/* The objective of Duality.dualProblem for Dist_KL (Duality.scala:74-79 over Dist_KL.scala:146-165): with z the
 * n dual variables (lambda, nu), B the n x nout matrix mat_B = (H; 1'; A) (Dist_KL.scala:134-140), w = vec_w
 * (:123-128) and R = 1/(nout e), e = 2.7182811828459045 (:114-116):
 *   valueAt(z) = w.z + R.exp(-B'z),  gradientAt(z) = w - B(R o exp(-B'z)),  hessianAt(z) = B diag(y) B'.
 * B is read row-major (row_major != 0, ldB >= nout) or column-major (ldB >= n). */
int cvxg_set_objective_kl(cvxg_ctx* ctx, const double* B, int ldB, int row_major, int nout, const double* w,
                          double R);

/* Dist_KL.objectiveFunction(n) (Dist_KL.scala:223-239), the KL distance from the uniform distribution on nout outcomes
 * (nout = the context's n for Dist_KL's own problems):
 *   valueAt(x) = x . log(x * nout),  gradientAt(x)_j = (1 + log x_j) + log nout,  hessianAt(x) = diag(1 / x).
 * Defined for x > 0 (Dist_KL's allCoordinatesPositive rows keep the iterates there).  The barrier solver and the
 * primal-dual solver (Dist_KL.scala:309-315, solverType "PD": its line-search residual takes the gradient afresh at
 * every trial point) run on it; cvxg_affine_from returns CVXG_E_UNSUPPORTED. */
int cvxg_set_objective_kl_primal(cvxg_ctx* ctx, int nout);

/* The LinearConstraint list r_i + a_i.x <= ub_i (LinearConstraint.scala:7-32), A row i = a_i in LIST
 * order (fold and forall order matter: BarrierSolver.scala:280-315, ConstraintSet.scala:34-38). */
int cvxg_set_ineq(cvxg_ctx* ctx, const double* A, int ldA, int row_major, const double* r,
                  const double* ub);

/* QuadraticConstraint(id, dim, ub, r, a, P): r + a.x + x'P x / 2 <= ub (QuadraticConstraint.scala:8-40).  Row
 * rows[k] (ascending) of the cvxg_set_ineq list holds its (a, r, ub); P_k is the n x n row-major block at
 * P + k n ldP (symmetric).  Call after cvxg_set_ineq (which clears the quadratic rows).  The barrier path
 * (value, gradient a + P x, Hessian terms G G'/d^2 + P/d, line search) and the primal-dual solver (KKT matrix
 * terms G G' lambda/d + lambda P, PrimalDualSolver.scala:224-238; gradients a + P x in rhs1, the dual residual and
 * dlambda) handle them. */
int cvxg_set_quad(cvxg_ctx* ctx, int q, const int* rows, const double* P, int ldP);

/* EqualityConstraint(A, b) (EqualityConstraint.scala:16). */
int cvxg_set_eq(cvxg_ctx* ctx, const double* Aeq, int ldAeq, int row_major, const double* beq);

/* Current iterate (device resident between calls): ConstraintSet.feasiblePoint / Solution.x. */
int cvxg_set_x(cvxg_ctx* ctx, const double* x);
int cvxg_get_x(cvxg_ctx* ctx, double* x);

/* ---- barrier oracles ---------------------------------------------------------------------------- */

/* BarrierSolver.barrierFunction / gradientBarrierFunction / hessianBarrierFunction
 * (BarrierSolver.scala:280-315) at (t, x).  g and H may be NULL; H is written n x n column-major
 * (symmetric).  Returns CVXG_E_INFEASIBLE_X when some d_i = ub_i - g_i(x) <= 0. */
int cvxg_barrier_eval(cvxg_ctx* ctx, double t, const double* x, double* f, double* g, double* H);

/* ConstraintSet.constraintFunctionAt without the -ub: g_i(x) = r_i + a_i.x (LinearConstraint.scala:22-24). */
int cvxg_constraint_values(cvxg_ctx* ctx, const double* x, double* gx);

/* Constraint.isActive (Constraint.scala:26): indices i with |g_i(x) - ub_i| < tol, ascending. */
int cvxg_active_set(cvxg_ctx* ctx, const double* x, double tol, int* idx, int* count);

/* ---- the hot path -------------------------------------------------------------------------------- */

/* Newton direction at (t, x) without the line search: MatrixUtils.choleskySolve(H, -grad) with its
 * UnconstrainedSolver fallbacks (UnconstrainedSolver.scala:54-67) when p == 0, KKTSystem.solve
 * (KKTSystem.scala:43-66) when p > 0.  grad may be NULL (then the engine's own barrier gradient at
 * (t, x) is used) or the caller's gradient (the reference passes `y` computed by the host).
 * dx[n]; w[p] may be NULL. */
int cvxg_newton_direction(cvxg_ctx* ctx, const cvxg_params* pars, double t, const double* x,
                          const double* grad, double* dx, double* w, cvxg_step_info* info);

/* Start the inner solver at barrier parameter t from the current iterate (new UnconstrainedSolver /
 * EqualityConstrainedSolver, BarrierSolver.scala:97,154). */
int cvxg_centering_begin(cvxg_ctx* ctx, double t);

/* Resume the inner solver in the middle of a centering, as the reference's loop state stands before inner iteration
 * `iter` (UnconstrainedSolver.scala:47-48): barrier parameter t, the trust radius frozen at iteration 0
 * (trustRadius, :86; ignored when iter == 0) and, when grad != NULL, the host's gradient y (:44,131) in place of the
 * engine's.  Lets a Scala caller that keeps its own loop hand over any iteration, and replays recorded steps. */
int cvxg_centering_resume(cvxg_ctx* ctx, double t, int iter, double trust_radius, const double* grad);

/* One inner Newton iteration on the device-resident iterate: assemble, equilibrate, factor, solve,
 * line search, update (UnconstrainedSolver.scala:47-134 or EqualityConstrainedSolver.scala:60-111).
 * info->done reports the loop condition for the next iteration. */
int cvxg_newton_step(cvxg_ctx* ctx, const cvxg_params* pars, cvxg_step_info* info);

/* The whole inner loop (UnconstrainedSolver.solve / EqualityConstrainedSolver.solve). */
int cvxg_centering(cvxg_ctx* ctx, const cvxg_params* pars, double t, cvxg_centering_info* info);

/* BarrierSolver.solve / solveSpecial (BarrierSolver.scala:70-188): the t-loop (mu = 10, t0 = 1) from
 * the current iterate.  termination: 0 = CvxUtils.standardTerminationCriterion, 1 =
 * CvxUtils.phase_I_TerminationCriterion (CvxUtils.scala:61-87). */
int cvxg_barrier_solve(cvxg_ctx* ctx, const cvxg_params* pars, int termination, cvxg_solution* sol);

/* ---- config C5 from one host process (a JVM caller): a batch of independent instances ------------------------ */

/* Run cvxg_barrier_solve / cvxg_newton_step on `count` distinct contexts concurrently, one host thread per context
 * (typically one context per GPU, each created on its own device with cvxg_create): the one-instance-per-GPU batch of
 * config C5 without a second process.  Nothing is exchanged between instances; afterwards each instance's x is read
 * with cvxg_get_x (the in-process counterpart of the RCCL gather of the multi-process path).  sols / infos[i] receive
 * context i's result (may be NULL), status[i] its return code (may be NULL); the call returns the first non-zero
 * status, CVXG_E_ARG for a NULL or repeated context. */
int cvxg_batch_barrier_solve(int count, cvxg_ctx* const* ctxs, const cvxg_params* pars, int termination,
                             cvxg_solution* sols, int* status);
int cvxg_batch_newton_step(int count, cvxg_ctx* const* ctxs, const cvxg_params* pars, cvxg_step_info* infos,
                           int* status);

/* ---- primal-dual interior-point solver (PrimalDualSolver.scala, solverType "PD") ---------------- */

/* One primal-dual iteration as PrimalDualSolver.solve_noEQs runs it (PrimalDualSolver.scala:421-427). */
typedef struct cvxg_pd_step_info {
  double t;                 /* the barrier-analogue parameter t = mu m / gap */
  double s0;                /* step bound min(1, -lambda_i / dlambda_i) (:331-338) */
  double step;              /* accepted step s (0.99 s0 beta^k) */
  double norm_residual;     /* |r_t| at (x, lambda) (:343, 350) */
  double rel_err;           /* choleskySolve residual ratio */
  int backtracks;           /* k of the accepted step */
  int fallback;             /* 0 choleskySolve(Q, s), 2 symSolve(Q, s) (SymmetricLinearSystem.scala:28-35) */
  int ruiz_sweeps;          /* SymmetricLinearSystem's own Ruiz sweeps (choleskySolve equilibrates Q again) */
  int regularized;          /* regularizedCholesky used Q + 1e-10 I */
} cvxg_pd_step_info;

/* Solution of PrimalDualSolver.solve (PrimalDualSolver.scala:455-459; with equality rows :615-620).  Filled after
 * every completed iteration, so after a failed one (CVXG_E_LINESEARCH) it describes the last accepted iterate. */
typedef struct cvxg_pd_solution {
  double duality_gap;       /* surrogate gap -h(x).lambda (:289-297) */
  double norm_dual_residual;/* |grad f + Dg' lambda| (:63-71); with equality rows the whole |r_t(x, lambda, nu)|
                               (residual_withEqs :133-145, as solve_withEQs reports it, :606) */
  double objective;         /* objF.valueAt(x) */
  int iter;                 /* iterations - 1 (reference semantics, :458) */
  int maxed_out;            /* iter == 2000/mu (1500/mu with equality rows, :577) */
  int newton_steps;         /* KKT solves performed (instrumentation) */
  double equality_gap;      /* |A x - b| with equality rows (:603), 0 without */
} cvxg_pd_solution;

/* The primal-dual search direction at (t, x, lambda) (PrimalDualSolver.scala:216-261, 184-209): the KKT
 * matrix H_pd = hessian f + sum_i [lambda_i grad2 g_i + (lambda_i / -f_i) G_i G_i'] (weighted SYRK over the gradient
 * rows G_i = a_i (+ P_i x), + lambda_k P_k), rhs1 = -grad f + sum_i G_i/(t f_i),
 * SymmetricLinearSystem(H_pd, rhs1).solve(tolEqSolve) (Ruiz, then choleskySolve with its own Ruiz, symSolve on any
 * failure), then dlambda.  lambda has m entries; dx (n) / dlambda (m) may be NULL.  No equality constraints. */
int cvxg_pd_direction(cvxg_ctx* ctx, const cvxg_params* pars, double t, const double* x, const double* lambda,
                      double* dx, double* dlambda, cvxg_pd_step_info* info);

/* The search direction of solve_withEQs (PrimalDualSolver.scala:590-593) at (t, x, lambda, nu) for a context with
 * p > 0 equality rows (cvxg_set_eq): kktSystem_withEqs (:271-285) = KKTSystem(H_pd, A, q = rhs1 + A'nu, b - A x)
 * solved as KKTSystem.solve does for the barrier's equality step (KKTSystem.scala:43-66: solvePD, solvePD on
 * H + A'A, kktSymSolve), giving dx (n) and dnu (p), then deltaLambda (m).  With p == 0 nu / dnu are ignored and this
 * is cvxg_pd_direction.  Output pointers may be NULL. */
int cvxg_pd_direction_eq(cvxg_ctx* ctx, const cvxg_params* pars, double t, const double* x, const double* lambda,
                         const double* nu, double* dx, double* dlambda, double* dnu, cvxg_pd_step_info* info);

/* PrimalDualSolver.solve (PrimalDualSolver.scala:628-633 -> solve_noEQs :381-460) from the current iterate
 * (cvxg_set_x: a strictly feasible point): lambda0 = -1/h(x0) (ConstraintSet.scala:116-120), t = mu m / gap,
 * residual-norm backtracking line search (:311-374), stop when gap < tolSolver and |r_dual| < tolSolver.
 * With equality rows (p > 0) solve_withEQs (:550-621) as written: nu0 = 0, the direction of cvxg_pd_direction_eq,
 * lineSearch_withEQs (:478-543) on |(r_dual + A'nu, r_central, A x - b)|, at most 1500/mu iterations.  The reference
 * passes q = rhs1 + A'nu to KKTSystem, which solves H dx + A'dnu = -q: the opposite sign of its own no-equality
 * system ("FIX ME", :284).  Its line search then fails after a few iterations on every problem we ran (the
 * reference's known-answer problems and random QPs, tests/test_oracle_known_answers.py); the engine reproduces the
 * same trajectory and returns CVXG_E_LINESEARCH at the same iteration, where the reference throws
 * LineSearchFailedException (sol and the iterate then hold the last accepted step). */
int cvxg_pd_solve(cvxg_ctx* ctx, const cvxg_params* pars, cvxg_pd_solution* sol);

/* The dual iterate lambda (m entries) after cvxg_pd_solve. */
int cvxg_get_lambda(cvxg_ctx* ctx, double* lambda);

/* The equality multipliers nu (p entries) after cvxg_pd_solve with equality rows. */
int cvxg_get_nu(cvxg_ctx* ctx, double* nu);

/* ---- affine re-parametrisation x = z0 + F u (BarrierSolver.affineTransformed / reduced) ----------- */

/* SolutionSpace(A, b) (SolutionSpace.scala:20-27 -> MatrixUtils.solveUnderdetermined, MatrixUtils.scala:536-550):
 * for A (p x n, p < n, full rank) the QR of A' (rocSOLVER dgeqrf + dorgqr with the full n x n Q, the LAPACK routines
 * Breeze's qr calls) gives F = Q(:, p..n-1) (column-major n x (n-p), leading dimension ldF >= n, orthonormal columns
 * spanning ker A) and z0 = Q(:, 0..p-1) y with R'y = b by forwardSolve (the minimum-norm solution).  No context:
 * errors are reported through cvxg_last_error(NULL). */
int cvxg_solution_space(int device, int p, int n, const double* A, int ldA, int row_major, const double* b,
                        double* z0, double* F, int ldF);

/* BarrierSolver.affineTransformed(z0, F, u0) (BarrierSolver.scala:209-232): load into `dst` (created with n = F.cols,
 * the same m and p as `src`, on the same device) the problem of `src` pulled back to u with x = z0 + F u.  The
 * reference composes its barrier functions (value at z0 + F u, F' gradient, (F' H) F); this engine transforms the
 * problem data once on the device instead — P_u = F'PF, a_u = F'(a + P z0), r0_u = f0(z0), constraint rows A F with
 * r + A z0 (LinearConstraint.affineTransformed, LinearConstraint.scala:46-52), quadratic rows F'(a + P_k z0) and
 * F'P_kF with r + a.z0 + z0'P_k z0/2 (QuadraticConstraint.scala:54-61), equalities (A_eq F) u = b - A_eq z0
 * (EqualityConstraint.scala:72-73) — so each Newton step runs in dimension F.cols at the cost of that dimension.
 * Equal to the reference's composition in exact arithmetic.  F is column-major (ldF >= src n).  The KL dual
 * objective is not transformable (CVXG_E_UNSUPPORTED).  dst keeps z0 and F for the two calls below. */
int cvxg_affine_from(cvxg_ctx* dst, cvxg_ctx* src, const double* z0, const double* F, int ldF);

/* SolutionSpace.parameter (SolutionSpace.scala:29-33): u0 = F'(x0 - z0) (x0 has src n entries, u0 dst n). */
int cvxg_affine_parameter(cvxg_ctx* dst, const double* x0, double* u0);

/* x = z0 + F u (the reporting map of the reduced solvers, UnconstrainedSolver.scala:199-200); u NULL = the current
 * iterate of dst. */
int cvxg_affine_map(cvxg_ctx* dst, const double* u, double* x);

/* ---- instrumentation ----------------------------------------------------------------------------- */

/* Per-phase device time (ms), the mean over the Newton steps (or PD iterations) since timing was enabled (at most the
 * last 63) that recorded the phase -- so a step whose assembly was prefetched before timing was enabled does not count
 * as a zero -- measured with HIP events on the stream each phase runs on; the steps never wait on them (only this call
 * synchronises): [0] assembly when not prefetched [1] Ruiz+scale [2] Cholesky (+fused forward solve)
 * [3] backward solve + residual [4] line search [5] the assembly SYRK alone (on its own stream when it was launched
 * behind the previous evaluation).  enabled = 1 records every phase; enabled = 2 records only the assembly and Cholesky
 * phases ([0], [2], [5]) -- every event record leaves the GPU idle a few microseconds between kernels. */
int cvxg_set_timing(cvxg_ctx* ctx, int enabled);
int cvxg_get_phase_times(cvxg_ctx* ctx, double* ms, int count);
/* cvxg_get_phase_times plus, per phase, the number of recorded occurrences its mean is over (occurrences may be NULL):
 * a phase that not every step runs (the inline assembly [0]) is then weighted by its occurrences, not by steps. */
int cvxg_get_phase_stats(cvxg_ctx* ctx, double* ms, int* occurrences, int count);
/* Diagnostic counters since cvxg_create (up to count of them): [0] Ruiz lookahead extensions, [1] speculative
 * regularized pairs launched (chol(Q) and chol(Q + 1e-10 I) side by side after a regularized direction), [2] pairs
 * whose second attempt was the one kept, [3] factorization attempts, [4] regularized directions. */
int cvxg_get_counters(cvxg_ctx* ctx, long long* out, int count);

/* The Newton step's Ruiz lookahead (cholesky_solve, MatrixUtils.scala:240-268 as restated in k_vec.hip): the next
 * step first launches `sweeps` Ruiz sweeps (the last step's count + 1 by default, RUIZ_MAX = 20 on a fresh
 * context), reads whether the loop is done, and launches 2 more at a time until it is, so results equal the full
 * loop's.  sweeps <= 0 leaves the setting; *relaunches (if given) receives how many extra batches were launched. */
int cvxg_set_ruiz_lookahead(cvxg_ctx* ctx, int sweeps, long long* relaunches);

/* Engine options.  cvxg_create sets every option to the product default; the other values are measured alternatives
 * kept for A/B runs and for the tests that hold the default to them.  None changes the reference's semantics, and the
 * library reads no environment variable that changes arithmetic (tracing aside). */
enum {
  CVXG_OPT_SPARSE_ROWS = 1,   /* 1 (default): rows with <= 4 nonzeros are summed per Hessian entry apart from the SYRK;
                                 0: every row through the SYRK.  Set before cvxg_set_ineq. */
  CVXG_OPT_EARLY_ABORT = 2,   /* 1 (default): regularizedCholesky's first attempt stops at its first 16-column block with
                                 min diag(L) <= 1e-7 (MatrixUtils.scala:458-460 discards that factor); 0: it runs on */
  CVXG_OPT_H_LOWER = 3,       /* 1 (default): the Newton step keeps H's lower triangle only; 0: H is mirrored */
  CVXG_OPT_KKT_FUSED_RHS = 4, /* 1..9: the KKT columns ride the fused forward solve when p + 1 <= value (default 9 below
                                 8 Cholesky blocks, else 1: the many-column dataflow solves) */
  CVXG_OPT_SPEC_REG = 5,      /* 1 (default): after a regularized direction, chol(Q) and chol(Q + 1e-10 I) run side by
                                 side and the device keeps the one regularizedCholesky keeps; 0: one after the other */
  CVXG_OPT_RUIZ_LOOP = 6,     /* 1: the whole Ruiz loop in one persistent launch (the default up to n = 1024;
                                 CVXG_E_UNSUPPORTED beyond its register batch of tiles); 0: each sweep a launch pair
                                 (the default above n = 1024).  Both give the same bits */
  CVXG_OPT_RUIZ_WG = 7        /* workgroups of the one-launch Ruiz loop (0, the default: one per CU) */
};
/* Returns CVXG_E_ARG for an unknown option or a value out of its range. */
int cvxg_set_option(cvxg_ctx* ctx, int option, long long value);

/* The worker task order of the dataflow Cholesky for nblk diagonal blocks and `workers` simulated workgroups,
 * exactly as cvxg_create builds it (host-only, no device needed): each entry (type << 30) | (k << 20) | (i << 10)
 * | j with type 1 TRSM(i,k), 2 UPDATE(i,j,k), 3 UPDATE4(i,j,k..k+3); the chain tasks are not listed.  Writes at
 * most cap entries and returns the task count (or a negative status). */
int cvxg_chol_schedule(int nblk, int workers, unsigned* order, int cap);

#ifdef __cplusplus
}
#endif
#endif /* CVXG_H */
