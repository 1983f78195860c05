// cvxg.cpp — C-ABI (include/cvxg.h) and host orchestration of the MI355X barrier Newton engine.
//
// Host side keeps only scalar control flow that the reference evaluates sequentially: the t-loop
// (BarrierSolver.scala:70-177), the inner Newton loop and its fallback chains
// (UnconstrainedSolver.scala:34-125, EqualityConstrainedSolver.scala:37-107, KKTSystem.scala:43-66,
// MatrixUtils.scala:452-516) and the backtracking decisions (UnconstrainedSolver.scala:83-113), read
// from one small device->host copy per decision point.  All vector/matrix work is HIP (k_*.hip).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <limits>
#include <queue>
#include <string>
#include <thread>
#include <vector>

#include "../../include/cvxg.h"
#include "kernels.hpp"

using namespace cvxg;

namespace {

constexpr int NT = 8;  // phase timers

// Phase timers: HIP events recorded on the stream each phase runs on, one ring slot per Newton step (or PD iteration),
// read only by cvxg_get_phase_times -- a step never waits on its own events, so timing does not serialise the
// pipeline (the prefetched assembly of the next step runs beside the host's reads).
constexpr int TRING = 64;
struct Timer {
  hipEvent_t ev[TRING][NT][2] = {};
  bool on = false, created = false;
  bool all = false;  // every phase; otherwise only the assembly and Cholesky phases (0, 2, 5): an event record is a
                     // marker packet that leaves the GPU idle ~3-4 us between kernels (microbench/hostcost.hip)
  bool rec[TRING][NT] = {};
  int tick = 0;      // the step being recorded: ring slot tick % TRING
  int steps = 0;     // steps recorded since timing was enabled (capped at TRING - 1)
  bool pf5 = false;  // slot 5 of the next tick already holds the prefetched assembly
};

}  // namespace

struct cvxg_ctx {
  int dev = 0, n = 0, m = 0, p = 0, np = 0, mp = 0, nblk = 0;
  hipStream_t s = nullptr;
  // problem
  double* P = nullptr;
  int hasP = 0;
  // KL dual objective (cvxg_set_objective_kl): KB = B' (nout x n, row-major, padded noutp x np), R = 1/(n e)
  int kl = 0, nout = 0, noutp = 0;
  double kl_R = 0.0;
  double *KB = nullptr, *kl_v = nullptr, *kl_y = nullptr, *kl_u = nullptr, *kl_negBy = nullptr;
  double *kl_part = nullptr, *kl_ls = nullptr;
  // certified line search of the KL dual: |B'||z|, |B'||s|; a fresh trial point's B'zt and y
  double *kl_vabs = nullptr, *kl_uabs = nullptr, *kl_vtr = nullptr, *kl_ytr = nullptr;
  // KL primal objective (cvxg_set_objective_kl_primal): f0 = x . log(n x), its gradient and diag(1/x) Hessian
  int klp = 0;
  double klp_n = 0.0;
  double *klp_lx = nullptr, *klp_g0 = nullptr, *klp_hd = nullptr, *klp_ab = nullptr, *klp_lxt = nullptr;
  double *klp_part = nullptr, *klp_ls = nullptr;
  double* a0 = nullptr;
  double r0 = 0.0;
  double *A = nullptr, *r = nullptr, *ub = nullptr;
  double *Aeq = nullptr, *beq = nullptr;
  int have_obj = 0, have_ineq = 0, have_eq = 0;
  // iterate and vectors
  double *x = nullptr, *y = nullptr, *dx = nullptr, *sdir = nullptr, *xtmp = nullptr, *vtmp = nullptr;
  double *Px = nullptr, *Ps = nullptr, *e = nullptr;
  double *c = nullptr, *d = nullptr, *invd = nullptr, *w = nullptr, *logd = nullptr;
  double *eqd = nullptr, *eqtmp = nullptr;  // b - Aeq x
  // KKT equality block (k_kkt.hip): X = Q^-1 [B' | Dq] in kY (np x kY_ld, row-major; the fused forward solve's rhs
  // and the backward solve's sol buffers instead when p + 1 <= kkt_fused_rhs), R = B X partials, S / z, w
  int kkt_fused_rhs = MAX_RHS;  // set at creation; CVXG_OPT_KKT_FUSED_RHS overrides (1: the many-column solves)
  double *kY = nullptr, *kYg = nullptr, *kgram = nullptr, *kS = nullptr, *kzp = nullptr;
  int kY_ld = 0, kY_chunks = 0, fm_gen = 0;
  // p > 64: S factored by the dataflow Cholesky on its own buffers (pS = p rounded up to 64), w by its backward solve
  double *sL = nullptr, *sLinv = nullptr, *sw = nullptr;
  unsigned* s_tasks = nullptr;
  int *s_work = nullptr, *s_bwd = nullptr;
  int s_nblk = 0, s_ntasks = 0, s_gen = 0;
  // matrices
  double *H = nullptr, *L = nullptr, *Linv = nullptr, *Hsave = nullptr;
  double *ruiz0 = nullptr, *ruiz1 = nullptr, *dfin = nullptr, *hdiag = nullptr;
  double *rhs = nullptr, *sol = nullptr;
  double* part = nullptr;
  size_t part_bytes = 0;
  double *kB = nullptr, *kw = nullptr, *kx = nullptr, *kz = nullptr;
  double *ls_plog = nullptr, *ls_log = nullptr, *ls_paux = nullptr;
  int *ls_pcnt = nullptr, *ls_cnt = nullptr;
  // certified line-search decisions: |r| + |a|.|x| per row, |a|.|s| per row, |P||x|, |P||s|; the fresh evaluation of
  // an ambiguous trial point xt = x + s t goes to its own buffers (the batch keeps reading c and e)
  double *cabs = nullptr, *eabs = nullptr, *Pxa = nullptr, *Psa = nullptr;
  double *xtr = nullptr, *Pxtr = nullptr, *c_tr = nullptr, *d_tr = nullptr, *invd_tr = nullptr, *w_tr = nullptr,
         *logd_tr = nullptr;
  // the speculative evaluation at x1 = x + dx t (k_ls_setup_eval, t = spec_t below), swapped with c/d/invd/w/logd/cabs
  // when the line search accepts that t
  double *x1 = nullptr, *c1 = nullptr, *d1 = nullptr, *invd1 = nullptr, *w1 = nullptr, *logd1 = nullptr,
         *cabs1 = nullptr;
  int* tiles = nullptr;
  int ntiles = 0, nsplit = 1;
  int ntiles_main = 0;  // tiles assembled without K split (whole waves of slots); the rest use nsplit
  int slots = 512;     // SYRK workgroup slots (2 per CU)
  // Sparse constraint rows (<= SPARSE_NNZ nonzeros: bounds, phase-I bound rows, box rows).  Their Hessian
  // terms are per-entry sums (k_sparse_hess); only the dense rows, packed into As, go through the SYRK.
  int sparse_rows = 1;          // CVXG_OPT_SPARSE_ROWS 0 disables the split (A/B)
  int early_abort = 1;          // regularizedCholesky's first attempt stops at min diag(L) <= 1e-7 (CVXG_OPT_EARLY_ABORT)
  // The Newton-step assembly with p == 0 stores H's lower triangle (and its diagonal tiles whole) only: Ruiz, the
  // Cholesky and the residual (a lower-triangle symv) read nothing else; consumers of the full matrix (eigen fallback,
  // KKT paths, cvxg_barrier_eval, the primal-dual solver) mirror it first (ensure_h_full).  CVXG_OPT_H_LOWER 0: mirror
  int h_lower = 1;
  bool h_full = true;           // the current H holds its upper triangle too
  double* hsv_part = nullptr;   // symv partials (nblk x np)
  // Ruiz: every sweep in one persistent launch (k_ruiz.hip; CVXG_OPT_RUIZ_LOOP; 0: two launches per sweep)
  int ruiz_loop = 0;            // (the default up to RUIZ_LOOP_MAX_BLOCKS blocks, cvxg_create)
  unsigned long long* ruiz_trace = nullptr;  // CVXG_RUIZ_TRACE=<file>: per-workgroup sweep stamps of the last loop
  std::string ruiz_trace_path;
  int ruiz_wg = 0;              // its workgroups (0: one per CU; CVXG_OPT_RUIZ_WG, tests: fewer -> streamed tiles)
  double* ruiz_S = nullptr;     // its data-tagged granules (ruiz_loop_doubles)
  unsigned long long ruiz_gen = 0;  // its launch generation (the granules' tags)
  int* ruiz_work = nullptr;     // its counters and flags (ruiz_loop_work_ints)
  int small_piv = 0;            // the last first attempt's stop row (DevCtrl::small_piv, or chol_info)
  int have_sparse = 0;          // set_ineq found sparse rows: the SYRK runs over As / wd / mdp
  int ndense = 0, mdp = 0;      // dense rows, padded to MPAD (>= MPAD)
  double *As = nullptr, *wd = nullptr;
  int* didx = nullptr;          // As row -> constraint index
  int sp_T = 0;                 // lower entries touched by sparse rows
  int *sp_ptr = nullptr, *sp_pq = nullptr, *sp_row = nullptr;
  double* sp_coef = nullptr;
  int kl_nsplit = 1;            // K split of the KL SYRK's tail tiles over the outcomes
  double* kl_spart = nullptr;   // its partials
  // QuadraticConstraint rows (cvxg_set_quad): row qrows[k] of A holds a_k, P_k stacked in Pq ((nq np) x np)
  int nq = 0;
  std::vector<int> qrows_h;
  std::vector<char> is_quad;     // per constraint row
  int *qrows = nullptr, *qslot = nullptr;  // device: row of constraint k, its row in As
  double *Pq = nullptr, *qPx = nullptr, *qPs = nullptr, *qextra = nullptr, *qf = nullptr;
  // certified line search of quadratic rows: |P_k||x|, |P_k||s| (stacked), the band's t^2 term per row, and a fresh
  // trial point's P_k xt and xt'P_k xt / 2
  double *qPxa = nullptr, *qPsa = nullptr, *qfabs = nullptr, *qPx_tr = nullptr, *qextra_tr = nullptr;
  // primal-dual solver state (PrimalDualSolver.scala; allocated on first use)
  double *lam = nullptr, *dlam = nullptr, *pd_rc = nullptr, *pd_w = nullptr;  // mp
  double *pd_rhs = nullptr, *pd_d1 = nullptr, *pd_R0 = nullptr, *pd_R1 = nullptr, *pd_R2 = nullptr;  // np
  double* pd_tmp = nullptr;
  double *pd_part_rows = nullptr, *pd_part_cols = nullptr, *pd_out = nullptr, *pd_hout = nullptr;
  // solve_withEQs: nu, dnu, A x - b, A dx (pe); the dual residual + A'nu and its step term (np); trial partials
  double *pd_nu = nullptr, *pd_dnu = nullptr, *pd_rp = nullptr, *pd_adx = nullptr;
  double *pd_R0e = nullptr, *pd_R1e = nullptr, *pd_part_eq = nullptr;
  // symSolve / kktSymSolve fallback buffers (allocated on first use; ldm = round_up(n + p, 128))
  int eig_ldm = 0;
  double *eig_M = nullptr, *eig_K = nullptr, *eig_d = nullptr, *eig_e = nullptr, *eig_dots = nullptr;
  double *eig_a = nullptr, *eig_z = nullptr, *eig_b = nullptr, *eig_x = nullptr, *eig_part = nullptr;
  int* eig_info = nullptr;
  int* bwd_flags = nullptr;
  int bwd_gen = 0;
  // Ruiz lookahead (cholesky_solve): the sweeps the next step launches first, and how often more had to follow
  int ruiz_launch = RUIZ_MAX;
  int ruiz_k1 = 0;            // Ruiz sweeps launched so far in this step (lookahead)
  bool ruiz_pending = false;  // the lookahead went out without a host read: the next factor attempt checks it
  long long ruiz_relaunches = 0;
  int ncu = 256;
  unsigned* df_tasks = nullptr;
  int df_ntasks = 0;
  int* df_work = nullptr;
  unsigned long long* df_trace = nullptr;  // CVXG_DF_TRACE=<file>: per-task timeline of the last factorization
  std::string df_trace_path;
  DevCtrl* ctrl = nullptr;
  DevCtrl* hctrl = nullptr;     // coherent pinned mirror of ctrl (written by k_publish_ctrl)
  DevCtrl* hctrl_dev = nullptr; // its device-side address
  unsigned* hflag = nullptr;    // coherent pinned sequence word of host_read, and its device-side address
  unsigned* hflag_dev = nullptr;
  unsigned hseq = 0;
  double* hls_dev = nullptr;    // device-side address of hls (coherent pinned)
  double* hls = nullptr;  // pinned: [3*LS_TRIALS] {log sum, its error bound, sum |log|} then [4*LS_TRIALS] counts as ints
  // centering state
  double t = 1.0;
  int iter = 0;
  double trust = NAN;
  int began = 0;
  double nd = 0.0;        // newton decrement
  double normGrad = 0.0;
  double eqGap = 0.0;
  double f_at_x = 0.0;    // barrier value at x
  int x_eval_valid = 0;   // c/d/w/y/scalars correspond to the current x and t
  // The next step's Hessian assembly, launched on the main stream as soon as the step's constraint values (w) exist,
  // while the rest of the evaluation (P x, A'(1/d), the gradient, the reductions) and the host's read of it run on s2
  // behind ev_w; the main stream then waits on ev_h (that tail) only if it has not finished.  h_valid: H holds the
  // assembly at the current x and t (x_eval_valid too).
  hipStream_t s2 = nullptr;
  hipEvent_t ev_w = nullptr, ev_h = nullptr;
  // speculative regularized pair (regularized_cholesky_spec): after a regularized Newton direction the next one runs
  // chol(Q) and chol(Q + 1e-10 I) side by side, each on half of the CUs (CVXG_OPT_SPEC_REG 0: one after the other)
  int spec_reg = 1;
  int prev_reg = 0;
  bool pair_active = false;
  double *L2 = nullptr, *Linv2 = nullptr, *rhs2 = nullptr;
  int* df_work2 = nullptr;
  DevCtrl* ctrl2 = nullptr;
  hipStream_t s3 = nullptr;
  hipEvent_t ev_p0 = nullptr, ev_p1 = nullptr;
  long long spec_pairs = 0, spec_pairs_used = 0;  // pairs launched / pairs whose second attempt was the one used
  long long n_attempts = 0, n_regularized = 0;
  bool h_valid = false;
  // The line search's setup (A s, P s, their dots) and first trial batch, enqueued behind each factorization attempt
  // of a Newton step with s = dx (the trust radius does not clamp in the common case), so the attempt's host read
  // carries them: spec_allowed (set by cvxg_newton_step), spec_launched (this attempt enqueued them), spec_have (the
  // last host read holds them for the current dx).
  bool spec_allowed = false, spec_launched = false, spec_have = false;
  // spec_eval_*: the setup's sweep over A also evaluated the constraints at x + dx (linear rows only)
  bool spec_eval_launched = false, spec_eval_have = false;
  double spec_beta = 0.5;
  // the step the speculative evaluation assumes: the previous step's accepted t (1 at a centering's start); late in
  // the path the line search takes the same beta^k step after step, early on mostly t = 1
  double spec_t = 1.0, spec_t_used = 1.0;
  double* spart = nullptr;  // SYRK split-K partials (ctx->part belongs to the evaluation's A'(1/d))
  // affine re-parametrisation (cvxg_affine_from): x = z0 + F u with F (aff_n x n, column-major, ld aff_n)
  double *aff_F = nullptr, *aff_z0 = nullptr;
  int aff_n = 0;
  Timer tm;
  std::string err;
};

// ------------------------------------------------------------------------------------------------
// helpers
// ------------------------------------------------------------------------------------------------
static int set_err(cvxg_ctx* ctx, int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (ctx) ctx->err = buf;
  return code;
}

#define HIPC(ctx, call)                                                                              \
  do {                                                                                               \
    hipError_t _e = (call);                                                                          \
    if (_e != hipSuccess) return set_err(ctx, CVXG_E_HIP, "%s failed: %s (%s:%d)", #call,           \
                                         hipGetErrorString(_e), __FILE__, __LINE__);                  \
  } while (0)

#define CHK(call)              \
  do {                         \
    int _rc = (call);          \
    if (_rc != CVXG_OK) return _rc; \
  } while (0)

static inline int round_up(int v, int a) { return (v + a - 1) / a * a; }

template <class T>
static int dalloc(cvxg_ctx* ctx, T** p, size_t count) {
  HIPC(ctx, hipMalloc((void**)p, std::max<size_t>(count, 1) * sizeof(T)));
  HIPC(ctx, hipMemsetAsync(*p, 0, std::max<size_t>(count, 1) * sizeof(T), ctx->s));
  return CVXG_OK;
}

static bool timed(const cvxg_ctx* ctx, int i) { return ctx->tm.on && (ctx->tm.all || i == 0 || i == 2 || i == 5); }
static void tstart(cvxg_ctx* ctx, int i) {
  if (timed(ctx, i)) (void)hipEventRecord(ctx->tm.ev[ctx->tm.tick % TRING][i][0], ctx->s);
}
static void tstop(cvxg_ctx* ctx, int i) {
  if (timed(ctx, i)) {
    (void)hipEventRecord(ctx->tm.ev[ctx->tm.tick % TRING][i][1], ctx->s);
    ctx->tm.rec[ctx->tm.tick % TRING][i] = true;
  }
}

static int copy_sync(cvxg_ctx* ctx, void* dst, const void* src, size_t bytes, hipMemcpyKind kind) {
  HIPC(ctx, hipMemcpyAsync(dst, src, bytes, kind, ctx->s));
  HIPC(ctx, hipStreamSynchronize(ctx->s));
  return CVXG_OK;
}

// Host reads behind everything enqueued so far on ctx->s, without a stream synchronisation: k_publish copies the
// ranges into coherent pinned host memory and then writes a sequence word that the host spins on (a stream
// synchronisation's wake-up left the GPU idle ~20-30 us per read, profiles/r03 timeline).  A failed launch or a
// faulted stream ends the spin through hipStreamQuery.
static int host_read(cvxg_ctx* ctx, const void* s0, void* d0, size_t b0, const void* s1 = nullptr, void* d1 = nullptr,
                     size_t b1 = 0, hipStream_t st = nullptr) {
  if (!st) st = ctx->s;
  const unsigned seq = ++ctx->hseq;
  launch_publish(st, s0, d0, b0, s1, d1, b1, ctx->hflag_dev, seq);
  HIPC(ctx, hipGetLastError());
  for (unsigned spins = 0;; ++spins) {
    if (__atomic_load_n(ctx->hflag, __ATOMIC_ACQUIRE) == seq) break;
    if ((spins & 1023) == 1023) {
      const hipError_t q = hipStreamQuery(st);
      if (q == hipSuccess) {  // the stream drained: the word must be there (re-read once, then report)
        if (__atomic_load_n(ctx->hflag, __ATOMIC_ACQUIRE) == seq) break;
        return set_err(ctx, CVXG_E_HIP, "host_read: stream idle but the sequence word was not published");
      }
      if (q != hipErrorNotReady)
        return set_err(ctx, CVXG_E_HIP, "HIP error %d (%s) during a host read", (int)q, hipGetErrorString(q));
    }
    __builtin_ia32_pause();
  }
  return CVXG_OK;
}

static int sync_ctrl(cvxg_ctx* ctx) { return host_read(ctx, ctx->ctrl, ctx->hctrl_dev, sizeof(DevCtrl)); }

// Upload an n-vector into a zero-padded device vector of length np.
static int upload_vec(cvxg_ctx* ctx, double* dst, const double* src, int n, int np) {
  std::vector<double> h(np, 0.0);
  memcpy(h.data(), src, sizeof(double) * n);
  HIPC(ctx, hipMemcpyAsync(dst, h.data(), sizeof(double) * np, hipMemcpyHostToDevice, ctx->s));
  HIPC(ctx, hipStreamSynchronize(ctx->s));
  return CVXG_OK;
}

// Pack a (rows x cols) matrix with leading dimension ld (row- or column-major) into a device row-major
// buffer of (rows_pad x ldd), zero padded.
static int upload_mat(cvxg_ctx* ctx, double* dst, int ldd, int rows_pad, const double* src, int rows, int cols,
                      int ld, int row_major) {
  std::vector<double> h((size_t)rows_pad * ldd, 0.0);
  for (int i = 0; i < rows; ++i)
    for (int j = 0; j < cols; ++j)
      h[(size_t)i * ldd + j] = row_major ? src[(size_t)i * ld + j] : src[(size_t)j * ld + i];
  HIPC(ctx, hipMemcpyAsync(dst, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice, ctx->s));
  HIPC(ctx, hipStreamSynchronize(ctx->s));
  return CVXG_OK;
}

// Lower-tile order for the assembly SYRK.  Workgroup b runs on XCD b % 8 (round-robin dispatch; used for
// locality only, never for correctness).  When nt % 4 == 0 the 32x32-tile triangle is cut into 4x4 block
// pairs of g = nt/4 tile rows: the 6 off-diagonal pairs (g*g tiles, 2g column panels each) and two groups
// of two diagonal pairs (g(g+1) tiles, 2g panels) give every XCD a tile set that touches only half of A's
// column panels, so each XCD's L2 streams half of A instead of all of it.  Each XCD gets the same number
// of full-K tiles (whole waves of its slots); the surplus of the diagonal groups (their diagonal tiles) is
// the split-K tail.  Other shapes: diagonal tiles first, whole waves, the rest is the tail.
static std::vector<int> syrk_tile_plan(int nt, int slots, int* nmain) {
  std::vector<int> tl;
  const int per_xcd = slots / 8;
  if (nt % 4 == 0 && nt >= 8 && slots % 8 == 0) {
    const int g = nt / 4;
    std::vector<std::vector<int>> grp;
    for (int a = 1; a < 4; ++a)
      for (int b = 0; b < a; ++b) {
        std::vector<int> v;
        for (int i = 0; i < g; ++i)
          for (int j = 0; j < g; ++j) v.push_back(((a * g + i) << 16) | (b * g + j));
        grp.push_back(v);
      }
    for (int pair = 0; pair < 2; ++pair) {
      std::vector<int> v, dg;
      for (int a = 2 * pair; a < 2 * pair + 2; ++a)
        for (int i = 0; i < g; ++i) {
          for (int j = 0; j < i; ++j) v.push_back(((a * g + i) << 16) | (a * g + j));
          dg.push_back(((a * g + i) << 16) | (a * g + i));
        }
      v.insert(v.end(), dg.begin(), dg.end());  // diagonal tiles last: they become the tail
      grp.push_back(v);
    }
    size_t shortest = grp[0].size();
    for (auto& v : grp) shortest = std::min(shortest, v.size());
    const int S = per_xcd > 0 ? (int)(shortest / per_xcd) * per_xcd : 0;
    if (S > 0) {
      for (int s = 0; s < S; ++s)
        for (int x = 0; x < 8; ++x) tl.push_back(grp[x][s]);
      for (int x = 0; x < 8; ++x) tl.insert(tl.end(), grp[x].begin() + S, grp[x].end());
      *nmain = 8 * S;
      return tl;
    }
  }
  for (int I = 0; I < nt; ++I) tl.push_back((I << 16) | I);
  for (int I = 0; I < nt; ++I)
    for (int J = 0; J < I; ++J) tl.push_back((I << 16) | J);
  *nmain = ((int)tl.size() / slots) * slots;
  return tl;
}

// Task order of the persistent dataflow Cholesky (k_dataflow.hip) for nb x nb tiles: the DAG
// POTRF(k) -> TRSM(i,k) -> UPDATE(i,j,k..) -> next UPDATE of tile (i,j) | POTRF(j) | TRSM(i,j) is list-scheduled on
// `workers` simulated workgroups with estimated task times, highest bottom level (longest path to the end)
// first among the ready tasks; the emitted order is the simulated start order, hence topological.  A tile's
// updates from panels k < j - `singles` are grouped four at a time (UPDATE4: one read-modify-write of the
// tile for four panels); the last `singles` panels stay single so that a tile's final update is not held
// back by its group.  The critical chain tasks POTRF(k), TRSM(k+1,k), UPDATE(k+1,k+1,k) are simulated but
// not emitted (workgroup 0 runs them in sequence); every transitive dependency of a chain task still precedes
// that task's dependents in the emitted order, which keeps the launch deadlock-free.
struct SchedTimes {  // estimated task times of the list scheduler (us)
  // round 5, after the worker fix: the measured medians (TRSM 5.7, UPDATE 4.1, UPDATE4 12.3 us) and a simulated chain
  // period potrf + trsm + 0.75 upd = 14 us.  Same-box A/Bs (profiles/r05/ab_sched, ab_sched2): the former 10 / 6 /
  // 5.5 / 16 1.083 ms, 7 / 5 / 4 / 12.5 1.064 ms, 6 / 5 / 4 / 12.5 1.048 ms; the order is sensitive to the ratio of the
  // simulated chain period to UPDATE4 (1.36: 1.094 ms, 1.04: 1.085 ms)
  double potrf = 6.0, trsm = 5.0, upd = 4.0, upd4 = 12.5;
};
static std::vector<unsigned> build_chol_schedule(int nb, int workers, int group, int singles, int near = 0,
                                                 double boost = 0.0, int band = 0, bool eager = true,
                                                 SchedTimes st = SchedTimes()) {
  struct Task {
    int type, i, j, k, cnt;
    double dur, bl, avail;
    int npred;
  };
  std::vector<Task> T;
  std::vector<int> potrf_id(nb), trsm_id((size_t)nb * nb, -1);
  std::vector<int> upd_base((size_t)nb * (nb + 1) / 2);
  auto tri = [](int i, int j) { return i * (i + 1) / 2 + j; };
  std::vector<int> upd_id;  // per tile (i,j) and panel k < j: the id of the update task that covers k
  {
    size_t tot = 0;
    for (int i = 0; i < nb; ++i)
      for (int j = 0; j <= i; ++j) {
        upd_base[tri(i, j)] = (int)tot;
        tot += j;
      }
    upd_id.assign(tot, -1);
  }
  // Estimated task times (us).  POTRF stands for the chain period minus the simulated TRSM + UPDATE of the chain
  // (measured ~22 us per block), UPDATE4 for its measured ~14 us plus the contention of a full chip.  With the
  // former 18 / 10 the simulated chain ran slower and the workers faster than on the device, so the emitted order
  // put TRSM(k+2, k) -- which the chain needs next -- behind trailing updates: 1.77 -> 1.57 ms per factorization.
  const double d_potrf = st.potrf, d_trsm = st.trsm, d_upd = st.upd, d_upd4 = st.upd4;
  for (int k = 0; k < nb; ++k) {  // (k, type) order is a topological order
    potrf_id[k] = (int)T.size();
    T.push_back({0, k, k, k, 1, d_potrf, 0, 0, k > 0 ? 1 : 0});
    for (int i = k + 1; i < nb; ++i) {
      trsm_id[(size_t)i * nb + k] = (int)T.size();
      T.push_back({1, i, k, k, 1, d_trsm, 0, 0, 1 + (k > 0 ? 1 : 0)});
    }
    for (int j = k + 1; j < nb; ++j)
      for (int i = j; i < nb; ++i) {
        const bool band = i - j < near;  // near-diagonal tiles: single updates (each panel as soon as it is done)
        // the group covering panel k: aligned four, else single
        int gs = k, cnt = 1;
        if (group && !band && (k & ~3) + 4 <= j - singles) {
          gs = k & ~3;
          cnt = 4;
        }
        if (gs != k) continue;  // covered by the group starting at gs
        const int id = (int)T.size();
        for (int kk = k; kk < k + cnt; ++kk) upd_id[upd_base[tri(i, j)] + kk] = id;
        const int npanel = (i == j) ? cnt : 2 * cnt;
        T.push_back({cnt == 4 ? 3 : 2, i, j, k, cnt, (cnt == 4 ? d_upd4 : d_upd) * (i == j ? 0.75 : 1.0), 0, 0,
                     npanel + (k > 0 ? 1 : 0)});
      }
  }
  auto succ = [&](int t, std::vector<int>& out) {
    out.clear();
    const Task& x = T[t];
    if (x.type == 0) {
      for (int i = x.k + 1; i < nb; ++i) out.push_back(trsm_id[(size_t)i * nb + x.k]);
    } else if (x.type == 1) {  // panel k of row i feeds tiles (i, j), k < j <= i, and (r, i), r > i
      const int i = x.i, k = x.k;
      for (int j = k + 1; j <= i; ++j) out.push_back(upd_id[upd_base[tri(i, j)] + k]);
      for (int r = i + 1; r < nb; ++r) out.push_back(upd_id[upd_base[tri(r, i)] + k]);
    } else {
      const int i = x.i, j = x.j, k1 = x.k + x.cnt;
      if (k1 < j) out.push_back(upd_id[upd_base[tri(i, j)] + k1]);
      else if (i == j) out.push_back(potrf_id[j]);
      else out.push_back(trsm_id[(size_t)i * nb + j]);
    }
  };
  std::vector<int> sv;
  for (int t = (int)T.size() - 1; t >= 0; --t) {
    succ(t, sv);
    double m = 0.0;
    for (int s : sv) m = std::max(m, T[s].bl);
    T[t].bl = T[t].dur + m;
    // priority bonus for the work the critical chain waits on: updates of near-diagonal tiles and the TRSMs
    // of the next block rows (their results feed TRSM(k+1, k) and UPDATE(k+1, k+1, k))
    const Task& x = T[t];
    if (boost > 0.0 && ((x.type >= 2 && x.i - x.j < band) || (x.type == 1 && x.i - x.k <= band))) T[t].bl += boost;
  }
  // list scheduling
  typedef std::pair<double, int> DI;
  std::priority_queue<DI, std::vector<DI>, std::greater<DI>> pending, wfree;  // by avail time / free time
  std::priority_queue<DI> ready;                                               // by bottom level
  for (int w = 0; w < workers; ++w) wfree.push({0.0, w});
  pending.push({0.0, potrf_id[0]});
  std::vector<unsigned> order;
  order.reserve(T.size());
  auto code = [](const Task& x) {  // task word: type 1 TRSM, 2 UPDATE, 3 UPDATE4 (POTRF is never listed)
    return ((unsigned)(x.type & 3) << 30) | ((unsigned)x.k << 20) | ((unsigned)x.i << 10) | (unsigned)x.j;
  };
  // the chain workgroups also apply panel b-2 to block row b (UPDATE(k+2,k+2,k), UPDATE(k+2,k+1,k); always
  // single-panel tasks: the groups of four end two panels before the diagonal)
  auto is_chain = [](const Task& x) {
    return x.type == 0 || (x.type == 1 && x.i == x.k + 1) || (x.type == 2 && x.i == x.j && x.j == x.k + 1) ||
           (x.type == 2 && x.i == x.k + 2 && (x.j == x.i || x.j == x.i - 1));
  };
  // the worker tasks the chain's staging of block k+2 waits on -- TRSM(k+2,k), UPDATE(k+2,k+1,k), UPDATE(k+2,k+2,k)
  // -- are emitted as soon as their last dependency is (not at their simulated start), so a worker claims them early
  // and starts the moment their inputs land, instead of when the queue reaches them behind trailing updates.  The
  // order stays topological: every dependency is emitted (or a chain task) before them.
  auto is_eager = [](const Task& x) {
    return (x.type == 1 && x.i == x.k + 2) || (x.type == 2 && x.i == x.k + 2 && (x.j == x.i || x.j == x.i - 1));
  };
  std::vector<char> emitted(T.size(), 0);
  size_t nsched = 0;
  while (nsched < T.size()) {
    DI wk = wfree.top();
    wfree.pop();
    double now = wk.first;
    while (!pending.empty() && pending.top().first <= now) {
      ready.push({T[pending.top().second].bl, pending.top().second});
      pending.pop();
    }
    if (ready.empty()) {
      now = pending.top().first;
      while (!pending.empty() && pending.top().first <= now) {
        ready.push({T[pending.top().second].bl, pending.top().second});
        pending.pop();
      }
    }
    const int t = ready.top().second;
    ready.pop();
    const Task& x = T[t];
    now = std::max(now, x.avail);  // a task moved to `ready` by a later worker is not available earlier
    if (!is_chain(x) && !emitted[t]) order.push_back(code(x));
    ++nsched;
    const double fin = now + x.dur;
    wfree.push({fin, wk.second});
    succ(t, sv);
    for (int s : sv) {
      T[s].avail = std::max(T[s].avail, fin);
      if (--T[s].npred == 0) {
        pending.push({T[s].avail, s});
        if (eager && is_eager(T[s]) && !is_chain(T[s])) {
          order.push_back(code(T[s]));
          emitted[s] = 1;
        }
      }
    }
  }
  return order;
}

// The production schedule: four-panel update groups (the last two panels of a tile single) and a priority boost
// of 100 us for the near-diagonal updates and next-row TRSMs the chain waits on (band 3).  A/B at C3 (boost 0 /
// band 2 -> 100 / 3): Cholesky 1.553, 1.552, 1.556 -> 1.498, 1.529, 1.502 ms.
// (singles >= 2: the chain's own panel b-2 tasks must stay single-panel.  Eight-panel groups and other estimates were
// measured in round 5 and not kept: DESIGN.md §7.)
static std::vector<unsigned> chol_schedule(int nblk, int workers) {
  return build_chol_schedule(nblk, workers, 1, 2, 0, 100.0, 3, true, SchedTimes());
}

extern "C" int cvxg_set_ruiz_lookahead(cvxg_ctx* ctx, int sweeps, long long* relaunches) {
  if (!ctx) return CVXG_E_ARG;
  if (relaunches) *relaunches = ctx->ruiz_relaunches;
  if (sweeps > 0) ctx->ruiz_launch = std::min(RUIZ_MAX, sweeps);
  return CVXG_OK;
}

constexpr int RUIZ_LOOP_MAX_BLOCKS = 16;  // the one-launch Ruiz loop is the default up to this many 64-row blocks

// The one-launch Ruiz loop's buffers (and, with CVXG_RUIZ_TRACE, its stamp buffer for every CU), on first use.
static int ruiz_loop_alloc(cvxg_ctx* ctx) {
  if (!ctx->ruiz_S) {
    CHK(dalloc(ctx, &ctx->ruiz_S, ruiz_loop_doubles(ctx->nblk)));
    CHK(dalloc(ctx, &ctx->ruiz_work, ruiz_loop_work_ints(ctx->nblk)));
  }
  if (!ctx->ruiz_trace_path.empty() && !ctx->ruiz_trace)
    CHK(dalloc(ctx, &ctx->ruiz_trace, (size_t)std::max(ctx->ncu, 1) * RUIZ_MAX * 4));
  return CVXG_OK;
}

extern "C" int cvxg_set_option(cvxg_ctx* ctx, int option, long long value) {
  if (!ctx) return CVXG_E_ARG;
  const bool bin = value == 0 || value == 1;
  switch (option) {
    case CVXG_OPT_SPARSE_ROWS:
      if (!bin) break;
      if (ctx->have_ineq) return set_err(ctx, CVXG_E_ARG, "CVXG_OPT_SPARSE_ROWS must be set before cvxg_set_ineq");
      ctx->sparse_rows = (int)value;
      return CVXG_OK;
    case CVXG_OPT_EARLY_ABORT:
      if (!bin) break;
      ctx->early_abort = (int)value;
      return CVXG_OK;
    case CVXG_OPT_H_LOWER:
      if (!bin) break;
      ctx->h_lower = (int)value;
      ctx->h_valid = false;  // (a prefetched assembly in the other form is not reused)
      return CVXG_OK;
    case CVXG_OPT_KKT_FUSED_RHS:
      if (value < 1 || value > MAX_RHS) break;
      ctx->kkt_fused_rhs = (int)value;
      return CVXG_OK;
    case CVXG_OPT_SPEC_REG:
      if (!bin) break;
      ctx->spec_reg = (int)value;
      return CVXG_OK;
    case CVXG_OPT_RUIZ_LOOP:
      if (!bin) break;
      if (value && !ruiz_loop_fits(ctx->nblk))
        return set_err(ctx, CVXG_E_UNSUPPORTED, "the one-launch Ruiz loop holds at most its register batch of tiles");
      if (value) CHK(ruiz_loop_alloc(ctx));
      ctx->ruiz_loop = (int)value;
      return CVXG_OK;
    case CVXG_OPT_RUIZ_WG:
      if (value < 0 || value > ctx->ncu) break;
      ctx->ruiz_wg = (int)value;
      return CVXG_OK;
    default:
      return set_err(ctx, CVXG_E_ARG, "cvxg_set_option: unknown option %d", option);
  }
  return set_err(ctx, CVXG_E_ARG, "cvxg_set_option: value %lld out of range for option %d", value, option);
}

extern "C" int cvxg_chol_schedule(int nblk, int workers, unsigned* order, int cap) {
  if (nblk < 1 || nblk > 1023 || workers < 1 || cap < 0 || (cap > 0 && !order)) return CVXG_E_ARG;
  const std::vector<unsigned> o = chol_schedule(nblk, workers);
  for (size_t t = 0; t < o.size() && (int)t < cap; ++t) order[t] = o[t];
  return (int)o.size();
}

// ------------------------------------------------------------------------------------------------
// Device pipeline pieces
// ------------------------------------------------------------------------------------------------

// objF.valueAt(x) from the reduced scalars: r + a.x (+ x'Px/2) (QuadraticObjectiveFunction.scala:31), or the
// KL dual  w.z + R.exp(-B'z)  (Dist_KL.scala:146-147 negated by Duality.scala:76)
static double objective_from_ctrl(const cvxg_ctx* ctx, const DevCtrl& h) {
  if (ctx->kl) return h.sc[SC_A0X] + h.sc[SC_KLSUM];
  if (ctx->klp) return h.sc[SC_KLP];  // x dot log(x*n)  (Dist_KL.scala:226)
  return ctx->r0 + h.sc[SC_A0X] + (ctx->hasP ? h.sc[SC_XPX] / 2 : 0.0);
}

// c = g(x), d, 1/d, 1/d^2, log d at ctx->x; QuadraticConstraint rows add x'P_k x / 2 (P_k x kept in qPx for the
// gradient, the Hessian rows and the line search).
// Certified line-search decisions (line_search): every configuration with inequality constraints -- linear and
// QuadraticConstraint rows, quadratic / linear / KL objectives.
static bool ls_certified(const cvxg_ctx* ctx) { return ctx->m > 0; }

static void constraint_eval_all(cvxg_ctx* ctx) {
  const int np = ctx->np;
  const bool cert = ls_certified(ctx);
  if (ctx->nq > 0) {
    if (cert) launch_rowdot_abs(ctx->s, ctx->Pq, np, ctx->nq * np, np, ctx->x, ctx->qPx, ctx->qPxa);
    else launch_rowdot(ctx->s, ctx->Pq, np, ctx->nq * np, np, ctx->x, ctx->qPx);
    launch_quad_xpx(ctx->s, ctx->qPx, ctx->x, ctx->qrows, ctx->nq, np, ctx->qextra);
  }
  launch_constraint_eval(ctx->s, ctx->A, np, ctx->mp, np, ctx->x, ctx->r, ctx->ub, ctx->c, ctx->d, ctx->invd, ctx->w,
                         ctx->logd, ctx->ctrl, ctx->nq > 0 ? ctx->qextra : nullptr, cert ? ctx->cabs : nullptr);
  if (cert && ctx->nq > 0)  // + |x|'|P_k||x| / 2 on the quadratic rows
    launch_quad_absdot(ctx->s, ctx->qPxa, ctx->x, ctx->qrows, ctx->nq, np, 0.5, 1, ctx->cabs);
}

// Barrier value / gradient pieces at the current x and ctrl->t (BarrierSolver.scala:280-301):
// c, d, w, invd, logd, Px, y, eqDiff, and sc[A0X, XPX, SUMLOG, GG, EQ2].
static int assemble_hessian(cvxg_ctx* ctx, const double* wts, const double* qw, hipStream_t st, bool full);
constexpr int ROWDOT_BESIDE_WG = 64;
// the Newton step's assembly: lower-only when nothing but Ruiz, the Cholesky and the symv residual reads H
static bool step_h_full(const cvxg_ctx* ctx) { return !(ctx->p == 0 && ctx->h_lower); }
// The setup sweep of a speculative line search also evaluates the constraints at x + dx (k_ls_setup_eval): linear
// rows, certified line search.
static bool spec_eval_ok(const cvxg_ctx* ctx) {
  return ls_certified(ctx) && ctx->nq == 0 && !ctx->kl && !ctx->klp && ctx->p == 0;
}
// taken: the line search accepted the speculated t along s = dx, and the speculative evaluation at x1 = x + dx t
// (bitwise the x + s t of the step) is the constraint evaluation at the new x
// ahead: the prefetched assembly belongs to the next step (the end-of-step prefetch, timed in ring slot tick + 1) or
// to this one (a step that starts without an evaluation, slot tick)
static int eval_at_x(cvxg_ctx* ctx, bool prefetch = false, bool taken = false, bool ahead = true) {
  hipStream_t s = ctx->s;
  const int np = ctx->np, mp = ctx->mp;
  if (taken) {
    std::swap(ctx->c, ctx->c1);
    std::swap(ctx->d, ctx->d1);
    std::swap(ctx->invd, ctx->invd1);
    std::swap(ctx->w, ctx->w1);
    std::swap(ctx->logd, ctx->logd1);
    std::swap(ctx->cabs, ctx->cabs1);
    // (the evaluation's counters are taken over on the stream that publishes them; with the prefetch that is s2)
    if (!prefetch || ctx->kl || ctx->klp) launch_ctrl_take_spec(s, ctx->ctrl);
  } else {
    launch_ctrl_reset_eval(s, ctx->ctrl);
    constraint_eval_all(ctx);
  }
  ctx->h_valid = false;
  prefetch = prefetch && !ctx->kl && !ctx->klp;  // (their Hessians need the evaluation's y / diag(1/x) first)
  if (prefetch) {  // the assembly needs w (and the quadratic rows' P_k x) only: it stays on the main stream, and the
                   // rest of the evaluation moves to s2 behind the constraint values
    // Taken: x (= x1, swapped in by the caller) and the constraint values were final before the line search's host
    // read, so s2 needs no wait on the main stream (one event marker less in front of the assembly)
    if (!taken) HIPC(ctx, hipEventRecord(ctx->ev_w, s));
    const int nx = (ctx->tm.tick + (ahead ? 1 : 0)) % TRING;  // timed as phase 5 of the step that will use it
    if (ctx->tm.on) HIPC(ctx, hipEventRecord(ctx->tm.ev[nx][5][0], s));
    CHK(assemble_hessian(ctx, nullptr, nullptr, s, step_h_full(ctx)));
    if (ctx->tm.on) {
      HIPC(ctx, hipEventRecord(ctx->tm.ev[nx][5][1], s));
      ctx->tm.rec[nx][5] = true;
      if (ahead) ctx->tm.pf5 = true;
    }
    // the second stream's wait is issued after the assembly's launches: the GPU is idle until they are (the host's
    // hipStreamWaitEvent costs ~8 us, microbench/hostcost.hip)
    if (!taken) HIPC(ctx, hipStreamWaitEvent(ctx->s2, ctx->ev_w, 0));
    s = ctx->s2;
    if (taken) launch_ctrl_take_spec(s, ctx->ctrl);
  }
  const bool quad = ctx->hasP && !ctx->kl;
  const bool cert = ls_certified(ctx);
  if (quad) {
    // beside the prefetched assembly (s2) on a bounded grid: 64 workgroups loop over the rows instead of 512 queueing
    // for the SYRK's CU slots (the same sums, bitwise)
    if (cert) launch_rowdot_abs(s, ctx->P, np, np, np, ctx->x, ctx->Px, ctx->Pxa, prefetch ? ROWDOT_BESIDE_WG : 0);
    else launch_rowdot(s, ctx->P, np, np, np, ctx->x, ctx->Px);
  }
  if (ctx->kl) {  // v = B'z, y = R exp(-v), -B y (the KL dual gradient is w - B y), sum_j y_j
    if (cert) launch_rowdot_abs(s, ctx->KB, np, ctx->noutp, np, ctx->x, ctx->kl_v, ctx->kl_vabs);
    else launch_rowdot(s, ctx->KB, np, ctx->noutp, np, ctx->x, ctx->kl_v);
    launch_kl_eval(s, ctx->kl_v, ctx->nout, ctx->noutp, ctx->kl_R, ctx->kl_y);
    launch_coldot_partials(s, ctx->KB, np, ctx->noutp, np, ctx->kl_y, ctx->kl_part);
    launch_sum_chunks(s, ctx->kl_part, coldot_chunks(ctx->noutp), np, ctx->kl_negBy);
    launch_axpy(s, ctx->kl_negBy, ctx->kl_negBy, -2.0, np, ctx->kl_negBy);  // -B y
    launch_sum(s, ctx->kl_y, ctx->noutp, ctx->ctrl, SC_KLSUM);
  }
  if (ctx->klp)  // log(n x), the gradient (1 + log x) + log n, diag(1/x) and the value terms' error scale
    launch_klp_eval(s, ctx->x, ctx->n, np, ctx->klp_n, ctx->klp_lx, ctx->klp_g0, ctx->klp_hd, ctx->klp_ab);
  launch_coldot_partials(s, ctx->A, np, mp, np, ctx->invd, ctx->part);
  // objF.gradientAt(x) * t: (a + P x) t, the KL dual's (w - B y) t, or the KL primal's (0 + g0) t = g0 t (a0 = 0)
  launch_gradient_finalize(s, ctx->a0, quad ? ctx->Px : (ctx->kl ? ctx->kl_negBy : (ctx->klp ? ctx->klp_g0 : nullptr)),
                           ctx->part, coldot_chunks(mp), np, ctx->ctrl, ctx->y);
  if (ctx->nq > 0) launch_quad_grad(s, ctx->qPx, ctx->invd, ctx->qrows, ctx->nq, np, ctx->y);  // + (P_k x)/d_k
  DotBatch db{};
  db.add(DOT_FMA, ctx->a0, ctx->x, np, SC_A0X);
  if (quad) db.add(DOT_FMA, ctx->x, ctx->Px, np, SC_XPX);
  if (ctx->klp) db.add(DOT_FMA, ctx->x, ctx->klp_lx, np, SC_KLP);
  db.add(DOT_SUM, ctx->logd, nullptr, mp, SC_SUMLOG);
  db.add(DOT_FMA, ctx->y, nullptr, np, SC_GG);
  if (cert) {  // error scales of f(x): |a0|.|x|, |x|.|P||x| (or the KL primal terms), sum cabs/d, sum |log d|
    if (db.full()) {
      launch_dots(s, db, ctx->ctrl);
      db.count = 0;
    }
    db.add(DOT_ABS, ctx->a0, ctx->x, np, SC_A0XA);
    if (quad) db.add(DOT_ABS, ctx->x, ctx->Pxa, np, SC_XPXA);
    if (ctx->klp) db.add(DOT_SUM, ctx->klp_ab, nullptr, np, SC_KLPA);
    if (ctx->kl) db.add(DOT_ABS, ctx->kl_y, ctx->kl_vabs, ctx->noutp, SC_KLA);
    db.add(DOT_ABS, ctx->cabs, ctx->invd, mp, SC_CAINV);
    db.add(DOT_ABS, ctx->logd, nullptr, mp, SC_LOGABS);
  }
  launch_dots(s, db, ctx->ctrl);
  if (ctx->p > 0) {
    launch_rowdot(s, ctx->Aeq, np, ctx->p, np, ctx->x, ctx->eqtmp);
    launch_axpy(s, ctx->beq, ctx->eqtmp, -1.0, ctx->p, ctx->eqd);  // b - A*x
    launch_dot(s, ctx->eqd, nullptr, ctx->p, ctx->ctrl, SC_EQ2);
  }
  HIPC(ctx, hipGetLastError());
  if (prefetch) HIPC(ctx, hipEventRecord(ctx->ev_h, s));  // the end of the evaluation's tail (before its publish)
  const int rc_sync = host_read(ctx, ctx->ctrl, ctx->hctrl_dev, sizeof(DevCtrl), nullptr, nullptr, 0, s);
  if (prefetch) {
    // the main stream (with the assembly) waits on the evaluation's tail only if it has not finished -- the host read
    // above has just seen it finish, so normally there is no cross-queue wait (a barrier packet costs 15-25 us on the
    // main stream, profiles/r03 timeline)
    hipError_t q = hipEventQuery(ctx->ev_h);
    for (int spins = 0; q == hipErrorNotReady && spins < 4096; ++spins) {
      __builtin_ia32_pause();
      q = hipEventQuery(ctx->ev_h);
    }
    if (q != hipSuccess) HIPC(ctx, hipStreamWaitEvent(ctx->s, ctx->ev_h, 0));
    ctx->h_valid = rc_sync == CVXG_OK;
  }
  CHK(rc_sync);
  const DevCtrl& h = *ctx->hctrl;
  const double f0 = objective_from_ctrl(ctx, h);
  ctx->f_at_x = ctx->t * f0 - h.sc[SC_SUMLOG];
  ctx->normGrad = sqrt(h.sc[SC_GG]);
  ctx->eqGap = ctx->p > 0 ? sqrt(h.sc[SC_EQ2]) : 0.0;
  ctx->x_eval_valid = 1;
  if (h.infeasible > 0)
    return set_err(ctx, CVXG_E_INFEASIBLE_X, "barrier: x not strictly feasible (%d constraints with d <= 0)",
                   h.infeasible);
  return CVXG_OK;
}

static double objective_at_x(cvxg_ctx* ctx) { return objective_from_ctrl(ctx, *ctx->hctrl); }

// H = t P + A' diag(wts) A (+ the sparse rows' entries) + sum_k qw_k P_k over the QuadraticConstraint rows; wts =
// ctx->w = 1/d^2 and qw = 1/d for the barrier Hessian (BarrierSolver.scala:314), or the primal-dual KKT weights
// lambda/d and qw = lambda (kktMatrix_noEqs, PrimalDualSolver.scala:226-238; then ctrl->t = 1).
static int assemble_hessian(cvxg_ctx* ctx, const double* wts = nullptr, const double* qw = nullptr,
                            hipStream_t st = nullptr, bool full = true) {
  const bool own = st == nullptr;  // on ctx->s (timed here as phase 5); otherwise the prefetch on s2 (timed there)
  if (own) st = ctx->s;
  if (own) tstart(ctx, 5);
  const double* wsrc = wts ? wts : ctx->w;
  // full tiles in whole waves of workgroup slots, then the leftover tiles split along K across all slots
  // (partials + ordered reduce) so the last wave is not a handful of tiles on an otherwise idle chip.
  const double* P = ctx->hasP ? ctx->P : nullptr;
  if (ctx->kl) {  // objF.hessianAt(z) = B diag(y) B' (Dist_KL.scala:158-165) into P: a weighted SYRK over the outcomes
    if (ctx->ntiles_main > 0)
      launch_syrk_assemble(st, ctx->KB, ctx->np, ctx->kl_y, ctx->noutp, nullptr, ctx->ctrl, ctx->P, ctx->np,
                           TileList{ctx->tiles, ctx->ntiles_main}, 1, ctx->part);
    if (ctx->ntiles > ctx->ntiles_main)  // the tail (all tiles for a small dual) split along the outcomes
      launch_syrk_assemble(st, ctx->KB, ctx->np, ctx->kl_y, ctx->noutp, nullptr, ctx->ctrl, ctx->P, ctx->np,
                           TileList{ctx->tiles + ctx->ntiles_main, ctx->ntiles - ctx->ntiles_main}, ctx->kl_nsplit,
                           ctx->kl_spart);
  }
  const double* A = ctx->A;
  const double* w = wsrc;
  int rows = ctx->mp;
  if (ctx->have_sparse) {  // dense rows only; the sparse rows' entries are added below
    if (ctx->nq > 0)  // gradient rows G_k = a_k + P_k x of the quadratic constraints
      launch_quad_rows(st, ctx->A, ctx->qPx, ctx->qrows, ctx->qslot, ctx->nq, ctx->np, ctx->As);
    launch_gather_w(st, wsrc, ctx->didx, ctx->ndense, ctx->mdp, ctx->wd);
    A = ctx->As;
    w = ctx->wd;
    rows = ctx->mdp;
  }
  const double* Pd = ctx->klp ? ctx->klp_hd : nullptr;  // the KL primal's diag(1/x) * t
  if (ctx->ntiles_main > 0)
    launch_syrk_assemble(st, A, ctx->np, w, rows, P, ctx->ctrl, ctx->H, ctx->np,
                         TileList{ctx->tiles, ctx->ntiles_main}, 1, ctx->spart, Pd, full);
  if (ctx->ntiles > ctx->ntiles_main)
    launch_syrk_assemble(st, A, ctx->np, w, rows, P, ctx->ctrl, ctx->H, ctx->np,
                         TileList{ctx->tiles + ctx->ntiles_main, ctx->ntiles - ctx->ntiles_main}, ctx->nsplit,
                         ctx->spart, Pd, full);
  ctx->h_full = full;
  if (ctx->have_sparse)
    launch_sparse_hess(st, ctx->sp_ptr, ctx->sp_pq, ctx->sp_row, ctx->sp_coef, wsrc, ctx->sp_T, ctx->H, ctx->np);
  if (ctx->nq > 0)  // + hessianAt/d = P_k / d_k  (BarrierSolver.scala:314), or grad2_gi * l_i (PrimalDualSolver.scala:236)
    launch_quad_hess(st, ctx->Pq, qw ? qw : ctx->invd, ctx->qrows, ctx->nq, ctx->np, ctx->H);
  if (own) tstop(ctx, 5);
  HIPC(ctx, hipGetLastError());
  return CVXG_OK;
}

// Ruiz equilibration of H into dfin (MatrixUtils.scala:240-268): sweeps k0 .. k1-1 (k0 = 0 starts from d = 1).
// A sweep whose rho[k] <= 1e-6 exits at once, so launching all RUIZ_MAX sweeps is the reference's loop; the
// final pass records the sweep count, or -1 when sweeps were left unlaunched and rho[k1] still exceeds 1e-6.
static void ruiz_sweeps(cvxg_ctx* ctx, int k0, int k1) {
  hipStream_t s = ctx->s;
  if (ctx->ruiz_loop) {  // the whole loop in one launch: k0 = 0, k1 = RUIZ_MAX always
    const int nwg = ctx->ruiz_wg > 0 ? ctx->ruiz_wg : ctx->ncu;
    launch_ruiz_loop(s, ctx->H, ctx->np, ctx->n, ctx->np, ctx->ruiz_S, ctx->ruiz_work, ctx->dfin, ctx->ctrl, nwg,
                     ++ctx->ruiz_gen, ctx->ruiz_trace);
    if (ctx->ruiz_trace) {  // instrumentation only
      std::vector<unsigned long long> tr((size_t)nwg * RUIZ_MAX * 4);
      if (copy_sync(ctx, tr.data(), ctx->ruiz_trace, tr.size() * 8, hipMemcpyDeviceToHost) == CVXG_OK)
        if (FILE* f = fopen(ctx->ruiz_trace_path.c_str(), "wb")) {
          fwrite(&nwg, 4, 1, f);
          fwrite(tr.data(), 8, tr.size(), f);
          fclose(f);
        }
    }
    return;
  }
  if (k0 == 0) launch_ruiz_init(s, ctx->ruiz0, ctx->np, ctx->ctrl);
  // (one launch per sweep, each forming the previous sweep's d from its partials, was measured in round 6: 0.463 vs
  // 0.235 ms per Ruiz at C3 -- the partials re-read per tile cost more than the row-pass launch it saves)
  for (int k = k0; k < k1; ++k) {
    const double* dc = (k & 1) ? ctx->ruiz1 : ctx->ruiz0;
    double* dn = (k & 1) ? ctx->ruiz0 : ctx->ruiz1;
    launch_ruiz_sweep_tri(s, ctx->H, ctx->np, ctx->n, ctx->np, dc, dn, ctx->part, ctx->ctrl, k);
  }
  launch_ruiz_final(s, ctx->ruiz0, ctx->ruiz1, ctx->np, ctx->dfin, ctx->ctrl, k1);
}
static void ruiz(cvxg_ctx* ctx) {
  ctx->ruiz_pending = false;
  ruiz_sweeps(ctx, 0, RUIZ_MAX);
}
// The Newton step's Ruiz launches only the sweeps the previous step needed plus RUIZ_MARGIN (a sweep that exits on
// rho <= 1e-6 still costs a launch pair, ~9 us), reads the control block, and launches RUIZ_CHUNK more at a time
// while the loop is not done.  The sweeps that run, dfin and the sweep count are those of the full loop; a short
// lookahead costs one more host round trip.
constexpr int RUIZ_MARGIN = 1, RUIZ_CHUNK = 2;
// The sweeps go out without a host read: the factorization attempt behind them is gated on the device (a launch that
// finds the loop still open leaves at once), and its one host read tells whether the loop was done (factor_attempt).
static int ruiz_lookahead(cvxg_ctx* ctx) {
  if (ctx->ruiz_loop) {  // (the one-launch loop runs to its end on the device: nothing to look ahead of)
    ruiz(ctx);
    HIPC(ctx, hipGetLastError());
    return CVXG_OK;
  }
  ctx->ruiz_k1 = ctx->ruiz_launch;
  ruiz_sweeps(ctx, 0, ctx->ruiz_k1);
  HIPC(ctx, hipGetLastError());
  ctx->ruiz_pending = true;
  return CVXG_OK;
}
// A short lookahead: RUIZ_CHUNK more sweeps at a time, each batch followed by a host read, until the loop is done.
static int ruiz_finish(cvxg_ctx* ctx) {
  while (ctx->hctrl->ruiz_sweeps < 0) {
    ++ctx->ruiz_relaunches;
    const int k2 = std::min(RUIZ_MAX, ctx->ruiz_k1 + RUIZ_CHUNK);
    ruiz_sweeps(ctx, ctx->ruiz_k1, k2);
    ctx->ruiz_k1 = k2;
    HIPC(ctx, hipGetLastError());
    CHK(sync_ctrl(ctx));
  }
  return CVXG_OK;
}
static void ruiz_learn(cvxg_ctx* ctx, int sweeps) {
  ctx->ruiz_launch = std::max(1, std::min(RUIZ_MAX, sweeps + RUIZ_MARGIN));
}

// The device-side failures an attempt's host read can carry (both forms of regularizedCholesky check them): a timed-out
// dependency wait of the dataflow Cholesky, or of the one-launch Ruiz loop it is gated on (ruiz_sweeps == -2; the
// factorization and the backward solve then left at once, so dx is stale).
static int attempt_status(cvxg_ctx* ctx) {
  if (ctx->hctrl->df_status != 0)
    return set_err(ctx, CVXG_E_HIP, "dataflow Cholesky: dependency wait timed out (status %d)", ctx->hctrl->df_status);
  if (ctx->hctrl->ruiz_sweeps == -2)
    return set_err(ctx, CVXG_E_HIP, "Ruiz loop: dependency wait timed out (abort word 0x%x)", ctx->hctrl->ruiz_abort);
  return CVXG_OK;
}

// One factorisation attempt of Q = DHD (+reg I) with the fused forward solve of nrhs right-hand sides,
// which `fill_rhs` writes into ctx->rhs first.  `after` enqueues the work that consumes the factor (the back
// substitution) before the one host read of the attempt, which returns chol_info / min_diag via hctrl; a caller
// discards that work when the attempt fails.
template <class F, class G>
static int factor_attempt(cvxg_ctx* ctx, double reg, int nrhs, F fill_rhs, G after) {
  hipStream_t s = ctx->s;
  ++ctx->n_attempts;
  launch_factor_prep(s, ctx->ctrl, reg, ctx->df_work, chol_dataflow_work_ints(ctx->nblk));  // reg, chol fields, work
  fill_rhs();
  // the whole factorization as one persistent launch over the 64 x 64 tile DAG (k_dataflow.hip); Q = (d d') o H
  // (+ reg I) is formed as each tile is first read (no separate k_form_q pass)
  // the first attempt (reg = 0) stops at the first block with min diag(L) <= 1e-7: its factor would be discarded
  // anyway (MatrixUtils.scala:458-460 refactors Q + 1e-10 I), so only the retry's L is ever used
  if (ctx->df_trace)  // (instrumentation: marks a launch does not reach read 0, not a previous launch's value)
    (void)hipMemsetAsync(ctx->df_trace, 0, (size_t)4 * (ctx->df_ntasks + 5 * ctx->nblk) * 8, s);
  launch_chol_dataflow(s, ctx->L, ctx->np, ctx->rhs, nrhs, ctx->Linv, ctx->ctrl, ctx->df_work, ctx->nblk, ctx->df_tasks,
                       ctx->df_ntasks, ctx->ncu, ctx->df_trace, false, ctx->H, ctx->dfin, ctx->n, ctx->ruiz_pending,
                       (reg == 0.0 && ctx->early_abort) ? 1e-7 : 0.0);
  ctx->spec_launched = false;
  after();
  HIPC(ctx, hipGetLastError());
  if (ctx->spec_launched) {  // the control block and the speculative line-search batch in one host read
    CHK(host_read(ctx, ctx->ctrl, ctx->hctrl_dev, sizeof(DevCtrl), ctx->ls_log, ctx->hls_dev,
                  5 * LS_TRIALS * sizeof(double)));
  } else {
    CHK(sync_ctrl(ctx));
  }
  if (ctx->ruiz_pending) {
    ctx->ruiz_pending = false;
    if (ctx->hctrl->ruiz_sweeps < 0) {  // the Ruiz loop was still open: this attempt was void (nothing factored)
      ctx->spec_launched = ctx->spec_eval_launched = false;
      CHK(ruiz_finish(ctx));
      tstart(ctx, 2);  // (phase 2 times the factorization that counts)
      return factor_attempt(ctx, reg, nrhs, fill_rhs, after);
    }
  }
  ctx->spec_have = ctx->spec_launched;
  ctx->spec_eval_have = ctx->spec_launched && ctx->spec_eval_launched;
  ctx->spec_launched = false;
  ctx->spec_eval_launched = false;
  CHK(attempt_status(ctx));
  if (ctx->df_trace) {  // instrumentation only: task order + timeline of this factorization
    std::vector<unsigned long long> tr((size_t)4 * (ctx->df_ntasks + 5 * ctx->nblk));
    std::vector<unsigned> ord(ctx->df_ntasks);
    CHK(copy_sync(ctx, tr.data(), ctx->df_trace, tr.size() * 8, hipMemcpyDeviceToHost));
    CHK(copy_sync(ctx, ord.data(), ctx->df_tasks, ord.size() * 4, hipMemcpyDeviceToHost));
    if (FILE* f = fopen(ctx->df_trace_path.c_str(), "wb")) {
      fwrite(&ctx->df_ntasks, 4, 1, f);
      fwrite(&ctx->nblk, 4, 1, f);
      fwrite(ord.data(), 4, ord.size(), f);
      fwrite(tr.data(), 8, tr.size(), f);
      fclose(f);
    }
  }
  return CVXG_OK;
}

static double min_diag_of(const DevCtrl& h) {
  double v;
  memcpy(&v, &h.min_diag, sizeof(v));
  return v;
}

// regularizedCholesky (MatrixUtils.scala:452-461): chol(Q); on failure or min diag(L) <= 1e-7 use
// chol(Q + 1e-10 I), whose failure propagates (CVXG_E_NOT_PD).
template <class F, class G>
static int regularized_cholesky(cvxg_ctx* ctx, int nrhs, F fill_rhs, int* regularized, double* mind, G after) {
  CHK(factor_attempt(ctx, 0.0, nrhs, fill_rhs, after));
  *regularized = 0;
  // where the first attempt stopped: its non-positive pivot, or the block where min diag(L) <= 1e-7 (0: it did not)
  ctx->small_piv = ctx->hctrl->small_piv ? ctx->hctrl->small_piv : ctx->hctrl->chol_info;
  if (ctx->hctrl->chol_info == 0 && min_diag_of(*ctx->hctrl) > 1e-7) {
    *mind = min_diag_of(*ctx->hctrl);
    return CVXG_OK;
  }
  CHK(factor_attempt(ctx, 1e-10, nrhs, fill_rhs, after));
  *regularized = 1;
  *mind = min_diag_of(*ctx->hctrl);
  if (ctx->hctrl->chol_info != 0)
    return set_err(ctx, CVXG_E_NOT_PD, "cholesky: matrix not positive definite (pivot %d)", ctx->hctrl->chol_info);
  return CVXG_OK;
}

static void backward_solve(cvxg_ctx* ctx, int nrhs, BwdEpilogue epi = {}) {
  BwdAlt alt;
  if (ctx->pair_active) alt = BwdAlt{ctx->L2, ctx->Linv2, ctx->rhs2};  // (the device picks by ctrl->spec_sel)
  launch_bwd_dataflow(ctx->s, ctx->L, ctx->np, ctx->Linv, ctx->rhs, ctx->sol, nrhs, ctx->nblk, ctx->bwd_flags,
                      ++ctx->bwd_gen, ctx->ctrl, epi, alt);
}

// The buffers of the speculative pair's second attempt (allocated on first use: 134 MB of L at C3).  All or nothing:
// ctx->L2 is set only once every piece exists, and a failure frees what was made (the caller then runs the sequential
// form, which needs none of it).
static void spec_free(double* L2, double* Linv2, double* rhs2, int* w2, DevCtrl* c2, hipStream_t s3, hipEvent_t e0,
                      hipEvent_t e1) {
  for (void* p : {(void*)L2, (void*)Linv2, (void*)rhs2, (void*)w2, (void*)c2})
    if (p) (void)hipFree(p);
  if (s3) (void)hipStreamDestroy(s3);
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
}
static int spec_alloc(cvxg_ctx* ctx) {
  if (ctx->L2) return CVXG_OK;
  const size_t np = ctx->np;
  double *L2 = nullptr, *Linv2 = nullptr, *rhs2 = nullptr;
  int* w2 = nullptr;
  DevCtrl* c2 = nullptr;
  hipStream_t s3 = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int rc = dalloc(ctx, &L2, np * np);
  if (rc == CVXG_OK) rc = dalloc(ctx, &Linv2, chol_dataflow_linv_doubles(ctx->nblk));
  if (rc == CVXG_OK) rc = dalloc(ctx, &rhs2, np * MAX_RHS);
  if (rc == CVXG_OK) rc = dalloc(ctx, &w2, chol_dataflow_work_ints(ctx->nblk));
  if (rc == CVXG_OK) rc = dalloc(ctx, &c2, 1);
  if (rc == CVXG_OK && hipStreamCreateWithFlags(&s3, hipStreamNonBlocking) != hipSuccess) rc = CVXG_E_HIP;
  if (rc == CVXG_OK && hipEventCreateWithFlags(&e0, hipEventDisableTiming) != hipSuccess) rc = CVXG_E_HIP;
  if (rc == CVXG_OK && hipEventCreateWithFlags(&e1, hipEventDisableTiming) != hipSuccess) rc = CVXG_E_HIP;
  if (rc != CVXG_OK) {
    spec_free(L2, Linv2, rhs2, w2, c2, s3, e0, e1);
    (void)hipGetLastError();  // (an allocation failure is not a sticky error for the sequential form)
    return rc;
  }
  ctx->Linv2 = Linv2;
  ctx->rhs2 = rhs2;
  ctx->df_work2 = w2;
  ctx->ctrl2 = c2;
  ctx->s3 = s3;
  ctx->ev_p0 = e0;
  ctx->ev_p1 = e1;
  ctx->L2 = L2;  // last: the pair's buffers are complete
  return CVXG_OK;
}

// regularizedCholesky (MatrixUtils.scala:452-461) with both attempts in flight together: chol(Q) (stopping at its
// first block with min diag(L) <= 1e-7, as factor_attempt) and chol(Q + 1e-10 I), each a dataflow launch on half of
// the CUs, on two streams.  The device picks the attempt the reference keeps (k_spec_select), the backward solve and
// everything behind it run on that one, and the one host read returns both verdicts.  The factors are bitwise those
// of the sequential form (the same launches, only concurrent).  Used after a regularized direction: late in the path
// the Q + 1e-10 I branch repeats step after step, and its first attempt fails in the last block (C3FULL stop rows
// 4081..4096), so the sequential form pays two whole factorizations.
template <class F, class G>
static int regularized_cholesky_spec(cvxg_ctx* ctx, int nrhs, F fill_rhs, int* regularized, double* mind, G after) {
  hipStream_t s = ctx->s;
  CHK(spec_alloc(ctx));
  ++ctx->spec_pairs;
  ctx->n_attempts += 2;
  launch_factor_prep(s, ctx->ctrl, 0.0, ctx->df_work, chol_dataflow_work_ints(ctx->nblk));
  launch_spec_prep2(s, ctx->ctrl2, ctx->ctrl, 1e-10);
  HIPC(ctx, hipMemsetAsync(ctx->df_work2, 0, chol_dataflow_work_ints(ctx->nblk) * sizeof(int), s));
  fill_rhs();
  HIPC(ctx, hipMemcpyAsync(ctx->rhs2, ctx->rhs, (size_t)ctx->np * nrhs * sizeof(double), hipMemcpyDeviceToDevice, s));
  HIPC(ctx, hipEventRecord(ctx->ev_p0, s));
  HIPC(ctx, hipStreamWaitEvent(ctx->s3, ctx->ev_p0, 0));
  const int half = std::max(3, ctx->ncu / 2);
  launch_chol_dataflow(s, ctx->L, ctx->np, ctx->rhs, nrhs, ctx->Linv, ctx->ctrl, ctx->df_work, ctx->nblk, ctx->df_tasks,
                       ctx->df_ntasks, half, nullptr, false, ctx->H, ctx->dfin, ctx->n, ctx->ruiz_pending,
                       ctx->early_abort ? 1e-7 : 0.0);
  launch_chol_dataflow(ctx->s3, ctx->L2, ctx->np, ctx->rhs2, nrhs, ctx->Linv2, ctx->ctrl2, ctx->df_work2, ctx->nblk,
                       ctx->df_tasks, ctx->df_ntasks, half, nullptr, false, ctx->H, ctx->dfin, ctx->n,
                       ctx->ruiz_pending, 0.0);
  HIPC(ctx, hipEventRecord(ctx->ev_p1, ctx->s3));
  HIPC(ctx, hipStreamWaitEvent(s, ctx->ev_p1, 0));
  launch_spec_select(s, ctx->ctrl, ctx->ctrl2);
  ctx->spec_launched = false;
  ctx->pair_active = true;
  after();
  ctx->pair_active = false;
  HIPC(ctx, hipGetLastError());
  if (ctx->spec_launched) {
    CHK(host_read(ctx, ctx->ctrl, ctx->hctrl_dev, sizeof(DevCtrl), ctx->ls_log, ctx->hls_dev,
                  5 * LS_TRIALS * sizeof(double)));
  } else {
    CHK(sync_ctrl(ctx));
  }
  if (ctx->ruiz_pending) {
    ctx->ruiz_pending = false;
    if (ctx->hctrl->ruiz_sweeps < 0) {  // the Ruiz loop was still open: both attempts were void
      ctx->spec_launched = ctx->spec_eval_launched = false;
      CHK(ruiz_finish(ctx));
      return regularized_cholesky(ctx, nrhs, fill_rhs, regularized, mind, after);
    }
  }
  ctx->spec_have = ctx->spec_launched;
  ctx->spec_eval_have = ctx->spec_launched && ctx->spec_eval_launched;
  ctx->spec_launched = false;
  ctx->spec_eval_launched = false;
  CHK(attempt_status(ctx));
  if (!ctx->hctrl->spec_sel) {
    *regularized = 0;
    ctx->small_piv = 0;
    *mind = min_diag_of(*ctx->hctrl);
    return CVXG_OK;
  }
  ++ctx->spec_pairs_used;
  *regularized = 1;
  ctx->small_piv = ctx->hctrl->small_piv ? ctx->hctrl->small_piv : ctx->hctrl->chol_info;
  double md2;
  memcpy(&md2, &ctx->hctrl->min_diag2, sizeof(md2));
  *mind = md2;
  if (ctx->hctrl->chol_info2 != 0)
    return set_err(ctx, CVXG_E_NOT_PD, "cholesky: matrix not positive definite (pivot %d)", ctx->hctrl->chol_info2);
  return CVXG_OK;
}

static void ls_setup_launch(cvxg_ctx* ctx, bool spec_eval = false, DotBatch db = {});
static void ls_batch_launch(cvxg_ctx* ctx, double tbase, double beta);

// MatrixUtils.choleskySolve(H, b = -grad, tol) (MatrixUtils.scala:468-516); result in ctx->dx.
static int cholesky_solve(cvxg_ctx* ctx, double tol, cvxg_step_info* info) {
  hipStream_t s = ctx->s;
  tstart(ctx, 1);
  CHK(ruiz_lookahead(ctx));
  tstop(ctx, 1);
  tstart(ctx, 2);
  int reg = 0;
  double mind = 0.0;
  // the back substitution and residual go out behind each factorization attempt, before its host read (one
  // round trip per step instead of two); a failed attempt's results are overwritten by the retry's
  auto solve_and_residual = [&]() {
    tstop(ctx, 2);
    tstart(ctx, 3);
    // x = d :* u, and for the speculative line search s = dx (x1 = x + s when the trial evaluation goes out too), in
    // the backward solve's epilogue
    const bool se = ctx->spec_allowed && spec_eval_ok(ctx);
    BwdEpilogue epi;
    epi.d = ctx->dfin;
    epi.dx = ctx->dx;
    if (ctx->spec_allowed) epi.s = ctx->sdir;
    if (se) {
      epi.x = ctx->x;
      epi.x1 = ctx->x1;
      epi.t1 = ctx->spec_t;
      epi.sctrl = ctx->ctrl;
      ctx->spec_t_used = ctx->spec_t;
    }
    backward_solve(ctx, 1, epi);
    // relativeSize(H*x - b, b, tol), b = -grad  (MatrixUtils.scala:437-442, 496)
    if (ctx->h_full) launch_rowdot_add(s, ctx->H, ctx->np, ctx->n, ctx->np, ctx->dx, ctx->y, ctx->vtmp);  // H x + grad
    else launch_symv_lower_add(s, ctx->H, ctx->np, ctx->n, ctx->dx, ctx->y, ctx->vtmp, ctx->hsv_part);
    DotBatch db{};
    db.add(DOT_FMA, ctx->vtmp, nullptr, ctx->n, SC_RES2);
    db.add(DOT_FMA, ctx->dx, ctx->y, ctx->np, SC_Q);
    if (!ctx->spec_allowed) launch_dots(s, db, ctx->ctrl);  // (else in one launch with the line search's dots)
    tstop(ctx, 3);
    if (ctx->spec_allowed) {  // the line search's setup and first batch for s = dx ride this attempt's host read
      tstart(ctx, 4);
      ls_setup_launch(ctx, se, db);  // (s = dx and x1 = x + s came with the backward solve)
      ls_batch_launch(ctx, 1.0, ctx->spec_beta);
      ctx->spec_launched = true;
      ctx->spec_eval_launched = se;
    }
  };
  auto fill = [&]() { launch_scaled_col(s, ctx->dfin, ctx->y, -1.0, ctx->n, ctx->np, 1, 0, ctx->rhs); };
  // the speculative pair needs 134 MB more at C3 (allocated on first use); without it the sequential form runs
  if (ctx->spec_reg && ctx->prev_reg && !ctx->df_trace && spec_alloc(ctx) != CVXG_OK) ctx->spec_reg = 0;
  int rc = (ctx->spec_reg && ctx->prev_reg && !ctx->df_trace)
               ? regularized_cholesky_spec(ctx, 1, fill, &reg, &mind, solve_and_residual)
               : regularized_cholesky(ctx, 1, fill, &reg, &mind, solve_and_residual);
  ctx->prev_reg = reg;
  ctx->n_regularized += reg;
  info->ruiz_sweeps = ctx->hctrl->ruiz_sweeps;
  if (info->ruiz_sweeps >= 0) ruiz_learn(ctx, info->ruiz_sweeps);
  info->regularized = reg;
  info->small_pivot = reg ? ctx->small_piv : 0;
  info->min_diag = mind;
  if (rc != CVXG_OK) return rc;
  const double nb = ctx->normGrad;
  const double f = nb < tol ? tol : tol + nb;
  const double rel = sqrt(ctx->hctrl->sc[SC_RES2]) / f;
  info->rel_err = rel;
  if (!(rel <= tol))
    return set_err(ctx, CVXG_E_LINSOLVE_TOL, "choleskySolve: ||Hx-b||/||b|| = %.5g exceeds tolerance", rel);
  return CVXG_OK;
}

// MatrixUtils.symSolve(Mat, b, tol) (MatrixUtils.scala:734-751 -> diagonalizationSolve :603-706) on the device.
// Mat: device row-major n2 x n2 with leading dimension eig_ldm and zero padding (kept for the residual);
// b: host vector of length n2.  The solution is left in ctx->eig_x (length eig_ldm, zero padded).
static int eig_alloc(cvxg_ctx* ctx) {
  if (ctx->eig_M) return CVXG_OK;
  const size_t l = (size_t)round_up(ctx->n + ctx->p, TILE);
  ctx->eig_ldm = (int)l;
  CHK(dalloc(ctx, &ctx->eig_M, l * l));
  if (ctx->p > 0) CHK(dalloc(ctx, &ctx->eig_K, l * l));
  for (double** v : {&ctx->eig_d, &ctx->eig_e, &ctx->eig_dots, &ctx->eig_a, &ctx->eig_z, &ctx->eig_b, &ctx->eig_x})
    CHK(dalloc(ctx, v, l));
  CHK(dalloc(ctx, &ctx->eig_part, (size_t)coldot_chunks((int)l) * l));
  CHK(dalloc(ctx, &ctx->eig_info, 1));
  return CVXG_OK;
}

static int sym_solve(cvxg_ctx* ctx, const double* Mat, int n2, const double* bdev, double tol) {
  hipStream_t s = ctx->s;
  const int l = ctx->eig_ldm;
  const size_t bytes = (size_t)l * l * sizeof(double);
  HIPC(ctx, hipMemcpyAsync(ctx->eig_M, Mat, bytes, hipMemcpyDeviceToDevice, s));
  const int info = sym_eig(s, ctx->eig_M, n2, l, ctx->eig_d, ctx->eig_e, ctx->eig_info);
  if (info != 0) return set_err(ctx, CVXG_E_UNSOLVABLE, "symSolve: eigSym failed (rocSOLVER dsyevd info %d)", info);
  // eigenvector j = row j of the row-major view; rows >= n2 and eigenvalues >= n2 are padding
  if (l > n2) {
    HIPC(ctx, hipMemsetAsync(ctx->eig_M + (size_t)n2 * l, 0, (size_t)(l - n2) * l * sizeof(double), s));
    HIPC(ctx, hipMemsetAsync(ctx->eig_d + n2, 0, (size_t)(l - n2) * sizeof(double), s));
  }
  // a_j = u_j.b (0 where d_j == 0), z_j = a_j / d_j
  launch_rowdot(s, ctx->eig_M, l, l, l, bdev, ctx->eig_dots);
  launch_eig_coeffs(s, ctx->eig_dots, ctx->eig_d, n2, l, ctx->eig_a, ctx->eig_z);
  // b0 = U a: the projection of b onto Im(A); relativeSize(b - b0, b, tol) > tol -> unsolvable (:626-632)
  launch_coldot_partials(s, ctx->eig_M, l, l, l, ctx->eig_a, ctx->eig_part);
  launch_sum_chunks(s, ctx->eig_part, coldot_chunks(l), l, ctx->eig_dots);
  launch_axpy(s, bdev, ctx->eig_dots, -1.0, l, ctx->eig_dots);
  launch_dot(s, ctx->eig_dots, nullptr, l, ctx->ctrl, SC_RES2);
  launch_dot(s, bdev, nullptr, l, ctx->ctrl, SC_B2);
  // w = V z (:640), residual relativeSize(A w - b, b, tol) (:641)
  launch_coldot_partials(s, ctx->eig_M, l, l, l, ctx->eig_z, ctx->eig_part);
  launch_sum_chunks(s, ctx->eig_part, coldot_chunks(l), l, ctx->eig_x);
  launch_rowdot(s, Mat, l, n2, l, ctx->eig_x, ctx->eig_dots);
  launch_axpy(s, ctx->eig_dots, bdev, -1.0, n2, ctx->eig_dots);
  launch_dot(s, ctx->eig_dots, nullptr, n2, ctx->ctrl, SC_RES2B);
  HIPC(ctx, hipGetLastError());
  CHK(sync_ctrl(ctx));
  const double nb = sqrt(ctx->hctrl->sc[SC_B2]);
  const double f = nb < tol ? tol : tol + nb;
  const double rel_dist = sqrt(ctx->hctrl->sc[SC_RES2]) / f, rel_err = sqrt(ctx->hctrl->sc[SC_RES2B]) / f;
  if (rel_dist > tol)
    return set_err(ctx, CVXG_E_UNSOLVABLE, "MatrixUtils.diagonalizationSolve: min_x||Ax-b||/||b|| = %.5g > tol = %g",
                   rel_dist, tol);
  if (rel_err > tol)  // the reference's regularization loop cannot change the outcome (see symsolve.cpp)
    return set_err(ctx, CVXG_E_UNSOLVABLE,
                   "MatrixUtils.diagonalizationSolve: system not solvable within tolerance tol = %g, error = %.5g",
                   tol, rel_err);
  return CVXG_OK;
}

// The full symmetric H for a consumer that reads its upper triangle (after a lower-only assembly).
static void ensure_h_full(cvxg_ctx* ctx) {
  if (ctx->h_full) return;
  launch_mirror_lower(ctx->s, ctx->H, ctx->np, ctx->n);
  ctx->h_full = true;
}

// UnconstrainedSolver Newton direction with its fallback chain (UnconstrainedSolver.scala:54-67).
static int newton_direction_p0(cvxg_ctx* ctx, const cvxg_params* pars, cvxg_step_info* info) {
  int rc = cholesky_solve(ctx, pars->tolEqSolve, info);
  info->fallback = 0;
  if (rc == CVXG_OK) return rc;
  if (rc == CVXG_E_HIP) return rc;
  // choleskySolve(H + 1e-9 I, -y)
  launch_copy_diag(ctx->s, ctx->H, ctx->np, ctx->n, ctx->hdiag);
  launch_add_diag(ctx->s, ctx->H, ctx->np, ctx->n, 1e-9);
  rc = cholesky_solve(ctx, pars->tolEqSolve, info);
  launch_set_diag(ctx->s, ctx->H, ctx->np, ctx->n, ctx->hdiag);
  info->fallback = 1;
  if (rc == CVXG_OK || rc == CVXG_E_HIP) return rc;
  info->fallback = 2;
  ctx->spec_have = false;  // (the speculative line-search setup belonged to a rejected direction)
  ctx->spec_eval_have = false;
  // symSolve(H, -y) (UnconstrainedSolver.scala:64)
  ensure_h_full(ctx);
  CHK(eig_alloc(ctx));
  HIPC(ctx, hipMemsetAsync(ctx->eig_b, 0, (size_t)ctx->eig_ldm * sizeof(double), ctx->s));
  launch_axpy(ctx->s, ctx->eig_b, ctx->y, -1.0, ctx->n, ctx->eig_b);
  CHK(sym_solve(ctx, ctx->H, ctx->n, ctx->eig_b, pars->tolEqSolve));
  HIPC(ctx, hipMemsetAsync(ctx->dx, 0, (size_t)ctx->np * sizeof(double), ctx->s));
  HIPC(ctx, hipMemcpyAsync(ctx->dx, ctx->eig_x, (size_t)ctx->n * sizeof(double), hipMemcpyDeviceToDevice, ctx->s));
  launch_dot(ctx->s, ctx->dx, ctx->y, ctx->np, ctx->ctrl, SC_Q);
  HIPC(ctx, hipGetLastError());
  CHK(sync_ctrl(ctx));
  return CVXG_OK;
}

// The accuracy check of KKTSystem.solveWithCholFactor (KKTSystem.scala:147-166) on the equilibrated system, with the
// solution y = ctx->kx (Q y + B'w = -Dq, B y = b) and w = ctx->kw; x = D y into ctx->dx.
static int kkt_residual_check(cvxg_ctx* ctx, const double* qv, const double* bv, double tol, cvxg_step_info* info) {
  hipStream_t s = ctx->s;
  const int n = ctx->n, np = ctx->np, p = ctx->p;
  // residual_1 = Q y + B' w + Dq  with  Q y = d o (H (d o y)), relative to -Dq   (:148-150)
  launch_scale_vec(s, ctx->kx, ctx->dfin, np, ctx->xtmp);
  launch_rowdot(s, ctx->H, np, n, np, ctx->xtmp, ctx->vtmp);
  launch_scale_vec(s, ctx->vtmp, ctx->dfin, n, ctx->vtmp);
  launch_scale_strided(s, ctx->dfin, qv, 1, 0, n, ctx->kz);  // Dq
  launch_btw_plus(s, ctx->kB, np, p, ctx->kw, ctx->kz, n, ctx->xtmp);
  launch_axpy(s, ctx->vtmp, ctx->xtmp, 1.0, n, ctx->vtmp);
  launch_dot(s, ctx->vtmp, nullptr, n, ctx->ctrl, SC_RES2);
  launch_dot(s, ctx->kz, nullptr, n, ctx->ctrl, SC_Q);  // |Dq|^2 (temporarily)
  // residual_2 = B y - b  (:152-153)
  launch_rowdot(s, ctx->kB, np, p, np, ctx->kx, ctx->eqtmp);
  launch_axpy(s, ctx->eqtmp, bv, -1.0, p, ctx->eqtmp);
  launch_dot(s, ctx->eqtmp, nullptr, p, ctx->ctrl, SC_RES2B);
  launch_dot(s, bv, nullptr, p, ctx->ctrl, SC_B2);
  launch_scale_vec(s, ctx->kx, ctx->dfin, np, ctx->dx);  // x = D y  (:244)
  tstop(ctx, 3);
  HIPC(ctx, hipGetLastError());
  CHK(sync_ctrl(ctx));
  if (ctx->hctrl->df_status != 0)
    return set_err(ctx, CVXG_E_HIP, "KKT Schur complement: dataflow dependency wait timed out (status %d)",
                   ctx->hctrl->df_status);
  if (ctx->hctrl->chol_info != 0) return set_err(ctx, CVXG_E_NOT_PD, "KKT Schur complement not positive definite");
  auto relsize = [&](double na, double nb_) { return na / (nb_ < tol ? tol : tol + nb_); };
  const double err1 = relsize(sqrt(ctx->hctrl->sc[SC_RES2]), sqrt(ctx->hctrl->sc[SC_Q]));
  const double err2 = relsize(sqrt(ctx->hctrl->sc[SC_RES2B]), sqrt(ctx->hctrl->sc[SC_B2]));
  info->rel_err = std::max(err1, err2);
  if (err1 > tol || err2 > tol)
    return set_err(ctx, CVXG_E_LINSOLVE_TOL, "KKT: Error in solution exceeds tolerance (%.3g, %.3g)", err1, err2);
  return CVXG_OK;
}

// Lazily, once per context: the buffers of the equality block (k_kkt.hip) for this p.
static int kkt_alloc(cvxg_ctx* ctx, bool fused) {
  const int np = ctx->np, p = ctx->p, nr = p + 1;
  if (!fused && !ctx->kY) {
    ctx->kY_chunks = (nr + 15) / 16;
    ctx->kY_ld = 16 * ctx->kY_chunks;
    CHK(dalloc(ctx, &ctx->kY, (size_t)np * ctx->kY_ld));
    HIPC(ctx, hipMemsetAsync(ctx->kY, 0, (size_t)np * ctx->kY_ld * sizeof(double), ctx->s));  // unused columns: 0
    const size_t g = trsm_many_granule_doubles(ctx->nblk, ctx->kY_chunks);
    CHK(dalloc(ctx, &ctx->kYg, g));
    HIPC(ctx, hipMemsetAsync(ctx->kYg, 0, g * sizeof(double), ctx->s));
  }
  if (!ctx->kgram) {
    CHK(dalloc(ctx, &ctx->kgram, schur_partial_doubles(np, p)));
    if (p <= NB) {
      CHK(dalloc(ctx, &ctx->kS, (size_t)p * p));
      CHK(dalloc(ctx, &ctx->kzp, (size_t)p));
    } else {  // the dataflow Cholesky of S on its own buffers
      const int ps = round_up(p, NB);
      ctx->s_nblk = ps / NB;
      CHK(dalloc(ctx, &ctx->sL, (size_t)ps * ps));
      HIPC(ctx, hipMemsetAsync(ctx->sL, 0, (size_t)ps * ps * sizeof(double), ctx->s));
      CHK(dalloc(ctx, &ctx->sLinv, chol_dataflow_linv_doubles(ctx->s_nblk)));
      CHK(dalloc(ctx, &ctx->kzp, (size_t)ps));
      CHK(dalloc(ctx, &ctx->sw, (size_t)ps));
      std::vector<unsigned> order = chol_schedule(ctx->s_nblk, ctx->ncu);
      ctx->s_ntasks = (int)order.size();
      CHK(dalloc(ctx, &ctx->s_tasks, std::max<size_t>(order.size(), 1)));
      if (!order.empty())
        CHK(copy_sync(ctx, ctx->s_tasks, order.data(), order.size() * sizeof(unsigned), hipMemcpyHostToDevice));
      CHK(dalloc(ctx, &ctx->s_work, chol_dataflow_work_ints(ctx->s_nblk)));
      CHK(dalloc(ctx, &ctx->s_bwd, bwd_work_ints(ctx->s_nblk)));
      HIPC(ctx, hipMemsetAsync(ctx->s_bwd, 0, bwd_work_ints(ctx->s_nblk) * sizeof(int), ctx->s));
    }
  }
  return CVXG_OK;
}

// KKTSystem.solvePD(Hm, Aeq, q, b) (KKTSystem.scala:200-246) with the block elimination of solveWithCholFactor
// (:99-167); Hm = ctx->H, q = qv (device n-vector), b = bv (device p-vector), on the factor L of Q = D Hm D
// (k_kkt.hip), in the reference's sequence: X = Q^-1 [B' | Dq] -- the factorization's fused forward solve and the
// one-launch backward solve when p + 1 <= MAX_RHS, otherwise the many-column dataflow solves with L and L' --,
// R = B X (MFMA partials + a fixed-order reduction), S = (R + R')/2, z = -(b + R[:, p]), w = S^-1 z (one
// workgroup for p <= 64, the dataflow Cholesky and backward solve beyond), y = -(X[:, p] + X[:, :p] w).
static int kkt_solve_pd(cvxg_ctx* ctx, const double* qv, const double* bv, double tol, cvxg_step_info* info) {
  hipStream_t s = ctx->s;
  const int n = ctx->n, np = ctx->np, p = ctx->p, nr = p + 1;
  const bool fused = nr <= std::min(ctx->kkt_fused_rhs, MAX_RHS);
  CHK(kkt_alloc(ctx, fused));
  tstart(ctx, 1);
  ruiz(ctx);
  tstop(ctx, 1);
  tstart(ctx, 2);
  int reg = 0;
  double mind = 0.0;
  int rc = regularized_cholesky(
      ctx, fused ? nr : 1,
      [&]() {
        if (fused) {
          launch_kkt_prep(s, ctx->Aeq, np, p, n, np, ctx->dfin, ctx->kB, ctx->rhs, nr);  // B = A diag(d), B'
          launch_scaled_col(s, ctx->dfin, qv, 1.0, n, np, nr, p, ctx->rhs);            // D q
        } else {
          launch_scaled_col(s, ctx->dfin, qv, 1.0, n, np, 1, 0, ctx->rhs);
        }
      },
      &reg, &mind, [] {});
  tstop(ctx, 2);
  info->ruiz_sweeps = ctx->hctrl->ruiz_sweeps;
  info->regularized = reg;
  info->small_pivot = reg ? ctx->small_piv : 0;
  info->min_diag = mind;
  if (rc != CVXG_OK) return rc;
  tstart(ctx, 3);
  const double* X = ctx->sol;
  int ldx = nr;
  if (fused) {
    backward_solve(ctx, nr);  // X = Q^-1 [B' | Dq]   (:120-121)
  } else {
    launch_kkt_prep(s, ctx->Aeq, np, p, n, np, ctx->dfin, ctx->kB, ctx->kY, ctx->kY_ld);  // [B' | Dq]
    launch_scaled_col(s, ctx->dfin, qv, 1.0, n, np, ctx->kY_ld, p, ctx->kY);
    launch_trsm_many(s, false, ctx->L, np, ctx->Linv, ctx->kY, ctx->kY_ld, ctx->nblk, ctx->kY_chunks, ctx->kYg,
                     ++ctx->fm_gen, ctx->ctrl);
    launch_trsm_many(s, true, ctx->L, np, ctx->Linv, ctx->kY, ctx->kY_ld, ctx->nblk, ctx->kY_chunks, ctx->kYg,
                     ++ctx->fm_gen, ctx->ctrl);
    X = ctx->kY;
    ldx = ctx->kY_ld;
  }
  launch_ctrl_reset_chol(s, ctx->ctrl);
  if (p <= NB) {
    launch_schur_form(s, ctx->kB, np, X, ldx, p, np, ctx->kgram, bv, p, p, ctx->kS, ctx->kzp);
    launch_schur_small(s, ctx->kS, p, ctx->kzp, ctx->kw, ctx->ctrl);
  } else {
    const int ps = ctx->s_nblk * NB;
    launch_schur_form(s, ctx->kB, np, X, ldx, p, np, ctx->kgram, bv, ps, ps, ctx->sL, ctx->kzp);
    launch_chol_dataflow(s, ctx->sL, ps, ctx->kzp, 1, ctx->sLinv, ctx->ctrl, ctx->s_work, ctx->s_nblk, ctx->s_tasks,
                         ctx->s_ntasks, ctx->ncu, nullptr);
    launch_bwd_dataflow(s, ctx->sL, ps, ctx->sLinv, ctx->kzp, ctx->sw, 1, ctx->s_nblk, ctx->s_bwd, ++ctx->s_gen,
                        ctx->ctrl);
    HIPC(ctx, hipMemcpyAsync(ctx->kw, ctx->sw, (size_t)p * sizeof(double), hipMemcpyDeviceToDevice, s));
  }
  launch_kkt_v(s, X, ldx, p, np, ctx->kw, ctx->kx);  // y = -(Hinv_q + Hinv_At w)   (:145)
  return kkt_residual_check(ctx, qv, bv, tol, info);
}

static int kkt_solve_any(cvxg_ctx* ctx, const double* qv, const double* bv, double tol, cvxg_step_info* info) {
  return kkt_solve_pd(ctx, qv, bv, tol, info);
}

// KKTSystem.solve (KKTSystem.scala:43-66): solvePD(H) -> solvePD(H + A'A, q - A'b) -> kktSymSolve.
static int newton_direction_kkt(cvxg_ctx* ctx, const cvxg_params* pars, cvxg_step_info* info) {
  hipStream_t s = ctx->s;
  int rc = kkt_solve_any(ctx, ctx->y, ctx->eqd, pars->tolEqSolve, info);
  info->fallback = 0;
  if (rc == CVXG_OK || rc == CVXG_E_HIP) return rc;
  const size_t bytes = (size_t)ctx->np * ctx->np * sizeof(double);
  HIPC(ctx, hipMemcpyAsync(ctx->Hsave, ctx->H, bytes, hipMemcpyDeviceToDevice, s));
  launch_add_ata(s, ctx->H, ctx->np, ctx->Aeq, ctx->p, ctx->n);
  launch_q_minus_atb(s, ctx->y, ctx->Aeq, ctx->np, ctx->p, ctx->eqd, ctx->n, ctx->e);
  rc = kkt_solve_any(ctx, ctx->e, ctx->eqd, pars->tolEqSolve, info);
  HIPC(ctx, hipMemcpyAsync(ctx->H, ctx->Hsave, bytes, hipMemcpyDeviceToDevice, s));
  info->fallback = 1;
  if (rc == CVXG_OK || rc == CVXG_E_HIP) {
    if (rc == CVXG_OK) {  // q for the decrement uses the original gradient
      launch_dot(s, ctx->dx, ctx->y, ctx->np, ctx->ctrl, SC_Q);
      CHK(sync_ctrl(ctx));
    }
    return rc;
  }
  info->fallback = 2;
  // kktSymSolve(H, A, g = y, r = b - A x) (KKTSystem.scala:283-310): symSolve([H A'; A 0], (-g, r))
  CHK(eig_alloc(ctx));
  const int n = ctx->n, p = ctx->p, l = ctx->eig_ldm;
  launch_kkt_matrix(s, ctx->H, ctx->np, ctx->Aeq, ctx->np, n, p, l, ctx->eig_K);
  HIPC(ctx, hipMemsetAsync(ctx->eig_b, 0, (size_t)l * sizeof(double), s));
  launch_axpy(s, ctx->eig_b, ctx->y, -1.0, n, ctx->eig_b);
  HIPC(ctx, hipMemcpyAsync(ctx->eig_b + n, ctx->eqd, (size_t)p * sizeof(double), hipMemcpyDeviceToDevice, s));
  CHK(sym_solve(ctx, ctx->eig_K, n + p, ctx->eig_b, pars->tolEqSolve));
  HIPC(ctx, hipMemsetAsync(ctx->dx, 0, (size_t)ctx->np * sizeof(double), s));
  HIPC(ctx, hipMemcpyAsync(ctx->dx, ctx->eig_x, (size_t)n * sizeof(double), hipMemcpyDeviceToDevice, s));
  HIPC(ctx, hipMemcpyAsync(ctx->kw, ctx->eig_x + n, (size_t)p * sizeof(double), hipMemcpyDeviceToDevice, s));
  launch_dot(s, ctx->dx, ctx->y, ctx->np, ctx->ctrl, SC_Q);
  HIPC(ctx, hipGetLastError());
  CHK(sync_ctrl(ctx));
  return CVXG_OK;
}

static int newton_direction(cvxg_ctx* ctx, const cvxg_params* pars, cvxg_step_info* info) {
  if (ctx->h_valid && ctx->x_eval_valid) {  // assembled on s2 behind this x's evaluation (s already waits on it)
  } else {
    tstart(ctx, 0);
    CHK(assemble_hessian(ctx, nullptr, nullptr, nullptr, step_h_full(ctx)));
    tstop(ctx, 0);
  }
  ctx->h_valid = false;
  int rc;
  if (ctx->p == 0) {
    rc = newton_direction_p0(ctx, pars, info);
  } else {
    rc = newton_direction_kkt(ctx, pars, info);
    if (rc == CVXG_OK && info->fallback == 0) {
      launch_dot(ctx->s, ctx->dx, ctx->y, ctx->np, ctx->ctrl, SC_Q);
      CHK(sync_ctrl(ctx));
    }
  }
  return rc;
}

// ------------------------------------------------------------------------------------------------
// Line search (UnconstrainedSolver.scala:83-113 / EqualityConstrainedSolver.scala:78-97)
// ------------------------------------------------------------------------------------------------
struct TrialBatch {
  int k0 = -1;
  double logs[LS_TRIALS];
  double lerr[LS_TRIALS];  // certified mode: bound of the log-sum error (inf: not certifiable)
  double labs[LS_TRIALS];  // certified mode: sum |log d_i|
  double kl[LS_TRIALS];    // KL dual: sum_j R exp(-(B'(x + t_k s))_j); KL primal: sum_j xt_j log(n xt_j)
  double kla[LS_TRIALS];   // KL primal: the error scale of kl (certified mode)
  int viol[LS_TRIALS], npos[LS_TRIALS], sure[LS_TRIALS], amb[LS_TRIALS];
};

static constexpr double U53 = 1.1102230246251565e-16;  // unit roundoff 2^-53
// gamma of the certified trial decisions: |fl(a.v) - a.v| <= (cols + 2) u |a|.|v| for any summation order, with a 4x
// margin and room for the few roundings around the dot (r +, x + s t, ub -)
static double ls_gamma(const cvxg_ctx* ctx) { return 4.0 * (ctx->np + 16) * U53; }

// The objective's own per-trial terms when it is not linear / quadratic in the step: the KL dual's R.exp(-B'(z + t s))
// or the KL primal's (x + s t).log(n (x + s t)) with its error scale; copied into b->kl / b->kla on the stream.
static int ls_objective_trials(cvxg_ctx* ctx, double tbase, double beta, TrialBatch* b) {
  if (ctx->kl) {
    const bool cert = ls_certified(ctx);
    launch_ls_kl(ctx->s, ctx->kl_v, ctx->kl_u, ctx->nout, ctx->kl_R, tbase, beta, ctx->kl_part, ctx->kl_ls,
                 cert ? ctx->kl_vabs : nullptr, cert ? ctx->kl_uabs : nullptr, ls_gamma(ctx));
    HIPC(ctx, hipMemcpyAsync(b->kl, ctx->kl_ls, LS_TRIALS * sizeof(double), hipMemcpyDeviceToHost, ctx->s));
    HIPC(ctx, hipMemcpyAsync(b->kla, ctx->kl_ls + LS_TRIALS, LS_TRIALS * sizeof(double), hipMemcpyDeviceToHost,
                             ctx->s));
  } else if (ctx->klp) {
    launch_ls_klp(ctx->s, ctx->x, ctx->sdir, ctx->n, ctx->klp_n, tbase, beta, ctx->klp_part, ctx->klp_ls);
    HIPC(ctx, hipMemcpyAsync(b->kl, ctx->klp_ls, LS_TRIALS * sizeof(double), hipMemcpyDeviceToHost, ctx->s));
    HIPC(ctx, hipMemcpyAsync(b->kla, ctx->klp_ls + LS_TRIALS, LS_TRIALS * sizeof(double), hipMemcpyDeviceToHost,
                             ctx->s));
  }
  return CVXG_OK;
}

// Launch one batch of LS_TRIALS trials t_k = tbase beta^k (inequality rows: the counts and log sums into ls_log).
static void ls_batch_launch(cvxg_ctx* ctx, double tbase, double beta) {
  const int nb = ls_blocks(ctx->m);
  const bool cert = ls_certified(ctx);
  launch_ls_trials(ctx->s, ctx->c, ctx->e, ctx->ub, ctx->m, tbase, beta, ctx->ls_plog, ctx->ls_pcnt,
                   ctx->nq > 0 ? ctx->qf : nullptr, cert ? ctx->cabs : nullptr, ctx->eabs, ls_gamma(ctx),
                   ctx->ls_paux, (cert && ctx->nq > 0) ? ctx->qfabs : nullptr);
  launch_ls_finalize(ctx->s, ctx->ls_plog, ctx->ls_pcnt, ctx->ls_paux, nb, ctx->ls_log, ctx->ls_cnt);
}
// The batch from its host copy (hls).
static void ls_batch_parse(const cvxg_ctx* ctx, int k0, TrialBatch* b) {
  b->k0 = k0;
  const int* cnt = (const int*)(ctx->hls + 3 * LS_TRIALS);
  for (int k = 0; k < LS_TRIALS; ++k) {
    b->logs[k] = ctx->hls[3 * k];
    b->lerr[k] = ctx->hls[3 * k + 1];
    b->labs[k] = ctx->hls[3 * k + 2];
    b->viol[k] = cnt[4 * k];
    b->npos[k] = cnt[4 * k + 1];
    b->sure[k] = cnt[4 * k + 2];
    b->amb[k] = cnt[4 * k + 3];
  }
}

static int ls_batch(cvxg_ctx* ctx, int k0, double tbase, double beta, TrialBatch* b) {
  if (ctx->m == 0) {  // no inequality constraints: every trial is in C and contributes no log terms
    CHK(ls_objective_trials(ctx, tbase, beta, b));
    HIPC(ctx, hipStreamSynchronize(ctx->s));
    b->k0 = k0;
    for (int k = 0; k < LS_TRIALS; ++k) {
      b->logs[k] = b->lerr[k] = b->labs[k] = 0.0;
      b->viol[k] = b->npos[k] = b->sure[k] = b->amb[k] = 0;
    }
    return CVXG_OK;
  }
  CHK(ls_objective_trials(ctx, tbase, beta, b));
  ls_batch_launch(ctx, tbase, beta);
  HIPC(ctx, hipGetLastError());
  if (ctx->kl || ctx->klp) {  // (their trial sums went out by hipMemcpyAsync into the host-stack batch)
    HIPC(ctx, hipMemcpyAsync(ctx->hls, ctx->ls_log, 5 * LS_TRIALS * sizeof(double), hipMemcpyDeviceToHost, ctx->s));
    HIPC(ctx, hipStreamSynchronize(ctx->s));
  } else {
    CHK(host_read(ctx, ctx->ls_log, ctx->hls_dev, 5 * LS_TRIALS * sizeof(double)));
  }
  ls_batch_parse(ctx, k0, b);
  return CVXG_OK;
}

// The reference's own evaluation of one trial point (UnconstrainedSolver.scala:93,102,107): xt = x + s*t, then
// isInSet(xt) (Constraint.scala:23 for every row) and barrierFunction(t, xt) (BarrierSolver.scala:280-289), through the
// same kernels and summation order as the barrier value at x.  Used for the trials whose batch margin is inside the
// rounding band (line_search).
struct FreshTrial {
  int viol = 0, npos = 0;
  double fv = 0.0;
};
static int trial_fresh(cvxg_ctx* ctx, double tt, FreshTrial* out) {
  hipStream_t s = ctx->s;
  const int np = ctx->np, mp = ctx->mp;
  launch_axpy(s, ctx->x, ctx->sdir, tt, np, ctx->xtr);  // x + s*t (contraction off: two roundings, as Breeze)
  launch_ctrl_reset_eval(s, ctx->ctrl);
  if (ctx->nq > 0) {  // QuadraticConstraint.valueAt(xt): r + a.xt + xt.(P xt)/2
    launch_rowdot(s, ctx->Pq, np, ctx->nq * np, np, ctx->xtr, ctx->qPx_tr);
    launch_quad_xpx(s, ctx->qPx_tr, ctx->xtr, ctx->qrows, ctx->nq, np, ctx->qextra_tr);
  }
  launch_constraint_eval(s, ctx->A, np, mp, np, ctx->xtr, ctx->r, ctx->ub, ctx->c_tr, ctx->d_tr, ctx->invd_tr, ctx->w_tr,
                         ctx->logd_tr, ctx->ctrl, ctx->nq > 0 ? ctx->qextra_tr : nullptr, nullptr);
  launch_sum(s, ctx->logd_tr, mp, ctx->ctrl, SC_TR_SUMLOG);
  launch_dot(s, ctx->a0, ctx->xtr, np, ctx->ctrl, SC_TR_A0X);
  const bool quad = ctx->hasP && !ctx->kl;
  if (quad) {
    launch_rowdot(s, ctx->P, np, np, np, ctx->xtr, ctx->Pxtr);
    launch_dot(s, ctx->xtr, ctx->Pxtr, np, ctx->ctrl, SC_TR_XPX);
  }
  if (ctx->klp) {  // Dist_KL.objectiveFunction(n).valueAt(xt) = xt dot log(xt*n)
    launch_klp_eval(s, ctx->xtr, ctx->n, np, ctx->klp_n, ctx->klp_lxt, nullptr, nullptr, nullptr);
    launch_dot(s, ctx->xtr, ctx->klp_lxt, np, ctx->ctrl, SC_TR_KLP);
  }
  if (ctx->kl) {  // -dualObjFAt(zt) = w.zt + R.exp(-B'zt)  (Dist_KL.scala:146-147, Duality.scala:76)
    launch_rowdot(s, ctx->KB, np, ctx->noutp, np, ctx->xtr, ctx->kl_vtr);
    launch_kl_eval(s, ctx->kl_vtr, ctx->nout, ctx->noutp, ctx->kl_R, ctx->kl_ytr);
    launch_sum(s, ctx->kl_ytr, ctx->noutp, ctx->ctrl, SC_TR_KLSUM);
  }
  HIPC(ctx, hipGetLastError());
  CHK(sync_ctrl(ctx));
  const DevCtrl& h = *ctx->hctrl;
  const double f0 = ctx->klp  ? h.sc[SC_TR_KLP]
                    : ctx->kl ? h.sc[SC_TR_A0X] + h.sc[SC_TR_KLSUM]
                              : ctx->r0 + h.sc[SC_TR_A0X] + (quad ? h.sc[SC_TR_XPX] / 2 : 0.0);
  out->fv = ctx->t * f0 - h.sc[SC_TR_SUMLOG];
  out->viol = h.not_strict;
  out->npos = h.infeasible;
  return CVXG_OK;
}

// Backtracking from x along s (device ctx->sdir).  limit = 200 / throw_at = 100 (Unconstrained) or
// 100 / 100 (EqualityConstrained).  Returns the accepted t and the two counters.
//
// Trials are scored in batches of LS_TRIALS from c = g(x) and e = A s (g(x + t s) = c + t e, O(m) per trial).  With
// linear constraints (ls_certified) the batch also bounds how far its arithmetic and the reference's fresh evaluation
// valueAt(x + s*t) can each lie from the exact value (any FP64 summation order), so every decision whose margin
// exceeds that band is the one any evaluation order makes.  Inside the band:
//  * feasibility (isInSet, Constraint.scala:23): the trial is evaluated fresh on the device (trial_fresh), exactly as
//    the reference forms it, and decided from that (*fresh counts these) -- a wrong "in C" would leave the domain;
//  * Armijo (UnconstrainedSolver.scala:107): |f(x + s t) - f - alpha t q| is below the rounding error of f itself, so
//    the decision is rounding noise in every implementation (numpy, Breeze and a fresh device evaluation disagree
//    among themselves).  It is taken from the batch value and counted in *ties.  (Deciding these from a fresh
//    evaluation was measured: late in the path -- t = 1e10 -- the noise then rejected trial after trial and a
//    centering ran into maxIter.)
// e = A s (and |A||s|), and the quadratic pieces of f0(x + s t), s = ctx->sdir: launches only.
// db: reductions already enqueued by the caller (the residual's), launched together with the setup's own
static void ls_setup_launch(cvxg_ctx* ctx, bool spec_eval, DotBatch db) {
  hipStream_t s = ctx->s;
  const bool cert = ls_certified(ctx);
  const bool quad = ctx->hasP && !ctx->kl;
  if (ctx->m > 0) {
    if (spec_eval)  // e, eabs and the constraint evaluation at x1 = x + s in one sweep over A
      launch_ls_setup_eval(s, ctx->A, ctx->np, ctx->mp, ctx->np, ctx->sdir, ctx->x1, ctx->e, ctx->eabs, ctx->r,
                           ctx->ub, ctx->c1, ctx->d1, ctx->invd1, ctx->w1, ctx->logd1, ctx->cabs1, ctx->ctrl);
    else if (cert) launch_rowdot_abs(s, ctx->A, ctx->np, ctx->m, ctx->np, ctx->sdir, ctx->e, ctx->eabs);
    else launch_rowdot(s, ctx->A, ctx->np, ctx->m, ctx->np, ctx->sdir, ctx->e);
  }
  if (ctx->nq > 0) {  // e_k = G_k.s and f_k = s'P_k s: g_k(x + t s) = g_k + t e_k + t^2 f_k / 2
    if (cert) launch_rowdot_abs(s, ctx->Pq, ctx->np, ctx->nq * ctx->np, ctx->np, ctx->sdir, ctx->qPs, ctx->qPsa);
    else launch_rowdot(s, ctx->Pq, ctx->np, ctx->nq * ctx->np, ctx->np, ctx->sdir, ctx->qPs);
    launch_quad_ls(s, ctx->qPx, ctx->qPs, ctx->sdir, ctx->qrows, ctx->nq, ctx->np, ctx->e, ctx->qf);
    if (cert) {  // eabs += |s|'|P_k||x|, fabs = |s|'|P_k||s|
      launch_quad_absdot(s, ctx->qPxa, ctx->sdir, ctx->qrows, ctx->nq, ctx->np, 1.0, 1, ctx->eabs);
      launch_quad_absdot(s, ctx->qPsa, ctx->sdir, ctx->qrows, ctx->nq, ctx->np, 1.0, 0, ctx->qfabs);
    }
  }
  if (ctx->kl) {  // u = B's (and |B'||s|)
    if (cert) launch_rowdot_abs(s, ctx->KB, ctx->np, ctx->noutp, ctx->np, ctx->sdir, ctx->kl_u, ctx->kl_uabs);
    else launch_rowdot(s, ctx->KB, ctx->np, ctx->noutp, ctx->np, ctx->sdir, ctx->kl_u);
  }
  if (quad) {
    if (cert) launch_rowdot_abs(s, ctx->P, ctx->np, ctx->np, ctx->np, ctx->sdir, ctx->Ps, ctx->Psa);
    else launch_rowdot(s, ctx->P, ctx->np, ctx->np, ctx->np, ctx->sdir, ctx->Ps);
  }
  auto add = [&](int k, const double* u, const double* v, int len, int sl) {
    if (db.full()) {
      launch_dots(s, db, ctx->ctrl);
      db.count = 0;
    }
    db.add(k, u, v, len, sl);
  };
  add(DOT_FMA, ctx->a0, ctx->sdir, ctx->np, SC_A0S);
  if (quad) {
    add(DOT_FMA, ctx->sdir, ctx->Px, ctx->np, SC_SPX);
    add(DOT_FMA, ctx->sdir, ctx->Ps, ctx->np, SC_SPS);
  }
  if (cert) {
    add(DOT_ABS, ctx->a0, ctx->sdir, ctx->np, SC_A0SA);
    if (quad) {
      add(DOT_ABS, ctx->sdir, ctx->Pxa, ctx->np, SC_SPXA);
      add(DOT_ABS, ctx->sdir, ctx->Psa, ctx->np, SC_SPSA);
    }
  }
  launch_dots(s, db, ctx->ctrl);
}

// use_spec: the setup and the first batch went out behind the factorization (cholesky_solve) and arrived with its host
// read; otherwise they are launched here.
static int line_search(cvxg_ctx* ctx, const cvxg_params* pars, double q, int limit, double* t_out, int* k_c,
                       int* k_a, int* fresh, int* ties, bool use_spec) {
  const double beta = pars->beta, alpha = pars->alpha;
  const bool cert = ls_certified(ctx);
  const bool quad = ctx->hasP && !ctx->kl;
  if (!use_spec) {
    ls_setup_launch(ctx);
    HIPC(ctx, hipGetLastError());
    CHK(sync_ctrl(ctx));
  }
  const DevCtrl h = *ctx->hctrl;
  const double tb = ctx->t, f = ctx->f_at_x;
  // r + a.(x+st) + (x+st)'P(x+st)/2, or w.(z+st) + R.exp(-B'(z+st)), or the KL primal (x+st).log(n (x+st))
  auto f0_at = [&](double tt, double klsum) {
    if (ctx->kl) return (h.sc[SC_A0X] + tt * h.sc[SC_A0S]) + klsum;
    if (ctx->klp) return klsum;
    double v = ctx->r0 + (h.sc[SC_A0X] + tt * h.sc[SC_A0S]);
    if (quad) v += (h.sc[SC_XPX] + 2 * tt * h.sc[SC_SPX] + tt * tt * h.sc[SC_SPS]) / 2;
    return v;
  };
  // error bounds (certified mode) of the objective part at x + s tt and of the barrier value f at x
  const double gam = ls_gamma(ctx);
  // error bound of f0 at x + s tt; klerr: the KL objectives' own term (the KL primal's error scale at the trial point,
  // or the KL dual's exponent error already scaled, k_ls_kl)
  auto ef0_at = [&](double tt, double klerr) {
    if (ctx->klp) return gam * klerr;
    if (ctx->kl) return gam * (h.sc[SC_A0XA] + tt * h.sc[SC_A0SA]) + klerr;
    double v = fabs(ctx->r0) + h.sc[SC_A0XA] + tt * h.sc[SC_A0SA];
    if (quad) v += (h.sc[SC_XPXA] + 2 * tt * h.sc[SC_SPXA] + tt * tt * h.sc[SC_SPSA]) / 2;
    return gam * v;
  };
  const double klerr_x = ctx->klp ? h.sc[SC_KLPA] : gam * h.sc[SC_KLA] + 4 * U53 * h.sc[SC_KLSUM];
  const double ef_x = tb * ef0_at(0.0, klerr_x) + 2.0 * gam * h.sc[SC_CAINV] + (ctx->mp + 8) * U53 * h.sc[SC_LOGABS] +
                      8 * U53 * fabs(f);
  TrialBatch b;
  double tcur = 1.0;
  double tbatch = 1.0;  // t at the start of the next batch (products of beta, UnconstrainedSolver.scala:93)
  int next_k0 = 0;
  if (use_spec) {  // batch 0 (t = 1 ... beta^63) is already on the host
    ls_batch_parse(ctx, 0, &b);
    for (int i = 0; i < LS_TRIALS; ++i) tbatch *= beta;
    next_k0 = LS_TRIALS;
  }
  auto ensure = [&](int k) -> int {
    while (!(b.k0 >= 0 && k >= b.k0 && k < b.k0 + LS_TRIALS)) {
      CHK(ls_batch(ctx, next_k0, tbatch, beta, &b));
      for (int i = 0; i < LS_TRIALS; ++i) tbatch *= beta;
      next_k0 += LS_TRIALS;
    }
    return CVXG_OK;
  };
  int fresh_it = -1;  // trial index of the cached fresh evaluation
  FreshTrial fr;
  auto fresh_at = [&](int it) -> int {
    if (fresh_it != it) {
      CHK(trial_fresh(ctx, tcur, &fr));
      fresh_it = it;
      ++*fresh;
    }
    return CVXG_OK;
  };
  int it = 0;
  // while (!C.isInSet(x + s*t) && it < limit) { t *= beta; it += 1 }
  while (true) {
    if (it >= limit) break;
    CHK(ensure(it));
    const int j = it - b.k0;
    bool in_set;
    if (!cert || b.sure[j] > 0 || b.amb[j] == 0) {
      in_set = b.viol[j] == 0;
    } else {
      CHK(fresh_at(it));
      in_set = fr.viol == 0;
    }
    if (in_set) break;
    tcur *= beta;
    ++it;
  }
  if (it == 100) return set_err(ctx, CVXG_E_LINESEARCH, "Line search: backtracking into the set C failed.");
  *k_c = it;
  // while (objF.valueAt(x + s*t) > f + alpha*t*q && it < limit) { t *= beta; it += 1 }
  double last_fv = 0.0, last_thr = 0.0;  // (diagnostics of a failed search)
  const int ties0 = *ties;
  while (it < limit) {
    CHK(ensure(it));
    const int j = it - b.k0;
    int npos = b.npos[j];
    double fv = tb * f0_at(tcur, b.kl[j]) - b.logs[j];
    const double thr = f + alpha * tcur * q;
    if (cert && fresh_it == it) {
      // this trial's feasibility was decided fresh: its d > 0 test and its value are the fresh evaluation's too (the
      // batch log sum skips rows whose own d <= 0 with no error bound, so it cannot stand in for barrierFunction here)
      npos = fr.npos;
      fv = fr.fv;
    }
    if (cert) {
      const double efv =
          tb * ef0_at(tcur, b.kla[j]) + b.lerr[j] + (ctx->mp + 8) * U53 * b.labs[j] + 8 * U53 * fabs(fv);
      const double ethr = ef_x + 8 * U53 * (fabs(f) + fabs(alpha * tcur * q));
      if (!(fabs(fv - thr) > efv + ethr)) ++*ties;  // a tie: decided by the batch value (see above)
    }
    if (npos > 0)
      return set_err(ctx, CVXG_E_INFEASIBLE_X, "barrierFunction: x not strictly feasible in line search");
    last_fv = fv;
    last_thr = thr;
    if (!(fv > thr)) break;
    tcur *= beta;
    ++it;
  }
  if (it == 100)
    return set_err(ctx, CVXG_E_LINESEARCH,
                   "Line search: sufficient decrease not reached (barrier t = %.17g, inner iteration %d, f = %.17g, "
                   "q = %.17g, %d halvings into C, last trial step %.17g: f(x + s t) = %.17g > f + alpha t q = %.17g; "
                   "%d of the Armijo decisions inside the rounding band of f)",
                   tb, ctx->iter, f, q, *k_c, tcur / beta, last_fv, last_thr, *ties - ties0);
  *k_a = it - *k_c;
  *t_out = tcur;
  return CVXG_OK;
}

static bool loop_cond(cvxg_ctx* ctx, const cvxg_params* pars) {
  const double tol = pars->tolSolver;
  if (!(ctx->iter < pars->maxIter)) return false;
  if (ctx->p == 0) return ctx->nd > tol && ctx->normGrad > tol;
  return (ctx->nd > tol && ctx->normGrad > tol) || ctx->eqGap > tol;
}

// End of a timed step: the next ring slot (its events are re-recorded; slot 5 may already hold the next step's
// prefetched assembly).
static void timing_collect(cvxg_ctx* ctx) {
  if (!ctx->tm.on) return;
  Timer& tm = ctx->tm;
  tm.tick += 1;
  tm.steps = std::min(tm.steps + 1, TRING - 1);
  const int sl = tm.tick % TRING;
  for (int i = 0; i < NT; ++i)
    if (i != 5 || !tm.pf5) tm.rec[sl][i] = false;
  tm.pf5 = false;
}

// ------------------------------------------------------------------------------------------------
// C-ABI
// ------------------------------------------------------------------------------------------------
extern "C" {

const char* cvxg_version(void) { return "cvxg 0.1 (gfx950, FP64 MFMA SYRK, blocked Cholesky NB=64)"; }

static thread_local std::string g_err;  // errors of the context-free entry points (cvxg_solution_space)
const char* cvxg_last_error(const cvxg_ctx* ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

// K split of the SYRK tail tiles: the leftover tiles share one wave of slots.
static int syrk_nsplit(const cvxg_ctx* ctx, int kchunks) {
  const int rest = ctx->ntiles - ctx->ntiles_main;
  return rest > 0 ? std::max(1, std::min(kchunks, ctx->slots / rest)) : 1;
}

int cvxg_create(int device, int n, int m, int p, cvxg_ctx** out) {
  if (!out) return CVXG_E_ARG;
  *out = nullptr;
  if (n <= 0 || m < 0 || p < 0) return CVXG_E_DIM;
  if (p > 0 && p >= n) return CVXG_E_DIM;  // EqualityConstraint: A.rows < A.cols (EqualityConstraint.scala:18-20)
  // the dataflow Cholesky encodes tile indices in 10 bits (nblk <= 1023, n <= 65472; H alone is 34 GB there)
  if (n > 1023 * NB) return CVXG_E_UNSUPPORTED;
  cvxg_ctx* ctx = new cvxg_ctx();
  *out = ctx;
  ctx->dev = device;
  ctx->n = n;
  ctx->m = m;
  ctx->p = p;
  ctx->np = round_up(n, TILE);
  ctx->mp = round_up(std::max(m, 1), MPAD);
  ctx->nblk = ctx->np / NB;
  HIPC(ctx, hipSetDevice(device));
  HIPC(ctx, hipStreamCreateWithFlags(&ctx->s, hipStreamNonBlocking));
  const size_t np = ctx->np, mp = ctx->mp;
  CHK(dalloc(ctx, &ctx->a0, np));
  CHK(dalloc(ctx, &ctx->A, mp * np));
  CHK(dalloc(ctx, &ctx->r, mp));
  CHK(dalloc(ctx, &ctx->ub, mp));
  {  // padded rows: ub = 1 so d = 1, log d = 0
    std::vector<double> one(mp, 1.0);
    CHK(copy_sync(ctx, ctx->ub, one.data(), mp * sizeof(double), hipMemcpyHostToDevice));
  }
  const size_t pe = std::max(p, CVXG_MAX_EQ);  // equality-row buffers
  if (p > 0) {
    CHK(dalloc(ctx, &ctx->Aeq, pe * np));
    CHK(dalloc(ctx, &ctx->beq, pe));
    CHK(dalloc(ctx, &ctx->kB, pe * np));
    CHK(dalloc(ctx, &ctx->Hsave, np * np));
  }
  CHK(dalloc(ctx, &ctx->kw, pe));
  CHK(dalloc(ctx, &ctx->kx, np));
  CHK(dalloc(ctx, &ctx->kz, np));
  CHK(dalloc(ctx, &ctx->eqd, pe));
  CHK(dalloc(ctx, &ctx->eqtmp, pe));
  for (double** v : {&ctx->x, &ctx->y, &ctx->dx, &ctx->sdir, &ctx->xtmp, &ctx->vtmp, &ctx->Px, &ctx->Ps, &ctx->ruiz0,
                     &ctx->ruiz1, &ctx->dfin, &ctx->hdiag})
    CHK(dalloc(ctx, v, np));
  for (double** v : {&ctx->c, &ctx->d, &ctx->invd, &ctx->w, &ctx->logd, &ctx->e}) CHK(dalloc(ctx, v, std::max(mp, np)));
  CHK(dalloc(ctx, &ctx->H, np * np));
  CHK(dalloc(ctx, &ctx->L, np * np));
  CHK(dalloc(ctx, &ctx->Linv, chol_dataflow_linv_doubles(ctx->nblk)));
  {  // dataflow Cholesky: task order for this tile count, work words
    (void)hipDeviceGetAttribute(&ctx->ncu, hipDeviceAttributeMultiprocessorCount, device);
    ctx->ncu = std::max(ctx->ncu, 1);
    std::vector<unsigned> order = chol_schedule(ctx->nblk, ctx->ncu);
    ctx->df_ntasks = (int)order.size();
    CHK(dalloc(ctx, &ctx->df_tasks, order.size()));
    CHK(copy_sync(ctx, ctx->df_tasks, order.data(), order.size() * sizeof(unsigned), hipMemcpyHostToDevice));
    CHK(dalloc(ctx, &ctx->df_work, chol_dataflow_work_ints(ctx->nblk)));
    if (const char* e = getenv("CVXG_DF_TRACE")) {  // instrumentation only: the task timeline of the last factorization
      ctx->df_trace_path = e;
      CHK(dalloc(ctx, &ctx->df_trace, (size_t)4 * (ctx->df_ntasks + 5 * ctx->nblk)));
    }
  }
  CHK(dalloc(ctx, &ctx->bwd_flags, bwd_work_ints(ctx->nblk)));
  CHK(dalloc(ctx, &ctx->rhs, np * MAX_RHS));
  CHK(dalloc(ctx, &ctx->sol, np * MAX_RHS));
  // SYRK tile list and wave plan (syrk_tile_plan): full-K tiles in whole waves of workgroup slots, the
  // remaining tiles split along K so that they fill one more wave.
  const int nt = ctx->np / TILE;
  int ncu = 256;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device);
  const int slots = 2 * std::max(ncu, 1);
  ctx->slots = slots;
  // the fused forward solve carries the KKT columns only on small problems: at C3 (64 blocks) the many-column solves
  // cost less than the 9-column chain (C3EQ8: 204.5 vs 191.5 solves/s)
  ctx->kkt_fused_rhs = ctx->nblk < 8 ? MAX_RHS : 1;
  const int kchunks = (int)(mp / KC);
  std::vector<int> tl = syrk_tile_plan(nt, slots, &ctx->ntiles_main);
  ctx->ntiles = (int)tl.size();
  ctx->nsplit = syrk_nsplit(ctx, kchunks);
  CHK(dalloc(ctx, &ctx->tiles, tl.size()));
  CHK(copy_sync(ctx, ctx->tiles, tl.data(), tl.size() * sizeof(int), hipMemcpyHostToDevice));
  size_t part = std::max((mp / 64) * np, (size_t)ctx->nblk * np);  // coldot partials, Ruiz tile partials
  if (ctx->nsplit > 1)
    part = std::max(part, (size_t)ctx->nsplit * (ctx->ntiles - ctx->ntiles_main) * TILE * TILE);
  CHK(dalloc(ctx, &ctx->part, part));
  CHK(dalloc(ctx, &ctx->hsv_part, (size_t)ctx->nblk * np));
  if (const char* e = getenv("CVXG_RUIZ_TRACE")) ctx->ruiz_trace_path = e;  // instrumentation only (the loop's stamps)
  // Ruiz by size (round 6): up to 16 blocks (n <= 1024, the triangle <= 4 MB) the one-launch loop
  // beats the launch pairs -- C2 0.105 vs 0.113 ms, C4 0.131 vs 0.141 ms per Ruiz, the same bits
  // (profiles/r06/workloads/ruiz_C*.json) -- and at C3 it loses (0.36-0.40 vs 0.245 ms, round 5)
  if (ctx->nblk <= RUIZ_LOOP_MAX_BLOCKS && ruiz_loop_fits(ctx->nblk)) {
    CHK(ruiz_loop_alloc(ctx));
    ctx->ruiz_loop = 1;
  }
  CHK(dalloc(ctx, &ctx->spart,
             ctx->nsplit > 1 ? (size_t)ctx->nsplit * (ctx->ntiles - ctx->ntiles_main) * TILE * TILE : (size_t)1));
  HIPC(ctx, hipStreamCreateWithFlags(&ctx->s2, hipStreamNonBlocking));
  HIPC(ctx, hipEventCreateWithFlags(&ctx->ev_w, hipEventDisableTiming));
  HIPC(ctx, hipEventCreateWithFlags(&ctx->ev_h, hipEventDisableTiming));
  const int lsb = ls_blocks(std::max(m, 1));
  CHK(dalloc(ctx, &ctx->ls_plog, (size_t)lsb * LS_TRIALS));
  CHK(dalloc(ctx, &ctx->ls_paux, (size_t)lsb * LS_TRIALS * 2));
  CHK(dalloc(ctx, &ctx->ls_pcnt, (size_t)lsb * LS_TRIALS * 4));
  CHK(dalloc(ctx, &ctx->ls_log, 5 * LS_TRIALS));  // {log sums} then the counts as ints: one host read for both
  ctx->ls_cnt = reinterpret_cast<int*>(ctx->ls_log + 3 * LS_TRIALS);
  for (double** v : {&ctx->Pxa, &ctx->Psa, &ctx->xtr, &ctx->Pxtr}) CHK(dalloc(ctx, v, np));
  for (double** v : {&ctx->cabs, &ctx->eabs, &ctx->c_tr, &ctx->d_tr, &ctx->invd_tr, &ctx->w_tr, &ctx->logd_tr,
                     &ctx->c1, &ctx->d1, &ctx->invd1, &ctx->w1, &ctx->logd1, &ctx->cabs1})
    CHK(dalloc(ctx, v, mp));
  CHK(dalloc(ctx, &ctx->x1, np));
  CHK(dalloc(ctx, &ctx->ctrl, 1));
  HIPC(ctx, hipHostMalloc((void**)&ctx->hctrl, sizeof(DevCtrl), hipHostMallocCoherent | hipHostMallocMapped));
  HIPC(ctx, hipHostMalloc((void**)&ctx->hflag, 64, hipHostMallocCoherent | hipHostMallocMapped));
  HIPC(ctx, hipHostGetDevicePointer((void**)&ctx->hctrl_dev, ctx->hctrl, 0));
  HIPC(ctx, hipHostGetDevicePointer((void**)&ctx->hflag_dev, ctx->hflag, 0));
  *ctx->hflag = 0;
  HIPC(ctx, hipHostMalloc((void**)&ctx->hls, 5 * LS_TRIALS * sizeof(double), hipHostMallocCoherent | hipHostMallocMapped));
  HIPC(ctx, hipHostGetDevicePointer((void**)&ctx->hls_dev, ctx->hls, 0));
  memset(ctx->hctrl, 0, sizeof(DevCtrl));
  HIPC(ctx, hipStreamSynchronize(ctx->s));
  return CVXG_OK;
}

void cvxg_destroy(cvxg_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->dev);
  if (ctx->s) (void)hipStreamSynchronize(ctx->s);
  void* ptrs[] = {ctx->P, ctx->a0, ctx->A, ctx->r, ctx->ub, ctx->Aeq, ctx->beq, ctx->x, ctx->y, ctx->dx, ctx->sdir,
                  ctx->xtmp, ctx->vtmp, ctx->Px, ctx->Ps, ctx->e, ctx->c, ctx->d, ctx->invd, ctx->w, ctx->logd,
                  ctx->eqd, ctx->eqtmp, ctx->H, ctx->L, ctx->Linv, ctx->Hsave, ctx->ruiz0, ctx->ruiz1, ctx->dfin,
                  ctx->hdiag, ctx->rhs, ctx->sol, ctx->part, ctx->hsv_part, ctx->ruiz_S, ctx->kB, ctx->kw, ctx->kx, ctx->kz, ctx->ls_plog,
                  ctx->ls_log, ctx->ls_pcnt, ctx->tiles, ctx->ctrl, ctx->df_tasks, ctx->df_work, ctx->df_trace, ctx->bwd_flags,
                  ctx->eig_M, ctx->eig_K, ctx->eig_d, ctx->eig_e, ctx->eig_dots, ctx->eig_a, ctx->eig_z,
                  ctx->eig_b, ctx->eig_x, ctx->eig_part, ctx->eig_info, ctx->KB, ctx->kl_v, ctx->kl_y, ctx->kl_u,
                  ctx->kl_negBy, ctx->kl_part, ctx->kl_ls, ctx->As, ctx->wd, ctx->didx, ctx->sp_ptr,
                  ctx->sp_pq, ctx->sp_row, ctx->sp_coef, ctx->kl_spart, ctx->lam, ctx->dlam, ctx->pd_rc,
                  ctx->pd_w, ctx->pd_rhs, ctx->pd_d1, ctx->pd_R0, ctx->pd_R1, ctx->pd_R2, ctx->pd_tmp, ctx->pd_part_rows,
                  ctx->pd_part_cols, ctx->pd_out, ctx->qrows, ctx->qslot, ctx->Pq, ctx->qPx, ctx->qPs,
                  ctx->qextra, ctx->qf, ctx->aff_F, ctx->aff_z0, ctx->ls_paux, ctx->cabs, ctx->eabs, ctx->Pxa,
                  ctx->Psa, ctx->xtr, ctx->Pxtr, ctx->c_tr, ctx->d_tr, ctx->invd_tr, ctx->w_tr, ctx->logd_tr,
                  ctx->klp_lx, ctx->klp_g0, ctx->klp_hd, ctx->klp_ab, ctx->klp_lxt, ctx->klp_part, ctx->klp_ls,
                  ctx->kl_vabs, ctx->kl_uabs, ctx->kl_vtr, ctx->kl_ytr, ctx->qPxa, ctx->qPsa, ctx->qfabs, ctx->qPx_tr,
                  ctx->qextra_tr, ctx->x1, ctx->c1, ctx->d1, ctx->invd1, ctx->w1, ctx->logd1, ctx->cabs1,
                  ctx->pd_nu, ctx->pd_dnu, ctx->pd_rp, ctx->pd_adx, ctx->pd_R0e, ctx->pd_R1e, ctx->pd_part_eq};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  for (void* p : {(void*)ctx->kY, (void*)ctx->kYg, (void*)ctx->kgram, (void*)ctx->kS, (void*)ctx->kzp,
                  (void*)ctx->sL, (void*)ctx->sLinv, (void*)ctx->sw, (void*)ctx->s_tasks, (void*)ctx->s_work,
                  (void*)ctx->s_bwd, (void*)ctx->ruiz_work})
    if (p) (void)hipFree(p);
  if (ctx->hctrl) (void)hipHostFree(ctx->hctrl);
  if (ctx->hflag) (void)hipHostFree(ctx->hflag);
  if (ctx->hls) (void)hipHostFree(ctx->hls);
  if (ctx->pd_hout) (void)hipHostFree(ctx->pd_hout);
  for (auto& slot : ctx->tm.ev)
    for (auto& pr : slot)
      for (hipEvent_t e : pr)
        if (e) (void)hipEventDestroy(e);
  if (ctx->s2) (void)hipStreamSynchronize(ctx->s2);
  if (ctx->s3) (void)hipStreamSynchronize(ctx->s3);
  for (void* p : {(void*)ctx->L2, (void*)ctx->Linv2, (void*)ctx->rhs2, (void*)ctx->df_work2, (void*)ctx->ctrl2})
    if (p) (void)hipFree(p);
  for (hipEvent_t e : {ctx->ev_p0, ctx->ev_p1})
    if (e) (void)hipEventDestroy(e);
  if (ctx->s3) (void)hipStreamDestroy(ctx->s3);
  if (ctx->spart) (void)hipFree(ctx->spart);
  for (hipEvent_t e : {ctx->ev_w, ctx->ev_h})
    if (e) (void)hipEventDestroy(e);
  if (ctx->s2) (void)hipStreamDestroy(ctx->s2);
  if (ctx->s) (void)hipStreamDestroy(ctx->s);
  delete ctx;
}

int cvxg_set_objective(cvxg_ctx* ctx, const double* P, int ldP, const double* a, double r) {
  if (!ctx || !a) return CVXG_E_ARG;
  HIPC(ctx, hipSetDevice(ctx->dev));
  const int n = ctx->n, np = ctx->np;
  if (P) {
    if (ldP < n) return set_err(ctx, CVXG_E_DIM, "ldP < n");
    if (!ctx->P) CHK(dalloc(ctx, &ctx->P, (size_t)np * np));
    CHK(upload_mat(ctx, ctx->P, np, np, P, n, n, ldP, 1));  // symmetric: either layout
    ctx->hasP = 1;
  } else {
    ctx->hasP = 0;
  }
  CHK(upload_vec(ctx, ctx->a0, a, n, np));
  ctx->r0 = r;
  ctx->kl = 0;
  ctx->klp = 0;
  ctx->have_obj = 1;
  ctx->x_eval_valid = 0;
  return CVXG_OK;
}

int cvxg_set_objective_kl(cvxg_ctx* ctx, const double* B, int ldB, int row_major, int nout, const double* w,
                          double R) {
  if (!ctx || !B || !w || nout <= 0) return CVXG_E_ARG;
  HIPC(ctx, hipSetDevice(ctx->dev));
  const int n = ctx->n, np = ctx->np;
  if (ldB < (row_major ? nout : n)) return set_err(ctx, CVXG_E_DIM, "ldB too small");
  const int noutp = round_up(nout, MPAD);
  if (noutp != ctx->noutp) {
    for (double** v : {&ctx->KB, &ctx->kl_v, &ctx->kl_y, &ctx->kl_u, &ctx->kl_negBy, &ctx->kl_part, &ctx->kl_ls,
                       &ctx->kl_vabs, &ctx->kl_uabs, &ctx->kl_vtr, &ctx->kl_ytr})
      if (*v) (void)hipFree(*v), *v = nullptr;
    CHK(dalloc(ctx, &ctx->KB, (size_t)noutp * np));
    for (double** v : {&ctx->kl_v, &ctx->kl_y, &ctx->kl_u, &ctx->kl_vabs, &ctx->kl_uabs, &ctx->kl_vtr, &ctx->kl_ytr})
      CHK(dalloc(ctx, v, noutp));
    CHK(dalloc(ctx, &ctx->kl_negBy, np));
    CHK(dalloc(ctx, &ctx->kl_part, std::max((size_t)coldot_chunks(noutp) * np,
                                            (size_t)ls_kl_blocks(noutp) * 2 * LS_TRIALS)));
    CHK(dalloc(ctx, &ctx->kl_ls, 2 * LS_TRIALS));
  }
  // KB = B' (nout x n): B row-major (ldB) is B' column-major with the same ld, and vice versa
  CHK(upload_mat(ctx, ctx->KB, np, noutp, B, nout, n, ldB, row_major ? 0 : 1));
  if (!ctx->P) CHK(dalloc(ctx, &ctx->P, (size_t)np * np));
  ctx->hasP = 1;  // the KL Hessian B diag(y) B' is assembled into P every step
  {
    const int rest = ctx->ntiles - ctx->ntiles_main;
    const int ns = syrk_nsplit(ctx, noutp / KC);
    if (rest > 0 && (ns != ctx->kl_nsplit || !ctx->kl_spart)) {
      if (ctx->kl_spart) (void)hipFree(ctx->kl_spart), ctx->kl_spart = nullptr;
      CHK(dalloc(ctx, &ctx->kl_spart, (size_t)ns * rest * TILE * TILE));
    }
    ctx->kl_nsplit = ns;
  }
  CHK(upload_vec(ctx, ctx->a0, w, n, np));
  ctx->r0 = 0.0;
  ctx->kl = 1;
  ctx->klp = 0;
  ctx->nout = nout;
  ctx->noutp = noutp;
  ctx->kl_R = R;
  ctx->have_obj = 1;
  ctx->x_eval_valid = 0;
  return CVXG_OK;
}

int cvxg_set_objective_kl_primal(cvxg_ctx* ctx, int nout) {
  if (!ctx || nout <= 0) return CVXG_E_ARG;
  HIPC(ctx, hipSetDevice(ctx->dev));
  const int np = ctx->np;
  if (!ctx->klp_lx) {
    for (double** v : {&ctx->klp_lx, &ctx->klp_g0, &ctx->klp_hd, &ctx->klp_ab, &ctx->klp_lxt}) CHK(dalloc(ctx, v, np));
    CHK(dalloc(ctx, &ctx->klp_part, (size_t)ls_klp_blocks(ctx->n) * 2 * LS_TRIALS));
    CHK(dalloc(ctx, &ctx->klp_ls, 2 * LS_TRIALS));
  }
  HIPC(ctx, hipMemsetAsync(ctx->a0, 0, (size_t)np * sizeof(double), ctx->s));  // no linear term: g = (0 + g0) t
  HIPC(ctx, hipStreamSynchronize(ctx->s));
  ctx->klp_n = (double)nout;  // Dist_KL: n.toDouble in x*n, log(n) in the gradient
  ctx->r0 = 0.0;
  ctx->hasP = 0;
  ctx->kl = 0;
  ctx->klp = 1;
  ctx->have_obj = 1;
  ctx->x_eval_valid = 0;
  return CVXG_OK;
}

// Split the constraint rows into dense rows (packed into As for the SYRK) and sparse rows (at most SPARSE_NNZ
// nonzeros), whose lower-triangle Hessian entries are listed per entry (p, q) with the rows in list order.
static constexpr int SPARSE_NNZ = 4;
static int plan_sparse_rows(cvxg_ctx* ctx, const double* A, int ldA, int row_major) {
  const int n = ctx->n, m = ctx->m;
  for (void** p : {(void**)&ctx->As, (void**)&ctx->wd, (void**)&ctx->didx, (void**)&ctx->sp_ptr, (void**)&ctx->sp_pq,
                   (void**)&ctx->sp_row, (void**)&ctx->sp_coef}) {
    if (*p) (void)hipFree(*p);
    *p = nullptr;
  }
  ctx->have_sparse = 0;
  ctx->sp_T = 0;
  ctx->nsplit = syrk_nsplit(ctx, ctx->mp / KC);
  if (!ctx->sparse_rows && ctx->nq == 0) return CVXG_OK;
  auto at = [&](int i, int j) { return row_major ? A[(size_t)i * ldA + j] : A[(size_t)j * ldA + i]; };
  struct Term {
    int p, q, row;
    double coef;
  };
  std::vector<Term> terms;
  std::vector<int> dense;
  std::vector<int> nzc;
  std::vector<double> nzv;
  for (int i = 0; i < m; ++i) {
    nzc.clear();
    nzv.clear();
    for (int j = 0; j < n && (int)nzc.size() <= SPARSE_NNZ; ++j) {
      const double v = at(i, j);
      if (v != 0.0) {
        nzc.push_back(j);
        nzv.push_back(v);
      }
    }
    if (!ctx->sparse_rows || (int)nzc.size() > SPARSE_NNZ || (!ctx->is_quad.empty() && ctx->is_quad[i])) {
      dense.push_back(i);  // QuadraticConstraint rows are always dense: their SYRK row G = a + P x changes with x
      continue;
    }
    for (size_t a = 0; a < nzc.size(); ++a)  // lower entries: p = nzc[a] >= q = nzc[b]
      for (size_t b = 0; b <= a; ++b) terms.push_back({nzc[a], nzc[b], i, nzv[a] * nzv[b]});
  }
  if ((int)dense.size() == m && ctx->nq == 0) return CVXG_OK;  // no sparse rows: the SYRK keeps using A itself
  std::stable_sort(terms.begin(), terms.end(),
                   [](const Term& x, const Term& y) { return x.p != y.p ? x.p < y.p : x.q < y.q; });
  std::vector<int> ptr, pq, row;
  std::vector<double> coef;
  for (size_t e = 0; e < terms.size(); ++e) {
    if (e == 0 || terms[e].p != terms[e - 1].p || terms[e].q != terms[e - 1].q) {
      ptr.push_back((int)e);
      pq.push_back(terms[e].p);
      pq.push_back(terms[e].q);
    }
    row.push_back(terms[e].row);
    coef.push_back(terms[e].coef);
  }
  ptr.push_back((int)terms.size());
  ctx->sp_T = (int)pq.size() / 2;
  ctx->ndense = (int)dense.size();
  ctx->mdp = std::max(round_up(ctx->ndense, MPAD), MPAD);
  const size_t np = ctx->np;
  CHK(dalloc(ctx, &ctx->As, (size_t)ctx->mdp * np));
  CHK(dalloc(ctx, &ctx->wd, ctx->mdp));
  CHK(dalloc(ctx, &ctx->didx, std::max(ctx->ndense, 1)));
  {
    std::vector<double> h((size_t)ctx->mdp * np, 0.0);
    for (int r = 0; r < ctx->ndense; ++r)
      for (int j = 0; j < n; ++j) h[(size_t)r * np + j] = at(dense[r], j);
    CHK(copy_sync(ctx, ctx->As, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice));
    if (ctx->ndense) CHK(copy_sync(ctx, ctx->didx, dense.data(), dense.size() * sizeof(int), hipMemcpyHostToDevice));
  }
  if (ctx->sp_T > 0) {
    CHK(dalloc(ctx, &ctx->sp_ptr, ptr.size()));
    CHK(dalloc(ctx, &ctx->sp_pq, pq.size()));
    CHK(dalloc(ctx, &ctx->sp_row, row.size()));
    CHK(dalloc(ctx, &ctx->sp_coef, coef.size()));
    CHK(copy_sync(ctx, ctx->sp_ptr, ptr.data(), ptr.size() * sizeof(int), hipMemcpyHostToDevice));
    CHK(copy_sync(ctx, ctx->sp_pq, pq.data(), pq.size() * sizeof(int), hipMemcpyHostToDevice));
    CHK(copy_sync(ctx, ctx->sp_row, row.data(), row.size() * sizeof(int), hipMemcpyHostToDevice));
    CHK(copy_sync(ctx, ctx->sp_coef, coef.data(), coef.size() * sizeof(double), hipMemcpyHostToDevice));
  }
  if (ctx->nq > 0) {  // As row of each quadratic constraint
    std::vector<int> slot(ctx->nq);
    for (int k = 0; k < ctx->nq; ++k)
      slot[k] = (int)(std::lower_bound(dense.begin(), dense.end(), ctx->qrows_h[k]) - dense.begin());
    if (ctx->qslot) (void)hipFree(ctx->qslot);
    CHK(dalloc(ctx, &ctx->qslot, ctx->nq));
    CHK(copy_sync(ctx, ctx->qslot, slot.data(), slot.size() * sizeof(int), hipMemcpyHostToDevice));
  }
  ctx->have_sparse = 1;
  ctx->nsplit = syrk_nsplit(ctx, ctx->mdp / KC);
  return CVXG_OK;
}

int cvxg_set_ineq(cvxg_ctx* ctx, const double* A, int ldA, int row_major, const double* r, const double* ub) {
  if (!ctx || (ctx->m > 0 && (!A || !r || !ub))) return CVXG_E_ARG;
  HIPC(ctx, hipSetDevice(ctx->dev));
  const int n = ctx->n, m = ctx->m;
  if (m > 0) {
    if (ldA < (row_major ? n : m)) return set_err(ctx, CVXG_E_DIM, "ldA too small");
    CHK(upload_mat(ctx, ctx->A, ctx->np, ctx->mp, A, m, n, ldA, row_major));
    std::vector<double> rr(ctx->mp, 0.0), uu(ctx->mp, 1.0);
    memcpy(rr.data(), r, m * sizeof(double));
    memcpy(uu.data(), ub, m * sizeof(double));
    CHK(copy_sync(ctx, ctx->r, rr.data(), ctx->mp * sizeof(double), hipMemcpyHostToDevice));
    CHK(copy_sync(ctx, ctx->ub, uu.data(), ctx->mp * sizeof(double), hipMemcpyHostToDevice));
    ctx->nq = 0;  // a new constraint list: quadratic rows are declared again with cvxg_set_quad
    ctx->is_quad.clear();
    CHK(plan_sparse_rows(ctx, A, ldA, row_major));
  }
  ctx->have_ineq = 1;
  ctx->x_eval_valid = 0;
  return CVXG_OK;
}

int cvxg_set_quad(cvxg_ctx* ctx, int q, const int* rows, const double* P, int ldP) {
  if (!ctx || q < 0 || (q > 0 && (!rows || !P))) return CVXG_E_ARG;
  if (!ctx->have_ineq) return set_err(ctx, CVXG_E_ARG, "cvxg_set_quad: call cvxg_set_ineq first");
  HIPC(ctx, hipSetDevice(ctx->dev));
  const int n = ctx->n, m = ctx->m;
  const size_t np = ctx->np;
  if (ldP < n) return set_err(ctx, CVXG_E_DIM, "ldP too small");
  std::vector<int> rs(rows, rows + q);
  for (int k = 0; k < q; ++k) {
    if (rs[k] < 0 || rs[k] >= m) return set_err(ctx, CVXG_E_DIM, "quadratic constraint row %d out of range", rs[k]);
    if (k > 0 && rs[k] <= rs[k - 1]) return set_err(ctx, CVXG_E_ARG, "quadratic constraint rows must ascend");
  }
  for (double** v : {&ctx->Pq, &ctx->qPx, &ctx->qPs, &ctx->qextra, &ctx->qf, &ctx->qPxa, &ctx->qPsa, &ctx->qfabs,
                     &ctx->qPx_tr, &ctx->qextra_tr})
    if (*v) (void)hipFree(*v), *v = nullptr;
  if (ctx->qrows) (void)hipFree(ctx->qrows), ctx->qrows = nullptr;
  ctx->nq = q;
  ctx->qrows_h = rs;
  ctx->is_quad.assign(m, 0);
  for (int r : rs) ctx->is_quad[r] = 1;
  if (q > 0) {
    CHK(dalloc(ctx, &ctx->Pq, (size_t)q * np * np));
    for (int k = 0; k < q; ++k)
      CHK(upload_mat(ctx, ctx->Pq + (size_t)k * np * np, (int)np, (int)np, P + (size_t)k * n * ldP, n, n, ldP, 1));
    CHK(dalloc(ctx, &ctx->qrows, q));
    CHK(copy_sync(ctx, ctx->qrows, rs.data(), q * sizeof(int), hipMemcpyHostToDevice));
    CHK(dalloc(ctx, &ctx->qPx, (size_t)q * np));
    CHK(dalloc(ctx, &ctx->qPs, (size_t)q * np));
    CHK(dalloc(ctx, &ctx->qextra, ctx->mp));  // zero on the linear rows
    CHK(dalloc(ctx, &ctx->qf, ctx->mp));
    for (double** v : {&ctx->qPxa, &ctx->qPsa, &ctx->qPx_tr}) CHK(dalloc(ctx, v, (size_t)q * np));
    CHK(dalloc(ctx, &ctx->qextra_tr, ctx->mp));
    CHK(dalloc(ctx, &ctx->qfabs, ctx->mp));
  }
  // re-split the rows (quadratic rows are dense SYRK rows with a changing gradient): A back from the device
  std::vector<double> hA((size_t)ctx->mp * np);
  CHK(copy_sync(ctx, hA.data(), ctx->A, hA.size() * sizeof(double), hipMemcpyDeviceToHost));
  CHK(plan_sparse_rows(ctx, hA.data(), (int)np, 1));
  ctx->x_eval_valid = 0;
  return CVXG_OK;
}

int cvxg_set_eq(cvxg_ctx* ctx, const double* Aeq, int ldAeq, int row_major, const double* beq) {
  if (!ctx) return CVXG_E_ARG;
  if (ctx->p == 0) return CVXG_OK;
  if (!Aeq || !beq) return CVXG_E_ARG;
  HIPC(ctx, hipSetDevice(ctx->dev));
  const int pe = std::max(ctx->p, CVXG_MAX_EQ);
  CHK(upload_mat(ctx, ctx->Aeq, ctx->np, pe, Aeq, ctx->p, ctx->n, ldAeq, row_major));
  std::vector<double> b(pe, 0.0);
  memcpy(b.data(), beq, ctx->p * sizeof(double));
  CHK(copy_sync(ctx, ctx->beq, b.data(), pe * sizeof(double), hipMemcpyHostToDevice));
  ctx->have_eq = 1;
  ctx->x_eval_valid = 0;
  return CVXG_OK;
}

int cvxg_set_x(cvxg_ctx* ctx, const double* x) {
  if (!ctx || !x) return CVXG_E_ARG;
  HIPC(ctx, hipSetDevice(ctx->dev));
  CHK(upload_vec(ctx, ctx->x, x, ctx->n, ctx->np));
  ctx->x_eval_valid = 0;
  return CVXG_OK;
}

int cvxg_get_x(cvxg_ctx* ctx, double* x) {
  if (!ctx || !x) return CVXG_E_ARG;
  HIPC(ctx, hipSetDevice(ctx->dev));
  HIPC(ctx, hipMemcpyAsync(x, ctx->x, ctx->n * sizeof(double), hipMemcpyDeviceToHost, ctx->s));
  HIPC(ctx, hipStreamSynchronize(ctx->s));
  return CVXG_OK;
}

static int check_ready(cvxg_ctx* ctx) {
  if (!ctx->have_obj || !ctx->have_ineq || (ctx->p > 0 && !ctx->have_eq))
    return set_err(ctx, CVXG_E_ARG, "objective / inequalities / equalities not set");
  return CVXG_OK;
}

static int set_t(cvxg_ctx* ctx, double t) {
  if (ctx->t != t) ctx->x_eval_valid = 0;
  ctx->t = t;
  launch_ctrl_set(ctx->s, ctx->ctrl, 0, t);
  HIPC(ctx, hipGetLastError());
  return CVXG_OK;
}

int cvxg_barrier_eval(cvxg_ctx* ctx, double t, const double* x, double* f, double* g, double* H) {
  if (!ctx || !x) return CVXG_E_ARG;
  HIPC(ctx, hipSetDevice(ctx->dev));
  CHK(check_ready(ctx));
  CHK(cvxg_set_x(ctx, x));
  CHK(set_t(ctx, t));
  CHK(eval_at_x(ctx));
  if (f) *f = ctx->f_at_x;
  if (g) CHK(copy_sync(ctx, g, ctx->y, ctx->n * sizeof(double), hipMemcpyDeviceToHost));
  if (H) {
    CHK(assemble_hessian(ctx));
    HIPC(ctx, hipMemcpy2DAsync(H, ctx->n * sizeof(double), ctx->H, ctx->np * sizeof(double), ctx->n * sizeof(double),
                               ctx->n, hipMemcpyDeviceToHost, ctx->s));
    HIPC(ctx, hipStreamSynchronize(ctx->s));
  }
  return CVXG_OK;
}

int cvxg_constraint_values(cvxg_ctx* ctx, const double* x, double* gx) {
  if (!ctx || !x || !gx) return CVXG_E_ARG;
  HIPC(ctx, hipSetDevice(ctx->dev));
  CHK(cvxg_set_x(ctx, x));
  launch_ctrl_reset_eval(ctx->s, ctx->ctrl);
  constraint_eval_all(ctx);
  HIPC(ctx, hipGetLastError());
  HIPC(ctx, hipMemcpyAsync(gx, ctx->c, ctx->m * sizeof(double), hipMemcpyDeviceToHost, ctx->s));
  HIPC(ctx, hipStreamSynchronize(ctx->s));
  ctx->x_eval_valid = 0;
  return CVXG_OK;
}

int cvxg_active_set(cvxg_ctx* ctx, const double* x, double tol, int* idx, int* count) {
  if (!ctx || !x || !count) return CVXG_E_ARG;
  std::vector<double> g(ctx->m), ub(ctx->m);
  CHK(cvxg_constraint_values(ctx, x, g.data()));
  CHK(copy_sync(ctx, ub.data(), ctx->ub, ctx->m * sizeof(double), hipMemcpyDeviceToHost));
  int k = 0;
  for (int i = 0; i < ctx->m; ++i)
    if (fabs(g[i] - ub[i]) < tol) {  // Constraint.isActive, Constraint.scala:26
      if (idx) idx[k] = i;
      ++k;
    }
  *count = k;
  return CVXG_OK;
}

int cvxg_newton_direction(cvxg_ctx* ctx, const cvxg_params* pars, double t, const double* x, const double* grad,
                          double* dx, double* w, cvxg_step_info* info) {
  if (!ctx || !pars || !x) return CVXG_E_ARG;
  HIPC(ctx, hipSetDevice(ctx->dev));
  CHK(check_ready(ctx));
  cvxg_step_info tmp;
  if (!info) info = &tmp;
  memset(info, 0, sizeof(*info));
  CHK(cvxg_set_x(ctx, x));
  CHK(set_t(ctx, t));
  CHK(eval_at_x(ctx));
  if (grad) {  // caller-supplied gradient (e.g. the host's y of UnconstrainedSolver.scala:44,131)
    std::vector<double> g(grad, grad + ctx->n);
    double gg = 0.0;
    for (double v : g) gg += v * v;
    CHK(upload_vec(ctx, ctx->y, g.data(), ctx->n, ctx->np));
    ctx->normGrad = sqrt(gg);
    ctx->x_eval_valid = 0;
  }
  info->t = t;
  info->f = ctx->f_at_x;
  info->norm_grad = ctx->normGrad;
  int rc = newton_direction(ctx, pars, info);
  if (rc != CVXG_OK) return rc;
  info->q = ctx->hctrl->sc[SC_Q];
  info->newton_decrement = -info->q / 2;
  if (dx) CHK(copy_sync(ctx, dx, ctx->dx, ctx->n * sizeof(double), hipMemcpyDeviceToHost));
  if (w && ctx->p > 0) CHK(copy_sync(ctx, w, ctx->kw, ctx->p * sizeof(double), hipMemcpyDeviceToHost));
  return CVXG_OK;
}

int cvxg_centering_begin(cvxg_ctx* ctx, double t) {
  if (!ctx) return CVXG_E_ARG;
  HIPC(ctx, hipSetDevice(ctx->dev));
  CHK(check_ready(ctx));
  CHK(set_t(ctx, t));
  ctx->iter = 0;
  ctx->trust = NAN;
  ctx->spec_t = 1.0;
  ctx->began = 1;
  CHK(eval_at_x(ctx));  // y = objF.gradientAt(x); normGrad; eqDiff   (UnconstrainedSolver.scala:44-46)
  ctx->nd = std::numeric_limits<double>::infinity();  // set to tol + 1 by the first cvxg_newton_step
  return CVXG_OK;
}

int cvxg_centering_resume(cvxg_ctx* ctx, double t, int iter, double trust_radius, const double* grad) {
  if (!ctx || iter < 0) return CVXG_E_ARG;
  HIPC(ctx, hipSetDevice(ctx->dev));
  CHK(check_ready(ctx));
  CHK(set_t(ctx, t));
  ctx->iter = iter;
  ctx->trust = iter == 0 ? NAN : trust_radius;
  ctx->spec_t = 1.0;
  ctx->began = 1;
  CHK(eval_at_x(ctx));
  if (grad) {  // the host's y (UnconstrainedSolver.scala:44,131): replaces the engine's gradient for this iteration
    double gg = 0.0;
    for (int i = 0; i < ctx->n; ++i) gg += grad[i] * grad[i];
    CHK(upload_vec(ctx, ctx->y, grad, ctx->n, ctx->np));
    ctx->normGrad = sqrt(gg);
  }
  ctx->nd = std::numeric_limits<double>::infinity();  // tol + 1 at the next cvxg_newton_step
  return CVXG_OK;
}

int cvxg_newton_step(cvxg_ctx* ctx, const cvxg_params* pars, cvxg_step_info* info) {
  if (!ctx || !pars) return CVXG_E_ARG;
  HIPC(ctx, hipSetDevice(ctx->dev));
  if (!ctx->began) return set_err(ctx, CVXG_E_ARG, "cvxg_newton_step before cvxg_centering_begin");
  cvxg_step_info tmp;
  if (!info) info = &tmp;
  memset(info, 0, sizeof(*info));
  info->t = ctx->t;
  info->iter = ctx->iter;
  if (ctx->nd == std::numeric_limits<double>::infinity()) ctx->nd = pars->tolSolver + 1;
  if (!loop_cond(ctx, pars)) {
    info->done = 1;
    info->newton_decrement = ctx->nd;
    info->norm_grad = ctx->normGrad;
    return CVXG_OK;
  }
  if (!ctx->x_eval_valid) CHK(eval_at_x(ctx, true, false, /*ahead=*/false));
  const double tol = pars->tolSolver;
  info->f = ctx->f_at_x;
  info->norm_grad = ctx->normGrad;
  ctx->spec_allowed = ctx->p == 0 && ctx->m > 0 && !ctx->kl && !ctx->klp;
  ctx->spec_beta = pars->beta;
  ctx->spec_have = false;
  ctx->spec_eval_have = false;
  int rc = newton_direction(ctx, pars, info);
  ctx->spec_allowed = false;
  const bool spec = ctx->spec_have;
  const bool spec_eval = spec && ctx->spec_eval_have;
  ctx->spec_have = false;
  ctx->spec_eval_have = false;
  if (rc != CVXG_OK) return rc;
  const double q = ctx->hctrl->sc[SC_Q];
  ctx->nd = -q / 2;
  info->q = q;
  info->newton_decrement = ctx->nd;
  if (ctx->nd > tol) {
    double scale = 1.0;
    int limit = 100;
    if (ctx->p == 0) {
      // trust region: rho = 1+1/4 == 1 (integer), radius frozen at |d_0|_H  (UnconstrainedSolver.scala:86-101)
      const double hNorm = sqrt(-q);
      if (ctx->iter == 0) ctx->trust = hNorm;
      info->hnorm = hNorm;
      info->trust_radius = ctx->trust;
      if (!(ctx->iter == 0 || hNorm <= ctx->trust)) scale = ctx->trust / hNorm;
      limit = 200;
    }
    const bool use_spec = spec && scale == 1.0;  // s = dx: the setup and first batch are already on the host
    if (!use_spec) tstart(ctx, 4);  // (else phase 4 began with the speculative launches)
    if (use_spec) {
    } else if (scale == 1.0) {
      launch_axpy_strided(ctx->s, nullptr, ctx->dx, 1, 0, 1.0, ctx->np, ctx->sdir);  // s = dx (a kernel: no blit gap)
    } else {
      launch_axpy_strided(ctx->s, nullptr, ctx->dx, 1, 0, scale, ctx->np, ctx->sdir);  // d * (radius/hNorm)
    }
    double tacc = 1.0;
    int kc = 0, ka = 0, fresh = 0, ties = 0;
    rc = line_search(ctx, pars, q, limit, &tacc, &kc, &ka, &fresh, &ties, use_spec);
    info->ls_fresh = fresh;
    info->ls_ties = ties;
    tstop(ctx, 4);
    if (rc != CVXG_OK) return rc;
    const bool taken = use_spec && spec_eval && tacc == ctx->spec_t_used;
    if (taken) std::swap(ctx->x, ctx->x1);  // x1 = x + s*t, formed (bitwise as below) before the host read
    else launch_axpy(ctx->s, ctx->x, ctx->sdir, tacc, ctx->np, ctx->x);  // x = x + s*t
    ctx->spec_t = scale == 1.0 ? tacc : 1.0;  // the next step's guess (s = dx there)
    HIPC(ctx, hipGetLastError());
    info->step = tacc;
    info->backtracks_c = kc;
    info->backtracks_armijo = ka;
    info->took_step = 1;
    // y = objF.gradientAt(x); normGrad (and eqDiff); the next step's assembly goes out behind the constraint values
    // when the loop will go on (UnconstrainedSolver.scala:38-41: iter + 1 < maxIter and this step's decrement > tol;
    // only normGrad <= tol, which the evaluation decides, could end it -- then the assembly is dropped)
    rc = eval_at_x(ctx, ctx->iter + 1 < pars->maxIter && ctx->nd > tol, taken);
    if (rc != CVXG_OK) return rc;
  }
  ctx->iter += 1;
  info->norm_grad_new = ctx->normGrad;
  info->equality_gap = ctx->eqGap;
  info->done = loop_cond(ctx, pars) ? 0 : 1;
  timing_collect(ctx);
  return CVXG_OK;
}

int cvxg_centering(cvxg_ctx* ctx, const cvxg_params* pars, double t, cvxg_centering_info* info) {
  if (!ctx || !pars) return CVXG_E_ARG;
  CHK(cvxg_centering_begin(ctx, t));
  cvxg_step_info si;
  while (true) {
    CHK(cvxg_newton_step(ctx, pars, &si));
    if (si.done) break;
  }
  if (info) {
    info->iter = ctx->iter;
    info->maxed_out = ctx->iter >= pars->maxIter;
    info->newton_decrement = ctx->nd;
    info->norm_grad = ctx->normGrad;
    info->equality_gap = ctx->eqGap;
  }
  return CVXG_OK;
}

int cvxg_barrier_solve(cvxg_ctx* ctx, const cvxg_params* pars, int termination, cvxg_solution* sol) {
  if (!ctx || !pars) return CVXG_E_ARG;
  HIPC(ctx, hipSetDevice(ctx->dev));
  CHK(check_ready(ctx));
  // assert(C.isInSet(startingPoint))  (BarrierSolver.scala:35)
  CHK(set_t(ctx, 1.0));
  int rc = eval_at_x(ctx);
  if (rc != CVXG_OK || ctx->hctrl->not_strict > 0)
    return set_err(ctx, CVXG_E_INFEASIBLE_X, "Starting point x not in set C");
  const double mu = 10.0;  // BarrierSolver.scala:73
  double t = 1.0;
  double gap = INFINITY, eqgap = INFINITY, fval = 1.7976931348623157e308;
  bool eq_defined = false;  // OptimizationState.equalityGap: None before the first pass without EQs
  const double maxIter = 1000 / mu;
  int outer = 0, total = 0;
  cvxg_centering_info ci{};
  auto tc = [&]() -> bool {
    if (termination == 1)  // CvxUtils.phase_I_TerminationCriterion
      return fval < 0 && (!eq_defined || eqgap < 1e-6);
    return gap < pars->tolSolver && (!eq_defined || eqgap < pars->tolSolver);  // standardTerminationCriterion
  };
  if (ctx->p > 0) eq_defined = true;  // solveWithEQs starts with Some(equalityGap = MaxValue)
  while (!tc() && outer < maxIter) {
    CHK(cvxg_centering(ctx, pars, t, &ci));
    total += ci.iter;
    fval = objective_at_x(ctx);  // objF.valueAt(x) at the centred point
    gap = ctx->m / t;            // dualityGap = numConstraints/t
    eqgap = ctx->p > 0 ? ci.equality_gap : 0.0;
    eq_defined = true;
    t = mu * t;
    ++outer;
  }
  if (sol) {
    sol->duality_gap = gap;
    sol->equality_gap = eqgap;
    sol->newton_decrement = ci.newton_decrement;
    sol->norm_grad = ci.norm_grad;
    sol->objective = fval;
    sol->iter = ci.iter;
    sol->maxed_out = ci.maxed_out;
    sol->outer_iters = outer;
    sol->newton_steps = total;
  }
  return CVXG_OK;
}

// ---- config C5 in one host process (SURVEY.md §8b cvxg_batch_*): independent contexts, one host thread each --------
// Each context owns its device, stream and buffers, so the solves run concurrently with no exchange; a context is only
// ever touched by the one thread that runs it (the contexts are not thread-safe, the batch is).  status[i] = the
// context's own return code; the call returns the first non-zero one (CVXG_OK when all succeed).
extern "C++" {
template <class F>
static int batch_run(int count, cvxg_ctx* const* ctxs, int* status, F one) {
  if (count < 0 || (count > 0 && !ctxs)) return CVXG_E_ARG;
  bool bad = false;
  for (int i = 0; i < count; ++i)
    for (int j = 0; j <= i; ++j)
      if (!ctxs[i] || (j < i && ctxs[i] == ctxs[j])) bad = true;  // one thread per distinct context
  if (bad) {  // nothing ran: every status says so (a caller reading status[] alone must not see success)
    if (status)
      for (int i = 0; i < count; ++i) status[i] = CVXG_E_ARG;
    return CVXG_E_ARG;
  }
  std::vector<int> rc(count, CVXG_OK);
  std::vector<std::thread> th;
  th.reserve(count);
  for (int i = 0; i < count; ++i) th.emplace_back([&, i]() { rc[i] = one(i); });
  for (auto& t : th) t.join();
  int first = CVXG_OK;
  for (int i = 0; i < count; ++i) {
    if (status) status[i] = rc[i];
    if (first == CVXG_OK) first = rc[i];
  }
  return first;
}
}  // extern "C++"

int cvxg_batch_barrier_solve(int count, cvxg_ctx* const* ctxs, const cvxg_params* pars, int termination,
                             cvxg_solution* sols, int* status) {
  if (!pars) return CVXG_E_ARG;
  return batch_run(count, ctxs, status,
                   [&](int i) { return cvxg_barrier_solve(ctxs[i], pars, termination, sols ? &sols[i] : nullptr); });
}

int cvxg_batch_newton_step(int count, cvxg_ctx* const* ctxs, const cvxg_params* pars, cvxg_step_info* infos,
                           int* status) {
  if (!pars) return CVXG_E_ARG;
  return batch_run(count, ctxs, status, [&](int i) {
    cvxg_step_info tmp;
    return cvxg_newton_step(ctxs[i], pars, infos ? &infos[i] : &tmp);
  });
}

int cvxg_set_timing(cvxg_ctx* ctx, int enabled) {
  if (!ctx) return CVXG_E_ARG;
  HIPC(ctx, hipSetDevice(ctx->dev));
  Timer& tm = ctx->tm;
  if (enabled && !tm.created) {
    for (auto& slot : tm.ev)
      for (auto& pr : slot)
        // timing only: no system-scope fence (its L2 writeback left a 5-10 us gap at every phase boundary)
        for (hipEvent_t& e : pr) HIPC(ctx, hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    tm.created = true;
  }
  if (enabled) {  // a fresh record: the steps from here on
    tm.steps = 0;
    tm.pf5 = false;
    for (auto& slot : tm.rec)
      for (bool& r : slot) r = false;
  }
  tm.on = enabled != 0;
  tm.all = enabled != 2;  // 1: every phase; 2: only the assembly and Cholesky phases (the bench's timed region)
  return CVXG_OK;
}

int cvxg_get_phase_times(cvxg_ctx* ctx, double* ms, int count) { return cvxg_get_phase_stats(ctx, ms, nullptr, count); }

int cvxg_get_counters(cvxg_ctx* ctx, long long* out, int count) {
  if (!ctx || !out) return CVXG_E_ARG;
  const long long v[5] = {ctx->ruiz_relaunches, ctx->spec_pairs, ctx->spec_pairs_used, ctx->n_attempts,
                          ctx->n_regularized};
  for (int i = 0; i < count && i < 5; ++i) out[i] = v[i];
  return CVXG_OK;
}

int cvxg_get_phase_stats(cvxg_ctx* ctx, double* ms, int* occurrences, int count) {
  if (!ctx || !ms) return CVXG_E_ARG;
  HIPC(ctx, hipSetDevice(ctx->dev));
  HIPC(ctx, hipStreamSynchronize(ctx->s));
  HIPC(ctx, hipStreamSynchronize(ctx->s2));
  const Timer& tm = ctx->tm;
  for (int i = 0; i < count && i < NT; ++i) {
    double sum = 0.0;
    int got = 0;
    for (int k = 1; k <= tm.steps; ++k) {  // the completed steps, newest first
      const int sl = ((tm.tick - k) % TRING + TRING) % TRING;
      float v = 0.f;
      if (tm.rec[sl][i] && hipEventElapsedTime(&v, tm.ev[sl][i][0], tm.ev[sl][i][1]) == hipSuccess) {
        sum += v;
        ++got;
      }
    }
    // per recorded occurrence: the first step after cvxg_set_timing may run an assembly prefetched before timing was on
    ms[i] = got > 0 ? sum / got : 0.0;
    if (occurrences) occurrences[i] = got;
  }
  (void)hipGetLastError();  // never leave a timing error sticky for the next launch check
  return CVXG_OK;
}

// ------------------------------------------------------------------------------------------------
// Primal-dual interior-point solver (PrimalDualSolver.scala, no equality constraints).  The host keeps the
// scalar loop; per iteration the device assembles H_pd with the shared SYRK (weights lambda_i/d_i), runs
// SymmetricLinearSystem's Ruiz + scaling and the shared choleskySolve pipeline, forms dlambda, and evaluates the
// residual-norm backtracking trials in batches of LS_TRIALS.
// ------------------------------------------------------------------------------------------------
static int pd_check(cvxg_ctx* ctx) {
  CHK(check_ready(ctx));
  if (ctx->kl)
    return set_err(ctx, CVXG_E_UNSUPPORTED, "primal-dual engine: quadratic, linear or KL primal objective only");
  if (ctx->m == 0) return set_err(ctx, CVXG_E_ARG, "primal-dual solver needs inequality constraints");
  if (ctx->lam) return CVXG_OK;
  const size_t np = ctx->np, mp = ctx->mp;
  for (double** v : {&ctx->lam, &ctx->dlam, &ctx->pd_rc, &ctx->pd_w}) CHK(dalloc(ctx, v, mp));
  for (double** v : {&ctx->pd_rhs, &ctx->pd_d1, &ctx->pd_R0, &ctx->pd_R1, &ctx->pd_R2, &ctx->pd_tmp})
    CHK(dalloc(ctx, v, np));
  CHK(dalloc(ctx, &ctx->pd_part_rows, (size_t)pd_row_blocks(ctx->m) * 2 * LS_TRIALS));
  CHK(dalloc(ctx, &ctx->pd_part_cols, (size_t)((ctx->n + 255) / 256) * LS_TRIALS));
  CHK(dalloc(ctx, &ctx->pd_out, 4 * LS_TRIALS));
  if (ctx->p > 0) {
    const size_t pe = std::max(ctx->p, CVXG_MAX_EQ);
    for (double** v : {&ctx->pd_nu, &ctx->pd_dnu, &ctx->pd_rp, &ctx->pd_adx}) CHK(dalloc(ctx, v, pe));
    for (double** v : {&ctx->pd_R0e, &ctx->pd_R1e}) CHK(dalloc(ctx, v, np));
    CHK(dalloc(ctx, &ctx->pd_part_eq, (size_t)((ctx->p + 255) / 256) * LS_TRIALS));
  }
  HIPC(ctx, hipHostMalloc((void**)&ctx->pd_hout, 4 * LS_TRIALS * sizeof(double), hipHostMallocDefault));
  return CVXG_OK;
}

// The objective gradient's x-dependent part at the evaluated x for the dual residual: P x, or the KL primal's
// (1 + log x) + log n (klp_g0; a0 = 0 there).
static const double* pd_grad_term(cvxg_ctx* ctx) {
  return ctx->klp ? ctx->klp_g0 : (ctx->hasP ? ctx->Px : nullptr);
}

// grad f(x) + Dg' v into out (the dual residual, :63-71): A' v, plus sum_k (P_k x) v_k over the QuadraticConstraint
// rows (their gradients a_k + P_k x; qPx from eval_at_x).  Px must hold P x.
static void pd_dual_residual(cvxg_ctx* ctx, const double* v, const double* a0, const double* Pv, double* out) {
  launch_coldot_partials(ctx->s, ctx->A, ctx->np, ctx->mp, ctx->np, v, ctx->part);
  launch_pd_finalize(ctx->s, a0, Pv, ctx->part, coldot_chunks(ctx->mp), ctx->np, out);
  if (ctx->nq > 0) launch_quad_grad(ctx->s, ctx->qPx, v, ctx->qrows, ctx->nq, ctx->np, out);
}

static int pd_delta_lambda(cvxg_ctx* ctx, double t);

// Search direction at (t, ctx->x, ctx->lam[, ctx->pd_nu]) into ctx->dx / ctx->dlam [/ ctx->pd_dnu]
// (PrimalDualSolver.scala:421-425; with equality rows :590-593).
static int pd_direction_dev(cvxg_ctx* ctx, const cvxg_params* pars, double t, cvxg_pd_step_info* info) {
  hipStream_t s = ctx->s;
  const int n = ctx->n, np = ctx->np;
  CHK(set_t(ctx, t));
  CHK(eval_at_x(ctx));  // c, d, invd, Px, y = t grad f + A'(1/d); d <= 0 fails (kktMatrix_noEqs asserts f_i < 0)
  launch_pd_rhs(s, ctx->y, t, n, np, ctx->pd_rhs);                       // rhs1 = -y / t        (:162-176)
  launch_pd_weights(s, ctx->lam, ctx->d, ctx->m, ctx->mp, ctx->pd_w);    // lambda_i / d_i      (:226-238)
  launch_ctrl_set(s, ctx->ctrl, 0, 1.0);                                 // hpd starts at objF.hessianAt(x)
  CHK(assemble_hessian(ctx, ctx->pd_w, ctx->lam));
  launch_ctrl_set(s, ctx->ctrl, 0, t);
  ctx->x_eval_valid = 0;  // y is reused below as the rhs of the shared choleskySolve
  if (ctx->p > 0) {
    // solve_withEQs (:590-593): kktSystem_withEqs (:271-285) = KKTSystem(H, A, q = rhs1 + A'nu, -(A x - b)),
    // KKTSystem.solve (H dx + A'dnu = -q, A dx = b - A x; KKTSystem.scala:43-66) -- the shared KKT path of the
    // equality-constrained barrier step (eqd = b - A x from eval_at_x).  As written: the reference's own "FIX ME"
    // (:284), q enters with the opposite sign of the no-equality system H dx = rhs1.
    launch_axpy(s, ctx->eqtmp, ctx->beq, -1.0, ctx->p, ctx->pd_rp);     // A x - b (eqtmp = A x; the KKT check reuses it)
    launch_btw_plus(s, ctx->Aeq, np, ctx->p, ctx->pd_nu, ctx->pd_rhs, n, ctx->y);  // q = rhs1 + A'nu
    HIPC(ctx, hipGetLastError());
    cvxg_step_info si;
    memset(&si, 0, sizeof(si));
    const int rc = newton_direction_kkt(ctx, pars, &si);
    info->fallback = si.fallback;
    info->regularized = si.regularized;
    info->rel_err = si.rel_err;
    info->ruiz_sweeps = si.ruiz_sweeps;
    CHK(rc);
    HIPC(ctx, hipMemcpyAsync(ctx->pd_dnu, ctx->kw, (size_t)ctx->p * sizeof(double), hipMemcpyDeviceToDevice, s));
    return pd_delta_lambda(ctx, t);
  }
  // SymmetricLinearSystem: d1 = Ruiz(H), Q = (d1 d1') o H, s = d1 o r (SymmetricLinearSystem.scala:20-23).  Q is
  // exactly symmetric (H is mirrored, d_i d_j = d_j d_i), so checkSymmetric(Q, 1e-13) holds and choleskySolve runs.
  tstart(ctx, 1);
  ruiz(ctx);
  tstop(ctx, 1);
  HIPC(ctx, hipMemcpyAsync(ctx->pd_d1, ctx->dfin, (size_t)np * sizeof(double), hipMemcpyDeviceToDevice, s));
  launch_scale_sym(s, ctx->H, np, np, ctx->pd_d1);
  launch_neg_scaled(s, ctx->pd_d1, ctx->pd_rhs, np, ctx->y);  // the pipeline solves H x = -y: y = -s
  launch_dot(s, ctx->y, nullptr, np, ctx->ctrl, SC_GG);
  HIPC(ctx, hipGetLastError());
  CHK(sync_ctrl(ctx));
  info->ruiz_sweeps = ctx->hctrl->ruiz_sweeps;
  ctx->normGrad = sqrt(ctx->hctrl->sc[SC_GG]);  // |s| for relativeSize inside choleskySolve
  cvxg_step_info si;
  memset(&si, 0, sizeof(si));
  int rc = cholesky_solve(ctx, pars->tolEqSolve, &si);  // choleskySolve(Q, s): Ruiz of Q, factor, solves, residual
  info->fallback = 0;
  info->regularized = si.regularized;
  info->rel_err = si.rel_err;
  if (rc == CVXG_E_HIP) return rc;
  if (rc != CVXG_OK) {  // any exception of choleskySolve -> symSolve(Q, s)  (SymmetricLinearSystem.scala:34)
    info->fallback = 2;
    CHK(eig_alloc(ctx));
    HIPC(ctx, hipMemsetAsync(ctx->eig_b, 0, (size_t)ctx->eig_ldm * sizeof(double), s));
    launch_axpy(s, ctx->eig_b, ctx->y, -1.0, n, ctx->eig_b);
    CHK(sym_solve(ctx, ctx->H, n, ctx->eig_b, pars->tolEqSolve));
    HIPC(ctx, hipMemsetAsync(ctx->dx, 0, (size_t)np * sizeof(double), s));
    HIPC(ctx, hipMemcpyAsync(ctx->dx, ctx->eig_x, (size_t)n * sizeof(double), hipMemcpyDeviceToDevice, s));
  }
  launch_scale_vec(s, ctx->dx, ctx->pd_d1, np, ctx->dx);  // x = d :* u  (:54)
  return pd_delta_lambda(ctx, t);
}

// deltaLambda (:184-209) with the step bound s0 and the central residual at (x, lambda); w = Dg dx (for a
// QuadraticConstraint row (a + P x).dx, with f = dx'P dx kept for the line-search trials)
static int pd_delta_lambda(cvxg_ctx* ctx, double t) {
  hipStream_t s = ctx->s;
  const int np = ctx->np;
  launch_rowdot(s, ctx->A, np, ctx->mp, np, ctx->dx, ctx->e);
  if (ctx->nq > 0) {
    launch_rowdot(s, ctx->Pq, np, ctx->nq * np, np, ctx->dx, ctx->qPs);
    launch_quad_ls(s, ctx->qPx, ctx->qPs, ctx->dx, ctx->qrows, ctx->nq, np, ctx->e, ctx->qf);
  }
  launch_pd_reset_s0(s, ctx->ctrl);
  launch_pd_dlambda(s, ctx->c, ctx->ub, ctx->lam, ctx->e, t, ctx->m, ctx->mp, ctx->dlam, ctx->pd_rc, ctx->ctrl);
  HIPC(ctx, hipGetLastError());
  return CVXG_OK;
}

// lineSearch_noEQs (PrimalDualSolver.scala:311-374) from (ctx->x, ctx->lam) along (dx, dlam); on success
// x += s dx, lambda += s dlam.  With equality rows lineSearch_withEQs (:478-543): the residual adds A'nu to the dual
// part and the primal part A x - b, nu moves with the step.  Needs ctx->c / ctx->Px at x (pd_direction_dev).
static int pd_line_search(cvxg_ctx* ctx, const cvxg_params* pars, double t, cvxg_pd_step_info* info) {
  hipStream_t s = ctx->s;
  const int n = ctx->n, np = ctx->np, p = ctx->p;
  pd_dual_residual(ctx, ctx->lam, ctx->a0, pd_grad_term(ctx), ctx->pd_R0);       // r_dual(x, lambda)
  if (ctx->hasP) launch_rowdot(s, ctx->P, np, np, np, ctx->dx, ctx->pd_tmp);     // P dx
  pd_dual_residual(ctx, ctx->dlam, nullptr, ctx->hasP ? ctx->pd_tmp : nullptr, ctx->pd_R1);
  if (ctx->nq > 0) {  // Dg(x + s dx)'(l + s dl): + s sum_k (P_k dx) l_k, + s^2 sum_k (P_k dx) dl_k
    launch_quad_grad(s, ctx->qPs, ctx->lam, ctx->qrows, ctx->nq, np, ctx->pd_R1);
    HIPC(ctx, hipMemsetAsync(ctx->pd_R2, 0, (size_t)np * sizeof(double), s));
    launch_quad_grad(s, ctx->qPs, ctx->dlam, ctx->qrows, ctx->nq, np, ctx->pd_R2);
  }
  const double* R0 = ctx->pd_R0;
  const double* R1 = ctx->pd_R1;
  if (p > 0) {  // + A'(nu + s dnu); A x_s - b = (A x - b) + s A dx
    launch_btw_plus(s, ctx->Aeq, np, p, ctx->pd_nu, ctx->pd_R0, n, ctx->pd_R0e);
    launch_btw_plus(s, ctx->Aeq, np, p, ctx->pd_dnu, ctx->pd_R1, n, ctx->pd_R1e);
    launch_rowdot(s, ctx->Aeq, np, p, np, ctx->dx, ctx->pd_adx);
    launch_dot(s, ctx->pd_rp, nullptr, p, ctx->ctrl, SC_EQ2);
    R0 = ctx->pd_R0e;
    R1 = ctx->pd_R1e;
  }
  launch_dot(s, R0, nullptr, p > 0 ? n : np, ctx->ctrl, SC_RES2);  // |r_dual(x, lambda) (+ A'nu)|^2
  const double* R0t = R0;  // the trials' constant term: with the KL primal objective only the constraint part (A'l
  if (ctx->klp) {          // (+ A'nu)); the objective's gradient at x_s is formed per trial
    pd_dual_residual(ctx, ctx->lam, nullptr, nullptr, ctx->pd_tmp);  // (no P with this objective: pd_tmp is free)
    if (p > 0) {  // (pd_rhs, rhs1 of this step's direction, is free after the solve)
      launch_btw_plus(s, ctx->Aeq, np, p, ctx->pd_nu, ctx->pd_tmp, n, ctx->pd_rhs);
      R0t = ctx->pd_rhs;
    } else {
      R0t = ctx->pd_tmp;
    }
  }
  launch_dot(s, ctx->pd_rc, nullptr, ctx->mp, ctx->ctrl, SC_RES2B);
  HIPC(ctx, hipGetLastError());
  CHK(sync_ctrl(ctx));
  double s0;
  memcpy(&s0, &ctx->hctrl->pd_s0, sizeof(s0));
  const double norm_rt =
      sqrt(ctx->hctrl->sc[SC_RES2] + ctx->hctrl->sc[SC_RES2B] + (p > 0 ? ctx->hctrl->sc[SC_EQ2] : 0.0));
  info->s0 = s0;
  info->norm_residual = norm_rt;
  const double alpha = pars->alpha, beta = pars->beta;
  const double maxIter = -30.0 / log(beta);  // a Double (:354)
  const int kmax = (int)floor(maxIter) + 1;   // the last k the while loop evaluates
  double sbase = 0.99 * s0;
  int k = 0, K = -1;
  double sK = 0.0;
  const int nout = p > 0 ? 4 : 3;
  while (K < 0) {
    launch_pd_trials(s, ctx->c, ctx->e, ctx->ub, ctx->lam, ctx->dlam, ctx->m, R0t, R1, ctx->n, sbase, beta, t,
                     ctx->pd_part_rows, ctx->pd_part_cols, ctx->pd_out, ctx->nq > 0 ? ctx->qf : nullptr,
                     ctx->nq > 0 ? ctx->pd_R2 : nullptr, ctx->pd_rp, ctx->pd_adx, p, ctx->pd_part_eq,
                     ctx->klp ? ctx->x : nullptr, ctx->klp ? ctx->dx : nullptr, ctx->klp_n);
    HIPC(ctx, hipGetLastError());
    CHK(copy_sync(ctx, ctx->pd_hout, ctx->pd_out, nout * LS_TRIALS * sizeof(double), hipMemcpyDeviceToHost));
    double sk = sbase;
    for (int j = 0; j < LS_TRIALS; ++j, ++k) {
      const double cent = ctx->pd_hout[2 * j], viol = ctx->pd_hout[2 * j + 1], dual = ctx->pd_hout[2 * LS_TRIALS + j];
      const double prim = p > 0 ? ctx->pd_hout[3 * LS_TRIALS + j] : 0.0;
      const bool ok = viol == 0.0 && sqrt(dual + cent + prim) < (1 - alpha * sk) * norm_rt;
      if (ok || k == kmax) {
        K = k;
        sK = sk;
        if (!ok) K = kmax;
        break;
      }
      sk *= beta;  // s *= beta (:358)
    }
    sbase = sk;
  }
  info->backtracks = K;
  info->step = sK;
  if (K >= maxIter) return set_err(ctx, CVXG_E_LINESEARCH, "PrimalDualSolver: Line search unsuccessful.");
  launch_axpy(s, ctx->x, ctx->dx, sK, np, ctx->x);           // x + dx*s
  launch_axpy(s, ctx->lam, ctx->dlam, sK, ctx->mp, ctx->lam);  // lambda + dLambda*s
  if (p > 0) launch_axpy(s, ctx->pd_nu, ctx->pd_dnu, sK, p, ctx->pd_nu);  // nu + dNu*s
  HIPC(ctx, hipGetLastError());
  ctx->x_eval_valid = 0;
  return CVXG_OK;
}

// gap = -h(x).lambda (:289-297) and |grad f + A' lambda| at the current (x, lambda); with equality rows (:600-606)
// the norm of the whole residual_withEqs(t, x, lambda, nu) -- t of the step just taken -- and |A x - b|.
static int pd_state(cvxg_ctx* ctx, double t, double* gap, double* norm_dual, double* eq_gap) {
  CHK(eval_at_x(ctx));
  const int p = ctx->p;
  pd_dual_residual(ctx, ctx->lam, ctx->a0, pd_grad_term(ctx), ctx->pd_R0);
  const double* R0 = ctx->pd_R0;
  if (p > 0) {
    launch_btw_plus(ctx->s, ctx->Aeq, ctx->np, p, ctx->pd_nu, ctx->pd_R0, ctx->n, ctx->pd_R0e);
    launch_pd_central(ctx->s, ctx->c, ctx->ub, ctx->lam, t, ctx->m, ctx->mp, ctx->pd_rc);
    launch_dot(ctx->s, ctx->pd_rc, nullptr, ctx->mp, ctx->ctrl, SC_PD_CENT);
    R0 = ctx->pd_R0e;
  }
  launch_dot(ctx->s, ctx->d, ctx->lam, ctx->mp, ctx->ctrl, SC_RES2B);
  launch_dot(ctx->s, R0, nullptr, p > 0 ? ctx->n : ctx->np, ctx->ctrl, SC_RES2);
  HIPC(ctx, hipGetLastError());
  CHK(sync_ctrl(ctx));
  const double* sc = ctx->hctrl->sc;
  *gap = sc[SC_RES2B];
  *norm_dual = p > 0 ? sqrt(sc[SC_RES2] + sc[SC_PD_CENT] + sc[SC_EQ2]) : sqrt(sc[SC_RES2]);
  if (eq_gap) *eq_gap = p > 0 ? sqrt(sc[SC_EQ2]) : 0.0;
  return CVXG_OK;
}

int cvxg_pd_direction(cvxg_ctx* ctx, const cvxg_params* pars, double t, const double* x, const double* lambda,
                      double* dx, double* dlambda, cvxg_pd_step_info* info) {
  if (!ctx || !pars || !x || !lambda) return CVXG_E_ARG;
  if (ctx->p > 0) return set_err(ctx, CVXG_E_ARG, "cvxg_pd_direction: equality rows present (cvxg_pd_direction_eq)");
  return cvxg_pd_direction_eq(ctx, pars, t, x, lambda, nullptr, dx, dlambda, nullptr, info);
}

int cvxg_pd_direction_eq(cvxg_ctx* ctx, const cvxg_params* pars, double t, const double* x, const double* lambda,
                         const double* nu, double* dx, double* dlambda, double* dnu, cvxg_pd_step_info* info) {
  if (!ctx || !pars || !x || !lambda || (ctx->p > 0 && !nu)) return CVXG_E_ARG;
  HIPC(ctx, hipSetDevice(ctx->dev));
  CHK(pd_check(ctx));
  cvxg_pd_step_info tmp;
  if (!info) info = &tmp;
  memset(info, 0, sizeof(*info));
  info->t = t;
  CHK(cvxg_set_x(ctx, x));
  CHK(upload_vec(ctx, ctx->lam, lambda, ctx->m, ctx->mp));
  if (ctx->p > 0) CHK(upload_vec(ctx, ctx->pd_nu, nu, ctx->p, std::max(ctx->p, CVXG_MAX_EQ)));
  CHK(pd_direction_dev(ctx, pars, t, info));
  CHK(sync_ctrl(ctx));
  memcpy(&info->s0, &ctx->hctrl->pd_s0, sizeof(double));
  if (dx) CHK(copy_sync(ctx, dx, ctx->dx, ctx->n * sizeof(double), hipMemcpyDeviceToHost));
  if (dlambda) CHK(copy_sync(ctx, dlambda, ctx->dlam, ctx->m * sizeof(double), hipMemcpyDeviceToHost));
  if (dnu && ctx->p > 0) CHK(copy_sync(ctx, dnu, ctx->pd_dnu, ctx->p * sizeof(double), hipMemcpyDeviceToHost));
  return CVXG_OK;
}

int cvxg_pd_solve(cvxg_ctx* ctx, const cvxg_params* pars, cvxg_pd_solution* sol) {
  if (!ctx || !pars) return CVXG_E_ARG;
  HIPC(ctx, hipSetDevice(ctx->dev));
  CHK(pd_check(ctx));
  const bool eqs = ctx->p > 0;
  const double tol = pars->tolSolver, mu = 10.0;
  const double m = ctx->m;
  // lambda = constraintSet.lambda(x) = -1/h (ConstraintSet.scala:116-120), gap = -h.lambda, t = mu m / gap; with
  // equality rows nu = 0 (:566-568)
  CHK(set_t(ctx, 1.0));
  CHK(eval_at_x(ctx));
  launch_pd_lambda0(ctx->s, ctx->invd, ctx->m, ctx->mp, ctx->lam);
  if (eqs) HIPC(ctx, hipMemsetAsync(ctx->pd_nu, 0, (size_t)ctx->p * sizeof(double), ctx->s));
  double gap = 0.0, norm_dual = 0.0, eq_gap = 0.0;
  CHK(pd_state(ctx, 1.0, &gap, &norm_dual, nullptr));
  norm_dual = std::numeric_limits<double>::max();  // OptimizationState(normDualResidual = Double.MaxValue)
  eq_gap = eqs ? std::numeric_limits<double>::max() : 0.0;
  double t = mu * m / gap;
  const double maxIter = (eqs ? 1500.0 : 2000.0) / mu;  // solve_withEQs :577, solve_noEQs :410
  int iter = 0;
  // sol holds the state after the last completed iteration, also when a later one fails (the reference throws)
  auto fill = [&]() {
    if (!sol) return;
    sol->duality_gap = gap;
    sol->norm_dual_residual = norm_dual;
    sol->objective = objective_at_x(ctx);
    sol->iter = iter - 1;
    sol->maxed_out = iter == (int)maxIter;
    sol->newton_steps = iter;
    sol->equality_gap = eq_gap;
  };
  fill();
  while (!(gap < tol && norm_dual < tol) && iter < maxIter) {
    cvxg_pd_step_info info;
    memset(&info, 0, sizeof(info));
    info.t = t;
    CHK(pd_direction_dev(ctx, pars, t, &info));
    CHK(pd_line_search(ctx, pars, t, &info));
    CHK(pd_state(ctx, t, &gap, &norm_dual, &eq_gap));
    t = mu * m / gap;  // JVM Double semantics: a zero gap gives +Infinity
    ++iter;
    fill();
    timing_collect(ctx);  // phase times of the last iteration (instrumentation, when enabled)
  }
  return CVXG_OK;
}

int cvxg_get_lambda(cvxg_ctx* ctx, double* lambda) {
  if (!ctx || !lambda) return CVXG_E_ARG;
  if (!ctx->lam) return set_err(ctx, CVXG_E_ARG, "no primal-dual iterate (call cvxg_pd_solve first)");
  HIPC(ctx, hipSetDevice(ctx->dev));
  return copy_sync(ctx, lambda, ctx->lam, ctx->m * sizeof(double), hipMemcpyDeviceToHost);
}

int cvxg_get_nu(cvxg_ctx* ctx, double* nu) {
  if (!ctx || !nu) return CVXG_E_ARG;
  if (ctx->p == 0 || !ctx->pd_nu)
    return set_err(ctx, CVXG_E_ARG, "no primal-dual equality multipliers (p = 0 or no cvxg_pd_solve yet)");
  HIPC(ctx, hipSetDevice(ctx->dev));
  return copy_sync(ctx, nu, ctx->pd_nu, ctx->p * sizeof(double), hipMemcpyDeviceToHost);
}

}  // extern "C"

// ------------------------------------------------------------------------------------------------
// Affine re-parametrisation x = z0 + F u (BarrierSolver.affineTransformed / reduced, BarrierSolver.scala:209-256)
// ------------------------------------------------------------------------------------------------
namespace {
// Device scratch freed on every exit path of the setup calls below.
struct DevBufs {
  std::vector<void*> p;
  template <class T>
  T* get(size_t count) {
    void* q = nullptr;
    if (hipMalloc(&q, std::max<size_t>(count, 1) * sizeof(T)) != hipSuccess) return nullptr;
    p.push_back(q);
    return (T*)q;
  }
  ~DevBufs() {
    for (void* q : p) (void)hipFree(q);
  }
};
}  // namespace

static int gerr(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

int cvxg_solution_space(int device, int p, int n, const double* A, int ldA, int row_major, const double* b,
                        double* z0, double* F, int ldF) {
  if (!A || !b || !z0 || !F) return gerr(CVXG_E_ARG, "cvxg_solution_space: null argument");
  if (p <= 0 || p >= n) return gerr(CVXG_E_DIM, "SolutionSpace: need 0 < rows(A) = %d < cols(A) = %d", p, n);
  if (ldA < (row_major ? n : p) || ldF < n) return gerr(CVXG_E_DIM, "cvxg_solution_space: leading dimension too small");
  if (hipSetDevice(device) != hipSuccess) return gerr(CVXG_E_HIP, "hipSetDevice(%d) failed", device);
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return gerr(CVXG_E_HIP, "stream create failed");
  int rc = CVXG_OK;
  {
    DevBufs B;
    const size_t nn = (size_t)n * n;
    double* M = B.get<double>(nn);
    double* Rc = B.get<double>((size_t)n * p);
    double* tau = B.get<double>(p);
    double* y = B.get<double>(p);
    double* z = B.get<double>(n);
    std::vector<double> h(nn, 0.0);
    for (int i = 0; i < p; ++i)  // column i of M = row i of A (M = A', column-major, ld n)
      for (int j = 0; j < n; ++j) h[(size_t)i * n + j] = row_major ? A[(size_t)i * ldA + j] : A[(size_t)j * ldA + i];
    std::vector<double> hR((size_t)n * p), hy(p);
    if (!M || !Rc || !tau || !y || !z) {
      rc = gerr(CVXG_E_HIP, "cvxg_solution_space: device allocation failed");
    } else if (hipMemcpyAsync(M, h.data(), nn * sizeof(double), hipMemcpyHostToDevice, s) != hipSuccess ||
               lib_qr_full(s, M, n, p, tau, Rc) != 0 ||
               hipMemcpyAsync(hR.data(), Rc, hR.size() * sizeof(double), hipMemcpyDeviceToHost, s) != hipSuccess ||
               hipStreamSynchronize(s) != hipSuccess) {
      rc = gerr(CVXG_E_HIP, "cvxg_solution_space: QR of A' failed");
    } else {
      // forwardSolve(R.t, b) (MatrixUtils.scala:383-403): L = R' is read on and below its diagonal, j ascending
      auto Lij = [&](int i, int j) { return hR[(size_t)i * n + j]; };  // L(i,j) = R(j,i) = column i, row j
      for (int i = 0; i < p && rc == CVXG_OK; ++i) {
        if (!(fabs(Lij(i, i)) > 0)) rc = gerr(CVXG_E_UNSOLVABLE, "Singular lower trianguar matrix L: zero on the diagonal");
        double acc = 0.0;
        for (int j = 0; j < i; ++j) acc += Lij(i, j) * hy[j];
        hy[i] = (b[i] - acc) / Lij(i, i);
      }
      std::vector<double> hz(n);
      if (rc == CVXG_OK &&
          (hipMemcpyAsync(y, hy.data(), p * sizeof(double), hipMemcpyHostToDevice, s) != hipSuccess ||
           lib_gemv(s, false, n, p, 1.0, M, n, y, 0.0, z) != 0 ||  // z0 = Q(:, 0 until p) y
           hipMemcpyAsync(hz.data(), z, n * sizeof(double), hipMemcpyDeviceToHost, s) != hipSuccess ||
           hipMemcpyAsync(h.data(), M, nn * sizeof(double), hipMemcpyDeviceToHost, s) != hipSuccess ||
           hipStreamSynchronize(s) != hipSuccess))
        rc = gerr(CVXG_E_HIP, "cvxg_solution_space: z0 / Q download failed");
      if (rc == CVXG_OK) {
        memcpy(z0, hz.data(), n * sizeof(double));
        for (int c = 0; c < n - p; ++c) memcpy(F + (size_t)c * ldF, h.data() + (size_t)(p + c) * n, n * sizeof(double));
      }
    }
  }
  (void)hipStreamDestroy(s);
  return rc;
}

#define LIBC(ctx, call)                                                                    \
  do {                                                                                     \
    if ((call) != 0) return set_err(ctx, CVXG_E_HIP, "%s failed (%s:%d)", #call, __FILE__, __LINE__); \
  } while (0)

int cvxg_affine_from(cvxg_ctx* dst, cvxg_ctx* src, const double* z0, const double* F, int ldF) {
  if (!dst || !src || !z0 || !F || dst == src) return dst ? set_err(dst, CVXG_E_ARG, "cvxg_affine_from: bad argument") : CVXG_E_ARG;
  if (dst->dev != src->dev) return set_err(dst, CVXG_E_ARG, "cvxg_affine_from: contexts on different devices");
  if (dst->m != src->m || dst->p != src->p)
    return set_err(dst, CVXG_E_DIM, "cvxg_affine_from: dst must have the m and p of src");
  if (ldF < src->n) return set_err(dst, CVXG_E_DIM, "cvxg_affine_from: ldF < n");
  if (!src->have_obj || !src->have_ineq || (src->p > 0 && !src->have_eq))
    return set_err(dst, CVXG_E_ARG, "cvxg_affine_from: the source problem is not complete");
  if (src->kl || src->klp) return set_err(dst, CVXG_E_UNSUPPORTED, "cvxg_affine_from: KL objective");
  HIPC(dst, hipSetDevice(src->dev));
  HIPC(dst, hipStreamSynchronize(src->s));
  const int n = src->n, k = dst->n, m = src->m, p = src->p, nq = src->nq;
  const int lds = src->np;
  hipStream_t s = dst->s;
  DevBufs B;
  double* dF = B.get<double>((size_t)n * k);
  double* dz = B.get<double>(n);
  double* dT = B.get<double>((size_t)n * k);
  double* dQ = B.get<double>((size_t)k * k);
  double* dv = B.get<double>(n);
  double* du = B.get<double>(k);
  double* dAu = B.get<double>((size_t)std::max(m, 1) * k);
  double* dr = B.get<double>(std::max(m, 1));
  double* dAe = B.get<double>((size_t)std::max(p, 1) * k);
  double* dbe = B.get<double>(std::max(p, 1));
  if (!dF || !dz || !dT || !dQ || !dv || !du || !dAu || !dr || !dAe || !dbe)
    return set_err(dst, CVXG_E_HIP, "cvxg_affine_from: device allocation failed");
  {
    std::vector<double> h((size_t)n * k);
    for (int c = 0; c < k; ++c) memcpy(h.data() + (size_t)c * n, F + (size_t)c * ldF, n * sizeof(double));
    CHK(copy_sync(dst, dF, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice));
    CHK(copy_sync(dst, dz, z0, n * sizeof(double), hipMemcpyHostToDevice));
  }
  // F' X F for a symmetric row-major X (ld lds): T = X F, Q = F' T; lower triangle mirrored (the engine reads H's
  // lower triangle, as dpotrf('L') reads the reference's (F'H)F)
  auto pullback = [&](const double* X, std::vector<double>& out) -> int {
    LIBC(dst, lib_gemm(s, false, false, n, k, n, X, lds, dF, n, dT, n));
    LIBC(dst, lib_gemm(s, true, false, k, k, n, dF, n, dT, n, dQ, k));
    out.resize((size_t)k * k);
    CHK(copy_sync(dst, out.data(), dQ, out.size() * sizeof(double), hipMemcpyDeviceToHost));
    for (int j = 0; j < k; ++j)
      for (int i = j + 1; i < k; ++i) out[(size_t)i * k + j] = out[(size_t)j * k + i];  // column-major: (i,j) -> (j,i)
    return CVXG_OK;
  };
  // objective: QuadraticObjectiveFunction / LinearObjectiveFunction under x = z0 + F u
  std::vector<double> Pu, au(k);
  double r0u = src->r0, dot = 0.0;
  CHK(copy_sync(dst, dv, src->a0, n * sizeof(double), hipMemcpyDeviceToDevice));
  LIBC(dst, lib_dot(s, n, src->a0, dz, &dot));
  r0u = r0u + dot;  // r + (a dot z)
  if (src->hasP) {
    CHK(pullback(src->P, Pu));
    LIBC(dst, lib_gemv(s, false, n, n, 1.0, src->P, lds, dz, 1.0, dv));  // v = a + P z0
    LIBC(dst, lib_gemv(s, false, n, n, 1.0, src->P, lds, dz, 0.0, dT));  // P z0
    LIBC(dst, lib_dot(s, n, dz, dT, &dot));
    r0u = r0u + dot / 2;  // + (z dot (P*z))/2
  }
  LIBC(dst, lib_gemv(s, true, n, k, 1.0, dF, n, dv, 0.0, du));  // a_u = F'(a + P z0)
  CHK(copy_sync(dst, au.data(), du, k * sizeof(double), hipMemcpyDeviceToHost));
  CHK(cvxg_set_objective(dst, src->hasP ? Pu.data() : nullptr, k, au.data(), r0u));
  // inequalities: rows a_i -> F'a_i, r_i -> r_i + a_i.z0 (the row-major A is the column-major A', ld lds)
  if (m > 0) {
    std::vector<double> Au((size_t)m * k), ru(m), ubh(m);
    LIBC(dst, lib_gemm(s, true, false, k, m, n, dF, n, src->A, lds, dAu, k));  // (A F)' = F' A'
    CHK(copy_sync(dst, dr, src->r, m * sizeof(double), hipMemcpyDeviceToDevice));
    LIBC(dst, lib_gemv(s, true, n, m, 1.0, src->A, lds, dz, 1.0, dr));
    std::vector<double> Pqu;
    if (nq > 0) {  // QuadraticConstraint.affineTransformed: F'(a + P z), F'PF, valueAt(z)
      Pqu.resize((size_t)nq * k * k);
      for (int q = 0; q < nq; ++q) {
        const double* Pk = src->Pq + (size_t)q * lds * lds;
        const int row = src->qrows_h[q];
        std::vector<double> Q;
        CHK(pullback(Pk, Q));
        memcpy(Pqu.data() + (size_t)q * k * k, Q.data(), Q.size() * sizeof(double));
        CHK(copy_sync(dst, dv, src->A + (size_t)row * lds, n * sizeof(double), hipMemcpyDeviceToDevice));
        LIBC(dst, lib_gemv(s, false, n, n, 1.0, Pk, lds, dz, 1.0, dv));        // a + P z
        LIBC(dst, lib_gemv(s, true, n, k, 1.0, dF, n, dv, 0.0, dAu + (size_t)row * k));
        LIBC(dst, lib_gemv(s, false, n, n, 1.0, Pk, lds, dz, 0.0, dT));        // P z
        LIBC(dst, lib_dot(s, n, dz, dT, &dot));
        double rq = 0.0;
        CHK(copy_sync(dst, &rq, dr + row, sizeof(double), hipMemcpyDeviceToHost));
        rq = rq + dot / 2;
        CHK(copy_sync(dst, dr + row, &rq, sizeof(double), hipMemcpyHostToDevice));
      }
    }
    CHK(copy_sync(dst, Au.data(), dAu, Au.size() * sizeof(double), hipMemcpyDeviceToHost));
    CHK(copy_sync(dst, ru.data(), dr, m * sizeof(double), hipMemcpyDeviceToHost));
    CHK(copy_sync(dst, ubh.data(), src->ub, m * sizeof(double), hipMemcpyDeviceToHost));
    CHK(cvxg_set_ineq(dst, Au.data(), k, 1, ru.data(), ubh.data()));
    if (nq > 0) CHK(cvxg_set_quad(dst, nq, src->qrows_h.data(), Pqu.data(), k));
  } else {
    CHK(cvxg_set_ineq(dst, nullptr, k, 1, nullptr, nullptr));
  }
  // equalities: (A F) u = b - A z0
  if (p > 0) {
    std::vector<double> Ae((size_t)p * k), be(p);
    LIBC(dst, lib_gemm(s, true, false, k, p, n, dF, n, src->Aeq, lds, dAe, k));
    CHK(copy_sync(dst, dbe, src->beq, p * sizeof(double), hipMemcpyDeviceToDevice));
    LIBC(dst, lib_gemv(s, true, n, p, -1.0, src->Aeq, lds, dz, 1.0, dbe));
    CHK(copy_sync(dst, Ae.data(), dAe, Ae.size() * sizeof(double), hipMemcpyDeviceToHost));
    CHK(copy_sync(dst, be.data(), dbe, p * sizeof(double), hipMemcpyDeviceToHost));
    CHK(cvxg_set_eq(dst, Ae.data(), k, 1, be.data()));
  }
  // keep z0 and F for cvxg_affine_parameter / cvxg_affine_map
  for (double** v : {&dst->aff_F, &dst->aff_z0})
    if (*v) (void)hipFree(*v), *v = nullptr;
  CHK(dalloc(dst, &dst->aff_F, (size_t)n * k));
  CHK(dalloc(dst, &dst->aff_z0, n));
  CHK(copy_sync(dst, dst->aff_F, dF, (size_t)n * k * sizeof(double), hipMemcpyDeviceToDevice));
  CHK(copy_sync(dst, dst->aff_z0, dz, n * sizeof(double), hipMemcpyDeviceToDevice));
  dst->aff_n = n;
  return CVXG_OK;
}

int cvxg_affine_parameter(cvxg_ctx* dst, const double* x0, double* u0) {
  if (!dst || !x0 || !u0) return CVXG_E_ARG;
  if (!dst->aff_F) return set_err(dst, CVXG_E_ARG, "cvxg_affine_parameter: no affine transform loaded");
  HIPC(dst, hipSetDevice(dst->dev));
  const int n = dst->aff_n, k = dst->n;
  DevBufs B;
  double* dx = B.get<double>(n);
  double* du = B.get<double>(k);
  if (!dx || !du) return set_err(dst, CVXG_E_HIP, "device allocation failed");
  CHK(copy_sync(dst, dx, x0, n * sizeof(double), hipMemcpyHostToDevice));
  launch_axpy(dst->s, dx, dst->aff_z0, -1.0, n, dx);  // x0 - z0
  HIPC(dst, hipGetLastError());
  LIBC(dst, lib_gemv(dst->s, true, n, k, 1.0, dst->aff_F, n, dx, 0.0, du));
  CHK(copy_sync(dst, u0, du, k * sizeof(double), hipMemcpyDeviceToHost));
  return CVXG_OK;
}

int cvxg_affine_map(cvxg_ctx* dst, const double* u, double* x) {
  if (!dst || !x) return CVXG_E_ARG;
  if (!dst->aff_F) return set_err(dst, CVXG_E_ARG, "cvxg_affine_map: no affine transform loaded");
  HIPC(dst, hipSetDevice(dst->dev));
  const int n = dst->aff_n, k = dst->n;
  DevBufs B;
  double* du = B.get<double>(k);
  double* dx = B.get<double>(n);
  if (!du || !dx) return set_err(dst, CVXG_E_HIP, "device allocation failed");
  if (u)
    CHK(copy_sync(dst, du, u, k * sizeof(double), hipMemcpyHostToDevice));
  else
    CHK(copy_sync(dst, du, dst->x, k * sizeof(double), hipMemcpyDeviceToDevice));
  CHK(copy_sync(dst, dx, dst->aff_z0, n * sizeof(double), hipMemcpyDeviceToDevice));
  LIBC(dst, lib_gemv(dst->s, false, n, k, 1.0, dst->aff_F, n, du, 1.0, dx));  // z0 + F u
  CHK(copy_sync(dst, x, dx, n * sizeof(double), hipMemcpyDeviceToHost));
  return CVXG_OK;
}
