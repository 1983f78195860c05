// common.hpp — shared device helpers and the device-side control block of the barrier engine.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cvxg {

constexpr int NB = 64;        // Cholesky / triangular-solve block (row-major lower L)
constexpr int TILE = 128;     // MFMA SYRK output tile
constexpr int KC = 16;        // SYRK contraction chunk staged per LDS buffer
constexpr int MPAD = 64;      // inequality rows padded to a multiple of this
constexpr int LS_TRIALS = 64; // backtracking trials evaluated per line-search batch
constexpr int MAX_RHS = 9;    // 1 + CVXG_MAX_EQ right-hand sides in the fused forward solve
constexpr int RUIZ_MAX = 20;  // MatrixUtils.scala:247
constexpr int COLDOT_ROWS = 128;  // row chunk of the A'v column reduction (partials summed in fixed order)

// Device control block: every scalar the graph-captured kernels need lives here, so launches can be
// replayed with fixed arguments.  A pinned host mirror is read back once per Newton step.
struct DevCtrl {
  double t;                       // barrier parameter of the current centering
  double reg;                     // diagonal shift added when forming Q (0 or 1e-10), MatrixUtils.scala:454
  int infeasible;                 // # rows with d_i <= 0 at the last constraint evaluation
  int not_strict;                 // # rows failing g_i*(1+3e-16) < ub_i
  int chol_info;                  // 1-based global pivot index of the first non-positive pivot, 0 = ok
  int ruiz_sweeps;                // Ruiz sweeps executed
  int df_status;                  // dataflow Cholesky: 2 = a dependency wait timed out (scheduling bug)
  unsigned long long min_diag;    // bits of min diag(L) (positive doubles order like uint64)
  unsigned long long pd_s0;       // bits of the primal-dual step bound s0 (PrimalDualSolver.scala:331-338)
  unsigned long long ruiz_rho[RUIZ_MAX + 2];
  double sc[40];                  // reduced scalars, see SC_* below
  int spec_infeasible;            // the speculative evaluation at x + s (k_ls_setup_eval): its infeasible / not_strict
  int spec_not_strict;
  int small_piv;                  // k_chol_dataflow with early_min > 0 (regularizedCholesky's first attempt): 1-based
                                  // first row of the 16-column block where it stopped on min diag(L) <= early_min
                                  // (min_diag holds that block's value); 0 = it did not stop
  int ruiz_abort;                 // k_ruiz_loop's abort word of its last launch (0 = none; else which wait gave up)
  // speculative regularized attempt (cvxg.cpp: regularized_cholesky_spec): chol(Q) and chol(Q + 1e-10 I) side by side;
  // spec_sel = 1 when the first is discarded (its pivot failed or min diag(L) <= 1e-7), the second's results beside
  int spec_sel;
  int chol_info2;
  int small_piv2;
  unsigned long long min_diag2;
};

enum {
  SC_A0X = 0,   // a0 . x
  SC_XPX,       // x . P x
  SC_SUMLOG,    // sum_i log d_i
  SC_GG,        // |grad|^2
  SC_Q,         // dx . grad
  SC_RES2,      // |H dx + grad|^2
  SC_A0S,       // a0 . s
  SC_SPX,       // s . P x
  SC_SPS,       // s . P s
  SC_EQ2,       // |b - Aeq x|^2
  SC_RES2B,     // second KKT residual |A x - b|^2
  SC_B2,        // |b|^2 (KKT)
  SC_KLSUM,     // KL dual: sum_j R exp(-(B'z)_j)
  // magnitudes for the certified line-search decisions (cvxg.cpp: line_search)
  SC_A0XA,      // |a0| . |x|
  SC_XPXA,      // |x| . |P| |x|
  SC_A0SA,      // |a0| . |s|
  SC_SPXA,      // |s| . |P| |x|
  SC_SPSA,      // |s| . |P| |s|
  SC_CAINV,     // sum_i cabs_i / d_i at x
  SC_LOGABS,    // sum_i |log d_i| at x
  // a fresh evaluation of one trial point (line_search: ambiguous trials)
  SC_TR_A0X,    // a0 . xt
  SC_TR_XPX,    // xt . P xt
  SC_TR_SUMLOG, // sum_i log d_i(xt)
  SC_KLP,       // KL primal objective x . log(n x) at x (Dist_KL.scala:223-227)
  SC_KLPA,      // its error scale sum_j |x_j log(n x_j)| + |x_j|
  SC_TR_KLP,    // the KL primal objective at a fresh trial point xt
  SC_KLA,       // KL dual: sum_j y_j (|B'||z|)_j, the error scale of its exponents at z
  SC_TR_KLSUM,  // KL dual: sum_j R exp(-(B'zt)_j) at a fresh trial point zt
  SC_PD_CENT,   // primal-dual with equalities: |r_cent(t, x, lambda)|^2 of the state after a step
  SC_COUNT
};
static_assert(SC_COUNT <= 40, "DevCtrl::sc too small");

// Bounded waits of the inter-workgroup hand-offs: a waiting workgroup gives up (and raises its abort / failure
// signal) after SPIN_LIMIT_TICKS of wall time on the 100 MHz real-time counter -- never a hung GPU on a scheduling
// bug, and no false alarm when other contexts' kernels share the device (a poll count bound fired under a batch of
// concurrent factorizations).  Callers test it every 256 polls.
constexpr unsigned long long SPIN_LIMIT_TICKS = 500000000ull;  // 5 s
__device__ __forceinline__ unsigned long long spin_clock() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ bool spin_expired(unsigned spins, unsigned long long t0) {
  return (spins & 255u) == 255u && spin_clock() - t0 > SPIN_LIMIT_TICKS;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}

// Deterministic block sum (fixed tree) for blockDim.x a multiple of 64, <= 1024.
__device__ __forceinline__ double block_sum(double v, double* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0) {
    for (int i = 0; i < nw; ++i) s += red[i];
    red[0] = s;
  }
  __syncthreads();
  s = red[0];
  __syncthreads();
  return s;
}

__device__ __forceinline__ void atomic_max_pos(unsigned long long* p, double v) {
  // v >= 0: IEEE ordering of non-negative doubles equals unsigned ordering of their bits.
  atomicMax(p, (unsigned long long)__double_as_longlong(v));
}
__device__ __forceinline__ void atomic_min_pos(unsigned long long* p, double v) {
  atomicMin(p, (unsigned long long)__double_as_longlong(v));
}

}  // namespace cvxg
