// k_chol.hip — the backward substitution L' u = w of the Cholesky solve (MatrixUtils.scala:410-430 backSolve,
// blocked): one persistent launch over the 64 x 64 blocks of L, using the diagonal-block inverses L_kk^-1 that the
// factorization (k_dataflow.hip) stores, so every block step is a product instead of a sequential substitution.
#include <math.h>

#include "potrf64.hpp"  // Sc1Mem

namespace cvxg {
// ------------------------------------------------------------------------------------------------
// The whole backward substitution L' u = w in ONE launch (MatrixUtils.scala:419-430 backSolve, blocked):
// workgroup g owns block b = nblk-1-g and accumulates  s_b = sum_{i>b} L_ib' u_i  as the u_i are published
// (L_ib is prefetched into registers before the wait), then  u_b = Linv_bb' (w_b - s_b)  and publishes u_b.
// Hand-off: every entry of u_b goes out as a data-tagged 16-B granule {value, gen} (one sc1 store, observed untorn
// on gfx950; MI355X_MICROARCH.md hand-off table: ~1.0 us for a small 1:1 hand-off against 1.7-1.9x that with a
// separate drained flag), and the consumers poll the granules themselves -- no flag round trip.  Workgroups only
// wait on lower blockIdx (dispatched earlier), so the launch is deadlock-free at any residency.  Thread (c, g)
// keeps the partial sums of column c over rows 16g..16g+15 of every tile; the four row groups are added once, in
// a fixed order.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_bwd_dataflow(const double* __restrict__ L, int ld,
                                                      const double* __restrict__ Linv, const double* __restrict__ rhs,
                                                      double* __restrict__ out, int nrhs, int nblk, int* flags, int gen,
                                                      const DevCtrl* ctrl, BwdEpilogue epi, BwdAlt alt) {
  if (ctrl->ruiz_sweeps < 0) return;  // a void factorization attempt
  if (alt.L && ctrl->spec_sel) {      // the speculative pair's second attempt is the one to use
    if (ctrl->chol_info2 != 0) return;
    L = alt.L;
    Linv = alt.Linv;
    rhs = alt.rhs;
  } else if (ctrl->chol_info != 0 || ctrl->small_piv != 0) {
    return;  // a failed attempt, or a first attempt stopped early (its factor is discarded: the retry's solve follows)
  }
  __shared__ double u[MAX_RHS][NB];
  __shared__ double part[4][MAX_RHS][NB];
  __shared__ int s_bad;
  const int b = nblk - 1 - (int)blockIdx.x;
  // the granules {u entry, gen} behind the nblk flag words (256-B aligned): entry (row, rho) at (row nrhs + rho)
  const Sc1Mem gr(reinterpret_cast<double*>(flags + ((nblk + 63) & ~63)), (unsigned)(nblk * NB * nrhs) * 16u);
  const double tag = __longlong_as_double((long long)gen);
  if (threadIdx.x == 0) s_bad = 0;
  const int g = threadIdx.x >> 6, c = threadIdx.x & 63;
  double acc[MAX_RHS];
#pragma unroll
  for (int rho = 0; rho < MAX_RHS; ++rho) acc[rho] = 0.0;
  double cur[16], nxt[16];
  // off the critical path: this block's w_b and L_bb^-1 (final before the launch) into registers up front
  double lin[16], wb[(MAX_RHS * NB + 255) / 256];
  {
    const double* li = Linv + (size_t)b * NB * NB;
#pragma unroll
    for (int r = 0; r < 16; ++r) lin[r] = li[(16 * g + r) * NB + c];
#pragma unroll
    for (int q = 0; q < (MAX_RHS * NB + 255) / 256; ++q) {
      const int t = threadIdx.x + 256 * q;
      wb[q] = (t < nrhs * NB) ? rhs[(size_t)(b * NB + t % NB) * nrhs + t / NB] : 0.0;
    }
  }
  auto load_tile = [&](double (&t)[16], int i) {  // rows 16g.. of tile (i, b), column c
    const double* tp = L + (size_t)i * NB * ld + (size_t)b * NB + c;
#pragma unroll
    for (int r = 0; r < 16; ++r) t[r] = __builtin_nontemporal_load(tp + (size_t)(16 * g + r) * ld);
  };
  if (b + 1 < nblk) load_tile(cur, nblk - 1);
  for (int i = nblk - 1; i > b; --i) {
    if (i - 1 > b) load_tile(nxt, i - 1);
    for (int t = threadIdx.x; t < nrhs * NB; t += 256) {  // each thread polls its own granules of u_i
      const int rho = t / NB, cc = t % NB;
      const int off = 2 * ((i * NB + cc) * nrhs + rho);
      f64x2 v = gr.ld2(off);
      const unsigned long long t0 = spin_clock();
      for (unsigned spins = 0; __double_as_longlong(v[1]) != (long long)gen; ++spins) {
        if (spin_expired(spins, t0)) {  // bounded wait: never hang the GPU on a scheduling bug
          s_bad = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        v = gr.ld2(off);
      }
      u[rho][cc] = v[0];
    }
    __syncthreads();
    if (s_bad) return;
    for (int rho = 0; rho < nrhs; ++rho) {
      double s = acc[rho];
#pragma unroll
      for (int r = 0; r < 16; ++r) s = fma(cur[r], u[rho][16 * g + r], s);
      acc[rho] = s;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) cur[r] = nxt[r];
    __syncthreads();  // u is rewritten next round
  }
  // y = w_b - s_b, then u_b = Linv_bb' y
  for (int rho = 0; rho < nrhs; ++rho) part[g][rho][c] = acc[rho];
  __syncthreads();
#pragma unroll
  for (int q = 0; q < (MAX_RHS * NB + 255) / 256; ++q) {
    const int t = threadIdx.x + 256 * q;
    if (t < nrhs * NB) {
      const int rho = t / NB, cc = t % NB;
      const double sb = ((part[0][rho][cc] + part[1][rho][cc]) + part[2][rho][cc]) + part[3][rho][cc];
      u[rho][cc] = wb[q] - sb;
    }
  }
  __syncthreads();
  for (int rho = 0; rho < nrhs; ++rho) {
    double s = 0.0;
#pragma unroll
    for (int r = 0; r < 16; ++r) s = fma(lin[r], u[rho][16 * g + r], s);
    part[g][rho][c] = s;
  }
  __syncthreads();
  if (g == 0) {
    for (int rho = 0; rho < nrhs; ++rho) {
      const double s = ((part[0][rho][c] + part[1][rho][c]) + part[2][rho][c]) + part[3][rho][c];
      gr.st2(2 * ((b * NB + c) * nrhs + rho), f64x2{s, tag});  // the hand-off granule first
      out[(size_t)(b * NB + c) * nrhs + rho] = s;              // the solution (read after the launch)
    }
    if (epi.d) {  // Newton step (nrhs = 1): dx = d :* u, and the line search's s = dx, x1 = x + s*t1 (k_scale_vec,
                  // k_spec_prep fused)
      const int i = b * NB + c;
      const double v = epi.d[i] * out[i];
      epi.dx[i] = v;
      if (epi.s) epi.s[i] = v;
      if (epi.x1) epi.x1[i] = epi.x[i] + v * epi.t1;
    }
  }
  if (epi.sctrl && b == 0 && threadIdx.x == 0) {
    epi.sctrl->spec_infeasible = 0;
    epi.sctrl->spec_not_strict = 0;
  }
}

size_t bwd_work_ints(int nblk) { return (size_t)((nblk + 63) & ~63) + (size_t)nblk * NB * MAX_RHS * 4; }

void launch_bwd_dataflow(hipStream_t s, const double* L, int ld, const double* Linv, const double* rhs, double* out,
                         int nrhs, int nblk, int* flags, int gen, const DevCtrl* ctrl, BwdEpilogue epi, BwdAlt alt) {
  // (flags: nblk words + the granules, bwd_work_ints)
  k_bwd_dataflow<<<nblk, 256, 0, s>>>(L, ld, Linv, rhs, out, nrhs, nblk, flags, gen, ctrl, epi, alt);
}

__global__ void k_spec_prep2(DevCtrl* ctrl2, const DevCtrl* ctrl, double reg) {
  ctrl2->reg = reg;
  ctrl2->small_piv = 0;
  ctrl2->chol_info = 0;
  ctrl2->df_status = 0;
  ctrl2->min_diag = (unsigned long long)__double_as_longlong(__builtin_inf());
  ctrl2->ruiz_sweeps = ctrl->ruiz_sweeps;
}
void launch_spec_prep2(hipStream_t s, DevCtrl* ctrl2, const DevCtrl* ctrl, double reg) {
  k_spec_prep2<<<1, 1, 0, s>>>(ctrl2, ctrl, reg);
}
// regularizedCholesky's test on the first attempt (MatrixUtils.scala:456-460): discarded when its pivot failed or
// min diag(L) <= 1e-7
__global__ void k_spec_select(DevCtrl* ctrl, const DevCtrl* ctrl2) {
  const double md = __longlong_as_double((long long)ctrl->min_diag);
  ctrl->spec_sel = (ctrl->chol_info == 0 && md > 1e-7) ? 0 : 1;
  ctrl->chol_info2 = ctrl2->chol_info;
  ctrl->small_piv2 = ctrl2->small_piv;
  ctrl->min_diag2 = ctrl2->min_diag;
  if (ctrl2->df_status) ctrl->df_status = ctrl2->df_status;
}
void launch_spec_select(hipStream_t s, DevCtrl* ctrl, const DevCtrl* ctrl2) { k_spec_select<<<1, 1, 0, s>>>(ctrl, ctrl2); }

}  // namespace cvxg
