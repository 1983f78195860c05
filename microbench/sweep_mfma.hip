// Microbenchmark of a 16 x 16 diagonal-block Cholesky kept in the f64 MFMA accumulator layout (one wave):
// the block is factored 4 columns at a time -- a 4 x 4 Cholesky and its inverse M = L4^-1 computed in every lane from
// ten broadcast entries, then the 16 x 4 panel L_p = C_s L4^-T and the rank-4 update C -= L_p L_p' as two
// v_mfma_f64_16x16x4 -- and L^-1 rides along (Y_s = M Y_s, Y -= L_p Y_s, two more MFMAs off the pivot chain).
// Against the row-per-lane sweep of potrf64w.hpp (120 column broadcasts by v_readlane per 16 columns) this
// broadcasts 40 values and moves the trailing updates onto the matrix core.
//
// Layouts (lane l, c = l & 15, g = l >> 4): accumulator register i holds C[g + 4i][c].  C stays exactly symmetric,
// so register s is also the A-fragment (row c, k = g) of column block s -- the panel operand needs no shuffle --
// and the TRSM's output register 0, L_p[c][g], is both the A- and the B-fragment of the update.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off microbench/sweep_mfma.hip -o microbench/sweep_mfma
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "../cvx_amd/csrc/potrf64.hpp"
using namespace cvxg;

#define MFMA(a, b, c) __builtin_amdgcn_mfma_f64_16x16x4f64((a), (b), (c), 0, 0, 0)

// One 4-column step s of the factorization (s compile-time).  C, Y: the block and L^-1 so far (accumulator layout);
// lfin[s] receives L[c][4s + g] (rows c >= 4s; the L^T accumulator layout).  Returns false on a non-positive pivot.
template <int S>
__device__ __forceinline__ void chol4_step(d4f& C, d4f& Y, double (&lfin)[4], double& pmin, int& firstbad, int lane) {
  const int c = lane & 15, g = lane >> 4;
  // the ten lower entries of the 4 x 4 diagonal block: D4[a][b] is register S of lane a*16 + 4S + b
  double d[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b <= a; ++b) d[a][b] = readlane_d(C[S], a * 16 + 4 * S + b);
  // 4 x 4 Cholesky (pivots p_j, s_j = p_j^-1/2, l_jj = p_j s_j) and M = L4^-1 (m_jj = s_j), wave-uniform
  double l[4][4], m[4][4], sv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double p = d[j][j];
#pragma unroll
    for (int k = 0; k < j; ++k) p = fma(-l[j][k], l[j][k], p);
    if (!(p > 0.0) && firstbad < 0) firstbad = 4 * S + j;
    pmin = fmin(pmin, p);
    sv[j] = rsqrt_nr(p);
    l[j][j] = p * sv[j];
#pragma unroll
    for (int i = j + 1; i < 4; ++i) {
      double t = d[i][j];
#pragma unroll
      for (int k = 0; k < j; ++k) t = fma(-l[i][k], l[j][k], t);
      l[i][j] = t * sv[j];
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    m[i][i] = sv[i];
#pragma unroll
    for (int j = 0; j < i; ++j) {
      double t = 0.0;
#pragma unroll
      for (int k = j; k < i; ++k) t = fma(l[i][k], m[k][j], t);
      m[i][j] = -(t * sv[i]);
    }
  }
  // A-fragment of M' (row c < 4, k = g): m[c][g] for g <= c, else 0
  double mf = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j <= i; ++j) mf = (c == i && g == j) ? m[i][j] : mf;
  // L_p = C_s L4^-T: B-fragment = register S (rows c < 4S are factored already: masked)
  const double cs = (c >= 4 * S) ? C[S] : 0.0;
  const d4f z = {0.0, 0.0, 0.0, 0.0};
  const d4f lp4 = MFMA(mf, cs, z);
  const double lp = lp4[0];  // L_p[c][g]: A- and B-fragment of the rank-4 update
  lfin[S] = lp;
  C = MFMA(-lp, lp, C);  // C -= L_p L_p'
  // L^-1 alongside: Y_s = M Y_s, then Y -= L_p Y_s (row block S of the result: Y_s)
  const d4f ys4 = MFMA(mf, Y[S], z);
  Y = MFMA(-lp, ys4[0], Y);
  Y[S] = ys4[0];
}

// Variant B: the LDL' form -- pivots by reciprocals only (U4 unit lower, p_j), the square roots off the pivot chain:
//   W = C_s U4^-T (MFMA), C -= (W diag(1/p)) W' (MFMA), L[:, 4s + k] = W[:, k] p_k^-1/2.
// L^-1 is formed after the four steps from the saved U4^-1 fragments and W diag(1/p) (Y_s = U4^-1 Y_s,
// Y -= (W/p) Y_s), rows scaled by p^-1/2 at the end.
template <int S>
__device__ __forceinline__ void ldl4_step(d4f& C, double (&wsc)[4], double (&uif)[4], double (&lfin)[4],
                                          double (&rs)[4], double& pmin, int& firstbad, int lane) {
  const int c = lane & 15, g = lane >> 4;
  double d[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b <= a; ++b) d[a][b] = readlane_d(C[S], a * 16 + 4 * S + b);
  // Gaussian elimination of the 4 x 4 block: e[i][j] = D_ij - sum_{k<j} e[i][k] e[j][k] / p_k (i > j), p_j = e[j][j]
  double e[4][4], r[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
#pragma unroll
    for (int i = j; i < 4; ++i) {
      double t = d[i][j];
#pragma unroll
      for (int k = 0; k < j; ++k) t = fma(-(e[i][k] * r[k]), e[j][k], t);
      e[i][j] = t;
    }
    if (!(e[j][j] > 0.0) && firstbad < 0) firstbad = 4 * S + j;
    pmin = fmin(pmin, e[j][j]);
    r[j] = rcp_nr(e[j][j]);
  }
  // U4 = unit lower, u_ij = e_ij / p_j; its inverse (unit lower) by forward substitution
  double ui[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < i; ++j) {
      double t = e[i][j] * r[j];
#pragma unroll
      for (int k = j + 1; k < i; ++k) t = fma(e[i][k] * r[k], ui[k][j], t);
      ui[i][j] = -t;
    }
  double mf = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j <= i; ++j) mf = (c == i && g == j) ? (i == j ? 1.0 : ui[i][j]) : mf;
  const double cs = (c >= 4 * S) ? C[S] : 0.0;
  const d4f z = {0.0, 0.0, 0.0, 0.0};
  const double w = MFMA(mf, cs, z)[0];  // W[c][g] = (C_s U4^-T)[c][g]
  double rg = r[0];
#pragma unroll
  for (int k = 1; k < 4; ++k) rg = (g == k) ? r[k] : rg;  // 1 / p_g
  const double wp = w * rg;
  C = MFMA(-wp, w, C);  // C -= (W / p) W'
  wsc[S] = wp;
  uif[S] = mf;
  rs[S] = rg;
  lfin[S] = w;  // scaled by p_g^-1/2 after the sweep
}

__global__ __launch_bounds__(64) void k_sweep_ldl(const double* __restrict__ D, double* __restrict__ out, int reps,
                                                  int reload, unsigned long long* cyc) {
  const int lane = threadIdx.x, c = lane & 15, g = lane >> 4;
  unsigned long long t0 = 0, t1 = 0;
  d4f C, Y, C0;
  double lfin[4], wsc[4], uif[4], rs[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) C0[i] = D[(g + 4 * i) * 16 + c];
  double pmin = 1e300;
  int firstbad = -1;
  for (int rep = 0; rep <= reps; ++rep) {
    if (rep == 1) t0 = __builtin_amdgcn_s_memtime();
    if (reload) {
#pragma unroll
      for (int i = 0; i < 4; ++i) C[i] = D[(g + 4 * i) * 16 + c];
    } else {
      C = C0;
    }
    ldl4_step<0>(C, wsc, uif, lfin, rs, pmin, firstbad, lane);
    ldl4_step<1>(C, wsc, uif, lfin, rs, pmin, firstbad, lane);
    ldl4_step<2>(C, wsc, uif, lfin, rs, pmin, firstbad, lane);
    ldl4_step<3>(C, wsc, uif, lfin, rs, pmin, firstbad, lane);
    // L = W p^-1/2 ; L^-1 = diag(p^-1/2) Lhat^-1 by the saved elimination steps
#pragma unroll
    for (int s = 0; s < 4; ++s) lfin[s] *= rsqrt_nr(1.0 / rs[s]);
#pragma unroll
    for (int i = 0; i < 4; ++i) Y[i] = (g + 4 * i == c) ? 1.0 : 0.0;
    const d4f z = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const double ys = __builtin_amdgcn_mfma_f64_16x16x4f64(uif[s], Y[s], z, 0, 0, 0)[0];
      Y = __builtin_amdgcn_mfma_f64_16x16x4f64(-wsc[s], ys, Y, 0, 0, 0);
      Y[s] = ys;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // row g + 4i of Lhat^-1 times p_{g+4i}^-1/2 (p of row-block i, entry g)
      Y[i] *= rsqrt_nr(1.0 / rs[i]);  // (rs[i] in this lane: 1 / p of entry g of block i)
    }
    C0[0] += 0.0 * (lfin[0] + lfin[3] + Y[3]);
    __builtin_amdgcn_sched_barrier(0);
  }
  t1 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int s = 0; s < 4; ++s) out[c * 16 + 4 * s + g] = (c >= 4 * s + g) ? lfin[s] : 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i) out[256 + (g + 4 * i) * 16 + c] = Y[i];
  if (lane == 0) {
    *cyc = (t1 - t0) / (reps > 0 ? reps : 1);
    out[512] = firstbad;
    out[513] = pmin;
  }
}

__global__ __launch_bounds__(64) void k_sweep_mfma(const double* __restrict__ D, double* __restrict__ out, int reps,
                                                   int reload, unsigned long long* cyc) {
  const int lane = threadIdx.x, c = lane & 15, g = lane >> 4;
  unsigned long long t0 = 0, t1 = 0;
  d4f C, Y;
  double lfin[4];
  d4f C0;
#pragma unroll
  for (int i = 0; i < 4; ++i) C0[i] = D[(g + 4 * i) * 16 + c];
  double pmin = 1e300;
  int firstbad = -1;
  for (int rep = 0; rep <= reps; ++rep) {
    if (rep == 1) t0 = __builtin_amdgcn_s_memtime();
    if (reload) {
#pragma unroll
      for (int i = 0; i < 4; ++i) C[i] = D[(g + 4 * i) * 16 + c];
    } else {
      C = C0;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) Y[i] = (g + 4 * i == c) ? 1.0 : 0.0;
    chol4_step<0>(C, Y, lfin, pmin, firstbad, lane);
    chol4_step<1>(C, Y, lfin, pmin, firstbad, lane);
    chol4_step<2>(C, Y, lfin, pmin, firstbad, lane);
    chol4_step<3>(C, Y, lfin, pmin, firstbad, lane);
    C0[0] += 0.0 * (lfin[0] + lfin[3] + Y[3]);  // keep the results live across reps
    __builtin_amdgcn_sched_barrier(0);
  }
  t1 = __builtin_amdgcn_s_memtime();
  // L[c][4s + g] = lfin[s] (rows c >= 4s + g), L^-1[g + 4i][c] = Y[i]
#pragma unroll
  for (int s = 0; s < 4; ++s) out[c * 16 + 4 * s + g] = (c >= 4 * s + g) ? lfin[s] : 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i) out[256 + (g + 4 * i) * 16 + c] = Y[i];
  if (lane == 0) {
    *cyc = (t1 - t0) / (reps > 0 ? reps : 1);
    out[512] = firstbad;
    out[513] = pmin;
  }
}

int main() {
  std::vector<double> B(256), D(256);
  srand(3);
  for (auto& v : B) v = (double)rand() / RAND_MAX - 0.5;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double s = 0;
      for (int k = 0; k < 16; ++k) s += B[i * 16 + k] * B[j * 16 + k];
      D[i * 16 + j] = s / 16 + (i == j ? 1.0 : 0.0);
    }
  std::vector<double> L(256, 0.0);
  double pminref = 1e300;
  for (int j = 0; j < 16; ++j) {
    double s = D[j * 16 + j];
    for (int k = 0; k < j; ++k) s -= L[j * 16 + k] * L[j * 16 + k];
    pminref = fmin(pminref, s);
    L[j * 16 + j] = sqrt(s);
    for (int i = j + 1; i < 16; ++i) {
      double t = D[i * 16 + j];
      for (int k = 0; k < j; ++k) t -= L[i * 16 + k] * L[j * 16 + k];
      L[i * 16 + j] = t / L[j * 16 + j];
    }
  }
  double *dD, *dO;
  unsigned long long* dc;
  hipMalloc(&dD, 256 * 8);
  hipMalloc(&dO, 514 * 8);
  hipMalloc(&dc, 8);
  hipMemcpy(dD, D.data(), 256 * 8, hipMemcpyHostToDevice);
  for (int run = 0; run < 4; ++run) {
    const int reload = run & 1, ldl = run >> 1;
    if (ldl) k_sweep_ldl<<<1, 64>>>(dD, dO, 100, reload, dc);
    else k_sweep_mfma<<<1, 64>>>(dD, dO, 100, reload, dc);
    hipDeviceSynchronize();
    std::vector<double> O(514);
    unsigned long long cyc;
    hipMemcpy(O.data(), dO, 514 * 8, hipMemcpyDeviceToHost);
    hipMemcpy(&cyc, dc, 8, hipMemcpyDeviceToHost);
    double eL = 0, eI = 0;
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        eL = fmax(eL, fabs(O[i * 16 + j] - L[i * 16 + j]));
        double s = 0;  // (L^-1 L)[i][j]
        for (int k = 0; k < 16; ++k) s += O[256 + i * 16 + k] * L[k * 16 + j];
        eI = fmax(eI, fabs(s - (i == j ? 1.0 : 0.0)));
      }
    printf("%s %s: %llu cycles per 16 columns  max|L - Lref| = %.3e  max|Linv L - I| = %.3e  firstbad %g "
           "pmin %.6g (ref %.6g)\n",
           ldl ? "ldl-form" : "mfma-layout", reload ? "(block reloaded from memory each rep, as sweep.hip)" : "(block in registers)", cyc, eL, eI,
           O[512], O[513], pminref);
  }
  return 0;
}
