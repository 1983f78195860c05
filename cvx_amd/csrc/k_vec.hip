// k_vec.hip — HBM-streaming kernels of the barrier Newton step (gfx950).
//
// Row-major constraint matrix A (row i = a_i, LinearConstraint.scala:7-32), 64-lane waves over rows so
// each row is read as 1 KiB coalesced double2 sweeps; column reductions write per-64-row-chunk partials
// that a second pass sums in a fixed order (results are bitwise reproducible run to run).
#include <math.h>

#include "kernels.hpp"
#include "ruiz_tile.hpp"

namespace cvxg {

// ------------------------------------------------------------------------------------------------
// Row dot products: two rows per wave, double2 loads, fixed-order wave reduction.
// ------------------------------------------------------------------------------------------------
typedef double vd2 __attribute__((ext_vector_type(2)));

// a.v (and |a|.|v|, which bounds the rounding error of every evaluation order of a.v: the line search's certified
// trial decisions) for two rows per wave.  cols is a multiple of 128 for every caller (padded layouts).  Per row each
// lane accumulates its double2 columns j = 2 lane + 128 k in two accumulators (k even / odd) with 4 sweeps in flight,
// then a fixed-order wave reduction: the result does not depend on the pairing or on ABS.  Each load of v serves both
// rows (with one row per wave every element of M costs two vector loads, and the sweep is load-issue bound below the
// HBM rate).  `two` is wave-uniform: false for the last row of an odd count.
template <bool ABS>
__device__ __forceinline__ void row_dot2_wave(const double* __restrict__ r0, const double* __restrict__ r1, bool two,
                                              const double* __restrict__ v, int cols, int lane, double (&dot)[2],
                                              double (&absdot)[2]) {
  const vd2 z = {0.0, 0.0};
  vd2 acc0[2] = {z, z}, acc1[2] = {z, z}, aab0[2] = {z, z}, aab1[2] = {z, z};
  const double* rows[2] = {r0, r1};
  int j = 2 * lane;
  for (; j + 384 < cols; j += 512) {
    const vd2 b0 = *reinterpret_cast<const vd2*>(v + j), b1 = *reinterpret_cast<const vd2*>(v + j + 128);
    const vd2 b2 = *reinterpret_cast<const vd2*>(v + j + 256), b3 = *reinterpret_cast<const vd2*>(v + j + 384);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      if (q == 1 && !two) break;
      const double* row = rows[q];
      const vd2 a0 = *reinterpret_cast<const vd2*>(row + j), a1 = *reinterpret_cast<const vd2*>(row + j + 128);
      const vd2 a2 = *reinterpret_cast<const vd2*>(row + j + 256), a3 = *reinterpret_cast<const vd2*>(row + j + 384);
      acc0[q] = __builtin_elementwise_fma(a0, b0, acc0[q]);
      acc1[q] = __builtin_elementwise_fma(a1, b1, acc1[q]);
      acc0[q] = __builtin_elementwise_fma(a2, b2, acc0[q]);
      acc1[q] = __builtin_elementwise_fma(a3, b3, acc1[q]);
      if (ABS) {
        aab0[q] = __builtin_elementwise_fma(__builtin_elementwise_abs(a0), __builtin_elementwise_abs(b0), aab0[q]);
        aab1[q] = __builtin_elementwise_fma(__builtin_elementwise_abs(a1), __builtin_elementwise_abs(b1), aab1[q]);
        aab0[q] = __builtin_elementwise_fma(__builtin_elementwise_abs(a2), __builtin_elementwise_abs(b2), aab0[q]);
        aab1[q] = __builtin_elementwise_fma(__builtin_elementwise_abs(a3), __builtin_elementwise_abs(b3), aab1[q]);
      }
    }
  }
  for (; j < cols; j += 128) {
    const vd2 b0 = *reinterpret_cast<const vd2*>(v + j);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      if (q == 1 && !two) break;
      const vd2 a0 = *reinterpret_cast<const vd2*>(rows[q] + j);
      acc0[q] = __builtin_elementwise_fma(a0, b0, acc0[q]);
      if (ABS)
        aab0[q] = __builtin_elementwise_fma(__builtin_elementwise_abs(a0), __builtin_elementwise_abs(b0), aab0[q]);
    }
  }
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    dot[q] = wave_sum((acc0[q][0] + acc0[q][1]) + (acc1[q][0] + acc1[q][1]));
    absdot[q] = ABS ? wave_sum((aab0[q][0] + aab0[q][1]) + (aab1[q][0] + aab1[q][1])) : 0.0;
  }
}

// one row's constraint evaluation from a.x (and |a|.|x|), lane 0
__device__ __forceinline__ void constraint_eval_row(int row, double dot, double adot, const double* __restrict__ r,
                                                    const double* __restrict__ ub, double* __restrict__ c,
                                                    double* __restrict__ d, double* __restrict__ invd,
                                                    double* __restrict__ w, double* __restrict__ logd, DevCtrl* ctrl,
                                                    const double* __restrict__ extra, double* __restrict__ cabs) {
  if (cabs) cabs[row] = fabs(r[row]) + adot;  // |r| + |a|.|x|: scale of the rounding error of r + a.x
  // r + (a dot x)  (LinearConstraint.scala:23), + (x dot P x)/2 for a QuadraticConstraint row (:31)
  const double ci = extra ? (r[row] + dot) + extra[row] : r[row] + dot;
  const double di = ub[row] - ci;          // d = ub - valueAt(x)    BarrierSolver.scala:283
  c[row] = ci;
  d[row] = di;
  invd[row] = 1.0 / di;
  w[row] = 1.0 / (di * di);                // GGt/(d*d)              BarrierSolver.scala:314
  logd[row] = (di > 0.0) ? log(di) : 0.0;
  if (!(di > 0.0)) atomicAdd(&ctrl->infeasible, 1);
  if (!(ci * (1 + 3e-16) < ub[row])) atomicAdd(&ctrl->not_strict, 1);  // Constraint.scala:23
}

template <bool ABS>
__global__ __launch_bounds__(256) void k_constraint_eval(const double* __restrict__ A, int ld, int mp, int cols,
                                                         const double* __restrict__ x,
                                                         const double* __restrict__ r,
                                                         const double* __restrict__ ub, double* __restrict__ c,
                                                         double* __restrict__ d, double* __restrict__ invd,
                                                         double* __restrict__ w, double* __restrict__ logd,
                                                         DevCtrl* ctrl, const double* __restrict__ extra,
                                                         double* __restrict__ cabs) {
  const int lane = threadIdx.x & 63;
  const int row = 2 * (blockIdx.x * 4 + (threadIdx.x >> 6));
  if (row >= mp) return;
  const bool two = row + 1 < mp;
  double dot[2], adot[2];
  row_dot2_wave<ABS>(A + (size_t)row * ld, A + (size_t)(two ? row + 1 : row) * ld, two, x, cols, lane, dot, adot);
  if (lane == 0) {
    constraint_eval_row(row, dot[0], adot[0], r, ub, c, d, invd, w, logd, ctrl, extra, cabs);
    if (two) constraint_eval_row(row + 1, dot[1], adot[1], r, ub, c, d, invd, w, logd, ctrl, extra, cabs);
  }
}

void launch_constraint_eval(hipStream_t s, const double* A, int ld, int mp, int n_cols, const double* x,
                            const double* r, const double* ub, double* c, double* d, double* invd,
                            double* w, double* logd, DevCtrl* ctrl, const double* extra, double* cabs) {
  const int grid = ((mp + 1) / 2 + 3) / 4;
  if (cabs) k_constraint_eval<true><<<grid, 256, 0, s>>>(A, ld, mp, n_cols, x, r, ub, c, d, invd, w, logd, ctrl, extra, cabs);
  else k_constraint_eval<false><<<grid, 256, 0, s>>>(A, ld, mp, n_cols, x, r, ub, c, d, invd, w, logd, ctrl, extra, cabs);
}

template <bool ABS>
__global__ __launch_bounds__(256) void k_rowdot(const double* __restrict__ M, int ld, int rows, int cols,
                                                const double* __restrict__ v, const double* __restrict__ add,
                                                double* __restrict__ y, double* __restrict__ yabs) {
  const int lane = threadIdx.x & 63;
  // one wave per row pair; a grid smaller than the pairs loops (the same per-row sums: bitwise the full grid)
  for (int row = 2 * (blockIdx.x * 4 + (threadIdx.x >> 6)); row < rows; row += 2 * 4 * gridDim.x) {
    const bool two = row + 1 < rows;
    double dot[2], adot[2];
    row_dot2_wave<ABS>(M + (size_t)row * ld, M + (size_t)(two ? row + 1 : row) * ld, two, v, cols, lane, dot, adot);
    if (lane == 0) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        if (q == 1 && !two) break;
        y[row + q] = add ? dot[q] + add[row + q] : dot[q];
        if (ABS) yabs[row + q] = adot[q];
      }
    }
  }
}
static int rowdot_grid(int rows) { return ((rows + 1) / 2 + 3) / 4; }

void launch_rowdot(hipStream_t s, const double* M, int ld, int rows, int cols, const double* v, double* y) {
  k_rowdot<false><<<rowdot_grid(rows), 256, 0, s>>>(M, ld, rows, cols, v, nullptr, y, nullptr);
}
void launch_rowdot_add(hipStream_t s, const double* M, int ld, int rows, int cols, const double* v,
                       const double* add, double* y) {
  k_rowdot<false><<<rowdot_grid(rows), 256, 0, s>>>(M, ld, rows, cols, v, add, y, nullptr);
}
void launch_rowdot_abs(hipStream_t s, const double* M, int ld, int rows, int cols, const double* v, double* y,
                       double* yabs, int max_wg) {
  const int g = rowdot_grid(rows);
  k_rowdot<true><<<(max_wg > 0 && max_wg < g) ? max_wg : g, 256, 0, s>>>(M, ld, rows, cols, v, nullptr, y, yabs);
}

// y = H v + add from the LOWER triangle of the symmetric H alone (the assembly leaves the strictly-upper part of its
// off-diagonal tiles unwritten, cvxg.cpp: assemble_hessian), in two fixed-order passes like the Ruiz sweep:
// tile (I, J), J <= I, of 64 x 64 writes
//   S[J][i] = sum_{j in J} H_ij v_j   for its rows i in I      (row partials; a diagonal tile: its whole rows, the
//                                                               assembly writes both triangles of diagonal tiles)
//   S[I][j] = sum_{i in I} H_ij v_i   for its columns j in J   (I > J: the rows of the upper tile H_JI = H_IJ')
// and k_symv_rows adds S[0..nbn)[r] in order, then add[r].  Deterministic; half the bytes of the full-row sweep.
__global__ __launch_bounds__(256) void k_symv_tiles(const double* __restrict__ H, int ld, int nbn,
                                                    const double* __restrict__ v, double* __restrict__ S) {
  const int t = blockIdx.x;
  int I = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while ((I + 1) * (I + 2) / 2 <= t) ++I;
  while (I * (I + 1) / 2 > t) --I;
  const int J = t - I * (I + 1) / 2;
  __shared__ double cred[4][NB];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int c2 = tid & 31, g = tid >> 5;  // column pair 2*c2, row group g: rows g + 8q
  const double* tile = H + (size_t)I * NB * ld + (size_t)J * NB;
  vd2 h[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) h[q] = *reinterpret_cast<const vd2*>(tile + (size_t)(g + 8 * q) * ld + 2 * c2);
  const vd2 vj = *reinterpret_cast<const vd2*>(v + J * NB + 2 * c2);
  vd2 csum = {0.0, 0.0};
  double rs[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const double vi = v[I * NB + g + 8 * q];
    rs[q] = fma(h[q][1], vj[1], h[q][0] * vj[0]);
    csum = __builtin_elementwise_fma(h[q], vd2{vi, vi}, csum);
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    double x = rs[q];
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    rs[q] = x;
  }
  if (c2 == 0) {
#pragma unroll
    for (int q = 0; q < 8; ++q) S[(size_t)J * (nbn * NB) + I * NB + g + 8 * q] = rs[q];
  }
  if (I == J) return;
  csum[0] += __shfl_xor(csum[0], 32, 64);
  csum[1] += __shfl_xor(csum[1], 32, 64);
  if (lane < 32) {
    cred[wid][2 * c2] = csum[0];
    cred[wid][2 * c2 + 1] = csum[1];
  }
  __syncthreads();
  if (tid < NB) S[(size_t)I * (nbn * NB) + J * NB + tid] = ((cred[0][tid] + cred[1][tid]) + cred[2][tid]) + cred[3][tid];
}
__global__ __launch_bounds__(256) void k_symv_rows(const double* __restrict__ S, int nbn, int n,
                                                   const double* __restrict__ add, double* __restrict__ y) {
  __shared__ double red[4][64];
  const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int row = blockIdx.x * 64 + lane;
  const int ldS = nbn * NB;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  if (row < n) {
    int X = q;
    for (; X + 12 < nbn; X += 16) {
      s0 += S[(size_t)X * ldS + row];
      s1 += S[(size_t)(X + 4) * ldS + row];
      s2 += S[(size_t)(X + 8) * ldS + row];
      s3 += S[(size_t)(X + 12) * ldS + row];
    }
    for (; X < nbn; X += 4) s0 += S[(size_t)X * ldS + row];
  }
  red[q][lane] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (q == 0 && row < n) {
    const double hv = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
    y[row] = add ? hv + add[row] : hv;
  }
}
void launch_symv_lower_add(hipStream_t s, const double* H, int ld, int n, const double* v, const double* add,
                           double* y, double* S) {
  const int nbn = (n + NB - 1) / NB;
  k_symv_tiles<<<nbn * (nbn + 1) / 2, 256, 0, s>>>(H, ld, nbn, v, S);
  k_symv_rows<<<(n + 63) / 64, 256, 0, s>>>(S, nbn, n, add, y);
}

// H_ji = H_ij for i > j (the full symmetric matrix from its lower triangle): 64 x 64 tiles (I, J), I > J, each
// transposed through LDS.
__global__ __launch_bounds__(256) void k_mirror_lower(double* __restrict__ H, int ld, int nbn) {
  const int t = blockIdx.x;
  int I = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while ((I + 1) * (I + 2) / 2 <= t) ++I;
  while (I * (I + 1) / 2 > t) --I;
  const int J = t - I * (I + 1) / 2;
  __shared__ double tl[NB][NB + 1];
  const int tid = threadIdx.x;
  for (int e = tid; e < NB * NB; e += 256) {
    const int r = e >> 6, c = e & 63;
    if (I != J || c < r) tl[r][c] = H[(size_t)(I * NB + r) * ld + J * NB + c];
  }
  __syncthreads();
  for (int e = tid; e < NB * NB; e += 256) {
    const int r = e >> 6, c = e & 63;  // H[J*NB + r][I*NB + c] = H[I*NB + c][J*NB + r]
    if (I != J || r < c) H[(size_t)(J * NB + r) * ld + I * NB + c] = tl[c][r];
  }
}
void launch_mirror_lower(hipStream_t s, double* H, int ld, int n) {
  const int nbn = (n + NB - 1) / NB;
  k_mirror_lower<<<nbn * (nbn + 1) / 2, 256, 0, s>>>(H, ld, nbn);
}

// The line search's setup sweep over A for s = dx (e = A s, eabs = |A| |s|) fused with the next step's constraint
// evaluation at x1 = x + s (k_constraint_eval's outputs and counters into a second set of buffers): when the line
// search accepts t = 1 -- the common case -- the next evaluation is already done and A is read once instead of twice.
// Each wave takes two rows, so every s / x1 load serves two rows of A (three vector loads per element of A would make
// the sweep load-issue bound, 3.7 instead of 5.3 TB/s).  Per row and vector the accumulation has row_dot2_wave's
// structure, so every output is bitwise the standalone kernels' (k_rowdot<true>, k_constraint_eval<true>).
struct RowAcc {
  vd2 sa0, sa1, sb0, sb1, xa0, xa1, xb0, xb1;  // s: dot, |.| dot; x1: dot, |.| dot (two accumulators each)
};
__device__ __forceinline__ void row_acc4(RowAcc& q, const double* __restrict__ a, int j, const vd2 (&sv)[4],
                                         const vd2 (&yv)[4]) {
  const vd2 a0 = *reinterpret_cast<const vd2*>(a + j), a1 = *reinterpret_cast<const vd2*>(a + j + 128);
  const vd2 a2 = *reinterpret_cast<const vd2*>(a + j + 256), a3 = *reinterpret_cast<const vd2*>(a + j + 384);
  const vd2 b0 = __builtin_elementwise_abs(a0), b1 = __builtin_elementwise_abs(a1);
  const vd2 b2 = __builtin_elementwise_abs(a2), b3 = __builtin_elementwise_abs(a3);
  q.sa0 = __builtin_elementwise_fma(a0, sv[0], q.sa0);
  q.sa1 = __builtin_elementwise_fma(a1, sv[1], q.sa1);
  q.sa0 = __builtin_elementwise_fma(a2, sv[2], q.sa0);
  q.sa1 = __builtin_elementwise_fma(a3, sv[3], q.sa1);
  q.sb0 = __builtin_elementwise_fma(b0, __builtin_elementwise_abs(sv[0]), q.sb0);
  q.sb1 = __builtin_elementwise_fma(b1, __builtin_elementwise_abs(sv[1]), q.sb1);
  q.sb0 = __builtin_elementwise_fma(b2, __builtin_elementwise_abs(sv[2]), q.sb0);
  q.sb1 = __builtin_elementwise_fma(b3, __builtin_elementwise_abs(sv[3]), q.sb1);
  q.xa0 = __builtin_elementwise_fma(a0, yv[0], q.xa0);
  q.xa1 = __builtin_elementwise_fma(a1, yv[1], q.xa1);
  q.xa0 = __builtin_elementwise_fma(a2, yv[2], q.xa0);
  q.xa1 = __builtin_elementwise_fma(a3, yv[3], q.xa1);
  q.xb0 = __builtin_elementwise_fma(b0, __builtin_elementwise_abs(yv[0]), q.xb0);
  q.xb1 = __builtin_elementwise_fma(b1, __builtin_elementwise_abs(yv[1]), q.xb1);
  q.xb0 = __builtin_elementwise_fma(b2, __builtin_elementwise_abs(yv[2]), q.xb0);
  q.xb1 = __builtin_elementwise_fma(b3, __builtin_elementwise_abs(yv[3]), q.xb1);
}
__device__ __forceinline__ void row_acc1(RowAcc& q, const double* __restrict__ a, int j, vd2 s0, vd2 y0) {
  const vd2 a0 = *reinterpret_cast<const vd2*>(a + j);
  q.sa0 = __builtin_elementwise_fma(a0, s0, q.sa0);
  q.sb0 = __builtin_elementwise_fma(__builtin_elementwise_abs(a0), __builtin_elementwise_abs(s0), q.sb0);
  q.xa0 = __builtin_elementwise_fma(a0, y0, q.xa0);
  q.xb0 = __builtin_elementwise_fma(__builtin_elementwise_abs(a0), __builtin_elementwise_abs(y0), q.xb0);
}
__device__ __forceinline__ void ls_setup_eval_row(const RowAcc& q, int row, double* __restrict__ e,
                                                  double* __restrict__ eabs, const double* __restrict__ r,
                                                  const double* __restrict__ ub, double* __restrict__ c,
                                                  double* __restrict__ d, double* __restrict__ invd,
                                                  double* __restrict__ w, double* __restrict__ logd,
                                                  double* __restrict__ cabs, DevCtrl* ctrl, int lane) {
  const double sab = wave_sum((q.sb0[0] + q.sb0[1]) + (q.sb1[0] + q.sb1[1]));
  const double sdt = wave_sum((q.sa0[0] + q.sa0[1]) + (q.sa1[0] + q.sa1[1]));
  const double xab = wave_sum((q.xb0[0] + q.xb0[1]) + (q.xb1[0] + q.xb1[1]));
  const double xdt = wave_sum((q.xa0[0] + q.xa0[1]) + (q.xa1[0] + q.xa1[1]));
  if (lane == 0) {
    e[row] = sdt;
    eabs[row] = sab;
    cabs[row] = fabs(r[row]) + xab;  // as k_constraint_eval (linear rows, certified)
    const double ci = r[row] + xdt;
    const double di = ub[row] - ci;
    c[row] = ci;
    d[row] = di;
    invd[row] = 1.0 / di;
    w[row] = 1.0 / (di * di);
    logd[row] = (di > 0.0) ? log(di) : 0.0;
    if (!(di > 0.0)) atomicAdd(&ctrl->spec_infeasible, 1);
    if (!(ci * (1 + 3e-16) < ub[row])) atomicAdd(&ctrl->spec_not_strict, 1);
  }
}
__global__ __launch_bounds__(256) void k_ls_setup_eval(const double* __restrict__ A, int ld, int mp, int cols,
                                                       const double* __restrict__ s, const double* __restrict__ x1,
                                                       double* __restrict__ e, double* __restrict__ eabs,
                                                       const double* __restrict__ r, const double* __restrict__ ub,
                                                       double* __restrict__ c, double* __restrict__ d,
                                                       double* __restrict__ invd, double* __restrict__ w,
                                                       double* __restrict__ logd, double* __restrict__ cabs,
                                                       DevCtrl* ctrl) {
  const int lane = threadIdx.x & 63;
  const int row = 2 * (blockIdx.x * 4 + (threadIdx.x >> 6));  // rows row, row + 1 (mp is even)
  if (row >= mp) return;
  const double* __restrict__ a0 = A + (size_t)row * ld;
  const double* __restrict__ a1 = a0 + ld;
  const vd2 z = {0.0, 0.0};
  RowAcc q0{z, z, z, z, z, z, z, z}, q1{z, z, z, z, z, z, z, z};
  int j = 2 * lane;
  for (; j + 384 < cols; j += 512) {
    vd2 sv[4], yv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      sv[u] = *reinterpret_cast<const vd2*>(s + j + 128 * u);
      yv[u] = *reinterpret_cast<const vd2*>(x1 + j + 128 * u);
    }
    row_acc4(q0, a0, j, sv, yv);
    row_acc4(q1, a1, j, sv, yv);
  }
  for (; j < cols; j += 128) {
    const vd2 s0 = *reinterpret_cast<const vd2*>(s + j), y0 = *reinterpret_cast<const vd2*>(x1 + j);
    row_acc1(q0, a0, j, s0, y0);
    row_acc1(q1, a1, j, s0, y0);
  }
  ls_setup_eval_row(q0, row, e, eabs, r, ub, c, d, invd, w, logd, cabs, ctrl, lane);
  ls_setup_eval_row(q1, row + 1, e, eabs, r, ub, c, d, invd, w, logd, cabs, ctrl, lane);
}
void launch_ls_setup_eval(hipStream_t st, const double* A, int ld, int mp, int cols, const double* s, const double* x1,
                          double* e, double* eabs, const double* r, const double* ub, double* c, double* d,
                          double* invd, double* w, double* logd, double* cabs, DevCtrl* ctrl) {
  k_ls_setup_eval<<<(mp / 2 + 3) / 4, 256, 0, st>>>(A, ld, mp, cols, s, x1, e, eabs, r, ub, c, d, invd, w, logd, cabs,
                                                    ctrl);
}

// s = dx and x1 = x + s * 1 (k_axpy's expression at t = 1); the speculative counters zeroed
__global__ void k_spec_prep(const double* __restrict__ dx, const double* __restrict__ x, int n, double* __restrict__ s,
                            double* __restrict__ x1, DevCtrl* ctrl) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const double v = dx[i];
    s[i] = v;
    x1[i] = x[i] + v * 1.0;
  }
  if (i == 0) {
    ctrl->spec_infeasible = 0;
    ctrl->spec_not_strict = 0;
  }
}
void launch_spec_prep(hipStream_t st, const double* dx, const double* x, int n, double* s, double* x1, DevCtrl* ctrl) {
  k_spec_prep<<<(n + 255) / 256, 256, 0, st>>>(dx, x, n, s, x1, ctrl);
}
// the evaluation's counters from the speculative ones (the evaluation at x1 is taken over)
__global__ void k_ctrl_take_spec(DevCtrl* ctrl) {
  ctrl->infeasible = ctrl->spec_infeasible;
  ctrl->not_strict = ctrl->spec_not_strict;
}
void launch_ctrl_take_spec(hipStream_t st, DevCtrl* ctrl) { k_ctrl_take_spec<<<1, 1, 0, st>>>(ctrl); }

// ------------------------------------------------------------------------------------------------
// Column reductions A' v: grid (cols/512, rows/64); thread owns 2 adjacent columns, loops 64 rows.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_coldot_partials(const double* __restrict__ M, int ld, int rows, int cols,
                                                         const double* __restrict__ v, double* __restrict__ part) {
  const int j = (blockIdx.x * 256 + threadIdx.x) * 2;
  const int r0 = blockIdx.y * COLDOT_ROWS;
  if (j >= cols) return;
  vd2 a0 = {0.0, 0.0}, a1 = {0.0, 0.0};
  const int rend = min(r0 + COLDOT_ROWS, rows);  // rows is a multiple of 64
  const double* mp = M + j;
  for (int i = r0; i < rend; i += 4) {
    const vd2 m0 = *reinterpret_cast<const vd2*>(mp + (size_t)i * ld);
    const vd2 m1 = *reinterpret_cast<const vd2*>(mp + (size_t)(i + 1) * ld);
    const vd2 m2 = *reinterpret_cast<const vd2*>(mp + (size_t)(i + 2) * ld);
    const vd2 m3 = *reinterpret_cast<const vd2*>(mp + (size_t)(i + 3) * ld);
    a0 = __builtin_elementwise_fma(m0, (vd2){v[i], v[i]}, a0);
    a1 = __builtin_elementwise_fma(m1, (vd2){v[i + 1], v[i + 1]}, a1);
    a0 = __builtin_elementwise_fma(m2, (vd2){v[i + 2], v[i + 2]}, a0);
    a1 = __builtin_elementwise_fma(m3, (vd2){v[i + 3], v[i + 3]}, a1);
  }
  *reinterpret_cast<vd2*>(part + (size_t)blockIdx.y * cols + j) = a0 + a1;
}

int coldot_chunks(int rows) { return (rows + COLDOT_ROWS - 1) / COLDOT_ROWS; }

void launch_coldot_partials(hipStream_t s, const double* M, int ld, int rows, int cols, const double* v,
                            double* part) {
  dim3 grid((cols / 2 + 255) / 256, coldot_chunks(rows));
  k_coldot_partials<<<grid, 256, 0, s>>>(M, ld, rows, cols, v, part);
}

__global__ void k_gradient_finalize(const double* __restrict__ a0, const double* __restrict__ Px,
                                    const double* __restrict__ part, int nchunks, int cols, const DevCtrl* ctrl,
                                    double* __restrict__ y) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= cols) return;
  const double t = ctrl->t;
  // objF.gradientAt(x) * t  (QuadraticObjectiveFunction.scala:32: a + P*x), then + sum_i a_i/d_i
  double g = (Px ? (a0[j] + Px[j]) : a0[j]) * t;
  double s = 0.0;
#pragma unroll 16
  for (int c = 0; c < nchunks; ++c) s += part[(size_t)c * cols + j];  // (loads in flight; the sum stays in order)
  y[j] = g + s;
}

void launch_gradient_finalize(hipStream_t s, const double* a0, const double* Px, const double* part,
                              int nchunks, int n_cols, const DevCtrl* ctrl, double* y) {
  k_gradient_finalize<<<(n_cols + 255) / 256, 256, 0, s>>>(a0, Px, part, nchunks, n_cols, ctrl, y);
}

// ------------------------------------------------------------------------------------------------
// Deterministic single-block reductions into ctrl->sc[slot].
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_dot(const double* __restrict__ u, const double* __restrict__ v, int n,
                                              DevCtrl* ctrl, int slot) {
  __shared__ double red[16];
  double acc = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) acc = fma(u[i], v ? v[i] : u[i], acc);
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) ctrl->sc[slot] = acc;
}

__global__ __launch_bounds__(1024) void k_sum(const double* __restrict__ u, int n, DevCtrl* ctrl, int slot) {
  __shared__ double red[16];
  double acc = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) acc += u[i];
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) ctrl->sc[slot] = acc;
}

// A batch of the reductions above, one block each: the per-thread loop and block_sum of each kind are those of
// k_dot / k_sum, so a batched sum is bitwise the single-launch one (one launch instead of up to 8).
__global__ __launch_bounds__(1024) void k_dots(DotBatch a, DevCtrl* ctrl) {
  __shared__ double red[16];
  const int b = blockIdx.x;
  const double* u = a.u[b];
  const double* v = a.v[b];
  const int n = a.n[b];
  double acc = 0.0;
  switch (a.kind[b]) {
    case DOT_FMA:
      for (int i = threadIdx.x; i < n; i += blockDim.x) acc = fma(u[i], v ? v[i] : u[i], acc);
      break;
    case DOT_SUM:
      for (int i = threadIdx.x; i < n; i += blockDim.x) acc += u[i];
      break;
    default:
      for (int i = threadIdx.x; i < n; i += blockDim.x) acc = fma(fabs(u[i]), v ? fabs(v[i]) : 1.0, acc);
      break;
  }
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) ctrl->sc[a.slot[b]] = acc;
}
void launch_dots(hipStream_t s, const DotBatch& a, DevCtrl* ctrl) {
  if (a.count > 0) k_dots<<<a.count, 1024, 0, s>>>(a, ctrl);
}
void launch_dot(hipStream_t s, const double* u, const double* v, int n, DevCtrl* ctrl, int slot) {
  k_dot<<<1, 1024, 0, s>>>(u, v, n, ctrl, slot);
}
void launch_sum(hipStream_t s, const double* u, int n, DevCtrl* ctrl, int slot) {
  k_sum<<<1, 1024, 0, s>>>(u, n, ctrl, slot);
}

__global__ void k_axpy(const double* __restrict__ u, const double* __restrict__ v, double alpha, int n,
                       double* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = u[i] + v[i] * alpha;  // x + s*t  (UnconstrainedSolver.scala:130)
}
void launch_axpy(hipStream_t s, const double* u, const double* v, double alpha, int n, double* out) {
  k_axpy<<<(n + 255) / 256, 256, 0, s>>>(u, v, alpha, n, out);
}

// diagonalizationSolve coefficients (MatrixUtils.scala:625, 639): a_j = (|d_j| > 0) ? u_j.b : 0, z_j = a_j / d_j
__global__ void k_eig_coeffs(const double* __restrict__ dots, const double* __restrict__ d, int n2, int npad,
                             double* __restrict__ a, double* __restrict__ z) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= npad) return;
  const bool nz = j < n2 && fabs(d[j]) > 0.0;
  a[j] = nz ? dots[j] : 0.0;
  z[j] = nz ? dots[j] / d[j] : 0.0;
}
void launch_eig_coeffs(hipStream_t s, const double* dots, const double* d, int n2, int npad, double* a, double* z) {
  k_eig_coeffs<<<(npad + 255) / 256, 256, 0, s>>>(dots, d, n2, npad, a, z);
}
// out_i = sum_c part[c][i] in a fixed order (column-reduction partials of k_coldot_partials)
__global__ void k_sum_chunks(const double* __restrict__ part, int nchunks, int cols, double* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cols) return;
  double s = 0.0;
#pragma unroll 8
  for (int c = 0; c < nchunks; ++c) s += part[(size_t)c * cols + i];
  out[i] = s;
}
void launch_sum_chunks(hipStream_t s, const double* part, int nchunks, int cols, double* out) {
  k_sum_chunks<<<(cols + 255) / 256, 256, 0, s>>>(part, nchunks, cols, out);
}
// KKT matrix [H A'; A 0] (KKTSystem.scala kktMatrix), row-major (n + p) x (n + p) with leading dimension ld
__global__ void k_kkt_matrix(const double* __restrict__ H, int ldh, const double* __restrict__ Aeq, int lda, int n,
                             int p, int ld, double* __restrict__ K) {
  const int i = blockIdx.y, j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= ld) return;
  double v = 0.0;
  if (i < n && j < n) v = H[(size_t)i * ldh + j];
  else if (i < n && j >= n && j < n + p) v = Aeq[(size_t)(j - n) * lda + i];
  else if (i >= n && i < n + p && j < n) v = Aeq[(size_t)(i - n) * lda + j];
  K[(size_t)i * ld + j] = v;
}
void launch_kkt_matrix(hipStream_t s, const double* H, int ldh, const double* Aeq, int lda, int n, int p, int ld,
                       double* K) {
  k_kkt_matrix<<<dim3((ld + 255) / 256, ld), 256, 0, s>>>(H, ldh, Aeq, lda, n, p, ld, K);
}

__global__ void k_scale_vec(const double* __restrict__ u, const double* __restrict__ d, int n,
                            double* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = d[i] * u[i];
}
void launch_scale_vec(hipStream_t s, const double* u, const double* d, int n, double* out) {
  k_scale_vec<<<(n + 255) / 256, 256, 0, s>>>(u, d, n, out);
}

// ------------------------------------------------------------------------------------------------
// Ruiz equilibration, MatrixUtils.scala:240-268 (Jacobi form: a sweep reads d of the previous sweep).
// Sweep k runs iff rho[k] > 1e-6 (rho[0] = 1); it writes d into the other buffer and max|1-u| into rho[k+1].
// ------------------------------------------------------------------------------------------------
__global__ void k_ruiz_init(double* d0, double* d1, int np, DevCtrl* ctrl, int* work, int nwork) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < np) {
    d0[i] = 1.0;
    if (d1) d1[i] = 1.0;
  }
  if (i < nwork) work[i] = 0;
  if (i < RUIZ_MAX + 2) ctrl->ruiz_rho[i] = (i == 0) ? (unsigned long long)__double_as_longlong(1.0) : 0ull;
}
void launch_ruiz_init(hipStream_t s, double* d0, int np, DevCtrl* ctrl, double* d1, int* work, size_t nwork) {
  const int m = np > (int)nwork ? np : (int)nwork;
  k_ruiz_init<<<(m + 255) / 256, 256, 0, s>>>(d0, d1, np, ctrl, work, (int)nwork);
}

// Lower-triangle form of the sweep: H is exactly symmetric (the assembly mirrors its lower triangle), so
// sum_j (d_j H_ij)^2 over a full row is assembled from the 64 x 64 tiles (I, J), J <= I, of the lower
// triangle alone -- half the bytes per sweep.  Tile (I, J) writes
//   S[J][i] = sum_{j in J} (d_j H_ij)^2   for its rows i in I      (row partials)
//   S[I][j] = sum_{i in I} (d_i H_ij)^2   for its columns j in J   (column partials = rows of H_JI, I > J)
// so every S[X][r] is written by exactly one tile, and k_ruiz_rows adds S[0..nbn)[r] in a fixed order.  The per-tile
// arithmetic is ruiz_tile.hpp's (shared with the one-launch loop, k_ruiz.hip).
__global__ __launch_bounds__(256) void k_ruiz_tiles(const double* __restrict__ H, int ld, int nbn,
                                                    const double* __restrict__ dcur, double* __restrict__ S,
                                                    const DevCtrl* ctrl, int k) {
  const double rho = __longlong_as_double((long long)ctrl->ruiz_rho[k]);
  if (!(rho > 1e-6)) return;
  // blockIdx.x -> (I, J), J <= I, row-major over the lower triangle
  const int t = blockIdx.x;
  int I = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while ((I + 1) * (I + 2) / 2 <= t) ++I;
  while (I * (I + 1) / 2 > t) --I;
  const int J = t - I * (I + 1) / 2;
  __shared__ double cred[8][NB];
  const int tid = threadIdx.x;
  const int c2 = tid & 31, g = tid >> 5;  // column pair 2*c2, row group g: rows g + 8q
  const double* tile = H + (size_t)I * NB * ld + (size_t)J * NB;
  vd2 h[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) h[q] = *reinterpret_cast<const vd2*>(tile + (size_t)(g + 8 * q) * ld + 2 * c2);
  const vd2 dj = *reinterpret_cast<const vd2*>(dcur + J * NB + 2 * c2);
  vd2 csum = {0.0, 0.0};
  double rs[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const double di = dcur[I * NB + g + 8 * q];
    const vd2 a = dj * h[q];
    rs[q] = a[0] * a[0] + a[1] * a[1];
    const vd2 b = h[q] * di;
    csum = __builtin_elementwise_fma(b, b, csum);
  }
  rz_rowgroup_sum8(rs);
  if (c2 == RZ_ROW_LANE) {
#pragma unroll
    for (int q = 0; q < 8; ++q) S[(size_t)J * (nbn * NB) + I * NB + g + 8 * q] = rs[q];
  }
  if (I == J) return;  // a diagonal tile's rows already cover its columns
  cred[g][2 * c2] = csum[0];
  cred[g][2 * c2 + 1] = csum[1];
  __syncthreads();
  if (tid < NB) {
    double v = cred[0][tid];
#pragma unroll
    for (int r = 1; r < 8; ++r) v += cred[r][tid];
    S[(size_t)I * (nbn * NB) + J * NB + tid] = v;
  }
}

__global__ __launch_bounds__(256) void k_ruiz_rows(const double* __restrict__ S, int nbn, int n, int np,
                                                   const double* __restrict__ dcur, double* __restrict__ dnext,
                                                   DevCtrl* ctrl, int k) {
  const double rho = __longlong_as_double((long long)ctrl->ruiz_rho[k]);
  if (!(rho > 1e-6)) return;
  // 64 rows per workgroup; wave q adds the partials X = q, q + 4, ... (independent loads in flight), then the
  // four wave sums are added in a fixed order.
  __shared__ double red[4][64];
  const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int row = blockIdx.x * 64 + lane;
  const int ldS = nbn * NB;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  if (row < n) {
    int X = q;
    for (; X + 12 < nbn; X += 16) {
      s0 += S[(size_t)X * ldS + row];
      s1 += S[(size_t)(X + 4) * ldS + row];
      s2 += S[(size_t)(X + 8) * ldS + row];
      s3 += S[(size_t)(X + 12) * ldS + row];
    }
    for (; X < nbn; X += 4) s0 += S[(size_t)X * ldS + row];
  }
  red[q][lane] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (q != 0) return;
  double m = 0.0;
  if (row < n) {
    const double ssum = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
    const double di = dcur[row];
    const double u = sqrt(di * sqrt(ssum));        // sqrt(norm(Q(i,::)))   MatrixUtils.scala:258
    const double v = (u > 0) ? 1.0 / u : 1.0;      // :259
    dnext[row] = di * v;                           // :260
    m = fabs(1.0 - u);                             // :261-262
  } else if (row < np) {
    dnext[row] = 1.0;
  }
  m = wave_max(m);  // every lane of wave 0 is live here
  if (lane == 0 && m > 0.0) atomic_max_pos(&ctrl->ruiz_rho[k + 1], m);
}

void launch_ruiz_sweep_tri(hipStream_t s, const double* H, int ld, int n, int np, const double* dcur, double* dnext,
                           double* S, DevCtrl* ctrl, int k) {
  const int nbn = (n + NB - 1) / NB;
  k_ruiz_tiles<<<nbn * (nbn + 1) / 2, 256, 0, s>>>(H, ld, nbn, dcur, S, ctrl, k);
  k_ruiz_rows<<<(np + 63) / 64, 256, 0, s>>>(S, nbn, n, np, dcur, dnext, ctrl, k);
}

// k1 = the sweeps launched so far.  K = the first k < k1 whose rho[k] <= 1e-6 (sweeps K.. exited), else k1;
// K == k1 < RUIZ_MAX with rho[k1] > 1e-6 means the loop is not done: ruiz_sweeps = -1 (cvxg.cpp: ruiz_lookahead).
__global__ void k_ruiz_final(const double* __restrict__ d0, const double* __restrict__ d1, int np,
                             double* __restrict__ dfin, DevCtrl* ctrl, int k1, const int* abortw) {
  int K = k1;
  for (int k = 0; k < k1; ++k) {
    if (!(__longlong_as_double((long long)ctrl->ruiz_rho[k]) > 1e-6)) {
      K = k;
      break;
    }
  }
  const bool open = K == k1 && k1 < RUIZ_MAX && __longlong_as_double((long long)ctrl->ruiz_rho[k1]) > 1e-6;
  const double* src = (K & 1) ? d1 : d0;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < np) dfin[i] = src[i];
  if (i == 0) ctrl->ruiz_sweeps = (abortw && *abortw) ? -2 : (open ? -1 : K);
}
void launch_ruiz_final(hipStream_t s, const double* d0, const double* d1, int np, double* dfin, DevCtrl* ctrl, int k1,
                       const int* abortw) {
  k_ruiz_final<<<(np + 255) / 256, 256, 0, s>>>(d0, d1, np, dfin, ctrl, k1, abortw);
}

// Q = (dd') o H (+ reg I), lower triangle into L; padded part: identity.   MatrixUtils.scala:267, :454
__global__ __launch_bounds__(256) void k_form_q(const double* __restrict__ H, double* __restrict__ L, int ld,
                                                int n, int np, const double* __restrict__ d,
                                                const DevCtrl* ctrl) {
  const int i = blockIdx.y;
  const int j = (blockIdx.x * 256 + threadIdx.x) * 2;
  if (j > i) return;
  const double reg = ctrl->reg;
  double2 o;
  if (i < n) {
    const double di = d[i];
    const double2 h = *reinterpret_cast<const double2*>(H + (size_t)i * ld + j);
    const double2 dj = *reinterpret_cast<const double2*>(d + j);
    o.x = (j < n) ? (di * dj.x) * h.x : 0.0;
    o.y = (j + 1 < n) ? (di * dj.y) * h.y : 0.0;
    if (j == i) o.x += reg;
    if (j + 1 == i) o.y += reg;
  } else {
    o.x = (j == i) ? 1.0 : 0.0;
    o.y = (j + 1 == i) ? 1.0 : 0.0;
  }
  *reinterpret_cast<double2*>(L + (size_t)i * ld + j) = o;
}
void launch_form_q(hipStream_t s, const double* H, double* L, int ld, int n, int np, const double* d,
                   const DevCtrl* ctrl) {
  dim3 grid((np / 2 + 255) / 256, np);
  k_form_q<<<grid, 256, 0, s>>>(H, L, ld, n, np, d, ctrl);
}

__global__ void k_add_diag(double* H, int ld, int n, double v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) H[(size_t)i * ld + i] += v;
}
__global__ void k_copy_diag(const double* H, int ld, int n, double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = H[(size_t)i * ld + i];
}
__global__ void k_set_diag(double* H, int ld, int n, const double* diag) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) H[(size_t)i * ld + i] = diag[i];
}
void launch_add_diag(hipStream_t s, double* H, int ld, int n, double v) {
  k_add_diag<<<(n + 255) / 256, 256, 0, s>>>(H, ld, n, v);
}
void launch_copy_diag(hipStream_t s, const double* H, int ld, int n, double* out) {
  k_copy_diag<<<(n + 255) / 256, 256, 0, s>>>(H, ld, n, out);
}
void launch_set_diag(hipStream_t s, double* H, int ld, int n, const double* diag) {
  k_set_diag<<<(n + 255) / 256, 256, 0, s>>>(H, ld, n, diag);
}

// ------------------------------------------------------------------------------------------------
// Line search trials (UnconstrainedSolver.scala:107-128): the reference evaluates g_i(x + s t) for the
// geometric sequence t = beta^k.  g is affine, so g_i(x + s t) = g_i(x) + t (a_i . s): one GEMV e = A s
// per Newton step, then O(m) per trial.  Each thread owns one constraint and sweeps LS_TRIALS trials.
// ------------------------------------------------------------------------------------------------
int ls_blocks(int m) { return (m + 255) / 256; }

// Certified decisions (cabs != nullptr): the trial value c_i + t e_i and the reference's fresh evaluation
// r_i + a_i.(x + s t) both lie within B_i(t) = gamma (cabs_i + t eabs_i) of the exact g_i(x + s t), with cabs_i = |r_i|
// + |a_i|.|x|, eabs_i = |a_i|.|s| and gamma = 4 (n + 16) u.  A QuadraticConstraint row (g = c + t e + t^2 f / 2 with
// e = (a + P x).s, f = s'P s) adds |x|'|P||x|/2 to cabs, |s|'|P||x| to eabs and the band term t^2 fabs / 2 with
// fabs = |s|'|P||s| (the expansion of |x + s t|'|P||x + s t| / 2).  A constraint whose feasibility margin is inside that
// band counts as ambiguous (the host then evaluates that trial fresh); per trial the kernel also sums the first-
// order bound of the log-sum error, sum_i (B_i + 4u(|g_i| + |ub_i|)) / d_i, and sum_i |log d_i| (+inf when some
// B_i is not small against d_i).
__global__ __launch_bounds__(256) void k_ls_trials(const double* __restrict__ c, const double* __restrict__ e,
                                                   const double* __restrict__ ub, int m, double tbase, double beta,
                                                   double* __restrict__ part_log, int* __restrict__ part_cnt,
                                                   const double* __restrict__ f, const double* __restrict__ cabs,
                                                   const double* __restrict__ eabs, double gamma,
                                                   double* __restrict__ part_aux, const double* __restrict__ fabsq) {
  // blockIdx.y = group of LS_GROUP consecutive trials (more workgroups than ceil(m/256) alone)
  constexpr int LS_GROUP = 8;
  constexpr double U = 1.1102230246251565e-16;  // 2^-53
  __shared__ double slog[4][LS_GROUP], serr[4][LS_GROUP], sabs[4][LS_GROUP];
  __shared__ int sviol[4][LS_GROUP], snpos[4][LS_GROUP], ssure[4][LS_GROUP], samb[4][LS_GROUP];
  const int k0 = blockIdx.y * LS_GROUP;
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const bool valid = i < m;
  const double ci = valid ? c[i] : 0.0, ei = valid ? e[i] : 0.0, ubi = valid ? ub[i] : 1.0;
  const double fi = (valid && f) ? f[i] : 0.0;  // s'P s of a QuadraticConstraint row (0: linear)
  const bool cert = cabs != nullptr;
  const double ca = (valid && cert) ? cabs[i] : 0.0, ea = (valid && cert) ? eabs[i] : 0.0;
  const double fa = (valid && cert && fabsq) ? fabsq[i] : 0.0;
  double t = tbase;
  for (int q = 0; q < k0; ++q) t *= beta;  // the same product chain as trial by trial
  for (int kk = 0; kk < LS_GROUP; ++kk) {
    const double g = f ? (ci + t * ei) + (t * t * fi) / 2 : ci + t * ei;
    const double dd = ubi - g;
    const double gs = g * (1 + 3e-16);
    const bool viol = valid && !(gs < ubi);   // Constraint.scala:23
    const bool npos = valid && !(dd > 0.0);   // BarrierSolver.scala:284
    const double lg = (valid && dd > 0.0) ? log(dd) : 0.0;
    bool sure = false, amb = false;
    double lerr = 0.0, labs = 0.0;
    if (valid && cert) {
      const double band = fabsq ? gamma * ((ca + t * ea) + (t * t * fa) / 2) : gamma * (ca + t * ea);
      const double bt = band * (1 + 3e-16) + 4 * U * (fabs(g) + fabs(ubi));
      const double margin = gs - ubi;  // >= 0: violated
      sure = margin > bt;
      amb = !sure && !(margin < -bt);
      if (dd > 0.0) {
        const double bd = band + 4 * U * (fabs(g) + fabs(ubi));
        lerr = (bd < 0.25 * dd) ? 2.0 * bd / dd : __builtin_inf();
        labs = fabs(lg);
      }
    }
    const double sl = wave_sum(lg), se = wave_sum(lerr), sa = wave_sum(labs);
    const unsigned long long bv = __ballot(viol), bn = __ballot(npos), bs = __ballot(sure), ba = __ballot(amb);
    if (lane == 0) {
      slog[wid][kk] = sl;
      serr[wid][kk] = se;
      sabs[wid][kk] = sa;
      sviol[wid][kk] = __popcll(bv);
      snpos[wid][kk] = __popcll(bn);
      ssure[wid][kk] = __popcll(bs);
      samb[wid][kk] = __popcll(ba);
    }
    t *= beta;  // t *= beta (repeated products, not pow)   UnconstrainedSolver.scala:93
  }
  __syncthreads();
  if (threadIdx.x < LS_GROUP) {
    const int kk = threadIdx.x, k = k0 + kk;
    double s = 0.0, se = 0.0, sa = 0.0;
    int v = 0, np_ = 0, su = 0, am = 0;
    for (int w = 0; w < 4; ++w) {
      s += slog[w][kk];
      se += serr[w][kk];
      sa += sabs[w][kk];
      v += sviol[w][kk];
      np_ += snpos[w][kk];
      su += ssure[w][kk];
      am += samb[w][kk];
    }
    const size_t o = (size_t)blockIdx.x * LS_TRIALS + k;
    part_log[o] = s;
    part_aux[2 * o] = se;
    part_aux[2 * o + 1] = sa;
    part_cnt[4 * o + 0] = v;
    part_cnt[4 * o + 1] = np_;
    part_cnt[4 * o + 2] = su;
    part_cnt[4 * o + 3] = am;
  }
}

void launch_ls_trials(hipStream_t s, const double* c, const double* e, const double* ub, int m, double tbase,
                      double beta, double* part_log, int* part_cnt, const double* f, const double* cabs,
                      const double* eabs, double gamma, double* part_aux, const double* fabsq) {
  k_ls_trials<<<dim3(ls_blocks(m), LS_TRIALS / 8), 256, 0, s>>>(c, e, ub, m, tbase, beta, part_log, part_cnt, f, cabs,
                                                                eabs, gamma, part_aux, fabsq);
}

// KL dual objective along the trial steps: per trial k, sum_j R exp(-(v_j + t_k u_j)) (v = B'z, u = B's),
// the vec_R dot exp(-B'(z + s t)) term of Dist_KL.dualObjFAt (Dist_KL.scala:146-147); t_k by repeated products.
// One 1024-thread block per trial, summed exactly as sum_j y_j at z is (k_sum over the noutp entries of k_kl_eval's y:
// per thread j = tid + 1024 i, then block_sum), so a trial whose exponents equal z's gives that sum bitwise (k_ls_klp).
// With vabs / uabs (= |B'||z|, |B'||s|; certified mode) also its error scale against any evaluation order of
// B'(z + s t): sum_j y_j (gamma (vabs_j + t_k uabs_j) + 4u) (the exponent's error propagated through exp).
__global__ __launch_bounds__(1024) void k_ls_kl(const double* __restrict__ v, const double* __restrict__ u, int nout,
                                                double R, double tbase, double beta, double* __restrict__ out,
                                                const double* __restrict__ vabs, const double* __restrict__ uabs,
                                                double gamma) {
  constexpr double U = 1.1102230246251565e-16;  // 2^-53
  __shared__ double red[16];
  const int k = blockIdx.x;
  double t = tbase;
  for (int q = 0; q < k; ++q) t *= beta;
  double sw = 0.0, se = 0.0;
  for (int j = threadIdx.x; j < nout; j += blockDim.x) {  // (j >= nout: k_kl_eval's y is 0 there, exact zeros)
    const double y = R * exp(-(v[j] + t * u[j]));
    sw += y;
    if (vabs) se += y * (gamma * (vabs[j] + t * uabs[j]) + 4 * U);
  }
  sw = block_sum(sw, red);
  se = block_sum(se, red);
  if (threadIdx.x == 0) {
    out[k] = sw;
    out[LS_TRIALS + k] = se;
  }
}
int ls_kl_blocks(int nout) { return (nout + 255) / 256; }
void launch_ls_kl(hipStream_t s, const double* v, const double* u, int nout, double R, double tbase, double beta,
                  double* part, double* out, const double* vabs, const double* uabs, double gamma) {
  (void)part;
  k_ls_kl<<<LS_TRIALS, 1024, 0, s>>>(v, u, nout, R, tbase, beta, out, vabs, uabs, gamma);
}

// KL primal objective Dist_KL.objectiveFunction(n) (Dist_KL.scala:223-239) at x, per coordinate j < n:
//   lx_j = log(x_j * n)                      (valueAt = x dot log(x*n.toDouble): the dot is taken over x and lx)
//   g0_j = (1 + log(x_j)) + log(n)            (gradientAt, left to right)
//   hd_j = 1 / x_j                            (hessianAt = diag(1/x))
//   ab_j = |x_j lx_j| + |x_j|                 (error scale of the value term, certified line search)
// zeros on the padding.
__global__ void k_klp_eval(const double* __restrict__ x, int n, int np, double nd, double* __restrict__ lx,
                           double* __restrict__ g0, double* __restrict__ hd, double* __restrict__ ab) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= np) return;
  double l = 0.0, g = 0.0, h = 0.0, a = 0.0;
  if (j < n) {
    const double xj = x[j];
    l = log(xj * nd);
    g = (1.0 + log(xj)) + log(nd);
    h = 1.0 / xj;
    a = fabs(xj * l) + fabs(xj);
  }
  lx[j] = l;
  if (g0) g0[j] = g;
  if (hd) hd[j] = h;
  if (ab) ab[j] = a;
}
void launch_klp_eval(hipStream_t s, const double* x, int n, int np, double nd, double* lx, double* g0, double* hd,
                     double* ab) {
  k_klp_eval<<<(np + 255) / 256, 256, 0, s>>>(x, n, np, nd, lx, g0, hd, ab);
}

// KL primal objective at the LS_TRIALS trial points xt = x + s*t_k (t_k = tbase beta^k by repeated products, as the
// host's backtracking; x + s*t with two roundings, as Breeze's x + s*t): per trial {sum_j xt_j log(xt_j n),
// sum_j |xt_j log(xt_j n)| + |xt_j|}.  One 1024-thread block per trial, and the value sum is formed exactly as the
// objective at x is (k_dots' DOT_FMA over x and log(n x): fma(xt_j, log(xt_j n), acc) per thread over j = tid +
// 1024 i, then block_sum), so a trial point equal to x gives bitwise the f(x) the Armijo test compares with -- as in
// the reference, where both sides are objF.valueAt (EqualityConstrainedSolver.scala:52, 88).  (A different summation
// order left f(x + s t) a few ulps of t f0 above f(x) at every small t: late in the path, where one ulp of f exceeds
// the decrease alpha t q, no trial could pass and the line search threw at it == 100.)  A trial outside the domain
// (some xt_j <= 0) gives a NaN / -inf sum; the backtracking into C has rejected it before Armijo reads it.
__global__ __launch_bounds__(1024) void k_ls_klp(const double* __restrict__ x, const double* __restrict__ sdir, int n,
                                                 double nd, double tbase, double beta, double* __restrict__ out) {
  __shared__ double red[16];
  const int k = blockIdx.x;
  double t = tbase;
  for (int q = 0; q < k; ++q) t *= beta;
  double v = 0.0, a = 0.0;
  for (int j = threadIdx.x; j < n; j += blockDim.x) {  // (j >= n: x = s = 0 adds exact zeros to the dot at x)
    const double xt = x[j] + sdir[j] * t;
    const double l = log(xt * nd);
    v = fma(xt, l, v);
    a += fabs(xt * l) + fabs(xt);
  }
  v = block_sum(v, red);
  a = block_sum(a, red);
  if (threadIdx.x == 0) {
    out[k] = v;
    out[LS_TRIALS + k] = a;
  }
}
int ls_klp_blocks(int n) { return (n + 255) / 256; }
void launch_ls_klp(hipStream_t s, const double* x, const double* sdir, int n, double nd, double tbase, double beta,
                   double* part, double* out) {
  (void)part;
  k_ls_klp<<<LS_TRIALS, 1024, 0, s>>>(x, sdir, n, nd, tbase, beta, out);
}

// KL dual at z (v = B'z given): y_j = R exp(-v_j) for j < nout (Dist_KL.scala:163, 170), 0 on the padding
__global__ void k_kl_eval(const double* __restrict__ v, int nout, int noutp, double R, double* __restrict__ y) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < noutp) y[j] = (j < nout) ? R * exp(-v[j]) : 0.0;
}
void launch_kl_eval(hipStream_t s, const double* v, int nout, int noutp, double R, double* y) {
  k_kl_eval<<<(noutp + 255) / 256, 256, 0, s>>>(v, nout, noutp, R, y);
}

// out: per trial k, out_log[3k..3k+2] = {sum log d, log-sum error bound, sum |log d|} and out_cnt[4k..4k+3] =
// {violations, d <= 0, sure violations, ambiguous}; blocks summed in a fixed order.
__global__ void k_ls_finalize(const double* __restrict__ part_log, const int* __restrict__ part_cnt,
                              const double* __restrict__ part_aux, int nblocks, double* __restrict__ out_log,
                              int* __restrict__ out_cnt) {
  const int k = threadIdx.x;
  if (k >= LS_TRIALS) return;
  double s = 0.0, se = 0.0, sa = 0.0;
  int c4[4] = {0, 0, 0, 0};
#pragma unroll 8
  for (int b = 0; b < nblocks; ++b) {  // (loads in flight; the sums stay in block order)
    const size_t o = (size_t)b * LS_TRIALS + k;
    s += part_log[o];
    se += part_aux[2 * o];
    sa += part_aux[2 * o + 1];
    for (int q = 0; q < 4; ++q) c4[q] += part_cnt[4 * o + q];
  }
  out_log[3 * k] = s;
  out_log[3 * k + 1] = se;
  out_log[3 * k + 2] = sa;
  for (int q = 0; q < 4; ++q) out_cnt[4 * k + q] = c4[q];
}
void launch_ls_finalize(hipStream_t s, const double* part_log, const int* part_cnt, const double* part_aux,
                        int nblocks, double* out_log, int* out_cnt) {
  k_ls_finalize<<<1, 64, 0, s>>>(part_log, part_cnt, part_aux, nblocks, out_log, out_cnt);
}

}  // namespace cvxg

// ------------------------------------------------------------------------------------------------
// Small control / vector helpers (stream-ordered, kernel arguments captured at launch).
// ------------------------------------------------------------------------------------------------
namespace cvxg {

__global__ void k_ctrl_set(DevCtrl* ctrl, int which, double v) {
  if (which == 0) ctrl->t = v;
  else if (which == 1) ctrl->reg = v;
}
__global__ void k_ctrl_reset_eval(DevCtrl* ctrl) {
  ctrl->infeasible = 0;
  ctrl->not_strict = 0;
}
__global__ void k_ctrl_reset_chol(DevCtrl* ctrl) {
  ctrl->chol_info = 0;
  ctrl->df_status = 0;
  ctrl->min_diag = (unsigned long long)__double_as_longlong(__builtin_inf());
}
void launch_ctrl_set(hipStream_t s, DevCtrl* ctrl, int which, double v) { k_ctrl_set<<<1, 1, 0, s>>>(ctrl, which, v); }
void launch_ctrl_reset_eval(hipStream_t s, DevCtrl* ctrl) { k_ctrl_reset_eval<<<1, 1, 0, s>>>(ctrl); }
void launch_ctrl_reset_chol(hipStream_t s, DevCtrl* ctrl) { k_ctrl_reset_chol<<<1, 1, 0, s>>>(ctrl); }
__global__ void k_factor_prep(DevCtrl* ctrl, double reg, int* __restrict__ work, int nwork) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nwork) work[i] = 0;
  if (i == 0) {
    ctrl->reg = reg;
    ctrl->small_piv = 0;
    ctrl->chol_info = 0;
    ctrl->df_status = 0;
    ctrl->min_diag = (unsigned long long)__double_as_longlong(__builtin_inf());
  }
}
void launch_factor_prep(hipStream_t s, DevCtrl* ctrl, double reg, int* work, size_t nwork) {
  k_factor_prep<<<(unsigned)((nwork + 255) / 256), 256, 0, s>>>(ctrl, reg, work, (int)nwork);
}

// A host read without a stream synchronisation: one workgroup copies up to two device ranges (8-byte words) into
// coherent (fine-grained) pinned host memory, makes its stores visible at system scope, then raises the sequence word
// the host spins on (cvxg.cpp: host_read).  Vector stores only.
__global__ __launch_bounds__(256) void k_publish(const unsigned long long* __restrict__ s0, unsigned long long* d0, int w0,
                                                 const unsigned long long* __restrict__ s1, unsigned long long* d1,
                                                 int w1, unsigned* flag, unsigned seq) {
  for (int i = threadIdx.x; i < w0; i += blockDim.x) d0[i] = s0[i];
  for (int i = threadIdx.x; i < w1; i += blockDim.x) d1[i] = s1[i];
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
void launch_publish(hipStream_t s, const void* s0, void* d0, size_t bytes0, const void* s1, void* d1, size_t bytes1,
                    unsigned* flag, unsigned seq) {
  k_publish<<<1, 256, 0, s>>>(static_cast<const unsigned long long*>(s0), static_cast<unsigned long long*>(d0),
                              (int)(bytes0 / 8), static_cast<const unsigned long long*>(s1),
                              static_cast<unsigned long long*>(d1), (int)(bytes1 / 8), flag, seq);
}

// rhs[i*nrhs + col] = d_i * sgn * v_i   (d*b with b = -grad for the Newton system)
__global__ void k_scaled_col(const double* __restrict__ d, const double* __restrict__ v, double sgn, int n, int np,
                             int nrhs, int col, double* __restrict__ rhs) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < np) rhs[(size_t)i * nrhs + col] = (i < n) ? d[i] * (sgn * v[i]) : 0.0;
}
void launch_scaled_col(hipStream_t s, const double* d, const double* v, double sgn, int n, int np, int nrhs, int col,
                       double* rhs) {
  k_scaled_col<<<(np + 255) / 256, 256, 0, s>>>(d, v, sgn, n, np, nrhs, col, rhs);
}

// B = Aeq diag(d) (p x ld), and rhs[i][a] = B[a][i]   (KKTSystem.scala:238, :116-118)
__global__ void k_kkt_prep(const double* __restrict__ Aeq, int ld, int p, int n, int np, const double* __restrict__ d,
                           double* __restrict__ B, double* __restrict__ rhs, int nrhs) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= np) return;
  for (int a = 0; a < p; ++a) {
    const double b = (i < n) ? d[i] * Aeq[(size_t)a * ld + i] : 0.0;
    B[(size_t)a * ld + i] = b;
    rhs[(size_t)i * nrhs + a] = b;
  }
}
void launch_kkt_prep(hipStream_t s, const double* Aeq, int ld, int p, int n, int np, const double* d, double* B,
                     double* rhs, int nrhs) {
  k_kkt_prep<<<(np + 255) / 256, 256, 0, s>>>(Aeq, ld, p, n, np, d, B, rhs, nrhs);
}

// out = u + alpha*v elementwise with a strided source column: out_i = u_i + alpha * v[i*vs + vc]
__global__ void k_axpy_strided(const double* __restrict__ u, const double* __restrict__ v, int vs, int vc,
                               double alpha, int n, double* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (u ? u[i] : 0.0) + alpha * v[(size_t)i * vs + vc];
}
void launch_axpy_strided(hipStream_t s, const double* u, const double* v, int vs, int vc, double alpha, int n,
                         double* out) {
  k_axpy_strided<<<(n + 255) / 256, 256, 0, s>>>(u, v, vs, vc, alpha, n, out);
}

// out_i = d_i * v[i*vs + vc]
__global__ void k_scale_strided(const double* __restrict__ d, const double* __restrict__ v, int vs, int vc, int n,
                                double* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = d[i] * v[(size_t)i * vs + vc];
}
void launch_scale_strided(hipStream_t s, const double* d, const double* v, int vs, int vc, int n, double* out) {
  k_scale_strided<<<(n + 255) / 256, 256, 0, s>>>(d, v, vs, vc, n, out);
}

// H += Aeq' Aeq (KKT fallback K = H + A'A, KKTSystem.scala:57), full symmetric update, p small.
__global__ void k_add_ata(double* __restrict__ H, int ld, const double* __restrict__ Aeq, int p, int n) {
  const int i = blockIdx.y;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || j >= n) return;
  double s = 0.0;
  for (int a = 0; a < p; ++a) s += Aeq[(size_t)a * ld + i] * Aeq[(size_t)a * ld + j];
  H[(size_t)i * ld + j] += s;
}
void launch_add_ata(hipStream_t s, double* H, int ld, const double* Aeq, int p, int n) {
  dim3 grid((n + 255) / 256, n);
  k_add_ata<<<grid, 256, 0, s>>>(H, ld, Aeq, p, n);
}

// z = q - A' b  (KKTSystem.scala:58)
__global__ void k_q_minus_atb(const double* __restrict__ q, const double* __restrict__ Aeq, int ld, int p,
                              const double* __restrict__ b, int n, double* __restrict__ z) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double s = 0.0;
  for (int a = 0; a < p; ++a) s += Aeq[(size_t)a * ld + i] * b[a];
  z[i] = q[i] - s;
}
void launch_q_minus_atb(hipStream_t s, const double* q, const double* Aeq, int ld, int p, const double* b, int n,
                        double* z) {
  k_q_minus_atb<<<(n + 255) / 256, 256, 0, s>>>(q, Aeq, ld, p, b, n, z);
}

// y = B' w + u (n), B p x ld
__global__ void k_btw_plus(const double* __restrict__ B, int ld, int p, const double* __restrict__ w,
                           const double* __restrict__ u, int n, double* __restrict__ y) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double s = u ? u[i] : 0.0;
  for (int a = 0; a < p; ++a) s += B[(size_t)a * ld + i] * w[a];
  y[i] = s;
}
void launch_btw_plus(hipStream_t s, const double* B, int ld, int p, const double* w, const double* u, int n,
                     double* y) {
  k_btw_plus<<<(n + 255) / 256, 256, 0, s>>>(B, ld, p, w, u, n, y);
}

// ------------------------------------------------------------------------------------------------
// Sparse constraint rows (bounds x_j >= 0, phase-I rows (e_j, -1), box and difference rows): their Hessian
// terms  a_ip a_iq / d_i^2  (BarrierSolver.scala:314) are summed per lower entry (p, q) over the rows that
// touch it, in list order, one wave per entry, and added to H after the dense-row SYRK (both triangles).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_sparse_hess(const int* __restrict__ ptr, const int* __restrict__ pq,
                                                     const int* __restrict__ row, const double* __restrict__ coef,
                                                     const double* __restrict__ w, int T, double* __restrict__ H,
                                                     int ld) {
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (t >= T) return;
  const int e0 = ptr[t], e1 = ptr[t + 1];
  double s = 0.0;
  for (int e = e0 + lane; e < e1; e += 64) s += coef[e] * w[row[e]];
  s = wave_sum(s);
  if (lane == 0) {
    const int p = pq[2 * t], q = pq[2 * t + 1];
    H[(size_t)p * ld + q] += s;
    if (p != q) H[(size_t)q * ld + p] += s;
  }
}
void launch_sparse_hess(hipStream_t s, const int* ptr, const int* pq, const int* row, const double* coef,
                        const double* w, int T, double* H, int ld) {
  if (T > 0) k_sparse_hess<<<(T + 3) / 4, 256, 0, s>>>(ptr, pq, row, coef, w, T, H, ld);
}

// wd[i] = w[idx[i]] for the dense rows packed for the SYRK (0 on the padding rows)
__global__ void k_gather_w(const double* __restrict__ w, const int* __restrict__ idx, int nd, int ndp,
                           double* __restrict__ wd) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < ndp) wd[i] = (i < nd) ? w[idx[i]] : 0.0;
}
void launch_gather_w(hipStream_t s, const double* w, const int* idx, int nd, int ndp, double* wd) {
  k_gather_w<<<(ndp + 255) / 256, 256, 0, s>>>(w, idx, nd, ndp, wd);
}

}  // namespace cvxg
