// k_quad.hip — QuadraticConstraint rows r + a'x + x'P x / 2 <= ub (QuadraticConstraint.scala:8-40) in the
// barrier path.  The P_k are stacked row-major as one (q np) x np matrix, so P_k x for every k is ONE rowdot
// launch.  With G_k = a_k + P_k x the barrier terms are (BarrierSolver.scala:291-315):
//   value     g_k = (r + a.x) + x.(P_k x)/2
//   gradient  sum_k G_k / d_k        (the a_k / d_k part comes from the shared column reduction)
//   Hessian   sum_k G_k G_k' / d_k^2 (the SYRK, with G_k written into the packed dense rows)  +  sum_k P_k / d_k
// and along a step s: g_k(x + t s) = g_k + t (G_k.s) + t^2 (s'P_k s)/2.
#include "kernels.hpp"

namespace cvxg {

// extra[row_k] = x.(P_k x) / 2   (one wave per constraint)
__global__ __launch_bounds__(256) void k_quad_xpx(const double* __restrict__ qPx, const double* __restrict__ x,
                                                  const int* __restrict__ qrows, int nq, int np,
                                                  double* __restrict__ extra) {
  const int k = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (k >= nq) return;
  double s = 0.0;
  for (int j = lane; j < np; j += 64) s = fma(x[j], qPx[(size_t)k * np + j], s);
  s = wave_sum(s);
  if (lane == 0) extra[qrows[k]] = s / 2;
}
void launch_quad_xpx(hipStream_t s, const double* qPx, const double* x, const int* qrows, int nq, int np,
                     double* extra) {
  k_quad_xpx<<<(nq + 3) / 4, 256, 0, s>>>(qPx, x, qrows, nq, np, extra);
}

// y[j] += sum_k (P_k x)_j / d_k, k ascending
__global__ void k_quad_grad(const double* __restrict__ qPx, const double* __restrict__ invd,
                            const int* __restrict__ qrows, int nq, int np, double* __restrict__ y) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= np) return;
  double s = 0.0;
  for (int k = 0; k < nq; ++k) s += qPx[(size_t)k * np + j] * invd[qrows[k]];
  y[j] += s;
}
void launch_quad_grad(hipStream_t s, const double* qPx, const double* invd, const int* qrows, int nq, int np,
                      double* y) {
  k_quad_grad<<<(np + 255) / 256, 256, 0, s>>>(qPx, invd, qrows, nq, np, y);
}

// As[slot_k] = a_k + P_k x: the gradient row G_k of the SYRK (QuadraticConstraint.gradientAt)
__global__ void k_quad_rows(const double* __restrict__ A, const double* __restrict__ qPx,
                            const int* __restrict__ qrows, const int* __restrict__ qslot, int nq, int np,
                            double* __restrict__ As) {
  const int k = blockIdx.y, j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= np) return;
  As[(size_t)qslot[k] * np + j] = A[(size_t)qrows[k] * np + j] + qPx[(size_t)k * np + j];
}
void launch_quad_rows(hipStream_t s, const double* A, const double* qPx, const int* qrows, const int* qslot, int nq,
                      int np, double* As) {
  k_quad_rows<<<dim3((np + 255) / 256, nq), 256, 0, s>>>(A, qPx, qrows, qslot, nq, np, As);
}

// H += sum_k P_k / d_k on the lower triangle, mirrored (H stays exactly symmetric)
__global__ void k_quad_hess(const double* __restrict__ Pq, const double* __restrict__ invd,
                            const int* __restrict__ qrows, int nq, int np, double* __restrict__ H) {
  const int i = blockIdx.y, j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j > i) return;
  double v = 0.0;
  for (int k = 0; k < nq; ++k) v += Pq[((size_t)k * np + i) * np + j] * invd[qrows[k]];
  H[(size_t)i * np + j] += v;
  if (i != j) H[(size_t)j * np + i] += v;
}
void launch_quad_hess(hipStream_t s, const double* Pq, const double* invd, const int* qrows, int nq, int np,
                      double* H) {
  k_quad_hess<<<dim3((np + 255) / 256, np), 256, 0, s>>>(Pq, invd, qrows, nq, np, H);
}

// Along the step s: e[row_k] += (P_k x).s (so e = G.s) and f[row_k] = s.(P_k s); one wave per constraint
__global__ __launch_bounds__(256) void k_quad_ls(const double* __restrict__ qPx, const double* __restrict__ qPs,
                                                 const double* __restrict__ sdir, const int* __restrict__ qrows,
                                                 int nq, int np, double* __restrict__ e, double* __restrict__ f) {
  const int k = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (k >= nq) return;
  double a = 0.0, b = 0.0;
  for (int j = lane; j < np; j += 64) {
    a = fma(qPx[(size_t)k * np + j], sdir[j], a);
    b = fma(sdir[j], qPs[(size_t)k * np + j], b);
  }
  a = wave_sum(a);
  b = wave_sum(b);
  if (lane == 0) {
    e[qrows[k]] += a;
    f[qrows[k]] = b;
  }
}
void launch_quad_ls(hipStream_t s, const double* qPx, const double* qPs, const double* sdir, const int* qrows, int nq,
                    int np, double* e, double* f) {
  k_quad_ls<<<(nq + 3) / 4, 256, 0, s>>>(qPx, qPs, sdir, qrows, nq, np, e, f);
}

// Error scales of the certified line search for QuadraticConstraint rows (k_ls_trials): out[row_k] (+)= scale *
// |v|.M_k for the stacked |P_k| products M (|P_k||x| or |P_k||s|), one wave per constraint.
__global__ __launch_bounds__(256) void k_quad_absdot(const double* __restrict__ M, const double* __restrict__ v,
                                                     const int* __restrict__ qrows, int nq, int np, double scale,
                                                     int accumulate, double* __restrict__ out) {
  const int k = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (k >= nq) return;
  double s = 0.0;
  for (int j = lane; j < np; j += 64) s = fma(fabs(v[j]), M[(size_t)k * np + j], s);
  s = wave_sum(s) * scale;
  if (lane == 0) out[qrows[k]] = accumulate ? out[qrows[k]] + s : s;
}
void launch_quad_absdot(hipStream_t s, const double* M, const double* v, const int* qrows, int nq, int np, double scale,
                        int accumulate, double* out) {
  k_quad_absdot<<<(nq + 3) / 4, 256, 0, s>>>(M, v, qrows, nq, np, scale, accumulate, out);
}

}  // namespace cvxg
