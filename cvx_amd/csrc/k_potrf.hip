// k_potrf.hip — 64x64 diagonal-block Cholesky (dpotrf 'L' semantics, MatrixUtils.scala:452-461 via
// Breeze cholesky) with the block inverse and the fused forward substitution, built for a short
// per-column critical path on one CU.
//
// Structure: 8 panels of 8 columns.  4 waves; lane r of every wave holds row r of three bordered
// systems for the columns of the wave's two panels {w, 7-w} (balanced early/late work):
//   a[] : row r of the block A_kk           -> L_kk
//   e[] : row r of the identity border      -> (L_kk^-1)^T   (Linv for the panel TRSM / back solve)
//   u[] : rhs vector r (lanes < nrhs)        -> w = L_kk^-1 b (forward substitution fused in)
// Panel p (owner wave o(p)): the owner publishes the raw 8x8 diagonal block, every owner lane factors it
// redundantly in registers (rsqrt + Newton, no divisions) and forward-substitutes its own row -> L / W
// panel values into LDS; ONE workgroup barrier; every wave then applies the rank-8 update to its owned
// later columns.  The owner of panel p+1 starts its panel right after its own update: the other waves'
// updates of panel p overlap it (intra-block lookahead).
#include <math.h>

#include "kernels.hpp"

namespace cvxg {

constexpr int PW = 8;            // panel width
constexpr int NPAN = NB / PW;    // 8 panels

__device__ __forceinline__ double rsqrt_nr(double p) {
  double y = __builtin_amdgcn_rsq(p);
  const double h = 0.5 * p;
  y = y * (1.5 - h * y * y);
  y = y * (1.5 - h * y * y);
  return y;
}

__device__ __forceinline__ int owner_of(int p) { return p < 4 ? p : 7 - p; }

__global__ __launch_bounds__(256) void k_potrf_blocked(double* __restrict__ L, int ld, int k, double* __restrict__ rhs,
                                                       int nrhs, double* __restrict__ Linv, DevCtrl* ctrl) {
  if (ctrl->chol_info != 0) return;
  __shared__ __attribute__((aligned(16))) double Lp[NPAN][NB][PW];    // final L, by panel
  __shared__ __attribute__((aligned(16))) double Ep[NPAN][NB][PW];    // final W = (L^-1)^T rows, by panel
  __shared__ __attribute__((aligned(16))) double Wp[NPAN][MAX_RHS][PW];
  __shared__ __attribute__((aligned(16))) double draw[PW][PW];
  __shared__ int fail;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int base = k * NB;
  const int q0 = w, q1 = 7 - w;  // owned panels
  double a[2][PW], e[2][PW], u[2][PW];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int q = s ? q1 : q0;
    const double* src = L + (size_t)(base + lane) * ld + base + PW * q;
    typedef double v2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int j = 0; j < PW; j += 2) {
      const v2 t = *reinterpret_cast<const v2*>(src + j);
      a[s][j] = (PW * q + j <= lane) ? t[0] : 0.0;
      a[s][j + 1] = (PW * q + j + 1 <= lane) ? t[1] : 0.0;
    }
#pragma unroll
    for (int j = 0; j < PW; ++j) {
      e[s][j] = (PW * q + j == lane) ? 1.0 : 0.0;
      u[s][j] = (lane < nrhs) ? rhs[(size_t)(base + PW * q + j) * nrhs + lane] : 0.0;
    }
  }
  if (tid == 0) fail = 0;
  double mind = __builtin_inf();
  __syncthreads();

#pragma unroll
  for (int p = 0; p < NPAN; ++p) {
    const int o = owner_of(p);
    const int so = p < 4 ? 0 : 1;  // owner's slot for panel p (static)
    // ---- phase A: owner wave factors the panel ---------------------------------------------------
    if (w == o) {
      if (lane >= PW * p && lane < PW * p + PW) {
#pragma unroll
        for (int j = 0; j < PW; ++j) draw[lane - PW * p][j] = a[so][j];
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      double Lb[PW][PW], rl[PW];
      bool bad = false;
#pragma unroll
      for (int j = 0; j < PW; ++j) {
        double dj = draw[j][j];
#pragma unroll
        for (int i = 0; i < j; ++i) dj = fma(-Lb[j][i], Lb[j][i], dj);
        bad = bad || !(dj > 0.0);
        rl[j] = rsqrt_nr(dj);
        Lb[j][j] = dj * rl[j];
        mind = fmin(mind, Lb[j][j]);
#pragma unroll
        for (int r = j + 1; r < PW; ++r) {
          double t = draw[r][j];
#pragma unroll
          for (int i = 0; i < j; ++i) t = fma(-Lb[r][i], Lb[j][i], t);
          Lb[r][j] = t * rl[j];
        }
      }
      // forward substitution of the owned rows: x = v[panel] L_bb^-T   (rows r < 8p are zero/upper)
      double xa[PW], xe[PW], xu[PW];
#pragma unroll
      for (int j = 0; j < PW; ++j) {
        double ta = a[so][j], te = e[so][j], tu = u[so][j];
#pragma unroll
        for (int i = 0; i < j; ++i) {
          ta = fma(-xa[i], Lb[j][i], ta);
          te = fma(-xe[i], Lb[j][i], te);
          tu = fma(-xu[i], Lb[j][i], tu);
        }
        xa[j] = ta * rl[j];
        xe[j] = te * rl[j];
        xu[j] = tu * rl[j];
      }
#pragma unroll
      for (int j = 0; j < PW; ++j) {
        const double va = (PW * p + j <= lane) ? xa[j] : 0.0;  // L is lower: zero above the diagonal
        a[so][j] = va;
        e[so][j] = xe[j];
        u[so][j] = xu[j];
        Lp[p][lane][j] = va;
        Ep[p][lane][j] = xe[j];
        if (lane < nrhs) Wp[p][lane][j] = xu[j];
      }
      if (bad && lane == 0) {
        fail = 1;
        atomicCAS(&ctrl->chol_info, 0, base + PW * p + 1);
      }
    }
    __syncthreads();
    if (fail) return;  // uniform: every wave reads the same flag after the barrier
    // ---- phase B: every wave applies panel p to its owned later columns --------------------------
    double xr[PW], er[PW], ur[PW];
#pragma unroll
    for (int j = 0; j < PW; ++j) {
      xr[j] = Lp[p][lane][j];
      er[j] = Ep[p][lane][j];
      ur[j] = (lane < nrhs) ? Wp[p][lane][j] : 0.0;
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int q = s ? q1 : q0;
      if (q > p) {
#pragma unroll
        for (int jj = 0; jj < PW; ++jj) {
          const int c = PW * q + jj;
          double sa = 0.0, se = 0.0, su = 0.0;
#pragma unroll
          for (int j = 0; j < PW; ++j) {
            const double lc = Lp[p][c][j];  // broadcast
            sa = fma(xr[j], lc, sa);
            se = fma(er[j], lc, se);
            su = fma(ur[j], lc, su);
          }
          a[s][jj] -= sa;
          e[s][jj] -= se;
          u[s][jj] -= su;
        }
      }
    }
  }
  __syncthreads();
  // ---- outputs: L block (lower), Linv[j][r] = W[r][j], w -------------------------------------------
  for (int t = tid; t < NB * NB; t += 256) {
    const int r = t / NB, c = t % NB;
    if (c <= r) L[(size_t)(base + r) * ld + base + c] = Lp[c / PW][r][c % PW];
    Linv[(size_t)k * NB * NB + t] = Ep[r / PW][c][r % PW];  // Linv[r][c] = W[c][r]
  }
  for (int t = tid; t < nrhs * NB; t += 256) {
    const int rho = t / NB, c = t % NB;
    rhs[(size_t)(base + c) * nrhs + rho] = Wp[c / PW][rho][c % PW];
  }
  if (lane == 0) atomic_min_pos(&ctrl->min_diag, mind);
}

void launch_potrf_diag(hipStream_t s, double* L, int ld, int k, double* rhs, int nrhs, double* Linv, DevCtrl* ctrl) {
  k_potrf_blocked<<<1, 256, 0, s>>>(L, ld, k, rhs, nrhs, Linv, ctrl);
}

}  // namespace cvxg
