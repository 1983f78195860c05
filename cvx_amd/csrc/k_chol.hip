// k_chol.hip — blocked right-looking Cholesky (row-major lower L, NB = 64) with the forward
// substitution fused in, and the backward-substitution steps.
//
// Reference: MatrixUtils.regularizedCholesky -> Breeze cholesky -> LAPACK dpotrf('L')
// (MatrixUtils.scala:452-461), then forwardSolve(L, d*b) / backSolve(L', w) (MatrixUtils.scala:383-430,
// 491-493).  The right-hand sides and the 64 unit vectors ride along as extra rows of each diagonal-block
// elimination (bordered form): the same sweep that produces L_kk yields w_k = L_kk^-1 b_k and
// L_kk^-1, so the panel TRSM and the backward substitution are products with L_kk^-1 instead of
// sequential substitutions.
#include <math.h>

#include "kernels.hpp"

namespace cvxg {

typedef double vd2c __attribute__((ext_vector_type(2)));
constexpr int TRSM_THREADS = 64;  // 16 rows per workgroup: the panel spreads over ~4x more CUs

// 1/sqrt(p) to full FP64 accuracy: hardware estimate + two Newton steps (no long div/sqrt sequences on
// the per-column critical path).
__device__ __forceinline__ double rsqrt_fp64(double p) {
  double y = __builtin_amdgcn_rsq(p);
  const double h = 0.5 * p;
  y = y * (1.5 - h * y * y);
  y = y * (1.5 - h * y * y);
  return y;
}

// ------------------------------------------------------------------------------------------------
// Diagonal block factorisation, row-owned: 3 waves run the same sweep, lane r of wave w owns ONE row of
// a 64-wide bordered system in 64 registers:
//   wave 0: row r of the block A_kk (lower part),
//   wave 1: row r of the identity border  -> row r of (L_kk^-1)^T,
//   wave 2: rhs column r (lanes < nrhs)    -> w = L_kk^-1 b (fused forward substitution).
// Step j (unrolled, static register index): wave 0 publishes column j to LDS, one barrier, then every
// row applies  v_c -= (v_j / l_jj) (a_cj / l_jj)  for c > j and finalises v_j /= l_jj.  One barrier per
// column, no divisions (rsqrt + Newton), outputs staged through LDS and written once, coalesced.
// Non-positive / NaN pivot -> ctrl->chol_info = global index + 1 (dpotrf info > 0).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(192) void k_potrf_diag(double* __restrict__ L, int ld, int k, double* __restrict__ rhs,
                                                    int nrhs, double* __restrict__ Linv, DevCtrl* ctrl) {
  if (ctrl->chol_info != 0) return;
  __shared__ __attribute__((aligned(16))) double col[NB];
  __shared__ double stage[NB][NB + 1];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int base = k * NB;
  double v[NB];
  if (wid == 0) {
    const double* src = L + (size_t)(base + lane) * ld + base;
#pragma unroll
    for (int c = 0; c < NB; c += 2) {
      const vd2c t = *reinterpret_cast<const vd2c*>(src + c);
      v[c] = (c <= lane) ? t[0] : 0.0;
      v[c + 1] = (c + 1 <= lane) ? t[1] : 0.0;
    }
  } else if (wid == 1) {
#pragma unroll
    for (int c = 0; c < NB; ++c) v[c] = (c == lane) ? 1.0 : 0.0;
  } else {
    const int rr = lane < nrhs ? lane : 0;
#pragma unroll
    for (int c = 0; c < NB; ++c) v[c] = rhs[(size_t)(base + c) * nrhs + rr];
  }
  double mind = __builtin_inf();
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    if (wid == 0) col[lane] = v[j];  // a_rj (unscaled) of every row
    __syncthreads();
    const double piv = col[j];
    if (!(piv > 0.0)) {  // uniform across the block
      if (tid == 0) atomicCAS(&ctrl->chol_info, 0, base + j + 1);
      return;
    }
    const double rl = rsqrt_fp64(piv);
    mind = fmin(mind, piv * rl);
    const double lr = v[j] * rl;  // final entry of column j (L_rj, W_rj or w_j)
    const double lrr = lr * rl;
    v[j] = lr;
#pragma unroll
    for (int c = j + 1; c < NB; c += 2) {
      if (c + 1 < NB) {
        const vd2c cc = *reinterpret_cast<const vd2c*>(&col[c]);  // broadcast read
        v[c] = fma(-lrr, cc[0], v[c]);
        v[c + 1] = fma(-lrr, cc[1], v[c + 1]);
      } else {
        v[c] = fma(-lrr, col[c], v[c]);
      }
    }
    __syncthreads();  // col is rewritten by the next step
  }
  // stage rows through LDS, write coalesced
  if (wid == 0) {
#pragma unroll
    for (int c = 0; c < NB; ++c) stage[lane][c] = v[c];
  }
  __syncthreads();
  for (int t = tid; t < NB * NB; t += 192) {
    const int r = t / NB, c = t % NB;
    if (c <= r) L[(size_t)(base + r) * ld + base + c] = stage[r][c];
  }
  __syncthreads();
  if (wid == 1) {  // lane r holds row r of W = (L^-1)^T, i.e. Linv[j][r] = v[j]
#pragma unroll
    for (int j = 0; j < NB; ++j) Linv[(size_t)k * NB * NB + j * NB + lane] = v[j];
  } else if (wid == 2 && lane < nrhs) {
#pragma unroll
    for (int c = 0; c < NB; ++c) rhs[(size_t)(base + c) * nrhs + lane] = v[c];
  }
  if (tid == 0) atomic_min_pos(&ctrl->min_diag, mind);
}

void launch_potrf_diag_rowowned(hipStream_t s, double* L, int ld, int k, double* rhs, int nrhs, double* Linv,
                                DevCtrl* ctrl) {
  k_potrf_diag<<<1, 192, 0, s>>>(L, ld, k, rhs, nrhs, Linv, ctrl);
}

// ------------------------------------------------------------------------------------------------
// Panel TRSM as a product with L_kk^-1:  L[i, kb] = A[i, kb] L_kk^-T, i.e. x_c = sum_{j<=c} a_j Linv[c][j].
// Four threads per row (each owns the outputs c = q + 4u), the row in registers, Linv broadcast from
// LDS.  Fused forward substitution: rhs[i] -= L[i, kb] . w_kb (shuffle-reduced over the 4 threads).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(TRSM_THREADS) void k_trsm_panel(double* __restrict__ L, int ld, int np, int k,
                                                    double* __restrict__ rhs, int nrhs,
                                                    const double* __restrict__ Linv, const DevCtrl* ctrl) {
  if (ctrl->chol_info != 0) return;
  __shared__ double li[NB][NB + 1];
  __shared__ double wk[MAX_RHS][NB];
  const int base = k * NB;
  const double* lsrc = Linv + (size_t)k * NB * NB;
  for (int t = threadIdx.x; t < NB * NB; t += TRSM_THREADS) li[t / NB][t % NB] = lsrc[t];
  for (int t = threadIdx.x; t < nrhs * NB; t += TRSM_THREADS) wk[t / NB][t % NB] = rhs[(size_t)(base + t % NB) * nrhs + t / NB];
  __syncthreads();
  const int q = threadIdx.x & 3;
  const int i = base + NB + blockIdx.x * (TRSM_THREADS / 4) + (threadIdx.x >> 2);
  const bool valid = i < np;
  const int ir = valid ? i : np - 1;
  double a[NB];
  double* row = L + (size_t)ir * ld + base;
#pragma unroll
  for (int c = 0; c < NB; c += 2) {
    const vd2c v = *reinterpret_cast<const vd2c*>(row + c);
    a[c] = v[0];
    a[c + 1] = v[1];
  }
  double x[NB / 4];
#pragma unroll
  for (int u = 0; u < NB / 4; ++u) {
    const int c = q + 4 * u;
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int j = 0; j < NB; j += 2) {  // Linv[c][j] = 0 for j > c
      s0 = fma(a[j], li[c][j], s0);
      s1 = fma(a[j + 1], li[c][j + 1], s1);
    }
    x[u] = s0 + s1;
  }
  if (valid) {
#pragma unroll
    for (int u = 0; u < NB / 4; ++u) row[q + 4 * u] = x[u];
  }
  for (int rho = 0; rho < nrhs; ++rho) {
    double s = 0.0;
#pragma unroll
    for (int u = 0; u < NB / 4; ++u) s = fma(x[u], wk[rho][q + 4 * u], s);
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    if (valid && q == 0) rhs[(size_t)i * nrhs + rho] -= s;
  }
}

void launch_trsm_panel(hipStream_t s, double* L, int ld, int np, int k, double* rhs, int nrhs, const double* Linv,
                       const DevCtrl* ctrl) {
  const int rows = np - (k + 1) * NB;
  if (rows <= 0) return;
  k_trsm_panel<<<(rows + TRSM_THREADS / 4 - 1) / (TRSM_THREADS / 4), TRSM_THREADS, 0, s>>>(L, ld, np, k, rhs, nrhs, Linv, ctrl);
}

// ------------------------------------------------------------------------------------------------
// Backward substitution L' u = w, block step k (k = nblk-1 .. 0):
//   u_k = Linv_kk' v_k  (every workgroup, redundantly),  workgroup b < k: v_b -= L[kb, bb]' u_k.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_bwd_step(const double* __restrict__ L, int ld,
                                                  const double* __restrict__ Linv, int k, double* __restrict__ rhs,
                                                  double* __restrict__ out, int nrhs, const DevCtrl* ctrl) {
  if (ctrl->chol_info != 0) return;
  __shared__ double v[MAX_RHS][NB];
  __shared__ double u[MAX_RHS][NB];
  __shared__ double part[4][MAX_RHS][NB];
  const int base = k * NB;
  const int g = threadIdx.x >> 6, c = threadIdx.x & 63;
  for (int t = threadIdx.x; t < nrhs * NB; t += 256) v[t / NB][t % NB] = rhs[(size_t)(base + t % NB) * nrhs + t / NB];
  __syncthreads();
  const double* li = Linv + (size_t)k * NB * NB;
  for (int rho = 0; rho < nrhs; ++rho) {
    double s = 0.0;
    for (int r = g * 16; r < g * 16 + 16; ++r) s = fma(li[r * NB + c], v[rho][r], s);
    part[g][rho][c] = s;
  }
  __syncthreads();
  if (g == 0) {
    for (int rho = 0; rho < nrhs; ++rho) {
      const double s = ((part[0][rho][c] + part[1][rho][c]) + part[2][rho][c]) + part[3][rho][c];
      u[rho][c] = s;
      if (blockIdx.x == 0) out[(size_t)(base + c) * nrhs + rho] = s;
    }
  }
  __syncthreads();
  if (k == 0) return;
  const int b = blockIdx.x;  // < k
  const double* tile = L + (size_t)base * ld + b * NB;  // rows kb, cols bb
  for (int rho = 0; rho < nrhs; ++rho) {
    double s = 0.0;
    for (int r = g * 16; r < g * 16 + 16; ++r) s = fma(tile[(size_t)r * ld + c], u[rho][r], s);
    part[g][rho][c] = s;
  }
  __syncthreads();
  if (g == 0) {
    for (int rho = 0; rho < nrhs; ++rho) {
      const double s = ((part[0][rho][c] + part[1][rho][c]) + part[2][rho][c]) + part[3][rho][c];
      rhs[(size_t)(b * NB + c) * nrhs + rho] -= s;
    }
  }
}

void launch_bwd_step(hipStream_t s, const double* L, int ld, const double* Linv, int k, double* rhs, double* out,
                     int nrhs, const DevCtrl* ctrl) {
  k_bwd_step<<<k > 0 ? k : 1, 256, 0, s>>>(L, ld, Linv, k, rhs, out, nrhs, ctrl);
}

// ------------------------------------------------------------------------------------------------
// The whole backward substitution L' u = w in ONE launch (MatrixUtils.scala:419-430 backSolve, blocked):
// workgroup g owns block b = nblk-1-g and accumulates  s_b = sum_{i>b} L_ib' u_i  as the u_i are published
// (flag[i] == gen; L_ib is prefetched into registers before the wait), then  u_b = Linv_bb' (w_b - s_b)  and
// publishes u_b.  Workgroups only wait on lower blockIdx (dispatched earlier), so the launch is deadlock-free
// at any residency.  Thread (c, g) keeps the partial sums of column c over rows 16g..16g+15 of every tile;
// the four row groups are added once, in a fixed order.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_bwd_dataflow(const double* __restrict__ L, int ld,
                                                      const double* __restrict__ Linv, const double* __restrict__ rhs,
                                                      double* __restrict__ out, int nrhs, int nblk, int* flags, int gen,
                                                      const DevCtrl* ctrl) {
  if (ctrl->chol_info != 0) return;
  __shared__ double u[MAX_RHS][NB];
  __shared__ double part[4][MAX_RHS][NB];
  __shared__ int s_ok;
  const int b = nblk - 1 - (int)blockIdx.x;
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
    if (threadIdx.x == 0) {
      unsigned spins = 0;
      while (__hip_atomic_load(flags + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != gen && ++spins < (1u << 24))
        __builtin_amdgcn_s_sleep(1);
      s_ok = spins < (1u << 24);
    }
    __syncthreads();
    if (!s_ok) return;  // bounded wait: never hang the GPU on a scheduling bug
    for (int t = threadIdx.x; t < nrhs * NB; t += 256)
      u[t / NB][t % NB] = __hip_atomic_load(out + (size_t)(i * NB + t % NB) * nrhs + t / NB, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
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
      __hip_atomic_store(out + (size_t)(b * NB + c) * nrhs + rho, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();  // every storing wave (wave 0) has drained
  if (threadIdx.x == 0) __hip_atomic_store(flags + b, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

void launch_bwd_dataflow(hipStream_t s, const double* L, int ld, const double* Linv, const double* rhs, double* out,
                         int nrhs, int nblk, int* flags, int gen, const DevCtrl* ctrl) {
  k_bwd_dataflow<<<nblk, 256, 0, s>>>(L, ld, Linv, rhs, out, nrhs, nblk, flags, gen, ctrl);
}

}  // namespace cvxg
