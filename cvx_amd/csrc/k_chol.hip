// k_chol.hip — the backward substitution L' u = w of the Cholesky solve (MatrixUtils.scala:410-430 backSolve,
// blocked): one persistent launch over the 64 x 64 blocks of L, using the diagonal-block inverses L_kk^-1 that the
// factorization (k_dataflow.hip) stores, so every block step is a product instead of a sequential substitution.
#include <math.h>

#include "kernels.hpp"

namespace cvxg {
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
