// Microbenchmark of the 16 x 16 elimination sweep (one wave) of the 64 x 64 diagonal-block Cholesky:
//   v0  lanes 0-15 D rows, lanes 16-31 identity-border rows, column broadcasts by v_readlane (potrf64w.hpp)
//   v3  as v0, the column broadcasts through LDS (one store + broadcast loads per column)
//   v2  as v0, two columns per step (one dependency bubble per pair; the second column updated uniformly)
//   v1  lanes 0-15 hold a D row and its border row in two register sets, column broadcasts by DPP row_newbcast
//       (64-bit v_mov_b64_dpp, folded into the FMAs where the compiler can), the pivot chain in VGPRs
// Checks both against a host Cholesky (L and L^-T) and reports cycles per sweep (s_memtime, 100 sweeps).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off microbench/sweep.hip -o microbench/sweep
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "../cvx_amd/csrc/potrf64.hpp"
using namespace cvxg;

template <int C>
__device__ __forceinline__ double bcast(double v) {
  return __builtin_amdgcn_update_dpp(0.0, v, 0x150 + C, 0xf, 0xf, false);  // row_newbcast:C
}

// ---- v1: DPP sweep ------------------------------------------------------------------------------------------
// step J: a[c] -= (a[J]/p_J) D_cJ, b[c] -= (b[J]/p_J) D_cJ for c > J (D_cJ = lane c's a[J], broadcast in the row);
// then the next pivot p_J+1 = lane J+1's a[J+1] (broadcast), and column J scaled by p_J^-1/2.
template <int J>
__device__ __forceinline__ void sweep_step(double (&a)[16], double (&b)[16], double& piv, double& rinv, double& pmin,
                                           int& firstbad) {
  if constexpr (J < 16) {
    if (!(piv > 0.0) && firstbad < 0) firstbad = J;
    pmin = fmin(pmin, piv);
    const double sj = rsqrt_nr(piv);
    const double nta = -(a[J] * rinv), ntb = -(b[J] * rinv);
    if constexpr (J + 1 < 16) {
      const double l1 = bcast<J + 1>(a[J]);
      a[J + 1] = fma(nta, l1, a[J + 1]);
      b[J + 1] = fma(ntb, l1, b[J + 1]);
      piv = bcast<J + 1>(a[J + 1]);
      rinv = rcp_nr(piv);
    }
    [&]<int... Cs>(std::integer_sequence<int, Cs...>) {
      (([&] {
         constexpr int C = J + 2 + Cs;
         const double l = bcast<C>(a[J]);
         a[C] = fma(nta, l, a[C]);
         b[C] = fma(ntb, l, b[C]);
       }()),
       ...);
    }(std::make_integer_sequence<int, (J + 2 < 16 ? 14 - J : 0)>{});
    a[J] *= sj;
    b[J] *= sj;
    sweep_step<J + 1>(a, b, piv, rinv, pmin, firstbad);
  }
}

__global__ __launch_bounds__(64) void k_sweep(const double* __restrict__ D, double* __restrict__ out, int variant,
                                              int reps, unsigned long long* cyc) {
  __shared__ double colbuf[2][16];  // v3: the finished column, broadcast through LDS
  const int lane = threadIdx.x, r = lane & 15;
  unsigned long long t0 = 0, t1 = 0;
  double a[16], b[16];
  for (int rep = 0; rep <= reps; ++rep) {
    if (rep == 1) t0 = __builtin_amdgcn_s_memtime();
    if (variant == 0) {
#pragma unroll
      for (int c = 0; c < 16; ++c)
        a[c] = (lane < 16) ? (c <= r ? D[r * 16 + c] : 0.0) : ((lane < 32 && c == r) ? 1.0 : 0.0);
      int firstbad = -1;
      double piv = readlane_d(a[0], 0);
      double rinv = rcp_nr(piv);
      double pmin = piv;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        double lc[16];
#pragma unroll
        for (int c = j + 1; c < 16; ++c) lc[c] = readlane_d(a[j], c);
        if (!(piv > 0.0) && firstbad < 0) firstbad = j;
        pmin = fmin(pmin, piv);
        const double rj = rinv;
        const double sj = rsqrt_nr(piv);
        if (j + 1 < 16) {
          const double dn = readlane_d(a[j + 1], j + 1);
          piv = fma(-(lc[j + 1] * rj), lc[j + 1], dn);
          rinv = rcp_nr(piv);
        }
        const double t = a[j] * rj;
#pragma unroll
        for (int c = j + 1; c < 16; ++c) a[c] = fma(-t, lc[c], a[c]);
        a[j] *= sj;
      }
      if (firstbad >= 0) a[0] = __builtin_nan("");
      a[1] += 0.0 * pmin;
#pragma unroll
      for (int c = 0; c < 16; ++c) b[c] = a[c];
    } else if (variant == 3) {
      // column broadcasts through LDS: lanes 0-15 store column j after its last update, every lane reads the
      // entries it needs back as uniform-address (broadcast) LDS loads -- one store + one read round trip per
      // column instead of 2 (15 - j) v_readlane
#pragma unroll
      for (int c = 0; c < 16; ++c)
        a[c] = (lane < 16) ? (c <= r ? D[r * 16 + c] : 0.0) : ((lane < 32 && c == r) ? 1.0 : 0.0);
      int firstbad = -1;
      double pmin = 1e300;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        double* cb = colbuf[j & 1];
        if (lane < 16) cb[lane] = a[j];  // column j (rows >= j are final; rows < j unused)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        double lc[16];
#pragma unroll
        for (int c = j; c < 16; ++c) lc[c] = cb[c];
        const double piv = lc[j];
        if (!(piv > 0.0) && firstbad < 0) firstbad = j;
        pmin = fmin(pmin, piv);
        const double rj = rcp_nr(piv);
        const double t = a[j] * rj;
#pragma unroll
        for (int c = j + 1; c < 16; ++c) a[c] = fma(-t, lc[c], a[c]);
        a[j] *= rsqrt_nr(piv);
      }
      if (firstbad >= 0) a[0] = __builtin_nan("");
      a[1] += 0.0 * pmin;
#pragma unroll
      for (int c = 0; c < 16; ++c) b[c] = a[c];
    } else if (variant == 2) {
      // two columns per step: both columns' broadcasts issued together behind one dependency bubble; the second
      // column's values get the first column's update uniformly (mc' = mc - lc * f), each row then applies the
      // rank-2 update
#pragma unroll
      for (int c = 0; c < 16; ++c)
        a[c] = (lane < 16) ? (c <= r ? D[r * 16 + c] : 0.0) : ((lane < 32 && c == r) ? 1.0 : 0.0);
      int firstbad = -1;
      double piv = readlane_d(a[0], 0);
      double rinv = rcp_nr(piv);
      double pmin = piv;
#pragma unroll
      for (int j = 0; j < 16; j += 2) {
        double lc[16], mc[16];
#pragma unroll
        for (int c = j + 1; c < 16; ++c) lc[c] = readlane_d(a[j], c);
#pragma unroll
        for (int c = j + 1; c < 16; ++c) mc[c] = readlane_d(a[j + 1], c);  // mc[j+1]: the diagonal D_j+1,j+1
        if (!(piv > 0.0) && firstbad < 0) firstbad = j;
        pmin = fmin(pmin, piv);
        const double f = lc[j + 1] * rinv;
        const double piv1 = fma(-lc[j + 1], f, mc[j + 1]);
        const double rinv1 = rcp_nr(piv1);
#pragma unroll
        for (int c = j + 2; c < 16; ++c) mc[c] = fma(-lc[c], f, mc[c]);
        double pivn = 1.0;
        if (j + 2 < 16) {  // next pair's pivot, uniformly: D_j+2,j+2 - lc^2 / p_j - mc'^2 / p_j+1
          const double dn = readlane_d(a[j + 2], j + 2);
          pivn = fma(-(mc[j + 2] * rinv1), mc[j + 2], fma(-(lc[j + 2] * rinv), lc[j + 2], dn));
        }
        if (!(piv1 > 0.0) && firstbad < 0) firstbad = j + 1;
        pmin = fmin(pmin, piv1);
        const double t1 = a[j] * rinv;
        a[j + 1] = fma(-t1, lc[j + 1], a[j + 1]);
        const double t2 = a[j + 1] * rinv1;
#pragma unroll
        for (int c = j + 2; c < 16; ++c) a[c] = fma(-t2, mc[c], fma(-t1, lc[c], a[c]));
        a[j] *= rsqrt_nr(piv);
        a[j + 1] *= rsqrt_nr(piv1);
        piv = pivn;
        rinv = rcp_nr(pivn);
      }
      if (firstbad >= 0) a[0] = __builtin_nan("");
      a[1] += 0.0 * pmin;
#pragma unroll
      for (int c = 0; c < 16; ++c) b[c] = a[c];
    } else {
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        a[c] = c <= r ? D[r * 16 + c] : 0.0;
        b[c] = (c == r) ? 1.0 : 0.0;
      }
      int firstbad = -1;
      double piv = bcast<0>(a[0]);
      double rinv = rcp_nr(piv);
      double pmin = piv;
      sweep_step<0>(a, b, piv, rinv, pmin, firstbad);
      if (firstbad >= 0) a[0] = __builtin_nan("");
      a[1] += 0.0 * pmin;
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (variant != 1) {  // v0 / v2: lanes 0-15 L rows, 16-31 L^-T rows
    if (lane < 32)
      for (int c = 0; c < 16; ++c) out[(lane < 16 ? 0 : 256) + r * 16 + c] = (lane >= 16 || c <= r) ? a[c] : 0.0;
  } else {
    if (lane < 16)
      for (int c = 0; c < 16; ++c) {
        out[r * 16 + c] = c <= r ? a[c] : 0.0;
        out[256 + r * 16 + c] = b[c];
      }
  }
  if (lane == 0) *cyc = (t1 - t0) / (reps > 0 ? reps : 1);
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
  // host Cholesky
  std::vector<double> L(256, 0.0), Li(256, 0.0);
  for (int j = 0; j < 16; ++j) {
    double s = D[j * 16 + j];
    for (int k = 0; k < j; ++k) s -= L[j * 16 + k] * L[j * 16 + k];
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
  hipMalloc(&dO, 512 * 8);
  hipMalloc(&dc, 8);
  hipMemcpy(dD, D.data(), 256 * 8, hipMemcpyHostToDevice);
  for (int v = 0; v < 4; ++v) {
    k_sweep<<<1, 64>>>(dD, dO, v, 100, dc);
    hipDeviceSynchronize();
    std::vector<double> O(512);
    unsigned long long cyc;
    hipMemcpy(O.data(), dO, 512 * 8, hipMemcpyDeviceToHost);
    hipMemcpy(&cyc, dc, 8, hipMemcpyDeviceToHost);
    double eL = 0, eI = 0;
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        eL = fmax(eL, fabs(O[i * 16 + j] - L[i * 16 + j]));
        // (L^-T)' L = I: row r of O[256..] is row r of L^-T
        double s = 0;
        for (int k = 0; k < 16; ++k) s += O[256 + k * 16 + i] * L[k * 16 + j];
        eI = fmax(eI, fabs(s - (i == j ? 1.0 : 0.0)));
      }
    printf("variant %d: %llu cycles per sweep  max|L - Lref| = %.3e  max|Linv L - I| = %.3e\n", v, cyc, eL, eI);
  }
  return 0;
}
