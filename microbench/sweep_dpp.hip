// Microbenchmark: the 16-column elimination sweep of potrf64w with every column broadcast folded into the update
// instruction itself -- v_fmac_f64 with DPP row_newbcast:c on its first source (gfx90a+ 64-bit DPP), in inline asm.
//
// Layout (one wave): lane l, lane-row g = l >> 4, r = l & 15.  Every lane-row holds a copy of the 16 x 16 block, row r
// in a[0..15] (the copies stay identical: the same instructions), so D_cj = lane c's a[j] is one row_newbcast:c away in
// every lane-row.  b[0..15] is the row the column operations also act on: lane-row 0 the identity border (-> U with
// D U = L~, i.e. L16^-T without its column scales, as potrf64w), lane-rows 1..3 up to 48 panel rows below the block
// (-> the panel times U: the TRSM T of potrf64w comes out of the sweep).  Per column j, c > j:
//   a[c] += D_cj * (-a[j] / p_j),   b[c] += D_cj * (-b[j] / p_j)       (two v_fmac_f64_dpp, no v_readlane)
// the next pivot p_j+1 = lane j+1's a[j+1] right after its update (one v_mov_b64_dpp), its reciprocal off the other
// updates.  Against the v_readlane sweep (microbench/sweep.hip v0: 2 (15 - j) readlanes + (15 - j) FMAs per column).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off microbench/sweep_dpp.hip -o microbench/sweep_dpp
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <utility>
#include <vector>

#include "../cvx_amd/csrc/potrf64.hpp"
using namespace cvxg;

// dst += bcast_C(src) * m   (row_newbcast:C = lane C of each row of 16 lanes)
template <int C>
__device__ __forceinline__ void fmac_bc(double& dst, double src, double m) {
  asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
               : "+v"(dst)
               : "v"(src), "v"(m), "i"(C));
}
template <int C>
__device__ __forceinline__ double bc(double src) {
  double d;
  asm volatile("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "=v"(d) : "v"(src), "i"(C));
  return d;
}

template <int J>
__device__ __forceinline__ void step(double (&a)[16], double (&b)[16], double& piv, double& rinv, double (&sv)[16],
                                     double& pmin, int& firstbad) {
  if constexpr (J < 16) {
    if (!(piv > 0.0) && firstbad < 0) firstbad = J;
    pmin = fmin(pmin, piv);
    sv[J] = rsqrt_nr(piv);
    const double nta = -(a[J] * rinv), ntb = -(b[J] * rinv);
    if constexpr (J + 1 < 16) {
      fmac_bc<J + 1>(a[J + 1], a[J], nta);
      fmac_bc<J + 1>(b[J + 1], a[J], ntb);
      piv = bc<J + 1>(a[J + 1]);
      rinv = rcp_nr(piv);
    }
    [&]<int... Cs>(std::integer_sequence<int, Cs...>) {
      ((fmac_bc<J + 2 + Cs>(a[J + 2 + Cs], a[J], nta), fmac_bc<J + 2 + Cs>(b[J + 2 + Cs], a[J], ntb)), ...);
    }(std::make_integer_sequence<int, (J + 2 < 16 ? 14 - J : 0)>{});
    step<J + 1>(a, b, piv, rinv, sv, pmin, firstbad);
  }
}

__global__ __launch_bounds__(64) void k_sweep_dpp(const double* __restrict__ D, const double* __restrict__ Pn,
                                                  double* __restrict__ out, int reps, unsigned long long* cyc) {
  const int lane = threadIdx.x, r = lane & 15, g = lane >> 4;
  unsigned long long t0 = 0, t1 = 0;
  double a[16], b[16], sv[16];
  double pmin = 1e300;
  int firstbad = -1;
  for (int rep = 0; rep <= reps; ++rep) {
    if (rep == 1) t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      a[c] = D[r * 16 + c];
      b[c] = (g == 0) ? ((c == r) ? 1.0 : 0.0) : Pn[(16 * (g - 1) + r) * 16 + c];
    }
    double piv = bc<0>(a[0]);
    double rinv = rcp_nr(piv);
    step<0>(a, b, piv, rinv, sv, pmin, firstbad);
    __builtin_amdgcn_sched_barrier(0);
  }
  t1 = __builtin_amdgcn_s_memtime();
  // lane-row 0: L = a diag(s) (lower), U diag(s) = L^-T; lane-rows 1..3: panel U diag(s) = P L^-T
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const double s = sv[c];
    if (g == 0) {
      out[r * 16 + c] = (c <= r) ? a[c] * s : 0.0;
      out[256 + r * 16 + c] = b[c] * s;
    } else {
      out[512 + (16 * (g - 1) + r) * 16 + c] = b[c] * s;
    }
  }
  if (lane == 0) {
    *cyc = (t1 - t0) / (reps > 0 ? reps : 1);
    out[512 + 768] = firstbad;
    out[512 + 769] = pmin;
  }
}

int main() {
  std::vector<double> B(256), D(256), Pn(768);
  srand(3);
  for (auto& v : B) v = (double)rand() / RAND_MAX - 0.5;
  for (auto& v : Pn) v = (double)rand() / RAND_MAX - 0.5;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double s = 0;
      for (int k = 0; k < 16; ++k) s += B[i * 16 + k] * B[j * 16 + k];
      D[i * 16 + j] = s / 16 + (i == j ? 1.0 : 0.0);
    }
  std::vector<double> L(256, 0.0);
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
  // panel reference: X L' = Pn  (row by row forward substitution)
  std::vector<double> X(768, 0.0);
  for (int i = 0; i < 48; ++i)
    for (int j = 0; j < 16; ++j) {
      double t = Pn[i * 16 + j];
      for (int k = 0; k < j; ++k) t -= X[i * 16 + k] * L[j * 16 + k];
      X[i * 16 + j] = t / L[j * 16 + j];
    }
  double *dD, *dP, *dO;
  unsigned long long* dc;
  hipMalloc(&dD, 256 * 8);
  hipMalloc(&dP, 768 * 8);
  hipMalloc(&dO, 1300 * 8);
  hipMalloc(&dc, 8);
  hipMemcpy(dD, D.data(), 256 * 8, hipMemcpyHostToDevice);
  hipMemcpy(dP, Pn.data(), 768 * 8, hipMemcpyHostToDevice);
  for (int run = 0; run < 3; ++run) {
    k_sweep_dpp<<<1, 64>>>(dD, dP, dO, 100, dc);
    hipDeviceSynchronize();
    std::vector<double> O(1300);
    unsigned long long cyc;
    hipMemcpy(O.data(), dO, 1300 * 8, hipMemcpyDeviceToHost);
    hipMemcpy(&cyc, dc, 8, hipMemcpyDeviceToHost);
    double eL = 0, eI = 0, eP = 0;
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        eL = fmax(eL, fabs(O[i * 16 + j] - L[i * 16 + j]));
        double s = 0;  // (L^-T)' L = I
        for (int k = 0; k < 16; ++k) s += O[256 + k * 16 + i] * L[k * 16 + j];
        eI = fmax(eI, fabs(s - (i == j ? 1.0 : 0.0)));
      }
    for (int i = 0; i < 768; ++i) eP = fmax(eP, fabs(O[512 + i] - X[i]));
    printf("dpp-fmac sweep (+48 panel rows): %llu cycles per 16 columns  max|L - Lref| = %.3e  max|Linv L - I| = %.3e"
           "  max|T - Tref| = %.3e  firstbad %g\n", cyc, eL, eI, eP, O[512 + 768]);
  }
  return 0;
}
