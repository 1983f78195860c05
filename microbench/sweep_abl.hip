// Ablations of the DPP elimination sweep (inputs held in registers, so no memory round trip is timed) (microbench/sweep_dpp.hip, potrf64w.hpp p64w_eliminate_dpp): where do the
// ~3 600 cycles per 16 columns go?  One wave, the same data layout as sweep_dpp.hip; every mode times 100 sweeps.
//   M0  the production sweep (rcp_nr: v_rcp_f64 + two mul/sub/mul Newton steps; column scale rsqrt in the loop)
//   M1  M0 without the column-scale rsqrt inside the loop (formed after the sweep from the kept pivots)
//   M2  M1 with the reciprocal's Newton steps in fma form (e = fma(-p, y, 1), y = fma(y, e, y), twice)
//   M3  M1 without the off-chain updates (columns j+2..15): the pivot chain alone
//   M4  M1 with the reciprocal replaced by the pivot itself: the update issue alone (numerically meaningless)
//   M5  M4 with plain v_fma_f64 (no DPP) on the updates: the DPP cost
//   M6  M1 with the off-chain updates of column j issued in two halves around the next pivot's reciprocal
//   M7  M1 with the reciprocal's seven steps as asm statements and the off-chain updates spread between them
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off microbench/sweep_abl.hip -o microbench/sweep_abl
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <utility>
#include <vector>

#include "../cvx_amd/csrc/potrf64.hpp"
using namespace cvxg;

template <int C>
__device__ __forceinline__ void fmac_bc(double& dst, double src, double m) {
  asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
               : "+v"(dst)
               : "v"(src), "v"(m), "i"(C));
}
template <int C>
__device__ __forceinline__ void fmac_plain(double& dst, double src, double m) {
  asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(dst) : "v"(src), "v"(m));
}
template <int C>
__device__ __forceinline__ double bc(double src) {
  double d;
  asm volatile("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "=v"(d) : "v"(src), "i"(C));
  return d;
}
__device__ __forceinline__ double rcp_fma(double p) {
  double y = __builtin_amdgcn_rcp(p);
  double e = fma(-p, y, 1.0);
  y = fma(y, e, y);
  e = fma(-p, y, 1.0);
  y = fma(y, e, y);
  return y;
}

// the reciprocal's steps as separate asm statements (the same instructions rcp_nr compiles to: v_rcp_f64, then twice
// t = p y; u = 2 - t; y = y u), so that they stay where they are written among the update fmacs
__device__ __forceinline__ double a_rcp(double p) {
  double y;
  asm volatile("v_rcp_f64 %0, %1\n\ts_nop 1" : "=v"(y) : "v"(p));  // (trans -> VALU use: wait states)
  return y;
}
__device__ __forceinline__ double a_mul(double x, double y) {
  double r;
  asm volatile("v_mul_f64 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
  return r;
}
__device__ __forceinline__ double a_two_minus(double t) {
  double r;
  asm volatile("v_add_f64 %0, -%1, 2.0" : "=v"(r) : "v"(t));
  return r;
}
// the I-th of the 2 R off-chain updates of column J (R = 14 - J columns c = J + 2 .., a then b)
template <int J, int I>
__device__ __forceinline__ void rest_one(double (&a)[16], double (&b)[16], double nta, double ntb) {
  constexpr int NR = (J + 2 < 16 ? 14 - J : 0);
  if constexpr (I < 2 * NR) {
    constexpr int c = J + 2 + I / 2;
    if constexpr (I % 2 == 0) fmac_bc<c>(a[c], a[J], nta);
    else fmac_bc<c>(b[c], a[J], ntb);
  }
}
template <int J, int I0, int N>
__device__ __forceinline__ void rest_range(double (&a)[16], double (&b)[16], double nta, double ntb) {
  if constexpr (N > 0) {
    rest_one<J, I0>(a, b, nta, ntb);
    rest_range<J, I0 + 1, N - 1>(a, b, nta, ntb);
  }
}

template <int M, int J, int... Cs>
__device__ __forceinline__ void rest(double (&a)[16], double (&b)[16], double nta, double ntb, int lo,
                                     std::integer_sequence<int, Cs...>) {
  if constexpr (M == 5) {
    ((fmac_plain<J + 2 + Cs>(a[J + 2 + Cs], a[J], nta), fmac_plain<J + 2 + Cs>(b[J + 2 + Cs], a[J], ntb)), ...);
  } else {
    ((fmac_bc<J + 2 + Cs>(a[J + 2 + Cs], a[J], nta), fmac_bc<J + 2 + Cs>(b[J + 2 + Cs], a[J], ntb)), ...);
  }
}

template <int M, int J>
__device__ __forceinline__ void step(double (&a)[16], double (&b)[16], double& piv, double& rinv, double (&sv)[16],
                                     double& pmin, int& firstbad) {
  if constexpr (J < 16) {
    if (!(piv > 0.0) && firstbad < 0) firstbad = J;
    pmin = fmin(pmin, piv);
    if constexpr (M == 0) sv[J] = rsqrt_nr(piv); else sv[J] = piv;
    const double nta = -(a[J] * rinv), ntb = -(b[J] * rinv);
    constexpr int NR = (J + 2 < 16 ? 14 - J : 0);
    if constexpr (J + 1 < 16) {
      if constexpr (M == 5) {
        fmac_plain<J + 1>(a[J + 1], a[J], nta);
        fmac_plain<J + 1>(b[J + 1], a[J], ntb);
      } else {
        fmac_bc<J + 1>(a[J + 1], a[J], nta);
        fmac_bc<J + 1>(b[J + 1], a[J], ntb);
      }
      piv = bc<J + 1>(a[J + 1]);
      if constexpr (M == 7) {
        // the reciprocal chain with the off-chain updates spread between its seven steps (K per gap)
        constexpr int K = (2 * NR + 6) / 7;
        double y = a_rcp(piv);
        rest_range<J, 0 * K, K>(a, b, nta, ntb);
        double t = a_mul(piv, y);
        rest_range<J, 1 * K, K>(a, b, nta, ntb);
        double u = a_two_minus(t);
        rest_range<J, 2 * K, K>(a, b, nta, ntb);
        y = a_mul(y, u);
        rest_range<J, 3 * K, K>(a, b, nta, ntb);
        t = a_mul(piv, y);
        rest_range<J, 4 * K, K>(a, b, nta, ntb);
        u = a_two_minus(t);
        rest_range<J, 5 * K, K>(a, b, nta, ntb);
        rinv = a_mul(y, u);
        rest_range<J, 6 * K, 2 * NR - 6 * K>(a, b, nta, ntb);
      } else if constexpr (M == 6) {
        // first half of the off-chain updates, then the reciprocal, then the second half
        rest<M, J>(a, b, nta, ntb, 0, std::make_integer_sequence<int, NR / 2>{});
        rinv = rcp_nr(piv);
        [&]<int... Cs>(std::integer_sequence<int, Cs...>) {
          ((fmac_bc<J + 2 + NR / 2 + Cs>(a[J + 2 + NR / 2 + Cs], a[J], nta),
            fmac_bc<J + 2 + NR / 2 + Cs>(b[J + 2 + NR / 2 + Cs], a[J], ntb)), ...);
        }(std::make_integer_sequence<int, NR - NR / 2>{});
      } else {
        if constexpr (M == 2) rinv = rcp_fma(piv);
        else if constexpr (M == 4 || M == 5) rinv = piv;
        else rinv = rcp_nr(piv);
      }
    }
    if constexpr (M != 3 && M != 6 && M != 7) rest<M, J>(a, b, nta, ntb, 0, std::make_integer_sequence<int, NR>{});
    step<M, J + 1>(a, b, piv, rinv, sv, pmin, firstbad);
  }
}

template <int M>
__global__ __launch_bounds__(64) void k_sweep(const double* __restrict__ D, const double* __restrict__ Pn,
                                              double* __restrict__ out, int reps, unsigned long long* cyc) {
  const int lane = threadIdx.x, r = lane & 15, g = lane >> 4;
  unsigned long long t0 = 0, t1 = 0;
  double a[16], b[16], sv[16];
  double pmin = 1e300;
  int firstbad = -1;
  double a0[16], b0[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    a0[c] = D[r * 16 + c];
    b0[c] = (g == 0) ? ((c == r) ? 1.0 : 0.0) : Pn[(16 * (g - 1) + r) * 16 + c];
  }
  for (int rep = 0; rep <= reps; ++rep) {
    if (rep == 1) t0 = __builtin_amdgcn_s_memtime();
    // the inputs are re-copied from registers each rep (global loads would put a memory round trip in the timing)
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      a[c] = a0[c];
      b[c] = b0[c];
    }
    double piv = bc<0>(a[0]);
    double rinv = (M == 4 || M == 5) ? piv : rcp_nr(piv);
    step<M, 0>(a, b, piv, rinv, sv, pmin, firstbad);
    __builtin_amdgcn_sched_barrier(0);
  }
  t1 = __builtin_amdgcn_s_memtime();
  if constexpr (M != 0) {
#pragma unroll
    for (int c = 0; c < 16; ++c) sv[c] = rsqrt_nr(sv[c]);
  }
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
  }
}

template <int M>
void run(const double* dD, const double* dP, double* dO, unsigned long long* dc, const std::vector<double>& L) {
  for (int rr = 0; rr < 2; ++rr) {
    k_sweep<M><<<1, 64>>>(dD, dP, dO, 100, dc);
    hipDeviceSynchronize();
    std::vector<double> O(1300);
    unsigned long long cyc;
    hipMemcpy(O.data(), dO, 1300 * 8, hipMemcpyDeviceToHost);
    hipMemcpy(&cyc, dc, 8, hipMemcpyDeviceToHost);
    double eL = 0;
    for (int i = 0; i < 256; ++i) eL = fmax(eL, fabs(O[i] - L[i]));
    printf("M%d: %llu cycles per 16 columns  max|L - Lref| = %.3e\n", M, cyc, eL);
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
  double *dD, *dP, *dO;
  unsigned long long* dc;
  hipMalloc(&dD, 256 * 8);
  hipMalloc(&dP, 768 * 8);
  hipMalloc(&dO, 1300 * 8);
  hipMalloc(&dc, 8);
  hipMemcpy(dD, D.data(), 256 * 8, hipMemcpyHostToDevice);
  hipMemcpy(dP, Pn.data(), 768 * 8, hipMemcpyHostToDevice);
  run<0>(dD, dP, dO, dc, L);
  run<1>(dD, dP, dO, dc, L);
  run<2>(dD, dP, dO, dc, L);
  run<3>(dD, dP, dO, dc, L);
  run<4>(dD, dP, dO, dc, L);
  run<5>(dD, dP, dO, dc, L);
  run<6>(dD, dP, dO, dc, L);
  run<7>(dD, dP, dO, dc, L);
  return 0;
}
