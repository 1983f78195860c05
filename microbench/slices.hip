// Microbenchmark of the chain's TRSM / UPDATE slices (k_dataflow.hip): one workgroup, operands in LDS.
//   slice cb:  L'[16 w.., 16 cb..] = A[16 w.., :] X[16 cb.., :]^T  (K = 16 (cb + 1)), then D -= L'[:, cb] L'[:, cb]^T on
//   the wave's lower 16 x 16 blocks (3 / 3 / 2 / 2), a workgroup barrier between the two.
// Variants (argv[1]): 0 LDS only; 1 + the sc1 global store of L' per slice; 2 = 1 + a global load issued after the
// stores and consumed in the next slice (the chain's next-row-block prefetch); 3 = UPDATE blocks interleaved (all of a
// wave's accumulators advance together, so independent MFMAs fill each other's latency).
// Bits: 4 skips the UPDATE, 8 the TRSM, 16 the barriers, 32 = batched operand reads (TRSM A fragments in
// registers across slices, one LDS wait per product); 64 = the UPDATE with per-wave compile-time blocks (with 32: batched TRSM too).  Prints shader-clock cycles (s_memtime) per slice.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 microbench/slices.hip -o microbench/slices
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "../cvx_amd/csrc/potrf64.hpp"
using namespace cvxg;

constexpr int SP = NB + 2;

// batched forms: every operand fragment read from LDS first (one wait), then the MFMAs back to back
template <int CB>
__device__ __forceinline__ d4f trsm_batched(const double (&af)[16], const double* Xr, int lane) {
  double xf[4 * (CB + 1)];
#pragma unroll
  for (int s = 0; s < 4 * (CB + 1); ++s) xf[s] = Xr[(lane & 15) * SP + 4 * s + (lane >> 4)];
  d4f acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int s = 0; s < 4 * (CB + 1); s += 2) {
    acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(af[s], xf[s], acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(af[s + 1], xf[s + 1], acc1, 0, 0, 0);
  }
  return acc0 + acc1;
}

// per-wave templated UPDATE: the wave's blocks (ib, jb) are compile-time, so the fragments are selected statically
constexpr int kIB[4][3] = {{0, 3, 3}, {1, 3, 2}, {1, 3, -1}, {2, 2, -1}};
constexpr int kJB[4][3] = {{0, 0, 3}, {0, 1, 2}, {1, 2, -1}, {0, 1, -1}};
template <int W>
__device__ __forceinline__ void update_static(d4f (&dacc)[3], const double* Lp, int cb, int lane) {
  constexpr bool use[4] = {kIB[W][0] == 0 || kJB[W][0] == 0 || kIB[W][1] == 0 || kJB[W][1] == 0 || kIB[W][2] == 0 || kJB[W][2] == 0,
                           kIB[W][0] == 1 || kJB[W][0] == 1 || kIB[W][1] == 1 || kJB[W][1] == 1 || kIB[W][2] == 1 || kJB[W][2] == 1,
                           kIB[W][0] == 2 || kJB[W][0] == 2 || kIB[W][1] == 2 || kJB[W][1] == 2 || kIB[W][2] == 2 || kJB[W][2] == 2,
                           kIB[W][0] == 3 || kJB[W][0] == 3 || kIB[W][1] == 3 || kJB[W][1] == 3 || kIB[W][2] == 3 || kJB[W][2] == 3};
  double lf[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
    if (use[r])
#pragma unroll
      for (int q = 0; q < 4; ++q) lf[r][q] = Lp[(16 * r + (lane & 15)) * SP + 16 * cb + 4 * q + (lane >> 4)];
#pragma unroll
  for (int st = 0; st < 4; ++st)
#pragma unroll
    for (int q = 0; q < 3; ++q)
      if (kIB[W][q] >= 0)
        dacc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(-lf[kIB[W][q]][st], lf[kJB[W][q]][st], dacc[q], 0, 0, 0);
}

__global__ __launch_bounds__(256) void k_slices(double* __restrict__ g, const double* __restrict__ src, int variant,
                                                int reps, unsigned long long* cyc, double* sink) {
  __shared__ double A[NB * SP], X[NB * SP], Lp[NB * SP], E[16 * SP];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int t = tid; t < NB * SP; t += 256) {
    A[t] = src[t % 4096] * 0.01;
    X[t] = src[(t * 7) % 4096] * 0.01;
    Lp[t] = 0.0;
  }
  const int blk_ib[4][3] = {{0, 3, 3}, {1, 3, 2}, {1, 3, -1}, {2, 2, -1}};
  const int blk_jb[4][3] = {{0, 0, 3}, {0, 1, 2}, {1, 2, -1}, {0, 1, -1}};
  d4f dacc[3];
  for (int q = 0; q < 3; ++q) dacc[q] = d4f{0.0, 0.0, 0.0, 0.0};
  const Sc1Mem mA(g, tile_bytes(NB));
  const Sc1Mem mI(g + NB * NB, tile_bytes(NB));
  __syncthreads();
  unsigned long long t0 = 0;
  f64x2 er[2] = {};
  double af[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) af[q] = A[(16 * wv + (lane & 15)) * SP + 4 * q + (lane >> 4)];
  for (int rep = 0; rep <= reps; ++rep) {
    if (rep == 1) t0 = __builtin_amdgcn_s_memtime();
    for (int cb = 0; cb < 4; ++cb) {
      if (variant == 2) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {  // consume the previous slice's prefetch
          const int e = tid + 256 * q;
          *reinterpret_cast<f64x2*>(E + (e >> 5) * SP + 2 * (e & 31)) = er[q];
        }
      }
      if (!(variant & 16)) __syncthreads();
      if (variant & 32) {
        const double* Xr = X + 16 * cb * SP;
        d4f acc;
        switch (cb) {
          case 0: acc = trsm_batched<0>(af, Xr, lane); break;
          case 1: acc = trsm_batched<1>(af, Xr, lane); break;
          case 2: acc = trsm_batched<2>(af, Xr, lane); break;
          default: acc = trsm_batched<3>(af, Xr, lane); break;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) Lp[(16 * wv + (lane >> 4) + 4 * r) * SP + 16 * cb + (lane & 15)] = acc[r];
      } else if (!(variant & 8)) {
        d4f acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
        const double* Ar = A + 16 * wv * SP;
        const double* Xr = X + 16 * cb * SP;
        for (int s2 = 0; s2 < 4 * (cb + 1); s2 += 2) {
          const int kk = 4 * s2 + (lane >> 4);
          acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(Ar[(lane & 15) * SP + kk], Xr[(lane & 15) * SP + kk], acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(Ar[(lane & 15) * SP + kk + 4], Xr[(lane & 15) * SP + kk + 4], acc1,
                                                      0, 0, 0);
        }
        const d4f acc = acc0 + acc1;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * wv + (lane >> 4) + 4 * r, col = 16 * cb + (lane & 15);
          Lp[row * SP + col] = acc[r];
          if (variant >= 1 && variant <= 2) mA.st(row * NB + col, acc[r]);
        }
      }
      if (!(variant & 16)) __syncthreads();
      if (variant == 2) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int e = tid + 256 * q;
          er[q] = mI.ld2((16 * ((cb + 1) & 3) + (e >> 5)) * NB + 2 * (e & 31));
        }
      }
      if (variant & 64) {
        switch (wv) {
          case 0: update_static<0>(dacc, Lp, cb, lane); break;
          case 1: update_static<1>(dacc, Lp, cb, lane); break;
          case 2: update_static<2>(dacc, Lp, cb, lane); break;
          default: update_static<3>(dacc, Lp, cb, lane); break;
        }
      } else if (variant & 32) {
        // the wave's row-blocks of L'[:, cb]: fragments of all four (A and B layouts coincide for A B^T)
        double lf[4][4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int q = 0; q < 4; ++q) lf[r][q] = Lp[(16 * r + (lane & 15)) * SP + 16 * cb + 4 * q + (lane >> 4)];
        d4f a[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) a[q] = dacc[q];
#pragma unroll
        for (int st = 0; st < 4; ++st)
#pragma unroll
          for (int q = 0; q < 3; ++q) {
            const int ib = blk_ib[wv][q] < 0 ? 0 : blk_ib[wv][q], jb = blk_ib[wv][q] < 0 ? 0 : blk_jb[wv][q];
            double x = 0, y = 0;  // (select the row-block fragments by the wave-uniform ib / jb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              x = ib == r ? lf[r][st] : x;
              y = jb == r ? lf[r][st] : y;
            }
            a[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(-x, y, a[q], 0, 0, 0);
          }
#pragma unroll
        for (int q = 0; q < 3; ++q)
          if (blk_ib[wv][q] >= 0) dacc[q] = a[q];
      } else if (variant == 3) {
        d4f a0 = dacc[0], a1 = dacc[1], a2 = dacc[2];
        const int i0 = blk_ib[wv][0], j0 = blk_jb[wv][0], i1 = blk_ib[wv][1], j1 = blk_jb[wv][1];
        const int i2 = blk_ib[wv][2] < 0 ? i1 : blk_ib[wv][2], j2 = blk_ib[wv][2] < 0 ? j1 : blk_jb[wv][2];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int k = 16 * cb + 4 * s + (lane >> 4), r = lane & 15;
          a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(-Lp[(16 * i0 + r) * SP + k], Lp[(16 * j0 + r) * SP + k], a0, 0, 0, 0);
          a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(-Lp[(16 * i1 + r) * SP + k], Lp[(16 * j1 + r) * SP + k], a1, 0, 0, 0);
          a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(-Lp[(16 * i2 + r) * SP + k], Lp[(16 * j2 + r) * SP + k], a2, 0, 0, 0);
        }
        dacc[0] = a0;
        dacc[1] = a1;
        if (blk_ib[wv][2] >= 0) dacc[2] = a2;
      } else if (!(variant & 4)) {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const int ib = blk_ib[wv][q], jb = blk_jb[wv][q];
          if (ib >= 0)
            dacc[q] = mfma16_abt(dacc[q], Lp + 16 * ib * SP + 16 * cb, SP, Lp + 16 * jb * SP + 16 * cb, SP, -1.0, lane);
        }
      }
    }
  }
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
  for (int q = 0; q < 3; ++q) s += dacc[q][0] + dacc[q][1] + dacc[q][2] + dacc[q][3];
  sink[tid] = s + er[0][0] + er[1][1];
  if (tid == 0) *cyc = (t1 - t0) / (reps * 4);
}

int main(int argc, char** argv) {
  double *g, *src, *sink;
  unsigned long long* cyc;
  hipMalloc(&g, 2 * NB * NB * 8);
  hipMalloc(&src, 4096 * 8);
  hipMalloc(&sink, 256 * 8);
  hipMalloc(&cyc, 8);
  double h[4096];
  for (int i = 0; i < 4096; ++i) h[i] = (double)rand() / RAND_MAX;
  hipMemcpy(src, h, sizeof h, hipMemcpyHostToDevice);
  hipMemset(g, 0, 2 * NB * NB * 8);
  const int vs[] = {0, 4, 8, 32, 48, 96, 112, 64 + 8, 64 + 16 + 8};
  for (int v : vs) {
    k_slices<<<1, 256>>>(g, src, v, 50, cyc, sink);
    hipDeviceSynchronize();
    unsigned long long c;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("variant %2d: %llu cycles per slice\n", v, c);
  }
  return 0;
}
