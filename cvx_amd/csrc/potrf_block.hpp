// potrf_block.hpp — 64x64 diagonal-block Cholesky (dpotrf 'L' semantics, MatrixUtils.scala:452-461 via
// Breeze cholesky) with the block inverse and the fused forward substitution, built for a short
// per-column critical path on one CU.
//
// Structure: NPAN panels of PW columns; 4 waves; lane r of every wave holds row r of three bordered
// systems for the columns of the panels the wave owns (snake order: early and late work balanced):
//   a[] : row r of the block A_kk           -> L_kk
//   e[] : row r of the identity border      -> (L_kk^-1)^T   (Linv for the panel TRSM / back solve)
//   u[] : rhs vector r (lanes < nrhs)        -> w = L_kk^-1 b (forward substitution fused in)
// Panel p: the owner wave eliminates the panel's columns right-looking inside the wave (pivots and
// multipliers broadcast with v_readlane, rsqrt + Newton, no divisions) and publishes the finished L / W
// panel to LDS; ONE workgroup barrier; every wave then applies the rank-PW update to its owned later
// columns.  The owner of panel p+1 starts its panel right after its own update, so the other waves'
// updates of panel p overlap it (intra-block lookahead).
//
// potrf_block<Mem> is shared by the per-block kernel (k_potrf.hip, plain accesses) and by the persistent
// dataflow factorization (k_dataflow.hip), where every access to handed-off data is an sc1 access.
#pragma once
#include <math.h>

#include "kernels.hpp"

namespace cvxg {

#ifndef POTRF_PW
#define POTRF_PW 8
#endif
constexpr int PW = POTRF_PW;     // panel width
constexpr int NPAN = NB / PW;    // panels
constexpr int NS = NPAN / 4;     // panels owned per wave

__device__ __forceinline__ double rsqrt_nr(double p) {
  double y = __builtin_amdgcn_rsq(p);
  const double h = 0.5 * p;
  y = y * (1.5 - h * y * y);
  y = y * (1.5 - h * y * y);
  return y;
}

__device__ __forceinline__ double readlane_d(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__host__ __device__ constexpr int owner_of(int p) { return ((p / 4) & 1) ? 3 - (p % 4) : (p % 4); }
__host__ __device__ constexpr int panel_of(int w, int s) { return 4 * s + ((s & 1) ? 3 - w : w); }

// Buffer descriptor over [base, base + bytes) built from values the compiler can see are wave-uniform
// (otherwise each buffer op is wrapped in a readfirstlane waterfall loop).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* base, unsigned bytes) {
  const unsigned long long a = reinterpret_cast<unsigned long long>(base);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  const unsigned nb = __builtin_amdgcn_readfirstlane(bytes);
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((unsigned long long)hi << 32) | lo), 0, nb,
                                           0x00020000);
}

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int AUX_SC1 = 16;  // cache-policy bits of a buffer access: sc1 (L1 bypass, write-through)

// Memory policies over one region (a tile, a rhs block), addressed by double offsets.
//   PlainMem: ordinary cached accesses (kernel boundaries order everything).
//   Sc1Mem:   buffer_load/store ... sc1 — the inter-workgroup hand-off form used inside one launch
//             (MI355X_MICROARCH.md, visibility: Valid forms, row 1).  Ordinary (non-atomic) loads, so
//             the compiler keeps many in flight.
struct PlainMem {
  double* p;
  __device__ PlainMem(double* base, unsigned) : p(base) {}
  __device__ __forceinline__ double ld(int off) const { return p[off]; }
  __device__ __forceinline__ void st(int off, double v) const { p[off] = v; }
};
typedef double f64x2 __attribute__((ext_vector_type(2)));
struct Sc1Mem {
  __amdgpu_buffer_rsrc_t r;
  __device__ Sc1Mem(double* base, unsigned bytes) : r(uniform_rsrc(base, bytes)) {}
  __device__ __forceinline__ double ld(int off) const {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off * 8, 0, AUX_SC1));
  }
  __device__ __forceinline__ void st(int off, double v) const {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, off * 8, 0, AUX_SC1);
  }
  __device__ __forceinline__ f64x2 ld2(int off) const {  // 16 B, off even
    return __builtin_bit_cast(f64x2, __builtin_amdgcn_raw_buffer_load_b128(r, off * 8, 0, AUX_SC1));
  }
};

// bytes spanned by a 64 x 64 tile with leading dimension ld (for a tile descriptor)
__host__ __device__ constexpr unsigned tile_bytes(int ld) { return (unsigned)((NB - 1) * ld + NB) * 8u; }

struct PotrfSmem {
  double Lp[NPAN][NB][PW];       // final L, by panel
  double Ep[NPAN][NB][PW];       // final W = (L^-1)^T rows, by panel
  double Wp[NPAN][MAX_RHS][PW];  // forward-solved rhs, by panel
  int fail;
};

#ifdef POTRF_STAMPS  // microbench/potrf_bench.hip: per-wave s_memtime stamps of the phases
__device__ unsigned long long g_potrf_stamps[4][64];
#define POTRF_STAMP(i)                                                        \
  do {                                                                        \
    if (lane == 0) g_potrf_stamps[w][(i)] = __builtin_amdgcn_s_memtime();     \
  } while (0)
#else
#define POTRF_STAMP(i) \
  do {                 \
  } while (0)
#endif

// Factor block k of L (lower part of the 64x64 diagonal block), write L_kk, Linv[k] = L_kk^-1 and the
// forward-solved rhs block.  Returns false (uniformly) on a non-positive pivot, after recording the
// 1-based global pivot index in ctrl->chol_info.
template <class M>
__device__ bool potrf_block(double* __restrict__ L, int ld, int k, double* __restrict__ rhs, int nrhs,
                            double* __restrict__ Linv, DevCtrl* ctrl, PotrfSmem& sm) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int base = k * NB;
  const M mL(L + (size_t)base * ld + base, tile_bytes(ld));                         // the diagonal tile
  const M mR(rhs + (size_t)base * nrhs, (unsigned)(NB * nrhs) * 8u);                // rhs block k
  const M mI(Linv + (size_t)k * NB * NB, (unsigned)(NB * NB) * 8u);                 // Linv[k]
  double a[NS][PW], e[NS][PW], u[NS][PW];  // slot s holds panel panel_of(w, s)
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int q = panel_of(w, s);
#pragma unroll
    for (int j = 0; j < PW; ++j) {
      const double t = mL.ld(lane * ld + PW * q + j);
      a[s][j] = (PW * q + j <= lane) ? t : 0.0;
      e[s][j] = (PW * q + j == lane) ? 1.0 : 0.0;
      const double b = mR.ld((PW * q + j) * nrhs + min(lane, nrhs - 1));
      u[s][j] = (lane < nrhs) ? b : 0.0;
    }
  }
  if (tid == 0) sm.fail = 0;
  double mind = __builtin_inf();
  POTRF_STAMP(0);
  __syncthreads();
  POTRF_STAMP(1);

#pragma unroll
  for (int p = 0; p < NPAN; ++p) {
    const int o = owner_of(p);
    const int so = p / 4;  // owner's slot for panel p (static)
    // ---- phase A: owner wave eliminates the panel -------------------------------------------------
    if (w == o) {
      bool bad = false;
#pragma unroll
      for (int j = 0; j < PW; ++j) {
        const double piv = readlane_d(a[so][j], PW * p + j);
        bad = bad || !(piv > 0.0);
        const double rl = rsqrt_nr(piv);
        mind = fmin(mind, piv * rl);
        a[so][j] *= rl;
        e[so][j] *= rl;
        u[so][j] *= rl;
#pragma unroll
        for (int c = j + 1; c < PW; ++c) {
          const double lcj = readlane_d(a[so][j], PW * p + c);
          a[so][c] = fma(-a[so][j], lcj, a[so][c]);
          e[so][c] = fma(-e[so][j], lcj, e[so][c]);
          u[so][c] = fma(-u[so][j], lcj, u[so][c]);
        }
      }
#pragma unroll
      for (int j = 0; j < PW; ++j) {
        const double va = (PW * p + j <= lane) ? a[so][j] : 0.0;  // L is lower: zero above the diagonal
        a[so][j] = va;
        sm.Lp[p][lane][j] = va;
        sm.Ep[p][lane][j] = e[so][j];
        if (lane < nrhs) sm.Wp[p][lane][j] = u[so][j];
      }
      if (bad && lane == 0) {
        sm.fail = 1;
        atomicCAS(&ctrl->chol_info, 0, base + PW * p + 1);
      }
      POTRF_STAMP(2 + 3 * p);
    }
    __syncthreads();
    POTRF_STAMP(3 + 3 * p);
    if (sm.fail) return false;  // uniform: every wave reads the same flag after the barrier
    // ---- phase B: every wave applies panel p to its owned later columns --------------------------
    double xr[PW], er[PW], ur[PW];
#pragma unroll
    for (int j = 0; j < PW; ++j) {
      xr[j] = sm.Lp[p][lane][j];
      er[j] = sm.Ep[p][lane][j];
      ur[j] = (lane < nrhs) ? sm.Wp[p][lane][j] : 0.0;
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int q = panel_of(w, s);
      if (q > p) {
        // the PW x PW block L[PW q.., PW p..] as broadcast LDS loads, issued in batches ahead of the FMAs
        constexpr int RH = PW < 8 ? PW : 4;
#pragma unroll
        for (int h = 0; h < PW / RH; ++h) {
          typedef double v2 __attribute__((ext_vector_type(2)));
          v2 lc[RH][PW / 2];
#pragma unroll
          for (int i = 0; i < RH; ++i)
#pragma unroll
            for (int jp = 0; jp < PW / 2; ++jp)
              lc[i][jp] = *reinterpret_cast<const v2*>(&sm.Lp[p][PW * q + RH * h + i][2 * jp]);
#pragma unroll
          for (int i = 0; i < RH; ++i) {
            const int jj = RH * h + i;
#pragma unroll
            for (int jp = 0; jp < PW / 2; ++jp)
#pragma unroll
              for (int t = 0; t < 2; ++t) {
                const double l = lc[i][jp][t];
                a[s][jj] = fma(-xr[2 * jp + t], l, a[s][jj]);
                e[s][jj] = fma(-er[2 * jp + t], l, e[s][jj]);
                u[s][jj] = fma(-ur[2 * jp + t], l, u[s][jj]);
              }
          }
        }
      }
      if (s == 0) POTRF_STAMP(4 + 3 * p);
    }
  }
  __syncthreads();
  POTRF_STAMP(60);
  // ---- outputs: L block (lower), Linv[r][c] = W[c][r], w -----------------------------------------
  for (int t = tid; t < NB * NB; t += 256) {
    const int r = t / NB, c = t % NB;
    if (c <= r) mL.st(r * ld + c, sm.Lp[c / PW][r][c % PW]);
    mI.st(t, sm.Ep[r / PW][c][r % PW]);
  }
  for (int t = tid; t < nrhs * NB; t += 256) {
    const int rho = t / NB, c = t % NB;
    mR.st(c * nrhs + rho, sm.Wp[c / PW][rho][c % PW]);
  }
  if (lane == 0) atomic_min_pos(&ctrl->min_diag, mind);
  POTRF_STAMP(61);
  return true;
}

}  // namespace cvxg
