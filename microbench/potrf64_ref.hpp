// potrf64_ref.hpp — the round-1 64 x 64 diagonal-block Cholesky with block inverse and fused forward solve (two
// workgroup barriers per 16-column step), kept as the A/B reference of microbench/potrf64_bench.hip.  The engine
// uses the wave-specialised form, cvx_amd/csrc/potrf64w.hpp.
//
// The 64 columns are processed as 4 steps of 16 (blocks kb = 0..3 of 16 x 16):
//   P  wave 0 eliminates the 16 x 16 diagonal block D_kb with one lane per row: lanes 0-15 hold the rows
//      of D (-> L16), lanes 16-31 the rows of the identity border (-> L16^-T), so ONE fma per column and
//      element serves both, with the pivots and L_cj broadcast by v_readlane (no LDS, no barrier).
//      Meanwhile waves 1..kb accumulate T_kb,j = sum_{m=j}^{kb-1} L_kb,m X_m,j (MFMA) for the off-diagonal
//      blocks X_kb,j of L^-1 (block forward substitution of the inverse).
//   T  waves 1..3: X_kb,j = -L16^-1 T_kb,j, or the panel TRSM L_ib,kb = A_ib,kb L16^-T (MFMA).
//   U  A_ib,jb -= L_ib,kb L_jb,kb^T for kb < jb <= ib (MFMA); wave 0 takes the next diagonal block first.
#pragma once
#include "../cvx_amd/csrc/potrf64.hpp"

#ifndef P64_KB_UNROLL
#define P64_KB_UNROLL 0
#endif

namespace cvxg {

struct Potrf64Smem {
  double S[NB * P64_SP];         // the tile: A -> L (lower blocks)
  double X[NB * P64_SP];         // L^-1 (lower blocks)
  double ET[4][16 * P64_EP];     // per step: L16^-T (row r = column r of L16^-1)
  double B[NB * MAX_RHS];        // rhs block, row-major [64][nrhs]
  double W[NB * MAX_RHS];        // forward-solved rhs block w = L^-1 b
  int fail;
};

// Stage the 64 x 64 tile at (r0, c0) of L into sm.S (all 256 threads; no barrier).
template <class M>
__device__ __forceinline__ void potrf64_stage_tile(const double* L, int ld, size_t off, Potrf64Smem& sm) {
  const int tid = threadIdx.x;
  const M mL(const_cast<double*>(L) + off, tile_bytes(ld));
  f64x2 v[NB * NB / 512];
#pragma unroll
  for (int q = 0; q < NB * NB / 512; ++q) {
    const int idx = q * 256 + tid;
    v[q] = mL.ld2((idx >> 5) * ld + 2 * (idx & 31));
  }
#pragma unroll
  for (int q = 0; q < NB * NB / 512; ++q) {
    const int idx = q * 256 + tid;
    const int r = idx >> 5, c = 2 * (idx & 31);
    sm.S[r * P64_SP + c] = v[q][0];
    sm.S[r * P64_SP + c + 1] = v[q][1];
  }
}
// Stage rhs block k into sm.B (no barrier).
template <class M>
__device__ __forceinline__ void potrf64_stage_rhs(const double* rhs, int k, int nrhs, Potrf64Smem& sm) {
  const M mR(const_cast<double*>(rhs) + (size_t)k * NB * nrhs, (unsigned)(NB * nrhs) * 8u);
  for (int t = threadIdx.x; t < NB * nrhs; t += 256) sm.B[t] = mR.ld(t);
}

// potrf64_factor: the tile is staged in sm.S and the rhs block in sm.B (barrier pending); on return sm.X holds
// L^-1 (exact zeros above the diagonal) and sm.W the solved rhs block.
//
// lflag != nullptr (dataflow chain): row-block kb of L^-1 is stored to Linv[k] as soon as it is final (after step
// kb's T phase) by wave 3, which then raises *lflag = kb + 1 (sc1 hand-off: its own stores drained first), so
// the other chain workgroup can start the next TRSM while this one is still factoring.  The L_kk tile is not
// stored here in either case: potrf64_store_L.
//
// fix(): called by every thread after the last step, before the forward solve (barrier after it) — the chain uses
// it to apply the last rhs correction, whose input (w of the other workgroup's block) is only ready by then.
template <class M, class Fix = NoFix>
__device__ bool potrf64_factor(double* __restrict__ L, int ld, int k, double* __restrict__ rhs, int nrhs,
                               double* __restrict__ Linv, DevCtrl* ctrl, Potrf64Smem& sm, int* lflag = nullptr,
                               Fix fix = Fix(), unsigned long long* pub_stamp = nullptr) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int base = k * NB;
  const M mR(rhs + (size_t)base * nrhs, (unsigned)(NB * nrhs) * 8u);                // rhs block k
  const M mI(Linv + (size_t)k * NB * NB, (unsigned)(NB * NB) * 8u);                 // Linv[k]
  double* S = sm.S;
  double* X = sm.X;
  {  // L^-1 is lower block-triangular: zero the six 16 x 16 blocks above the diagonal (read by callers' MFMAs)
    for (int t = tid; t < 6 * 256; t += 256) {
      const int b = t >> 8, e = t & 255;
      const int ib = (b < 3) ? 0 : ((b < 5) ? 1 : 2), jb = (b < 3) ? 1 + b : ((b < 5) ? b - 1 : 3);
      X[(16 * ib + (e >> 4)) * P64_SP + 16 * jb + (e & 15)] = 0.0;
    }
    if (tid == 0) sm.fail = 0;
  }
  double mind = __builtin_inf();
  P64_STAMP(0);
  __syncthreads();
  P64_STAMP(1);

#if P64_KB_UNROLL
#pragma unroll
#else
#pragma unroll 1  // one copy of the step body: the instruction stream stays resident in the I-cache
#endif
  for (int kb = 0; kb < 4; ++kb) {
    const int o = 16 * kb;
    d4f T = {0.0, 0.0, 0.0, 0.0};
    // ---- P: wave 0 eliminates D_kb; waves 1..kb accumulate T_kb,j (j = w - 1) --------------------------
    if (w == 0) {
      // lanes 0-15: row r of D (lower triangle), lanes 16-31: row r of the identity border.  Step j reads the
      // still-unscaled column j with v_readlane and applies  v_c -= (v_j / p_j) D_cj  for c > j, then scales v_j
      // by p_j^-1/2 — one fma per element serves the L rows and the L^-T border rows alike.  The next pivot is
      // formed from uniform values, p_j+1 = D_j+1,j+1 - (D_j+1,j / p_j) D_j+1,j (bit-identical to lane j+1's own
      // update), so the per-column dependency chain is only 1/p (rcp + Newton) and one fma; the rsqrt of the
      // column scale and the element updates fill the issue slots beside it.
      const int r = lane & 15;
      double a[16];
      {
        const double* src = S + (o + r) * P64_SP + o;
#pragma unroll
        for (int c = 0; c < 16; c += 2) {
          const f64x2 v = *reinterpret_cast<const f64x2*>(src + c);
          a[c] = (lane < 16) ? ((c <= r) ? v[0] : 0.0) : ((lane < 32 && c == r) ? 1.0 : 0.0);
          a[c + 1] = (lane < 16) ? ((c + 1 <= r) ? v[1] : 0.0) : ((lane < 32 && c + 1 == r) ? 1.0 : 0.0);
        }
      }
      P64_STAMP(22 + 3 * kb);
      int firstbad = -1;
      double piv = readlane_d(a[0], 0);
      double rinv = rcp_nr(piv);
      double mypiv = 1.0;  // lane j keeps p_j: the column scales p_j^-1/2 are formed once, after the sweep
      double pmin = piv;   // min_j L_jj = sqrt(min_j p_j)
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        double lc[16];
#pragma unroll
        for (int c = j + 1; c < 16; ++c) lc[c] = readlane_d(a[j], c);  // D_cj, c > j (lower: lane c, column j)
        if (!(piv > 0.0) && firstbad < 0) firstbad = j;
        pmin = fmin(pmin, piv);
        if (r == j) mypiv = piv;
        const double rj = rinv;
        if (j + 1 < 16) {
          const double dn = readlane_d(a[j + 1], j + 1);
          piv = fma(-(lc[j + 1] * rj), lc[j + 1], dn);
          rinv = rcp_nr(piv);
        }
        const double t = a[j] * rj;
#pragma unroll
        for (int c = j + 1; c < 16; ++c) a[c] = fma(-t, lc[c], a[c]);
      }
      P64_STAMP(23 + 3 * kb);
      {  // column scales: lane j forms p_j^-1/2, broadcast back per column
        const double rlv = rsqrt_nr(mypiv);
        mind = fmin(mind, pmin * rsqrt_nr(pmin));
#pragma unroll
        for (int j = 0; j < 16; ++j) a[j] *= readlane_d(rlv, j);
      }
      if (lane < 32) {  // lanes 0-15: L16 row r -> S; lanes 16-31: L16^-T row r -> ET (one store stream)
        double* dst = (lane < 16) ? S + (o + r) * P64_SP + o : sm.ET[kb] + r * P64_EP;
#pragma unroll
        for (int c = 0; c < 16; c += 2) {
          f64x2 v;
          v[0] = (lane >= 16 || c <= r) ? a[c] : 0.0;
          v[1] = (lane >= 16 || c + 1 <= r) ? a[c + 1] : 0.0;
          *reinterpret_cast<f64x2*>(dst + c) = v;
        }
      }
      P64_STAMP(24 + 3 * kb);
      if (firstbad >= 0) {
        if (lane == 0) atomicCAS(&ctrl->chol_info, 0, base + o + firstbad + 1);
        sm.fail = 1;
      }
    } else if (w <= kb) {
      const int j = w - 1;
#pragma unroll
      for (int m = j; m < kb; ++m)
        T = mfma16_ab(T, S + o * P64_SP + 16 * m, P64_SP, X + 16 * m * P64_SP + 16 * j, P64_SP, 1.0, lane);
    }
    P64_STAMP(2 + 4 * kb);
    __syncthreads();
    P64_STAMP(3 + 4 * kb);
    if (sm.fail) return false;  // uniform: every wave reads the same flag after the barrier
    // ---- T: X_kb,j = -L16^-1 T (waves 1..kb) / panel TRSM L_ib,kb = A_ib,kb L16^-T (waves kb+1..3) --------
    const double* ET = sm.ET[kb];
    if (w == 0) {  // the L^-1 diagonal block is the transpose of L16^-T: X[o+c][o+r] = ET[r][c]
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int e = lane + 64 * i, rr = e >> 4, cc = e & 15;
        X[(o + cc) * P64_SP + o + rr] = ET[rr * P64_EP + cc];
      }
    } else if (w <= kb) {
      const int j = w - 1;
      d4f acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s = 0; s < 4; ++s)  // A = L16^-1 (row r = column r of ET), B slab s = T register s
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-ET[(4 * s + (lane >> 4)) * P64_EP + (lane & 15)], T[s], acc, 0, 0,
                                                   0);
      c16_store(X + o * P64_SP + 16 * j, P64_SP, acc, lane);
    } else if (w > kb) {
      const int ib = w;
      d4f acc = {0.0, 0.0, 0.0, 0.0};
      acc = mfma16_ab(acc, S + 16 * ib * P64_SP + o, P64_SP, ET, P64_EP, 1.0, lane);
      c16_store(S + 16 * ib * P64_SP + o, P64_SP, acc, lane);
    }
    P64_STAMP(4 + 4 * kb);
    __syncthreads();
    if (lflag && w == 3) {  // publish row-block kb of L^-1 (final after the T phase)
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int e = lane + 64 * q, rr = o + (e >> 5), cc = 2 * (e & 31);
        mI.st2(rr * NB + cc, *reinterpret_cast<const f64x2*>(X + rr * P64_SP + cc));
      }
    }
    // ---- U: A_ib,jb -= L_ib,kb L_jb,kb^T, kb < jb <= ib; wave 0 takes the next diagonal block ------------
    if (kb < 3) {
      int idx = 0;
#pragma unroll
      for (int jb = kb + 1; jb < 4; ++jb)
#pragma unroll
        for (int ib = jb; ib < 4; ++ib) {
          const bool next_diag = (ib == kb + 1 && jb == kb + 1);
          const int owner = next_diag ? 0 : 1 + (idx++ % 3);
          if (w == owner) {
            double* C = S + 16 * ib * P64_SP + 16 * jb;
            d4f acc = c16_load(C, P64_SP, lane);
            acc = mfma16_abt(acc, S + 16 * ib * P64_SP + o, P64_SP, S + 16 * jb * P64_SP + o, P64_SP, -1.0, lane);
            c16_store(C, P64_SP, acc, lane);
          }
        }
    }
    if (lflag && w == 3) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_store(lflag, kb + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (pub_stamp && lane == 0 && kb == 3) *pub_stamp = __builtin_amdgcn_s_memrealtime();  // trace only
    }
    P64_STAMP(5 + 4 * kb);
  }
  __syncthreads();
  P64_STAMP(20);
  if (!fix()) return false;  // (uniform)
  __syncthreads();
  // ---- outputs: Linv = L^-1 (unless published progressively), w = L^-1 b (4 threads per rhs entry) --------
  if (!lflag) {
    for (int t = tid; t < NB * NB / 2; t += 256) {
      const int r = t >> 5, c = 2 * (t & 31);
      mI.st2(r * NB + c, *reinterpret_cast<const f64x2*>(X + r * P64_SP + c));
    }
  }
  for (int t0 = 0; t0 < NB * nrhs * 4; t0 += 256) {
    const int t = t0 + tid, q = t & 3, e = t >> 2;
    const int r = e / nrhs, rho = e - r * nrhs;
    double s = 0.0;
    if (e < NB * nrhs) {
      const int c0 = 16 * q, cend = min(c0 + 16, (r | 15) + 1);  // X is zero beyond the diagonal block of row r
      for (int c = c0; c < cend; ++c) s = fma(X[r * P64_SP + c], sm.B[c * nrhs + rho], s);
    }
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    if (q == 0 && e < NB * nrhs) {
      mR.st(e, s);
      sm.W[e] = s;
    }
  }
  if (tid == 0) atomic_min_pos(&ctrl->min_diag, mind);  // the pivots are wave-uniform on wave 0
  P64_STAMP(21);
  return true;
}

// Store the factored diagonal tile L_kk (lower triangle) from sm.S (after potrf64_factor).
template <class M>
__device__ __forceinline__ void potrf64_store_L(double* __restrict__ L, int ld, int k, const Potrf64Smem& sm) {
  const M mL(L + (size_t)k * NB * ld + (size_t)k * NB, tile_bytes(ld));
  for (int t = threadIdx.x; t < NB * NB / 2; t += 256) {
    const int r = t >> 5, c = 2 * (t & 31);
    const f64x2 l = *reinterpret_cast<const f64x2*>(sm.S + r * P64_SP + c);
    if (c + 1 <= r) mL.st2(r * ld + c, l);
    else if (c <= r) mL.st(r * ld + c, l[0]);
  }
}

// Factor block k of L (lower part of the 64x64 diagonal block), write L_kk, Linv[k] = L_kk^-1 and the
// forward-solved rhs block.  Returns false (uniformly) on a non-positive pivot, after recording the
// 1-based global pivot index in ctrl->chol_info.  Needs blockDim.x == 256.
template <class M>
__device__ bool potrf64(double* __restrict__ L, int ld, int k, double* __restrict__ rhs, int nrhs,
                        double* __restrict__ Linv, DevCtrl* ctrl, Potrf64Smem& sm) {
  potrf64_stage_tile<M>(L, ld, (size_t)k * NB * ld + (size_t)k * NB, sm);
  potrf64_stage_rhs<M>(rhs, k, nrhs, sm);
  if (!potrf64_factor<M>(L, ld, k, rhs, nrhs, Linv, ctrl, sm)) return false;
  potrf64_store_L<M>(L, ld, k, sm);
  return true;
}

}  // namespace cvxg
