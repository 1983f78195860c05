// potrf64w_dpp.hpp (measured and rejected in round 5, microbench A/B only) — the 64 x 64 diagonal-block Cholesky (dpotrf 'L' semantics, MatrixUtils.scala:452-461) with the
// block inverse L^-1 and the fused forward solve, wave-specialised for latency: wave 0 runs only the critical path,
// waves 1..3 everything else, synchronised through LDS flags instead of workgroup barriers.
//
// The block is 4 x 4 tiles of 16.  Step kb:
//   wave 0   the column sweep of block column kb (p64w_sweep): every lane-row of 16 lanes holds a copy of D_kb, row r
//            in lane r, so the column D_cj of each elimination step is one DPP row_newbcast:c away and rides in the
//            update instruction itself (v_fmac_f64_dpp, no v_readlane); the same column operations act on a second
//            register row: the identity border in lane-row 0 (-> L16^-T without its column scales) and the panel
//            tiles A_kb+1..3,kb in lane-rows 1..3 (-> the panel L_ib,kb = A_ib,kb L16^-T, the TRSM, in the same
//            instructions).  -> S(kb,kb), ET[kb], SV[kb], S(ib,kb); flag fP = kb + 1
//            U   D_kb+1 -= L_kb+1,kb L_kb+1,kb^T (4 MFMAs), behind cntU[kb-1] == 3
//   waves 1..3, behind fP(kb) and all of step kb-1 (cntU[kb-1] == 3):
//            C   the updates of block column kb+1 below the diagonal (what the next sweep reads); cntC[kb] += 1
//            A   row kb of L^-1 (X_kb,j = -L16^-1 sum_m L_kb,m X_m,j and the transposed diagonal block); cntT[kb] += 1
//            B   the other trailing updates except the next diagonal block; cntU[kb] += 1
// Wave 0 starts sweep kb + 1 once cntC[kb] == 3.  All flag waits are bounded; a failed pivot or a timeout raises
// sm.fail and every wave leaves at its next wait.
//
// Round 4's form (microbench/potrf64w_r04.hpp) eliminated one lane per row with 2 (15 - j) v_readlane broadcasts per
// column (~44 cycles each) and formed the panel tiles as MFMA products with L16^-T afterwards (wave 0's T).  The
// pivots, L16 and L16^-T are bitwise those of that sweep (the same fma per entry); the panel tiles come from the
// column operations instead of the MFMA product, so they round differently.
#pragma once
#include <utility>

#include "potrf64.hpp"

namespace cvxg {

#ifndef PUBLISH_ONLY
#define PUBLISH_ONLY (reinterpret_cast<int*>(1))  // lflag: store the L^-1 row-blocks progressively, raise no flag
#endif

struct Potrf64wSmem {
  double S[NB * P64_SP];      // the tile: A -> L (lower blocks)
  double X[NB * P64_SP];      // L^-1 (lower blocks)
  double ET[4][16 * P64_EP];  // per step: L16^-T without its column scales (row r = column r of L16^-1 / s_r)
  double SV[4][16];           // per step: the column scales s_j = p_j^-1/2 of L16 (L16 = L~16 diag(s))
  double B[NB * MAX_RHS];     // rhs block, row-major [64][nrhs]
  double W[NB * MAX_RHS];     // forward-solved rhs block w = L^-1 b
  int fail;
  int fP;                     // wave 0: steps whose sweep (diagonal block, L16^-T, scales, panel tiles) is published
  int cntC[4], cntT[4], cntU[4];  // waves 1..3 done with phase C / A / B of step kb
};

__device__ __forceinline__ int p64w_load(const int* f) {
  return __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void p64w_publish(int* f, int v) {  // one lane, after this wave's LDS writes
  __hip_atomic_store(f, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void p64w_add(int* f) { __hip_atomic_fetch_add(f, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP); }

// Wait (whole wave) until *f >= want.  False when the factorization failed or after ~2^20 polls (raises sm.fail = 2).
__device__ __forceinline__ bool p64w_wait(Potrf64wSmem& sm, const int* f, int want) {
  for (unsigned spins = 0;; ++spins) {
    if (p64w_load(f) >= want) return true;
    if (__hip_atomic_load(&sm.fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return false;
    if (spins > (1u << 20)) {
      __hip_atomic_store(&sm.fail, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// Stage the tile / rhs (as potrf64_stage_*), reset the flags; caller syncs.
template <class M>
__device__ __forceinline__ void potrf64w_stage(const double* L, int ld, size_t off, const double* rhs, int k, int nrhs,
                                               Potrf64wSmem& sm) {
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
    *reinterpret_cast<f64x2*>(sm.S + (idx >> 5) * P64_SP + 2 * (idx & 31)) = v[q];
  }
  const M mR(const_cast<double*>(rhs) + (size_t)k * NB * nrhs, (unsigned)(NB * nrhs) * 8u);
  for (int t = tid; t < NB * nrhs; t += 256) sm.B[t] = mR.ld(t);
}

// 16 x 16 block ops on LDS operands (one wave)
__device__ __forceinline__ void p64w_U(Potrf64wSmem& sm, int ib, int jb, int kb, int lane) {  // A_ib,jb -= L_ib,kb L_jb,kb'
  double* C = sm.S + 16 * ib * P64_SP + 16 * jb;
  d4f acc = c16_load(C, P64_SP, lane);
  acc = mfma16_abt(acc, sm.S + 16 * ib * P64_SP + 16 * kb, P64_SP, sm.S + 16 * jb * P64_SP + 16 * kb, P64_SP, -1.0,
                   lane);
  c16_store(C, P64_SP, acc, lane);
}
__device__ __forceinline__ void p64w_X(Potrf64wSmem& sm, int kb, int j, int lane) {  // X_kb,j, j < kb
  d4f T = {0.0, 0.0, 0.0, 0.0};
  for (int m = j; m < kb; ++m)
    T = mfma16_ab(T, sm.S + 16 * kb * P64_SP + 16 * m, P64_SP, sm.X + 16 * m * P64_SP + 16 * j, P64_SP, 1.0, lane);
  const double* ET = sm.ET[kb];
  d4f acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int s = 0; s < 4; ++s)  // A = L16^-1 / s_row (row r = column r of ET), B slab s = T register s
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-ET[(4 * s + (lane >> 4)) * P64_EP + (lane & 15)], T[s], acc, 0, 0, 0);
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] *= sm.SV[kb][(lane >> 4) + 4 * i];  // row scales (C layout: row (lane>>4) + 4i)
  c16_store(sm.X + 16 * kb * P64_SP + 16 * j, P64_SP, acc, lane);
}
// X_kb,kb = (L16^-T)' with the column scales, and the scales of the L16 block of S (L16 = L~16 diag(s))
__device__ __forceinline__ void p64w_Xdiag(Potrf64wSmem& sm, int kb, int lane) {
  const double* ET = sm.ET[kb];
  const double* sv = sm.SV[kb];
  const int o = 16 * kb;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e = lane + 64 * i, rr = e >> 4, cc = e & 15;
    sm.X[(o + cc) * P64_SP + o + rr] = ET[rr * P64_EP + cc] * sv[cc];
    double* sd = sm.S + (o + rr) * P64_SP + o + cc;
    *sd = (cc <= rr) ? *sd * sv[cc] : 0.0;
  }
}

// ---- wave 0's column sweep ---------------------------------------------------------------------------------------
// dst += bcast_C(src) * m, bcast_C = DPP row_newbcast:C (lane C of each row of 16 lanes; 64-bit DPP, gfx90a+).  The
// DPP source is read two or more instructions after its last write (the step below keeps it so; the explicit s_nop
// covers the one read right behind a write).
template <int C>
__device__ __forceinline__ void p64w_fmac_bc(double& dst, double src, double m) {
  asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
               : "+v"(dst)
               : "v"(src), "v"(m), "i"(C));
}
template <int C>
__device__ __forceinline__ double p64w_bc(double src) {
  double d;
  asm volatile("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf"
               : "=v"(d)
               : "v"(src), "i"(C));
  return d;
}
// the updates of column J beyond the next pivot's: c = J + 2 .. 15
template <int J, int... Cs>
__device__ __forceinline__ void p64w_rest(double (&a)[16], double (&b)[16], double nta, double ntb,
                                          std::integer_sequence<int, Cs...>) {
  ((p64w_fmac_bc<J + 2 + Cs>(a[J + 2 + Cs], a[J], nta), p64w_fmac_bc<J + 2 + Cs>(b[J + 2 + Cs], a[J], ntb)), ...);
}
// Column J of the sweep: for c > J, a[c] += D_cJ (-a[J] / p_J) and b[c] += D_cJ (-b[J] / p_J) with D_cJ = lane c's a[J];
// the next pivot p_J+1 = lane J+1's a[J+1] right after its update, its reciprocal beside the remaining updates.  Per
// entry the fma of the round-4 v_readlane sweep: fma(D_cJ, -(a[J] r_J), a[c]).
template <int J>
__device__ __forceinline__ void p64w_step(double (&a)[16], double (&b)[16], double& piv, double& rinv,
                                          double (&pv)[16], double& pmin, int& firstbad) {
  if constexpr (J < 16) {
    if (!(piv > 0.0) && firstbad < 0) firstbad = J;
    pmin = fmin(pmin, piv);
    pv[J] = piv;
    const double nta = -(a[J] * rinv), ntb = -(b[J] * rinv);
    if constexpr (J + 1 < 16) {
      p64w_fmac_bc<J + 1>(a[J + 1], a[J], nta);
      p64w_fmac_bc<J + 1>(b[J + 1], a[J], ntb);
      piv = p64w_bc<J + 1>(a[J + 1]);
      rinv = rcp_nr(piv);
    }
    p64w_rest<J>(a, b, nta, ntb, std::make_integer_sequence<int, (J + 2 < 16 ? 14 - J : 0)>{});
    p64w_step<J + 1>(a, b, piv, rinv, pv, pmin, firstbad);
  }
}

// wave 0: the sweep of block column kb (D_kb and the panel tiles below it with every panel < kb applied) -> L~16 into
// S(kb,kb) and L~16^-T into ET[kb] without their column scales, the scales s_j = p_j^-1/2 into SV[kb] (the consumers
// scale: p64w_X, p64w_Xdiag), the panel tiles L_ib,kb (scaled) into S(ib,kb).  Returns false on a non-positive pivot
// (chol_info recorded) or, with early_min > 0, on a block min diag(L) <= early_min (min_diag / small_piv recorded).
__device__ __forceinline__ bool p64w_sweep(Potrf64wSmem& sm, int kb, int base, DevCtrl* ctrl, double& mind, int lane,
                                           double early_min) {
  const int o = 16 * kb, r = lane & 15, g = lane >> 4;
  const int ib = kb + g;
  const bool pan = g > 0 && ib <= 3;
  double a[16], b[16];
  {
    const double* src = sm.S + (o + r) * P64_SP + o;
    const double* bsrc = sm.S + (16 * (pan ? ib : kb) + r) * P64_SP + o;
#pragma unroll
    for (int c = 0; c < 16; c += 2) {
      const f64x2 v = *reinterpret_cast<const f64x2*>(src + c);
      const f64x2 u = *reinterpret_cast<const f64x2*>(bsrc + c);
      a[c] = (c <= r) ? v[0] : 0.0;
      a[c + 1] = (c + 1 <= r) ? v[1] : 0.0;
      b[c] = pan ? u[0] : ((g == 0 && c == r) ? 1.0 : 0.0);
      b[c + 1] = pan ? u[1] : ((g == 0 && c + 1 == r) ? 1.0 : 0.0);
    }
  }
  int firstbad = -1;
  double pv[16];
  double piv = p64w_bc<0>(a[0]);
  double rinv = rcp_nr(piv);
  double pmin = piv;
  p64w_step<0>(a, b, piv, rinv, pv, pmin, firstbad);
  double sv[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) sv[c] = rsqrt_nr(pv[c]);
  const double bmin = pmin * rsqrt_nr(pmin);  // this block's min diag(L) (the value min_diag would take)
  mind = fmin(mind, bmin);
  {
    double myv = sv[0];
#pragma unroll
    for (int c = 1; c < 16; ++c) myv = (r == c) ? sv[c] : myv;
    if (lane < 16) sm.SV[kb][r] = myv;
  }
  if (g == 0) {
    double* ds = sm.S + (o + r) * P64_SP + o;
    double* de = sm.ET[kb] + r * P64_EP;
#pragma unroll
    for (int c = 0; c < 16; c += 2) {
      f64x2 v, e;
      v[0] = (c <= r) ? a[c] : 0.0;
      v[1] = (c + 1 <= r) ? a[c + 1] : 0.0;
      e[0] = b[c];
      e[1] = b[c + 1];
      *reinterpret_cast<f64x2*>(ds + c) = v;
      *reinterpret_cast<f64x2*>(de + c) = e;
    }
  } else if (pan) {
    double* dp = sm.S + (16 * ib + r) * P64_SP + o;
#pragma unroll
    for (int c = 0; c < 16; c += 2) {
      f64x2 v;
      v[0] = b[c] * sv[c];
      v[1] = b[c + 1] * sv[c + 1];
      *reinterpret_cast<f64x2*>(dp + c) = v;
    }
  }
  if (firstbad >= 0) {
    if (lane == 0) atomicCAS(&ctrl->chol_info, 0, base + o + firstbad + 1);
    return false;
  }
  // regularizedCholesky's first attempt (MatrixUtils.scala:458-460): once some diag(L) <= 1e-7 the factor is discarded
  // and chol(Q + 1e-10 I) taken instead, so the rest of this factorization cannot matter -- stop here.  The test is on
  // the same value min_diag accumulates, so the host's decision (min_diag <= 1e-7) is the one the full attempt gives.
  if (early_min > 0.0 && !(bmin > early_min)) {
    if (lane == 0) {
      atomic_min_pos(&ctrl->min_diag, bmin);
      atomicCAS(&ctrl->small_piv, 0, base + o + 1);
    }
    return false;
  }
  return true;
}

// Phase C / A / B work of waves 1..3 at step kb (static assignment, see the header).
__device__ __forceinline__ void p64w_phaseC(Potrf64wSmem& sm, int kb, int w, int lane) {  // block column kb + 1
  if (kb == 0) {
    if (w == 1) p64w_U(sm, 2, 1, 0, lane);
    if (w == 2) p64w_U(sm, 3, 1, 0, lane);
  } else if (kb == 1) {
    if (w == 1) p64w_U(sm, 3, 2, 1, lane);
  }
}
__device__ __forceinline__ void p64w_phaseA(Potrf64wSmem& sm, int kb, int w, int lane) {
  if (kb == 0) {
    if (w == 3) p64w_Xdiag(sm, 0, lane);
  } else if (kb == 1) {
    if (w == 2) p64w_X(sm, 1, 0, lane);
    if (w == 3) p64w_Xdiag(sm, 1, lane);
  } else if (kb == 2) {
    if (w == 1) p64w_X(sm, 2, 0, lane);
    if (w == 2) p64w_X(sm, 2, 1, lane);
    if (w == 3) p64w_Xdiag(sm, 2, lane);
  } else {
    if (w == 1) p64w_X(sm, 3, 0, lane);
    if (w == 2) p64w_X(sm, 3, 1, lane);
    if (w == 3) {
      p64w_X(sm, 3, 2, lane);
      p64w_Xdiag(sm, 3, lane);
    }
  }
}
__device__ __forceinline__ void p64w_phaseB(Potrf64wSmem& sm, int kb, int w, int lane) {
  if (kb == 0) {
    if (w == 1) p64w_U(sm, 2, 2, 0, lane);
    if (w == 2) p64w_U(sm, 3, 2, 0, lane);
    if (w == 3) p64w_U(sm, 3, 3, 0, lane);
  } else if (kb == 1) {
    if (w == 1) p64w_U(sm, 3, 3, 1, lane);
  }
}

// The factorization of block k: tile staged in sm.S, rhs block in sm.B, flags reset (potrf64w_reset), a barrier
// behind.  On return (uniformly true / false) sm.X = L^-1 (exact zeros above the diagonal), sm.W = w = L^-1 b (also
// stored to rhs block k); Linv[k] = L^-1 is stored row-block by row-block as it becomes final (wave 3), and *lflag
// (when given) counts the stored row-blocks (sc1 hand-off: the stores drained first).  fix() runs on all threads
// between the factorization and the forward solve (barrier behind it).  L_kk is not stored (potrf64w_store_L).
template <class M, class Fix = NoFix>
__device__ __forceinline__ bool potrf64w_factor(int k, double* __restrict__ rhs, int nrhs, double* __restrict__ Linv,
                                                DevCtrl* ctrl, Potrf64wSmem& sm, int* lflag = nullptr,
                                                Fix fix = Fix(), double early_min = 0.0) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int base = k * NB;
  const M mI(Linv + (size_t)k * NB * NB, (unsigned)(NB * NB) * 8u);  // Linv[k]
  double mind = __builtin_inf();
  bool ok = true;
  if (w == 0) {
#pragma unroll 1
    for (int kb = 0; kb < 4 && ok; ++kb) {
      if (kb >= 1 && !p64w_wait(sm, &sm.cntC[kb - 1], 3)) {  // block column kb carries panel kb - 1
        ok = false;
        break;
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      P64_STAMP(1 + 4 * kb);
      ok = p64w_sweep(sm, kb, base, ctrl, mind, lane, early_min);
      P64_STAMP(2 + 4 * kb);
      if (!ok) {
        if (lane == 0) __hip_atomic_store(&sm.fail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        break;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) p64w_publish(&sm.fP, kb + 1);
      if (kb < 3) {
        if (kb >= 1 && !p64w_wait(sm, &sm.cntU[kb - 1], 3)) {  // D_kb+1 carries every panel < kb
          ok = false;
          break;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        P64_STAMP(3 + 4 * kb);
        p64w_U(sm, kb + 1, kb + 1, kb, lane);
        P64_STAMP(4 + 4 * kb);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // the next sweep reads this wave's U result
      }
    }
  } else {
#pragma unroll 1
    for (int kb = 0; kb < 4 && ok; ++kb) {
      ok = p64w_wait(sm, &sm.fP, kb + 1) && (kb == 0 || p64w_wait(sm, &sm.cntU[kb - 1], 3));
      if (!ok) break;
      P64_STAMP(1 + 4 * kb);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      p64w_phaseC(sm, kb, w, lane);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) p64w_add(&sm.cntC[kb]);
      p64w_phaseA(sm, kb, w, lane);
      P64_STAMP(2 + 4 * kb);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) p64w_add(&sm.cntT[kb]);
      if (lflag && w == 3) {  // row-block kb of L^-1 is final once every wave's phase A is
        if (!p64w_wait(sm, &sm.cntT[kb], 3)) {
          ok = false;
          break;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int e = lane + 64 * q, rr = 16 * kb + (e >> 5), cc = 2 * (e & 31);
          mI.st2(rr * NB + cc, *reinterpret_cast<const f64x2*>(sm.X + rr * P64_SP + cc));
        }
        if (lflag != PUBLISH_ONLY) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          if (lane == 0) __hip_atomic_store(lflag, kb + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      P64_STAMP(3 + 4 * kb);
      p64w_phaseB(sm, kb, w, lane);
      P64_STAMP(4 + 4 * kb);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) p64w_add(&sm.cntU[kb]);
    }
  }
  P64_STAMP(17);
  __syncthreads();
  P64_STAMP(18);
  if (sm.fail) return false;  // uniform after the barrier
  if (!fix()) return false;   // (uniform)
  __syncthreads();
  // ---- outputs: Linv (unless stored progressively), w = L^-1 b (4 threads per rhs entry) ----
  const M mR(rhs + (size_t)base * nrhs, (unsigned)(NB * nrhs) * 8u);  // rhs block k
  if (!lflag) {
    for (int t = tid; t < NB * NB / 2; t += 256) {
      const int r = t >> 5, c = 2 * (t & 31);
      mI.st2(r * NB + c, *reinterpret_cast<const f64x2*>(sm.X + r * P64_SP + c));
    }
  }
  for (int t0 = 0; t0 < NB * nrhs * 4; t0 += 256) {
    const int t = t0 + tid, q = t & 3, e = t >> 2;
    const int r = e / nrhs, rho = e - r * nrhs;
    double s = 0.0;
    if (e < NB * nrhs) {
      const int c0 = 16 * q, cend = min(c0 + 16, (r | 15) + 1);  // X is zero beyond the diagonal block of row r
      for (int c = c0; c < cend; ++c) s = fma(sm.X[r * P64_SP + c], sm.B[c * nrhs + rho], s);
    }
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    if (q == 0 && e < NB * nrhs) {
      mR.st(e, s);
      sm.W[e] = s;
    }
  }
  if (tid == 0) atomic_min_pos(&ctrl->min_diag, mind);  // the pivots are wave-uniform on wave 0
  P64_STAMP(19);
  return true;
}

// Before potrf64w_factor: zero the upper blocks of L^-1 (read by callers' MFMAs) and the flags (a barrier must
// follow).
__device__ __forceinline__ void potrf64w_reset(Potrf64wSmem& sm) {
  const int tid = threadIdx.x;
  for (int t = tid; t < 6 * 256; t += 256) {
    const int b = t >> 8, e = t & 255;
    const int ib = (b < 3) ? 0 : ((b < 5) ? 1 : 2), jb = (b < 3) ? 1 + b : ((b < 5) ? b - 1 : 3);
    sm.X[(16 * ib + (e >> 4)) * P64_SP + 16 * jb + (e & 15)] = 0.0;
  }
  if (tid < 4) {
    sm.cntC[tid] = 0;
    sm.cntT[tid] = 0;
    sm.cntU[tid] = 0;
  }
  if (tid == 0) {
    sm.fail = 0;
    sm.fP = 0;
  }
}

// Store the factored diagonal tile L_kk (lower triangle) from sm.S.
template <class M>
__device__ __forceinline__ void potrf64w_store_L(double* __restrict__ L, int ld, int k, const Potrf64wSmem& sm) {
  const M mL(L + (size_t)k * NB * ld + (size_t)k * NB, tile_bytes(ld));
  for (int t = threadIdx.x; t < NB * NB / 2; t += 256) {
    const int r = t >> 5, c = 2 * (t & 31);
    const f64x2 l = *reinterpret_cast<const f64x2*>(sm.S + r * P64_SP + c);
    if (c + 1 <= r) mL.st2(r * ld + c, l);
    else if (c <= r) mL.st(r * ld + c, l[0]);
  }
}

}  // namespace cvxg
