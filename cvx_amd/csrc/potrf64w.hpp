// potrf64w.hpp — the 64 x 64 diagonal-block Cholesky (dpotrf 'L' semantics, MatrixUtils.scala:452-461) with the
// block inverse L^-1 and the fused forward solve, wave-specialised for latency: wave 0 runs only the critical path,
// waves 1..3 everything else, synchronised through LDS flags instead of workgroup barriers.
//
// The block is 4 x 4 tiles of 16.  Step kb:
//   wave 0   P   eliminates D_kb (one lane per row, the identity border beside it: L16 and L16^-T in one sweep, the
//                column scales p_j^-1/2 applied as each column finishes) -> S(kb,kb), ET[kb]; flag fP = kb + 1
//            T   L_kb+1,kb = A_kb+1,kb L16^-T (4 MFMAs) -> S(kb+1,kb); flag fT = kb + 1
//            U   D_kb+1 -= L_kb+1,kb L_kb+1,kb^T (4 MFMAs) -> S(kb+1,kb+1), the next diagonal block
//   waves 1..3, behind fP(kb) and all of step kb-1 (cntU[kb-1] == 3):
//            A   the other panel tiles L_ib,kb (ib >= kb+2), row kb of L^-1 (X_kb,j = -L16^-1 sum_m L_kb,m X_m,j and
//                the transposed diagonal block); cntT[kb] += 1
//            B   behind fT(kb) and cntT[kb] == 3: the trailing updates except the next diagonal block; cntU[kb] += 1
// Wave 0 waits only for cntU[kb-1] == 3 (A_kb+1,kb and D_kb+1 carry every panel < kb) between its P and T of step
// kb, i.e. while it eliminated D_kb the other waves finished step kb-1.  All flag waits are bounded; a failed pivot
// or a timeout raises sm.fail and every wave leaves at its next wait.
//
// Against potrf64.hpp (two workgroup barriers per step, the column scales as a separate pass, T and U phases
// shared by all waves between the barriers) the chain of wave 0 per step is the sweep, 8 MFMAs and two LDS round
// trips.
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
  int fP, fT;                 // wave 0: steps whose P / T are published
  int cntT[4], cntU[4];       // waves 1..3 done with phase A / B of step kb
  int cntD;                   // (wait_d) waves 1..3 done storing their blocks of the staged tile
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
__device__ __forceinline__ void p64w_T(Potrf64wSmem& sm, int ib, int kb, int lane) {  // L_ib,kb = A_ib,kb L16^-T
  double* C = sm.S + 16 * ib * P64_SP + 16 * kb;
  d4f acc = {0.0, 0.0, 0.0, 0.0};
  acc = mfma16_ab(acc, C, P64_SP, sm.ET[kb], P64_EP, 1.0, lane);
  acc *= sm.SV[kb][lane & 15];  // the column scales of L16^-T (C layout: column = lane & 15)
  c16_store(C, P64_SP, acc, lane);
}
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
    const double x = ET[rr * P64_EP + cc] * sv[cc];
    sm.X[(o + cc) * P64_SP + o + rr] = x;
    double* sd = sm.S + (o + rr) * P64_SP + o + cc;
    *sd = (cc <= rr) ? *sd * sv[cc] : 0.0;
  }
}

// wave 0: eliminate D_kb (S diagonal block kb, all panels < kb applied) -> L~16 into S, L~16^-T into ET[kb], the column
// scales s_j = p_j^-1/2 into SV[kb] (L16 = L~16 diag(s)).  Returns false on a non-positive pivot (chol_info recorded) or
// an early stop.  Every lane-row of 16 lanes holds a copy of D_kb (row r in lane r), so D_cj is one DPP row_newbcast:c
// away and rides in v_fmac_f64_dpp (64-bit DPP, gfx90a+); the identity border beside it (-> L~16^-T) is a second
// register row of lane-row 0.  (Round 5: bitwise equal to the v_readlane sweep it replaced, 3 170 vs 4 500 cycles.)
// (microbench/sweep_dpp.hip: 3 600 cycles per 16 columns with 48 panel rows riding along.)
template <int C>
__device__ __forceinline__ void p64w_fmac_bc(double& dst, double src, double m) {
  asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(dst) : "v"(src), "v"(m), "i"(C));
}
template <int C>
__device__ __forceinline__ double p64w_bc(double src) {
  double d;
  asm volatile("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "=v"(d) : "v"(src), "i"(C));
  return d;
}
template <int J, int... Cs>
__device__ __forceinline__ void p64w_rest(double (&a)[16], double (&b)[16], double nta, double ntb,
                                          std::integer_sequence<int, Cs...>) {
  ((p64w_fmac_bc<J + 2 + Cs>(a[J + 2 + Cs], a[J], nta), p64w_fmac_bc<J + 2 + Cs>(b[J + 2 + Cs], a[J], ntb)), ...);
}
// (the per-column bookkeeping stays off wave-uniform branches: the minimum pivot is one v_min_f64 per column -- IEEE
// minNum, as fmin for the quiet values a pivot can take -- and the first bad pivot is found after the sweep from the
// pivots the lanes keep, by one ballot)
__device__ __forceinline__ double p64w_vmin(double x, double y) {
  double r;
  asm volatile("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
  return r;
}
template <int J>
__device__ __forceinline__ void p64w_dstep(double (&a)[16], double (&b)[16], double& piv, double& rinv, double& mypiv,
                                           int r, double& pmin, int& firstbad) {
  if constexpr (J < 16) {
    pmin = fmin(pmin, piv);
    if (r == J) mypiv = piv;
    const double nta = -(a[J] * rinv), ntb = -(b[J] * rinv);
    if constexpr (J + 1 < 16) {
      p64w_fmac_bc<J + 1>(a[J + 1], a[J], nta);
      p64w_fmac_bc<J + 1>(b[J + 1], a[J], ntb);
      piv = p64w_bc<J + 1>(a[J + 1]);
      rinv = rcp_nr(piv);
    }
    p64w_rest<J>(a, b, nta, ntb, std::make_integer_sequence<int, (J + 2 < 16 ? 14 - J : 0)>{});
    p64w_dstep<J + 1>(a, b, piv, rinv, mypiv, r, pmin, firstbad);
  }
}
__device__ __forceinline__ bool p64w_eliminate_dpp(Potrf64wSmem& sm, int kb, int base, DevCtrl* ctrl, double& mind,
                                                   int lane, double early_min) {
  const int o = 16 * kb, r = lane & 15, g = lane >> 4;
  // The row's entries above the diagonal (c > r) are loaded as they are and never masked: they only ever feed other
  // entries above the diagonal (lane r's multiplier for column j > r is its own a[j], c > j > r), never a pivot, an
  // entry on or below the diagonal, or a broadcast (lane c's a[j], j < c), and the stores below keep c <= r only.
  double a[16], b[16];
  {
    const double* src = sm.S + (o + r) * P64_SP + o;
#pragma unroll
    for (int c = 0; c < 16; c += 2) {
      const f64x2 v = *reinterpret_cast<const f64x2*>(src + c);
      a[c] = v[0];
      a[c + 1] = v[1];
      b[c] = (g == 0 && c == r) ? 1.0 : 0.0;
      b[c + 1] = (g == 0 && c + 1 == r) ? 1.0 : 0.0;
    }
  }
  int firstbad = -1;
  double piv = p64w_bc<0>(a[0]);
  double rinv = rcp_nr(piv);
  double pmin = piv;
  double mypiv = 1.0;
  p64w_dstep<0>(a, b, piv, rinv, mypiv, r, pmin, firstbad);
  {  // the first column whose pivot is not > 0 (lane r of lane-row 0 holds p_r)
    const unsigned long long bad = __ballot(!(mypiv > 0.0)) & 0xffffull;
    if (bad) firstbad = __builtin_ctzll(bad);
  }
  const double bmin = pmin * rsqrt_nr(pmin);
  mind = fmin(mind, bmin);
  if (lane < 16) {
    sm.SV[kb][r] = rsqrt_nr(mypiv);
    double* dS = sm.S + (o + r) * P64_SP + o;
    double* dE = sm.ET[kb] + r * P64_EP;
    // (the entries above the diagonal go out as they are: nothing reads the upper part of a diagonal block of S,
    // and potrf64w_store_L keeps c <= r)
#pragma unroll
    for (int c = 0; c < 16; c += 2) {
      *reinterpret_cast<f64x2*>(dS + c) = f64x2{a[c], a[c + 1]};
      *reinterpret_cast<f64x2*>(dE + c) = f64x2{b[c], b[c + 1]};
    }
  }
  if (firstbad >= 0) {
    if (lane == 0) atomicCAS(&ctrl->chol_info, 0, base + o + firstbad + 1);
    return false;
  }
  if (early_min > 0.0 && !(bmin > early_min)) {
    if (lane == 0) {
      atomic_min_pos(&ctrl->min_diag, bmin);
      atomicCAS(&ctrl->small_piv, 0, base + o + 1);
    }
    return false;
  }
  return true;
}

// Phase A / B work of waves 1..3 at step kb (static assignment, see the header).
__device__ __forceinline__ void p64w_phaseA(Potrf64wSmem& sm, int kb, int w, int lane) {
  if (kb == 0) {
    if (w == 1) p64w_T(sm, 2, 0, lane);
    if (w == 2) p64w_T(sm, 3, 0, lane);
    if (w == 3) p64w_Xdiag(sm, 0, lane);
  } else if (kb == 1) {
    if (w == 1) p64w_T(sm, 3, 1, lane);
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
    if (w == 1) {
      p64w_U(sm, 2, 1, 0, lane);
      p64w_U(sm, 3, 3, 0, lane);
    }
    if (w == 2) {
      p64w_U(sm, 3, 1, 0, lane);
      p64w_U(sm, 2, 2, 0, lane);
    }
    if (w == 3) p64w_U(sm, 3, 2, 0, lane);
  } else if (kb == 1) {
    if (w == 1) p64w_U(sm, 3, 2, 1, lane);
    if (w == 2) p64w_U(sm, 3, 3, 1, lane);
  }
}

// The factorization of block k: tile staged in sm.S, rhs block in sm.B, flags reset (potrf64w_reset), a barrier
// behind.  On return (uniformly true / false) sm.X = L^-1 (exact zeros above the diagonal), sm.W = w = L^-1 b (also
// stored to rhs block k); Linv[k] = L^-1 is stored row-block by row-block as it becomes final (wave 3), and *lflag
// (when given) counts the stored row-blocks (sc1 hand-off: the stores drained first).  fix() runs on all threads
// between the factorization and the forward solve (barrier behind it).  L_kk is not stored (potrf64w_store_L).
template <class M, class Fix = NoFix, class Pre = NoPre>
__device__ __forceinline__ bool potrf64w_factor(int k, double* __restrict__ rhs, int nrhs, double* __restrict__ Linv,
                                                DevCtrl* ctrl, Potrf64wSmem& sm, int* lflag = nullptr,
                                                Fix fix = Fix(), double early_min = 0.0, Pre pre = Pre(),
                                                unsigned long long* rb_stamp = nullptr, bool wait_d = false) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int base = k * NB;
  const M mI(Linv + (size_t)k * NB * NB, (unsigned)(NB * NB) * 8u);  // Linv[k]
  double mind = __builtin_inf();
  bool ok = true;
  if (w == 0) {
#pragma unroll 1
    for (int kb = 0; kb < 4 && ok; ++kb) {
      P64_STAMP(1 + 4 * kb);
      ok = p64w_eliminate_dpp(sm, kb, base, ctrl, mind, lane, early_min);
      P64_STAMP(2 + 4 * kb);
      if (!ok) {
        if (lane == 0) __hip_atomic_store(&sm.fail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        break;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) p64w_publish(&sm.fP, kb + 1);
      if (kb < 3) {
        // (wait_d: the caller entered without a barrier behind the staged tile; wave 0 factored its own block D_00
        // and waits here for waves 1..3's blocks before the first T / U)
        if ((kb >= 1 && !p64w_wait(sm, &sm.cntU[kb - 1], 3)) || (kb == 0 && wait_d && !p64w_wait(sm, &sm.cntD, 3))) {
          ok = false;
          break;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        P64_STAMP(3 + 4 * kb);
        p64w_T(sm, kb + 1, kb, lane);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) p64w_publish(&sm.fT, kb + 1);
        p64w_U(sm, kb + 1, kb + 1, kb, lane);
        P64_STAMP(4 + 4 * kb);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // the next sweep reads this wave's U result
      }
    }
  } else {
    pre(w, lane);
#pragma unroll 1
    for (int kb = 0; kb < 4 && ok; ++kb) {
      ok = p64w_wait(sm, &sm.fP, kb + 1) && (kb == 0 ? (!wait_d || p64w_wait(sm, &sm.cntD, 3))
                                                      : p64w_wait(sm, &sm.cntU[kb - 1], 3));
      if (!ok) break;
      P64_STAMP(1 + 4 * kb);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
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
          if (rb_stamp && lane == 0) rb_stamp[kb] = __builtin_amdgcn_s_memrealtime();  // (instrumentation)
        }
      }
      if (kb < 3) {
        ok = p64w_wait(sm, &sm.fT, kb + 1) && p64w_wait(sm, &sm.cntT[kb], 3);
        if (!ok) break;
        P64_STAMP(3 + 4 * kb);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        p64w_phaseB(sm, kb, w, lane);
        P64_STAMP(4 + 4 * kb);
      }
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
    sm.cntT[tid] = 0;
    sm.cntU[tid] = 0;
  }
  if (tid == 0) {
    sm.cntD = 0;
    sm.fail = 0;
    sm.fP = 0;
    sm.fT = 0;
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
