// k_dataflow.hip — the whole regularized-Cholesky factorization (right-looking dpotrf('L'),
// MatrixUtils.scala:452-461) with the fused forward solve, as ONE persistent launch over a tile DAG.
//
// Tiles are 64 x 64 (NB).  Tasks, in an order fixed on the host by list-scheduling the DAG with its
// critical-path priorities (cvxg.cpp, build_chol_schedule):
//   POTRF(k)      factor the diagonal tile, L_kk^-1 into Linv[k], forward-solve rhs block k
//   TRSM(i,k)     L_ik = A_ik L_kk^-T (MFMA, product with L_kk^-1); rhs_i -= L_ik w_k
//   UPDATE(i,j,k) A_ij -= L_ik L_jk^T (MFMA), k < j <= i
// Per lower tile (i,j) one state word counts the operations applied to it: UPDATE(i,j,k) needs
// state(i,j) == k, state(i,k) == state(j,k) == k + 1; POTRF(k) / TRSM(i,k) need state == k (and the
// finished diagonal tile).  Workgroups (one per CU) claim tasks with an atomic counter; a task only waits
// on tasks earlier in the order, so the launch cannot deadlock whatever the residency.  Every wait is
// bounded: on a timeout or a failed pivot the abort word is set and every workgroup drains.
//
// Inter-workgroup hand-off (MI355X_MICROARCH.md, visibility: Valid forms, row 1): every load and store of
// handed-off bytes is an sc1 access (relaxed agent-scope atomics), each storing wave drains with
// s_waitcnt vmcnt(0), a workgroup barrier, then ONE lane stores the state word; the consumer polls the
// word with sc1 loads, then a workgroup barrier, then sc1 loads of the data.  One workgroup per CU.
#include "potrf64w.hpp"

namespace cvxg {


constexpr int DF_SP = NB + 2;  // LDS row stride (doubles) of a staged 64 x 64 operand: conflict-free fragments
constexpr int DF_SMEM = 4 * NB * (NB + 2) + 2 * 16 * (NB + 2) + 512;  // doubles (~142 KB): > half the CU's LDS, so one workgroup per CU

// LDS of the critical-chain workgroup: POTRF's workspace (tile, L^-1, rhs) + the TRSM tile L_k+1,k + L' w_k
struct ChainSmem {
  Potrf64wSmem p;
  double Sa[NB * (NB + 2)];       // A_b,b-1 during the TRSM slices, then L_b,b-1 (for the last rhs correction)
  double E2[2][16 * (NB + 2)];    // double-buffered row-blocks of L_b-1,b-1^-1
  double V[NB * MAX_RHS];
  int lpub;                       // waves of POTRF(b) done storing L_b,b-1 (deferred publication)
};
static_assert(sizeof(ChainSmem) <= DF_SMEM * sizeof(double), "chain workspace exceeds the dataflow LDS");

__device__ __forceinline__ int df_tri(int i, int j) { return i * (i + 1) / 2 + j; }

// Q = (d d') o H (+ reg I), padded part identity — k_form_q's entries (MatrixUtils.scala:267, :454), formed as each
// tile is first read (POTRF(0), the chain's staging of block 1, TRSM(i,0), UPDATE(i,j,0)) instead of by a separate
// pass over the lower triangle.  The same expression in the same order as k_form_q, so the factor is bit-identical.
struct QFold {
  const double* H;  // nullptr: L already holds the matrix to factor
  const double* d;
  int n;
  double reg;
};
__device__ __forceinline__ double qf_entry(const QFold& f, int r, int c, double h) {
  if (r < f.n && c < f.n) {
    double v = (f.d[r] * f.d[c]) * h;
    if (r == c) v += f.reg;
    return v;
  }
  return (r == c) ? 1.0 : 0.0;
}
// a 64 x 64 tile's loads (df_load layout) of Q(r0.., c0..) from H
__device__ __forceinline__ void qf_load(f64x2 (&v)[NB * NB / 512], const QFold& f, int ld, int r0, int c0) {
  const int tid = threadIdx.x;
  const Sc1Mem mH(const_cast<double*>(f.H) + (size_t)r0 * ld + c0, tile_bytes(ld));
#pragma unroll
  for (int q = 0; q < NB * NB / 512; ++q) {
    const int idx = q * 256 + tid;
    v[q] = mH.ld2((idx >> 5) * ld + 2 * (idx & 31));
  }
#pragma unroll
  for (int q = 0; q < NB * NB / 512; ++q) {
    const int idx = q * 256 + tid;
    const int r = r0 + (idx >> 5), c = c0 + 2 * (idx & 31);
    v[q][0] = qf_entry(f, r, c, v[q][0]);
    v[q][1] = qf_entry(f, r, c + 1, v[q][1]);
  }
}

__device__ __forceinline__ int df_poll(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void df_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Thread 0 waits until state[idx] >= want.  Returns false when the launch aborts (failed pivot elsewhere)
// or after SPIN_LIMIT_TICKS of wall time (then it raises the abort word itself with code 2: a scheduling bug, not a
// hang).
__device__ bool df_wait(const int* state, int idx, int want, int* abortw, DevCtrl* ctrl) {
  const unsigned long long t0 = spin_clock();
  for (unsigned spins = 0;; ++spins) {
    if (df_poll(state + idx) >= want) return true;
    if ((spins & 15) == 15 && df_poll(abortw)) return false;
    if (spin_expired(spins, t0)) {
      __hip_atomic_store(abortw, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      atomicExch(&ctrl->df_status, 2);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// Thread 0 waits until p0[0] >= w0, p1[0] >= w1 and p2[0] >= w2 (p2 may be null) -- the worker's dependency test.  The
// polls are loaded together, so a task whose inputs are already final starts after one memory round trip instead of one
// per input; only the words still short are polled again.  Same exits as df_wait (the abort word at the first spin
// that finds an input short, then every 16th).
__device__ bool df_wait3(const int* p0, int w0, const int* p1, int w1, const int* p2, int w2, int* abortw, DevCtrl* ctrl) {
  const unsigned long long t0 = spin_clock();
  bool n0 = true, n1 = true, n2 = p2 != nullptr;
  for (unsigned spins = 0;; ++spins) {
    const int v0 = n0 ? df_poll(p0) : w0;
    const int v1 = n1 ? df_poll(p1) : w1;
    const int v2 = n2 ? df_poll(p2) : w2;
    n0 = v0 < w0;
    n1 = v1 < w1;
    n2 = v2 < w2;
    if (!(n0 || n1 || n2)) return true;
    if ((spins & 15) == 0 && df_poll(abortw)) return false;
    if (spin_expired(spins, t0)) {
      __hip_atomic_store(abortw, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      atomicExch(&ctrl->df_status, 2);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// Stage a 64 x 64 tile (descriptor m, leading dimension ld) into LDS [64][DF_SP]: 8 x 16-B sc1 loads per thread.
__device__ __forceinline__ void df_stage(double* __restrict__ dst, const Sc1Mem& m, int ld) {
  const int tid = threadIdx.x;
  f64x2 v[NB * NB / 512];
#pragma unroll
  for (int q = 0; q < NB * NB / 512; ++q) {
    const int idx = q * 256 + tid;
    v[q] = m.ld2((idx >> 5) * ld + 2 * (idx & 31));
  }
#pragma unroll
  for (int q = 0; q < NB * NB / 512; ++q) {
    const int idx = q * 256 + tid;
    const int r = idx >> 5, c = 2 * (idx & 31);
    dst[r * DF_SP + c] = v[q][0];
    dst[r * DF_SP + c + 1] = v[q][1];
  }
}

// The two halves of df_stage, for software pipelining: loads into registers, then LDS stores.
__device__ __forceinline__ void df_load(f64x2 (&v)[NB * NB / 512], const Sc1Mem& m, int ld) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int q = 0; q < NB * NB / 512; ++q) {
    const int idx = q * 256 + tid;
    v[q] = m.ld2((idx >> 5) * ld + 2 * (idx & 31));
  }
}
__device__ __forceinline__ void df_put(double* __restrict__ dst, const f64x2 (&v)[NB * NB / 512]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int q = 0; q < NB * NB / 512; ++q) {
    const int idx = q * 256 + tid;
    const int r = idx >> 5, c = 2 * (idx & 31);
    *reinterpret_cast<f64x2*>(dst + r * DF_SP + c) = v[q];
  }
}

// acc (wave (wr, wc): 32 x 32 block = 2 x 2 MFMA tiles) += sgn * P_i[rows] . P_j[cols]^T over K = 64.
__device__ __forceinline__ void df_mfma(d4f (&acc)[2][2], const double* Pi, const double* Pj, double sgn, int wr,
                                        int wc, int lane) {
#pragma unroll
  for (int s = 0; s < NB / 4; ++s) {
    const int kk = 4 * s + (lane >> 4);
    double fa[2], fb[2];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) fa[mi] = sgn * Pi[(wr * 32 + mi * 16 + (lane & 15)) * DF_SP + kk];
#pragma unroll
    for (int nj = 0; nj < 2; ++nj) fb[nj] = Pj[(wc * 32 + nj * 16 + (lane & 15)) * DF_SP + kk];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int nj = 0; nj < 2; ++nj)
        acc[mi][nj] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[mi], fb[nj], acc[mi][nj], 0, 0, 0);
  }
  // issue order for the unrolled loop (the LDS reads of two k-steps pair into ds_read2): the next pair's four reads
  // right after the first two MFMAs of the current pair, so their round trip hides behind the other six
  __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
  for (int p = 0; p < NB / 8; ++p) {
    __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
    if (p + 1 < NB / 8) __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
  }
}

// The updates run df_mfma on the negated tile with sgn = +1, df_neg before and after: with round-to-nearest every
// step of the MFMA's sum is symmetric under a sign flip, so -((-C) + sum a b) is C + sum (-a) b bit for bit, and the
// inner loop has no sign flip between an LDS read and its MFMA (with the issue order in df_mfma: Cholesky 1.052 ->
// 1.043 ms, the same fingerprints; profiles/r05/ab_pipe)
__device__ __forceinline__ void df_neg(d4f (&acc)[2][2]) {
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int nj = 0; nj < 2; ++nj) acc[mi][nj] = -acc[mi][nj];
}

// UPDATE(i,j,k): A_ij -= L_ik L_jk^T.  On a diagonal tile the strictly-upper 32 x 32 wave block is skipped.
// The tile's C operand in MFMA accumulator layout: from L, or on its first touch (k == 0) Q from H.
__device__ __forceinline__ void df_load_c(d4f (&acc)[2][2], const Sc1Mem& mC, int ld, int i, int j, bool fold,
                                          const QFold& qf, int wr, int wc, int lane) {
  if (fold) {
    const Sc1Mem mH(const_cast<double*>(qf.H) + (size_t)i * NB * ld + (size_t)j * NB, tile_bytes(ld));
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int nj = 0; nj < 2; ++nj)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = wr * 32 + mi * 16 + (lane >> 4) + 4 * r, col = wc * 32 + nj * 16 + (lane & 15);
          acc[mi][nj][r] = mH.ld(row * ld + col);
        }
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int nj = 0; nj < 2; ++nj)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = wr * 32 + mi * 16 + (lane >> 4) + 4 * r, col = wc * 32 + nj * 16 + (lane & 15);
          acc[mi][nj][r] = qf_entry(qf, i * NB + row, j * NB + col, acc[mi][nj][r]);
        }
    return;
  }
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int nj = 0; nj < 2; ++nj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wr * 32 + mi * 16 + (lane >> 4) + 4 * r, col = wc * 32 + nj * 16 + (lane & 15);
        acc[mi][nj][r] = mC.ld(row * ld + col);
      }
}

__device__ void df_update(double* __restrict__ L, int ld, int i, int j, int k, double* smem, const QFold& qf) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const bool active = !(i == j && wc > wr);
  const Sc1Mem mC(L + (size_t)i * NB * ld + (size_t)j * NB, tile_bytes(ld));
  d4f acc[2][2];
  df_load_c(acc, mC, ld, i, j, qf.H && k == 0, qf, wr, wc, lane);
  double* Pi = smem;
  double* Pj = (i == j) ? smem : smem + NB * DF_SP;
  {  // both panel tiles' loads in flight together (one round trip, behind the C loads), then the LDS stores
    f64x2 vi[NB * NB / 512], vj[NB * NB / 512];
    df_load(vi, Sc1Mem(L + (size_t)i * NB * ld + (size_t)k * NB, tile_bytes(ld)), ld);
    if (i != j) df_load(vj, Sc1Mem(L + (size_t)j * NB * ld + (size_t)k * NB, tile_bytes(ld)), ld);
    df_put(Pi, vi);
    if (i != j) df_put(Pj, vj);
  }
  __syncthreads();
  if (active) {
    df_neg(acc);
    df_mfma(acc, Pi, Pj, 1.0, wr, wc, lane);
    df_neg(acc);
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int nj = 0; nj < 2; ++nj)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = wr * 32 + mi * 16 + (lane >> 4) + 4 * r, col = wc * 32 + nj * 16 + (lane & 15);
          mC.st(row * ld + col, acc[mi][nj][r]);
        }
  }
}

// UPDATE4 (G = 4)(i,j,k0): A_ij -= sum_{k=k0}^{k0+G-1} L_ik L_jk^T — one read-modify-write of the tile for G panels,
// with the operand tiles of panel k+1 loaded into registers while the MFMAs of panel k run (two LDS buffers).  The
// accumulator is the FP64 tile itself, so G panels in one task are the same bits as G single-panel tasks.
template <int G>
__device__ void df_updateg(double* __restrict__ L, int ld, int i, int j, int k0, double* smem, const QFold& qf) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const bool active = !(i == j && wc > wr);
  const bool diag = (i == j);
  const Sc1Mem mC(L + (size_t)i * NB * ld + (size_t)j * NB, tile_bytes(ld));
  d4f acc[2][2];
  df_load_c(acc, mC, ld, i, j, qf.H && k0 == 0, qf, wr, wc, lane);
  df_neg(acc);
  f64x2 vi[NB * NB / 512], vj[NB * NB / 512];
  auto tile = [&](int r, int k) { return Sc1Mem(L + (size_t)r * NB * ld + (size_t)k * NB, tile_bytes(ld)); };
  df_load(vi, tile(i, k0), ld);
  if (!diag) df_load(vj, tile(j, k0), ld);
  df_put(smem, vi);
  if (!diag) df_put(smem + NB * DF_SP, vj);
#pragma unroll 1
  for (int q = 0; q < G; ++q) {
    double* Pi = smem + (q & 1) * 2 * NB * DF_SP;
    double* Pj = diag ? Pi : Pi + NB * DF_SP;
    if (q < G - 1) {
      df_load(vi, tile(i, k0 + q + 1), ld);
      if (!diag) df_load(vj, tile(j, k0 + q + 1), ld);
    }
    __syncthreads();  // panel q staged; every wave is done with panel q - 1 (the other buffer)
    if (active) df_mfma(acc, Pi, Pj, 1.0, wr, wc, lane);
    if (q < G - 1) {
      double* Ni = smem + ((q + 1) & 1) * 2 * NB * DF_SP;
      df_put(Ni, vi);
      if (!diag) df_put(Ni + NB * DF_SP, vj);
    }
  }
  if (active) {
    df_neg(acc);
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int nj = 0; nj < 2; ++nj)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = wr * 32 + mi * 16 + (lane >> 4) + 4 * r, col = wc * 32 + nj * 16 + (lane & 15);
          mC.st(row * ld + col, acc[mi][nj][r]);
        }
  }
}

// TRSM(i,k): X = A_ik Linv_kk^T into tile (i,k); rhs_i -= X w_k (w_k = rhs block k after POTRF(k)).  The task
// starts once all of Linv_kk is published (chain flag) and waits for w_k (state(k,k) == k + 1, the end of POTRF(k))
// only before the rhs update, so the L tile is not held back by POTRF's forward solve.  False: the launch aborted.
__device__ bool df_trsm(double* __restrict__ L, int ld, int i, int k, double* __restrict__ rhs, int nrhs,
                        double* __restrict__ Linv, double* smem, int* state, int* rhscnt, int* abortw, DevCtrl* ctrl,
                        int* s_ok, const QFold& qf) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  double* Pi = smem;
  double* Pj = smem + NB * DF_SP;
  const Sc1Mem mA(L + (size_t)i * NB * ld + (size_t)k * NB, tile_bytes(ld));
  const Sc1Mem mW(rhs + (size_t)k * NB * nrhs, (unsigned)(NB * nrhs) * 8u);
  const Sc1Mem mR(rhs + (size_t)i * NB * nrhs, (unsigned)(NB * nrhs) * 8u);
  {  // both operand tiles' loads in flight together, then the LDS stores
    f64x2 va[NB * NB / 512], vl[NB * NB / 512];
    if (qf.H && k == 0) qf_load(va, qf, ld, i * NB, 0);
    else df_load(va, mA, ld);
    df_load(vl, Sc1Mem(Linv + (size_t)k * NB * NB, tile_bytes(NB)), NB);
    df_put(Pi, va);
    df_put(Pj, vl);
  }
  __syncthreads();
  // Linv_kk is lower triangular: output column block c needs K < 16 (c + 1) only.  Wave (rh, cp) takes rows
  // 32 rh.. and the column blocks {0, 3} (cp = 0) or {1, 2} (cp = 1): 40 MFMAs per wave instead of 64, balanced.
  // (The skipped products are exact zeros: the sums are the full-K ones bit for bit.)
  const int rh = wid >> 1, cp = wid & 1;
  const int cb0 = cp ? 1 : 0, cb1 = cp ? 2 : 3;
  const int lim0 = 4 * (cb0 + 1), lim1 = 4 * (cb1 + 1);
  d4f acc[2][2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int t = 0; t < 2; ++t) acc[mi][t] = d4f{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int st = 0; st < NB / 4; ++st) {
    const int kk = 4 * st + (lane >> 4);
    double fa[2];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) fa[mi] = Pi[(rh * 32 + mi * 16 + (lane & 15)) * DF_SP + kk];
    if (st < lim0) {
      const double fb = Pj[(cb0 * 16 + (lane & 15)) * DF_SP + kk];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) acc[mi][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[mi], fb, acc[mi][0], 0, 0, 0);
    }
    if (st < lim1) {
      const double fb = Pj[(cb1 * 16 + (lane & 15)) * DF_SP + kk];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) acc[mi][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[mi], fb, acc[mi][1], 0, 0, 0);
    }
  }
  __syncthreads();  // every wave is done reading Pi / Pj: reuse them for X and w_k
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rh * 32 + mi * 16 + (lane >> 4) + 4 * r, col = (t ? cb1 : cb0) * 16 + (lane & 15);
        mA.st(row * ld + col, acc[mi][t][r]);
        Pi[row * DF_SP + col] = acc[mi][t][r];
      }
  // L_ik is published before the rhs update: its consumers (the updates of row i and column i) start a rhs update
  // earlier.  The rhs updates of block row i stay in panel order through rhscnt[i] (applied TRSM(i, .) updates):
  // this one waits for w_k and for rhscnt[i] == k, and POTRF(i)'s fix hook on the chain waits for rhscnt[i] == i - 1.
  df_drain();
  __syncthreads();
  if (tid == 0) {
    __hip_atomic_store(state + df_tri(i, k), k + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int v0 = df_poll(state + df_tri(k, k)), v1 = df_poll(rhscnt + i);
    *s_ok = (v0 >= k + 1 || df_wait(state, df_tri(k, k), k + 1, abortw, ctrl)) &&
            (v1 >= k || df_wait(rhscnt, i, k, abortw, ctrl));
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keep the w_k and rhs loads behind the polls
  __syncthreads();
  if (!*s_ok) return false;
  double* wk = Pj;  // [64][nrhs]
  for (int t = tid; t < NB * nrhs; t += 256) wk[t] = mW.ld(t);
  __syncthreads();
  for (int t = tid; t < NB * nrhs; t += 256) {
    const int row = t / nrhs, rho = t % nrhs;
    double s = 0.0;
#pragma unroll 8
    for (int c = 0; c < NB; ++c) s = fma(Pi[row * DF_SP + c], wk[c * nrhs + rho], s);
    mR.st(t, mR.ld(t) - s);
  }
  df_drain();
  __syncthreads();
  if (tid == 0) __hip_atomic_store(rhscnt + i, k + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

// ---- chain slices (ping-pong consumer below): operands read from LDS in one batch, then the MFMAs back to back.
// One wave per SIMD cannot hide an LDS round trip behind another wave, so interleaving reads and MFMAs costs a round
// trip per MFMA pair (microbench/slices.hip: 4650 -> 2840 cycles per slice).
// TRSM slice CB: L'[16 w.., 16 CB..] = A[16 w.., :] L^-1[16 CB.., :]^T (K = 16 (CB + 1): L^-1 is lower); af = the
// wave's row-block of A as MFMA A-fragments (loaded once per block), E = row-block CB of L^-1 (row stride DF_SP).
template <int CB>
__device__ __forceinline__ d4f ch_trsm(const double (&af)[16], const double* E, int lane) {
  double xf[4 * (CB + 1)];
#pragma unroll
  for (int s = 0; s < 4 * (CB + 1); ++s) xf[s] = E[(lane & 15) * DF_SP + 4 * s + (lane >> 4)];
  d4f acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int s = 0; s < 4 * (CB + 1); s += 2) {
    acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(af[s], xf[s], acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(af[s + 1], xf[s + 1], acc1, 0, 0, 0);
  }
  return acc0 + acc1;
}
// the 10 lower 16 x 16 blocks of a 64 x 64 tile, 3 / 3 / 2 / 2 per wave (-1: none)
// (wave 0 holds only D_00, which POTRF's first sweep reads: with a deferred publication it goes from its last slice
// straight into the sweep while waves 1..3 finish and store the other nine blocks, ps.cntD)
constexpr int kChIB[4][3] = {{0, -1, -1}, {1, 1, 2}, {2, 2, 3}, {3, 3, 3}};
constexpr int kChJB[4][3] = {{0, -1, -1}, {0, 1, 2}, {0, 1, 3}, {0, 1, 2}};
// UPDATE slice: D -= L'[:, 16 cb..] L'[:, 16 cb..]^T on wave W's blocks (compile-time, so fragments are picked
// statically); Lp = L' with row stride DF_SP
template <int W>
__device__ __forceinline__ void ch_update(d4f (&dacc)[3], const double* Lp, int cb, int lane) {
  constexpr auto uses = [](int r) {
    for (int q = 0; q < 3; ++q)
      if (kChIB[W][q] == r || kChJB[W][q] == r) return true;
    return false;
  };
  double lf[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
    if (uses(r))
#pragma unroll
      for (int q = 0; q < 4; ++q) lf[r][q] = Lp[(16 * r + (lane & 15)) * DF_SP + 16 * cb + 4 * q + (lane >> 4)];
#pragma unroll
  for (int st = 0; st < 4; ++st)
#pragma unroll
    for (int q = 0; q < 3; ++q)
      if (kChIB[W][q] >= 0)
        dacc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(-lf[kChIB[W][q] < 0 ? 0 : kChIB[W][q]][st],
                                                       lf[kChJB[W][q] < 0 ? 0 : kChJB[W][q]][st], dacc[q], 0, 0, 0);
}

// The chain applies panel b-2 to block row b itself, L_b,b-1 is stored / published inside POTRF(b) by its waves 1..3,
// and POTRF's column sweep rides its broadcasts in DPP (round 6: the measured-and-rejected variants -- workers applying
// panel b-2, L_b,b-1 published before POTRF(b), the v_readlane sweep, data-tagged L^-1 row-blocks, eight-panel update
// groups -- are gone from the product; DESIGN.md §7 keeps their numbers).
__global__ __launch_bounds__(256, 1) void k_chol_dataflow(double* __restrict__ L, int ld, double* __restrict__ rhs,
                                                          int nrhs, double* __restrict__ Linv, DevCtrl* ctrl,
                                                          int* __restrict__ work, const unsigned* __restrict__ tasks,
                                                          int ntasks, int nblk, unsigned long long* __restrict__ trace,
                                                          const double* __restrict__ Hq, const double* __restrict__ dq,
                                                          int nq, int ruiz_gate, double early_min) {
  // the Ruiz loop launched ahead of the factorization without a host read may still be open (k_ruiz_final: -1): then
  // the launch is void and the host finishes the loop and factors again
  if (ruiz_gate && ctrl->ruiz_sweeps < 0) return;
  __shared__ __attribute__((aligned(16))) double smem[DF_SMEM];
  __shared__ unsigned s_task;
  __shared__ int s_ok;
  __shared__ int s_next;
  int* counter = work;
  int* abortw = work + 32;  // own cache line: the claim counter's line takes every worker's atomic
  int* state = work + 64;  // own cache lines
  int* cflag = work + 64 + nblk * (nblk + 1) / 2;  // cflag[k]: row-blocks of L_kk^-1 published (0..4)
  int* rhscnt = cflag + nblk;  // rhscnt[i]: worker TRSM(i, .) rhs updates applied to rhs block i (in panel order)
  const int tid = threadIdx.x;
  const QFold qf{Hq, dq, nq, Hq ? ctrl->reg : 0.0};
  // Roles by residency, not by blockIdx: the first two workgroups to start run the chain.  Workgroups are not
  // dispatched in blockIdx order across the XCDs, and with other work on the device (several contexts sharing one
  // GPU) blockIdx 1 may wait for a free CU behind workers that wait on it; with tickets, any three resident
  // workgroups of a launch make progress.
  __shared__ int s_role;
  if (tid == 0) s_role = atomicAdd(work + 2, 1);
  __syncthreads();
  const int role = s_role;
  if (role < 2) {
    // ---- roles 0 and 1: the critical chain, ping-pong.  The workgroup of role c factors the diagonal blocks b = c,
    // c + 2, ...  Before POTRF(b) it runs TRSM(b, b-1) and UPDATE(b, b, b-1) in four 16-column slices, each
    // started as soon as the other workgroup's POTRF(b-1) has published that row-block of L_b-1^-1
    // (chain flags), so the next factorization starts ~one slice after the previous one ends.  The updated
    // diagonal tile goes straight from the MFMA accumulators into this workgroup's POTRF workspace.
    ChainSmem& cs = *reinterpret_cast<ChainSmem*>(smem);
    Potrf64wSmem& ps = cs.p;
    const int lane = tid & 63, wv = tid >> 6;
    auto mark = [&](int k, int step, int field) {
      if (trace && tid == 0) trace[4 * (size_t)(ntasks + 5 * k + step) + field] = __builtin_amdgcn_s_memrealtime();
    };
    auto publish = [&](int idx, int v) {
      df_drain();  // every storing wave: its sc1 stores have left
      __syncthreads();
      if (tid == 0) __hip_atomic_store(state + idx, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    auto wait = [&](const int* base, int idx, int want) -> bool {
      if (tid == 0) s_ok = df_wait(base, idx, want, abortw, ctrl);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      __syncthreads();
      return s_ok;
    };
    constexpr int NBLK16 = 3;  // (kChIB / kChJB: this wave's lower 16 x 16 blocks)
    for (int b = role; b < nblk; b += 2) {
      if (b == 0) {
        if (qf.H) {
          f64x2 v[NB * NB / 512];
          qf_load(v, qf, ld, 0, 0);
#pragma unroll
          for (int q = 0; q < NB * NB / 512; ++q) {
            const int idx = q * 256 + tid;
            *reinterpret_cast<f64x2*>(ps.S + (idx >> 5) * P64_SP + 2 * (idx & 31)) = v[q];
          }
          const Sc1Mem mR(rhs, (unsigned)(NB * nrhs) * 8u);
          for (int t = tid; t < NB * nrhs; t += 256) ps.B[t] = mR.ld(t);
        } else {
          potrf64w_stage<Sc1Mem>(L, ld, 0, rhs, 0, nrhs, ps);
        }
      } else {
        const int k = b - 1;
        mark(k, 1, 0);
        const Sc1Mem mA(L + (size_t)b * NB * ld + (size_t)k * NB, tile_bytes(ld));
        const Sc1Mem mI(Linv + (size_t)k * NB * NB, (unsigned)(NB * NB) * 8u);
        // the row-blocks of L_kk^-1 already published (cflag, read while the tile loads are in flight) are loaded
        // at once into ps.S (free until the diagonal tile goes there at the end of the slices) and applied as one
        // batch below
        int pv = 0;
        d4f dacc[NBLK16];
        if (b >= 2) {
          // Panel j = b-2 of block row b on this workgroup (the tasks UPDATE(b,b,j) and UPDATE(b,k,j), not in the
          // worker list), in two waits (below).  The MFMA sequences are the workers' (df_update's K = 0..63 chain), so the factor is
          // bitwise the same; the worker -> state word -> staging hop of both tiles is gone from the chain.
          const int j = b - 2;
          // (1) A_b,k and D_b with every panel < j: final long before (the workers' updates of panel j-1), so their
          // loads go out first and land while (2) waits for the two fresh L tiles
          if (tid == 0) {
            const int v0 = df_poll(state + df_tri(b, k)), v1 = df_poll(state + df_tri(b, b));
            s_ok = (v0 >= j || df_wait(state, df_tri(b, k), j, abortw, ctrl)) &&
                   (v1 >= j || df_wait(state, df_tri(b, b), j, abortw, ctrl));
          }
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          __syncthreads();
          if (!s_ok) return;
          const int wr = wv >> 1, wc = wv & 1;
          d4f acc[2][2];
          const bool fold = qf.H && j == 0;  // block 2: A_2,1 and D_2 are first read here (Q formed from H)
          df_load_c(acc, mA, ld, b, k, fold, qf, wr, wc, lane);
          {
            const Sc1Mem mD(const_cast<double*>(fold ? qf.H : L) + (size_t)b * NB * ld + (size_t)b * NB, tile_bytes(ld));
#pragma unroll
            for (int q = 0; q < NBLK16; ++q) {
              const int ib = kChIB[wv][q], jb = kChJB[wv][q];
              if (ib >= 0) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                  const int rr = 16 * ib + (lane >> 4) + 4 * r, cc = 16 * jb + (lane & 15);
                  const double h = mD.ld(rr * ld + cc);
                  dacc[q][r] = fold ? qf_entry(qf, b * NB + rr, b * NB + cc, h) : h;
                }
              }
            }
          }
          // (2) L_b,j (worker TRSM(b,j)) and L_k,j (the other chain workgroup's TRSM, published inside its POTRF(k));
          // the rhs block is read in POTRF(b)'s fix hook, which it first feeds
          if (tid == 0) {
            const int v3 = df_poll(state + df_tri(b, j)), v4 = df_poll(state + df_tri(k, j));
            s_ok = (v3 >= j + 1 || df_wait(state, df_tri(b, j), j + 1, abortw, ctrl)) &&
                   (v4 >= j + 1 || df_wait(state, df_tri(k, j), j + 1, abortw, ctrl));
          }
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          __syncthreads();
          if (!s_ok) return;
          mark(k, 2, 3);  // trace: the b-2 panel's inputs are in (field 3 of the fix record)
          {
            f64x2 vl[NB * NB / 512], vk[NB * NB / 512];
            df_load(vl, Sc1Mem(L + (size_t)b * NB * ld + (size_t)j * NB, tile_bytes(ld)), ld);
            df_load(vk, Sc1Mem(L + (size_t)k * NB * ld + (size_t)j * NB, tile_bytes(ld)), ld);
            df_put(ps.X, vl);  // (POTRF's L^-1 workspace and tile: free until the reset / the batch below)
            df_put(ps.S, vk);
          }
          __syncthreads();
          for (int cb = 0; cb < 4; ++cb) {
            switch (wv) {  // D_b -= L_b,j L_b,j^T on this wave's lower blocks
              case 0: ch_update<0>(dacc, ps.X, cb, lane); break;
              case 1: ch_update<1>(dacc, ps.X, cb, lane); break;
              case 2: ch_update<2>(dacc, ps.X, cb, lane); break;
              default: ch_update<3>(dacc, ps.X, cb, lane); break;
            }
          }
          df_mfma(acc, ps.X, ps.S, -1.0, wr, wc, lane);  // A_b,k -= L_b,j L_k,j^T
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int nj = 0; nj < 2; ++nj)
#pragma unroll
              for (int r = 0; r < 4; ++r)
                cs.Sa[(wr * 32 + mi * 16 + (lane >> 4) + 4 * r) * DF_SP + wc * 32 + nj * 16 + (lane & 15)] = acc[mi][nj][r];
          // the row-blocks of L_kk^-1 published by now (after this panel's MFMAs, so the batch below takes as many as
          // it can)
          if (tid == 0) pv = __hip_atomic_load(cflag + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          mark(k, 0, 3);  // trace: the b-2 panel applied (field 3 of POTRF(k)'s record)
        } else {
        // A_b,k and D_b with every panel < k applied (state >= k): one wait for both states, then every load in
        // flight together (the rhs block is read in POTRF(b)'s fix hook)
        if (tid == 0) {  // (the polls in flight together: usually the other inputs are final when the first is)
          const int v0 = df_poll(state + df_tri(b, k)), v1 = df_poll(state + df_tri(b, b));
          s_ok = (v0 >= k || df_wait(state, df_tri(b, k), k, abortw, ctrl)) &&
                 (v1 >= k || df_wait(state, df_tri(b, b), k, abortw, ctrl));
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        __syncthreads();
        if (!s_ok) return;
        {
          f64x2 va[NB * NB / 512];
          const bool fold = qf.H && k == 0;  // block 1: A_1,0 and D_1 are first read here
          if (fold) qf_load(va, qf, ld, b * NB, 0);
          else df_load(va, mA, ld);
          const Sc1Mem mD(const_cast<double*>(fold ? qf.H : L) + (size_t)b * NB * ld + (size_t)b * NB, tile_bytes(ld));
#pragma unroll
          for (int q = 0; q < NBLK16; ++q) {
            const int ib = kChIB[wv][q], jb = kChJB[wv][q];
            if (ib >= 0) {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int rr = 16 * ib + (lane >> 4) + 4 * r, cc = 16 * jb + (lane & 15);
                const double h = mD.ld(rr * ld + cc);
                dacc[q][r] = fold ? qf_entry(qf, b * NB + rr, b * NB + cc, h) : h;
              }
            }
          }
          if (tid == 0) pv = __hip_atomic_load(cflag + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          df_put(cs.Sa, va);
        }
        }
        if (tid == 0) s_next = pv;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        __syncthreads();
        const int nbat = min(s_next, 4);
        {
          f64x2 vb[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const int e = tid + 256 * q;
            if (q < 2 * nbat) vb[q] = mI.ld2((e >> 5) * NB + 2 * (e & 31));
          }
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const int e = tid + 256 * q;
            if (q < 2 * nbat) *reinterpret_cast<f64x2*>(ps.S + (e >> 5) * P64_SP + 2 * (e & 31)) = vb[q];
          }
        }
        potrf64w_reset(ps);  // the slices leave POTRF's L^-1 workspace and flags alone: clear them off the chain
        if (tid == 0) cs.lpub = 0;  // (POTRF(b-2)'s pre hook is long done; the barrier below orders it)
        mark(k, 1, 1);
        // L_b,k, row stride DF_SP: written over A_b,k in Sa (every wave holds its row-block of A in af before the first
        // slice's barrier), where it stays for the rhs correction at the end of POTRF(b) — no copy before POTRF
        double* Lp = cs.Sa;
        // row-block cb of L_kk^-1 (published by the other workgroup's POTRF(k) as cflag[k] reaches cb + 1) is
        // loaded into registers one slice ahead when it is already published, so its latency hides behind the
        // MFMAs of the current slice
        f64x2 er[2];
        auto eload = [&](int cb) {
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const int e = tid + 256 * q;
            er[q] = mI.ld2((16 * cb + (e >> 5)) * NB + 2 * (e & 31));
          }
        };
        __syncthreads();  // Sa and the batch's row-blocks in ps.S complete
        mark(k, 4, 0);    // trace: every wave's staging loads landed (record 4: the batch's phases)
        double af[16];  // this wave's row-block of A_b,k as MFMA A-fragments
#pragma unroll
        for (int q = 0; q < 16; ++q) af[q] = cs.Sa[(16 * wv + (lane & 15)) * DF_SP + 4 * q + (lane >> 4)];
        if (nbat > 0) {
          // the batch: the same MFMA sequence per output as the per-slice form below, so the same bits
          d4f acc[4];
          acc[0] = ch_trsm<0>(af, ps.S, lane);
          if (nbat > 1) acc[1] = ch_trsm<1>(af, ps.S + 16 * P64_SP, lane);
          if (nbat > 2) acc[2] = ch_trsm<2>(af, ps.S + 32 * P64_SP, lane);
          if (nbat > 3) acc[3] = ch_trsm<3>(af, ps.S + 48 * P64_SP, lane);
          __syncthreads();  // every wave holds its fragments of A (Sa takes L')
          mark(k, 4, 1);
#pragma unroll
          for (int cb = 0; cb < 4; ++cb)
            if (cb < nbat)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int row = 16 * wv + (lane >> 4) + 4 * r, col = 16 * cb + (lane & 15);
                Lp[row * DF_SP + col] = acc[cb][r];
              }
          __syncthreads();
          for (int cb = 0; cb < nbat; ++cb) {
            switch (wv) {  // D -= L'[:, cb] L'[:, cb]^T on this wave's lower blocks
              case 0: ch_update<0>(dacc, Lp, cb, lane); break;
              case 1: ch_update<1>(dacc, Lp, cb, lane); break;
              case 2: ch_update<2>(dacc, Lp, cb, lane); break;
              default: ch_update<3>(dacc, Lp, cb, lane); break;
            }
          }
          mark(k, 4, 2);
        }
        if (nbat < 4) {
          if (!wait(cflag, k, nbat + 1)) return;
          eload(nbat);
        }
        bool have_next = nbat < 4;
#pragma unroll 1
        for (int cb = nbat; cb < 4; ++cb) {
          double* E = cs.E2[cb & 1];
          if (cb == 3) mark(k + 1, 0, 1);  // trace: slice 2 done (field 1 of the next POTRF record)
          if (!have_next) {
            if (!wait(cflag, k, cb + 1)) return;
            eload(cb);
          }
          if (cb == 3) mark(k, 1, 3);  // trace: last row-block of L_kk^-1 in hand
          // non-blocking look at the next row-block: the sc1 poll is issued here and its value consumed only after
          // this slice's MFMAs, so its round trip stays off the chain
          int pollv = 0;
          if (cb < 3 && tid == 0) pollv = __hip_atomic_load(cflag + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const int e = tid + 256 * q;
            *reinterpret_cast<f64x2*>(E + (e >> 5) * DF_SP + 2 * (e & 31)) = er[q];
          }
          __syncthreads();
          {  // L'[16 wv.., 16 cb..] = A[16 wv.., :] L^-1[16 cb.., :]^T, K = 16 (cb + 1), two MFMA chains
            d4f acc;
            switch (cb) {
              case 0: acc = ch_trsm<0>(af, E, lane); break;
              case 1: acc = ch_trsm<1>(af, E, lane); break;
              case 2: acc = ch_trsm<2>(af, E, lane); break;
              default: acc = ch_trsm<3>(af, E, lane); break;
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int row = 16 * wv + (lane >> 4) + 4 * r, col = 16 * cb + (lane & 15);
              Lp[row * DF_SP + col] = acc[r];
            }
          }
          if (tid == 0) s_next = (cb < 3) && pollv >= cb + 2;  // own word: read between this barrier and the next
          __syncthreads();
          have_next = s_next;
          if (have_next) eload(cb + 1);  // lands behind the diagonal update below
          switch (wv) {  // D -= L'[:, cb] L'[:, cb]^T on this wave's lower blocks
            case 0: ch_update<0>(dacc, Lp, cb, lane); break;
            case 1: ch_update<1>(dacc, Lp, cb, lane); break;
            case 2: ch_update<2>(dacc, Lp, cb, lane); break;
            default: ch_update<3>(dacc, Lp, cb, lane); break;
          }
        }
#pragma unroll
        for (int q = 0; q < NBLK16; ++q) {
          const int ib = kChIB[wv][q], jb = kChJB[wv][q];
          if (ib >= 0) c16_store(ps.S + 16 * ib * P64_SP + 16 * jb, P64_SP, dacc[q], lane);
        }
        // L_b,k goes to HBM off the chain: waves 1..3 of POTRF(b) store it from Sa and raise state(b, k) (pre hook
        // below), while wave 0 runs the first sweep -- no drain round trip between the last slice and POTRF(b).  No
        // barrier either: wave 0 starts the sweep on its own D_00, and waves 1..3 count their stored blocks into
        // ps.cntD, which POTRF's first T / U and phase A wait for.
        if (wv > 0) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          if (lane == 0) p64w_add(&ps.cntD);
        }
        mark(k, 1, 2);
      }
      // POTRF(b): tile and rhs block staged in LDS; L_bb^-1 row-blocks published progressively; before the
      // forward solve, the rhs block gets its last correction  - L_b,b-1 w_b-1  (w_b-1: POTRF(b-1) done)
      mark(b, 0, 0);
      auto fix = [&]() -> bool {
        if (b == 0) return true;
        const int k = b - 1;
        mark(k, 2, 0);
        // w_k (POTRF(k) done) and the rhs block b with every worker TRSM(b, j < k)'s update (rhscnt[b] == k)
        if (tid == 0) {
          const int v0 = df_poll(state + df_tri(k, k)), v1 = df_poll(rhscnt + b);
          s_ok = (v0 >= k + 1 || df_wait(state, df_tri(k, k), k + 1, abortw, ctrl)) &&
                 (v1 >= k || df_wait(rhscnt, b, k, abortw, ctrl));
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        __syncthreads();
        if (!s_ok) return false;
        mark(k, 2, 1);
        const Sc1Mem mW(rhs + (size_t)k * NB * nrhs, (unsigned)(NB * nrhs) * 8u);
        const Sc1Mem mRb(rhs + (size_t)b * NB * nrhs, (unsigned)(NB * nrhs) * 8u);
        for (int t = tid; t < NB * nrhs; t += 256) {
          cs.V[t] = mW.ld(t);
          ps.B[t] = mRb.ld(t);
        }
        __syncthreads();
        for (int t0 = 0; t0 < NB * nrhs * 4; t0 += 256) {
          const int t = t0 + tid, q = t & 3, e = t >> 2;
          const int r = e / nrhs, rho = e - r * nrhs;
          double sv = 0.0;
          if (e < NB * nrhs) {
            for (int c = 16 * q; c < 16 * q + 16; ++c) sv = fma(cs.Sa[r * DF_SP + c], cs.V[c * nrhs + rho], sv);
          }
          sv += __shfl_xor(sv, 1, 64);
          sv += __shfl_xor(sv, 2, 64);
          if (q == 0 && e < NB * nrhs) ps.B[e] -= sv;
        }
        mark(k, 2, 2);
        return true;
      };
      if (b == 0) {
        potrf64w_reset(ps);
        __syncthreads();
      }  // b > 0: reset behind the staging, the tile's LDS stores behind publish()'s barrier
      auto pre = [&](int w, int ln) {  // waves 1..3: L_b,b-1 from Sa to HBM, the last one to drain raises its state
        if (b == 0) return;
        const int k = b - 1;
        const Sc1Mem mL(L + (size_t)b * NB * ld + (size_t)k * NB, tile_bytes(ld));
        for (int e = 64 * (w - 1) + ln; e < NB * NB / 2; e += 192) {
          const int r = e >> 5, c = 2 * (e & 31);
          mL.st2(r * ld + c, *reinterpret_cast<const f64x2*>(cs.Sa + r * DF_SP + c));
        }
        df_drain();
        if (ln == 0 && atomicAdd(&cs.lpub, 1) == 2)
          __hip_atomic_store(state + df_tri(b, k), k + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      };
      if (!potrf64w_factor<Sc1Mem>(b, rhs, nrhs, Linv, ctrl, ps, cflag + b, fix, early_min, pre,
                                   trace ? trace + 4 * (size_t)(ntasks + 5 * b + 3) : nullptr, b > 0)) {
        if (tid == 0) __hip_atomic_store(abortw, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
      }
      publish(df_tri(b, b), b + 1);  // w_b and L_bb^-1 stored
      mark(b, 0, 2);
      potrf64w_store_L<Sc1Mem>(L, ld, b, ps);  // only the final backward solve reads L_bb
      __syncthreads();  // the potrf workspace is reused by the next TRSM slices
    }
    return;
  }
  // ---- roles 2..: claim the remaining tasks in the host-built order ---------------------------
  // The claim is one atomic on the counter; the abort word lives on its own cache line and is read only by the waits
  // (a task that finds an input short), not before every claim.  With the abort word beside the counter, every
  // worker's claim-time poll queued behind the other workers' atomics on that one line: Cholesky 1.29 -> 1.09 ms at
  // C3 once it moved.  The dependency polls of a task go out together (df_wait3).
  int my_idx = -1;  // thread 0: claimed task index (trace)
  for (;;) {
    if (tid == 0) {
      unsigned t = 0xffffffffu;
      const int idx = atomicAdd(counter, 1);
      if (idx < ntasks) t = tasks[idx];
      my_idx = idx;
      if (trace && idx < ntasks) trace[4 * idx] = __builtin_amdgcn_s_memrealtime();
      s_task = t;
    }
    __syncthreads();
    const unsigned task = s_task;
    if (task == 0xffffffffu) break;
    const int type = task >> 30, k = (task >> 20) & 1023, i = (task >> 10) & 1023, j = task & 1023;
    if (tid == 0) {
      bool ok;
      if (type == 1) {  // all of Linv_kk published (w_k is awaited inside the task)
        ok = df_wait3(cflag + k, 4, state + df_tri(i, k), k, nullptr, 0, abortw, ctrl);
      } else if (type == 3) {  // panels k..k+3: TRSM(., k+3) done implies the earlier ones
        ok = df_wait3(state + df_tri(i, k + 3), k + 4, state + df_tri(j, k + 3), k + 4, state + df_tri(i, j), k,
                      abortw, ctrl);
      } else {
        ok = df_wait3(state + df_tri(i, k), k + 1, state + df_tri(j, k), k + 1, state + df_tri(i, j), k, abortw, ctrl);
      }
      s_ok = ok;
      if (trace) trace[4 * my_idx + 1] = __builtin_amdgcn_s_memrealtime();
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keep the data loads behind the poll
    __syncthreads();
    if (!s_ok) break;
    int done_idx, done_val = k + 1;
    if (type == 1) {
      if (!df_trsm(L, ld, i, k, rhs, nrhs, Linv, smem, state, rhscnt, abortw, ctrl, &s_ok, qf)) break;
      done_idx = df_tri(i, k);
    } else if (type == 3) {
      df_updateg<4>(L, ld, i, j, k, smem, qf);
      done_idx = df_tri(i, j);
      done_val = k + 4;
    } else {
      df_update(L, ld, i, j, k, smem, qf);
      done_idx = df_tri(i, j);
    }
    df_drain();  // every storing wave: its sc1 stores have left
    __syncthreads();
    if (tid == 0) {
      __hip_atomic_store(state + done_idx, done_val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (trace) {
        trace[4 * my_idx + 2] = __builtin_amdgcn_s_memrealtime();
        trace[4 * my_idx + 3] = blockIdx.x;
      }
    }
  }
}

// work: [0] counter, [2] role ticket, [32] abort word, [64 ..) one state word per lower tile, then one chain flag and
// one rhs counter per diagonal block; zeroed before every launch.
size_t chol_dataflow_work_ints(int nblk) { return 64 + (size_t)nblk * (nblk + 1) / 2 + 2 * (size_t)nblk; }

void launch_chol_dataflow(hipStream_t s, double* L, int ld, double* rhs, int nrhs, double* Linv, DevCtrl* ctrl,
                          int* work, int nblk, const unsigned* tasks, int ntasks, int nwg,
                          unsigned long long* trace, bool zero_work, const double* Hq, const double* dq, int nq,
                          bool ruiz_gate, double early_min) {
  if (zero_work) (void)hipMemsetAsync(work, 0, chol_dataflow_work_ints(nblk) * sizeof(int), s);
  k_chol_dataflow<<<nwg, 256, 0, s>>>(L, ld, rhs, nrhs, Linv, ctrl, work, tasks, ntasks, nblk, trace, Hq, dq, nq,
                                      ruiz_gate ? 1 : 0, early_min);
}

}  // namespace cvxg
