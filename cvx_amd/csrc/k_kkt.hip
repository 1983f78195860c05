// k_kkt.hip — the equality block of the Newton system, KKTSystem.solveWithCholFactor (KKTSystem.scala:99-167), on the
// factor Q + reg I = L L' the engine already holds, in the reference's own sequence:
//   X = Q^-1 [B' | Dq]           (B = Aeq diag(d); :114-121, MatrixUtils.triangularSolve with L, then with L')
//   R = B X,  S = (R + R')/2     (:126, :139)
//   z = -(b + R[:, p])           (:141)
//   w = S^-1 z                   (:140-144, cholesky(S) + two triangular solves; failure = not positive definite)
//   y = -(X[:, p] + X[:, :p] w)  (:145)
// X comes from the factorization's fused forward solve + k_bwd_dataflow when p + 1 <= MAX_RHS, otherwise from the
// many-column dataflow solves k_trsm_many<false> (L) and k_trsm_many<true> (L') below.
#include "potrf64.hpp"  // Sc1Mem, f64x2, d4f

namespace cvxg {

constexpr int FM_CW = 16;      // right-hand-side columns per k_trsm_many workgroup (one MFMA column block)
constexpr int FM_SP = NB + 2;  // LDS row stride of the staged L tile: conflict-free A fragments either way round

// ------------------------------------------------------------------------------------------------
// Triangular solve with many right-hand sides (nchunk * FM_CW columns, row-major, leading dimension ldy), in place, in
// ONE launch:  BWD = false: L Z = Y (blocks b = 0, 1, ...),  BWD = true: L' X = Y (blocks b = nblk-1, ..., 0).
// Workgroup (b, c) owns row block b and column chunk c.  With T_i the off-diagonal tile that couples block b to an
// earlier-solved block i (L_bi, or L_ib'), Minv the diagonal-block inverse the factorization stored (Linv_bb, or its
// transpose) and i* the block solved just before b:
//   Z_b = Minv (Y_b - sum_{i != i*} T_i Z_i) - (Minv T_i*) Z_i* = V_b - M_b Z_i*.
// M_b (a 64^3 MFMA product) and V_b (MFMAs over the blocks solved two or more hops earlier, the L tiles staged through
// LDS with the next tile's loads in flight) are formed while the chain is still upstream, so once Z_i* is published
// the critical path is one chain of 16 MFMAs per wave whose B fragments are polled straight from Z_i*'s granules (no
// LDS, no barrier).  Hand-off: every entry of Z_b goes out as a data-tagged 16-B granule {value, gen} (one sc1 store)
// and consumers poll the granules themselves (the k_bwd_dataflow scheme).  Workgroups only wait on lower blockIdx
// (dispatched earlier), so the launch is deadlock-free at any residency; every wait is bounded (a timeout raises
// ctrl->df_status = 2 and the launch completes with the granules published).
// MFMA f64 16x16x4: A lane l = (row l&15, k l>>4), B lane l = (k l>>4, col l&15), C/D reg r = (row (l>>4)+4r, col l&15).
// ------------------------------------------------------------------------------------------------
template <bool BWD>
__global__ __launch_bounds__(256) void k_trsm_many(const double* __restrict__ L, int ld, const double* __restrict__ Linv,
                                                   double* __restrict__ Y, int ldy, int nblk, int nchunk,
                                                   double* __restrict__ gran, int gen, DevCtrl* ctrl) {
  if (ctrl->chol_info != 0) return;
  __shared__ __attribute__((aligned(16))) double Ls[NB * FM_SP];
  __shared__ double Zs[NB * FM_CW];
  __shared__ int s_bad;
  const int q0 = (int)blockIdx.x / nchunk, c = (int)blockIdx.x - q0 * nchunk;
  const int b = BWD ? nblk - 1 - q0 : q0;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r16 = 16 * w + (lane & 15), k4 = lane >> 4;  // A-fragment row, B-fragment k offset
  const double tag = __longlong_as_double((long long)gen);
  if (tid == 0) s_bad = 0;
  auto granules = [&](int i) {  // chunk c of block i: [64 rows][16 cols] granules of 16 B
    return Sc1Mem(gran + (size_t)(i * nchunk + c) * NB * FM_CW * 2, (unsigned)(NB * FM_CW) * 16u);
  };
  auto minv_nonzero = [&](int s) { return BWD ? s >= 4 * w : s < 4 * (w + 1); };  // wave-uniform
  // this block's rhs chunk (C layout) and the A fragments of Minv
  double yb[4], lin[16];
#pragma unroll
  for (int r = 0; r < 4; ++r)
    yb[r] = Y[(size_t)(b * NB + 16 * w + k4 + 4 * r) * ldy + c * FM_CW + (lane & 15)];
  {
    const double* li = Linv + (size_t)b * NB * NB;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int k = 4 * s + k4;
      lin[s] = minv_nonzero(s) ? (BWD ? li[k * NB + r16] : li[r16 * NB + k]) : 0.0;
    }
  }
  f64x2 lt[NB * NB / 512];  // an L tile in flight: this thread's eight 16-B pieces
  auto load_tile = [&](int i) {
    const double* tp = BWD ? L + (size_t)i * NB * ld + (size_t)b * NB : L + (size_t)b * NB * ld + (size_t)i * NB;
#pragma unroll
    for (int q = 0; q < NB * NB / 512; ++q) {
      const int idx = q * 256 + tid;
      lt[q] = *reinterpret_cast<const f64x2*>(tp + (size_t)(idx >> 5) * ld + 2 * (idx & 31));
    }
  };
  auto stage_tile = [&]() {
#pragma unroll
    for (int q = 0; q < NB * NB / 512; ++q) {
      const int idx = q * 256 + tid;
      *reinterpret_cast<f64x2*>(Ls + (idx >> 5) * FM_SP + 2 * (idx & 31)) = lt[q];
    }
  };
  auto tile_a = [&](int s) {  // T_i[r16][4s + k4] from the staged tile
    const int k = 4 * s + k4;
    return BWD ? Ls[k * FM_SP + r16] : Ls[r16 * FM_SP + k];
  };
  const int nsteps = BWD ? nblk - 1 - b : b;
  auto step_block = [&](int t) { return BWD ? nblk - 1 - t : t; };
  const int istar = nsteps > 0 ? step_block(nsteps - 1) : 0;
  // ---- M_b = Minv T_i*, kept as negated A fragments
  double mf[16];
  if (nsteps > 0) {
    load_tile(istar);
    stage_tile();
    __syncthreads();
    d4f m[4];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      m[nb] = d4f{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s = 0; s < 16; ++s)
        if (minv_nonzero(s)) {
          const int k = 4 * s + k4, col = 16 * nb + (lane & 15);  // B = T_i*[k][col]
          m[nb] = __builtin_amdgcn_mfma_f64_16x16x4f64(lin[s], BWD ? Ls[col * FM_SP + k] : Ls[k * FM_SP + col], m[nb],
                                                       0, 0, 0);
        }
    }
    __syncthreads();  // every wave is done with T_i*: the tile buffer takes M
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) Ls[(16 * w + k4 + 4 * r) * FM_SP + 16 * nb + (lane & 15)] = m[nb][r];
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 16; ++s) mf[s] = -Ls[r16 * FM_SP + 4 * s + k4];
    __syncthreads();  // the buffer is the accumulation's again
  }
  // ---- acc = sum over the blocks solved before i*
  d4f acc = {0.0, 0.0, 0.0, 0.0};
  if (nsteps > 1) load_tile(step_block(0));
  for (int t = 0; t + 1 < nsteps; ++t) {
    const Sc1Mem g = granules(step_block(t));
    f64x2 zv[NB * FM_CW / 256];
#pragma unroll
    for (int q = 0; q < NB * FM_CW / 256; ++q) zv[q] = g.ld2(2 * (tid + 256 * q));
    const unsigned long long t0 = spin_clock();
    for (unsigned spins = 0;; ++spins) {  // all four granules polled together
      bool ready = true;
#pragma unroll
      for (int q = 0; q < NB * FM_CW / 256; ++q) ready = ready && __double_as_longlong(zv[q][1]) == (long long)gen;
      if (ready) break;
      if (spin_expired(spins, t0)) {  // bounded wait: never hang the GPU on a scheduling bug
        s_bad = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
#pragma unroll
      for (int q = 0; q < NB * FM_CW / 256; ++q)
        if (__double_as_longlong(zv[q][1]) != (long long)gen) zv[q] = g.ld2(2 * (tid + 256 * q));
    }
#pragma unroll
    for (int q = 0; q < NB * FM_CW / 256; ++q) Zs[tid + 256 * q] = zv[q][0];
    stage_tile();
    __syncthreads();
    if (s_bad) break;
    if (t + 2 < nsteps) load_tile(step_block(t + 1));  // in flight behind this tile's MFMAs
#pragma unroll
    for (int s = 0; s < NB / 4; ++s)
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(tile_a(s), Zs[(4 * s + k4) * FM_CW + (lane & 15)], acc, 0, 0, 0);
    __syncthreads();  // Ls / Zs are rewritten next round
  }
  // ---- V_b = Minv (Y_b - acc)
#pragma unroll
  for (int r = 0; r < 4; ++r) Zs[(16 * w + k4 + 4 * r) * FM_CW + (lane & 15)] = yb[r] - acc[r];
  __syncthreads();
  d4f v = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int s = 0; s < NB / 4; ++s)
    if (minv_nonzero(s))
      v = __builtin_amdgcn_mfma_f64_16x16x4f64(lin[s], Zs[(4 * s + k4) * FM_CW + (lane & 15)], v, 0, 0, 0);
  // ---- the chain step: Z_b = V_b - M_b Z_i*, Z_i*'s B fragments polled straight from its granules (per wave)
  bool bad = s_bad != 0;
  if (nsteps > 0) {
    const Sc1Mem g = granules(istar);
    f64x2 zf[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) zf[s] = g.ld2(2 * ((4 * s + k4) * FM_CW + (lane & 15)));
    const unsigned long long t0 = spin_clock();
    for (unsigned spins = 0; !bad; ++spins) {
      bool ready = true;
#pragma unroll
      for (int s = 0; s < 16; ++s) ready = ready && __double_as_longlong(zf[s][1]) == (long long)gen;
      if (ready) break;
      if (spin_expired(spins, t0)) {
        bad = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
#pragma unroll
      for (int s = 0; s < 16; ++s)
        if (__double_as_longlong(zf[s][1]) != (long long)gen) zf[s] = g.ld2(2 * ((4 * s + k4) * FM_CW + (lane & 15)));
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) v = __builtin_amdgcn_mfma_f64_16x16x4f64(mf[s], zf[s][0], v, 0, 0, 0);
  }
  if (bad) atomicExch(&ctrl->df_status, 2);
  const Sc1Mem gb = granules(b);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = 16 * w + k4 + 4 * r, col = lane & 15;
    gb.st2(2 * (row * FM_CW + col), f64x2{v[r], tag});         // the hand-off granule first
    Y[(size_t)(b * NB + row) * ldy + c * FM_CW + col] = v[r];  // the solution (read after the launch)
  }
}

size_t trsm_many_granule_doubles(int nblk, int nchunk) { return (size_t)nblk * nchunk * NB * FM_CW * 2; }

void launch_trsm_many(hipStream_t s, bool transposed, const double* L, int ld, const double* Linv, double* Y, int ldy,
                      int nblk, int nchunk, double* gran, int gen, DevCtrl* ctrl) {
  if (transposed)
    k_trsm_many<true><<<nblk * nchunk, 256, 0, s>>>(L, ld, Linv, Y, ldy, nblk, nchunk, gran, gen, ctrl);
  else
    k_trsm_many<false><<<nblk * nchunk, 256, 0, s>>>(L, ld, Linv, Y, ldy, nblk, nchunk, gran, gen, ctrl);
}

// ------------------------------------------------------------------------------------------------
// R = B X (KKTSystem.scala:126, :141): B row-major p x ldb, X row-major np x ldx with ncols = p + 1 columns.  64 x 64
// output tiles x row chunks of kch rows of X; each wave a 32 x 32 block (2 x 2 MFMAs, operands straight from L2).
// (An f64 MFMA is a chain of IEEE fused multiply-adds in k order, microbench/mfma_f64_semantics.hip, so each partial
// is the sequential fma sum over its rows.)
// part[(kc * ntile + ti * tjn + tj) * 4096 + r * 64 + cc] = sum_{k in chunk kc} B[64ti+r][k] X[k][64tj+cc]
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_bx_partials(const double* __restrict__ B, int ldb, int p,
                                                     const double* __restrict__ X, int ldx, int ncols, int np, int kch,
                                                     int tjn, int ntile, double* __restrict__ part) {
  const int tile = (int)blockIdx.x % ntile, kc = (int)blockIdx.x / ntile;
  const int ti = tile / tjn, tj = tile - ti * tjn;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, wr = wv >> 1, wc = wv & 1;
  const int k0 = kc * kch, k1 = min(np, k0 + kch);
  int ra[2], cb[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    ra[q] = NB * ti + 32 * wr + 16 * q + (lane & 15);
    cb[q] = NB * tj + 32 * wc + 16 * q + (lane & 15);
  }
  d4f acc[2][2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int nj = 0; nj < 2; ++nj) acc[mi][nj] = d4f{0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
  for (int k = k0 + (lane >> 4); k < k1; k += 4) {
    double fa[2], fb[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      fa[q] = ra[q] < p ? B[(size_t)ra[q] * ldb + k] : 0.0;
      fb[q] = cb[q] < ncols ? X[(size_t)k * ldx + cb[q]] : 0.0;
    }
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int nj = 0; nj < 2; ++nj)
        acc[mi][nj] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[mi], fb[nj], acc[mi][nj], 0, 0, 0);
  }
  double* out = part + ((size_t)kc * ntile + tile) * NB * NB;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int nj = 0; nj < 2; ++nj)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        out[(32 * wr + 16 * mi + (lane >> 4) + 4 * r) * NB + 32 * wc + 16 * nj + (lane & 15)] = acc[mi][nj][r];
}

// R = the row-chunk partials summed in chunk order (row-major p x (p + 1))
__global__ void k_bx_reduce(const double* __restrict__ part, int nk, int tjn, int ntile, int p,
                            double* __restrict__ R) {
  const int ncol = p + 1;
  const int idx = (int)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= p * ncol) return;
  const int i = idx / ncol, j = idx - i * ncol;
  const double* src = part + ((size_t)((i / NB) * tjn + j / NB)) * NB * NB + (i % NB) * NB + (j % NB);
  const size_t stride = (size_t)ntile * NB * NB;
  double sum = 0.0;
#pragma unroll 8
  for (int kc = 0; kc < nk; ++kc) sum += src[kc * stride];
  R[idx] = sum;
}

// S = (R + R')/2 (:139; lower triangle, leading dimension lds; rows p..ps-1 the identity padding of the dataflow
// factorization) and z = -(b + R[:, p]) (:141, zero-padded)
__global__ void k_schur_form(const double* __restrict__ R, int p, int ps, int lds, const double* __restrict__ bvec,
                             double* __restrict__ S, double* __restrict__ z) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (size_t)ps * ps) return;
  const int a = (int)(idx / ps), c = (int)(idx % ps);
  const size_t ncol = (size_t)p + 1;
  if (c <= a) S[(size_t)a * lds + c] = (a < p) ? (R[a * ncol + c] + R[c * ncol + a]) * 0.5 : (a == c ? 1.0 : 0.0);
  if (c == 0) z[a] = (a < p) ? -(bvec[a] + R[a * ncol + p]) : 0.0;
}

static int bx_tjn(int p) { return (p + 1 + NB - 1) / NB; }
static int bx_ntile(int p) { return ((p + NB - 1) / NB) * bx_tjn(p); }
static int bx_chunks(int np, int p) {  // row chunks: >= 64 workgroups where the rows allow, >= 64 rows each
  const int want = (64 + bx_ntile(p) - 1) / bx_ntile(p);
  return std::max(1, std::min(np / NB, want));
}
size_t schur_partial_doubles(int np, int p) {
  return (size_t)bx_chunks(np, p) * bx_ntile(p) * NB * NB + (size_t)p * (p + 1);
}

void launch_schur_form(hipStream_t s, const double* B, int ldb, const double* X, int ldx, int p, int np, double* part,
                       const double* bvec, int ps, int lds, double* S, double* z) {
  const int tjn = bx_tjn(p), ntile = bx_ntile(p), nk = bx_chunks(np, p);
  const int kch = ((np + nk - 1) / nk + 3) & ~3;
  double* R = part + (size_t)nk * ntile * NB * NB;
  k_bx_partials<<<ntile * nk, 256, 0, s>>>(B, ldb, p, X, ldx, p + 1, np, kch, tjn, ntile, part);
  k_bx_reduce<<<(p * (p + 1) + 255) / 256, 256, 0, s>>>(part, nk, tjn, ntile, p, R);
  const size_t cnt = (size_t)ps * ps;
  k_schur_form<<<(unsigned)((cnt + 255) / 256), 256, 0, s>>>(R, p, ps, lds, bvec, S, z);
}

// ------------------------------------------------------------------------------------------------
// w = S^-1 z for p <= 64 in one wave, in the reference's arithmetic:
//  * cholesky(S) = LAPACK dpotrf('L'), which for p <= 64 (its block size) is the unblocked dpotf2: per column j,
//    ajj = S_jj - ddot(L_j,0:j, L_j,0:j); a non-positive (or NaN) ajj fails (chol_info = -1: Breeze's
//    NotConvergedException -> KKTSystem.solve's fallback); the column below is S_ij + sum_l (-L_jl) L_il (dgemv,
//    sequential in l) scaled by 1/ajj (dscal);
//  * forwardSolve(K, z) and backSolve(K', u) (MatrixUtils.scala:383-430): x_i = (b_i - sum_j ...) / diag with the
//    sum sequential in the reference's j order.
// Products are rounded before they are added (-ffp-contract=off), as in the reference's Fortran / Java.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_schur_small(const double* __restrict__ S, int p, const double* __restrict__ z,
                                                    double* __restrict__ w, DevCtrl* ctrl) {
  // One wave; lane i keeps row i in registers.  dpotf2's left-looking sums are formed right-looking: when column l is
  // final, entry (i, j) gains (-L_jl) L_il and lane i's diagonal dot gains L_il^2 -- per entry the same terms in the
  // same order (l ascending) as ddot / dgemv.  Column l reaches the lanes through LDS (broadcast reads); everything is
  // unrolled, so the register indices are static and the updates need no predicates (lanes outside the trailing
  // triangle only write their unused upper part).
  __shared__ double K[NB][NB + 1];
  __shared__ double col[NB];
  const int lane = threadIdx.x;
  double kr[NB];
#pragma unroll
  for (int l = 0; l < NB; ++l) kr[l] = (lane < p && l <= lane) ? S[lane * p + l] : 0.0;
  double sjj = 0.0;  // S_ii (the diagonal takes S_ii - dot, not the dgemv updates)
#pragma unroll
  for (int l = 0; l < NB; ++l)
    if (l == lane) sjj = kr[l];
  double dsum = 0.0;  // ddot(L_i,0:i, L_i,0:i) so far
#pragma unroll
  for (int l = 0; l < NB; ++l) {
    if (l >= p) continue;  // (not break: the loop stays fully unrolled, kr stays in registers)
    double ajj = readlane_d(sjj - dsum, l);
    if (!(ajj > 0.0)) {  // wave-uniform
      if (lane == 0) ctrl->chol_info = -1;
      return;
    }
    ajj = sqrt(ajj);
    const double rinv = 1.0 / ajj;
    const double lil = lane == l ? ajj : rinv * kr[l];
    kr[l] = lil;
    col[lane] = lil;
    __syncthreads();
    dsum = dsum + lil * lil;
#pragma unroll
    for (int j = l + 1; j < NB; ++j) kr[j] = kr[j] + (-col[j]) * lil;
    __syncthreads();
  }
#pragma unroll
  for (int l = 0; l < NB; ++l) K[lane][l] = kr[l];
  // forwardSolve(K, z) (:143): lane i's sum gains K_ij u_j as u_j is broadcast, j ascending
  const double zi = lane < p ? z[lane] : 0.0;
  double sum = 0.0, ui = 0.0;
#pragma unroll
  for (int j = 0; j < NB; ++j)
    if (j < p) {
      if (lane == j) ui = (zi - sum) / kr[j];
      const double uj = readlane_d(ui, j);
      if (lane > j) sum = sum + kr[j] * uj;
    }
  __syncthreads();
  // backSolve(K', u) (:144): U_ij = K_ji, j descending
  sum = 0.0;
  double wi = 0.0;
#pragma unroll
  for (int j = NB - 1; j >= 0; --j)
    if (j < p) {
      if (lane == j) wi = (ui - sum) / kr[j];
      const double wj = readlane_d(wi, j);
      if (lane < j) sum = sum + K[j][lane] * wj;
    }
  if (lane < p) w[lane] = wi;
}

void launch_schur_small(hipStream_t s, const double* S, int p, const double* z, double* w, DevCtrl* ctrl) {
  k_schur_small<<<1, 64, 0, s>>>(S, p, z, w, ctrl);
}

// y = -(X[:, p] + X[:, :p] w)   (KKTSystem.scala:145), one thread per row, the sum over a in the reference's dgemv
// order (sequential, rounded products)
__global__ __launch_bounds__(256) void k_kkt_v(const double* __restrict__ X, int ldx, int p, int np,
                                               const double* __restrict__ w, double* __restrict__ y) {
  const int row = (int)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= np) return;
  const double* xr = X + (size_t)row * ldx;
  double s = 0.0;
  for (int a = 0; a < p; ++a) s = s + xr[a] * w[a];
  y[row] = -(xr[p] + s);
}

void launch_kkt_v(hipStream_t s, const double* X, int ldx, int p, int np, const double* w, double* y) {
  k_kkt_v<<<(np + 255) / 256, 256, 0, s>>>(X, ldx, p, np, w, y);
}

}  // namespace cvxg
