// k_syrk.hip — FP64 MFMA (v_mfma_f64_16x16x4_f64) symmetric rank-k kernels for gfx950.
//
// 1) Barrier Hessian assembly  H = t*P + A' diag(w) A,  w_i = 1/d_i^2
//    (the fold of BarrierSolver.scala:303-315 as ONE weighted SYRK; the reference forms m rank-1
//    outer products G*G.t/(d*d) in list order).  A is row-major m x n, so a contraction chunk of KC
//    constraint rows is KC coalesced 1 KiB row segments per 128-column panel.
// 2) Cholesky trailing update  C -= Pn Pn'  (right-looking blocked dpotrf, MatrixUtils.scala:456).
//
// Tile 128x128, 4 waves as 2x2, each wave a 64x64 block = 4x4 MFMA 16x16 accumulators (64 f64 per lane).
// f64 MFMA operand maps (gfx950): A-frag lane l = A[row l&15][k l>>4], B-frag = B[k l>>4][col l&15],
// C/D reg r of lane l = C[row (l>>4)+4r][col l&15].
#include <stdlib.h>

#include "kernels.hpp"

namespace cvxg {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));

#define MFMA64(a, b, c) __builtin_amdgcn_mfma_f64_16x16x4f64((a), (b), (c), 0, 0, 0)

// [k][col] panel stride: (k*SA + col) mod 32 distinct for the 32 lanes of one ds_read_b64 group.
constexpr int SA = TILE + 16;
// [row][k] panel stride for the trailing update (K chunk 32): (2*row + k) mod 32 distinct.
constexpr int KU = 32;
constexpr int SU = KU + 2;

__device__ __forceinline__ void tile_of(int t, int& I, int& J) {
  int i = 0;
  while ((i + 1) * (i + 2) / 2 <= t) ++i;
  I = i;
  J = t - i * (i + 1) / 2;
}

// ------------------------------------------------------------------------------------------------
// Assembly SYRK.  grid = (ntiles, nsplit); each workgroup owns one lower tile (I,J) and a K range.
// Register-staged double buffering: the next chunk's global loads are issued before the MFMAs of the
// current chunk and written to the other LDS buffer after them (one barrier per chunk).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256, 2) void k_syrk_assemble(const double* __restrict__ A, int lda,
                                                          const double* __restrict__ w, int mp,
                                                          const double* __restrict__ P, const DevCtrl* ctrl,
                                                          double* __restrict__ H, int ldh,
                                                          const int* __restrict__ tiles, int ntiles, int nsplit,
                                                          double* __restrict__ partials) {
  __shared__ __attribute__((aligned(16))) double lds[2][2][KC][SA];
  const int tile = blockIdx.x, split = blockIdx.y;
  const int ij = tiles[tile];
  const int I = ij >> 16, J = ij & 0xffff;
  const bool diag = (I == J);
  const int kchunks = mp / KC;
  const int per = (kchunks + nsplit - 1) / nsplit;
  const int c0 = split * per, c1 = min(kchunks, c0 + per);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const bool active = !(diag && wc > wr);  // strictly-upper 64x64 block of a diagonal tile: skip

  d4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};

  const int colI = I * TILE + lane * 2, colJ = J * TILE + lane * 2;

  // Unconditional, statically indexed staging (a predicated assignment sends the staging registers to
  // scratch); a diagonal tile simply stages panel I twice.  Two register sets (sa, sb) keep loads two
  // chunks ahead of their LDS write, so about 2 x 4096 MFMA cycles of latency are covered.
  const double* srcI = A + colI;
  const double* srcJ = A + colJ;
  // The weights w_k = 1/d_k^2 scale the J panel as it is written to LDS (row k of the slab is wave-uniform:
  // wave `wid` stages rows wid + 4q), so the MFMA loop has no FP64 VALU work.
  auto gload = [&](d2 (&st)[8], double (&wv)[4], int chunk) {
    const size_t k0 = (size_t)min(chunk, kchunks - 1) * KC;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      st[q] = *reinterpret_cast<const d2*>(srcI + (k0 + wid + 4 * q) * lda);
      st[q + 4] = *reinterpret_cast<const d2*>(srcJ + (k0 + wid + 4 * q) * lda);
      wv[q] = w[k0 + wid + 4 * q];
    }
  };
  auto swrite = [&](const d2 (&st)[8], const double (&wv)[4], int buf) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      *reinterpret_cast<d2*>(&lds[buf][0][wid + 4 * q][lane * 2]) = st[q];
      *reinterpret_cast<d2*>(&lds[buf][1][wid + 4 * q][lane * 2]) = st[q + 4] * wv[q];
    }
  };
  auto compute = [&](int buf) {
    if (!active) return;
    const double* PI = &lds[buf][0][0][0];
    const double* PJ = &lds[buf][1][0][0];
#pragma unroll
    for (int s = 0; s < KC / 4; ++s) {
      const int kk = 4 * s + (lane >> 4);
      double fa[4], fb[4];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) fa[mi] = PI[kk * SA + wr * 64 + mi * 16 + (lane & 15)];
#pragma unroll
      for (int nj = 0; nj < 4; ++nj) fb[nj] = PJ[kk * SA + wc * 64 + nj * 16 + (lane & 15)];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int nj = 0; nj < 4; ++nj) acc[mi][nj] = MFMA64(fa[mi], fb[nj], acc[mi][nj]);
    }
  };

  d2 sa[8], sb[8];
  double wa[4], wb[4];
  gload(sa, wa, c0);
  swrite(sa, wa, 0);
  gload(sb, wb, c0 + 1);
  __syncthreads();
  for (int c = c0; c < c1; c += 2) {
    gload(sa, wa, c + 2);
    compute(0);
    swrite(sb, wb, 1);
    __syncthreads();
    if (c + 1 >= c1) break;
    gload(sb, wb, c + 3);
    compute(1);
    swrite(sa, wa, 0);
    __syncthreads();
  }
  if (!active) return;

  if (nsplit == 1) {
    const double t = ctrl->t;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int nj = 0; nj < 4; ++nj)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int li = wr * 64 + mi * 16 + (lane >> 4) + 4 * r;
          const int lj = wc * 64 + nj * 16 + (lane & 15);
          if (diag && lj > li) continue;
          const int gi = I * TILE + li, gj = J * TILE + lj;
          // fold starts at objF.hessianAt(x)*t (BarrierSolver.scala:304); lower entry mirrored so H is
          // exactly symmetric (the reference's Breeze cholesky checks symmetry).
          const double v = (P ? P[(size_t)gi * ldh + gj] * t : 0.0) + acc[mi][nj][r];
          H[(size_t)gi * ldh + gj] = v;
          if (gi != gj) H[(size_t)gj * ldh + gi] = v;
        }
  } else {
    double* out = partials + ((size_t)split * ntiles + tile) * (TILE * TILE);
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int nj = 0; nj < 4; ++nj)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int li = wr * 64 + mi * 16 + (lane >> 4) + 4 * r;
          const int lj = wc * 64 + nj * 16 + (lane & 15);
          out[li * TILE + lj] = acc[mi][nj][r];
        }
  }
}

// ------------------------------------------------------------------------------------------------
// Assembly SYRK, register-direct form: no LDS and no barriers.  Each wave streams its own MFMA operands
// from L2 (all resident tiles walk the same k-slab of A, so the slab is L2-resident) with 16-B loads kept
// SYRK_DEPTH k-steps ahead.  Lane l of a k-step loads row k0 + (l >> 4), columns 2 (l & 15) + {0, 1} (+ 32):
// exactly the f64 MFMA A/B fragment map (lane l = (row l & 15, k l >> 4)) for four column-interleaved 16-wide
// blocks, block mi = 2h + e covering tile columns 32 h + 2 r + e.  The epilogue undoes the interleave.
// ------------------------------------------------------------------------------------------------
template <int SYRK_DEPTH>
__global__ __launch_bounds__(256, 2) void k_syrk_direct(const double* __restrict__ A, int lda,
                                                        const double* __restrict__ w, int mp,
                                                        const double* __restrict__ P, const DevCtrl* ctrl,
                                                        double* __restrict__ H, int ldh,
                                                        const int* __restrict__ tiles, int ntiles, int nsplit,
                                                        double* __restrict__ partials) {
  const int tile = blockIdx.x, split = blockIdx.y;
  const int ij = tiles[tile];
  const int I = ij >> 16, J = ij & 0xffff;
  const bool diag = (I == J);
  const int kchunks = mp / KC;
  const int per = (kchunks + nsplit - 1) / nsplit;
  const int c0 = split * per, c1 = min(kchunks, c0 + per);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  if (diag && wc > wr) return;  // strictly-upper 64x64 block of a diagonal tile (no barriers in this kernel)
  const int nsteps = (c1 > c0) ? (c1 - c0) * (KC / 4) : 0;

  d4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};

  const int lk = lane >> 4, l15 = lane & 15;
  const size_t kbase = (size_t)c0 * KC + lk;
  const double* pI = A + kbase * lda + I * TILE + wr * 64 + 2 * l15;
  const double* pJ = A + kbase * lda + J * TILE + wc * 64 + 2 * l15;
  const double* pw = w + kbase;
  struct Op {
    d2 a0, a1, b0, b1;
    double wk;
  };
  auto load = [&](Op& o, int st) {
    st = min(st, max(nsteps - 1, 0));
    const size_t off = (size_t)(4 * st) * lda;
    o.a0 = *reinterpret_cast<const d2*>(pI + off);
    o.a1 = *reinterpret_cast<const d2*>(pI + off + 32);
    o.b0 = *reinterpret_cast<const d2*>(pJ + off);
    o.b1 = *reinterpret_cast<const d2*>(pJ + off + 32);
    o.wk = pw[4 * st];
  };
  Op buf[SYRK_DEPTH];
  if (nsteps > 0) {
#pragma unroll
    for (int d = 0; d < SYRK_DEPTH; ++d) {
      load(buf[d], d);  // in stage order, as in the loop: the loop-header wait then needs only stage 0
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  static_assert((KC / 4) % SYRK_DEPTH == 0 || SYRK_DEPTH % (KC / 4) == 0, "depth vs chunk");
  for (int s0 = 0; s0 < nsteps; s0 += SYRK_DEPTH) {  // nsteps is a multiple of KC / 4 (and of SYRK_DEPTH)
#pragma unroll
    for (int d = 0; d < SYRK_DEPTH; ++d) {
      const Op& o = buf[d];
      const double fa[4] = {o.a0[0], o.a0[1], o.a1[0], o.a1[1]};
      const double fb[4] = {o.b0[0] * o.wk, o.b0[1] * o.wk, o.b1[0] * o.wk, o.b1[1] * o.wk};
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int nj = 0; nj < 4; ++nj) acc[mi][nj] = MFMA64(fa[mi], fb[nj], acc[mi][nj]);
      // pin the order: the refill of this stage is issued after its MFMAs and is not sunk to its use
      // SYRK_DEPTH - 1 steps later (the scheduler otherwise moves loads next to their consumers)
      __builtin_amdgcn_sched_barrier(0);
      load(buf[d], s0 + d + SYRK_DEPTH);
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  // acc[mi][nj] reg r of lane l: MFMA (row R = (l >> 4) + 4 r, col C = l & 15) -> tile (li, lj) below
  const double t = ctrl->t;
  double* out = (nsplit == 1) ? nullptr : partials + ((size_t)split * ntiles + tile) * (TILE * TILE);
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int nj = 0; nj < 4; ++nj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int li = wr * 64 + 32 * (mi >> 1) + 2 * (lk + 4 * r) + (mi & 1);
        const int lj = wc * 64 + 32 * (nj >> 1) + 2 * l15 + (nj & 1);
        if (out) {
          out[li * TILE + lj] = acc[mi][nj][r];
          continue;
        }
        if (diag && lj > li) continue;
        const int gi = I * TILE + li, gj = J * TILE + lj;
        const double v = (P ? P[(size_t)gi * ldh + gj] * t : 0.0) + acc[mi][nj][r];
        H[(size_t)gi * ldh + gj] = v;
        if (gi != gj) H[(size_t)gj * ldh + gi] = v;
      }
}

// Split-K reduce: H = t*P + sum_splits partial (fixed split order), lower entries mirrored.
__global__ __launch_bounds__(TILE) void k_syrk_reduce(const double* __restrict__ partials, int ntiles, int nsplit,
                                                      const int* __restrict__ tiles, const double* __restrict__ P,
                                                      const DevCtrl* ctrl, double* __restrict__ H, int ldh) {
  const int tile = blockIdx.x, li = blockIdx.y, lj = threadIdx.x;
  const int ij = tiles[tile];
  const int I = ij >> 16, J = ij & 0xffff;
  if (I == J && lj > li) return;
  double s = 0.0;
  for (int sp = 0; sp < nsplit; ++sp) s += partials[((size_t)sp * ntiles + tile) * (TILE * TILE) + li * TILE + lj];
  const int gi = I * TILE + li, gj = J * TILE + lj;
  const double v = (P ? P[(size_t)gi * ldh + gj] * ctrl->t : 0.0) + s;
  H[(size_t)gi * ldh + gj] = v;
  if (gi != gj) H[(size_t)gj * ldh + gi] = v;
}

void launch_syrk_assemble(hipStream_t s, const double* A, int lda, const double* w, int mp, const double* P,
                          const DevCtrl* ctrl, double* H, int ldh, TileList tiles, int nsplit, double* partials) {
  static int direct = -1;  // CVXG_SYRK_DIRECT: 0 = LDS-staged kernel, else the prefetch depth of the direct one
  if (direct < 0) {
    const char* e = getenv("CVXG_SYRK_DIRECT");
    direct = e ? atoi(e) : 4;
  }
  dim3 grid(tiles.count, nsplit);
  if (direct == 2)
    k_syrk_direct<2><<<grid, 256, 0, s>>>(A, lda, w, mp, P, ctrl, H, ldh, tiles.ij, tiles.count, nsplit, partials);
  else if (direct != 0)
    k_syrk_direct<4><<<grid, 256, 0, s>>>(A, lda, w, mp, P, ctrl, H, ldh, tiles.ij, tiles.count, nsplit, partials);
  else
    k_syrk_assemble<<<grid, 256, 0, s>>>(A, lda, w, mp, P, ctrl, H, ldh, tiles.ij, tiles.count, nsplit, partials);
  if (nsplit > 1) {
    dim3 g2(tiles.count, TILE);
    k_syrk_reduce<<<g2, TILE, 0, s>>>(partials, tiles.count, nsplit, tiles.ij, P, ctrl, H, ldh);
  }
}

// ------------------------------------------------------------------------------------------------
// Cholesky trailing update on the lower tiles of C[r0:np, r0:np], r0 = k0 + NB, panel Pn = C[r0:, k0:k0+NB].
// Two K chunks of 32, single-buffered [row][k] LDS panels (2 workgroups per CU overlap each other's loads).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256, 2) void k_syrk_update(double* __restrict__ C, int ld, int np, int k0,
                                                        const DevCtrl* ctrl) {
  if (ctrl->chol_info != 0) return;
  __shared__ __attribute__((aligned(16))) double pi_[TILE][SU];
  __shared__ __attribute__((aligned(16))) double pj_[TILE][SU];
  const int r0 = k0 + NB;
  int I, J;
  tile_of(blockIdx.x, I, J);
  const bool diag = (I == J);
  const int rowI = r0 + I * TILE, rowJ = r0 + J * TILE;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const bool active = !(diag && wc > wr);

  d4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = d4{0.0, 0.0, 0.0, 0.0};

  const int lr = tid >> 4;        // 0..15
  const int lc = (tid & 15) * 2;  // 0..30
  for (int kc = 0; kc < NB; kc += KU) {
    d2 si[8], sj[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int row = lr + 16 * q;
      const int gi = rowI + row, gj = rowJ + row;
      // clamped unconditional loads + selects keep si/sj in registers (no scratch)
      const d2 vi = *reinterpret_cast<const d2*>(C + (size_t)min(gi, np - 1) * ld + k0 + kc + lc);
      const d2 vj = *reinterpret_cast<const d2*>(C + (size_t)min(gj, np - 1) * ld + k0 + kc + lc);
      si[q] = gi < np ? vi : d2{0.0, 0.0};
      sj[q] = gj < np ? vj : d2{0.0, 0.0};
    }
    if (kc) __syncthreads();
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int row = lr + 16 * q;
      *reinterpret_cast<d2*>(&pi_[row][lc]) = si[q];
      *reinterpret_cast<d2*>(&pj_[row][lc]) = sj[q];
    }
    __syncthreads();
    if (active) {
      const double* PI = &pi_[0][0];
      const double* PJ = diag ? PI : &pj_[0][0];
#pragma unroll
      for (int s = 0; s < KU / 4; ++s) {
        const int kk = 4 * s + (lane >> 4);
        double fa[4], fb[4];
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) fa[mi] = PI[(wr * 64 + mi * 16 + (lane & 15)) * SU + kk];
#pragma unroll
        for (int nj = 0; nj < 4; ++nj) fb[nj] = PJ[(wc * 64 + nj * 16 + (lane & 15)) * SU + kk];
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int nj = 0; nj < 4; ++nj) acc[mi][nj] = MFMA64(fa[mi], fb[nj], acc[mi][nj]);
      }
    }
  }
  if (!active) return;
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int nj = 0; nj < 4; ++nj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int li = wr * 64 + mi * 16 + (lane >> 4) + 4 * r;
        const int lj = wc * 64 + nj * 16 + (lane & 15);
        const int gi = rowI + li, gj = rowJ + lj;
        if (gi >= np || gj > gi) continue;
        C[(size_t)gi * ld + gj] -= acc[mi][nj][r];
      }
}

void launch_syrk_update(hipStream_t s, double* C, int ld, int np, int k0, const DevCtrl* ctrl) {
  const int r0 = k0 + NB;
  if (r0 >= np) return;
  const int nt = (np - r0 + TILE - 1) / TILE;
  k_syrk_update<<<nt * (nt + 1) / 2, 256, 0, s>>>(C, ld, np, k0, ctrl);
}

}  // namespace cvxg
