// k_syrk.hip — FP64 MFMA (v_mfma_f64_16x16x4_f64) symmetric rank-k kernels for gfx950.
//
// 1) Barrier Hessian assembly  H = t*P + A' diag(w) A,  w_i = 1/d_i^2
//    (the fold of BarrierSolver.scala:303-315 as ONE weighted SYRK; the reference forms m rank-1
//    outer products G*G.t/(d*d) in list order).  A is row-major m x n, so a contraction chunk of KC
//    constraint rows is KC coalesced 1 KiB row segments per 128-column panel.
//
// Tile 128x128, 4 waves as 2x2, each wave a 64x64 block = 4x4 MFMA 16x16 accumulators (64 f64 per lane).
// f64 MFMA operand maps (gfx950): A-frag lane l = A[row l&15][k l>>4], B-frag = B[k l>>4][col l&15],
// C/D reg r of lane l = C[row (l>>4)+4r][col l&15].
#include "kernels.hpp"

namespace cvxg {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));

#define MFMA64(a, b, c) __builtin_amdgcn_mfma_f64_16x16x4f64((a), (b), (c), 0, 0, 0)

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
                                                        double* __restrict__ partials,
                                                        const double* __restrict__ Pd, int mirror) {
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
        const double v = (P ? P[(size_t)gi * ldh + gj] * t : (Pd && gi == gj ? Pd[gi] * t : 0.0)) + acc[mi][nj][r];
        H[(size_t)gi * ldh + gj] = v;
        if (gi != gj && (mirror || diag)) H[(size_t)gj * ldh + gi] = v;
      }
}

// Split-K reduce: H = t*P + sum_splits partial (fixed split order), lower entries mirrored (all, or those of diagonal
// tiles only).
__global__ __launch_bounds__(TILE) void k_syrk_reduce(const double* __restrict__ partials, int ntiles, int nsplit,
                                                      const int* __restrict__ tiles, const double* __restrict__ P,
                                                      const DevCtrl* ctrl, double* __restrict__ H, int ldh,
                                                      const double* __restrict__ Pd, int mirror) {
  const int tile = blockIdx.x, li = blockIdx.y, lj = threadIdx.x;
  const int ij = tiles[tile];
  const int I = ij >> 16, J = ij & 0xffff;
  if (I == J && lj > li) return;
  double s = 0.0;
  for (int sp = 0; sp < nsplit; ++sp) s += partials[((size_t)sp * ntiles + tile) * (TILE * TILE) + li * TILE + lj];
  const int gi = I * TILE + li, gj = J * TILE + lj;
  const double v = (P ? P[(size_t)gi * ldh + gj] * ctrl->t : (Pd && gi == gj ? Pd[gi] * ctrl->t : 0.0)) + s;
  H[(size_t)gi * ldh + gj] = v;
  if (gi != gj && (mirror || I == J)) H[(size_t)gj * ldh + gi] = v;
}

void launch_syrk_assemble(hipStream_t s, const double* A, int lda, const double* w, int mp, const double* P,
                          const DevCtrl* ctrl, double* H, int ldh, TileList tiles, int nsplit, double* partials,
                          const double* Pd, bool mirror) {
  dim3 grid(tiles.count, nsplit);
  k_syrk_direct<4><<<grid, 256, 0, s>>>(A, lda, w, mp, P, ctrl, H, ldh, tiles.ij, tiles.count, nsplit, partials, Pd,
                                        mirror ? 1 : 0);
  if (nsplit > 1) {
    dim3 g2(tiles.count, TILE);
    k_syrk_reduce<<<g2, TILE, 0, s>>>(partials, tiles.count, nsplit, tiles.ij, P, ctrl, H, ldh, Pd, mirror ? 1 : 0);
  }
}

}  // namespace cvxg
