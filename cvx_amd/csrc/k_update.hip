// k_update.hip — FP64 MFMA kernels of the two-level blocked Cholesky (right-looking dpotrf('L'),
// MatrixUtils.scala:452-461): the panel TRSM L21 = A21 L_kk^-T and the rank-kw updates
//   C[r, c] -= sum_{k in [k0, k0+kw)} L[r][k] L[c][k]      (r >= c, r in [r0, np), c in [c0, c1))
// used both for the narrow in-panel updates (kw = 64) and for the trailing update after a 256-wide outer
// panel (kw = 256: four times fewer read-modify-write passes over the trailing matrix than NB = 64).
#include "kernels.hpp"

namespace cvxg {

typedef double d4u __attribute__((ext_vector_type(4)));
typedef double d2u __attribute__((ext_vector_type(2)));

#define MFMA64U(a, b, c) __builtin_amdgcn_mfma_f64_16x16x4f64((a), (b), (c), 0, 0, 0)

// ------------------------------------------------------------------------------------------------
// Panel TRSM by MFMA:  X = A21 Linv_kk^T  for rows i in [(k+1)*NB, np), written in place of A21.
// One wave = 16 rows x 64 columns (4 accumulator tiles), operands straight from L2 (A21 rows are read
// once; Linv_kk is 32 KB and shared by every wave).  Fused forward substitution: rhs[i] -= X[i,:] w_k.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_trsm_mfma(double* __restrict__ L, int ld, int np, int k,
                                                   double* __restrict__ rhs, int nrhs,
                                                   const double* __restrict__ Linv, const DevCtrl* ctrl) {
  if (ctrl->chol_info != 0) return;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int base = k * NB;
  const int r0 = base + NB + (blockIdx.x * 4 + wid) * 16;
  if (r0 >= np) return;
  const double* li = Linv + (size_t)k * NB * NB;
  const int ar = min(r0 + (lane & 15), np - 1);
  const double* arow = L + (size_t)ar * ld + base;
  d4u acc[4];
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) acc[ct] = d4u{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int ks = 0; ks < NB / 4; ++ks) {
    const int kk = 4 * ks + (lane >> 4);
    const double a = arow[kk];  // A21[r0 + (l&15)][kk]
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      const double b = li[(16 * ct + (lane & 15)) * NB + kk];  // B[kk][c] = Linv[c][kk]
      acc[ct] = MFMA64U(a, b, acc[ct]);
    }
  }
  // C/D: reg r of lane l -> row (l>>4) + 4r, col 16ct + (l&15)
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = r0 + (lane >> 4) + 4 * r;
      if (row < np) L[(size_t)row * ld + base + 16 * ct + (lane & 15)] = acc[ct][r];
    }
#pragma unroll
  for (int rho = 0; rho < MAX_RHS; ++rho) {
    if (rho >= nrhs) break;
    double bw[4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) bw[ct] = rhs[(size_t)(base + 16 * ct + (lane & 15)) * nrhs + rho];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      double s = acc[0][r] * bw[0];
#pragma unroll
      for (int ct = 1; ct < 4; ++ct) s = fma(acc[ct][r], bw[ct], s);
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      s += __shfl_xor(s, 4, 64);
      s += __shfl_xor(s, 8, 64);
      const int row = r0 + (lane >> 4) + 4 * r;
      if ((lane & 15) == 0 && row < np) rhs[(size_t)row * nrhs + rho] -= s;
    }
  }
}

void launch_trsm_mfma(hipStream_t s, double* L, int ld, int np, int k, double* rhs, int nrhs, const double* Linv,
                      const DevCtrl* ctrl) {
  const int rows = np - (k + 1) * NB;
  if (rows <= 0) return;
  k_trsm_mfma<<<(rows + 63) / 64, 256, 0, s>>>(L, ld, np, k, rhs, nrhs, Linv, ctrl);
}

// ------------------------------------------------------------------------------------------------
// Region update C[r0:np, c0:c1] (lower part) -= P_r P_c^T over contraction columns [k0, k0+kw).
// 128x128 tiles on a rectangular grid (tiles wholly above the diagonal exit at once), 4 waves as 2x2,
// K in chunks of 32 through [row][k] LDS panels with stride 34 (conflict-free f64 fragment reads),
// register-staged so the next chunk's loads are in flight during the current chunk's MFMAs.
// ------------------------------------------------------------------------------------------------
// Buffer descriptor from values the compiler can see are wave-uniform (otherwise every buffer op is
// wrapped in a readfirstlane waterfall loop).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const double* base, int bytes) {
  const unsigned long long a = reinterpret_cast<unsigned long long>(base);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  const int nb = __builtin_amdgcn_readfirstlane(bytes);
  void* p = reinterpret_cast<void*>(((unsigned long long)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(p, 0, nb, 0x00020000);
}

constexpr int UKC = 32;
constexpr int USTR = UKC + 2;

__global__ __launch_bounds__(256, 2) void k_chol_update(double* __restrict__ C, int ld, int np, int k0, int kw,
                                                        int r0, int c0, int c1, int ncol_tiles,
                                                        const DevCtrl* ctrl) {
  if (ctrl->chol_info != 0) return;
  __shared__ __attribute__((aligned(16))) double pi_[TILE][USTR];
  __shared__ __attribute__((aligned(16))) double pj_[TILE][USTR];
  const int I = blockIdx.x / ncol_tiles, J = blockIdx.x % ncol_tiles;
  const int rowI = r0 + I * TILE, colJ = c0 + J * TILE;
  if (rowI + TILE - 1 < colJ) return;  // tile strictly above the diagonal
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const bool active = !(rowI + wr * 64 + 63 < colJ + wc * 64);  // wave block strictly upper: skip MFMAs

  d4u acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = d4u{0.0, 0.0, 0.0, 0.0};

  const int lr = tid >> 4;        // 0..15
  const int lc = (tid & 15) * 2;  // 0..30
  // Buffer loads through per-tile descriptors: rows past np (or past c1 for the column operand) fall outside
  // the descriptor range and read as zero, and the per-lane address is one 32-bit voffset (the row stride
  // q*16*ld goes to the scalar soffset), which keeps the 64 staging registers + 128 accumulators spill-free.
  const int rows_i = min(TILE, np - rowI), rows_j = max(0, min(TILE, min(np, c1) - colJ));
  const __amdgpu_buffer_rsrc_t ri = uniform_rsrc(C + (size_t)rowI * ld + k0, rows_i * ld * 8);
  const __amdgpu_buffer_rsrc_t rj = uniform_rsrc(C + (size_t)min(colJ, np - 1) * ld + k0, rows_j * ld * 8);
  const int voff = (lr * ld + lc) * 8;
  d2u si[8], sj[8];
  auto gload = [&](int kc) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int soff = (16 * q * ld + kc) * 8;
      si[q] = __builtin_bit_cast(d2u, __builtin_amdgcn_raw_buffer_load_b128(ri, voff, soff, 0));
      sj[q] = __builtin_bit_cast(d2u, __builtin_amdgcn_raw_buffer_load_b128(rj, voff, soff, 0));
    }
  };
  // single-buffered LDS (69.6 KB: two workgroups per CU overlap each other's loads); the next chunk is
  // fetched into registers while the current one feeds the MFMAs.
  const int nch = kw / UKC;
  gload(0);
  for (int ch = 0; ch < nch; ++ch) {
    if (ch) __syncthreads();
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int row = lr + 16 * q;
      *reinterpret_cast<d2u*>(&pi_[row][lc]) = si[q];
      *reinterpret_cast<d2u*>(&pj_[row][lc]) = sj[q];
    }
    __syncthreads();
    if (ch + 1 < nch) gload((ch + 1) * UKC);
    if (active) {
      const double* PI = &pi_[0][0];
      const double* PJ = &pj_[0][0];
#pragma unroll
      for (int s = 0; s < UKC / 4; ++s) {
        const int kk = 4 * s + (lane >> 4);
        double fa[4], fb[4];
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) fa[mi] = PI[(wr * 64 + mi * 16 + (lane & 15)) * USTR + kk];
#pragma unroll
        for (int nj = 0; nj < 4; ++nj) fb[nj] = PJ[(wc * 64 + nj * 16 + (lane & 15)) * USTR + kk];
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int nj = 0; nj < 4; ++nj) acc[mi][nj] = MFMA64U(fa[mi], fb[nj], acc[mi][nj]);
      }
    }
  }
  if (!active) return;
  // epilogue: read-modify-write of the tile, 16 loads in flight per row group (rows >= np read as zero
  // through the descriptor; stores are predicated to the lower part of [c0, c1)).
  const __amdgpu_buffer_rsrc_t rc = uniform_rsrc(C + (size_t)rowI * ld, rows_i * ld * 8);
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
    double old[4][4];
    const int li0 = wr * 64 + mi * 16 + (lane >> 4);
#pragma unroll
    for (int nj = 0; nj < 4; ++nj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int lj = colJ + wc * 64 + nj * 16 + (lane & 15);
        old[nj][r] = __builtin_bit_cast(
            double, __builtin_amdgcn_raw_buffer_load_b64(rc, ((li0 + 4 * r) * ld + lj) * 8, 0, 0));
      }
#pragma unroll
    for (int nj = 0; nj < 4; ++nj)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gi = rowI + li0 + 4 * r;
        const int gj = colJ + wc * 64 + nj * 16 + (lane & 15);
        if (gi < np && gj < c1 && gj <= gi) C[(size_t)gi * ld + gj] = old[nj][r] - acc[mi][nj][r];
      }
  }
}

void launch_chol_update(hipStream_t s, double* C, int ld, int np, int k0, int kw, int r0, int c0, int c1,
                        const DevCtrl* ctrl) {
  if (r0 >= np || c0 >= c1 || kw <= 0) return;
  const int nI = (np - r0 + TILE - 1) / TILE;
  const int nJ = (c1 - c0 + TILE - 1) / TILE;
  k_chol_update<<<nI * nJ, 256, 0, s>>>(C, ld, np, k0, kw, r0, c0, c1, nJ, ctrl);
}

}  // namespace cvxg
