// ruiz_tile.hpp — the per-tile arithmetic of a Ruiz sweep (MatrixUtils.scala:240-268) over the lower triangle, shared
// by the multi-launch form (k_vec.hip: k_ruiz_tiles) and the one-launch loop (k_ruiz.hip), so both give the same bits.
//
// Thread layout of a 64 x 64 tile (256 threads): c2 = tid & 31 holds columns 2 c2, 2 c2 + 1; g = tid >> 5 holds rows
// g + 8 q, q = 0..7.  Row partial of row r: sum_c (d_c H_rc)^2, the thread pair's two squares, then the 32 lanes of
// its row group added with DPP (quad_perm, row_half_mirror, row_mirror within each 16-lane row, row_bcast:15 across
// the two rows): the total sits in lane c2 == 16 (RZ_ROW_LANE).  Column partial of column c: sum over the tile's rows
// of (d_r H_rc)^2 -- each thread's 8 rows as an fma chain, then the 8 row groups in order g = 0..7 through LDS.
#pragma once
#include "common.hpp"

namespace cvxg {

constexpr int RZ_ROW_LANE = 16;  // (tid & 31) of the lanes that hold a row group's total

template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ double rz_dppd(double v) {  // a 64-bit DPP move as two 32-bit ones (lanes masked off: 0)
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, ROW_MASK, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, ROW_MASK, 0xf, false);
  return __hiloint2double(hi, lo);
}

// the sum over the 32 lanes of v's row group (lanes 0-31 or 32-63 of the wave), valid at (lane & 31) >= 16
__device__ __forceinline__ double rz_rowgroup_sum(double v) {
  v = v + rz_dppd<0xB1>(v);        // quad_perm [1,0,3,2]
  v = v + rz_dppd<0x4E>(v);        // quad_perm [2,3,0,1]
  v = v + rz_dppd<0x141>(v);       // row_half_mirror
  v = v + rz_dppd<0x140>(v);       // row_mirror: every lane of a 16-lane row holds the row's sum
  return v + rz_dppd<0x142, 0xA>(v);  // row_bcast:15 into rows 1 and 3: + the other row's sum
}

// eight independent row-group sums, level by level so their DPP chains interleave
__device__ __forceinline__ void rz_rowgroup_sum8(double (&v)[8]) {
#pragma unroll
  for (int q = 0; q < 8; ++q) v[q] = v[q] + rz_dppd<0xB1>(v[q]);
#pragma unroll
  for (int q = 0; q < 8; ++q) v[q] = v[q] + rz_dppd<0x4E>(v[q]);
#pragma unroll
  for (int q = 0; q < 8; ++q) v[q] = v[q] + rz_dppd<0x141>(v[q]);
#pragma unroll
  for (int q = 0; q < 8; ++q) v[q] = v[q] + rz_dppd<0x140>(v[q]);
#pragma unroll
  for (int q = 0; q < 8; ++q) v[q] = v[q] + rz_dppd<0x142, 0xA>(v[q]);
}

}  // namespace cvxg
