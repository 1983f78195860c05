// potrf64.hpp — building blocks of the 64 x 64 diagonal-block Cholesky (dpotrf 'L' semantics,
// MatrixUtils.scala:452-461 via Breeze cholesky) and of the dataflow tile tasks, sized by the measured gfx950
// latencies (microbench/lat.hip: v_readlane f64 ~44 cycles, rsq + 2 Newton ~50, FP64 FMA ~5, FP64 MFMA 16x16x4
// 64 cycles, LDS store->load ~130): the Newton-refined reciprocal / rsqrt, the f64 lane broadcast, buffer
// descriptors with plain or sc1 (inter-workgroup hand-off) accesses, the 16 x 16 MFMA products on LDS operands.
// The factorization itself is potrf64w.hpp (wave-specialised); the round-1 barrier-per-step form it replaced is
// kept as the A/B reference of microbench/potrf64_bench.hip (microbench/potrf64_ref.hpp).
#pragma once
#include <math.h>

#include "kernels.hpp"

namespace cvxg {

typedef double d4f __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int AUX_SC1 = 16;  // cache-policy bits of a buffer access: sc1 (L1 bypass, write-through)

__device__ __forceinline__ double rsqrt_nr(double p) {
  double y = __builtin_amdgcn_rsq(p);
  const double h = 0.5 * p;
  y = y * (1.5 - h * y * y);
  y = y * (1.5 - h * y * y);
  return y;
}

__device__ __forceinline__ double rcp_nr(double p) {
  double y = __builtin_amdgcn_rcp(p);
  y = y * (2.0 - p * y);
  y = y * (2.0 - p * y);
  return y;
}

__device__ __forceinline__ double readlane_d(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

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

// Memory policies over one region (a tile, a rhs block), addressed by double offsets.
//   PlainMem: ordinary cached accesses (kernel boundaries order everything).
//   Sc1Mem:   buffer_load/store ... sc1 — the inter-workgroup hand-off form used inside one launch
//             (MI355X_MICROARCH.md, visibility: Valid forms, row 1).
struct PlainMem {
  double* p;
  __device__ PlainMem(double* base, unsigned) : p(base) {}
  __device__ __forceinline__ double ld(int off) const { return p[off]; }
  __device__ __forceinline__ void st(int off, double v) const { p[off] = v; }
  __device__ __forceinline__ f64x2 ld2(int off) const { return *reinterpret_cast<const f64x2*>(p + off); }
  __device__ __forceinline__ void st2(int off, f64x2 v) const { *reinterpret_cast<f64x2*>(p + off) = v; }
};
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
  __device__ __forceinline__ void st2(int off, f64x2 v) const {  // 16 B, off even
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off * 8, 0, AUX_SC1);
  }
};

// bytes spanned by a 64 x 64 tile with leading dimension ld (for a tile descriptor)
__host__ __device__ constexpr unsigned tile_bytes(int ld) { return (unsigned)((NB - 1) * ld + NB) * 8u; }

// ---- 16 x 16 MFMA building blocks on LDS operands (f64 16x16x4: A lane l = (row l&15, k l>>4), B lane l =
// (k l>>4, col l&15), C/D lane l reg i = (row (l>>4) + 4i, col l&15)) ----------------------------------------
// acc += sgn * A B^T with A, B row-major 16 x 16 (B^T: the row of B is the column of the product)
__device__ __forceinline__ d4f mfma16_abt(d4f acc, const double* a, int lda, const double* b, int ldb, double sgn,
                                          int lane) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int k = 4 * s + (lane >> 4);
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(sgn * a[(lane & 15) * lda + k], b[(lane & 15) * ldb + k], acc, 0, 0, 0);
  }
  return acc;
}
// acc += sgn * A B with A, B row-major
__device__ __forceinline__ d4f mfma16_ab(d4f acc, const double* a, int lda, const double* b, int ldb, double sgn,
                                         int lane) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int k = 4 * s + (lane >> 4);
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(sgn * a[(lane & 15) * lda + k], b[k * ldb + (lane & 15)], acc, 0, 0, 0);
  }
  return acc;
}
__device__ __forceinline__ d4f c16_load(const double* c, int ldc, int lane) {
  d4f v;
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = c[((lane >> 4) + 4 * i) * ldc + (lane & 15)];
  return v;
}
__device__ __forceinline__ void c16_store(double* c, int ldc, d4f v, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) c[((lane >> 4) + 4 * i) * ldc + (lane & 15)] = v[i];
}

#ifdef POTRF_STAMPS  // microbench/potrf64_bench.hip: per-wave s_memtime stamps of the phases
__device__ unsigned long long g_potrf_stamps[4][64];
#define P64_STAMP(i)                                                          \
  do {                                                                        \
    if (lane == 0) g_potrf_stamps[w][(i)] = __builtin_amdgcn_s_memtime();     \
  } while (0)
#else
#define P64_STAMP(i) \
  do {               \
  } while (0)
#endif

constexpr int P64_SP = NB + 2;  // LDS row stride (doubles) of the 64 x 64 work arrays: conflict-free fragments
constexpr int P64_EP = 16 + 2;  // row stride of the 16 x 16 L16^-T blocks

// fix() hook of the factorizations (potrf64w.hpp): runs between the factorization and the forward solve
struct NoFix {
  __device__ bool operator()() const { return true; }
};
// pre(w, lane) hook (potrf64w.hpp): waves 1..3 run it first, while wave 0 starts the first sweep
struct NoPre {
  __device__ void operator()(int, int) const {}
};

}  // namespace cvxg
