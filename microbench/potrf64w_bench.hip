// Microbenchmark of the wave-specialised 64x64 diagonal-block Cholesky (potrf64w.hpp) in isolation: correctness against a
// host Cholesky / inverse / forward solve, kernel time via hipEvents over many launches on fresh copies,
// and per-wave phase stamps (built with -DPOTRF_STAMPS).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DPOTRF_STAMPS microbench/potrf64w_bench.hip -o microbench/potrf64w_bench
// -DWITH_LFLAG: progressive L^-1 stores + flag (the chain's form); -Icvx_amd/csrc -DPOTRF_HDR='"potrf64w_dpp.hpp"': the
// round-5 DPP column-sweep variant (microbench/potrf64w_dpp.hpp, measured and rejected: DESIGN.md §7);
// -DP64_DPP_ON=true: potrf64w's own DPP sweep (same structure as the v_readlane sweep, bitwise the same factor)
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#ifndef P64_DPP_ON
#define P64_DPP_ON false  // -DP64_DPP_ON=true: the DPP column sweep (potrf64w.hpp p64w_eliminate_dpp)
#endif
#ifndef POTRF_HDR
#define POTRF_HDR "../cvx_amd/csrc/potrf64w.hpp"
#endif
#include POTRF_HDR
namespace cvxg {
__device__ int g_lflag;  // -DWITH_LFLAG: the progressive L^-1 row-block stores and flag of the chain's POTRF
__device__ double* g_src;  // pristine copy of the tile (warm-I$ repetition)
__device__ int g_reps = 1;
__global__ __launch_bounds__(256) void k_p64(double* L, int ld, int k, double* rhs, int nrhs, double* Linv, DevCtrl* ctrl) {
  __shared__ __attribute__((aligned(16))) Potrf64wSmem sm;
  for (int rep = 0; rep < g_reps; ++rep) {
    if (rep > 0) {
      for (int t = threadIdx.x; t < 64 * 64; t += 256) L[t] = g_src[t];
      __threadfence();
      __syncthreads();
    }
    {
      const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
      P64_STAMP(0);
    }
    potrf64w_stage<PlainMem>(L, ld, (size_t)k * NB * ld + (size_t)k * NB, rhs, k, nrhs, sm);
    potrf64w_reset(sm);
    __syncthreads();
#ifdef WITH_LFLAG
    if (potrf64w_factor<Sc1Mem>(k, rhs, nrhs, Linv, ctrl, sm, &g_lflag, NoFix(), 0.0, NoPre()))
      potrf64w_store_L<Sc1Mem>(L, ld, k, sm);
#else
    if (potrf64w_factor<PlainMem>(k, rhs, nrhs, Linv, ctrl, sm, nullptr, NoFix(), 0.0, NoPre()))
      potrf64w_store_L<PlainMem>(L, ld, k, sm);
#endif
    __syncthreads();
  }
}
void launch_potrf_diag(hipStream_t s, double* L, int ld, int k, double* rhs, int nrhs, double* Linv, DevCtrl* ctrl) {
  k_p64<<<1, 256, 0, s>>>(L, ld, k, rhs, nrhs, Linv, ctrl);
}
}

using namespace cvxg;

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 200;
  const int nrhs = argc > 2 ? atoi(argv[2]) : 1, ld = 64;
  std::vector<double> A(64 * 64), B(64 * 64), rhs(64 * nrhs);
  srand(7);
  for (auto& v : B) v = (double)rand() / RAND_MAX - 0.5;
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j < 64; ++j) {
      double s = 0;
      for (int k = 0; k < 64; ++k) s += B[i * 64 + k] * B[j * 64 + k];
      A[i * 64 + j] = s / 64 + (i == j ? 1.0 : 0.0);
    }
  for (auto& v : rhs) v = (double)rand() / RAND_MAX;
  double *dA, *dL, *dR, *dR0, *dLinv;
  DevCtrl* dc;
  CK(hipMalloc(&dA, 64 * 64 * 8));
  CK(hipMalloc(&dL, 64 * 64 * 8));
  CK(hipMalloc(&dR, 64 * nrhs * 8));
  CK(hipMalloc(&dR0, 64 * nrhs * 8));
  CK(hipMalloc(&dLinv, 64 * 64 * 8));
  CK(hipMalloc(&dc, sizeof(DevCtrl)));
  CK(hipMemset(dc, 0, sizeof(DevCtrl)));
  CK(hipMemcpy(dA, A.data(), 64 * 64 * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dR0, rhs.data(), 64 * nrhs * 8, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  {
    double* src;
    CK(hipMalloc(&src, 64 * 64 * 8));
    CK(hipMemcpy(src, A.data(), 64 * 64 * 8, hipMemcpyHostToDevice));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_src), &src, sizeof(src)));
    const int reps = argc > 3 ? atoi(argv[3]) : 1;
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_reps), &reps, sizeof(reps)));
  }
  // warm + correctness
  CK(hipMemcpy(dL, dA, 64 * 64 * 8, hipMemcpyDeviceToDevice));
  CK(hipMemcpy(dR, dR0, 64 * nrhs * 8, hipMemcpyDeviceToDevice));
  launch_potrf_diag(0, dL, ld, 0, dR, nrhs, dLinv, dc);
  CK(hipDeviceSynchronize());
  std::vector<double> L(64 * 64), Li(64 * 64), w(64 * nrhs);
  CK(hipMemcpy(L.data(), dL, 64 * 64 * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(Li.data(), dLinv, 64 * 64 * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(w.data(), dR, 64 * nrhs * 8, hipMemcpyDeviceToHost));
  double e_llt = 0, e_inv = 0, e_w = 0;
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j <= i; ++j) {
      double s = 0;
      for (int k = 0; k <= j; ++k) s += L[i * 64 + k] * L[j * 64 + k];
      e_llt = fmax(e_llt, fabs(s - A[i * 64 + j]));
    }
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j < 64; ++j) {
      double s = 0;
      for (int k = 0; k < 64; ++k) s += Li[i * 64 + k] * (k >= j ? L[k * 64 + j] : 0.0);
      e_inv = fmax(e_inv, fabs(s - (i == j ? 1.0 : 0.0)));
    }
  for (int i = 0; i < 64; ++i) {  // L w = b
    double s = 0;
    for (int k = 0; k <= i; ++k) s += L[i * 64 + k] * w[k * nrhs];
    e_w = fmax(e_w, fabs(s - rhs[i * nrhs]));
  }
  printf("max|LL'-A|=%.3e  max|Linv L - I|=%.3e  max|Lw-b|=%.3e\n", e_llt, e_inv, e_w);
#ifdef POTRF_STAMPS
  unsigned long long st[4][64];
  CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(g_potrf_stamps), sizeof(st)));
  for (int wv = 0; wv < 4; ++wv) {
    printf("wave %d:", wv);
    for (int i = 1; i < 20; ++i) printf(" %lld", (long long)(st[wv][i] - st[0][0]));
    printf("\n");
  }
#endif
  // timing: copy + potrf pairs, then copies alone
  float ms_pair = 0, ms_copy = 0;
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) {
    CK(hipMemcpyAsync(dL, dA, 64 * 64 * 8, hipMemcpyDeviceToDevice));
    launch_potrf_diag(0, dL, ld, 0, dR, nrhs, dLinv, dc);
  }
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms_pair, e0, e1));
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) CK(hipMemcpyAsync(dL, dA, 64 * 64 * 8, hipMemcpyDeviceToDevice));
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms_copy, e0, e1));
  printf("potrf: %.2f us per launch (pairs %.2f us, copies %.2f us)\n", 1e3 * (ms_pair - ms_copy) / reps,
         1e3 * ms_pair / reps, 1e3 * ms_copy / reps);
  return 0;
}
