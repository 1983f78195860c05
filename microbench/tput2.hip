// Microbenchmark: back-to-back issue cost of broadcast primitives on gfx950 (one wave), each measured as
// a block of independent instructions between two s_memtime stamps, consumers outside the block.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 microbench/tput2.hip -o microbench/tput2
#include <hip/hip_runtime.h>
#include <stdio.h>

#define REP16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

__global__ void k_b(double* out, long long* res, double x) {
  __shared__ __attribute__((aligned(16))) double sh[256];
  const int lane = threadIdx.x & 63;
  double a[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) a[i] = x + lane * 0.01 + i;
  sh[lane] = x * lane;
  sh[lane + 64] = x * lane + 1;
  __syncthreads();
  long long t0, t1;
  unsigned s[32];
  // 0: 32 v_readlane_b32 back to back
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n s_nop 7" ::: "memory");
  t0 = __builtin_amdgcn_s_memtime();
#define RL(i) s[2 * i] = __builtin_amdgcn_readlane((int)__double_as_longlong(a[i]), i); \
              s[2 * i + 1] = __builtin_amdgcn_readlane((int)(__double_as_longlong(a[i]) >> 32), i);
  REP16(RL)
  asm volatile("" ::"s"(s[0]), "s"(s[31]));
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) res[0] = t1 - t0;
  unsigned acc = 0;
  for (int i = 0; i < 32; ++i) acc += s[i];
  // 1: 16 v_fmac_f64 with SGPR operands (independent)
  asm volatile("s_nop 7" ::: "memory");
  t0 = __builtin_amdgcn_s_memtime();
  const double sv = __longlong_as_double(((long long)s[1] << 32) | s[0]);
#define FM(i) a[i] = fma(sv, a[(i + 1) & 15], a[i]);
  REP16(FM)
  asm volatile("" ::"v"(a[0]), "v"(a[15]));
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) res[1] = t1 - t0;
  // 2: 16 pairs of v_mov_b32_dpp row_newbcast
  int d[32];
  asm volatile("s_nop 7" ::: "memory");
  t0 = __builtin_amdgcn_s_memtime();
#define DP(i) d[2 * i] = __builtin_amdgcn_mov_dpp((int)__double_as_longlong(a[i]), 0x150 + i, 0xf, 0xf, true); \
              d[2 * i + 1] = __builtin_amdgcn_mov_dpp((int)(__double_as_longlong(a[i]) >> 32), 0x150 + i, 0xf, 0xf, true);
  REP16(DP)
  asm volatile("" ::"v"(d[0]), "v"(d[31]));
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) res[2] = t1 - t0;
  for (int i = 0; i < 32; ++i) acc += d[i];
  // 3: 8 ds_read_b128 broadcast (uniform address) + wait
  typedef double v2 __attribute__((ext_vector_type(2)));
  v2 l[8];
  const int base = __builtin_amdgcn_readfirstlane((int)(x * 0.0));
  asm volatile("s_nop 7" ::: "memory");
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int i = 0; i < 8; ++i) l[i] = *reinterpret_cast<const v2*>(&sh[base + 2 * i]);
  asm volatile("s_waitcnt lgkmcnt(0)" ::"v"(l[0]), "v"(l[7]));
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) res[3] = t1 - t0;
  double ls = 0;
  for (int i = 0; i < 8; ++i) ls += l[i][0] + l[i][1];
  // 4: 16 v_fmac_f64_dpp row_newbcast (independent)
  asm volatile("s_nop 7" ::: "memory");
  t0 = __builtin_amdgcn_s_memtime();
#define FD(i) asm volatile("v_fmac_f64_dpp %0, %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "+v"(a[i]) : "v"(sv), "i"(i));
  REP16(FD)
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) res[4] = t1 - t0;
  // 5: 16 v_readfirstlane-free SGPR-broadcast alternative: v_permlane32_swap pairs? skipped; ds_bpermute x16
  int bp[16];
  asm volatile("s_nop 7" ::: "memory");
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int i = 0; i < 16; ++i) bp[i] = __builtin_amdgcn_ds_bpermute(i * 4, (int)__double_as_longlong(a[i]));
  asm volatile("s_waitcnt lgkmcnt(0)" ::"v"(bp[0]), "v"(bp[15]));
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) res[5] = t1 - t0;
  for (int i = 0; i < 16; ++i) acc += bp[i];
  double sum = ls + acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) sum += a[i];
  out[threadIdx.x] = sum;
}

int main() {
  double* o;
  long long* r;
  (void)hipMalloc(&o, 1 << 16);
  (void)hipMalloc(&r, 1024);
  const char* names[] = {"32 v_readlane_b32", "16 v_fmac_f64 (sgpr)", "32 v_mov_b32_dpp newbcast", "8 ds_read_b128 bcast+wait",
                         "16 v_fmac_f64_dpp", "16 ds_bpermute+wait"};
  const double cnt[] = {32, 16, 32, 8, 16, 16};
  for (int rep = 0; rep < 3; ++rep) k_b<<<1, 64>>>(o, r, 0.5);
  (void)hipDeviceSynchronize();
  long long h[8];
  (void)hipMemcpy(h, r, sizeof(h), hipMemcpyDeviceToHost);
  for (int s = 0; s < 6; ++s) printf("  %-28s %6lld cycles  %6.2f per instr\n", names[s], h[s], h[s] / cnt[s]);
  return 0;
}
