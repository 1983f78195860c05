// HBM stream microbenchmark (re-measure the HBM ceiling on the box).  Three kernels over 1 GiB
// double buffers with 16-B accesses, grid-stride, 8 workgroups of 256 threads per CU: read (sum into a per-thread
// register, one store per thread), copy (b = a), triad (c = a + s b).  Best of 10 timed launches after 2 warm-ups;
// bytes = the algorithmic bytes each kernel moves.  Also the same three at 64 MiB (fits the 256 MiB Infinity
// Cache: the regime of the Ruiz sweeps over the 67 MB lower triangle).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 microbench/stream.hip -o microbench/stream
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double d2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_read(const d2* __restrict__ a, size_t n2, double* __restrict__ out) {
  d2 s = {0.0, 0.0};
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256) s += a[i];
  out[blockIdx.x * 256 + threadIdx.x] = s[0] + s[1];
}
__global__ __launch_bounds__(256) void k_copy(const d2* __restrict__ a, d2* __restrict__ b, size_t n2) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256) b[i] = a[i];
}
__global__ __launch_bounds__(256) void k_triad(const d2* __restrict__ a, const d2* __restrict__ b, d2* __restrict__ c,
                                               double s, size_t n2) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256) c[i] = a[i] + s * b[i];
}

int main() {
  int dev = 0, ncu = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const int grid = ncu * 8;
  double *a, *b, *c, *out;
  const size_t big = (size_t)1 << 30;
  hipMalloc(&a, big);
  hipMalloc(&b, big);
  hipMalloc(&c, big);
  hipMalloc(&out, (size_t)grid * 256 * 8);
  hipMemset(a, 0, big);
  hipMemset(b, 0, big);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (size_t bytes : {big, (size_t)64 << 20}) {
    const size_t n2 = bytes / 16;
    for (int kind = 0; kind < 3; ++kind) {
      float best = 1e30f;
      for (int r = 0; r < 12; ++r) {
        hipEventRecord(e0);
        if (kind == 0) k_read<<<grid, 256>>>((const d2*)a, n2, out);
        if (kind == 1) k_copy<<<grid, 256>>>((const d2*)a, (d2*)b, n2);
        if (kind == 2) k_triad<<<grid, 256>>>((const d2*)a, (const d2*)b, (d2*)c, 1.5, n2);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        if (r >= 2 && ms < best) best = ms;
      }
      const double moved = (double)bytes * (kind == 0 ? 1 : kind == 1 ? 2 : 3);
      printf("%-5s %5zu MiB per array: %.3f ms, %.2f TB/s\n", kind == 0 ? "read" : kind == 1 ? "copy" : "triad",
             bytes >> 20, best, moved / (best * 1e-3) / 1e12);
    }
  }
  return 0;
}
