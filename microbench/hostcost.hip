// Host-side cost of the HIP calls the Newton step issues between kernels, and the GPU idle they leave: an empty kernel
// launch, hipEventRecord (default and disable-timing events), hipStreamWaitEvent on a second stream, and a kernel
// launch behind each.  For each call sequence: host microseconds per sequence (steady_clock) and the GPU time from the
// end of a spin kernel to the start of the next kernel (s_memrealtime stamps, 100 MHz).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 microbench/hostcost.hip -o microbench/hostcost
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <chrono>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);   \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

__global__ void k_stamp(unsigned long long* t, int i, int end) {
  if (threadIdx.x == 0) t[2 * i + end] = __builtin_amdgcn_s_memrealtime();
}
__global__ void k_spin(unsigned long long* t, int i, long long ticks) {  // busy ~ticks of the 100 MHz clock
  if (threadIdx.x == 0) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    t[2 * i] = t0;
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)ticks) {
    }
    t[2 * i + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  hipStream_t s, s2;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t ev, evt0, evt1;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  CK(hipEventCreate(&evt0));
  CK(hipEventCreate(&evt1));
  unsigned long long* t;
  CK(hipMalloc(&t, 2 * 64 * sizeof(unsigned long long)));
  const char* names[] = {"launch only",
                         "record(disable-timing) + launch",
                         "record(timing) + launch",
                         "record + waitEvent(s2) + launch",
                         "record + waitEvent(s2) + record(timing) + launch",
                         "5 launches"};
  for (int variant = 0; variant < 6; ++variant) {
    double host = 0, gap = 0;
    const int reps = 50;
    for (int r = 0; r < reps + 5; ++r) {
      k_spin<<<1, 64, 0, s>>>(t, 0, 5000);  // 50 us of GPU work: the host calls below are issued while it runs
      const double h0 = now_us();
      switch (variant) {
        case 0: k_stamp<<<1, 64, 0, s>>>(t, 1, 0); break;
        case 1:
          CK(hipEventRecord(ev, s));
          k_stamp<<<1, 64, 0, s>>>(t, 1, 0);
          break;
        case 2:
          CK(hipEventRecord(evt0, s));
          k_stamp<<<1, 64, 0, s>>>(t, 1, 0);
          break;
        case 3:
          CK(hipEventRecord(ev, s));
          CK(hipStreamWaitEvent(s2, ev, 0));
          k_stamp<<<1, 64, 0, s>>>(t, 1, 0);
          break;
        case 4:
          CK(hipEventRecord(ev, s));
          CK(hipStreamWaitEvent(s2, ev, 0));
          CK(hipEventRecord(evt1, s));
          k_stamp<<<1, 64, 0, s>>>(t, 1, 0);
          break;
        case 5:
          for (int q = 0; q < 5; ++q) k_stamp<<<1, 64, 0, s>>>(t, 1, 0);
          break;
      }
      const double h1 = now_us();
      CK(hipStreamSynchronize(s));
      CK(hipStreamSynchronize(s2));
      unsigned long long ht[4];
      CK(hipMemcpy(ht, t, sizeof(ht), hipMemcpyDeviceToHost));
      if (r >= 5) {
        host += h1 - h0;
        gap += (double)(ht[2] - ht[1]) / 100.0;  // 100 MHz ticks -> us
      }
    }
    printf("%-52s host %7.2f us   GPU gap spin-end -> next kernel %7.2f us\n", names[variant], host / reps, gap / reps);
  }
  // the same when the GPU is idle at the time of the calls (the host issues after a synchronize)
  for (int variant = 0; variant < 2; ++variant) {
    double host = 0;
    const int reps = 50;
    for (int r = 0; r < reps + 5; ++r) {
      CK(hipStreamSynchronize(s));
      const double h0 = now_us();
      if (variant == 1) CK(hipEventRecord(ev, s));
      k_stamp<<<1, 64, 0, s>>>(t, 1, 0);
      const double h1 = now_us();
      if (r >= 5) host += h1 - h0;
    }
    CK(hipStreamSynchronize(s));
    printf("idle GPU: %-42s host %7.2f us\n", variant ? "record + launch" : "launch", host / reps);
  }
  return 0;
}
