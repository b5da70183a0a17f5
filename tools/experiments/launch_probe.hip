// Launch-cost probe (round 6): what a dependent launch, an event record, a
// hipExtLaunchKernelGGL with events, a cross-stream join and a large kernarg
// cost on one MI355X stream.  Each case runs ITERS times between two events;
// prints microseconds per iteration.  Build: hipcc --offload-arch=gfx950 -O2.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

__global__ void k_tiny(int *p) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1;
}
struct Big {
  void *p[48];
};
__global__ void k_bigarg(Big b) {
  if (threadIdx.x == 0 && blockIdx.x == 0) static_cast<int *>(b.p[0])[0] += 1;
}
__global__ __launch_bounds__(1024) void k_wide(int *p) {
  __shared__ int s[12288];
  s[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += s[5];
}

int main() {
  const int ITERS = 2000, K = 10;
  int *d;
  CK(hipMalloc(&d, 4096));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t t0, t1, e1, e2, ea, eb;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  CK(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&e2, hipEventDisableTiming));
  CK(hipEventCreate(&ea));
  CK(hipEventCreate(&eb));
  Big big{};
  big.p[0] = d;
  auto run = [&](const char *name, auto body) {
    for (int w = 0; w < 50; w++) body();
    CK(hipStreamSynchronize(s1));
    CK(hipStreamSynchronize(s2));
    CK(hipEventRecord(t0, s1));
    for (int i = 0; i < ITERS; i++) body();
    CK(hipEventRecord(t1, s1));
    CK(hipEventSynchronize(t1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, t0, t1));
    std::printf("%-58s %8.2f us/iter\n", name, ms * 1e3f / ITERS);
  };
  run("10 dependent k_tiny", [&] {
    for (int k = 0; k < K; k++) hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s1, d);
  });
  run("10 k_tiny, a timing event record after each", [&] {
    for (int k = 0; k < K; k++) {
      hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s1, d);
      CK(hipEventRecord(k & 1 ? eb : ea, s1));
    }
  });
  run("10 k_tiny, a no-timing event record after each", [&] {
    for (int k = 0; k < K; k++) {
      hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s1, d);
      CK(hipEventRecord(e1, s1));
    }
  });
  run("10 k_tiny by hipExtLaunchKernelGGL with start/stop events", [&] {
    for (int k = 0; k < K; k++)
      hipExtLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s1, ea, eb, 0, d);
  });
  run("10 k_bigarg (384-B kernarg)", [&] {
    for (int k = 0; k < K; k++) hipLaunchKernelGGL(k_bigarg, dim3(1), dim3(64), 0, s1, big);
  });
  run("10 k_wide (1024 threads, 48 KB LDS)", [&] {
    for (int k = 0; k < K; k++) hipLaunchKernelGGL(k_wide, dim3(1), dim3(1024), 0, s1, d);
  });
  run("10 k_tiny, s1->s2->s1 ping-pong each (2 joins)", [&] {
    for (int k = 0; k < K; k++) {
      hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s1, d);
      CK(hipEventRecord(e1, s1));
      CK(hipStreamWaitEvent(s2, e1, 0));
      hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s2, d + 64);
      CK(hipEventRecord(e2, s2));
      CK(hipStreamWaitEvent(s1, e2, 0));
    }
  });
  run("fork at start, 10 k_tiny on s1, join of s2's 1 k_tiny at end", [&] {
    CK(hipEventRecord(e1, s1));
    CK(hipStreamWaitEvent(s2, e1, 0));
    hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s2, d + 64);
    CK(hipEventRecord(e2, s2));
    for (int k = 0; k < K; k++) hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s1, d);
    CK(hipStreamWaitEvent(s1, e2, 0));
    hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s1, d);
  });
  run("11 dependent k_tiny (the same without the streams)", [&] {
    for (int k = 0; k < K + 1; k++) hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s1, d);
  });
  return 0;
}
