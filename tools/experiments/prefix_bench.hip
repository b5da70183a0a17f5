// prefix_bench.hip -- k_canon_prefix's one-workgroup prefix over T+1 rounds of two
// u64 arrays (C3: 10 001 rounds), three forms timed with HIP events (round 5 experiment):
//   0  canon_prefix_block<1024> (the run form shipped to round 4: thread t owns rounds t*per ..)
//   1  an LDS-transposed tile form (shipped in round 5 up to v14): coalesced loads into LDS, each thread scans 4
//      contiguous rounds out of LDS, one block scan per tile, coalesced stores
//   2  canon_prefix_block<256>
//   3  k_canon_prefix<1024> as shipped since round 5's v14 (canon_prefix_regs: every round
//      of the chunk in registers, DPP wave scans, two LDS-only barriers)
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../dag_rider_amd/csrc prefix_bench.hip -o prefix_bench
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "kernels.hpp"

using dr::u64;

template <int NT, int PT = 4>
__global__ __launch_bounds__(NT) void k_prefix_lds(int T, const u64 *__restrict__ a, const u64 *__restrict__ b,
                                                   u64 *__restrict__ A, u64 *__restrict__ B) {
  constexpr int TILE = NT * PT;
  __shared__ u64 sa[TILE], sb[TILE];
  __shared__ u64 part[NT / 64];
  const int tid = threadIdx.x, n = T + 1;
  u64 ca = 0, cb = 0;
  for (int t0 = 0; t0 < n; t0 += TILE) {
#pragma unroll
    for (int j = 0; j < PT; j++) {  // coalesced: lane-consecutive rounds
      const int r = t0 + j * NT + tid;
      const bool in = r >= 1 && r < n;
      const int rc = in ? r : 0;
      const u64 x = a[rc], y = b[rc];
      sa[j * NT + tid] = in ? x : 0ULL;
      sb[j * NT + tid] = in ? y : 0ULL;
    }
    __syncthreads();
    u64 xa[PT], xb[PT], la = 0, lb = 0;
#pragma unroll
    for (int j = 0; j < PT; j++) {
      xa[j] = sa[tid * PT + j];
      xb[j] = sb[tid * PT + j];
      la += xa[j];
      lb += xb[j];
    }
    u64 ta, tb;
    u64 ea = ca + dr::block_scan_excl<NT>(la, part, ta);
    u64 eb = cb + dr::block_scan_excl<NT>(lb, part, tb);
#pragma unroll
    for (int j = 0; j < PT; j++) {
      ea += xa[j];
      eb += xb[j];
      sa[tid * PT + j] = ea;
      sb[tid * PT + j] = eb;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PT; j++) {
      const int r = t0 + j * NT + tid;
      if (r < n) {
        A[r] = sa[j * NT + tid];
        B[r] = sb[j * NT + tid];
      }
    }
    ca += ta;
    cb += tb;
    __syncthreads();
  }
}

template <int NT>
__global__ __launch_bounds__(NT) void k_prefix_block(int T, const u64 *a, const u64 *b, u64 *A, u64 *B) {
  dr::canon_prefix_block<NT>(T, a, b, A, B, nullptr);
}

int main(int argc, char **argv) {
  const int T = argc > 1 ? atoi(argv[1]) : 10000;
  const int n = T + 1;
  std::vector<u64> ha(n), hb(n);
  for (int i = 0; i < n; i++) { ha[i] = (u64)(i * 7 + 3); hb[i] = (u64)(i % 13); }
  u64 *a, *b, *A, *B;
  hipMalloc(&a, n * 8); hipMalloc(&b, n * 8); hipMalloc(&A, n * 8); hipMalloc(&B, n * 8);
  hipMemcpy(a, ha.data(), n * 8, hipMemcpyHostToDevice);
  hipMemcpy(b, hb.data(), n * 8, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  std::vector<u64> wantA(n), wantB(n);
  u64 sa = 0, sb = 0;
  for (int i = 0; i < n; i++) { if (i >= 1) { sa += ha[i]; sb += hb[i]; } wantA[i] = sa; wantB[i] = sb; }
  for (int form = 0; form < 4; form++) {
    float best = 1e9;
    for (int it = 0; it < 50; it++) {
      hipMemset(A, 0, n * 8);
      hipEventRecord(e0);
      if (form == 0) hipLaunchKernelGGL((k_prefix_block<1024>), dim3(1), dim3(1024), 0, 0, T, a, b, A, B);
      if (form == 1) hipLaunchKernelGGL((k_prefix_lds<1024>), dim3(1), dim3(1024), 0, 0, T, a, b, A, B);
      if (form == 2) hipLaunchKernelGGL((k_prefix_block<256>), dim3(1), dim3(256), 0, 0, T, a, b, A, B);
      if (form == 3) hipLaunchKernelGGL((dr::k_canon_prefix<1024>), dim3(1), dim3(1024), 0, 0, T, a, b, A, B);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    std::vector<u64> gA(n), gB(n);
    hipMemcpy(gA.data(), A, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(gB.data(), B, n * 8, hipMemcpyDeviceToHost);
    const bool ok = gA == wantA && gB == wantB;
    printf("form %d T %d best %.2f us %s\n", form, T, best * 1e3, ok ? "ok" : "WRONG");
  }
  return 0;
}
