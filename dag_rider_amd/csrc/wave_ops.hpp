// wave_ops.hpp -- wave64 helpers shared by the engine (kernels.hpp) and the
// column-sharded path (shard.hip): popcount, agent-scope loads, the delivered-
// sequence digest term and DPP/readlane wave reductions.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dr {

typedef unsigned long long u64;

__device__ __forceinline__ int popc64(u64 x) { return __popcll(x); }

__device__ __forceinline__ u64 ld_agent(const u64 *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ u64 mix64(u64 z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
__device__ __forceinline__ u64 digest_term(uint32_t round, uint32_t source, u64 k) {
  u64 key = ((u64)round << 32) | source;
  return mix64(key ^ mix64(k + 0x9E3779B97F4A7C15ULL));
}

// ---------------------------------------------------------------------------
// Wave reductions on DPP row operations (rows of 16 lanes) + readlane: no LDS
// traffic, no ds_bpermute latency chain.  Every lane of the wave must be active.
// ---------------------------------------------------------------------------
// every control used here (quad_perm, row_half_mirror, row_mirror) reads a lane of
// the same row, so no lane is out of bounds: old = x and bound_ctrl leave the
// destination uninitialised (no v_mov of a zero old value per step) and let the
// compiler fold the move into the OR / add that consumes it
template <int CTRL>
__device__ __forceinline__ uint32_t dpp32(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, CTRL, 0xF, 0xF, true);
}
template <int CTRL>
__device__ __forceinline__ u64 dpp64(u64 x) {
  return ((u64)dpp32<CTRL>((uint32_t)(x >> 32)) << 32) | (u64)dpp32<CTRL>((uint32_t)x);
}

enum : int { DPP_QP_1032 = 0xB1, DPP_QP_2301 = 0x4E, DPP_ROW_MIRROR = 0x140, DPP_ROW_HALF_MIRROR = 0x141,
             DPP_ROW_ROR = 0x120 };
// OR over the lanes of a row with equal (lane mod C), C a power of two < 16:
// afterwards lane l of every row holds the OR of its row's class l mod C.
template <int C>
__device__ __forceinline__ u64 row_or_stride(u64 x) {
  if constexpr (C <= 1) x |= dpp64<DPP_ROW_ROR + 1>(x);
  if constexpr (C <= 2) x |= dpp64<DPP_ROW_ROR + 2>(x);
  if constexpr (C <= 4) x |= dpp64<DPP_ROW_ROR + 4>(x);
  if constexpr (C <= 8) x |= dpp64<DPP_ROW_ROR + 8>(x);
  return x;
}
__device__ __forceinline__ u64 readlane64(u64 x, int l) {
  return ((u64)(uint32_t)__builtin_amdgcn_readlane((int)(x >> 32), l) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, l);
}
// lane l's value (ds_bpermute on both halves); every lane of the wave must be active
__device__ __forceinline__ u64 shfl64(u64 x, int l) {
  return ((u64)(uint32_t)__shfl((int)(x >> 32), l) << 32) | (uint32_t)__shfl((int)(uint32_t)x, l);
}
// Workgroup barrier that orders LDS only: the release waits for this thread's LDS
// accesses (lgkmcnt), not for its global loads in flight, so loads prefetched ahead of a
// barrier stay in flight across it (__syncthreads waits for every vmcnt event).  For
// loops whose threads share data through LDS alone.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
// lane (lane ^ m)'s value; every lane of the wave must be active
__device__ __forceinline__ u64 shfl_xor64(u64 x, int m) {
  return ((u64)(uint32_t)__shfl_xor((int)(x >> 32), m) << 32) | (uint32_t)__shfl_xor((int)(uint32_t)x, m);
}
// lane (lane - d)'s value, own value for lane < d
__device__ __forceinline__ u64 shfl_up64(u64 x, int d) {
  return ((u64)(uint32_t)__shfl_up((int)(x >> 32), d) << 32) | (uint32_t)__shfl_up((int)(uint32_t)x, d);
}
// OR of all 64 lanes (wave-uniform result)
__device__ __forceinline__ u64 wave_or(u64 x) {
  x |= dpp64<DPP_QP_1032>(x);
  x |= dpp64<DPP_QP_2301>(x);
  x |= dpp64<DPP_ROW_HALF_MIRROR>(x);
  x |= dpp64<DPP_ROW_MIRROR>(x);
  return readlane64(x, 0) | readlane64(x, 16) | readlane64(x, 32) | readlane64(x, 48);
}
// 64-bit DPP move with zero where the source lane is out of the row or the row is masked
// off (old = 0, bound_ctrl off)
template <int CTRL, int ROWS>
__device__ __forceinline__ u64 dpp64z(u64 x) {
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(x >> 32), CTRL, ROWS, 0xF, false);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)x, CTRL, ROWS, 0xF, false);
  return ((u64)hi << 32) | lo;
}
// inclusive prefix sum over the 64 lanes: row_shr 1, 2, 4, 8 inside each row of 16, then
// row_bcast:15 (rows 1, 3 add the last lane of the row below) and row_bcast:31 (rows 2, 3
// add lane 31); every lane of the wave must be active
__device__ __forceinline__ u64 wave_scan_incl(u64 x) {
  x += dpp64z<0x111, 0xF>(x);
  x += dpp64z<0x112, 0xF>(x);
  x += dpp64z<0x114, 0xF>(x);
  x += dpp64z<0x118, 0xF>(x);
  x += dpp64z<0x142, 0xA>(x);
  x += dpp64z<0x143, 0xC>(x);
  return x;
}
// sum of all 64 lanes (wave-uniform result)
__device__ __forceinline__ u64 wave_sum(u64 x) {
  x += dpp64<DPP_QP_1032>(x);
  x += dpp64<DPP_QP_2301>(x);
  x += dpp64<DPP_ROW_HALF_MIRROR>(x);
  x += dpp64<DPP_ROW_MIRROR>(x);
  return readlane64(x, 0) + readlane64(x, 16) + readlane64(x, 32) + readlane64(x, 48);
}
}  // namespace dr
