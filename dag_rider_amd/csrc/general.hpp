// general.hpp -- reachability on a mirror whose vertices carry edges outside the
// round contract.
//
// uponDeliver checks only the strong-edge count (process/process.go:165) and
// path() is a BFS with a visited set (:89-148), so the reference answers for any
// graph: a strong edge to a round other than r-1, a weak edge to round r-1 or
// above -- even edges to the same or a later round, i.e. cycles.  The mirror
// keeps such "irregular" edges per round beside the packed rows (entry: own
// source, strong flag, target round and source) and, while it holds any, answers
// every query with the general sweep below; the round-by-round kernels
// (kernels.hpp) assume edges point down and stay for contract DAGs.
//
//   k_gsweep    one workgroup per query: the reach set over every round of the
//               DAG, F (reached ids, dangling targets included) and E (expanded),
//               kept in global memory.  A pass walks rounds from the highest one
//               with unexpanded bits down to 0 and expands F & P & ~E of each:
//               strong rows into r-1, weak columns and far edges into their
//               rounds, irregular edges anywhere; a target in the same round
//               repeats the round, one above starts another pass from there.
//               Ends when a pass adds nothing above it (every pass expands at
//               least one new vertex, so at most |V| passes).  Outputs: the hit
//               bit of a tested target, the degree sum of the expanded present
//               vertices in a round range, the reach rows.
//   k_gpaper    PAPER delivery (Alg. 3 line 54) over the pops in order: each
//               pop's mask rows minus the delivered set, which grows by them.
//   k_gdeg      the strong + weak degree sum of each pop's delivered ids.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.hpp"

namespace dr {

// irregular edge entry: bits 0-10 target source - 1, 11-30 target round, 31 strong, 32-42 own source - 1
__host__ __device__ inline uint64_t irr_pack(int own0, bool strong, int tr, int ts0) {
  return ((uint64_t)own0 << 32) | ((uint64_t)(strong ? 1u : 0u) << 31) | ((uint64_t)tr << 11) | (uint64_t)ts0;
}

struct GView {
  const uint64_t *irr;      // irregular edges, grouped by round (irr_roff), sorted by own source
  const uint32_t *irr_roff; // [R+1]
};

struct GQuery {
  int32_t r0, s0;       // start vertex (0-based source; -1: no vertex, nothing reached)
  int32_t strong_only;  // 1: strong edges only (path(.., true), chains, votes)
  int32_t tr, ts;       // tested target (0-based source), -1: none
  int32_t elo, ehi;     // degree sum over expanded present vertices of rounds [elo, ehi]
  int64_t mask_off;     // word offset of this query's F rows [0..T] in masks
  int32_t bot;          // lowest round expanded (rows below stay empty; 0: every round)
  int32_t pad;
};

// T: the last round the reach rows cover (irregular edges may target rounds past
// the mirrored ones, NR: those hold no vertex).
// U (optional): the rounds' strong-row unions (k_summary_commit / k_round_summary, valid
// for the rows whatever irregular edges the mirror holds): a round whose present vertices
// are all newly expanded sends U_r to round r-1 instead of its rows.  Strong rows are
// ORed in registers and reduced through LDS (one global OR per word and round); every F
// row belongs to this workgroup alone, so the weak and irregular scatters' atomics are
// ordered by the round's barriers (no device-scope fence per round: round 4 had one, and
// a global atomic per row word -- C4 scale: ~160 us a round, profiles/r05/v13_*).
template <int WS>
__global__ __launch_bounds__(256) void k_gsweep(DagView g, GView gv, const GQuery *__restrict__ qs, int nq, int T,
                                                int NR, u64 *__restrict__ masks, u64 *__restrict__ scratch,
                                                uint8_t *__restrict__ hit, u64 *__restrict__ edges,
                                                const u64 *__restrict__ U) {
  constexpr int NT = 256;
  const int qi = blockIdx.x;
  if (qi >= nq) return;
  const GQuery q = qs[qi];
  const int tid = threadIdx.x, lane = tid & 63;
  u64 *F = masks + q.mask_off, *E = scratch + (size_t)qi * (T + 1) * WS;
  __shared__ u64 NEW[WS], ACC[WS];
  __shared__ int s_any, s_same, s_up, s_full;
  __shared__ u64 s_e;
  for (size_t i = tid; i < (size_t)(T + 1) * WS; i += NT) {
    F[i] = 0;
    E[i] = 0;
  }
  if (tid == 0) s_e = 0;
  if (tid < WS) ACC[tid] = 0;
  __syncthreads();
  if (q.s0 < 0 || q.r0 < 0 || q.r0 > T) {
    if (tid == 0) {
      if (hit) hit[qi] = 0;
      if (edges) edges[qi] = 0;
    }
    return;
  }
  if (tid == 0) atomicOr(&F[(size_t)q.r0 * WS + (q.s0 >> 6)], 1ULL << (q.s0 & 63));
  __syncthreads();
  const int bot = max(q.bot, 0);
  int hi = q.r0;
  while (hi >= bot) {
    int up = -1;
    int r = hi;
    while (r >= bot) {
      if (tid < 64) {
        u64 nw = 0, p = 0;
        if (lane < WS) {
          const u64 f = ld_agent(&F[(size_t)r * WS + lane]);
          p = r < NR ? g.present[(size_t)r * WS + lane] : 0ULL;
          nw = f & p & ~E[(size_t)r * WS + lane];
          E[(size_t)r * WS + lane] |= nw;
          NEW[lane] = nw;
        }
        const bool any = __ballot(nw != 0ULL) != 0ULL;
        const bool full = __ballot(lane < WS && nw != p) == 0ULL;  // every present vertex new
        if (lane == 0) {
          s_any = any;
          s_full = full;
          s_same = 0;
          s_up = -1;
        }
      }
      __syncthreads();
      const int any = s_any;
      // every wave has read s_any before wave 0 rewrites it (and NEW) for the next round
      __syncthreads();
      if (!any) {
        r--;
        continue;
      }
      // degrees of the vertices expanded now (edge totals of the caller's round range)
      if (r >= q.elo && r <= q.ehi) {
        u64 e = 0;
        for (int s = tid; s < g.n; s += NT)
          if ((NEW[s >> 6] >> (s & 63)) & 1ULL) {
            const size_t at = (size_t)r * g.n + s;
            e += g.sdeg[at] + (q.strong_only ? 0 : g.wdeg[at]);
          }
        e = wave_sum(e);
        if (lane == 0 && e) atomicAdd(&s_e, e);
      }
      // strong rows -> round r-1
      if (r >= 1 && r - 1 >= bot) {
        if (U && s_full) {  // block-uniform
          if (tid < WS) {
            const u64 x = U[(size_t)r * WS + tid];
            if (x) atomicOr(&F[(size_t)(r - 1) * WS + tid], x);
          }
        } else {
          const u64 *rows = g.strong + (size_t)r * g.n * WS;
          u64 acc[WS];
#pragma unroll
          for (int w = 0; w < WS; w++) acc[w] = 0;
          for (int s = tid; s < g.n; s += NT) {
            if (!((NEW[s >> 6] >> (s & 63)) & 1ULL)) continue;
#pragma unroll
            for (int w = 0; w < WS; w++) acc[w] |= rows[(size_t)s * WS + w];
          }
#pragma unroll
          for (int w = 0; w < WS; w++) {
            const u64 v = wave_or(acc[w]);
            if (lane == 0 && v) atomicOr(&ACC[w], v);
          }
          __syncthreads();
          if (tid < WS) {
            const u64 x = ACC[tid];
            ACC[tid] = 0;
            if (x) atomicOr(&F[(size_t)(r - 1) * WS + tid], x);
          }
        }
      }
      if (!q.strong_only) {
        // weak columns of round r (entry: delta, target; its sources' row)
        for (uint32_t j = g.wc_roff[r] + tid; j < g.wc_roff[r + 1]; j += NT) {
          const u64 *row = g.wc_rows + (size_t)j * WS;
          u64 h = 0;
          for (int w = 0; w < WS; w++) h |= row[w] & NEW[w];
          if (!h) continue;
          const uint32_t key = g.wc_key[j];
          const int tr = r - (int)(key >> 11), ts = (int)(key & 2047u);
          if (tr >= bot) atomicOr(&F[(size_t)tr * WS + (ts >> 6)], 1ULL << (ts & 63));
        }
        // far weak edges (delta > 1023): own source - 1 << 32 | target round << 11 | target source - 1
        for (uint32_t j = g.far_roff[r] + tid; j < g.far_roff[r + 1]; j += NT) {
          const u64 x = g.far[j];
          const int own = (int)(x >> 32), tr = (int)((x >> 11) & 0x1FFFFFu), ts = (int)(x & 2047u);
          if (!((NEW[own >> 6] >> (own & 63)) & 1ULL) || tr < bot) continue;
          atomicOr(&F[(size_t)tr * WS + (ts >> 6)], 1ULL << (ts & 63));
        }
      }
      // irregular edges: any target round; the same round repeats r, a later one another pass
      for (uint32_t j = gv.irr_roff[r] + tid; j < gv.irr_roff[r + 1]; j += NT) {
        const uint64_t x = gv.irr[j];
        const int own = (int)((x >> 32) & 2047u), tr = (int)((x >> 11) & 0xFFFFFu), ts = (int)(x & 2047u);
        const bool strong = (x >> 31) & 1u;
        if (q.strong_only && !strong) continue;
        if (!((NEW[own >> 6] >> (own & 63)) & 1ULL) || tr < bot) continue;
        const u64 bit = 1ULL << (ts & 63);
        const u64 old = atomicOr(&F[(size_t)tr * WS + (ts >> 6)], bit);
        if (!(old & bit) && tr >= r) {
          if (tr == r) atomicOr(&s_same, 1);
          else atomicMax(&s_up, tr);
        }
      }
      __syncthreads();  // (waits for this workgroup's atomics: wave 0 reads F from L2 next)
      if (s_up > up) up = s_up;
      if (!s_same) r--;  // a new bit in round r itself: expand r again
      __syncthreads();
    }
    hi = up;  // a later round gained a bit: another pass from there (-1: done)
  }
  __syncthreads();
  if (tid == 0) {
    if (hit) hit[qi] = (q.tr >= 0 && q.tr <= T && q.ts >= 0)
                           ? (uint8_t)((ld_agent(&F[(size_t)q.tr * WS + (q.ts >> 6)]) >> (q.ts & 63)) & 1ULL)
                           : 0;
    if (edges) edges[qi] = s_e;
  }
}

// PAPER delivery over pops in order (one workgroup; lane w < WS of wave k handles
// rounds k, k + 4, ...): mask_p(r) := mask_p(r) & P_r & ~D_r, D_r |= mask_p(r),
// for r in [1, last_p]; rows outside that range are cleared.  D: [T+1][WS], zeroed.
template <int WS>
__global__ __launch_bounds__(256) void k_gpaper(DagView g, u64 *__restrict__ masks, const int64_t *__restrict__ moff,
                                                const int32_t *__restrict__ last, int np, int T, u64 *__restrict__ D) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int p = 0; p < np; p++) {
    u64 *m = masks + moff[p];
    for (int r = wv; r <= T; r += 4) {
      if (lane >= WS) continue;
      const size_t i = (size_t)r * WS + lane;
      u64 x = 0;
      if (r >= 1 && r <= last[p]) {
        x = m[i] & g.present[i] & ~D[i];
        D[i] |= x;
      }
      m[i] = x;
    }
    __syncthreads();
  }
}

// Per mask p: the degree sum (strong, + weak with `weak`) of the present ids of its
// rows [first[p], last[p]] (an id's edges once).  One workgroup per mask.
template <int WS>
__global__ __launch_bounds__(256) void k_gdeg(DagView g, const u64 *__restrict__ masks, const int64_t *__restrict__ moff,
                                              const int32_t *__restrict__ first, const int32_t *__restrict__ last,
                                              int weak, u64 *__restrict__ out) {
  __shared__ u64 s_e;
  const int p = blockIdx.x, tid = threadIdx.x;
  if (tid == 0) s_e = 0;
  __syncthreads();
  const u64 *m = masks + moff[p];
  u64 e = 0;
  for (int r = first[p]; r <= last[p]; r++)
    for (int s = tid; s < g.n; s += 256) {
      const size_t i = (size_t)r * WS + (s >> 6);
      if ((m[i] & g.present[i]) >> (s & 63) & 1ULL)
        e += g.sdeg[(size_t)r * g.n + s] + (weak ? g.wdeg[(size_t)r * g.n + s] : 0);
    }
  e = wave_sum(e);
  if ((tid & 63) == 0 && e) atomicAdd(&s_e, e);
  __syncthreads();
  if (tid == 0) out[p] = s_e;
}

}  // namespace dr
