// shard.hip -- process-column sharded reachability, commit and delivery
// (include/dagrider_shard.h).
//
// for a DAG split across the GPUs of one node, GPU g keeps the
// target columns [g*C, (g+1)*C) of every strong row and the weak edges whose
// target falls there; every GPU also keeps the small per-vertex metadata
// (presence, slot order, strong/weak degrees), so each one can emit the
// delivered sequences itself once it holds a full frontier.
//
// Sweeps (path(), the leader chain of waveReady, the cones of orderVertices).
// A batch of up to 64 queries sweeps the rounds top-down; the frontier of a
// round is held TRANSPOSED: FT[s] = u64 mask of the queries that reached source
// s, so one all-gather of C words per shard per round moves the frontier of all
// 64 queries.  Per round r:
//
//   1. write round r's reach rows (the ballot of bit b over 64 sources is query
//      b's bitset word -- a 64x64 bit transpose per wave, shard 0 only);
//   2. chain queries (process.go:341-350) at a leader round: when the wave's
//      leader is present and in a chain's frontier, push that wave and restart
//      the chain's frontier at the leader alone -- every shard takes the same
//      decision from the same full FT_r;
//   3. strong expansion into the pending frontier of r-1: each wave takes 64
//      sources; for every (source with a non-empty mask) x (row word) it walks
//      the active sources with a scalar loop (readlane) and lane j ORs the
//      source's query mask when the row has target bit j: one atomic per target;
//   4. weak expansion: the shard's weak edges of round r (sorted by (delta,
//      target)) OR the source's mask into the pending frontier of r - delta;
//   5. produce: drain the pending frontier of r-1, inject the queries that start
//      there, publish the shard's columns of FT_{r-1}.
//
// Local mode (all shards in one context, one device) runs a whole batch as ONE
// cooperative launch (k_shard_sweep): steps 1-4, a grid barrier, step 5 spread
// over every workgroup, a second barrier, next round -- no per-round launch.
// RCCL mode launches k_shard_round per round (the last workgroup of the shard
// produces into the send buffer) followed by ncclAllGather on the same stream.
//
// Commit (waveReady's vote, process.go:326-339) for many waves at once: three
// steps S_k = {v in round 4w-3+k : row(v) & S_{k-1} != 0}; shard g tests its
// columns of each row against its columns of S_{k-1} and writes a partial hit
// bitset; the partials of all shards are OR-ed by the next step (RCCL mode: one
// all-gather of [nwaves][W] words per step).  vcount = |S_3|.
//
// Delivery (orderVertices, process.go:404-443): one cone per distinct popped
// leader (rows for rounds bottom..top), then on every GPU: paper-mode dedup (a
// per-round scan over the leaders in pop order against the delivered set),
// per-(leader, round) counts and edge sums, a per-leader scan for positions, and
// the order-sensitive digest over the round's slots in insertion order.
//
// Semantics are those of dagrider_gpu.h (dr_reach_sets, dr_path_batch,
// dr_wave_commit, dr_wave_ready, dr_order_vertices, dr_replay): the reach set
// is defined over the id space (a dangling target counts as reached,
// process.go:123,136), an absent vertex has an all-zero row (no edges,
// :111-116), and the start vertex is in its own set (self path, :91-93).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "dagrider_gpu.h"
#include "dagrider_shard.h"
#include "shard_fused.hpp"
#include "shard_memo.hpp"
#include "shard_step.hpp"
#include "wave_ops.hpp"

namespace {

using dr::u64;
constexpr int SH_NT = 256;  // threads per workgroup (4 waves)
constexpr int SH_BATCH = 64;
enum : int32_t { QF_CHAIN = 1 };

thread_local std::string g_shard_err;

struct SBuf {
  void *p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t c = std::max<size_t>(bytes, 4096);
    hipError_t e = hipMalloc(&p, c);
    if (e == hipSuccess) cap = c;
    return e;
  }
  // grow keeping the first `keep` bytes
  hipError_t grow(size_t bytes, size_t keep, hipStream_t s) {
    if (bytes <= cap) return hipSuccess;
    const size_t c = std::max<size_t>({bytes, cap * 2, 4096});
    void *q = nullptr;
    hipError_t e = hipMalloc(&q, c);
    if (e != hipSuccess) return e;
    if (p && keep) {
      e = hipMemcpyAsync(q, p, keep, hipMemcpyDeviceToDevice, s);
      if (e == hipSuccess) e = hipStreamSynchronize(s);
      if (e != hipSuccess) { (void)hipFree(q); return e; }
    }
    if (p) (void)hipFree(p);
    p = q;
    cap = c;
    return hipSuccess;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T> T *as() const { return static_cast<T *>(p); }
};

struct QInfo {
  int32_t top, bottom, src0, flags;  // src0 = 0-based source of `from`, -1 none; flags QF_*
  int64_t obase;                     // word offset of round `bottom` in the batch output
  int32_t push_base;                 // QF_CHAIN: first slot of the query's push list
  int32_t last;                      // pops: last emitted round, min(p.round, top)
};

struct ShardArgs {
  const u64 *strong;        // [nlocal][max_rounds][n][SP] (words >= WSs zero)
  const uint32_t *weak;     // per local shard: edges (target col 0-10, source 11-21, delta 22-31)
  const uint64_t *woff;     // [nlocal][max_rounds+1] edge offsets (absolute in weak)
  const u64 *pres;          // [max_rounds][W] presence (chain restarts)
  const uint16_t *lead;     // [nlead] chooseLeader(w), 1-based source
  const uint16_t *sdeg;     // [max_rounds][n] strong degree of the whole row (chain edges)
  u64 *ftb0, *ftb1;         // FT_r for even / odd r: [G*C] query masks (full width)
  u64 *send;                // RCCL mode: this shard's columns of FT_{r-1}
  u64 *pend;                // [nlocal][depth][C]
  unsigned *cnt;            // [nlocal] workgroups done this round (k_shard_round)
  unsigned *bar;            // grid barrier counter (k_shard_sweep)
  int32_t *err;             // grid barrier timeout flag
  u64 *out;                 // batch reach rows
  const QInfo *q;           // [nq]
  int32_t *push_out;        // chain pushes (waves), query b's list at q[b].push_base
  int32_t *push_n;          // [64] pushes per chain query
  u64 *cedges;              // [64] chain edges per query
  int32_t n, W, WSs, SP, C, depth, shard0, nlocal, local, max_rounds, nq, strong_only, nlead;
  int64_t strong_shard_stride;  // words between local shards' rows of one round (n * SP)
  int64_t strong_round_stride;  // words per round, every local shard (nlocal * n * SP)
};

__device__ __forceinline__ u64 shfl_xor64(u64 v, int m) {
  const int lo = __shfl_xor((int)(uint32_t)v, m, 64), hi = __shfl_xor((int)(uint32_t)(v >> 32), m, 64);
  return ((u64)(uint32_t)hi << 32) | (uint32_t)lo;
}

// per-round query masks, one query per lane (wave-uniform results)
struct RMasks { u64 exp, out, inj, chk; };
__device__ __forceinline__ RMasks round_masks(const QInfo *q, int nq, int r, int lane) {
  bool e = false, o = false, i = false, k = false;
  if (lane < nq) {
    const QInfo x = q[lane];
    const bool chain = (x.flags & QF_CHAIN) != 0;
    e = x.bottom < r && r <= x.top;             // expand round r
    o = !chain && x.bottom <= r && r <= x.top;  // write round r's reach row
    i = x.top == r - 1;                         // starts at r-1
    k = chain && x.bottom <= r && r < x.top;    // leader test at r (chain)
  }
  return RMasks{__ballot(e), __ballot(o), __ballot(i), __ballot(k)};
}

// The full frontier of round r, read per source.  FtGathered: the FT_r buffer
// (produced by step 5, or all-gathered).  FtPending (the persistent local-mode
// kernel): straight from the pending ring slot of round r -- every shard's
// columns are in this context -- plus the queries that start at r, so a round
// needs one grid barrier instead of two.
struct FtGathered {
  const u64 *ft;
  __device__ __forceinline__ u64 operator()(int s) const { return dr::ld_agent(&ft[s]); }
};
struct FtPending {
  const u64 *pend;
  const QInfo *qs;
  int depth, C, slot;
  u64 starts;  // queries whose top is r
  __device__ __forceinline__ u64 operator()(int s) const {
    const int l = s / C;
    u64 v = dr::ld_agent(&pend[((size_t)l * depth + slot) * C + (s - l * C)]);
    for (u64 im = starts; im; im &= im - 1) {
      const int b = __builtin_ctzll(im);
      if (qs[b].src0 == s) v |= 1ULL << b;
    }
    return v;
  }
};

// Steps 1-4 of round r for local shard l (see the file comment).  ft(s) = FT_r[s].
// ledges: LDS chain-edge accumulators; writer: the one thread that records pushes.
template <class Ft>
__device__ void sweep_round(const ShardArgs &a, const Ft &ft, int r, int l, int gw, int nwv, int lane,
                            const RMasks &m, u64 chainq, u64 *ledges, bool writer) {
  const int C = a.C;
  u64 *pend = a.pend + (size_t)l * a.depth * C;
  // 2: chain restarts (every thread takes the same decision)
  u64 rst = 0;
  int L = -1;
  if (m.chk && ((r - 1) & 3) == 0) {
    const int w2 = ((r - 1) >> 2) + 1;
    L = (w2 < a.nlead ? (int)a.lead[w2] : 1) - 1;
    if ((a.pres[(size_t)r * a.W + (L >> 6)] >> (L & 63)) & 1ULL) rst = ft(L) & m.chk;
    if (writer)
      for (u64 x = rst; x; x &= x - 1) {
        const int b = __builtin_ctzll(x);
        a.push_out[a.q[b].push_base + a.push_n[b]] = w2;
        a.push_n[b] += 1;
      }
  }
  // 1 + 3: reach rows and strong expansion.  A wave's work item is (64-source
  // chunk, target word): nchunks * WSs items spread over every wave of the grid.
  const int nchunks = (a.n + 63) >> 6;
  for (int it = gw; it < nchunks * a.WSs; it += nwv) {
    const int s0 = (it / a.WSs) * 64, tw = it % a.WSs;
    const int s = s0 + lane;
    u64 mv = s < a.n ? ft(s) : 0ULL;
    if (s != L) mv &= ~rst;
    if (l == 0 && tw == 0) {
      if (m.out) {
        u64 mine = 0;
        for (u64 om = m.out; om; om &= om - 1) {
          const int b = __builtin_ctzll(om);
          const u64 word = __ballot((mv >> b) & 1ULL);
          if (lane == b) mine = word;
        }
        if ((m.out >> lane) & 1ULL) {
          const QInfo qi = a.q[lane];
          a.out[qi.obase + (int64_t)(r - qi.bottom) * a.W + (s0 >> 6)] = mine;
        }
      }
      const u64 ce = mv & m.exp & chainq;
      if (ce && ledges) {
        const u64 d = a.sdeg[(size_t)r * a.n + s];
        for (u64 x = ce; x; x &= x - 1) atomicAdd(&ledges[__builtin_ctzll(x)], d);
      }
    }
    const u64 me = mv & m.exp;
    if (r < 1 || __ballot(me != 0ULL) == 0ULL) continue;
    const u64 row = (me != 0ULL)
                        ? a.strong[(size_t)r * a.strong_round_stride + (size_t)l * a.strong_shard_stride + (size_t)s * a.SP + tw]
                        : 0ULL;
    u64 act = __ballot(row != 0ULL);
    u64 acc = 0;
    while (act) {  // wave-uniform loop over the sources that contribute
      const int src = __builtin_ctzll(act);
      act &= act - 1;
      const u64 rs = dr::readlane64(row, src), ms = dr::readlane64(me, src);
      if ((rs >> lane) & 1ULL) acc |= ms;
    }
    if (acc) atomicOr(&pend[(size_t)((r - 1) & (a.depth - 1)) * C + tw * 64 + lane], acc);
  }
  // 4: weak expansion
  if (!a.strong_only && r >= 2) {
    const size_t e0 = a.woff[(size_t)l * (a.max_rounds + 1) + r], e1 = a.woff[(size_t)l * (a.max_rounds + 1) + r + 1];
    for (size_t base = e0 + (size_t)gw * 64; base < e1; base += (size_t)nwv * 64) {
      const size_t e = base + lane;
      u64 mv = 0;
      uint32_t key = 0xFFFFFFFFu;
      if (e < e1) {
        const uint32_t w = a.weak[e];
        const int src = (int)((w >> 11) & 2047u);
        mv = ft(src) & m.exp;
        if (src != L) mv &= ~rst;
        const int slot = (r - (int)(w >> 22)) & (a.depth - 1);
        key = (uint32_t)slot * (uint32_t)C + (w & 2047u);
      }
      const u64 act = __ballot(mv != 0ULL);
      if (!act) continue;
      const int first = __builtin_ctzll(act);
      const uint32_t kf = (uint32_t)__builtin_amdgcn_readlane((int)key, first);
      if (__ballot(mv != 0ULL && key != kf) == 0ULL) {
        u64 v = mv;
        for (int d = 32; d; d >>= 1) v |= shfl_xor64(v, d);
        if (lane == first) atomicOr(&pend[kf], v);
      } else if (mv) {
        atomicOr(&pend[key], mv);
      }
    }
  }
}

// step 5 for column t of local shard l: FT_{r1}[col] = pending | starts
__device__ __forceinline__ u64 produce_col(const ShardArgs &a, const QInfo *q, int l, int t, int r1, u64 inj) {
  u64 *slotp = a.pend + ((size_t)l * a.depth + (size_t)(r1 & (a.depth - 1))) * a.C;
  u64 v = atomicExch(&slotp[t], 0ULL);
  const int col = (a.shard0 + l) * a.C + t;
  for (u64 im = inj; im; im &= im - 1) {
    const int b = __builtin_ctzll(im);
    if (q[b].src0 == col) v |= 1ULL << b;
  }
  return v;
}

// Grid-wide barrier of a cooperative launch: monotone arrival counter.  The
// wait is bounded (2 s of the 100 MHz real-time clock) and sticky: a timed-out
// barrier sets *err, every other waiter sees it and the kernel ends instead of
// hanging (the host reports DR_E_HIP).  Returns false once *err is set.
__device__ __forceinline__ bool grid_sync(unsigned *bar, unsigned nblk, unsigned &target, int32_t *err) {
  __shared__ int bad;
  __syncthreads();
  target += nblk;
  if (threadIdx.x == 0) {
    __threadfence();
    atomicAdd(bar, 1u);
    const unsigned long long t0 = wall_clock64();
    int e = 0;
    while (__hip_atomic_load(bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(2);
      if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) { e = 1; break; }
      if (wall_clock64() - t0 > 200000000ULL) {
        atomicOr(err, 1);
        e = 1;
        break;
      }
    }
    __threadfence();
    bad = e;
  }
  __syncthreads();
  return !bad;
}

__device__ __forceinline__ void load_queries(const ShardArgs &a, QInfo *qs, u64 *ledges) {
  if ((int)threadIdx.x < a.nq) qs[threadIdx.x] = a.q[threadIdx.x];
  if (threadIdx.x < SH_BATCH) ledges[threadIdx.x] = 0;
  __syncthreads();
}
__device__ __forceinline__ void flush_edges(const ShardArgs &a, const u64 *ledges) {
  __syncthreads();
  if ((int)threadIdx.x < a.nq && ledges[threadIdx.x]) atomicAdd(&a.cedges[threadIdx.x], ledges[threadIdx.x]);
}

// Local mode: a whole batch, rounds T..Bm, in one cooperative launch.  Round r
// reads its frontier from the pending ring slot of r (FtPending), clears the slot
// of r+1 that the previous round read (the ring has depth >= dmax + 2, so no
// expansion of round r or r+1 targets that slot), expands, and ends at one grid
// barrier.
__global__ void __launch_bounds__(SH_NT) k_shard_sweep(ShardArgs a, int T, int Bm) {
  __shared__ QInfo qs[SH_BATCH];
  __shared__ u64 ledges[SH_BATCH];
  load_queries(a, qs, ledges);
  const int lane = threadIdx.x & 63;
  const u64 chainq = __ballot(lane < a.nq && (qs[lane].flags & QF_CHAIN));
  const int l = blockIdx.y;
  const int nwv = gridDim.x * (SH_NT / 64);
  const int gw = blockIdx.x * (SH_NT / 64) + (threadIdx.x >> 6);
  const unsigned nblk = gridDim.x * gridDim.y;
  const int gthreads = (int)nblk * SH_NT;
  const int gtid = (int)(blockIdx.y * gridDim.x + blockIdx.x) * SH_NT + (int)threadIdx.x;
  const bool writer = blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0;
  const int dm = a.depth - 1;
  unsigned target = 0;
  for (int r = T; r >= Bm; r--) {
    const RMasks m = round_masks(qs, a.nq, r, lane);
    const u64 starts = __ballot(lane < a.nq && qs[lane].top == r);
    if (r < T)
      for (int t = gtid; t < a.nlocal * a.C; t += gthreads) {
        const int ll = t / a.C;
        __hip_atomic_store(&a.pend[((size_t)ll * a.depth + ((r + 1) & dm)) * a.C + (t - ll * a.C)], 0ULL,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // same coherence point as the ORs
      }
    sweep_round(a, FtPending{a.pend, qs, a.depth, a.C, r & dm, starts}, r, l, gw, nwv, lane, m, chainq, ledges,
                writer);
    if (r - 1 < Bm) break;
    if (!grid_sync(a.bar, nblk, target, a.err)) break;
  }
  flush_edges(a, ledges);
}

// One round per launch (RCCL mode, or local mode without cooperative launch):
// the last workgroup of each shard produces its columns of FT_{r-1}.
__global__ void __launch_bounds__(SH_NT) k_shard_round(ShardArgs a, int r, int produce) {
  __shared__ QInfo qs[SH_BATCH];
  __shared__ u64 ledges[SH_BATCH];
  __shared__ int last;
  load_queries(a, qs, ledges);
  const int lane = threadIdx.x & 63;
  const u64 chainq = __ballot(lane < a.nq && (qs[lane].flags & QF_CHAIN));
  const int l = blockIdx.y;
  const int nwv = gridDim.x * (SH_NT / 64);
  const int gw = blockIdx.x * (SH_NT / 64) + (threadIdx.x >> 6);
  const RMasks m = round_masks(qs, a.nq, r, lane);
  const bool writer = blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0;
  sweep_round(a, FtGathered{(r & 1) ? a.ftb1 : a.ftb0}, r, l, gw, nwv, lane, m, chainq, ledges, writer);
  flush_edges(a, ledges);
  if (!produce) return;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    last = atomicAdd(&a.cnt[l], 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  u64 *ftn = ((r - 1) & 1) ? a.ftb1 : a.ftb0;
  for (int t = threadIdx.x; t < a.C; t += SH_NT) {
    const u64 v = produce_col(a, qs, l, t, r - 1, m.inj);
    if (a.local) ftn[(size_t)(a.shard0 + l) * a.C + t] = v;
    else a.send[t] = v;
  }
  if (threadIdx.x == 0) a.cnt[l] = 0;
}

// Commit step k (1..3) of waves w0..w0+nw-1: partial hits of shard g,
// P[g][wi][word] bit s <=> row_g(4w-3+k, s) & S_{k-1}[cols of g] != 0.
// S_0 = S0 (leader bits, [nw][W]); S_{k-1} = OR over the G partials of Pin.
__global__ void __launch_bounds__(SH_NT) k_shard_vote(ShardArgs a, int w0, int nw, int k, int G, const u64 *S0,
                                                      const u64 *Pin, u64 *Pout) {
  __shared__ u64 S[64];
  const int l = blockIdx.y, g = a.shard0 + l;
  const int bpw = (a.n + SH_NT - 1) / SH_NT;
  const int wi = blockIdx.x / bpw, sb = blockIdx.x % bpw;
  if (wi >= nw) return;
  const int r = 4 * (w0 + wi - 1) + 1 + k;
  if ((int)threadIdx.x < a.WSs) {
    const int cw = g * a.WSs + (int)threadIdx.x;
    u64 v = 0;
    if (cw < a.W) {
      if (k == 1) v = S0[(size_t)wi * a.W + cw];
      else
        for (int gg = 0; gg < G; gg++) v |= Pin[((size_t)gg * nw + wi) * a.W + cw];
    }
    S[threadIdx.x] = v;
  }
  __syncthreads();
  const int s = sb * SH_NT + (int)threadIdx.x;
  bool hit = false;
  if (s < a.n) {
    const u64 *row = a.strong + (size_t)r * a.strong_round_stride + (size_t)l * a.strong_shard_stride + (size_t)s * a.SP;
    for (int j = 0; j < a.WSs; j++) hit |= (row[j] & S[j]) != 0ULL;
  }
  const u64 b = __ballot(hit);
  if ((threadIdx.x & 63) == 0 && s < a.n)
    Pout[((size_t)(a.local ? g : 0) * nw + wi) * a.W + (s >> 6)] = b;
}

// vcount = |S_3|: one wave per wave index, lane = word, the G partials OR-ed
__global__ __launch_bounds__(SH_NT) void k_shard_vcount(const u64 *P, int G, int nw, int W, int32_t *vc) {
  const int wi = blockIdx.x * (SH_NT / 64) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (wi >= nw) return;
  u64 v = 0;
  if (lane < W)
    for (int g = 0; g < G; g++) v |= P[((size_t)g * nw + wi) * W + lane];
  const u64 c = dr::wave_sum((u64)__popcll(v));
  if (lane == 0) vc[wi] = (int32_t)c;
}

// Delivery masks, one wave per round r (lane = word): X = reach & present, and
// in paper mode & ~delivered, the leaders scanned in pop order (Alg. 3 line 54).
__global__ void __launch_bounds__(SH_NT) k_shard_dmask(u64 *out, const QInfo *q, int nq, int rmax, int W,
                                                       const u64 *pres, u64 *D, int paper) {
  const int r = 1 + (int)(blockIdx.x * (SH_NT / 64) + (threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  if (r > rmax || lane >= W) return;
  const u64 pw = pres[(size_t)r * W + lane];
  u64 Dw = paper ? D[(size_t)r * W + lane] : 0ULL;
  for (int b = 0; b < nq; b++) {
    const QInfo x = q[b];
    if (r < x.bottom || r > x.last) continue;
    u64 *p = &out[x.obase + (int64_t)(r - x.bottom) * W + lane];
    const u64 v = *p & pw & ~Dw;  // Dw stays 0 in ref mode
    if (paper) Dw |= v;
    *p = v;
  }
  if (paper) D[(size_t)r * W + lane] = Dw;
}

// Per (query, round): delivered count and the strong + weak degree sum
// (rdeg[r] for a round delivered whole).  cnt: [nq][rstride].
__global__ void __launch_bounds__(SH_NT) k_shard_count(const u64 *out, const QInfo *q, int W, int n, int rstride,
                                                       const u64 *pres, const uint16_t *sdeg, const uint16_t *wdeg,
                                                       const u64 *rdeg, uint32_t *cnt, u64 *qedges) {
  const int b = blockIdx.y;
  const int r = 1 + (int)(blockIdx.x * (SH_NT / 64) + (threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  const QInfo x = q[b];
  if (r > x.last || r < x.bottom) return;
  const u64 v = lane < W ? out[x.obase + (int64_t)(r - x.bottom) * W + lane] : 0ULL;
  const u64 pw = lane < W ? pres[(size_t)r * W + lane] : 0ULL;
  const uint32_t c = (uint32_t)dr::wave_sum((u64)__popcll(v));
  u64 e;
  if (__ballot(v != pw) == 0ULL) {
    e = rdeg[r];
  } else {
    u64 acc = 0;
    for (u64 y = v; y; y &= y - 1) {
      const size_t at = (size_t)r * n + lane * 64 + __builtin_ctzll(y);
      acc += (u64)sdeg[at] + wdeg[at];
    }
    e = dr::wave_sum(acc);
  }
  if (lane == 0) {
    cnt[(size_t)b * rstride + r] = c;
    if (e) atomicAdd(&qedges[b], e);
  }
}

// Per query: exclusive scan of the per-round counts -> positions; total count.
__global__ void __launch_bounds__(SH_NT) k_shard_scan(const QInfo *q, int rstride, uint32_t *cnt, u64 *qcount) {
  __shared__ u64 part[SH_NT];
  const int b = blockIdx.x;
  const QInfo x = q[b];
  const int lo = std::max(1, x.bottom), hi = x.last;  // rounds lo..hi
  uint32_t *c = cnt + (size_t)b * rstride;
  const int span = hi >= lo ? hi - lo + 1 : 0;
  const int per = (span + SH_NT - 1) / SH_NT;
  const int a0 = lo + (int)threadIdx.x * per, a1 = std::min(hi + 1, a0 + per);
  u64 s = 0;
  for (int r = a0; r < a1; r++) s += c[r];
  part[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    u64 run = 0;
    for (int t = 0; t < SH_NT; t++) {
      const u64 v = part[t];
      part[t] = run;
      run += v;
    }
    qcount[b] = run;
  }
  __syncthreads();
  u64 run = part[threadIdx.x];
  for (int r = a0; r < a1; r++) {  // counts -> exclusive positions, in place (u32: < 2^32 per pop)
    const uint32_t v = c[r];
    c[r] = (uint32_t)run;
    run += v;
  }
}

// Per (query, round): sum of digest_term(r, s, k) over the delivered slots of
// round r in insertion order, k = the query's position.
__global__ void __launch_bounds__(SH_NT) k_shard_digest(const u64 *out, const QInfo *q, int W, int rstride,
                                                        const uint32_t *pos, const uint32_t *slot_off,
                                                        const uint16_t *slot_src, u64 *qdigest) {
  const int b = blockIdx.y;
  const int r = 1 + (int)(blockIdx.x * (SH_NT / 64) + (threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  const QInfo x = q[b];
  if (r > x.last || r < x.bottom) return;
  const u64 xw = lane < W ? out[x.obase + (int64_t)(r - x.bottom) * W + lane] : 0ULL;
  u64 k = pos[(size_t)b * rstride + r];
  u64 acc = 0;
  const uint32_t s0 = slot_off[r], s1 = slot_off[r + 1];
  for (uint32_t base = s0; base < s1; base += 64) {
    const uint32_t sl = base + lane;
    const int s = sl < s1 ? (int)slot_src[sl] : 0;
    const int wd = s > 0 ? (s - 1) >> 6 : 0;
    const u64 word = ((u64)(uint32_t)__shfl((int)(xw >> 32), wd, 64) << 32) | (uint32_t)__shfl((int)(uint32_t)xw, wd, 64);
    const bool in = s > 0 && ((word >> ((s - 1) & 63)) & 1ULL);
    const u64 bal = __ballot(in);
    if (in) acc += dr::digest_term((uint32_t)r, (uint32_t)s, k + (u64)__popcll(bal & ((1ULL << lane) - 1ULL)));
    k += (u64)__popcll(bal);
  }
  const u64 t = dr::wave_sum(acc);
  if (lane == 0 && t) atomicAdd(&qdigest[b], t);
}

}  // namespace

struct dr_shard {
  int n = 0, f = 0, W = 0, G = 1, shard0 = 0, nlocal = 1, WSs = 1, SP = 1, C = 64, max_rounds = 0, dev = 0;
  bool local = true;
  int persistent = 1;  // DR_SHARD_OPT_PERSISTENT
  int memo = 1;        // DR_SHARD_OPT_MEMO
  int stepped = 0;     // DR_SHARD_OPT_STEPPED: the memo replay's stepped form even when every column is here
  int phase_timing = 1;  // DR_SHARD_OPT_PHASE_TIMING
  // a phase boundary of the memo replay (recorded only with phase timing)
  hipError_t mark(int k) { return phase_timing ? hipEventRecord(evs[k], stream) : hipSuccess; }
  int pass_geo = 0;    // k_ms_pass geometry (tuning: DR_SHARD_PASS_GEO)
  // k_ms_wu on the side stream beside the pass (tuning: DR_SHARD_WU_SIDE=1); by default
  // before it on the main stream: C4 G = 1 0.348 vs 0.358 ms, G = 8 0.380 vs 0.398 ms, the
  // pass's workgroups queue behind the side stream's (profiles/r04/)
  int wu_side = 0;
  int emit_fused = 0;  // REF emission inside the fused sweep (tuning: DR_SHARD_EMIT_FUSED=1)
  int step_nt = 256;   // k_ms_step2 threads per query (tuning: DR_SHARD_STEP_NT=128)
  int keep4 = 1;       // stepped pass: round 4w's rows with cached loads, re-read by the third vote step (off: DR_SHARD_KEEP4=0)
  int nrounds = 0, dmax = 1, depth = 2;
  size_t max_weak_round = 0;
  hipStream_t stream = nullptr;
  hipStream_t side = nullptr;                       // k_ms_wu beside k_ms_pass (fork / join events)
  hipEvent_t fork = nullptr, join = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
  hipEvent_t evs[5] = {};  // the memo replay's phase boundaries
  ncclComm_t comm = nullptr;
  SBuf strong, weak, woff, ft[2], send, pend, cnt, out, qinfo;
  // per-vertex metadata, full width on every shard
  SBuf pres, sdeg, wdeg, rdeg, slot_off, slot_src, lead;
  // per-call scratch
  SBuf bar, errf, push_out, push_n, cedges, vote_s0, vote_p[2], vote_send, vcount, D, pcnt, qcnt, qedges, qdig;
  // memoized replay (shard_memo.hpp): strong degree per round, round summaries,
  // canonical cone and prefixes, the stepped queries' buffers
  SBuf sdr, mU, mWU, mK, mgood, mRD, mCE, mRG, mC, mE, mG, mksend, mkrecv, mq, mpend, mrecv[2], msend, mmasks,
      mpush, mqidx, mqout;
  // stepped form: the canonical walk's query; S_1 per wave (k_ms_lcol; RCCL mode: the
  // exchanged partials, lcol_g slots of lcol_nw waves), valid until an append or a coin change
  SBuf mcq, mlcol, mlcolp;
  // the stepped canonical walk's own pending ring and exchanged frontiers: a walk resumed
  // after the batch steps ran (a continuation, replay_memo) finds them as it left them
  SBuf cpend, crecv[2], csend;
  bool lcol_ok = false;
  int lcol_nw = 1, lcol_g = 1;
  uint64_t lead_version = 0;  // bumped by every coin change
  uint64_t pops_key[4] = {};  // what the device's pop query table was built for (upload_pops)
  uint64_t syncs = 0;  // host waits of the last query call (dr_shard_host_syncs)
  std::vector<uint64_t> h_sdr;  // strong degree sum per round (host copy)
  int hint_canon = 8, hint_batch = 12;  // steps the last replay's canonical walk / query batch took
  // pinned staging for the memo replay's small transfers (queries in, results out);
  // reset at each replay's start, grown after a stream sync
  char *pin = nullptr;
  size_t pin_cap = 0, pin_used = 0;
  SBuf ppref;                   // [round] |P_1| + .. + |P_r| (present vertices, round 0 excluded)
  std::vector<u64> h_ppref;
  SBuf mSG, mout;               // speculative canonical digests; the memo replay's output region
  std::vector<std::vector<uint32_t>> h_weak;  // per local shard
  std::vector<std::vector<uint64_t>> h_woff;  // per local shard, absolute offsets, size nrounds+1
  // weak columns per local shard (the memoized replay, shard_memo.hpp): one entry per
  // distinct weak target (delta, column) of a round whose column is this shard's, key
  // delta << 11 | local column, and the W-word bitset of the round's sources with it
  std::vector<std::vector<uint32_t>> h_wck;
  std::vector<std::vector<u64>> h_wcr;
  std::vector<std::vector<uint64_t>> h_wcro;  // per local shard, absolute offsets, size nrounds+1
  SBuf wck, wcr, wcro;
  std::vector<u64> h_pres;                    // [nrounds][W]
  std::vector<uint64_t> h_deg;                // strong degree sum per round
  std::vector<uint32_t> h_slot_off{0};
  std::vector<uint16_t> h_lead;
  bool weak_dirty = false;
  float last_ms = 0;
  uint64_t last_rounds = 0, last_xbytes = 0;
  float ms_vote = 0, ms_sweep = 0, ms_emit = 0;
  std::string err;
  int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    err = buf;
    return code;
  }
  int lead_src(int w) const { return (w >= 0 && w < (int)h_lead.size()) ? h_lead[w] : 1; }
  bool is_present(int r, int s /*1-based*/) const {
    if (r < 0 || r >= nrounds || s < 1 || s > n) return false;
    return (h_pres[(size_t)r * W + ((s - 1) >> 6)] >> ((s - 1) & 63)) & 1ULL;
  }
};

#define SHCHK(c, x)                                                                                  \
  do {                                                                                               \
    hipError_t e_ = (x);                                                                             \
    if (e_ != hipSuccess) return (c)->fail(DR_E_HIP, "%s: %s (%s:%d)", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
  } while (0)
#define SHNCCL(c, x)                                                                                 \
  do {                                                                                               \
    ncclResult_t r_ = (x);                                                                           \
    if (r_ != ncclSuccess) return (c)->fail(DR_E_RCCL, "%s: %s", #x, ncclGetErrorString(r_));        \
  } while (0)

namespace {

int sh_set_device(dr_shard *c) {
  hipError_t e = hipSetDevice(c->dev);
  if (e != hipSuccess) return c->fail(DR_E_HIP, "hipSetDevice(%d): %s", c->dev, hipGetErrorString(e));
  return DR_OK;
}

// upload the weak edges appended since the last query (kept on the host until then)
int sync_weak(dr_shard *c) {
  if (!c->weak_dirty) return DR_OK;
  size_t total = 0;
  for (auto &v : c->h_weak) total += v.size();
  SHCHK(c, c->weak.ensure(std::max<size_t>(total, 1) * 4));
  SHCHK(c, c->woff.ensure((size_t)c->nlocal * (c->max_rounds + 1) * 8));
  std::vector<uint64_t> offs((size_t)c->nlocal * (c->max_rounds + 1), 0);
  size_t base = 0;
  for (int l = 0; l < c->nlocal; l++) {
    const auto &w = c->h_weak[l];
    if (!w.empty())
      SHCHK(c, hipMemcpyAsync(c->weak.as<uint32_t>() + base, w.data(), w.size() * 4, hipMemcpyHostToDevice, c->stream));
    uint64_t *o = &offs[(size_t)l * (c->max_rounds + 1)];
    for (int r = 0; r <= c->max_rounds; r++)
      o[r] = base + c->h_woff[l][std::min<size_t>(r, c->h_woff[l].size() - 1)];
    base += w.size();
  }
  SHCHK(c, hipMemcpyAsync(c->woff.p, offs.data(), offs.size() * 8, hipMemcpyHostToDevice, c->stream));
  // weak columns, concatenated over the local shards; wcro absolute like woff
  size_t ncol = 0;
  for (auto &v : c->h_wck) ncol += v.size();
  SHCHK(c, c->wck.ensure(std::max<size_t>(ncol, 1) * 4));
  SHCHK(c, c->wcr.ensure(std::max<size_t>(ncol, 1) * c->W * 8));
  SHCHK(c, c->wcro.ensure((size_t)c->nlocal * (c->max_rounds + 1) * 8));
  std::vector<uint64_t> coffs((size_t)c->nlocal * (c->max_rounds + 1), 0);
  size_t cb = 0;
  for (int l = 0; l < c->nlocal; l++) {
    const auto &k = c->h_wck[l];
    if (!k.empty()) {
      SHCHK(c, hipMemcpyAsync(c->wck.as<uint32_t>() + cb, k.data(), k.size() * 4, hipMemcpyHostToDevice, c->stream));
      SHCHK(c, hipMemcpyAsync(c->wcr.as<u64>() + cb * c->W, c->h_wcr[l].data(), k.size() * c->W * 8,
                              hipMemcpyHostToDevice, c->stream));
    }
    uint64_t *o = &coffs[(size_t)l * (c->max_rounds + 1)];
    for (int r = 0; r <= c->max_rounds; r++)
      o[r] = cb + c->h_wcro[l][std::min<size_t>(r, c->h_wcro[l].size() - 1)];
    cb += k.size();
  }
  SHCHK(c, hipMemcpyAsync(c->wcro.p, coffs.data(), coffs.size() * 8, hipMemcpyHostToDevice, c->stream));
  c->syncs++;
  SHCHK(c, hipStreamSynchronize(c->stream));
  c->weak_dirty = false;
  return DR_OK;
}

ShardArgs make_args(dr_shard *c, int nq, int strong_only) {
  ShardArgs a{};
  a.strong = c->strong.as<u64>();
  a.weak = c->weak.as<uint32_t>();
  a.woff = c->woff.as<uint64_t>();
  a.pres = c->pres.as<u64>();
  a.lead = c->lead.as<uint16_t>();
  a.sdeg = c->sdeg.as<uint16_t>();
  a.ftb0 = c->ft[0].as<u64>();
  a.ftb1 = c->ft[1].as<u64>();
  a.send = c->send.as<u64>();
  a.pend = c->pend.as<u64>();
  a.cnt = c->cnt.as<unsigned>();
  a.bar = c->bar.as<unsigned>();
  a.err = c->errf.as<int32_t>();
  a.out = c->out.as<u64>();
  a.q = c->qinfo.as<QInfo>();
  a.push_out = c->push_out.as<int32_t>();
  a.push_n = c->push_n.as<int32_t>();
  a.cedges = c->cedges.as<u64>();
  a.n = c->n;
  a.W = c->W;
  a.WSs = c->WSs;
  a.SP = c->SP;
  a.C = c->C;
  a.depth = c->depth;
  a.shard0 = c->shard0;
  a.nlocal = c->nlocal;
  a.local = c->local ? 1 : 0;
  a.max_rounds = c->max_rounds;
  a.nq = nq;
  a.strong_only = strong_only;
  a.nlead = (int32_t)c->h_lead.size();
  a.strong_shard_stride = (int64_t)c->n * c->SP;
  a.strong_round_stride = (int64_t)c->nlocal * c->n * c->SP;
  return a;
}

// One batch of <= 64 sweep queries (rounds max top .. min bottom).  Reach rows
// land in c->out at dq[i].obase; chain pushes / edges in c->push_* / c->cedges.
int sweep_batch(dr_shard *c, std::vector<QInfo> &dq, int strong_only) {
  const int nq = (int)dq.size();
  int T = 0, Bm = 1 << 30;
  for (auto &q : dq) {
    T = std::max(T, q.top);
    Bm = std::min(Bm, q.bottom);
  }
  const int NT = c->G * c->C;
  SHCHK(c, hipMemcpyAsync(c->qinfo.p, dq.data(), nq * sizeof(QInfo), hipMemcpyHostToDevice, c->stream));
  SHCHK(c, hipMemsetAsync(c->pend.p, 0, (size_t)c->nlocal * c->depth * c->C * 8, c->stream));
  SHCHK(c, hipMemsetAsync(c->cnt.p, 0, (size_t)c->nlocal * 4, c->stream));
  std::vector<u64> ft0(NT, 0);
  for (int i = 0; i < nq; i++)
    if (dq[i].top == T && dq[i].src0 >= 0) ft0[dq[i].src0] |= 1ULL << i;
  SHCHK(c, hipMemcpyAsync(c->ft[T & 1].p, ft0.data(), (size_t)NT * 8, hipMemcpyHostToDevice, c->stream));
  ShardArgs a = make_args(c, nq, strong_only);
  const int item_waves = (c->n + 63) / 64 * c->WSs;  // (source chunk, target word) items
  const size_t weak_waves = strong_only ? 0 : (c->max_weak_round + 63) / 64;
  int gx = (int)std::max<size_t>((item_waves + 3) / 4, std::min<size_t>(128, (weak_waves + 3) / 4));
  if (c->local && c->persistent) {
    // every workgroup must be resident: cap the grid by the occupancy of this device
    int per_cu = 0, ncu = 0;
    SHCHK(c, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_shard_sweep, SH_NT, 0));
    SHCHK(c, hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->dev));
    // every workgroup arrives at each round's barrier: keep the grid small (the
    // round's work is a few hundred waves) and resident
    const int cap = std::max(1, std::min(per_cu * ncu, 128) / std::max(1, c->nlocal));
    gx = std::max(1, std::min(gx, cap));
    SHCHK(c, hipMemsetAsync(c->bar.p, 0, 4, c->stream));
    void *args[] = {&a, &T, &Bm};
    SHCHK(c, hipLaunchCooperativeKernel(reinterpret_cast<const void *>(k_shard_sweep), dim3(gx, c->nlocal),
                                        dim3(SH_NT), args, 0, c->stream));
    c->last_rounds += (uint64_t)(T - Bm + 1);
    return DR_OK;
  }
  const dim3 grid(gx, c->nlocal), block(SH_NT);
  for (int r = T; r >= Bm; r--) {
    const int produce = r - 1 >= Bm;
    hipLaunchKernelGGL(k_shard_round, grid, block, 0, c->stream, a, r, produce);
    SHCHK(c, hipGetLastError());
    if (produce && !c->local) {
      SHNCCL(c, ncclAllGather(c->send.p, c->ft[(r - 1) & 1].p, (size_t)c->C, ncclUint64, c->comm, c->stream));
      c->last_xbytes += (uint64_t)c->C * 8;
    }
    c->last_rounds++;
  }
  return DR_OK;
}

int check_barrier(dr_shard *c) {
  int32_t e = 0;
  SHCHK(c, hipMemcpyAsync(&e, c->errf.p, 4, hipMemcpyDeviceToHost, c->stream));
  SHCHK(c, hipStreamSynchronize(c->stream));
  if (e) return c->fail(DR_E_HIP, "k_shard_sweep: grid barrier timed out (workgroups not co-resident)");
  return DR_OK;
}

int prepare_queries(dr_shard *c, int strong_only) {
  if (int rc = sync_weak(c)) return rc;
  (void)strong_only;
  SHCHK(c, c->qinfo.ensure(SH_BATCH * sizeof(QInfo)));
  SHCHK(c, c->bar.ensure(64));
  SHCHK(c, c->errf.ensure(64));
  SHCHK(c, c->push_n.ensure(SH_BATCH * 4));
  SHCHK(c, c->cedges.ensure(SH_BATCH * 8));
  SHCHK(c, hipMemsetAsync(c->errf.p, 0, 4, c->stream));
  return DR_OK;
}

// reach-set queries, in batches of 64, timed with HIP events; rows land in host `out` at hbase[i]
int run_queries(dr_shard *c, const std::vector<QInfo> &qs, const std::vector<size_t> &hbase, int strong_only,
                uint64_t *out) {
  if (int rc = prepare_queries(c, strong_only)) return rc;
  c->last_rounds = 0;
  c->last_xbytes = 0;
  SHCHK(c, hipEventRecord(c->ev0, c->stream));
  for (size_t i0 = 0; i0 < qs.size(); i0 += SH_BATCH) {
    const size_t i1 = std::min(qs.size(), i0 + SH_BATCH);
    std::vector<QInfo> dq(qs.begin() + i0, qs.begin() + i1);
    int64_t words = 0;
    for (auto &q : dq) {
      q.obase = words;
      words += (int64_t)(q.top - q.bottom + 1) * c->W;
    }
    SHCHK(c, c->out.ensure(std::max<int64_t>(words, 1) * 8));
    if (int rc = sweep_batch(c, dq, strong_only)) return rc;
    std::vector<u64> tmp(words);
    SHCHK(c, hipMemcpyAsync(tmp.data(), c->out.p, words * 8, hipMemcpyDeviceToHost, c->stream));
    SHCHK(c, hipStreamSynchronize(c->stream));
    for (size_t i = 0; i < dq.size(); i++)
      std::memcpy(out + hbase[i0 + i], &tmp[dq[i].obase], (size_t)(dq[i].top - dq[i].bottom + 1) * c->W * 8);
  }
  SHCHK(c, hipEventRecord(c->ev1, c->stream));
  SHCHK(c, hipEventSynchronize(c->ev1));
  SHCHK(c, hipEventElapsedTime(&c->last_ms, c->ev0, c->ev1));
  return check_barrier(c);
}

// waveReady's commit decision for waves w0..w1 (all evaluable; see votes())
int vote_range(dr_shard *c, int w0, int nw, uint8_t *commit, int32_t *vcount) {
  const int W = c->W, G = c->G;
  std::vector<u64> s0((size_t)nw * W, 0);
  std::vector<uint8_t> has(nw, 0);
  for (int i = 0; i < nw; i++) {
    const int w = w0 + i, L = c->lead_src(w);
    if (c->is_present(4 * (w - 1) + 1, L)) {
      has[i] = 1;
      s0[(size_t)i * W + ((L - 1) >> 6)] = 1ULL << ((L - 1) & 63);
    }
  }
  const size_t pw = (size_t)G * nw * W * 8;
  SHCHK(c, c->vote_s0.ensure(s0.size() * 8));
  SHCHK(c, c->vote_p[0].ensure(pw));
  SHCHK(c, c->vote_p[1].ensure(pw));
  SHCHK(c, c->vote_send.ensure((size_t)nw * W * 8));
  SHCHK(c, c->vcount.ensure((size_t)nw * 4));
  SHCHK(c, hipMemcpyAsync(c->vote_s0.p, s0.data(), s0.size() * 8, hipMemcpyHostToDevice, c->stream));
  ShardArgs a = make_args(c, 0, 1);
  const int bpw = (c->n + SH_NT - 1) / SH_NT;
  for (int k = 1; k <= 3; k++) {
    u64 *pin = c->vote_p[(k + 1) & 1].as<u64>(), *pout = c->vote_p[k & 1].as<u64>();
    u64 *dst = c->local ? pout : c->vote_send.as<u64>();
    hipLaunchKernelGGL(k_shard_vote, dim3(nw * bpw, c->nlocal), dim3(SH_NT), 0, c->stream, a, w0, nw, k, G,
                       c->vote_s0.as<u64>(), pin, dst);
    SHCHK(c, hipGetLastError());
    if (!c->local) {
      SHNCCL(c, ncclAllGather(c->vote_send.p, pout, (size_t)nw * W, ncclUint64, c->comm, c->stream));
      c->last_xbytes += (uint64_t)nw * W * 8;
    }
  }
  hipLaunchKernelGGL(k_shard_vcount, dim3((nw + SH_NT / 64 - 1) / (SH_NT / 64)), dim3(SH_NT), 0, c->stream,
                     c->vote_p[1].as<u64>(), G, nw,
                     W, c->vcount.as<int32_t>());
  SHCHK(c, hipGetLastError());
  std::vector<int32_t> vc(nw);
  SHCHK(c, hipMemcpyAsync(vc.data(), c->vcount.p, (size_t)nw * 4, hipMemcpyDeviceToHost, c->stream));
  SHCHK(c, hipStreamSynchronize(c->stream));
  for (int i = 0; i < nw; i++) {
    vcount[i] = has[i] ? vc[i] : -1;
    commit[i] = has[i] && vc[i] >= 2 * c->f + 1;
  }
  return DR_OK;
}

// dr_wave_commit semantics (engine.hip commit_range): waves past the DAG panic
// (Go: index out of range) unless their leader is absent.
int votes(dr_shard *c, int w0, int w1, uint8_t *commit, int32_t *vcount) {
  if (w0 < 1 || w1 < w0) return c->fail(DR_E_INVAL, "wave range [%d,%d] invalid (waves are 1-based)", w0, w1);
  int wk = w0 - 1;
  while (wk + 1 <= w1 && 4 * (wk + 1) < c->nrounds) wk++;
  for (int w = wk + 1; w <= w1; w++) {
    const int r1 = 4 * (w - 1) + 1;
    if (r1 >= c->nrounds) return c->fail(DR_E_INVAL, "wave %d: leader round %d not in the DAG (Go: index out of range)", w, r1);
    if (c->is_present(r1, c->lead_src(w))) return c->fail(DR_E_INVAL, "wave %d: round %d not in the DAG (Go: index out of range)", w, 4 * w);
    commit[w - w0] = 0;
    vcount[w - w0] = -1;
  }
  if (wk < w0) return DR_OK;
  return vote_range(c, w0, wk - w0 + 1, commit, vcount);
}

struct ChainTask { int wave, floor; };

// Leader chains (process.go:341-350): pushes[i] = waves pushed by task i, in push order.
int chains(dr_shard *c, const std::vector<ChainTask> &tasks, std::vector<std::vector<int32_t>> &pushes,
           uint64_t *edges_total) {
  pushes.assign(tasks.size(), {});
  std::vector<QInfo> qv;
  std::vector<int> qi;
  for (size_t i = 0; i < tasks.size(); i++) {
    pushes[i].push_back(tasks[i].wave);
    if (tasks[i].wave - 1 < tasks[i].floor + 1) continue;
    if (tasks[i].floor < 0) return c->fail(DR_E_INVAL, "decidedWave %d < 0 (Go: waveRound(0,1) index out of range)", tasks[i].floor);
    QInfo q{};
    q.top = 4 * (tasks[i].wave - 1) + 1;
    q.bottom = 4 * tasks[i].floor + 1;
    q.src0 = c->lead_src(tasks[i].wave) - 1;
    q.flags = QF_CHAIN;
    qv.push_back(q);
    qi.push_back((int)i);
  }
  if (edges_total) *edges_total = 0;
  if (qv.empty()) return DR_OK;
  if (int rc = prepare_queries(c, 1)) return rc;
  for (size_t i0 = 0; i0 < qv.size(); i0 += SH_BATCH) {
    const size_t i1 = std::min(qv.size(), i0 + SH_BATCH);
    std::vector<QInfo> dq(qv.begin() + i0, qv.begin() + i1);
    int32_t off = 0;
    for (auto &q : dq) {
      q.push_base = off;
      off += (q.top - q.bottom) / 4 + 1;
    }
    SHCHK(c, c->push_out.ensure((size_t)std::max(off, 1) * 4));
    SHCHK(c, hipMemsetAsync(c->push_n.p, 0, SH_BATCH * 4, c->stream));
    SHCHK(c, hipMemsetAsync(c->cedges.p, 0, SH_BATCH * 8, c->stream));
    if (int rc = sweep_batch(c, dq, 1)) return rc;
    std::vector<int32_t> pn(dq.size()), po(off);
    std::vector<u64> ce(dq.size());
    SHCHK(c, hipMemcpyAsync(pn.data(), c->push_n.p, dq.size() * 4, hipMemcpyDeviceToHost, c->stream));
    SHCHK(c, hipMemcpyAsync(po.data(), c->push_out.p, (size_t)off * 4, hipMemcpyDeviceToHost, c->stream));
    SHCHK(c, hipMemcpyAsync(ce.data(), c->cedges.p, dq.size() * 8, hipMemcpyDeviceToHost, c->stream));
    SHCHK(c, hipStreamSynchronize(c->stream));
    for (size_t j = 0; j < dq.size(); j++) {
      auto &p = pushes[qi[i0 + j]];
      for (int x = 0; x < pn[j]; x++) p.push_back(po[dq[j].push_base + x]);
      if (edges_total) *edges_total += ce[j];
    }
  }
  return check_barrier(c);
}

struct Pop { int round, source, cur; };

// orderVertices deliveries of `pops` in pop order: one cone per distinct
// (round, source), emitted over rounds 1..min(cur, round).
int deliver(dr_shard *c, const std::vector<Pop> &pops, int mode, uint64_t *pcount, uint64_t *pdigest,
            uint64_t *pedges) {
  const int W = c->W;
  std::map<std::pair<int, int>, int> key;
  std::vector<int> kidx(pops.size());
  std::vector<Pop> uniq;
  std::vector<uint8_t> first(pops.size(), 0);
  for (size_t i = 0; i < pops.size(); i++) {
    auto it = key.find({pops[i].round, pops[i].source});
    if (it == key.end()) {
      it = key.emplace(std::make_pair(pops[i].round, pops[i].source), (int)uniq.size()).first;
      uniq.push_back(pops[i]);
      first[i] = 1;
    }
    kidx[i] = it->second;
  }
  const int K = (int)uniq.size();
  std::vector<u64> kc(K), kd(K), ke(K);
  if (int rc = prepare_queries(c, 0)) return rc;
  int rmax = 1;
  for (auto &p : uniq) rmax = std::max(rmax, std::min(p.cur, p.round));
  const int rstride = c->nrounds + 1;
  SHCHK(c, c->pcnt.ensure((size_t)SH_BATCH * rstride * 4));
  SHCHK(c, c->qcnt.ensure(SH_BATCH * 8));
  SHCHK(c, c->qedges.ensure(SH_BATCH * 8));
  SHCHK(c, c->qdig.ensure(SH_BATCH * 8));
  if (mode == DR_DELIVER_PAPER) {
    SHCHK(c, c->D.ensure((size_t)c->nrounds * W * 8));
    SHCHK(c, hipMemsetAsync(c->D.p, 0, (size_t)c->nrounds * W * 8, c->stream));
  }
  float ms_sw = 0, ms_em = 0;
  for (int i0 = 0; i0 < K; i0 += SH_BATCH) {
    const int i1 = std::min(K, i0 + SH_BATCH);
    std::vector<QInfo> dq;
    int64_t words = 0;
    int bmax = 1;
    for (int i = i0; i < i1; i++) {
      QInfo q{};
      q.top = uniq[i].round;
      q.bottom = std::min(1, q.top);  // round 0 is never delivered nor expanded from
      q.src0 = (uniq[i].source >= 1 && uniq[i].source <= c->n) ? uniq[i].source - 1 : -1;
      q.last = std::min(uniq[i].cur, q.top);
      q.obase = words;
      words += (int64_t)(q.top - q.bottom + 1) * W;
      bmax = std::max(bmax, q.last);
      dq.push_back(q);
    }
    const int nq = (int)dq.size();
    SHCHK(c, c->out.ensure(std::max<int64_t>(words, 1) * 8));
    SHCHK(c, hipEventRecord(c->ev0, c->stream));
    if (int rc = sweep_batch(c, dq, 0)) return rc;
    SHCHK(c, hipEventRecord(c->ev1, c->stream));
    SHCHK(c, hipMemsetAsync(c->qedges.p, 0, SH_BATCH * 8, c->stream));
    SHCHK(c, hipMemsetAsync(c->qdig.p, 0, SH_BATCH * 8, c->stream));
    const int rb = (bmax + 3) / 4;  // 4 rounds (waves) per workgroup
    const QInfo *qd = c->qinfo.as<QInfo>();
    hipLaunchKernelGGL(k_shard_dmask, dim3(rb), dim3(SH_NT), 0, c->stream, c->out.as<u64>(), qd, nq, bmax, W,
                       c->pres.as<u64>(), c->D.as<u64>(), mode == DR_DELIVER_PAPER ? 1 : 0);
    SHCHK(c, hipGetLastError());
    hipLaunchKernelGGL(k_shard_count, dim3(rb, nq), dim3(SH_NT), 0, c->stream, c->out.as<u64>(), qd, W, c->n,
                       rstride, c->pres.as<u64>(), c->sdeg.as<uint16_t>(), c->wdeg.as<uint16_t>(), c->rdeg.as<u64>(),
                       c->pcnt.as<uint32_t>(), c->qedges.as<u64>());
    SHCHK(c, hipGetLastError());
    hipLaunchKernelGGL(k_shard_scan, dim3(nq), dim3(SH_NT), 0, c->stream, qd, rstride, c->pcnt.as<uint32_t>(),
                       c->qcnt.as<u64>());
    SHCHK(c, hipGetLastError());
    hipLaunchKernelGGL(k_shard_digest, dim3(rb, nq), dim3(SH_NT), 0, c->stream, c->out.as<u64>(), qd, W, rstride,
                       c->pcnt.as<uint32_t>(), c->slot_off.as<uint32_t>(), c->slot_src.as<uint16_t>(),
                       c->qdig.as<u64>());
    SHCHK(c, hipGetLastError());
    SHCHK(c, hipEventRecord(c->ev2, c->stream));
    SHCHK(c, hipMemcpyAsync(&kc[i0], c->qcnt.p, (size_t)nq * 8, hipMemcpyDeviceToHost, c->stream));
    SHCHK(c, hipMemcpyAsync(&ke[i0], c->qedges.p, (size_t)nq * 8, hipMemcpyDeviceToHost, c->stream));
    SHCHK(c, hipMemcpyAsync(&kd[i0], c->qdig.p, (size_t)nq * 8, hipMemcpyDeviceToHost, c->stream));
    SHCHK(c, hipStreamSynchronize(c->stream));
    float a = 0, b = 0;
    SHCHK(c, hipEventElapsedTime(&a, c->ev0, c->ev1));
    SHCHK(c, hipEventElapsedTime(&b, c->ev1, c->ev2));
    ms_sw += a;
    ms_em += b;
  }
  c->ms_sweep = ms_sw;
  c->ms_emit = ms_em;
  // a repeated leader in paper mode delivers nothing new (its whole cone is in
  // the delivered set) and expands nothing (the pruned leader)
  for (size_t i = 0; i < pops.size(); i++) {
    const int k = kidx[i];
    const bool zero = mode == DR_DELIVER_PAPER && !first[i];
    if (pcount) pcount[i] = zero ? 0 : kc[k];
    if (pdigest) pdigest[i] = zero ? 0 : kd[k];
    if (pedges) pedges[i] = zero ? 0 : ke[k];
  }
  return check_barrier(c);
}


// ---------------------------------------------------------------------------
// Memoized replay (shard_memo.hpp).  Every shard holds the full canonical cone
// and every query's full frontier after each exchange, so each one takes the
// same decisions; only the row work is split by column.
// ---------------------------------------------------------------------------
drs::MArgs make_margs(dr_shard *c, int nq, int T = -1) {
  drs::MArgs a{};
  a.strong = c->strong.as<u64>();
  a.strong_stride = (int64_t)c->n * c->SP;
  a.strong_rstride = (int64_t)c->nlocal * c->n * c->SP;
  a.wck = c->wck.as<uint32_t>();
  a.wcr = c->wcr.as<u64>();
  a.wcro = c->wcro.as<uint64_t>();
  a.pres = c->pres.as<u64>();
  a.sdeg = c->sdeg.as<uint16_t>();
  a.wdeg = c->wdeg.as<uint16_t>();
  a.sdr = c->sdr.as<u64>();
  a.rdeg = c->rdeg.as<u64>();
  a.lead = c->lead.as<uint16_t>();
  a.U = c->mU.as<u64>();
  a.WU = c->mWU.as<u64>();
  a.K = c->mK.as<u64>();
  a.q = c->mq.as<drs::MQuery>();
  a.pend = c->mpend.as<u64>();
  a.masks = c->mmasks.as<u64>();
  a.push_out = c->mpush.as<int32_t>();
  a.n = c->n;
  a.W = c->W;
  a.WSs = c->WSs;
  a.SP = c->SP;
  a.G = c->G;
  a.shard0 = c->shard0;
  a.nlocal = c->nlocal;
  a.local = c->local ? 1 : 0;
  a.nq = nq;
  a.depth = c->depth;
  a.dd = std::max(0, c->dmax - 1);
  a.dmax = std::max(1, c->dmax);
  a.summary = 1;
  a.R = c->max_rounds;
  a.nlead = (int32_t)c->h_lead.size();
  a.good = c->mgood.as<uint8_t>();
  a.slot_off = c->slot_off.as<uint32_t>();
  a.slot_src = c->slot_src.as<uint16_t>();
  a.T = T >= 0 ? T : c->nrounds - 1;
  return a;
}

bool memo_applies(const dr_shard *c) { return c->memo && c->dmax <= 65; }

// every host wait of a query call goes through here (dr_shard_host_syncs counts them)
hipError_t host_sync(dr_shard *c) {
  c->syncs++;
  return hipStreamSynchronize(c->stream);
}

// n bytes of the pinned staging area (256-B aligned); nullptr on failure
char *stage(dr_shard *c, size_t n) {
  const size_t at = (c->pin_used + 255) & ~(size_t)255;
  if (at + n > c->pin_cap) {
    if (host_sync(c) != hipSuccess) return nullptr;  // staged copies still in flight
    const size_t cap = std::max<size_t>({(size_t)4 << 20, 2 * c->pin_cap, 2 * (at + n)});
    char *q = nullptr;
    if (hipHostMalloc((void **)&q, cap, hipHostMallocDefault) != hipSuccess) return nullptr;
    if (c->pin) (void)hipHostFree(c->pin);
    c->pin = q;
    c->pin_cap = cap;
    c->pin_used = 0;
    return stage(c, n);
  }
  c->pin_used = at + n;
  return c->pin + at;
}

// The memo replay's outputs, carved from one device region that comes back in
// one copy: header, commits, vcounts, every query's state (the stepped form
// steps them in place), the canonical walk's state (stepped form), chain pushes,
// per-pop count | digest | edges.
struct MOut {
  int32_t *hdr;
  uint8_t *commit;
  int32_t *vcount;
  drs::MState *fin, *canon;
  int32_t *push;
  u64 *qout;
  size_t bytes;
};
MOut carve_out(char *base, int nw, int nq, int64_t pcap, int npop) {
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char *p = base + off;
    off = (off + bytes + 63) & ~(size_t)63;
    return p;
  };
  MOut m{};
  m.hdr = reinterpret_cast<int32_t *>(take(drs::FH_N * 4));
  m.commit = reinterpret_cast<uint8_t *>(take((size_t)nw));
  m.vcount = reinterpret_cast<int32_t *>(take((size_t)nw * 4));
  m.fin = reinterpret_cast<drs::MState *>(take((size_t)std::max(nq, 1) * sizeof(drs::MState)));
  m.canon = reinterpret_cast<drs::MState *>(take(sizeof(drs::MState)));
  m.push = reinterpret_cast<int32_t *>(take((size_t)std::max<int64_t>(pcap, 1) * 4));
  m.qout = reinterpret_cast<u64 *>(take((size_t)3 * std::max(npop, 1) * 8));
  m.bytes = off;
  return m;
}

// k_ms_pass at the context's row stride.  Vote modes: VOTE_FULL (fused), VOTE_STEP2 /
// VOTE_STEP3 (stepped: Sout = this context's partial of the tested round's set, Sin =
// Gin exchanged slots of [sin_nw][W] it is tested against)
struct PassIO {
  u64 *Sout = nullptr;
  const u64 *Sin = nullptr;
  int Gin = 0, sin_nw = 0;
  hipStream_t st = nullptr;  // the context's stream if null
};
template <int SP, int NT, int GR>
hipError_t launch_pass_g(dr_shard *c, const drs::MArgs &a, const drs::FArgs &f, int nw, int mode, const PassIO &io) {
  const int T = c->nrounds - 1, nl = c->nlocal;
  const size_t lds = ((size_t)2 * nl * SP + c->W) * 8;
  hipStream_t st = io.st ? io.st : c->stream;
  if (nl == 1)
    hipLaunchKernelGGL((drs::k_ms_pass<SP, NT, GR, true>), dim3((T + 3) / 4), dim3(NT), lds, st, a, f, nw, mode,
                       c->mU.as<u64>(), io.Sout, io.Sin, io.Gin, io.sin_nw);
  else
    hipLaunchKernelGGL((drs::k_ms_pass<SP, NT, GR, false>), dim3((T + 3) / 4), dim3(NT), lds, st, a, f, nw, mode,
                       c->mU.as<u64>(), io.Sout, io.Sin, io.Gin, io.sin_nw);
  return hipGetLastError();
}
template <int SP>
hipError_t launch_pass_t(dr_shard *c, const drs::MArgs &a, const drs::FArgs &f, int nw, int mode, const PassIO &io) {
  // 512 threads, 8 chunks in flight: at C4, G = 8 (SP 2) 147 us vs 179 us at 1024 x 2,
  // G = 1 (SP 16) the same (profiles/r04/ pass geometries)
  if constexpr (SP == 2 || SP == 16) {  // the C4 shapes: the other geometries, for tuning
    switch (c->pass_geo) {
      case 1: return launch_pass_g<SP, 1024, 4>(c, a, f, nw, mode, io);
      case 2: return launch_pass_g<SP, 512, 4>(c, a, f, nw, mode, io);
      case 3: return launch_pass_g<SP, 1024, 2>(c, a, f, nw, mode, io);
    }
  }
  return launch_pass_g<SP, 512, 8>(c, a, f, nw, mode, io);
}
// the pass, after k_ms_wu (with_wu: WU and the speculative digests; the third vote
// step reads no summary)
hipError_t launch_pass(dr_shard *c, const drs::MArgs &a, const drs::FArgs &f, int nw, int mode, const PassIO &io,
                       bool with_wu = true) {
  const int T = c->nrounds - 1;
  const bool wu = with_wu && T >= 1;
  const bool side = wu && c->wu_side;
  if (wu) {
    const size_t lds = std::max<size_t>((size_t)4 * c->nlocal * a.dd * c->SP * 8, 8);
    if (side) {
      if (hipError_t e = hipEventRecord(c->fork, c->stream)) return e;
      if (hipError_t e = hipStreamWaitEvent(c->side, c->fork, 0)) return e;
    }
    hipLaunchKernelGGL((drs::k_ms_wu<256>), dim3((T + 3) / 4), dim3(256), lds, side ? c->side : c->stream, a, f,
                       c->mWU.as<u64>());
    if (hipError_t e = hipGetLastError()) return e;
    if (side)
      if (hipError_t e = hipEventRecord(c->join, c->side)) return e;
  }
  hipError_t e = hipErrorInvalidValue;
  switch (c->SP) {
    case 1: e = launch_pass_t<1>(c, a, f, nw, mode, io); break;
    case 2: e = launch_pass_t<2>(c, a, f, nw, mode, io); break;
    case 4: e = launch_pass_t<4>(c, a, f, nw, mode, io); break;
    case 8: e = launch_pass_t<8>(c, a, f, nw, mode, io); break;
    case 16: e = launch_pass_t<16>(c, a, f, nw, mode, io); break;
    case 32: e = launch_pass_t<32>(c, a, f, nw, mode, io); break;
  }
  if (e == hipSuccess && side) e = hipStreamWaitEvent(c->stream, c->join, 0);
  return e;
}

int paper_emit(dr_shard *c, const drs::MArgs &a, const std::vector<drs::MQuery> &qs,
               const std::vector<drs::MState> &fin, const std::vector<int> &pop_query, std::vector<uint64_t> &qout,
               int npop);

// ---------------------------------------------------------------------------
// The stepped form (shard_step.hpp).  Every launch goes out on the context's
// stream (RCCL mode: each exchange on it too); the host waits once, for the
// results.
// ---------------------------------------------------------------------------
// S_1 of every mirrored wave (k_ms_lcol), after an append or a coin change: the
// rank holding the leader's column finds it, one exchange gives it to every rank
int ensure_lcol(dr_shard *c) {
  const int T = c->nrounds - 1, nwl = std::max(0, (T + 2) / 4);
  if (c->lcol_ok) return DR_OK;
  drs::MArgs a = make_margs(c, 1, T);
  const size_t words = (size_t)std::max(nwl, 1) * c->W;
  SHCHK(c, c->mlcol.ensure((size_t)(c->local ? 1 : c->G) * words * 8));
  if (nwl > 0) {
    if (c->local) {
      hipLaunchKernelGGL(drs::k_ms_lcol, dim3((nwl + 3) / 4), dim3(256), 0, c->stream, a, nwl, c->mlcol.as<u64>());
      SHCHK(c, hipGetLastError());
    } else {
      SHCHK(c, c->mlcolp.ensure(words * 8));
      hipLaunchKernelGGL(drs::k_ms_lcol, dim3((nwl + 3) / 4), dim3(256), 0, c->stream, a, nwl, c->mlcolp.as<u64>());
      SHCHK(c, hipGetLastError());
      SHNCCL(c, ncclAllGather(c->mlcolp.p, c->mlcol.p, words, ncclUint64, c->comm, c->stream));
      c->last_xbytes += words * 8;
    }
  }
  c->lcol_nw = std::max(nwl, 1);
  c->lcol_g = c->local ? 1 : c->G;
  c->lcol_ok = true;
  return DR_OK;
}

// Launch steps [j0, j1) of a batch of nq queries (states st, in place), each
// followed by its exchange in RCCL mode.
int launch_steps(dr_shard *c, const drs::MArgs &a, const drs::FArgs &f, drs::MState *st, int nq, int j0, int j1,
                 int batch) {
  const int WL = c->nlocal * c->WSs;
  const size_t lds = ((size_t)c->depth * WL + c->W) * 8;
  // the canonical walk (batch 0, one query) and the batch steps keep separate buffers
  SBuf &pend = batch ? c->mpend : c->cpend, &send = batch ? c->msend : c->csend;
  SBuf *recv = batch ? c->mrecv : c->crecv;
  SHCHK(c, pend.ensure((size_t)std::max(nq, 1) * c->depth * WL * 8));
  SHCHK(c, recv[0].ensure((size_t)c->G * std::max(nq, 1) * c->WSs * 8));
  SHCHK(c, recv[1].ensure((size_t)c->G * std::max(nq, 1) * c->WSs * 8));
  SHCHK(c, send.ensure((size_t)std::max(nq, 1) * c->WSs * 8));
  drs::MArgs b = a;
  b.pend = pend.as<u64>();
  for (int j = j0; j < j1; j++) {
    u64 *rin = recv[j & 1].as<u64>();
    u64 *rout = c->local ? recv[(j + 1) & 1].as<u64>() : send.as<u64>();
    if (c->step_nt == 128)
      hipLaunchKernelGGL((drs::k_ms_step2<128>), dim3(nq), dim3(128), lds, c->stream, b, f, j, st, (const u64 *)rin,
                         rout, batch);
    else
      hipLaunchKernelGGL((drs::k_ms_step2<256>), dim3(nq), dim3(256), lds, c->stream, b, f, j, st, (const u64 *)rin,
                         rout, batch);
    SHCHK(c, hipGetLastError());
    if (!c->local) {
      SHNCCL(c, ncclAllGather(send.p, recv[(j + 1) & 1].p, (size_t)nq * c->WSs, ncclUint64, c->comm, c->stream));
      c->last_xbytes += (uint64_t)nq * c->WSs * 8;
    }
    c->last_rounds++;
  }
  return DR_OK;
}

// The stepped commit phase: S_1 (cached), the pass with the partial S_2, the S_2
// exchange, the third vote step (with K^cand in RCCL mode: one exchange for both),
// then k_ms_kfin: K, good, the RD / CE defaults, vcount / commit, the walk's query.
int stepped_commit(dr_shard *c, int nw, const drs::FArgs &f, const MOut &m) {
  const int T = c->nrounds - 1, W = c->W, G = c->G;
  drs::MArgs a1 = make_margs(c, 1, T);
  if (int rc = ensure_lcol(c)) return rc;
  const size_t pw = (size_t)std::max(nw, 1) * W * 8;
  SHCHK(c, c->vote_p[0].ensure((c->local ? 1 : G) * pw));  // S_2 partials, exchanged
  SHCHK(c, c->vote_p[1].ensure(pw));                        // local: S_3; RCCL: this rank's S_2
  u64 *S2 = c->vote_p[0].as<u64>();
  PassIO p2;
  p2.Sout = c->local ? S2 : c->vote_p[1].as<u64>();
  p2.Sin = c->mlcol.as<u64>();
  p2.Gin = c->lcol_g;
  p2.sin_nw = c->lcol_nw;
  SHCHK(c, launch_pass(c, a1, f, nw, drs::VOTE_STEP2, p2));
  if (!c->local) {
    SHNCCL(c, ncclAllGather(c->vote_p[1].p, S2, (size_t)nw * W, ncclUint64, c->comm, c->stream));
    c->last_xbytes += (uint64_t)nw * W * 8;
  }
  PassIO p3;
  p3.Sin = S2;
  p3.Gin = c->local ? 1 : G;
  p3.sin_nw = nw;
  const int rb = (T + 1 + 3) / 4, nb = rb + (nw + 3) / 4;
  if (c->local) {
    p3.Sout = c->vote_p[1].as<u64>();
    SHCHK(c, launch_pass(c, a1, f, nw, drs::VOTE_STEP3, p3, false));
    hipLaunchKernelGGL(drs::k_ms_kfin, dim3(nb), dim3(256), 0, c->stream, a1, f, (const u64 *)nullptr, (int64_t)0,
                       (const u64 *)p3.Sout, 1, c->mcq.as<drs::MQuery>(), m.canon);
    SHCHK(c, hipGetLastError());
  } else {
    // one send buffer: this rank's K^cand columns [(T+1) * WSs], then its partial S_3 [nw * W]
    const int64_t ks = (int64_t)(T + 1) * c->WSs + (int64_t)nw * W;
    SHCHK(c, c->mksend.ensure((size_t)ks * 8));
    SHCHK(c, c->mkrecv.ensure((size_t)G * ks * 8));
    hipLaunchKernelGGL(drs::k_ms_kcand, dim3(rb, c->nlocal), dim3(drs::MS_NT), 0, c->stream, a1, T,
                       c->mksend.as<u64>());
    SHCHK(c, hipGetLastError());
    p3.Sout = c->mksend.as<u64>() + (size_t)(T + 1) * c->WSs;
    SHCHK(c, launch_pass(c, a1, f, nw, drs::VOTE_STEP3, p3, false));
    SHNCCL(c, ncclAllGather(c->mksend.p, c->mkrecv.p, (size_t)ks, ncclUint64, c->comm, c->stream));
    c->last_xbytes += (uint64_t)ks * 8;
    hipLaunchKernelGGL(drs::k_ms_kfin, dim3(nb), dim3(256), 0, c->stream, a1, f, (const u64 *)c->mkrecv.as<u64>(), ks,
                       (const u64 *)nullptr, G, c->mcq.as<drs::MQuery>(), m.canon);
    SHCHK(c, hipGetLastError());
  }
  return DR_OK;
}

// What follows the canonical walk: the vote counts, its positions, the E prefix and
// the chain plan (k_ms_cpos), the canonical digests and their G prefix.
int stepped_canon_tail(dr_shard *c, const drs::FArgs &f, const MOut &m, int nq, int64_t pcap) {
  const int T = c->nrounds - 1, rb = (T + 1 + 3) / 4;
  drs::MArgs a = make_margs(c, nq, T);
  a.push_out = m.push;
  hipLaunchKernelGGL((drs::k_ms_cpos<1024>), dim3(1), dim3(1024), 0, c->stream, a, f, (const drs::MState *)m.canon,
                     c->mq.as<drs::MQuery>(), (int)pcap);
  SHCHK(c, hipGetLastError());
  hipLaunchKernelGGL(drs::k_ms_rg_full, dim3(rb), dim3(256), 0, c->stream, a, f);
  SHCHK(c, hipGetLastError());
  hipLaunchKernelGGL((drs::k_ms_gprefix<1024>), dim3(1), dim3(1024), 0, c->stream, a, f);
  SHCHK(c, hipGetLastError());
  return DR_OK;
}

// The pop queries of a stepped replay (one per wave whose leader is present, mask rows
// laid out in wave order): uploaded when the DAG, the leaders or the wave count changed.
int upload_pops(dr_shard *c, const std::vector<drs::MQuery> &qs, int nw) {
  const uint64_t key[4] = {(uint64_t)c->nrounds, c->lead_version, (uint64_t)nw, (uint64_t)(uintptr_t)c->mq.p};
  if (std::equal(key, key + 4, c->pops_key) || qs.empty()) return DR_OK;
  auto *hq = reinterpret_cast<drs::MQuery *>(stage(c, qs.size() * sizeof(drs::MQuery)));
  if (!hq) return c->fail(DR_E_HIP, "pinned staging allocation failed");
  std::copy(qs.begin(), qs.end(), hq);
  SHCHK(c, hipMemcpyAsync(c->mq.p, hq, qs.size() * sizeof(drs::MQuery), hipMemcpyHostToDevice, c->stream));
  std::copy(key, key + 4, c->pops_key);
  return DR_OK;
}

// dr_shard_replay on the memo path.  Fused form (the context holds every column:
// local mode, a one-rank group): every kernel reads all columns, so nothing is
// exchanged and each query runs to its end in one launch -- the pass (U, WU,
// speculative digests and the complete vote), K^cand, the canonical walk, the
// canonical digests and prefixes, the chain plan, one sweep launch for every pop
// and chain, the emission: eight launches and one copy back.  Stepped form
// (shard_step.hpp): the launches of each phase back to back, as many steps as the
// last replay took, one copy back; more steps only if a query was still live.
// REF emission k_ms_emit; PAPER paper_emit after the copy.
int replay_memo(dr_shard *c, int nwaves, int chain_mode, int deliver_mode, dr_replay_out *o) {
  const auto th0 = std::chrono::steady_clock::now();
  static const bool th_on = getenv("DR_SHARD_HOST_TIMING") != nullptr;  // investigation only
  std::chrono::steady_clock::time_point th1 = th0, th2 = th0, th3 = th0;
  const bool paper = deliver_mode == DR_DELIVER_PAPER, persistent = chain_mode == DR_CHAIN_PERSISTENT;
  const bool fused = c->nlocal == c->G && !c->stepped;
  const int T = c->nrounds - 1, W = c->W, nw = nwaves;
  c->syncs = 0;
  if (int rc = sync_weak(c)) return rc;  // uploads the weak edges and columns after an append
  c->pin_used = 0;
  // one cone query per wave whose leader is present (a superset of the leaders any chain can push)
  std::vector<drs::MQuery> qs;
  std::vector<int> popq(nw + 1, -1);
  int64_t moff = 0;
  for (int w = 1; w <= nw; w++) {
    const int r1 = 4 * (w - 1) + 1, L = c->lead_src(w);
    if (!c->is_present(r1, L)) continue;
    drs::MQuery q{};
    q.type = drs::MQ_POP;
    q.top = r1;
    q.bottom = 0;
    q.src0 = L - 1;
    q.mask_off = moff;
    moff += (int64_t)(r1 + 1) * W;
    popq[w] = (int)qs.size();
    qs.push_back(q);
  }
  const int npop = (int)qs.size(), nq = npop + nw;
  const int64_t pcap = persistent ? (int64_t)nw : (int64_t)nw * (nw + 1) / 2;
  if (pcap > ((int64_t)1 << 26)) return c->fail(DR_E_CAPACITY, "literal chains of %d waves: push bound %lld", nw, (long long)pcap);
  // buffers
  const size_t R = (size_t)c->max_rounds;
  const int nl = c->nlocal, dd = std::max(0, c->dmax - 1);
  SHCHK(c, c->mU.ensure((size_t)nl * R * c->SP * 8));
  SHCHK(c, c->mWU.ensure(std::max<size_t>((size_t)nl * R * dd * c->SP, 1) * 8));
  SHCHK(c, c->mK.ensure((size_t)(T + 1) * W * 8));
  SHCHK(c, c->mgood.ensure((size_t)T + 16));
  for (SBuf *b : {&c->mRD, &c->mCE, &c->mRG, &c->mC, &c->mE, &c->mG, &c->mSG}) SHCHK(c, b->ensure((size_t)(T + 1) * 8));
  SHCHK(c, c->mmasks.ensure((size_t)std::max<int64_t>(moff, 1) * 8));
  SHCHK(c, c->mq.ensure((size_t)std::max(nq, 1) * sizeof(drs::MQuery)));  // pops and chains: planned on the device
  SHCHK(c, c->mcq.ensure(sizeof(drs::MQuery)));                           // the stepped canonical walk
  MOut m = carve_out(nullptr, nw, nq, pcap, npop);
  SHCHK(c, c->mout.ensure(m.bytes));
  m = carve_out(c->mout.as<char>(), nw, nq, pcap, npop);
  drs::FArgs f{};
  f.ppref = c->ppref.as<u64>();
  f.SG = c->mSG.as<u64>();
  f.RD = c->mRD.as<u64>();
  f.CE = c->mCE.as<u64>();
  f.RG = c->mRG.as<u64>();
  f.Cc = c->mC.as<u64>();
  f.Ec = c->mE.as<u64>();
  f.Gc = c->mG.as<u64>();
  f.good = c->mgood.as<uint8_t>();
  f.hdr = m.hdr;
  f.commit = m.commit;
  f.vcount = m.vcount;
  f.fin = m.fin;
  f.quorum = 2 * c->f + 1;
  f.nw = nw;
  f.npop = npop;
  f.persistent = persistent ? 1 : 0;
  f.qcount = m.qout;
  f.qdigest = m.qout + npop;
  f.qedges = m.qout + 2 * npop;
  // the fused sweep emitting each pop itself (DR_SHARD_EMIT_FUSED=1, tuning): 101 us against
  // 68 + 22 us as two launches at C4 G = 1 (profiles/r04/)
  f.emit = fused && !paper && c->emit_fused ? 1 : 0;
  f.keep4 = c->keep4;
  SHCHK(c, c->mark(0));
  th1 = std::chrono::steady_clock::now();
  c->last_rounds = 0;
  drs::MArgs a = make_margs(c, nq);
  a.push_out = m.push;
  drs::MArgs ac = make_margs(c, 1, T);  // the stepped canonical walk: one query
  ac.q = c->mcq.as<drs::MQuery>();
  auto emit = [&]() -> int {  // REF emission of every pop query (PAPER needs the pop order, below)
    if (npop > 0 && !paper && !f.emit) {
      hipLaunchKernelGGL(drs::k_ms_emit, dim3(npop), dim3(drs::MS_NT), 0, c->stream, a, (const int32_t *)nullptr,
                         (const drs::MState *)m.fin, c->slot_off.as<uint32_t>(), c->slot_src.as<uint16_t>(),
                         (const u64 *)f.Cc, (const u64 *)f.Gc, (const u64 *)f.Ec, m.qout, m.qout + npop,
                         m.qout + 2 * npop);
      SHCHK(c, hipGetLastError());
    }
    return DR_OK;
  };
  int jc = 0, jb = 0;  // stepped form: canonical walk / batch steps launched
  if (fused) {
    a.good = f.good;
    SHCHK(c, launch_pass(c, a, f, nw, drs::VOTE_FULL, PassIO{}));
    SHCHK(c, c->mark(1));
    // K^cand, the canonical walk, the canonical digests and prefixes, the plan (pops and chains).
    // (As one workgroup's tail of the parallel launch before it -- a done counter behind an
    // agent-scope fence per workgroup -- these took 108 + 92 us against 40 + 33 us apart:
    // every fence writes back the XCD's L2; profiles/r04/.)
    const int rb = (T + 1 + 3) / 4;
    const size_t lds_ring = ((size_t)c->depth * W + 2 * W) * 8;
    hipLaunchKernelGGL(drs::k_ms_kcand_full, dim3(rb), dim3(256), 0, c->stream, a, f);
    SHCHK(c, hipGetLastError());
    hipLaunchKernelGGL((drs::k_ms_canon_full<512>), dim3(1), dim3(512), lds_ring, c->stream, a, f);
    SHCHK(c, hipGetLastError());
    hipLaunchKernelGGL(drs::k_ms_rg_full, dim3(rb), dim3(256), 0, c->stream, a, f);
    SHCHK(c, hipGetLastError());
    hipLaunchKernelGGL((drs::k_ms_prefix_plan<1024>), dim3(1), dim3(1024), 0, c->stream, a, f,
                       c->mq.as<drs::MQuery>(), (int)pcap);
    SHCHK(c, hipGetLastError());
    SHCHK(c, c->mark(2));
    // every pop and chain to its end, REF pops emitted by their own workgroup
    hipLaunchKernelGGL((drs::k_ms_sweep_full<256>), dim3(nq), dim3(256), lds_ring, c->stream, a, f);
    SHCHK(c, hipGetLastError());
  } else {
    if (int rc = stepped_commit(c, nw, f, m)) return rc;
    SHCHK(c, c->mark(1));
    if (int rc = upload_pops(c, qs, nw)) return rc;
    jc = std::max(1, c->hint_canon);
    if (int rc = launch_steps(c, ac, f, m.canon, 1, 0, jc, 0)) return rc;
    if (int rc = stepped_canon_tail(c, f, m, nq, pcap)) return rc;
    SHCHK(c, c->mark(2));
    jb = std::max(1, c->hint_batch);
    if (int rc = launch_steps(c, a, f, m.fin, nq, 0, jb, 1)) return rc;
  }
  SHCHK(c, c->mark(3));
  if (int rc = emit()) return rc;
  SHCHK(c, c->mark(4));
  char *hb = stage(c, m.bytes);
  if (!hb) return c->fail(DR_E_HIP, "pinned staging allocation failed");
  SHCHK(c, hipMemcpyAsync(hb, c->mout.p, m.bytes, hipMemcpyDeviceToHost, c->stream));
  th2 = std::chrono::steady_clock::now();
  SHCHK(c, host_sync(c));
  th3 = std::chrono::steady_clock::now();
  const MOut h = carve_out(hb, nw, nq, pcap, npop);
  if (!fused) {
    // a query still live after the launched steps (the DAG changed since the step
    // counts were taken): step on from where it is, then everything that reads it again
    const int bound = T + 2 * std::max(1, c->nrounds) + 8;
    for (;;) {
      const bool cdone = h.canon->done != 0;
      bool bdone = cdone;
      for (int i = 0; bdone && i < nq; i++) bdone = h.fin[i].done != 0;
      if (cdone && bdone) break;
      if (!cdone) {
        const int more = std::max(4, jc);
        if (jc + more > bound) return c->fail(DR_E_HIP, "memo replay: the canonical walk is live after %d steps", jc);
        if (int rc = launch_steps(c, ac, f, m.canon, 1, jc, jc + more, 0)) return rc;
        jc += more;
        if (int rc = stepped_canon_tail(c, f, m, nq, pcap)) return rc;
        jb = std::max(1, c->hint_batch);
        if (int rc = launch_steps(c, a, f, m.fin, nq, 0, jb, 1)) return rc;
      } else {
        const int more = std::max(4, jb);
        if (jb + more > bound) return c->fail(DR_E_HIP, "memo replay: queries live after %d steps", jb);
        if (int rc = launch_steps(c, a, f, m.fin, nq, jb, jb + more, 1)) return rc;
        jb += more;
      }
      if (int rc = emit()) return rc;
      SHCHK(c, hipMemcpyAsync(hb, c->mout.p, m.bytes, hipMemcpyDeviceToHost, c->stream));
      SHCHK(c, host_sync(c));
    }
    c->hint_canon = std::max(1, h.canon->steps);
    int need = 1;
    for (int i = 0; i < nq; i++) need = std::max(need, h.fin[i].steps);
    c->hint_batch = need;
  }
  if (c->phase_timing) {
    SHCHK(c, hipEventElapsedTime(&o->ms_commit, c->evs[0], c->evs[1]));
    SHCHK(c, hipEventElapsedTime(&o->ms_summary, c->evs[1], c->evs[2]));
    SHCHK(c, hipEventElapsedTime(&o->ms_deliver, c->evs[2], c->evs[3]));
    SHCHK(c, hipEventElapsedTime(&o->ms_emit, c->evs[3], c->evs[4]));
  }
  o->ms_chain = 0;
  if (h.hdr[drs::FH_ERR]) return c->fail(DR_E_CAPACITY, "chain pushes exceed the bound %lld", (long long)pcap);
  std::memcpy(o->commit, h.commit, (size_t)nw);
  std::memcpy(o->vcount, h.vcount, (size_t)nw * 4);
  o->canon_segments = h.hdr[drs::FH_NSEG];
  uint64_t ce = 0;
  for (int w = 1; w <= nw; w++)
    if (o->vcount[w - 1] >= 0) ce += c->h_deg[4 * w - 2] + c->h_deg[4 * w - 1] + c->h_deg[4 * w];
  o->commit_edges = ce;
  // the chain tasks plan_body made (k_ms_prefix_plan, k_ms_cpos), in the same order: chain i is query npop + i
  struct Task { int wave, q; int32_t pbase; };
  std::vector<Task> tasks;  // every commit, q = -1 without a chain query
  {
    int lastw = 0, nch = 0;
    int32_t pb = 0;
    for (int w = 1; w <= nw; w++)
      if (o->commit[w - 1]) {
        const int fl = persistent ? lastw : 0;
        Task t{w, -1, 0};
        if (w - 1 >= fl + 1) {
          t.q = npop + nch++;
          t.pbase = pb;
          pb += w - fl;
        }
        tasks.push_back(t);
        lastw = w;
      }
    if (nch != h.hdr[drs::FH_NCHAIN]) return c->fail(DR_E_HIP, "memo replay: %d chains planned on the device, %d on the host", h.hdr[drs::FH_NCHAIN], nch);
  }
  uint64_t chain_e = 0;
  int64_t np = 0;
  for (const Task &t : tasks) {
    np += 1 + (t.q >= 0 ? h.fin[t.q].npush : 0);
    if (t.q >= 0) chain_e += h.fin[t.q].edges;
  }
  o->chain_edges = chain_e;
  o->n_push = np;
  if (np > o->push_cap || !o->push_wave || !o->pop_count || !o->pop_digest)
    return c->fail(DR_E_CAPACITY, "%lld pushed leaders, capacity %lld", (long long)np, (long long)o->push_cap);
  int64_t at = 0;
  size_t ti = 0;
  std::vector<int> pop_query;
  for (int w = 1; w <= nw; w++) {
    o->push_off[w - 1] = (uint32_t)at;
    if (ti < tasks.size() && tasks[ti].wave == w) {
      const Task &t = tasks[ti];
      const int64_t a0 = at;
      o->push_wave[at++] = w;
      if (t.q >= 0)
        for (int x = 0; x < h.fin[t.q].npush; x++) o->push_wave[at++] = h.push[t.pbase + x];
      for (int64_t y = at - 1; y >= a0; y--) {  // pops: the stack's LIFO order
        const int q = popq[o->push_wave[y]];
        if (q < 0) return c->fail(DR_E_HIP, "memo replay: pushed wave %d has no cone query", o->push_wave[y]);
        pop_query.push_back(q);
      }
      ti++;
    }
  }
  o->push_off[nw] = (uint32_t)at;
  std::vector<uint64_t> qout;  // PAPER: paper_emit's counts; REF reads the copied region
  const uint64_t *qo = reinterpret_cast<const uint64_t *>(h.qout);
  int steps = c->hint_batch;
  if (fused) {
    steps = 0;
    for (int i = 0; i < npop; i++) steps = std::max(steps, qs[i].top - h.fin[i].stop + 1);
  }
  if (paper && !pop_query.empty()) {
    std::vector<drs::MState> fin(h.fin, h.fin + npop);
    SHCHK(c, c->mark(3));
    qout.assign(qo, qo + (size_t)3 * std::max(npop, 1));
    if (int rc = paper_emit(c, a, qs, fin, pop_query, qout, npop)) return rc;
    qo = qout.data();
    SHCHK(c, c->mark(4));
    if (c->phase_timing) {
      SHCHK(c, hipEventSynchronize(c->evs[4]));
      SHCHK(c, hipEventElapsedTime(&o->ms_emit, c->evs[3], c->evs[4]));
    }
  }
  uint64_t de = 0;
  std::vector<uint8_t> seen(paper ? npop : 0, 0);
  for (size_t pi = 0; pi < pop_query.size(); pi++) {
    const int q = pop_query[pi];
    const bool zero = paper && seen[q];  // a repeated leader delivers nothing new (its cone is delivered)
    if (paper) seen[q] = 1;
    o->pop_count[pi] = zero ? 0 : qo[q];
    o->pop_digest[pi] = zero ? 0 : qo[npop + q];
    const uint64_t e = zero ? 0 : qo[2 * npop + q];
    if (o->pop_edges) o->pop_edges[pi] = e;
    de += e;
  }
  o->deliver_edges = de;
  o->sweep_count = (uint64_t)npop;
  o->sweep_partial = (uint64_t)steps;
  c->last_rounds = (uint64_t)steps;
  if (th_on) {
    auto us = [](std::chrono::steady_clock::time_point x, std::chrono::steady_clock::time_point y) {
      return std::chrono::duration<double, std::micro>(y - x).count();
    };
    fprintf(stderr, "[shard host] prep %.1f us, enqueue %.1f us, wait %.1f us, assemble %.1f us, %zu B back\n",
            us(th0, th1), us(th1, th2), us(th2, th3), us(th3, std::chrono::steady_clock::now()), m.bytes);
  }
  return DR_OK;
}

// PAPER on the memo path: the first pop of each distinct leader delivers its cone
// minus the cones of the pops before it (k_ms_paper).  qout: [count | digest |
// edges] per query index.
int paper_emit(dr_shard *c, const drs::MArgs &a, const std::vector<drs::MQuery> &qs,
               const std::vector<drs::MState> &fin, const std::vector<int> &pop_query, std::vector<uint64_t> &qout,
               int npop) {
  std::vector<int> first;
  std::vector<uint8_t> seen(npop, 0);
  for (int q : pop_query)
    if (!seen[q]) {
      seen[q] = 1;
      first.push_back(q);
    }
  const int m = (int)first.size();
  std::vector<drs::MPaper> qp(m);
  int rmax = 1;
  for (int i = 0; i < m; i++) {
    const drs::MQuery &Q = qs[first[i]];
    const drs::MState &S = fin[first[i]];
    drs::MPaper x{};
    x.top = Q.top;
    if (S.merged) {
      x.cut = std::min(S.stop + a.dmax - 1, Q.top);
      x.lo = x.cut + 1;
    } else {
      x.cut = 0;
      x.lo = std::max(1, S.stop);
    }
    x.mask_off = Q.mask_off;
    qp[i] = x;
    rmax = std::max(rmax, Q.top);
  }
  const int rstride = rmax + 1;
  SHCHK(c, c->mqidx.ensure((size_t)m * sizeof(drs::MPaper)));
  SHCHK(c, c->pcnt.ensure((size_t)m * rstride * 4));
  SHCHK(c, c->mqout.ensure((size_t)3 * m * 8));
  u64 *qo = c->mqout.as<u64>();
  SHCHK(c, hipMemcpyAsync(c->mqidx.p, qp.data(), (size_t)m * sizeof(drs::MPaper), hipMemcpyHostToDevice, c->stream));
  SHCHK(c, hipMemsetAsync(c->pcnt.p, 0, (size_t)m * rstride * 4, c->stream));
  SHCHK(c, hipMemsetAsync(qo, 0, (size_t)3 * m * 8, c->stream));
  const drs::MPaper *dqp = c->mqidx.as<drs::MPaper>();
  const dim3 grid((rmax + 3) / 4), block(drs::MS_NT);
  hipLaunchKernelGGL(drs::k_ms_paper<false>, grid, block, 0, c->stream, a, rmax, dqp, m, c->pcnt.as<uint32_t>(),
                     rstride, c->slot_off.as<uint32_t>(), c->slot_src.as<uint16_t>(), qo + 2 * m, qo + m);
  SHCHK(c, hipGetLastError());
  hipLaunchKernelGGL(drs::k_ms_paper_scan, dim3(m), block, 0, c->stream, rmax, c->pcnt.as<uint32_t>(), rstride, qo);
  SHCHK(c, hipGetLastError());
  hipLaunchKernelGGL(drs::k_ms_paper<true>, grid, block, 0, c->stream, a, rmax, dqp, m, c->pcnt.as<uint32_t>(),
                     rstride, c->slot_off.as<uint32_t>(), c->slot_src.as<uint16_t>(), qo + 2 * m, qo + m);
  SHCHK(c, hipGetLastError());
  std::vector<uint64_t> h((size_t)3 * m);
  SHCHK(c, hipMemcpyAsync(h.data(), qo, h.size() * 8, hipMemcpyDeviceToHost, c->stream));
  SHCHK(c, hipStreamSynchronize(c->stream));
  qout.assign((size_t)3 * std::max(npop, 1), 0);
  for (int i = 0; i < m; i++) {
    qout[first[i]] = h[i];
    qout[npop + first[i]] = h[m + i];
    qout[2 * npop + first[i]] = h[2 * m + i];
  }
  return DR_OK;
}

}  // namespace

extern "C" int dr_shard_unique_id(uint8_t *id) {
  if (!id) return DR_E_INVAL;
  ncclUniqueId u;
  ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) {
    g_shard_err = std::string("ncclGetUniqueId: ") + ncclGetErrorString(r);
    return DR_E_RCCL;
  }
  static_assert(sizeof(ncclUniqueId) == DR_SHARD_ID_BYTES, "RCCL unique id size");
  std::memcpy(id, &u, sizeof u);
  return DR_OK;
}

extern "C" int dr_shard_create(int n, int faulty, int max_rounds, int device, int nshards, int rank, const uint8_t *id,
                               dr_shard **out) {
  if (!out) return DR_E_INVAL;
  *out = nullptr;
  if (n < 1 || n > 2048 || faulty < 0 || max_rounds < 1 || max_rounds > (1 << 20) || device < 0 || nshards < 1 ||
      nshards > 64 || rank < 0 || rank >= nshards || (!id && rank != 0)) {
    g_shard_err = "dr_shard_create: n in [1,2048], faulty >= 0, max_rounds in [1,2^20], device >= 0, "
                  "nshards in [1,64], 0 <= rank < nshards (rank 0 in local mode)";
    return DR_E_INVAL;
  }
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || device >= ndev) {
    g_shard_err = std::string("dr_shard_create: no usable HIP device (") +
                  (e != hipSuccess ? hipGetErrorString(e) : "ordinal out of range") + "); there is no CPU fallback";
    return DR_E_HIP;
  }
  dr_shard *c = new dr_shard();
  c->n = n;
  c->f = faulty;
  c->W = (n + 63) / 64;
  c->G = nshards;
  c->WSs = (c->W + nshards - 1) / nshards;
  c->C = c->WSs * 64;
  c->SP = 1;
  while (c->SP < c->WSs) c->SP <<= 1;  // row stride: a power of two (fixed lane -> column maps)
  c->local = id == nullptr;
  if (const char *g = getenv("DR_SHARD_PASS_GEO")) c->pass_geo = atoi(g) & 3;  // tuning only
  if (const char *g = getenv("DR_SHARD_WU_SIDE")) c->wu_side = atoi(g) != 0;
  if (const char *g = getenv("DR_SHARD_EMIT_FUSED")) c->emit_fused = atoi(g) != 0;
  if (const char *g = getenv("DR_SHARD_KEEP4")) c->keep4 = atoi(g) != 0;
  if (const char *g = getenv("DR_SHARD_STEP_NT")) c->step_nt = atoi(g) == 128 ? 128 : 256;
  c->shard0 = c->local ? 0 : rank;
  c->nlocal = c->local ? nshards : 1;
  c->max_rounds = max_rounds;
  c->dev = device;
  c->h_weak.resize(c->nlocal);
  c->h_woff.assign(c->nlocal, std::vector<uint64_t>(1, 0));
  c->h_wck.resize(c->nlocal);
  c->h_wcr.resize(c->nlocal);
  c->h_wcro.assign(c->nlocal, std::vector<uint64_t>(1, 0));
  c->h_lead.assign((size_t)max_rounds / 4 + 2, 1);
  if (sh_set_device(c) != DR_OK || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev0, hipEventReleaseToDevice) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev1, hipEventReleaseToDevice) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev2, hipEventReleaseToDevice) != hipSuccess ||
      hipEventCreateWithFlags(&c->evs[0], hipEventReleaseToDevice) != hipSuccess ||
      hipEventCreateWithFlags(&c->evs[1], hipEventReleaseToDevice) != hipSuccess ||
      hipEventCreateWithFlags(&c->evs[2], hipEventReleaseToDevice) != hipSuccess ||
      hipEventCreateWithFlags(&c->evs[3], hipEventReleaseToDevice) != hipSuccess ||
      hipEventCreateWithFlags(&c->evs[4], hipEventReleaseToDevice) != hipSuccess ||
      hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->join, hipEventDisableTiming) != hipSuccess) {
    g_shard_err = "dr_shard_create: stream/event creation failed";
    dr_shard_destroy(c);
    return DR_E_HIP;
  }
  const size_t NT = (size_t)c->G * c->C;
  if (c->strong.ensure((size_t)c->nlocal * max_rounds * n * c->SP * 8) != hipSuccess ||
      c->ft[0].ensure(NT * 8) != hipSuccess || c->ft[1].ensure(NT * 8) != hipSuccess ||
      c->send.ensure((size_t)c->C * 8) != hipSuccess || c->cnt.ensure(c->nlocal * 4) != hipSuccess ||
      c->pres.ensure((size_t)max_rounds * c->W * 8) != hipSuccess ||
      c->sdeg.ensure((size_t)max_rounds * n * 2) != hipSuccess ||
      c->wdeg.ensure((size_t)max_rounds * n * 2) != hipSuccess ||
      c->rdeg.ensure((size_t)max_rounds * 8) != hipSuccess || c->sdr.ensure((size_t)max_rounds * 8) != hipSuccess ||
      c->ppref.ensure((size_t)max_rounds * 8) != hipSuccess ||
      c->slot_off.ensure(((size_t)max_rounds + 1) * 4) != hipSuccess ||
      c->lead.ensure(c->h_lead.size() * 2) != hipSuccess ||
      hipMemcpy(c->lead.p, c->h_lead.data(), c->h_lead.size() * 2, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(c->slot_off.p, 0, 4) != hipSuccess) {
    g_shard_err = "dr_shard_create: device allocation failed";
    dr_shard_destroy(c);
    return DR_E_HIP;
  }
  if (!c->local) {
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    ncclResult_t r = ncclCommInitRank(&c->comm, nshards, u, rank);
    if (r != ncclSuccess) {
      g_shard_err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
      c->comm = nullptr;
      dr_shard_destroy(c);
      return DR_E_RCCL;
    }
  }
  *out = c;
  return DR_OK;
}

extern "C" void dr_shard_destroy(dr_shard *c) {
  if (!c) return;
  (void)hipSetDevice(c->dev);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->comm) (void)ncclCommDestroy(c->comm);
  for (SBuf *b : {&c->wck, &c->wcr, &c->wcro, &c->sdr, &c->mU, &c->mWU, &c->mK, &c->mgood, &c->mRD, &c->mCE, &c->mRG,
                  &c->mC, &c->mE, &c->mG, &c->mksend, &c->mkrecv, &c->mq, &c->mpend, &c->mrecv[0],
                  &c->mrecv[1], &c->msend, &c->mmasks, &c->mpush, &c->mqidx, &c->mqout, &c->ppref, &c->mSG,
                  &c->mout, &c->mcq, &c->mlcol, &c->mlcolp, &c->cpend, &c->crecv[0], &c->crecv[1], &c->csend})
    b->release();
  if (c->pin) (void)hipHostFree(c->pin);
  for (SBuf *b : {&c->strong, &c->weak, &c->woff, &c->ft[0], &c->ft[1], &c->send, &c->pend, &c->cnt, &c->out,
                  &c->qinfo, &c->pres, &c->sdeg, &c->wdeg, &c->rdeg, &c->slot_off, &c->slot_src, &c->lead, &c->bar,
                  &c->errf, &c->push_out, &c->push_n, &c->cedges, &c->vote_s0, &c->vote_p[0], &c->vote_p[1],
                  &c->vote_send, &c->vcount, &c->D, &c->pcnt, &c->qcnt, &c->qedges, &c->qdig})
    b->release();
  for (hipEvent_t ev : {c->ev0, c->ev1, c->ev2, c->evs[0], c->evs[1], c->evs[2], c->evs[3], c->evs[4], c->fork, c->join})
    if (ev) (void)hipEventDestroy(ev);
  if (c->side) (void)hipStreamDestroy(c->side);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

extern "C" const char *dr_shard_last_error(const dr_shard *c) { return c ? c->err.c_str() : g_shard_err.c_str(); }
extern "C" int dr_shard_num_rounds(const dr_shard *c) { return c ? c->nrounds : -1; }

extern "C" int dr_shard_info(const dr_shard *c, int *nshards, int *shard0, int *nlocal, int *col0, int *col1) {
  if (!c) return DR_E_INVAL;
  if (nshards) *nshards = c->G;
  if (shard0) *shard0 = c->shard0;
  if (nlocal) *nlocal = c->nlocal;
  if (col0) *col0 = std::min(c->n, c->shard0 * c->C) + 1;
  if (col1) *col1 = std::min(c->n, (c->shard0 + c->nlocal) * c->C) + 1;
  return DR_OK;
}

extern "C" int dr_shard_set_option(dr_shard *c, int option, int value) {
  if (!c) return DR_E_INVAL;
  if (option == DR_SHARD_OPT_PERSISTENT) {
    c->persistent = value ? 1 : 0;
    return DR_OK;
  }
  if (option == DR_SHARD_OPT_MEMO) {
    c->memo = value ? 1 : 0;
    return DR_OK;
  }
  if (option == DR_SHARD_OPT_STEPPED) {
    c->stepped = value ? 1 : 0;
    return DR_OK;
  }
  if (option == DR_SHARD_OPT_PHASE_TIMING) {
    c->phase_timing = value ? 1 : 0;
    return DR_OK;
  }
  if (option == DR_SHARD_OPT_STEP_HINTS) {
    if (value < 1) return c->fail(DR_E_INVAL, "step hint %d < 1", value);
    c->hint_canon = c->hint_batch = value;
    return DR_OK;
  }
  return c->fail(DR_E_INVAL, "unknown option %d", option);
}

extern "C" int dr_shard_set_leader_coin(dr_shard *c, int mode, uint64_t seed, int k, const int32_t *table) {
  if (!c) return DR_E_INVAL;
  if (int rc = sh_set_device(c)) return rc;
  std::vector<uint16_t> L(c->h_lead.size(), 1);
  if (mode == DR_LEADER_SEEDED) {
    for (size_t w = 1; w < L.size(); w++) L[w] = (uint16_t)dr_coin_leader(seed, (int)w, c->n);
  } else if (mode == DR_LEADER_TABLE) {
    if (k < 0 || (k > 0 && !table)) return c->fail(DR_E_INVAL, "bad leader table");
    for (int w = 1; w <= k && w < (int)L.size(); w++) {
      if (table[w - 1] < 1 || table[w - 1] > c->n)
        return c->fail(DR_E_INVAL, "leader of wave %d: source %d outside [1, %d]", w, table[w - 1], c->n);
      L[w] = (uint16_t)table[w - 1];
    }
  } else if (mode != DR_LEADER_CONST1) {
    return c->fail(DR_E_INVAL, "unknown leader coin mode %d", mode);
  }
  c->h_lead = std::move(L);
  c->lcol_ok = false;  // the stepped vote's S_1 follows the leaders
  c->lead_version++;
  SHCHK(c, hipMemcpyAsync(c->lead.p, c->h_lead.data(), c->h_lead.size() * 2, hipMemcpyHostToDevice, c->stream));
  SHCHK(c, hipStreamSynchronize(c->stream));
  return DR_OK;
}

extern "C" int dr_shard_append_rounds_packed(dr_shard *c, int r0, int k, const uint32_t *slot_off,
                                             const uint16_t *slot_src, const uint64_t *strong,
                                             const uint32_t *weak_off, const uint32_t *weak_tgt) {
  if (!c) return DR_E_INVAL;
  if (int rc = sh_set_device(c)) return rc;
  if (r0 != c->nrounds) return c->fail(DR_E_STATE, "append at round %d but %d rounds mirrored", r0, c->nrounds);
  if (k < 0 || r0 + k > c->max_rounds) return c->fail(DR_E_INVAL, "append of %d rounds exceeds max_rounds %d", k, c->max_rounds);
  if (k == 0) return DR_OK;
  if (!slot_off || !slot_src || !strong || !weak_off) return c->fail(DR_E_INVAL, "null array");
  const int n = c->n, W = c->W, WSs = c->WSs, SP = c->SP, C = c->C;
  const u64 lastmask = (n % 64) ? ((1ULL << (n % 64)) - 1ULL) : ~0ULL;
  std::vector<u64> pres((size_t)k * W, 0);
  std::vector<u64> rows((size_t)c->nlocal * k * n * SP, 0);
  std::vector<uint16_t> sd((size_t)k * n, 0), wd((size_t)k * n, 0);
  std::vector<u64> rd(k, 0);
  std::vector<uint64_t> deg(k, 0);
  std::vector<std::vector<uint32_t>> wnew(c->nlocal);
  std::vector<std::vector<uint64_t>> wro(c->nlocal, std::vector<uint64_t>(k + 1, 0));
  std::vector<std::vector<uint32_t>> wck_new(c->nlocal);
  std::vector<std::vector<u64>> wcr_new(c->nlocal);
  std::vector<std::vector<uint64_t>> wcro_new(c->nlocal, std::vector<uint64_t>(k + 1, 0));
  int dmax = c->dmax;
  size_t maxw = c->max_weak_round;
  for (int i = 0; i < k; i++) {
    const int r = r0 + i;
    u64 *P = &pres[(size_t)i * W];
    for (uint32_t sl = slot_off[i]; sl < slot_off[i + 1]; sl++) {
      const int s = slot_src[sl];
      if (s > n) return c->fail(DR_E_CONTRACT, "round %d slot %u: source %d > n=%d", r, sl - slot_off[i], s, n);
      if (s == 0) continue;
      const u64 bit = 1ULL << ((s - 1) & 63);
      if ((P[(s - 1) >> 6] & bit) && r >= 1) return c->fail(DR_E_CONTRACT, "round %d: duplicate vertex id (%d,%d)", r, r, s);
      P[(s - 1) >> 6] |= bit;
    }
    for (int l = 0; l < c->nlocal; l++) wro[l][i] = wnew[l].size();
    for (int s0 = 0; s0 < n; s0++) {
      const bool here = (P[s0 >> 6] >> (s0 & 63)) & 1ULL;
      const uint64_t *row = strong + ((size_t)i * n + s0) * W;
      uint64_t d = 0;
      for (int w = 0; w < W; w++) d += (uint64_t)__builtin_popcountll(row[w]);
      if (d && !here) return c->fail(DR_E_CONTRACT, "round %d: strong edges on absent vertex (%d,%d)", r, r, s0 + 1);
      if (d && r == 0) return c->fail(DR_E_CONTRACT, "round 0 vertex (0,%d) has strong edges", s0 + 1);
      if (row[W - 1] & ~lastmask) return c->fail(DR_E_CONTRACT, "round %d vertex (%d,%d): strong target source > n", r, r, s0 + 1);
      for (int l = 0; l < c->nlocal; l++) {
        const int g = c->shard0 + l;
        u64 *dst = &rows[(((size_t)i * c->nlocal + l) * n + s0) * SP];
        for (int w = 0; w < WSs; w++) {
          const int gw = g * WSs + w;
          dst[w] = gw < W ? row[gw] : 0ULL;
        }
      }
      const uint32_t ea = weak_off[(size_t)i * n + s0], eb = weak_off[(size_t)i * n + s0 + 1];
      if (eb < ea) return c->fail(DR_E_INVAL, "weak_off not monotone at round %d", r);
      if (eb > ea && !here) return c->fail(DR_E_CONTRACT, "round %d: weak edges on absent vertex (%d,%d)", r, r, s0 + 1);
      sd[(size_t)i * n + s0] = (uint16_t)d;
      wd[(size_t)i * n + s0] = (uint16_t)std::min<uint32_t>(eb - ea, 65535u);
      deg[i] += d;
      rd[i] += d + (eb - ea);
      for (uint32_t e = ea; e < eb; e++) {
        const uint32_t t = weak_tgt[e];
        const int tr = (int)((t >> 11) & 0xFFFFFu), ts = (int)(t & 2047u);
        if (t >> 31)  // dagrider_gpu.h: bit 31 marks a strong edge outside r-1 (App. A Q8)
          return c->fail(DR_E_CONTRACT, "strong edge (%d,%d)->(%d,%d) outside r-1: not supported by dr_shard", r,
                         s0 + 1, tr, ts + 1);
        if (ts >= n) return c->fail(DR_E_CONTRACT, "weak edge (%d,%d)->(%d,%d): source > n", r, s0 + 1, tr, ts + 1);
        if (tr > r - 2) return c->fail(DR_E_CONTRACT, "weak edge (%d,%d)->(%d,%d) must target a round < r-1", r, s0 + 1, tr, ts + 1);
        const int delta = r - tr;
        if (delta > 1023) return c->fail(DR_E_CONTRACT, "weak edge (%d,%d)->(%d,%d): delta %d > 1023 (sharded path)", r, s0 + 1, tr, ts + 1, delta);
        dmax = std::max(dmax, delta);
        const int l = ts / C - c->shard0;
        if (l < 0 || l >= c->nlocal) continue;  // another shard's column
        wnew[l].push_back(((uint32_t)delta << 22) | ((uint32_t)s0 << 11) | (uint32_t)(ts % C));
      }
    }
    for (int l = 0; l < c->nlocal; l++) {
      auto &w = wnew[l];
      // (delta, target) order inside the round: the kernel's wave-uniform OR path
      std::sort(w.begin() + wro[l][i], w.end(), [](uint32_t x, uint32_t y) {
        const uint32_t kx = ((x >> 22) << 11) | (x & 2047u), ky = ((y >> 22) << 11) | (y & 2047u);
        return kx < ky;
      });
      maxw = std::max<size_t>(maxw, w.size() - wro[l][i]);
      // the round's weak columns: runs of equal (delta, target) in the sorted edges
      auto &ck = wck_new[l];
      auto &cr = wcr_new[l];
      wcro_new[l][i] = ck.size();
      for (size_t e = wro[l][i]; e < w.size(); e++) {
        const uint32_t key = ((w[e] >> 22) << 11) | (w[e] & 2047u);
        if (e == wro[l][i] || key != ck.back()) {
          ck.push_back(key);
          cr.resize(cr.size() + W, 0ULL);
        }
        const uint32_t src = (w[e] >> 11) & 2047u;
        cr[(ck.size() - 1) * W + (src >> 6)] |= 1ULL << (src & 63);
      }
    }
  }
  // per-vertex metadata (every shard holds all of it) and the slot order
  const uint32_t S0 = c->h_slot_off.back();
  for (int i = 0; i < k; i++) c->h_slot_off.push_back(S0 + (slot_off[i + 1] - slot_off[0]));
  const size_t ns = (size_t)(slot_off[k] - slot_off[0]);
  SHCHK(c, c->slot_src.grow(((size_t)S0 + ns) * 2 + 64, (size_t)S0 * 2, c->stream));
  if (ns)
    SHCHK(c, hipMemcpyAsync(c->slot_src.as<uint16_t>() + S0, slot_src + slot_off[0], ns * 2, hipMemcpyHostToDevice,
                            c->stream));
  SHCHK(c, hipMemcpyAsync(c->slot_off.as<uint32_t>() + r0 + 1, &c->h_slot_off[r0 + 1], (size_t)k * 4,
                          hipMemcpyHostToDevice, c->stream));
  SHCHK(c, hipMemcpyAsync(c->pres.as<u64>() + (size_t)r0 * W, pres.data(), pres.size() * 8, hipMemcpyHostToDevice,
                          c->stream));
  SHCHK(c, hipMemcpyAsync(c->sdeg.as<uint16_t>() + (size_t)r0 * n, sd.data(), sd.size() * 2, hipMemcpyHostToDevice,
                          c->stream));
  SHCHK(c, hipMemcpyAsync(c->wdeg.as<uint16_t>() + (size_t)r0 * n, wd.data(), wd.size() * 2, hipMemcpyHostToDevice,
                          c->stream));
  SHCHK(c, hipMemcpyAsync(c->rdeg.as<u64>() + r0, rd.data(), rd.size() * 8, hipMemcpyHostToDevice, c->stream));
  SHCHK(c, hipMemcpyAsync(c->sdr.as<u64>() + r0, deg.data(), deg.size() * 8, hipMemcpyHostToDevice, c->stream));
  {  // presence prefix (the canonical positions when every round below is full)
    const size_t base = c->h_ppref.size();
    for (int i = 0; i < k; i++) {
      uint64_t np = 0;
      for (int w = 0; w < W; w++) np += (uint64_t)__builtin_popcountll(pres[(size_t)i * W + w]);
      const int r = r0 + i;
      c->h_ppref.push_back(r == 0 ? 0 : (c->h_ppref.empty() ? 0 : c->h_ppref.back()) + np);
    }
    SHCHK(c, hipMemcpyAsync(c->ppref.as<u64>() + r0, c->h_ppref.data() + base, (size_t)k * 8, hipMemcpyHostToDevice,
                            c->stream));
  }
  // rows are round-major over the local shards ([round][shard][n][SP]): the k new
  // rounds are one contiguous block
  SHCHK(c, hipMemcpyAsync(c->strong.as<u64>() + (size_t)r0 * c->nlocal * n * SP, rows.data(),
                          (size_t)k * c->nlocal * n * SP * 8, hipMemcpyHostToDevice, c->stream));
  for (int l = 0; l < c->nlocal; l++) {
    wro[l][k] = wnew[l].size();
    const uint64_t base = c->h_weak[l].size();
    c->h_weak[l].insert(c->h_weak[l].end(), wnew[l].begin(), wnew[l].end());
    for (int i = 1; i <= k; i++) c->h_woff[l].push_back(base + wro[l][i]);
    wcro_new[l][k] = wck_new[l].size();
    const uint64_t cbase = c->h_wck[l].size();
    c->h_wck[l].insert(c->h_wck[l].end(), wck_new[l].begin(), wck_new[l].end());
    c->h_wcr[l].insert(c->h_wcr[l].end(), wcr_new[l].begin(), wcr_new[l].end());
    for (int i = 1; i <= k; i++) c->h_wcro[l].push_back(cbase + wcro_new[l][i]);
  }
  SHCHK(c, hipStreamSynchronize(c->stream));
  c->h_pres.insert(c->h_pres.end(), pres.begin(), pres.end());
  c->h_deg.insert(c->h_deg.end(), deg.begin(), deg.end());
  c->weak_dirty = true;
  c->lcol_ok = false;
  c->dmax = dmax;
  int depth = 2;
  while (depth < dmax + 2) depth <<= 1;  // k_shard_sweep clears a slot one round after reading it
  if (depth != c->depth || !c->pend.p) {
    SHCHK(c, c->pend.ensure((size_t)c->nlocal * depth * C * 8));
    c->depth = depth;
  }
  c->max_weak_round = maxw;
  c->nrounds += k;
  return DR_OK;
}

extern "C" int dr_shard_reach_sets(dr_shard *c, int q, const int32_t *from, const int32_t *bottom, int strong_only,
                                   uint64_t *out, size_t cap_words, size_t *out_words) {
  if (!c) return DR_E_INVAL;
  if (q < 0 || (q > 0 && (!from || !bottom))) return c->fail(DR_E_INVAL, "bad query arrays");
  if (int rc = sh_set_device(c)) return rc;
  size_t need = 0;
  std::vector<QInfo> qs(q);
  std::vector<size_t> hb(q);
  for (int i = 0; i < q; i++) {
    const int fr = from[2 * i], fs = from[2 * i + 1], b = bottom[i];
    if (fr < 0 || fr >= c->nrounds || b < 0 || b > fr)
      return c->fail(DR_E_INVAL, "query %d: rounds [%d,%d] outside the DAG", i, b, fr);
    qs[i] = QInfo{fr, b, (fs >= 1 && fs <= c->n) ? fs - 1 : -1, 0, 0, 0, fr};
    hb[i] = need;
    need += (size_t)(fr - b + 1) * c->W;
  }
  if (out_words) *out_words = need;
  if (need > cap_words || (!out && need)) return c->fail(DR_E_CAPACITY, "reach sets need %zu words", need);
  if (q == 0) return DR_OK;
  return run_queries(c, qs, hb, strong_only, out);
}

extern "C" int dr_shard_path_batch(dr_shard *c, int q, const int32_t *from, const int32_t *to, int strong_only,
                                   uint8_t *out) {
  if (!c) return DR_E_INVAL;
  if (q < 0 || (q > 0 && (!from || !to || !out))) return c->fail(DR_E_INVAL, "bad query arrays");
  if (int rc = sh_set_device(c)) return rc;
  std::vector<QInfo> qs;
  std::vector<size_t> hb;
  std::vector<int> idx;
  size_t need = 0;
  for (int i = 0; i < q; i++) {
    const int fr = from[2 * i], fs = from[2 * i + 1], tr = to[2 * i], ts = to[2 * i + 1];
    if (fr == tr && fs == ts) { out[i] = 1; continue; }  // process.go:91-93
    if (fr < 0 || fr >= c->nrounds)
      return c->fail(DR_E_INVAL, "query %d: from round %d outside the DAG (Go: index out of range)", i, fr);
    out[i] = 0;
    if (tr < 0 || tr >= fr || ts < 1 || ts > c->n || fs < 1 || fs > c->n) continue;
    // only the row of round tr is needed: a one-round output window
    qs.push_back(QInfo{fr, tr, fs - 1, 0, 0, 0, fr});
    hb.push_back(need);
    need += (size_t)(fr - tr + 1) * c->W;
    idx.push_back(i);
  }
  if (qs.empty()) return DR_OK;
  std::vector<uint64_t> sets(need);
  if (int rc = run_queries(c, qs, hb, strong_only, sets.data())) return rc;
  for (size_t k = 0; k < idx.size(); k++) {
    const int i = idx[k], ts = to[2 * i + 1] - 1;
    out[i] = (sets[hb[k] + (ts >> 6)] >> (ts & 63)) & 1ULL;  // round tr is the first row
  }
  return DR_OK;
}

extern "C" int dr_shard_wave_commit(dr_shard *c, int w0, int w1, uint8_t *commit, int32_t *vcount) {
  if (!c) return DR_E_INVAL;
  if (!commit || !vcount) return c->fail(DR_E_INVAL, "null output");
  if (int rc = sh_set_device(c)) return rc;
  c->last_xbytes = 0;
  return votes(c, w0, w1, commit, vcount);
}

extern "C" int dr_shard_wave_ready(dr_shard *c, int wave, int decided_wave, uint8_t *commit, int32_t *vcount,
                                   int32_t *pushed_waves, int cap, int *n_pushed) {
  if (!c) return DR_E_INVAL;
  if (!commit || !vcount || !n_pushed) return c->fail(DR_E_INVAL, "null output");
  if (int rc = sh_set_device(c)) return rc;
  *n_pushed = 0;
  c->last_xbytes = 0;
  c->last_rounds = 0;
  if (int rc = votes(c, wave, wave, commit, vcount)) return rc;
  if (!*commit) return DR_OK;
  std::vector<std::vector<int32_t>> pushes;
  if (int rc = chains(c, {ChainTask{wave, decided_wave}}, pushes, nullptr)) return rc;
  *n_pushed = (int)pushes[0].size();
  if ((int)pushes[0].size() > cap || (!pushed_waves && !pushes[0].empty()))
    return c->fail(DR_E_CAPACITY, "%zu pushed leaders, capacity %d", pushes[0].size(), cap);
  std::copy(pushes[0].begin(), pushes[0].end(), pushed_waves);
  return DR_OK;
}

extern "C" int dr_shard_order_vertices(dr_shard *c, const int32_t *stack_rs, int nstack, int cur_round, int mode,
                                       size_t *out_n, uint64_t *pop_count, uint64_t *pop_digest) {
  if (!c) return DR_E_INVAL;
  if (nstack < 0 || (nstack > 0 && !stack_rs)) return c->fail(DR_E_INVAL, "bad stack");
  if (mode != DR_DELIVER_REF && mode != DR_DELIVER_PAPER) return c->fail(DR_E_INVAL, "bad mode %d", mode);
  if (int rc = sh_set_device(c)) return rc;
  if (out_n) *out_n = 0;
  if (nstack == 0) return DR_OK;
  if (cur_round >= c->nrounds) return c->fail(DR_E_INVAL, "p.round %d beyond the DAG (Go: index out of range)", cur_round);
  std::vector<Pop> pops;
  for (int t = nstack - 1; t >= 0; t--) {  // LIFO (stack/stack.go:23-28)
    Pop p{stack_rs[2 * t], stack_rs[2 * t + 1], cur_round};
    if (cur_round >= 1 && (p.round < 0 || p.round >= c->nrounds))
      return c->fail(DR_E_INVAL, "popped vertex round %d outside the DAG (Go: index out of range)", p.round);
    if (p.source < 1 || p.source > c->n)
      return c->fail(DR_E_CONTRACT, "popped vertex (%d,%d): source outside [1,n]", p.round, p.source);
    if (cur_round < 1) p.round = std::max(0, std::min(p.round, c->nrounds - 1));
    pops.push_back(p);
  }
  std::vector<uint64_t> cnt(pops.size()), dg(pops.size());
  c->last_xbytes = 0;
  c->last_rounds = 0;
  if (int rc = deliver(c, pops, mode, cnt.data(), dg.data(), nullptr)) return rc;
  uint64_t tot = 0;
  for (auto x : cnt) tot += x;
  if (out_n) *out_n = (size_t)tot;
  if (pop_count) std::copy(cnt.begin(), cnt.end(), pop_count);
  if (pop_digest) std::copy(dg.begin(), dg.end(), pop_digest);
  return DR_OK;
}

extern "C" int dr_shard_replay(dr_shard *c, int nwaves, int chain_mode, int deliver_mode, dr_replay_out *o) {
  if (!c) return DR_E_INVAL;
  if (!o || !o->commit || !o->vcount || !o->push_off) return c->fail(DR_E_INVAL, "null output");
  if (nwaves < 1 || 4 * nwaves >= c->nrounds) return c->fail(DR_E_INVAL, "nwaves %d needs rounds 0..%d mirrored", nwaves, 4 * nwaves);
  if (chain_mode != DR_CHAIN_LITERAL && chain_mode != DR_CHAIN_PERSISTENT) return c->fail(DR_E_INVAL, "bad chain mode");
  if (deliver_mode != DR_DELIVER_REF && deliver_mode != DR_DELIVER_PAPER) return c->fail(DR_E_INVAL, "bad deliver mode");
  if (o->ids && o->ids_cap > 0) return c->fail(DR_E_INVAL, "the sharded replay reports counts and digests, not ids");
  if (int rc = sh_set_device(c)) return rc;
  o->ms_commit = o->ms_chain = o->ms_deliver = o->ms_emit = o->ms_summary = 0;
  o->sweep_count = o->sweep_partial = o->sweep_row_bytes = o->sweep_weak_scanned = o->sweep_shortcut = 0;
  o->n_ids = 0;
  o->canon_segments = -1;
  c->last_xbytes = 0;
  c->last_rounds = 0;
  if (memo_applies(c)) return replay_memo(c, nwaves, chain_mode, deliver_mode, o);
  hipEvent_t t0 = nullptr, t1 = nullptr, t2 = nullptr;
  SHCHK(c, hipEventCreate(&t0));
  SHCHK(c, hipEventCreate(&t1));
  SHCHK(c, hipEventCreate(&t2));
  struct EvGuard { hipEvent_t *e[3]; ~EvGuard() { for (auto p : e) if (*p) (void)hipEventDestroy(*p); } } eg{{&t0, &t1, &t2}};
  SHCHK(c, hipEventRecord(t0, c->stream));
  // 1. commit decisions of every wave
  if (int rc = votes(c, 1, nwaves, o->commit, o->vcount)) return rc;
  SHCHK(c, hipEventRecord(t1, c->stream));
  uint64_t ce = 0;
  for (int w = 1; w <= nwaves; w++)
    if (o->vcount[w - 1] >= 0) ce += c->h_deg[4 * w - 2] + c->h_deg[4 * w - 1] + c->h_deg[4 * w];
  o->commit_edges = ce;
  // 2. chains
  std::vector<ChainTask> tasks;
  int lastw = 0;
  for (int w = 1; w <= nwaves; w++)
    if (o->commit[w - 1]) {
      tasks.push_back(ChainTask{w, chain_mode == DR_CHAIN_PERSISTENT ? lastw : 0});
      lastw = w;
    }
  std::vector<std::vector<int32_t>> pushes;
  if (int rc = chains(c, tasks, pushes, &o->chain_edges)) return rc;
  SHCHK(c, hipEventRecord(t2, c->stream));
  SHCHK(c, hipEventSynchronize(t2));
  SHCHK(c, hipEventElapsedTime(&o->ms_commit, t0, t1));
  SHCHK(c, hipEventElapsedTime(&o->ms_chain, t1, t2));
  int64_t np = 0;
  for (auto &p : pushes) np += (int64_t)p.size();
  o->n_push = np;
  if (np > o->push_cap || !o->push_wave || !o->pop_count || !o->pop_digest)
    return c->fail(DR_E_CAPACITY, "%lld pushed leaders, capacity %lld", (long long)np, (long long)o->push_cap);
  // 3. pops (stack order: the oldest pushed leader first)
  std::vector<Pop> pops;
  int64_t at = 0;
  size_t t = 0;
  for (int w = 1; w <= nwaves; w++) {
    o->push_off[w - 1] = (uint32_t)at;
    if (t < tasks.size() && tasks[t].wave == w) {
      for (int32_t pw : pushes[t]) o->push_wave[at++] = pw;
      for (auto it = pushes[t].rbegin(); it != pushes[t].rend(); ++it)
        pops.push_back(Pop{4 * (*it - 1) + 1, c->lead_src(*it), 4 * w});
      t++;
    }
  }
  o->push_off[nwaves] = (uint32_t)at;
  std::vector<uint64_t> pe(pops.size());
  if (!pops.empty())
    if (int rc = deliver(c, pops, deliver_mode, o->pop_count, o->pop_digest, pe.data())) return rc;
  o->ms_deliver = c->ms_sweep;
  o->ms_emit = c->ms_emit;
  uint64_t de = 0;
  for (size_t i = 0; i < pops.size(); i++) {
    de += pe[i];
    if (o->pop_edges) o->pop_edges[i] = pe[i];
  }
  o->deliver_edges = de;
  o->sweep_count = (uint64_t)pops.size();
  return DR_OK;
}

extern "C" int dr_shard_stats(const dr_shard *c, float *ms, uint64_t *rounds, uint64_t *exchange_bytes) {
  if (!c) return DR_E_INVAL;
  if (ms) *ms = c->last_ms;
  if (rounds) *rounds = c->last_rounds;
  if (exchange_bytes) *exchange_bytes = c->last_xbytes;
  return DR_OK;
}

extern "C" int dr_shard_host_syncs(const dr_shard *c, uint64_t *syncs) {
  if (!c || !syncs) return DR_E_INVAL;
  *syncs = c->syncs;
  return DR_OK;
}

#ifdef DR_SWEEP_TIMING
// profiling build only: the per-query ticks of the last k_ms_sweep_full
// (shard_fused.hpp g_ms_timing; 8 u64 per query, wall-clock ticks)
extern "C" int dr_debug_ms_timing(uint64_t *out, int nq) {
  if (nq < 0 || nq > drs::kMsTimingQ) return DR_E_INVAL;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(drs::g_ms_timing), (size_t)nq * 64, 0, hipMemcpyDeviceToHost) ==
                 hipSuccess
             ? DR_OK
             : DR_E_HIP;
}
#endif
