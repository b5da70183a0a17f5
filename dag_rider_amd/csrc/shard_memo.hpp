// shard_memo.hpp -- kernels of the memoized replay on the column-sharded DAG
// (dr_shard_replay, include/dagrider_shard.h).
//
// The single-GPU replay's memo carried over to column shards:
//
//   k_ms_summary   per round and shard: U_r = OR of the shard's columns of every
//                  strong row, WU_r[d] = the shard's weak targets at delta d+2
//                  (from its weak columns).  Every shard reads only its own
//                  columns of the rows: the HBM-bound pass splits G ways.
//   k_ms_kcand     K^cand_r = U_{r+1} | OR_d WU_{r+d+2}[d] on the shard's columns
//                  (K^cand_T = P_T); the shards' columns are all-gathered into a
//                  full-width K on every shard, and good_r = K^cand_r covers P_r.
//   k_ms_step      one round of every live query, one workgroup per (query,
//                  shard): the query's full frontier of round r (all-gathered),
//                  its decisions -- chain restart (process.go:341-350), merge with
//                  K (the cone below is K's), stop -- taken alike on every shard,
//                  then the shard's columns of the rounds below: U / WU on a full
//                  round, else the frontier's strong rows and weak columns into a
//                  per-query ring of pending rounds; the shard's columns of round
//                  r-1 go to the exchange.  Queries step together by RELATIVE
//                  round: query q is at round top_q - j at step j, so a batch of
//                  pops (each stopping a few rounds under its top) costs a handful
//                  of steps, not the depth of the DAG.
//     query kinds: MQ_POP (orderVertices cone, strong + weak, merges with K),
//                  MQ_CHAIN (waveReady's leader chain, strong only, restarts),
//                  MQ_CANON (a canonical segment below a bad round: K rows).
//   k_ms_cstats / k_ms_prefix / k_ms_rg   canonical counts, edges, digests and
//                  their prefixes C, E, G over rounds (every shard alike).
//   k_ms_emit      per pop query: the canonical prefix at its cut plus its own
//                  rounds above the cut (counts, order-sensitive digest, edges).
//
// Semantics are dr_replay's (engine.hip): same commits, pushes, per-pop counts,
// digests and edge totals, bit for bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "wave_ops.hpp"

namespace drs {

using dr::u64;
using dr::shfl_xor64;
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

constexpr int MS_NT = 256;  // threads per workgroup (4 waves)
enum : int32_t { MQ_POP = 0, MQ_CHAIN = 1, MQ_CANON = 2 };

struct MQuery {
  int32_t type, top, bottom, src0;
  int64_t mask_off;   // MQ_POP: word offset of the mask row of round `top` (row j = round top - j)
  int32_t push_base;  // MQ_CHAIN: first slot of the query's pushes in push_out
  int32_t pad;
};

// Per-query state, double-buffered by step parity (every shard reads the state
// before step j; the shard-0 workgroup writes the state after it).
struct MState {
  int32_t done, run, low, stop;  // stop: the round where the query merged / ended
  int32_t merged, npush;         // MQ_CANON: npush counts the segments walked
  int32_t cur, fresh;            // MQ_CANON: its current round; 1 = start the next segment below cur
  int32_t steps, pad;            // stepped form: launches the query was live in
  u64 edges;                     // MQ_CHAIN: strong degrees of the expanded vertices
};

struct MArgs {
  const u64 *strong;        // [max_rounds][nlocal][n][SP]: round-major over the local shards
  int64_t strong_stride;    // words between local shards' rows of one round (n * SP)
  int64_t strong_rstride;   // words per round (nlocal * n * SP)
  const uint32_t *wck;      // weak columns: key delta << 11 | local column
  const u64 *wcr;           // [column][W] sources with that weak edge
  const uint64_t *wcro;     // [nlocal][R+1] absolute column offsets per round
  const u64 *pres;          // [R][W]
  const uint16_t *sdeg;     // [R][n] strong degree
  const uint16_t *wdeg;     // [R][n] weak degree
  const u64 *sdr;           // [R] strong degree sum of a round
  const u64 *rdeg;          // [R] strong + weak degree sum of a round
  const uint16_t *lead;     // [nlead] chooseLeader(w), 1-based
  const u64 *U;             // [nlocal][R][SP]
  const u64 *WU;            // [nlocal][R][dd][SP]
  u64 *K;                   // [R][W] canonical cone, full width
  const MQuery *q;
  MState *st0, *st1;
  u64 *pend;                // [nlocal][nq][depth][SP]
  u64 *recv0, *recv1;       // [G][nq][WSs]: step j reads recv_{j&1}, local mode writes recv_{(j+1)&1}
  u64 *send;                // RCCL mode: [nq][WSs]
  u64 *masks;               // MQ_POP frontier rows
  int32_t *push_out;
  const uint8_t *good;       // [T+1] K^cand_r covers P_r (MQ_CANON: where segments start)
  const uint32_t *slot_off;  // [R+1] slot order (insertion order of every round)
  const uint16_t *slot_src;  // 1-based source per slot (0 = ghost)
  int32_t n, W, WSs, SP, G, shard0, nlocal, local, nq, depth, dd, dmax, summary, R, nlead, T;
};

// Round summaries of one shard: one workgroup per (round, local shard).  Thread t's
// 16-B chunks hold columns (2t) mod SP and (2t+1) mod SP of every row it reads
// (2 * MS_NT is a multiple of SP); lanes of a column are OR-ed by xor-shuffles.
__global__ __launch_bounds__(MS_NT) void k_ms_summary(MArgs a, int T, u64 *__restrict__ U, u64 *__restrict__ WU) {
  const int r = blockIdx.x + 1, l = blockIdx.y, tid = threadIdx.x, lane = tid & 63;
  if (r > T) return;
  const int SP = a.SP;
  __shared__ u64 sU[32];
  __shared__ u64 sWU[64 * 32];
  if (tid < SP) sU[tid] = 0;
  for (int i = tid; i < a.dd * SP; i += MS_NT) sWU[i] = 0;
  __syncthreads();
  const u64 *rows = a.strong + (size_t)r * a.strong_rstride + (size_t)l * a.strong_stride;
  const size_t nw = (size_t)a.n * SP;
  if (SP >= 2) {
    const u64x2 *p = reinterpret_cast<const u64x2 *>(rows);
    u64 x0 = 0, x1 = 0;
    for (size_t i = tid; i < nw / 2; i += MS_NT) {
      const u64x2 v = __builtin_nontemporal_load(p + i);
      x0 |= v.x;
      x1 |= v.y;
    }
    for (int off = SP / 2; off < 64; off <<= 1) {
      x0 |= shfl_xor64(x0, off);
      x1 |= shfl_xor64(x1, off);
    }
    if (lane < SP / 2) {
      if (x0) atomicOr(&sU[2 * lane], x0);
      if (x1) atomicOr(&sU[2 * lane + 1], x1);
    }
  } else {
    u64 x = 0;
    for (size_t i = tid; i < nw; i += MS_NT) x |= __builtin_nontemporal_load(rows + i);
    x = dr::wave_or(x);
    if (lane == 0 && x) atomicOr(&sU[0], x);
  }
  const uint64_t c0 = a.wcro[(size_t)l * (a.R + 1) + r], c1 = a.wcro[(size_t)l * (a.R + 1) + r + 1];
  for (uint64_t j = c0 + tid; j < c1; j += MS_NT) {
    const uint32_t key = a.wck[j];
    const int d = (int)(key >> 11) - 2, tc = (int)(key & 2047u);
    atomicOr(&sWU[d * SP + (tc >> 6)], 1ULL << (tc & 63));
  }
  __syncthreads();
  const size_t ub = (size_t)l * a.R + r;
  if (tid < SP) U[ub * SP + tid] = sU[tid];
  for (int i = tid; i < a.dd * SP; i += MS_NT) WU[ub * a.dd * SP + i] = sWU[i];
}

// K^cand on the shard's columns, one wave per round (lane = column word).  Local
// mode writes the full-width K directly; RCCL mode writes ksend[r][WSs] for the
// all-gather (k_ms_kunpack lays it out).
__global__ __launch_bounds__(MS_NT) void k_ms_kcand(MArgs a, int T, u64 *__restrict__ ksend) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), l = blockIdx.y, cw = threadIdx.x & 63;
  if (r > T || cw >= a.WSs) return;
  const int g = a.shard0 + l, w = g * a.WSs + cw;
  u64 v = 0;
  if (w < a.W) {
    if (r == T) {
      v = a.pres[(size_t)r * a.W + w];
    } else {
      const size_t ub = (size_t)l * a.R;
      v = a.U[(ub + r + 1) * a.SP + cw];
      for (int d = 0; d < a.dd && r + d + 2 <= T; d++) v |= a.WU[((ub + r + d + 2) * a.dd + d) * a.SP + cw];
    }
  }
  if (a.local) {
    if (w < a.W) a.K[(size_t)r * a.W + w] = v;
  } else {
    ksend[(size_t)r * a.WSs + cw] = v;
  }
}

// RCCL mode: krecv [G][T+1][WSs] -> K [T+1][W]
__global__ void k_ms_kunpack(MArgs a, int T, const u64 *__restrict__ krecv) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)(T + 1) * a.W) return;
  const int r = (int)(i / a.W), w = (int)(i % a.W);
  a.K[i] = krecv[((size_t)(w / a.WSs) * (T + 1) + r) * a.WSs + w % a.WSs];
}

// good_r = K_r covers P_r, one wave per round
__global__ __launch_bounds__(MS_NT) void k_ms_good(MArgs a, int T, uint8_t *__restrict__ good) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r > T) return;
  bool bad = false;
  if (lane < a.W) {
    const u64 p = a.pres[(size_t)r * a.W + lane];
    bad = (a.K[(size_t)r * a.W + lane] & p) != p;
  }
  bad = __ballot(bad) != 0ULL;
  if (lane == 0) good[r] = bad ? 0 : 1;
}

// A canonical segment below bad round b (MQ_CANON): its ring of pending rounds
// starts with what the full rounds above b put below b (the WU of rounds b+1 ..
// b+dd+1), exactly as k_canon (kernels.hpp) starts it.  Every thread of the
// workgroup calls it; the caller synchronises after.
__device__ __forceinline__ void canon_ring_init(const MArgs &a, u64 *pend, int l, int b) {
  const int tid = threadIdx.x, SP = a.SP, dm = a.depth - 1;
  for (int i = tid; i < a.depth * SP; i += MS_NT) pend[i] = 0;
  __syncthreads();
  if (tid >= SP) return;
  const size_t ub = (size_t)l * a.R;
  for (int x = b - 1; x >= 0 && x >= b - a.dd; x--) {
    u64 v = 0;
    for (int y = max(b + 1, x + 2); y <= a.T && y <= x + a.dd + 1; y++)
      v |= a.WU[((ub + y) * a.dd + (y - x - 2)) * SP + tid];
    pend[(size_t)(x & dm) * SP + tid] = v;
  }
}

// The highest bad round below `below` (-1: none), one wave (every lane gets it).
// The 0/1 flags are read 8 at a time (u64 words, a byte != 1 is a bad round), 16
// words per lane in flight: one pass covers 8192 rounds.
__device__ __forceinline__ int next_bad(const MArgs &a, int below) {
  constexpr int PL = 16;
  constexpr uint64_t ONES = 0x0101010101010101ULL;
  const int lane = threadIdx.x & 63;
  if (below <= 0) return -1;
  const uint64_t *g = reinterpret_cast<const uint64_t *>(a.good);
  const int wtop = (below - 1) >> 3, nb = below - 8 * wtop;  // rounds of word wtop below `below`: its low nb bytes
  const uint64_t topmask = nb >= 8 ? ~0ULL : (1ULL << (8 * nb)) - 1ULL;
  for (int top = wtop; top >= 0; top -= 64 * PL) {
    uint64_t v[PL];
#pragma unroll
    for (int k = 0; k < PL; k++) {
      const int x = top - PL * lane - k;
      v[k] = x >= 0 ? g[x] : ONES;
    }
    int best = -1;
#pragma unroll
    for (int k = PL - 1; k >= 0; k--) {
      const int x = top - PL * lane - k;
      uint64_t bad = v[k] ^ ONES;
      if (x == wtop) bad &= topmask;
      if (bad) best = 8 * x + (63 - __clzll(bad)) / 8;
    }
    for (int off = 32; off > 0; off >>= 1) best = max(best, __shfl_xor(best, off));
    if (best >= 0) return best;
  }
  return -1;
}

// One step (see the file comment).  Grid (nq, nlocal).
__global__ __launch_bounds__(MS_NT) void k_ms_step(MArgs a, int j) {
  const int qi = blockIdx.x, l = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const bool writer = l == 0;
  const MState *sc = (j & 1) ? a.st1 : a.st0;
  MState *sn = (j & 1) ? a.st0 : a.st1;
  const MState S = sc[qi];
  if (S.done) {
    if (writer && tid == 0) sn[qi] = S;
    return;
  }
  const MQuery Q = a.q[qi];
  const int W = a.W, SP = a.SP, dm = a.depth - 1;
  __shared__ u64 sFE[32];
  __shared__ u64 sAcc[32];
  __shared__ int sCtl[2];
  __shared__ int sStart;
  u64 *pend = a.pend + ((size_t)l * a.nq + qi) * a.depth * SP;
  // MQ_CANON walks the canonical segments top down on its own (k_canon's walk): at a
  // segment start it finds the next bad round below its current round, resets its
  // ring there, and starts from K^cand; it is done when no bad round is left
  int r = Q.top - j;
  bool start = false;
  MState S1 = S;
  if (Q.type == MQ_CANON) {
    r = S.cur;
    if (S.fresh) {
      if (wv == 0) {
        const int b = next_bad(a, S.cur);
        if (lane == 0) sStart = b;
      }
      __syncthreads();
      const int b = sStart;
      if (b < 0) {
        if (writer && tid == 0) {
          S1.done = 1;
          sn[qi] = S1;
        }
        return;
      }
      canon_ring_init(a, pend, l, b);
      __syncthreads();
      r = b;
      start = true;
      S1.run = 0;
      S1.low = b;
      S1.npush = S.npush + 1;
    }
  }
  if (tid < SP) sAcc[tid] = 0;
  if (wv == 0) {
    const bool act = lane < W;
    u64 f = 0, p = 0;
    if (act) {
      if (start) {
        f = a.K[(size_t)r * W + lane];
      } else if (j == 0) {
        f = (Q.src0 >= 0 && lane == (Q.src0 >> 6)) ? 1ULL << (Q.src0 & 63) : 0ULL;
      } else {
        const u64 *rv = (j & 1) ? a.recv1 : a.recv0;
        f = rv[((size_t)(lane / a.WSs) * a.nq + qi) * a.WSs + lane % a.WSs];
      }
      p = a.pres[(size_t)r * W + lane];
    }
    // waveReady's chain (process.go:342-350): a reachable, present leader of wave
    // wv' is pushed and the chain goes on from it alone
    bool restart = false;
    int wvv = 0;
    if (Q.type == MQ_CHAIN && r < Q.top && ((r - 1) & 3) == 0) {
      wvv = ((r - 1) >> 2) + 1;
      const int L = (wvv < a.nlead ? (int)a.lead[wvv] : 1) - 1;
      const u64 fl = __shfl(f & p, L >> 6);
      if ((fl >> (L & 63)) & 1ULL) {
        f = lane == (L >> 6) ? 1ULL << (L & 63) : 0ULL;
        restart = true;
      }
    }
    const u64 fe = f & p;
    const bool nz = __ballot(act && f != 0ULL) != 0ULL;
    const bool full = __ballot(act && fe != p) == 0ULL;
    int run = S1.run, low = S1.low;
    if (nz) low = min(low, r - 1);
    bool merged = false, done;
    if (Q.type == MQ_POP) {
      const u64 k = act ? a.K[(size_t)r * W + lane] : 0ULL;
      run = __ballot(act && f != k) == 0ULL ? run + 1 : 0;
      merged = a.summary && run >= a.dmax;
      done = merged || r <= Q.bottom || (!nz && low >= r);
    } else if (Q.type == MQ_CHAIN) {
      done = r <= Q.bottom || (!nz && low >= r);
    } else {  // MQ_CANON: the segment ends where dmax full rounds restore the regime
      run = full ? run + 1 : 0;
      done = run >= a.dmax || r == 0;
    }
    if (writer && act) {
      if (Q.type == MQ_POP) a.masks[Q.mask_off + (int64_t)j * W + lane] = f;
      else if (Q.type == MQ_CANON) a.K[(size_t)r * W + lane] = f;
    }
    const bool summary = !done && a.summary && full;
    u64 edges = S.edges;
    if (Q.type == MQ_CHAIN && !done && writer) {
      if (summary) {
        edges += a.sdr[r];
      } else {
        u64 e = 0;
        for (u64 x = act ? fe : 0ULL; x; x &= x - 1) e += a.sdeg[(size_t)r * a.n + lane * 64 + __builtin_ctzll(x)];
        edges += dr::wave_sum(e);
      }
    }
    if (!done && Q.type != MQ_CHAIN && __ballot(act && fe != 0ULL) != 0ULL) low = min(low, r - a.dmax);
    if (writer && lane == 0) {
      MState o = S1;
      o.done = done;
      o.run = run;
      o.low = low;
      o.stop = done ? r : 0;
      o.merged = merged;
      o.npush = S1.npush + (restart ? 1 : 0);
      o.edges = edges;
      if (Q.type == MQ_CANON) {  // a finished segment: look for the next one below r
        o.done = 0;
        o.fresh = done ? 1 : 0;
        o.cur = done ? r : r - 1;
      }
      if (restart) a.push_out[Q.push_base + S1.npush] = wvv;
      sn[qi] = o;
    }
    if (act) sFE[lane] = fe;
    if (lane == 0) {
      sCtl[0] = done;
      sCtl[1] = summary;
    }
  }
  __syncthreads();
  if (sCtl[0]) return;
  const bool weak = Q.type != MQ_CHAIN;
  if (sCtl[1]) {  // full round: the union of its rows and weak columns
    if (tid < SP) {
      const size_t ub = (size_t)l * a.R + r;
      sAcc[tid] = a.U[ub * SP + tid];
      if (weak)
        for (int d = 0; d < a.dd; d++) {
          const int tr = r - d - 2;
          if (tr < Q.bottom) break;
          pend[(size_t)(tr & dm) * SP + tid] |= a.WU[(ub * a.dd + d) * SP + tid];
        }
    }
  } else {
    // strong rows of the frontier: wave wv takes frontier words wv, wv + 4, ...;
    // lane reads words lane + 64 i of the word's 64 rows (column lane mod SP)
    const u64 *rows = a.strong + (size_t)r * a.strong_rstride + (size_t)l * a.strong_stride;
    // saturation (as the unsharded sweep's expand_round): once the OR of the rows a
    // wave has read equals U_r, the union of every row of round r, no further row
    // can add a bit and the wave stops reading
    const u64 ur = lane < SP ? a.U[((size_t)l * a.R + r) * SP + lane] : 0ULL;
    u64 acc = 0;
    for (int w = wv; w < W; w += MS_NT / 64) {
      const u64 bits = sFE[w];
      if (!bits) continue;
      const u64 *blk = rows + (size_t)w * 64 * SP;
      for (int i = 0; i < SP; i++) {
        const int k = lane + 64 * i;
        if ((bits >> (k / SP)) & 1ULL) acc |= blk[k];
      }
      u64 red = acc;
      for (int off = SP; off < 64; off <<= 1) red |= shfl_xor64(red, off);
      if (__ballot(lane < SP && red != ur) == 0ULL) break;
    }
    for (int off = SP; off < 64; off <<= 1) acc |= shfl_xor64(acc, off);
    if (lane < SP && acc) atomicOr(&sAcc[lane], acc);
    if (weak) {  // weak columns of round r whose target is this shard's
      const uint64_t c0 = a.wcro[(size_t)l * (a.R + 1) + r], c1 = a.wcro[(size_t)l * (a.R + 1) + r + 1];
      for (uint64_t jj = c0 + tid; jj < c1; jj += MS_NT) {
        const u64 *row = a.wcr + jj * W;
        u64 hit = 0;
        for (int w = 0; w < W; w++) hit |= row[w] & sFE[w];
        if (!hit) continue;
        const uint32_t key = a.wck[jj];
        const int tr = r - (int)(key >> 11), tc = (int)(key & 2047u);
        if (tr < Q.bottom) continue;
        atomicOr(&pend[(size_t)(tr & dm) * SP + (tc >> 6)], 1ULL << (tc & 63));
      }
    }
  }
  __syncthreads();
  // the shard's columns of round r-1 (complete: weak contributions came from the
  // rounds above, already expanded) leave the ring for the exchange
  if (tid < a.WSs) {
    u64 *ps = &pend[(size_t)((r - 1) & dm) * SP + tid];
    const u64 v = *ps | sAcc[tid];
    *ps = 0ULL;
    if (a.local) {
      u64 *rv = (j & 1) ? a.recv0 : a.recv1;
      rv[((size_t)(a.shard0 + l) * a.nq + qi) * a.WSs + tid] = v;
    } else {
      a.send[(size_t)qi * a.WSs + tid] = v;
    }
  }
}

// number of live queries in the state buffer (host polls it every few steps)
__global__ __launch_bounds__(MS_NT) void k_ms_alive(const MState *__restrict__ st, int nq, int *__restrict__ out) {
  __shared__ int s;
  if (threadIdx.x == 0) s = 0;
  __syncthreads();
  int c = 0;
  for (int i = threadIdx.x; i < nq; i += MS_NT) c += st[i].done ? 0 : 1;
  if (c) atomicAdd(&s, c);
  __syncthreads();
  if (threadIdx.x == 0) *out = s;
}

// canonical per-round terms, one wave per round: RD = |K & P| (round 0: 0), CE =
// the strong + weak degrees of K & P (the round total when K covers P)
__global__ __launch_bounds__(MS_NT) void k_ms_cstats(MArgs a, int T, u64 *__restrict__ RD, u64 *__restrict__ CE) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r > T) return;
  u64 kp = 0, p = 0;
  if (lane < a.W) {
    p = a.pres[(size_t)r * a.W + lane];
    kp = a.K[(size_t)r * a.W + lane] & p;
  }
  const u64 cnt = dr::wave_sum((u64)__popcll(kp));
  u64 e;
  if (__ballot(kp != p) == 0ULL) {
    e = a.rdeg[r];
  } else {
    u64 acc = 0;
    for (u64 x = kp; x; x &= x - 1) {
      const size_t at = (size_t)r * a.n + lane * 64 + __builtin_ctzll(x);
      acc += (u64)a.sdeg[at] + a.wdeg[at];
    }
    e = dr::wave_sum(acc);
  }
  if (lane == 0) {
    RD[r] = r == 0 ? 0 : cnt;
    CE[r] = r == 0 ? 0 : e;
  }
}

// exclusive scan over one workgroup of MS_NT threads (wave shuffles + one LDS hop)
__device__ __forceinline__ u64 ms_block_scan(u64 v, u64 *s, u64 &total) {
  constexpr int NW = MS_NT / 64;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  u64 x = v;
  for (int off = 1; off < 64; off <<= 1) {
    const u64 y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  if (lane == 63) s[wid] = x;
  __syncthreads();
  u64 base = 0;
  total = 0;
  for (int w = 0; w < NW; w++) {
    if (w < wid) base += s[w];
    total += s[w];
  }
  __syncthreads();
  return base + x - v;
}

// inclusive prefix over rounds 0..T of up to two arrays, one workgroup of NT
// threads: tiles of NT * CH rounds, wave v's CH chunks of 64 consecutive rounds
// loaded together (coalesced, one memory latency per tile), scanned across the
// lanes with the wave's running carry, then offset by the waves before it
template <int NT>
__device__ __forceinline__ void ms_prefix_one(int n, const u64 *__restrict__ a, u64 *__restrict__ b, u64 *part) {
  constexpr int NW = NT / 64, CH = 8, TILE = NT * CH;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  u64 tile_carry = 0;
  for (int t0 = 0; t0 < n; t0 += TILE) {
    const int base = t0 + wv * CH * 64 + lane;
    u64 v[CH];
#pragma unroll
    for (int c = 0; c < CH; c++) v[c] = base + c * 64 < n ? a[base + c * 64] : 0ULL;
    u64 run = 0;
#pragma unroll
    for (int c = 0; c < CH; c++) {
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const u64 y = __shfl_up(v[c], off);
        if (lane >= off) v[c] += y;
      }
      v[c] += run;
      run = __shfl(v[c], 63);
    }
    if (lane == 0) part[wv] = run;
    __syncthreads();
    u64 off = tile_carry, tot = 0;
    for (int w = 0; w < NW; w++) {
      if (w < wv) off += part[w];
      tot += part[w];
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < CH; c++)
      if (base + c * 64 < n) b[base + c * 64] = off + v[c];
    tile_carry += tot;
  }
}
// inclusive prefixes of two arrays (a1 may be null) over 0..n-1 in one pass of one
// workgroup of NT threads: tiles of NT * CH elements, thread t owns CH consecutive
// elements (serial sums), one wave scan of the threads' totals for both arrays, one
// LDS hop for the waves' totals.  part: 2 * NT / 64 words of LDS.
template <int NT, int CH = 4>
__device__ __forceinline__ void ms_prefix_two(int n, const u64 *__restrict__ a0, u64 *__restrict__ b0,
                                              const u64 *__restrict__ a1, u64 *__restrict__ b1, u64 *part) {
  constexpr int NW = NT / 64, TILE = NT * CH;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  u64 cx = 0, cy = 0;  // carries from the tiles before
  for (int t0 = 0; t0 < n; t0 += TILE) {
    const int base = t0 + (int)threadIdx.x * CH;
    u64 x[CH], y[CH];
#pragma unroll
    for (int c = 0; c < CH; c++) {
      x[c] = base + c < n ? a0[base + c] : 0ULL;
      y[c] = (a1 && base + c < n) ? a1[base + c] : 0ULL;
    }
#pragma unroll
    for (int c = 1; c < CH; c++) {
      x[c] += x[c - 1];
      y[c] += y[c - 1];
    }
    const u64 sx = x[CH - 1], sy = y[CH - 1];
    u64 ix = sx, iy = sy;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const u64 tx = dr::shfl_up64(ix, off), ty = dr::shfl_up64(iy, off);
      if (lane >= off) {
        ix += tx;
        iy += ty;
      }
    }
    if (lane == 63) {
      part[wv] = ix;
      part[NW + wv] = iy;
    }
    __syncthreads();
    u64 ox = cx, oy = cy, tx = 0, ty = 0;
    for (int w = 0; w < NW; w++) {
      const u64 px = part[w], py = part[NW + w];
      if (w < wv) {
        ox += px;
        oy += py;
      }
      tx += px;
      ty += py;
    }
    __syncthreads();
    ox += ix - sx;
    oy += iy - sy;
#pragma unroll
    for (int c = 0; c < CH; c++)
      if (base + c < n) {
        b0[base + c] = ox + x[c];
        if (b1) b1[base + c] = oy + y[c];
      }
    cx += tx;
    cy += ty;
  }
}
template <int NT>
__global__ __launch_bounds__(NT) void k_ms_prefix(int T, const u64 *__restrict__ a0, u64 *__restrict__ b0,
                                                  const u64 *__restrict__ a1, u64 *__restrict__ b1) {
  __shared__ u64 part[NT / 64];
  ms_prefix_one<NT>(T + 1, a0, b0, part);
  if (a1) ms_prefix_one<NT>(T + 1, a1, b1, part);
}

// One wave emits round y's slots whose source bit is set in mw (lane w < W holds
// word w) in insertion order from position pos: digest terms and, with sdeg, the
// strong + weak degrees (this lane's shares).  Lane l takes SPT consecutive slots
// of each 64*SPT block: every slot and degree load of a block goes out at once
// (three memory latencies per round, not two per 64 slots), and an exclusive scan
// of the lanes' hit counts keeps the slot order.
__device__ __forceinline__ void ms_wave_emit(const uint32_t *__restrict__ slot_off, const uint16_t *__restrict__ slot_src,
                                             int y, u64 mw, u64 pos, int W, const uint16_t *sdeg, const uint16_t *wdeg,
                                             int n, u64 &dg, u64 &ed) {
  constexpr int SPT = 16;
  const int lane = threadIdx.x & 63;
  const uint32_t s0 = slot_off[y], s1 = slot_off[y + 1];
  const uint32_t hi32 = (uint32_t)(mw >> 32), lo32 = (uint32_t)mw;
  for (uint32_t c0 = s0; c0 < s1; c0 += 64 * SPT) {
    const uint32_t i0 = c0 + (uint32_t)lane * SPT;
    int src[SPT];
#pragma unroll
    for (int q = 0; q < SPT; q++) src[q] = i0 + q < s1 ? (int)slot_src[i0 + q] : 0;
    uint32_t inm = 0;  // bit q: slot i0 + q is delivered
#pragma unroll
    for (int q = 0; q < SPT; q++) {
      const int sv = src[q];
      const int wd = sv > 0 ? (sv - 1) >> 6 : 0;
      const u64 word = ((u64)(uint32_t)__shfl((int)hi32, wd, 64) << 32) | (uint32_t)__shfl((int)lo32, wd, 64);
      inm |= (sv > 0 && ((word >> ((sv - 1) & 63)) & 1ULL)) ? 1u << q : 0u;
    }
    uint16_t d1[SPT], d2[SPT];
    if (sdeg) {
#pragma unroll
      for (int q = 0; q < SPT; q++) {
        const size_t at = (size_t)y * n + (src[q] > 0 ? src[q] - 1 : 0);
        d1[q] = (inm >> q) & 1u ? sdeg[at] : (uint16_t)0;
        d2[q] = (inm >> q) & 1u ? wdeg[at] : (uint16_t)0;
      }
    }
    const uint32_t cnt = (uint32_t)__popc(inm);
    uint32_t inc = cnt;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t t = __shfl_up(inc, off);
      if (lane >= off) inc += t;
    }
    u64 k = pos + (inc - cnt);
#pragma unroll
    for (int q = 0; q < SPT; q++)
      if ((inm >> q) & 1u) dg += dr::digest_term((uint32_t)y, (uint32_t)src[q], k++);
    if (sdeg) {
#pragma unroll
      for (int q = 0; q < SPT; q++) ed += (u64)d1[q] + d2[q];
    }
    pos += __shfl(inc, 63);
  }
  (void)W;
}

// canonical digest of each round r >= 1 (positions from C_{r-1}), one wave per round
__global__ __launch_bounds__(MS_NT) void k_ms_rg(MArgs a, int T, const uint32_t *__restrict__ slot_off,
                                                 const uint16_t *__restrict__ slot_src, const u64 *__restrict__ Cc,
                                                 u64 *__restrict__ RG) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r > T) return;
  if (r == 0) {
    if (lane == 0) RG[0] = 0;
    return;
  }
  const u64 mw = lane < a.W ? a.K[(size_t)r * a.W + lane] & a.pres[(size_t)r * a.W + lane] : 0ULL;
  u64 dg = 0, ed = 0;
  ms_wave_emit(slot_off, slot_src, r, mw, Cc[r - 1], a.W, nullptr, nullptr, a.n, dg, ed);
  dg = dr::wave_sum(dg);
  if (lane == 0) RG[r] = dg;
}

// REF emission of one pop query by one workgroup of MS_NT threads (every thread
// calls it): the canonical prefix at the cut (C, G, E) plus the query's own
// rounds cut+1 .. top from its mask rows, 64 rounds at a time (counts, exclusive
// scan, digests and degrees).  The fused sweep calls it right after its own
// wave 0 wrote the mask rows: a workgroup barrier orders them (one CU, its L1
// writes through).
__device__ __forceinline__ void ms_emit_query(const MArgs &a, const MQuery &Q, const MState &S,
                                              const uint32_t *__restrict__ slot_off,
                                              const uint16_t *__restrict__ slot_src, const u64 *__restrict__ Cc,
                                              const u64 *__restrict__ Gc, const u64 *__restrict__ Ec, int b,
                                              u64 *__restrict__ qcount, u64 *__restrict__ qdigest,
                                              u64 *__restrict__ qedges) {
  __shared__ uint32_t sCnt[64];
  __shared__ u64 sPos[64];
  __shared__ u64 sTot, sDg, sEd;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int top = Q.top;
  int cut, lo;
  if (S.merged) {
    cut = min(S.stop + a.dmax - 1, top);
    lo = cut + 1;
  } else {
    cut = 0;
    lo = max(1, S.stop);
  }
  if (tid == 0) {
    sDg = 0;
    sEd = 0;
  }
  auto mask_word = [&](int y) -> u64 {
    if (lane >= a.W) return 0ULL;
    return a.masks[Q.mask_off + (int64_t)(top - y) * a.W + lane] & a.pres[(size_t)y * a.W + lane];
  };
  u64 run = Cc[cut];
  for (int y0 = lo; y0 <= top; y0 += 64) {
    const int ny = min(64, top - y0 + 1);
    for (int i = wv; i < ny; i += MS_NT / 64) {
      const u64 c = dr::wave_sum((u64)__popcll(mask_word(y0 + i)));
      if (lane == 0) sCnt[i] = (uint32_t)c;
    }
    __syncthreads();
    if (wv == 0) {
      u64 x = lane < ny ? sCnt[lane] : 0;
      const u64 v = x;
      for (int off = 1; off < 64; off <<= 1) {
        const u64 yv = __shfl_up(x, off);
        if (lane >= off) x += yv;
      }
      if (lane < ny) sPos[lane] = run + x - v;
      if (lane == 63) sTot = x;
    }
    __syncthreads();
    u64 dg = 0, ed = 0;
    for (int i = wv; i < ny; i += MS_NT / 64) {
      const int y = y0 + i;
      ms_wave_emit(slot_off, slot_src, y, mask_word(y), sPos[i], a.W, a.sdeg, a.wdeg, a.n, dg, ed);
    }
    dg = dr::wave_sum(dg);
    ed = dr::wave_sum(ed);
    if (lane == 0) {
      atomicAdd(&sDg, dg);
      atomicAdd(&sEd, ed);
    }
    run += sTot;
    __syncthreads();
  }
  if (tid == 0) {
    qcount[b] = run;
    qdigest[b] = sDg + Gc[cut];
    qedges[b] = sEd + Ec[cut];
  }
}

// REF emission, one workgroup per pop query (qidx; null: query b)
__global__ __launch_bounds__(MS_NT) void k_ms_emit(MArgs a, const int32_t *__restrict__ qidx, const MState *__restrict__ st,
                                                   const uint32_t *__restrict__ slot_off,
                                                   const uint16_t *__restrict__ slot_src, const u64 *__restrict__ Cc,
                                                   const u64 *__restrict__ Gc, const u64 *__restrict__ Ec,
                                                   u64 *__restrict__ qcount, u64 *__restrict__ qdigest,
                                                   u64 *__restrict__ qedges) {
  const int b = blockIdx.x, qi = qidx ? qidx[b] : b;
  ms_emit_query(a, a.q[qi], st[qi], slot_off, slot_src, Cc, Gc, Ec, b, qcount, qdigest, qedges);
}

// ---------------------------------------------------------------------------
// PAPER delivery (Alg. 3 line 54: a pop delivers its cone minus everything
// delivered before it).  The delivered set is downward closed, so every vertex
// goes to the FIRST pop whose cone holds it; only the first pop
// of each distinct leader delivers.  Per round r, one wave walks the distinct
// queries in first-pop order: base_q(r) = K_r for r <= cut_q, the query's own
// mask row for lo_q <= r <= top_q, else nothing; delivered = base & P & ~D,
// D |= base.  Pass 1 counts (and sums degrees), a per-query scan gives
// positions, pass 2 the order-sensitive digests.
// ---------------------------------------------------------------------------
struct MPaper {
  int32_t top, cut, lo, pad;
  int64_t mask_off;
};

__device__ __forceinline__ u64 paper_base(const MArgs &a, const MPaper &x, int r, u64 kr, int lane) {
  if (r <= x.cut) return kr;
  if (r < x.lo || r > x.top || lane >= a.W) return 0ULL;
  return a.masks[x.mask_off + (int64_t)(x.top - r) * a.W + lane];
}

template <bool DIGEST>
__global__ __launch_bounds__(MS_NT) void k_ms_paper(MArgs a, int rmax, const MPaper *__restrict__ qp, int m,
                                                    uint32_t *__restrict__ cnt, int rstride,
                                                    const uint32_t *__restrict__ slot_off,
                                                    const uint16_t *__restrict__ slot_src, u64 *__restrict__ qedges,
                                                    u64 *__restrict__ qdigest) {
  const int r = 1 + blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r > rmax) return;
  const u64 p = lane < a.W ? a.pres[(size_t)r * a.W + lane] : 0ULL;
  const u64 kr = lane < a.W ? a.K[(size_t)r * a.W + lane] : 0ULL;
  u64 D = 0;
  for (int i = 0; i < m; i++) {
    const MPaper x = qp[i];
    if (r > x.top) continue;  // wave-uniform
    const u64 base = paper_base(a, x, r, kr, lane) & p;
    const u64 dl = base & ~D;
    D |= base;
    if (__ballot(dl != 0ULL) == 0ULL) continue;
    if constexpr (!DIGEST) {
      const u64 c = dr::wave_sum((u64)__popcll(dl));
      u64 acc = 0;
      for (u64 y = dl; y; y &= y - 1) {
        const size_t at = (size_t)r * a.n + lane * 64 + __builtin_ctzll(y);
        acc += (u64)a.sdeg[at] + a.wdeg[at];
      }
      acc = dr::wave_sum(acc);
      if (lane == 0) {
        cnt[(size_t)i * rstride + r] = (uint32_t)c;
        atomicAdd(&qedges[i], acc);
      }
    } else {
      u64 dg = 0, ed = 0;
      ms_wave_emit(slot_off, slot_src, r, dl, cnt[(size_t)i * rstride + r], a.W, nullptr, nullptr, a.n, dg, ed);
      dg = dr::wave_sum(dg);
      if (lane == 0 && dg) atomicAdd(&qdigest[i], dg);
    }
  }
}

// per query: counts over rounds 1..rmax -> exclusive positions in place; total
__global__ __launch_bounds__(MS_NT) void k_ms_paper_scan(int rmax, uint32_t *__restrict__ cnt, int rstride,
                                                         u64 *__restrict__ qcount) {
  __shared__ u64 part[MS_NT];
  const int i = blockIdx.x, tid = threadIdx.x;
  uint32_t *c = cnt + (size_t)i * rstride;
  const int span = rmax, per = (span + MS_NT - 1) / MS_NT;
  const int a0 = 1 + tid * per, a1 = min(rmax + 1, a0 + per);
  u64 s = 0;
  for (int r = a0; r < a1; r++) s += c[r];
  part[tid] = s;
  __syncthreads();
  if (tid == 0) {
    u64 run = 0;
    for (int t = 0; t < MS_NT; t++) {
      const u64 v = part[t];
      part[t] = run;
      run += v;
    }
    qcount[i] = run;
  }
  __syncthreads();
  u64 run = part[tid];
  for (int r = a0; r < a1; r++) {
    const uint32_t v = c[r];
    c[r] = (uint32_t)run;
    run += v;
  }
}

}  // namespace drs
