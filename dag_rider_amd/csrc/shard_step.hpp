// shard_step.hpp -- the stepped form of the column-sharded memoized replay
// (dr_shard_replay, include/dagrider_shard.h): what every rank of an
// RCCL group of G > 1 runs, and what a local-mode context runs with
// DR_SHARD_OPT_STEPPED so one device can check it.
//
// A rank holds only its columns of the strong rows and weak edges, so every round
// of every query needs the other ranks' columns of its next frontier: one exchange
// (all-gather) per round.  The host enqueues the whole replay with no round trip:
//
//   k_ms_lcol       (after an append or a coin change only) the vote's S_1 per
//                   wave: the sources of round 4w-2 whose row holds the leader's
//                   bit -- the rank that stores the leader's column finds it, the
//                   others write zeros, one exchange.  Derived DAG metadata like
//                   the degrees; it makes S_1 known on every rank.
//   k_ms_wu, k_ms_pass (VOTE_STEP2)   one read of the rank's columns of every
//                   strong row: U per round and, from the replicated S_1, this
//                   rank's partial S_2 (process.go:326-339) -> exchange.
//   k_ms_pass (VOTE_STEP3)   round 4w's rows against S_2 only: partial S_3,
//                   exchanged together with K^cand (k_ms_kcand) in RCCL mode.
//   k_ms_kfin       K (= K^cand), good_r, the full-round defaults of RD / CE, the
//                   vote count and commit of every wave, the walk's query and state.
//   k_ms_step2 x s  the canonical walk (one query), one round per launch.
//   k_ms_cpos       the canonical positions C over the walked rounds, the E
//                   prefix, and the leader chains planned on the device from the
//                   commit flags (the pop queries are a cached table).
//   k_ms_rg_full, k_ms_gprefix   the canonical digests and their prefix G.
//   k_ms_step2 x s  every pop and chain, one round per launch.
//   k_ms_emit       REF emission; one copy back, one host sync.
//
// Tried and not kept (profiles/r05/): the third vote step on a second stream beside
// the canonical walk (the walk's one-workgroup launches queued behind its
// workgroups: summary phase 0.062 -> 0.146 ms at G = 1), and each REF pop emitting
// in the step where it ends (every such step grew by the slowest emission: deliver
// + emit 0.101 -> 0.122 ms); 64 threads per query (0.43 -> 0.51 ms).
//
// k_ms_step2 is one workgroup per query (every local shard's columns in the same
// workgroup): the query's pending ring of rounds below lives in LDS during the
// launch and in global memory between launches, its state is read and written in
// place, and a finished query's workgroup exits at once.  The number of launches
// s is what the same replay took last time; the final states come back with the
// results, and the host steps on only if one was still live (the DAG changed).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "shard_fused.hpp"
#include "wave_ops.hpp"

namespace drs {

// S_1 of every wave w whose round 4w-2 is mirrored (partial: this context's shard
// holds the leader's column, else zeros).  One wave per wave index, lane = source
// word; out [nwl][W].
__global__ __launch_bounds__(256) void k_ms_lcol(MArgs a, int nwl, u64 *__restrict__ out) {
  const int wi = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (wi >= nwl) return;
  const int w = wi + 1, r = 4 * w - 2, L = (w < a.nlead ? (int)a.lead[w] : 1) - 1;
  const int gl = (L >> 6) / a.WSs, l = gl - a.shard0, cw = (L >> 6) - gl * a.WSs;
  const bool mine = l >= 0 && l < a.nlocal && r <= a.T;
  const u64 *rows = a.strong + (size_t)r * a.strong_rstride + (size_t)(mine ? l : 0) * a.strong_stride + cw;
  for (int w0 = 0; w0 < a.W; w0++) {  // 64 sources per pass, one per lane
    const int s = w0 * 64 + lane;
    const bool hit = mine && s < a.n && ((rows[(size_t)s * a.SP] >> (L & 63)) & 1ULL);
    const u64 b = __ballot(hit);
    if (lane == 0) out[(size_t)wi * a.W + w0] = b;
  }
}

// Local-mode K^cand over every local shard (kcand_round), good_r, the RD / CE
// defaults; RCCL mode: the same from the all-gathered K^cand columns (krecv:
// [G][kstride], each rank's [(T+1) * WSs] K^cand words then its [nw * W] partial
// S_3).  Extra workgroups: vcount / commit of every wave from the S_3 partials (P3:
// [Gp][nw][W] in local mode, inside krecv in RCCL mode; -1 / no commit where the
// leader is absent, process.go:327-329); block 0 also writes the canonical walk's
// query and initial state.
__global__ __launch_bounds__(256) void k_ms_kfin(MArgs a, FArgs f, const u64 *__restrict__ krecv, int64_t kstride,
                                                 const u64 *__restrict__ P3, int Gp, MQuery *__restrict__ cq,
                                                 MState *__restrict__ cst) {
  const int rb = (a.T + 1 + 3) / 4, lane = threadIdx.x & 63;
  if ((int)blockIdx.x < rb) {
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      MQuery q{};
      q.type = MQ_CANON;
      q.top = a.T;
      q.bottom = 0;
      q.src0 = -1;
      *cq = q;
      MState s{};
      s.cur = a.T;
      s.fresh = 1;
      s.stop = a.T + 1;  // lowest round a segment stopped at (T + 1: none)
      *cst = s;
    }
    if (!krecv) {
      kcand_round(a, f, r);
      return;
    }
    if (r > a.T) return;
    bool bad = false;
    int cnt = 0;
    if (lane < a.W) {
      const u64 p = a.pres[(size_t)r * a.W + lane];
      const int g = lane / a.WSs, cw = lane - g * a.WSs;
      const u64 v = krecv[(size_t)g * kstride + (size_t)r * a.WSs + cw];
      a.K[(size_t)r * a.W + lane] = v;
      bad = (v & p) != p;
      cnt = __popcll(v & p);
    }
    const bool ok = __ballot(bad) == 0ULL;
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
    if (lane == 0) {
      f.good[r] = ok;
      f.RD[r] = r == 0 ? 0 : (u64)cnt;
      f.CE[r] = r == 0 ? 0 : a.rdeg[r];
    }
    return;
  }
  const int wi = (blockIdx.x - rb) * 4 + (threadIdx.x >> 6);
  if (wi >= f.nw) return;
  const int w = wi + 1, r1 = 4 * wi + 1, L = (w < a.nlead ? (int)a.lead[w] : 1) - 1;
  const bool has = (a.pres[(size_t)r1 * a.W + (L >> 6)] >> (L & 63)) & 1ULL;
  u64 v = 0;
  if (lane < a.W) {
    if (krecv) {
      for (int g = 0; g < a.G; g++) v |= krecv[(size_t)g * kstride + (size_t)(a.T + 1) * a.WSs + (size_t)wi * a.W + lane];
    } else {
      for (int g = 0; g < Gp; g++) v |= P3[((size_t)g * f.nw + wi) * a.W + lane];
    }
  }
  const int c = (int)dr::wave_sum((u64)__popcll(v));
  if (lane == 0) {
    f.vcount[wi] = has ? c : -1;
    f.commit[wi] = has && c >= f.quorum ? 1 : 0;
  }
}

// After the stepped walk (one workgroup): the canonical positions C (B = its lowest
// stop round), the E prefix (CE is final), and the chain tasks of the batch from the
// commit flags (plan_body; the pop queries are the context's cached table and start
// from their initial state in the first step).
template <int NT>
__global__ __launch_bounds__(NT) void k_ms_cpos(MArgs a, FArgs f, const MState *__restrict__ cst,
                                                MQuery *__restrict__ q, int push_cap) {
  __shared__ u64 part[2 * NT / 64];
  const MState S = *cst;
  canon_positions<NT>(a, f, min(S.stop, a.T + 1), S.npush);
  ms_prefix_two<NT>(a.T + 1, f.CE, f.Ec, nullptr, nullptr, part);
  plan_body<NT>(a, f, q, push_cap, 0);
}

// the G prefix of the canonical digests (one workgroup; RG is final)
template <int NT>
__global__ __launch_bounds__(NT) void k_ms_gprefix(MArgs a, FArgs f) {
  __shared__ u64 part[2 * NT / 64];
  ms_prefix_two<NT>(a.T + 1, f.RG, f.Gc, nullptr, nullptr, part);
}

// Partial round r of one query (every local shard's columns): the frontier FE's
// strong rows into ring slot r-1, and (weak) its weak columns into the slots of
// their target rounds >= bottom.  ring: LDS, WL = nlocal * WSs LOCAL words per slot
// (word l * WSs + c = column word c of local shard l).  Saturation as in the fused
// sweep: once the OR of the rows a wave has read equals U_r on its words, no
// further row adds a bit.  Every thread calls it.
// strong = false: the rows are done (wave 0 saturated on the first word, k_ms_step2).
template <int NT>
__device__ __forceinline__ void expand_partial_local(const MArgs &a, int r, int bottom, const u64 *FE, u64 *ring, int WL,
                                                     int dm, bool weak, bool strong) {
  constexpr int NW = NT / 64;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int SP = a.SP, W = a.W, WSs = a.WSs, NL = a.nlocal, WP = NL * SP;
  u64 *dst = ring + (size_t)((r - 1) & dm) * WL;
  if (!strong) {
  } else if (WP <= 64 && (64 % WP) == 0) {
    const int l0 = (lane % WP) / SP, c0 = lane % SP;  // this lane's word of the concatenated row
    const u64 *base = a.strong + (size_t)r * a.strong_rstride + (size_t)l0 * a.strong_stride + c0;
    const u64 ur = lane < WP ? a.U[((size_t)l0 * a.R + r) * SP + c0] : 0ULL;
    const int RPL = 64 / WP;  // rows per load instruction
    u64 acc = 0;
    for (int w = wv; w < W; w += NW) {
      const u64 bits = FE[w];
      if (!bits) continue;
      const int rb = w * 64;
      for (int i = 0; i < WP; i++) {
        const int row = i * RPL + lane / WP;
        if ((bits >> row) & 1ULL) acc |= base[(size_t)(rb + row) * SP];
      }
      u64 red = acc;
      for (int off = WP; off < 64; off <<= 1) red |= shfl_xor64(red, off);
      if (__ballot(lane < WP && red != ur) == 0ULL) break;
    }
    for (int off = WP; off < 64; off <<= 1) acc |= shfl_xor64(acc, off);
    if (lane < WP && c0 < WSs && acc) atomicOr(&dst[l0 * WSs + c0], acc);
  } else {
    for (int l = 0; l < NL; l++) {
      const u64 *rows = a.strong + (size_t)r * a.strong_rstride + (size_t)l * a.strong_stride;
      const u64 ur = lane < SP ? a.U[((size_t)l * a.R + r) * SP + lane] : 0ULL;
      u64 acc = 0;
      for (int w = wv; w < W; w += NW) {
        const u64 bits = FE[w];
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
      if (lane < SP && lane < WSs && acc) atomicOr(&dst[l * WSs + lane], acc);
    }
  }
  if (!weak) return;
  // the frontier's nonzero words: a column's source words are read only there (a query's
  // first step has one source, one word of W)
  u64 fm = 0;
  for (int w = 0; w < W; w++) fm |= FE[w] ? 1ULL << w : 0ULL;
  const bool per_wave = NL >= NW;
  for (int l = per_wave ? wv : 0; l < NL; l += per_wave ? NW : 1) {
    const uint64_t c0 = a.wcro[(size_t)l * (a.R + 1) + r], c1 = a.wcro[(size_t)l * (a.R + 1) + r + 1];
    for (uint64_t jj = c0 + (per_wave ? lane : tid); jj < c1; jj += per_wave ? 64 : NT) {
      const u64 *row = a.wcr + jj * W;
      const uint32_t key = a.wck[jj];
      u64 hit = 0;
      for (u64 m = fm; m; m &= m - 1) {
        const int w = __builtin_ctzll(m);
        hit |= row[w] & FE[w];
      }
      if (!hit) continue;
      const int tr = r - (int)(key >> 11), cb = l * WSs * 64 + (int)(key & 2047u);  // local bit
      if (tr < bottom) continue;
      atomicOr(&ring[(size_t)(tr & dm) * WL + (cb >> 6)], 1ULL << (cb & 63));
    }
  }
}

// One round of one query per launch (see the file comment).  Grid: one workgroup
// per query.  st: the queries' states, read and written in place (a query's state
// belongs to its workgroup).  rin: [G][nq][WSs] the exchanged frontier columns of
// this step's rounds; rout: local mode the same layout for the next step (this
// context's shards), RCCL mode [nq][WSs] (the send buffer).  Dynamic LDS:
// ring[depth][WL] | FE[W].
// batch: the pops and chains (their first step starts them from their query; chain
// slots past the planned chains end there), else the canonical walk.
template <int NT>
__global__ __launch_bounds__(NT) void k_ms_step2(MArgs a, FArgs f, int j, MState *__restrict__ st,
                                                 const u64 *__restrict__ rin, u64 *__restrict__ rout, int batch) {
  extern __shared__ __attribute__((aligned(16))) u64 lds[];
  const int qi = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const MQuery Q = a.q[qi];
  MState S = st[qi];
  if (batch && j == 0) {
    if (qi >= f.npop + f.hdr[FH_NCHAIN]) {  // an unused chain slot
      if (tid == 0) {
        MState d{};
        d.done = 1;
        st[qi] = d;
      }
      return;
    }
    S = MState{};
    S.low = Q.top;
    S.cur = Q.top;
  }
  if (S.done) return;
  const int W = a.W, WSs = a.WSs, WL = a.nlocal * WSs, dm = a.depth - 1, D = a.depth, SP = a.SP;
  u64 *ring = lds, *FE = lds + (size_t)D * WL;
  __shared__ int s_ctl[3];
  __shared__ u64 s_e;
  __shared__ MState s_st;
  __shared__ u64 sAcc[64];  // wave 0's rows of the first frontier word, local words of slot r-1
  u64 *gring = a.pend + (size_t)qi * D * WL;
  const bool pop = Q.type == MQ_POP, chain = Q.type == MQ_CHAIN, canon = Q.type == MQ_CANON;
  int r = canon ? S.cur : Q.top - j;
  bool start = false;
  MState S1 = S;
  S1.steps = S.steps + 1;
  // wave 0's words of round r go out before the ring copy below (which waits for its own
  // loads before it writes LDS), unless a canonical segment starts (its round is found first)
  const bool early = !(canon && S.fresh);
  u64 e_fw = 0, e_p = 0, e_k = 0;
  if (early && wv == 0 && lane < a.W) {
    if (j == 0 && !canon) e_fw = (Q.src0 >= 0 && lane == (Q.src0 >> 6)) ? 1ULL << (Q.src0 & 63) : 0ULL;
    else e_fw = rin[((size_t)(lane / a.WSs) * a.nq + qi) * a.WSs + lane % a.WSs];
    e_p = a.pres[(size_t)r * a.W + lane];
    if (pop) e_k = a.K[(size_t)r * a.W + lane];
  }
  if (canon && S.fresh) {
    // the next canonical segment: the highest bad round below cur; its ring starts
    // with what the full rounds above it put below it (canon_ring_init)
    if (wv == 0) {
      const int b = next_bad(a, S.cur);
      if (lane == 0) s_ctl[0] = b;
    }
    for (int i = tid; i < D * WL; i += NT) ring[i] = 0;
    __syncthreads();
    const int b = s_ctl[0];
    if (b < 0) {
      if (tid == 0) {
        S1.done = 1;
        S1.fresh = 0;
        st[qi] = S1;
      }
      return;
    }
    if (tid < WL) {
      const int l = tid / WSs, cw = tid - l * WSs;
      const size_t ub = (size_t)l * a.R;
      for (int x = b - 1; x >= 0 && x >= b - a.dd; x--) {
        u64 v = 0;
        for (int y = max(b + 1, x + 2); y <= a.T && y <= x + a.dd + 1; y++)
          v |= a.WU[((ub + y) * a.dd + (y - x - 2)) * SP + cw];
        ring[(size_t)(x & dm) * WL + tid] = v;
      }
    }
    r = b;
    start = true;
    S1.run = 0;
    S1.low = b;
    S1.npush = S.npush + 1;
    S1.fresh = 0;
  } else if (j == 0 && !canon) {
    for (int i = tid; i < D * WL; i += NT) ring[i] = 0;
  } else {
    for (int i = tid; i < D * WL; i += NT) ring[i] = gring[i];
  }
  if (wv == 0) {
    const bool act = lane < W;
    u64 fw = 0, p = 0, k = 0;
    if (act) {
      if (start) {
        fw = a.K[(size_t)r * W + lane];
        p = a.pres[(size_t)r * W + lane];
      } else {
        fw = e_fw;
        p = e_p;
        k = e_k;
      }
    }
    // waveReady's chain (process.go:342-350): a reachable, present leader of wave
    // wvv is pushed and the chain goes on from it alone
    bool restart = false;
    int wvv = 0;
    if (chain && r < Q.top && ((r - 1) & 3) == 0) {
      wvv = ((r - 1) >> 2) + 1;
      const int L = (wvv < a.nlead ? (int)a.lead[wvv] : 1) - 1;
      const u64 fl = __shfl(fw & p, L >> 6);
      if ((fl >> (L & 63)) & 1ULL) {
        fw = lane == (L >> 6) ? 1ULL << (L & 63) : 0ULL;
        restart = true;
      }
    }
    const u64 fe = fw & p;
    const bool nz = __ballot(act && fw != 0ULL) != 0ULL;
    const bool anyfe = __ballot(act && fe != 0ULL) != 0ULL;
    const bool full = __ballot(act && fe != p) == 0ULL;
    int run = S1.run, low = S1.low;
    if (nz) low = min(low, r - 1);
    bool merged = false, done;
    if (pop) {
      run = __ballot(act && fw != k) == 0ULL ? run + 1 : 0;
      merged = run >= a.dmax;
      done = merged || r <= Q.bottom || (!nz && low >= r);
    } else if (chain) {
      done = r <= Q.bottom || (!nz && low >= r);
    } else {  // the canonical segment ends where dmax full rounds restore the regime
      run = full ? run + 1 : 0;
      done = run >= a.dmax || r == 0;
    }
    if (act) {
      if (pop) a.masks[Q.mask_off + (int64_t)j * W + lane] = fw;
      else if (canon) a.K[(size_t)r * W + lane] = fw;
    }
    if (canon) {  // RD_r of a walked round (CE_r of a partial one: below)
      int cnt = __popcll(fe);
      for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
      if (lane == 0) f.RD[r] = r == 0 ? 0 : (u64)cnt;
    }
    const bool summary = !done && full;
    // A partial round's rows, first frontier word, by wave 0 alone: in a quorum DAG the
    // OR of 64 rows is already U_r, the OR of every row of the round (saturation), and
    // the other waves then read no row at all (they would each read a word of their own)
    const int WP = a.nlocal * SP;
    int sat = 0;
    if (lane < WL) sAcc[lane] = 0;
    if (!done && !summary && anyfe && WP <= 64 && (64 % WP) == 0) {
      const int l0 = (lane % WP) / SP, c0 = lane % SP, RPL = 64 / WP;
      const u64 *base = a.strong + (size_t)r * a.strong_rstride + (size_t)l0 * a.strong_stride + c0;
      const u64 ur = lane < WP ? a.U[((size_t)l0 * a.R + r) * SP + c0] : 0ULL;
      const int w0 = __ffsll((long long)__ballot(act && fe != 0ULL)) - 1;
      const u64 bits = dr::shfl64(fe, w0);
      u64 acc = 0;
      for (int i = 0; i < WP; i++) {
        const int row = i * RPL + lane / WP;
        if ((bits >> row) & 1ULL) acc |= base[(size_t)(w0 * 64 + row) * SP];
      }
      for (int off = WP; off < 64; off <<= 1) acc |= shfl_xor64(acc, off);
      sat = __ballot(lane < WP && acc != ur) == 0ULL;
      if (lane < WP && c0 < WSs) sAcc[l0 * WSs + c0] = acc;
    }
    u64 edges = S.edges;
    if (chain && summary) edges += a.sdr[r];
    if (!done && !chain && anyfe) low = min(low, r - a.dmax);
    if (act) FE[lane] = fe;
    if (lane == 0) {
      MState o = S1;
      o.done = done;
      o.run = run;
      o.low = low;
      o.stop = done ? r : 0;
      o.merged = merged;
      o.npush = S1.npush + (restart ? 1 : 0);
      o.edges = edges;
      if (canon) {  // a finished segment: look for the next one below r
        o.done = 0;
        o.fresh = done ? 1 : 0;
        o.cur = done ? r : r - 1;
        o.stop = done ? r : S1.stop;
      }
      if (restart) a.push_out[Q.push_base + S1.npush] = wvv;
      s_st = o;
      s_ctl[0] = done;
      s_ctl[1] = summary;
      s_ctl[2] = sat;
      s_e = 0;
    }
  }
  __syncthreads();
  if (s_ctl[0]) {
    if (tid == 0) st[qi] = s_st;
    return;
  }
  const bool weak = !chain;
  if (s_ctl[1]) {  // full round: ring[r-1] |= U_r, ring[r-d-2] |= WU_r[d] (distinct slots)
    const int terms = weak ? 1 + a.dd : 1;
    for (int i = tid; i < WL * terms; i += NT) {
      const int lw = i % WL, d = i / WL - 1, l = lw / WSs, cw = lw - l * WSs;
      const size_t ub = (size_t)l * a.R + r;
      if (d < 0) {
        ring[(size_t)((r - 1) & dm) * WL + lw] |= a.U[ub * SP + cw];
      } else {
        const int tr = r - d - 2;
        if (tr >= Q.bottom) ring[(size_t)(tr & dm) * WL + lw] |= a.WU[(ub * a.dd + d) * SP + cw];
      }
    }
  } else {
    // degrees of the partial round's frontier (chains: strong, the edges followed;
    // the canonical walk: strong + weak, CE_r), loaded before the rows
    if (!pop) {
      u64 e = 0;
      for (int s = tid; s < a.n; s += NT)
        if ((FE[s >> 6] >> (s & 63)) & 1ULL) {
          const size_t at = (size_t)r * a.n + s;
          e += a.sdeg[at] + (canon ? a.wdeg[at] : 0);
        }
      e = dr::wave_sum(e);
      if (lane == 0 && e) atomicAdd(&s_e, e);
    }
    expand_partial_local<NT>(a, r, Q.bottom, FE, ring, WL, dm, weak, !s_ctl[2]);
  }
  __syncthreads();
  // the ring goes back to global memory; slot r-1 (complete: every contribution
  // from the rounds above is in) leaves it for the exchange
  const int so = ((r - 1) & dm) * WL;
  for (int i = tid; i < D * WL; i += NT) {
    u64 v = ring[i];
    if (i >= so && i < so + WL) {
      const int lw = i - so, l = lw / WSs, cw = lw - l * WSs;
      v |= sAcc[lw];
      if (a.local) rout[((size_t)(a.shard0 + l) * a.nq + qi) * WSs + cw] = v;
      else rout[(size_t)qi * WSs + cw] = v;
      gring[i] = 0;
    } else {
      gring[i] = v;
    }
  }
  if (tid == 0) {
    MState o = s_st;
    if (chain) o.edges += s_e;
    if (canon && !s_ctl[1]) f.CE[r] = s_e;  // a partial walked round (full ones keep the round total)
    st[qi] = o;
  }
}

}  // namespace drs
