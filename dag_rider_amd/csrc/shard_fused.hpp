// shard_fused.hpp -- kernels of the column-sharded memoized replay
// (dr_shard_replay, include/dagrider_shard.h) that read every
// column a context holds in one workgroup.
//
//   k_ms_wu          one workgroup per round: WU_r (from the weak-column keys)
//                    and the round's speculative canonical digest.
//   k_ms_pass        one workgroup per wave (rounds 4w-3 .. 4w): streams every
//                    local shard's columns of the wave's strong rows once and
//                    builds, from that one read, U_r (per shard) and waveReady's
//                    vote (process.go:326-339).  When the
//                    context holds every column (local mode, a one-rank group:
//                    "fused") the vote is complete: S_1..S_3, vcount, commit.
//                    Otherwise (one rank of G > 1) the pass writes this shard's
//                    partial S_1 for the exchange; steps 2 and 3 follow the
//                    exchanges (shard.hip k_shard_vote).
//   k_ms_kcand_full  K^cand_r, good_r and the full-round defaults of RD, CE.
//   k_ms_canon_full  one workgroup walks the canonical segments below the bad
//                    rounds (k_canon's walk, kernels.hpp) over the shard arrays,
//                    then the canonical positions C (the presence prefix below
//                    the lowest walked round) and the lowest round whose
//                    speculative digest is stale.
//   k_ms_rg_full     per-round canonical digests (speculative below that round).
//   k_ms_prefix_plan the G, E prefixes and waveReady's chain tasks from the device
//                    commit flags (persistent decidedWave: the previous commit;
//                    literal: 0), plan_body.
//   k_ms_sweep_full  one workgroup per query (orderVertices cone / leader chain),
//                    round by round to its end: no exchange is needed when the
//                    workgroup sees every column, so a query never waits for the
//                    others (the stepped form, shard_memo.hpp k_ms_step, moves one
//                    round per launch with an exchange between launches).
//
// Semantics are dr_replay's (engine.hip): the same commits, pushes, per-pop
// counts, digests and edge totals, bit for bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "shard_memo.hpp"
#include "wave_ops.hpp"

namespace drs {

#ifdef DR_SWEEP_TIMING
// profiling build only (libdagrider_gpu_timing.so, tools/ms_timing.py): per
// query of k_ms_sweep_full, wall-clock ticks at start / end, rounds wave 0
// applied alone, workgroup rounds, ticks inside workgroup rounds, type, top, stop
constexpr int kMsTimingQ = 8192;
__device__ u64 g_ms_timing[8 * kMsTimingQ];
#define DR_MT(...) __VA_ARGS__
#else
#define DR_MT(...)
#endif

// k_ms_pass vote modes: VOTE_FULL every step of the vote (the context holds every
// column); VOTE_STEP2 this context's partial S_2 from the replicated S_1 (one rank
// of G > 1, or the stepped form on one device); VOTE_STEP3 round 4w's rows only,
// against S_2: the partial S_3
enum : int { VOTE_FULL = 1, VOTE_STEP2 = 2, VOTE_STEP3 = 3 };

// extra inputs/outputs of the fused replay (every pointer device memory)
struct FArgs {
  const u64 *ppref;    // [R] |P_1| + .. + |P_r| (present vertices, round 0 excluded)
  u64 *SG;             // [T+1] speculative canonical digest (every round 1..r full)
  u64 *RD, *CE, *RG;   // [T+1] canonical count, edges, digest of each round
  u64 *Cc, *Ec, *Gc;   // [T+1] their prefixes
  uint8_t *good;       // [T+8] K^cand_r covers P_r
  int32_t *hdr;        // FH_* slots
  uint8_t *commit;     // [nw]
  int32_t *vcount;     // [nw]
  MState *fin;         // [nq] final state of every query
  u64 *qcount, *qdigest, *qedges;  // [npop] REF emission of each pop (k_ms_sweep_full with emit)
  int32_t quorum, nw, npop, persistent, emit;
  int32_t keep4;  // VOTE_STEP2: round 4w's rows with cached loads (read again by VOTE_STEP3; tuning)
};
enum : int { FH_NCHAIN = 0, FH_NSEG = 1, FH_RLO = 2, FH_PUSHES = 3, FH_ERR = 4, FH_N = 8 };

// exclusive scan of v over one workgroup of NT threads (every thread calls it);
// s: NT/64 slots of LDS; op: 0 sum, 1 max
template <int NT>
__device__ __forceinline__ int64_t fblock_scan(int64_t v, int64_t *s, int64_t &total, int op) {
  constexpr int NW = NT / 64;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int64_t x = v;
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t y = (int64_t)__shfl_up((long long)x, off);
    if (lane >= off) x = op ? max(x, y) : x + y;
  }
  if (lane == 63) s[wid] = x;
  __syncthreads();
  int64_t base = 0, tot = 0;
  for (int w = 0; w < NW; w++) {
    const int64_t t = s[w];
    if (w < wid) base = op ? max(base, t) : base + t;
    tot = op ? max(tot, t) : tot + t;
  }
  __syncthreads();
  total = tot;
  const int64_t ex = (int64_t)__shfl_up((long long)x, 1);
  const int64_t lex = lane == 0 ? 0 : ex;
  return op ? max(base, lex) : base + lex;
}

// ---------------------------------------------------------------------------
// k_ms_wu: one wave per round r >= 1 (NT/64 rounds per workgroup): WU_r of every
// local shard from the round's weak-column keys (LDS atomics, then every word
// written, zeros included), and the speculative canonical digest SG_r (every
// present vertex of the round delivered in slot order at positions from
// ppref[r-1]).  Dynamic LDS: sWU[NT/64][NL*dd*SP].  It reads no strong row, so it is kept out of
// k_ms_pass, whose row stream it would stall at every round.
// ---------------------------------------------------------------------------
template <int NT>
__global__ __launch_bounds__(NT) void k_ms_wu(MArgs a, FArgs f, u64 *__restrict__ WU) {
  extern __shared__ __attribute__((aligned(16))) u64 lds[];
  constexpr int NW = NT / 64;
  const int NL = a.nlocal, SP = a.SP, dd = a.dd, words = NL * dd * SP;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, r = blockIdx.x * NW + wid + 1;
  u64 *sWU = lds + (size_t)wid * words;  // this wave's round
  for (int i = lane; i < words; i += 64) sWU[i] = 0;
  if (r > a.T) return;  // (wave-uniform; no workgroup barrier below)
  for (int l = 0; l < NL; l++) {  // every key has a source
    const uint64_t c0 = a.wcro[(size_t)l * (a.R + 1) + r], c1 = a.wcro[(size_t)l * (a.R + 1) + r + 1];
    for (uint64_t jj = c0 + lane; jj < c1; jj += 64) {
      const uint32_t key = a.wck[jj];
      const int d = (int)(key >> 11) - 2, tc = (int)(key & 2047u);
      atomicOr(&sWU[((size_t)l * dd + d) * SP + (tc >> 6)], 1ULL << (tc & 63));
    }
  }
  {  // speculative canonical digest of round r
    constexpr int SPT = 8;
    const uint32_t sa = a.slot_off[r], sb = a.slot_off[r + 1];
    u64 pos = f.ppref[r - 1], dg = 0;
    for (uint32_t c0 = sa; c0 < sb; c0 += 64 * SPT) {
      const uint32_t i0 = c0 + (uint32_t)lane * SPT;
      uint32_t src[SPT];
      uint32_t cnt = 0;
#pragma unroll
      for (int q = 0; q < SPT; q++) {
        src[q] = i0 + q < sb ? a.slot_src[i0 + q] : 0u;
        cnt += src[q] != 0;
      }
      uint32_t inc = cnt;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(inc, off);
        if (lane >= off) inc += y;
      }
      u64 k = pos + (inc - cnt);
#pragma unroll
      for (int q = 0; q < SPT; q++)
        if (src[q]) dg += dr::digest_term((uint32_t)r, src[q], k++);
      pos += __shfl(inc, 63);
    }
    dg = dr::wave_sum(dg);
    if (lane == 0) f.SG[r] = dg;
  }
  for (int i = lane; i < words; i += 64) {  // (LDS ops of one wave complete in order)
    const int l = i / (dd * SP), rest = i - l * dd * SP;
    WU[((size_t)l * a.R + r) * dd * SP + rest] = sWU[i];
  }
}

// ---------------------------------------------------------------------------
// k_ms_pass (see the file comment).  Dynamic LDS: sU[NL*SP] | Sp[NL*SP] |
// Tn[W].  SP (the row stride) is a template parameter, so the
// chunk geometry is static: thread t owns 16-B chunk column j = t mod CPR of
// rows t / CPR + p * RPP of every local shard, and its OR accumulator holds that
// column.  A round is NL * CPT (shard, pass) elements per thread, loaded GR at a
// time (nontemporal: each row is read once); a shard's U column is reduced when
// its last pass is consumed (the pass index is uniform over the workgroup).
// ---------------------------------------------------------------------------
// ONE: the context holds one shard (G = 1 fused, or one rank of an RCCL group):
// the element index is the pass, and the S chunk a thread tests is read once per
// round.
// Sin (VOTE_STEP2 / 3): the set the tested round is checked against, Gin slots of
// [sin_nw][W] OR-ed (the exchanged partials); Sout: this context's partial of the
// tested round's set, [nwc][W].
template <int SP, int NT, int GR, bool ONE>
__global__ __launch_bounds__(NT) void k_ms_pass(MArgs a, FArgs f, int nwc, int vote_mode, u64 *__restrict__ U,
                                                u64 *__restrict__ Sout, const u64 *__restrict__ Sin, int Gin,
                                                int sin_nw) {
  constexpr int CW = SP >= 2 ? 2 : 1, CPR = SP / CW, RPP = NT / CPR;
  static_assert(NT % 64 == 0 && NT % CPR == 0 && CPR <= 16, "block must tile rows");
  extern __shared__ __attribute__((aligned(16))) u64 lds[];
  const int NL = ONE ? 1 : a.nlocal, W = a.W, WSs = a.WSs, n = a.n, T = a.T;
  u64 *sU = lds, *Sp = lds + NL * SP, *Tn = Sp + NL * SP;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, j = tid % CPR, row0 = tid / CPR;
  const int w = blockIdx.x + 1, r1 = 4 * (w - 1) + 1;
  const int nr = min(T, r1 + 3) - r1 + 1;
  const bool do_commit = w <= nwc;
  const int L = do_commit ? (w < a.nlead ? (int)a.lead[w] : 1) - 1 : 0;
  const bool leader = do_commit && ((a.pres[(size_t)r1 * W + (L >> 6)] >> (L & 63)) & 1ULL);
  const int CPT = (n + RPP - 1) / RPP, E = NL * CPT;
  const int ktest = vote_mode == VOTE_STEP2 ? 2 : 3;  // the stepped modes test one round
  if (vote_mode == VOTE_STEP3 && !(leader && nr == 4)) {  // no vote: nothing to read
    if (do_commit)
      for (int i = tid; i < W; i += NT) Sout[(size_t)(w - 1) * W + i] = 0;
    return;
  }
  for (int i = tid; i < NL * SP; i += NT) {
    sU[i] = 0;
    const int l = i / SP, c = i % SP, gw = (a.shard0 + l) * WSs + c;
    u64 v = 0;
    if (vote_mode == VOTE_FULL) {
      v = (c < WSs && gw == (L >> 6)) ? 1ULL << (L & 63) : 0ULL;
    } else if (leader && c < WSs && gw < W) {
      for (int g = 0; g < Gin; g++) v |= Sin[((size_t)g * sin_nw + (w - 1)) * W + gw];
    }
    Sp[i] = v;
  }
  for (int i = tid; i < W; i += NT) Tn[i] = 0;
  __syncthreads();
  for (int k = vote_mode == VOTE_STEP3 ? 3 : 0; k < nr; k++) {
    const int r = r1 + k;
    const bool test = leader && (vote_mode == VOTE_FULL ? k >= 1 : k == ktest);
    const bool keep = f.keep4 && vote_mode == VOTE_STEP2 && k == 3;
    const u64 *rbase = a.strong + (size_t)r * a.strong_rstride + (size_t)row0 * SP + j * CW;
    u64 a0 = 0, a1 = 0;
    u64 t0 = 0, t1 = 0;  // ONE: this thread's chunk of S_{k-1}
    if (ONE && test) {
      t0 = Sp[j * CW];
      t1 = CW == 2 ? Sp[j * CW + 1] : 0ULL;
    }
    int lc = 0, pc = 0;  // (shard, pass) of element e0, carried from group to group
    for (int e0 = 0; e0 < E; e0 += GR) {
      u64 x0[GR], x1[GR];
      {
        int l = lc, p = pc;
#pragma unroll
        for (int q = 0; q < GR; q++) {
          x0[q] = 0;
          x1[q] = 0;
          const int s = row0 + p * RPP;
          if (e0 + q < E && s < n) {
            const u64 *src = rbase + (size_t)l * a.strong_stride + (size_t)p * RPP * SP;
            if constexpr (CW == 2) {
              const u64x2 v = keep ? *reinterpret_cast<const u64x2 *>(src)
                                   : __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(src));
              x0[q] = v.x;
              x1[q] = v.y;
            } else {
              x0[q] = keep ? *src : __builtin_nontemporal_load(src);
            }
          }
          if (++p == CPT) {
            p = 0;
            l++;
          }
        }
      }
      int l = lc, p = pc;
#pragma unroll
      for (int q = 0; q < GR; q++) {
        if (e0 + q >= E) break;  // uniform
        a0 |= x0[q];
        a1 |= x1[q];
        if (test) {  // rows of round r reaching S_{k-1} on this shard's columns
          const u64 s0 = ONE ? t0 : Sp[l * SP + j * CW], s1 = ONE ? t1 : (CW == 2 ? Sp[l * SP + j * CW + 1] : 0ULL);
          u64 m = __ballot(((x0[q] & s0) | (x1[q] & s1)) != 0ULL);
          const int rowbase = (wid * 64) / CPR + p * RPP;  // the wave's first row
          if (lane == 0 && m && rowbase < n) {
            u64 bits = m;
            if constexpr (CPR > 1) {
#pragma unroll
              for (int sh = 1; sh < CPR; sh <<= 1) m |= m >> sh;
              bits = 0;
#pragma unroll
              for (int gI = 0; gI < 64 / CPR; gI++) bits |= ((m >> (gI * CPR)) & 1ULL) << gI;
            }
            atomicOr(&Tn[rowbase >> 6], bits << (rowbase & 63));
          }
        }
        if (p == CPT - 1) {  // the shard's columns of round r are done: U
          if constexpr (CPR < 16) {
            a0 = dr::row_or_stride<CPR>(a0);
            if constexpr (CW == 2) a1 = dr::row_or_stride<CPR>(a1);
          }
          if ((lane & 15) < CPR) {
            if (a0) atomicOr(&sU[l * SP + (lane & 15) * CW], a0);
            if (CW == 2 && a1) atomicOr(&sU[l * SP + (lane & 15) * CW + 1], a1);
          }
          a0 = a1 = 0;
        }
        if (++p == CPT) {
          p = 0;
          l++;
        }
      }
      lc = l;
      pc = p;
    }
    __syncthreads();
    if (vote_mode != VOTE_STEP3)
      for (int i = tid; i < NL * SP; i += NT) {
        const int l = i / SP, c = i % SP;
        U[((size_t)l * a.R + r) * SP + c] = sU[i];
        sU[i] = 0;
      }
    if (test) {  // S_k: the sources of round r that reach S_{k-1} (this context's shards' columns of it)
      for (int i = tid; i < W; i += NT) {
        const u64 v = Tn[i];
        Tn[i] = 0;
        const int l = i / WSs - a.shard0, c = i % WSs;
        if (l >= 0 && l < NL) Sp[l * SP + c] = v;
        if (vote_mode != VOTE_FULL && Sout) Sout[(size_t)(w - 1) * W + i] = v;
      }
    }
    __syncthreads();
  }
  if (do_commit && vote_mode == VOTE_STEP2 && !(leader && nr >= 3) && Sout)
    for (int i = tid; i < W; i += NT) Sout[(size_t)(w - 1) * W + i] = 0;
  if (do_commit && vote_mode == VOTE_FULL && tid == 0) {
    if (!leader) {  // leader is bottom (process.go:327-329)
      f.commit[w - 1] = 0;
      f.vcount[w - 1] = -1;
    } else {
      int vc = 0;
      for (int i = 0; i < NL * SP; i++) vc += __popcll(Sp[i]);
      f.vcount[w - 1] = vc;
      f.commit[w - 1] = vc >= f.quorum ? 1 : 0;
    }
  }
}

// K^cand over the full width (every local shard's U / WU), good_r, and the
// full-round defaults RD_r = |K^cand_r & P_r|, CE_r = the round's degree sum.
// One wave per round, lane w < W owns word w (shard w / WSs, column w mod WSs).
__device__ __forceinline__ void kcand_round(const MArgs &a, const FArgs &f, int r) {
  const int w = threadIdx.x & 63, T = a.T;
  if (r > T) return;
  bool bad = false;
  int cnt = 0;
  if (w < a.W) {
    const int l = w / a.WSs, cw = w - l * a.WSs;
    const u64 p = a.pres[(size_t)r * a.W + w];
    u64 v;
    if (r == T) {
      v = p;
    } else {
      const size_t ub = (size_t)l * a.R;
      v = a.U[(ub + r + 1) * a.SP + cw];
      for (int d = 0; d < a.dd && r + d + 2 <= T; d++) v |= a.WU[((ub + r + d + 2) * a.dd + d) * a.SP + cw];
    }
    a.K[(size_t)r * a.W + w] = v;
    bad = (v & p) != p;
    cnt = __popcll(v & p);
  }
  const bool ok = __ballot(bad) == 0ULL;
  for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
  if (w == 0) {
    f.good[r] = ok;
    f.RD[r] = r == 0 ? 0 : (u64)cnt;
    f.CE[r] = r == 0 ? 0 : a.rdeg[r];
  }
}
__global__ __launch_bounds__(256) void k_ms_kcand_full(MArgs a, FArgs f) {
  kcand_round(a, f, blockIdx.x * 4 + (threadIdx.x >> 6));
}

// Full-width expansion of a partial round r of a query held by one workgroup:
// the frontier FE's strong rows (every local shard's columns) -> ring slot of
// r-1, and (weak) its weak columns -> the ring slots of their target rounds
// (>= bottom).  Saturation as in k_ms_step: once the OR of the rows a wave has
// read equals U_r, no further row adds a bit.  Every thread calls it; ring / FE
// are LDS (W words per round slot).
//
// The local shards' row pieces are read as one row of WP = nlocal * SP words:
// the 64 rows of frontier word w are 64 * WP words, lane k's i-th load is
// element k + 64 i (row (k + 64 i) / WP, word (k mod WP)), so with WP dividing
// 64 a lane always accumulates the same word of the concatenated row, whatever
// the shard count, and every load of a frontier word is issued before its
// saturation check.  Other shard counts take the per-shard loop.
template <int NT>
__device__ __forceinline__ void expand_partial_full(const MArgs &a, int r, int bottom, const u64 *FE, u64 *ring,
                                                    int dm, bool weak, const u64 *Ur = nullptr,
                                                    int64_t wc0 = -1, int64_t wc1 = -1) {
  constexpr int NW = NT / 64;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int SP = a.SP, W = a.W, WSs = a.WSs, NL = a.nlocal, WP = NL * SP;
  u64 *dst = ring + (size_t)((r - 1) & dm) * W;
  // one local shard: its weak-column range goes out with the U word and the rows
  // (the columns' loads then wait on one memory latency, not two)
  if (weak && NL == 1 && wc0 < 0) {
    wc0 = (int64_t)a.wcro[r];
    wc1 = (int64_t)a.wcro[r + 1];
  }
  if (WP <= 64 && (64 % WP) == 0) {
    const int l0 = (lane % WP) / SP, c0 = lane % SP;  // this lane's word of the concatenated row
    const u64 *base = a.strong + (size_t)r * a.strong_rstride + (size_t)l0 * a.strong_stride + c0;
    // U_r of this lane's word: from LDS when the caller staged it (W words), else loaded
    const u64 ur = lane < WP ? (Ur ? (c0 < WSs ? Ur[l0 * WSs + c0] : 0ULL) : a.U[((size_t)l0 * a.R + r) * SP + c0]) : 0ULL;
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
  // weak columns: one wave per local shard when there are as many shards as
  // waves (their offsets load in parallel), else every thread on each shard
  const bool per_wave = NL >= NW;
  for (int l = per_wave ? wv : 0; l < NL; l += per_wave ? NW : 1) {
    // (a prefetched range: one local shard)
    const uint64_t c0 = wc0 >= 0 ? (uint64_t)wc0 : a.wcro[(size_t)l * (a.R + 1) + r];
    const uint64_t c1 = wc0 >= 0 ? (uint64_t)wc1 : a.wcro[(size_t)l * (a.R + 1) + r + 1];
    for (uint64_t jj = c0 + (per_wave ? lane : tid); jj < c1; jj += per_wave ? 64 : NT) {
      const u64 *row = a.wcr + jj * W;
      const uint32_t key = a.wck[jj];  // with the row: one memory latency
      u64 hit = 0;
      for (int w = 0; w < W; w++) hit |= row[w] & FE[w];
      if (!hit) continue;
      const int tr = r - (int)(key >> 11), cg = (a.shard0 + l) * WSs * 64 + (int)(key & 2047u);
      if (tr < bottom) continue;
      atomicOr(&ring[(size_t)(tr & dm) * W + (cg >> 6)], 1ULL << (cg & 63));
    }
  }
}

// full round r: ring[r-1] |= U_r, (weak) ring[r-d-2] |= WU_r[d] (>= bottom); lane w < W
__device__ __forceinline__ void expand_full_round(const MArgs &a, int r, int bottom, u64 *ring, int dm, bool weak,
                                                  int w) {
  const int l = w / a.WSs, cw = w - l * a.WSs, W = a.W;
  const size_t ub = (size_t)l * a.R + r;
  ring[(size_t)((r - 1) & dm) * W + w] |= a.U[ub * a.SP + cw];
  if (weak)
    for (int d = 0; d < a.dd; d++) {
      const int tr = r - d - 2;
      if (tr < bottom) break;
      ring[(size_t)(tr & dm) * W + w] |= a.WU[(ub * a.dd + d) * a.SP + cw];
    }
}

// sum over the vertices of FE (LDS, W words) of sdeg (+ wdeg): every thread calls
// it, thread t takes sources t, t + NT, ...; returns the block total in *out (LDS)
template <int NT>
__device__ __forceinline__ void fe_degrees(const MArgs &a, int r, const u64 *FE, bool with_weak, u64 *out) {
  u64 e = 0;
  for (int s = threadIdx.x; s < a.n; s += NT)
    if ((FE[s >> 6] >> (s & 63)) & 1ULL) {
      const size_t at = (size_t)r * a.n + s;
      e += a.sdeg[at] + (with_weak ? a.wdeg[at] : 0);
    }
  e = dr::wave_sum(e);
  if ((threadIdx.x & 63) == 0 && e) atomicAdd(out, e);
}

// Per-round words of lane w < W (global word w = shard w / WSs, column w mod
// WSs) that do not depend on the frontier, loaded one round ahead by wave 0:
// presence, canonical row, U and the first FDD weak-summary slots.
// Also the leader of the wave whose first round r is (chains), and the round's
// weak-column range when the context holds one shard (pops).
constexpr int FDD = 3;
struct FRound {
  u64 P, K, U, WU[FDD];
  uint64_t C0, C1;
  u64 SD;  // chains: the round's strong-degree sum
  int L;
};
// Every lane of wave 0 calls it (lanes >= W load nothing), so no part of the
// record is assigned under a lane-divergent branch.
// EXTRA: also the weak range, SD and the wave leader (the canonical walk uses the range).
template <bool EXTRA = true>
__device__ __forceinline__ void fload_round(const MArgs &a, int r, bool pop, int w, FRound &x, bool wantK = true) {
  const bool on = w < a.W;
  const int l = on ? w / a.WSs : 0, cw = on ? w - l * a.WSs : 0;
  const size_t ub = (size_t)l * a.R + r;
  x.P = on ? a.pres[(size_t)r * a.W + w] : 0ULL;
  x.K = (on && pop && wantK) ? a.K[(size_t)r * a.W + w] : 0ULL;
  x.U = on ? a.U[ub * a.SP + cw] : 0ULL;
#pragma unroll
  for (int d = 0; d < FDD; d++) x.WU[d] = (on && pop && d < a.dd) ? a.WU[(ub * a.dd + d) * a.SP + cw] : 0ULL;
  if constexpr (EXTRA) {
    x.C0 = (pop && a.nlocal == 1) ? a.wcro[r] : 0;
    x.C1 = (pop && a.nlocal == 1) ? a.wcro[r + 1] : 0;
    x.SD = pop ? 0ULL : a.sdr[r];
    const int wvv = ((r - 1) >> 2) + 1;
    x.L = (!pop && r >= 1 && ((r - 1) & 3) == 0) ? (wvv < a.nlead ? (int)a.lead[wvv] : 1) - 1 : -1;
  }
}

// A full round's weak summaries: ring[r-d-2] |= WU_r[d] for d < dd and r-d-2 >=
// bottom.  Every lane of wave 0 calls it: lane w < W applies the FDD prefetched
// slots (pre) of word w; the deeper slots are spread over all 64 lanes (64/W per
// word, each every (64/W)-th slot), 8 loads in flight per lane before their ORs.
__device__ __forceinline__ void full_weak_round(const MArgs &a, int r, int bottom, u64 *ring, int dm, const u64 *pre,
                                                int lane) {
  const int W = a.W, dlim = min(a.dd, r - 1 - bottom);
  if (lane < W) {
#pragma unroll
    for (int d = 0; d < FDD; d++)
      if (d < dlim) ring[(size_t)((r - d - 2) & dm) * W + lane] |= pre[d];
  }
  const int LPW = (W <= 64 && 64 % W == 0) ? 64 / W : 1;
  const int w = lane % W, j = lane / W;
  if (j >= LPW) return;
  const int l = w / a.WSs, cw = w - l * a.WSs;
  for (int d0 = FDD + j; d0 < dlim; d0 += 8 * LPW) {
    u64 v[8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int d = d0 + q * LPW;
      v[q] = d < dlim ? a.WU[(((size_t)l * a.R + r) * a.dd + d) * a.SP + cw] : 0ULL;
    }
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int d = d0 + q * LPW;
      if (d < dlim) ring[(size_t)((r - d - 2) & dm) * W + w] |= v[q];
    }
  }
}

// canonical positions C: the presence prefix below the lowest walked round B, a
// scan of RD over [B, T] above it; FH_RLO = the first round whose prefix differs
// from the presence prefix (the speculative digests are exact below it), FH_NSEG.
// Shared by the fused walk (canon_walk's tail) and the stepped one.
template <int NT>
__device__ __forceinline__ void canon_positions(const MArgs &a, const FArgs &f, int B, int segs) {
  __shared__ int64_t s_scan[NT / 64];
  __shared__ int s_bad;
  const int tid = threadIdx.x, T = a.T;
  for (int x = tid; x < B && x <= T; x += NT) f.Cc[x] = f.ppref[x];
  const int span = T + 1 - B, per = span > 0 ? (span + NT - 1) / NT : 0;
  const int ra = B + tid * per, rb = min(T + 1, ra + per);
  int64_t loc = 0;
  for (int x = ra; x < rb; x++) loc += (int64_t)f.RD[x];
  int64_t tot;
  u64 run = (B >= 1 ? f.ppref[B - 1] : 0ULL) + (u64)fblock_scan<NT>(loc, s_scan, tot, 0);
  int bad = INT_MAX;
  for (int x = ra; x < rb; x++) {
    run += f.RD[x];
    f.Cc[x] = run;
    if (bad == INT_MAX && x >= 1 && run != f.ppref[x]) bad = x;
  }
  if (tid == 0) s_bad = INT_MAX;
  __syncthreads();
  if (bad != INT_MAX) atomicMin(&s_bad, bad);
  __syncthreads();
  if (tid == 0) {
    f.hdr[FH_NSEG] = segs;
    f.hdr[FH_RLO] = s_bad;
  }
}

// ---------------------------------------------------------------------------
// k_ms_canon_full: one workgroup, the canonical segments top down (k_canon).
// Dynamic LDS: ring[depth*W] | FE[W] | Ur[W].  As in k_ms_sweep_full, wave 0
// walks with the round words loaded three rounds ahead and applies full rounds
// alone; partial rounds take the workgroup (degrees loaded before the rows).
// ---------------------------------------------------------------------------
template <int NT>
__device__ __forceinline__ void canon_walk(const MArgs &a, const FArgs &f, u64 *lds) {
  const int W = a.W, dm = a.depth - 1, T = a.T;
  u64 *ring = lds, *FE = lds + (size_t)a.depth * W, *Ur = FE + W;
  __shared__ int s_ctl[4];
  __shared__ int64_t s_wc[2];
  __shared__ u64 s_e;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  int pos = T, segs = 0, lo_w = T + 1;
  while (true) {
    if (wv == 0) {
      const int b = next_bad(a, pos);
      if (lane == 0) s_ctl[0] = b;
    }
    __syncthreads();
    const int b = s_ctl[0];
    __syncthreads();
    if (b < 0) break;
    segs++;
    for (int i = tid; i < a.depth * W; i += NT) ring[i] = 0;
    __syncthreads();
    if (tid < W) {  // F_b = K^cand_b; pending below b from the full rounds above it
      ring[(size_t)(b & dm) * W + tid] = a.K[(size_t)b * W + tid];
      const int l = tid / a.WSs, cw = tid - l * a.WSs;
      for (int x = b - 1; x >= 0 && x >= b - a.dd; x--) {
        u64 v = 0;
        for (int y = max(b + 1, x + 2); y <= T && y <= x + a.dd + 1; y++)
          v |= a.WU[(((size_t)l * a.R + y) * a.dd + (y - x - 2)) * a.SP + cw];
        ring[(size_t)(x & dm) * W + tid] |= v;
      }
    }
    __syncthreads();
    int run = 0, r = b;
    const bool act = lane < W;
    // wave 0: the round words three rounds ahead; full rounds applied alone
    FRound c0{}, c1{}, c2{}, c3{};
    if (wv == 0) {
      fload_round(a, r, true, lane, c0, false);
      if (r >= 1) fload_round(a, r - 1, true, lane, c1, false);
      if (r >= 2) fload_round(a, r - 2, true, lane, c2, false);
    }
    for (;;) {
      if (wv == 0) {
        for (;;) {
          if (r >= 3) fload_round(a, r - 3, true, lane, c3, false);
          u64 fw = 0;
          const u64 p = c0.P;
          if (act) {
            u64 *slot = &ring[(size_t)(r & dm) * W + lane];
            fw = *slot;
            *slot = 0;
            a.K[(size_t)r * W + lane] = fw;
          }
          const u64 fe = fw & p;
          const bool full = __ballot(act && fe != p) == 0ULL;
          int cnt = __popcll(fe);
          for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
          run = full ? run + 1 : 0;
          if (lane == 0) f.RD[r] = r == 0 ? 0 : (u64)cnt;
          if (run >= a.dmax || r == 0) {  // regime restored at r (CE_r keeps the full-round total)
            if (lane == 0) s_ctl[1] = 1;
            break;
          }
          if (!full) {  // partial: the workgroup expands it
            if (act) {
              FE[lane] = fe;
              Ur[lane] = c0.U;
            }
            if (lane == 0) {
              s_ctl[1] = 0;
              s_ctl[2] = r;
              s_wc[0] = a.nlocal == 1 ? (int64_t)c0.C0 : -1;
              s_wc[1] = (int64_t)c0.C1;
              s_e = 0;
            }
            break;
          }
          // full: ring[r-1] |= U_r, ring[r-d-2] |= WU_r[d]
          if (act) ring[(size_t)((r - 1) & dm) * W + lane] |= c0.U;
          full_weak_round(a, r, 0, ring, dm, c0.WU, lane);
          c0 = c1;
          c1 = c2;
          c2 = c3;
          --r;
        }
      }
      __syncthreads();
      if (s_ctl[1]) break;
      r = s_ctl[2];
      // the partial round's strong + weak degrees (loaded before the rows) and expansion
      constexpr int KS = 2048 / NT;
      uint32_t dg[KS];
#pragma unroll
      for (int k = 0; k < KS; k++) {
        const int sv = tid + k * NT;
        const size_t at = (size_t)r * a.n + sv;
        dg[k] = (sv < a.n && ((FE[sv >> 6] >> (sv & 63)) & 1ULL)) ? (uint32_t)a.sdeg[at] + a.wdeg[at] : 0u;
      }
      expand_partial_full<NT>(a, r, 0, FE, ring, dm, true, Ur, s_wc[0], s_wc[1]);
      u64 e = 0;
#pragma unroll
      for (int k = 0; k < KS; k++) e += dg[k];
      e = dr::wave_sum(e);
      if (lane == 0 && e) atomicAdd(&s_e, e);
      __syncthreads();
      if (tid == 0) f.CE[r] = s_e;
      if (wv == 0) {
        c0 = c1;
        c1 = c2;
        c2 = c3;
      }
      --r;
    }
    if (tid == 0) s_ctl[3] = r;  // wave 0's stop round
    __syncthreads();
    r = s_ctl[3];
    __syncthreads();
    pos = r;
    lo_w = min(lo_w, r);
  }
  // canonical positions: below the lowest walked round every round is full (C
  // is the presence prefix); the scan covers the walked region only
  canon_positions<NT>(a, f, lo_w, segs);
}
template <int NT>
__global__ __launch_bounds__(NT) void k_ms_canon_full(MArgs a, FArgs f) {
  extern __shared__ __attribute__((aligned(16))) u64 lds[];
  canon_walk<NT>(a, f, lds);
}


// canonical digest of round r >= 1 (one wave per round): the speculative one
// below the first round whose position prefix differs from the presence prefix
__device__ __forceinline__ void rg_round(const MArgs &a, const FArgs &f, int r) {
  const int lane = threadIdx.x & 63;
  if (r > a.T) return;
  if (r == 0) {
    if (lane == 0) f.RG[0] = 0;
    return;
  }
  if (r < f.hdr[FH_RLO]) {
    if (lane == 0) f.RG[r] = f.SG[r];
    return;
  }
  const u64 mw = lane < a.W ? a.K[(size_t)r * a.W + lane] & a.pres[(size_t)r * a.W + lane] : 0ULL;
  u64 dg = 0, ed = 0;
  ms_wave_emit(a.slot_off, a.slot_src, r, mw, f.Cc[r - 1], a.W, nullptr, nullptr, a.n, dg, ed);
  dg = dr::wave_sum(dg);
  if (lane == 0) f.RG[r] = dg;
}
__global__ __launch_bounds__(256) void k_ms_rg_full(MArgs a, FArgs f) {
  rg_round(a, f, blockIdx.x * 4 + (threadIdx.x >> 6));
}

// ---------------------------------------------------------------------------
// plan_body: waveReady's chain tasks (process.go:341-350) from the device commit
// flags, one workgroup (k_ms_prefix_plan, k_ms_cpos).  Committed wave w's floor is
// the previous committed wave (persistent decidedWave) or 0 (Q1 literal); it has a
// chain query when w - 1 >= floor + 1.  Chain i takes query slot npop + i, its
// pushes from the exclusive prefix of the chains' push bounds (w - floor each).
// make_pops: also the pop queries (the fused form).
// ---------------------------------------------------------------------------
template <int NT>
__device__ __forceinline__ void plan_body(const MArgs &a, const FArgs &f, MQuery *__restrict__ q, int push_cap,
                                          int make_pops) {
  __shared__ int64_t s_scan[NT / 64];
  const int nw = f.nw, tid = threadIdx.x;
  const int per = (nw + NT - 1) / NT, wa = 1 + tid * per, wb = min(nw + 1, wa + per);
  if (make_pops) {
    // the pop queries (one per wave whose leader is present, in wave order; mask
    // rows top..0 each), as the host lists them: no upload before the sweeps
    auto leader_present = [&](int w, int &L) {
      const int r1 = 4 * (w - 1) + 1;
      L = (w < a.nlead ? (int)a.lead[w] : 1) - 1;
      return ((a.pres[(size_t)r1 * a.W + (L >> 6)] >> (L & 63)) & 1ULL) != 0ULL;
    };
    int64_t pc = 0, pm = 0;
    for (int w = wa; w < wb; w++) {
      int L;
      if (leader_present(w, L)) {
        pc++;
        pm += (int64_t)(4 * (w - 1) + 2) * a.W;
      }
    }
    int64_t t0, t1;
    int64_t pi = fblock_scan<NT>(pc, s_scan, t0, 0);
    int64_t mo = fblock_scan<NT>(pm, s_scan, t1, 0);
    for (int w = wa; w < wb; w++) {
      int L;
      if (leader_present(w, L)) {
        MQuery x{};
        x.type = MQ_POP;
        x.top = 4 * (w - 1) + 1;
        x.bottom = 0;
        x.src0 = L;
        x.mask_off = mo;
        q[pi++] = x;
        mo += (int64_t)(x.top + 1) * a.W;
      }
    }
  }
  // floors: exclusive prefix max of (commit ? w : 0)
  int64_t m = 0;
  for (int w = wa; w < wb; w++)
    if (f.commit[w - 1]) m = w;
  int64_t tot;
  int64_t prev = fblock_scan<NT>(m, s_scan, tot, 1);
  int64_t cnt = 0, pushes = 0;
  {
    int64_t pv = prev;
    for (int w = wa; w < wb; w++)
      if (f.commit[w - 1]) {
        const int fl = f.persistent ? (int)pv : 0;
        if (w - 1 >= fl + 1) {
          cnt++;
          pushes += w - fl;
        }
        pv = w;
      }
  }
  int64_t ctot, ptot;
  int64_t ci = fblock_scan<NT>(cnt, s_scan, ctot, 0);
  int64_t pb = fblock_scan<NT>(pushes, s_scan, ptot, 0);
  {
    int64_t pv = prev;
    for (int w = wa; w < wb; w++)
      if (f.commit[w - 1]) {
        const int fl = f.persistent ? (int)pv : 0;
        if (w - 1 >= fl + 1) {
          MQuery x{};
          x.type = MQ_CHAIN;
          x.top = 4 * (w - 1) + 1;
          x.bottom = 4 * fl + 1;
          x.src0 = (w < a.nlead ? (int)a.lead[w] : 1) - 1;
          x.push_base = (int32_t)pb;
          const int qi = f.npop + (int)ci;
          q[qi] = x;
          ci++;
          pb += w - fl;
        }
        pv = w;
      }
  }
  if (tid == 0) {
    f.hdr[FH_NCHAIN] = (int32_t)ctot;
    f.hdr[FH_PUSHES] = (int32_t)min<int64_t>(ptot, INT32_MAX);
    f.hdr[FH_ERR] = ptot > push_cap ? 1 : 0;
  }
}

// The canonical prefixes G, E (RG, CE -> Gc, Ec) and the plan (pops and chains)
// in one single-workgroup launch (the fused form: both read only what earlier
// launches wrote)
template <int NT>
__global__ __launch_bounds__(NT) void k_ms_prefix_plan(MArgs a, FArgs f, MQuery *__restrict__ q, int push_cap) {
  __shared__ u64 part[2 * NT / 64];
  ms_prefix_two<NT>(a.T + 1, f.RG, f.Gc, f.CE, f.Ec, part);
  plan_body<NT>(a, f, q, push_cap, 1);
}


// ---------------------------------------------------------------------------
// k_ms_sweep_full: one workgroup per query, every round to its end (the same
// decisions as k_ms_step, shard_memo.hpp).  Grid npop + nw: workgroups past the
// planned chains exit.  Dynamic LDS: ring[depth*W] | FE[W].
//
// Wave 0 decides each round from words it loaded one round ahead and applies,
// without a workgroup barrier, every round it can expand alone: a full round
// (ring |= U_r, WU_r from the prefetched words), a round whose frontier is one
// vertex (the query's top, a chain's restart: that row and its weak columns)
// and an empty one.  Only a partial round with several vertices is expanded by
// the whole workgroup (expand_partial_full).
// ---------------------------------------------------------------------------
// (4 waves per SIMD: every C4 query resident at once -- at 130 VGPRs, 3 per SIMD, the
// last quarter of the pops started after the first had finished, profiles/r04/)
template <int NT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4))) void k_ms_sweep_full(MArgs a, FArgs f) {
  extern __shared__ __attribute__((aligned(16))) u64 lds[];
  const int qi = blockIdx.x;
  DR_MT(const u64 tt0 = wall_clock64(); u64 tt_wg = 0, n_w0 = 0, n_wg = 0;)
  if (qi >= f.npop + f.hdr[FH_NCHAIN]) return;
  const int W = a.W, dm = a.depth - 1, WSs = a.WSs;
  u64 *ring = lds, *FE = lds + (size_t)a.depth * W;
  __shared__ int s_ctl[2];
  __shared__ u64 s_e;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const MQuery Q = a.q[qi];
  const bool pop = Q.type == MQ_POP, weak = pop;
  for (int i = tid; i < a.depth * W; i += NT) ring[i] = 0;
  __syncthreads();
  if (tid == 0 && Q.src0 >= 0) ring[(size_t)(Q.top & dm) * W + (Q.src0 >> 6)] = 1ULL << (Q.src0 & 63);
  __syncthreads();
  int run = 0, low = Q.top, npush = 0;
  u64 edges = 0;
  int r = Q.top;
  bool merged = false;
  const bool act = lane < W;
  FRound cur{}, nxt{}, nx2{};  // wave 0: rounds r, r-1 (loaded), r-2 (issued at round r)
  if (wv == 0 && act) {
    fload_round<false>(a, r, pop, lane, cur);
    if (r >= 1) fload_round<false>(a, r - 1, pop, lane, nxt);
  }
  for (;;) {
    if (wv == 0) {
      for (;;) {
        if (act && r >= 2) fload_round<false>(a, r - 2, pop, lane, nx2);
        u64 fw = 0;
        const u64 p = cur.P;
        if (act) {
          u64 *slot = &ring[(size_t)(r & dm) * W + lane];
          fw = *slot;
          *slot = 0;
        }
        int single = r == Q.top ? Q.src0 : -1;  // a round whose frontier is one known vertex
        // waveReady's chain (process.go:342-350): a reachable, present leader of
        // wave wvv is pushed and the chain goes on from it alone
        if (!pop && r < Q.top && ((r - 1) & 3) == 0) {
          const int wvv = ((r - 1) >> 2) + 1;
          const int L = (wvv < a.nlead ? (int)a.lead[wvv] : 1) - 1;
          const u64 fl = __shfl(fw & p, L >> 6);
          if ((fl >> (L & 63)) & 1ULL) {
            fw = lane == (L >> 6) ? 1ULL << (L & 63) : 0ULL;
            if (lane == 0) a.push_out[Q.push_base + npush] = wvv;
            npush++;
            single = L;
          }
        }
        const u64 fe = fw & p;
        const bool nz = __ballot(act && fw != 0ULL) != 0ULL;
        const bool anyfe = __ballot(act && fe != 0ULL) != 0ULL;
        const bool full = __ballot(act && fe != p) == 0ULL;
        if (nz) low = min(low, r - 1);
        bool done;
        if (pop) {
          run = __ballot(act && fw != cur.K) == 0ULL ? run + 1 : 0;
          merged = run >= a.dmax;
          done = merged || r <= Q.bottom || (!nz && low >= r);
          if (act) a.masks[Q.mask_off + (int64_t)(Q.top - r) * W + lane] = fw;
        } else {
          done = r <= Q.bottom || (!nz && low >= r);
        }
        const bool summary = !done && full;
        if (!pop && !done && summary) edges += a.sdr[r];
        if (!done && pop && anyfe) low = min(low, r - a.dmax);
        if (done) {
          if (lane == 0) {
            s_ctl[0] = 1;
            s_ctl[1] = r;
          }
          break;
        }
        if (summary) {  // ring[r-1] |= U_r, ring[r-d-2] |= WU_r[d]
          if (act) ring[(size_t)((r - 1) & dm) * W + lane] |= cur.U;
          if (weak) full_weak_round(a, r, Q.bottom, ring, dm, cur.WU, lane);  // every lane of wave 0
        } else if (anyfe && single >= 0 && ((__shfl(fe, single >> 6) >> (single & 63)) & 1ULL)) {
          // FE = {single}: its row (every local shard's piece) and its weak columns
          if (!pop) edges += a.sdeg[(size_t)r * a.n + single];
          if (act) {
            const int l = lane / WSs, cw = lane - l * WSs;
            ring[(size_t)((r - 1) & dm) * W + lane] |=
                a.strong[(size_t)r * a.strong_rstride + (size_t)l * a.strong_stride + (size_t)single * a.SP + cw];
          }
          if (weak)
            for (int l = 0; l < a.nlocal; l++) {
              const uint64_t c0 = a.wcro[(size_t)l * (a.R + 1) + r], c1 = a.wcro[(size_t)l * (a.R + 1) + r + 1];
              for (uint64_t jj = c0 + lane; jj < c1; jj += 64) {
                if (!((a.wcr[jj * W + (single >> 6)] >> (single & 63)) & 1ULL)) continue;
                const uint32_t key = a.wck[jj];
                const int tr = r - (int)(key >> 11), cg = (a.shard0 + l) * WSs * 64 + (int)(key & 2047u);
                if (tr < Q.bottom) continue;
                atomicOr(&ring[(size_t)(tr & dm) * W + (cg >> 6)], 1ULL << (cg & 63));
              }
            }
        } else if (anyfe) {  // a partial round: the workgroup expands it
          if (act) FE[lane] = fe;
          if (lane == 0) {
            s_ctl[0] = 0;
            s_ctl[1] = r;
            s_e = 0;
          }
          break;
        }
        DR_MT(n_w0++;)
        cur = nxt;
        nxt = nx2;
        --r;
      }
    }
    __syncthreads();
    if (s_ctl[0]) break;
    r = s_ctl[1];
    DR_MT(const u64 tw = wall_clock64();)
    constexpr int KS = 2048 / NT;  // sources per thread (n <= 2048)
    uint16_t dg[KS];
    if (!pop) {  // a chain's strong degrees of FE (the edges it traverses), loaded before the rows
#pragma unroll
      for (int k = 0; k < KS; k++) {
        const int sv = tid + k * NT;
        dg[k] = (sv < a.n && ((FE[sv >> 6] >> (sv & 63)) & 1ULL)) ? a.sdeg[(size_t)r * a.n + sv] : (uint16_t)0;
      }
    }
    expand_partial_full<NT>(a, r, Q.bottom, FE, ring, dm, weak);
    if (!pop) {
      u64 e = 0;
#pragma unroll
      for (int k = 0; k < KS; k++) e += dg[k];
      e = dr::wave_sum(e);
      if (lane == 0 && e) atomicAdd(&s_e, e);
    }
    __syncthreads();
    DR_MT(tt_wg += wall_clock64() - tw; n_wg++;)
    if (wv == 0) {
      if (!pop) edges += s_e;
      cur = nxt;
      nxt = nx2;
    }
    --r;
  }
  __shared__ MState s_fin;
  if (tid == 0) {
    MState o{};
    o.done = 1;
    o.run = run;
    o.low = low;
    o.stop = r;
    o.merged = pop && merged;
    o.npush = npush;
    o.edges = edges;
    o.cur = r;
    f.fin[qi] = o;
    s_fin = o;
    DR_MT(if (qi < kMsTimingQ) {
      u64 *t = g_ms_timing + 8 * (size_t)qi;
      t[0] = tt0; t[1] = wall_clock64(); t[2] = n_w0; t[3] = n_wg; t[4] = tt_wg;
      t[5] = (u64)Q.type; t[6] = (u64)Q.top; t[7] = (u64)(int64_t)r;
    })
  }
  if (pop && f.emit) {  // REF emission of this pop here (wave 0's mask rows: same CU, after the barrier)
    static_assert(NT == MS_NT, "ms_emit_query assumes MS_NT threads");
    __syncthreads();
    const MState S = s_fin;
    ms_emit_query(a, Q, S, a.slot_off, a.slot_src, f.Cc, f.Gc, f.Ec, qi, f.qcount, f.qdigest, f.qedges);
  }
}

}  // namespace drs
