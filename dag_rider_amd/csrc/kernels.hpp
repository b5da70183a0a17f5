// kernels.hpp -- CDNA4 (gfx950) kernels of the causal-history reachability engine.
//
// Device layout, WS = row stride in u64 words = next_pow2(ceil(n/64)):
//   strong  [rounds][n][WS]  bit t of row (r,s) <=> strong edge (r,s) -> (r-1,t+1)
//   present [rounds][WS]     bit s-1 <=> source s has a vertex in round r
//   weak_roff  prefix of each round's weak-edge count (the edges themselves live
//           in the weak columns below; only counts are needed per edge)
//   far     u64 per edge with delta > 1023: (own source-1) << 32 | (r' << 11 | t-1)
//   wc      weak columns, grouped by round (wc_roff[r]..wc_roff[r+1]): one entry per
//           distinct near weak target of the round, key (delta << 11 | t-1), and a
//           WS-word row of the round's sources with that edge.  A late vertex
//           collects hundreds of weak edges, so the columns are ~1/16 of the edge
//           list at C4; the sweeps and the weak union read them instead.
//
// Kernels (all integer/boolean; HBM-bound, no MFMA):
//   k_commit  waveReady's commit decision (process.go:326-339) for a range of
//             waves, one workgroup per wave: backward strong sweep from the leader
//             over rounds 4w-2..4w with ballot-compacted "row AND S != 0" tests.
//   k_sweep   forward reachability (path(), process.go:89-148) from one vertex per
//             workgroup, round by round: OR of the rows in the frontier (coalesced
//             16-B row chunks, wave64 xor-shuffle OR reduction, LDS 64-bit atomic OR
//             into a ring of future-round frontiers) plus weak-edge scatter into that
//             ring.  Variants: chain (waveReady's leader chain, :341-350), prune
//             (paper-mode orderVertices dedup), masks (reach sets for delivery).
//   k_emit_*  orderVertices emission (process.go:417-441): per (pop, round) counts,
//             scan, then (round asc, slot asc) positions via ballot ranks, the
//             order-sensitive digest and optional id list.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <climits>

#include "wave_ops.hpp"

namespace dr {



typedef unsigned long long u64;
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#ifdef DR_SWEEP_TIMING
// profiling build only (libdagrider_gpu_timing.so, tools/sweep_timing.py): per
// query, wall-clock ticks of the prologue, wave 0's phase A (summary rounds
// included), the partial rounds' expansion, the total, and the round counts
constexpr int kSweepTimingQ = 8192;
__device__ u64 g_sweep_timing[16 * kSweepTimingQ];
__device__ u64 g_canon_timing[8];  // k_canon: start, segments walked, positions done, segment count, rounds walked
#define DR_TT(...) __VA_ARGS__
#else
#define DR_TT(...)
#endif

// Q_REGULAR: follow only the regular graph -- strong rows and weak columns of delta
// <= MemoView::dreg, no far edge (the exception test, engine.hip ensure_exceptions)
// Q_FAST (merge sweeps with summaries, dd <= DDR): also stop at the first round r whose
// frontier equals K_r while the pending ring equals K's pending contributions from the
// rounds above (sweep_body: kring); the cut is then r itself
enum : int32_t { Q_STRONG_ONLY = 1, Q_CHAIN = 2, Q_MASKS = 4, Q_PRUNE = 8, Q_SHORTCUT = 16, Q_MERGE = 32, Q_REGULAR = 64,
                 Q_FAST = 128 };

struct SweepQuery {
  int32_t top;       // start round (the `from` vertex's round)
  int32_t bottom;    // last round of the sweep (not expanded)
  int32_t src0;      // 0-based source of `from`; -1 = nothing to expand
  int32_t flags;     // Q_*
  int64_t mask_off;  // word offset of round `bottom` in masks (Q_MASKS)
  int32_t out_off;   // Q_CHAIN: first entry in push_out
  int32_t tgt0;      // path: 0-based target source tested at round `bottom`, -1 none
  int32_t cur_round; // Q_PRUNE: rounds 1..cur_round enter the delivered set
  int32_t pad;
};

// The single-stream REF replay (engine.hip replay_planned): the delivery sweeps run from
// the static per-wave query table before the leader chains are known, so a query is live
// when its wave committed or a chain pushed its leader (pushed[w] == epoch, the replay's
// stamp: no clearing between replays).  Chain sweeps stamp pushed[]; delivery sweeps,
// their emission and the upward-edge check skip a query that is not live.
struct PopMark {
  const uint8_t *commit;  // [wave-1]; null: no filter / no stamping
  int32_t *pushed;        // [wave]
  int32_t epoch;
  __device__ bool live(int top) const {
    const int w = (top - 1) / 4 + 1;
    return commit[w - 1] || pushed[w] == epoch;
  }
};

struct DagView {
  const u64 *strong;
  const u64 *present;
  const uint32_t *weak_roff;  // prefix of weak-edge counts per round (edge accounting)
  const u64 *far;
  const uint32_t *far_roff;
  const uint32_t *wc_key;
  const u64 *wc_rows;
  const uint32_t *wc_roff;
  const uint16_t *sdeg;  // [rounds][n] strong degree per vertex
  const uint16_t *wdeg;  // [rounds][n] weak degree per vertex (far edges included)
  const uint16_t *lead;  // [wave] chooseLeader(w) (process.go:386-392), 1-based source
  // repeated ids (uponDeliver / the buffer loop append an id already in the
  // round, process.go:158-169, :229): null when the mirror has none.  dup_src
  // lists the source of every slot after the first of its id, per round
  // (dup_off[r] .. dup_off[r+1]); slot_rep[slot] = 1 for those slots.  Edges
  // come from the id's last slot (path's lookup, :112-116); vCount and REF
  // delivery count every slot (:332, :418-429).
  const uint32_t *dup_off;
  const uint16_t *dup_src;
  const uint8_t *slot_rep;
  // [round] strong edges kept beside the rows (App. A Q8: to a round other than r-1),
  // counted in sdeg but not in the rows' popcount: the round summaries' SD adds them.
  // Null when the mirror has none.
  const uint32_t *sdx;
  int32_t n;
  int32_t nrounds;
  // wave-range slice (dr_set_slice): digest keys use global rounds (round + roff);
  // rounds >= seed_lo are taken as full canonical rounds (K covers P; INT_MAX: none)
  int32_t roff;
  int32_t seed_lo;
};

// repeated slots of round r whose source is in the set X (lane w < WS holds word
// w of X; every lane of the wave calls it and gets the count)
template <int WS>
__device__ __forceinline__ int dup_count(const DagView &g, int r, u64 xw) {
  if (!g.dup_off) return 0;
  const uint32_t a = g.dup_off[r], b = g.dup_off[r + 1];
  int c = 0;
  for (uint32_t j = a; j < b; j++) {  // wave-uniform
    const int s = (int)g.dup_src[j] - 1;
    const u64 w = __shfl(xw, (s >> 6) & (WS - 1));
    c += (int)((w >> (s & 63)) & 1ULL);
  }
  return c;
}

// Geometry per row stride: chunks are 16 B (two words) for WS >= 2, one word for WS == 1.
template <int WS, int NT>
struct Geo {
  static constexpr int CW = WS >= 2 ? 2 : 1;    // words per chunk
  static constexpr int CPR = WS / CW;           // chunks per row
  static constexpr int RPP = NT / CPR;          // rows per pass
  static constexpr int NMAX = 64 * WS;          // max n for this stride
  static constexpr int CPT = (NMAX + RPP - 1) / RPP;  // passes (chunks per thread)
  static_assert(NT % 64 == 0 && NT % CPR == 0, "block must tile rows");
};

// ---------------------------------------------------------------------------
// k_commit: one workgroup per wave.  S0 = {leader}; S_{k+1} = {v in round
// r1+k+1 : row(v) & S_k != 0}; vcount = |S_3|.  Every row load of the wave goes out
// before the first is used: round r1+1 as the word holding the leader's bit of each
// row (one source per thread), rounds r1+2, r1+3 whole (16-B chunks; they do not
// depend on S).  An absent vertex's row is zero (the append rejects strong edges on
// one), so no presence test is needed.  (Round by round, each round's loads waited
// for the previous round's S: three memory round trips a wave, 21 us for a rank's
// 125-wave share at N = 8, 0.20 of peak, profiles/r05/final_bench_share8.json.)
// ---------------------------------------------------------------------------
template <int WS, int NT>
__global__ __launch_bounds__(NT) void k_commit(DagView g, int w0, int nw, int quorum,
                                               uint8_t *__restrict__ commit,
                                               int32_t *__restrict__ vcount) {
  using G = Geo<WS, NT>;
  constexpr int CW = G::CW, CPR = G::CPR, RPP = G::RPP, CPT = G::CPT;
  constexpr int NS = (64 * WS + NT - 1) / NT;  // passes over the sources of round r1+1
  __shared__ u64 S[WS];
  __shared__ u64 T[WS];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int bi = blockIdx.x;
  if (bi >= nw) return;
  const int w = w0 + bi;
  const int r1 = 4 * (w - 1) + 1;
  const int n = g.n;
  const int l = g.lead[w] - 1;  // chooseLeader(w), 0-based
  if (!((g.present[(size_t)r1 * WS + (l >> 6)] >> (l & 63)) & 1ULL)) {  // leader is bottom (process.go:327-329)
    if (tid == 0) { commit[bi] = 0; vcount[bi] = -1; }
    return;
  }
  const int j = tid % CPR;  // this thread's chunk column in rounds r1+2, r1+3
  const u64 *rows1 = g.strong + (size_t)(r1 + 1) * n * WS;
  u64 x1[NS];
#pragma unroll
  for (int i = 0; i < NS; i++) {
    const int s = i * NT + tid;
    x1[i] = rows1[(size_t)(s < n ? s : 0) * WS + (l >> 6)];
  }
  // both rounds in registers when they fit (n = 2048: 16 chunks a round, round r1+3 then
  // loads once round r1+2 is consumed)
  constexpr int PRE = CPT <= 8 ? 2 : 1;
  u64 v0[PRE][CPT], v1[PRE][CPT];
  auto load = [&](int k, int slot) {
    const u64 *rows = g.strong + (size_t)(r1 + 2 + k) * n * WS;
#pragma unroll
    for (int p = 0; p < CPT; p++) {
      const int s = tid / CPR + p * RPP;
      const size_t at = (size_t)(s < n ? s : 0) * WS;  // clamped: unconditional loads
      if constexpr (CW == 2) {
        const ulonglong2 x = *reinterpret_cast<const ulonglong2 *>(rows + at + 2 * j);
        v0[slot][p] = x.x;
        v1[slot][p] = x.y;
      } else {
        v0[slot][p] = rows[at];
        v1[slot][p] = 0;
      }
    }
  };
#pragma unroll
  for (int k = 0; k < PRE; k++) load(k, k);
  if (tid < WS) T[tid] = 0;
  // S_1: the sources of round r1+1 whose row holds the leader (wave = 64 sources)
#pragma unroll
  for (int i = 0; i < NS; i++) {
    const int s = i * NT + tid;
    const u64 m = __ballot(s < n && ((x1[i] >> (l & 63)) & 1ULL));
    const int word = (i * NT) / 64 + wid;
    if (lane == 0 && word < WS) S[word] = m;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const int kk = PRE == 2 ? k : 0;
    if (PRE == 1 && k == 1) load(1, 0);
    // S chunk this thread ANDs with
    const u64 s0 = S[j * CW], s1 = CW == 2 ? S[j * CW + 1] : 0ULL;
#pragma unroll
    for (int p = 0; p < CPT; p++) {
      const int rowbase = (wid * 64) / CPR + p * RPP;  // first row of this wave's pass
      if (rowbase >= n) break;                         // wave-uniform
      const int s = tid / CPR + p * RPP;
      const bool hit = s < n && ((v0[kk][p] & s0) | (v1[kk][p] & s1)) != 0ULL;
      u64 m = __ballot(hit);
      if (lane == 0 && m) {
        u64 bits;
        if constexpr (CPR == 1) {
          bits = m;
        } else {
#pragma unroll
          for (int sh = 1; sh < CPR; sh <<= 1) m |= m >> sh;
          bits = 0;
#pragma unroll
          for (int gI = 0; gI < 64 / CPR; gI++) bits |= ((m >> (gI * CPR)) & 1ULL) << gI;
        }
        atomicOr(&T[rowbase >> 6], bits << (rowbase & 63));
      }
    }
    __syncthreads();
    if (tid < WS) { S[tid] = T[tid]; T[tid] = 0; }
    __syncthreads();
  }
  if (wid == 0) {  // vCount counts slots (process.go:330-335): repeated ids once per slot
    const int dc = dup_count<WS>(g, r1 + 3, lane < WS ? S[lane] : 0ULL);
    if (tid == 0) {
      int vc = dc;
#pragma unroll
      for (int i = 0; i < WS; i++) vc += popc64(S[i]);
      vcount[bi] = vc;
      commit[bi] = vc >= quorum ? 1 : 0;
    }
  }
}

// ---------------------------------------------------------------------------
// k_commit_split: the same commit rule for a short wave range (a rank's share of
// the all-waves commit sweep leaves most CUs idle with one workgroup per wave):
// KS workgroups per wave, no barrier between them.  Every workgroup of wave w
// computes S_1 (the rows of round 2 holding the leader's bit: one 16-B chunk per
// row) and S_2 (rows of round 3 reaching S_1: the whole round) itself, then its
// own share of S_3 -- rows [j*RS, (j+1)*RS) of round 4, RS = P3 passes of rows --
// and adds |S_3 share| (+ its repeated slots) to the wave's sum.  Count and sum
// share one 64-bit word (arrivals << 32 | votes) added by one atomic, so the
// last workgroup to arrive holds the complete sum with no fence (an agent-scope
// release per workgroup would write back the XCD's L2); it writes commit /
// vcount and zeroes the word.  Every load goes out before the first ballot (none
// depends on S).
// The KS workgroups of a wave sit on one XCD (blockIdx = (group*KS + j)*8 + xcd,
// wave = group*8 + xcd), so the rounds they all read come from one L2.
// ---------------------------------------------------------------------------
template <int WS, int NT, int P3>
__global__ __launch_bounds__(NT) void k_commit_split(DagView g, int w0, int nw, int KS, int quorum,
                                                     unsigned long long *__restrict__ acc,
                                                     uint8_t *__restrict__ commit, int32_t *__restrict__ vcount) {
  using G = Geo<WS, NT>;
  constexpr int CW = G::CW, CPR = G::CPR, RPP = G::RPP, CPT = G::CPT, NMAX = G::NMAX;
  constexpr int L1 = (NMAX + NT - 1) / NT;  // round-2 rows per thread
  __shared__ u64 S1[WS], S2[WS], S3[WS];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, grp = slot / KS, j = slot - grp * KS;
  const int bi = grp * 8 + xcd;
  if (bi >= nw) return;  // a slot of the last group past the range: no wave
  const int w = w0 + bi, r1 = 4 * (w - 1) + 1, n = g.n;
  const int l = g.lead[w] - 1;
  if (!((g.present[(size_t)r1 * WS + (l >> 6)] >> (l & 63)) & 1ULL)) {  // leader is bottom (process.go:327-329)
    if (j == 0 && tid == 0) { commit[bi] = 0; vcount[bi] = -1; }
    return;
  }
  // every load first: round 2's leader word of each row, round 3 whole, round 4's share
  u64 a[L1];
  const u64 *rows2 = g.strong + (size_t)(r1 + 1) * n * WS + (l >> 6);
#pragma unroll
  for (int k = 0; k < L1; k++) {
    const int s = tid + k * NT;
    a[k] = s < n ? __builtin_nontemporal_load(rows2 + (size_t)s * WS) : 0ULL;
  }
  const int jj = tid % CPR;
  u64 v0[CPT], v1[CPT];
  const u64 *rows3 = g.strong + (size_t)(r1 + 2) * n * WS;
#pragma unroll
  for (int p = 0; p < CPT; p++) {
    const int s = tid / CPR + p * RPP;
    v0[p] = 0;
    v1[p] = 0;
    if (s < n) {
      const u64 *q = rows3 + (size_t)s * WS + jj * CW;
      if constexpr (CW == 2) {
        const u64x2 x = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(q));
        v0[p] = x.x;
        v1[p] = x.y;
      } else {
        v0[p] = __builtin_nontemporal_load(q);
      }
    }
  }
  u64 u0[P3], u1[P3];
  const u64 *rows4 = g.strong + (size_t)(r1 + 3) * n * WS;
#pragma unroll
  for (int p = 0; p < P3; p++) {
    const int s = j * P3 * RPP + tid / CPR + p * RPP;
    u0[p] = 0;
    u1[p] = 0;
    if (s < n) {
      const u64 *q = rows4 + (size_t)s * WS + jj * CW;
      if constexpr (CW == 2) {
        const u64x2 x = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(q));
        u0[p] = x.x;
        u1[p] = x.y;
      } else {
        u0[p] = __builtin_nontemporal_load(q);
      }
    }
  }
  if (tid < WS) {
    S1[tid] = 0;
    S2[tid] = 0;
    S3[tid] = 0;
  }
  __syncthreads();
  // S_1: a wave's ballot is one word of rows
#pragma unroll
  for (int k = 0; k < L1; k++) {
    const int s0 = wid * 64 + k * NT;
    const u64 m = __ballot(tid + k * NT < n && ((a[k] >> (l & 63)) & 1ULL));
    if (lane == 0 && s0 < n && m) S1[s0 >> 6] = m;
  }
  __syncthreads();
  // the rows of a pass that reach S (ballot of CPR-lane groups -> one bit per row)
  auto pass_bits = [&](u64 x0, u64 x1, const u64 *S) -> u64 {
    const u64 sa = S[jj * CW], sb = CW == 2 ? S[jj * CW + 1] : 0ULL;
    u64 m = __ballot(((x0 & sa) | (x1 & sb)) != 0ULL);
    if constexpr (CPR == 1) return m;
    u64 bits = 0;
#pragma unroll
    for (int sh = 1; sh < CPR; sh <<= 1) m |= m >> sh;
#pragma unroll
    for (int gI = 0; gI < 64 / CPR; gI++) bits |= ((m >> (gI * CPR)) & 1ULL) << gI;
    return bits;
  };
#pragma unroll
  for (int p = 0; p < CPT; p++) {
    const int rowbase = (wid * 64) / CPR + p * RPP;  // first row of this wave's pass
    if (rowbase >= n) break;                         // wave-uniform
    const u64 bits = pass_bits(v0[p], v1[p], S1);
    if (lane == 0 && bits) atomicOr(&S2[rowbase >> 6], bits << (rowbase & 63));
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < P3; p++) {
    const int rowbase = j * P3 * RPP + (wid * 64) / CPR + p * RPP;
    if (rowbase >= n) break;
    const u64 bits = pass_bits(u0[p], u1[p], S2);
    if (lane == 0 && bits) atomicOr(&S3[rowbase >> 6], bits << (rowbase & 63));
  }
  __syncthreads();
  // |S_3 share| (+ its repeated slots, process.go:330-335) into the wave's sum
  if (wid == 0) {
    const int dc = dup_count<WS>(g, r1 + 3, lane < WS ? S3[lane] : 0ULL);
    int c = lane < WS ? popc64(S3[lane]) : 0;
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
    if (lane == 0) {
      const unsigned long long old = atomicAdd(&acc[bi], (1ULL << 32) | (unsigned long long)(c + dc));
      if ((old >> 32) == (unsigned long long)KS - 1ULL) {  // the last of the wave: every share is in
        const int vc = (int)(uint32_t)old + c + dc;
        vcount[bi] = vc;
        commit[bi] = vc >= quorum ? 1 : 0;
        acc[bi] = 0;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Round summaries (memo): per round r, U_r = OR of every strong row, WU_r[d] =
// union of the weak targets at delta d+2, SD_r = total strong degree.  A sweep
// whose frontier covers every present vertex of r (a "full" round) expands it
// as U_r / WU_r -- the same bits the rows would give -- without reading rows.
// K is the canonical cone: the reach sets of "every vertex of the top round";
// once a sweep's frontier equals K on dmax consecutive rounds, the rest of its
// cone is K.
// ---------------------------------------------------------------------------
struct MemoView {
  const u64 *U;
  const u64 *WU;
  const u64 *SD;
  const u64 *K;
  int32_t dd;    // dense weak slots (deltas 2 .. dd+1); 0 with no weak edges
  int32_t dmax;  // merge window = max(1, largest regular weak delta)
  int32_t dreg;  // the regular window: weak columns of larger delta (and far edges) are exceptions
  const u64 *CE;  // the canonical rounds' edges (Q_FAST: the rounds a fast merge skips)
};

// One partial round r of a sweep: the frontier FE's strong rows -> ring slot of
// round r-1, and (WEAK) its weak columns -> the ring slots (or far mask rows,
// mask_bottom) of their target rounds.  Returns the lowest target round.
// Every load that does not depend on another goes out first -- the round's weak
// columns (WPF passes of WS-lane entries), the frontier's strong degrees and the
// first group of rows -- so a round costs a few memory latencies, not one per
// loop step.  Edges: the frontier's strong degrees from sdeg (2 B per vertex, the
// rows' exact popcount) plus one per followed weak edge.  Rows: GRP 16-B chunks
// per thread in flight; with Ur (round r's union of rows, from the round
// summaries) a wave stops loading rows once the OR of what it has read equals Ur
// -- no further row can add a bit.  wc0/wc1: the round's weak-column range when
// the caller prefetched it (-1: read it here).  row_bytes counts bytes read.
// dreg: weak columns of larger delta and far edges are not followed (Q_REGULAR); the
// weak edges counted are every weak edge of the frontier's vertices (their weak degree,
// exceptions included: the edge totals are the reference's).
template <int WS, int NT, bool WEAK>
__device__ __forceinline__ int expand_round(const DagView &g, int r, int bottom, const u64 *FE, u64 *ring, int depth,
                                            u64 *mask_bottom, const u64 *Ur, u64 &my_edges, u64 &my_wedges,
                                            u64 &row_bytes, int64_t wc0 = -1, int64_t wc1 = -1, u64 *tsub = nullptr,
                                            int dreg = 0x7fffffff) {
  using G = Geo<WS, NT>;
  constexpr int CW = G::CW, CPR = G::CPR, RPP = G::RPP, CPT = G::CPT, NMAX = G::NMAX;
  constexpr int GRP = CPT < 4 ? CPT : 4;  // 4 x RPP rows per step: a C4 frontier saturates in one
  constexpr int SPT = (NMAX + NT - 1) / NT;  // sources per thread for the degree sum
  static_assert(WS <= 64 && (64 % WS) == 0, "WS lanes per weak-column entry");
  constexpr int EPP = NT / WS;  // weak-column entries per pass
  constexpr int WPF = 4;        // weak passes loaded up front
  const int tid = threadIdx.x, lane = tid & 63, j = tid % CPR, n = g.n, dmask = depth - 1;
  const int w = tid % WS, gbase = lane & ~(WS - 1);
  int lowmin = 0x7fffffff;
  DR_TT(u64 t0 = wall_clock64(); (void)t0;)
  // ---- independent loads first ----
  uint32_t c0 = 0, c1 = 0;
  u64 wv[WPF];
  uint32_t wk[WPF];
  if constexpr (WEAK) {
    c0 = wc0 >= 0 ? (uint32_t)wc0 : g.wc_roff[r];
    c1 = wc1 >= 0 ? (uint32_t)wc1 : g.wc_roff[r + 1];
#pragma unroll
    for (int p = 0; p < WPF; p++) {
      const uint32_t jj = c0 + (uint32_t)(p * EPP + tid / WS);
      wv[p] = jj < c1 ? g.wc_rows[(size_t)jj * WS + w] : 0ULL;
      wk[p] = jj < c1 ? g.wc_key[jj] : 0u;
    }
  }
  const uint16_t *deg = g.sdeg + (size_t)r * n;
  const uint16_t *wdg = g.wdeg + (size_t)r * n;
  uint16_t dg[SPT], dw[SPT];  // loaded now, used after the rows: no wait here
  uint32_t din = 0;  // bit k: source tid*SPT+k is in the frontier
#pragma unroll
  for (int k = 0; k < SPT; k++) {
    const int s = tid * SPT + k;
    const bool in = s < n && ((FE[s >> 6] >> (s & 63)) & 1ULL);
    din |= (in ? 1u : 0u) << k;
    dg[k] = in ? deg[s] : (uint16_t)0;
    dw[k] = (WEAK && in) ? wdg[s] : (uint16_t)0;
  }
  const u64 *rows = g.strong + (size_t)r * n * WS;
  u64 a0 = 0, a1 = 0;
  u64 u0 = ~0ULL, u1 = ~0ULL;  // never equal to a partial OR when Ur is absent
  if (Ur) {
    u0 = Ur[CW * j];
    u1 = CW == 2 ? Ur[CW * j + 1] : 0ULL;
  }
  DR_TT(if (tsub && tid == 0) { const u64 t = wall_clock64(); tsub[0] += t - t0; t0 = t; })
  // ---- strong rows until the OR saturates ----
#pragma unroll 1
  for (int p0 = 0; p0 < CPT; p0 += GRP) {
    if ((tid / CPR) + p0 * RPP - (tid & ~63) / CPR >= n) break;  // wave-uniform: rows of this wave done
    u64 v0[GRP], v1[GRP];
#pragma unroll
    for (int p = 0; p < GRP; p++) {
      const int s = tid / CPR + (p0 + p) * RPP;
      v0[p] = 0;
      v1[p] = 0;
      if (s < n && ((FE[s >> 6] >> (s & 63)) & 1ULL)) {
        if constexpr (CW == 2) {
          const ulonglong2 x = *reinterpret_cast<const ulonglong2 *>(rows + (size_t)s * WS + 2 * j);
          v0[p] = x.x;
          v1[p] = x.y;
        } else {
          v0[p] = rows[s];
        }
        row_bytes += CW * 8;
      }
    }
#pragma unroll
    for (int p = 0; p < GRP; p++) {
      a0 |= v0[p];
      a1 |= v1[p];
    }
    if (Ur) {  // the wave's OR so far (lanes of one chunk class j) against U_r
      u64 r0 = a0, r1 = a1;
#pragma unroll
      for (int off = CPR; off < 64; off <<= 1) {
        r0 |= __shfl_xor(r0, off);
        if (CW == 2) r1 |= __shfl_xor(r1, off);
      }
      if (__ballot(r0 != u0 || r1 != u1) == 0ULL) break;  // saturated: no row can add a bit
    }
  }
  DR_TT(if (tsub && tid == 0) { const u64 t = wall_clock64(); tsub[1] += t - t0; t0 = t; })
  // chunk j = lane mod CPR: fold each row's lanes of class j, then one LDS OR per row
  if constexpr (CPR < 16) {
    a0 = row_or_stride<CPR>(a0);
    if constexpr (CW == 2) a1 = row_or_stride<CPR>(a1);
  }
  if ((lane & 15) < CPR) {
    u64 *dst = ring + (size_t)((r - 1) & dmask) * WS + (lane & 15) * CW;
    if (a0) atomicOr(dst, a0);
    if (CW == 2 && a1) atomicOr(dst + 1, a1);
  }
#pragma unroll
  for (int k = 0; k < SPT; k++) {
    my_edges += dg[k];
    if constexpr (WEAK) my_wedges += dw[k];
  }
  row_bytes += 2 * (u64)__popc(din);
  DR_TT(if (tsub && tid == 0) { const u64 t = wall_clock64(); tsub[2] += t - t0; t0 = t; })
  if constexpr (!WEAK) return lowmin;
  // ---- weak columns: lane group of entry jj (WS lanes, lane w owns word w)
  // ANDs the entry's source row with the frontier; a hit sets the target bit
  // (one atomic per entry); the popcount is the number of weak edges followed
  const u64 fe = FE[w];
  const u64 gm = WS >= 64 ? ~0ULL : (((1ULL << WS) - 1ULL) << gbase);
  auto column = [&](u64 row, uint32_t key) {
    const u64 v = row & fe;
    const u64 bal = __ballot(v != 0ULL);
    if (w == 0 && (bal & gm) && (int)(key >> 11) <= dreg) {
      const int delta = (int)(key >> 11), ts = (int)(key & 2047u), tr = r - delta;
      if (tr >= bottom) {
        const u64 bit = 1ULL << (ts & 63);
        lowmin = min(lowmin, tr);
        if (delta < depth) atomicOr(ring + (size_t)(tr & dmask) * WS + (ts >> 6), bit);
        else atomicOr(mask_bottom + (int64_t)(tr - bottom) * WS + (ts >> 6), bit);
      }
    }
  };
#pragma unroll
  for (int p = 0; p < WPF; p++)
    if (c0 + (uint32_t)(p * EPP) < c1) column(wv[p], wk[p]);  // wave-uniform
  // the rest CB passes at a time: their loads in flight together (a deep window's
  // round holds ~1000 columns: one load latency per pass had made the weak columns
  // ~90 us of each partial round at c4-deep)
  constexpr int CB = 8;
  for (uint32_t j0 = c0 + (uint32_t)(WPF * EPP); j0 < c1; j0 += CB * EPP) {
    u64 rv[CB];
    uint32_t kv[CB];
#pragma unroll
    for (int q = 0; q < CB; q++) {
      const uint32_t jj = j0 + (uint32_t)(q * EPP) + (uint32_t)(tid / WS);
      rv[q] = jj < c1 ? g.wc_rows[(size_t)jj * WS + w] : 0ULL;
      kv[q] = jj < c1 ? g.wc_key[jj] : 0u;
    }
#pragma unroll
    for (int q = 0; q < CB; q++)
      if (j0 + (uint32_t)(q * EPP) < c1) column(rv[q], kv[q]);  // wave-uniform
  }
  const uint32_t f0 = g.far_roff[r], f1 = dreg > 1023 ? g.far_roff[r + 1] : f0;
  for (uint32_t e = f0 + tid; e < f1; e += NT) {
    const u64 y = g.far[e];
    const int own = (int)(y >> 32);
    const uint32_t t = (uint32_t)y;
    if (!((FE[own >> 6] >> (own & 63)) & 1ULL)) continue;
    const int tr = (int)(t >> 11), ts = (int)(t & 2047u);
    if (tr < bottom) continue;
    const u64 bit = 1ULL << (ts & 63);
    if (r - tr < depth) atomicOr(ring + (size_t)(tr & dmask) * WS + (ts >> 6), bit);
    else atomicOr(mask_bottom + (int64_t)(tr - bottom) * WS + (ts >> 6), bit);
    lowmin = min(lowmin, tr);
  }
  DR_TT(if (tsub && tid == 0) { const u64 t = wall_clock64(); tsub[3] += t - t0; t0 = t; })
  return lowmin;
}

// Per-round data that does not depend on the frontier, prefetched one round
// ahead by lane w < WS (word w): presence, canonical word, U and the first
// DDR weak-summary slots (later slots are read when used).
constexpr int DDR = 3;
struct RoundWords {
  u64 P, K, U, WU[DDR];
  uint32_t C0, C1;  // the round's weak-column range
  u64 SD;           // the round's strong-degree sum (summary rounds' edge count)
  uint32_t NW0, NW1;  // weak_roff[r], weak_roff[r+1]: the round's weak edges = NW1 - NW0, subtracted where
                      // used (a subtraction here waits on every load in flight, prefetches included)
  __device__ __forceinline__ uint32_t NW() const { return NW1 - NW0; }
};

template <int WS, bool MERGE, bool SUMMARY, bool WEAK>
__device__ __forceinline__ void load_round(const DagView &g, const MemoView &mv, int r, RoundWords &x) {
  const int w = threadIdx.x;
  x.P = g.present[(size_t)r * WS + w];
  if constexpr (WEAK) {
    x.C0 = g.wc_roff[r];
    x.C1 = g.wc_roff[r + 1];
  }
  if constexpr (MERGE) x.K = mv.K[(size_t)r * WS + w];
  if constexpr (SUMMARY) {
    if (w == 0) {
      x.SD = mv.SD[r];
      if constexpr (WEAK) {
        x.NW0 = g.weak_roff[r];
        x.NW1 = g.weak_roff[r + 1];
      }
    }
    x.U = mv.U[(size_t)r * WS + w];
    if constexpr (WEAK) {
#pragma unroll
      for (int d = 0; d < DDR; d++) x.WU[d] = d < mv.dd ? mv.WU[((size_t)r * mv.dd + d) * WS + w] : 0ULL;
    }
  }
}

// full round r: ring[r-1] |= U_r, ring[r-d-2] |= WU_r[d] (lane w < WS owns word w)
// Threads 0 .. NTH-1 call it (wave 0: NTH = 64; a whole workgroup: NTH = its size);
// x is thread w's prefetched words for w < WS.
template <int WS, bool WEAK, int NTH = 64>
__device__ __forceinline__ void expand_summary_t(const MemoView &mv, const RoundWords &x, int r, int bottom,
                                                 u64 *ring, int dmask) {
  const int lane = threadIdx.x;
  if (lane < WS) {
    ring[(size_t)((r - 1) & dmask) * WS + lane] |= x.U;
    if constexpr (WEAK) {
#pragma unroll
      for (int d = 0; d < DDR; d++) {
        const int tr = r - d - 2;
        if (d < mv.dd && tr >= bottom) ring[(size_t)(tr & dmask) * WS + lane] |= x.WU[d];
      }
    }
  }
  if constexpr (!WEAK) return;
  // deeper slots (a deep window: dd up to 254) over all NTH threads -- NTH/WS per
  // word, each taking every (NTH/WS)-th slot -- B loads in flight per thread, then
  // their ORs (every (slot, word) is its own ring word).  Wave 0 alone (NTH = 64):
  // B = 24, one round trip per round up to dd = 99 at WS = 16 (8 took three at dd = 79)
  constexpr int LPW = WS >= NTH ? 1 : NTH / WS;
  constexpr int B = (NTH == 64 && WS >= 16) ? 24 : 8;  // (24 at WS = 4 took the WS = 4 sweeps from 4 to 3 waves/SIMD)
  const int w = lane % WS, j = lane / WS;
  const int dlim = min(mv.dd, r - 1 - bottom);  // tr = r - d - 2 >= bottom
  if (j >= LPW) return;
  for (int d0 = DDR + j; d0 < dlim; d0 += B * LPW) {
    u64 v[B];
#pragma unroll
    for (int q = 0; q < B; q++) {
      const int d = d0 + q * LPW;
      v[q] = d < dlim ? mv.WU[((size_t)r * mv.dd + d) * WS + w] : 0ULL;
    }
#pragma unroll
    for (int q = 0; q < B; q++) {
      const int d = d0 + q * LPW;
      if (d < dlim) ring[(size_t)((r - d - 2) & dmask) * WS + w] |= v[q];
    }
  }
}
// The deep slots of a full round preloaded one round ahead (k_canon's walk): thread
// t holds slots DDR + t/WS + q*LPW, q < PF, of word t % WS (PF = 4 covers dd <= 66 at
// WS = 16, NT = 512); later slots load when used.  Threads 0 .. NTH-1 call both.
template <int WS, int NTH, int PF>
__device__ __forceinline__ void deep_slots_load(const MemoView &mv, int r, int bottom, u64 (&v)[PF]) {
  constexpr int LPW = WS >= NTH ? 1 : NTH / WS;
  const int w = threadIdx.x % WS, j = threadIdx.x / WS;
  const int dlim = min(mv.dd, r - 1 - bottom);
#pragma unroll
  for (int q = 0; q < PF; q++) {
    const int d = DDR + j + q * LPW;
    v[q] = (j < LPW && d < dlim) ? mv.WU[((size_t)r * mv.dd + d) * WS + w] : 0ULL;
  }
}
template <int WS, int NTH, int PF>
__device__ __forceinline__ void expand_summary_pre(const MemoView &mv, const RoundWords &x, int r, int bottom,
                                                   u64 *ring, int dmask, const u64 (&v)[PF]) {
  const int lane = threadIdx.x;
  if (lane < WS) {
    ring[(size_t)((r - 1) & dmask) * WS + lane] |= x.U;
#pragma unroll
    for (int d = 0; d < DDR; d++) {
      const int tr = r - d - 2;
      if (d < mv.dd && tr >= bottom) ring[(size_t)(tr & dmask) * WS + lane] |= x.WU[d];
    }
  }
  constexpr int LPW = WS >= NTH ? 1 : NTH / WS;
  const int w = lane % WS, j = lane / WS;
  if (j >= LPW) return;
  const int dlim = min(mv.dd, r - 1 - bottom);
#pragma unroll
  for (int q = 0; q < PF; q++) {
    const int d = DDR + j + q * LPW;
    if (d < dlim) ring[(size_t)((r - d - 2) & dmask) * WS + w] |= v[q];
  }
  for (int d = DDR + j + PF * LPW; d < dlim; d += LPW)  // beyond the preloaded slots
    ring[(size_t)((r - d - 2) & dmask) * WS + w] |= mv.WU[((size_t)r * mv.dd + d) * WS + w];
}
template <int WS, bool WEAK>
__device__ __forceinline__ void expand_summary(const MemoView &mv, const RoundWords &x, int r, int bottom, u64 *ring,
                                               int dmask) {
  expand_summary_t<WS, WEAK, 64>(mv, x, r, bottom, ring, dmask);
}

// ---------------------------------------------------------------------------
// k_sweep: one workgroup per query (or, with seq != 0, one workgroup walking all
// queries in order -- paper-mode dedup needs that order).  MODE (compile time):
//   SW_WEAK   follow weak edges too (path(.., false), orderVertices)
//   SW_CHAIN  waveReady's leader chain: restart at every reachable leader
//   SW_PRUNE  paper-mode orderVertices: skip delivered vertices
//   SW_MERGE  stop once the frontier equals the canonical cone K on dmax
//             consecutive rounds (the cone below is K)
// Per round r (top .. bottom):
//   phase A (wave 0, lane w < WS): F[w] = ring[r][w] (| far-scatter mask word)
//           (& ~delivered); chain restart; masks/delivered writes; ring slot freed;
//           full / merge tests.  Round r-1's frontier-independent words are
//           prefetched meanwhile.
//   phase B (all): full round with Q_SHORTCUT -> summaries; else strong rows of
//           F -> ring[r-1] and weak edges of F -> ring[r'].
// LDS: F[WS] | FE[WS] | ring[depth][WS] | ctl (int[8]) | edges (u64[2]).
// ---------------------------------------------------------------------------
// SW_FAST (with SW_WEAK | SW_MERGE): the fast merge of Q_FAST queries compiled in (its second
// ring costs registers: a launch of queries without Q_FAST keeps the plain merge sweep)
enum : int { SW_WEAK = 1, SW_CHAIN = 2, SW_PRUNE = 4, SW_MERGE = 8, SW_FAST = 16 };

// exclusive scan over one workgroup; s = NT/64 scratch slots; every thread calls
template <int NT, class T>
__device__ __forceinline__ T block_scan_excl(T v, T *s, T &total) {
  constexpr int NW = NT / 64;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  T x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const T y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  if (lane == 63) s[wid] = x;
  __syncthreads();
  if (wid == 0) {
    T t = lane < NW ? s[lane] : T(0);
#pragma unroll
    for (int off = 1; off < NW; off <<= 1) {
      const T y = __shfl_up(t, off);
      if (lane >= off) t += y;
    }
    if (lane < NW) s[lane] = t;
  }
  __syncthreads();
  const T base = wid ? s[wid - 1] : T(0);
  total = s[NW - 1];
  __syncthreads();
  return base + x - v;
}

template <int NT, int MAXP = 16>
__device__ __forceinline__ void canon_prefix_block(int T, const u64 *__restrict__ a, const u64 *__restrict__ b,
                                                   u64 *__restrict__ A, u64 *__restrict__ B,
                                                   uint32_t *__restrict__ rbase) {
  __shared__ u64 s[NT / 64];
  const int tid = threadIdx.x;
  const int n = T + 1, per = (n + NT - 1) / NT;
  const int ra = tid * per, rb = min(n, ra + per);
  if (per <= MAXP) {  // block-uniform: every load in flight at once, values kept in registers
    u64 va[MAXP], vb[MAXP], sa = 0, sb = 0;
#pragma unroll
    for (int j = 0; j < MAXP; j++) {
      const int r = ra + j;
      const bool in = r >= 1 && r < rb;
      va[j] = in ? a[r] : 0ULL;
      vb[j] = in && b ? b[r] : 0ULL;
      sa += va[j];
      sb += vb[j];
    }
    u64 ta, tb;
    u64 xa = block_scan_excl<NT>(sa, s, ta);
    u64 xb = b ? block_scan_excl<NT>(sb, s, tb) : 0ULL;
#pragma unroll
    for (int j = 0; j < MAXP; j++) {
      const int r = ra + j;
      if (r >= rb) break;
      if (rbase) rbase[r] = (uint32_t)xa;
      xa += va[j];
      xb += vb[j];
      A[r] = xa;
      if (b) B[r] = xb;
    }
    return;
  }
  // more rounds per thread (C3: 10 000 rounds, 20 per thread at NT = 512): eight
  // rounds' loads in flight at a time, in both passes (one load at a time left the
  // thread ~20 memory latencies deep)
  constexpr int CH = 8;
  u64 sa = 0, sb = 0;
  for (int r0 = ra; r0 < rb; r0 += CH) {
    u64 va[CH], vb[CH];
#pragma unroll
    for (int j = 0; j < CH; j++) {
      const int r = r0 + j;
      const bool in = r >= 1 && r < rb;
      va[j] = in ? a[r] : 0ULL;
      vb[j] = in && b ? b[r] : 0ULL;
    }
#pragma unroll
    for (int j = 0; j < CH; j++) {
      sa += va[j];
      sb += vb[j];
    }
  }
  u64 ta, tb;
  u64 xa = block_scan_excl<NT>(sa, s, ta);
  u64 xb = b ? block_scan_excl<NT>(sb, s, tb) : 0ULL;  // b is uniform
  for (int r0 = ra; r0 < rb; r0 += CH) {
    u64 va[CH], vb[CH];
#pragma unroll
    for (int j = 0; j < CH; j++) {
      const int r = r0 + j;
      const bool in = r >= 1 && r < rb;
      va[j] = in ? a[r] : 0ULL;
      vb[j] = in && b ? b[r] : 0ULL;
    }
#pragma unroll
    for (int j = 0; j < CH; j++) {
      const int r = r0 + j;
      if (r >= rb) break;
      if (rbase) rbase[r] = (uint32_t)xa;
      xa += va[j];
      xb += vb[j];
      A[r] = xa;
      if (b) B[r] = xb;
    }
  }
}

// plan[] slots (int32, device)
// (PL_NLIVE: the delivery queries a replay swept -- the static table's live ones -- for the
// sweep statistics; PL_NQD counts the launched table)
enum : int { PL_NTASK = 0, PL_NQC = 1, PL_NPUSH = 2, PL_CAPERR = 3, PL_NQD = 4, PL_NDESC = 5, PL_NLIVE = 6, PL_N = 8 };
// header written to host memory by k_plan_final (u64)
// (PH_MINSTOP .. PH_PROBE + 23: a sliced context's outputs, dr_slice_result)
enum : int {
  PH_NPUSH = 0, PH_CHAIN_E = 1, PH_DELIVER_E = 2, PH_PARTIAL = 3, PH_ROWS = 4, PH_WEAK = 5, PH_SHORT = 6,
  PH_NQD = 7, PH_NSEG = 8, PH_CAPERR = 9, PH_MINSTOP = 10, PH_OWN_CE = 11, PH_UPBAD = 12, PH_PROBE = 16, PH_N = 40
};
constexpr int kMaxProbe = 8;

// Host-visible output region of a planned replay (packed, one copy back).
struct FinalOut {
  uint8_t *commit;
  int32_t *vcount;
  uint32_t *push_off;
  int32_t *push_wave;
  u64 *pc, *pd, *pe, *hdr;
};

// Inputs of the planned replay's last pass (replay_final_block).
struct FinalArgs {
  int T, nw;
  const u64 *RG, *CE;  // canonical per-round digests and edges
  u64 *Gc, *Ec;        // their prefixes (k_own_emit's last workgroup)
  const u64 *Cc;
  const uint8_t *commit;
  const int32_t *vcount;
  const uint32_t *push_off;
  const int32_t *push_wave, *pop_q, *pop_cur;
  const SweepQuery *dq;
  const int32_t *stops;
  const u64 *dedges, *cedges, *dstats;
  const int32_t *nseg, *plan;
  const int32_t *firstpop;  // PAPER (k_paper_*): the first pop of each query; later pops deliver nothing
  const u64 *qedges;        // PAPER: the query's delivered edges
  FinalOut o;
  // a sliced context (dr_set_slice; own_w0 = 0: none): the owned commits' min pop stop
  // and chain edges (task_wave / task_q: k_plan_chains' tasks), C, G, E at the probes
  const int32_t *task_wave, *task_q;
  const int32_t *upbad;  // k_verify_up's count (null: no upward edges checked)
  int32_t own_w0, nprobe;
  int32_t probe[kMaxProbe];
  // the canonical walk's lowest round (nseg + 1): the final pass first rescans the G, E
  // prefixes from there (the speculative prefixes are exact below it; null: no rescan here)
  const int32_t *lo_w;
};

// The planned replay's per-query emission outputs (k_own_emit, k_paper_emit):
// the count and order-sensitive digest of what each query's first pop delivers
// beyond the canonical prefix (REF: its own rounds above the cut).
struct EmitArgs {
  const uint32_t *slot_off;
  const uint16_t *slot_src;
  const u64 *Cc;  // canonical prefix counts (k_canon)
  u64 *count;     // [query] delivered vertex count (REF: own rounds)
  u64 *digest;    // [query] own-round digest terms
  int32_t *cut;   // [query] the canonical rounds are 1..cut (-1: none)
  FinalArgs fin;
};

// One wave emits round y: the delivered slots (source bit set in mw, lane w
// holding word w) in insertion order, vertex k at position pos + rank.  Returns
// this lane's share of the digest sum.
// SPL: slots per lane per pass (16 in the sweep would cost it a wave per SIMD of occupancy).
// DEG: also add the strong + weak degrees of the delivered vertices to *edges
// (this lane's share; sdeg/wdeg indexed [round][source-1], row length n).
// wave_emit_slots: the same with the round's slot range [sa, sb) already loaded.
// first_only (PAPER, slot_rep non-null): a repeated id's later slots deliver nothing.
template <int WS, int SPL = 8, bool DEG = false>
__device__ __forceinline__ u64 wave_emit_slots(const uint16_t *__restrict__ slot_src, int y, uint32_t sa,
                                               uint32_t sb, u64 mw, u64 pos,
                                               const uint16_t *__restrict__ sdeg = nullptr,
                                               const uint16_t *__restrict__ wdeg = nullptr, int n = 0,
                                               u64 *edges = nullptr, const uint8_t *__restrict__ first_only = nullptr,
                                               int koff = 0) {
  const int lane = threadIdx.x & 63;
  u64 dg = 0;
  for (uint32_t c0 = sa; c0 < sb; c0 += 64 * SPL) {
    const uint32_t i0 = c0 + (uint32_t)lane * SPL;
    int src[SPL];
#pragma unroll
    for (int j = 0; j < SPL; j++) src[j] = i0 + j < sb ? (int)slot_src[i0 + j] : 0;
    if (first_only)
#pragma unroll
      for (int j = 0; j < SPL; j++)
        if (i0 + j < sb && first_only[i0 + j]) src[j] = 0;
    uint32_t bits = 0;
#pragma unroll
    for (int j = 0; j < SPL; j++) {
      const int s = src[j] - 1;
      const u64 w = __shfl(mw, s >= 0 ? (s >> 6) & (WS - 1) : 0);
      if (s >= 0 && ((w >> (s & 63)) & 1ULL)) bits |= 1u << j;
    }
    const int cnt = __popc(bits);
    int x = cnt;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int yv = __shfl_up(x, off);
      if (lane >= off) x += yv;
    }
    const int total = __shfl(x, 63);
    u64 k = pos + (u64)(x - cnt);
#pragma unroll
    for (int j = 0; j < SPL; j++) {
      if (!((bits >> j) & 1u)) continue;
      dg += digest_term((uint32_t)(y + koff), (uint32_t)src[j], k);
      if constexpr (DEG) {
        const size_t at = (size_t)y * n + (src[j] - 1);
        *edges += (u64)sdeg[at] + wdeg[at];
      }
      k++;
    }
    pos += (u64)total;
  }
  return dg;
}
template <int WS, int SPL = 8, bool DEG = false>
__device__ __forceinline__ u64 wave_emit_round(const uint32_t *__restrict__ slot_off,
                                               const uint16_t *__restrict__ slot_src, int y, u64 mw, u64 pos,
                                               const uint16_t *__restrict__ sdeg = nullptr,
                                               const uint16_t *__restrict__ wdeg = nullptr, int n = 0,
                                               u64 *edges = nullptr, const uint8_t *__restrict__ first_only = nullptr,
                                               int koff = 0) {
  return wave_emit_slots<WS, SPL, DEG>(slot_src, y, slot_off[y], slot_off[y + 1], mw, pos, sdeg, wdeg, n, edges,
                                       first_only, koff);
}



// The planned replay's last pass (k_replay_final, after k_own_emit or
// k_paper_emit): per pop, the canonical terms at its
// query's cut (C, G) and merge round (E) plus the query's own-round count,
// digest and edges (what k_plan_emit + k_emit_ids + k_plan_final did in three
// launches), the commits and pushes, and the totals, into the packed output
// region.  Every pop of a replay has cur_round >= top (a leader is popped at a
// wave's end, above its own round): checked, a violation reports PH_CAPERR = 3.
template <int NT, int J, class LA, class LB>
__device__ __forceinline__ void canon_prefix_gen(int r0, int T, u64 ca, u64 cb, LA la, LB lb, u64 *__restrict__ A,
                                                 u64 *__restrict__ B);
template <int NT>
__device__ void replay_final_block(const FinalArgs &f, const EmitArgs &ea) {
  __shared__ u64 acc[8];
  __shared__ int s_bad;
  const int tid = threadIdx.x;
  if (f.lo_w) {  // (block-uniform) G, E from the walk's lowest round up (DR_OPT_FUSE bit 32)
    const int lw = *f.lo_w;
    if (lw <= f.T)
      canon_prefix_gen<NT, 8>(
          lw, f.T, lw >= 1 ? f.Gc[lw - 1] : 0ULL, lw >= 1 ? f.Ec[lw - 1] : 0ULL, [&](int r) { return f.RG[r]; },
          [&](int r) { return f.CE[r]; }, f.Gc, f.Ec);
    __syncthreads();
  }
  if (tid < 8) acc[tid] = 0;
  if (tid == 0) s_bad = 0;
  const int caperr = f.plan[PL_CAPERR];
  const int64_t np = caperr ? 0 : f.plan[PL_NPUSH];
  const int nqc = f.plan[PL_NQC], nqd = f.plan[PL_NQD];
  u64 de = 0, ce = 0, st[4] = {0, 0, 0, 0};
  bool bad = false;
  __shared__ int s_minstop;
  __shared__ u64 s_owce;
  if (tid == 0) {
    s_minstop = INT_MAX;
    s_owce = 0;
  }
  // a slice: the pops of owned commits start at push_off[own_w0 - 1]
  const int64_t pown = f.own_w0 > 0 && !caperr ? (int64_t)f.push_off[f.own_w0 - 1] : INT64_MAX;
  int minstop = INT_MAX;
  // every load of a pop before any store (the stores could alias for the compiler)
  for (int64_t p = tid; p < np; p += NT) {
    const int q = f.pop_q[p];
    const int cur = f.pop_cur[p], pw = f.push_wave[p];
    const int stop = f.stops[q], cut = ea.cut[q], top = f.dq[q].top;
    u64 c = ea.count[q], d = ea.digest[q], e = f.dedges[q];
    if (f.firstpop) {  // PAPER: everything the query delivers goes to its first pop
      const bool mine = f.firstpop[q] == (int32_t)p;
      c = mine ? c : 0ULL;
      d = mine ? d : 0ULL;
      e = mine ? f.qedges[q] : 0ULL;
    } else {
      if (cut >= 0) {
        c += f.Cc[cut];
        d += f.Gc[cut];
      }
      if (stop >= 0) e += f.Ec[stop];  // the sweep counted the edges of rounds above stop
    }
    bad |= cur < top;
    if (p >= pown) minstop = min(minstop, stop);
    f.o.push_wave[p] = pw;
    f.o.pc[p] = c;
    f.o.pd[p] = d;
    f.o.pe[p] = e;
    de += e;
  }
  for (int q = tid; q < nqc; q += NT) ce += f.cedges[q];
  u64 owce = 0;
  if (f.own_w0 > 0) {
    const int ntask = f.plan[PL_NTASK];
    for (int t = tid; t < ntask; t += NT) {
      const int q = f.task_q[t];
      if (q >= 0 && f.task_wave[t] >= f.own_w0) owce += f.cedges[q];
    }
  }
  for (int q = tid; q < nqd; q += NT)
#pragma unroll
    for (int k = 0; k < 4; k++) st[k] += f.dstats[4 * q + k];
  for (int w = tid; w < f.nw; w += NT) {
    const uint8_t cm = f.commit[w];
    const int32_t vc = f.vcount[w];
    f.o.commit[w] = cm;
    f.o.vcount[w] = vc;
  }
  if (!caperr)
    for (int w = tid; w <= f.nw; w += NT) f.o.push_off[w] = f.push_off[w];
  de = wave_sum(de);
  ce = wave_sum(ce);
#pragma unroll
  for (int k = 0; k < 4; k++) st[k] = wave_sum(st[k]);
  __syncthreads();  // acc, s_bad initialised
  if ((tid & 63) == 0) {
    atomicAdd(&acc[0], de);
    atomicAdd(&acc[1], ce);
#pragma unroll
    for (int k = 0; k < 4; k++) atomicAdd(&acc[2 + k], st[k]);
  }
  if (bad) s_bad = 1;
  if (f.own_w0 > 0) {
    owce = wave_sum(owce);
    if ((tid & 63) == 0 && owce) atomicAdd(&s_owce, owce);
    if (minstop != INT_MAX) atomicMin(&s_minstop, minstop);
  }
  if (tid < f.nprobe) {
    const int r = f.probe[tid];
    f.o.hdr[PH_PROBE + tid] = f.Cc[r];
    f.o.hdr[PH_PROBE + kMaxProbe + tid] = f.Gc[r];
    f.o.hdr[PH_PROBE + 2 * kMaxProbe + tid] = f.Ec[r];
  }
  __syncthreads();
  if (tid == 0) {
    u64 *h = f.o.hdr;
    h[PH_MINSTOP] = (u64)(int64_t)s_minstop;
    h[PH_UPBAD] = f.upbad ? (u64)*f.upbad : 0ULL;
    h[PH_OWN_CE] = s_owce;
    h[PH_NPUSH] = (u64)f.plan[PL_NPUSH];
    h[PH_CHAIN_E] = acc[1];
    h[PH_DELIVER_E] = acc[0];
    for (int k = 0; k < 4; k++) h[PH_PARTIAL + k] = acc[2 + k];
    h[PH_NQD] = (u64)f.plan[PL_NLIVE];
    h[PH_NSEG] = (u64)(int64_t)*f.nseg;
    h[PH_CAPERR] = (u64)(caperr ? caperr : s_bad ? 3 : 0);
  }
}

// The sweep of query bidx (seq: every query in turn), the body of k_sweep and of the
// fused canonical-walk + chains launch (k_canon_chains).
template <int WS, int NT, int MODE>
__device__ __forceinline__ void sweep_body(const int bidx, DagView g, MemoView mv, const SweepQuery *__restrict__ qs,
                                           int nq, int seq, int depth_log2,
                                           u64 *__restrict__ masks, u64 *__restrict__ dlv,
                                           int32_t *__restrict__ push_out,
                                           int32_t *__restrict__ push_n,
                                           u64 *__restrict__ edges_out,
                                           u64 *__restrict__ wedges_out,
                                           uint8_t *__restrict__ hit_out,
                                           int32_t *__restrict__ stop_out,
                                           u64 *__restrict__ stats_out, const int *__restrict__ nq_dev,
                                           uint32_t *__restrict__ rcnt, const PopMark pm) {
  if (nq_dev) {  // grid sized by an upper bound, count on the device (planned replay)
    const int m = *nq_dev;
    if (seq) nq = m;
    else if (bidx >= m) return;
  }
  constexpr bool WEAK = MODE & SW_WEAK, CHAIN = MODE & SW_CHAIN, PRUNE = MODE & SW_PRUNE,
                 MERGE = MODE & SW_MERGE, FASTM = (MODE & SW_FAST) && WEAK && MERGE;
  constexpr u64 WMASK = WS >= 64 ? ~0ULL : ((1ULL << WS) - 1ULL);  // lanes owning a frontier word
  extern __shared__ __attribute__((aligned(16))) u64 smem[];
  u64 *F = smem;                // WS: frontier (reached ids, dangling included)
  u64 *FE = smem + WS;          // WS: F & present (the vertices that expand)
  u64 *ring = smem + 2 * WS;    // depth * WS
  const int depth = 1 << depth_log2, dmask = depth - 1;
  // ctl: [0] low water [1] round [2] status (0 partial, 1 stop) [3] merged [4] stop round
  //      [5] [6] the partial round's weak-column range
  int *s_ctl = reinterpret_cast<int *>(ring + (size_t)depth * WS);
  u64 *s_edges = reinterpret_cast<u64 *>(s_ctl + 8);  // [0] all edges, [1] weak edges, [2] row bytes
  // Q_FAST: K's contributions pending for the rounds below, from the rounds the sweep has
  // passed (depth x WS, after the control words: sweep_lds(dl, true))
  u64 *kring = reinterpret_cast<u64 *>(reinterpret_cast<char *>(smem) + (size_t)(2 * WS + depth * WS) * 8 + 64);
  const int tid = threadIdx.x;
  const bool w0 = tid < 64;     // wave 0 runs phase A and every summary round
  const bool act = tid < WS;    // lane w owns frontier word w

  const int qa = seq ? 0 : bidx;
  const int qb = seq ? nq : bidx + 1;
  for (int qi = qa; qi < qb; qi++) {
    const SweepQuery q = qs[qi];
    if (!CHAIN && pm.commit && !pm.live(q.top)) {  // (block-uniform) a wave nobody pops
      if (stats_out && threadIdx.x < 4) stats_out[4 * qi + threadIdx.x] = 0;
      continue;
    }
    const bool has_masks = q.flags & Q_MASKS;
    const bool shortcut = q.flags & Q_SHORTCUT;
    const int dreg = (q.flags & Q_REGULAR) ? mv.dreg : 0x7fffffff;
    const bool fast = FASTM && shortcut && (q.flags & Q_FAST) && mv.dd <= DDR;
    for (int i = tid; i < depth * WS; i += NT) {
      ring[i] = 0;
      if (FASTM && fast) kring[i] = 0;
    }
    if (tid == 0) {
      s_ctl[0] = q.top; s_ctl[1] = q.top; s_ctl[2] = 0; s_ctl[3] = 0; s_ctl[4] = q.bottom;
      s_edges[0] = 0; s_edges[1] = 0; s_edges[2] = 0;
    }
    __syncthreads();
    if (tid == 0 && q.src0 >= 0)
      ring[(size_t)(q.top & dmask) * WS + (q.src0 >> 6)] = 1ULL << (q.src0 & 63);
    int npush = 0;  // thread 0
    u64 st_partial = 0, st_scan = 0, st_short = 0;  // thread 0: work counters
    DR_TT(u64 tt0 = wall_clock64(); u64 tt_a = 0, tt_b = 0, tt_pro = 0, tt_ns = 0, tt_np = 0, tt_end = 0, tt_emit = 0;
          u64 tt_sub[4] = {0, 0, 0, 0};)
    int run = 0;    // wave 0: consecutive rounds equal to K
    int kfrun = 0;  // wave 0 (Q_FAST): consecutive rounds passed whose K covers the round
    u64 my_edges = 0, my_wedges = 0, my_rowb = 0;
    RoundWords cur{}, nxt{};
    if (act) {
      if (shortcut) load_round<WS, MERGE, true, WEAK>(g, mv, q.top, cur);
      else load_round<WS, MERGE, false, WEAK>(g, mv, q.top, cur);
    }
    __syncthreads();
    int r = q.top;
    DR_TT(tt_pro = wall_clock64() - tt0;)
    for (;;) {
      // ---------- wave 0: phase A of round r; summary rounds end here ----------
      DR_TT(const u64 tta = wall_clock64();)
      if (w0) {
        for (;;) {
          if (act && r > q.bottom) {  // prefetch round r-1 (frontier-independent)
            if (shortcut) load_round<WS, MERGE, true, WEAK>(g, mv, r - 1, nxt);
            else load_round<WS, MERGE, false, WEAK>(g, mv, r - 1, nxt);
          }
          u64 f = 0, p = 0;
          if (act) {
            const int slot = (r & dmask) * WS + tid;
            f = ring[slot];
            ring[slot] = 0;
            if (FASTM && fast) kring[slot] = 0;
            u64 *mrow = has_masks ? masks + q.mask_off + (int64_t)(r - q.bottom) * WS : nullptr;
            if constexpr (WEAK && !MERGE) {
              if (has_masks) f |= ld_agent(mrow + tid);  // far weak scatters
            }
            if constexpr (PRUNE) f &= ~ld_agent(dlv + (size_t)r * WS + tid);
            p = cur.P;
          }
          int single = (r == q.top) ? q.src0 : -1;  // a round whose frontier is one known vertex
          if constexpr (CHAIN) {
            if (r < q.top && ((r - 1) & 3) == 0) {
              const int wv = (r - 1) / 4 + 1, l = g.lead[wv] - 1;  // leader of wave wv, 0-based
              const u64 fl = __shfl(f, l >> 6), pl = __shfl(p, l >> 6);
              if (((fl & pl) >> (l & 63)) & 1ULL) {  // v' present, strong_path(leader, v'): push v' (process.go:344-349)
                f = tid == (l >> 6) ? 1ULL << (l & 63) : 0ULL;
                if (tid == 0) {
                  push_out[q.out_off + npush++] = wv;
                  if (pm.pushed) pm.pushed[wv] = pm.epoch;  // (a delivery query of wave wv is live)
                }
                single = l;  // the chain restarts at v' alone
              }
            }
          }
          if (act) {
            F[tid] = f;
            FE[tid] = f & p;
            if (has_masks) masks[q.mask_off + (int64_t)(r - q.bottom) * WS + tid] = f;
            if constexpr (PRUNE) {
              if (r >= 1 && r <= q.cur_round) {
                const u64 add = f & p;
                if (add) atomicOr(dlv + (size_t)r * WS + tid, add);
              }
            }
          }
          const bool nz = (__ballot(act && f != 0ULL) & WMASK) != 0;
          const bool full = (__ballot(act && (f & p) != p) & WMASK) == 0;
          bool eq = false;
          if constexpr (MERGE) {
            eq = (__ballot(act && f != cur.K) & WMASK) == 0;
            run = eq ? run + 1 : 0;
          }
          // Q_FAST: F_r = K_r and the ring's pending words for r-1 .. r-dmax+1 equal K's
          // (the contributions of rounds r+1 .. r+dmax-1, every one covered by K: WU) -- the
          // sweep's state at r is K's, so its cone below r+1 is K's
          bool fastm = false;
          if constexpr (FASTM) {
            if (fast) {
              const bool kf = (__ballot(act && (cur.K & p) != p) & WMASK) == 0;
              if (eq && kfrun >= mv.dmax - 1 && r - mv.dmax + 1 >= max(q.bottom, 0)) {
                bool diff = false;
                if (act)
                  for (int j = 1; j < mv.dmax; j++) {
                    const size_t sl = (size_t)((r - j) & dmask) * WS + tid;
                    diff |= ring[sl] != kring[sl];
                  }
                fastm = (__ballot(diff) & WMASK) == 0;
              }
              if (kf && act)  // K_r covers the round: its contributions below are WU_r
#pragma unroll
                for (int d = 0; d < DDR; d++) {
                  const int tr = r - d - 2;
                  if (d < mv.dd && tr >= q.bottom) kring[(size_t)(tr & dmask) * WS + tid] |= cur.WU[d];
                }
              kfrun = kf ? kfrun + 1 : 0;
            }
          }
          const bool merged = MERGE && (run >= mv.dmax || fastm);
          if (FASTM && fastm && run < mv.dmax) {  // the cut is r: the canonical edges of r - dmax + 2 .. r
            u64 ce = 0;
            if (tid < mv.dmax - 1) ce = mv.CE[r - tid];
            ce = wave_sum(ce);
            if (tid == 0) my_edges += ce;
          }
          int low = s_ctl[0];
          if (nz && r - 1 < low) low = r - 1;
          const bool stop = merged || r <= q.bottom || (!nz && low >= r);
          const bool summary = !stop && shortcut && full;
          if (rcnt && has_masks) {  // |mask_r & P_r|: the emission's per-round counts
            int pc = act ? popc64(f & p) : 0;
#pragma unroll
            for (int off = 1; off < WS; off <<= 1) pc += __shfl_xor(pc, off);
            pc += dup_count<WS>(g, r, act ? f & p : 0ULL);  // REF: every slot of a reached id
            if (tid == 0) rcnt[q.mask_off / WS + (r - q.bottom)] = (uint32_t)pc;
          }
          if (stats_out && tid == 0 && !stop) {
            if (summary) st_short++;
            else { st_partial++; if (WEAK) st_scan += cur.C1 - cur.C0; }
          }
          if (summary) {  // the round is the union of its rows: apply the summaries, stay in wave 0
            expand_summary<WS, WEAK>(mv, cur, r, q.bottom, ring, dmask);  // every lane of wave 0
            if (tid == 0) {
              my_edges += cur.SD;
              if (WEAK) my_wedges += cur.NW();
            }
            low = min(low, WEAK ? r - 1 - mv.dd : r - 1);
            if (tid == 0) s_ctl[0] = low;
            DR_TT(tt_ns++;)
            cur = nxt;
            --r;
            continue;
          }
          // The query's own top round holds one vertex (its `from`), and so does a
          // chain's restart round (its pushed leader): wave 0 expands it here -- one
          // row, the round's weak-column words of that source -- instead of a
          // workgroup round (no far edges: merge sweeps run on the memo path, which
          // has none; strong-only sweeps never read them).
          if ((!PRUNE && (MERGE || !WEAK)) && !stop && single >= 0) {
            const int s0 = single;
            const bool in = (__shfl(f & p, s0 >> 6) >> (s0 & 63)) & 1ULL;  // FE = {s0}
            int lowmin = 0x7fffffff;
            if (in) {
              if (act) ring[(size_t)((r - 1) & dmask) * WS + tid] |= g.strong[((size_t)r * g.n + s0) * WS + tid];
              if (tid == 0) {
                my_edges += g.sdeg[(size_t)r * g.n + s0];
                my_rowb += WS * 8 + 2;
              }
              if constexpr (WEAK) {
                if (tid == 0) my_wedges += g.wdeg[(size_t)r * g.n + s0];  // every weak edge of the vertex
                const uint32_t c0 = (uint32_t)__shfl((int)cur.C0, 0), c1 = (uint32_t)__shfl((int)cur.C1, 0);
                for (uint32_t jj = c0 + tid; jj < c1; jj += 64) {
                  if (!((g.wc_rows[(size_t)jj * WS + (s0 >> 6)] >> (s0 & 63)) & 1ULL)) continue;
                  const uint32_t key = g.wc_key[jj];
                  const int delta = (int)(key >> 11), ts = (int)(key & 2047u), tr = r - delta;
                  if (tr < q.bottom || delta > dreg) continue;
                  const u64 bit = 1ULL << (ts & 63);
                  lowmin = min(lowmin, tr);
                  if (delta < depth) atomicOr(ring + (size_t)(tr & dmask) * WS + (ts >> 6), bit);
                  else atomicOr(masks + q.mask_off + (int64_t)(tr - q.bottom) * WS + (ts >> 6), bit);
                }
#pragma unroll
                for (int off = 1; off < 64; off <<= 1) lowmin = min(lowmin, __shfl_xor(lowmin, off));
              }
            }
            low = min(low, min(r - 1, lowmin));
            if (tid == 0) s_ctl[0] = low;
            cur = nxt;
            --r;
            continue;
          }
          if (tid == 0) {
            s_ctl[0] = low;
            s_ctl[1] = r;
            s_ctl[2] = stop ? 1 : 0;
            s_ctl[3] = merged ? 1 : 0;
            if (stop && (merged || r > q.bottom)) s_ctl[4] = (FASTM && fastm && run < mv.dmax) ? r - mv.dmax + 1 : r;
            if constexpr (WEAK) {  // the round's weak-column range, prefetched with its words
              s_ctl[5] = (int)cur.C0;
              s_ctl[6] = (int)cur.C1;
            }
          }
          break;
        }
      }
      __syncthreads();
      DR_TT(const u64 ttb = wall_clock64(); tt_a += ttb - tta;)
      r = s_ctl[1];
      if (s_ctl[2]) break;
      // ---------- all threads: rows and weak edges of partial round r ----------
      if (s_ctl[0] < r || true) {
        const int lowmin = expand_round<WS, NT, WEAK>(g, r, q.bottom, FE, ring, depth, masks + q.mask_off,
                                                      shortcut ? mv.U + (size_t)r * WS : nullptr, my_edges,
                                                      my_wedges, my_rowb, WEAK ? s_ctl[5] : -1, WEAK ? s_ctl[6] : -1,
#ifdef DR_SWEEP_TIMING
                                                      tt_sub,
#else
                                                      nullptr,
#endif
                                                      dreg);
        if (WEAK && lowmin != 0x7fffffff) atomicMin(&s_ctl[0], lowmin);
      }
      __syncthreads();
      DR_TT(tt_b += wall_clock64() - ttb; tt_np++;)
      cur = nxt;
      --r;
    }
    DR_TT(const u64 tte = wall_clock64();)
    // results
    DR_TT(tt_end = wall_clock64(); tt_emit = tt_end - tte;)
    my_edges += my_wedges;
    // one LDS atomic per wave and counter (a workgroup of same-address atomics serialises)
    my_edges = wave_sum(my_edges);
    my_wedges = wave_sum(my_wedges);
    my_rowb = wave_sum(my_rowb);
    if ((tid & 63) == 0) {
      if (my_edges) atomicAdd(&s_edges[0], my_edges);
      if (my_wedges) atomicAdd(&s_edges[1], my_wedges);
      if (my_rowb) atomicAdd(&s_edges[2], my_rowb);
    }
    __syncthreads();
    if (tid == 0) {
      if (edges_out) edges_out[qi] = s_edges[0];
      if (wedges_out) wedges_out[qi] = s_edges[1];
      if (hit_out) hit_out[qi] = q.tgt0 >= 0 ? (uint8_t)((F[q.tgt0 >> 6] >> (q.tgt0 & 63)) & 1ULL) : 0;
      if (push_n) push_n[qi] = npush;
      if (stop_out) stop_out[qi] = s_ctl[3] ? s_ctl[4] : -1 - s_ctl[4];  // >= 0 merged there; < 0 ended at -1-x
#ifdef DR_SWEEP_TIMING
      if (qi < kSweepTimingQ) {
        u64 *t = g_sweep_timing + 16 * (size_t)qi;
        t[0] = tt_pro; t[1] = tt_a; t[2] = tt_b; t[3] = wall_clock64() - tt0; t[4] = tt_ns; t[5] = tt_np;
        t[6] = (u64)q.top; t[7] = (u64)(int64_t)s_ctl[4];
        t[8] = tt_sub[0]; t[9] = tt_sub[1]; t[10] = tt_sub[2]; t[11] = tt_sub[3]; t[12] = wall_clock64() - tt_end;
        t[13] = tt0; t[14] = wall_clock64(); t[15] = tt_emit;
      }
#endif
      if (stats_out) {
        stats_out[4 * qi + 0] = st_partial;
        stats_out[4 * qi + 1] = s_edges[2];  // strong-row bytes read
        stats_out[4 * qi + 2] = st_scan;
        stats_out[4 * qi + 3] = st_short;
      }
    }
    __syncthreads();
  }
}

// Leader chains (SW_CHAIN: strong only, process.go:341-350) for n <= 64 * WS, WS <=
// 4, one wavefront per chain and every round in registers: lane l holds the WS rows
// of sources l*WS .. l*WS + WS-1 (WS * WS contiguous words), loaded PF rounds ahead
// with the round's presence and the lane's strong degrees.  A round is the OR of the
// lane's rows whose source is in F & P and one OR across the wave of WS words; a
// strong-only frontier has nothing pending below r-1, so there is no ring, no LDS and
// no barrier.  The chain sweep of k_sweep walks a long leader gap round by round in
// wave 0 with two workgroup barriers and a row read per round (C3: ~2 us a round, one
// chain the critical path of the replay).  Same outputs as k_sweep's chain mode:
// pushes, push count, edges (strong degrees of every expanded vertex), hits (no
// target: 0), stop (-1 - the round the sweep ended at).  Four chains per workgroup.
template <int WS, int PF>
__device__ __forceinline__ void chain_reg_body(const int bidx, DagView g, const SweepQuery *__restrict__ qs,
                                               const int *__restrict__ nq_dev, int32_t *__restrict__ push_out,
                                               int32_t *__restrict__ push_n, u64 *__restrict__ edges_out,
                                               u64 *__restrict__ wedges_out, uint8_t *__restrict__ hit_out,
                                               int32_t *__restrict__ stop_out, const PopMark pm) {
  static_assert(WS >= 1 && WS <= 4 && PF >= 2, "register-resident rounds");
  constexpr int RW = WS * WS;  // words of the lane's rows per round
  const int lane = threadIdx.x & 63, qi = bidx * 4 + (int)(threadIdx.x >> 6);
  if (qi >= *nq_dev) return;  // wave-uniform
  const SweepQuery q = qs[qi];
  constexpr int PB = 64;  // pushes buffered per chain
  __shared__ int32_t s_push[4][PB];
  int32_t *pbuf = s_push[threadIdx.x >> 6];
  const int n = g.n, s0 = lane * WS, wd = s0 >> 6, sh = s0 & 63;  // a lane's WS sources share a word
  u64 rows[PF][RW], P[PF][WS];
  uint32_t dg[PF][WS];
  int LD[PF];
  // Every load unconditional and unmasked: branch-free loads whose values are not
  // touched until their round lets the compiler count them (s_waitcnt vmcnt(k)) instead of
  // draining the queue (vmcnt(0)) before each round -- conditional loads, a select right
  // after each load and the wave leader read inside the loop had made every round a full
  // memory latency (C3: 46 us for the longest chain, 36 rounds).  A lane past n reads row
  // 0 and a source past n is never in F & P, so neither value is ever used.  The leader of
  // the wave starting at round r travels with the round (every lane loads it: a wave-wide
  // value must not come from a lane-divergent load).
  const int s_safe = s0 < n ? s0 : 0;
  auto load = [&](u64 (&rw)[RW], u64 (&pw)[WS], uint32_t (&dd)[WS], int &ld, int r) {
    r = max(r, 0);
    const u64 *src = g.strong + ((size_t)r * n + (size_t)s_safe) * WS;
    if constexpr (RW % 2 == 0) {
      typedef u64 u64v2 __attribute__((ext_vector_type(2)));
#pragma unroll
      for (int i = 0; i < RW; i += 2) {
        const u64v2 x = *reinterpret_cast<const u64v2 *>(src + i);
        rw[i] = x.x;
        rw[i + 1] = x.y;
      }
    } else {
#pragma unroll
      for (int i = 0; i < RW; i++) rw[i] = src[i];
    }
#pragma unroll
    for (int w = 0; w < WS; w++) pw[w] = g.present[(size_t)r * WS + w];
#pragma unroll
    for (int k = 0; k < WS; k++) dd[k] = g.sdeg[(size_t)r * n + min(s_safe + k, n - 1)];
    ld = g.lead[((r - 1) >> 2) + 1];  // (used only when r starts a wave)
  };
  u64 F[WS];
#pragma unroll
  for (int w = 0; w < WS; w++) F[w] = (q.src0 >= 0 && w == (q.src0 >> 6)) ? 1ULL << (q.src0 & 63) : 0ULL;
  int r = q.top;
#pragma unroll
  for (int k = 0; k < PF; k++) load(rows[k], P[k], dg[k], LD[k], r - k);  // (rounds below lo: loaded, never used)
  int npush = 0, stop_r = q.bottom;
  u64 e = 0;
  bool ended = false;
  while (!ended) {
#pragma unroll
    for (int k = 0; k < PF; k++) {  // round r is in slot k
      // waveReady's chain: a reachable, present leader of wave wv is pushed and the
      // chain goes on from it alone (also at the bottom round, before the sweep stops)
      // (every loaded value is consumed every round, through selects: a value a branch
      // may skip leaves its load's register in doubt, and the compiler then drains the
      // whole queue before reusing it)
      const int L = LD[k] - 1;
      u64 fl = 0;
#pragma unroll
      for (int w = 0; w < WS; w++) fl = w == (L >> 6) ? F[w] & P[k][w] : fl;
      if (r < q.top && ((r - 1) & 3) == 0) {
        const int wv = (r - 1) / 4 + 1;
        if ((fl >> (L & 63)) & 1ULL) {
#pragma unroll
          for (int w = 0; w < WS; w++) F[w] = w == (L >> 6) ? 1ULL << (L & 63) : 0ULL;
          // pushes collect in LDS (no global store inside the loop: stores count in vmcnt
          // too, and a conditional one defeats the compiler's count of the loads in flight)
          if (lane == 0) pbuf[npush & (PB - 1)] = wv;
          npush++;
          if ((npush & (PB - 1)) == 0) {  // (a chain of more than PB pushes: flush)
            if (lane < PB) {
              push_out[q.out_off + npush - PB + lane] = pbuf[lane];
              if (pm.pushed) pm.pushed[pbuf[lane]] = pm.epoch;
            }
          }
        }
      }
      if (r <= q.bottom) {
        ended = true;
        break;
      }
      u64 any = 0;
#pragma unroll
      for (int w = 0; w < WS; w++) any |= F[w];
      if (!any) {  // nothing reached in round r: nothing below either
        stop_r = r;
        ended = true;
        break;
      }
      u64 fw = 0;
#pragma unroll
      for (int w = 0; w < WS; w++) fw = w == wd ? F[w] & P[k][w] : fw;
      const uint32_t fe = (uint32_t)(fw >> sh);
      u64 acc[WS];
#pragma unroll
      for (int w = 0; w < WS; w++) acc[w] = 0;
#pragma unroll
      for (int j = 0; j < WS; j++) {
        const u64 m = 0ULL - (u64)((fe >> j) & 1u);
        e += dg[k][j] & (uint32_t)m;
#pragma unroll
        for (int w = 0; w < WS; w++) acc[w] |= rows[k][j * WS + w] & m;
      }
#pragma unroll
      for (int w = 0; w < WS; w++) F[w] = wave_or(acc[w]);
      load(rows[k], P[k], dg[k], LD[k], r - PF);  // slot k is free: round r - PF
      --r;
    }
  }
  {
    const int left = npush & (PB - 1);
    if (lane < left) {
      push_out[q.out_off + npush - left + lane] = pbuf[lane];
      if (pm.pushed) pm.pushed[pbuf[lane]] = pm.epoch;  // (a delivery query of that wave is live)
    }
  }
  e = wave_sum(e);
  if (lane == 0) {
    if (push_n) push_n[qi] = npush;
    if (edges_out) edges_out[qi] = e;
    if (wedges_out) wedges_out[qi] = 0;
    if (hit_out) hit_out[qi] = 0;
    if (stop_out) stop_out[qi] = -1 - stop_r;
  }
}

template <int WS, int PF>
__global__ __launch_bounds__(256) void k_chain_reg(DagView g, const SweepQuery *__restrict__ qs,
                                                   const int *__restrict__ nq_dev, int32_t *__restrict__ push_out,
                                                   int32_t *__restrict__ push_n, u64 *__restrict__ edges_out,
                                                   u64 *__restrict__ wedges_out, uint8_t *__restrict__ hit_out,
                                                   int32_t *__restrict__ stop_out, const PopMark pm) {
  chain_reg_body<WS, PF>((int)blockIdx.x, g, qs, nq_dev, push_out, push_n, edges_out, wedges_out, hit_out, stop_out,
                         pm);
}

// The planned replay's final pass (one workgroup), after the emitting sweep.
template <int NT>
__global__ __launch_bounds__(NT) void k_replay_final(const EmitArgs ea) {
  replay_final_block<NT>(ea.fin, ea);
}

// ---------------------------------------------------------------------------
// k_summary_commit: one workgroup per wave w (rounds 4w-3 .. 4w, clipped to T):
// the round summaries U_r (OR of every strong row) and SD_r (strong degree sum)
// AND waveReady's commit decision from one read of each strong row.  Commit:
// S_0 = {leader}; for the wave's rounds 2..4, S_k = {v : row(v) & S_{k-1} != 0}
// by ballot; vcount = |S_3| (process.go:326-339).  Waves past nwc get
// summaries only.  Each thread owns 16-B chunk column j of rows tid/CPR + p*RPP;
// loads go out GRP chunks at a time (nontemporal: every row is read once).
// PIPE: the next group's loads -- the next round's first group at a round end
// -- are issued before the current group is consumed, so the two barriers that
// publish a round's U, SD and S overlap the next round's loads.
// ---------------------------------------------------------------------------
template <int WS>
__device__ __forceinline__ void weak_union_round(const DagView &g, int r, int dd, u64 *__restrict__ WU, u64 *sW,
                                                 const u64 *__restrict__ ppref, const uint32_t *__restrict__ slot_off,
                                                 const uint16_t *__restrict__ slot_src, u64 *__restrict__ RG,
                                                 int lane);

// The weak unions and speculative digests (weak_union_round) in the row pass's launch:
// workgroups nsum .. nsum + nwug - 1 of the grid, after every row workgroup, take the
// rounds nwv at a time (one wave each, the other waves idle).  They depend on the
// weak-column keys and the slot lists alone, so they fill the CUs the row pass's last
// workgroups leave idle instead of a launch of their own after it (C4: 12 us).
struct WUArgs {
  int nsum;  // row-pass workgroups ((T + 3) / 4); 0: no weak-union workgroups
  int dd, nwv;
  u64 *WU;
  const u64 *ppref;
  const uint32_t *slot_off;
  const uint16_t *slot_src;
  u64 *RG;
};

template <int WS, int NT, int GRP, bool PIPE>
__global__ __launch_bounds__(NT) void k_summary_commit(DagView g, int T, int nwc, int quorum, u64 *__restrict__ U,
                                                       u64 *__restrict__ SD, uint8_t *__restrict__ commit,
                                                       int32_t *__restrict__ vcount, const WUArgs wa) {
  if (wa.nsum > 0 && (int)blockIdx.x >= wa.nsum) {  // (block-uniform) a weak-union workgroup
    extern __shared__ __attribute__((aligned(16))) u64 wu_lds[];
    const int wid = threadIdx.x >> 6;
    const int r = ((int)blockIdx.x - wa.nsum) * wa.nwv + wid + 1;
    if (wid >= wa.nwv || r > T) return;  // wave-uniform
    weak_union_round<WS>(g, r, wa.dd, wa.WU, wu_lds + (size_t)wid * wa.dd * WS, wa.ppref, wa.slot_off, wa.slot_src,
                         wa.RG, threadIdx.x & 63);
    return;
  }
  using G = Geo<WS, NT>;
  constexpr int CW = G::CW, CPR = G::CPR, RPP = G::RPP, CPT = G::CPT;
  constexpr int GR = CPT < GRP ? CPT : GRP;  // chunks per group
  constexpr int NGR = (CPT + GR - 1) / GR;   // groups per round
  __shared__ u64 sU[WS], S[WS], Tn[WS], P[WS];
  __shared__ u64 sSD;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, j = tid % CPR, n = g.n;
  const int w = blockIdx.x + 1;
  const int r1 = 4 * (w - 1) + 1;
  const int nr = min(T, r1 + 3) - r1 + 1;
  const bool do_commit = w <= nwc;
  const int l = do_commit ? g.lead[w] - 1 : 0;  // chooseLeader(w), 0-based
  const bool leader = do_commit && ((g.present[(size_t)r1 * WS + (l >> 6)] >> (l & 63)) & 1ULL);
  if (tid < WS) {
    sU[tid] = 0;
    S[tid] = tid == (l >> 6) ? 1ULL << (l & 63) : 0ULL;
    Tn[tid] = 0;
    P[tid] = g.present[(size_t)r1 * WS + tid];
  }
  if (tid == 0) sSD = 0;
  __syncthreads();
  const int NG = nr * NGR;
  u64 A0[GR], A1[GR], B0[GR], B1[GR];
  u64 a0 = 0, a1 = 0, deg = 0, s0 = 0, s1 = 0;
  bool test = false;
  auto load = [&](u64 *x0, u64 *x1, int gi) {
    const int k = gi / NGR, p0 = (gi - k * NGR) * GR;
    const u64 *rows = g.strong + (size_t)(r1 + k) * n * WS;
#pragma unroll
    for (int p = 0; p < GR; p++) {
      const int s = tid / CPR + (p0 + p) * RPP;
      x0[p] = 0;
      x1[p] = 0;
      if (p0 + p < CPT && s < n) {
        if constexpr (CW == 2) {
          const u64x2 x = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(rows + (size_t)s * WS + 2 * j));
          x0[p] = x.x;
          x1[p] = x.y;
        } else {
          x0[p] = __builtin_nontemporal_load(rows + s);
        }
      }
    }
  };
  auto round_begin = [&](int k) {  // S_{k-1} is published: the chunk of it this thread tests
    test = leader && k >= 1;
    s0 = test ? S[j * CW] : 0ULL;
    s1 = (test && CW == 2) ? S[j * CW + 1] : 0ULL;
  };
  auto consume = [&](const u64 *x0, const u64 *x1, int gi) {
    const int k = gi / NGR, p0 = (gi - k * NGR) * GR;
#pragma unroll
    for (int p = 0; p < GR; p++) {
      a0 |= x0[p];
      a1 |= x1[p];
      deg += (u64)(popc64(x0[p]) + popc64(x1[p]));
    }
    if (test) {  // commit: rows of round r that reach S (wave rounds 2..4)
#pragma unroll
      for (int p = 0; p < GR; p++) {
        const int rowbase = (wid * 64) / CPR + (p0 + p) * RPP;
        if (p0 + p >= CPT || rowbase >= n) break;  // wave-uniform
        const int s = tid / CPR + (p0 + p) * RPP;
        const bool pres = s < n && ((P[s >> 6] >> (s & 63)) & 1ULL);
        const bool hit = pres && ((x0[p] & s0) | (x1[p] & s1)) != 0ULL;
        u64 m = __ballot(hit);
        if (lane == 0 && m) {
          u64 bits;
          if constexpr (CPR == 1) {
            bits = m;
          } else {
#pragma unroll
            for (int sh = 1; sh < CPR; sh <<= 1) m |= m >> sh;
            bits = 0;
#pragma unroll
            for (int gI = 0; gI < 64 / CPR; gI++) bits |= ((m >> (gI * CPR)) & 1ULL) << gI;
          }
          atomicOr(&Tn[rowbase >> 6], bits << (rowbase & 63));
        }
      }
    }
  };
  auto round_end = [&](int k) {  // publish U_r, SD_r, S_k; load the next round's presence
    const int r = r1 + k;
    if constexpr (CPR < 16) {
      a0 = row_or_stride<CPR>(a0);
      if constexpr (CW == 2) a1 = row_or_stride<CPR>(a1);
    }
    deg = wave_sum(deg);
    if ((lane & 15) < CPR) {
      if (a0) atomicOr(&sU[(lane & 15) * CW], a0);
      if (CW == 2 && a1) atomicOr(&sU[(lane & 15) * CW + 1], a1);
    }
    if (lane == 0 && deg) atomicAdd(&sSD, deg);
    a0 = a1 = deg = 0;
    __syncthreads();
    if (tid < WS) {
      U[(size_t)r * WS + tid] = sU[tid];
      sU[tid] = 0;
      if (test) { S[tid] = Tn[tid]; Tn[tid] = 0; }
      if (k + 1 < nr) P[tid] = g.present[(size_t)(r + 1) * WS + tid];
    }
    if (tid == 0) { SD[r] = sSD + (g.sdx ? g.sdx[r] : 0u); sSD = 0; }
    __syncthreads();
    round_begin(k + 1);
  };
  round_begin(0);
  if constexpr (PIPE) {
    load(A0, A1, 0);
    for (int gi = 0; gi < NG; gi += 2) {
      if (gi + 1 < NG) load(B0, B1, gi + 1);
      consume(A0, A1, gi);
      if (gi % NGR == NGR - 1) round_end(gi / NGR);
      if (gi + 1 >= NG) break;
      if (gi + 2 < NG) load(A0, A1, gi + 2);
      consume(B0, B1, gi + 1);
      if ((gi + 1) % NGR == NGR - 1) round_end((gi + 1) / NGR);
    }
  } else {
    (void)B0;
    (void)B1;
    for (int gi = 0; gi < NG; gi++) {
      load(A0, A1, gi);
      consume(A0, A1, gi);
      if (gi % NGR == NGR - 1) round_end(gi / NGR);
    }
  }
  if (do_commit && wid == 0) {
    // vCount counts slots (process.go:330-335): repeated ids once per slot
    const int dc = leader ? dup_count<WS>(g, r1 + 3, lane < WS ? S[lane] : 0ULL) : 0;
    if (tid == 0) {
      if (!leader) {  // leader is bottom (process.go:327-329)
        commit[w - 1] = 0;
        vcount[w - 1] = -1;
      } else {
        int vc = dc;
#pragma unroll
        for (int i = 0; i < WS; i++) vc += popc64(S[i]);
        vcount[w - 1] = vc;
        commit[w - 1] = vc >= quorum ? 1 : 0;
      }
    }
  }
}

// The rounds an append touched: up to kRoundListMax of them travel in the launch's
// arguments (the per-call waveReady's four: no copy before the launch), more in
// device memory (ext).
constexpr int kRoundListMax = 16;
struct RoundList {
  int n;
  int32_t r[kRoundListMax];
  const int32_t *ext;
};
__device__ __forceinline__ int round_at(const RoundList &l, int i) { return l.ext ? l.ext[i] : l.r[i]; }

// U_r and SD_r of the listed rounds (the incremental summaries of rounds an
// append touched): one workgroup per round, the row stream of k_summary_commit
// without the commit rule.  With dd > 0 the workgroups after the first rl.n take
// the listed rounds' weak unions WU_r, nwv rounds each (one wave per round, the
// others idle; dynamic LDS nwv x dd x WS words): they read the weak-column keys
// alone, so they run beside the row workgroups instead of in a launch after them.
template <int WS, int NT>
__global__ __launch_bounds__(NT) void k_round_summary(DagView g, const RoundList rl, u64 *__restrict__ U,
                                                      u64 *__restrict__ SD, int dd, int nwv,
                                                      u64 *__restrict__ WU) {
  if ((int)blockIdx.x >= rl.n) {  // (block-uniform) a weak-union workgroup
    extern __shared__ __attribute__((aligned(16))) u64 wu_lds[];
    const int wid = threadIdx.x >> 6;
    const int i = ((int)blockIdx.x - rl.n) * nwv + wid;
    if (wid >= nwv || i >= rl.n) return;  // wave-uniform
    weak_union_round<WS>(g, round_at(rl, i), dd, WU, wu_lds + (size_t)wid * dd * WS, nullptr, nullptr, nullptr,
                         nullptr, threadIdx.x & 63);
    return;
  }
  using G = Geo<WS, NT>;
  constexpr int CW = G::CW, CPR = G::CPR, RPP = G::RPP, CPT = G::CPT;
  __shared__ u64 sU[WS];
  __shared__ u64 sSD;
  const int tid = threadIdx.x, lane = tid & 63, j = tid % CPR, n = g.n;
  const int r = round_at(rl, blockIdx.x);
  if (tid < WS) sU[tid] = 0;
  if (tid == 0) sSD = 0;
  __syncthreads();
  const u64 *rows = g.strong + (size_t)r * n * WS;
  u64 a0 = 0, a1 = 0, deg = 0;
#pragma unroll 4
  for (int p = 0; p < CPT; p++) {
    const int s = tid / CPR + p * RPP;
    if (s >= n) break;
    u64 x0, x1 = 0;
    if constexpr (CW == 2) {
      const u64x2 x = *reinterpret_cast<const u64x2 *>(rows + (size_t)s * WS + 2 * j);
      x0 = x.x;
      x1 = x.y;
    } else {
      x0 = rows[s];
    }
    a0 |= x0;
    a1 |= x1;
    deg += (u64)(popc64(x0) + popc64(x1));
  }
  if constexpr (CPR < 16) {
    a0 = row_or_stride<CPR>(a0);
    if constexpr (CW == 2) a1 = row_or_stride<CPR>(a1);
  }
  deg = wave_sum(deg);
  if ((lane & 15) < CPR) {
    if (a0) atomicOr(&sU[(lane & 15) * CW], a0);
    if (CW == 2 && a1) atomicOr(&sU[(lane & 15) * CW + 1], a1);
  }
  if (lane == 0 && deg) atomicAdd(&sSD, deg);
  __syncthreads();
  if (tid < WS) U[(size_t)r * WS + tid] = sU[tid];
  if (tid == 0) SD[r] = sSD + (g.sdx ? g.sdx[r] : 0u);
}

// ---------------------------------------------------------------------------
// k_set_weak: setWeakEdges (process.go:298-310) for a new vertex v of round r0
// whose strong row is srow, paper semantics (path over v's own edges, weak edges
// added so far included).  One workgroup walks rounds r0-1 .. 1:
//   F_r = the ring slot of r (| far-scatter row);  for r <= r0-2:
//   add_r = P_r & ~F_r (present vertices v cannot reach: they become weak edges,
//   process.go:305-307), F_r |= add_r (v now reaches them);  expand F_r & P_r.
// add_r is written to out[r]; the host lists its slots in (round desc, slot asc)
// order.  far[r] (zeroed by the host) takes weak scatters beyond the ring.
// ---------------------------------------------------------------------------
template <int WS, int NT>
__global__ __launch_bounds__(NT) void k_set_weak(DagView g, int r0, int depth_log2, const u64 *__restrict__ srow,
                                                 u64 *__restrict__ out, u64 *__restrict__ far) {
  constexpr u64 WMASK = WS >= 64 ? ~0ULL : ((1ULL << WS) - 1ULL);
  extern __shared__ __attribute__((aligned(16))) u64 smem[];
  u64 *F = smem, *FE = smem + WS, *ring = smem + 2 * WS;
  const int depth = 1 << depth_log2, dmask = depth - 1, tid = threadIdx.x;
  __shared__ int s_nz;
  for (int i = tid; i < depth * WS; i += NT) ring[i] = 0;
  __syncthreads();
  if (tid < WS) ring[(size_t)((r0 - 1) & dmask) * WS + tid] = srow[tid];
  __syncthreads();
  u64 e_dummy = 0, rb_dummy = 0, we_dummy = 0;
  for (int r = r0 - 1; r >= 1; r--) {
    if (tid < 64) {
      u64 f = 0, p = 0;
      if (tid < WS) {
        const int slot = (r & dmask) * WS + tid;
        f = ring[slot] | ld_agent(far + (size_t)r * WS + tid);
        ring[slot] = 0;
        p = g.present[(size_t)r * WS + tid];
        const u64 add = r <= r0 - 2 ? (p & ~f) : 0ULL;
        out[(size_t)r * WS + tid] = add;
        f |= add;
        F[tid] = f;
        FE[tid] = f & p;
      }
      const bool nz = (__ballot(tid < WS && (f & p) != 0ULL) & WMASK) != 0;
      if (tid == 0) s_nz = nz;
    }
    __syncthreads();
    if (s_nz) {
      expand_round<WS, NT, true>(g, r, 1, FE, ring, depth, far + WS, nullptr, e_dummy, we_dummy, rb_dummy);
    }
    __syncthreads();
  }
}

// WU_r[delta] = the union of round r's weak targets at distance delta, one
// wavefront per round, four rounds per workgroup: round r = 4 blockIdx.x + wave
// + 1 <= T (or rounds[4 blockIdx.x + wave] for the first nr entries:
// incremental).  No workgroup barrier: each wave ORs the round's weak-column keys
// into its own LDS slice (dynamic LDS, 4 x dd x WS u64).
//
// With RG (a full replay): also the speculative canonical digest of round r,
// assuming every round 1..r full (K_y covers P_y): every present vertex of r
// (every non-ghost slot, in slot order) delivered at positions from ppref[r-1]
// = |P_1| + .. + |P_{r-1}|.  k_canon lowers *rlo to the lowest round where that
// assumption fails; the canonical emission recomputes only rounds >= *rlo.
// One round's WU_r and speculative digest RG[r] on one wavefront, in the wave's LDS
// slice sW (dd x WS words).  No workgroup barrier.
template <int WS>
__device__ __forceinline__ void weak_union_round(const DagView &g, int r, int dd, u64 *__restrict__ WU, u64 *sW,
                                                 const u64 *__restrict__ ppref, const uint32_t *__restrict__ slot_off,
                                                 const uint16_t *__restrict__ slot_src, u64 *__restrict__ RG,
                                                 int lane) {
  if (dd <= 0 && !RG) return;
  // 16-B LDS and HBM accesses when every row is 16-B aligned (WS even)
  typedef u64 u64v2 __attribute__((ext_vector_type(2)));
  if constexpr (WS % 2 == 0) {
    for (int k = lane; k < dd * WS / 2; k += 64) reinterpret_cast<u64v2 *>(sW)[k] = u64v2{0, 0};
  } else {
    for (int k = lane; k < dd * WS; k += 64) sW[k] = 0;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  // every weak-column entry has at least one source: its key alone is the union
  for (uint32_t j = g.wc_roff[r] + lane; j < g.wc_roff[r + 1]; j += 64) {
    const uint32_t key = g.wc_key[j];
    const uint32_t d = (key >> 11) - 2;  // keys beyond the regular window are exceptions (no slot)
    if (d < (uint32_t)dd) atomicOr(&sW[d * WS + ((key & 2047u) >> 6)], 1ULL << (key & 63u));
  }
  if (RG) {  // the round's slots in lane-contiguous runs of SPT
    constexpr int SPT = 8;
    const uint32_t sa = slot_off[r], sb = slot_off[r + 1];
    u64 pos = ppref[r - 1], dg = 0;
    for (uint32_t c0 = sa; c0 < sb; c0 += 64 * SPT) {
      const uint32_t i0 = c0 + (uint32_t)lane * SPT;
      uint32_t src[SPT];
      uint32_t cnt = 0;
#pragma unroll
      for (int j = 0; j < SPT; j++) {
        src[j] = i0 + j < sb ? slot_src[i0 + j] : 0u;
        cnt += src[j] != 0;
      }
      uint32_t inc = cnt;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(inc, off);
        if (lane >= off) inc += y;
      }
      u64 k = pos + (inc - cnt);
#pragma unroll
      for (int j = 0; j < SPT; j++)
        if (src[j]) dg += digest_term((uint32_t)(r + g.roff), src[j], k++);
      pos += __shfl(inc, 63);
    }
    dg = wave_sum(dg);
    if (lane == 0) RG[r] = dg;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  if constexpr (WS % 2 == 0) {
    u64v2 *dst = reinterpret_cast<u64v2 *>(WU + (size_t)r * dd * WS);
    for (int k = lane; k < dd * WS / 2; k += 64) dst[k] = reinterpret_cast<const u64v2 *>(sW)[k];
  } else {
    for (int k = lane; k < dd * WS; k += 64) WU[(size_t)r * dd * WS + k] = sW[k];
  }
}

template <int WS>
__global__ __launch_bounds__(256) void k_weak_union(DagView g, int T, int nr, int dd, u64 *__restrict__ WU,
                                                    const int32_t *__restrict__ rounds,
                                                    const u64 *__restrict__ ppref, const uint32_t *__restrict__ slot_off,
                                                    const uint16_t *__restrict__ slot_src, u64 *__restrict__ RG) {
  extern __shared__ __attribute__((aligned(16))) u64 wu_lds[];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int i = blockIdx.x * (int)(blockDim.x >> 6) + wid;  // one wave per round
  int r;
  if (rounds) {
    if (i >= nr) return;
    r = rounds[i];
  } else {
    r = i + 1;
  }
  if (r > T) return;  // wave-uniform: this wave alone
  weak_union_round<WS>(g, r, dd, WU, wu_lds + (size_t)wid * dd * WS, ppref, slot_off, slot_src, RG, lane);
}

// K^cand_r = U_{r+1} | OR_d WU_{r+d+2}[d] (the cone of round r when every round
// above it is full); K^cand_T = P_T.  good_r = K^cand_r covers P_r.  CE_r (the
// canonical round's edges) defaults to the full-round total, RD_r (its vertex
// count |K_r & P_r|) to K^cand's.  One wave per round, lane w < WS owns word w;
// the window's WU terms are spread over all 64 lanes (64/WS classes of delta d,
// OR-reduced across lanes): a deep window (dd = 79) has 79 terms per word.
template <int WS>
__device__ __forceinline__ void kcand_body(DagView g, MemoView mv, int T, u64 *__restrict__ K,
                                           uint8_t *__restrict__ good, u64 *__restrict__ CE,
                                           u64 *__restrict__ RD, int *__restrict__ rlo, int lo,
                                           const u64 *__restrict__ ppref, u64 *__restrict__ Cc,
                                           uint32_t *__restrict__ crbase) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), w = threadIdx.x & 63;
  if (rlo && blockIdx.x == 0 && threadIdx.x == 0) *rlo = lo;  // k_canon_diff / k_canon lower it
  if (r > T) return;  // wave-uniform
  constexpr int G = WS >= 64 ? 1 : 64 / WS;  // delta classes
  const int wl = w % WS, cls = w / WS;
  u64 k = 0;
  if (r < T && cls < G) {
    if (cls == 0) k = mv.U[(size_t)(r + 1) * WS + wl];
#pragma unroll 4
    for (int d = cls; d < mv.dd && r + d + 2 <= T; d += G) k |= mv.WU[((size_t)(r + d + 2) * mv.dd + d) * WS + wl];
  }
#pragma unroll
  for (int m = WS; m < 64; m <<= 1) k |= shfl_xor64(k, m);
  bool bad = false;
  int cnt = 0;
  if (w < WS) {
    const u64 p = g.present[(size_t)r * WS + w];
    if (r == T) k = p;
    else if (r >= g.seed_lo) k |= p;  // a seeded slice top: the rank above reports these rounds full
    K[(size_t)r * WS + w] = k;
    bad = (k & p) != p;
    cnt = popc64(k & p);
  }
  const bool ok = __ballot(bad) == 0ULL;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
  // REF delivers every slot of a reached id (process.go:418-429): repeated ones count too
  if (g.dup_off && r >= 1) {
    u64 kp = 0;
    if (w < WS) kp = K[(size_t)r * WS + w] & g.present[(size_t)r * WS + w];
    cnt += dup_count<WS>(g, r, kp);
  }
  if (w == 0) {
    good[r] = ok;
    CE[r] = r == 0 ? 0 : mv.SD[r] + (g.weak_roff[r + 1] - g.weak_roff[r]);
    RD[r] = r == 0 ? 0 : (u64)cnt;
  }
  if (ppref && w == 1) {  // a full cone: positions default to the presence prefix (k_canon
    // rewrites the rounds from its lowest walked round up)
    Cc[r] = ppref[r];
    crbase[r] = r >= 1 ? (uint32_t)ppref[r - 1] : 0u;
  }
}
template <int WS>
__global__ __launch_bounds__(256) void k_kcand(DagView g, MemoView mv, int T, u64 *__restrict__ K,
                                               uint8_t *__restrict__ good, u64 *__restrict__ CE,
                                               u64 *__restrict__ RD, int *__restrict__ rlo, int lo,
                                               const u64 *__restrict__ ppref, u64 *__restrict__ Cc,
                                               uint32_t *__restrict__ crbase) {
  kcand_body<WS>(g, mv, T, K, good, CE, RD, rlo, lo, ppref, Cc, crbase);
}

// Incremental canonical emission: the lowest round r < lo whose canonical
// vertices K_r & P_r differ from the previous cone's (rounds >= lo changed or are
// new) -> atomicMin(*rlo).  Rounds below *rlo keep their per-round digests, and
// their positions are unchanged (every count below them is).  One wave per round.
template <int WS>
__global__ __launch_bounds__(256) void k_canon_diff(DagView g, int lo, const u64 *__restrict__ K,
                                                    const u64 *__restrict__ Kprev, int *__restrict__ rlo) {
  const int r = 1 + blockIdx.x * 4 + (threadIdx.x >> 6), w = threadIdx.x & 63;
  if (r >= lo) return;
  bool diff = false;
  if (w < WS) {
    const size_t i = (size_t)r * WS + w;
    diff = ((K[i] ^ Kprev[i]) & g.present[i]) != 0ULL;
  }
  if (__ballot(diff) != 0ULL && w == 0) atomicMin(rlo, r);
}

// ---------------------------------------------------------------------------
// k_canon: one workgroup walks the canonical cone from the top.  Rounds whose
// K^cand covers the round (good) and whose dmax-window above is full are exact
// already; at each bad round b a segment sweep (rows where partial, summaries
// where full) runs until dmax consecutive full rounds restore the regime.  The
// next bad round below is found 8 rounds per thread (one 8-B load of good[]).
// Then the canonical positions: C_r = sum of RD over rounds 1..r, crbase_r =
// C_{r-1} (k_kcand's counts, rewritten here for the segment rounds).
// ---------------------------------------------------------------------------
template <int WS, int NT>
__device__ __forceinline__ void canon_body(DagView g, MemoView mv, int T, int depth_log2,
                                           u64 *__restrict__ K, const uint8_t *__restrict__ good,
                                           u64 *__restrict__ CE, int32_t *__restrict__ nseg,
                                           u64 *__restrict__ RD, u64 *__restrict__ Cc,
                                           uint32_t *__restrict__ crbase, const u64 *__restrict__ ppref,
                                           int *__restrict__ rlo) {
  extern __shared__ __attribute__((aligned(16))) u64 smem[];
  u64 *F = smem, *FE = smem + WS, *ring = smem + 2 * WS;
  const int depth = 1 << depth_log2, dmask = depth - 1;
  int *s_ctl = reinterpret_cast<int *>(ring + (size_t)depth * WS);  // [0] next bad [1] full [2] done
  u64 *s_edges = reinterpret_cast<u64 *>(s_ctl + 8);
  const int tid = threadIdx.x;
  int pos = T;  // rounds >= pos are final; the regime holds below pos until the next bad round
  int segs = 0;
  int lo_w = T + 1;  // the lowest round a segment walk reached (RD below it is the full count)
  DR_TT(int walked = 0; if (tid == 0) { g_canon_timing[0] = wall_clock64(); g_canon_timing[5] = 0; })
  while (true) {
    // next bad round below pos: thread t looks at the 64 rounds of block (pos-1)/64 - t -
    // i*NT (four 16-B loads of good[], one pass over C3's 10 001 rounds; 8 rounds a
    // thread took five dependent passes there)
    if (tid == 0) s_ctl[0] = -1;
    __syncthreads();
    for (int b0 = (pos - 1) >> 6; b0 >= 0; b0 -= NT) {
      const int b = b0 - tid;
      if (b >= 0) {
        typedef u64 u64v2 __attribute__((ext_vector_type(2)));
        const u64v2 *gp = reinterpret_cast<const u64v2 *>(good + 64 * (size_t)b);
        u64 v[8];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const u64v2 x = gp[k];
          v[2 * k] = x.x;
          v[2 * k + 1] = x.y;
        }
        int hit = -1;  // the highest round x < pos of the block with good[x] == 0
#pragma unroll
        for (int k = 7; k >= 0; k--) {
          const int x0 = 64 * b + 8 * k;  // rounds x0 .. x0+7, one byte (0 or 1) each
          u64 m = ~v[k] & 0x0101010101010101ULL;  // bit 8j: round x0 + j is bad
          const int lim = pos - x0;              // rounds below pos only
          if (lim < 8) m &= lim <= 0 ? 0ULL : (1ULL << (8 * lim)) - 1ULL;
          if (hit < 0 && m) hit = x0 + (63 - __clzll(m)) / 8;
        }
        if (hit >= 0) atomicMax(&s_ctl[0], hit);
      }
      __syncthreads();
      if (s_ctl[0] >= 0) break;
      __syncthreads();
    }
    const int b = s_ctl[0];
    __syncthreads();
    if (b < 0) break;
    segs++;
    DR_TT(const u64 t_init = wall_clock64();)
    // state at b: F_b = K^cand_b; pending for rounds below from the full rounds above b
    for (int i = tid; i < depth * WS; i += NT) ring[i] = 0;
    __syncthreads();
    // the walk's per-round words three rounds ahead, in four register sets that the
    // unrolled loop below uses in turn (one round ahead, every round paid a load
    // latency: ~2.2 us a round at c4-deep; rotating the sets through moves waits for the
    // loads in flight, so the sets keep their registers and the rounds take turns).  The
    // walk's threads share the round through LDS only: its barriers order LDS alone and
    // leave the prefetches in flight (lds_barrier).
    constexpr int PF = 4;
    RoundWords rw[4] = {};
    u64 dv[4][PF];
    if (tid < WS) {
      ring[(size_t)(b & dmask) * WS + tid] = K[(size_t)b * WS + tid];
      load_round<WS, false, true, true>(g, mv, b, rw[0]);
      if (b >= 1) load_round<WS, false, true, true>(g, mv, b - 1, rw[1]);
      if (b >= 2) load_round<WS, false, true, true>(g, mv, b - 2, rw[2]);
    }
    // (round x, word w) pairs over every thread: a deep window has dd^2/2 terms per word
    for (int it = tid; it < mv.dd * WS; it += NT) {
      const int x = b - 1 - it / WS, w = it % WS;
      if (x < 0) continue;
      u64 v = 0;
#pragma unroll 8
      for (int y = max(b + 1, x + 2); y <= T && y <= x + mv.dd + 1; y++)
        v |= mv.WU[((size_t)y * mv.dd + (y - x - 2)) * WS + w];
      ring[(size_t)(x & dmask) * WS + w] = v;
    }
    __syncthreads();
    int run = 0;
    int r = b;
    deep_slots_load<WS, NT, PF>(mv, b, 0, dv[0]);
    deep_slots_load<WS, NT, PF>(mv, max(b - 1, 0), 0, dv[1]);
    deep_slots_load<WS, NT, PF>(mv, max(b - 2, 0), 0, dv[2]);
    DR_TT(if (tid == 0) g_canon_timing[5] += wall_clock64() - t_init;)
    bool done = false;
    while (!done) {
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const RoundWords &cur = rw[k];
        if (r >= 3) {  // round r-3's words, in flight
          deep_slots_load<WS, NT, PF>(mv, r - 3, 0, dv[(k + 3) & 3]);
          if (tid < WS) load_round<WS, false, true, true>(g, mv, r - 3, rw[(k + 3) & 3]);
        }
        if (tid < 64) {
          int cnt = 0;
          bool full = true;
          if (tid < WS) {
            const int slot = (r & dmask) * WS + tid;
            const u64 f = ring[slot];
            ring[slot] = 0;
            const u64 p = cur.P;
            F[tid] = f;
            FE[tid] = f & p;
            K[(size_t)r * WS + tid] = f;
            full = (f & p) == p;
            cnt = popc64(f & p);
          }
          full = __all(full);
#pragma unroll
          for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
          if (g.dup_off && r >= 1) cnt += dup_count<WS>(g, r, tid < WS ? FE[tid] : 0ULL);  // every slot (REF)
          run = full ? run + 1 : 0;
          if (tid == 0) {
            s_ctl[1] = full;
            s_ctl[2] = (run >= mv.dmax) || r == 0;
            s_edges[0] = 0;
            RD[r] = r == 0 ? 0 : (u64)cnt;
          }
        }
        lds_barrier();
        if (s_ctl[2]) {  // regime restored at r (or bottom reached): CE_r stays the full total
          done = true;
          break;
        }
        u64 e = 0, we = 0;
        if (s_ctl[1]) {
          expand_summary_pre<WS, NT, PF>(mv, cur, r, 0, ring, dmask, dv[k]);  // the whole workgroup
          if (tid == 0) e = cur.SD + cur.NW();  // prefetched with the round's words
        } else {
          u64 rb = 0;
          expand_round<WS, NT, true>(g, r, 0, FE, ring, depth, K, mv.U + (size_t)r * WS, e, we, rb, -1, -1, nullptr,
                                     mv.dreg);  // G_reg: exceptions are benign (engine.hip ensure_exceptions)
        }
        e += we;
        if (e) atomicAdd(&s_edges[0], e);
        DR_TT(walked++;)
        lds_barrier();
        // (no barrier before the next round: every thread read this round's s_ctl before
        // the one above, the ring's contributions are in, and s_edges is read and reset
        // by thread 0 alone)
        if (tid == 0) CE[r] = s_edges[0];
        --r;
      }
    }
    pos = r;
    lo_w = min(lo_w, r);
  }
  if (tid == 0 && nseg) {
    nseg[0] = segs;
    nseg[1] = lo_w;  // (T + 1: no walk) below it K is K^cand, every round full, CE the full total
  }
  DR_TT(if (tid == 0) {
    g_canon_timing[1] = wall_clock64();
    g_canon_timing[3] = segs;
    g_canon_timing[4] = walked;
  })
  // canonical positions (the RD writes above are this workgroup's own: visible after the barrier)
  // With ppref (a full cone), every round below the lowest walked one holds all its
  // present vertices (a bad round starts a walk): C there is the presence prefix,
  // copied; the scan covers the walked region only (C4, C3: the top ~10 rounds).
  __syncthreads();
  __shared__ u64 part[NT / 64];
  const int B = ppref ? lo_w : 0;  // (rounds below B: k_kcand wrote the presence prefix)
  // (ppref[0]: the slice's position base, 0 for a whole DAG; round 0 is never delivered)
  const u64 base0 = ppref ? ppref[B >= 1 ? B - 1 : 0] : 0ULL;
  const int per = (T + 1 - B + NT - 1) / NT;
  const int ra = B + tid * per, rb = min(T + 1, ra + per);
  int bad = INT_MAX;  // ppref: the lowest round whose C differs from the all-full prefix
  constexpr int MAXP = 16;
  if (per <= MAXP) {  // block-uniform: every load in flight at once
    u64 v[MAXP], pp[MAXP], loc = 0;
#pragma unroll
    for (int j = 0; j < MAXP; j++) {
      const int x = ra + j;
      v[j] = x < rb ? RD[x] : 0ULL;
      pp[j] = ppref && x < rb ? ppref[x] : 0ULL;
      loc += v[j];
    }
    u64 tot;
    u64 run = base0 + block_scan_excl<NT>(loc, part, tot);
#pragma unroll
    for (int j = 0; j < MAXP; j++) {
      const int x = ra + j;
      if (x >= rb) break;
      crbase[x] = (uint32_t)run;
      run += v[j];
      Cc[x] = run;
      if (ppref && bad == INT_MAX && x >= 1 && run != pp[j]) bad = x;
    }
  } else {
    u64 loc = 0;
    for (int x = ra; x < rb; x++) loc += RD[x];
    u64 tot;
    u64 run = base0 + block_scan_excl<NT>(loc, part, tot);
    for (int x = ra; x < rb; x++) {
      crbase[x] = (uint32_t)run;
      run += RD[x];
      Cc[x] = run;
      if (ppref && bad == INT_MAX && x >= 1 && run != ppref[x]) bad = x;
    }
  }
  if (ppref) {
    __shared__ int s_bad;
    if (tid == 0) s_bad = INT_MAX;
    __syncthreads();
    if (bad != INT_MAX) atomicMin(&s_bad, bad);
    __syncthreads();
    if (tid == 0 && s_bad != INT_MAX) atomicMin(rlo, s_bad);
  }
  DR_TT(if (tid == 0) g_canon_timing[2] = wall_clock64();)
}

template <int WS, int NT>
__global__ __launch_bounds__(NT) void k_canon(DagView g, MemoView mv, int T, int depth_log2,
                                              u64 *__restrict__ K, const uint8_t *__restrict__ good,
                                              u64 *__restrict__ CE, int32_t *__restrict__ nseg,
                                              u64 *__restrict__ RD, u64 *__restrict__ Cc,
                                              uint32_t *__restrict__ crbase, const u64 *__restrict__ ppref,
                                              int *__restrict__ rlo) {
  canon_body<WS, NT>(g, mv, T, depth_log2, K, good, CE, nseg, RD, Cc, crbase, ppref, rlo);
}

// The canonical walk (workgroup 0) and the leader chains (every other workgroup) in one
// launch: the chains need only the commits and the rows, the walk only the summaries, so
// neither waits for the other and no second stream (no fork or join event, ~18 us on
// MI355X, tools/experiments/launch_probe.hip) is needed.  CREG: the chains on one
// wavefront each (chain_reg_body, NT = 256), else k_sweep's chain mode.
struct CanonArgs {
  int T, depth_log2;
  u64 *K;
  const uint8_t *good;
  u64 *CE;
  int32_t *nseg;
  u64 *RD, *Cc;
  uint32_t *crbase;
  const u64 *ppref;
  int *rlo;
};
struct ChainArgs {
  const SweepQuery *q;
  const int *nq_dev;
  int32_t *push_out, *push_n;
  u64 *edges, *wedges;
  uint8_t *hits;
  int32_t *stops;
  PopMark pm;
};
// The canonical prefixes A, B of two per-round arrays over rounds 0..T (round 0 counted
// as 0), one workgroup, every round of a chunk of J * NT in registers: column j of the
// chunk (NT rounds) is loaded lane-consecutively (coalesced, all 2J loads in flight at
// once), each wave scans its 64 rounds of every column by DPP (no LDS, no barrier), and
// wave 0 turns the J * NT/64 wave totals into offsets through LDS: two LDS-only barriers
// per chunk, one memory round trip.  C3 (10 001 rounds, J = 10): one chunk, 11.4 us against
// 16.8 us for an LDS-tiled form and 18.8 us for canon_prefix_block's per-thread runs
// (profiles/r05/v15_prefix_bench.txt; a single-CU pass either way).
template <int NT, int J, class LA, class LB>
__device__ __forceinline__ void canon_prefix_gen(int r0, int T, u64 ca, u64 cb, LA la, LB lb, u64 *__restrict__ A,
                                                 u64 *__restrict__ B) {
  constexpr int NW = NT / 64, E = J * NW, PL = (E + 63) / 64;
  __shared__ u64 oa[E + 1], ob[E + 1];  // wave totals -> exclusive offsets; [E] = the chunk total
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, n = T + 1, lo = r0 > 1 ? r0 : 1;
  for (int c0 = r0; c0 < n; c0 += J * NT) {
    u64 xa[J], xb[J];
#pragma unroll
    for (int j = 0; j < J; j++) {  // clamped addresses: unconditional loads, all in flight
      const int r = c0 + j * NT + tid;
      const int rc = (r >= lo && r < n) ? r : lo;
      xa[j] = la(rc);
      xb[j] = lb(rc);
    }
#pragma unroll
    for (int j = 0; j < J; j++) {
      const int r = c0 + j * NT + tid;
      const bool in = r >= lo && r < n;  // round 0 is never delivered
      xa[j] = wave_scan_incl(in ? xa[j] : 0ULL);
      xb[j] = wave_scan_incl(in ? xb[j] : 0ULL);
      if (lane == 63) {
        oa[j * NW + wid] = xa[j];
        ob[j * NW + wid] = xb[j];
      }
    }
    lds_barrier();
    if (wid == 0) {  // exclusive offsets of the E (column, wave) totals, in round order
      u64 va[PL], vb[PL], sa = 0, sb = 0;
#pragma unroll
      for (int k = 0; k < PL; k++) {
        const int e = lane * PL + k;
        va[k] = e < E ? oa[e] : 0ULL;
        vb[k] = e < E ? ob[e] : 0ULL;
        sa += va[k];
        sb += vb[k];
      }
      const u64 ia = wave_scan_incl(sa), ib = wave_scan_incl(sb);
      u64 pa = ia - sa, pb = ib - sb;
#pragma unroll
      for (int k = 0; k < PL; k++) {
        const int e = lane * PL + k;
        if (e < E) {
          oa[e] = pa;
          ob[e] = pb;
        }
        pa += va[k];
        pb += vb[k];
      }
      if (lane == 63) {
        oa[E] = ia;
        ob[E] = ib;
      }
    }
    lds_barrier();
#pragma unroll
    for (int j = 0; j < J; j++) {
      const int r = c0 + j * NT + tid;
      if (r < n) {
        A[r] = ca + oa[j * NW + wid] + xa[j];
        B[r] = cb + ob[j * NW + wid] + xb[j];
      }
    }
    ca += oa[E];
    cb += ob[E];
    lds_barrier();  // the offsets are rewritten by the next chunk
  }
}
template <int NT, int J>
__device__ __forceinline__ void canon_prefix_regs(int T, const u64 *__restrict__ a, const u64 *__restrict__ b,
                                                  u64 *__restrict__ A, u64 *__restrict__ B) {
  canon_prefix_gen<NT, J>(0, T, 0ULL, 0ULL, [&](int r) { return a[r]; }, [&](int r) { return b[r]; }, A, B);
}

// The speculative canonical prefixes (the grid's last workgroup of k_canon_chains when
// on): G, E over every round as if every round were full -- the weak-union launch's
// per-round digests RG and the full-round edge totals SD + weak counts (k_kcand's CE
// default) -- exact below the canonical walk's lowest round; k_own_emit's workgroup 0
// then rescans only the rounds from there up (C3: 10 001 rounds, five chunks of one
// workgroup, off the critical path).
struct SpecPrefix {
  int on;
  const u64 *RG, *SD;
  const uint32_t *weak_roff;
  u64 *Gc, *Ec;
};
template <int WS, int NT, bool CREG>
__global__ __launch_bounds__(NT) void k_canon_chains(DagView g, MemoView mv, const CanonArgs ca, const ChainArgs xa,
                                                     const SpecPrefix sp) {
  if (sp.on && blockIdx.x == gridDim.x - 1) {
    canon_prefix_gen<NT, 8>(
        0, ca.T, 0ULL, 0ULL, [&](int r) { return sp.RG[r]; },
        [&](int r) { return sp.SD[r] + (u64)(sp.weak_roff[r + 1] - sp.weak_roff[r]); }, sp.Gc, sp.Ec);
    return;
  }
  if (blockIdx.x == 0) {
    canon_body<WS, NT>(g, mv, ca.T, ca.depth_log2, ca.K, ca.good, ca.CE, ca.nseg, ca.RD, ca.Cc, ca.crbase, ca.ppref,
                       ca.rlo);
    return;
  }
  if constexpr (CREG) {
    chain_reg_body<WS, 3>((int)blockIdx.x - 1, g, xa.q, xa.nq_dev, xa.push_out, xa.push_n, xa.edges, xa.wedges,
                          xa.hits, xa.stops, xa.pm);
  } else {
    sweep_body<WS, NT, SW_CHAIN>((int)blockIdx.x - 1, g, mv, xa.q, 0, 0, ca.depth_log2, nullptr, nullptr, xa.push_out,
                                 xa.push_n, xa.edges, xa.wedges, xa.hits, xa.stops, nullptr, xa.nq_dev, nullptr,
                                 xa.pm);
  }
}

// ---------------------------------------------------------------------------
// Emission.  A pop's delivered sequence is the concatenation, in round order,
// of segments; each segment is a PopDesc: rounds [first, last] read from a
// mask image (the pop's own masks, or the canonical cone K), positions starting
// at pos0 within the pop.
// ---------------------------------------------------------------------------
struct PopDesc {
  int64_t mask_off;   // word offset of round 0 in its image
  int64_t rbase_off;  // int offset of round `first` in rbase
  int64_t pos0;       // position of the segment's first vertex within its pop
  int32_t first, last;
  int32_t out;        // pop index (count / digest / ids slot)
  int32_t use_k;      // mask image: 0 = masks, 1 = canonical K
  int32_t flags;      // PD_FIRST_ONLY: a repeated id is delivered at its first slot only (PAPER)
};
enum : int32_t { PD_FIRST_ONLY = 1 };

// part 1: one workgroup per segment: c_r = |mask_r & present_r|, exclusive scan
// over the segment's rounds -> rbase, total -> count[seg]
template <int WS, int NT>
__global__ __launch_bounds__(NT) void k_emit_count(DagView g, const PopDesc *__restrict__ pd,
                                                   const u64 *__restrict__ masks, const u64 *__restrict__ K,
                                                   uint32_t *__restrict__ rbase, u64 *__restrict__ count,
                                                   const int *__restrict__ nd_dev) {
  __shared__ uint32_t part[NT];
  if (nd_dev && (int)blockIdx.x >= *nd_dev) return;  // grid sized by an upper bound
  const PopDesc d = pd[blockIdx.x];
  const u64 *img = (d.use_k ? K : masks) + d.mask_off;
  const int tid = threadIdx.x;
  const int nr = d.last - d.first + 1;
  const int per = nr > 0 ? (nr + NT - 1) / NT : 0;
  const int ra = d.first + tid * per, rb = min(d.last + 1, ra + per);
  // repeated ids: every slot counts in REF, the first slot only in PAPER
  const bool reps = g.dup_off && !(d.flags & PD_FIRST_ONLY);
  auto rep_cnt = [&](int r, const u64 *m) -> uint32_t {
    uint32_t c = 0;
    for (uint32_t j = g.dup_off[r]; j < g.dup_off[r + 1]; j++) {
      const int s = (int)g.dup_src[j] - 1;
      c += (uint32_t)((m[s >> 6] >> (s & 63)) & 1ULL);
    }
    return c;
  };
  uint32_t loc = 0;
  for (int r = ra; r < rb; r++) {
    const u64 *m = img + (int64_t)r * WS;
    const u64 *p = g.present + (size_t)r * WS;
#pragma unroll
    for (int w = 0; w < WS; w++) loc += popc64(m[w] & p[w]);
    if (reps) loc += rep_cnt(r, m);
  }
  part[tid] = loc;
  __syncthreads();
  for (int off = 1; off < NT; off <<= 1) {  // inclusive scan over NT partials
    uint32_t v = tid >= off ? part[tid - off] : 0;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  uint32_t run = part[tid] - loc;
  for (int r = ra; r < rb; r++) {
    rbase[d.rbase_off + (r - d.first)] = run;
    const u64 *m = img + (int64_t)r * WS;
    const u64 *p = g.present + (size_t)r * WS;
    uint32_t c = 0;
#pragma unroll
    for (int w = 0; w < WS; w++) c += popc64(m[w] & p[w]);
    if (reps) c += rep_cnt(r, m);
    run += c;
  }
  if (tid == NT - 1) count[blockIdx.x] = nr > 0 ? part[NT - 1] : 0;
}

// part 2: grid (round blocks, segments).  Each wave walks one round's slots in
// order, 64 at a time: the ballot of "slot's source in mask" ranks the round's
// delivered vertices, so vertex k of the pop (k = pos0 + rbase + rank) adds
// digest_term(round, source, k); ids land at pop_pos[out] + k.  With
// round_out != nullptr the per-round digest sums are written instead.
template <int WS, int NT, int RPB>
__device__ __forceinline__ void emit_block(const DagView &g, const uint32_t *__restrict__ slot_off,
                                           const uint16_t *__restrict__ slot_src, const PopDesc &d, int blk,
                                           const u64 *__restrict__ masks, const u64 *__restrict__ K,
                                           const uint32_t *__restrict__ rbase, const int64_t *__restrict__ pop_pos,
                                           u64 *__restrict__ digest, u64 *__restrict__ round_out,
                                           int32_t *__restrict__ ids, int64_t ids_cap, u64 *s_dg,
                                           const uint32_t *__restrict__ rcnt, u64 *__restrict__ pcount,
                                           int skip_below = -1) {
  constexpr int SPL = 16;  // slots per lane per pass: one wave covers 1024 slots with one load latency
  const u64 *img = (d.use_k ? K : masks) + d.mask_off;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  constexpr int NWAVE = NT / 64;
  if (tid == 0) *s_dg = 0;
  __syncthreads();
  u64 dg = 0;
  const int ra = d.first + blk * RPB;
  const int rb = min(d.last + 1, ra + RPB);
  const int64_t pbase = pop_pos ? pop_pos[d.out] : 0;
  for (int r = ra + wid; r < rb; r += NWAVE) {
    if (r < skip_below) continue;  // wave-uniform (round_out mode: nothing to add up)
    const u64 mw = lane < WS ? img[(int64_t)r * WS + lane] : 0ULL;  // lane w holds mask word w
    u64 pos;
    if (rcnt) {  // the sweep's per-round counts: position = pos0 + counts of rounds first..r-1
      const uint32_t *rc = rcnt + d.mask_off / WS;
      u64 below = 0;
      for (int x = d.first + lane; x < r; x += 64) below += rc[x];
      pos = (u64)d.pos0 + wave_sum(below);
      if (lane == 0 && rc[r]) atomicAdd(pcount + d.out, (u64)rc[r]);
    } else {
      pos = (u64)d.pos0 + rbase[d.rbase_off + (r - d.first)];
    }
    u64 rdg = 0;
    const uint32_t sa = slot_off[r], sb = slot_off[r + 1];
    for (uint32_t c0 = sa; c0 < sb; c0 += 64 * SPL) {
      const uint32_t i0 = c0 + (uint32_t)lane * SPL;  // this lane's slots, in slot order
      int src[SPL];
#pragma unroll
      for (int j = 0; j < SPL; j++) src[j] = i0 + j < sb ? (int)slot_src[i0 + j] : 0;
      if (g.slot_rep && (d.flags & PD_FIRST_ONLY))  // PAPER: a repeated id's later slots deliver nothing
#pragma unroll
        for (int j = 0; j < SPL; j++)
          if (i0 + j < sb && g.slot_rep[i0 + j]) src[j] = 0;
      uint32_t bits = 0;
#pragma unroll
      for (int j = 0; j < SPL; j++) {
        const int s = src[j] - 1;
        const u64 w = __shfl(mw, s >= 0 ? (s >> 6) : 0);
        if (s >= 0 && ((w >> (s & 63)) & 1ULL)) bits |= 1u << j;
      }
      const int cnt = __popc(bits);
      int x = cnt;  // inclusive scan of the lanes' counts = ranks in slot order
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(x, off);
        if (lane >= off) x += y;
      }
      const int total = __shfl(x, 63);
      u64 k = pos + (u64)(x - cnt);
#pragma unroll
      for (int j = 0; j < SPL; j++) {
        if (!((bits >> j) & 1u)) continue;
        rdg += digest_term((uint32_t)(r + g.roff), (uint32_t)src[j], k);
        if (ids) {
          const int64_t at = pbase + (int64_t)k;
          if (at < ids_cap) { ids[2 * at] = r + g.roff; ids[2 * at + 1] = src[j]; }
        }
        k++;
      }
      pos += (u64)total;
    }
    if (round_out) {
      rdg = wave_sum(rdg);
      if (lane == 0) round_out[r] = rdg;
    } else {
      dg += rdg;
    }
  }
  if (round_out) return;  // uniform: no barrier follows
  dg = wave_sum(dg);
  if (lane == 0 && dg) atomicAdd(s_dg, dg);
  __syncthreads();
  if (tid == 0 && *s_dg) atomicAdd(digest + d.out, *s_dg);
}

// Two launch shapes: grid (round blocks, segments) when item_pref is null; else
// a fixed grid striding over the work items of ctl[0] segments, segment i owning
// items [item_pref[i], item_pref[i+1]) (device-planned replay).  There, with rcnt
// (the delivery sweep's per-round counts, indexed like the mask rows), positions
// come from rcnt and the pop totals accumulate in pcount[out]: no count pass.
template <int WS, int NT, int RPB>
__global__ __launch_bounds__(NT) void k_emit_ids(DagView g, const uint32_t *__restrict__ slot_off,
                                                 const uint16_t *__restrict__ slot_src,
                                                 const PopDesc *__restrict__ pd, const PopDesc d1,
                                                 const u64 *__restrict__ masks, const u64 *__restrict__ K,
                                                 const uint32_t *__restrict__ rbase,
                                                 const int64_t *__restrict__ pop_pos,
                                                 u64 *__restrict__ digest, u64 *__restrict__ round_out,
                                                 int32_t *__restrict__ ids, int64_t ids_cap,
                                                 const int64_t *__restrict__ item_pref, const int *__restrict__ ctl,
                                                 const uint32_t *__restrict__ rcnt, u64 *__restrict__ pcount,
                                                 const int *__restrict__ skip_below) {
  __shared__ u64 s_dg;
  if (!item_pref) {
    const PopDesc d = pd ? pd[blockIdx.y] : d1;
    int lo = -1;
    if (skip_below) {  // per-round outputs of rounds >= *skip_below only (incremental canon)
      lo = *skip_below;
      if (d.first + ((int)blockIdx.x + 1) * RPB <= lo) return;
    }
    emit_block<WS, NT, RPB>(g, slot_off, slot_src, d, blockIdx.x, masks, K, rbase, pop_pos, digest, round_out, ids,
                            ids_cap, &s_dg, nullptr, nullptr, lo);
    return;
  }
  // item_pref[nd] = item count; item_pref[nd + 1 + it] = the segment owning item it
  const int nd = ctl[0];
  const int64_t nit = item_pref[nd];
  for (int64_t it = blockIdx.x; it < nit; it += gridDim.x) {
    const int lo = (int)item_pref[nd + 1 + it];
    emit_block<WS, NT, RPB>(g, slot_off, slot_src, pd[lo], (int)(it - item_pref[lo]), masks, K, rbase, pop_pos,
                            digest, round_out, ids, ids_cap, &s_dg, rcnt, pcount);
    __syncthreads();
  }
}



template <int NT>
__global__ __launch_bounds__(NT) void k_canon_prefix(int T, const u64 *__restrict__ a, const u64 *__restrict__ b,
                                                     u64 *__restrict__ A, u64 *__restrict__ B) {
  canon_prefix_regs<NT, 10>(T, a, b, A, B);
}

// Multi-segment copy between device memory and pinned (device-mapped) host
// memory: one launch moves every small result of a call, instead of one blit
// (and one queue round trip) per array.  blockIdx.y = segment.
struct CopySeg { const uint8_t *src; uint8_t *dst; uint64_t n; };
constexpr int kCopySegs = 16;
struct CopyList { CopySeg s[kCopySegs]; };

__global__ __launch_bounds__(256) void k_copy(CopyList L) {
  const CopySeg sg = L.s[blockIdx.y];
  const size_t stride = (size_t)gridDim.x * 256, t = (size_t)blockIdx.x * 256 + threadIdx.x;
  size_t head = 0;
  if ((((uintptr_t)sg.src | (uintptr_t)sg.dst) & 15) == 0) {
    head = sg.n & ~(uint64_t)15;
    const u32x4 *a = reinterpret_cast<const u32x4 *>(sg.src);
    u32x4 *b = reinterpret_cast<u32x4 *>(sg.dst);
    for (size_t i = t; i < head / 16; i += stride) b[i] = a[i];
  }
  for (size_t i = head + t; i < sg.n; i += stride) sg.dst[i] = sg.src[i];
}

// Calibration: read n16 16-B words (grid-stride, 4 in flight per thread) and
// fold them so nothing is dead-code eliminated.  The practical ceiling for the
// streaming kernels (dr_profile_kernel).
template <int NT>
__global__ __launch_bounds__(NT) void k_stream_read(const u64x2 *__restrict__ p, size_t n16, u64 *__restrict__ out) {
  u64 acc = 0;
  const size_t stride = (size_t)gridDim.x * NT;
  size_t i = (size_t)blockIdx.x * NT + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const u64x2 a = __builtin_nontemporal_load(p + i), b = __builtin_nontemporal_load(p + i + stride);
    const u64x2 c = __builtin_nontemporal_load(p + i + 2 * stride), d = __builtin_nontemporal_load(p + i + 3 * stride);
    acc ^= a.x ^ a.y ^ b.x ^ b.y ^ c.x ^ c.y ^ d.x ^ d.y;
  }
  for (; i < n16; i += stride) { const u64x2 a = __builtin_nontemporal_load(p + i); acc ^= a.x ^ a.y; }
  if (acc == 0x9E3779B97F4A7C15ULL) out[0] = acc;  // practically never taken
}

// Calibration, blocked pattern: workgroup b reads its own contiguous chunk
// (the access shape of one-workgroup-per-wave kernels).
template <int NT>
__global__ __launch_bounds__(NT) void k_stream_read_blocked(const u64x2 *__restrict__ p, size_t n16,
                                                            u64 *__restrict__ out) {
  u64 acc = 0;
  const size_t per = (n16 + gridDim.x - 1) / gridDim.x;
  const size_t a = (size_t)blockIdx.x * per, b = min(n16, a + per);
  size_t i = a + threadIdx.x;
  for (; i + 3 * NT < b; i += 4 * NT) {
    const u64x2 x = __builtin_nontemporal_load(p + i), y = __builtin_nontemporal_load(p + i + NT);
    const u64x2 z = __builtin_nontemporal_load(p + i + 2 * NT), w = __builtin_nontemporal_load(p + i + 3 * NT);
    acc ^= x.x ^ x.y ^ y.x ^ y.y ^ z.x ^ z.y ^ w.x ^ w.y;
  }
  for (; i < b; i += NT) { const u64x2 x = __builtin_nontemporal_load(p + i); acc ^= x.x ^ x.y; }
  if (acc == 0x9E3779B97F4A7C15ULL) out[0] = acc;
}

}  // namespace dr
