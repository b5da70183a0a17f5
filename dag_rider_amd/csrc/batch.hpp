// batch.hpp -- fused replay of many small DAGs: one workgroup of four wavefronts
// per DAG.
//
// thousands of independent replays (one Process mirror
// each, n <= 128, up to 64 waves).  A per-DAG dr_replay would spend its time in
// launches and host round trips; here one kernel replays every DAG of a batch,
// everything between the DAG in HBM and the per-pop results on the device.
// At N GPUs each GPU holds 4096 / N DAGs, so what bounds a GPU's share is one
// DAG's critical path, not the batch's total work: the workgroup splits it.
//
// Per DAG (T = 4*(nw-1)+1, the highest leader round; lane b = leader of wave
// b+1, lane 63 = the canonical cone K = every present vertex of round T):
//   1. commits (waveReady's rule, process.go:326-339) on waves 1-3, one
//      DAG-wave per wavefront at a time: S0 = {leader}; S_k = ballot(row(v) &
//      S_{k-1} != 0) over rounds 4w-2..4w.
//   2. two independent top-down passes over rounds T..1, bit-sliced (lane b
//      holds leader b's cone in the current round as a vertex set, 2 words),
//      each loading its rounds kSmallPF ahead into a register ring:
//      wave 0 (2F): F_b over strong and weak edges (orderVertices' path(..,
//      false)).  Rows are OR-reduced over the set's members; a weak column (one
//      distinct weak target of the round) puts its target into b's pending
//      round iff its sources meet F_b.  A leader whose set equals K's takes K's
//      expansion and weak targets; only the others (a leader in the few rounds
//      under its top) expand on their own.  Per round it stores every lane's
//      set, |F_b & P_r| and the leaders whose set differs from K's.
//      wave 1 (2G, after the commits): G_b over strong edges only (the chains'
//      strong_path, while a chain can still inspect it), the leaders whose
//      strong cone holds each leader vertex (QL), and per leader the strong
//      degrees summed over G_b (the chains' edge counts).
//      waves 2-3 (2D): the strong + weak degree of every slot's vertex.
//   3. chains (process.go:341-350) from QL: wave w' is pushed after leader L
//      iff L's strong cone holds leader(w'); pops = reverse pushes.  Chain
//      edges = per segment the strong degrees summed over its rounds
//      (differences of step 2's suffix sums).
//   4. emission, parallel over rounds.  The order-sensitive digest (DESIGN.md
//      s3.3) needs each vertex's position in its pop's sequence, so counts come
//      first: |F_b & P_r| (ids do not repeat here), prefix sums give positions,
//      then every (round, leader) contribution is computed with lanes = slots
//      (ballot ranks; wave sums of digests and edges).
//      REF: b's cone equals K in every round below the lowest round d_b where
//      they differ, so b's sequence is K's prefix below d_b followed by b's own
//      rounds d_b..top_b (DESIGN.md s3.2's identity): K's rounds are emitted
//      once, and only the (round, leader) pairs of the leaders' own rounds
//      beside them.
//      PAPER: vertex v of round r goes to the first popped leader (first-pop
//      order) whose set holds it: per round the sets minus an exclusive prefix
//      OR over the leaders in first-pop order, then counts, per-leader prefix
//      sums and contributions.
// Supported: n <= 128, nw <= 64, weak deltas < ring slots (<= 32), no far
// edges, no repeated ids (dr_replay_batch takes dr_replay otherwise).
#pragma once
#include "kernels.hpp"

namespace dr {

struct SmallJob {
  const u64 *strong;
  const u64 *present;
  const uint32_t *wc_key;   // weak columns (kernels.hpp DagView::wc_*)
  const u64 *wc_rows;
  const uint32_t *wc_roff;
  const uint16_t *wdeg;     // [rounds][n] weak degree per vertex
  const uint16_t *sdeg;     // [rounds][n] strong degree per vertex (the wave form's emission)
  const uint32_t *slot_off;
  const uint16_t *slot_src;
  const uint16_t *lead;     // [wave] chooseLeader(w), 1-based source
  // scratch: cone sets F [T+1][2 words][64 leaders], per-leader strong-degree suffix
  // sums at the leader rounds [65][64], strong + weak degree per slot
  u64 *cone;
  uint32_t *sufl;
  uint32_t *deg;
  // outputs
  uint8_t *commit;      // [nw]
  int32_t *vcount;      // [nw]
  uint32_t *push_off;   // [nw + 1]
  int32_t *push_wave;   // [push_cap]
  u64 *pop_count;       // [push_cap]
  u64 *pop_digest;      // [push_cap]
  u64 *pop_edges;       // [push_cap]
  u64 *totals;          // [4]: commit edges, chain edges, deliver edges, n_push
  int32_t n, WS, push_cap, quorum;  // quorum = 2f+1 (process.go:337)
};

constexpr int kSmallMaxPops = 64 * 65 / 2;  // literal chains: wave w pushes up to w leaders
constexpr int kSmallNT = 256;               // four wavefronts per DAG
constexpr int kSmallPF = 4;                 // rounds loaded ahead by the cone passes
// u64 words of a job's cone scratch per round: the workgroup form's dense [2][64] sets, or
// the wave form's record (K, mask, up to 64 lanes' sets: 3 + 128 words)
constexpr int kConeRecWords = 131;

// dynamic LDS of k_replay_small (D = ring slots, a power of two above the
// largest weak delta): pass 2F's weak ring [D][2][64] u64 and K's weak targets
// [D][D][2] u64 (round x's targets at delta d, slot x mod D), then the
// per-(round, leader) counts / positions [T+1][64] u16
inline size_t small_lds_bytes(int D, int nw) {
  const int T = 4 * (nw - 1) + 1;
  return (size_t)D * 128 * 8 + (size_t)D * D * 2 * 8 + (size_t)(T + 1) * 64 * 2;
}

// global address space (loads and stores through these are global_*, not flat_*)
#define DR_GLOBAL __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ T DR_GLOBAL *as_global(T *p) {
  return (T DR_GLOBAL *)p;
}

// wavefront-local LDS ordering: a wave's LDS operations execute in order; this
// keeps the compiler from moving them across the point
__device__ __forceinline__ void wave_lds_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

// round r's data for a cone pass, loaded kSmallPF rounds ahead
struct SmallRound {
  u64 x0, x1, y0, y1;  // rows of vertices lane and lane + 64 (2 words each)
  u64 p0, p1;          // presence
  u64 cw0, cw1;        // the first 64 weak columns: lane j's source row ...
  uint32_t ckey;       // ... and key
  uint32_t c0, c1;     // the round's weak columns
};
// round r's data for the emission: every lane's set (lane = leader) and the
// first 128 slots (lane = slot)
struct EmitRound {
  u64 f0, f1;
  int s[2];
  uint32_t dg[2];
};

template <int D, bool PAPER, bool PERSIST>
__global__ __launch_bounds__(kSmallNT) void k_replay_small(const SmallJob *__restrict__ jobs, int njobs, int nw) {
  static_assert(D >= 2 && D <= 32 && (D & (D - 1)) == 0, "ring slots: a power of two");
  constexpr bool chain_persistent = PERSIST;  // persistent chains push every wave at most once: <= 64 pops
  constexpr int kMaxPops = PERSIST ? 64 : kSmallMaxPops;
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int jb = blockIdx.x;
  if (jb >= njobs) return;
  const SmallJob J = jobs[jb];
  // the job's arrays as global-memory pointers: flat accesses would also count
  // against lgkmcnt, so every LDS wait would wait for the rounds loaded ahead
  auto g_strong = as_global(J.strong);
  auto g_present = as_global(J.present);
  auto g_wc_key = as_global(J.wc_key);
  auto g_wc_rows = as_global(J.wc_rows);
  auto g_wc_roff = as_global(J.wc_roff);
  auto g_wdeg = as_global(J.wdeg);
  auto g_slot_off = as_global(J.slot_off);
  auto g_slot_src = as_global(J.slot_src);
  auto g_lead = as_global(J.lead);
  auto g_cone = as_global(J.cone);
  auto g_sufl = as_global(J.sufl);
  auto g_deg = as_global(J.deg);
  auto g_commit = as_global(J.commit);
  auto g_vcount = as_global(J.vcount);
  auto g_push_off = as_global(J.push_off);
  auto g_push_wave = as_global(J.push_wave);
  auto g_pop_count = as_global(J.pop_count);
  auto g_pop_digest = as_global(J.pop_digest);
  auto g_pop_edges = as_global(J.pop_edges);
  auto g_totals = as_global(J.totals);
  const int n = J.n, WS = J.WS;
  const int T = 4 * (nw - 1) + 1;
  const bool haveK = nw <= 63;         // lane 63 carries K when it is not a leader
  const bool kmemo = !PAPER && haveK;  // REF: leaders take K's prefix below their lowest difference
  extern __shared__ __attribute__((aligned(16))) u64 arena[];
  constexpr int M = D - 1;                                                     // ring slot = round & M
  u64 *ring = arena;                                                           // [D][2][64], pass 2F
  u64 *KWt = arena + (size_t)D * 128;                                          // [D][D][2], pass 2F
  uint16_t *cnt = reinterpret_cast<uint16_t *>(KWt + (size_t)D * D * 2);      // [T+1][64]
  __shared__ uint32_t s_roff[256], s_soff[256];  // weak-column and slot offsets of rounds 0..T+1
  __shared__ uint16_t s_lead[65];
  __shared__ u64 Dm[256];  // REF: leaders whose set differs from K's in round r; PAPER: leaders delivering in r
  __shared__ u64 QL[64];
  __shared__ u64 s_commit, s_lead_mask, s_cedges;
  __shared__ int s_done, s_npush, s_npop;
  __shared__ int32_t vc_s[64];
  __shared__ int16_t first_pop[64], d_lo[64];
  __shared__ int8_t ord[64];
  __shared__ int8_t coef[64 * 65];
  __shared__ uint8_t pop_lead[kMaxPops];
  __shared__ uint32_t kx[256];        // K's delivered vertices in rounds < r
  __shared__ u64 dKx[256], eKx[256];  // K's per-round digest / edges, then their exclusive prefixes
  __shared__ u64 res[64 * 3];         // per leader: count, digest, edges
  // profiling build: wall-clock stamps at the phase boundaries (tools/batch_timing.py)
  DR_TT(u64 *tt = jb < kSweepTimingQ ? g_sweep_timing + (size_t)jb * 16 : nullptr;
        auto stamp = [&](int k) { if (tt && lane == 0) tt[k] = wall_clock64(); };
        if (tid == 0) stamp(0);)

  for (int i = tid; i <= T + 1; i += kSmallNT) {
    s_roff[i] = g_wc_roff[i];
    s_soff[i] = g_slot_off[i];
  }
  for (int i = tid; i <= nw; i += kSmallNT) s_lead[i] = g_lead[i];
  if (tid == 0) {
    s_commit = 0;
    s_lead_mask = 0;
    s_cedges = 0;
    s_done = 0;
  }
  for (int i = tid; i < 64 * 3; i += kSmallNT) res[i] = 0;
  __syncthreads();
  const int my_lead = lane < nw ? s_lead[lane + 1] - 1 : 0;  // lane w-1: chooseLeader(w), 0-based

  auto row2 = [&](int r, int v, u64 &a, u64 &b) {  // row of (r, v+1); zero for v >= n
    a = 0;
    b = 0;
    if (v < n) {
      const u64 DR_GLOBAL *p = g_strong + ((size_t)r * n + v) * WS;
      if (WS == 2) {
        const u64x2 x = *reinterpret_cast<const u64x2 DR_GLOBAL *>(p);
        a = x.x;
        b = x.y;
      } else {
        a = p[0];
      }
    }
  };
  // a cone pass's loads are branch-free (a load under a lane-divergent branch makes
  // the compiler wait for it where the paths join): a vertex >= n is read at n-1
  // (it is never in a set, so its row is never used), a weak column past the
  // round's last at the last one (masked where it is used)
  auto row_raw = [&](int r, int v, u64 &a, u64 &b) {
    const int vc = v < n ? v : n - 1;
    const u64 DR_GLOBAL *p = g_strong + ((size_t)r * n + vc) * WS;
    if (WS == 2) {
      const u64x2 x = *reinterpret_cast<const u64x2 DR_GLOBAL *>(p);
      a = x.x;
      b = x.y;
    } else {
      a = p[0];
      b = 0;
    }
  };
  auto load_round = [&](int r, SmallRound &d, bool weak) {
    row_raw(r, lane, d.x0, d.x1);
    row_raw(r, lane + 64, d.y0, d.y1);
    d.p0 = g_present[(size_t)r * WS];
    d.p1 = WS > 1 ? g_present[(size_t)r * WS + 1] : 0ULL;
    if (weak) {
      d.c0 = s_roff[r];
      d.c1 = s_roff[r + 1];
      const uint32_t c1 = d.c1, jc = d.c0 + lane;
      const uint32_t jl = jc < c1 ? jc : (c1 > 0 ? c1 - 1 : 0);
      d.ckey = g_wc_key[jl];
      d.cw0 = g_wc_rows[(size_t)jl * WS];
      d.cw1 = WS > 1 ? g_wc_rows[(size_t)jl * WS + 1] : 0ULL;
    } else {
      d.ckey = 0;
      d.cw0 = d.cw1 = 0;
      d.c0 = d.c1 = 0;
    }
  };
  // OR of the rows of the set (s0, s1) (wave-uniform), and optionally the sum of
  // its members' strong degrees
  auto expand = [&](const SmallRound &d, u64 s0, u64 s1, u64 &n0, u64 &n1, uint32_t *dsum) {
    const bool m0 = (s0 >> lane) & 1ULL, m1 = (s1 >> lane) & 1ULL;
    n0 = wave_or((m0 ? d.x0 : 0ULL) | (m1 ? d.y0 : 0ULL));
    n1 = WS > 1 ? wave_or((m0 ? d.x1 : 0ULL) | (m1 ? d.y1 : 0ULL)) : 0ULL;
    if (dsum) {
      const uint32_t a = m0 ? (uint32_t)(__popcll(d.x0) + __popcll(d.x1)) : 0u;
      const uint32_t b = m1 ? (uint32_t)(__popcll(d.y0) + __popcll(d.y1)) : 0u;
      *dsum = (uint32_t)wave_sum((u64)(a + b));
    }
  };
  // a cone pass: rounds T down to 1, round r in register-ring slot (T - r) %
  // kSmallPF (a compile-time index in the unrolled body), refilled with round
  // r - kSmallPF as round r is taken
  auto cone_pass = [&](bool weak, auto &&body) {
    SmallRound pf[kSmallPF];
#pragma unroll
    for (int u = 0; u < kSmallPF; u++)
      if (T - u >= 1) load_round(T - u, pf[u], weak);
    for (int base = T; base >= 1; base -= kSmallPF) {
#pragma unroll
      for (int u = 0; u < kSmallPF; u++) {
        const int r = base - u;
        if (r < 1) break;
        const SmallRound cur = pf[u];
        if (r - kSmallPF >= 1) load_round(r - kSmallPF, pf[u], weak);
        body(r, cur);
      }
    }
  };

  if (wv == 0) {
    // ---------------- 2F. F_b over strong + weak edges (wave 0) ----------------
    for (int i = lane; i < D * 128 + D * D * 2; i += 64) ring[i] = 0;  // ring and KWt
    wave_lds_fence();
    u64 F0 = 0, F1 = 0;
    uint32_t E = 0;  // bit d-1: this lane's set was K's in round r+d (it takes K's weak targets from there)
    DR_TT(u64 cyc[6] = {0, 0, 0, 0, 0, 0}; u64 tc = __builtin_readcyclecounter();
          auto tick = [&](int k) { const u64 x = __builtin_readcyclecounter(); cyc[k] += x - tc; tc = x; };)
    cone_pass(true, [&](int r, const SmallRound &d) {
      DR_TT(tick(0);)  // waiting for the round's loads and the loop
      const int sl = r & M;
      F0 |= ring[(sl * 2) * 64 + lane];
      F1 |= ring[(sl * 2 + 1) * 64 + lane];
      ring[(sl * 2) * 64 + lane] = 0;
      ring[(sl * 2 + 1) * 64 + lane] = 0;
      if (haveK) {  // K's weak targets from rounds r+d, for the lanes whose set was K's there
        u64x2 kw[D];
#pragma unroll
        for (int dl = 2; dl < D; dl++) kw[dl] = *reinterpret_cast<const u64x2 *>(KWt + (((r + dl) & M) * D + dl) * 2);
#pragma unroll
        for (int dl = 2; dl < D; dl++)
          if ((E >> (dl - 1)) & 1u) {
            F0 |= kw[dl].x;
            F1 |= kw[dl].y;
          }
      }
      if (haveK && r == T && lane == 63) {  // K: every present vertex of the top round
        F0 |= d.p0;
        F1 |= d.p1;
      }
      if (((r - 1) & 3) == 0) {  // leader round of wave w: seed its lane with the leader's vertex
        const int w = (r - 1) / 4 + 1;
        const int l = __builtin_amdgcn_readlane(my_lead, w - 1);
        const bool present = (((l < 64) ? d.p0 : d.p1) >> (l & 63)) & 1ULL;
        if (present && lane == w - 1) {
          if (l < 64) F0 |= 1ULL << l; else F1 |= 1ULL << (l - 64);
        }
      }
      g_cone[((size_t)r * 2) * 64 + lane] = F0;
      g_cone[((size_t)r * 2 + 1) * 64 + lane] = F1;
      u64 K0 = 0, K1 = 0;
      if (haveK) {
        K0 = readlane64(F0, 63);
        K1 = readlane64(F1, 63);
      }
      // emission inputs: |F_b & P_r| and the leaders whose set differs from K's
      cnt[r * 64 + lane] = (uint16_t)(__popcll(F0 & d.p0) + __popcll(F1 & d.p1));
      const u64 dm = __ballot(lane < nw && (((F0 ^ K0) & d.p0) | ((F1 ^ K1) & d.p1)) != 0ULL);
      if (lane == 0) Dm[r] = dm;
      const bool eqF = haveK && F0 == K0 && F1 == K1;
      const u64 soloF = __ballot(!eqF && (F0 | F1) != 0ULL);
      DR_TT(tick(1);)
      // weak columns of round r (64 per batch, lane j holding column j; the first
      // batch came with the round): a column's target joins b's pending round iff
      // its sources meet F_b
      const uint32_t c0 = d.c0, c1 = d.c1;
      if (lane < 2 * D) KWt[(size_t)sl * D * 2 + lane] = 0;  // round r+D's targets: consumed above r
      wave_lds_fence();
      u64 cw0 = d.cw0, cw1 = d.cw1;
      uint32_t ckey = d.ckey;
      for (uint32_t cb = c0; cb < c1; cb += 64) {
        if (cb != c0) {
          const uint32_t jc = cb + lane, jl = jc < c1 ? jc : c1 - 1;
          ckey = g_wc_key[jl];
          cw0 = g_wc_rows[(size_t)jl * WS];
          cw1 = WS > 1 ? g_wc_rows[(size_t)jl * WS + 1] : 0ULL;
        }
        const int delta = (int)(ckey >> 11), ts = (int)(ckey & 2047u);
        const bool live = cb + lane < c1 && (cw0 | cw1) != 0ULL && r - delta >= 1;
        const u64 tb = 1ULL << (ts & 63);
        const int tw = ts >> 6, tsl = (r - delta) & M;
        if (haveK && live && ((cw0 & K0) | (cw1 & K1)) != 0ULL) atomicOr(&KWt[((size_t)sl * D + delta) * 2 + tw], tb);
        for (u64 m = soloF; m; m &= m - 1) {
          const int b = __builtin_ctzll(m);
          const u64 s0 = readlane64(F0, b), s1 = readlane64(F1, b);
          if (live && ((cw0 & s0) | (cw1 & s1)) != 0ULL) atomicOr(&ring[(tsl * 2 + tw) * 64 + b], tb);
        }
      }
      wave_lds_fence();
      DR_TT(tick(2);)
      E = (E << 1) | (eqF ? 1u : 0u);
      DR_TT(tick(3);)
      // strong edges: round r-1's sets
      u64 N0 = 0, N1 = 0;
      if (haveK) {
        u64 a, b;
        expand(d, K0, K1, a, b, nullptr);
        if (eqF) { N0 = a; N1 = b; }
      }
      DR_TT(tick(4);)
      for (u64 m = soloF; m; m &= m - 1) {
        const int b = __builtin_ctzll(m);
        u64 x, y;
        expand(d, readlane64(F0, b), readlane64(F1, b), x, y, nullptr);
        if (lane == b) { N0 = x; N1 = y; }
      }
      F0 = N0;
      F1 = N1;
      wave_lds_fence();
      DR_TT(tick(5);)
    });
    DR_TT(stamp(1); if (tt && lane == 0) for (int k = 0; k < 6; k++) tt[8 + k] = cyc[k];)
  } else {
    // ---------------- 1. commits (waves 1-3) ----------------
    u64 cm = 0, lm = 0, ce = 0;
    for (int w = wv; w <= nw; w += 3) {
      const int r1 = 4 * (w - 1) + 1;
      const int l = s_lead[w] - 1;  // chooseLeader(w), 0-based (< 128)
      const u64 pl = g_present[(size_t)r1 * WS + (l >> 6)];
      u64 a[3][2], b[3][2], p[3][2];
#pragma unroll
      for (int k = 0; k < 3; k++) {
        row2(r1 + 1 + k, lane, a[k][0], b[k][0]);
        row2(r1 + 1 + k, lane + 64, a[k][1], b[k][1]);
        p[k][0] = g_present[(size_t)(r1 + 1 + k) * WS];
        p[k][1] = WS > 1 ? g_present[(size_t)(r1 + 1 + k) * WS + 1] : 0ULL;
      }
      if (!((pl >> (l & 63)) & 1ULL)) {  // leader is bottom (process.go:327-329)
        if (lane == 0) vc_s[w - 1] = -1;
        continue;
      }
      lm |= 1ULL << (w - 1);
      u64 s0 = l < 64 ? 1ULL << l : 0ULL, s1 = l >= 64 ? 1ULL << (l - 64) : 0ULL, deg = 0;
#pragma unroll
      for (int k = 0; k < 3; k++) {
        const bool h0 = ((p[k][0] >> lane) & 1ULL) && (((a[k][0] & s0) | (b[k][0] & s1)) != 0ULL);
        const bool h1 = ((p[k][1] >> lane) & 1ULL) && (((a[k][1] & s0) | (b[k][1] & s1)) != 0ULL);
        s0 = __ballot(h0);
        s1 = __ballot(h1);
        deg += (u64)(__popcll(a[k][0]) + __popcll(b[k][0]) + __popcll(a[k][1]) + __popcll(b[k][1]));
      }
      ce += wave_sum(deg);
      const int vc = __popcll(s0) + __popcll(s1);
      if (lane == 0) vc_s[w - 1] = vc;
      if (vc >= J.quorum) cm |= 1ULL << (w - 1);
    }
    if (lane == 0) {
      atomicOr(&s_commit, cm);
      atomicOr(&s_lead_mask, lm);
      atomicAdd(&s_cedges, ce);
      __hip_atomic_fetch_add(&s_done, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (wv == 1) {
      // ---------------- 2G. G_b over strong edges only, QL, suffix sums (wave 1) ----------------
      // waves 1-3 of this workgroup are resident and finish the commits unconditionally
      while (__hip_atomic_load(&s_done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < 3)
        __builtin_amdgcn_s_sleep(1);
      const u64 commit_mask = __hip_atomic_load(&s_commit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      const u64 lead_mask = __hip_atomic_load(&s_lead_mask, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      // chains (process.go:341-350) inspect leader b's strong cone only down to the
      // floor round of the commit whose chain can push b: 4*decidedWave + 1, with
      // decidedWave the last commit below wave b+1 (never inspected without a
      // commit at or above wave b+1)
      int my_floor = 0x7fff;
      if (lane < nw && (commit_mask >> lane) != 0ULL) {
        const u64 below = commit_mask & ((1ULL << lane) - 1ULL);
        const int lastc = below ? 64 - __builtin_clzll(below) : 0;
        my_floor = chain_persistent ? 4 * lastc + 1 : 1;
      }
      u64 G0 = 0, G1 = 0;
      uint32_t suf = 0;  // strong degrees summed over G_b, rounds r..T
      cone_pass(false, [&](int r, const SmallRound &d) {
        const bool alive = (lane < nw && my_floor <= r) || (haveK && lane == 63);
        if (!alive) G0 = G1 = 0;
        if (haveK && r == T && lane == 63) {
          G0 = d.p0;
          G1 = d.p1;
        }
        if (((r - 1) & 3) == 0) {
          const int w = (r - 1) / 4 + 1;
          const int l = __builtin_amdgcn_readlane(my_lead, w - 1);
          if ((lead_mask >> (w - 1)) & 1ULL) {
            if (lane == w - 1 && alive) {
              if (l < 64) G0 |= 1ULL << l; else G1 |= 1ULL << (l - 64);
            }
            // the leaders whose strong cone holds this leader's vertex (the chains' test)
            const u64 ql = __ballot(lane < nw && ((((l < 64) ? G0 : G1) >> (l & 63)) & 1ULL));
            if (lane == 0) QL[w - 1] = ql;
          } else if (lane == 0) {
            QL[w - 1] = 0;
          }
        }
        u64 K0 = 0, K1 = 0;
        if (haveK) {
          K0 = readlane64(G0, 63);
          K1 = readlane64(G1, 63);
        }
        const bool eqG = haveK && G0 == K0 && G1 == K1;
        const u64 soloG = __ballot(!eqG && (G0 | G1) != 0ULL);
        u64 H0 = 0, H1 = 0;
        if (haveK) {
          u64 a, b;
          uint32_t ds;
          expand(d, K0, K1, a, b, &ds);
          if (eqG) { H0 = a; H1 = b; suf += ds; }
        }
        for (u64 m = soloG; m; m &= m - 1) {
          const int b = __builtin_ctzll(m);
          u64 x, y;
          uint32_t ds;
          expand(d, readlane64(G0, b), readlane64(G1, b), x, y, &ds);
          if (lane == b) { H0 = x; H1 = y; suf += ds; }
        }
        if (r >= 2 && ((r - 2) & 3) == 0) g_sufl[((r - 2) / 4 + 1) * 64 + lane] = suf;  // Suf_b(4(x-1)+2)
        G0 = H0;
        G1 = H1;
      });
    } else {
      // ---------------- 2D. strong + weak degree per slot (waves 2-3) ----------------
      for (int r = wv - 1; r <= T; r += 2) {
        const uint32_t sa = s_soff[r], sb = s_soff[r + 1];
        for (uint32_t s = sa + lane; s < sb; s += 64) {
          const int src = g_slot_src[s];
          uint32_t dg = 0;
          if (src > 0) {
            u64 a, b;
            row2(r, src - 1, a, b);
            dg = (uint32_t)(__popcll(a) + __popcll(b)) + g_wdeg[(size_t)r * n + src - 1];
          }
          g_deg[s] = dg;
        }
      }
    }
  }
  __syncthreads();
  DR_TT(if (tid == 0) stamp(2);)

  // ---------------- 3. chains and pops (wave 0: lane j holds QL[j]) ----------------
  const u64 commit_mask = s_commit;
  for (int i = tid; i < 64 * 65; i += kSmallNT) coef[i] = 0;
  if (tid < 64) first_pop[tid] = -1;
  __syncthreads();
  if (wv == 0) {
    const u64 ql = QL[lane], lmask = s_lead_mask;
    int npush = 0, npop = 0, last = 0;
    for (int w = 1; w <= nw; w++) {
      if (lane == 0) g_push_off[w - 1] = (uint32_t)npush;
      if (!((commit_mask >> (w - 1)) & 1ULL)) continue;
      const int floor_w = chain_persistent ? last : 0;
      // pushed leaders of this commit in push order, lane i holding the i-th
      int k = 1, L = w, myL = lane == 0 ? w : 0;
      for (int w2 = w - 1; w2 >= floor_w + 1; w2--) {
        if (((lmask >> (w2 - 1)) & 1ULL) && ((readlane64(ql, w2 - 1) >> (L - 1)) & 1ULL)) {
          if (lane == k) myL = w2;
          k++;
          L = w2;
        }
      }
      const int nextL = __shfl_down(myL, 1);
      if (lane < k) {
        // chain edges: segment i expands leader list[i]'s strong cone over rounds
        // (round(list[i+1]), round(list[i])], the last one down to round(floor+1)
        const int lo = lane + 1 < k ? nextL : floor_w + 1;
        coef[(myL - 1) * 65 + myL] += 1;
        coef[(myL - 1) * 65 + lo] -= 1;
        if (npush + lane < J.push_cap) g_push_wave[npush + lane] = myL;
        const int j = npop + (k - 1 - lane);  // pops: reverse push order (stack/stack.go:23-28)
        if (j < kMaxPops) pop_lead[j] = (uint8_t)myL;
        if (first_pop[myL - 1] < 0) first_pop[myL - 1] = (int16_t)j;
      }
      wave_lds_fence();
      npush += k;
      npop += k;
      last = w;
    }
    if (lane == 0) {
      g_push_off[nw] = (uint32_t)npush;
      s_npush = npush;
      s_npop = npop;
    }
  }
  __syncthreads();
  const int npush = s_npush, npop = s_npop;
  DR_TT(if (tid == 0) stamp(3);)

  // ---------------- 4. emission ----------------
  const int myfirst = first_pop[lane];
  const u64 popped = __ballot(lane < nw && myfirst >= 0);
  const int npopped = __popcll(popped);
  int myrank = 0;  // PAPER: leaders first popped before b
  for (int x = 0; x < 64; x++) {
    const int fp = first_pop[x];
    myrank += (fp >= 0 && myfirst >= 0 && fp < myfirst) ? 1 : 0;
  }
  if (PAPER && wv == 0 && myfirst >= 0) ord[myrank] = (int8_t)lane;
  // chain edges: segment sums are differences of the suffix sums at the leader
  // rounds (every leader's coefficients sum to zero; Suf = 0 above round T)
  u64 chain = 0;
  if (wv == 0) {
    for (int x = 1; x < nw; x++) {
      const int c = coef[lane * 65 + x];
      if (c) chain -= (u64)((int64_t)c * (int64_t)g_sufl[x * 64 + lane]);
    }
    chain = wave_sum(chain);
  }
  auto load_emit = [&](int r, EmitRound &e) {  // branch-free: slots past the round's end masked in contrib
    e.f0 = g_cone[((size_t)r * 2) * 64 + lane];
    e.f1 = g_cone[((size_t)r * 2 + 1) * 64 + lane];
    const uint32_t sa = s_soff[r], sb = s_soff[r + 1];
#pragma unroll
    for (int i = 0; i < 2; i++) {
      const uint32_t sl = sa + 64 * i + lane, sc = sl < sb ? sl : (sb > 0 ? sb - 1 : 0);
      e.s[i] = (int)g_slot_src[sc];
      e.dg[i] = g_deg[sc];
    }
  };
  // contribution of the set (s0, s1) to round r's delivery, positions from k0
  // (lanes = slots in insertion order): digest and edges (wave-uniform)
  auto contrib = [&](int r, const EmitRound &e, u64 s0, u64 s1, u64 k0, u64 &dg, u64 &ed) {
    const uint32_t sa = s_soff[r], sb = s_soff[r + 1];
    u64 k = k0, dacc = 0, eacc = 0;
    for (uint32_t c0 = sa, i = 0; c0 < sb; c0 += 64, i++) {
      int s;
      uint32_t dgv;
      if (i < 2) {
        s = c0 + lane < sb ? e.s[i] : 0;  // 0: ghost / none
        dgv = e.dg[i];
      } else {
        const uint32_t sl = c0 + lane;
        s = sl < sb ? (int)g_slot_src[sl] : 0;
        dgv = sl < sb ? g_deg[sl] : 0u;
      }
      const int v = s - 1;
      const bool in = s > 0 && ((((v < 64) ? s0 : s1) >> (v & 63)) & 1ULL);
      const u64 bal = __ballot(in);
      if (in) {
        dacc += digest_term((uint32_t)r, (uint32_t)s, k + (u64)__popcll(bal & ((1ULL << lane) - 1ULL)));
        eacc += dgv;
      }
      k += (u64)__popcll(bal);
    }
    dg = wave_sum(dacc);
    ed = wave_sum(eacc);
  };
  // rounds 1 + wv, 5 + wv, ... of this wave, each loaded kEPF of them ahead
  // (register ring, compile-time slots in the unrolled body)
  constexpr int kEPF = 4;
  auto emit_rounds = [&](auto &&body) {
    EmitRound pf[kEPF];
#pragma unroll
    for (int u = 0; u < kEPF; u++)
      if (1 + wv + 4 * u <= T) load_emit(1 + wv + 4 * u, pf[u]);
    for (int base = 1 + wv; base <= T; base += 4 * kEPF) {
#pragma unroll
      for (int u = 0; u < kEPF; u++) {
        const int r = base + 4 * u;
        if (r > T) break;
        const EmitRound cur = pf[u];
        if (r + 4 * kEPF <= T) load_emit(r + 4 * kEPF, pf[u]);
        body(r, cur);
      }
    }
  };
  __syncthreads();
  if (!PAPER) {
    // 4a. K's positions (wave 0); each popped leader's lowest round differing from K (wave 1)
    if (wv == 0 && haveK) {
      constexpr int PER = 4;  // rounds per lane: T + 2 <= 256
      uint32_t v[PER], loc = 0;
#pragma unroll
      for (int j = 0; j < PER; j++) {
        const int r = lane * PER + j;
        v[j] = (r >= 1 && r <= T) ? cnt[r * 64 + 63] : 0u;
        loc += v[j];
      }
      uint32_t inc = loc;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(inc, off);
        if (lane >= off) inc += y;
      }
      uint32_t run = inc - loc;
#pragma unroll
      for (int j = 0; j < PER; j++) {
        kx[lane * PER + j] = run;
        run += v[j];
      }
    }
    if (wv == 1) {
      int d = 0x7fff;
      if ((popped >> lane) & 1ULL) {
        const int top = 4 * lane + 1;
        d = kmemo ? top + 1 : 1;
        if (kmemo)
          for (int r = 1; r <= top; r++)
            if ((Dm[r] >> lane) & 1ULL) {
              d = r;
              break;
            }
      }
      d_lo[lane] = (int16_t)d;
    }
    __syncthreads();
    // 4b. each popped leader's own rounds d_b..top_b: positions = K's count below
    //     d_b + its own counts (lane b, counts -> positions in place)
    if (wv == 0 && ((popped >> lane) & 1ULL)) {
      const int d = d_lo[lane], top = 4 * lane + 1;
      uint32_t run = kmemo ? kx[d] : 0u;
      for (int r = d; r <= top; r++) {
        const uint32_t c = cnt[r * 64 + lane];
        cnt[r * 64 + lane] = (uint16_t)run;
        run += c;
      }
      if (d <= top) res[lane * 3 + 0] = run;
    }
    // own rounds of round r: the popped leaders with d_b <= r <= top_b
    const int my_d = d_lo[lane];
    __syncthreads();
    // 4c. contributions, parallel over rounds: K's (per round) and the leaders' own
    emit_rounds([&](int r, const EmitRound &e) {
      if (haveK) {
        u64 dg, ed;
        contrib(r, e, readlane64(e.f0, 63), readlane64(e.f1, 63), kx[r], dg, ed);
        if (lane == 0) {
          dKx[r] = dg;
          eKx[r] = ed;
        }
      }
      for (u64 m = __ballot(((popped >> lane) & 1ULL) && my_d <= r && r <= 4 * lane + 1); m; m &= m - 1) {
        const int b = __builtin_ctzll(m);
        u64 dg, ed;
        contrib(r, e, readlane64(e.f0, b), readlane64(e.f1, b), cnt[r * 64 + b], dg, ed);
        if (lane == 0) {
          atomicAdd(&res[b * 3 + 1], dg);
          atomicAdd(&res[b * 3 + 2], ed);
        }
      }
    });
    __syncthreads();
    // 4d. K's digest / edge prefixes, then each leader's totals
    if (wv == 0 && haveK) {
      constexpr int PER = 4;
      u64 v0[PER], v1[PER], l0 = 0, l1 = 0;
#pragma unroll
      for (int j = 0; j < PER; j++) {
        const int r = lane * PER + j;
        v0[j] = (r >= 1 && r <= T) ? dKx[r] : 0ULL;
        v1[j] = (r >= 1 && r <= T) ? eKx[r] : 0ULL;
        l0 += v0[j];
        l1 += v1[j];
      }
      u64 i0 = l0, i1 = l1;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const u64 y0 = shfl_up64(i0, off), y1 = shfl_up64(i1, off);
        if (lane >= off) {
          i0 += y0;
          i1 += y1;
        }
      }
      u64 a0 = i0 - l0, a1 = i1 - l1;
      wave_lds_fence();
#pragma unroll
      for (int j = 0; j < PER; j++) {
        dKx[lane * PER + j] = a0;
        eKx[lane * PER + j] = a1;
        a0 += v0[j];
        a1 += v1[j];
      }
      wave_lds_fence();
      if ((popped >> lane) & 1ULL) {
        const int d = my_d, top = 4 * lane + 1;
        if (d > top) {  // equal to K up to its own round: K's prefix through it
          res[lane * 3 + 0] = kx[top + 1];
          res[lane * 3 + 1] = dKx[top + 1];
          res[lane * 3 + 2] = eKx[top + 1];
        } else {        // K's prefix below d, then its own rounds
          res[lane * 3 + 1] += dKx[d];
          res[lane * 3 + 2] += eKx[d];
        }
      }
    }
  } else {
    // per round: what each popped leader delivers -- its set minus what the
    // leaders popped before it hold (exclusive prefix OR in first-pop order)
    auto paper_sets = [&](int r, const EmitRound &e, u64 &x0, u64 &x1) -> u64 {
      const u64 P0 = g_present[(size_t)r * WS], P1 = WS > 1 ? g_present[(size_t)r * WS + 1] : 0ULL;
      const u64 active = popped & __ballot(lane < nw && 4 * lane + 1 >= r);  // leaders whose top >= r
      const int src = lane < npopped ? (int)ord[lane] : 0;
      u64 y0 = shfl64(e.f0, src), y1 = shfl64(e.f1, src);
      if (lane >= npopped) y0 = y1 = 0;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const u64 z0 = shfl_up64(y0, off), z1 = shfl_up64(y1, off);
        if (lane >= off) {
          y0 |= z0;
          y1 |= z1;
        }
      }
      u64 e0 = shfl_up64(y0, 1), e1 = shfl_up64(y1, 1);
      if (lane == 0) e0 = e1 = 0;
      x0 = e.f0 & ~shfl64(e0, myrank);
      x1 = e.f1 & ~shfl64(e1, myrank);
      const u64 m = __ballot(((x0 & P0) | (x1 & P1)) != 0ULL) & active;
      x0 &= P0;
      x1 &= P1;
      return m;
    };
    // 4a. counts per (round, leader)
    emit_rounds([&](int r, const EmitRound &e) {
      u64 x0, x1;
      const u64 m = paper_sets(r, e, x0, x1);
      cnt[r * 64 + lane] = ((m >> lane) & 1ULL) ? (uint16_t)(__popcll(x0) + __popcll(x1)) : (uint16_t)0;
      if (lane == 0) Dm[r] = m;
    });
    __syncthreads();
    // 4b. per leader (lane): positions = exclusive prefix of its counts over rounds
    if (wv == 0 && lane < nw) {
      uint32_t run = 0;
      for (int r = 1; r <= T; r++) {
        const uint32_t c = cnt[r * 64 + lane];
        cnt[r * 64 + lane] = (uint16_t)run;
        run += c;
      }
      res[lane * 3 + 0] = run;
    }
    __syncthreads();
    // 4c. contributions, parallel over rounds
    emit_rounds([&](int r, const EmitRound &e) {
      u64 x0, x1;
      paper_sets(r, e, x0, x1);
      for (u64 m = Dm[r]; m; m &= m - 1) {
        const int b = __builtin_ctzll(m);
        u64 dg, ed;
        contrib(r, e, readlane64(x0, b), readlane64(x1, b), cnt[r * 64 + b], dg, ed);
        if (lane == 0) {
          atomicAdd(&res[b * 3 + 1], dg);
          atomicAdd(&res[b * 3 + 2], ed);
        }
      }
    });
  }
  __syncthreads();
  DR_TT(if (tid == 0) stamp(4);)

  // ---------------- 5. outputs ----------------
  if (wv == 0) {
    u64 dsum = 0;
    const int np = min(npop, min(J.push_cap, kMaxPops));
    for (int j = lane; j < np; j += 64) {
      const int lb = pop_lead[j] - 1;
      u64 c = 0, d = 0, e = 0;  // PAPER: a leader's cone goes to its first pop only
      if (!PAPER || first_pop[lb] == j) {
        c = res[lb * 3 + 0];
        d = res[lb * 3 + 1];
        e = res[lb * 3 + 2];
      }
      g_pop_count[j] = c;
      g_pop_digest[j] = d;
      g_pop_edges[j] = e;
      dsum += e;
    }
    dsum = wave_sum(dsum);
    if (lane < nw) {
      g_vcount[lane] = vc_s[lane];
      g_commit[lane] = (uint8_t)((commit_mask >> lane) & 1ULL);
    }
    if (lane == 0) {
      g_totals[0] = s_cedges;
      g_totals[1] = chain;
      g_totals[2] = dsum;
      g_totals[3] = (u64)npush;
    }
  }
  DR_TT(if (tid == 0) stamp(5);)
}

}  // namespace dr
