// batch1w.hpp -- the throughput form of the fused small-DAG replay: one
// wavefront per DAG (batch.hpp holds the workgroup-per-DAG form and the job
// layout).  A wave walks its DAG's phases in order: commits, one bit-sliced
// top-down cone pass (lane b = leader b, lane 63 = the canonical cone K) for the
// strong+weak sets F_b and their strong-only twins G_b, chains from the leaders'
// strong cones, then a bottom-up emission in which a leader equal to K below its
// top takes K's prefix.  Sixteen DAGs share a CU, so when a
// batch holds many DAGs per CU (C5 on one GPU: 4096 / 256 CUs) the SIMDs stay
// busy and the batch's total work bounds it; dr_replay_batch picks this form
// there and the four-wave form when each CU holds only a few DAGs (one GPU's
// share at N = 8).  Same semantics and limits as batch.hpp.
#pragma once
#include "batch.hpp"

namespace dr {

// Materialise a value here: an empty asm that reads it keeps the compiler from sinking its
// computation (and the wait for the load it came from) below the next round's prefetch,
// where the wait's in-order count then covered the prefetch's loads too.
__device__ __forceinline__ void pin_vgpr(u64 x) { asm volatile("" : : "v"(x)); }
__device__ __forceinline__ void pin_vgpr(uint32_t x) { asm volatile("" : : "v"(x)); }

// dynamic LDS of k_replay_small_1w: the weak ring (rsl slots of 128 u64) or the
// later phases' arrays, whichever is larger
template <bool PAPER, bool PERSIST>
constexpr int small1w_late_bytes() {  // coef, pop list, per-leader results
  return 64 * 65 + (((PERSIST ? 64 : kSmallMaxPops) + 255) & ~255) + 64 * (PAPER ? 6 : 3) * 8;
}
template <bool PAPER, bool PERSIST>
inline size_t small1w_lds_bytes(int rsl) {
  const size_t ring = (size_t)rsl * 128 * 8, late = (size_t)small1w_late_bytes<PAPER, PERSIST>();
  return ring > late ? ring : late;
}

template <bool PAPER, bool PERSIST>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) void k_replay_small_1w(const SmallJob *__restrict__ jobs, int njobs, int nw, int rsl) {
  constexpr bool paper = PAPER;  // REF mode skips the paper-mode digests entirely
  constexpr bool chain_persistent = PERSIST;  // persistent chains push every wave at most once: <= 64 pops
  // LDS is what limits DAGs per CU: the weak ring (phase 2 only) shares its
  // bytes with the chain coefficients, pop list and per-leader results (phases
  // 3-5, which start after phase 2's last barrier).
  constexpr int kMaxPops = PERSIST ? 64 : kSmallMaxPops;
  constexpr int RS = PAPER ? 6 : 3;  // per-leader results kept
  constexpr int kCoefB = 64 * 65, kPopB = (kMaxPops + 255) & ~255, kResB = 64 * RS * 8;
  static_assert(kCoefB + kPopB + kResB == small1w_late_bytes<PAPER, PERSIST>(), "LDS layout");
  // lane 63 carries the canonical cone K when it is not a leader
  const bool haveK = nw <= 63;
  const bool kmemo = !PAPER && haveK;  // REF memo: leaders take K's prefix below their first difference
  extern __shared__ __attribute__((aligned(16))) u64 arena[];                  // small_lds_bytes(rsl)
  u64 *ring = arena;                                                            // [rsl][2][64], phase 2
  int8_t *coef = reinterpret_cast<int8_t *>(arena);                             // [64 * 65], phases 3-4
  uint8_t *pop_lead = reinterpret_cast<uint8_t *>(arena) + kCoefB;              // [kSmallMaxPops], 3-5
  u64 *res = reinterpret_cast<u64 *>(reinterpret_cast<char *>(arena) + ((kCoefB + kPopB + 7) & ~7));  // 4-5
  __shared__ u64 KW[64];            // K's weak targets of the current round, [delta][word]
  __shared__ uint32_t DG[128];
  __shared__ u64 QL[64];
  __shared__ int32_t vc_s[64];
  __shared__ int16_t first_pop[64];
  __shared__ int8_t lst[64];
  __shared__ int8_t ord[64];        // PAPER: popped leaders in first-pop order
  const int lane = threadIdx.x;
  const int jb = blockIdx.x;
  if (jb >= njobs) return;
  // profiling build: wall-clock stamps at the phase boundaries, cycle counts of the cone
  // pass's parts (tools/batch_timing.py)
  DR_TT(u64 *tt = jb < kSweepTimingQ ? g_sweep_timing + (size_t)jb * 16 : nullptr;
        auto stamp = [&](int k) { if (tt && lane == 0) tt[k] = wall_clock64(); };
        stamp(0);)
  const SmallJob J = jobs[jb];
  auto g_strong = as_global(J.strong);
  auto g_present = as_global(J.present);
  auto g_wc_key = as_global(J.wc_key);
  auto g_wc_rows = as_global(J.wc_rows);
  auto g_wc_roff = as_global(J.wc_roff);
  auto g_wdeg = as_global(J.wdeg);
  auto g_sdeg = as_global(J.sdeg);
  auto g_slot_off = as_global(J.slot_off);
  auto g_slot_src = as_global(J.slot_src);
  auto g_lead = as_global(J.lead);
  auto g_cone = as_global(J.cone);
  auto g_sufl = as_global(J.sufl);
  auto g_commit = as_global(J.commit);
  auto g_vcount = as_global(J.vcount);
  auto g_push_off = as_global(J.push_off);
  auto g_push_wave = as_global(J.push_wave);
  auto g_pop_count = as_global(J.pop_count);
  auto g_pop_digest = as_global(J.pop_digest);
  auto g_pop_edges = as_global(J.pop_edges);
  auto g_totals = as_global(J.totals);
  const int n = J.n, WS = J.WS;
  const int q = J.quorum;
  const int T = 4 * (nw - 1) + 1;
  auto row = [&](int r, int v, u64 &a, u64 &b) {  // row of (r, v+1); zero for v >= n
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
  auto pres_word = [&](int r, int w) -> u64 { return w < WS ? g_present[(size_t)r * WS + w] : 0ULL; };
  // The per-round weak-column and slot offsets (rounds 0..T+1 <= 254) and the leaders
  // (waves 0..nw <= 64) in registers -- lane l holds entries l, 64+l, 128+l, 192+l --
  // read by wave-uniform readlane.  The prefetches of the passes below take their
  // addresses from them: an address that came from a load just issued made the wave
  // wait for that load, and for every load issued before it, so each round had paid a
  // full memory latency (profiles/r05/v20_batch_timing.jsonl).
  uint32_t roffv[4], soffv[4], leadv[2];  // (soffv: loaded for the emission, phase 4)
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int i = 64 * k + lane, ic = i <= T + 1 ? i : T + 1;
    roffv[k] = g_wc_roff[ic];
  }
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const int i = 64 * k + lane;
    leadv[k] = g_lead[i <= nw ? i : nw];
  }
  auto tab4 = [&](const uint32_t (&v)[4], int i) -> uint32_t {  // i wave-uniform
    const int k = i >> 6;
    const uint32_t x = k == 0 ? v[0] : k == 1 ? v[1] : k == 2 ? v[2] : v[3];
    return (uint32_t)__builtin_amdgcn_readlane((int)x, i & 63);
  };
  auto lead_of = [&](int w) -> int {  // chooseLeader(w), 1-based source
    return __builtin_amdgcn_readlane((int)(w < 64 ? leadv[0] : leadv[1]), w & 63);
  };

  // ---------------- 1. leaders ----------------
  // (the commit rule runs inside the cone pass below, on the rows it reads anyway: a
  // separate pass had re-read three of every four rounds, profiles/r05/)
  u64 commit_mask = 0, commit_edges = 0;
  u64 lead_mask;
  {
    bool lp = false;
    if (lane < nw) {
      const int l = g_lead[lane + 1] - 1;  // chooseLeader(w), 0-based (< 128)
      lp = (pres_word(4 * lane + 1, l >> 6) >> (l & 63)) & 1ULL;
    }
    lead_mask = __ballot(lp);
    if (lane < nw && !lp) vc_s[lane] = -1;
  }
  DR_TT(stamp(1); u64 cyc[6] = {0, 0, 0, 0, 0, 0}; u64 tc = __builtin_readcyclecounter();
        auto tick = [&](int k) { const u64 x = __builtin_readcyclecounter(); cyc[k] += x - tc; tc = x; };)

  // ---------------- 2. top-down cone pass (lane b: leader b's sets) ----------------
  for (int i = lane; i < rsl * 128; i += 64) ring[i] = 0;
  KW[lane] = 0;
  __syncthreads();
  // leader b's strong cone is followed to round 1 (the chains read its degree sums only
  // from their floor up; the commits, which would set the floors, are decided in this pass)
  const bool alive = lane < nw || (haveK && lane == 63);
  // the commit rule (process.go:326-339) of the wave whose leader round is r: rows and
  // presence of rounds r+1 .. r+3, kept from the iterations above (lanes v, v + 64)
  // hp[k]: bit i = vertex lane + 64 i present (two bits instead of two presence words)
  u64 ha[3][2], hb[3][2];
  uint32_t hp[3];
  auto pbits = [&](u64 p0, u64 p1) -> uint32_t {
    return (uint32_t)((p0 >> lane) & 1ULL) | ((uint32_t)((p1 >> lane) & 1ULL) << 1);
  };
#pragma unroll
  for (int k = 0; k < 3; k++) {  // rounds T+1 .. T+3 (the top wave's; the DAG holds 4 nw + 1 rounds)
    row(T + 1 + k, lane, ha[k][0], hb[k][0]);
    row(T + 1 + k, lane + 64, ha[k][1], hb[k][1]);
    hp[k] = pbits(pres_word(T + 1 + k, 0), pres_word(T + 1 + k, 1));
  }
  uint32_t crec = (uint32_t)(T + 1) * kConeRecWords;  // the cone records (below)
  u64 F0 = 0, F1 = 0;  // F_b: round-r vertices in leader b's cone
  u64 G0 = 0, G1 = 0;  // G_b: the same over strong edges only
  uint32_t suf = 0;    // strong degrees summed over G_b, rounds r..T
  // round r's vertices (lanes v, v + 64): rows, strong degrees; b's expansion over its set
  u64 ra[2], rb[2];
  uint32_t sd[2];
  auto expand = [&](u64 s0, u64 s1, u64 &n0, u64 &n1, uint32_t *dsum) {  // s: wave-uniform
    const bool m0 = (s0 >> lane) & 1ULL, m1 = (s1 >> lane) & 1ULL;
    n0 = wave_or((m0 ? ra[0] : 0ULL) | (m1 ? ra[1] : 0ULL));
    n1 = WS > 1 ? wave_or((m0 ? rb[0] : 0ULL) | (m1 ? rb[1] : 0ULL)) : 0ULL;
    if (dsum) *dsum = (uint32_t)wave_sum((u64)((m0 ? sd[0] : 0u) + (m1 ? sd[1] : 0u)));
  };
  // software pipeline: round r-1's rows, presence, weak degrees and first 64 weak
  // columns (they do not depend on the cones) load while round r is processed, into
  // one of two register sets that the 2x unrolled loop below uses in turn (one set
  // rotated through moves at the loop's back edge made the wave wait there for the
  // loads it had just issued; the offsets come from registers, tab4)
  struct Pf {
    u64 ra[2], rb[2], w0, w1;
    uint32_t pr[2];  // the 32-bit half of each presence word that holds this lane's bit
    uint32_t key, c0, c1;
  };
  // Every load unconditional, at a clamped address, its value masked only where the round
  // uses it (cone_round): a conditional load, or a select right after a load, made the
  // wave wait for the loads just issued.  A row is one 16-B load (WS = 1: the second word
  // is the next row's, masked; the mirror's strong buffer has a row of slack); a column
  // index past the round's columns reads column 0 (the key buffers hold >= 4 KiB).
  auto prefetch2 = [&](int r, Pf &p) {
    p.c0 = tab4(roffv, r);
    p.c1 = tab4(roffv, r + 1);
    const uint32_t jc = p.c0 + lane, jcc = jc < p.c1 ? jc : 0u;
    p.key = g_wc_key[jcc];
    p.w0 = g_wc_rows[(size_t)jcc * WS];
    p.w1 = g_wc_rows[(size_t)jcc * WS + (WS > 1 ? 1 : 0)];
#pragma unroll
    for (int i = 0; i < 2; i++) {
      const int v = lane + 64 * i, vc = v < n ? v : 0;
      const u64x2 x = *reinterpret_cast<const u64x2 DR_GLOBAL *>(g_strong + ((size_t)r * n + vc) * WS);
      p.ra[i] = x.x;
      p.rb[i] = x.y;
    }
    const uint32_t DR_GLOBAL *ph = reinterpret_cast<const uint32_t DR_GLOBAL *>(g_present + (size_t)r * WS);
    p.pr[0] = ph[lane >> 5];
    p.pr[1] = ph[(WS > 1 ? 2 : 0) + (lane >> 5)];
  };
  auto cone_round = [&](int r, const Pf &cur, Pf &nxt) {
    DR_TT(tick(0);)  // the loop and the round's loads
#pragma unroll
    for (int i = 0; i < 2; i++) {  // the prefetched words, masked (prefetch2)
      const bool in = lane + 64 * i < n;
      ra[i] = in ? cur.ra[i] : 0ULL;
      rb[i] = in && WS > 1 ? cur.rb[i] : 0ULL;
      sd[i] = (uint32_t)(__popcll(ra[i]) + __popcll(rb[i]));
    }
    const uint32_t cpb = ((cur.pr[0] >> (lane & 31)) & 1u) | (WS > 1 ? ((cur.pr[1] >> (lane & 31)) & 1u) << 1 : 0u);
    if (((r - 1) & 3) == 0) {  // leader round of wave w: its vote from rounds r+1 .. r+3
      const int w = (r - 1) / 4 + 1;
      if ((lead_mask >> (w - 1)) & 1ULL) {
        const int l = lead_of(w) - 1;
        u64 s0 = l < 64 ? 1ULL << l : 0ULL, s1 = l >= 64 ? 1ULL << (l - 64) : 0ULL, deg = 0;
#pragma unroll
        for (int k = 0; k < 3; k++) {
          const bool h0 = (hp[k] & 1u) && (((ha[k][0] & s0) | (hb[k][0] & s1)) != 0ULL);
          const bool h1 = (hp[k] & 2u) && (((ha[k][1] & s0) | (hb[k][1] & s1)) != 0ULL);
          s0 = __ballot(h0);
          s1 = __ballot(h1);
          deg += (u64)(__popcll(ha[k][0]) + __popcll(hb[k][0]) + __popcll(ha[k][1]) + __popcll(hb[k][1]));
        }
        commit_edges += wave_sum(deg);
        const int vc = __popcll(s0) + __popcll(s1);
        if (lane == 0) vc_s[w - 1] = vc;
        if (vc >= q) commit_mask |= 1ULL << (w - 1);
      }
    }
    DR_TT(tick(1);)  // the commit rule
#pragma unroll
    for (int i = 0; i < 2; i++) {  // round r joins the history (r+1 .. r+3 for the next leader round)
      ha[2][i] = ha[1][i];
      hb[2][i] = hb[1][i];
      ha[1][i] = ha[0][i];
      hb[1][i] = hb[0][i];
      ha[0][i] = ra[i];
      hb[0][i] = rb[i];
    }
    hp[2] = hp[1];
    hp[1] = hp[0];
    hp[0] = cpb;
    const bool cin = cur.c0 + lane < cur.c1;
    u64 cw0 = cin ? cur.w0 : 0ULL, cw1 = cin && WS > 1 ? cur.w1 : 0ULL;
    uint32_t ckey = cin ? cur.key : 0u;
    const uint32_t c0 = cur.c0, c1 = cur.c1;
    // this round's words are in before the next round's loads go out
#pragma unroll
    for (int i = 0; i < 2; i++) {
      pin_vgpr(ra[i]);
      pin_vgpr(rb[i]);
      pin_vgpr(sd[i]);
    }
    pin_vgpr(cw0);
    pin_vgpr(cw1);
    pin_vgpr(ckey);
    if (r > 1) prefetch2(r - 1, nxt);
    {  // pending weak targets of round r
      const int sl = r % rsl;
      F0 |= ring[(sl * 2) * 64 + lane];
      F1 |= ring[(sl * 2 + 1) * 64 + lane];
      ring[(sl * 2) * 64 + lane] = 0;
      ring[(sl * 2 + 1) * 64 + lane] = 0;
    }
    if (!alive) G0 = G1 = 0;
    if (haveK && r == T && lane == 63) {  // K: every present vertex of the top round
      F0 |= pres_word(T, 0);
      F1 |= pres_word(T, 1);
      G0 = F0;
      G1 = F1;
    }
    if (((r - 1) & 3) == 0) {  // leader round of wave w: seed its lane with the leader's vertex
      const int w = (r - 1) / 4 + 1;
      const int l = lead_of(w) - 1;
      if ((lead_mask >> (w - 1)) & 1ULL) {
        const u64 bit = 1ULL << (l & 63);
        if (lane == w - 1) {
          if (l < 64) F0 |= bit; else F1 |= bit;
          if (alive) { if (l < 64) G0 |= bit; else G1 |= bit; }
        }
        // the leaders whose strong cone holds this leader's vertex (the chains' test)
        const u64 ql = __ballot(lane < nw && ((((l < 64) ? G0 : G1) >> (l & 63)) & 1ULL));
        if (lane == 0) QL[w - 1] = ql;
      } else if (lane == 0) {
        QL[w - 1] = 0;
      }
    }
    // K (lane 63) and the leaders whose sets differ from it ("solo": expanded on their own)
    u64 K0 = 0, K1 = 0, KG0 = 0, KG1 = 0;
    if (haveK) {
      K0 = readlane64(F0, 63);
      K1 = readlane64(F1, 63);
      KG0 = readlane64(G0, 63);
      KG1 = readlane64(G1, 63);
    }
    {  // round r's cone record for the emission: K, the lanes whose set differs from K, their sets
      // (a leader's lane above its own round holds nothing, and a lane past the leaders is
      // empty: the emission knows both, so neither is stored)
      const bool own = (lane < nw && r <= 4 * lane + 1) || (haveK && lane == 63);
      const u64 dm = __ballot(own && (F0 != K0 || F1 != K1));
      crec -= 3u + 2u * (uint32_t)__popcll(dm);
      u64 DR_GLOBAL *rec = g_cone + crec;
      if (lane == 0) {
        rec[0] = K0;
        rec[1] = K1;
        rec[2] = dm;
      }
      if ((dm >> lane) & 1ULL) {
        const uint32_t at = 3u + 2u * (uint32_t)__popcll(dm & ((1ULL << lane) - 1ULL));
        rec[at] = F0;
        rec[at + 1] = F1;
      }
    }
    const bool eqF = haveK && F0 == K0 && F1 == K1, eqG = haveK && G0 == KG0 && G1 == KG1;
    const u64 soloF = __ballot(!eqF && (F0 | F1) != 0ULL), soloG = __ballot(!eqG && (G0 | G1) != 0ULL);
    DR_TT(tick(2);)  // ring, seeds, cone and degree stores, solo ballots
    // weak columns of round r (64 per batch, lane j holding column j; the first
    // batch was prefetched): a column's target joins b's pending round iff its
    // sources meet F_b
    for (uint32_t cb = c0; cb < c1; cb += 64) {
      if (cb != c0) {
        const uint32_t jc = cb + lane;
        ckey = 0;
        cw0 = cw1 = 0;
        if (jc < c1) {
          ckey = g_wc_key[jc];
          cw0 = g_wc_rows[(size_t)jc * WS];
          cw1 = WS > 1 ? g_wc_rows[(size_t)jc * WS + 1] : 0ULL;
        }
      }
      const int delta = (int)(ckey >> 11), ts = (int)(ckey & 2047u);
      const bool live = (cw0 | cw1) != 0ULL && r - delta >= 1;
      const u64 tb = 1ULL << (ts & 63);
      const int tw = ts >> 6, tsl = live ? (r - delta) % rsl : 0;
      if (haveK && live && ((cw0 & K0) | (cw1 & K1)) != 0ULL) atomicOr(&KW[delta * 2 + tw], tb);
      for (u64 m = soloF; m; m &= m - 1) {
        const int b = __builtin_ctzll(m);
        const u64 s0 = readlane64(F0, b), s1 = readlane64(F1, b);
        if (live && ((cw0 & s0) | (cw1 & s1)) != 0ULL) atomicOr(&ring[(tsl * 2 + tw) * 64 + b], tb);
      }
    }
    __syncthreads();
    if (haveK && c0 < c1) {  // K's weak targets to every lane whose set is K's
      for (int d = 1; d < rsl && r - d >= 1; d++) {
        const u64 k0 = KW[d * 2], k1 = KW[d * 2 + 1];
        if ((k0 | k1) && eqF) {
          const int tsl = (r - d) % rsl;
          ring[(tsl * 2) * 64 + lane] |= k0;
          ring[(tsl * 2 + 1) * 64 + lane] |= k1;
        }
      }
      __syncthreads();
      KW[lane] = 0;
    }
    DR_TT(tick(3);)  // weak columns, K's weak targets spread
    // strong edges: round r-1's sets, and the strong degrees summed over G
    u64 N0 = 0, N1 = 0, H0 = 0, H1 = 0;
    if (haveK) {
      u64 a, b;
      uint32_t ds;
      expand(K0, K1, a, b, nullptr);
      if (eqF) { N0 = a; N1 = b; }
      expand(KG0, KG1, a, b, &ds);
      if (eqG) { H0 = a; H1 = b; suf += ds; }
    }
    DR_TT(tick(4);)  // K's two expansions
    for (u64 m = soloF; m; m &= m - 1) {
      const int b = __builtin_ctzll(m);
      u64 x, y;
      expand(readlane64(F0, b), readlane64(F1, b), x, y, nullptr);
      if (lane == b) { N0 = x; N1 = y; }
    }
    for (u64 m = soloG; m; m &= m - 1) {
      const int b = __builtin_ctzll(m);
      u64 x, y;
      uint32_t ds;
      expand(readlane64(G0, b), readlane64(G1, b), x, y, &ds);
      if (lane == b) { H0 = x; H1 = y; suf += ds; }
    }
    if (r >= 2 && ((r - 2) & 3) == 0) g_sufl[((r - 2) / 4 + 1) * 64 + lane] = suf;  // Suf_b(4(x-1)+2)
    F0 = N0;
    F1 = N1;
    G0 = H0;
    G1 = H1;
    __syncthreads();
    DR_TT(tick(5);)  // the leaders' own expansions
  };
  // crec: the cone records, written top down from the end of the job's scratch (round T's
  // highest): round 1's is the lowest, and each round's follows the one below it, so the
  // bottom-up emission reads them in address order.  A record is K (2 words), the mask of
  // the lanes whose set differs from K, and those lanes' sets in lane order: C5's leaders
  // equal K below their top few rounds, so this is ~1/10 of all 64 lanes' sets per round
  // (the dense [round][2][64] image was ~35 % of the kernel's HBM traffic)
  Pf pa, pb;
  prefetch2(T, pa);
  for (int r = T; r >= 1; r -= 2) {
    cone_round(r, pa, pb);
    if (r >= 2) cone_round(r - 1, pb, pa);
  }
  DR_TT(stamp(2); if (tt && lane == 0) for (int k = 0; k < 6; k++) tt[8 + k] = cyc[k];)

  // ---------------- 3. chains and pops (wave-uniform scalar code) ----------------
  for (int i = lane; i < 64 * 65; i += 64) coef[i] = 0;
  if (lane < 64) first_pop[lane] = -1;
  __syncthreads();
  int npush = 0, npop = 0, last = 0;
  for (int w = 1; w <= nw; w++) {
    if (lane == 0) g_push_off[w - 1] = (uint32_t)npush;
    if (!((commit_mask >> (w - 1)) & 1ULL)) continue;
    const int floor_w = chain_persistent ? last : 0;
    // pushed leaders of this commit, push order (every lane writes the same
    // values to lst: the list stays in LDS, not in per-lane scratch)
    int k = 0;
    lst[k++] = (int8_t)w;
    int L = w;
    for (int w2 = w - 1; w2 >= floor_w + 1; w2--) {
      if (((lead_mask >> (w2 - 1)) & 1ULL) && ((QL[w2 - 1] >> (L - 1)) & 1ULL)) {
        lst[k++] = (int8_t)w2;
        L = w2;
      }
    }
    __syncthreads();
    // chain edges: segment i expands leader list[i]'s strong cone over rounds
    // (round(list[i+1]), round(list[i])], the last one down to round(floor+1)
    if (lane == 0) {
      for (int i = 0; i < k; i++) {
        const int hi = lst[i], lo = i + 1 < k ? lst[i + 1] : floor_w + 1;
        coef[(lst[i] - 1) * 65 + hi] += 1;
        coef[(lst[i] - 1) * 65 + lo] -= 1;
        if (npush + i < J.push_cap) g_push_wave[npush + i] = lst[i];
      }
      for (int i = k - 1; i >= 0; i--) {  // pops: reverse push order (stack/stack.go:23-28)
        const int j = npop + (k - 1 - i);
        pop_lead[j] = (uint8_t)lst[i];
        if (first_pop[lst[i] - 1] < 0) first_pop[lst[i] - 1] = (int16_t)j;
      }
    }
    npush += k;
    npop += k;
    last = w;
    __syncthreads();
  }
  if (lane == 0) g_push_off[nw] = (uint32_t)npush;
  __syncthreads();
  DR_TT(stamp(3);)

  // ---------------- 4. bottom-up emission ----------------
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int i = 64 * k + lane, ic = i <= T + 1 ? i : T + 1;
    soffv[k] = g_slot_off[ic];
  }
  // lane b = leader wave b+1 for the per-leader bookkeeping
  const int myfirst = first_pop[lane];
  int myrank = 0;  // PAPER: leaders first popped before b
  for (int x = 0; x < 64; x++) {
    const int fp = first_pop[x];
    myrank += (fp >= 0 && myfirst >= 0 && fp < myfirst) ? 1 : 0;
  }
  if (PAPER && myfirst >= 0) ord[myrank] = (int8_t)lane;
  for (int k = 0; k < RS; k++) res[lane * RS + k] = 0;
  // chain edges: segment sums are differences of the suffix sums at the leader
  // rounds (every leader's coefficients sum to zero; Suf = 0 above round T)
  u64 chain = 0;
  for (int x = 1; x < nw; x++) {
    const int c = coef[lane * 65 + x];
    if (c) chain -= (u64)((int64_t)c * (int64_t)g_sufl[x * 64 + lane]);
  }
  chain = wave_sum(chain);
  const u64 popped = __ballot(myfirst >= 0);
  const int npopped = __popcll(popped);
  __syncthreads();
  u64 neq = kmemo ? 0ULL : ~0ULL;   // leaders whose cone differs from K in some round <= r
  u64 kK = 0, dK = 0, eK = 0;       // K's count, digest, edges through round r-1
  // delivered vertices of round r (the set s0|s1) in slot order, positions from
  // k0: count, digest, edges (wave-uniform); lanes = slots (sa, sb: the round's
  // slots; slo / shi: its first 128 slot sources, lane-held)
  auto contrib = [&](int r, u64 s0, u64 s1, u64 k0, uint32_t sa, uint32_t sb, int slo, int shi, u64 &cnt, u64 &dg,
                     u64 &ed) {
    u64 k = k0, dacc = 0, eacc = 0;
    for (uint32_t c0 = sa; c0 < sb; c0 += 64) {
      const uint32_t sl = c0 + lane;
      const int s = c0 == sa ? slo : c0 == sa + 64 ? shi : (sl < sb ? (int)g_slot_src[sl] : 0);  // 0: ghost / none
      const int v = s - 1;
      const bool in = s > 0 && ((((v < 64) ? s0 : s1) >> (v & 63)) & 1ULL);
      const u64 bal = __ballot(in);
      if (in) {
        dacc += digest_term((uint32_t)r, (uint32_t)s, k + (u64)__popcll(bal & ((1ULL << lane) - 1ULL)));
        eacc += DG[v];
      }
      k += (u64)__popcll(bal);
    }
    cnt = k - k0;
    dg = wave_sum(dacc);
    ed = wave_sum(eacc);
  };
  // software pipeline: round r+1's sets, degrees, presence and slots load while
  // round r is processed
  // the cone records in two stages: round r+1's header (K, mask) was loaded a round ago,
  // its lanes' sets load now, and round r+2's header, whose address follows from r+1's mask
  u64 pf0 = 0, pf1 = 0, pp0 = 0, pp1 = 0;
  u64 pk0 = 0, pk1 = 0, pm = 0;  // the header of the round whose sets pf0 / pf1 hold
  u64 hk0 = 0, hk1 = 0, hm = 0;  // the next round's header
  uint32_t hat = crec;           // the next round's record
  auto load_hdr = [&](uint32_t at) {
    hk0 = g_cone[at];
    hk1 = g_cone[at + 1];
    hm = g_cone[at + 2];
  };
  auto load_sets = [&]() {  // the sets of the round whose header is in hk / hm: unconditional loads
    pk0 = hk0;
    pk1 = hk1;
    pm = hm;
    const bool in = (pm >> lane) & 1ULL;
    const uint32_t at = in ? hat + 3u + 2u * (uint32_t)__popcll(pm & ((1ULL << lane) - 1ULL)) : hat;
    pf0 = g_cone[at];
    pf1 = g_cone[at + 1];
    hat += 3u + 2u * (uint32_t)__popcll(pm);
  };
  uint16_t psd[2] = {0, 0}, pwd[2] = {0, 0};  // (16-bit: no widening right after the loads)
  uint32_t psa = 0, psb = 0;
  int pslo = 0, pshi = 0;
  auto prefetch4 = [&](int r) {
    load_sets();
    if (r < T) load_hdr(hat);
#pragma unroll
    for (int i = 0; i < 2; i++) {
      const int v = lane + 64 * i;
      const size_t at = (size_t)r * n + (v < n ? v : 0);  // (a lane past n: never read)
      psd[i] = g_sdeg[at];
      pwd[i] = g_wdeg[at];
    }
    pp0 = pres_word(r, 0);
    pp1 = pres_word(r, 1);
    psa = tab4(soffv, r);
    psb = tab4(soffv, r + 1);
    pslo = psa + lane < psb ? (int)g_slot_src[psa + lane] : 0;
    pshi = psa + 64 + lane < psb ? (int)g_slot_src[psa + 64 + lane] : 0;
  };
  load_hdr(hat);
  prefetch4(1);
  for (int r = 1; r <= T; r++) {
    __syncthreads();
    const bool own = (pm >> lane) & 1ULL;  // this lane's set differs from K in round r
    const bool held = (lane < nw && r <= 4 * lane + 1) || (haveK && lane == 63);  // else empty
    const u64 f0 = own ? pf0 : held ? pk0 : 0ULL, f1 = own ? pf1 : held ? pk1 : 0ULL, P0 = pp0, P1 = pp1;
    const uint32_t sa = psa, sb = psb;
    const int slo = pslo, shi = pshi;
#pragma unroll
    for (int i = 0; i < 2; i++) {
      const int v = lane + 64 * i;
      if (v < n) DG[v] = (uint32_t)psd[i] + (uint32_t)pwd[i];  // strong + weak degree
    }
    if (r < T) prefetch4(r + 1);
    __syncthreads();
    const u64 active = popped & __ballot(lane < nw && 4 * lane + 1 >= r);  // leaders whose top >= r
    if (!PAPER) {
      if (kmemo) {  // leaders whose cone first differs from K in round r take K's prefix
        const u64 K0 = readlane64(f0, 63), K1 = readlane64(f1, 63);
        const u64 newly = __ballot((((f0 ^ K0) & P0) | ((f1 ^ K1) & P1)) != 0ULL) & active & ~neq;
        if ((newly >> lane) & 1ULL) {
          res[lane * RS + 0] = kK;
          res[lane * RS + 1] = dK;
          res[lane * RS + 2] = eK;
        }
        neq |= newly;
        u64 c, d, e;
        contrib(r, K0, K1, kK, sa, sb, slo, shi, c, d, e);
        kK += c;
        dK += d;
        eK += e;
      }
      __syncthreads();
      for (u64 m = neq & active; m; m &= m - 1) {
        const int b = __builtin_ctzll(m);
        u64 c, d, e;
        contrib(r, readlane64(f0, b), readlane64(f1, b), res[b * RS + 0], sa, sb, slo, shi, c, d, e);
        __syncthreads();
        if (lane == 0) {
          res[b * RS + 0] += c;
          res[b * RS + 1] += d;
          res[b * RS + 2] += e;
        }
        __syncthreads();
      }
      if (kmemo && ((r - 1) & 3) == 0) {  // a leader equal to K up to its own round: K's prefix
        const int b = (r - 1) / 4;
        if (lane == 0 && b < nw && ((popped >> b) & 1ULL) && !((neq >> b) & 1ULL)) {
          res[b * RS + 0] = kK;
          res[b * RS + 1] = dK;
          res[b * RS + 2] = eK;
        }
      }
    } else if (active) {
      // what the leaders popped before b hold: exclusive prefix OR over the popped
      // leaders in first-pop order (lane j = the j-th), read back at b's rank
      const int src = lane < npopped ? (int)ord[lane] : 0;
      u64 y0 = shfl64(f0, src), y1 = shfl64(f1, src);
      if (lane >= npopped) y0 = y1 = 0;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const u64 z0 = shfl_up64(y0, off), z1 = shfl_up64(y1, off);
        if (lane >= off) { y0 |= z0; y1 |= z1; }
      }
      u64 e0 = shfl_up64(y0, 1), e1 = shfl_up64(y1, 1);
      if (lane == 0) e0 = e1 = 0;
      const u64 x0 = f0 & ~shfl64(e0, myrank), x1 = f1 & ~shfl64(e1, myrank);
      for (u64 m = __ballot(((x0 & P0) | (x1 & P1)) != 0ULL) & active; m; m &= m - 1) {
        const int b = __builtin_ctzll(m);
        u64 c, d, e;
        contrib(r, readlane64(x0, b), readlane64(x1, b), res[b * RS + 3], sa, sb, slo, shi, c, d, e);
        __syncthreads();
        if (lane == 0) {
          res[b * RS + 3] += c;
          res[b * RS + 4] += d;
          res[b * RS + 5] += e;
        }
        __syncthreads();
      }
    }
  }
  __syncthreads();
  DR_TT(stamp(4);)

  // ---------------- 5. outputs ----------------
  u64 dsum = 0;
  const int np = min(npop, min(J.push_cap, kMaxPops));
  for (int j = lane; j < np; j += 64) {
    const int lb = pop_lead[j] - 1;
    u64 c, d, e;
    if (!paper) {
      c = res[lb * RS + 0]; d = res[lb * RS + 1]; e = res[lb * RS + 2];
    } else if (first_pop[lb] == j) {
      c = res[lb * RS + (RS - 3)]; d = res[lb * RS + (RS - 2)]; e = res[lb * RS + (RS - 1)];
    } else {
      c = 0; d = 0; e = 0;  // the leader's cone was delivered by its first pop
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
    g_totals[0] = commit_edges;
    g_totals[1] = chain;
    g_totals[2] = dsum;
    g_totals[3] = (u64)npush;
  }
  DR_TT(stamp(5);)
}

}  // namespace dr
