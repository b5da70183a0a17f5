// batch.hpp -- fused replay of many small DAGs: one wavefront per DAG.
//
// thousands of independent replays (one Process mirror
// each, n <= 128, up to 64 waves).  A per-DAG dr_replay would spend its time in
// launches and host round trips; here one kernel replays every DAG of a batch,
// a wavefront per DAG, everything between the DAG in HBM and the per-pop
// results on the device.
//
// Per DAG (T = 4*(nw-1)+1, the highest leader round):
//   1. commits (waveReady's rule, process.go:326-339), wave by wave: S0 =
//      {leader}; S_k = ballot(row(v) & S_{k-1} != 0) over rounds 4w-2..4w.
//   2. one top-down pass over rounds T..1 computing, for every vertex v, the
//      set of leader waves whose cone contains v: Qs (strong edges only, the
//      chains' strong_path) and Qf (strong + weak, orderVertices' path(.., false)).
//      Strong: lane u of round r-1 ORs Q(v) of every v of round r whose row has
//      bit u (rows broadcast by readlane).  Weak: per weak column (one distinct
//      weak target of the round), the wave-OR of Qf over the column's sources
//      goes into a ring of pending rounds (one LDS atomic per column).  Q and
//      degrees go to a per-DAG scratch.
//   3. chains (process.go:341-350) from the leaders' Qs: wave w' is pushed
//      after leader L iff L's bit is in Qs(leader(w')); pops = reverse pushes.
//   4. bottom-up emission.  Vertex v is delivered by leader b (REF) iff b in
//      Qf(v), or (PAPER) iff additionally no leader popped before b's first pop
//      is in Qf(v).  A leader's contribution of a round is computed with lanes =
//      slots: ballot ranks give the positions, the order-sensitive digest
//       and edge sums are wave reductions.  REF memo (nw <= 63):
//      bit 63 of Qf is the canonical cone K (every present vertex of round T);
//      below the first round where b's cone differs from K, b's prefix equals K's,
//      so only K and the leaders that already differ (those a few rounds under
//      their top) are computed per round (the same identity as the
//      engine's memo).  PAPER computes a leader only in rounds where it delivers
//      something.  Chain edges: per-leader sums of strong degrees over Qs, only
//      in the rounds the leader's chain segments cover.
//   Qs bits are kept only in the rounds the chains can inspect (a leader's bit
//   dies below its chain's floor round), and sources with an empty Qs skip the
//   strong-only half of the expansion.
// Supported: n <= 128, nw <= 64, weak deltas < ring depth (<= 32), no far edges.
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
  const uint32_t *slot_off;
  const uint16_t *slot_src;
  const uint16_t *lead;     // [wave] chooseLeader(w), 1-based source
  // scratch, rounds 0..T: Qf, Qs, (deg << 16 | strong deg)
  u64 *qf;
  u64 *qs;
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

// dynamic LDS of k_replay_small: the weak ring (rsl slots of 128 u64) or the
// later phases' arrays, whichever is larger
template <bool PAPER, bool PERSIST>
constexpr int small_late_bytes() {  // coef, pop list, per-leader results, chain sums, paper "before" masks
  return 64 * 65 + (((PERSIST ? 64 : kSmallMaxPops) + 255) & ~255) + 64 * (PAPER ? 6 : 3) * 8 + 64 * 8 +
         (PAPER ? 64 * 8 : 0);
}
template <bool PAPER, bool PERSIST>
inline size_t small_lds_bytes(int rsl) {
  const size_t ring = (size_t)rsl * 128 * 8, late = (size_t)small_late_bytes<PAPER, PERSIST>();
  return ring > late ? ring : late;
}

// rsl = ring slots = largest weak delta + 1 (round x's slot is reused by round
// x + rsl, which is drained before any contribution to x arrives)
template <int DEPTH, bool PAPER, bool PERSIST>
__global__ __launch_bounds__(64) void k_replay_small(const SmallJob *__restrict__ jobs, int njobs, int nw, int rsl) {
  constexpr bool paper = PAPER;  // REF mode skips the paper-mode digests entirely
  constexpr bool chain_persistent = PERSIST;  // persistent chains push every wave at most once: <= 64 pops
  // LDS is what limits DAGs per CU: the weak ring (phase 2 only) shares its
  // bytes with the chain coefficients, pop list and per-leader results (phases
  // 3-5, which start after phase 2's last barrier).
  constexpr int kMaxPops = PERSIST ? 64 : kSmallMaxPops;
  constexpr int RS = PAPER ? 6 : 3;  // per-leader results kept
  constexpr int kCoefB = 64 * 65, kPopB = (kMaxPops + 255) & ~255, kResB = 64 * RS * 8;
  static_assert(kCoefB + kPopB + kResB + 64 * 8 + (PAPER ? 64 * 8 : 0) == small_late_bytes<PAPER, PERSIST>(),
                "LDS layout");
  // REF memo: bit 63 of Qf carries the canonical cone K (needs a free leader bit)
  const bool kmemo = !PAPER && nw <= 63;
  extern __shared__ __attribute__((aligned(16))) u64 arena[];                  // small_lds_bytes(rsl)
  u64 *ring = arena;                                                            // [rsl * 128], phase 2
  int8_t *coef = reinterpret_cast<int8_t *>(arena);                             // [64 * 65], phases 3-4
  uint8_t *pop_lead = reinterpret_cast<uint8_t *>(arena) + kCoefB;              // [kSmallMaxPops], 3-5
  u64 *res = reinterpret_cast<u64 *>(reinterpret_cast<char *>(arena) + ((kCoefB + kPopB + 7) & ~7));  // 4-5
  u64 *CS = res + 64 * RS;   // [64] chain: running strong-degree sums over Qs, phase 4
  u64 *BEF = CS + 64;        // [64] PAPER: leaders first popped before b, phase 4
  __shared__ u64 QF[128];
  __shared__ uint32_t DG[128];
  __shared__ u64 QL[64];
  __shared__ int32_t vc_s[64];
  __shared__ int16_t first_pop[64];
  __shared__ int16_t qs_floor[64];  // lowest round where leader b's strong cone is still inspected
  __shared__ int8_t lst[64];
  const int lane = threadIdx.x;
  const int jb = blockIdx.x;
  if (jb >= njobs) return;
  const SmallJob J = jobs[jb];
  const int n = J.n, WS = J.WS;
  const int q = J.quorum;
  const int T = 4 * (nw - 1) + 1;
  auto row = [&](int r, int v, u64 &a, u64 &b) {  // row of (r, v+1); zero for v >= n
    a = 0;
    b = 0;
    if (v < n) {
      const u64 *p = J.strong + ((size_t)r * n + v) * WS;
      if (WS == 2) {
        const u64x2 x = *reinterpret_cast<const u64x2 *>(p);
        a = x.x;
        b = x.y;
      } else {
        a = p[0];
      }
    }
  };
  auto pres_word = [&](int r, int w) -> u64 { return w < WS ? J.present[(size_t)r * WS + w] : 0ULL; };

  // ---------------- 1. commits ----------------
  u64 commit_mask = 0, lead_mask = 0, commit_edges = 0;
  for (int w = 1; w <= nw; w++) {
    const int r1 = 4 * (w - 1) + 1;
    const int l = J.lead[w] - 1;  // chooseLeader(w), 0-based (< 128)
    const bool lead = (pres_word(r1, l >> 6) >> (l & 63)) & 1ULL;
    if (!lead) {
      if (lane == 0) vc_s[w - 1] = -1;
      continue;
    }
    lead_mask |= 1ULL << (w - 1);
    u64 a[3][2], b[3][2];
#pragma unroll
    for (int k = 0; k < 3; k++) {
      row(r1 + 1 + k, lane, a[k][0], b[k][0]);
      row(r1 + 1 + k, lane + 64, a[k][1], b[k][1]);
    }
    u64 s0 = l < 64 ? 1ULL << l : 0ULL, s1 = l >= 64 ? 1ULL << (l - 64) : 0ULL, deg = 0;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const int r = r1 + 1 + k;
      const u64 p0 = pres_word(r, 0), p1 = pres_word(r, 1);
      const bool h0 = ((p0 >> lane) & 1ULL) && (((a[k][0] & s0) | (b[k][0] & s1)) != 0ULL);
      const bool h1 = ((p1 >> lane) & 1ULL) && (((a[k][1] & s0) | (b[k][1] & s1)) != 0ULL);
      s0 = __ballot(h0);
      s1 = __ballot(h1);
      deg += (u64)(__popcll(a[k][0]) + __popcll(b[k][0]) + __popcll(a[k][1]) + __popcll(b[k][1]));
    }
    commit_edges += wave_sum(deg);
    const int vc = __popcll(s0) + __popcll(s1);
    if (lane == 0) vc_s[w - 1] = vc;
    if (vc >= q) commit_mask |= 1ULL << (w - 1);
  }

  // ---------------- 2. top-down Q pass ----------------
  for (int i = lane; i < rsl * 128; i += 64) ring[i] = 0;
  // chains (process.go:341-350) inspect leader b's strong cone only down to the
  // floor round of the commit whose chain can push b: 4*decidedWave + 1
  qs_floor[lane] = 0x7fff;
  __syncthreads();
  if (lane == 0) {
    int lastc = 0;
    for (int w = 1; w <= nw; w++)
      if ((commit_mask >> (w - 1)) & 1ULL) {
        for (int b = lastc + 1; b <= w; b++) qs_floor[b - 1] = (int16_t)(chain_persistent ? 4 * lastc + 1 : 1);
        lastc = w;
      }
  }
  __syncthreads();
  const int my_floor = qs_floor[lane];
  u64 qf[2] = {0, 0}, qs[2] = {0, 0};
  // software pipeline: round r-1's rows and first 64 weak columns (they do not
  // depend on the frontier) load while round r is processed
  u64 nra[2], nrb[2], nw0 = 0, nw1 = 0;
  uint32_t nkey = 0, nc0 = 0, nc1 = 0;
  auto prefetch2 = [&](int r) {
    row(r, lane, nra[0], nrb[0]);
    row(r, lane + 64, nra[1], nrb[1]);
    nc0 = J.wc_roff[r];
    nc1 = J.wc_roff[r + 1];
    const uint32_t jc = nc0 + lane;
    nkey = 0;
    nw0 = nw1 = 0;
    if (jc < nc1) {
      nkey = J.wc_key[jc];
      nw0 = J.wc_rows[(size_t)jc * WS];
      nw1 = WS > 1 ? J.wc_rows[(size_t)jc * WS + 1] : 0ULL;
    }
  };
  prefetch2(T);
  for (int r = T; r >= 1; r--) {
    const u64 alive = __ballot(lane < nw && my_floor <= r);
    u64 ra[2] = {nra[0], nra[1]}, rb[2] = {nrb[0], nrb[1]};
    u64 cw0 = nw0, cw1 = nw1;
    uint32_t ckey = nkey;
    const uint32_t c0 = nc0, c1 = nc1;
    if (r > 1) prefetch2(r - 1);
#pragma unroll
    for (int i = 0; i < 2; i++) {
      const int v = lane + 64 * i;
      qf[i] |= ring[(r % rsl) * 128 + v];
      ring[(r % rsl) * 128 + v] = 0;
      qs[i] &= alive;
    }
    if (kmemo && r == T) {  // K: every present vertex of the top round
      if ((pres_word(T, 0) >> lane) & 1ULL) qf[0] |= 1ULL << 63;
      if ((pres_word(T, 1) >> lane) & 1ULL) qf[1] |= 1ULL << 63;
    }
    if (((r - 1) & 3) == 0) {  // leader round of wave w: seed its bit at the leader's source
      const int w = (r - 1) / 4 + 1;
      const int l = J.lead[w] - 1;
      if ((lead_mask >> (w - 1)) & 1ULL) {
        if (lane == (l & 63)) {  // register arrays: constant indices only
          const u64 sb = (alive >> (w - 1)) & 1ULL;
          if (l < 64) {
            qf[0] |= 1ULL << (w - 1);
            qs[0] |= sb << (w - 1);
            QL[w - 1] = qs[0];
          } else {
            qf[1] |= 1ULL << (w - 1);
            qs[1] |= sb << (w - 1);
            QL[w - 1] = qs[1];
          }
        }
      } else if (lane == 0) {
        QL[w - 1] = 0;
      }
    }
    // weak columns of round r (64 per batch, lane j holding column j; the first
    // batch was prefetched): Qf of the column's sources into the pending round
    for (uint32_t cb = c0; cb < c1; cb += 64) {
      if (cb != c0) {
        const uint32_t jc = cb + lane;
        ckey = 0;
        cw0 = cw1 = 0;
        if (jc < c1) {
          ckey = J.wc_key[jc];
          cw0 = J.wc_rows[(size_t)jc * WS];
          cw1 = WS > 1 ? J.wc_rows[(size_t)jc * WS + 1] : 0ULL;
        }
      }
      const int m = (int)min(64u, c1 - cb);
      for (int t = 0; t < m; t++) {  // wave-uniform
        const u64 w0 = readlane64(cw0, t), w1 = readlane64(cw1, t);
        const uint32_t key = (uint32_t)__builtin_amdgcn_readlane((int)ckey, t);
        u64 v = ((w0 >> lane) & 1ULL) ? qf[0] : 0ULL;
        v |= ((w1 >> lane) & 1ULL) ? qf[1] : 0ULL;
        v = wave_or(v);
        const int delta = (int)(key >> 11), ts = (int)(key & 2047u);
        if (lane == 0 && v && r - delta >= 1) atomicOr(&ring[((r - delta) % rsl) * 128 + ts], v);
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 2; i++) {
      const int v = lane + 64 * i;
      if (v < n) {
        const uint32_t sd = (uint32_t)(__popcll(ra[i]) + __popcll(rb[i]));
        const size_t at = (size_t)r * n + v;
        J.qf[at] = qf[i];
        J.qs[at] = qs[i];
        J.deg[at] = ((sd + J.wdeg[at]) << 16) | sd;
      }
    }
    // strong edges: Q of round r-1, lane u owns targets u and u+64
    // (Qs is a subset of Qf per vertex: the strong-only half runs only for the
    // sources with a live Qs)
    u64 nf0 = 0, nf1 = 0, ns0 = 0, ns1 = 0;
#pragma unroll
    for (int i = 0; i < 2; i++) {
      u64 m = __ballot(qf[i] != 0ULL);
      while (m) {
        const int l = __builtin_ctzll(m);
        m &= m - 1;
        const u64 a = readlane64(ra[i], l), b = readlane64(rb[i], l), f = readlane64(qf[i], l);
        nf0 |= ((a >> lane) & 1ULL) ? f : 0ULL;
        nf1 |= ((b >> lane) & 1ULL) ? f : 0ULL;
      }
      u64 ms = __ballot(qs[i] != 0ULL);
      while (ms) {
        const int l = __builtin_ctzll(ms);
        ms &= ms - 1;
        const u64 a = readlane64(ra[i], l), b = readlane64(rb[i], l), sq = readlane64(qs[i], l);
        ns0 |= ((a >> lane) & 1ULL) ? sq : 0ULL;
        ns1 |= ((b >> lane) & 1ULL) ? sq : 0ULL;
      }
    }
    qf[0] = nf0;
    qf[1] = nf1;
    qs[0] = ns0;
    qs[1] = ns1;
    __syncthreads();
  }

  // ---------------- 3. chains and pops (wave-uniform scalar code) ----------------
  for (int i = lane; i < 64 * 65; i += 64) coef[i] = 0;
  if (lane < 64) first_pop[lane] = -1;
  __syncthreads();
  int npush = 0, npop = 0, last = 0;
  for (int w = 1; w <= nw; w++) {
    if (lane == 0) J.push_off[w - 1] = (uint32_t)npush;
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
        if (npush + i < J.push_cap) J.push_wave[npush + i] = lst[i];
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
  if (lane == 0) J.push_off[nw] = (uint32_t)npush;
  __syncthreads();

  // ---------------- 4. bottom-up emission ----------------
  // lane b = leader wave b+1 for the per-leader bookkeeping
  const int myfirst = first_pop[lane];
  {
    u64 bef = 0;  // leaders first popped before b (PAPER: they own shared vertices)
    for (int x = 0; x < 64; x++) {
      const int fp = first_pop[x];
      if (fp >= 0 && myfirst >= 0 && fp < myfirst) bef |= 1ULL << x;
    }
    if (PAPER) BEF[lane] = bef;
    CS[lane] = 0;
    for (int k = 0; k < RS; k++) res[lane * RS + k] = 0;
  }
  // chain segments of leader b cover rounds (lo_b, hi_b]
  int seg_lo = 0x7fff, seg_hi = -1;
  for (int x = 0; x <= 64; x++)
    if (coef[lane * 65 + x]) {
      seg_lo = min(seg_lo, 4 * (x - 1) + 1);
      seg_hi = max(seg_hi, 4 * (x - 1) + 1);
    }
  const u64 popped = __ballot(myfirst >= 0);
  u64 neq = kmemo ? 0ULL : ~0ULL;   // leaders whose cone differs from K in some round <= r
  u64 kK = 0, dK = 0, eK = 0;       // K's count, digest, edges through round r-1
  u64 chain = 0;
  // one leader's (or K's, b = 63) delivered vertices of round r in slot order,
  // positions from k0: count, digest, edges (wave-uniform); lanes = slots
  // (sa, sb: the round's slots; slo / shi: its first 128 slot sources, lane-held)
  auto contrib = [&](int r, int b, u64 k0, u64 befb, uint32_t sa, uint32_t sb, int slo, int shi, u64 &cnt, u64 &dg,
                     u64 &ed) {
    u64 k = k0, dacc = 0, eacc = 0;
    for (uint32_t c0 = sa; c0 < sb; c0 += 64) {
      const uint32_t sl = c0 + lane;
      const int s = c0 == sa ? slo : c0 == sa + 64 ? shi : (sl < sb ? (int)J.slot_src[sl] : 0);  // 0: ghost / none
      const u64 f = s > 0 ? QF[s - 1] : 0ULL;
      const bool in = ((f >> b) & 1ULL) && !(f & befb);
      const u64 bal = __ballot(in);
      if (in) {
        dacc += digest_term((uint32_t)r, (uint32_t)s, k + (u64)__popcll(bal & ((1ULL << lane) - 1ULL)));
        eacc += DG[s - 1] >> 16;
      }
      k += (u64)__popcll(bal);
    }
    cnt = k - k0;
    dg = wave_sum(dacc);
    ed = wave_sum(eacc);
  };
  // software pipeline: round r+1's Q, degrees, presence and slots load while
  // round r is processed
  u64 pf[2] = {0, 0}, ps[2] = {0, 0}, pp[2] = {0, 0};
  uint32_t pd[2] = {0, 0}, psa = 0, psb = 0;
  int pslo = 0, pshi = 0;
  auto prefetch4 = [&](int r) {
#pragma unroll
    for (int i = 0; i < 2; i++) {
      const int v = lane + 64 * i;
      if (v < n) {
        const size_t at = (size_t)r * n + v;
        pf[i] = J.qf[at];
        ps[i] = J.qs[at];
        pd[i] = J.deg[at];
      }
      pp[i] = pres_word(r, i);
    }
    psa = J.slot_off[r];
    psb = J.slot_off[r + 1];
    pslo = psa + lane < psb ? (int)J.slot_src[psa + lane] : 0;
    pshi = psa + 64 + lane < psb ? (int)J.slot_src[psa + 64 + lane] : 0;
  };
  prefetch4(1);
  for (int r = 1; r <= T; r++) {
    __syncthreads();
    const u64 f2[2] = {pf[0], pf[1]}, s2[2] = {ps[0], ps[1]}, p2[2] = {pp[0], pp[1]};
    const uint32_t d2[2] = {pd[0], pd[1]}, sa = psa, sb = psb;
    const int slo = pslo, shi = pshi;
#pragma unroll
    for (int i = 0; i < 2; i++) {
      const int v = lane + 64 * i;
      if (v < n) {
        QF[v] = f2[i];
        DG[v] = d2[i];
      }
    }
    if (r < T) prefetch4(r + 1);
    __syncthreads();
    const u64 active = popped & ~0ULL & __ballot(lane < nw && 4 * lane + 1 >= r);  // leaders whose top >= r
    if (!PAPER) {
      if (kmemo) {  // leaders whose cone first differs from K in round r take K's prefix
        u64 x = 0;
#pragma unroll
        for (int i = 0; i < 2; i++)
          if ((p2[i] >> lane) & 1ULL) x |= f2[i] ^ (((f2[i] >> 63) & 1ULL) ? ~0ULL : 0ULL);
        const u64 newly = wave_or(x) & active & ~neq;
        if ((newly >> lane) & 1ULL) {
          res[lane * RS + 0] = kK;
          res[lane * RS + 1] = dK;
          res[lane * RS + 2] = eK;
        }
        neq |= newly;
        u64 c, d, e;
        contrib(r, 63, kK, 0ULL, sa, sb, slo, shi, c, d, e);
        kK += c;
        dK += d;
        eK += e;
      }
      __syncthreads();
      for (u64 m = neq & active; m; m &= m - 1) {
        const int b = __builtin_ctzll(m);
        u64 c, d, e;
        contrib(r, b, res[b * RS + 0], 0ULL, sa, sb, slo, shi, c, d, e);
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
    } else {
      for (u64 m = active; m; m &= m - 1) {
        const int b = __builtin_ctzll(m);
        const u64 befb = BEF[b];
        bool any = false;
#pragma unroll
        for (int i = 0; i < 2; i++)
          any |= ((p2[i] >> lane) & 1ULL) && ((f2[i] >> b) & 1ULL) && !(f2[i] & befb);
        if (__ballot(any) == 0ULL) continue;
        u64 c, d, e;
        contrib(r, b, res[b * RS + 3], befb, sa, sb, slo, shi, c, d, e);
        __syncthreads();
        if (lane == 0) {
          res[b * RS + 3] += c;
          res[b * RS + 4] += d;
          res[b * RS + 5] += e;
        }
        __syncthreads();
      }
    }
    // chain edges: strong-degree sums over Qs in the leaders' segment rounds
    for (u64 m = __ballot(lane < nw && seg_lo < r && r <= seg_hi); m; m &= m - 1) {
      const int b = __builtin_ctzll(m);
      u64 x = 0;
#pragma unroll
      for (int i = 0; i < 2; i++)
        if ((s2[i] >> b) & 1ULL) x += d2[i] & 0xFFFFu;
      x = wave_sum(x);
      if (lane == 0) CS[b] += x;
    }
    __syncthreads();
    if (((r - 1) & 3) == 0) {
      const int x = (r - 1) / 4 + 1;
      const int c = coef[lane * 65 + x];
      if (c) chain += (u64)(int64_t)c * CS[lane];
    }
  }
  chain = wave_sum(chain);
  __syncthreads();

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
    J.pop_count[j] = c;
    J.pop_digest[j] = d;
    J.pop_edges[j] = e;
    dsum += e;
  }
  dsum = wave_sum(dsum);
  if (lane < nw) {
    J.vcount[lane] = vc_s[lane];
    J.commit[lane] = (uint8_t)((commit_mask >> lane) & 1ULL);
  }
  if (lane == 0) {
    J.totals[0] = commit_edges;
    J.totals[1] = chain;
    J.totals[2] = dsum;
    J.totals[3] = (u64)npush;
  }
}

}  // namespace dr
