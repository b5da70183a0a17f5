/*
 * ref_bitset.c -- packed-bitset CPU restatement of the same hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Same outputs as ref_literal.c on
 * contract DAGs (strong edges target round r-1, weak edges rounds < r-1),
 * computed by round sweeps.  An id may repeat in a round (process.go:158-169,
 * :229): the packed row is its last slot's (path()'s lookup, :112-116), vCount
 * and REF delivery count every slot (:332, :418-429), PAPER delivers an id at
 * its first slot, edge totals count an id's edges once.
 *   path(from,to)   process.go:89-148  -> forward sweep from `from`, bit test
 *   waveReady       process.go:314-354 -> backward strong sweep from the
 *                   leader over rounds 4w-2..4w; chain = one forward strong
 *                   sweep that restarts at every pushed leader
 *   orderVertices   process.go:404-443 -> forward strong+weak cone sweep per
 *                   pop, then (round asc, slot asc) emission
 * OpenMP parallelises over independent waves / chains / pops.
 * Edges outside the round contract that target a lower
 * round ride in weak_tgt: a weak edge to r-1, and with bit 31 set a strong edge
 * to a round < r-1 (oracle.h).  Edges to the same or a later round are the
 * literal restatement's alone.
 */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static inline const uint64_t *row_of(const or_pdag *p, int r, int s0) {
  return p->strong + ((size_t)r * p->n + s0) * p->W;
}
static inline int present(const or_pdag *p, int r, int src) {
  for (uint32_t i = p->slot_off[r]; i < p->slot_off[r + 1]; i++)
    if (p->slot_src[i] == src) return 1;
  return 0;
}
static inline int popc(uint64_t x) { return __builtin_popcountll(x); }
/* weak_tgt entry: target round, and bit 31 = a strong edge outside the row (App. A Q8) */
static inline int tgt_round(uint32_t t) { return (int)((t >> 11) & 0xFFFFFu); }
static inline int tgt_strong(uint32_t t) { return (int)(t >> 31); }
static int has_strong_extras(const or_pdag *p) {
  const uint32_t ne = p->weak_off[(size_t)p->nrounds * p->n];
  for (uint32_t e = p->weak_off[0]; e < ne; e++)
    if (tgt_strong(p->weak_tgt[e])) return 1;
  return 0;
}

/* Forward sweep from (top, src0) down to `bottom`.  masks: (top-bottom+1)*W
 * words, round r at (r-bottom)*W, caller-zeroed, bit src0 seeded by caller.
 * Rows of rounds > bottom are expanded; `prune` (paper mode) holds the
 * delivered set per round (same indexing, NULL = none): pruned bits are
 * removed from the frontier before expansion.  Returns edges traversed. */
static uint64_t sweep(const or_pdag *p, int top, int bottom, int strong_only, uint64_t *masks,
                      const uint64_t *prune_base) {
  const int W = p->W, n = p->n;
  uint64_t edges = 0;
  for (int r = top; r > bottom; r--) {
    uint64_t *F = masks + (size_t)(r - bottom) * W;
    if (prune_base) {
      const uint64_t *D = prune_base + (size_t)r * W;
      for (int w = 0; w < W; w++) F[w] &= ~D[w];
    }
    uint64_t *N = F - W;
    for (int w = 0; w < W; w++) {
      uint64_t x = F[w];
      while (x) {
        int b = __builtin_ctzll(x);
        x &= x - 1;
        int s0 = w * 64 + b;
        if (s0 >= n) continue;
        const uint64_t *row = row_of(p, r, s0);
        for (int k = 0; k < W; k++) { N[k] |= row[k]; edges += (uint64_t)popc(row[k]); }
        size_t g = (size_t)r * n + s0;
        for (uint32_t e = p->weak_off[g]; e < p->weak_off[g + 1]; e++) {
          uint32_t t = p->weak_tgt[e];
          if (strong_only && !tgt_strong(t)) continue;
          int tr = tgt_round(t), ts = (int)(t & 2047u);
          edges++;
          if (tr < bottom) continue;
          masks[(size_t)(tr - bottom) * W + (ts >> 6)] |= 1ULL << (ts & 63);
        }
      }
    }
  }
  if (prune_base && top >= bottom) {
    uint64_t *F = masks;
    const uint64_t *D = prune_base + (size_t)bottom * W;
    for (int w = 0; w < W; w++) F[w] &= ~D[w];
  }
  return edges;
}

int or_bs_cone(const or_pdag *p, or_vid from, int bottom, int strong_only, uint64_t *masks,
               uint64_t *edges) {
  if (from.round < 0 || from.round >= p->nrounds || bottom < 0 || bottom > from.round) return OR_PANIC;
  size_t nw = (size_t)(from.round - bottom + 1) * p->W;
  memset(masks, 0, nw * sizeof(uint64_t));
  uint64_t e = 0;
  if (from.source >= 1 && from.source <= p->n) {
    masks[(size_t)(from.round - bottom) * p->W + ((from.source - 1) >> 6)] |= 1ULL << ((from.source - 1) & 63);
    e = sweep(p, from.round, bottom, strong_only, masks, NULL);
  }
  if (edges) *edges = e;
  return 0;
}

/* process.go:89-148 path() by bitset reachability */
int or_bs_path(const or_pdag *p, or_vid from, or_vid to, int strong_path) {
  if (from.round == to.round && from.source == to.source) return 1;
  if (from.round < 0 || from.round >= p->nrounds) return OR_PANIC;
  if (to.round < 0 || to.round >= from.round || to.source < 1 || to.source > p->n) return 0;
  uint64_t *m = (uint64_t *)calloc((size_t)(from.round - to.round + 1) * p->W, sizeof(uint64_t));
  or_bs_cone(p, from, to.round, strong_path, m, NULL);
  int hit = (int)((m[(to.source - 1) >> 6] >> ((to.source - 1) & 63)) & 1);
  free(m);
  return hit;
}

/* waveReady commit decision for one wave: backward strong sweep from the
 * leader (source 1 of round 4w-3).  vcount = #slots of round 4w with a strong
 * path to the leader (process.go:331-336).  -1 when the leader is absent. */
static int commit_one(const or_pdag *p, int faulty, int w, uint8_t *commit, int32_t *vcount,
                      uint64_t *edges) {
  const int W = p->W, n = p->n;
  int r1 = 4 * (w - 1) + 1;
  if (w < 1 || r1 + 3 >= p->nrounds) return OR_PANIC;
  *edges = 0;
  const int L = or_leader(p->leader, p->nleader, w) - 1; /* chooseLeader(w), 0-based */
  if (!present(p, r1, L + 1)) { *commit = 0; *vcount = -1; return 0; }
  /* S[k]: the ids of round r1+k with a strong path to the leader (W <= 32) */
  uint64_t S[4][64];
  memset(S, 0, sizeof S);
  S[0][L >> 6] = 1ULL << (L & 63);
  uint64_t seen[64];
  for (int r = r1 + 1; r <= r1 + 3; r++) {
    uint64_t *T = S[r - r1];
    memset(seen, 0, sizeof seen);
    for (uint32_t i = p->slot_off[r]; i < p->slot_off[r + 1]; i++) {
      int src = p->slot_src[i];
      if (src == 0) continue;
      const uint64_t bit = 1ULL << ((src - 1) & 63);
      if (seen[(src - 1) >> 6] & bit) continue; /* a repeated id: one row, its edges once */
      seen[(src - 1) >> 6] |= bit;
      const uint64_t *row = row_of(p, r, src - 1);
      int hit = 0;
      for (int k = 0; k < W; k++) { hit |= (row[k] & S[r - r1 - 1][k]) != 0; *edges += (uint64_t)popc(row[k]); }
      const size_t g = (size_t)r * n + (src - 1);
      for (uint32_t e = p->weak_off[g]; e < p->weak_off[g + 1]; e++) { /* strong edges skipping rounds */
        const uint32_t t = p->weak_tgt[e];
        if (!tgt_strong(t)) continue;
        const int tr = tgt_round(t), ts = (int)(t & 2047u);
        (*edges)++;
        if (tr >= r1 && tr < r - 1) hit |= (int)((S[tr - r1][ts >> 6] >> (ts & 63)) & 1);
      }
      if (hit) T[(src - 1) >> 6] |= bit;
    }
  }
  const uint64_t *Sv = S[3];
  int vc = 0; /* every slot of round 4w whose id reaches the leader (process.go:331-336) */
  for (uint32_t i = p->slot_off[r1 + 3]; i < p->slot_off[r1 + 4]; i++) {
    int src = p->slot_src[i];
    if (src != 0 && ((Sv[(src - 1) >> 6] >> ((src - 1) & 63)) & 1)) vc++;
  }
  *vcount = vc;
  *commit = vc >= 2 * faulty + 1;
  return 0;
}

int or_bs_commit_sweep(const or_pdag *p, int faulty, int w0, int w1, uint8_t *commit,
                       int32_t *vcount, uint64_t *edges) {
  int bad = 0;
  uint64_t tot = 0;
#pragma omp parallel for schedule(dynamic, 4) reduction(+ : tot) reduction(| : bad)
  for (int w = w0; w <= w1; w++) {
    uint64_t e = 0;
    if (commit_one(p, faulty, w, &commit[w - w0], &vcount[w - w0], &e) < 0) bad = 1;
    tot += e;
  }
  if (edges) *edges = tot;
  return bad ? OR_PANIC : 0;
}

/* Leader chain of a commit at wave w (process.go:341-350): one forward strong
 * sweep from round 4w-3 down to round(floor+1, 1), restarting the frontier at
 * every leader it reaches.  Writes pushed waves (push order) to out. */
/* The same with strong edges that skip rounds (extras): the frontier of every round
 * below the current one is pending in M (rounds bottom..top); a restart drops it. */
static int chain_one_x(const or_pdag *p, int w, int floor_w, int32_t *out, uint64_t *edges) {
  const int W = p->W, n = p->n;
  int top = 4 * (w - 1) + 1, bottom = 4 * floor_w + 1;
  int np = 0;
  out[np++] = w;
  uint64_t *M = (uint64_t *)calloc((size_t)(top - bottom + 1) * W, sizeof(uint64_t));
  const int L0 = or_leader(p->leader, p->nleader, w) - 1;
  M[(size_t)(top - bottom) * W + (L0 >> 6)] = 1ULL << (L0 & 63);
  uint64_t e = 0;
  for (int r = top;; r--) {
    uint64_t *F = M + (size_t)(r - bottom) * W;
    if (r < top && ((r - 1) & 3) == 0) {
      int w2 = (r - 1) / 4 + 1;
      const int L2 = or_leader(p->leader, p->nleader, w2) - 1;
      if (((F[L2 >> 6] >> (L2 & 63)) & 1) && present(p, r, L2 + 1)) {
        out[np++] = w2;
        memset(M, 0, (size_t)(r - bottom + 1) * W * sizeof(uint64_t));
        F[L2 >> 6] = 1ULL << (L2 & 63);
      }
    }
    if (r <= bottom) break;
    uint64_t *N = F - W;
    for (int k = 0; k < W; k++) {
      uint64_t x = F[k];
      while (x) {
        int b = __builtin_ctzll(x);
        x &= x - 1;
        int s0 = k * 64 + b;
        if (s0 >= n) continue;
        const uint64_t *row = row_of(p, r, s0);
        for (int j = 0; j < W; j++) { N[j] |= row[j]; e += (uint64_t)popc(row[j]); }
        const size_t g = (size_t)r * n + s0;
        for (uint32_t q = p->weak_off[g]; q < p->weak_off[g + 1]; q++) {
          const uint32_t t = p->weak_tgt[q];
          if (!tgt_strong(t)) continue;
          const int tr = tgt_round(t), ts = (int)(t & 2047u);
          e++;
          if (tr >= bottom) M[(size_t)(tr - bottom) * W + (ts >> 6)] |= 1ULL << (ts & 63);
        }
      }
    }
  }
  free(M);
  *edges = e;
  return np;
}

static int chain_one(const or_pdag *p, int w, int floor_w, int32_t *out, uint64_t *edges) {
  const int W = p->W, n = p->n;
  int top = 4 * (w - 1) + 1, bottom = 4 * floor_w + 1;
  int np = 0;
  out[np++] = w;
  uint64_t F[64], N[64];
  memset(F, 0, sizeof F);
  const int L0 = or_leader(p->leader, p->nleader, w) - 1;
  F[L0 >> 6] = 1ULL << (L0 & 63);
  uint64_t e = 0;
  for (int r = top;; r--) {
    if (r < top && ((r - 1) & 3) == 0) {
      int w2 = (r - 1) / 4 + 1;
      const int L2 = or_leader(p->leader, p->nleader, w2) - 1;
      if (((F[L2 >> 6] >> (L2 & 63)) & 1) && present(p, r, L2 + 1)) {
        out[np++] = w2;
        memset(F, 0, sizeof F);
        F[L2 >> 6] = 1ULL << (L2 & 63);
      }
    }
    if (r <= bottom) break;
    memset(N, 0, sizeof N);
    int any = 0;
    for (int k = 0; k < W; k++) {
      uint64_t x = F[k];
      while (x) {
        int b = __builtin_ctzll(x);
        x &= x - 1;
        int s0 = k * 64 + b;
        if (s0 >= n) continue;
        const uint64_t *row = row_of(p, r, s0);
        for (int j = 0; j < W; j++) { N[j] |= row[j]; e += (uint64_t)popc(row[j]); }
      }
    }
    for (int k = 0; k < W; k++) { F[k] = N[k]; any |= N[k] != 0; }
    if (!any) break;
  }
  *edges = e;
  return np;
}

typedef struct { int leader_wave, cur_round, pop_index; } pop_t;

/* first_only (PAPER): a repeated id is delivered at its first slot only; REF
 * delivers every slot of a reached id */
static void emit_pop(const or_pdag *p, const uint64_t *masks, int bottom, int top, int cur_round,
                     uint64_t *count, uint64_t *digest, or_vid *ids, int64_t ids_cap, int64_t *ids_n,
                     int first_only) {
  const int W = p->W;
  uint64_t k = 0, dg = 0;
  uint64_t seen[64];
  int last = cur_round < top ? cur_round : top;
  for (int r = 1; r <= last; r++) {
    if (r < bottom) continue;
    const uint64_t *F = masks + (size_t)(r - bottom) * W;
    if (first_only) memset(seen, 0, sizeof seen);
    for (uint32_t i = p->slot_off[r]; i < p->slot_off[r + 1]; i++) {
      int s = p->slot_src[i];
      if (s == 0) continue; /* ghost {0,0}: never reachable (no edge targets source 0) */
      if (!((F[(s - 1) >> 6] >> ((s - 1) & 63)) & 1)) continue;
      if (first_only) {
        const uint64_t bit = 1ULL << ((s - 1) & 63);
        if (seen[(s - 1) >> 6] & bit) continue;
        seen[(s - 1) >> 6] |= bit;
      }
      dg += or_digest_term(r, s, k);
      if (ids) {
        if (*ids_n < ids_cap) { ids[*ids_n].round = r; ids[*ids_n].source = s; }
        (*ids_n)++;
      }
      k++;
    }
  }
  *count = k;
  *digest = dg;
}

int or_bs_replay(const or_pdag *p, int faulty, int nwaves, int chain_mode, int deliver_mode,
                 int nthreads, or_replay_out *o) {
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#else
  (void)nthreads;
#endif
  const int W = p->W;
  o->n_ids = 0;
  o->commit_edges = o->chain_edges = o->deliver_edges = 0;
  int rc = or_bs_commit_sweep(p, faulty, 1, nwaves, o->commit, o->vcount, &o->commit_edges);
  if (rc) return rc;
  /* chains: independent given the commit bits */
  int *cw = (int *)malloc((size_t)(nwaves + 1) * sizeof(int));
  int *cfloor = (int *)malloc((size_t)(nwaves + 1) * sizeof(int));
  int nc = 0, last = 0;
  for (int w = 1; w <= nwaves; w++)
    if (o->commit[w - 1]) {
      cw[nc] = w;
      cfloor[nc] = chain_mode == OR_CHAIN_PERSISTENT ? last : 0;
      nc++;
      last = w;
    }
  int32_t *pushbuf = (int32_t *)malloc((size_t)nc * (nwaves + 1) * sizeof(int32_t) + 4);
  int *npush = (int *)calloc((size_t)nc + 1, sizeof(int));
  uint64_t chain_e = 0;
  const int sx = has_strong_extras(p);
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : chain_e)
  for (int c = 0; c < nc; c++) {
    uint64_t e = 0;
    npush[c] = (sx ? chain_one_x : chain_one)(p, cw[c], cfloor[c], pushbuf + (size_t)c * (nwaves + 1), &e);
    chain_e += e;
  }
  o->chain_edges = chain_e;
  /* push lists + pop schedule */
  int64_t tot = 0;
  for (int c = 0; c < nc; c++) tot += npush[c];
  if (tot > o->push_cap) { free(cw); free(cfloor); free(pushbuf); free(npush); return OR_PANIC; }
  pop_t *pops = (pop_t *)malloc((size_t)(tot + 1) * sizeof(pop_t));
  int64_t np = 0, npop = 0;
  for (int w = 1, c = 0; w <= nwaves; w++) {
    o->push_off[w - 1] = (uint32_t)np;
    if (c < nc && cw[c] == w) {
      const int32_t *pb = pushbuf + (size_t)c * (nwaves + 1);
      for (int i = 0; i < npush[c]; i++) o->push_wave[np++] = pb[i];
      for (int i = npush[c] - 1; i >= 0; i--) {
        pops[npop].leader_wave = pb[i];
        pops[npop].cur_round = 4 * w;
        pops[npop].pop_index = (int)npop;
        npop++;
      }
      c++;
    }
  }
  o->push_off[nwaves] = (uint32_t)np;
  o->n_push = np;
  uint64_t del_e = 0;
  if (deliver_mode == OR_DELIVER_REF && !o->ids) {
    /* a pop's outputs depend only on its leader (the emission window 1..min(cur,
     * top) is 1..top in a replay): one cone per distinct leader wave, which keeps
     * the literal-chain replay (O(w^2) pops) tractable */
    uint64_t *wc = (uint64_t *)calloc((size_t)nwaves + 1, sizeof(uint64_t));
    uint64_t *wd = (uint64_t *)calloc((size_t)nwaves + 1, sizeof(uint64_t));
    uint64_t *we = (uint64_t *)calloc((size_t)nwaves + 1, sizeof(uint64_t));
    uint8_t *need = (uint8_t *)calloc((size_t)nwaves + 1, 1);
    for (int64_t j = 0; j < npop; j++) need[pops[j].leader_wave] = 1;
#pragma omp parallel for schedule(dynamic, 1)
    for (int lw = 1; lw <= nwaves; lw++) {
      if (!need[lw]) continue;
      int top = 4 * (lw - 1) + 1;
      uint64_t *m = (uint64_t *)calloc((size_t)(top + 1) * W, sizeof(uint64_t));
      or_vid from = {top, or_leader(p->leader, p->nleader, lw)};
      or_bs_cone(p, from, 0, 0, m, &we[lw]);
      emit_pop(p, m, 0, top, top, &wc[lw], &wd[lw], NULL, 0, NULL, 0);
      free(m);
    }
    for (int64_t j = 0; j < npop; j++) {
      const int lw = pops[j].leader_wave;
      o->pop_count[j] = wc[lw];
      o->pop_digest[j] = wd[lw];
      o->pop_edges[j] = we[lw];
      del_e += we[lw];
    }
    free(wc);
    free(wd);
    free(we);
    free(need);
  } else {
    /* sequential: needed for the ids list order and for paper-mode dedup */
    uint64_t *D = NULL;
    if (deliver_mode == OR_DELIVER_PAPER) D = (uint64_t *)calloc((size_t)p->nrounds * W, sizeof(uint64_t));
    for (int64_t j = 0; j < npop; j++) {
      int top = 4 * (pops[j].leader_wave - 1) + 1;
      uint64_t *m = (uint64_t *)calloc((size_t)(top + 1) * W, sizeof(uint64_t));
      const int L = or_leader(p->leader, p->nleader, pops[j].leader_wave) - 1;
      m[(size_t)top * W + (L >> 6)] |= 1ULL << (L & 63);
      uint64_t e = sweep(p, top, 0, 0, m, D);
      emit_pop(p, m, 0, top, pops[j].cur_round, &o->pop_count[j], &o->pop_digest[j], o->ids,
               o->ids_cap, &o->n_ids, deliver_mode == OR_DELIVER_PAPER);
      if (D) { /* delivered := delivered U (new cone restricted to present, rounds 1..cur) */
        int lastr = pops[j].cur_round < top ? pops[j].cur_round : top;
        for (int r = 1; r <= lastr; r++)
          for (uint32_t i = p->slot_off[r]; i < p->slot_off[r + 1]; i++) {
            int s = p->slot_src[i];
            if (s == 0) continue;
            uint64_t bit = 1ULL << ((s - 1) & 63);
            if (m[(size_t)r * W + ((s - 1) >> 6)] & bit) D[(size_t)r * W + ((s - 1) >> 6)] |= bit;
          }
        /* edges: only the expanded (new) vertices of rounds >= 1 count, which
         * sweep() already restricted by pruning; round-0 bits expand nothing */
      }
      o->pop_edges[j] = e;
      del_e += e;
      free(m);
    }
    free(D);
  }
  o->deliver_edges = del_e;
  free(pops);
  free(cw);
  free(cfloor);
  free(pushbuf);
  free(npush);
  return 0;
}

/* orderVertices (process.go:404-443) for an arbitrary stack: pops top first,
 * delivering in (round asc, slot asc) order over rounds 1..cur_round.  PAPER
 * skips vertices delivered by an earlier pop of this call. */
int or_bs_order_vertices(const or_pdag *p, const or_vid *stack, int stack_len, int cur_round, int mode,
                         or_vid *out, int64_t out_cap, int64_t *out_n, uint64_t *pop_count,
                         uint64_t *pop_digest) {
  const int W = p->W;
  *out_n = 0;
  if (stack_len == 0) return 0;
  if (cur_round >= p->nrounds) return OR_PANIC;
  uint64_t *D = NULL;
  if (mode == OR_DELIVER_PAPER) D = (uint64_t *)calloc((size_t)p->nrounds * W, sizeof(uint64_t));
  int j = 0;
  for (int t = stack_len - 1; t >= 0; t--, j++) {
    or_vid v = stack[t];
    if (cur_round >= 1 && (v.round < 0 || v.round >= p->nrounds)) { free(D); return OR_PANIC; }
    int top = v.round < 0 ? 0 : (v.round >= p->nrounds ? p->nrounds - 1 : v.round);
    uint64_t *m = (uint64_t *)calloc((size_t)(top + 1) * W, sizeof(uint64_t));
    if (v.source >= 1 && v.source <= p->n)
      m[(size_t)top * W + ((v.source - 1) >> 6)] |= 1ULL << ((v.source - 1) & 63);
    sweep(p, top, 0, 0, m, D);
    emit_pop(p, m, 0, top, cur_round, &pop_count[j], &pop_digest[j], out, out_cap, out_n, mode == OR_DELIVER_PAPER);
    if (D) {
      int lastr = cur_round < top ? cur_round : top;
      for (int r = 1; r <= lastr; r++)
        for (uint32_t i = p->slot_off[r]; i < p->slot_off[r + 1]; i++) {
          int s = p->slot_src[i];
          if (s == 0) continue;
          uint64_t bit = 1ULL << ((s - 1) & 63);
          if (m[(size_t)r * W + ((s - 1) >> 6)] & bit) D[(size_t)r * W + ((s - 1) >> 6)] |= bit;
        }
    }
    free(m);
  }
  free(D);
  return 0;
}
