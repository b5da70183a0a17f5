/*
 * ref_literal.c -- literal CPU restatement of process/process.go's hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Follows the reference algorithm as
 * written, including its cost structure (per-dequeue linear id scan, hash-set
 * visited map, one BFS per orderVertices candidate); debug logging
 * (process.go:109) is omitted.
 */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>

static inline int vid_eq(or_vid a, or_vid b) { return a.round == b.round && a.source == b.source; }
static inline uint64_t vid_key(or_vid a) {
  return ((uint64_t)(uint32_t)a.round << 32) | (uint32_t)a.source;
}

static inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

uint64_t or_digest_term(int32_t round, int32_t source, uint64_t k) {
  uint64_t key = ((uint64_t)(uint32_t)round << 32) | (uint32_t)source;
  return mix64(key ^ mix64(k + 0x9E3779B97F4A7C15ULL));
}

/* ---- the `visited` map: open addressing, generation-stamped clear ---- */
typedef struct {
  uint64_t *keys;
  uint32_t *stamp;
  uint32_t gen;
  size_t cap, used;
} hset;

static void hs_reset(hset *h) {
  h->gen++;
  h->used = 0;
  if (h->gen == 0) { /* wrapped: really clear */
    memset(h->stamp, 0, h->cap * sizeof(uint32_t));
    h->gen = 1;
  }
}
static void hs_init(hset *h, size_t cap) {
  h->cap = cap;
  h->keys = (uint64_t *)malloc(cap * sizeof(uint64_t));
  h->stamp = (uint32_t *)calloc(cap, sizeof(uint32_t));
  h->gen = 1;
  h->used = 0;
}
static void hs_free(hset *h) { free(h->keys); free(h->stamp); memset(h, 0, sizeof *h); }

static int hs_insert(hset *h, uint64_t k);
static void hs_grow(hset *h) {
  hset g;
  hs_init(&g, h->cap * 2);
  for (size_t i = 0; i < h->cap; i++)
    if (h->stamp[i] == h->gen) hs_insert(&g, h->keys[i]);
  hs_free(h);
  *h = g;
}
static inline size_t hs_slot(uint64_t k, size_t cap) { return (size_t)(mix64(k) & (cap - 1)); }
static int hs_has(const hset *h, uint64_t k) {
  size_t i = hs_slot(k, h->cap);
  while (h->stamp[i] == h->gen) {
    if (h->keys[i] == k) return 1;
    i = (i + 1) & (h->cap - 1);
  }
  return 0;
}
static int hs_insert(hset *h, uint64_t k) {
  if ((h->used + 1) * 2 > h->cap) hs_grow(h);
  size_t i = hs_slot(k, h->cap);
  while (h->stamp[i] == h->gen) {
    if (h->keys[i] == k) return 0;
    i = (i + 1) & (h->cap - 1);
  }
  h->stamp[i] = h->gen;
  h->keys[i] = k;
  h->used++;
  return 1;
}

/* per-thread scratch, so OpenMP callers (cpu baseline) can run BFSs in parallel */
static __thread hset tl_visited;
static __thread or_vid *tl_queue;
static __thread size_t tl_qcap;

static void q_reserve(size_t need) {
  if (need <= tl_qcap) return;
  size_t c = tl_qcap ? tl_qcap : 1024;
  while (c < need) c *= 2;
  tl_queue = (or_vid *)realloc(tl_queue, c * sizeof(or_vid));
  tl_qcap = c;
}

/* process.go:89-148  func (p Process) path(from, to vertexID, strongPath bool) bool */
int or_lit_path(const or_ldag *d, or_vid from, or_vid to, int strong_path) {
  if (vid_eq(from, to)) return 1; /* :91-93 self path */
  if (!tl_visited.cap) hs_init(&tl_visited, 1 << 12);
  hs_reset(&tl_visited);
  size_t head = 0, tail = 0;
  q_reserve(64);
  hs_insert(&tl_visited, vid_key(from)); /* :102-103 */
  tl_queue[tail++] = from;
  while (head < tail) { /* :105 */
    or_vid v = tl_queue[head++];
    if (v.round < 0 || v.round >= d->nrounds) return OR_PANIC; /* p.dag[vID.round] out of range */
    /* :111-116 linear scan, LAST match wins (no break) */
    int64_t idx = -1;
    for (uint32_t i = d->slot_off[v.round]; i < d->slot_off[v.round + 1]; i++)
      if (vid_eq(d->slot_id[i], v)) idx = i;
    if (idx < 0) continue; /* zero-valued vertex: no edges */
    /* :121-130 strong edges */
    for (uint32_t e = d->strong_off[idx]; e < d->strong_off[idx + 1]; e++) {
      or_vid t = d->strong_ids[e];
      if (!hs_has(&tl_visited, vid_key(t))) {
        if (vid_eq(t, to)) return 1;
        hs_insert(&tl_visited, vid_key(t));
        q_reserve(tail + 1);
        tl_queue[tail++] = t;
      }
    }
    if (!strong_path) { /* :132-144 weak edges */
      for (uint32_t e = d->weak_off[idx]; e < d->weak_off[idx + 1]; e++) {
        or_vid t = d->weak_ids[e];
        if (!hs_has(&tl_visited, vid_key(t))) {
          if (vid_eq(t, to)) return 1;
          hs_insert(&tl_visited, vid_key(t));
          q_reserve(tail + 1);
          tl_queue[tail++] = t;
        }
      }
    }
  }
  return 0;
}

static inline int wave_round(int w, int k) { return 4 * (w - 1) + k; } /* process.go:400-402 */
static inline int choose_leader(const or_ldag *d, int w) { return or_leader(d->leader, d->nleader, w); } /* :390-392 */

/* process.go:357-371 getWaveVertexLeader: FIRST slot with source == leader */
int or_lit_leader(const or_ldag *d, int wave, or_vid *leader) {
  int src = choose_leader(d, wave);
  int r = wave_round(wave, 1);
  if (r < 0 || r >= d->nrounds) return OR_PANIC;
  for (uint32_t i = d->slot_off[r]; i < d->slot_off[r + 1]; i++)
    if (d->slot_id[i].source == src) { *leader = d->slot_id[i]; return 1; }
  return 0;
}

/* process.go:314-354 waveReady (without the decidedWave write, which the caller
 * owns: Q1, value receiver). Returns 1 commit, 0 no commit, -1 panic. */
static int wave_ready_impl(const or_ldag *d, int faulty, int wave, int decided_wave, or_vid *stack,
                           int *stack_len, int stack_cap, int *vcount, int nthreads) {
  or_vid leader;
  *vcount = -1;
  int rc = or_lit_leader(d, wave, &leader);
  if (rc < 0) return OR_PANIC;
  if (rc == 0) return 0; /* :327-329 */
  int r4 = wave_round(wave, 4);
  if (r4 < 0 || r4 >= d->nrounds) return OR_PANIC;
  int vc = 0, panic = 0; /* :331-336 voter loop over every SLOT of dag[round(w,4)] (independent BFSs) */
  const int64_t a = d->slot_off[r4], b = d->slot_off[r4 + 1];
#pragma omp parallel for schedule(dynamic, 8) num_threads(nthreads > 1 ? nthreads : 1) reduction(+ : vc, panic)
  for (int64_t i = a; i < b; i++) {
    int p = or_lit_path(d, d->slot_id[i], leader, 1);
    if (p < 0) panic++;
    else vc += p;
  }
  if (panic) return OR_PANIC;
  *vcount = vc;
  if (vc < 2 * faulty + 1) return 0; /* :337-339 */
  if (*stack_len >= stack_cap) return OR_PANIC;
  stack[(*stack_len)++] = leader; /* :341 */
  for (int w = wave - 1; w >= decided_wave + 1; w--) { /* :342-350 */
    or_vid v;
    int ok = or_lit_leader(d, w, &v);
    if (ok < 0) return OR_PANIC;
    if (!ok) continue;
    int p = or_lit_path(d, leader, v, 1);
    if (p < 0) return OR_PANIC;
    if (!p) continue;
    if (*stack_len >= stack_cap) return OR_PANIC;
    stack[(*stack_len)++] = v;
    leader = v;
  }
  return 1;
}

int or_lit_wave_ready(const or_ldag *d, int faulty, int wave, int decided_wave,
                      or_vid *stack, int *stack_len, int stack_cap, int *vcount) {
  return wave_ready_impl(d, faulty, wave, decided_wave, stack, stack_len, stack_cap, vcount, 1);
}

static uint64_t slot_degree(const or_ldag *d, uint32_t i) {
  return (uint64_t)(d->strong_off[i + 1] - d->strong_off[i]) + (d->weak_off[i + 1] - d->weak_off[i]);
}

/* Repeated ids in a round (uponDeliver / the buffer loop append whatever they are
 * handed, process.go:158-169, :229).  The edge totals (this
 * repo's metric) count an id's edges once, those of the vertex path()'s lookup
 * finds: its LAST slot (:112-116).  slot_first: slot i is its id's first slot in
 * round r; slot_last: the id's last slot. */
static int slot_first(const or_ldag *d, int r, uint32_t i) {
  for (uint32_t j = d->slot_off[r]; j < i; j++)
    if (vid_eq(d->slot_id[j], d->slot_id[i])) return 0;
  return 1;
}
static uint32_t slot_last(const or_ldag *d, int r, uint32_t i) {
  uint32_t last = i;
  for (uint32_t j = i + 1; j < d->slot_off[r + 1]; j++)
    if (vid_eq(d->slot_id[j], d->slot_id[i])) last = j;
  return last;
}

/* process.go:404-443 orderVertices.  One pop per stack entry, top first.
 * mode REF: the delivered filter is a no-op (Q2, :423-427), so each pop
 * delivers its full causal history in rounds 1..cur_round.  mode PAPER:
 * skip ids already in `delivered` (Alg.3 line 54), which persists. */
/* nthreads > 1: the candidates' path() calls (independent BFSs) run on that
 * many OpenMP threads first; emission then walks them in order as above. */
static int order_pop(const or_ldag *d, or_vid popped, int cur_round, int mode, hset *delivered,
                     or_vid *out, int64_t out_cap, int64_t *out_n, uint64_t *count,
                     uint64_t *digest, uint64_t *edges, int nthreads) {
  uint64_t k = 0, dg = 0, ed = 0;
  int8_t *hit = NULL;
  uint32_t base = 0;
  if (nthreads > 1 && cur_round >= 1) {
    if (cur_round >= d->nrounds) return OR_PANIC;
    base = d->slot_off[1];
    const int64_t m = (int64_t)d->slot_off[cur_round + 1] - base;
    hit = (int8_t *)malloc((size_t)(m > 0 ? m : 1));
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads)
    for (int64_t i = 0; i < m; i++) hit[i] = (int8_t)or_lit_path(d, popped, d->slot_id[base + i], 0);
  }
  for (int r = 1; r <= cur_round; r++) { /* :417 */
    if (r >= d->nrounds) { free(hit); return OR_PANIC; }
    for (uint32_t i = d->slot_off[r]; i < d->slot_off[r + 1]; i++) { /* :418 */
      or_vid t = d->slot_id[i];
      int p = hit ? hit[i - base] : or_lit_path(d, popped, t, 0); /* :419 */
      if (p < 0) { free(hit); return OR_PANIC; }
      if (!p) continue;
      if (mode == OR_DELIVER_PAPER) {
        if (hs_has(delivered, vid_key(t))) continue;
      }
      /* :433-441 deliver (Broadcast + deliveredVertices append) */
      if (mode == OR_DELIVER_PAPER) hs_insert(delivered, vid_key(t));
      if (out && *out_n < out_cap) out[*out_n] = t;
      (*out_n)++;
      dg += or_digest_term(t.round, t.source, k);
      if (slot_first(d, r, i)) ed += slot_degree(d, slot_last(d, r, i)); /* an id's edges once */
      k++;
    }
  }
  free(hit);
  *count = k;
  *digest = dg;
  if (edges) *edges = ed;
  return 0;
}

int or_lit_order_vertices(const or_ldag *d, const or_vid *stack, int stack_len, int cur_round,
                          int mode, uint8_t *unused, or_vid *out, int64_t out_cap,
                          int64_t *out_n, uint64_t *pop_count, uint64_t *pop_digest) {
  (void)unused;
  hset del;
  hs_init(&del, 1 << 10);
  *out_n = 0;
  int j = 0;
  for (int top = stack_len - 1; top >= 0; top--, j++) { /* :412-413 LIFO pops */
    int rc = order_pop(d, stack[top], cur_round, mode, &del, out, out_cap, out_n,
                       &pop_count[j], &pop_digest[j], NULL, 1);
    if (rc < 0) { hs_free(&del); return rc; }
  }
  hs_free(&del);
  return 0;
}

/* Replay harness: the wiring process.go lacks (Q3): for each wave w, waveReady
 * and, on commit, orderVertices with p.round = round(w,4).  decidedWave is
 * 0 forever in CHAIN_LITERAL (Q1) or the last committed wave in
 * CHAIN_PERSISTENT. */
int or_lit_replay(const or_ldag *d, int faulty, int nwaves, int chain_mode, int deliver_mode,
                  or_replay_out *o) {
  return or_lit_replay_mt(d, faulty, nwaves, chain_mode, deliver_mode, 1, o);
}

/* The same replay with orderVertices' candidate path() calls spread over
 * nthreads OpenMP threads (the reference's algorithm and cost, one BFS per
 * candidate, on every core; results identical). */
int or_lit_replay_mt(const or_ldag *d, int faulty, int nwaves, int chain_mode, int deliver_mode, int nthreads,
                     or_replay_out *o) {
  hset del;
  hs_init(&del, 1 << 10);
  int decided = 0;
  int64_t npush = 0, npop = 0;
  o->n_ids = 0;
  o->commit_edges = o->chain_edges = o->deliver_edges = 0;
  or_vid *stack = (or_vid *)malloc((size_t)(nwaves + 1) * sizeof(or_vid));
  int rc = 0;
  for (int w = 1; w <= nwaves && rc == 0; w++) {
    int slen = 0, vc = -1;
    int c = wave_ready_impl(d, faulty, w, chain_mode == OR_CHAIN_PERSISTENT ? decided : 0, stack, &slen,
                            nwaves + 1, &vc, nthreads);
    if (c < 0) { rc = c; break; }
    o->commit[w - 1] = (uint8_t)c;
    o->vcount[w - 1] = vc;
    o->push_off[w - 1] = (uint32_t)npush;
    if (vc >= 0) { /* leader present: the voter loop examined rounds 4w-2..4w */
      for (int r = wave_round(w, 2); r <= wave_round(w, 4); r++)
        for (uint32_t i = d->slot_off[r]; i < d->slot_off[r + 1]; i++) {
          if (!slot_first(d, r, i)) continue; /* an id's row once: its last slot's */
          const uint32_t j = slot_last(d, r, i);
          o->commit_edges += d->strong_off[j + 1] - d->strong_off[j];
        }
    }
    if (!c) continue;
    if (npush + slen > o->push_cap) { rc = OR_PANIC; break; }
    for (int i = 0; i < slen; i++) o->push_wave[npush++] = (stack[i].round - 1) / 4 + 1;
    if (chain_mode == OR_CHAIN_PERSISTENT) decided = w; /* :352 */
    for (int top = slen - 1; top >= 0; top--, npop++) {
      uint64_t ed = 0;
      rc = order_pop(d, stack[top], wave_round(w, 4), deliver_mode, &del, o->ids, o->ids_cap,
                     &o->n_ids, &o->pop_count[npop], &o->pop_digest[npop], &ed, nthreads);
      if (rc < 0) break;
      o->pop_edges[npop] = ed;
      o->deliver_edges += ed;
    }
  }
  if (rc == 0) o->push_off[nwaves] = (uint32_t)npush;
  o->n_push = npush;
  free(stack);
  hs_free(&del);
  return rc;
}

/* ---- packed -> list expansion (what a Go caller's [][]vertex looks like) ---- */
int or_ldag_from_packed(const or_pdag *p, int nrounds, or_ldag *out) {
  if (nrounds > p->nrounds) nrounds = p->nrounds;
  uint32_t nslots = p->slot_off[nrounds];
  uint32_t *slot_off = (uint32_t *)malloc((size_t)(nrounds + 1) * sizeof(uint32_t));
  or_vid *slot_id = (or_vid *)malloc((size_t)(nslots + 1) * sizeof(or_vid));
  uint32_t *so = (uint32_t *)malloc((size_t)(nslots + 1) * sizeof(uint32_t));
  uint32_t *wo = (uint32_t *)malloc((size_t)(nslots + 1) * sizeof(uint32_t));
  /* count */
  uint64_t ns = 0, nw = 0;
  for (int r = 0; r <= nrounds; r++) slot_off[r] = p->slot_off[r];
  for (int r = 0; r < nrounds; r++)
    for (uint32_t i = p->slot_off[r]; i < p->slot_off[r + 1]; i++) {
      int s = p->slot_src[i];
      so[i] = (uint32_t)ns;
      wo[i] = (uint32_t)nw;
      if (s == 0) { slot_id[i].round = 0; slot_id[i].source = 0; continue; }
      slot_id[i].round = r;
      slot_id[i].source = s;
      const uint64_t *row = p->strong + ((size_t)r * p->n + (s - 1)) * p->W;
      for (int w = 0; w < p->W; w++) ns += (uint64_t)__builtin_popcountll(row[w]);
      size_t g = (size_t)r * p->n + (s - 1);
      for (uint32_t k = p->weak_off[g]; k < p->weak_off[g + 1]; k++) /* bit 31: a strong edge off r-1 */
        (p->weak_tgt[k] >> 31) ? ns++ : nw++;
    }
  so[nslots] = (uint32_t)ns;
  wo[nslots] = (uint32_t)nw;
  or_vid *sid = (or_vid *)malloc((size_t)(ns + 1) * sizeof(or_vid));
  or_vid *wid = (or_vid *)malloc((size_t)(nw + 1) * sizeof(or_vid));
  for (int r = 0; r < nrounds; r++)
    for (uint32_t i = p->slot_off[r]; i < p->slot_off[r + 1]; i++) {
      int s = p->slot_src[i];
      if (s == 0) continue;
      const uint64_t *row = p->strong + ((size_t)r * p->n + (s - 1)) * p->W;
      uint32_t e = so[i];
      for (int w = 0; w < p->W; w++) {
        uint64_t x = row[w];
        while (x) {
          int b = __builtin_ctzll(x);
          x &= x - 1;
          sid[e].round = r - 1;
          sid[e].source = w * 64 + b + 1;
          e++;
        }
      }
      size_t g = (size_t)r * p->n + (s - 1);
      uint32_t f = wo[i];
      for (uint32_t k = p->weak_off[g]; k < p->weak_off[g + 1]; k++) {
        uint32_t t = p->weak_tgt[k];
        or_vid *dst = (t >> 31) ? &sid[e++] : &wid[f++];
        dst->round = (int32_t)((t >> 11) & 0xFFFFFu);
        dst->source = (int32_t)(t & 2047u) + 1;
      }
    }
  out->nrounds = nrounds;
  out->slot_off = slot_off;
  out->slot_id = slot_id;
  out->strong_off = so;
  out->strong_ids = sid;
  out->weak_off = wo;
  out->weak_ids = wid;
  out->leader = p->leader;
  out->nleader = p->nleader;
  return 0;
}

void or_ldag_free(or_ldag *d) {
  free((void *)d->slot_off);
  free((void *)d->slot_id);
  free((void *)d->strong_off);
  free((void *)d->strong_ids);
  free((void *)d->weak_off);
  free((void *)d->weak_ids);
  memset(d, 0, sizeof *d);
}
