/*
 * dagrider_gen.h -- deterministic synthetic DAG-Rider DAGs (host side).
 *
 * Produces DAGs in the packed layout dr_append_rounds_packed() consumes
 * (dagrider_gpu.h).  There is no counterpart in the reference (it has no
 * generator or benchmark); the spec is SURVEY.md s8(d):
 *
 *   round 0      n genesis vertices (0,s), slot order 1..n, no edges
 *   round r>=1   source s present w.p. p_present (source 1 on a leader round
 *                r = 4w-3 absent w.p. p_la instead); topped up to >= 2f+1
 *                present; slot order = seeded Fisher-Yates of the present set
 *   late L(r)    up to f present vertices (each w.p. p_late, capped so that
 *                >= 2f+1 stay eligible) that round r+1 never references
 *   strong(r,s)  k ~ U[2f+1, m] distinct targets drawn by selection sampling
 *                from E(r-1) = present(r-1) \ L(r-1), m = |E(r-1)|
 *   weak(r,s)    each u in L(r') for r' in [max(1, r-D), r-2], w.p. p_w,
 *                sorted by (r', source)
 *
 * Every draw comes from a splitmix64 stream keyed by (seed, round, source,
 * purpose), so generation is parallel and bit-reproducible.
 */
#ifndef DAGRIDER_GEN_H
#define DAGRIDER_GEN_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int32_t n;          /* processes, sources 1..n (n <= 2048) */
  int32_t last_round; /* R: rounds 0..R are generated */
  uint64_t seed;
  double p_present, p_late, p_w, p_la;
  int32_t weak_depth; /* D */
  int32_t nthreads;   /* 0 = library default */
} dr_gen_params;

typedef struct dr_gen_dag dr_gen_dag;

/* Generate.  The handle owns the arrays; views stay valid until dr_gen_free. */
int dr_gen_create(const dr_gen_params *prm, dr_gen_dag **out);
void dr_gen_free(dr_gen_dag *g);

/* Views (packed layout; W = ceil(n/64)):
 *   slot_off  [R+2]          slots of round r: [slot_off[r], slot_off[r+1])
 *   slot_src  [slot_off[R+1]] source per slot (1..n)
 *   strong    [(R+1)*n*W]    row of (r, s) at ((r*n) + s-1) * W, bit t-1 <=> edge to (r-1, t)
 *   weak_off  [(R+1)*n + 1]  weak edges of (r, s): [weak_off[r*n+s-1], weak_off[r*n+s])
 *   weak_tgt  [weak_off[(R+1)*n]]  (round << 11) | (source-1) */
int dr_gen_info(const dr_gen_dag *g, int32_t *n, int32_t *W, int32_t *nrounds, uint64_t *nslots,
                uint64_t *nweak);
const uint32_t *dr_gen_slot_off(const dr_gen_dag *g);
const uint16_t *dr_gen_slot_src(const dr_gen_dag *g);
const uint64_t *dr_gen_strong(const dr_gen_dag *g);
const uint32_t *dr_gen_weak_off(const dr_gen_dag *g);
const uint32_t *dr_gen_weak_tgt(const dr_gen_dag *g);

#ifdef __cplusplus
}
#endif
#endif
