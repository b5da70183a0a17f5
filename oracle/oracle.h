/*
 * oracle.h -- CPU restatement of DAG-Rider's causal-history reachability path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (dag_rider_amd/, include/)
 * may include, link or call this code.  It is imported solely by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker.
 *
 * Parity pinning: the reference is Go (xenowits/dag-rider, /root/reference) and
 * no Go toolchain exists in this image, so the oracle is a restatement.  It is
 * pinned against the reference's own known answers (TestPath,
 * process/process_internal_test.go:20-83 on the Figure-1 DAG built at :86-283)
 * and the hand-derived answers of SURVEY.md s4 (tests/golden/figure1.json).
 *
 * Two restatements with identical outputs:
 *   lit_*  -- the reference algorithm as written: BFS with a hash-set
 *             `visited`, last-match linear id lookup per dequeue, one BFS per
 *             (leader, candidate) in orderVertices.  General graphs.
 *   bs_*   -- packed-bitset round sweeps (OpenMP over independent units).
 *             Edges to lower rounds only (rows: strong edges to r-1; weak_tgt: the rest).
 * They are cross-checked on thousands of seeded DAGs (tests/test_oracle.py).
 */
#ifndef DAGRIDER_ORACLE_H
#define DAGRIDER_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* vertexID, process/process.go:20-23 */
typedef struct { int32_t round, source; } or_vid;

/* List-form DAG: the literal shape of Process.dag [][]vertex (process.go:79),
 * flattened.  Round r owns slots [slot_off[r], slot_off[r+1]); slot i has id
 * slot_id[i] and edge lists strong_ids[strong_off[i]..strong_off[i+1]) and
 * weak_ids[weak_off[i]..weak_off[i+1]). */
typedef struct {
  int32_t nrounds;
  const uint32_t *slot_off;
  const or_vid *slot_id;
  const uint32_t *strong_off;
  const or_vid *strong_ids;
  const uint32_t *weak_off;
  const or_vid *weak_ids;
  const int32_t *leader; /* chooseLeader(w) = leader[w-1] for w <= nleader, else 1 (NULL: always 1) */
  int32_t nleader;
} or_ldag;

/* Packed DAG: strong rows indexed by (round, source-1), W = ceil(n/64) u64
 * words, bit (t-1) <=> strong edge to (round-1, t).  weak CSR indexed by the
 * vertex index r*n + (s-1); each weak target packed (round << 11) | (source-1).
 * With bit 31 set an entry is a strong edge to a round < r-1 (App. A Q8; the
 * bitset restatement takes those and weak edges to r-1, no edge upward).
 * slot_src holds the source of each slot (0 = ghost slot, id {0,0}). */
typedef struct {
  int32_t n, W, nrounds;
  const uint32_t *slot_off;
  const uint16_t *slot_src;
  const uint64_t *strong;
  const uint32_t *weak_off;
  const uint32_t *weak_tgt;
  const int32_t *leader; /* as or_ldag */
  int32_t nleader;
} or_pdag;

/* chooseLeader (process.go:386-392): the reference's constant 1, or the
 * caller's coin table (the engine's DR_LEADER_* modes) */
static inline int or_leader(const int32_t *leader, int32_t nleader, int w) {
  return (leader && w >= 1 && w <= nleader) ? leader[w - 1] : 1;
}

enum { OR_CHAIN_LITERAL = 0, OR_CHAIN_PERSISTENT = 1 };
enum { OR_DELIVER_REF = 0, OR_DELIVER_PAPER = 1 };
#define OR_PANIC (-1)

/* Replay outputs (caller-owned).  Waves are 1..nwaves; arrays indexed w-1.
 * push_off has nwaves+1 entries; the leaders pushed by wave w (in push order,
 * as wave numbers) are push_wave[push_off[w-1] .. push_off[w]).  Pops run in
 * reverse push order; pop j of the whole replay (global pop order) has
 * pop_count[j], pop_digest[j], pop_edges[j].  ids (optional, may be NULL)
 * receives the delivered vertex sequence, up to ids_cap entries. */
typedef struct {
  uint8_t *commit;
  int32_t *vcount;
  uint32_t *push_off;
  int32_t *push_wave;
  int64_t push_cap;
  uint64_t *pop_count;
  uint64_t *pop_digest;
  uint64_t *pop_edges;
  or_vid *ids;
  int64_t ids_cap;
  /* filled by the call */
  int64_t n_push;
  int64_t n_ids;
  uint64_t commit_edges, chain_edges, deliver_edges;
} or_replay_out;

/* digest term of the k-th delivered vertex (order-sensitive, summed mod 2^64) */
uint64_t or_digest_term(int32_t round, int32_t source, uint64_t k);

/* ---- literal restatement (process/process.go) ---- */
int or_lit_path(const or_ldag *d, or_vid from, or_vid to, int strong_path);
int or_lit_leader(const or_ldag *d, int wave, or_vid *leader); /* 1 found, 0 bottom, -1 panic */
int or_lit_wave_ready(const or_ldag *d, int faulty, int wave, int decided_wave,
                      or_vid *stack, int *stack_len, int stack_cap, int *vcount);
int or_lit_order_vertices(const or_ldag *d, const or_vid *stack, int stack_len,
                          int cur_round, int mode, uint8_t *delivered_rs /* nullable, paper mode */,
                          or_vid *out, int64_t out_cap, int64_t *out_n,
                          uint64_t *pop_count, uint64_t *pop_digest);
int or_lit_replay(const or_ldag *d, int faulty, int nwaves, int chain_mode,
                  int deliver_mode, or_replay_out *o);
int or_lit_replay_mt(const or_ldag *d, int faulty, int nwaves, int chain_mode, int deliver_mode, int nthreads,
                     or_replay_out *o);

/* expand a packed DAG (rounds [0, nrounds)) to list form; buffers malloc'd,
 * release with or_ldag_free */
int or_ldag_from_packed(const or_pdag *p, int nrounds, or_ldag *out);
void or_ldag_free(or_ldag *d);

/* ---- bitset restatement ---- */
int or_bs_path(const or_pdag *p, or_vid from, or_vid to, int strong_path);
int or_bs_cone(const or_pdag *p, or_vid from, int bottom, int strong_only,
               uint64_t *masks /* (from.round-bottom+1)*W, round-major from bottom */,
               uint64_t *edges);
int or_bs_commit_sweep(const or_pdag *p, int faulty, int w0, int w1,
                       uint8_t *commit, int32_t *vcount, uint64_t *edges);
int or_bs_order_vertices(const or_pdag *p, const or_vid *stack, int stack_len, int cur_round, int mode,
                         or_vid *out, int64_t out_cap, int64_t *out_n, uint64_t *pop_count,
                         uint64_t *pop_digest);
int or_bs_replay(const or_pdag *p, int faulty, int nwaves, int chain_mode,
                 int deliver_mode, int nthreads, or_replay_out *o);

#ifdef __cplusplus
}
#endif
#endif
