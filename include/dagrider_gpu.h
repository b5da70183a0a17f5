/*
 * dagrider_gpu.h -- C ABI of the MI355X causal-history reachability engine.
 *
 * Drop-in boundary for xenowits/dag-rider's hot path (process/process.go).
 * The reference has no FFI; its hot path is unexported methods of
 * process.Process.  Each entry point below names the Go function it replaces;
 * INTEGRATION.md shows the cgo binding a maintainer would add.
 *
 * Contract (cgo rules): only C scalars and flat caller-owned arrays cross the
 * boundary; the library keeps no host pointer after a call returns; calls on one
 * context are not thread-safe (the caller serialises them, as the reference's
 * single Start goroutine does); every call selects the context's device itself,
 * so goroutine/OS-thread migration is harmless.  Calls are synchronous.
 * Errors are negative status codes, never exceptions or aborts; the reference's
 * panics (index out of range, empty Pop) map to DR_E_INVAL.  dr_last_error()
 * describes the last failure.
 *
 * There is no CPU fallback: dr_create fails with DR_E_HIP when no gfx950
 * device is usable.
 *
 * Vertex ids travel as int32 pairs {round, source} (vertexID,
 * process/process.go:20-23).  Waves are 1-based; round(w, k) = 4(w-1)+k
 * (waveRound, process.go:400-402); the leader of wave w is chooseLeader(w)
 * (process.go:390-392): source 1 unless dr_set_leader_coin says otherwise.
 */
#ifndef DAGRIDER_GPU_H
#define DAGRIDER_GPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: dr_last_kernel_ms and dr_last_batch_phases added, dr_profile_kernel moved to the
 * profiling build (dagrider_tuning.h), repeated ids accepted by every append (Q6),
 * dr_replay_batch's ms_* fields keep their device meaning */
#define DR_ABI_VERSION 2

enum {
  DR_OK = 0,
  DR_E_INVAL = -1,    /* bad argument / reference would panic */
  DR_E_CAPACITY = -2, /* output buffer too small; required size reported */
  DR_E_HIP = -3,      /* device / runtime failure: the call may have stopped part-way (e.g. an append
                         whose rounds are mirrored without their irregular edges); destroy the context */
  DR_E_RCCL = -4,     /* collective failure */
  DR_E_CONTRACT = -5, /* DAG outside the mirrored contract (see dr_append_rounds_lists) */
  DR_E_STATE = -6     /* call order violated (e.g. append not contiguous) */
};
enum { DR_CHAIN_LITERAL = 0, DR_CHAIN_PERSISTENT = 1 };
enum { DR_OPT_MEMO = 1, DR_OPT_DEVICE_PLAN = 2, DR_OPT_PHASE_TIMING = 3, DR_OPT_BATCH_FORM = 4, DR_OPT_COMMIT_SPLIT = 5,
       DR_OPT_REPLAY_GRAPH = 6, DR_OPT_FUSE = 7, DR_OPT_CALL_OVERLAP = 8 };
enum { DR_BATCH_AUTO = 0, DR_BATCH_WORKGROUP = 1, DR_BATCH_WAVE = 2 };
enum { DR_DELIVER_REF = 0, DR_DELIVER_PAPER = 1 };
enum { DR_WEAK_LITERAL = 0, DR_WEAK_PAPER = 1 };

typedef struct dr_ctx dr_ctx;

int dr_abi_version(void);

/* New(index, faulty, tp) (process.go:34-60) minus the protocol state: one
 * device mirror of Process.dag (process.go:79) for n processes (sources
 * 1..n, n <= 2048), faulty = f (2f+1 thresholds, process.go:337).
 * max_rounds bounds the rounds that may be appended (device memory is sized
 * from it).  device >= 0 is a HIP ordinal. */
int dr_create(int n, int faulty, int max_rounds, int device, dr_ctx **out);
/* dr_create with flags.  DR_CREATE_SHARED_STREAM: the context enqueues on one HIP
 * stream shared by every such context of the device (created with the first, destroyed
 * with the last) instead of a stream of its own -- for batches of many small mirrors
 * (dr_replay_batch over thousands of contexts), where a device-wide synchronize walks
 * every stream of the process.  Calls on such contexts still return when their own work
 * is done; they may also wait for work other shared-stream contexts queued before it.
 * DR_OPT_REPLAY_GRAPH does not capture on a shared stream. */
enum { DR_CREATE_SHARED_STREAM = 1 };
int dr_create_ex(int n, int faulty, int max_rounds, int device, int flags, dr_ctx **out);
void dr_destroy(dr_ctx *ctx);
const char *dr_last_error(const dr_ctx *ctx);
/* Provenance: the sha256 (first 16 hex digits) of the sources this library was built
 * from (dag_rider_amd/csrc/{*.hip,*.hpp,*.cpp} and include/{*.h}, concatenated in byte
 * order of their paths), stamped by the Makefile.  Static string, never NULL. */
const char *dr_build_id(void);
/* number of rounds currently mirrored (len(p.dag)) */
int dr_num_rounds(const dr_ctx *ctx);
/* chooseLeader(w) (process.go:386-392): "a global perfect coin"; the
 * reference returns process 1 for every wave.
 *   DR_LEADER_CONST1  leader(w) = 1 (the default: parity with the code)
 *   DR_LEADER_SEEDED  leader(w) = dr_coin_leader(seed, w, n): a seeded coin
 *                     every process computes alike (agreement, fairness)
 *   DR_LEADER_TABLE   leader(w) = table[w-1] for w <= k (the caller's coin,
 *                     e.g. an (f+1)-of-n threshold signature), 1 beyond
 * Applies to every later waveReady / getWaveVertexLeader / replay. */
enum { DR_LEADER_CONST1 = 0, DR_LEADER_SEEDED = 1, DR_LEADER_TABLE = 2 };
int dr_set_leader_coin(dr_ctx *ctx, int mode, uint64_t seed, int k, const int32_t *table);
/* The seeded coin: 1 + splitmix64(seed + wave * 0x9E3779B97F4A7C15) mod n
 * (n = the context's process count). */
int dr_coin_leader(uint64_t seed, int wave, int n);
/* chooseLeader(wave) as the context currently decides it (1-based source). */
int dr_wave_leader(const dr_ctx *ctx, int wave);

/* DR_OPT_MEMO (default 1): use round summaries + the canonical cone for
 * orderVertices / path sweeps (identical results; 0 = sweep every cone).  It
 * applies while every weak delta is <= 65 and no weak edge spans more than
 * 1023 rounds.
 * DR_OPT_DEVICE_PLAN (default 1): dr_replay plans its chain, pop and emission
 * phases on the device (one host synchronisation per replay) when summaries
 * are on and no ids are requested, in both delivery modes; 0 = plan on the
 * host between phases (identical results).
 * DR_OPT_PHASE_TIMING (default 2): HIP events time every phase of a
 * device-planned dr_replay (ms_* outputs); 1 = the summary pass only, 0 = none
 * (untimed ms_* are 0).  Each timed event costs the stream a few microseconds.
 * DR_OPT_BATCH_FORM (default DR_BATCH_AUTO), read from the first context of a
 * dr_replay_batch: the fused small-DAG kernel's form.  DR_BATCH_WORKGROUP =
 * one workgroup of four wavefronts per DAG (shortest time per DAG),
 * DR_BATCH_WAVE = one wavefront per DAG (most DAGs per CU); AUTO takes the
 * wave form when the batch holds more than 6 DAGs per CU of the device.
 * DR_OPT_COMMIT_SPLIT (default 2): 1 = dr_wave_commit / dr_wave_ready on a
 * wave range shorter than the device's CU count split each wave's vote over
 * several workgroups (each computes S_1, S_2 whole and a share of S_3); 0 = one
 * workgroup per wave, the faster on MI355X at C4's 125-wave shares (DESIGN.md
 * s7); 2 = split ranges of at most 4 waves (the per-call waveReady).  Identical
 * results.
 * DR_OPT_REPLAY_GRAPH (default 0): 1 = a device-planned dr_replay called again
 * with the same DAG version, options, wave count, modes and push capacity is
 * captured once as a hipGraph (both streams' launches after the summary pass
 * and the copy of the outputs into pinned memory) and later such calls launch
 * the graph (with DR_OPT_PHASE_TIMING <= 1).  0 = launch every kernel per call,
 * as fast on MI355X at C3/C4.  Identical results.
 * DR_OPT_FUSE (default 23, bits): which independent phases of a device-planned REF
 * dr_replay share a launch with the phase beside them: 1 = the weak unions with the row
 * pass, 2 = the canonical re-emission with the delivery sweeps, 4 = the speculative
 * canonical prefixes with the canonical walk and the pop plan with the delivery sweeps;
 * 0 = each phase its own launch; + 8 = the delivery sweeps' queries
 * grouped by XCD (adjacent waves on one L2); + 16 = the delivery sweeps stop at the first
 * round whose state equals the canonical cone's (n > 512).  Identical results.
 * DR_OPT_CALL_OVERLAP (default 1): once the context answered a DR_DELIVER_REF
 * dr_order_vertices, dr_wave_ready launches the canonical cone of the new top round (what
 * the next REF dr_order_vertices merges with) without waiting for it: 1 = behind the
 * commit rule on the context's stream when no leader chain can follow (decided_wave >=
 * wave - 1), else after the wave's commit is known; 2 = on a second stream beside the
 * commit rule; 0 = dr_order_vertices computes it.  Identical results. */
int dr_set_option(dr_ctx *ctx, int option, int value);
/* The form of the context's last dr_replay: 1 = a captured graph was launched,
 * 0 = kernels launched one by one, -1 = one by one after a failed capture
 * (DR_OPT_REPLAY_GRAPH then stays off until set again). */
int dr_replay_graph_state(const dr_ctx *ctx);

/* p.dag[r] = append(p.dag[r], v) (process.go:229) for whole rounds
 * [r0, r0+k), r0 == dr_num_rounds(ctx): the flattened [][]vertex.
 *   slot_off   [k+1]   slots of round r0+i: [slot_off[i], slot_off[i+1])
 *   slot_id    [2*S]   vertex id per slot, in insertion order
 *   strong_off [S+1], strong_ids [2*E]   strongEdges per slot
 *   weak_off   [S+1], weak_ids   [2*E']  weakEdges per slot
 * Contract (else DR_E_CONTRACT): a slot's id is (r, s), 1 <= s <= n, or the
 * zero id {0,0} with no edges (the Figure-1 ghost slot,
 * process_internal_test.go:91); every edge targets an id (r', t) with
 * 0 <= r' < max_rounds, 1 <= t <= n.  Targets need not exist (a dangling
 * target counts as reached, process.go:123,136).  Strong edges to (r-1, t) and
 * weak edges below r-1 are the round contract the reference's own vertices
 * keep; any other edge (uponDeliver checks only the
 * strong-edge count, process.go:165 -- a strong edge to another round, a weak
 * edge to round r-1 or above, even a cycle) is kept too.  One that targets a
 * lower round is an exception (as are weak edges past the memo window and far
 * weak edges): the next query tests each new exception u -> v with one sweep
 * (is v in u's cone without the exceptions? then the edge changes no cone) and
 * the memoized path stays on while every one is (dr_exception_stats).  While
 * the mirror holds an edge to the same or a later round, or an exception
 * that changes a cone, every query runs on the general sweep (general.hpp:
 * exact for any graph, slower; dr_set_weak_edges then returns
 * DR_E_CONTRACT).  An id may
 * repeat within a round, as uponDeliver and the buffer loop let it
 * (process.go:158-169, :229): every slot is kept, path() sees the id's LAST
 * slot (:112-116), vCount and REF delivery count every slot (:332, :418-429),
 * PAPER delivers an id once, at its first slot; edge totals count an id's
 * edges once (its last slot). */
int dr_append_rounds_lists(dr_ctx *ctx, int r0, int k, const uint32_t *slot_off,
                           const int32_t *slot_id, const uint32_t *strong_off,
                           const int32_t *strong_ids, const uint32_t *weak_off,
                           const int32_t *weak_ids);

/* Same, pre-packed (the layout of dagrider_gen.h; W = ceil(n/64)):
 *   slot_src [slot_off[k]] source per slot (0 = ghost)
 *   strong   [k*n*W]  row of (r0+i, s) at (i*n + s-1)*W, zero for absent s
 *   weak_off [k*n+1]  relative offsets into weak_tgt (weak_off[0] may be != 0)
 *   weak_tgt          (round << 11) | (source-1): a weak edge; with bit 31 set, a
 *                     strong edge outside the row's round r-1 (App. A Q8).  A weak
 *                     edge to round r-1 or above is one too (dr_append_rounds_lists'
 *                     contract). */
int dr_append_rounds_packed(dr_ctx *ctx, int r0, int k, const uint32_t *slot_off,
                            const uint16_t *slot_src, const uint64_t *strong,
                            const uint32_t *weak_off, const uint32_t *weak_tgt);

/* p.dag[v.id.round] = append(p.dag[v.id.round], v) (process.go:229), one
 * vertex at a time, for k vertices in order -- the buffer loop's append, into
 * any mirrored round, not only new ones.  Vertex i goes to p.dag[r_i], r_i =
 * slot_round[i] (slot_round may be NULL: r_i = ids[2i], the Go index);
 * r_i == dr_num_rounds() opens that round, as growing p.dag by one would (a
 * larger r_i: DR_E_INVAL, Go's index out of range).  Its slot follows the
 * round's existing slots.  ids[2i], ids[2i+1] = (round, source); strong edges
 * strong_ids[2e..] for e in [strong_off[i], strong_off[i+1]), weak likewise.
 * Same contract as dr_append_rounds_lists (else DR_E_CONTRACT); a vertex whose
 * id is already in the round becomes the one path() sees (the last slot).  All or nothing: on
 * any error the mirror is unchanged.  Only the rounds touched are re-read when
 * round summaries or the canonical cone are next needed.  An edge may target
 * any round below max_rounds, also one not mirrored yet: such a target is a
 * dangling id (reached, never expanded), where Go's path() would index past
 * p.dag and panic once its BFS dequeued it (process.go:111) -- whether it does
 * depends on the BFS order, so this case answers instead of failing (parity
 * unpinned for it). */
int dr_append_vertices(dr_ctx *ctx, int k, const int32_t *slot_round, const int32_t *ids,
                       const uint32_t *strong_off, const int32_t *strong_ids, const uint32_t *weak_off,
                       const int32_t *weak_ids);

/* path(from, to, strongPath) (process.go:89-148) for q queries at once.
 * out[i] = 1 iff to_i is reachable from from_i (self-path included).
 * from.round outside the mirrored rounds (Go: index out of range) -> DR_E_INVAL. */
int dr_path_batch(dr_ctx *ctx, int q, const int32_t *from, const int32_t *to, int strong_only,
                  uint8_t *out);

/* Reach sets: for each query i, the set of ids reachable from from_i in rounds
 * [bottom_i, from_i.round], as W-word bitsets per round, round-major from
 * bottom_i, concatenated over queries (words_needed written to *out_words). */
int dr_reach_sets(dr_ctx *ctx, int q, const int32_t *from, const int32_t *bottom, int strong_only,
                  uint64_t *out, size_t cap_words, size_t *out_words);

/* setWeakEdges(v, round) (process.go:298-310) for a vertex v of round `round`
 * (1 <= round <= dr_num_rounds: v may belong to the next, not yet appended
 * round) whose strong edges are strong_ids (nstrong ids (round-1, t)).  Writes,
 * in the reference's order -- rounds round-2 down to 1, slots in insertion
 * order -- the ids that become v's weak edges:
 *   DR_WEAK_LITERAL  the code as written: v.id is still {0,0} when it runs
 *                    (SURVEY.md App. A Q5), so path() reaches nothing and
 *                    every slot except the zero id becomes a weak edge;
 *   DR_WEAK_PAPER    Alg. 2 lines 29-31: u is added iff no path from v, over
 *                    v's strong edges and the weak edges added so far, reaches
 *                    u (no DAG edge targets a ghost slot {0,0}: the first one
 *                    becomes a weak edge, which then reaches the others).
 * out_ids (may be NULL): 2 int32 per id, up to cap; *out_n = total (an
 * undersized out_ids gives DR_E_CAPACITY with *out_n set). */
int dr_set_weak_edges(dr_ctx *ctx, int round, int nstrong, const int32_t *strong_ids, int mode,
                      int32_t *out_ids, size_t cap, size_t *out_n);

/* One pass of the buffer loop (process.go:200-234) with present()
 * (process.go:374-384) as a presence-bitset test on the device, replacing the
 * reference's O(R*n) scan per predecessor.  The q buffered vertices, in buffer
 * order, have ids ids[2i], ids[2i+1] (round, source; 0 <= source <= n, else
 * DR_E_CONTRACT) and predecessors (strong then weak edges, any order)
 * preds[2e..] for e in [pred_off[i], pred_off[i+1]).  admit[i] = 1 iff
 * round_i <= cur_round and every predecessor is present in the mirrored rounds
 * 0..cur_round or is the id of a vertex j < i admitted earlier in the same
 * pass -- exactly the sequential pass.  The caller appends the admitted
 * vertices (buffer order) to the DAG (dr_append_vertices); the rest form the
 * new buffer.  The pass's Go panics return DR_E_INVAL: with cur_round >=
 * dr_num_rounds, present() runs off p.dag for any vertex of a round <=
 * cur_round that stays buffered (process.go:375-376); an admitted vertex of a
 * round >= dr_num_rounds panics at p.dag[v.id.round] (:229). */
int dr_buffer_admit(dr_ctx *ctx, int cur_round, int q, const int32_t *ids, const uint32_t *pred_off,
                    const int32_t *preds, uint8_t *admit);

/* The commit decision of waveReady (process.go:326-339) for waves w0..w1:
 * commit[i] = leader exists && vcount >= 2f+1; vcount[i] = number of slots of
 * round(w,4) with a strong path to the leader, -1 when the leader is bottom. */
int dr_wave_commit(dr_ctx *ctx, int w0, int w1, uint8_t *commit, int32_t *vcount);

/* waveReady(wave) (process.go:314-354) given decidedWave: commit decision and,
 * on commit, the leaders pushed onto leadersStack in push order (as waves),
 * leader first, then each w' in wave-1..decided_wave+1 strongly reachable from
 * the last pushed leader. */
int dr_wave_ready(dr_ctx *ctx, int wave, int decided_wave, uint8_t *commit, int32_t *vcount,
                  int32_t *pushed_waves, int cap, int *n_pushed);

/* orderVertices() (process.go:404-443) with leadersStack = stack_rs (bottom to
 * top, ids) and p.round = cur_round.  Pops run top first; each delivers, in
 * (round asc, slot asc) order over rounds 1..cur_round, every vertex reachable
 * from the popped leader -- all of them in DR_DELIVER_REF (the reference's
 * no-op filter, :423-427) or only those not delivered by an earlier pop of
 * this call in DR_DELIVER_PAPER (Alg. 3 line 54).  out_ids (may be NULL)
 * receives up to cap ids; *out_n = total delivered.  pop_count / pop_digest
 * (length nstack, may be NULL): per pop count and order-sensitive digest
 * sum_k mix(id_k, k). */
int dr_order_vertices(dr_ctx *ctx, const int32_t *stack_rs, int nstack, int cur_round, int mode,
                      int32_t *out_ids, size_t cap, size_t *out_n, uint64_t *pop_count,
                      uint64_t *pop_digest);

/* Whole replay (the wiring the reference omits): for
 * w = 1..nwaves, waveReady(w) and on commit orderVertices with
 * p.round = round(w,4); decidedWave stays 0 (DR_CHAIN_LITERAL, Q1) or becomes
 * the committed wave (DR_CHAIN_PERSISTENT). */
typedef struct {
  /* per wave (length nwaves) */
  uint8_t *commit;
  int32_t *vcount;
  /* pushed leaders, push order; wave w's are push_wave[push_off[w-1] .. push_off[w]) */
  uint32_t *push_off; /* nwaves + 1 */
  int32_t *push_wave;
  int64_t push_cap;
  /* per pop, global pop order (length >= total pushes) */
  uint64_t *pop_count;
  uint64_t *pop_digest;
  uint64_t *pop_edges;
  /* optional delivered ids (2 int32 each), may be NULL */
  int32_t *ids;
  int64_t ids_cap;
  /* results */
  int64_t n_push;
  int64_t n_ids;
  uint64_t commit_edges, chain_edges, deliver_edges;
  /* device time (ms) of each phase of the last call, HIP events (ms_summary: the
   * rows + commit pass k_summary_commit; the weak union that follows it is not
   * included).  A fused dr_replay_batch sets ms_deliver = the fused kernel in every
   * output and, in the first output only, the call's host phases: ms_commit = host
   * preparation before the launch, ms_summary = launch to results on the host,
   * ms_chain = the copy back (device), ms_emit = unpacking into the outputs.  A
   * device-planned REF dr_replay runs its leader chains inside the canonical walk's
   * launch and reports ms_chain = 0 */
  float ms_commit, ms_chain, ms_deliver, ms_emit, ms_summary;
  int32_t canon_segments; /* partial-round segments of the canonical cone (-1: summaries off) */
  /* work done by the delivery sweeps (identical leaders share one sweep):
   * sweeps, rounds expanded from rows (+ weak columns), strong-row bytes read
   * there (rows, plus 2-B degrees of rows skipped once the OR saturated), weak
   * columns scanned there, rounds expanded from the round summaries */
  uint64_t sweep_count, sweep_partial, sweep_row_bytes, sweep_weak_scanned, sweep_shortcut;
} dr_replay_out;

int dr_replay(dr_ctx *ctx, int nwaves, int chain_mode, int deliver_mode, dr_replay_out *o);

/* A batch of independent replays: dr_replay(ctxs[i], nwaves, chain_mode,
 * deliver_mode, &outs[i]) for i in [0, nctx), each context a separate
 * Process mirror (thousands of n=128 replays on one GPU).
 * Contexts must be distinct and on one device; errors name the context.
 * Outputs, semantics and capacities are exactly dr_replay's.  When every
 * context has n <= 128, nwaves <= 64, weak deltas < 32 and no ids are
 * requested, the whole batch runs as one fused kernel in one of two forms
 * (DR_OPT_BATCH_FORM): a workgroup of four wavefronts per DAG
 * (dag_rider_amd/csrc/batch.hpp) when each CU holds few DAGs, a wavefront per
 * DAG (batch1w.hpp) when it holds many; outs[i].ms_deliver = the launch's device
 * time, the other ms_* fields 0.  Otherwise the contexts replay one after
 * another through dr_replay. */
int dr_replay_batch(dr_ctx *const *ctxs, int nctx, int nwaves, int chain_mode, int deliver_mode,
                    dr_replay_out *outs);

/* The results of one context of a fused dr_replay_batch_view, in place: every
 * pointer is into one host region owned by the batch's first context, valid until
 * the next dr_replay_batch / dr_replay_batch_view on it or its destruction. */
typedef struct dr_replay_view {
  const uint8_t *commit;     /* [nwaves], as dr_replay_out.commit */
  const int32_t *vcount;     /* [nwaves] */
  const uint32_t *push_off;  /* [nwaves + 1] */
  const int32_t *push_wave;  /* [n_push] */
  const uint64_t *pop_count, *pop_digest, *pop_edges;  /* [n_push] */
  int64_t n_push;
  uint64_t commit_edges, chain_edges, deliver_edges;
  float ms_deliver;  /* the fused launch's device time (HIP events), as dr_replay_out.ms_deliver */
} dr_replay_view;

/* dr_replay_batch without copying each context's results out: views[i] points at
 * context i's results where the batch's single copy back left them (C5: 4096
 * contexts, ~0.3 ms of per-context copies saved).  Only for a batch that runs
 * fused (see dr_replay_batch; DR_E_INVAL otherwise); push_cap bounds each
 * context's pushes, as dr_replay_out.push_cap. */
int dr_replay_batch_view(dr_ctx *const *ctxs, int nctx, int nwaves, int chain_mode, int deliver_mode,
                         int64_t push_cap, dr_replay_view *views);

/* Device time (ms, HIP events) of the commit-rule kernel of the last
 * dr_wave_commit / dr_wave_ready / dr_replay on this context (observability,
 * like dr_shard_stats; no reference counterpart). */
int dr_last_kernel_ms(const dr_ctx *ctx, float *ms);
/* The exception test's state (dr_append_rounds_lists): out[0] exceptions mirrored,
 * out[1] of them found to change a cone at the last test, out[2] exception sweeps
 * run so far, out[3] the regular weak window (largest delta kept in the memo's
 * summaries), out[4] edges to the same or a later round, out[5] 1 while the
 * memoized path serves queries (every exception tested and benign, none upward). */
int dr_exception_stats(const dr_ctx *ctx, int64_t *out6);
/* The mirror's sizes (the bench's algorithmic byte counts): out[0] rounds, out[1] slots,
 * out[2] weak-column entries (distinct near weak targets per round), out[3] weak edges;
 * the first min(k, 4) are written. */
int dr_mirror_stats(const dr_ctx *ctx, int64_t *out, int k);

/* Host-side phases (ms, steady clock) of the last fused dr_replay_batch whose
 * first context is ctx: ms4[0] preparation before the launch (checks, job
 * table), [1] launch until the results are on the host, [2] the copy back
 * (device events), [3] unpacking into the callers' outputs (observability). */
int dr_last_batch_phases(const dr_ctx *ctx, float *ms4);
/* The fused form the last dr_replay_batch led by ctx ran: DR_BATCH_WORKGROUP
 * (k_replay_small) or DR_BATCH_WAVE (k_replay_small_1w); 0 when its shapes took one
 * dr_replay per context (or none ran yet). */
int dr_last_batch_form(const dr_ctx *ctx);
/* Host time of the last dr_append_rounds_packed (ms): ms4[0] validation and the rounds'
 * host state (weak columns), [1] rows and degrees staged, [2] the flattened per-round
 * arrays staged, [3] the copy launch (the call does not wait for the device: later
 * calls of the context run behind the copy on its stream). */
int dr_last_append_phases(const dr_ctx *ctx, float *ms4);

/* The path the last dr_replay took: 0 the memoized (or full-cone) replay on the
 * regular graph; 1 the same with weak edges to the same or a later round (App. A
 * Q8) checked against every cone it computed and found not to change one
 * (k_verify_up); 2 the general sweep after that check found a cone they change; 3 the
 * general sweep (strong edges upward, too many such edges, or PAPER delivery); -1
 * none yet. */
int dr_last_replay_path(const dr_ctx *ctx);

/* Wave-range slice of one DAG (SURVEY.md s8(e) row 1 widened to the whole replay:
 * waveReady :314-354 and orderVertices :404-443 of a contiguous wave range on the GPU
 * that holds only those rounds; dag_rider_amd/split.py).  The context mirrors global
 * rounds [round_offset, round_offset + nrounds) as its rounds 0.. (weak edges below
 * round_offset dropped, round 0's rows empty) and dr_replay then reports what the
 * whole DAG's replay reports for the slice's waves, up to additive offsets that the
 * ranks' dr_slice_out exchange supplies:
 *   - digest keys use global rounds (slice round + round_offset);
 *   - canonical positions start at pos_base, the canonical vertices of global rounds
 *     1..round_offset (so pop counts are global);
 *   - seeded_top > 0: the top seeded_top rounds are taken as full canonical rounds
 *     (K covers every present vertex) -- the rounds above a lower rank's waves, whose
 *     canonical cone the rank above reports (its C probes);
 *   - own_w0: the first slice wave this rank owns (1-based, slice numbering): the
 *     replay's min pop stop and owned chain edges count the commits from it on;
 *   - probes: the canonical prefixes C (count, from pos_base), G (digest, from 0) and
 *     E (edges, from 0) at up to 8 slice rounds.
 * Only dr_replay (REF delivery, persistent chains, memo path) runs on a sliced
 * context; the other query calls return DR_E_STATE while a slice is set.  NULL
 * clears it. */
typedef struct dr_slice_cfg {
  int32_t round_offset;
  int32_t seeded_top;
  uint64_t pos_base;
  int32_t own_w0;
  int32_t nprobe;
  int32_t probe[8];
} dr_slice_cfg;
typedef struct dr_slice_out {
  uint64_t C[8], G[8], E[8];   /* the canonical prefixes at cfg.probe[] */
  int32_t min_stop;            /* lowest merge round (slice numbering) of the pops of owned
                                  commits; < 0: one did not merge inside the slice */
  int32_t pad_;
  uint64_t own_chain_edges;    /* chain edges of the owned commits */
} dr_slice_out;
int dr_set_slice(dr_ctx *ctx, const dr_slice_cfg *cfg);
/* the slice outputs of the last dr_replay on a sliced context */
int dr_slice_result(const dr_ctx *ctx, dr_slice_out *out);

#ifdef __cplusplus
}
#endif
#endif
