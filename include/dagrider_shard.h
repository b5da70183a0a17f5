/*
 * dagrider_shard.h -- process-column sharded reachability.
 *
 * The same path()/reach-set queries as dagrider_gpu.h (process/process.go:89-148),
 * waveReady's commit and leader chain (:314-354) and orderVertices (:404-443),
 * for a DAG whose edge rows are split by TARGET column across G shards: shard g
 * stores, for every vertex (r, s), the words [g*C, (g+1)*C) of its strong row
 * (C = 64 * ceil(ceil(n/64) / G) target sources per shard) and the weak edges whose
 * target source lies in those columns.  A sweep keeps the whole frontier of the
 * current round on every shard (one u64 query mask per source: bit b <=> query b
 * reached it), expands it into its own columns of the rounds below, and the shards'
 * columns of the next frontier are all-gathered (one RCCL all-gather over xGMI per
 * round, in a batch of up to 64 queries).  Results are bit-identical to
 * dr_reach_sets / dr_path_batch on the unsharded DAG.
 *
 * Two exchange modes, chosen at creation:
 *   - RCCL: one process per GPU; the nshards ranks build a communicator from a
 *     unique id (dr_shard_unique_id on rank 0, broadcast by the caller).
 *   - local (id == NULL): one context holds all nshards column shards on one
 *     device and the exchange is the shared frontier buffer.  Same kernels, same
 *     column split; it is how the decomposition is tested on a 1-GPU box.
 *
 * Contract as dagrider_gpu.h: C scalars and caller-owned flat arrays, no host
 * pointer kept after a call, synchronous calls, negative status codes
 * (DR_E_* of dagrider_gpu.h), one caller thread per context.  In RCCL mode every
 * rank must make the same calls with the same arguments (the collective runs
 * inside them); every rank receives the full results.
 */
#ifndef DAGRIDER_SHARD_H
#define DAGRIDER_SHARD_H
#include <stddef.h>
#include <stdint.h>

#include "dagrider_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

#define DR_SHARD_ID_BYTES 128

typedef struct dr_shard dr_shard;

/* RCCL unique id for a new shard group (ncclGetUniqueId); rank 0 makes it and the
 * caller hands the bytes to every rank (e.g. torch.distributed broadcast). */
int dr_shard_unique_id(uint8_t *id);

/* dr_create (dagrider_gpu.h) for one column shard group.  nshards in [1, 64];
 * id != NULL: this process is shard `rank` of an RCCL group of nshards ranks;
 * id == NULL: local mode, this context holds every shard (rank must be 0). */
int dr_shard_create(int n, int faulty, int max_rounds, int device, int nshards, int rank, const uint8_t *id,
                    dr_shard **out);
void dr_shard_destroy(dr_shard *ctx);
const char *dr_shard_last_error(const dr_shard *ctx);
int dr_shard_num_rounds(const dr_shard *ctx);
/* this context's shards [*shard0, *shard0 + *nlocal) and the target sources
 * [*col0, *col1) (1-based, half-open) it stores */
int dr_shard_info(const dr_shard *ctx, int *nshards, int *shard0, int *nlocal, int *col0, int *col1);

/* p.dag[r] = append(...) (process.go:229): dr_append_rounds_packed's arguments and
 * contract; the context keeps only its columns.  Weak edges must satisfy
 * 2 <= r - r' <= 1023, and an id may not repeat within a round >= 1 (else
 * DR_E_CONTRACT; repeated ids replay on the unsharded engine).  The packed
 * format's irregular entries -- bit 31 of weak_tgt, a strong edge outside r-1,
 * and weak edges to r-1 or above (App. A Q8) -- are not supported here either
 * (DR_E_CONTRACT naming the edge); dr_append_rounds_packed takes them. */
int dr_shard_append_rounds_packed(dr_shard *ctx, int r0, int k, const uint32_t *slot_off, const uint16_t *slot_src,
                                  const uint64_t *strong, const uint32_t *weak_off, const uint32_t *weak_tgt);

/* dr_reach_sets (dagrider_gpu.h) on the sharded DAG: same arguments and output layout. */
int dr_shard_reach_sets(dr_shard *ctx, int q, const int32_t *from, const int32_t *bottom, int strong_only,
                        uint64_t *out, size_t cap_words, size_t *out_words);

/* dr_path_batch (path(), process.go:89-148) on the sharded DAG. */
int dr_shard_path_batch(dr_shard *ctx, int q, const int32_t *from, const int32_t *to, int strong_only,
                        uint8_t *out);

/* Options: DR_SHARD_OPT_PERSISTENT (default 1) runs a local-mode sweep batch as
 * one cooperative launch with grid barriers between rounds; 0 launches one
 * kernel per round (the RCCL mode's shape).  Results are identical. */
#define DR_SHARD_OPT_PERSISTENT 1
/* DR_SHARD_OPT_MEMO (default 1): dr_shard_replay runs the memoized path when
 * every weak delta is <= 65 -- per-shard round summaries, the canonical cone,
 * and every leader chain and delivery cone stepped together by relative round
 * (a cone stops where its frontier merges with the canonical cone; one exchange
 * per step for all queries); PAPER delivery assigns each vertex to the first
 * pop whose cone holds it.  0 = the batched full sweeps.  Results are
 * identical. */
#define DR_SHARD_OPT_MEMO 2
/* DR_SHARD_OPT_STEPPED (default 0): when the context holds every column (local
 * mode, a one-rank group) the memoized replay runs "fused": each kernel reads all
 * columns, so every query runs to its end in one launch and nothing is
 * exchanged.  1 runs the stepped form instead -- one round of every live query
 * per launch with the columns exchanged between launches, what each rank of a
 * group of G > 1 runs -- so one device can check it.  Results are identical. */
#define DR_SHARD_OPT_STEPPED 3
/* DR_SHARD_OPT_PHASE_TIMING (default 1): the memoized replay records HIP events
 * between its phases and reports them in dr_replay_out.ms_*; 0 leaves them 0
 * (reading the events back costs the host ~20 us per replay). */
#define DR_SHARD_OPT_PHASE_TIMING 4
/* DR_SHARD_OPT_STEP_HINTS (tuning and tests): the stepped form launches as many
 * steps of the canonical walk and of the query batch as the last replay needed
 * (8 and 12 before the first) and continues a query still live after them; value
 * (>= 1) resets both counts, e.g. 1 forces every continuation path.  Results are
 * identical. */
#define DR_SHARD_OPT_STEP_HINTS 5
int dr_shard_set_option(dr_shard *ctx, int option, int value);

/* chooseLeader (process.go:386-392): dr_set_leader_coin's modes and semantics. */
int dr_shard_set_leader_coin(dr_shard *ctx, int mode, uint64_t seed, int k, const int32_t *table);

/* dr_wave_commit (waveReady's commit decision, process.go:326-339) on the sharded
 * DAG: each shard tests its columns of every row of rounds 4w-2..4w against its
 * columns of the previous step's set; the partial hits are OR-ed across shards
 * (one all-gather per step in RCCL mode).  Same outputs as dr_wave_commit. */
int dr_shard_wave_commit(dr_shard *ctx, int w0, int w1, uint8_t *commit, int32_t *vcount);

/* dr_wave_ready (waveReady, process.go:314-354) on the sharded DAG. */
int dr_shard_wave_ready(dr_shard *ctx, int wave, int decided_wave, uint8_t *commit, int32_t *vcount,
                        int32_t *pushed_waves, int cap, int *n_pushed);

/* dr_order_vertices (orderVertices, process.go:404-443) on the sharded DAG:
 * per-pop counts and digests (no id list); *out_n = total delivered. */
int dr_shard_order_vertices(dr_shard *ctx, const int32_t *stack_rs, int nstack, int cur_round, int mode,
                            size_t *out_n, uint64_t *pop_count, uint64_t *pop_digest);

/* dr_replay on the sharded DAG: commit, chains and delivery of waves 1..nwaves,
 * every output of dr_replay_out except the id list (o->ids must be NULL or
 * ids_cap 0) and the memo statistics.  ms_commit / ms_chain / ms_deliver
 * (cone sweeps) / ms_emit (dedup, counts, digests) are HIP-event times. */
int dr_shard_replay(dr_shard *ctx, int nwaves, int chain_mode, int deliver_mode, dr_replay_out *o);

/* Last query call: device time (ms, HIP events around the sweeps, exchange
 * included), rounds stepped, and bytes this rank sent through the exchange. */
int dr_shard_stats(const dr_shard *ctx, float *ms, uint64_t *rounds, uint64_t *exchange_bytes);

/* Host waits (stream synchronisations) of the last dr_shard_replay on the memoized
 * path: 1 when every launch of the replay went out back to back and the host
 * waited once, for the results (more after an append, whose weak columns upload
 * first, or when a query was still live after the launched steps). */
int dr_shard_host_syncs(const dr_shard *ctx, uint64_t *syncs);

#ifdef __cplusplus
}
#endif
#endif
