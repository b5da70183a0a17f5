// engine.hip -- host side of the C ABI (include/dagrider_gpu.h): the device
// mirror of Process.dag, validation, kernel orchestration.
//
// One dr_ctx per reference Process.  The DAG lives in HBM in the packed layout
// of kernels.hpp; host keeps only slot lists, presence bits and per-round
// degree sums (for leader lookups, emission bounds and edge accounting).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <thread>
#include <climits>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <functional>
#include <mutex>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "dagrider_gpu.h"
#include "host_rounds.hpp"
#include "kernels.hpp"
#include "replay_plan.hpp"
#include "batch.hpp"
#include "batch1w.hpp"
#include "general.hpp"

using dr::u64;

namespace {

thread_local std::string g_create_err;

// Context generations: every ABI call that may change a context (appends, options,
// replays that grow its buffers) gives it a new generation from one process-wide
// counter, and so does dr_create -- a generation is never reused, so a destroyed
// context whose address comes back in a new one cannot match.  A cached
// dr_replay_batch plan is valid while every member context keeps the generation it
// was built at.
std::atomic<uint64_t> g_ctx_gen{1};
uint64_t next_gen() { return g_ctx_gen.fetch_add(1, std::memory_order_relaxed) + 1; }

// The memo's weak-delta window: WU holds dmax - 1 unions per
// round and a merge needs dmax equal rounds, so a deeper window costs every pop
// sweep more rounds; beyond it the full sweeps run.
constexpr int kMemoMaxDelta = 255;

int next_pow2(int x) {
  int p = 1;
  while (p < x) p <<= 1;
  return p;
}

struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    // a buffer that grows (per-call paths on a growing DAG: masks, plan arena, summaries)
    // takes 1.5x, so that it is not freed every call: hipFree waits for the device
    const size_t c = std::max<size_t>({bytes, cap ? cap + cap / 2 : 0, 4096});
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(&p, c);
    if (e == hipSuccess) cap = c;
    return e;
  }
  // grow keeping the first `keep` bytes
  hipError_t grow(size_t bytes, size_t keep, hipStream_t s) {
    if (bytes <= cap) return hipSuccess;
    size_t c = std::max<size_t>({bytes, cap * 2, 4096});
    void *q = nullptr;
    hipError_t e = hipMalloc(&q, c);
    if (e != hipSuccess) return e;
    if (p && keep) {
      e = hipMemcpyAsync(q, p, keep, hipMemcpyDeviceToDevice, s);
      if (e == hipSuccess) e = hipStreamSynchronize(s);
      if (e != hipSuccess) { (void)hipFree(q); return e; }
    }
    if (p) (void)hipFree(p);
    p = q;
    cap = c;
    return hipSuccess;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T> T *as() const { return static_cast<T *>(p); }
};

// Host copy of one round of Process.dag (process.go:79): what the kernels need
// beyond the fixed-stride device arrays.  Variable-size per-round data lives
// here and is flattened to the device from the lowest changed round on
// (dr_ctx::upload_suffix), so a vertex appended to an old round
// (process.go:229) rewrites only the rounds from there to the top.
using dr_host::HostRound;

}  // namespace

struct dr_ctx {
  int n = 0, f = 0, W = 0, WS = 0, max_rounds = 0, dev = 0;
  int nrounds = 0;
  int dmax_near = 1;  // largest weak delta stored in the near format
  hipStream_t stream = nullptr;
  bool shared_stream = false;  // DR_CREATE_SHARED_STREAM: stream is the device's shared one
  hipEvent_t ev[8] = {};
  // device DAG
  DevBuf strong, present, slot_off, slot_src, weak_roff, far, far_roff;
  DevBuf ppref;  // [round] |P_1| + .. + |P_r| (present vertices, round 0 excluded)
  size_t nfar = 0;
  // weak columns (kernels.hpp DagView::wc_*): one entry per distinct near weak
  // target (delta, t) of a round + the bitset of the round's sources pointing at it
  DevBuf wc_key, wc_rows, wc_roff;
  DevBuf sdeg;  // [max_rounds][n] u16 strong degree per vertex (kernels.hpp expand_rows)
  DevBuf setweak;  // dr_set_weak_edges scratch
  DevBuf admit_buf;  // dr_buffer_admit scratch
  DevBuf wdeg;     // [max_rounds][n] u16 weak degree per vertex (batch.hpp)
  DevBuf put_buf;  // dr_append_vertices staging on the device
  // chooseLeader (process.go:386-392): leader source of every wave, index w
  // (DR_LEADER_CONST1: 1, the reference's constant), mirrored on the device
  DevBuf lead;
  std::vector<uint16_t> h_lead;
  // repeated ids (DagView::dup_*): slots after the first of their id, per round
  DevBuf slot_rep, dup_off, dup_src;
  std::vector<uint32_t> h_dup_off{0};
  int64_t ndups = 0;  // repeated slots in rounds >= 1 (round 0 may repeat ids: never read)
  // edges outside the round contract (App. A Q8: a strong edge not to r-1, a weak
  // edge not below r-1): while any is mirrored every query takes the general sweep
  int64_t nirr = 0;
  int irr_tmax = 0;  // the highest round an irregular edge targets (the general sweep's row extent)
  DevBuf irr, irr_roff, gscratch, gquery, gaux;
  std::vector<uint32_t> h_irr_roff{0};
  // Exceptions: the regular graph G_reg holds the strong rows and the weak
  // columns of delta <= reg_max(); every other edge below its round -- a weak column past
  // the window, a far weak edge, an irregular edge to a lower round -- is an exception.
  // An exception u -> v with v in u's G_reg cone (its strong cone for a strong edge) is
  // benign: it changes no cone, so every query may run on G_reg's summaries and canonical
  // cone.  ensure_exceptions tests the exceptions of the rounds touched since its last
  // test, one sweep each; an irregular edge to the same or a later round (irr_up) always
  // takes the general sweep.  Per round (upload_suffix): the largest regular delta, the
  // exception count, the irr_up count; per round (ensure_exceptions): exceptions found
  // not benign.
  std::vector<int32_t> h_rdreg, h_rexc, h_rup, h_rbad;
  // upward irregular edges that are strong ones (h_rups): a weak-only upward set may take
  // the verified memo replay (dr_replay: up_verify, replay_plan.hpp k_verify_up)
  std::vector<int32_t> h_rups;
  int64_t nirr_ups = 0;
  bool up_verify = false;
  DevBuf upe, upbad;            // the upward weak edges (ru, su0, rv, tv0), the violation count
  std::vector<uint64_t> upe_key;
  int upe_n = 0;
  int last_path = -1;           // dr_last_replay_path
  std::vector<uint32_t> h_sdx;  // [round] strong edges outside the rows (DagView::sdx)
  DevBuf sdx;
  bool sdx_valid = false;       // the device copy holds every mirrored round's h_sdx
  int dreg = 1;            // largest regular weak delta (1: none)
  int64_t nexc = 0, nirr_up = 0, nirr_down = 0, nbad = 0;
  int exc_lo = 0;          // lowest round touched since the last exception test
  uint64_t exc_sweeps = 0; // exception sweeps run (dr_exception_stats)
  int depth_cap() const {
    const int cap_words = (65536 - 64) / 8 - 2 * WS;
    int cap = 1;
    while (cap * 2 * WS <= cap_words) cap *= 2;
    return cap;
  }
  int reg_max() const { return std::min(kMemoMaxDelta, depth_cap() - 1); }
  // the lowest round holding an edge to the same or a later round (INT_MAX: none): a
  // general sweep toward a target in round t never needs the rounds below t unless some
  // path climbs back from there, which only such an edge below t allows
  // wave-range slice (dr_set_slice): dr_replay only, REF + persistent on the memo path
  bool slice_on = false;
  dr_slice_cfg slice{};
  dr_slice_out slice_res{};
  // (cached in up_min: upload_suffix recomputes it from the lowest round it rewrote)
  int up_min = INT_MAX;
  int min_up_round() const { return nirr_up == 0 ? INT_MAX : up_min; }
  int gsweep_bottom(int t) const { return (t >= 0 && min_up_round() >= t) ? t : 0; }
  // every exception known benign (the last test covers every round)
  bool exc_clear() const { return nexc == 0 || (exc_lo >= nrounds && nbad == 0); }
  bool general() const { return (nirr_up > 0 && !up_verify) || (nirr_down > 0 && !exc_clear()); }
  // dr_replay may take the memo path with a per-replay check of the upward edges: weak ones
  // only, a bounded number of them, every downward exception benign
  static constexpr int64_t kMaxUpVerify = 1 << 14;
  // (the downward exceptions are worth testing: a verified replay can use the memo)
  bool up_verifiable_structure() const { return nirr_ups == 0 && nirr_up <= kMaxUpVerify; }
  bool up_verifiable() const {
    return nirr_up > 0 && nirr_ups == 0 && nirr_up <= kMaxUpVerify && (nirr_down == 0 || exc_clear());
  }
  dr::GView gview() const { return dr::GView{irr.as<uint64_t>(), irr_roff.as<uint32_t>()}; }
  int lead_src(int w) const { return (w >= 0 && w < (int)h_lead.size()) ? h_lead[w] : 1; }
  // host mirror: per-round data, presence [rounds][WS], and the prefix offsets
  // of the flattened device arrays (valid for rounds < up_lo)
  std::vector<HostRound> hr;
  // per vertex [round][n]: strong degree and weak-edge count of the id's current
  // vertex (its last slot), so a repeated id can take back the one it replaces
  std::vector<uint16_t> h_sdeg, h_wcnt;
  dr_host::BuildScratch build_scr;  // dr_append_rounds_packed's per-thread column tables
  std::vector<u64> h_present;
  std::vector<uint32_t> h_slot_off{0}, h_wc_roff{0}, h_far_roff{0}, h_weak_roff{0};
  std::vector<u64> h_ppref;
  int up_lo = 0;  // lowest round whose flattened device arrays are stale
  // round summaries (U, SD, WU) per round: sdirty[r] = stale; the canonical cone
  // and its prefixes (K, C, G, E) describe the DAG as of the last canon build
  bool use_memo = true;
  uint64_t version = 0;  // bumped by every change of the DAG or the leader coin
  std::vector<uint8_t> sdirty;
  int sum_dd = -1;            // WU layout the summaries were built with (memo_dd())
  bool canon_ok = false;      // K/C/G/E describe the current DAG
  int32_t canon_segments = 0;
  DevBuf U, WU, SD, K, good, CE, RD, Cc, Gc, Ec, crbase, ccount, nseg, stops, qstats, srounds;
  // incremental canonical cone: the previous cone, per-round
  // canonical digests, the lowest round to re-emit; canon_lo = lowest round
  // touched since the last cone
  DevBuf Kprev, RG, rlo;
  // k_commit_split: [wave] arrivals << 32 | |S_3| sum, kept zero between launches
  DevBuf split_ctl;
  size_t split_nw = 0;
  int split_cap = 0;  // CUs of this device (0: not read yet): ranges shorter than this split
  // DR_OPT_COMMIT_SPLIT: 2 (default) splits ranges of at most kSplitAuto waves -- the
  // per-call waveReady's single wave: k_commit's one workgroup reads its three rounds
  // alone (C4: 16 us, profiles/r05/v10_timeline_loop.txt); at C4's N = 8 share (125 waves)
  // k_commit_split took 29 us against 22 us for k_commit (profiles/r04/); 1 = every range
  // shorter than the CU count, 0 = never
  int commit_split = 2;
  // the planned replay's leader chains on one register-resident wavefront each at n <= 256
  // (k_chain_reg; DR_CHAIN_REG=0: k_sweep's chain mode)
  int chain_reg = getenv("DR_CHAIN_REG") ? atoi(getenv("DR_CHAIN_REG")) : 1;
  // DR_OPT_FUSE: bit 0 = a full replay's weak unions ride in the row pass's launch
  // (dr::WUArgs, the chain plan then in k_kcand_plan); bit 1 = the canonical re-emission
  // rides in the delivery sweeps' launch; bit 2 = the speculative G, E prefixes beside the
  // canonical walk (k_canon_chains) and the pop plan beside the delivery sweeps; bit 3 = the
  // delivery sweeps' queries grouped by XCD (dr::CanonEmit::xcd); bit 4 = the static delivery queries merge
  // fast (dr::Q_FAST); bit 5 = each query's own rounds emitted by its sweep workgroup (dr::OwnEmit)
  int fuse = getenv("DR_FUSE") ? atoi(getenv("DR_FUSE")) : 23;
  // DR_OPT_CALL_OVERLAP: once a REF orderVertices was answered, dr_wave_ready starts the
  // canonical cone of the new top on stream2 beside the commit rule (the next
  // dr_order_vertices merges with it); s2_detached: that work is in flight, the waits
  // inside dr_wave_ready skip stream2 and its end joins it on the device (ev_join)
  int call_overlap = getenv("DR_CALL_OVERLAP") ? atoi(getenv("DR_CALL_OVERLAP")) : 1;
  bool ref_seen = false, s2_detached = false;
  int last_split = 0;   // workgroups per wave of the last commit launch (0: k_commit)
  int canon_lo = 0, canon_dd = -1;
  bool kprev_ok = false;
  int ndirty = 0;     // rounds with sdirty set
  int canon_T = -1;   // top round of the last canonical build
  std::vector<uint64_t> hC, hG, hE;
  bool canon_host = false;
  // DR_OPT_PHASE_TIMING: 2 = HIP events around every replay phase, 1 = around the
  // summary pass only (ev[6], ev[7]), 0 = none.  Each timed event record costs the
  // stream a few microseconds.
  int phase_timing = 2;
  bool timed(int i) const { return phase_timing >= 2 || (phase_timing == 1 && (i == 6 || i == 7)); }
  hipError_t rec(int i) { return timed(i) ? hipEventRecord(ev[i], stream) : hipSuccess; }
  // DR_OPT_REPLAY_GRAPH (default 0): a device-planned dr_replay whose configuration
  // (graph_key) matches the previous call's is captured once as a hipGraph --
  // every launch, both streams, the copy of the outputs into pinned memory -- and
  // later calls with the same key launch that graph.  The summary pass stays outside the
  // graph, between its timing events (an event record inside a capture needs
  // hipEventRecordExternal, which the HIP runtime torch loads refuses).  Off by default:
  // C4 0.220 ms per step with the graph, 0.214 without; C3 0.272 / 0.270
  // (profiles/r04/v6_graph_*) -- the device-side gaps between dependent kernels stay
  int replay_graph = 0;
  int graph_fail = 0;      // a capture or instantiation failed: eager launches from then on
  int graph_state = 0;     // dr_replay_graph_state: the last dr_replay's form
  uint64_t cfg_gen = 0;    // bumped by dr_set_option
  std::vector<uint64_t> last_key, rg_key;
  hipGraphExec_t rg_exec = nullptr;
  int plan_mode = 1;        // DR_OPT_DEVICE_PLAN: dr_replay planned on the device when it applies
  int batch_form = DR_BATCH_AUTO;  // DR_OPT_BATCH_FORM (dr_replay_batch, first context)
  int last_batch_form = 0;         // dr_last_batch_form: the fused form this context's last batch ran
  float append_phases[4] = {};     // dr_last_append_phases: the last dr_append_rounds_packed (host ms)
  int cu_count = 0;         // compute units of the device (dr_replay_batch's form choice)
  float last_commit_ms = 0;  // dr_last_kernel_ms: the last commit-rule launch (HIP events)
  float batch_phases[4] = {};
  std::vector<dr_replay_out> view_outs;  // dr_replay_batch_view's capacities (this context first)
  uint64_t gen = 0;  // context generation (g_ctx_gen): bumped by every call that may change the context
  void touch() { gen = next_gen(); }  // dr_last_batch_phases: host prep, launch -> host, copy back, unpack
  // REF planned replay: the static delivery-query table, one query per wave whose leader
  // is present (highest wave first, masks of rounds 0..top each), wave -> query index, and
  // a constant plan header {PL_NQD = count, PL_CAPERR = 0} for the launches that must not
  // read the chain planner's (it runs on the second stream)
  DevBuf sdq, sqidx, splan;
  DevBuf pushed;            // [wave] the replay stamp of a chain push (dr::PopMark)
  int32_t pop_epoch = 0;
  std::vector<uint64_t> sdq_key;
  int sdq_n = 0;
  bool sdq_fast = false;  // the static table's queries carry Q_FAST
  DevBuf plan_arena;        // device-planned replay (replay_plan.hpp)
  DevBuf plan_out;          // its outputs, packed for one copy back
  std::vector<char> plan_host;
  DevBuf batch_arena;       // dr_replay_batch scratch + outputs (batch.hpp)
  char *batch_pin = nullptr;     // dr_replay_batch output region, host side (pinned: ~5 MB at C5)
  size_t batch_pin_cap = 0;
  std::vector<dr::SmallJob> batch_jobs;  // the job table last uploaded to the arena
  // the last fused batch this context led (dr_replay_batch's first context): a call with
  // the same contexts, modes and output buffers, and no ABI call that could change a
  // member since (its generation), reuses its checks, job table and output layout
  struct BatchPlan {
    bool valid = false;
    int nw = 0, chain_mode = 0, deliver_mode = 0, dmax = 0;
    size_t out0 = 0, out1 = 0, jobs_at = 0;  // output region, job table (arena offsets)
    std::vector<dr_ctx *> ctxs;
    std::vector<uint64_t> gens;  // each member's generation when the plan was built
    std::vector<char> out_keys;  // each output's caller-set prefix (commit .. ids_cap)
  } batch_plan;
  hipError_t batch_host(size_t n, char **out) {
    if (n > batch_pin_cap) {
      if (batch_pin) (void)hipHostFree(batch_pin);
      batch_pin = nullptr;
      batch_pin_cap = 0;
      const size_t cap = std::max<size_t>(n, (size_t)1 << 20);
      hipError_t e = hipHostMalloc((void **)&batch_pin, cap, hipHostMallocMapped);
      if (e != hipSuccess) return e;
      batch_pin_cap = cap;
    }
    *out = batch_pin;
    return hipSuccess;
  }
  // memo (round summaries + canonical cone) over the regular graph: weak deltas up to
  // reg_max() (WU holds dd = dreg - 1 slots per round, the merge window is dreg rounds,
  // the sweeps' LDS ring holds them), every exception benign, no irregular edge upward
  bool memo_struct_ok() const { return nirr_up == 0 || up_verify; }
  bool memo_ok() const { return memo_struct_ok() && exc_clear(); }
  // repeated ids: the summaries' counts and the emission count every slot of a
  // reached id (REF), PAPER delivers an id at its first slot (slot_rep)
  bool memo_on() const { return use_memo && memo_ok(); }
  int memo_dd() const { return std::max(0, dreg - 1); }
  // scratch
  DevBuf q_buf, masks, dlv, push_out, push_n, edges, wedges, hits, commit, vcount, popdesc, rbase, counts,
      digest, pop_pos, ids;
  // pinned, device-mapped staging for the per-call transfers.  H2D: staged and
  // copied by k_copy at once.  D2H: deferred to sync(), where one k_copy launch
  // moves every pending small array into pinned memory (callers sync before
  // launching anything that overwrites a pending source).  sync() spins on an
  // event: the host waits microseconds, not an interrupt round trip.
  char *pin = nullptr;
  size_t pin_cap = 0, pin_used = 0;
  struct Pending { void *dst; void *stage; const void *src; size_t n; };
  std::vector<Pending> pend;
  hipEvent_t ev_sync = nullptr, ev_sync2 = nullptr, ev_fork = nullptr, ev_join = nullptr, ev_start = nullptr,
            ev_wu = nullptr, ev_commit = nullptr;  // ev_commit: system fence (commit_range's early wait)
  hipStream_t stream2 = nullptr;  // second queue: canonical cone beside the leader chains
  hipError_t launch_copies(const dr::CopySeg *sg, int k) {
    for (int i0 = 0; i0 < k; i0 += dr::kCopySegs) {
      dr::CopyList L{};
      const int m = std::min(dr::kCopySegs, k - i0);
      uint64_t mx = 1;
      for (int i = 0; i < m; i++) { L.s[i] = sg[i0 + i]; mx = std::max<uint64_t>(mx, sg[i0 + i].n); }
      // bytes per workgroup (DR_COPY_BLK, measurement only: 512-4096 B moved nothing on the
      // per-call loop, profiles/r06/cb_loop_*.json)
      static const uint64_t blk = getenv("DR_COPY_BLK") ? std::max(256, atoi(getenv("DR_COPY_BLK"))) : 4096;
      const unsigned bx = (unsigned)std::min<uint64_t>(256, (mx + blk - 1) / blk);
      hipLaunchKernelGGL(dr::k_copy, dim3(bx, m), dim3(256), 0, stream, L);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  // H2D segments staged while defer_h2d is set: one k_copy launch for all of them
  // (an append stages ~a dozen small arrays) at flush_h2d() or the next sync()
  bool defer_h2d = false;
  std::vector<dr::CopySeg> h2q;
  hipError_t flush_h2d() {
    if (h2q.empty()) return hipSuccess;
    hipError_t e = launch_copies(h2q.data(), (int)h2q.size());
    h2q.clear();
    return e;
  }
  bool async_pending = false;  // an append returned before its copies ran (dr_replay_batch waits)
  // A host wait: poll the event for up to kSpinUs (a per-call query's results are
  // usually back within tens of microseconds, and an interrupt round trip costs more),
  // then block in hipEventSynchronize, so a long wait does not hold a host core.
  // (DR_WAIT_SPIN_US overrides the bound: measurement only)
  static hipError_t wait_event(hipEvent_t ev) {
    static const int kSpinUs = getenv("DR_WAIT_SPIN_US") ? atoi(getenv("DR_WAIT_SPIN_US")) : 200;
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      const hipError_t e = hipEventQuery(ev);
      if (e != hipErrorNotReady) return e;
      if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(kSpinUs)) return hipEventSynchronize(ev);
      std::this_thread::yield();
    }
  }
  // the append whose copies may still be in flight (a HIP error before the next completed
  // wait names it: fail() appends it to the message)
  std::string async_what;
  hipError_t sync() {
    async_pending = false;
    hipError_t e = flush_h2d();
    if (e == hipSuccess && !pend.empty()) {
      std::vector<dr::CopySeg> small;
      for (auto &p : pend) {
        if (p.n >= ((size_t)1 << 22))  // bulk: DMA engine
          e = hipMemcpyAsync(p.stage, p.src, p.n, hipMemcpyDeviceToHost, stream);
        else
          small.push_back(dr::CopySeg{static_cast<const uint8_t *>(p.src), static_cast<uint8_t *>(p.stage), p.n});
        if (e != hipSuccess) break;
      }
      if (e == hipSuccess && !small.empty()) e = launch_copies(small.data(), (int)small.size());
    }
    if (e == hipSuccess) e = hipEventRecord(ev_sync, stream);
    if (e == hipSuccess && stream2 && !s2_detached) e = hipEventRecord(ev_sync2, stream2);
    if (e == hipSuccess) e = wait_event(ev_sync);
    if (e == hipSuccess && stream2 && !s2_detached) e = wait_event(ev_sync2);
    if (e == hipSuccess) {
      for (auto &p : pend) std::memcpy(p.dst, p.stage, p.n);
      async_what.clear();
    }
    pend.clear();
    pin_used = 0;
    return e;
  }
  hipError_t stage(size_t n, void **out) {
    n = (n + 63) & ~(size_t)63;
    if (pin_used + n > pin_cap) {
      hipError_t e = sync();
      if (e != hipSuccess) return e;
      if (n > pin_cap) {
        if (pin) (void)hipHostFree(pin);
        pin = nullptr;
        pin_cap = 0;
        const size_t cap = std::max<size_t>(n, (size_t)8 << 20);
        e = hipHostMalloc((void **)&pin, cap, hipHostMallocMapped);
        if (e != hipSuccess) return e;
        pin_cap = cap;
      }
    }
    *out = pin + pin_used;
    pin_used += n;
    return hipSuccess;
  }
  hipError_t d2h(void *host, const void *dev, size_t n) {
    if (!n) return hipSuccess;
    void *p = nullptr;
    hipError_t e = stage(n, &p);
    if (e == hipSuccess) pend.push_back(Pending{host, p, dev, n});
    return e;
  }
  hipError_t h2d(void *dev, const void *host, size_t n) {
    if (!n) return hipSuccess;
    void *p = nullptr;
    hipError_t e = stage(n, &p);
    if (e != hipSuccess) return e;
    std::memcpy(p, host, n);
    return h2d_staged(dev, p, n);
  }
  // the copy of n bytes the caller already wrote at p (from stage())
  hipError_t h2d_staged(void *dev, void *p, size_t n) {
    if (n >= ((size_t)1 << 22)) return hipMemcpyAsync(dev, p, n, hipMemcpyHostToDevice, stream);
    const dr::CopySeg sg{static_cast<const uint8_t *>(p), static_cast<uint8_t *>(dev), n};
    if (defer_h2d) {
      h2q.push_back(sg);
      return hipSuccess;
    }
    return launch_copies(&sg, 1);
  }
  std::string err;
  int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    err = buf;
    if (code == DR_E_HIP && !async_what.empty()) err += " (pending before this call: " + async_what + ")";
    return code;
  }
  dr::MemoView memo_view() const {
    dr::MemoView m;
    m.U = U.as<u64>();
    m.WU = WU.as<u64>();
    m.SD = SD.as<u64>();
    m.K = K.as<u64>();
    m.dd = memo_dd();
    m.dmax = std::max(1, dreg);
    // exceptions present: the canonical walk and Q_REGULAR sweeps follow G_reg alone
    m.dreg = nexc > 0 ? dreg : 0x7fffffff;
    m.CE = CE.as<u64>();
    return m;
  }
  dr::DagView view() const {
    dr::DagView v;
    v.strong = strong.as<u64>();
    v.present = present.as<u64>();
    v.weak_roff = weak_roff.as<uint32_t>();
    v.far = far.as<u64>();
    v.far_roff = far_roff.as<uint32_t>();
    v.wc_key = wc_key.as<uint32_t>();
    v.wc_rows = wc_rows.as<u64>();
    v.wc_roff = wc_roff.as<uint32_t>();
    v.sdeg = sdeg.as<uint16_t>();
    v.wdeg = wdeg.as<uint16_t>();
    v.lead = lead.as<uint16_t>();
    v.dup_off = ndups ? dup_off.as<uint32_t>() : nullptr;
    v.dup_src = ndups ? dup_src.as<uint16_t>() : nullptr;
    v.slot_rep = ndups ? slot_rep.as<uint8_t>() : nullptr;
    v.sdx = nirr > 0 ? sdx.as<uint32_t>() : nullptr;
    v.n = n;
    v.nrounds = nrounds;
    v.roff = slice_on ? slice.round_offset : 0;
    v.seed_lo = slice_on && slice.seeded_top > 0 ? nrounds - slice.seeded_top : INT_MAX;
    return v;
  }
  bool is_present(int r, int s /*1-based*/) const {
    if (r < 0 || r >= nrounds || s < 1 || s > n) return false;
    return (h_present[(size_t)r * WS + ((s - 1) >> 6)] >> ((s - 1) & 63)) & 1ULL;
  }
  int depth_log2() const {
    int need = next_pow2(std::max(2, dmax_near + 1));
    int cap_words = (65536 - 64) / 8 - 2 * WS;
    int cap = 1;
    while (cap * 2 * WS <= cap_words) cap *= 2;
    int d = std::min(need, cap);
    int l = 0;
    while ((1 << l) < d) l++;
    return l;
  }
  // (+ a second ring for Q_FAST merge sweeps: kring, kernels.hpp sweep_body)
  size_t sweep_lds(int dl, bool fast = false) const { return (size_t)((2 + (fast ? 2 : 1) * (1 << dl)) * WS) * 8 + 64; }
  uint64_t round_deg(int r) const { return hr[r].deg; }
  bool has_ghost(int r) const {
    for (uint16_t s : hr[r].slots)
      if (s == 0) return true;
    return false;
  }
  // a round changed: its summaries are stale, and so is every canonical prefix
  void touch(int r) {
    version++;
    while ((int)sdirty.size() <= r) { sdirty.push_back(1); ndirty++; }
    if (!sdirty[r]) { sdirty[r] = 1; ndirty++; }
    canon_ok = false;
    canon_lo = std::min(canon_lo, r);
    up_lo = std::min(up_lo, r);
    exc_lo = std::min(exc_lo, r);
  }
  // round r's regular window, exceptions and upward irregular edges (upload_suffix)
  void round_exceptions(int r) {
    const HostRound &h = hr[r];
    const int X = reg_max();
    int d = 1, ex = (int)h.far.size(), up = 0, ups = 0;
    for (size_t j = 0; j < h.wc_key.size(); j++) {
      const int delta = (int)(h.wc_key[j] >> 11);
      if (delta <= X) { d = std::max(d, delta); continue; }
      for (int w = 0; w < WS; w++) ex += __builtin_popcountll(h.wc_rows[j * WS + w]);
    }
    uint32_t sx = 0;
    for (uint64_t x : h.irr) {
      const bool upw = (int)((x >> 11) & 0xFFFFFu) >= r;
      upw ? up++ : ex++;
      if (upw && ((x >> 31) & 1u)) ups++;
      sx += (uint32_t)((x >> 31) & 1u);
    }
    h_sdx[r] = sx;
    h_rdreg[r] = d;
    h_rexc[r] = ex;
    h_rup[r] = up;
    h_rups[r] = ups;
  }
  // Flatten rounds [up_lo, nrounds) of the variable-size per-round arrays
  // (slots, weak columns, far edges, weak counts, presence) and copy them to
  // the device after the unchanged prefix.  One staged copy per array.
  hipError_t upload_suffix() {
    const int R = nrounds, lo = up_lo;
    if (lo >= R) { up_lo = R; return hipSuccess; }
    h_slot_off.resize(R + 1);
    h_dup_off.resize(R + 1);
    h_wc_roff.resize(R + 1);
    h_far_roff.resize(R + 1);
    h_irr_roff.resize(R + 1);
    h_weak_roff.resize(R + 1);
    h_ppref.resize(R);
    for (int r = lo; r < R; r++) {
      const HostRound &h = hr[r];
      u64 np = 0;
      if (r >= 1)
        for (uint16_t sl : h.slots) np += sl != 0;
      h_ppref[r] = (r ? h_ppref[r - 1] : (slice_on ? slice.pos_base : 0)) + np;
      h_slot_off[r + 1] = h_slot_off[r] + (uint32_t)h.slots.size();
      h_wc_roff[r + 1] = h_wc_roff[r] + (uint32_t)h.wc_key.size();
      h_far_roff[r + 1] = h_far_roff[r] + (uint32_t)h.far.size();
      h_irr_roff[r + 1] = h_irr_roff[r] + (uint32_t)h.irr.size();
      h_weak_roff[r + 1] = h_weak_roff[r] + (uint32_t)h.nweak;
    }
    {  // the exception counters of rounds [lo, R), the totals updated in place (an append at
       // the top touches only its rounds; the largest regular delta is recomputed whole only
       // when a round that held it changed)
      const int Rold = (int)h_rexc.size();
      bool dreg_drop = false;
      for (int r = lo; r < std::min(Rold, R); r++) {
        nexc -= h_rexc[r];
        nirr_up -= h_rup[r];
        nirr_ups -= h_rups[r];
        dreg_drop |= h_rdreg[r] == dreg;
      }
      h_rdreg.resize(R, 1);
      h_rexc.resize(R, 0);
      h_rup.resize(R, 0);
      h_rups.resize(R, 0);
      h_rbad.resize(R, 0);
      h_sdx.resize(R, 0);
      for (int r = lo; r < R; r++) {
        round_exceptions(r);
        nexc += h_rexc[r];
        nirr_up += h_rup[r];
        nirr_ups += h_rups[r];
      }
      if (dreg_drop) {
        dreg = 1;
        for (int r = 0; r < R; r++) dreg = std::max(dreg, h_rdreg[r]);
      } else {
        for (int r = lo; r < R; r++) dreg = std::max(dreg, h_rdreg[r]);
      }
      nirr_down = nirr - nirr_up;
      if (up_min >= lo) {  // rounds below lo kept their counts
        up_min = INT_MAX;
        for (int r = lo; r < R; r++)
          if (h_rup[r]) {
            up_min = r;
            break;
          }
      }
    }
    const size_t s0 = h_slot_off[lo], s1 = h_slot_off[R], k0 = h_wc_roff[lo], k1 = h_wc_roff[R];
    const size_t f0 = h_far_roff[lo], f1 = h_far_roff[R];
    // repeated ids: the slots after the first of their id, per round (rounds >= 1)
    std::vector<uint8_t> rep;
    std::vector<uint16_t> dsrc;
    rep.reserve(s1 - s0);
    {
      std::vector<u64> seen(WS);
      for (int r = lo; r < R; r++) {
        HostRound &h = hr[r];
        ndups -= h.ndup;
        h.ndup = 0;
        std::fill(seen.begin(), seen.end(), 0ULL);
        for (uint16_t sl : h.slots) {
          bool again = false;
          if (sl != 0 && r >= 1) {
            const u64 bit = 1ULL << ((sl - 1) & 63);
            again = (seen[(sl - 1) >> 6] & bit) != 0;
            seen[(sl - 1) >> 6] |= bit;
          }
          rep.push_back(again ? 1 : 0);
          if (again) {
            dsrc.push_back(sl);
            h.ndup++;
          }
        }
        ndups += h.ndup;
        h_dup_off[r + 1] = h_dup_off[r] + h.ndup;
      }
    }
    const size_t d0 = h_dup_off[lo], d1 = h_dup_off[R];
    hipError_t e;
    if ((e = slot_rep.grow(s1 + 64, s0, stream)) != hipSuccess) return e;
    if ((e = dup_src.grow(d1 * 2 + 64, d0 * 2, stream)) != hipSuccess) return e;
    if ((e = dup_off.grow(((size_t)R + 1) * 4 + 64, ((size_t)lo + 1) * 4, stream)) != hipSuccess) return e;
    if ((e = slot_src.grow(s1 * 2 + 64, s0 * 2, stream)) != hipSuccess) return e;
    if ((e = wc_key.grow(k1 * 4 + 64, k0 * 4, stream)) != hipSuccess) return e;
    if ((e = wc_rows.grow(k1 * WS * 8 + 64, k0 * WS * 8, stream)) != hipSuccess) return e;
    if ((e = far.grow(f1 * 8 + 64, f0 * 8, stream)) != hipSuccess) return e;
    const size_t i0 = h_irr_roff[lo], i1 = h_irr_roff[R];
    if ((e = irr.grow(i1 * 8 + 64, i0 * 8, stream)) != hipSuccess) return e;
    if ((e = irr_roff.grow(((size_t)R + 1) * 4 + 64, ((size_t)lo + 1) * 4, stream)) != hipSuccess) return e;
    std::vector<uint16_t> sl;
    sl.reserve(s1 - s0);
    std::vector<uint32_t> kk;
    kk.reserve(k1 - k0);
    std::vector<u64> rows, ff, ii;
    rows.reserve((k1 - k0) * WS);
    ff.reserve(f1 - f0);
    ii.reserve(i1 - i0);
    for (int r = lo; r < R; r++) {
      const HostRound &h = hr[r];
      sl.insert(sl.end(), h.slots.begin(), h.slots.end());
      kk.insert(kk.end(), h.wc_key.begin(), h.wc_key.end());
      rows.insert(rows.end(), h.wc_rows.begin(), h.wc_rows.end());
      ff.insert(ff.end(), h.far.begin(), h.far.end());
      ii.insert(ii.end(), h.irr.begin(), h.irr.end());
    }
    const size_t nr = (size_t)(R - lo);
    if ((e = h2d(slot_src.as<uint16_t>() + s0, sl.data(), sl.size() * 2)) != hipSuccess) return e;
    if ((e = h2d(slot_rep.as<uint8_t>() + s0, rep.data(), rep.size())) != hipSuccess) return e;
    if (d1 > d0 && (e = h2d(dup_src.as<uint16_t>() + d0, dsrc.data(), dsrc.size() * 2)) != hipSuccess) return e;
    if ((e = h2d(dup_off.as<uint32_t>() + lo, &h_dup_off[lo], (nr + 1) * 4)) != hipSuccess) return e;
    if ((e = h2d(wc_key.as<uint32_t>() + k0, kk.data(), kk.size() * 4)) != hipSuccess) return e;
    if ((e = h2d(wc_rows.as<u64>() + k0 * WS, rows.data(), rows.size() * 8)) != hipSuccess) return e;
    if ((e = h2d(far.as<u64>() + f0, ff.data(), ff.size() * 8)) != hipSuccess) return e;
    if (i1 > i0 && (e = h2d(irr.as<u64>() + i0, ii.data(), ii.size() * 8)) != hipSuccess) return e;
    if ((e = h2d(irr_roff.as<uint32_t>() + lo + 1, &h_irr_roff[lo + 1], nr * 4)) != hipSuccess) return e;
    if ((e = h2d(slot_off.as<uint32_t>() + lo + 1, &h_slot_off[lo + 1], nr * 4)) != hipSuccess) return e;
    if ((e = h2d(ppref.as<u64>() + lo, &h_ppref[lo], nr * 8)) != hipSuccess) return e;
    if ((e = h2d(wc_roff.as<uint32_t>() + lo + 1, &h_wc_roff[lo + 1], nr * 4)) != hipSuccess) return e;
    if ((e = h2d(far_roff.as<uint32_t>() + lo + 1, &h_far_roff[lo + 1], nr * 4)) != hipSuccess) return e;
    if ((e = h2d(weak_roff.as<uint32_t>() + lo + 1, &h_weak_roff[lo + 1], nr * 4)) != hipSuccess) return e;
    if ((e = h2d(present.as<u64>() + (size_t)lo * WS, &h_present[(size_t)lo * WS], nr * WS * 8)) != hipSuccess)
      return e;
    if (nirr > 0) {  // the rounds from lo, or every round when the device copy is not current
      if ((e = sdx.ensure(((size_t)max_rounds + 1) * 4)) != hipSuccess) return e;
      const int x0 = sdx_valid ? lo : 0;
      if ((e = h2d(sdx.as<uint32_t>() + x0, h_sdx.data() + x0, (size_t)(R - x0) * 4)) != hipSuccess) return e;
      sdx_valid = true;
    } else {
      sdx_valid = false;
    }
    up_lo = R;
    return hipSuccess;
  }
};

#define HIPCHK(ctx, call)                                                                   \
  do {                                                                                      \
    hipError_t e_ = (call);                                                                 \
    if (e_ != hipSuccess)                                                                   \
      return (ctx)->fail(DR_E_HIP, "%s failed: %s (%s:%d)", #call, hipGetErrorString(e_),   \
                         __FILE__, __LINE__);                                               \
  } while (0)

namespace {

// Scope in which dr_ctx::h2d stages instead of launching; the staged copies go
// out in one launch at the scope's sync() (or here, on an early error return).
struct DeferH2D {
  dr_ctx *c;
  explicit DeferH2D(dr_ctx *cc) : c(cc) { c->defer_h2d = true; }
  ~DeferH2D() {
    c->defer_h2d = false;
    (void)c->flush_h2d();
  }
};

template <int WS>
constexpr int block_for() {
  return WS == 1 ? 64 : WS == 2 ? 128 : WS == 4 ? 256 : WS == 8 ? 512 : 1024;
}
// k_summary_commit: 512 threads at WS 16 (two workgroups per CU overlap each
// other's per-round barriers: 274 vs 291 us on C4, profiles/r01/v4_tune.txt)
template <int WS>
constexpr int summary_block() {
  return WS == 16 ? 512 : block_for<WS>();
}
// sweeps keep more state live across a round: cap the block at 512 threads
// (256 VGPRs per lane) so nothing spills
template <int WS>
constexpr int sweep_block() {
  return WS == 1 ? 64 : WS == 2 ? 128 : WS == 4 ? 256 : 512;
}
// many independent sweeps (delivery pops, path/reach batches): at WS = 16 half
// the block lets every C4 pop be resident at once (4 waves/SIMD at 107 VGPRs);
// the saturating row reads keep the row passes short.  Chains and the single
// canonical sweep keep the wide block.  C4: pops 96 -> 75 us.
template <int WS, int MODE>
constexpr int sweep_block_m() {
  // merging pop sweeps at n = 1024: 3 waves, so every query of a C4 replay is
  // resident at once at 3 waves per SIMD (168 VGPRs: the emission fits unspilled)
  if constexpr ((MODE & dr::SW_MERGE) && WS == 16) return 192;
  return (MODE & dr::SW_CHAIN) ? sweep_block<WS>() : WS == 16 ? 256 : sweep_block<WS>();
}

// ---- kernel launch dispatch over the row stride ----
constexpr int kSplitNT = 512, kSplitP3 = 2, kSplitAuto = 4;
// A short wave range (fewer waves than CUs): KS workgroups per wave
// (k_commit_split), each deciding S_1, S_2 in full and a share of S_3.  Returns
// 1 when the range is long enough for one workgroup per wave (the caller
// launches k_commit), else a hipError_t; *split = KS.
template <int WS>
int launch_commit_split_t(dr_ctx *c, int w0, int nw, uint8_t *cm, int32_t *vc, int *split) {
  *split = 0;
  if (WS < 2 || !c->commit_split || (c->commit_split == 2 && nw > kSplitAuto)) return 1;
  if (c->split_cap == 0) {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->dev) != hipSuccess) return 1;
    c->split_cap = std::max(1, ncu);
  }
  if (nw >= c->split_cap) return 1;
  using G = dr::Geo<WS, kSplitNT>;
  const int RS = G::RPP * kSplitP3;  // rows of round 4 per workgroup
  const int KS = (c->n + RS - 1) / RS;
  if (KS < 2) return 1;
  if ((size_t)nw > c->split_nw) {  // counters start at zero; the kernel leaves them at zero
    hipError_t e;
    if ((e = c->split_ctl.ensure((size_t)nw * 8 + 64)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(c->split_ctl.p, 0, (size_t)nw * 8 + 64, c->stream)) != hipSuccess) return e;
    c->split_nw = (size_t)nw;
  }
  const int groups = (nw + 7) / 8;
  hipLaunchKernelGGL((dr::k_commit_split<WS, kSplitNT, kSplitP3>), dim3(groups * 8 * KS), dim3(kSplitNT), 0,
                     c->stream, c->view(), w0, nw, KS, 2 * c->f + 1, c->split_ctl.as<unsigned long long>(), cm, vc);
  *split = KS;
  return hipGetLastError();
}

template <int WS>
hipError_t launch_commit_t(dr_ctx *c, int w0, int nw, uint8_t *cm, int32_t *vc) {
  constexpr int NT = block_for<WS>();
  c->last_split = 0;
  const int rc = launch_commit_split_t<WS>(c, w0, nw, cm, vc, &c->last_split);
  if (rc != 1) return (hipError_t)rc;
  hipLaunchKernelGGL((dr::k_commit<WS, NT>), dim3(nw), dim3(NT), 0, c->stream, c->view(), w0, nw,
                     2 * c->f + 1, cm, vc);
  return hipGetLastError();
}
hipError_t launch_commit(dr_ctx *c, int w0, int nw, uint8_t *cm, int32_t *vc) {
  switch (c->WS) {
    case 1: return launch_commit_t<1>(c, w0, nw, cm, vc);
    case 2: return launch_commit_t<2>(c, w0, nw, cm, vc);
    case 4: return launch_commit_t<4>(c, w0, nw, cm, vc);
    case 8: return launch_commit_t<8>(c, w0, nw, cm, vc);
    case 16: return launch_commit_t<16>(c, w0, nw, cm, vc);
    case 32: return launch_commit_t<32>(c, w0, nw, cm, vc);
  }
  return hipErrorInvalidValue;
}

struct SweepArgs {  // (every field initialised: a launch never reads a stale pointer)
  const dr::SweepQuery *q = nullptr;
  int nq = 0, seq = 0;
  u64 *masks = nullptr, *dlv = nullptr;
  int32_t *push_out = nullptr, *push_n = nullptr;
  u64 *edges = nullptr, *wedges = nullptr;
  uint8_t *hits = nullptr;
  int32_t *stops = nullptr;
  u64 *stats = nullptr;
  const int *nq_dev = nullptr;  // planned replay: query count on the device, nq = grid upper bound
  uint32_t *rcnt = nullptr;     // planned delivery: per-mask-row vertex counts for the emission
  dr::PopMark pm{};             // REF planned replay: live delivery queries / chain stamps
  dr::CanonEmit ce{};           // merge sweeps: the canonical re-emission's workgroups (first in the grid)
  dr::PopPlanArgs pp{};         // merge sweeps: the pop plan's workgroup (last in the grid; pp.active)
  bool fast = false;            // some query has Q_FAST: the second ring in LDS
  dr::OwnEmit oe{};             // merge sweeps: each query's own-round emission after its sweep
};
// The REF replay's leader chains inside the single-stream launches: the chain plan in the
// weak-union launch (k_wu_plan), the chain sweeps beside the canonical walk (k_canon_chains)
struct ChainFuse {
  dr::ChainPlanArgs pa;
  dr::ChainArgs xa;
  bool plan_in_kcand = false;  // the weak unions rode in the row pass: the plan rides in k_kcand_plan
  bool emit_in_sweep = false;  // the canonical re-emission rides in the delivery sweeps' launch
  dr::SpecPrefix sp{};         // the speculative G, E prefixes beside the canonical walk (last workgroup)
};

// Raise a kernel's dynamic-LDS limit once per (device, size it has not seen yet):
// a host call per launch otherwise, and the replay launches sweeps every step.
constexpr int kLdsDevs = 16;
inline hipError_t lds_limit(const void *fn, std::atomic<int> *seen, int dev, size_t lds) {
  std::atomic<int> *sl = dev >= 0 && dev < kLdsDevs ? &seen[dev] : nullptr;
  if (sl && (int)lds <= sl->load(std::memory_order_relaxed)) return hipSuccess;
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e == hipSuccess && sl) {
    int cur = sl->load(std::memory_order_relaxed);
    while ((int)lds > cur && !sl->compare_exchange_weak(cur, (int)lds)) {
    }
  }
  return e;
}

template <int WS, int MODE>
hipError_t launch_sweep_m(dr_ctx *c, const SweepArgs &a) {
  constexpr int NT = sweep_block_m<WS, MODE>();
  const int dl = c->depth_log2();
  const size_t lds = c->sweep_lds(dl, a.fast);
  static std::atomic<int> seen[kLdsDevs] = {};
  hipError_t e = lds_limit((const void *)dr::k_sweep<WS, NT, MODE>, seen, c->dev, lds);
  if (e != hipSuccess) return e;
  const int ne = (MODE & dr::SW_MERGE) ? a.ce.nblk : 0;  // (a multiple of 8, CanonEmit::xcd)
  const int np = (MODE & dr::SW_MERGE) && a.pp.active ? 1 : 0;
  const int grid = (a.seq ? 1 : a.nq) + ne + np;
  dr::CanonEmit ce = a.ce;
  ce.nblk = ne;
  dr::PopPlanArgs pp = a.pp;
  pp.active = np;
  hipLaunchKernelGGL((dr::k_sweep<WS, NT, MODE>), dim3(grid), dim3(NT), lds, c->stream,
                     c->view(), c->memo_view(), a.q, a.nq, a.seq, dl, a.masks, a.dlv, a.push_out,
                     a.push_n, a.edges, a.wedges, a.hits, a.stops, a.stats, a.nq_dev, a.rcnt, a.pm, ce, pp,
                     (MODE & dr::SW_MERGE) ? a.oe : dr::OwnEmit{});
  return hipGetLastError();
}
template <int WS>
hipError_t launch_sweep_t(dr_ctx *c, const SweepArgs &a, int mode) {
  switch (mode) {
    case 0: return launch_sweep_m<WS, 0>(c, a);
    case dr::SW_WEAK: return launch_sweep_m<WS, dr::SW_WEAK>(c, a);
    case dr::SW_CHAIN: return launch_sweep_m<WS, dr::SW_CHAIN>(c, a);
    case dr::SW_WEAK | dr::SW_PRUNE: return launch_sweep_m<WS, dr::SW_WEAK | dr::SW_PRUNE>(c, a);
    case dr::SW_WEAK | dr::SW_MERGE: return launch_sweep_m<WS, dr::SW_WEAK | dr::SW_MERGE>(c, a);
    case dr::SW_WEAK | dr::SW_MERGE | dr::SW_FAST:
      return launch_sweep_m<WS, dr::SW_WEAK | dr::SW_MERGE | dr::SW_FAST>(c, a);
  }
  return hipErrorInvalidValue;
}
// the compile-time mode of a query (every query of one launch shares it)
int sweep_mode(const dr::SweepQuery &q) {
  int m = 0;
  if (!(q.flags & dr::Q_STRONG_ONLY)) m |= dr::SW_WEAK;
  if (q.flags & dr::Q_CHAIN) m |= dr::SW_CHAIN;
  if (q.flags & dr::Q_PRUNE) m |= dr::SW_PRUNE;
  if (q.flags & dr::Q_MERGE) m |= dr::SW_MERGE;
  if ((q.flags & dr::Q_FAST) && (m & dr::SW_MERGE) && (m & dr::SW_WEAK)) m |= dr::SW_FAST;
  return m;
}
// The planned replay's leader chains (a device-counted batch): n <= 256 on one
// wavefront per chain with every round in registers (k_chain_reg), else k_sweep.
template <int WS, int PF>
hipError_t launch_chain_reg(dr_ctx *c, const SweepArgs &a) {
  hipLaunchKernelGGL((dr::k_chain_reg<WS, PF>), dim3((a.nq + 3) / 4), dim3(256), 0, c->stream, c->view(), a.q,
                     a.nq_dev, a.push_out, a.push_n, a.edges, a.wedges, a.hits, a.stops, a.pm);
  return hipGetLastError();
}
hipError_t launch_sweep(dr_ctx *c, const SweepArgs &a, int mode);
hipError_t launch_chains(dr_ctx *c, const SweepArgs &a) {
  if (a.nq <= 0) return hipSuccess;
  if (a.nq_dev && !a.seq && c->chain_reg) {
    switch (c->WS) {
      case 1: return launch_chain_reg<1, 4>(c, a);
      case 2: return launch_chain_reg<2, 4>(c, a);
      case 4: return launch_chain_reg<4, 3>(c, a);
    }
  }
  return launch_sweep(c, a, dr::SW_CHAIN);
}
hipError_t launch_sweep(dr_ctx *c, const SweepArgs &a, int mode) {
  // (with no query, the launch still runs the canonical re-emission and pop plan riding in it)
  if (a.nq <= 0 && !((mode & dr::SW_MERGE) && (a.ce.nblk > 0 || a.pp.active))) return hipSuccess;
  switch (c->WS) {
    case 1: return launch_sweep_t<1>(c, a, mode);
    case 2: return launch_sweep_t<2>(c, a, mode);
    case 4: return launch_sweep_t<4>(c, a, mode);
    case 8: return launch_sweep_t<8>(c, a, mode);
    case 16: return launch_sweep_t<16>(c, a, mode);
    case 32: return launch_sweep_t<32>(c, a, mode);
  }
  return hipErrorInvalidValue;
}

constexpr int kEmitRPB = 4;  // rounds per emit workgroup: one per wave
// workgroups of the delivery sweeps' launch that re-emit the canonical rounds (C4: a
// top segment of a few dozen rounds, a wave each)
constexpr int kCanonEmitBlocks = 16;

// Planned mode (plan != nullptr, device-planned replay): the count pass runs
// ndesc = an upper bound of workgroups and reads the true count from plan[0];
// the digest pass strides a fixed grid over the work items item_pref describes.
// pd == nullptr: one segment, described by d1 (passed by value).
template <int WS>
hipError_t launch_emit_t(dr_ctx *c, int ndesc, int span, const dr::PopDesc *pd, uint32_t *rbase, u64 *cnt, u64 *dg,
                         u64 *round_out, const int64_t *pos, int32_t *ids, int64_t cap, bool count_phase,
                         const int *plan, const int64_t *item_pref, const dr::PopDesc &d1, const uint32_t *rcnt,
                         const int *skip) {
  if (count_phase) {
    hipLaunchKernelGGL((dr::k_emit_count<WS, 256>), dim3(ndesc), dim3(256), 0, c->stream, c->view(), pd,
                       c->masks.as<u64>(), c->K.as<u64>(), rbase, cnt, plan);
  } else if (plan) {
    hipLaunchKernelGGL((dr::k_emit_ids<WS, 256, kEmitRPB>), dim3(2048), dim3(256), 0, c->stream, c->view(),
                       c->slot_off.as<uint32_t>(), c->slot_src.as<uint16_t>(), pd, d1, c->masks.as<u64>(),
                       c->K.as<u64>(), rbase, pos, dg, round_out, ids, cap, item_pref, plan, rcnt, cnt,
                       (const int *)nullptr);
  } else {
    const int bx = std::max(1, (span + kEmitRPB - 1) / kEmitRPB);
    hipLaunchKernelGGL((dr::k_emit_ids<WS, 256, kEmitRPB>), dim3(bx, ndesc), dim3(256), 0, c->stream, c->view(),
                       c->slot_off.as<uint32_t>(), c->slot_src.as<uint16_t>(), pd, d1, c->masks.as<u64>(),
                       c->K.as<u64>(), rbase, pos, dg, round_out, ids, cap, (const int64_t *)nullptr,
                       (const int *)nullptr, (const uint32_t *)nullptr, (u64 *)nullptr, skip);
  }
  return hipGetLastError();
}
hipError_t launch_emit(dr_ctx *c, int ndesc, int span, const dr::PopDesc *pd, uint32_t *rbase, u64 *cnt, u64 *dg,
                       u64 *round_out, const int64_t *pos, int32_t *ids, int64_t cap, bool count_phase,
                       const int *plan = nullptr, const int64_t *item_pref = nullptr,
                       const dr::PopDesc &d1 = dr::PopDesc{}, const uint32_t *rcnt = nullptr,
                       const int *skip = nullptr) {
  if (ndesc <= 0) return hipSuccess;
  switch (c->WS) {
    case 1: return launch_emit_t<1>(c, ndesc, span, pd, rbase, cnt, dg, round_out, pos, ids, cap, count_phase, plan, item_pref, d1, rcnt, skip);
    case 2: return launch_emit_t<2>(c, ndesc, span, pd, rbase, cnt, dg, round_out, pos, ids, cap, count_phase, plan, item_pref, d1, rcnt, skip);
    case 4: return launch_emit_t<4>(c, ndesc, span, pd, rbase, cnt, dg, round_out, pos, ids, cap, count_phase, plan, item_pref, d1, rcnt, skip);
    case 8: return launch_emit_t<8>(c, ndesc, span, pd, rbase, cnt, dg, round_out, pos, ids, cap, count_phase, plan, item_pref, d1, rcnt, skip);
    case 16: return launch_emit_t<16>(c, ndesc, span, pd, rbase, cnt, dg, round_out, pos, ids, cap, count_phase, plan, item_pref, d1, rcnt, skip);
    case 32: return launch_emit_t<32>(c, ndesc, span, pd, rbase, cnt, dg, round_out, pos, ids, cap, count_phase, plan, item_pref, d1, rcnt, skip);
  }
  return hipErrorInvalidValue;
}

// k_summary_commit geometry (block, chunks in flight per thread, software
// pipelining); dr_profile_kernel's variants time the alternatives.
// rounds (waves) per k_weak_union workgroup: four, fewer when a deep window's
// per-wave LDS slice (dd x WS words) would take the workgroup past 64 KiB
inline int weak_union_waves(int dd, int WS, int cap = 4) {
  const size_t per = (size_t)std::max(dd, 1) * WS * 8;
  return (int)std::max<size_t>(1, std::min<size_t>(cap, 65536 / per));
}
// wu: the weak unions and speculative digests ride in the same launch (dr::WUArgs)
template <int WS, int NT, int GRP, bool PIPE>
hipError_t launch_sc(dr_ctx *c, int T, int nwc, uint8_t *cm, int32_t *vc, bool wu = false) {
  dr::WUArgs wa{};
  const int nsum = (T + 3) / 4;
  int grid = nsum;
  size_t lds = 0;
  if (wu) {
    wa.nsum = nsum;
    wa.dd = c->memo_dd();
    wa.nwv = weak_union_waves(wa.dd, WS, NT / 64);
    wa.WU = c->WU.as<u64>();
    wa.ppref = c->ppref.as<u64>();
    wa.slot_off = c->slot_off.as<uint32_t>();
    wa.slot_src = c->slot_src.as<uint16_t>();
    wa.RG = c->RG.as<u64>();
    grid += (T + wa.nwv - 1) / wa.nwv;
    lds = (size_t)wa.nwv * std::max(wa.dd, 1) * WS * 8;  // <= 64 KiB: no attribute needed
  }
  hipLaunchKernelGGL((dr::k_summary_commit<WS, NT, GRP, PIPE>), dim3(grid), dim3(NT), lds, c->stream, c->view(), T,
                     nwc, 2 * c->f + 1, c->U.as<u64>(), c->SD.as<u64>(), cm, vc, wa);
  return hipGetLastError();
}
// WS = 16 (n = 1024): 1024 threads, 2 chunks per thread per group: 80.8 us
// for C4's 524.8 MB (6.5 TB/s), faster than a bare blocked streaming read of
// the same rows (profiles/r02/v29_tune.txt: 82.5 us)
// A short DAG (fewer waves than CUs: a wave-split rank's slice, 134 waves at N = 8) leaves
// most CUs idle, and a CU's bandwidth is its bytes in flight over the latency: each thread
// then keeps all 8 of its chunks of a round in flight (GRP 8).
template <int WS>
hipError_t launch_sc_shipped(dr_ctx *c, int T, int nwc, uint8_t *cm, int32_t *vc, bool wu = false) {
  if constexpr (WS == 16) {
    if (c->cu_count <= 0) {
      int cus = 0;
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->dev) == hipSuccess) c->cu_count = cus;
    }
    if ((T + 3) / 4 < c->cu_count) return launch_sc<WS, 1024, 8, false>(c, T, nwc, cm, vc, wu);
    return launch_sc<WS, 1024, 2, false>(c, T, nwc, cm, vc, wu);
  }
  return launch_sc<WS, summary_block<WS>(), 8, false>(c, T, nwc, cm, vc, wu);
}

// rows + commit decisions (U, SD); the weak-edge unions (WU) come from the
// weak-column keys alone: with wu, as extra workgroups after the row workgroups of the
// same launch (they take the CUs the pass's last workgroups leave idle), else
// launch_weak_union after it.  (Inside the row pass's workgroups, one wave per round
// after the rows, they lengthened the pass by as much as the separate launch took:
// C4 89 -> 105 us, profiles/r05/v7_*.)
template <int WS>
hipError_t launch_summary_t(dr_ctx *c, int T, int nwc, uint8_t *cm, int32_t *vc, bool wu) {
  hipError_t e = launch_sc_shipped<WS>(c, T, nwc, cm, vc, wu);
  if (e == hipSuccess) e = c->rec(7);  // ms_summary times k_summary_commit alone (the roofline kernel)
  return e;
}
// every round's WU, and its speculative canonical digest into RG (k_canon's spec check)
// one LDS limit per k_weak_union instantiation (both launch sites share it)
template <int WS>
hipError_t weak_union_lds(const dr_ctx *c, size_t lds) {
  static std::atomic<int> seen[kLdsDevs] = {};
  return lds_limit((const void *)dr::k_weak_union<WS>, seen, c->dev, lds);
}
template <int WS>
hipError_t launch_weak_union_t(dr_ctx *c, int T, hipStream_t st) {
  const int dd = c->memo_dd(), nwv = weak_union_waves(dd, WS);
  const size_t lds = (size_t)nwv * std::max(dd, 1) * WS * 8;
  hipError_t e = weak_union_lds<WS>(c, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((dr::k_weak_union<WS>), dim3((T + nwv - 1) / nwv), dim3(64 * nwv), lds, st, c->view(), T, 0, dd,
                     c->WU.as<u64>(), (const int32_t *)nullptr, c->ppref.as<u64>(), c->slot_off.as<uint32_t>(),
                     c->slot_src.as<uint16_t>(), c->RG.as<u64>());
  return hipGetLastError();
}
// ... and with cf (the REF replay): the chain plan as the launch's last workgroup
// (k_wu_plan; a deep window's smaller workgroups take a separate k_plan_chains)
template <int WS>
hipError_t launch_wu_plan_t(dr_ctx *c, int T, const ChainFuse &cf) {
  const int dd = c->memo_dd(), nwv = weak_union_waves(dd, WS);
  if (nwv != 4) {
    hipError_t e = launch_weak_union_t<WS>(c, T, c->stream);
    if (e != hipSuccess) return e;
    const dr::ChainPlanArgs &pa = cf.pa;
    hipLaunchKernelGGL((dr::k_plan_chains<1024>), dim3(1), dim3(1024), 0, c->stream, pa.commit, pa.lead, pa.nw,
                       pa.persistent, pa.qflags, pa.task_wave, pa.task_q, pa.cq, pa.plan);
    return hipGetLastError();
  }
  const size_t lds = (size_t)4 * std::max(dd, 1) * WS * 8;
  static std::atomic<int> seen[kLdsDevs] = {};
  hipError_t e = lds_limit((const void *)dr::k_wu_plan<WS>, seen, c->dev, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((dr::k_wu_plan<WS>), dim3((T + 3) / 4 + 1), dim3(256), lds, c->stream, c->view(), T, dd,
                     c->WU.as<u64>(), c->ppref.as<u64>(), c->slot_off.as<uint32_t>(), c->slot_src.as<uint16_t>(),
                     c->RG.as<u64>(), cf.pa);
  return hipGetLastError();
}
hipError_t launch_weak_union(dr_ctx *c, int T, hipStream_t st, const ChainFuse *cf = nullptr) {
  switch (c->WS) {
#define DR_WU(W) \
  case W: return cf ? launch_wu_plan_t<W>(c, T, *cf) : launch_weak_union_t<W>(c, T, st);
    DR_WU(1) DR_WU(2) DR_WU(4) DR_WU(8) DR_WU(16) DR_WU(32)
#undef DR_WU
  }
  return hipErrorInvalidValue;
}

// incremental summaries of the listed rounds (device list of nr rounds)
template <int WS>
hipError_t launch_round_summary_t(dr_ctx *c, const dr::RoundList &rl) {
  constexpr int NT = block_for<WS>() < 256 ? 256 : block_for<WS>();
  const dr::MemoView mv = c->memo_view();
  // the weak unions in the same launch: nwv rounds per workgroup within 64 KB of LDS
  const int nwv = mv.dd > 0 ? weak_union_waves(mv.dd, WS, NT / 64) : 1;
  const int nwu = mv.dd > 0 ? (rl.n + nwv - 1) / nwv : 0;
  const size_t lds = mv.dd > 0 ? (size_t)nwv * mv.dd * WS * 8 : 0;
  hipLaunchKernelGGL((dr::k_round_summary<WS, NT>), dim3(rl.n + nwu), dim3(NT), lds, c->stream, c->view(), rl,
                     c->U.as<u64>(), c->SD.as<u64>(), mv.dd, nwv, c->WU.as<u64>());
  return hipGetLastError();
}
hipError_t launch_round_summary(dr_ctx *c, const dr::RoundList &rounds) {
  switch (c->WS) {
    case 1: return launch_round_summary_t<1>(c, rounds);
    case 2: return launch_round_summary_t<2>(c, rounds);
    case 4: return launch_round_summary_t<4>(c, rounds);
    case 8: return launch_round_summary_t<8>(c, rounds);
    case 16: return launch_round_summary_t<16>(c, rounds);
    case 32: return launch_round_summary_t<32>(c, rounds);
  }
  return hipErrorInvalidValue;
}

// canonical cone: K^cand per round, then the exact cone at the bad rounds;
// spec (a full cone, lo == 1): the round summaries carry every round's
// speculative canonical digest (k_weak_union), k_canon sets *rlo to the lowest
// round where it fails, and the canonical emission re-emits from there.
template <int WS>
hipError_t launch_canon_cone_t(dr_ctx *c, int T, int lo, bool spec, const ChainFuse *cf = nullptr) {
  const dr::MemoView mv = c->memo_view();
  if (cf && cf->plan_in_kcand)
    hipLaunchKernelGGL((dr::k_kcand_plan<WS>), dim3((T + 1 + 3) / 4 + 1), dim3(256), 0, c->stream, c->view(), mv, T,
                       c->K.as<u64>(), c->good.as<uint8_t>(), c->CE.as<u64>(), c->RD.as<u64>(), c->rlo.as<int>(),
                       spec ? T + 1 : lo, spec ? c->ppref.as<u64>() : nullptr, c->Cc.as<u64>(),
                       c->crbase.as<uint32_t>(), cf->pa);
  else
    hipLaunchKernelGGL((dr::k_kcand<WS>), dim3((T + 1 + 3) / 4), dim3(256), 0, c->stream, c->view(), mv, T,
                       c->K.as<u64>(), c->good.as<uint8_t>(), c->CE.as<u64>(), c->RD.as<u64>(), c->rlo.as<int>(),
                       spec ? T + 1 : lo, spec ? c->ppref.as<u64>() : nullptr, c->Cc.as<u64>(),
                       c->crbase.as<uint32_t>());
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int dl = c->depth_log2();
  const size_t lds = c->sweep_lds(dl);
  constexpr int NTS = sweep_block<WS>();
  if (cf) {  // workgroup 0 walks the canonical cone, the others sweep the leader chains
    const dr::CanonArgs ca{T, dl, c->K.as<u64>(), c->good.as<uint8_t>(), c->CE.as<u64>(), c->nseg.as<int32_t>(),
                           c->RD.as<u64>(), c->Cc.as<u64>(), c->crbase.as<uint32_t>(),
                           spec ? c->ppref.as<u64>() : nullptr, c->rlo.as<int>()};
    const int nq = std::max(cf->pa.nw, 1);
    bool creg = false;
    if constexpr (WS == 4) creg = c->chain_reg != 0;
    if (creg) {
      if constexpr (WS == 4) {
        static std::atomic<int> seen_r[kLdsDevs] = {};
        e = lds_limit((const void *)dr::k_canon_chains<WS, NTS, true>, seen_r, c->dev, lds);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL((dr::k_canon_chains<WS, NTS, true>), dim3(1 + (nq + 3) / 4 + (cf->sp.on ? 1 : 0)),
                           dim3(NTS), lds, c->stream, c->view(), mv, ca, cf->xa, cf->sp);
      }
    } else {
      static std::atomic<int> seen_s[kLdsDevs] = {};
      e = lds_limit((const void *)dr::k_canon_chains<WS, NTS, false>, seen_s, c->dev, lds);
      if (e != hipSuccess) return e;
      hipLaunchKernelGGL((dr::k_canon_chains<WS, NTS, false>), dim3(1 + nq + (cf->sp.on ? 1 : 0)), dim3(NTS), lds,
                         c->stream, c->view(), mv, ca, cf->xa, cf->sp);
    }
    e = hipGetLastError();
    if (e != hipSuccess || lo <= 1) return e;
  } else {
    static std::atomic<int> seen[kLdsDevs] = {};
    e = lds_limit((const void *)dr::k_canon<WS, NTS>, seen, c->dev, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((dr::k_canon<WS, NTS>), dim3(1), dim3(NTS), lds, c->stream, c->view(), mv, T, dl,
                       c->K.as<u64>(), c->good.as<uint8_t>(), c->CE.as<u64>(), c->nseg.as<int32_t>(), c->RD.as<u64>(),
                       c->Cc.as<u64>(), c->crbase.as<uint32_t>(), spec ? c->ppref.as<u64>() : nullptr,
                       c->rlo.as<int>());
  }
  e = hipGetLastError();
  if (e != hipSuccess || lo <= 1) return e;
  hipLaunchKernelGGL((dr::k_canon_diff<WS>), dim3((lo - 1 + 3) / 4), dim3(256), 0, c->stream, c->view(), lo,
                     c->K.as<u64>(), c->Kprev.as<u64>(), c->rlo.as<int>());
  return hipGetLastError();
}
hipError_t launch_canon_cone(dr_ctx *c, int T, int lo, bool spec, const ChainFuse *cf = nullptr) {
  switch (c->WS) {
    case 1: return launch_canon_cone_t<1>(c, T, lo, spec, cf);
    case 2: return launch_canon_cone_t<2>(c, T, lo, spec, cf);
    case 4: return launch_canon_cone_t<4>(c, T, lo, spec, cf);
    case 8: return launch_canon_cone_t<8>(c, T, lo, spec, cf);
    case 16: return launch_canon_cone_t<16>(c, T, lo, spec, cf);
    case 32: return launch_canon_cone_t<32>(c, T, lo, spec, cf);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_summary(dr_ctx *c, int T, int nwc, uint8_t *cm, int32_t *vc, bool wu = false) {
  switch (c->WS) {
    case 1: return launch_summary_t<1>(c, T, nwc, cm, vc, wu);
    case 2: return launch_summary_t<2>(c, T, nwc, cm, vc, wu);
    case 4: return launch_summary_t<4>(c, T, nwc, cm, vc, wu);
    case 8: return launch_summary_t<8>(c, T, nwc, cm, vc, wu);
    case 16: return launch_summary_t<16>(c, T, nwc, cm, vc, wu);
    case 32: return launch_summary_t<32>(c, T, nwc, cm, vc, wu);
  }
  return hipErrorInvalidValue;
}

int set_device(dr_ctx *c) {
  hipError_t e = hipSetDevice(c->dev);
  if (e != hipSuccess) return c->fail(DR_E_HIP, "hipSetDevice(%d): %s", c->dev, hipGetErrorString(e));
  return DR_OK;
}

template <class T>
int h2d(dr_ctx *c, DevBuf &b, const std::vector<T> &v) {
  HIPCHK(c, b.ensure(std::max<size_t>(v.size(), 1) * sizeof(T)));
  if (!v.empty())
    HIPCHK(c, hipMemcpyAsync(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, c->stream));
  return DR_OK;
}

}  // namespace

// ===========================================================================
// lifecycle
// ===========================================================================
extern "C" int dr_abi_version(void) { return DR_ABI_VERSION; }

// DR_CREATE_SHARED_STREAM: one HIP stream per device shared by every such context
// (reference-counted, created with the first): a batch of thousands of small contexts
// (C5) otherwise holds thousands of streams, and a device-wide synchronize walks each
namespace {
struct SharedStream {
  hipStream_t s = nullptr;
  int refs = 0;
};
std::mutex g_ss_mu;
SharedStream g_ss[kLdsDevs];
hipError_t shared_stream_get(int dev, hipStream_t *out) {
  if (dev < 0 || dev >= kLdsDevs) return hipErrorInvalidDevice;
  std::lock_guard<std::mutex> lk(g_ss_mu);
  SharedStream &x = g_ss[dev];
  if (!x.s) {
    hipError_t e = hipStreamCreateWithFlags(&x.s, hipStreamNonBlocking);
    if (e != hipSuccess) return e;
  }
  x.refs++;
  *out = x.s;
  return hipSuccess;
}
void shared_stream_put(int dev) {
  std::lock_guard<std::mutex> lk(g_ss_mu);
  SharedStream &x = g_ss[dev];
  if (--x.refs == 0) {
    (void)hipStreamDestroy(x.s);
    x.s = nullptr;
  }
}
}  // namespace

extern "C" int dr_create(int n, int faulty, int max_rounds, int device, dr_ctx **out) {
  return dr_create_ex(n, faulty, max_rounds, device, 0, out);
}

extern "C" int dr_create_ex(int n, int faulty, int max_rounds, int device, int flags, dr_ctx **out) {
  if (!out) return DR_E_INVAL;
  *out = nullptr;
  if (n < 1 || n > 2048 || faulty < 0 || max_rounds < 1 || max_rounds > (1 << 20) || device < 0) {
    g_create_err = "dr_create: n must be in [1,2048], faulty >= 0, max_rounds in [1,2^20], device >= 0";
    return DR_E_INVAL;
  }
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || device >= ndev) {
    g_create_err = std::string("dr_create: no usable HIP device (") +
                   (e != hipSuccess ? hipGetErrorString(e) : "ordinal out of range") +
                   "); this library has no CPU fallback";
    return DR_E_HIP;
  }
  dr_ctx *c = new dr_ctx();
  c->touch();
  c->n = n;
  c->f = faulty;
  c->W = (n + 63) / 64;
  c->WS = next_pow2(c->W);
  c->max_rounds = max_rounds;
  c->dev = device;
  // (stream2 is created at the first fork, ensure_stream2: a context that never forks --
  // one DAG of a C5 batch -- keeps one HIP stream, and a device-wide synchronize walks
  // every stream of the process: 4096 contexts x 2 streams cost it ~2.7 ms)
  if ((flags & ~DR_CREATE_SHARED_STREAM) != 0) {
    g_create_err = "dr_create_ex: unknown flags";
    delete c;
    return DR_E_INVAL;
  }
  c->shared_stream = (flags & DR_CREATE_SHARED_STREAM) != 0;
  if (set_device(c) != DR_OK ||
      (c->shared_stream ? shared_stream_get(device, &c->stream)
                        : hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess) {
    g_create_err = "dr_create: stream creation failed";
    c->shared_stream = false;
    c->stream = nullptr;
    delete c;
    return DR_E_HIP;
  }
  // Timing and stream-to-stream events need only a device-scope release: the
  // default system-scope fence (L2 writeback + invalidate) cost the stream ~7 us
  // per record.  ev_sync / ev_sync2 order the kernels' writes to pinned host
  // memory before the host reads them, so they keep the system fence.
  for (auto &ev : c->ev) (void)hipEventCreateWithFlags(&ev, hipEventReleaseToDevice);
  for (hipEvent_t *e : {&c->ev_fork, &c->ev_join, &c->ev_start, &c->ev_wu})
    (void)hipEventCreateWithFlags(e, hipEventDisableTiming | hipEventReleaseToDevice);
  for (hipEvent_t *e : {&c->ev_sync, &c->ev_sync2, &c->ev_commit}) (void)hipEventCreateWithFlags(e, hipEventDisableTiming);
  // (+ a lane's WS rows of slack: k_chain_reg reads each lane's WS rows whole, past n
  // in the last round when WS does not divide n)
  const size_t rows = (size_t)max_rounds * n * c->WS * sizeof(u64) + (size_t)c->WS * c->WS * sizeof(u64);
  if (c->strong.ensure(rows) != hipSuccess ||
      c->present.ensure((size_t)max_rounds * c->WS * sizeof(u64)) != hipSuccess ||
      c->slot_off.ensure((size_t)(max_rounds + 1) * sizeof(uint32_t)) != hipSuccess ||
      c->ppref.ensure((size_t)(max_rounds + 1) * sizeof(u64)) != hipSuccess ||
      c->weak_roff.ensure((size_t)(max_rounds + 1) * sizeof(uint32_t)) != hipSuccess ||
      c->far_roff.ensure((size_t)(max_rounds + 1) * sizeof(uint32_t)) != hipSuccess ||
      c->far.ensure(4096) != hipSuccess || c->irr.ensure(4096) != hipSuccess ||
      c->irr_roff.ensure((size_t)(max_rounds + 1) * sizeof(uint32_t)) != hipSuccess ||
      c->wc_roff.ensure((size_t)(max_rounds + 1) * sizeof(uint32_t)) != hipSuccess ||
      c->wc_key.ensure(4096) != hipSuccess || c->wc_rows.ensure(4096) != hipSuccess ||
      c->sdeg.ensure((size_t)max_rounds * n * sizeof(uint16_t)) != hipSuccess ||
      c->wdeg.ensure((size_t)max_rounds * n * sizeof(uint16_t)) != hipSuccess ||
      c->slot_src.ensure(4096) != hipSuccess || c->lead.ensure(((size_t)max_rounds / 4 + 2) * 2) != hipSuccess) {
    g_create_err = "dr_create: device allocation failed";
    dr_destroy(c);
    return DR_E_HIP;
  }
  uint32_t zero = 0;
  (void)hipMemcpy(c->slot_off.p, &zero, 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(c->weak_roff.p, &zero, 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(c->far_roff.p, &zero, 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(c->irr_roff.p, &zero, 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(c->wc_roff.p, &zero, 4, hipMemcpyHostToDevice);
  c->h_lead.assign((size_t)max_rounds / 4 + 2, 1);  // chooseLeader(w) = 1 (process.go:390-392)
  (void)hipMemcpy(c->lead.p, c->h_lead.data(), c->h_lead.size() * 2, hipMemcpyHostToDevice);
  *out = c;
  return DR_OK;
}

extern "C" void dr_destroy(dr_ctx *c) {
  if (!c) return;
  (void)hipSetDevice(c->dev);
  if (c->stream) (void)c->sync();
  if (c->pin) (void)hipHostFree(c->pin);
  if (c->batch_pin) (void)hipHostFree(c->batch_pin);
  DevBuf *bufs[] = {&c->strong,  &c->present, &c->slot_off, &c->ppref, &c->slot_src, &c->put_buf,
                    &c->weak_roff, &c->far,   &c->far_roff, &c->q_buf,    &c->masks,
                    &c->dlv,     &c->push_out, &c->push_n,  &c->edges,    &c->hits, &c->wedges,
                    &c->commit,  &c->vcount,  &c->popdesc,  &c->rbase,    &c->counts,
                    &c->digest,  &c->pop_pos, &c->ids,      &c->U,        &c->WU,
                    &c->SD,      &c->K,       &c->Kprev,    &c->RG,       &c->rlo,      &c->good,     &c->CE,       &c->RD,
                    &c->Cc,      &c->Gc,      &c->Ec,       &c->crbase,   &c->ccount,
                    &c->nseg,    &c->stops,   &c->qstats, &c->plan_arena, &c->batch_arena, &c->srounds, &c->plan_out,
                    &c->wc_key,  &c->wc_rows, &c->wc_roff, &c->sdeg, &c->setweak, &c->wdeg,
                    &c->admit_buf, &c->lead, &c->split_ctl, &c->irr, &c->irr_roff, &c->gscratch,
                    &c->gquery, &c->gaux};
  for (DevBuf *b : bufs) b->release();
  for (auto &ev : c->ev)
    if (ev) (void)hipEventDestroy(ev);
  for (hipEvent_t e : {c->ev_sync, c->ev_sync2, c->ev_fork, c->ev_join, c->ev_start, c->ev_wu, c->ev_commit})
    if (e) (void)hipEventDestroy(e);
  if (c->rg_exec) (void)hipGraphExecDestroy(c->rg_exec);
  if (c->stream2) (void)hipStreamDestroy(c->stream2);
  if (c->stream) {
    if (c->shared_stream) shared_stream_put(c->dev);
    else (void)hipStreamDestroy(c->stream);
  }
  delete c;
}

extern "C" const char *dr_last_error(const dr_ctx *c) {
  return c ? c->err.c_str() : g_create_err.c_str();
}

extern "C" int dr_num_rounds(const dr_ctx *c) { return c ? c->nrounds : -1; }

// ===========================================================================
// DAG append (validation + packing)
// ===========================================================================
namespace {
// Set bit `own` (0-based source) of the weak column `key` of round h, keeping
// the keys sorted (the order the bulk path produces; no kernel depends on it).
void wc_add(HostRound &h, int WS, uint32_t key, int own) {
  auto it = std::lower_bound(h.wc_key.begin(), h.wc_key.end(), key);
  const size_t j = (size_t)(it - h.wc_key.begin());
  if (it == h.wc_key.end() || *it != key) {
    h.wc_key.insert(it, key);
    h.wc_rows.insert(h.wc_rows.begin() + (ptrdiff_t)(j * WS), (size_t)WS, 0ULL);
  }
  h.wc_rows[j * WS + (own >> 6)] |= 1ULL << (own & 63);
}

// rows, strong and weak degrees of individually appended vertices (vidx = r*n + s-1)
__global__ __launch_bounds__(256) void k_put_vertices(const u64 *__restrict__ rows, const uint32_t *__restrict__ vidx,
                                                      const uint16_t *__restrict__ sd,
                                                      const uint16_t *__restrict__ wd, int nv, int WS,
                                                      u64 *__restrict__ strong, uint16_t *__restrict__ sdeg,
                                                      uint16_t *__restrict__ wdeg) {
  const int64_t total = (int64_t)nv * WS;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int64_t v = t / WS, w = t - v * WS;
    strong[(size_t)vidx[v] * WS + w] = rows[t];
    if (w == 0) {
      sdeg[vidx[v]] = sd[v];
      wdeg[vidx[v]] = wd[v];
    }
  }
}
}  // namespace

extern "C" int dr_append_rounds_packed(dr_ctx *c, int r0, int k, const uint32_t *slot_off,
                                       const uint16_t *slot_src, const uint64_t *strong,
                                       const uint32_t *weak_off, const uint32_t *weak_tgt) {
  if (c) c->touch();
  if (!c) return DR_E_INVAL;
  if (int rc = set_device(c)) return rc;
  if (r0 != c->nrounds) return c->fail(DR_E_STATE, "append at round %d but %d rounds mirrored", r0, c->nrounds);
  if (k < 0 || r0 + k > c->max_rounds) return c->fail(DR_E_INVAL, "append of %d rounds exceeds max_rounds %d", k, c->max_rounds);
  if (k == 0) return DR_OK;
  if (!slot_off || (!slot_src && slot_off[k] > slot_off[0]) || !strong || !weak_off)
    return c->fail(DR_E_INVAL, "null array");
  const int n = c->n, W = c->W, WS = c->WS;
  dr_host::PackedRounds in;
  in.n = n;
  in.W = W;
  in.WS = WS;
  in.r0 = r0;
  in.k = k;
  in.max_rounds = c->max_rounds;
  in.slot_off = slot_off;
  in.slot_src = slot_src;
  in.strong = strong;
  in.weak_off = weak_off;
  in.weak_tgt = weak_tgt;
  dr_host::BuiltRounds built;
  const size_t row_words = (size_t)n * WS;
  const bool staged = WS == W && (size_t)k * row_words * 8 <= ((size_t)16 << 20);
  void *row_stage = nullptr;  // per-round appends: the build's chunk tasks copy the rows into pinned staging
  const auto ta0 = std::chrono::steady_clock::now();
  if (staged) {
    HIPCHK(c, c->stage((size_t)k * row_words * 8, &row_stage));
    in.strong_stage = static_cast<uint64_t *>(row_stage);
  }
  if (int rc = dr_host::build_packed_rounds(in, c->dmax_near, built, c->err, c->build_scr)) return rc;
  const auto ta1 = std::chrono::steady_clock::now();
  std::vector<HostRound> &nh = built.rounds;
  const size_t nfar = built.nfar;
  const int dmax = built.dmax;
  // ---- commit: rows and per-vertex degrees, then the flattened per-round arrays ----
  DeferH2D batch(c);  // every staged copy below goes out in one launch at sync()
  if (staged) {  // per-round appends: pinned staging, written by the build
    HIPCHK(c, c->h2d_staged(c->strong.as<u64>() + (size_t)r0 * row_words, row_stage, (size_t)k * row_words * 8));
  } else if (WS == W) {  // bulk loads: straight from the caller's memory
    HIPCHK(c, hipMemcpyAsync(c->strong.as<u64>() + (size_t)r0 * row_words, strong,
                             (size_t)k * row_words * 8, hipMemcpyHostToDevice, c->stream));
  } else {
    std::vector<u64> pad((size_t)k * row_words, 0);
    for (size_t v = 0; v < (size_t)k * n; v++)
      std::memcpy(&pad[v * WS], strong + v * W, (size_t)W * 8);
    HIPCHK(c, hipMemcpyAsync(c->strong.as<u64>() + (size_t)r0 * row_words, pad.data(), pad.size() * 8,
                             hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  HIPCHK(c, c->h2d(c->sdeg.as<uint16_t>() + (size_t)r0 * n, built.sdeg.data(), built.sdeg.size() * 2));
  HIPCHK(c, c->h2d(c->wdeg.as<uint16_t>() + (size_t)r0 * n, built.wdeg.data(), built.wdeg.size() * 2));
  for (auto &h : nh) c->hr.push_back(std::move(h));
  c->h_sdeg.insert(c->h_sdeg.end(), built.sdeg.begin(), built.sdeg.end());
  c->h_wcnt.insert(c->h_wcnt.end(), built.wdeg.begin(), built.wdeg.end());
  c->h_present.insert(c->h_present.end(), built.pres.begin(), built.pres.end());
  c->nfar += nfar;
  c->nirr += (int64_t)built.nirr;
  if (built.nirr) c->irr_tmax = std::max(c->irr_tmax, built.irr_tmax);
  c->dmax_near = dmax;
  c->nrounds += k;
  for (int r = r0; r < r0 + k; r++) c->touch(r);
  const auto ta2 = std::chrono::steady_clock::now();
  HIPCHK(c, c->upload_suffix());
  const auto ta3 = std::chrono::steady_clock::now();
  // one copy launch for everything staged, no wait: every later call of this context runs
  // behind it on the same stream, the caller's arrays were copied into pinned staging
  // memory (kept until the next wait), and a copy error surfaces at the next call.  (A bulk
  // load's rows went straight from the caller's memory: wait for them.)
  HIPCHK(c, staged ? c->flush_h2d() : c->sync());
  c->async_pending = staged;
  if (staged) {
    char what[96];
    std::snprintf(what, sizeof what, "the copies of dr_append_rounds_packed rounds %d..%d", r0, r0 + k - 1);
    c->async_what = what;
  }
  const auto ta4 = std::chrono::steady_clock::now();
  auto ms = [](auto a, auto b) { return std::chrono::duration<float, std::milli>(b - a).count(); };
  c->append_phases[0] = ms(ta0, ta1);  // validation + host rounds (weak columns)
  c->append_phases[1] = ms(ta1, ta2);  // rows and degrees staged
  c->append_phases[2] = ms(ta2, ta3);  // flattened per-round arrays staged
  c->append_phases[3] = ms(ta3, ta4);  // one copy launch (no wait)
  return DR_OK;
}

extern "C" int dr_append_vertices(dr_ctx *c, int k, const int32_t *slot_round, const int32_t *ids,
                                  const uint32_t *strong_off, const int32_t *strong_ids, const uint32_t *weak_off,
                                  const int32_t *weak_ids) {
  if (c) c->touch();
  if (!c) return DR_E_INVAL;
  if (k < 0) return c->fail(DR_E_INVAL, "negative vertex count");
  if (k == 0) return DR_OK;
  if (!ids || !strong_off || !weak_off) return c->fail(DR_E_INVAL, "null array");
  if (int rc = set_device(c)) return rc;
  const int n = c->n, WS = c->WS, R0 = c->nrounds;
  // pass 1: validate every vertex against the mirror plus the vertices before it
  // in this call; nothing changes unless all of them are inside the contract
  int R = R0;
  for (int i = 0; i < k; i++) {
    const int vr = ids[2 * i], vs = ids[2 * i + 1];
    const int r = slot_round ? slot_round[i] : vr;
    if (r < 0 || r > R)
      return c->fail(DR_E_INVAL, "vertex %d: p.dag[%d] with %d rounds (Go: index out of range)", i, r, R);
    if (r == R) {
      if (R >= c->max_rounds) return c->fail(DR_E_INVAL, "vertex %d opens round %d beyond max_rounds %d", i, r, c->max_rounds);
      R++;
    }
    const uint32_t sa = strong_off[i], sb = strong_off[i + 1], wa = weak_off[i], wb = weak_off[i + 1];
    if (sb < sa || wb < wa) return c->fail(DR_E_INVAL, "vertex %d: edge offsets not monotone", i);
    if ((sb > sa && !strong_ids) || (wb > wa && !weak_ids)) return c->fail(DR_E_INVAL, "null edge array");
    if (vr == 0 && vs == 0) {  // ghost slot: zero vertexID (process_internal_test.go:89-100)
      if (sb != sa || wb != wa) return c->fail(DR_E_CONTRACT, "p.dag[%d]: ghost slot {0,0} with edges", r);
      continue;
    }
    if (vr != r || vs < 1 || vs > n)
      return c->fail(DR_E_CONTRACT, "p.dag[%d]: id (%d,%d) outside the mirrored contract", r, vr, vs);
    // any target id the mirror can hold: edges outside the round contract (App. A Q8)
    // are kept as irregular edges and answered by the general sweep (general.hpp)
    for (uint32_t e = sa; e < sb; e++) {
      const int tr = strong_ids[2 * e], ts = strong_ids[2 * e + 1];
      if (tr < 0 || tr >= c->max_rounds || ts < 1 || ts > n)
        return c->fail(DR_E_CONTRACT, "strong edge (%d,%d)->(%d,%d): target outside rounds [0,%d), sources [1,%d]", r, vs,
                       tr, ts, c->max_rounds, n);
    }
    for (uint32_t e = wa; e < wb; e++) {
      const int tr = weak_ids[2 * e], ts = weak_ids[2 * e + 1];
      if (tr < 0 || tr >= c->max_rounds || ts < 1 || ts > n)
        return c->fail(DR_E_CONTRACT, "weak edge (%d,%d)->(%d,%d): target outside rounds [0,%d), sources [1,%d]", r, vs, tr,
                       ts, c->max_rounds, n);
    }
  }
  // pass 2: apply
  DeferH2D batch(c);
  if (R > R0) {  // opened rounds start empty: zero rows and degrees
    const size_t a = (size_t)R0 * n, b = (size_t)R * n;
    HIPCHK(c, hipMemsetAsync(c->strong.as<u64>() + a * WS, 0, (b - a) * WS * 8, c->stream));
    HIPCHK(c, hipMemsetAsync(c->sdeg.as<uint16_t>() + a, 0, (b - a) * 2, c->stream));
    HIPCHK(c, hipMemsetAsync(c->wdeg.as<uint16_t>() + a, 0, (b - a) * 2, c->stream));
    c->hr.resize(R);
    c->h_present.resize((size_t)R * WS, 0);
    c->h_sdeg.resize((size_t)R * n, 0);
    c->h_wcnt.resize((size_t)R * n, 0);
    c->nrounds = R;
  }
  std::vector<u64> rows((size_t)k * WS, 0);
  std::vector<uint32_t> vidx(k);
  std::vector<uint16_t> sd(k), wd(k);
  std::unordered_map<uint32_t, int> put_at;  // vertex index -> its entry (a repeated id rewrites it)
  int nv = 0, dmax = c->dmax_near;
  for (int i = 0; i < k; i++) {
    const int vr = ids[2 * i], vs = ids[2 * i + 1];
    const int r = slot_round ? slot_round[i] : vr;
    HostRound &h = c->hr[r];
    c->touch(r);
    if (vr == 0 && vs == 0) {
      h.slots.push_back(0);
      continue;
    }
    h.slots.push_back((uint16_t)vs);
    const size_t vi = (size_t)r * n + vs - 1;
    u64 &pw = c->h_present[(size_t)r * WS + ((vs - 1) >> 6)];
    const u64 pbit = 1ULL << ((vs - 1) & 63);
    if (pw & pbit) {  // the id is already in the round: this vertex replaces it for path()'s
      // lookup (the last slot, process.go:112-116): take back its degree and weak edges
      h.deg -= c->h_sdeg[vi];
      h.nweak -= c->h_wcnt[vi];
      const int o = vs - 1;
      for (size_t j = 0; j < h.wc_key.size();) {
        uint64_t *wr = &h.wc_rows[j * WS];
        wr[o >> 6] &= ~(1ULL << (o & 63));
        bool any = false;
        for (int w = 0; w < WS; w++) any |= wr[w] != 0ULL;
        if (any) { j++; continue; }
        h.wc_key.erase(h.wc_key.begin() + (ptrdiff_t)j);
        h.wc_rows.erase(h.wc_rows.begin() + (ptrdiff_t)(j * WS), h.wc_rows.begin() + (ptrdiff_t)((j + 1) * WS));
      }
      const size_t nf = h.far.size();
      h.far.erase(std::remove_if(h.far.begin(), h.far.end(), [&](uint64_t x) { return (int)(x >> 32) == o; }),
                  h.far.end());
      c->nfar -= nf - h.far.size();
      const size_t ni = h.irr.size();
      h.irr.erase(std::remove_if(h.irr.begin(), h.irr.end(),
                                 [&](uint64_t x) { return (int)((x >> 32) & 2047u) == o; }),
                  h.irr.end());
      c->nirr -= ni - h.irr.size();
    }
    pw |= pbit;
    auto pa = put_at.find((uint32_t)vi);
    const int slot_nv = pa == put_at.end() ? nv : pa->second;
    u64 *row = &rows[(size_t)slot_nv * WS];
    std::fill(row, row + WS, 0ULL);
    uint64_t nirr_s = 0;  // strong edges outside the round contract (App. A Q8)
    for (uint32_t e = strong_off[i]; e < strong_off[i + 1]; e++) {
      const int tr = strong_ids[2 * e], ts = strong_ids[2 * e + 1] - 1;
      if (tr != r - 1) {
        h.irr.push_back(dr::irr_pack(vs - 1, true, tr, ts));
        c->irr_tmax = std::max(c->irr_tmax, tr);
        nirr_s++;
        continue;
      }
      row[ts >> 6] |= 1ULL << (ts & 63);
    }
    c->nirr += (int64_t)nirr_s;
    uint64_t d = nirr_s;
    for (int w = 0; w < WS; w++) d += (uint64_t)__builtin_popcountll(row[w]);
    h.deg += d;
    const uint32_t wa = weak_off[i], wb = weak_off[i + 1];
    for (uint32_t e = wa; e < wb; e++) {
      const int tr = weak_ids[2 * e], ts = weak_ids[2 * e + 1] - 1, delta = r - tr;
      if (delta < 2) {  // a weak edge not below r-1 (App. A Q8)
        h.irr.push_back(dr::irr_pack(vs - 1, false, tr, ts));
        c->irr_tmax = std::max(c->irr_tmax, tr);
        c->nirr++;
        continue;
      }
      if (delta <= 1023) {
        wc_add(h, WS, ((uint32_t)delta << 11) | (uint32_t)ts, vs - 1);
        dmax = std::max(dmax, delta);
      } else {
        h.far.push_back(((u64)(vs - 1) << 32) | ((uint32_t)tr << 11) | (uint32_t)ts);
        c->nfar++;
      }
    }
    h.nweak += wb - wa;
    c->h_sdeg[vi] = (uint16_t)d;
    c->h_wcnt[vi] = (uint16_t)std::min<uint32_t>(wb - wa, 65535u);
    vidx[slot_nv] = (uint32_t)vi;
    sd[slot_nv] = (uint16_t)d;
    wd[slot_nv] = (uint16_t)std::min<uint32_t>(wb - wa, 65535u);
    if (pa == put_at.end()) put_at.emplace((uint32_t)vi, nv++);
  }
  c->dmax_near = dmax;
  if (nv) {
    const size_t o_idx = (size_t)nv * WS * 8, o_sd = o_idx + (size_t)nv * 4, o_wd = o_sd + (size_t)nv * 2;
    HIPCHK(c, c->put_buf.ensure(o_wd + (size_t)nv * 2));
    char *b = c->put_buf.as<char>();
    HIPCHK(c, c->h2d(b, rows.data(), o_idx));
    HIPCHK(c, c->h2d(b + o_idx, vidx.data(), (size_t)nv * 4));
    HIPCHK(c, c->h2d(b + o_sd, sd.data(), (size_t)nv * 2));
    HIPCHK(c, c->h2d(b + o_wd, wd.data(), (size_t)nv * 2));
    HIPCHK(c, c->flush_h2d());  // k_put_vertices reads them
    const int blocks = (int)std::min<int64_t>(1024, ((int64_t)nv * WS + 255) / 256);
    hipLaunchKernelGGL(k_put_vertices, dim3(blocks), dim3(256), 0, c->stream, reinterpret_cast<const u64 *>(b),
                       reinterpret_cast<const uint32_t *>(b + o_idx), reinterpret_cast<const uint16_t *>(b + o_sd),
                       reinterpret_cast<const uint16_t *>(b + o_wd), nv, WS, c->strong.as<u64>(),
                       c->sdeg.as<uint16_t>(), c->wdeg.as<uint16_t>());
    HIPCHK(c, hipGetLastError());
  }
  HIPCHK(c, c->upload_suffix());
  HIPCHK(c, c->sync());
  return DR_OK;
}

extern "C" int dr_append_rounds_lists(dr_ctx *c, int r0, int k, const uint32_t *slot_off,
                                      const int32_t *slot_id, const uint32_t *strong_off,
                                      const int32_t *strong_ids, const uint32_t *weak_off,
                                      const int32_t *weak_ids) {
  if (c) c->touch();
  if (!c) return DR_E_INVAL;
  if (k < 0) return c->fail(DR_E_INVAL, "negative round count");
  if (k == 0) return DR_OK;
  if (!slot_off || !slot_id || !strong_off || !weak_off) return c->fail(DR_E_INVAL, "null array");
  const int n = c->n, W = c->W;
  const uint32_t S0 = slot_off[0], S1 = slot_off[k];
  std::vector<uint32_t> so(k + 1);
  std::vector<uint16_t> src(std::max<uint32_t>(S1 - S0, 1));
  std::vector<uint64_t> rows((size_t)k * n * W, 0);
  std::vector<std::vector<uint32_t>> wl((size_t)k * n);
  std::vector<std::vector<uint64_t>> irl((size_t)k * n);  // edges outside the round contract (App. A Q8)
  if (r0 < 0 || k > c->max_rounds || r0 > c->max_rounds - k)
    return c->fail(DR_E_INVAL, "append of rounds [%d, %d) exceeds max_rounds %d", r0, r0 + k, c->max_rounds);
  for (int i = 0; i <= k; i++) so[i] = slot_off[i] - S0;
  for (int i = 0; i < k; i++) {
    const int r = r0 + i;
    for (uint32_t sl = slot_off[i]; sl < slot_off[i + 1]; sl++) {
      const int vr = slot_id[2 * sl], vs = slot_id[2 * sl + 1];
      const uint32_t sa = strong_off[sl], sb = strong_off[sl + 1];
      const uint32_t wa = weak_off[sl], wb = weak_off[sl + 1];
      if (vr == 0 && vs == 0) {  // ghost slot: zero vertexID (process_internal_test.go:89-100)
        if (sb != sa || wb != wa) return c->fail(DR_E_CONTRACT, "round %d: ghost slot {0,0} with edges", r);
        src[sl - S0] = 0;
        continue;
      }
      if (vr != r || vs < 1 || vs > n)
        return c->fail(DR_E_CONTRACT, "round %d slot %u: id (%d,%d) outside the mirrored contract", r, sl - slot_off[i], vr, vs);
      src[sl - S0] = (uint16_t)vs;
      uint64_t *row = &rows[((size_t)i * n + (vs - 1)) * W];
      // a repeated id: path()'s lookup takes the last slot (process.go:112-116), so
      // its edges replace the earlier slot's
      std::fill(row, row + W, 0ULL);
      wl[(size_t)i * n + (vs - 1)].clear();
      std::vector<uint64_t> &I = irl[(size_t)i * n + (vs - 1)];
      I.clear();
      for (uint32_t e = sa; e < sb; e++) {
        const int tr = strong_ids[2 * e], ts = strong_ids[2 * e + 1];
        if (tr < 0 || tr >= c->max_rounds || ts < 1 || ts > n)
          return c->fail(DR_E_CONTRACT, "strong edge (%d,%d)->(%d,%d): target outside rounds [0,%d), sources [1,%d]", r,
                         vs, tr, ts, c->max_rounds, n);
        if (tr != r - 1) I.push_back(dr::irr_pack(vs - 1, true, tr, ts - 1));
        else row[(ts - 1) >> 6] |= 1ULL << ((ts - 1) & 63);
      }
      std::vector<uint32_t> &L = wl[(size_t)i * n + (vs - 1)];
      for (uint32_t e = wa; e < wb; e++) {
        const int tr = weak_ids[2 * e], ts = weak_ids[2 * e + 1];
        if (tr < 0 || tr >= c->max_rounds || ts < 1 || ts > n)
          return c->fail(DR_E_CONTRACT, "weak edge (%d,%d)->(%d,%d): target outside rounds [0,%d), sources [1,%d]", r,
                         vs, tr, ts, c->max_rounds, n);
        if (tr > r - 2) I.push_back(dr::irr_pack(vs - 1, false, tr, ts - 1));
        else L.push_back(((uint32_t)tr << 11) | (uint32_t)(ts - 1));
      }
    }
  }
  std::vector<uint32_t> woff((size_t)k * n + 1, 0);
  std::vector<uint32_t> wt;
  for (size_t v = 0; v < (size_t)k * n; v++) {
    woff[v] = (uint32_t)wt.size();
    wt.insert(wt.end(), wl[v].begin(), wl[v].end());
  }
  woff[(size_t)k * n] = (uint32_t)wt.size();
  if (int rc = dr_append_rounds_packed(c, r0, k, so.data(), src.data(), rows.data(), woff.data(), wt.data()))
    return rc;
  // the irregular edges of the appended rounds: kept per round, counted in the vertices'
  // degrees (edge totals count every edge of an id once)
  bool any = false;
  for (int i = 0; i < k; i++)
    for (int s = 0; s < n; s++) {
      const std::vector<uint64_t> &I = irl[(size_t)i * n + s];
      if (I.empty()) continue;
      any = true;
      HostRound &h = c->hr[r0 + i];
      uint32_t ns = 0, nwk = 0;
      for (uint64_t x : I) {
        ((x >> 31) & 1u) ? ns++ : nwk++;
        c->irr_tmax = std::max(c->irr_tmax, (int)((x >> 11) & 0xFFFFFu));
      }
      h.irr.insert(h.irr.end(), I.begin(), I.end());
      c->nirr += (int64_t)I.size();
      const size_t vi = (size_t)(r0 + i) * n + s;
      c->h_sdeg[vi] = (uint16_t)std::min<uint32_t>(c->h_sdeg[vi] + ns, 65535u);
      c->h_wcnt[vi] = (uint16_t)std::min<uint32_t>(c->h_wcnt[vi] + nwk, 65535u);
      h.deg += ns;
      h.nweak += nwk;
    }
  if (!any) return DR_OK;
  for (int r = r0; r < r0 + k; r++) c->touch(r);
  HIPCHK(c, c->h2d(c->sdeg.as<uint16_t>() + (size_t)r0 * n, &c->h_sdeg[(size_t)r0 * n], (size_t)k * n * 2));
  HIPCHK(c, c->h2d(c->wdeg.as<uint16_t>() + (size_t)r0 * n, &c->h_wcnt[(size_t)r0 * n], (size_t)k * n * 2));
  HIPCHK(c, c->upload_suffix());
  HIPCHK(c, c->sync());
  return DR_OK;
}

// ===========================================================================
// queries
// ===========================================================================
namespace {

// Run sweep queries in batches bounded by the mask budget.  qv: queries with
// mask_off filled here per batch (Q_MASKS).  On return the per-query edges /
// hits / pushes / stop rounds are in host arrays.  Each batch's masks are
// handed to `on_batch` before the next batch overwrites them.  Masks are
// zeroed unless every query of the batch is a merge sweep (those write every
// round they report).
template <class OnBatch>
int run_sweeps(dr_ctx *c, std::vector<dr::SweepQuery> &qv, bool seq, std::vector<uint64_t> *edges,
               std::vector<uint64_t> *wedges, std::vector<uint8_t> *hits, std::vector<int32_t> *push_n,
               int32_t *push_out_dev, std::vector<int32_t> *stops, OnBatch on_batch, float *ms,
               std::vector<uint64_t> *qstats = nullptr, const std::function<int()> &pre_sync = {}) {
  const size_t budget_words = (size_t)1 << 29;  // 4 GiB of frontier masks per batch
  const int WS = c->WS;
  if (edges) edges->assign(qv.size(), 0);
  if (wedges) wedges->assign(qv.size(), 0);
  if (hits) hits->assign(qv.size(), 0);
  if (push_n) push_n->assign(qv.size(), 0);
  if (stops) stops->assign(qv.size(), 0);
  if (qstats) qstats->assign(qv.size() * 4, 0);
  size_t i0 = 0;
  float total_ms = 0;
  while (i0 < qv.size()) {
    // batch [i0, i1): as many queries as the mask budget allows (sequential
    // mode keeps its order across batches: the delivered set persists)
    size_t i1 = i0, words = 0;
    bool all_merge = true;
    while (i1 < qv.size()) {
      const size_t w = (qv[i1].flags & dr::Q_MASKS) ? (size_t)(qv[i1].top - qv[i1].bottom + 1) * WS : 0;
      if (i1 > i0 && (words + w > budget_words || sweep_mode(qv[i1]) != sweep_mode(qv[i0]))) break;
      qv[i1].mask_off = (int64_t)words;
      all_merge &= (qv[i1].flags & dr::Q_MERGE) != 0;
      words += w;
      i1++;
    }
    const int nq = (int)(i1 - i0);
    HIPCHK(c, c->masks.ensure(std::max<size_t>(words, 1) * 8));
    if (words && !all_merge) HIPCHK(c, hipMemsetAsync(c->masks.p, 0, words * 8, c->stream));
    HIPCHK(c, c->q_buf.ensure((size_t)nq * sizeof(dr::SweepQuery)));
    HIPCHK(c, c->h2d(c->q_buf.p, qv.data() + i0, (size_t)nq * sizeof(dr::SweepQuery)));
    HIPCHK(c, c->edges.ensure((size_t)nq * 8));
    HIPCHK(c, c->wedges.ensure((size_t)nq * 8));
    HIPCHK(c, c->hits.ensure((size_t)nq));
    HIPCHK(c, c->push_n.ensure((size_t)nq * 4));
    HIPCHK(c, c->stops.ensure((size_t)nq * 4));
    HIPCHK(c, c->qstats.ensure((size_t)nq * 32));
    SweepArgs a;
    a.q = c->q_buf.as<dr::SweepQuery>();
    a.nq = nq;
    a.seq = seq ? 1 : 0;
    a.masks = c->masks.as<u64>();
    a.dlv = c->dlv.as<u64>();
    a.push_out = push_out_dev;
    a.push_n = c->push_n.as<int32_t>();
    a.edges = c->edges.as<u64>();
    a.wedges = c->wedges.as<u64>();
    a.hits = c->hits.as<uint8_t>();
    a.stops = c->stops.as<int32_t>();
    a.stats = qstats ? c->qstats.as<u64>() : nullptr;
    HIPCHK(c, hipEventRecord(c->ev[0], c->stream));
    HIPCHK(c, launch_sweep(c, a, sweep_mode(qv[i0])));
    HIPCHK(c, hipEventRecord(c->ev[1], c->stream));
    if (edges) HIPCHK(c, c->d2h(edges->data() + i0, c->edges.p, (size_t)nq * 8));
    if (wedges) HIPCHK(c, c->d2h(wedges->data() + i0, c->wedges.p, (size_t)nq * 8));
    if (hits) HIPCHK(c, c->d2h(hits->data() + i0, c->hits.p, (size_t)nq));
    if (push_n) HIPCHK(c, c->d2h(push_n->data() + i0, c->push_n.p, (size_t)nq * 4));
    if (stops) HIPCHK(c, c->d2h(stops->data() + i0, c->stops.p, (size_t)nq * 4));
    if (qstats) HIPCHK(c, c->d2h(qstats->data() + 4 * i0, c->qstats.p, (size_t)nq * 32));
    if (pre_sync && i1 == qv.size())
      if (int rc = pre_sync()) return rc;
    HIPCHK(c, c->sync());
    float t = 0;
    HIPCHK(c, hipEventElapsedTime(&t, c->ev[0], c->ev[1]));
    total_ms += t;
    if (int rc = on_batch(i0, i1)) return rc;
    i0 = i1;
  }
  if (ms) *ms = total_ms;
  return DR_OK;
}

// Emission of npop pops from their segments pd (pd[i].out in [0, npop),
// rbase_off assigned here).  count_out[p] = extra[p] (vertices the caller
// accounts for, may be null) + the segments' vertices; digest_out[p] = the
// segments' digest sum.  ids (optional): pop p's vertices at ids_base + the
// pops before it (then every vertex must be in a segment).
int run_emit(dr_ctx *c, std::vector<dr::PopDesc> &pd, int npop, const uint64_t *extra, uint64_t *count_out,
             uint64_t *digest_out, int32_t *ids_host, int64_t ids_cap, int64_t ids_base, int64_t *ids_total,
             float *ms) {
  const int nd = (int)pd.size();
  std::vector<uint64_t> cnt(npop, 0);
  if (extra) std::copy(extra, extra + npop, cnt.begin());
  std::fill(digest_out, digest_out + npop, 0);
  if (nd == 0) {
    std::copy(cnt.begin(), cnt.end(), count_out);
    if (ids_total) { *ids_total = 0; for (auto x : cnt) *ids_total += (int64_t)x; }
    return DR_OK;
  }
  int64_t rb_words = 0;
  int span = 0;
  for (auto &d : pd) {
    d.rbase_off = rb_words;
    rb_words += d.last - d.first + 1;
    span = std::max(span, d.last - d.first + 1);
  }
  HIPCHK(c, c->rbase.ensure((size_t)std::max<int64_t>(rb_words, 1) * 4));
  HIPCHK(c, c->popdesc.ensure((size_t)nd * sizeof(dr::PopDesc)));
  HIPCHK(c, c->counts.ensure((size_t)nd * 8));
  HIPCHK(c, c->digest.ensure((size_t)npop * 8));
  HIPCHK(c, c->h2d(c->popdesc.p, pd.data(), (size_t)nd * sizeof(dr::PopDesc)));
  HIPCHK(c, hipMemsetAsync(c->digest.p, 0, (size_t)npop * 8, c->stream));
  HIPCHK(c, hipEventRecord(c->ev[2], c->stream));
  HIPCHK(c, launch_emit(c, nd, span, c->popdesc.as<dr::PopDesc>(), c->rbase.as<uint32_t>(), c->counts.as<u64>(),
                        nullptr, nullptr, nullptr, nullptr, 0, true));
  int32_t *ids_dev = nullptr;
  int64_t cap_here = 0, tot = 0;
  if (ids_host && ids_base < ids_cap) {
    std::vector<uint64_t> dc(nd);
    HIPCHK(c, c->d2h(dc.data(), c->counts.p, (size_t)nd * 8));
    HIPCHK(c, c->sync());
    std::vector<uint64_t> pc(cnt);
    for (int i = 0; i < nd; i++) pc[pd[i].out] += dc[i];
    for (int p = 0; p < npop; p++) tot += (int64_t)pc[p];
    cap_here = std::min<int64_t>(tot, ids_cap - ids_base);
    std::vector<int64_t> pos(npop);
    int64_t run = 0;
    for (int p = 0; p < npop; p++) { pos[p] = run; run += (int64_t)pc[p]; }
    HIPCHK(c, c->pop_pos.ensure((size_t)npop * 8));
    HIPCHK(c, c->h2d(c->pop_pos.p, pos.data(), (size_t)npop * 8));
    HIPCHK(c, c->ids.ensure((size_t)std::max<int64_t>(cap_here, 1) * 8));
    ids_dev = c->ids.as<int32_t>();
  }
  HIPCHK(c, launch_emit(c, nd, span, c->popdesc.as<dr::PopDesc>(), c->rbase.as<uint32_t>(), nullptr,
                        c->digest.as<u64>(), nullptr, ids_dev ? c->pop_pos.as<int64_t>() : nullptr, ids_dev,
                        cap_here, false));
  HIPCHK(c, hipEventRecord(c->ev[3], c->stream));
  std::vector<uint64_t> dc(nd);
  HIPCHK(c, c->d2h(dc.data(), c->counts.p, (size_t)nd * 8));
  HIPCHK(c, c->d2h(digest_out, c->digest.p, (size_t)npop * 8));
  if (ids_dev && cap_here > 0)
    HIPCHK(c, c->d2h(ids_host + 2 * ids_base, ids_dev, (size_t)cap_here * 8));
  HIPCHK(c, c->sync());
  for (int i = 0; i < nd; i++) cnt[pd[i].out] += dc[i];
  std::copy(cnt.begin(), cnt.end(), count_out);
  if (ids_total) {
    *ids_total = 0;
    for (auto x : cnt) *ids_total += (int64_t)x;
  }
  if (ms) {
    float t = 0;
    HIPCHK(c, hipEventElapsedTime(&t, c->ev[2], c->ev[3]));
    *ms += t;
  }
  return DR_OK;
}

// Summary and canonical-cone buffers, sized once for max_rounds (WU for the
// current weak window; a wider window reallocates it and rebuilds every round).
int ensure_summary_bufs(dr_ctx *c) {
  const size_t R = (size_t)c->max_rounds + 1, WS = c->WS, dd = (size_t)c->memo_dd();
  HIPCHK(c, c->U.ensure(R * WS * 8));
  HIPCHK(c, c->WU.ensure(std::max<size_t>(R * dd * WS, 1) * 8));
  HIPCHK(c, c->SD.ensure(R * 8));
  HIPCHK(c, c->K.ensure(R * WS * 8));
  HIPCHK(c, c->good.ensure(R + 64));  // k_canon reads good[] 64 rounds at a time
  HIPCHK(c, c->CE.ensure(R * 8));
  HIPCHK(c, c->RD.ensure(R * 8));
  HIPCHK(c, c->Kprev.ensure(R * WS * 8));
  HIPCHK(c, c->RG.ensure(R * 8));
  HIPCHK(c, c->rlo.ensure(8));
  HIPCHK(c, c->Cc.ensure(R * 8));
  HIPCHK(c, c->Gc.ensure(R * 8));
  HIPCHK(c, c->Ec.ensure(R * 8));
  HIPCHK(c, c->crbase.ensure((R + 1) * 4));
  HIPCHK(c, c->ccount.ensure(8));
  HIPCHK(c, c->nseg.ensure(4));
  HIPCHK(c, c->srounds.ensure(R * 4));
  return DR_OK;
}

void mark_rounds_clean(dr_ctx *c) {
  std::fill(c->sdirty.begin(), c->sdirty.end(), 0);
  c->ndirty = 0;
  c->sum_dd = c->memo_dd();
}

// Incremental round summaries (U, SD, WU) of the rounds appended or changed
// since they were last built: one workgroup per stale round.  A DAG that left
// the memo contract (far weak edges, deltas > 65) keeps none.
int refresh_rounds(dr_ctx *c, bool any = false) {
  // G_reg's summaries, exceptions tested or not (any: also with edges upward, for k_gsweep)
  if (!c->use_memo || (!any && !c->memo_struct_ok())) return DR_OK;
  const int T = c->nrounds - 1;
  if (T < 1) return DR_OK;
  const int dd = c->memo_dd();
  const bool all = dd != c->sum_dd;
  if (!all && c->ndirty == 0) return DR_OK;
  if (int rc = ensure_summary_bufs(c)) return rc;
  std::vector<int32_t> list;
  for (int r = 1; r <= T; r++)
    if (all || c->sdirty[r]) list.push_back(r);
  if (!list.empty()) {
    dr::RoundList rl{};
    rl.n = (int)list.size();
    if (rl.n <= dr::kRoundListMax) {  // in the launch's arguments
      std::copy(list.begin(), list.end(), rl.r);
    } else {
      HIPCHK(c, c->h2d(c->srounds.p, list.data(), list.size() * 4));
      rl.ext = c->srounds.as<int32_t>();
    }
    HIPCHK(c, launch_round_summary(c, rl));
  }
  mark_rounds_clean(c);
  return DR_OK;
}

// The exception test: every exception u -> v of a round touched since
// the last test is benign iff v is in u's cone over G_reg (strong cone for a strong
// edge): one sweep from u down to v's round per exception, Q_REGULAR (weak columns of
// delta <= dreg, no far edge), on G_reg's round summaries (Q_SHORTCUT).  A test covers a
// round for good: later rounds cannot change the cone of u below u's round, and an
// append or replacement in round r re-tests rounds >= r (touch).  Nothing to do with
// no exceptions, or with an upward irregular edge (the general sweep serves everything).
int ensure_exceptions(dr_ctx *c) {
  const int R = c->nrounds;
  if (c->exc_lo >= R) return DR_OK;
  if (c->nexc == 0 || (c->nirr_up > 0 && !c->up_verifiable_structure())) {
    c->exc_lo = c->nexc == 0 ? INT_MAX : c->exc_lo;
    return DR_OK;
  }
  const int lo = std::max(0, c->exc_lo), WS = c->WS, X = c->reg_max();
  std::vector<dr::SweepQuery> qs, qw;  // strong-only, weak
  std::vector<int32_t> rs, rw;         // each query's round
  auto add = [&](int r, int src0, int tr, int ts0, bool strong) {
    dr::SweepQuery q{};
    q.top = r;
    q.bottom = tr;
    q.src0 = src0;
    q.tgt0 = ts0;
    q.flags = strong ? dr::Q_STRONG_ONLY : dr::Q_REGULAR;
    (strong ? qs : qw).push_back(q);
    (strong ? rs : rw).push_back(r);
  };
  for (int r = lo; r < R; r++) {
    c->nbad -= c->h_rbad[r];
    c->h_rbad[r] = 0;
    if (!c->h_rexc[r]) continue;
    const HostRound &h = c->hr[r];
    for (size_t j = 0; j < h.wc_key.size(); j++) {
      const int delta = (int)(h.wc_key[j] >> 11), ts = (int)(h.wc_key[j] & 2047u);
      if (delta <= X) continue;
      for (int w = 0; w < WS; w++)
        for (u64 x = h.wc_rows[j * WS + w]; x; x &= x - 1) add(r, w * 64 + __builtin_ctzll(x), r - delta, ts, false);
    }
    for (uint64_t x : h.far) {
      const uint32_t t = (uint32_t)x;
      add(r, (int)(x >> 32), (int)(t >> 11), (int)(t & 2047u), false);
    }
    for (uint64_t x : h.irr) {
      const int tr = (int)((x >> 11) & 0xFFFFFu);
      if (tr < r) add(r, (int)((x >> 32) & 2047u), tr, (int)(x & 2047u), ((x >> 31) & 1u) != 0);
    }
  }
  if (int rc = refresh_rounds(c)) return rc;
  const int sc = (c->use_memo && c->ndirty == 0 && c->sum_dd == c->memo_dd() && R >= 2) ? dr::Q_SHORTCUT : 0;
  for (int pass = 0; pass < 2; pass++) {
    std::vector<dr::SweepQuery> &qv = pass ? qw : qs;
    const std::vector<int32_t> &rv = pass ? rw : rs;
    if (qv.empty()) continue;
    for (auto &q : qv) q.flags |= sc;
    std::vector<uint8_t> hits;
    int rc = run_sweeps(c, qv, false, nullptr, nullptr, &hits, nullptr, nullptr, nullptr,
                        [](size_t, size_t) { return 0; }, nullptr);
    if (rc) return rc;
    c->exc_sweeps += qv.size();
    for (size_t i = 0; i < qv.size(); i++)
      if (!hits[i]) {
        c->h_rbad[rv[i]]++;
        c->nbad++;
      }
  }
  c->exc_lo = INT_MAX;
  return DR_OK;
}

// every query entry point: the device, then the exception test of the rounds changed
// since the last one (general() and memo_on() read its verdict)
int prep_query(dr_ctx *c, bool slice_ok = false) {
  if (c->slice_on && !slice_ok)
    return c->fail(DR_E_STATE, "a sliced context (dr_set_slice) answers dr_replay only");
  if (int rc = set_device(c)) return rc;
  return ensure_exceptions(c);
}

// Canonical cone K of the current top round + canonical prefixes C, G, E
// (DESIGN.md s3.2), from fresh round summaries.
// fork: the canonical chain runs on stream2 (joined by the caller through
// ev_join) while the caller's next phases use stream.  side (optional, with
// fork): work launched on stream2 first, beside the canonical chain, which then
// stays on the main stream; ev_join marks its end.  forked: stream2 already
// waits on an event of the main stream (build_summary's).
// prefix = false: the caller's emitting sweep computes the G, E prefixes.
// spec: RG holds every round's speculative digest (build_summary's weak union).
// the second stream, created at the first fork (dr_create)
inline hipError_t ensure_stream2(dr_ctx *c) {
  return c->stream2 ? hipSuccess : hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking);
}

int launch_canon(dr_ctx *c, bool fork, const std::function<int()> *side, bool forked = false,
                 bool incremental = false, bool prefix = true, bool spec_rg = false, const ChainFuse *cf = nullptr) {
  const int T = c->nrounds - 1;
  // incremental (the per-call path): rounds below the lowest one that changed
  // since the last cone, and whose canonical vertices are unchanged, keep their
  // per-round digests (RG); a replay recomputes every round
  const bool inc = incremental && c->kprev_ok && c->canon_dd == c->memo_dd();
  const int lo = inc ? std::max(1, std::min(c->canon_lo, c->canon_T + 1)) : 1;
  if (c->kprev_ok) std::swap(c->K, c->Kprev);  // Kprev: the last cone (every round of K is rewritten)
  struct Swap {  // launch helpers use c->stream: point it at stream2 for the canonical chain
    dr_ctx *c;
    bool on;
    Swap(dr_ctx *c_, bool on_) : c(c_), on(on_) { if (on) std::swap(c->stream, c->stream2); }
    ~Swap() { if (on) std::swap(c->stream, c->stream2); }
  };
  if (fork) HIPCHK(c, ensure_stream2(c));
  if (fork && !forked) {
    HIPCHK(c, hipEventRecord(c->ev_fork, c->stream));
    HIPCHK(c, hipStreamWaitEvent(c->stream2, c->ev_fork, 0));
  }
  if (fork && side) {
    Swap sw(c, true);
    if (int rc = (*side)()) return rc;
    HIPCHK(c, hipEventRecord(c->ev_join, c->stream));  // c->stream is stream2 here
  }
  Swap sw(c, fork && !side);
  // canonical cone, per-round counts and positions (k_kcand + k_canon), then the
  // per-round digests (emission) and their prefixes
  const bool spec = spec_rg && lo <= 1;  // a full cone: re-emission from the first non-full round
  HIPCHK(c, launch_canon_cone(c, T, lo, spec, cf));  // *rlo = the lowest round to re-emit
  dr::PopDesc d{};
  d.mask_off = 0;
  d.rbase_off = 1;  // crbase is indexed by round; rbase_off addresses round `first`
  d.pos0 = 0;
  d.first = 1;
  d.last = T;
  d.out = 0;
  d.use_k = 1;
  if (!(cf && cf->emit_in_sweep && spec))  // (else the delivery sweeps' launch re-emits, dr::CanonEmit)
    HIPCHK(c, launch_emit(c, 1, T, nullptr, c->crbase.as<uint32_t>(), nullptr, nullptr, c->RG.as<u64>(), nullptr,
                          nullptr, 0, false, nullptr, nullptr, d, nullptr,
                          c->rlo.as<int>()));  // the descriptor travels by value
  if (prefix)
    hipLaunchKernelGGL((dr::k_canon_prefix<1024>), dim3(1), dim3(1024), 0, c->stream, T, c->RG.as<u64>(),
                       c->CE.as<u64>(), c->Gc.as<u64>(), c->Ec.as<u64>());
  HIPCHK(c, hipGetLastError());
  if (fork && !side) HIPCHK(c, hipEventRecord(c->ev_join, c->stream));  // c->stream is stream2 here
  c->kprev_ok = true;
  c->canon_dd = c->memo_dd();
  c->canon_lo = INT_MAX;
  c->canon_T = T;
  c->canon_ok = true;
  c->canon_host = false;
  return DR_OK;
}

// host copies of the canonical prefixes (after a planned replay left them on the device)
int fetch_canon(dr_ctx *c) {
  if (c->canon_host) return DR_OK;
  const size_t R = (size_t)c->canon_T + 1;
  c->hC.resize(R);
  c->hG.resize(R);
  c->hE.resize(R);
  HIPCHK(c, c->d2h(c->hC.data(), c->Cc.p, R * 8));
  HIPCHK(c, c->d2h(c->hG.data(), c->Gc.p, R * 8));
  HIPCHK(c, c->d2h(c->hE.data(), c->Ec.p, R * 8));
  HIPCHK(c, c->d2h(&c->canon_segments, c->nseg.p, 4));
  HIPCHK(c, c->sync());
  c->canon_host = true;
  return DR_OK;
}

// Bring the round summaries and the canonical cone up to date with the DAG
// (the per-call path: only stale rounds are re-read).
int refresh_canon(dr_ctx *c) {
  if (!(c->memo_on()) || c->nrounds < 2) return DR_OK;
  if (int rc = refresh_rounds(c)) return rc;
  if (!c->canon_ok) {
    if (int rc = ensure_summary_bufs(c)) return rc;
    if (int rc = launch_canon(c, false, nullptr, false, true)) return rc;
  }
  return DR_OK;  // host copies of the prefixes: fetch_canon, when a host-planned path needs them
}

// Full summary pass (dr_replay): every strong row of rounds 1..T read once by
// k_summary_commit, which with nwc > 0 also decides the commits of waves
// 1..nwc (host arrays), then the canonical cone and prefixes.  Every replay
// re-reads the whole DAG; nothing carries over from earlier calls.
// parts: 1 = the row pass (k_summary_commit between its timing events), 2 = the rest
// (a replay graph holds part 2 alone), 3 = both.
int build_summary(dr_ctx *c, float *ms_summary, int nwc = 0, uint8_t *commit = nullptr, int32_t *vcount = nullptr,
                  bool host_out = true, bool fork = false, const std::function<int()> *side = nullptr,
                  bool prefix = true, int parts = 3, const ChainFuse *cf = nullptr) {
  const int T = c->nrounds - 1;
  if (T < 1) return c->fail(DR_E_STATE, "summary needs rounds 0..1 at least");
  const bool wu_fused = (c->fuse & 1) != 0;  // (the same for both parts of one replay)
  if (parts & 1) {
    if (int rc = ensure_summary_bufs(c)) return rc;
    HIPCHK(c, c->commit.ensure((size_t)std::max(nwc, 1)));
    HIPCHK(c, c->vcount.ensure((size_t)std::max(nwc, 1) * 4));
    // rows + commits and the weak unions from the weak-column keys, as the same launch's
    // last workgroups or a launch after it (on a second stream beside the row pass they
    // only queued behind its workgroups and paid a cross-stream join:
    // profiles/r02/v30_timeline.txt)
    HIPCHK(c, c->rec(6));
    HIPCHK(c, launch_summary(c, T, nwc, c->commit.as<uint8_t>(), c->vcount.as<int32_t>(), wu_fused));  // records ev[7]
  }
  if (!(parts & 2)) return DR_OK;
  ChainFuse cfk;
  if (cf && wu_fused) {  // the chain plan rides in K^cand's launch instead of the weak unions'
    cfk = *cf;
    cfk.plan_in_kcand = true;
    cf = &cfk;
  }
  const bool early = fork && side;
  if (early) HIPCHK(c, ensure_stream2(c));
  if (early) {  // stream2's work (side) needs only the rows' summaries and commits: fork here,
    // on the summary's end event when it is recorded anyway (each event costs the
    // stream ~7 us: profiles/r02/v34_timeline.txt)
    hipEvent_t fe = c->ev_fork;
    if (c->timed(7) && (parts & 1))  // (a capture forks on an event of its own)
      fe = c->ev[7];
    else
      HIPCHK(c, hipEventRecord(fe, c->stream));
    HIPCHK(c, hipStreamWaitEvent(c->stream2, fe, 0));
  }
  if (!wu_fused) HIPCHK(c, launch_weak_union(c, T, c->stream, cf));
  mark_rounds_clean(c);
  if (int rc = launch_canon(c, fork, side, early, false, prefix, true, cf)) return rc;
  if (!host_out) return DR_OK;  // planned replay: results stay on the device
  if (nwc > 0) {
    HIPCHK(c, c->d2h(commit, c->commit.p, (size_t)nwc));
    HIPCHK(c, c->d2h(vcount, c->vcount.p, (size_t)nwc * 4));
  }
  if (int rc = fetch_canon(c)) return rc;  // syncs
  if (ms_summary) {
    *ms_summary = 0;
    if (c->timed(6)) HIPCHK(c, hipEventElapsedTime(ms_summary, c->ev[6], c->ev[7]));
  }
  return DR_OK;
}

}  // namespace

namespace {
// Round summaries usable for this context's current DAG (Q_SHORTCUT), and the
// canonical cone too (Q_MERGE).
bool rounds_fresh(const dr_ctx *c) {
  return c->memo_on() && c->ndirty == 0 && c->sum_dd == c->memo_dd() && c->nrounds >= 2;
}
bool summary_fresh(const dr_ctx *c) { return rounds_fresh(c) && c->canon_ok && c->canon_T == c->nrounds - 1; }
int shortcut_flag(const dr_ctx *c) { return rounds_fresh(c) ? dr::Q_SHORTCUT : 0; }
}  // namespace

extern "C" int dr_set_leader_coin(dr_ctx *c, int mode, uint64_t seed, int k, const int32_t *table) {
  if (c) c->touch();
  if (!c) return DR_E_INVAL;
  if (int rc = set_device(c)) return rc;
  std::vector<uint16_t> L(c->h_lead.size(), 1);
  if (mode == DR_LEADER_SEEDED) {
    for (size_t w = 1; w < L.size(); w++) L[w] = (uint16_t)dr_coin_leader(seed, (int)w, c->n);
  } else if (mode == DR_LEADER_TABLE) {
    if (k < 0 || (k > 0 && !table)) return c->fail(DR_E_INVAL, "bad leader table");
    for (int w = 1; w <= k && w < (int)L.size(); w++) {
      if (table[w - 1] < 1 || table[w - 1] > c->n)
        return c->fail(DR_E_INVAL, "leader of wave %d: source %d outside [1, %d]", w, table[w - 1], c->n);
      L[w] = (uint16_t)table[w - 1];
    }
  } else if (mode != DR_LEADER_CONST1) {
    return c->fail(DR_E_INVAL, "unknown leader coin mode %d", mode);
  }
  c->h_lead = std::move(L);
  c->version++;
  HIPCHK(c, c->h2d(c->lead.p, c->h_lead.data(), c->h_lead.size() * 2));
  HIPCHK(c, c->sync());
  return DR_OK;
}

extern "C" int dr_wave_leader(const dr_ctx *c, int wave) { return c ? c->lead_src(wave) : -1; }
extern "C" int dr_replay_graph_state(const dr_ctx *c) { return c ? c->graph_state : 0; }

#ifdef DR_SWEEP_TIMING
// profiling build only: the per-query phase timings of the last k_sweep launch
// (kernels.hpp g_sweep_timing; 16 u64 per query, wall-clock ticks)
extern "C" int dr_debug_sweep_timing(uint64_t *out, int nq) {
  if (nq < 0 || nq > dr::kSweepTimingQ) return DR_E_INVAL;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(dr::g_sweep_timing), (size_t)nq * 128, 0, hipMemcpyDeviceToHost) ==
                 hipSuccess ? DR_OK : DR_E_HIP;
}
// k_canon's stamps of the last canonical cone (kernels.hpp g_canon_timing, 8 u64)
extern "C" int dr_debug_canon_timing(uint64_t *out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(dr::g_canon_timing), 64, 0, hipMemcpyDeviceToHost) == hipSuccess
             ? DR_OK : DR_E_HIP;
}
#endif

extern "C" int dr_coin_leader(uint64_t seed, int wave, int n) {
  if (n < 1) return 1;
  uint64_t z = seed + (uint64_t)(uint32_t)wave * 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  z ^= z >> 31;
  return 1 + (int)(z % (uint64_t)n);
}

extern "C" int dr_set_option(dr_ctx *c, int option, int value) {
  if (c) c->touch();
  if (!c) return DR_E_INVAL;
  c->cfg_gen++;
  if (option == DR_OPT_REPLAY_GRAPH) {
    c->replay_graph = value != 0;
    c->graph_fail = 0;
    return DR_OK;
  }
  if (option == DR_OPT_MEMO) {
    c->use_memo = value != 0;
    return DR_OK;
  }
  if (option == DR_OPT_FUSE) {
    if (value < 0 || value > 63) return c->fail(DR_E_INVAL, "DR_OPT_FUSE is a mask of bits 1, 2, 4, 8, 16, 32");
    c->fuse = value;
    return DR_OK;
  }
  if (option == DR_OPT_CALL_OVERLAP) {
    if (value < 0 || value > 2) return c->fail(DR_E_INVAL, "DR_OPT_CALL_OVERLAP is 0, 1 or 2");
    c->call_overlap = value;
    return DR_OK;
  }
  if (option == DR_OPT_DEVICE_PLAN) {
    c->plan_mode = value != 0;
    return DR_OK;
  }
  if (option == DR_OPT_COMMIT_SPLIT) {
    if (value < 0 || value > 2) return c->fail(DR_E_INVAL, "DR_OPT_COMMIT_SPLIT is 0, 1 or 2");
    c->commit_split = value;
    return DR_OK;
  }
  if (option == DR_OPT_BATCH_FORM) {
    if (value < DR_BATCH_AUTO || value > DR_BATCH_WAVE) return c->fail(DR_E_INVAL, "DR_OPT_BATCH_FORM is 0, 1 or 2");
    c->batch_form = value;
    return DR_OK;
  }
  if (option == DR_OPT_PHASE_TIMING) {
    if (value < 0 || value > 2) return c->fail(DR_E_INVAL, "DR_OPT_PHASE_TIMING is 0, 1 or 2");
    c->phase_timing = value;
    return DR_OK;
  }
  return c->fail(DR_E_INVAL, "unknown option %d", option);
}

#ifdef DR_TUNING  // tuning build only (libdagrider_gpu_timing.so, include/dagrider_tuning.h)
namespace {
// dr_profile_kernel variants of k_summary_commit (WS = 16 geometries; other
// strides run the shipped one)
template <int WS>
hipError_t launch_sv_t(dr_ctx *c, int T, int variant) {
  uint8_t *cm = c->commit.as<uint8_t>();
  int32_t *vc = c->vcount.as<int32_t>();
  const int nwc = T / 4;
  if constexpr (WS == 16) {
    switch (variant) {
      case 1: return launch_sc<WS, 512, 8, false>(c, T, nwc, cm, vc);
      case 2: return launch_sc<WS, 512, 8, true>(c, T, nwc, cm, vc);
      case 3: return launch_sc<WS, 512, 4, true>(c, T, nwc, cm, vc);
      case 4: return launch_sc<WS, 1024, 4, true>(c, T, nwc, cm, vc);
      case 5: return launch_sc<WS, 1024, 8, false>(c, T, nwc, cm, vc);
      case 6: return launch_sc<WS, 256, 8, true>(c, T, nwc, cm, vc);
      case 7: return launch_sc<WS, 1024, 2, true>(c, T, nwc, cm, vc);
      case 8: return launch_sc<WS, 512, 16, false>(c, T, nwc, cm, vc);
      case 9: return launch_sc<WS, 256, 16, false>(c, T, nwc, cm, vc);
      case 10: return launch_sc<WS, 512, 2, true>(c, T, nwc, cm, vc);
      case 11: return launch_sc<WS, 1024, 1, true>(c, T, nwc, cm, vc);
      case 12: return launch_sc<WS, 256, 4, true>(c, T, nwc, cm, vc);
      case 13: return launch_sc<WS, 1024, 4, false>(c, T, nwc, cm, vc);
      case 14: return launch_sc<WS, 1024, 2, false>(c, T, nwc, cm, vc);
      case 15: return launch_sc<WS, 1024, 1, false>(c, T, nwc, cm, vc);
      case 16: return launch_sc<WS, 512, 2, false>(c, T, nwc, cm, vc);
      case 17: return launch_sc<WS, 512, 4, false>(c, T, nwc, cm, vc);
      case 18: return launch_sc<WS, 256, 2, false>(c, T, nwc, cm, vc);
      case 19: return launch_sc<WS, 256, 4, false>(c, T, nwc, cm, vc);
    }
  }
  return launch_sc_shipped<WS>(c, T, nwc, cm, vc);
}
}  // namespace

// Tuning hook: average device time (HIP events) of `iters` launches of one
// kernel variant on the resident DAG.  kernel 0: k_summary_commit (variant 0
// shipped, 1-9 the geometries of launch_sv_t); kernel 1: streaming read of the
// strong rows (variant 0 grid-stride, 2 one block per wave's rows); kernel 2:
// the whole dr_replay summary phase (k_summary_commit + canonical cone).
extern "C" int dr_profile_kernel(dr_ctx *c, int kernel, int variant, int iters, float *avg_ms) {
  if (c) c->touch();
  if (!c || !avg_ms || iters < 1) return DR_E_INVAL;
  if (int rc = set_device(c)) return rc;
  const int T = c->nrounds - 1;
  if (T < 4) return c->fail(DR_E_STATE, "profiling needs a DAG");
  const size_t R = (size_t)T + 1;
  if (int rc = ensure_summary_bufs(c)) return rc;
  HIPCHK(c, c->commit.ensure(R));
  HIPCHK(c, c->vcount.ensure(R * 4));
  HIPCHK(c, c->edges.ensure(64));
  auto one = [&]() -> hipError_t {
    if (kernel == 0) {
      if (!c->memo_ok()) return hipErrorInvalidValue;
      switch (c->WS) {
        case 1: return launch_sv_t<1>(c, T, variant);
        case 2: return launch_sv_t<2>(c, T, variant);
        case 4: return launch_sv_t<4>(c, T, variant);
        case 8: return launch_sv_t<8>(c, T, variant);
        case 16: return launch_sv_t<16>(c, T, variant);
        case 32: return launch_sv_t<32>(c, T, variant);
      }
      return hipErrorInvalidValue;
    }
    if (kernel == 1) {
      const size_t a16 = (size_t)c->nrounds * c->n * c->WS / 2;
      if (variant == 2) {  // blocked pattern: one workgroup per 4-round wave's worth of rows
        hipLaunchKernelGGL((dr::k_stream_read_blocked<1024>), dim3(1000), dim3(1024), 0, c->stream,
                           reinterpret_cast<const dr::u64x2 *>(c->strong.p), a16, c->edges.as<u64>());
        return hipGetLastError();
      }
      hipLaunchKernelGGL((dr::k_stream_read<256>), dim3(2048), dim3(256), 0, c->stream,
                         reinterpret_cast<const dr::u64x2 *>(c->strong.p), a16, c->edges.as<u64>());
      return hipGetLastError();
    }
    return hipErrorInvalidValue;
  };
  if (kernel == 2) {
    float t = 0, tot = 0;
    for (int i = 0; i < iters; i++) {
      if (int rc = build_summary(c, &t)) return rc;
      tot += t;
    }
    *avg_ms = tot / iters;
    return DR_OK;
  }
  HIPCHK(c, one());  // warm
  HIPCHK(c, hipEventRecord(c->ev[0], c->stream));
  for (int i = 0; i < iters; i++) HIPCHK(c, one());
  HIPCHK(c, hipEventRecord(c->ev[1], c->stream));
  HIPCHK(c, c->sync());
  float ms = 0;
  HIPCHK(c, hipEventElapsedTime(&ms, c->ev[0], c->ev[1]));
  *avg_ms = ms / iters;
  return DR_OK;
}

#endif  // DR_TUNING

extern "C" int dr_exception_stats(const dr_ctx *c, int64_t *out) {
  if (!c || !out) return DR_E_INVAL;
  out[0] = c->nexc;
  out[1] = c->nbad;
  out[2] = (int64_t)c->exc_sweeps;
  out[3] = c->dreg;
  out[4] = c->nirr_up;
  out[5] = c->memo_on() ? 1 : 0;
  return DR_OK;
}

extern "C" int dr_mirror_stats(const dr_ctx *c, int64_t *out, int k) {
  if (!c || !out || k < 0) return DR_E_INVAL;
  const int64_t v[4] = {c->nrounds, (int64_t)c->h_slot_off.back(), (int64_t)c->h_wc_roff.back(),
                        (int64_t)c->h_weak_roff.back()};
  for (int i = 0; i < k && i < 4; i++) out[i] = v[i];
  return DR_OK;
}

extern "C" int dr_last_kernel_ms(const dr_ctx *c, float *ms) {
  if (!c || !ms) return DR_E_INVAL;
  *ms = c->last_commit_ms;
  return DR_OK;
}

extern "C" int dr_last_batch_form(const dr_ctx *c) { return c ? c->last_batch_form : DR_E_INVAL; }

extern "C" int dr_last_append_phases(const dr_ctx *c, float *ms4) {
  if (!c || !ms4) return DR_E_INVAL;
  std::memcpy(ms4, c->append_phases, sizeof c->append_phases);
  return DR_OK;
}

extern "C" int dr_last_batch_phases(const dr_ctx *c, float *ms4) {
  if (!c || !ms4) return DR_E_INVAL;
  for (int i = 0; i < 4; i++) ms4[i] = c->batch_phases[i];
  return DR_OK;
}

// one orderVertices pop: the popped leader's id and p.round at its delivery
struct Pop { int32_t round, source, cur_round; };

// ===========================================================================
// General graphs: every query of a mirror holding edges
// outside the round contract, on the general sweep (general.hpp).  One sweep per
// start vertex gives its whole reach set (every round, cycles included); the
// reference's functions are then bit tests on it: path() the target's bit,
// waveReady's vote the leader's bit in the strong sets of round 4w's ids, the
// chain the first present leader below in the last pushed leader's strong set,
// orderVertices the set's rows 1..p.round in slot order.
// ===========================================================================
namespace {

template <int WS>
hipError_t launch_gsweep_t(dr_ctx *c, const dr::GQuery *q, int nq, int Tg, u64 *masks, u64 *scratch, uint8_t *hit,
                           u64 *edges, const u64 *U) {
  hipLaunchKernelGGL((dr::k_gsweep<WS>), dim3(nq), dim3(256), 0, c->stream, c->view(), c->gview(), q, nq, Tg,
                     c->nrounds, masks, scratch, hit, edges, U);
  return hipGetLastError();
}
template <int WS>
hipError_t launch_gdeg_t(dr_ctx *c, const int64_t *moff, const int32_t *first, const int32_t *last, int np, int weak,
                         u64 *out) {
  hipLaunchKernelGGL((dr::k_gdeg<WS>), dim3(np), dim3(256), 0, c->stream, c->view(), c->masks.as<u64>(), moff, first,
                     last, weak, out);
  return hipGetLastError();
}
template <int WS>
hipError_t launch_gpaper_t(dr_ctx *c, const int64_t *moff, const int32_t *last, int np, int Tg, u64 *D) {
  hipLaunchKernelGGL((dr::k_gpaper<WS>), dim3(1), dim3(256), 0, c->stream, c->view(), c->masks.as<u64>(), moff, last,
                     np, Tg, D);
  return hipGetLastError();
}
#define DR_WS_SWITCH(c, call)                         \
  switch ((c)->WS) {                                  \
    case 1: { constexpr int WS_ = 1; return call; }   \
    case 2: { constexpr int WS_ = 2; return call; }   \
    case 4: { constexpr int WS_ = 4; return call; }   \
    case 8: { constexpr int WS_ = 8; return call; }   \
    case 16: { constexpr int WS_ = 16; return call; } \
    case 32: { constexpr int WS_ = 32; return call; } \
  }                                                   \
  return hipErrorInvalidValue
hipError_t launch_gsweep(dr_ctx *c, const dr::GQuery *q, int nq, int Tg, u64 *m, u64 *s, uint8_t *h, u64 *ed,
                         const u64 *U) {
  DR_WS_SWITCH(c, launch_gsweep_t<WS_>(c, q, nq, Tg, m, s, h, ed, U));
}
hipError_t launch_gdeg(dr_ctx *c, const int64_t *moff, const int32_t *first, const int32_t *last, int np, int weak,
                       u64 *out) {
  DR_WS_SWITCH(c, launch_gdeg_t<WS_>(c, moff, first, last, np, weak, out));
}
hipError_t launch_gpaper(dr_ctx *c, const int64_t *moff, const int32_t *last, int np, int Tg, u64 *D) {
  DR_WS_SWITCH(c, launch_gpaper_t<WS_>(c, moff, last, np, Tg, D));
}
#undef DR_WS_SWITCH

int gsweep_rows(const dr_ctx *c) { return std::max(c->nrounds - 1, c->irr_tmax) + 1; }

// General sweeps of qv in batches (reach rows of every query at qv[i].mask_off in
// c->masks, assigned here per batch); hits / edges to the host; on_batch(i0, i1)
// sees each batch's rows before the next overwrites them.  whole: one batch or
// DR_E_CAPACITY (callers that keep every query's rows).
int run_gsweeps(dr_ctx *c, std::vector<dr::GQuery> &qv, std::vector<uint8_t> *hits, std::vector<u64> *edges,
                const std::function<int(size_t, size_t)> &on_batch, bool whole = false) {
  const int WS = c->WS, Tg = gsweep_rows(c) - 1;
  const size_t per = (size_t)(Tg + 1) * WS, budget = (size_t)1 << 27;  // words of rows (and as many of scratch)
  const size_t bq = std::max<size_t>(1, budget / per);
  if (whole && qv.size() > bq) return c->fail(DR_E_CAPACITY, "general sweeps: %zu reach sets of %zu words exceed one batch", qv.size(), per);
  if (hits) hits->assign(qv.size(), 0);
  if (edges) edges->assign(qv.size(), 0);
  // the rows' unions U_r (valid whatever irregular edges the mirror holds): full rounds
  // skip their rows
  const u64 *U = nullptr;
  if (c->use_memo && c->nrounds >= 2) {
    if (int rc = refresh_rounds(c, true)) return rc;
    if (c->ndirty == 0 && c->sum_dd == c->memo_dd()) U = c->U.as<u64>();
  }
  for (size_t i0 = 0; i0 < qv.size(); i0 += bq) {
    const size_t i1 = std::min(qv.size(), i0 + bq), nq = i1 - i0;
    for (size_t i = i0; i < i1; i++) qv[i].mask_off = (int64_t)((i - i0) * per);
    HIPCHK(c, c->masks.ensure(nq * per * 8));
    HIPCHK(c, c->gscratch.ensure(nq * per * 8));
    const size_t o_hit = nq * sizeof(dr::GQuery), o_e = (o_hit + nq + 7) & ~(size_t)7;
    HIPCHK(c, c->gquery.ensure(o_e + nq * 8));
    char *qb = c->gquery.as<char>();
    HIPCHK(c, c->h2d(qb, qv.data() + i0, nq * sizeof(dr::GQuery)));
    uint8_t *dh = reinterpret_cast<uint8_t *>(qb + o_hit);
    u64 *de = reinterpret_cast<u64 *>(qb + o_e);
    HIPCHK(c, launch_gsweep(c, reinterpret_cast<const dr::GQuery *>(qb), (int)nq, Tg, c->masks.as<u64>(),
                            c->gscratch.as<u64>(), dh, de, U));
    if (hits) HIPCHK(c, c->d2h(hits->data() + i0, dh, nq));
    if (edges) HIPCHK(c, c->d2h(edges->data() + i0, de, nq * 8));
    HIPCHK(c, c->sync());
    if (on_batch)
      if (int rc = on_batch(i0, i1)) return rc;
  }
  return DR_OK;
}

int general_path(dr_ctx *c, int q, const int32_t *from, const int32_t *to, int strong_only, uint8_t *out) {
  const int Tg = gsweep_rows(c) - 1;
  std::vector<dr::GQuery> qv;
  std::vector<int> idx;
  for (int i = 0; i < q; i++) {
    const int fr = from[2 * i], fs = from[2 * i + 1], tr = to[2 * i], ts = to[2 * i + 1];
    if (fr == tr && fs == ts) { out[i] = 1; continue; }  // process.go:91-93
    if (fr < 0 || fr >= c->nrounds)
      return c->fail(DR_E_INVAL, "query %d: from round %d outside the DAG (Go: index out of range)", i, fr);
    out[i] = 0;
    if (fs < 1 || fs > c->n || tr < 0 || tr > Tg || ts < 1 || ts > c->n) continue;  // no edges / not an id any edge holds
    qv.push_back(dr::GQuery{fr, fs - 1, strong_only ? 1 : 0, tr, ts - 1, 1, 0, 0, c->gsweep_bottom(tr), 0});
    idx.push_back(i);
  }
  std::vector<uint8_t> hits;
  if (int rc = run_gsweeps(c, qv, &hits, nullptr, {})) return rc;
  for (size_t k = 0; k < idx.size(); k++) out[idx[k]] = hits[k];
  return DR_OK;
}

int general_reach(dr_ctx *c, int q, const int32_t *from, const int32_t *bottom, int strong_only, uint64_t *out) {
  const int W = c->W, WS = c->WS;
  std::vector<dr::GQuery> qv(q);
  std::vector<size_t> obase(q);
  size_t acc = 0;
  for (int i = 0; i < q; i++) {
    const int fs = from[2 * i + 1];
    qv[i] = dr::GQuery{from[2 * i], (fs >= 1 && fs <= c->n) ? fs - 1 : -1, strong_only ? 1 : 0, -1, -1, 1, 0, 0};
    obase[i] = acc;
    acc += (size_t)(from[2 * i] - bottom[i] + 1) * W;
  }
  std::vector<u64> tmp;
  return run_gsweeps(c, qv, nullptr, nullptr, [&](size_t i0, size_t i1) -> int {
    const size_t per = (size_t)gsweep_rows(c) * WS;
    tmp.resize((i1 - i0) * per);
    HIPCHK(c, hipMemcpy(tmp.data(), c->masks.p, tmp.size() * 8, hipMemcpyDeviceToHost));
    for (size_t i = i0; i < i1; i++)
      for (int r = bottom[i]; r <= from[2 * i]; r++)
        std::memcpy(out + obase[i] + (size_t)(r - bottom[i]) * W, &tmp[qv[i].mask_off + (size_t)r * WS], (size_t)W * 8);
    return 0;
  });
}

// waveReady's vote (process.go:326-339) for waves w0 .. w0+nw-1, all evaluable:
// vcount = the slots of round 4w whose id's strong reach set holds the leader.
int general_votes(dr_ctx *c, int w0, int nw, uint8_t *commit, int32_t *vcount) {
  const int n = c->n;
  std::vector<dr::GQuery> qv;
  std::vector<int32_t> qw;  // wave index of each query
  for (int i = 0; i < nw; i++) {
    const int w = w0 + i, r1 = 4 * (w - 1) + 1, L = c->lead_src(w), r4 = 4 * w;
    commit[i] = 0;
    vcount[i] = -1;
    if (!c->is_present(r1, L)) continue;  // leader is bottom (process.go:327-329)
    vcount[i] = 0;
    for (int s = 1; s <= n; s++)
      if (c->is_present(r4, s)) {
        qv.push_back(dr::GQuery{r4, s - 1, 1, r1, L - 1, 1, 0, 0, c->gsweep_bottom(r1), 0});
        qw.push_back(i);
      }
  }
  std::vector<uint8_t> hits;
  if (int rc = run_gsweeps(c, qv, &hits, nullptr, {})) return rc;
  std::vector<uint8_t> reach((size_t)nw * (n + 1), 0);  // (wave, source) -> the leader is in its strong set
  for (size_t k = 0; k < qv.size(); k++) reach[(size_t)qw[k] * (n + 1) + qv[k].s0 + 1] = hits[k];
  for (int i = 0; i < nw; i++) {
    if (vcount[i] < 0) continue;
    int vc = 0;
    for (uint16_t s : c->hr[4 * (w0 + i)].slots) vc += s != 0 && reach[(size_t)i * (n + 1) + s];  // every slot (:332)
    vcount[i] = vc;
    commit[i] = vc >= 2 * c->f + 1 ? 1 : 0;
  }
  return DR_OK;
}

// The leader chain of a commit of wave `wave` (process.go:341-350) above decidedWave
// `floor`: pushes (task wave first) and the strong degrees of each segment's reach set
// above the round where the next leader takes over (the last: above round(floor+1,1)).
int general_chain(dr_ctx *c, int wave, int floor, std::vector<int32_t> &push, uint64_t *edges) {
  push.assign(1, wave);
  if (edges) *edges = 0;
  if (wave - 1 < floor + 1) return DR_OK;
  if (floor < 0) return c->fail(DR_E_INVAL, "decidedWave %d < 0 (Go: waveRound(0,1) index out of range)", floor);
  const int WS = c->WS, bottom = 4 * floor + 1, T = c->nrounds - 1;
  int vr = 4 * (wave - 1) + 1, vs = c->lead_src(wave), cur = wave;
  std::vector<u64> rows;
  while (true) {
    std::vector<dr::GQuery> qv{dr::GQuery{vr, vs - 1, 1, -1, -1, 1, 0, 0, c->gsweep_bottom(bottom), 0}};
    int next = -1;
    if (int rc = run_gsweeps(c, qv, nullptr, nullptr, [&](size_t, size_t) -> int {
          const size_t per = (size_t)gsweep_rows(c) * WS;
          rows.resize(per);
          HIPCHK(c, hipMemcpy(rows.data(), c->masks.p, per * 8, hipMemcpyDeviceToHost));
          for (int w = cur - 1; w >= floor + 1 && next < 0; w--) {  // process.go:342-349
            const int r = 4 * (w - 1) + 1, L = c->lead_src(w);
            if (c->is_present(r, L) && ((rows[(size_t)r * WS + ((L - 1) >> 6)] >> ((L - 1) & 63)) & 1ULL)) next = w;
          }
          return 0;
        }))
      return rc;
    if (edges) {  // the segment's strong degrees: rows above the round the next leader restarts at
      const int lo = (next > 0 ? 4 * (next - 1) + 1 : bottom) + 1, hi = T;
      if (lo <= hi) {
        HIPCHK(c, c->gaux.ensure(64));
        int64_t mo = 0;
        int32_t fl[2] = {lo, hi};
        char *a = c->gaux.as<char>();
        HIPCHK(c, c->h2d(a, &mo, 8));
        HIPCHK(c, c->h2d(a + 8, fl, 8));
        HIPCHK(c, launch_gdeg(c, reinterpret_cast<const int64_t *>(a), reinterpret_cast<const int32_t *>(a + 8),
                              reinterpret_cast<const int32_t *>(a + 12), 1, 0, reinterpret_cast<u64 *>(a + 16)));
        u64 e = 0;
        HIPCHK(c, c->d2h(&e, a + 16, 8));
        HIPCHK(c, c->sync());
        *edges += e;
      }
    }
    if (next < 0) break;
    push.push_back(next);
    vr = 4 * (next - 1) + 1;
    vs = c->lead_src(next);
    cur = next;
  }
  return DR_OK;
}

// orderVertices (process.go:404-443) for pops in pop order: each pop's reach set
// (strong + weak) on rounds 1..min(p.round, T) in slot order; PAPER minus what the
// pops before it delivered (an id once, at its first slot).  counts, digests, edges
// (strong + weak degrees of the delivered ids) per pop; ids optional.
int general_deliver(dr_ctx *c, const std::vector<Pop> &pops, int mode, uint64_t *cnt, uint64_t *dg, uint64_t *pe,
                    int32_t *ids, int64_t ids_cap, int64_t *ids_total) {
  const int np = (int)pops.size(), WS = c->WS, T = c->nrounds - 1;
  if (ids_total) *ids_total = 0;
  if (np == 0) return DR_OK;
  std::vector<dr::GQuery> qv(np);
  for (int i = 0; i < np; i++) {
    const Pop &p = pops[i];
    const bool ok = p.round >= 0 && p.round <= T && p.source >= 1 && p.source <= c->n;
    qv[i] = dr::GQuery{ok ? p.round : 0, ok ? p.source - 1 : -1, 0, -1, -1, 1, 0, 0};
  }
  if (int rc = run_gsweeps(c, qv, nullptr, nullptr, {}, true)) return rc;  // every pop's rows stay in c->masks
  std::vector<int64_t> moff(np);
  std::vector<int32_t> first(np, 1), last(np);
  for (int i = 0; i < np; i++) {
    moff[i] = qv[i].mask_off;
    last[i] = std::min(pops[i].cur_round, T);
  }
  HIPCHK(c, c->gaux.ensure((size_t)np * 24 + 64));
  char *a = c->gaux.as<char>();
  int64_t *d_moff = reinterpret_cast<int64_t *>(a);
  int32_t *d_first = reinterpret_cast<int32_t *>(a + (size_t)np * 8), *d_last = d_first + np;
  u64 *d_e = reinterpret_cast<u64 *>(a + (size_t)np * 16);
  HIPCHK(c, c->h2d(d_moff, moff.data(), (size_t)np * 8));
  HIPCHK(c, c->h2d(d_first, first.data(), (size_t)np * 4));
  HIPCHK(c, c->h2d(d_last, last.data(), (size_t)np * 4));
  if (mode == DR_DELIVER_PAPER) {  // Alg. 3 line 54: minus the delivered set, pop by pop
    const size_t dw = (size_t)gsweep_rows(c) * WS;
    HIPCHK(c, c->dlv.ensure(dw * 8));
    HIPCHK(c, hipMemsetAsync(c->dlv.p, 0, dw * 8, c->stream));
    HIPCHK(c, launch_gpaper(c, d_moff, d_last, np, gsweep_rows(c) - 1, c->dlv.as<u64>()));
  }
  HIPCHK(c, launch_gdeg(c, d_moff, d_first, d_last, np, 1, d_e));
  HIPCHK(c, c->d2h(pe, d_e, (size_t)np * 8));
  HIPCHK(c, c->sync());
  std::vector<dr::PopDesc> pd;
  for (int i = 0; i < np; i++) {
    if (last[i] < 1) continue;
    dr::PopDesc d{};
    d.mask_off = moff[i];
    d.first = 1;
    d.last = last[i];
    d.out = i;
    d.use_k = 0;
    d.flags = mode == DR_DELIVER_PAPER ? dr::PD_FIRST_ONLY : 0;
    pd.push_back(d);
  }
  return run_emit(c, pd, np, nullptr, cnt, dg, ids, ids_cap, 0, ids_total, nullptr);
}

int general_replay(dr_ctx *c, int nw, int chain_mode, int deliver_mode, dr_replay_out *o) {
  if (int rc = general_votes(c, 1, nw, o->commit, o->vcount)) return rc;
  uint64_t ce = 0;
  for (int w = 1; w <= nw; w++)
    if (o->vcount[w - 1] >= 0) ce += c->round_deg(4 * w - 2) + c->round_deg(4 * w - 1) + c->round_deg(4 * w);
  o->commit_edges = ce;
  std::vector<Pop> pops;
  int64_t np = 0;
  uint64_t chain_e = 0;
  int last = 0;
  std::vector<int32_t> push;
  for (int w = 1; w <= nw; w++) {
    o->push_off[w - 1] = (uint32_t)np;
    if (!o->commit[w - 1]) continue;
    uint64_t e = 0;
    if (int rc = general_chain(c, w, chain_mode == DR_CHAIN_PERSISTENT ? last : 0, push, &e)) return rc;
    chain_e += e;
    last = w;
    if (np + (int64_t)push.size() > o->push_cap || !o->push_wave)
      return c->fail(DR_E_CAPACITY, "%lld pushed leaders, capacity %lld", (long long)(np + (int64_t)push.size()),
                     (long long)o->push_cap);
    for (int32_t pw : push) o->push_wave[np++] = pw;
    for (auto it = push.rbegin(); it != push.rend(); ++it)  // the stack's LIFO order
      pops.push_back(Pop{4 * (*it - 1) + 1, c->lead_src(*it), 4 * w});
  }
  o->push_off[nw] = (uint32_t)np;
  o->n_push = np;
  o->chain_edges = chain_e;
  if (!pops.empty() && (!o->pop_count || !o->pop_digest))
    return c->fail(DR_E_CAPACITY, "%zu pops, no pop outputs", pops.size());
  std::vector<uint64_t> pe(pops.size());
  int64_t tot = 0;
  const bool want_ids = o->ids && o->ids_cap > 0;
  if (int rc = general_deliver(c, pops, deliver_mode, o->pop_count, o->pop_digest, pe.data(),
                               want_ids ? o->ids : nullptr, want_ids ? o->ids_cap : 0, &tot))
    return rc;
  uint64_t de = 0;
  for (size_t i = 0; i < pops.size(); i++) {
    de += pe[i];
    if (o->pop_edges) o->pop_edges[i] = pe[i];
  }
  o->deliver_edges = de;
  o->n_ids = want_ids ? tot : 0;
  o->sweep_count = pops.size();
  if (want_ids && tot > o->ids_cap) return c->fail(DR_E_CAPACITY, "%lld delivered ids, capacity %lld", (long long)tot, (long long)o->ids_cap);
  return DR_OK;
}

}  // namespace

extern "C" int dr_path_batch(dr_ctx *c, int q, const int32_t *from, const int32_t *to, int strong_only,
                             uint8_t *out) {
  if (c) c->touch();
  if (!c) return DR_E_INVAL;
  if (q < 0 || (q > 0 && (!from || !to || !out))) return c->fail(DR_E_INVAL, "bad query arrays");
  if (int rc = prep_query(c)) return rc;
  if (c->general()) return general_path(c, q, from, to, strong_only, out);
  if (int rc = refresh_rounds(c)) return rc;
  std::vector<dr::SweepQuery> qv;
  std::vector<int> idx;
  for (int i = 0; i < q; i++) {
    const int fr = from[2 * i], fs = from[2 * i + 1], tr = to[2 * i], ts = to[2 * i + 1];
    if (fr == tr && fs == ts) { out[i] = 1; continue; }  // process.go:91-93
    if (fr < 0 || fr >= c->nrounds)
      return c->fail(DR_E_INVAL, "query %d: from round %d outside the DAG (Go: index out of range)", i, fr);
    out[i] = 0;
    if (tr < 0 || tr >= fr || ts < 1 || ts > c->n) continue;  // unreachable by construction
    if (fs < 1 || fs > c->n) continue;                         // unknown `from`: no edges
    dr::SweepQuery sq{};
    sq.top = fr;
    sq.bottom = tr;
    sq.src0 = fs - 1;
    sq.flags = (strong_only ? dr::Q_STRONG_ONLY : dr::Q_MASKS) | shortcut_flag(c);
    sq.tgt0 = ts - 1;
    qv.push_back(sq);
    idx.push_back(i);
  }
  std::vector<uint8_t> hits;
  int rc = run_sweeps(c, qv, false, nullptr, nullptr, &hits, nullptr, nullptr, nullptr,
                      [](size_t, size_t) { return 0; }, nullptr);
  if (rc) return rc;
  for (size_t k = 0; k < idx.size(); k++) out[idx[k]] = hits[k];
  return DR_OK;
}

extern "C" int dr_reach_sets(dr_ctx *c, int q, const int32_t *from, const int32_t *bottom, int strong_only,
                             uint64_t *out, size_t cap_words, size_t *out_words) {
  if (c) c->touch();
  if (!c) return DR_E_INVAL;
  if (int rc = prep_query(c)) return rc;
  if (int rc = refresh_rounds(c)) return rc;
  size_t need = 0;
  for (int i = 0; i < q; i++) {
    const int fr = from[2 * i], b = bottom[i];
    if (fr < 0 || fr >= c->nrounds || b < 0 || b > fr)
      return c->fail(DR_E_INVAL, "query %d: rounds [%d,%d] outside the DAG", i, b, fr);
    need += (size_t)(fr - b + 1) * c->W;
  }
  if (out_words) *out_words = need;
  if (need > cap_words || (!out && need)) return c->fail(DR_E_CAPACITY, "reach sets need %zu words", need);
  if (c->general()) return general_reach(c, q, from, bottom, strong_only, out);
  std::vector<dr::SweepQuery> qv(q);
  std::vector<size_t> obase(q);
  size_t acc = 0;
  for (int i = 0; i < q; i++) {
    dr::SweepQuery &s = qv[i];
    s = dr::SweepQuery{};
    s.top = from[2 * i];
    s.bottom = bottom[i];
    const int fs = from[2 * i + 1];
    s.src0 = (fs >= 1 && fs <= c->n) ? fs - 1 : -1;
    s.flags = dr::Q_MASKS | (strong_only ? dr::Q_STRONG_ONLY : 0) | shortcut_flag(c);
    s.tgt0 = -1;
    obase[i] = acc;
    acc += (size_t)(s.top - s.bottom + 1) * c->W;
  }
  const int W = c->W, WS = c->WS;
  std::vector<u64> tmp;
  return run_sweeps(c, qv, false, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                    [&](size_t i0, size_t i1) -> int {
                      size_t words = 0;
                      for (size_t i = i0; i < i1; i++) words += (size_t)(qv[i].top - qv[i].bottom + 1) * WS;
                      tmp.resize(words);
                      HIPCHK(c, hipMemcpy(tmp.data(), c->masks.p, words * 8, hipMemcpyDeviceToHost));
                      for (size_t i = i0; i < i1; i++) {
                        const int nr = qv[i].top - qv[i].bottom + 1;
                        for (int r = 0; r < nr; r++)
                          std::memcpy(out + obase[i] + (size_t)r * W, &tmp[qv[i].mask_off + (size_t)r * WS], (size_t)W * 8);
                      }
                      return 0;
                    },
                    nullptr);
}

namespace {

// Commit decisions for waves [w0, w1] (host handles waves whose round(w,4) is
// not mirrored: legal only when their leader is bottom).
// pre_sync: launches queued while the commit rule runs; behind (on the same stream): the
// host waits for the commit rule alone (ev_commit), not for them
int commit_range(dr_ctx *c, int w0, int w1, uint8_t *commit, int32_t *vcount, float *ms,
                 const std::function<int()> *pre_sync = nullptr, const std::function<int()> *behind = nullptr) {
  if (w0 < 1 || w1 < w0) return c->fail(DR_E_INVAL, "wave range [%d,%d] invalid (waves are 1-based)", w0, w1);
  int wk = w0 - 1;  // last wave the kernel can evaluate
  while (wk + 1 <= w1 && 4 * (wk + 1) < c->nrounds) wk++;
  for (int w = wk + 1; w <= w1; w++) {
    const int r1 = 4 * (w - 1) + 1;
    if (r1 >= c->nrounds) return c->fail(DR_E_INVAL, "wave %d: leader round %d not in the DAG (Go: index out of range)", w, r1);
    if (c->is_present(r1, c->lead_src(w))) return c->fail(DR_E_INVAL, "wave %d: round %d not in the DAG (Go: index out of range)", w, 4 * w);
    commit[w - w0] = 0;
    vcount[w - w0] = -1;
  }
  const int nw = wk - w0 + 1;
  if (nw <= 0) return DR_OK;
  if (c->general()) return general_votes(c, w0, nw, commit, vcount);
  // the flags and counts straight into pinned, device-mapped staging: no copy launch
  // after the commit rule (the per-call waveReady waits on this one kernel)
  // (one stage call: a second could sync and reuse the first's space)
  const size_t hv_off = ((size_t)nw + 15) & ~(size_t)15;
  void *hc = nullptr;
  HIPCHK(c, c->stage(hv_off + (size_t)nw * 4, &hc));
  void *hv = static_cast<char *>(hc) + hv_off;
  HIPCHK(c, hipEventRecord(c->ev[4], c->stream));
  HIPCHK(c, launch_commit(c, w0, nw, static_cast<uint8_t *>(hc), static_cast<int32_t *>(hv)));
  HIPCHK(c, hipEventRecord(c->ev[5], c->stream));
  if (pre_sync)  // launches the host queues while the commit rule runs
    if (int rc = (*pre_sync)()) return rc;
  if (behind && c->pend.empty() && c->h2q.empty()) {
    HIPCHK(c, hipEventRecord(c->ev_commit, c->stream));
    if (int rc = (*behind)()) return rc;
    HIPCHK(c, dr_ctx::wait_event(c->ev_commit));
  } else {
    HIPCHK(c, c->sync());
  }
  std::memcpy(commit, hc, (size_t)nw);
  std::memcpy(vcount, hv, (size_t)nw * 4);
  HIPCHK(c, hipEventElapsedTime(&c->last_commit_ms, c->ev[4], c->ev[5]));
  if (ms) *ms = c->last_commit_ms;
  return DR_OK;
}

struct ChainTask { int wave, floor; };

// Leader chains of commits (process.go:341-350).  pushes[i] receives the waves
// pushed by task i in push order (task wave first).
int run_chains(dr_ctx *c, const std::vector<ChainTask> &tasks, std::vector<std::vector<int32_t>> &pushes,
               uint64_t *edges_total, float *ms) {
  pushes.assign(tasks.size(), {});
  std::vector<dr::SweepQuery> qv;
  std::vector<int> qi;
  int64_t off = 0;
  for (size_t i = 0; i < tasks.size(); i++) {
    pushes[i].push_back(tasks[i].wave);
    if (tasks[i].wave - 1 < tasks[i].floor + 1) continue;
    if (tasks[i].floor < 0) return c->fail(DR_E_INVAL, "decidedWave %d < 0 (Go: waveRound(0,1) index out of range)", tasks[i].floor);
    dr::SweepQuery s{};
    s.top = 4 * (tasks[i].wave - 1) + 1;
    s.bottom = 4 * tasks[i].floor + 1;
    s.src0 = c->lead_src(tasks[i].wave) - 1;
    s.flags = dr::Q_CHAIN | dr::Q_STRONG_ONLY | shortcut_flag(c);
    s.out_off = (int32_t)off;
    s.tgt0 = -1;
    off += tasks[i].wave - tasks[i].floor - 1;
    qv.push_back(s);
    qi.push_back((int)i);
  }
  if (edges_total) *edges_total = 0;
  if (ms) *ms = 0;
  if (qv.empty()) return DR_OK;
  if (off > INT32_MAX) return c->fail(DR_E_INVAL, "chain output too large");
  HIPCHK(c, c->push_out.ensure((size_t)std::max<int64_t>(off, 1) * 4));
  std::vector<uint64_t> edges;
  std::vector<int32_t> pn;
  std::vector<int32_t> po((size_t)off);
  // chain queries carry no masks: one batch, whose sync also brings push_out
  int rc = run_sweeps(c, qv, false, &edges, nullptr, nullptr, &pn, c->push_out.as<int32_t>(), nullptr,
                      [](size_t, size_t) { return 0; }, ms, nullptr, [&]() -> int {
                        HIPCHK(c, c->d2h(po.data(), c->push_out.p, (size_t)off * 4));
                        return 0;
                      });
  if (rc) return rc;
  uint64_t et = 0;
  for (size_t k = 0; k < qv.size(); k++) {
    et += edges[k];
    auto &P = pushes[qi[k]];
    for (int j = 0; j < pn[k]; j++) P.push_back(po[qv[k].out_off + j]);
  }
  if (edges_total) *edges_total = et;
  return DR_OK;
}

struct SweepStats { uint64_t sweeps = 0, partial = 0, rows = 0, weak_scanned = 0, shortcut = 0; };

// Deliver pops (in pop order).
//  REF + fresh summaries: one merge sweep per distinct leader; the cone below
//    the merge round is the canonical K, counted from the canonical prefixes.
//  REF otherwise: every distinct leader's cone swept to round 0.
//  PAPER: one workgroup walks the pops in order, pruning at delivered vertices.
// With ids requested, sweeps run one per pop in pop order.
int run_deliver(dr_ctx *c, const std::vector<Pop> &pops, int mode, uint64_t *pcount, uint64_t *pdigest,
                uint64_t *pedges, SweepStats *stats, int32_t *ids, int64_t ids_cap, int64_t *ids_total,
                float *ms_sweep, float *ms_emit) {
  const int WS = c->WS;
  if (ms_sweep) *ms_sweep = 0;
  if (ms_emit) *ms_emit = 0;
  if (stats) *stats = SweepStats{};
  if (ids_total) *ids_total = 0;
  if (pops.empty()) return DR_OK;
  const bool want_ids = ids && ids_cap > 0;
  const bool paper = mode == DR_DELIVER_PAPER;
  const bool memo = !paper && summary_fresh(c);
  if (memo)
    if (int rc = fetch_canon(c)) return rc;
  std::vector<dr::SweepQuery> qv;
  std::vector<int> pop2q(pops.size());
  if (!paper && !want_ids) {
    // distinct leaders, longest first
    std::vector<int> order(pops.size());
    for (size_t i = 0; i < pops.size(); i++) order[i] = (int)i;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
      if (pops[a].round != pops[b].round) return pops[a].round > pops[b].round;
      return pops[a].source < pops[b].source;
    });
    for (size_t k = 0; k < order.size(); k++) {
      const Pop &p = pops[order[k]];
      if (k > 0 && pops[order[k - 1]].round == p.round && pops[order[k - 1]].source == p.source) {
        pop2q[order[k]] = (int)qv.size() - 1;
        continue;
      }
      dr::SweepQuery s{};
      s.top = p.round;
      s.src0 = (p.source >= 1 && p.source <= c->n) ? p.source - 1 : -1;
      qv.push_back(s);
      pop2q[order[k]] = (int)qv.size() - 1;
    }
  } else {
    if (paper) {
      HIPCHK(c, c->dlv.ensure((size_t)c->nrounds * WS * 8));
      HIPCHK(c, hipMemsetAsync(c->dlv.p, 0, (size_t)c->nrounds * WS * 8, c->stream));
    }
    for (size_t i = 0; i < pops.size(); i++) {
      dr::SweepQuery s{};
      s.top = pops[i].round;
      s.src0 = (pops[i].source >= 1 && pops[i].source <= c->n) ? pops[i].source - 1 : -1;
      s.cur_round = pops[i].cur_round;
      qv.push_back(s);
      pop2q[i] = (int)i;
    }
  }
  for (auto &s : qv) {
    s.bottom = 0;
    s.tgt0 = -1;
    s.flags = dr::Q_MASKS | (paper ? dr::Q_PRUNE : 0) | (memo ? (dr::Q_SHORTCUT | dr::Q_MERGE) : 0);
  }
  std::vector<std::vector<int>> q2pop(qv.size());
  for (size_t i = 0; i < pops.size(); i++) q2pop[pop2q[i]].push_back((int)i);
  std::vector<uint64_t> qedges, qwedges, qst;
  std::vector<int32_t> qstop;
  std::vector<uint64_t> cnt(pops.size()), dg(pops.size());
  float ms_e = 0;
  int64_t id_run = 0;
  int rc = run_sweeps(
      c, qv, paper, &qedges, &qwedges, nullptr, nullptr, nullptr, &qstop,
      [&](size_t i0, size_t i1) -> int {
        // pops served by this batch, in pop order (contiguous when ids are wanted)
        std::vector<int> pl;
        for (size_t k = i0; k < i1; k++) pl.insert(pl.end(), q2pop[k].begin(), q2pop[k].end());
        std::sort(pl.begin(), pl.end());
        std::vector<dr::PopDesc> pd;
        std::vector<uint64_t> extra(pl.size(), 0), extra_dg(pl.size(), 0);
        for (size_t t = 0; t < pl.size(); t++) {
          const Pop &p = pops[pl[t]];
          const dr::SweepQuery &s = qv[pop2q[pl[t]]];
          const int stop = memo ? qstop[pop2q[pl[t]]] : -1;
          const int last = std::min(p.cur_round, s.top);
          int own_first = 1;
          uint64_t pos0 = 0;
          if (memo) {
            if (stop >= 0) {  // merged at m = stop: rounds 1..min(m, cur) are canonical
              const int cm = std::min(stop, p.cur_round);
              if (want_ids) {
                if (cm >= 1) {
                  dr::PopDesc d{};
                  d.mask_off = 0;
                  d.pos0 = 0;
                  d.first = 1;
                  d.last = cm;
                  d.out = (int32_t)t;
                  d.use_k = 1;
                  pd.push_back(d);
                }
              } else {
                extra[t] = c->hC[cm];
                extra_dg[t] = c->hG[cm];
              }
              pos0 = c->hC[cm];
              own_first = stop + 1;
            } else {
              own_first = std::max(1, -1 - stop);  // swept to (-1-stop); rounds below it are empty
            }
          }
          if (own_first <= last) {
            dr::PopDesc d{};
            d.mask_off = s.mask_off;  // bottom = 0: the image starts at round 0
            d.pos0 = (int64_t)pos0;
            d.first = own_first;
            d.last = last;
            d.out = (int32_t)t;
            d.use_k = 0;
            d.flags = paper ? dr::PD_FIRST_ONLY : 0;  // PAPER dedups by id (Alg. 3 line 54)
            pd.push_back(d);
          }
        }
        std::vector<uint64_t> bc(pl.size()), bd(pl.size());
        int64_t tot = 0;
        int r2 = run_emit(c, pd, (int)pl.size(), extra.data(), bc.data(), bd.data(), want_ids ? ids : nullptr,
                          ids_cap, id_run, &tot, &ms_e);
        if (r2) return r2;
        id_run += tot;
        for (size_t t = 0; t < pl.size(); t++) { cnt[pl[t]] = bc[t]; dg[pl[t]] = bd[t] + extra_dg[t]; }
        return 0;
      },
      ms_sweep, &qst);
  if (rc) return rc;
  for (size_t k = 0; k < qv.size(); k++) {
    const int stop = memo ? qstop[k] : -1;
    const uint64_t canon_e = (memo && stop >= 0) ? c->hE[stop] : 0;
    if (stats) {
      stats->sweeps++;
      stats->partial += qst[4 * k + 0];
      stats->rows += qst[4 * k + 1];
      stats->weak_scanned += qst[4 * k + 2];
      stats->shortcut += qst[4 * k + 3];
    }
    for (int p : q2pop[k]) {
      pcount[p] = cnt[p];
      pdigest[p] = dg[p];
      if (pedges) pedges[p] = qedges[k] + canon_e;
    }
  }
  if (ids_total) *ids_total = id_run;
  if (ms_emit) *ms_emit = ms_e;
  return DR_OK;
}

}  // namespace

namespace {
template <int WS>
hipError_t launch_set_weak_t(dr_ctx *c, int r0, const u64 *srow, u64 *out, u64 *far) {
  constexpr int NT = sweep_block<WS>();
  const int dl = c->depth_log2();
  const size_t lds = c->sweep_lds(dl);
  hipError_t e = hipFuncSetAttribute((const void *)dr::k_set_weak<WS, NT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((dr::k_set_weak<WS, NT>), dim3(1), dim3(NT), lds, c->stream, c->view(), r0, dl, srow, out, far);
  return hipGetLastError();
}
hipError_t launch_set_weak(dr_ctx *c, int r0, const u64 *srow, u64 *out, u64 *far) {
  switch (c->WS) {
    case 1: return launch_set_weak_t<1>(c, r0, srow, out, far);
    case 2: return launch_set_weak_t<2>(c, r0, srow, out, far);
    case 4: return launch_set_weak_t<4>(c, r0, srow, out, far);
    case 8: return launch_set_weak_t<8>(c, r0, srow, out, far);
    case 16: return launch_set_weak_t<16>(c, r0, srow, out, far);
    case 32: return launch_set_weak_t<32>(c, r0, srow, out, far);
  }
  return hipErrorInvalidValue;
}

// One sweep of the buffer pass (process.go:200-234): wavefront i admits
// buffered vertex i once every predecessor is present (process.go:374-384) in
// the mirrored rounds <= cur, or was admitted earlier in the same pass by a
// buffered vertex j < i (first[] = least admitted buffer index per id of the
// buffered round span).  The 64 lanes stride the predecessor list (a vertex
// has ~2f+1 of them) and vote with __all.  first[] only falls, so repeated
// sweeps reach the sequential pass's unique fixed point.
__global__ void __launch_bounds__(256) k_buffer_admit(const u64 *__restrict__ present, int WS, int n, int lim,
                                                      int cur, int ghost_round, int rlo, int rhi, int q,
                                                      const int32_t *__restrict__ ids, const uint32_t *__restrict__ poff,
                                                      const int32_t *__restrict__ preds, uint32_t *first,
                                                      uint8_t *admit, uint32_t *changed) {
  const int i = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);  // wave-uniform
  const int lane = threadIdx.x & 63;
  if (i >= q || admit[i]) return;
  const int vr = ids[2 * i], vs = ids[2 * i + 1];
  if (vr > cur) return;  // process.go:203: stays buffered
  bool ok = true;
  for (uint32_t e = poff[i] + lane; ok && e < poff[i + 1]; e += 64) {
    const int pr = preds[2 * e], ps = preds[2 * e + 1];
    bool here = false;
    if (pr == 0 && ps == 0) here = ghost_round <= cur;  // a ghost slot {0,0} in rounds 0..cur
    else if (pr >= 0 && pr <= lim && ps >= 1 && ps <= n)
      here = (present[(size_t)pr * WS + ((ps - 1) >> 6)] >> ((ps - 1) & 63)) & 1ULL;
    if (!here && pr >= rlo && pr <= rhi && ps >= 0 && ps <= n)
      here = __atomic_load_n(&first[(size_t)(pr - rlo) * (n + 1) + ps], __ATOMIC_RELAXED) < (uint32_t)i;
    ok = here;
  }
  if (!__all(ok)) return;
  if (lane == 0) {
    admit[i] = 1;
    atomicMin(&first[(size_t)(vr - rlo) * (n + 1) + vs], (uint32_t)i);
    atomicOr(changed, 1u);
  }
}
}  // namespace

extern "C" int dr_buffer_admit(dr_ctx *c, int cur_round, int q, const int32_t *ids, const uint32_t *pred_off,
                               const int32_t *preds, uint8_t *admit) {
  if (c) c->touch();
  if (!c) return DR_E_INVAL;
  if (q < 0 || (q > 0 && (!ids || !pred_off || !admit))) return c->fail(DR_E_INVAL, "bad buffer arrays");
  if (q == 0) return DR_OK;
  const uint32_t ne = pred_off[q];
  if (pred_off[0] != 0 || (ne > 0 && !preds)) return c->fail(DR_E_INVAL, "bad pred_off/preds");
  for (int i = 0; i < q; i++)
    if (pred_off[i + 1] < pred_off[i]) return c->fail(DR_E_INVAL, "pred_off not monotone at %d", i);
  int rlo = INT32_MAX, rhi = -1;
  for (int i = 0; i < q; i++) {
    const int r = ids[2 * i], s = ids[2 * i + 1];
    if (r < 0 || s < 0 || s > c->n)
      return c->fail(DR_E_CONTRACT, "buffered vertex %d: id (%d,%d) outside rounds >= 0, sources 0..n", i, r, s);
    if (r <= cur_round) { rlo = std::min(rlo, r); rhi = std::max(rhi, r); }
  }
  std::fill(admit, admit + q, 0);
  if (rhi < 0) return DR_OK;  // every buffered vertex is ahead of the current round
  if (int rc = prep_query(c)) return rc;
  int ghost_round = INT32_MAX;
  for (int r = 0; r < c->nrounds && ghost_round == INT32_MAX; r++)
    if (c->has_ghost(r)) ghost_round = r;
  const int lim = std::min(cur_round, c->nrounds - 1);
  const size_t nfirst = (size_t)(rhi - rlo + 1) * (c->n + 1);
  const size_t b_ids = (size_t)q * 8, b_off = (size_t)(q + 1) * 4, b_pr = (size_t)std::max<uint32_t>(ne, 1) * 8;
  const size_t o_off = (b_ids + 15) & ~15ull, o_pr = (o_off + b_off + 15) & ~15ull,
               o_first = (o_pr + b_pr + 15) & ~15ull, o_adm = (o_first + nfirst * 4 + 15) & ~15ull,
               o_chg = (o_adm + q + 15) & ~15ull, total = o_chg + 16;
  HIPCHK(c, c->admit_buf.ensure(total));
  char *base = static_cast<char *>(c->admit_buf.p);
  int32_t *d_ids = reinterpret_cast<int32_t *>(base);
  uint32_t *d_off = reinterpret_cast<uint32_t *>(base + o_off);
  int32_t *d_pr = reinterpret_cast<int32_t *>(base + o_pr);
  uint32_t *d_first = reinterpret_cast<uint32_t *>(base + o_first), *d_chg = reinterpret_cast<uint32_t *>(base + o_chg);
  uint8_t *d_adm = reinterpret_cast<uint8_t *>(base + o_adm);
  HIPCHK(c, hipMemcpyAsync(d_ids, ids, b_ids, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(d_off, pred_off, b_off, hipMemcpyHostToDevice, c->stream));
  if (ne) HIPCHK(c, hipMemcpyAsync(d_pr, preds, (size_t)ne * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemsetAsync(d_first, 0xff, nfirst * 4, c->stream));
  HIPCHK(c, hipMemsetAsync(d_adm, 0, q, c->stream));
  // dependency chains inside one pass are at most q long: at most q+1 sweeps
  for (int sweep = 0; sweep <= q; sweep++) {
    uint32_t chg = 0;
    HIPCHK(c, hipMemsetAsync(d_chg, 0, 4, c->stream));
    hipLaunchKernelGGL(k_buffer_admit, dim3((q + 3) / 4), dim3(256), 0, c->stream, c->present.as<u64>(), c->WS,
                       c->n, lim, cur_round, ghost_round, rlo, rhi, q, d_ids, d_off, d_pr, d_first, d_adm, d_chg);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(&chg, d_chg, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (!chg) break;
  }
  HIPCHK(c, hipMemcpyAsync(admit, d_adm, q, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  // Go panics.  present() scans p.dag[0..p.round] (process.go:375-376): with
  // p.round >= len(p.dag) each absent predecessor it evaluates runs off the end,
  // and a vertex of a round <= p.round that stays buffered evaluated one.  An
  // admitted vertex of a round >= len(p.dag) panics at p.dag[v.id.round] (:229).
  for (int i = 0; i < q; i++) {
    const int r = ids[2 * i];
    if (r > cur_round) continue;
    if (!admit[i] && cur_round >= c->nrounds)
      return c->fail(DR_E_INVAL, "buffered vertex %d (%d,%d): present() scans p.dag[%d] of %d rounds (Go: index out of range)",
                     i, r, ids[2 * i + 1], cur_round, c->nrounds);
    if (admit[i] && r >= c->nrounds)
      return c->fail(DR_E_INVAL, "admitted vertex %d: p.dag[%d] of %d rounds (Go: index out of range)", i, r,
                     c->nrounds);
  }
  return DR_OK;
}

extern "C" int dr_set_weak_edges(dr_ctx *c, int round, int nstrong, const int32_t *strong_ids, int mode,
                                 int32_t *out_ids, size_t cap, size_t *out_n) {
  if (c) c->touch();
  if (!c) return DR_E_INVAL;
  if (out_n) *out_n = 0;
  if (round < 1 || round > c->nrounds)
    return c->fail(DR_E_INVAL, "setWeakEdges: round %d outside [1, %d] (Go: index out of range)", round, c->nrounds);
  if (mode != DR_WEAK_LITERAL && mode != DR_WEAK_PAPER) return c->fail(DR_E_INVAL, "unknown mode %d", mode);
  if (nstrong < 0 || (nstrong > 0 && !strong_ids)) return c->fail(DR_E_INVAL, "bad strong edge array");
  if (int rc = prep_query(c)) return rc;
  if (c->general())
    return c->fail(DR_E_CONTRACT, "setWeakEdges on a mirror with edges outside the round contract (App. A Q8) "
                                  "is not supported");
  const int WS = c->WS;
  std::vector<u64> srow(WS, 0);
  for (int i = 0; i < nstrong; i++) {
    const int tr = strong_ids[2 * i], ts = strong_ids[2 * i + 1];
    if (tr != round - 1 || ts < 1 || ts > c->n)
      return c->fail(DR_E_CONTRACT, "strong edge %d -> (%d,%d) must target (round-1, 1..n)", i, tr, ts);
    srow[(ts - 1) >> 6] |= 1ULL << ((ts - 1) & 63);
  }
  const int lo = 1, hi = round - 2;  // process.go:304: r = round-2 down to 1
  std::vector<u64> add;
  if (mode == DR_WEAK_PAPER && hi >= lo) {
    const size_t rows = (size_t)round + 1;
    HIPCHK(c, c->setweak.ensure((WS + 2 * rows * WS) * 8));
    u64 *d_srow = c->setweak.as<u64>(), *d_out = d_srow + WS, *d_far = d_out + rows * WS;
    HIPCHK(c, hipMemsetAsync(d_out, 0, 2 * rows * WS * 8, c->stream));
    HIPCHK(c, hipMemcpyAsync(d_srow, srow.data(), WS * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, launch_set_weak(c, round, d_srow, d_out, d_far));
    add.resize(rows * WS);
    HIPCHK(c, hipMemcpyAsync(add.data(), d_out, rows * WS * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  // emission in the reference's order: rounds hi..lo, slots in insertion order
  size_t k = 0;
  bool ghost_edge = false;  // paper: once v has a weak edge to {0,0}, path(v, {0,0}) holds
  for (int r = hi; r >= lo; r--) {
    for (const uint16_t s : c->hr[r].slots) {
      bool take;
      if (mode == DR_WEAK_LITERAL) take = s != 0;  // v.id == {0,0}: path() reaches nothing but itself
      else if (s == 0) { take = !ghost_edge; ghost_edge = true; }  // no DAG edge targets {0,0}
      else take = (add[(size_t)r * WS + ((s - 1) >> 6)] >> ((s - 1) & 63)) & 1ULL;
      if (!take) continue;
      if (out_ids && k < cap) {
        out_ids[2 * k] = s == 0 ? 0 : r;
        out_ids[2 * k + 1] = s;
      }
      k++;
    }
  }
  if (out_n) *out_n = k;
  if (k > cap && out_ids) return c->fail(DR_E_CAPACITY, "setWeakEdges: %zu ids, capacity %zu", k, cap);
  return DR_OK;
}

extern "C" int dr_wave_commit(dr_ctx *c, int w0, int w1, uint8_t *commit, int32_t *vcount) {
  if (c) c->touch();
  if (!c) return DR_E_INVAL;
  if (!commit || !vcount) return c->fail(DR_E_INVAL, "null output");
  if (int rc = prep_query(c)) return rc;
  return commit_range(c, w0, w1, commit, vcount, nullptr);
}

extern "C" int dr_wave_ready(dr_ctx *c, int wave, int decided_wave, uint8_t *commit, int32_t *vcount,
                             int32_t *pushed_waves, int cap, int *n_pushed) {
  if (c) c->touch();
  if (!c) return DR_E_INVAL;
  if (!commit || !vcount || !n_pushed) return c->fail(DR_E_INVAL, "null output");
  if (int rc = prep_query(c)) return rc;
  if (int rc = refresh_rounds(c)) return rc;
  *n_pushed = 0;
  // DR_OPT_CALL_OVERLAP: the canonical cone of the new top (what the next REF
  // dr_order_vertices merges with, refresh_canon) on stream2, forked after the round
  // summaries and launched while the commit rule runs; every later launch on the main
  // stream waits for it on the device (the join below), none on the host
  const bool spec = c->call_overlap == 2 && c->ref_seen && c->memo_on() && c->nrounds >= 2 && !c->canon_ok;
  std::function<int()> fork = [c]() -> int {
    c->s2_detached = true;
    return launch_canon(c, true, nullptr, true, true);
  };
  if (spec) {
    if (int rc = ensure_summary_bufs(c)) return rc;
    HIPCHK(c, ensure_stream2(c));
    HIPCHK(c, hipEventRecord(c->ev_fork, c->stream));
    HIPCHK(c, hipStreamWaitEvent(c->stream2, c->ev_fork, 0));
  }
  struct Join {  // (on every return below)
    dr_ctx *c;
    ~Join() {
      if (!c->s2_detached) return;
      c->s2_detached = false;
      (void)hipStreamWaitEvent(c->stream, c->ev_join, 0);
    }
  } join{c};
  // DR_OPT_CALL_OVERLAP 1, when no leader chain can follow (the previous wave is decided):
  // the canonical cone goes in behind the commit rule before it is known whether the wave
  // commits -- its launches overlap the commit rule, and the host waits for the rule alone
  const bool behind = c->call_overlap == 1 && decided_wave >= wave - 1 && c->ref_seen && c->memo_on() &&
                      c->nrounds >= 2 && !c->canon_ok;
  std::function<int()> canon_behind = [c]() -> int { return launch_canon(c, false, nullptr, false, true); };
  if (behind)
    if (int rc = ensure_summary_bufs(c)) return rc;
  if (int rc = commit_range(c, wave, wave, commit, vcount, nullptr, spec ? &fork : nullptr,
                            behind ? &canon_behind : nullptr))
    return rc;
  if (!*commit) return DR_OK;
  std::vector<std::vector<int32_t>> pushes(1);
  if (c->general()) {
    if (int rc = general_chain(c, wave, decided_wave, pushes[0], nullptr)) return rc;
  } else if (int rc = run_chains(c, {ChainTask{wave, decided_wave}}, pushes, nullptr, nullptr)) {
    return rc;
  }
  *n_pushed = (int)pushes[0].size();
  if ((int)pushes[0].size() > cap || (!pushed_waves && !pushes[0].empty()))
    return c->fail(DR_E_CAPACITY, "%zu pushed leaders, capacity %d", pushes[0].size(), cap);
  std::copy(pushes[0].begin(), pushes[0].end(), pushed_waves);
  // DR_OPT_CALL_OVERLAP 1: a commit, so orderVertices follows -- its canonical cone runs on
  // the device while the caller prepares the pops (no wait here)
  if (c->call_overlap == 1 && c->ref_seen && c->memo_on() && c->nrounds >= 2 && !c->canon_ok) {
    if (int rc = ensure_summary_bufs(c)) return rc;
    if (int rc = launch_canon(c, false, nullptr, false, true)) return rc;
  }
  return DR_OK;
}

namespace {
int deliver_planned(dr_ctx *c, const std::vector<Pop> &pops, uint64_t *pcount, uint64_t *pdigest);
}

extern "C" int dr_order_vertices(dr_ctx *c, const int32_t *stack_rs, int nstack, int cur_round, int mode,
                                 int32_t *out_ids, size_t cap, size_t *out_n, uint64_t *pop_count,
                                 uint64_t *pop_digest) {
  if (c) c->touch();
  if (!c) return DR_E_INVAL;
  if (nstack < 0 || (nstack > 0 && !stack_rs)) return c->fail(DR_E_INVAL, "bad stack");
  if (mode != DR_DELIVER_REF && mode != DR_DELIVER_PAPER) return c->fail(DR_E_INVAL, "bad mode %d", mode);
  if (int rc = prep_query(c)) return rc;
  if (out_n) *out_n = 0;
  if (nstack == 0) return DR_OK;
  if (cur_round >= c->nrounds) return c->fail(DR_E_INVAL, "p.round %d beyond the DAG (Go: index out of range)", cur_round);
  std::vector<Pop> pops;
  for (int t = nstack - 1; t >= 0; t--) {  // LIFO (stack/stack.go:23-28)
    Pop p{stack_rs[2 * t], stack_rs[2 * t + 1], cur_round};
    if (cur_round >= 1 && (p.round < 0 || p.round >= c->nrounds))
      return c->fail(DR_E_INVAL, "popped vertex round %d outside the DAG (Go: index out of range)", p.round);
    if (p.source < 1 || p.source > c->n)
      return c->fail(DR_E_CONTRACT, "popped vertex (%d,%d): source outside [1,n]", p.round, p.source);
    if (cur_round < 1) p.round = std::max(0, std::min(p.round, c->nrounds - 1));
    pops.push_back(p);
  }
  std::vector<uint64_t> cnt(pops.size()), dg(pops.size());
  int64_t tot = 0;
  if (c->general()) {  // edges outside the round contract (App. A Q8): the general sweep
    std::vector<uint64_t> pe(pops.size());
    if (int rc = general_deliver(c, pops, mode, cnt.data(), dg.data(), pe.data(), out_ids, (int64_t)cap, &tot))
      return rc;
    if (out_n) *out_n = (size_t)tot;
    if (pop_count) std::copy(cnt.begin(), cnt.end(), pop_count);
    if (pop_digest) std::copy(dg.begin(), dg.end(), pop_digest);
    if (out_ids && (size_t)tot > cap) return c->fail(DR_E_CAPACITY, "%lld delivered ids, capacity %zu", (long long)tot, cap);
    return DR_OK;
  }
  if (mode == DR_DELIVER_REF) {  // stale rounds' summaries + the canonical cone of the current top
    c->ref_seen = true;
    if (int rc = refresh_canon(c)) return rc;
  }
  // REF mode on fresh summaries without ids: planned on the device, one copy back
  int rc = 1;
  if (mode == DR_DELIVER_REF && !out_ids && c->plan_mode != 0 && summary_fresh(c))
    rc = deliver_planned(c, pops, cnt.data(), dg.data());
  if (rc == 1)
    rc = run_deliver(c, pops, mode, cnt.data(), dg.data(), nullptr, nullptr, out_ids, (int64_t)cap, &tot, nullptr,
                     nullptr);
  if (rc) return rc;
  if (!out_ids) {
    tot = 0;
    for (auto x : cnt) tot += (int64_t)x;
  }
  if (out_n) *out_n = (size_t)tot;
  if (pop_count) std::copy(cnt.begin(), cnt.end(), pop_count);
  if (pop_digest) std::copy(dg.begin(), dg.end(), pop_digest);
  if (out_ids && (size_t)tot > cap) return c->fail(DR_E_CAPACITY, "%lld delivered ids, capacity %zu", (long long)tot, cap);
  return DR_OK;
}

namespace {
// bump allocator over one device buffer (sizing pass with base == nullptr)
template <int WS>
hipError_t launch_paper_emit_t(dr_ctx *c, int nw, const int32_t *plan, const dr::SweepQuery *dq,
                               const int32_t *firstpop, const int32_t *qcut, const int32_t *qlo,
                               const uint32_t *firstK, const uint32_t *qr_off, const int32_t *qr_list, u64 *qcount,
                               u64 *qdigest, u64 *qedges) {
  hipLaunchKernelGGL((dr::k_paper_emit<WS, 512>), dim3(nw), dim3(512), 0, c->stream, c->view(), c->K.as<u64>(),
                     c->masks.as<u64>(), plan, dq, firstpop, qcut, qlo, firstK, qr_off, qr_list,
                     c->slot_off.as<uint32_t>(), c->slot_src.as<uint16_t>(), qcount, qdigest, qedges);
  return hipGetLastError();
}
hipError_t launch_paper_emit(dr_ctx *c, int nw, const int32_t *plan, const dr::SweepQuery *dq,
                             const int32_t *firstpop, const int32_t *qcut, const int32_t *qlo, const uint32_t *firstK,
                             const uint32_t *qr_off, const int32_t *qr_list, u64 *qcount, u64 *qdigest,
                             u64 *qedges) {
  switch (c->WS) {
#define DR_PE(W) \
  case W: return launch_paper_emit_t<W>(c, nw, plan, dq, firstpop, qcut, qlo, firstK, qr_off, qr_list, qcount, qdigest, qedges);
    DR_PE(1) DR_PE(2) DR_PE(4) DR_PE(8) DR_PE(16) DR_PE(32)
#undef DR_PE
  }
  return hipErrorInvalidValue;
}


template <int WS>
hipError_t launch_own_emit_t(dr_ctx *c, int nq, const int32_t *plan, const dr::SweepQuery *dq, const int32_t *stops,
                             u64 *qcount, u64 *qdigest, int32_t *qcut, const dr::PopMark &pm,
                             const dr::PopPlanArgs &pp, const int *lo_w) {
  // 256 threads per query at n <= 256 (C3: 41 -> 37 us, more queries resident); above it
  // see own_nt below (round 3: C4 at 256 12.8 -> 18.8 us, when the own ranges were longer,
  // profiles/r03/v18_timeline_*_own256.txt).  Workgroup 0: the
  // canonical prefixes G, E (every DAG length: canon_prefix_regs walks chunks); the last,
  // with pp.active: the pop plan.
  // At WS > 4 256 threads too (round 6: a query's own range is the few rounds above its cut,
  // and at 512 threads, 90 VGPRs, C4's 977 queries took two passes over the CUs: 17.0 ->
  // 14.8 us, profiles/r06/i_timeline_c4_own256.txt).  DR_OWN_NT=512: the wide block.
  static const int own_nt = getenv("DR_OWN_NT") ? atoi(getenv("DR_OWN_NT")) : 256;
  if (WS > 4 && own_nt == 256) {
    hipLaunchKernelGGL((dr::k_own_emit<WS, 256>), dim3(1 + nq + (pp.active ? 1 : 0)), dim3(256), 0, c->stream,
                       c->view(), c->masks.as<u64>(), c->memo_view().dmax, plan, dq, stops, c->Cc.as<u64>(),
                       c->slot_off.as<uint32_t>(), c->slot_src.as<uint16_t>(), qcount, qdigest, qcut, c->nrounds - 1,
                       c->RG.as<u64>(), c->CE.as<u64>(), c->Gc.as<u64>(), c->Ec.as<u64>(), pm, pp, lo_w);
    return hipGetLastError();
  }
  constexpr int NT = WS <= 4 ? 256 : 512;
  hipLaunchKernelGGL((dr::k_own_emit<WS, NT>), dim3(1 + nq + (pp.active ? 1 : 0)), dim3(NT), 0, c->stream,
                     c->view(), c->masks.as<u64>(), c->memo_view().dmax, plan, dq, stops, c->Cc.as<u64>(),
                     c->slot_off.as<uint32_t>(), c->slot_src.as<uint16_t>(), qcount, qdigest, qcut, c->nrounds - 1,
                     c->RG.as<u64>(), c->CE.as<u64>(), c->Gc.as<u64>(), c->Ec.as<u64>(), pm, pp, lo_w);
  return hipGetLastError();
}
hipError_t launch_own_emit(dr_ctx *c, int nq, const int32_t *plan, const dr::SweepQuery *dq, const int32_t *stops,
                           u64 *qcount, u64 *qdigest, int32_t *qcut, const dr::PopMark &pm,
                           const dr::PopPlanArgs &pp, const int *lo_w) {
  switch (c->WS) {
#define DR_OE(W) \
  case W: return launch_own_emit_t<W>(c, nq, plan, dq, stops, qcount, qdigest, qcut, pm, pp, lo_w);
    DR_OE(1) DR_OE(2) DR_OE(4) DR_OE(8) DR_OE(16) DR_OE(32)
#undef DR_OE
  }
  return hipErrorInvalidValue;
}

struct Carve {
  char *base = nullptr;
  size_t off = 0;
  size_t align = 256;  // a power of two
  template <class T> T *take(size_t n) {
    off = (off + align - 1) & ~(align - 1);
    T *p = reinterpret_cast<T *>(base + off);
    off += std::max<size_t>(n, 1) * sizeof(T);
    return p;
  }
};

// orderVertices (DR_DELIVER_REF, fresh summaries, no ids) planned on the device:
// one query per distinct popped leader (longest first), the delivery sweeps,
// emission segments from the sweeps' stops, per-pop totals, one copy back --
// replay_planned's delivery half for a caller-given stack.  Returns 1 when the
// bounds do not fit (the caller takes run_deliver), else a DR_* status.
int deliver_planned(dr_ctx *c, const std::vector<Pop> &pops, uint64_t *pcount, uint64_t *pdigest) {
  const int WS = c->WS, T = c->nrounds - 1, np = (int)pops.size();
  std::vector<int> order(np);
  for (int i = 0; i < np; i++) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
    if (pops[a].round != pops[b].round) return pops[a].round > pops[b].round;
    return pops[a].source < pops[b].source;
  });
  std::vector<dr::SweepQuery> qv;
  std::vector<int32_t> pq(np), pcur(np);
  int64_t mw = 0;
  for (int k = 0; k < np; k++) {
    const Pop &p = pops[order[k]];
    if (k == 0 || pops[order[k - 1]].round != p.round || pops[order[k - 1]].source != p.source) {
      dr::SweepQuery s{};
      s.top = p.round;
      s.bottom = 0;
      s.src0 = (p.source >= 1 && p.source <= c->n) ? p.source - 1 : -1;
      s.flags = dr::Q_MASKS | dr::Q_SHORTCUT | dr::Q_MERGE;
      s.mask_off = mw;
      s.tgt0 = -1;
      mw += (int64_t)(p.round + 1) * WS;
      qv.push_back(s);
    }
    pq[order[k]] = (int32_t)qv.size() - 1;
  }
  for (int i = 0; i < np; i++) pcur[i] = pops[i].cur_round;
  const int nq = (int)qv.size();
  const int64_t rb_cap = (int64_t)np * (T + 1);
  if (mw > ((int64_t)1 << 29) || rb_cap > ((int64_t)1 << 28)) return 1;
  // arena: the inputs first (one copy), then device-only scratch
  Carve cv;
  int32_t *plan = nullptr, *pop_q, *pop_cur, *dstops, *desc_of_pop;
  dr::SweepQuery *dq;
  u64 *dedges, *dwedges, *extra_c, *extra_g, *pedges, *counts, *digest, *outv;
  int64_t *item_pref;
  dr::PopDesc *pd;
  uint32_t *rcnt;
  size_t in_bytes = 0;
  for (int pass = 0; pass < 2; pass++) {
    cv.off = 0;
    plan = cv.take<int32_t>(dr::PL_N);
    dq = cv.take<dr::SweepQuery>(nq);
    pop_q = cv.take<int32_t>(np);
    pop_cur = cv.take<int32_t>(np);
    in_bytes = cv.off;
    dedges = cv.take<u64>(nq);
    dwedges = cv.take<u64>(nq);
    dstops = cv.take<int32_t>(nq);
    desc_of_pop = cv.take<int32_t>(np);
    extra_c = cv.take<u64>(np);
    extra_g = cv.take<u64>(np);
    pedges = cv.take<u64>(np);
    counts = cv.take<u64>(np);
    digest = cv.take<u64>(np);
    outv = cv.take<u64>(2 * (size_t)np);
    item_pref = cv.take<int64_t>(np + 1 + (size_t)rb_cap / kEmitRPB + np);
    pd = cv.take<dr::PopDesc>(np);
    rcnt = cv.take<uint32_t>((size_t)mw / WS);
    if (pass == 0) {
      HIPCHK(c, c->plan_arena.ensure(cv.off));
      cv.base = static_cast<char *>(c->plan_arena.p);
    }
  }
  HIPCHK(c, c->masks.ensure((size_t)mw * 8));
  {  // inputs, laid out as in the arena
    std::vector<char> hb(in_bytes, 0);
    char *db = cv.base;
    auto at = [&](void *p) { return hb.data() + (static_cast<char *>(p) - db); };
    int32_t *hp = reinterpret_cast<int32_t *>(at(plan));
    hp[dr::PL_NPUSH] = np;
    hp[dr::PL_NQD] = nq;
    hp[dr::PL_NLIVE] = nq;
    std::memcpy(at(dq), qv.data(), (size_t)nq * sizeof(dr::SweepQuery));
    std::memcpy(at(pop_q), pq.data(), (size_t)np * 4);
    std::memcpy(at(pop_cur), pcur.data(), (size_t)np * 4);
    HIPCHK(c, c->h2d(db, hb.data(), in_bytes));
  }
  SweepArgs a{};
  a.q = dq;
  a.nq = nq;
  a.seq = 0;
  a.masks = c->masks.as<u64>();
  a.edges = dedges;
  a.wedges = dwedges;
  a.stops = dstops;
  a.rcnt = rcnt;
  HIPCHK(c, launch_sweep(c, a, dr::SW_WEAK | dr::SW_MERGE));
  hipLaunchKernelGGL((dr::k_plan_emit<1024>), dim3(1), dim3(1024), 0, c->stream, pop_cur, pop_q, dq, dstops,
                     c->Cc.as<u64>(), c->Gc.as<u64>(), c->Ec.as<u64>(), dedges, kEmitRPB, rb_cap, pd, desc_of_pop,
                     extra_c, extra_g, pedges, digest, counts, item_pref, plan);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, launch_emit(c, np, 0, pd, nullptr, counts, digest, nullptr, nullptr, nullptr, 0, false,
                        plan + dr::PL_NDESC, item_pref, dr::PopDesc{}, rcnt));
  // the per-pop totals straight into pinned, device-mapped staging (no copy launch)
  void *ho = nullptr;
  HIPCHK(c, c->stage((size_t)np * 16, &ho));
  u64 *hout = static_cast<u64 *>(ho);
  hipLaunchKernelGGL((dr::k_pop_final<256>), dim3(std::max(1, std::min(64, (np + 255) / 256))), dim3(256), 0,
                     c->stream, plan, desc_of_pop, extra_c, extra_g, counts, digest, hout, hout + np);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, c->sync());
  std::memcpy(pcount, hout, (size_t)np * 8);
  std::memcpy(pdigest, hout + np, (size_t)np * 8);
  (void)outv;
  return DR_OK;
}

// Device-planned replay (memo summaries, DR_DELIVER_REF, no ids): the same
// phases as the host-planned path below, planned by replay_plan.hpp's kernels,
// with one host synchronisation.  Returns 1 when the bounds do not fit (the
// caller then takes the host-planned path), else a DR_* status.
// paper: DR_DELIVER_PAPER through the same pipeline, the delivery sweeps' masks
// turned into first-pop ownership (replay_plan.hpp k_paper_*)
// Everything dr_replay's device-planned launch sequence depends on besides the
// DAG's contents (version): options, sizes, and the buffers it names.
std::vector<uint64_t> graph_key(const dr_ctx *c, int nw, int chain_mode, bool paper, int64_t pcap) {
  auto P = [](const void *p) { return (uint64_t)reinterpret_cast<uintptr_t>(p); };
  return {c->version,          c->cfg_gen,         (uint64_t)c->nrounds, (uint64_t)nw,          (uint64_t)chain_mode,
          (uint64_t)paper,     (uint64_t)pcap,     (uint64_t)c->phase_timing, (uint64_t)c->dmax_near,
          (uint64_t)c->use_memo, (uint64_t)c->kprev_ok, (uint64_t)c->pin_cap, P(c->pin),  P(c->K.p), P(c->Kprev.p),
          P(c->plan_arena.p), P(c->plan_out.p),   P(c->masks.p),       P(c->U.p),    P(c->WU.p),  P(c->SD.p),
          P(c->commit.p),      P(c->vcount.p),     P(c->strong.p),       P(c->RG.p),   P(c->slot_src.p),
          P(c->ppref.p),       P(c->present.p),    P(c->wc_rows.p),      P(c->wc_key.p), P(c->wc_roff.p),
          P(c->weak_roff.p),   P(c->far.p),        P(c->far_roff.p),     P(c->sdeg.p), P(c->wdeg.p),
          P(c->lead.p),        P(c->slot_off.p),   P(c->dup_off.p),      P(c->dup_src.p), P(c->slot_rep.p),
          P(c->Cc.p),          P(c->CE.p),         P(c->RD.p),           P(c->Gc.p),   P(c->Ec.p),
          P(c->good.p),        P(c->nseg.p),       P(c->crbase.p),       P(c->rlo.p),  (uint64_t)c->ndups,
          P(c->view().sdx),    (uint64_t)c->dreg,  (uint64_t)c->nexc};
}

// The static delivery-query table of an nw-wave REF replay (rebuilt when the DAG, the
// leader coin or the wave count changed): pops no longer wait for the leader chains --
// a pop's cone depends on its leader alone, and every pushed leader is a present one.
int ensure_static_pops(dr_ctx *c, int nw) {
  // DR_OPT_FUSE bit 16: the fast merge (Q_FAST) where every weak slot rides in the sweep's
  // round words (dd <= DDR), at n > 512: the SW_FAST sweep's second ring costs registers
  // (C4, WS 16: 156 -> 161 VGPRs, 3 waves/SIMD either way, pop sweep 32.7 -> 29.3 us; C3, WS 4:
  // 126 -> 141, 4 -> 3 waves/SIMD, 50.6 -> 63.6 us: profiles/r06/j_*)
  const bool fast = (c->fuse & 16) && c->memo_dd() <= dr::DDR && c->WS >= 16;
  const std::vector<uint64_t> key{c->version, (uint64_t)nw, (uint64_t)c->WS, (uint64_t)(uintptr_t)c->sdq.p,
                                  (uint64_t)fast, (uint64_t)c->memo_dd()};
  if (key == c->sdq_key) return DR_OK;
  std::vector<dr::SweepQuery> q;
  std::vector<int32_t> qi((size_t)nw + 1, -1);
  int64_t moff = 0;
  for (int w = nw; w >= 1; w--) {
    const int top = 4 * (w - 1) + 1, L = c->lead_src(w);
    if (!c->is_present(top, L)) continue;
    dr::SweepQuery x{};
    x.top = top;
    x.bottom = 0;
    x.src0 = L - 1;
    x.flags = dr::Q_MASKS | dr::Q_SHORTCUT | dr::Q_MERGE | (fast ? dr::Q_FAST : 0);
    x.mask_off = moff;
    x.tgt0 = -1;
    moff += (int64_t)(top + 1) * c->WS;
    qi[w] = (int32_t)q.size();
    q.push_back(x);
  }
  HIPCHK(c, c->sdq.ensure(std::max<size_t>(q.size(), 1) * sizeof(dr::SweepQuery)));
  HIPCHK(c, c->sqidx.ensure(qi.size() * 4));
  HIPCHK(c, c->splan.ensure(dr::PL_N * 4));
  std::vector<int32_t> sp(dr::PL_N, 0);
  sp[dr::PL_NQD] = (int32_t)q.size();
  if (!q.empty()) HIPCHK(c, c->h2d(c->sdq.p, q.data(), q.size() * sizeof(dr::SweepQuery)));
  HIPCHK(c, c->h2d(c->sqidx.p, qi.data(), qi.size() * 4));
  HIPCHK(c, c->h2d(c->splan.p, sp.data(), sp.size() * 4));
  HIPCHK(c, c->flush_h2d());
  c->sdq_n = (int)q.size();
  c->sdq_fast = fast;
  c->sdq_key = {c->version, (uint64_t)nw, (uint64_t)c->WS, (uint64_t)(uintptr_t)c->sdq.p, (uint64_t)fast,
                (uint64_t)c->memo_dd()};
  return DR_OK;
}

// The upward weak edges (ru, su0, rv, tv0) for k_verify_up (rebuilt when the DAG changed).
int ensure_up_edges(dr_ctx *c) {
  const std::vector<uint64_t> key{c->version, (uint64_t)(uintptr_t)c->upe.p};
  if (key == c->upe_key) return DR_OK;
  std::vector<int32_t> e;
  for (int r = 0; r < c->nrounds; r++)
    for (uint64_t x : c->hr[r].irr) {
      const int tr = (int)((x >> 11) & 0xFFFFFu);
      if (tr < r || ((x >> 31) & 1u)) continue;
      e.insert(e.end(), {r, (int32_t)((x >> 32) & 2047u), tr, (int32_t)(x & 2047u)});
    }
  HIPCHK(c, c->upe.ensure(std::max<size_t>(e.size(), 4) * 4));
  HIPCHK(c, c->upbad.ensure(64));
  if (!e.empty()) HIPCHK(c, c->h2d(c->upe.p, e.data(), e.size() * 4));
  HIPCHK(c, c->flush_h2d());
  c->upe_n = (int)(e.size() / 4);
  c->upe_key = {c->version, (uint64_t)(uintptr_t)c->upe.p};
  return DR_OK;
}

template <int WS>
hipError_t launch_verify_up_t(dr_ctx *c, const int32_t *stops, const int32_t *qcut, const dr::PopMark &pm) {
  const int64_t n = (int64_t)c->upe_n * (c->sdq_n + 1);
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(1024, (n + 255) / 256));
  hipError_t e = hipMemsetAsync(c->upbad.p, 0, 4, c->stream);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((dr::k_verify_up<WS>), dim3(grid), dim3(256), 0, c->stream, c->K.as<u64>(), c->masks.as<u64>(),
                     c->sdq.as<dr::SweepQuery>(), c->sdq_n, stops, qcut, c->upe.as<int4>(), c->upe_n,
                     c->upbad.as<int32_t>(), pm);
  return hipGetLastError();
}
hipError_t launch_verify_up(dr_ctx *c, const int32_t *stops, const int32_t *qcut, const dr::PopMark &pm) {
  switch (c->WS) {
    case 1: return launch_verify_up_t<1>(c, stops, qcut, pm);
    case 2: return launch_verify_up_t<2>(c, stops, qcut, pm);
    case 4: return launch_verify_up_t<4>(c, stops, qcut, pm);
    case 8: return launch_verify_up_t<8>(c, stops, qcut, pm);
    case 16: return launch_verify_up_t<16>(c, stops, qcut, pm);
    case 32: return launch_verify_up_t<32>(c, stops, qcut, pm);
  }
  return hipErrorInvalidValue;
}

int replay_planned(dr_ctx *c, int nw, int chain_mode, bool paper, dr_replay_out *o) {
  const int WS = c->WS, T = c->nrounds - 1;
  const bool persistent = chain_mode == DR_CHAIN_PERSISTENT;
  const int64_t pbound = persistent ? 2 * (int64_t)nw + 1 : (int64_t)nw * (nw + 1) / 2;
  const int64_t pcap = std::max<int64_t>(1, std::min<int64_t>(o->push_cap, pbound));
  const int64_t chain_slots = persistent ? nw : (int64_t)nw * (nw - 1) / 2;
  size_t mask_words = 0;  // every wave's leader a distinct query: rounds 0..4(w-1)+1
  for (int w = 1; w <= nw; w++) mask_words += (size_t)(4 * (w - 1) + 2) * WS;
  if (mask_words > ((size_t)1 << 29) || chain_slots > INT32_MAX) return 1;
  // A replay that launches kernel by kernel starts the row pass first: the host's planning
  // below (arena, static query table, launch arguments) then runs beside it instead of
  // before it (the row pass needs only the summary buffers and the commit flags)
  const bool early = !(c->replay_graph && !c->graph_fail && c->phase_timing <= 1 && !c->shared_stream);
  if (early) {
    HIPCHK(c, c->commit.ensure((size_t)std::max(nw, 1)));
    HIPCHK(c, c->vcount.ensure((size_t)std::max(nw, 1) * 4));
    if (int rc = build_summary(c, nullptr, nw, nullptr, nullptr, false, false, nullptr, false, 1)) return rc;
  }
  // device arena
  Carve cv;
  int32_t *plan = nullptr, *task_wave, *task_q, *cpush_n, *push_out, *push_wave, *pop_wave, *pop_cur, *pop_q,
          *qidx, *dstops;
  int64_t *task_pos;
  uint32_t *push_off;
  uint8_t *seen, *hits;
  dr::SweepQuery *cq, *dq;
  u64 *cedges, *cwedges, *dedges, *dwedges, *dstats, *qcount, *qdigest, *qedges = nullptr;
  int32_t *cstops, *qcut, *firstpop = nullptr, *qlo = nullptr, *qr_list = nullptr;
  uint32_t *firstK = nullptr, *qr_cnt = nullptr, *qr_off = nullptr;
  for (int pass = 0; pass < 2; pass++) {
    cv.off = 0;
    plan = cv.take<int32_t>(dr::PL_N);
    task_wave = cv.take<int32_t>(nw);
    task_q = cv.take<int32_t>(nw);
    task_pos = cv.take<int64_t>(nw);
    cq = cv.take<dr::SweepQuery>(nw);
    dq = cv.take<dr::SweepQuery>(nw);
    cpush_n = cv.take<int32_t>(nw);
    cedges = cv.take<u64>(nw);
    cwedges = cv.take<u64>(nw);
    cstops = cv.take<int32_t>(nw);
    hits = cv.take<uint8_t>(nw);
    push_out = cv.take<int32_t>((size_t)chain_slots);
    dedges = cv.take<u64>(nw);
    dwedges = cv.take<u64>(nw);
    dstops = cv.take<int32_t>(nw);
    dstats = cv.take<u64>(4 * (size_t)nw);
    qcount = cv.take<u64>(nw);
    qdigest = cv.take<u64>(nw);
    qcut = cv.take<int32_t>(nw);
    if (paper) {
      firstpop = cv.take<int32_t>(nw);
      qlo = cv.take<int32_t>(nw);
      qedges = cv.take<u64>(nw);
      firstK = cv.take<uint32_t>((size_t)T + 2);
      qr_cnt = cv.take<uint32_t>((size_t)T + 2);
      qr_off = cv.take<uint32_t>((size_t)T + 3);
      qr_list = cv.take<int32_t>(3 * (mask_words / WS));  // (owner, mask row offset) per entry: every
                                                           // query's own range lies in its mask rows
    }
    seen = cv.take<uint8_t>(nw + 1);
    qidx = cv.take<int32_t>(nw + 1);
    push_off = cv.take<uint32_t>(nw + 1);
    push_wave = cv.take<int32_t>(pcap);
    pop_wave = cv.take<int32_t>(pcap);
    pop_cur = cv.take<int32_t>(pcap);
    pop_q = cv.take<int32_t>(pcap);
    if (pass == 0) {
      HIPCHK(c, c->plan_arena.ensure(cv.off));
      cv.base = static_cast<char *>(c->plan_arena.p);
    }
  }
  HIPCHK(c, c->masks.ensure(mask_words * 8));
  // outputs: the emitting sweep's final pass packs them into one device region, which comes back
  // in one copy (writing them straight into pinned host memory from the kernel
  // took 19.5 us, profiles/r02/v27_timeline.txt)
  const size_t h_bytes = dr::PH_N * 8 + (size_t)nw + 4 * (size_t)nw + 4 * ((size_t)nw + 1) + 4 * (size_t)pcap +
                         3 * 8 * (size_t)pcap + 8 * 256;
  HIPCHK(c, c->plan_out.ensure(h_bytes));
  Carve hv;
  hv.base = c->plan_out.as<char>();
  u64 *h_hdr = hv.take<u64>(dr::PH_N);
  uint8_t *h_commit = hv.take<uint8_t>(nw);
  int32_t *h_vcount = hv.take<int32_t>(nw);
  uint32_t *h_push_off = hv.take<uint32_t>(nw + 1);
  int32_t *h_push_wave = hv.take<int32_t>(pcap);
  u64 *h_pc = hv.take<u64>(pcap), *h_pd = hv.take<u64>(pcap), *h_pe = hv.take<u64>(pcap);
  const size_t out_bytes = hv.off;

  // REF: the delivery sweeps run from the static per-wave query table, beside the chains
  const bool stat = !paper;
  if (stat)
    if (int rc = ensure_static_pops(c, nw)) return rc;
  dr::SweepQuery *sdq = c->sdq.as<dr::SweepQuery>();
  const int32_t *splan = c->splan.as<int32_t>();
  // graph form (DR_OPT_REPLAY_GRAPH): launch the captured graph when nothing the
  // launch sequence depends on changed since it was captured; capture when this
  // call's configuration matches the previous call's (every buffer is sized then)
  enum { EAGER, CAPTURE, LAUNCH } form = EAGER;
  if (c->replay_graph && !c->graph_fail && c->phase_timing <= 1 && !c->shared_stream) {
    if (c->pin_used || !c->pend.empty() || !c->h2q.empty()) HIPCHK(c, c->sync());  // the stage starts at pin
    const std::vector<uint64_t> key = graph_key(c, nw, chain_mode, paper, pcap);
    if (c->rg_exec && key == c->rg_key)
      form = LAUNCH;
    else if (key == c->last_key && c->pin_cap >= out_bytes)
      form = CAPTURE;
  }
  // REF (stat): one stream.  The chain plan rides in the weak-union launch and the chain
  // sweeps beside the canonical walk (k_wu_plan, k_canon_chains); the delivery sweeps run
  // from the static table at once, a query live when its wave committed or a chain pushed
  // its leader (dr::PopMark); the pop plan and the canonical prefixes G, E ride in the
  // emission launch (k_own_emit).  A second stream would cost a fork and a join, ~18 us on
  // MI355X even when the other stream's work is long done (launch_probe.hip).
  // PAPER: the chains and the pop plan on stream2 beside the canonical cone, as before.
  int32_t *pushed = nullptr;
  // the commit flags' buffer before any pointer to it is taken below (build_summary would
  // size it, but the chain plan's and the pop filter's arguments are built first: on a
  // context's first replay the buffer did not exist yet)
  HIPCHK(c, c->commit.ensure((size_t)std::max(nw, 1)));
  HIPCHK(c, c->vcount.ensure((size_t)std::max(nw, 1) * 4));
  // ... and the summaries' and prefixes' buffers (the speculative prefixes' arguments hold
  // RG, SD, Gc, Ec before build_summary runs)
  if (int rc = ensure_summary_bufs(c)) return rc;
  if (stat) {
    const size_t need = ((size_t)nw + 2) * 4;
    if (c->pushed.cap < need) {
      HIPCHK(c, c->pushed.ensure(need));
      HIPCHK(c, hipMemsetAsync(c->pushed.p, 0, c->pushed.cap, c->stream));
    }
    pushed = c->pushed.as<int32_t>();
    if (++c->pop_epoch <= 0) c->pop_epoch = 1;
  }
  const dr::PopMark pmark{stat ? c->commit.as<uint8_t>() : nullptr, pushed, c->pop_epoch};
  auto enqueue = [&](char *stage, int parts) -> int {
    const int sc = dr::Q_SHORTCUT;
    SweepArgs a;
    ChainFuse cf{};
    if (stat) {
      cf.pa = dr::ChainPlanArgs{c->commit.as<uint8_t>(), c->lead.as<uint16_t>(), nw, persistent ? 1 : 0,
                                dr::Q_CHAIN | dr::Q_STRONG_ONLY | sc, task_wave, task_q, cq, plan};
      cf.xa = dr::ChainArgs{cq, plan + dr::PL_NQC, push_out, cpush_n, cedges, cwedges, hits, cstops, pmark};
      cf.emit_in_sweep = (c->fuse & 2) != 0;
      if (c->fuse & 4)  // the speculative prefixes beside the walk; k_own_emit rescans from its lowest round
        cf.sp = dr::SpecPrefix{1, c->RG.as<u64>(), c->SD.as<u64>(), c->weak_roff.as<uint32_t>(), c->Gc.as<u64>(),
                               c->Ec.as<u64>()};
    }
    std::function<int()> side = [&]() -> int {
      // 2. leader chains
      hipLaunchKernelGGL((dr::k_plan_chains<1024>), dim3(1), dim3(1024), 0, c->stream, c->commit.as<uint8_t>(),
                         c->lead.as<uint16_t>(), nw,
                         persistent ? 1 : 0, dr::Q_CHAIN | dr::Q_STRONG_ONLY | sc, task_wave, task_q, cq, plan);
      HIPCHK(c, hipGetLastError());
      a.q = cq;
      a.nq = nw;
      a.seq = 0;
      a.masks = c->masks.as<u64>();
      a.dlv = nullptr;
      a.push_out = push_out;
      a.push_n = cpush_n;
      a.edges = cedges;
      a.wedges = cwedges;
      a.hits = hits;
      a.stops = cstops;
      a.stats = nullptr;
      a.nq_dev = plan + dr::PL_NQC;
      HIPCHK(c, c->rec(0));
      HIPCHK(c, launch_chains(c, a));
      HIPCHK(c, c->rec(1));
      // 3. pops
      hipLaunchKernelGGL((dr::k_plan_pops<1024>), dim3(1), dim3(1024), 0, c->stream, nw, WS,
                         dr::Q_MASKS | dr::Q_SHORTCUT | dr::Q_MERGE, c->lead.as<uint16_t>(), task_wave, task_q, cq, cpush_n, push_out, pcap,
                         task_pos, push_off, push_wave, pop_wave, pop_cur, pop_q, seen, qidx, dq, plan,
                         (const int32_t *)nullptr, 0);
      HIPCHK(c, hipGetLastError());
      return 0;
    };
    // PAPER computes no canonical prefixes G, E; REF's come from k_own_emit's workgroup 0
    if (stat) {
      if (int rc = build_summary(c, nullptr, nw, nullptr, nullptr, false, false, nullptr, false, parts, &cf)) return rc;
    } else {
      if (int rc = build_summary(c, nullptr, nw, nullptr, nullptr, false, true, &side, false, parts)) return rc;
      c->canon_ok = false;  // no canonical prefixes G, E from this replay: a later call rebuilds the cone
    }
    // 3+4. delivery sweeps (merging with K), then each query's emission (every field: the
    // side lambda that used to fill some of them runs for PAPER only)
    a.seq = 0;
    a.masks = c->masks.as<u64>();
    a.dlv = nullptr;
    a.nq = nw;
    a.q = stat ? sdq : dq;
    a.push_out = nullptr;
    a.push_n = nullptr;  // the chains' push counts: stream2's pop plan may still read them
    a.hits = nullptr;
    a.edges = dedges;
    a.wedges = dwedges;
    a.stops = dstops;
    a.stats = dstats;
    a.nq_dev = stat ? nullptr : plan + dr::PL_NQD;  // (static: the table's count)
    if (stat) a.nq = c->sdq_n;
    a.rcnt = nullptr;
    a.pm = pmark;
    if (stat && cf.emit_in_sweep)  // the canonical re-emission beside the delivery sweeps
      a.ce = dr::CanonEmit{kCanonEmitBlocks, 0, T, c->slot_off.as<uint32_t>(), c->slot_src.as<uint16_t>(),
                           c->K.as<u64>(), c->crbase.as<uint32_t>(), c->RG.as<u64>(), c->rlo.as<int>()};
    if (stat) a.ce.xcd = (c->fuse & 8) ? 1 : 0;
    a.fast = stat && c->sdq_fast;
    // DR_OPT_FUSE bit 32 (with the speculative prefixes): the own rounds emitted by each query's
    // sweep workgroup, the G, E rescan in the final pass; no k_own_emit launch
    const bool own_in_sweep = stat && cf.sp.on && (c->fuse & 32);
    if (own_in_sweep)
      a.oe = dr::OwnEmit{1, c->Cc.as<u64>(), c->slot_off.as<uint32_t>(), c->slot_src.as<uint16_t>(), qcount, qdigest,
                         qcut};
    if (stat && cf.sp.on)  // the pop plan (the chains' pushes, the launch before) beside the delivery sweeps
      a.pp = dr::PopPlanArgs{1, nw, WS, dr::Q_MASKS | dr::Q_SHORTCUT | dr::Q_MERGE, c->lead.as<uint16_t>(), task_wave,
                             task_q, cq, cpush_n, push_out, pcap, task_pos, push_off, push_wave, pop_wave, pop_cur,
                             pop_q, seen, qidx, dq, plan, c->sqidx.as<int32_t>(), c->sdq_n};
    dr::EmitArgs em{c->slot_off.as<uint32_t>(), c->slot_src.as<uint16_t>(), c->Cc.as<u64>(), qcount, qdigest, qcut,
                          dr::FinalArgs{}};
    {
      dr::FinalArgs &f = em.fin;
      f.T = T;
      f.nw = nw;
      f.RG = c->RG.as<u64>();
      f.CE = c->CE.as<u64>();
      f.Gc = c->Gc.as<u64>();
      f.Ec = c->Ec.as<u64>();
      f.Cc = c->Cc.as<u64>();
      f.commit = c->commit.as<uint8_t>();
      f.vcount = c->vcount.as<int32_t>();
      f.push_off = push_off;
      f.push_wave = push_wave;
      f.pop_q = pop_q;
      f.pop_cur = pop_cur;
      f.dq = stat ? sdq : dq;
      f.stops = dstops;
      f.dedges = dedges;
      f.cedges = cedges;
      f.dstats = dstats;
      f.nseg = c->nseg.as<int32_t>();
      f.plan = plan;
      f.o = dr::FinalOut{h_commit, h_vcount, h_push_off, h_push_wave, h_pc, h_pd, h_pe, h_hdr};
      f.task_wave = task_wave;
      f.task_q = task_q;
      f.upbad = c->up_verify ? c->upbad.as<int32_t>() : nullptr;
      f.own_w0 = c->slice_on ? c->slice.own_w0 : 0;
      f.nprobe = c->slice_on ? c->slice.nprobe : 0;
      for (int i = 0; i < dr::kMaxProbe; i++) f.probe[i] = c->slice_on && i < c->slice.nprobe ? c->slice.probe[i] : 0;
    }
    dr::SweepQuery probe{};
    probe.flags = dr::Q_MASKS | dr::Q_SHORTCUT | dr::Q_MERGE | (stat && c->sdq_fast ? dr::Q_FAST : 0);
    if (!stat) HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_join, 0));  // PAPER: the pops planned on stream2
    HIPCHK(c, c->rec(2));
    HIPCHK(c, launch_sweep(c, a, sweep_mode(probe)));
    if (paper) {  // first-pop ownership, then each query's delivered rounds
      hipLaunchKernelGGL((dr::k_paper_plan<1024>), dim3(1), dim3(1024), 0, c->stream, T, c->memo_view().dmax, plan,
                         pop_q, dq, dstops, firstpop, qcut, qlo, firstK, qr_cnt, qr_off, qr_list);
      HIPCHK(c, hipGetLastError());
      HIPCHK(c, launch_paper_emit(c, nw, plan, dq, firstpop, qcut, qlo, firstK, qr_off, qr_list, qcount, qdigest,
                                  qedges));
      em.fin.firstpop = firstpop;
      em.fin.qedges = qedges;
    } else {  // REF: own rounds above the cut; workgroup 0 the canonical prefixes G, E, the last the pop plan
      dr::PopPlanArgs pp{1, nw, WS, dr::Q_MASKS | dr::Q_SHORTCUT | dr::Q_MERGE, c->lead.as<uint16_t>(), task_wave,
                         task_q, cq, cpush_n, push_out, pcap, task_pos, push_off, push_wave, pop_wave, pop_cur,
                         pop_q, seen, qidx, dq, plan, c->sqidx.as<int32_t>(), c->sdq_n};
      if (cf.sp.on) pp.active = 0;  // (the delivery sweeps' launch planned the pops)
      if (!own_in_sweep)
        HIPCHK(c, launch_own_emit(c, c->sdq_n, splan, sdq, dstops, qcount, qdigest, qcut, pmark, pp,
                                  cf.sp.on ? c->nseg.as<int32_t>() + 1 : nullptr));
      else
        em.fin.lo_w = c->nseg.as<int32_t>() + 1;
      if (c->up_verify) HIPCHK(c, launch_verify_up(c, dstops, qcut, pmark));  // the upward edges against the cones
    }
    HIPCHK(c, c->rec(3));
    // 5. per-pop totals and outputs (the canonical prefixes came from the sweep launch's extra workgroup)
    hipLaunchKernelGGL((dr::k_replay_final<1024>), dim3(1), dim3(1024), 0, c->stream, em);
    HIPCHK(c, hipGetLastError());
    if (stage) {  // graph: the outputs into pinned memory inside the graph
      const dr::CopySeg sg{c->plan_out.as<uint8_t>(), reinterpret_cast<uint8_t *>(stage), out_bytes};
      HIPCHK(c, c->launch_copies(&sg, 1));
    }
    return DR_OK;
  };  // enqueue
  char *hb = nullptr;
  bool enqueued = false;
  if (form != EAGER)  // the row pass, timed, ahead of the graph
    if (int rc = build_summary(c, nullptr, nw, nullptr, nullptr, false, true, nullptr, false, 1)) return rc;
  if (form == CAPTURE) {
    hipError_t e = hipStreamBeginCapture(c->stream, hipStreamCaptureModeRelaxed);
    int rc = e == hipSuccess ? enqueue(c->pin, 2) : DR_E_HIP;
    hipGraph_t g = nullptr;
    if (e == hipSuccess) {
      const hipError_t e2 = hipStreamEndCapture(c->stream, &g);
      if (e2 != hipSuccess) e = e2;
    }
    hipGraphExec_t x = nullptr;
    if (rc == DR_OK && e == hipSuccess && g) e = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
    if (g) (void)hipGraphDestroy(g);
    if (rc != DR_OK || e != hipSuccess || !x) {  // eager from here on, this call included
      std::fprintf(stderr, "dagrider: replay graph capture failed (%s; %s); launching kernel by kernel\n",
                   hipGetErrorString(e), rc != DR_OK ? c->err.c_str() : "launch sequence ok");
      (void)hipGetLastError();
      if (x) (void)hipGraphExecDestroy(x);
      c->graph_fail = 1;
      if (int rc2 = enqueue(nullptr, 2)) return rc2;  // after the row pass already launched
      enqueued = true;
      form = EAGER;
    } else {
      if (c->rg_exec) (void)hipGraphExecDestroy(c->rg_exec);
      c->rg_exec = x;
      c->rg_key = graph_key(c, nw, chain_mode, paper, pcap);  // after the capture's own K <-> Kprev swap
      form = LAUNCH;
    }
  } else if (form == LAUNCH) {  // the host state a captured replay leaves behind
    mark_rounds_clean(c);
    c->kprev_ok = true;
    c->canon_dd = c->memo_dd();
    c->canon_lo = INT_MAX;
    c->canon_T = T;
    c->canon_host = false;
    c->canon_ok = !paper;
  }
  if (form == LAUNCH) {
    HIPCHK(c, hipGraphLaunch(c->rg_exec, c->stream));
    HIPCHK(c, hipEventRecord(c->ev_sync, c->stream));
    HIPCHK(c, hipEventSynchronize(c->ev_sync));  // (a blocking wait: no host core spinning while the graph runs)
    hb = c->pin;
    c->graph_state = 1;
  } else {
    if (!enqueued)
      if (int rc = enqueue(nullptr, early ? 2 : 3)) return rc;
    c->plan_host.resize(out_bytes);
    HIPCHK(c, c->d2h(c->plan_host.data(), c->plan_out.p, out_bytes));
    HIPCHK(c, c->sync());
    hb = c->plan_host.data();
    c->graph_state = c->graph_fail ? -1 : 0;
  }
  c->last_key = graph_key(c, nw, chain_mode, paper, pcap);
  {  // device addresses -> the same offsets in the host copy
    char *db = c->plan_out.as<char>();
    auto H = [&](auto *p) { return reinterpret_cast<decltype(p)>(hb + (reinterpret_cast<char *>(p) - db)); };
    h_hdr = H(h_hdr);
    h_commit = H(h_commit);
    h_vcount = H(h_vcount);
    h_push_off = H(h_push_off);
    h_push_wave = H(h_push_wave);
    h_pc = H(h_pc);
    h_pd = H(h_pd);
    h_pe = H(h_pe);
  }
  // outputs
  o->ms_summary = o->ms_chain = o->ms_deliver = o->ms_emit = 0;
  if (c->timed(6)) HIPCHK(c, hipEventElapsedTime(&o->ms_summary, c->ev[6], c->ev[7]));
  if (c->timed(0)) {  // (REF: the chains run inside the canonical walk's launch, not timed apart)
    if (!stat) HIPCHK(c, hipEventElapsedTime(&o->ms_chain, c->ev[0], c->ev[1]));
    HIPCHK(c, hipEventElapsedTime(&o->ms_deliver, c->ev[2], c->ev[3]));  // sweeps + emission + final pass
  }
  std::memcpy(o->commit, h_commit, (size_t)nw);
  std::memcpy(o->vcount, h_vcount, (size_t)nw * 4);
  c->canon_segments = (int32_t)(int64_t)h_hdr[dr::PH_NSEG];
  o->canon_segments = c->canon_segments;
  uint64_t ce = 0;
  for (int w = 1; w <= nw; w++)
    if (o->vcount[w - 1] >= 0) ce += c->round_deg(4 * w - 2) + c->round_deg(4 * w - 1) + c->round_deg(4 * w);
  o->commit_edges = ce;
  o->chain_edges = h_hdr[dr::PH_CHAIN_E];
  const int64_t np = (int64_t)h_hdr[dr::PH_NPUSH];
  o->n_push = np;
  if (h_hdr[dr::PH_CAPERR] == 2) return c->fail(DR_E_STATE, "replay planner: segment bound exceeded");
  if (h_hdr[dr::PH_CAPERR] == 3) return c->fail(DR_E_STATE, "replay planner: a pop below its leader's round");
  if (h_hdr[dr::PH_CAPERR] || np > o->push_cap)
    return c->fail(DR_E_CAPACITY, "%lld pushed leaders, capacity %lld", (long long)np, (long long)o->push_cap);
  std::memcpy(o->push_off, h_push_off, ((size_t)nw + 1) * 4);
  std::memcpy(o->push_wave, h_push_wave, (size_t)np * 4);
  std::memcpy(o->pop_count, h_pc, (size_t)np * 8);
  std::memcpy(o->pop_digest, h_pd, (size_t)np * 8);
  if (o->pop_edges) std::memcpy(o->pop_edges, h_pe, (size_t)np * 8);
  o->deliver_edges = h_hdr[dr::PH_DELIVER_E];
  o->sweep_count = h_hdr[dr::PH_NQD];
  o->sweep_partial = h_hdr[dr::PH_PARTIAL];
  o->sweep_row_bytes = h_hdr[dr::PH_ROWS];
  o->sweep_weak_scanned = h_hdr[dr::PH_WEAK];
  o->sweep_shortcut = h_hdr[dr::PH_SHORT];
  o->n_ids = 0;
  if (c->up_verify && h_hdr[dr::PH_UPBAD] > 0) return 2;  // an upward edge changes a cone: the general sweep
  if (c->slice_on) {
    dr_slice_out &so = c->slice_res;
    so = dr_slice_out{};
    for (int i = 0; i < c->slice.nprobe; i++) {
      so.C[i] = h_hdr[dr::PH_PROBE + i];
      so.G[i] = h_hdr[dr::PH_PROBE + dr::kMaxProbe + i];
      so.E[i] = h_hdr[dr::PH_PROBE + 2 * dr::kMaxProbe + i];
    }
    const int64_t ms = (int64_t)h_hdr[dr::PH_MINSTOP];
    so.min_stop = ms >= INT_MAX ? INT_MAX : (int32_t)ms;
    so.own_chain_edges = h_hdr[dr::PH_OWN_CE];
  }
  return DR_OK;
}
}  // namespace

extern "C" int dr_replay(dr_ctx *c, int nwaves, int chain_mode, int deliver_mode, dr_replay_out *o) {
  if (c) c->touch();
  if (!c) return DR_E_INVAL;
  if (!o || !o->commit || !o->vcount || !o->push_off) return c->fail(DR_E_INVAL, "null output");
  if (nwaves < 1 || 4 * nwaves >= c->nrounds) return c->fail(DR_E_INVAL, "nwaves %d needs rounds 0..%d mirrored", nwaves, 4 * nwaves);
  if (chain_mode != DR_CHAIN_LITERAL && chain_mode != DR_CHAIN_PERSISTENT) return c->fail(DR_E_INVAL, "bad chain mode");
  if (deliver_mode != DR_DELIVER_REF && deliver_mode != DR_DELIVER_PAPER) return c->fail(DR_E_INVAL, "bad deliver mode");
  if (int rc = prep_query(c, true)) return rc;
  if (c->slice_on) {  // a slice replays on the device-planned memo path alone (its outputs come from there)
    if (chain_mode != DR_CHAIN_PERSISTENT || deliver_mode != DR_DELIVER_REF)
      return c->fail(DR_E_STATE, "a sliced context replays persistent chains with REF delivery only");
    if (c->general() || !c->memo_on() || c->plan_mode == 0 || (o->ids && o->ids_cap > 0) || !o->push_wave ||
        !o->pop_count || !o->pop_digest)
      return c->fail(DR_E_STATE, "a sliced context needs the memoized device-planned replay (no ids, every output)");
    if (c->slice.own_w0 > nwaves) return c->fail(DR_E_INVAL, "slice: own_w0 %d > nwaves %d", c->slice.own_w0, nwaves);
    for (int i = 0; i < c->slice.nprobe; i++)
      if (c->slice.probe[i] >= c->nrounds) return c->fail(DR_E_INVAL, "slice: probe round %d beyond the mirror", c->slice.probe[i]);
  }
  o->ms_commit = o->ms_chain = o->ms_deliver = o->ms_emit = o->ms_summary = 0;
  o->sweep_count = o->sweep_partial = o->sweep_row_bytes = o->sweep_weak_scanned = o->sweep_shortcut = 0;
  o->n_ids = 0;
  o->canon_segments = -1;
  if (c->general()) {
    // weak edges to the same or a later round (App. A Q8): the memo replay on the regular
    // graph, then a check that no such edge changes a cone it computed (k_verify_up)
    if (c->up_verifiable() && deliver_mode == DR_DELIVER_REF && c->use_memo && c->plan_mode != 0 &&
        !(o->ids && o->ids_cap > 0) && o->push_wave && o->pop_count && o->pop_digest) {
      c->up_verify = true;
      int rc = ensure_up_edges(c);
      if (rc == DR_OK) rc = replay_planned(c, nwaves, chain_mode, false, o);
      c->up_verify = false;
      c->canon_ok = false;  // (the cone is the regular graph's: the general paths never read it)
      if (rc == DR_OK) {
        c->last_path = 1;
        return DR_OK;
      }
      if (rc != 1 && rc != 2) return rc;
      c->last_path = rc == 2 ? 2 : 3;
    } else {
      c->last_path = 3;
    }
    return general_replay(c, nwaves, chain_mode, deliver_mode, o);
  }
  c->last_path = 0;
  if (c->plan_mode != 0 && c->memo_on() && !(o->ids && o->ids_cap > 0) && o->push_wave &&
      o->pop_count && o->pop_digest) {
    const int rc = replay_planned(c, nwaves, chain_mode, deliver_mode == DR_DELIVER_PAPER, o);
    if (rc != 1) return rc;
  }
  // 0+1. round summaries + canonical cone, fused with the commit decisions of
  // every wave (one pass over the DAG per replay); without summaries, k_commit
  if (c->memo_on()) {
    if (int rc = build_summary(c, &o->ms_summary, nwaves, o->commit, o->vcount)) return rc;
    o->canon_segments = c->canon_segments;
  } else if (int rc = commit_range(c, 1, nwaves, o->commit, o->vcount, &o->ms_commit)) {
    return rc;
  }
  uint64_t ce = 0;
  for (int w = 1; w <= nwaves; w++)
    if (o->vcount[w - 1] >= 0) ce += c->round_deg(4 * w - 2) + c->round_deg(4 * w - 1) + c->round_deg(4 * w);
  o->commit_edges = ce;
  // 2. chains
  std::vector<ChainTask> tasks;
  int last = 0;
  for (int w = 1; w <= nwaves; w++)
    if (o->commit[w - 1]) {
      tasks.push_back(ChainTask{w, chain_mode == DR_CHAIN_PERSISTENT ? last : 0});
      last = w;
    }
  std::vector<std::vector<int32_t>> pushes;
  if (int rc = run_chains(c, tasks, pushes, &o->chain_edges, &o->ms_chain)) return rc;
  int64_t np = 0;
  for (auto &p : pushes) np += (int64_t)p.size();
  o->n_push = np;
  if (np > o->push_cap || !o->push_wave || !o->pop_count || !o->pop_digest)
    return c->fail(DR_E_CAPACITY, "%lld pushed leaders, capacity %lld", (long long)np, (long long)o->push_cap);
  // 3. pops
  std::vector<Pop> pops;
  int64_t at = 0;
  size_t t = 0;
  for (int w = 1; w <= nwaves; w++) {
    o->push_off[w - 1] = (uint32_t)at;
    if (t < tasks.size() && tasks[t].wave == w) {
      for (int32_t pw : pushes[t]) o->push_wave[at++] = pw;
      for (auto it = pushes[t].rbegin(); it != pushes[t].rend(); ++it)
        pops.push_back(Pop{4 * (*it - 1) + 1, c->lead_src(*it), 4 * w});
      t++;
    }
  }
  o->push_off[nwaves] = (uint32_t)at;
  int64_t tot = 0;
  std::vector<uint64_t> pe(pops.size());
  SweepStats st;
  int rc = run_deliver(c, pops, deliver_mode, o->pop_count, o->pop_digest, pe.data(), &st, o->ids, o->ids_cap,
                       &tot, &o->ms_deliver, &o->ms_emit);
  if (rc) return rc;
  o->sweep_count = st.sweeps;
  o->sweep_partial = st.partial;
  o->sweep_row_bytes = st.rows;
  o->sweep_weak_scanned = st.weak_scanned;
  o->sweep_shortcut = st.shortcut;
  uint64_t de = 0;
  for (size_t i = 0; i < pops.size(); i++) {
    de += pe[i];
    if (o->pop_edges) o->pop_edges[i] = pe[i];
  }
  o->deliver_edges = de;
  o->n_ids = tot;
  return DR_OK;
}

// ===========================================================================
// batch of independent replays
// ===========================================================================
namespace {
// the fused small-DAG path (batch.hpp) covers this context's DAG
bool small_ok(const dr_ctx *c, int nwaves) {
  return c->n <= 128 && nwaves <= 64 && c->nfar == 0 && c->dmax_near < 32 && c->ndups == 0 && c->nirr == 0;
}

template <int D, bool PAPER, bool PERSIST>
hipError_t launch_small_t(const dr_ctx *c, const dr::SmallJob *jobs, int nj, int nw) {
  const size_t lds = dr::small_lds_bytes(D, nw);
  static std::atomic<int> seen[kLdsDevs] = {};
  hipError_t e = lds_limit((const void *)dr::k_replay_small<D, PAPER, PERSIST>, seen, c->dev, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((dr::k_replay_small<D, PAPER, PERSIST>), dim3(nj), dim3(dr::kSmallNT), lds, c->stream, jobs, nj,
                     nw);
  return hipGetLastError();
}
template <int D>
hipError_t launch_small_d(const dr_ctx *c, const dr::SmallJob *jobs, int nj, int nw, int persistent, int paper) {
  if (paper) return persistent ? launch_small_t<D, true, true>(c, jobs, nj, nw)
                               : launch_small_t<D, true, false>(c, jobs, nj, nw);
  return persistent ? launch_small_t<D, false, true>(c, jobs, nj, nw)
                    : launch_small_t<D, false, false>(c, jobs, nj, nw);
}
template <bool PAPER, bool PERSIST>
hipError_t launch_small_1w_t(const dr_ctx *c, const dr::SmallJob *jobs, int nj, int nw, int rsl) {
  const size_t lds = dr::small1w_lds_bytes<PAPER, PERSIST>(rsl);
  static std::atomic<int> seen[kLdsDevs] = {};
  hipError_t e = lds_limit((const void *)dr::k_replay_small_1w<PAPER, PERSIST>, seen, c->dev, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((dr::k_replay_small_1w<PAPER, PERSIST>), dim3(nj), dim3(64), lds, c->stream, jobs, nj, nw,
                     rsl);
  return hipGetLastError();
}
// one wavefront per DAG (batch1w.hpp); rsl = ring slots = largest weak delta + 1
hipError_t launch_small_1w(const dr_ctx *c, const dr::SmallJob *jobs, int nj, int nw, int persistent, int paper,
                           int dmax) {
  const int rsl = dmax + 1;
  if (paper) return persistent ? launch_small_1w_t<true, true>(c, jobs, nj, nw, rsl)
                               : launch_small_1w_t<true, false>(c, jobs, nj, nw, rsl);
  return persistent ? launch_small_1w_t<false, true>(c, jobs, nj, nw, rsl)
                    : launch_small_1w_t<false, false>(c, jobs, nj, nw, rsl);
}
// one workgroup per DAG (batch.hpp); D = ring slots, a power of two above the largest weak delta
hipError_t launch_small(const dr_ctx *c, const dr::SmallJob *jobs, int nj, int nw, int persistent, int paper,
                        int dmax) {
  const int need = next_pow2(dmax + 1);
  if (need <= 8) return launch_small_d<8>(c, jobs, nj, nw, persistent, paper);
  if (need <= 16) return launch_small_d<16>(c, jobs, nj, nw, persistent, paper);
  return launch_small_d<32>(c, jobs, nj, nw, persistent, paper);
}
}  // namespace

namespace {
// dr_replay_batch (views == nullptr: results copied into outs) and dr_replay_batch_view
// (views: pointers into the copied-back region; outs holds only the capacities)
int replay_batch_impl(dr_ctx *const *ctxs, int nctx, int nwaves, int chain_mode, int deliver_mode,
                      dr_replay_out *outs, dr_replay_view *views) {
  if (!ctxs || nctx < 1 || !outs) return DR_E_INVAL;
  for (int i = 0; i < nctx; i++)
    if (!ctxs[i]) return DR_E_INVAL;
  for (int i = 0; i < nctx; i++)
    if (ctxs[i]->slice_on) return ctxs[0]->fail(DR_E_STATE, "context %d is sliced (dr_set_slice): dr_replay only", i);
  dr_ctx *c0 = ctxs[0];
  // the fused launch reads every member's mirror on the first context's stream: appends
  // still in flight on a member's own stream finish first
  for (int i = 0; i < nctx; i++)
    if (ctxs[i]->async_pending) {
      if (int rc = set_device(ctxs[i])) return rc;
      HIPCHK(ctxs[i], ctxs[i]->sync());
    }
  const auto h0 = std::chrono::steady_clock::now();
  // each output's caller-set fields, commit .. ids_cap
  constexpr size_t kKey = offsetof(dr_replay_out, n_push);
  dr_ctx::BatchPlan &P = c0->batch_plan;
  bool hit = P.valid && P.nw == nwaves && P.chain_mode == chain_mode && P.deliver_mode == deliver_mode &&
             P.ctxs.size() == (size_t)nctx && std::memcmp(P.ctxs.data(), ctxs, sizeof(dr_ctx *) * nctx) == 0;
  for (int i = 0; hit && i < nctx; i++)
    hit = P.gens[i] == ctxs[i]->gen && std::memcmp(P.out_keys.data() + kKey * i, &outs[i], kKey) == 0;
  const int nw = nwaves, T = 4 * (nw - 1) + 1;
  if (!hit) {
    P.valid = false;
    bool fused = true;
    int dmax = 1;
    for (int i = 0; i < nctx; i++) {
      dr_ctx *c = ctxs[i];
      dr_replay_out *o = &outs[i];
      if (c->dev != c0->dev) return c0->fail(DR_E_INVAL, "batch contexts on devices %d and %d", c0->dev, c->dev);
      if (!o->commit || !o->vcount || !o->push_off) return c0->fail(DR_E_INVAL, "null output (context %d)", i);
      if (nwaves < 1 || 4 * nwaves >= c->nrounds)
        return c0->fail(DR_E_INVAL, "context %d: nwaves %d needs rounds 0..%d mirrored", i, nwaves, 4 * nwaves);
      for (int j = 0; j < i && nctx <= 64; j++)
        if (ctxs[j] == c) return c0->fail(DR_E_INVAL, "context %d repeated in the batch", i);
      if (!small_ok(c, nwaves) || (o->ids && o->ids_cap > 0)) fused = false;
      dmax = std::max(dmax, c->dmax_near);
    }
    if (chain_mode != DR_CHAIN_LITERAL && chain_mode != DR_CHAIN_PERSISTENT)
      return c0->fail(DR_E_INVAL, "bad chain mode");
    if (deliver_mode != DR_DELIVER_REF && deliver_mode != DR_DELIVER_PAPER)
      return c0->fail(DR_E_INVAL, "bad deliver mode");
    if (!fused && views) return c0->fail(DR_E_INVAL, "dr_replay_batch_view: the batch does not run fused");
    if (!fused) {  // general shapes: one dr_replay per context (all on the GPU)
      for (int i = 0; i < nctx; i++)
        if (int rc = dr_replay(ctxs[i], nwaves, chain_mode, deliver_mode, &outs[i])) {
          if (ctxs[i] != c0) c0->err = "context " + std::to_string(i) + ": " + ctxs[i]->err;
          return rc;
        }
      return DR_OK;
    }
    if (int rc = set_device(c0)) return rc;
    const int64_t pbound = chain_mode == DR_CHAIN_PERSISTENT ? nw : (int64_t)nw * (nw + 1) / 2;
    // device arena: per job scratch + outputs, then the job table
    Carve cv;
    std::vector<dr::SmallJob> jobs(nctx);
    // scratch of every job first, then every job's outputs in one region: only that
    // region comes back to the host (C5: ~5 MB instead of the 1.3 GB arena)
    size_t out0 = 0, out1 = 0;
    dr::SmallJob *jt = nullptr;
    for (int pass = 0; pass < 2; pass++) {
      cv.off = 0;
      for (int i = 0; i < nctx; i++) {
        dr_ctx *c = ctxs[i];
        dr::SmallJob &J = jobs[i];
        J.cone = cv.take<u64>((size_t)(T + 1) * dr::kConeRecWords);
        J.sufl = cv.take<uint32_t>(65 * 64);
        // per slot of rounds 0..T (workgroup form) or per (round, vertex) (wave form)
        J.deg = cv.take<uint32_t>(std::max<size_t>(c->h_slot_off[T + 1], (size_t)(T + 1) * c->n));
      }
      cv.off = (cv.off + 255) & ~(size_t)255;
      out0 = cv.off;
      cv.align = 16;  // the output region comes back whole: no padding between small arrays
      for (int i = 0; i < nctx; i++) {
        dr::SmallJob &J = jobs[i];
        const int64_t pcap = std::max<int64_t>(1, std::min<int64_t>(outs[i].push_wave ? outs[i].push_cap : 0, pbound));
        J.push_cap = (int32_t)pcap;
        J.commit = cv.take<uint8_t>(nw);
        J.vcount = cv.take<int32_t>(nw);
        J.push_off = cv.take<uint32_t>(nw + 1);
        J.push_wave = cv.take<int32_t>(pcap);
        J.pop_count = cv.take<u64>(pcap);
        J.pop_digest = cv.take<u64>(pcap);
        J.pop_edges = cv.take<u64>(pcap);
        J.totals = cv.take<u64>(4);
      }
      out1 = cv.off;
      cv.align = 256;
      jt = cv.take<dr::SmallJob>(nctx);
      if (pass == 0) {
        HIPCHK(c0, c0->batch_arena.ensure(cv.off));
        cv.base = c0->batch_arena.as<char>();
      }
    }
    for (int i = 0; i < nctx; i++) {
      dr_ctx *c = ctxs[i];
      dr::SmallJob &J = jobs[i];
      J.strong = c->strong.as<u64>();
      J.present = c->present.as<u64>();
      J.wc_key = c->wc_key.as<uint32_t>();
      J.wc_rows = c->wc_rows.as<u64>();
      J.wc_roff = c->wc_roff.as<uint32_t>();
      J.wdeg = c->wdeg.as<uint16_t>();
      J.sdeg = c->sdeg.as<uint16_t>();
      J.slot_off = c->slot_off.as<uint32_t>();
      J.slot_src = c->slot_src.as<uint16_t>();
      J.lead = c->lead.as<uint16_t>();
      J.n = c->n;
      J.WS = c->WS;
      J.quorum = 2 * c->f + 1;
    }
    // appends are synchronous (dr_append_rounds_*), so every DAG is resident; the
    // job table goes up only when it differs from the arena's (a repeated batch:
    // same contexts, buffers and arena)
    const size_t jb = jobs.size() * sizeof(dr::SmallJob);
    if (c0->batch_jobs.size() != jobs.size() || std::memcmp(c0->batch_jobs.data(), jobs.data(), jb) != 0) {
      HIPCHK(c0, c0->h2d(jt, jobs.data(), jb));
      c0->batch_jobs.swap(jobs);
    }
    P.nw = nwaves;
    P.chain_mode = chain_mode;
    P.deliver_mode = deliver_mode;
    P.dmax = dmax;
    P.out0 = out0;
    P.out1 = out1;
    P.jobs_at = (size_t)(reinterpret_cast<char *>(jt) - c0->batch_arena.as<char>());
    P.ctxs.assign(ctxs, ctxs + nctx);
    P.gens.resize(nctx);
    for (int i = 0; i < nctx; i++) P.gens[i] = ctxs[i]->gen;
    P.out_keys.resize(kKey * nctx);
    for (int i = 0; i < nctx; i++) std::memcpy(P.out_keys.data() + kKey * i, &outs[i], kKey);
    P.valid = true;
  } else if (int rc = set_device(c0)) {
    return rc;
  }
  const std::vector<dr::SmallJob> &jobs = c0->batch_jobs;
  const size_t out0 = P.out0, out1 = P.out1;
  const dr::SmallJob *jt = reinterpret_cast<const dr::SmallJob *>(c0->batch_arena.as<char>() + P.jobs_at);
  const auto h1 = std::chrono::steady_clock::now();
  const int persistent = chain_mode == DR_CHAIN_PERSISTENT, paper = deliver_mode == DR_DELIVER_PAPER;
  HIPCHK(c0, hipEventRecord(c0->ev[0], c0->stream));
  // small_ok: dmax < 32.  The wave form when the CUs each hold many DAGs (throughput),
  // the workgroup form when they hold few (each DAG's critical path bounds the launch)
  if (c0->cu_count <= 0) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c0->dev) != hipSuccess || cus <= 0)
      cus = 256;
    c0->cu_count = cus;
  }
  const bool wave_form = c0->batch_form == DR_BATCH_WAVE ||
                         (c0->batch_form == DR_BATCH_AUTO && nctx > 6 * c0->cu_count);
  c0->last_batch_form = wave_form ? DR_BATCH_WAVE : DR_BATCH_WORKGROUP;
  HIPCHK(c0, wave_form ? launch_small_1w(c0, jt, nctx, nw, persistent, paper, P.dmax)
                       : launch_small(c0, jt, nctx, nw, persistent, paper, P.dmax));
  HIPCHK(c0, hipEventRecord(c0->ev[1], c0->stream));
  // results: one bulk copy of the output region of the arena
  char *host = nullptr;
  HIPCHK(c0, c0->batch_host(out1 - out0, &host));
  // (DR_BATCH_COPY=dma: the DMA engine; default: k_copy's workgroups write the pinned, device-mapped region)
  static const bool dma = getenv("DR_BATCH_COPY") && std::strcmp(getenv("DR_BATCH_COPY"), "dma") == 0;
  if (dma) {
    HIPCHK(c0, hipMemcpyAsync(host, c0->batch_arena.as<char>() + out0, out1 - out0, hipMemcpyDeviceToHost, c0->stream));
  } else {
    const dr::CopySeg sg{reinterpret_cast<const uint8_t *>(c0->batch_arena.as<char>() + out0),
                         reinterpret_cast<uint8_t *>(host), out1 - out0};
    HIPCHK(c0, c0->launch_copies(&sg, 1));
  }
  HIPCHK(c0, hipEventRecord(c0->ev[2], c0->stream));
  HIPCHK(c0, hipStreamSynchronize(c0->stream));
  const auto h2 = std::chrono::steady_clock::now();
  float ms = 0, ms_copy = 0;
  (void)hipEventElapsedTime(&ms, c0->ev[0], c0->ev[1]);
  (void)hipEventElapsedTime(&ms_copy, c0->ev[1], c0->ev[2]);
  auto at = [&](const void *dev) {
    return host + (reinterpret_cast<const char *>(dev) - (c0->batch_arena.as<char>() + out0));
  };
  // unpack every context's outputs (one thread: no faster with more on the GPU box
  // (round 2, v67), the copies are memory-bound)
  int bad = -1;
  int64_t bad_np = 0;
  for (int i = 0; i < nctx; i++) {
    const dr::SmallJob &J = jobs[i];
    dr_replay_out *o = &outs[i];
    const u64 *tot = reinterpret_cast<const u64 *>(at(J.totals));
    const int64_t np = (int64_t)tot[3];
    if (views) {  // in place: pointers into the copied-back region
      dr_replay_view &v = views[i];
      v.commit = reinterpret_cast<const uint8_t *>(at(J.commit));
      v.vcount = reinterpret_cast<const int32_t *>(at(J.vcount));
      v.push_off = reinterpret_cast<const uint32_t *>(at(J.push_off));
      v.push_wave = reinterpret_cast<const int32_t *>(at(J.push_wave));
      v.pop_count = reinterpret_cast<const uint64_t *>(at(J.pop_count));
      v.pop_digest = reinterpret_cast<const uint64_t *>(at(J.pop_digest));
      v.pop_edges = reinterpret_cast<const uint64_t *>(at(J.pop_edges));
      v.n_push = np;
      v.commit_edges = tot[0];
      v.chain_edges = tot[1];
      v.deliver_edges = tot[2];
      v.ms_deliver = ms;
      if (np > o->push_cap && bad < 0) {
        bad = i;
        bad_np = np;
      }
      continue;
    }
    std::memcpy(o->commit, at(J.commit), nw);
    std::memcpy(o->vcount, at(J.vcount), 4 * (size_t)nw);
    std::memcpy(o->push_off, at(J.push_off), 4 * (size_t)(nw + 1));
    o->n_push = np;
    o->n_ids = 0;
    o->commit_edges = tot[0];
    o->chain_edges = tot[1];
    o->deliver_edges = tot[2];
    o->ms_commit = o->ms_chain = o->ms_emit = o->ms_summary = 0;
    o->ms_deliver = ms;  // the whole fused replay kernel
    o->canon_segments = -1;
    o->sweep_count = o->sweep_partial = o->sweep_row_bytes = o->sweep_weak_scanned = o->sweep_shortcut = 0;
    if (np > o->push_cap || !o->push_wave || !o->pop_count || !o->pop_digest) {
      if (bad < 0) {
        bad = i;
        bad_np = np;
      }
      continue;
    }
    std::memcpy(o->push_wave, at(J.push_wave), 4 * (size_t)np);
    std::memcpy(o->pop_count, at(J.pop_count), 8 * (size_t)np);
    std::memcpy(o->pop_digest, at(J.pop_digest), 8 * (size_t)np);
    if (o->pop_edges) std::memcpy(o->pop_edges, at(J.pop_edges), 8 * (size_t)np);
  }
  // the call's host phases (dr_last_batch_phases on the first context; every output's
  // ms_* fields keep their device meaning: ms_deliver = the fused kernel, the rest 0)
  auto msd = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
    return std::chrono::duration<float, std::milli>(b - a).count();
  };
  c0->batch_phases[0] = msd(h0, h1);
  c0->batch_phases[1] = msd(h1, h2);
  c0->batch_phases[2] = ms_copy;
  c0->batch_phases[3] = msd(h2, std::chrono::steady_clock::now());
  if (bad >= 0)
    return c0->fail(DR_E_CAPACITY, "context %d: %lld pushed leaders, capacity %lld", bad, (long long)bad_np,
                    (long long)outs[bad].push_cap);
  return DR_OK;
}
}  // namespace

extern "C" int dr_replay_batch(dr_ctx *const *ctxs, int nctx, int nwaves, int chain_mode, int deliver_mode,
                               dr_replay_out *outs) {
  return replay_batch_impl(ctxs, nctx, nwaves, chain_mode, deliver_mode, outs, nullptr);
}

extern "C" int dr_replay_batch_view(dr_ctx *const *ctxs, int nctx, int nwaves, int chain_mode, int deliver_mode,
                                    int64_t push_cap, dr_replay_view *views) {
  if (!ctxs || nctx < 1 || !views || push_cap < 1 || !ctxs[0]) return DR_E_INVAL;
  // capacities only: the outputs' pointers are never written in view mode (a stable
  // array per first context, so a repeated batch reuses its plan)
  std::vector<dr_replay_out> &outs = ctxs[0]->view_outs;
  static uint8_t dummy[8];
  if (outs.size() != (size_t)nctx) outs.assign(nctx, dr_replay_out{});
  for (dr_replay_out &o : outs) {
    o.commit = dummy;
    o.vcount = reinterpret_cast<int32_t *>(dummy);
    o.push_off = reinterpret_cast<uint32_t *>(dummy);
    o.push_wave = reinterpret_cast<int32_t *>(dummy);
    o.pop_count = reinterpret_cast<uint64_t *>(dummy);
    o.pop_digest = reinterpret_cast<uint64_t *>(dummy);
    o.pop_edges = reinterpret_cast<uint64_t *>(dummy);
    o.push_cap = push_cap;
  }
  return replay_batch_impl(ctxs, nctx, nwaves, chain_mode, deliver_mode, outs.data(), views);
}

extern "C" int dr_set_slice(dr_ctx *c, const dr_slice_cfg *cfg) {
  if (c) c->touch();
  if (!c) return DR_E_INVAL;
  if (int rc = set_device(c)) return rc;
  const uint64_t old_base = c->slice_on ? c->slice.pos_base : 0;
  if (!cfg) {
    c->slice_on = false;
    c->slice = dr_slice_cfg{};
  } else {
    if (cfg->round_offset < 0 || cfg->seeded_top < 0 || cfg->seeded_top >= std::max(1, c->nrounds) ||
        cfg->own_w0 < 0 || cfg->nprobe < 0 || cfg->nprobe > dr::kMaxProbe)
      return c->fail(DR_E_INVAL, "bad slice configuration");
    for (int i = 0; i < cfg->nprobe; i++)
      if (cfg->probe[i] < 0) return c->fail(DR_E_INVAL, "slice probe %d: negative round", i);
    c->slice_on = true;
    c->slice = *cfg;
  }
  c->slice_res = dr_slice_out{};
  c->cfg_gen++;          // a captured replay graph is stale
  c->canon_ok = false;   // positions and digests change with the base and the key offset
  c->kprev_ok = false;
  const uint64_t base = c->slice_on ? c->slice.pos_base : 0;
  if (base != old_base && !c->h_ppref.empty()) {  // positions start at the new base: every round's prefix
    for (u64 &x : c->h_ppref) x = x - old_base + base;
    HIPCHK(c, c->h2d(c->ppref.as<u64>(), c->h_ppref.data(), c->h_ppref.size() * 8));
    HIPCHK(c, c->sync());
  }
  return DR_OK;
}

extern "C" int dr_slice_result(const dr_ctx *c, dr_slice_out *out) {
  if (!c || !out) return DR_E_INVAL;
  if (!c->slice_on) return DR_E_STATE;
  *out = c->slice_res;
  return DR_OK;
}

extern "C" int dr_last_replay_path(const dr_ctx *c) { return c ? c->last_path : DR_E_INVAL; }
