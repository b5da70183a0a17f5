// replay_plan.hpp -- device-side planning of dr_replay (memo + DR_DELIVER_REF).
//
// The host-planned replay (engine.hip: run_chains / run_deliver) returns to the
// CPU after the commit pass, after the leader chains and after the delivery
// sweeps, to turn each phase's results into the next phase's queries.  These
// single-workgroup kernels do that planning on the device, so a whole replay is
// one stream of launches and one host synchronisation:
//
//   k_summary_commit, k_weak_union   round summaries, commits, speculative
//                                    canonical digests
//   k_kcand, k_canon, k_emit_ids     canonical cone, re-emission from the first
//                                    non-full round
//   k_plan_chains     commit[] -> leader-chain queries   (process.go:341-350)
//   k_sweep (chains)
//   k_plan_pops       pushes -> leadersStack pops, distinct-leader queries
//                     (process.go:404-412: pops run top first)
//   k_sweep (delivery, SW_EMIT: merge with the canonical cone, emit the own
//                     rounds; one extra workgroup: canonical prefixes G, E)
//   k_replay_final    per-pop totals, outputs (kernels.hpp replay_final_block)
//
// (k_plan_emit / k_pop_final serve the per-call dr_order_vertices path.)
// Every rule here restates the host planner line for line (same floors, same
// query order), so both paths produce identical replays;
// tests/test_gpu_parity.py runs both.
#pragma once
#include "kernels.hpp"
#include <climits>

namespace dr {

// Two exclusive scans over one workgroup at once (one set of barriers); s holds
// 2 * NT/64 slots; every thread calls.
template <int NT>
__device__ __forceinline__ void block_scan2_excl(int64_t &a, int64_t &b, int64_t *s, int64_t &ta, int64_t &tb) {
  constexpr int NW = NT / 64;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int64_t x = a, y = b;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t u = __shfl_up(x, off), v = __shfl_up(y, off);
    if (lane >= off) {
      x += u;
      y += v;
    }
  }
  if (lane == 63) {
    s[wid] = x;
    s[NW + wid] = y;
  }
  __syncthreads();
  if (wid == 0) {
    int64_t t = lane < NW ? s[lane] : 0, z = lane < NW ? s[NW + lane] : 0;
#pragma unroll
    for (int off = 1; off < NW; off <<= 1) {
      const int64_t u = __shfl_up(t, off), v = __shfl_up(z, off);
      if (lane >= off) {
        t += u;
        z += v;
      }
    }
    if (lane < NW) {
      s[lane] = t;
      s[NW + lane] = z;
    }
  }
  __syncthreads();
  ta = s[NW - 1];
  tb = s[2 * NW - 1];
  a = (wid ? s[wid - 1] : 0) + x - a;
  b = (wid ? s[NW + wid - 1] : 0) + y - b;
  __syncthreads();
}

// K consecutive items per thread (item tid*K + j of the chunk): their exclusive
// prefixes in ex[], the chunk total returned.  s: 2 * NT/64 slots.
template <int NT, int K>
__device__ __forceinline__ int64_t block_scan_items(const int64_t (&v)[K], int64_t (&ex)[K], int64_t *s) {
  int64_t sum = 0, zero = 0, tot, tz;
#pragma unroll
  for (int j = 0; j < K; j++) {
    ex[j] = sum;
    sum += v[j];
  }
  block_scan2_excl<NT>(sum, zero, s, tot, tz);
#pragma unroll
  for (int j = 0; j < K; j++) ex[j] += sum;
  return tot;
}
// the same for two item sequences at once
template <int NT, int K>
__device__ __forceinline__ void block_scan2_items(const int64_t (&va)[K], const int64_t (&vb)[K], int64_t (&ea)[K],
                                                  int64_t (&eb)[K], int64_t *s, int64_t &ta, int64_t &tb) {
  int64_t sa = 0, sb = 0;
#pragma unroll
  for (int j = 0; j < K; j++) {
    ea[j] = sa;
    eb[j] = sb;
    sa += va[j];
    sb += vb[j];
  }
  block_scan2_excl<NT>(sa, sb, s, ta, tb);
#pragma unroll
  for (int j = 0; j < K; j++) {
    ea[j] += sa;
    eb[j] += sb;
  }
}

// Planning kernels take kPlanK consecutive items per thread: one pass of
// barriers covers NT * kPlanK waves (C3's 2500 waves in one pass at NT = 1024).
constexpr int kPlanK = 4;

// Committed waves -> tasks (wave, floor) -> leader-chain queries.  Persistent
// decidedWave: floor = the previous committed wave; literal: 0.  A task with
// wave - floor >= 2 walks rounds 4(w-1)+1 .. 4 floor + 1 and may push up to
// wave - floor - 1 leaders at out_off.
template <int NT>
__device__ __forceinline__ void plan_chains_body(const uint8_t *__restrict__ commit, const uint16_t *__restrict__ lead,
                                                 int nw, int persistent, int qflags, int32_t *__restrict__ task_wave,
                                                 int32_t *__restrict__ task_q, SweepQuery *__restrict__ cq,
                                                 int32_t *__restrict__ plan) {
  constexpr int K = kPlanK, CH = NT * K;
  __shared__ int64_t s[2 * (NT / 64)];
  const int tid = threadIdx.x;
  int64_t c0 = 0, c1 = 0, c2 = 0;  // running totals (block-uniform)
  for (int w0 = 0; w0 < nw; w0 += CH) {
    int64_t f[K], ex[K];
#pragma unroll
    for (int j = 0; j < K; j++) {
      const int w = w0 + tid * K + j;
      f[j] = (w < nw && commit[w]) ? 1 : 0;
    }
    const int64_t tot = block_scan_items<NT, K>(f, ex, s);
#pragma unroll
    for (int j = 0; j < K; j++)
      if (f[j]) task_wave[c0 + ex[j]] = w0 + tid * K + j + 1;
    c0 += tot;
  }
  __syncthreads();  // task_wave written
  const int ntask = (int)c0;
  for (int t0 = 0; t0 < ntask; t0 += CH) {
    int w[K], fl[K];
    int64_t len[K], has[K], qi[K], off[K];
#pragma unroll
    for (int j = 0; j < K; j++) {
      const int t = t0 + tid * K + j;
      w[j] = fl[j] = 0;
      len[j] = has[j] = 0;
      if (t < ntask) {
        w[j] = task_wave[t];
        fl[j] = (persistent && t > 0) ? task_wave[t - 1] : 0;
        len[j] = w[j] - fl[j] - 1;
        has[j] = len[j] >= 1 ? 1 : 0;
        if (!has[j]) len[j] = 0;
      }
    }
    int64_t tq, tl;
    block_scan2_items<NT, K>(has, len, qi, off, s, tq, tl);
#pragma unroll
    for (int j = 0; j < K; j++) {
      const int t = t0 + tid * K + j;
      if (t < ntask) task_q[t] = has[j] ? (int32_t)(c1 + qi[j]) : -1;
      if (has[j]) {
        SweepQuery q{};
        q.top = 4 * (w[j] - 1) + 1;
        q.bottom = 4 * fl[j] + 1;
        q.src0 = lead[w[j]] - 1;
        q.flags = qflags;
        q.mask_off = 0;
        q.out_off = (int32_t)(c2 + off[j]);
        q.tgt0 = -1;
        cq[c1 + qi[j]] = q;
      }
    }
    c1 += tq;
    c2 += tl;
  }
  if (tid == 0) {
    plan[PL_NTASK] = ntask;
    plan[PL_NQC] = (int32_t)c1;
    plan[PL_CAPERR] = 0;
    plan[PL_NQD] = 0;
    plan[PL_NLIVE] = 0;
    plan[PL_NDESC] = 0;
  }
}

template <int NT>
__global__ __launch_bounds__(NT) void k_plan_chains(const uint8_t *__restrict__ commit, const uint16_t *__restrict__ lead,
                                                    int nw, int persistent, int qflags, int32_t *__restrict__ task_wave,
                                                    int32_t *__restrict__ task_q, SweepQuery *__restrict__ cq,
                                                    int32_t *__restrict__ plan) {
  plan_chains_body<NT>(commit, lead, nw, persistent, qflags, task_wave, task_q, cq, plan);
}

// The round summaries' weak unions and speculative digests (k_weak_union, four rounds a
// workgroup) and, in the grid's last workgroup, the leader-chain plan (plan_chains_body):
// the chains' queries need only the commits, so they are ready when the canonical walk's
// launch starts its chain workgroups (k_canon_chains).
struct ChainPlanArgs {
  const uint8_t *commit;
  const uint16_t *lead;
  int nw, persistent, qflags;
  int32_t *task_wave, *task_q;
  SweepQuery *cq;
  int32_t *plan;
};
template <int WS>
__global__ __launch_bounds__(256) void k_wu_plan(DagView g, int T, int dd, u64 *__restrict__ WU,
                                                 const u64 *__restrict__ ppref, const uint32_t *__restrict__ slot_off,
                                                 const uint16_t *__restrict__ slot_src, u64 *__restrict__ RG,
                                                 const ChainPlanArgs pa) {
  if (blockIdx.x == gridDim.x - 1) {
    plan_chains_body<256>(pa.commit, pa.lead, pa.nw, pa.persistent, pa.qflags, pa.task_wave, pa.task_q, pa.cq, pa.plan);
    return;
  }
  extern __shared__ __attribute__((aligned(16))) u64 wu_lds[];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = (int)blockIdx.x * 4 + wid + 1;  // one wave per round
  if (r > T) return;  // wave-uniform
  weak_union_round<WS>(g, r, dd, WU, wu_lds + (size_t)wid * dd * WS, ppref, slot_off, slot_src, RG, lane);
}

// K^cand (kcand_body, one wave per round) and, in the grid's last workgroup, the
// leader-chain plan: with the weak unions inside the row pass's launch (WUArgs), the
// commits are final when this launch starts.
template <int WS>
__global__ __launch_bounds__(256) void k_kcand_plan(DagView g, MemoView mv, int T, u64 *__restrict__ K,
                                                    uint8_t *__restrict__ good, u64 *__restrict__ CE,
                                                    u64 *__restrict__ RD, int *__restrict__ rlo, int lo,
                                                    const u64 *__restrict__ ppref, u64 *__restrict__ Cc,
                                                    uint32_t *__restrict__ crbase, const ChainPlanArgs pa) {
  if (blockIdx.x == gridDim.x - 1) {
    plan_chains_body<256>(pa.commit, pa.lead, pa.nw, pa.persistent, pa.qflags, pa.task_wave, pa.task_q, pa.cq, pa.plan);
    return;
  }
  kcand_body<WS>(g, mv, T, K, good, CE, RD, rlo, lo, ppref, Cc, crbase);
}

// Pushes (task wave, then its chain's pushes in push order) -> pops in pop
// order (each task's pushes reversed, process.go:406-412), push_off per wave,
// and one delivery query per distinct leader, highest round first, with
// cumulative mask images (rounds 0..top).  qidx_static (REF): the delivery
// queries were swept already from the static table of every wave whose leader is
// present (no dependence on the chains); a pop takes its leader wave's entry.
template <int NT>
__device__ __forceinline__ void plan_pops_body(int nw, int WS, int qflags, const uint16_t *__restrict__ lead,
                                                  const int32_t *__restrict__ task_wave,
                                                  const int32_t *__restrict__ task_q,
                                                  const SweepQuery *__restrict__ cq,
                                                  const int32_t *__restrict__ push_n,
                                                  const int32_t *__restrict__ push_out, int64_t pcap,
                                                  int64_t *__restrict__ task_pos, uint32_t *__restrict__ push_off,
                                                  int32_t *__restrict__ push_wave, int32_t *__restrict__ pop_wave,
                                                  int32_t *__restrict__ pop_cur, int32_t *__restrict__ pop_q,
                                                  uint8_t *__restrict__ seen, int32_t *__restrict__ qidx,
                                                  SweepQuery *__restrict__ dq, int32_t *__restrict__ plan,
                                                  const int32_t *__restrict__ qidx_static,
                                                  int nqd_static) {
  constexpr int K = kPlanK, CH = NT * K;
  __shared__ int64_t s[2 * (NT / 64)];
  const int tid = threadIdx.x;
  const int ntask = plan[PL_NTASK];
  for (int i = tid; i <= nw; i += NT) seen[i] = 0;
  int64_t np = 0;  // running total (block-uniform)
  for (int t0 = 0; t0 < ntask; t0 += CH) {
    int64_t cnt[K], ex[K];
#pragma unroll
    for (int j = 0; j < K; j++) {
      const int t = t0 + tid * K + j;
      const int q = t < ntask ? task_q[t] : -1;
      cnt[j] = t < ntask ? 1 + (q >= 0 ? push_n[q] : 0) : 0;
    }
    const int64_t tot = block_scan_items<NT, K>(cnt, ex, s);
#pragma unroll
    for (int j = 0; j < K; j++) {
      const int t = t0 + tid * K + j;
      if (t < ntask) task_pos[t] = np + ex[j];
    }
    np += tot;
  }
  if (tid == 0) plan[PL_NPUSH] = (int32_t)np;
  if (np > pcap) {  // uniform; the host reports DR_E_CAPACITY with n_push = np
    if (tid == 0) plan[PL_CAPERR] = 1;
    return;
  }
  __syncthreads();  // task_pos written, seen cleared
  for (int t = tid; t < ntask; t += NT) {
    const int w = task_wave[t];
    const int64_t P = task_pos[t];
    const int q = task_q[t];
    const int k = q >= 0 ? push_n[q] : 0;
    const int base = q >= 0 ? cq[q].out_off : 0;
    const int cnt = 1 + k;
    for (int i = 0; i < cnt; i++) push_wave[P + i] = i == 0 ? w : push_out[base + i - 1];
    for (int j = 0; j < cnt; j++) {
      const int i = cnt - 1 - j;
      const int pw = i == 0 ? w : push_out[base + i - 1];
      pop_wave[P + j] = pw;
      pop_cur[P + j] = 4 * w;
      seen[pw] = 1;
    }
  }
  // pushes before wave w = the position of the first task with wave >= w (np
  // past the last): task t owns the waves after its predecessor's, up to its own
  // (task waves increase), so each writes its range -- no search per wave
  for (int t = tid; t <= ntask; t += NT) {
    const int wlo = t == 0 ? 1 : task_wave[t - 1] + 1;
    const int whi = t < ntask ? task_wave[t] : nw + 1;
    const uint32_t v = (uint32_t)(t < ntask ? task_pos[t] : np);
    for (int w = wlo; w <= whi; w++) push_off[w - 1] = v;
  }
  if (qidx_static) {  // the delivery queries are the static per-wave table (one per present leader)
    __syncthreads();  // pop_wave written, seen set (block-uniform branch: a kernel argument)
    if (tid == 0) plan[PL_NQD] = nqd_static;
    for (int64_t p = tid; p < np; p += NT) pop_q[p] = qidx_static[pop_wave[p]];
    int64_t live = 0, zero = 0, tl, tz;  // the distinct popped leaders: the table's queries that swept
    for (int w = 1 + tid; w <= nw; w += NT) live += seen[w];
    block_scan2_excl<NT>(live, zero, s, tl, tz);
    if (tid == 0) plan[PL_NLIVE] = (int32_t)tl;
    return;
  }
  __syncthreads();  // seen written
  int64_t c0 = 0, c1 = 0;  // running totals (block-uniform)
  for (int i0 = 0; i0 < nw; i0 += CH) {
    int64_t f[K], mw[K], qi[K], mo[K];
#pragma unroll
    for (int j = 0; j < K; j++) {
      const int i = i0 + tid * K + j, w = nw - i;
      f[j] = (i < nw && seen[w]) ? 1 : 0;
      mw[j] = f[j] ? (int64_t)(4 * (w - 1) + 2) * WS : 0;  // rounds 0..top
    }
    int64_t tq, tm;
    block_scan2_items<NT, K>(f, mw, qi, mo, s, tq, tm);
#pragma unroll
    for (int j = 0; j < K; j++) {
      if (!f[j]) continue;
      const int w = nw - (i0 + tid * K + j);
      qidx[w] = (int32_t)(c0 + qi[j]);
      SweepQuery q{};
      q.top = 4 * (w - 1) + 1;
      q.bottom = 0;
      q.src0 = lead[w] - 1;
      q.flags = qflags;
      q.mask_off = c1 + mo[j];
      q.tgt0 = -1;
      dq[c0 + qi[j]] = q;
    }
    c0 += tq;
    c1 += tm;
  }
  if (tid == 0) {
    plan[PL_NQD] = (int32_t)c0;
    plan[PL_NLIVE] = (int32_t)c0;
  }
  __syncthreads();  // qidx written
  for (int64_t p = tid; p < np; p += NT) pop_q[p] = qidx[pop_wave[p]];
}
template <int NT>
__global__ __launch_bounds__(NT) void k_plan_pops(int nw, int WS, int qflags, const uint16_t *__restrict__ lead,
                                                  const int32_t *__restrict__ task_wave,
                                                  const int32_t *__restrict__ task_q,
                                                  const SweepQuery *__restrict__ cq,
                                                  const int32_t *__restrict__ push_n,
                                                  const int32_t *__restrict__ push_out, int64_t pcap,
                                                  int64_t *__restrict__ task_pos, uint32_t *__restrict__ push_off,
                                                  int32_t *__restrict__ push_wave, int32_t *__restrict__ pop_wave,
                                                  int32_t *__restrict__ pop_cur, int32_t *__restrict__ pop_q,
                                                  uint8_t *__restrict__ seen, int32_t *__restrict__ qidx,
                                                  SweepQuery *__restrict__ dq, int32_t *__restrict__ plan,
                                                  const int32_t *__restrict__ qidx_static = nullptr,
                                                  int nqd_static = 0) {
  plan_pops_body<NT>(nw, WS, qflags, lead, task_wave, task_q, cq, push_n, push_out, pcap, task_pos, push_off,
                     push_wave, pop_wave, pop_cur, pop_q, seen, qidx, dq, plan, qidx_static, nqd_static);
}
// plan_pops_body's arguments, for the workgroup of k_own_emit that runs it
struct PopPlanArgs {
  int active;  // 0: no plan workgroup
  int nw, WS, qflags;
  const uint16_t *lead;
  const int32_t *task_wave, *task_q;
  const SweepQuery *cq;
  const int32_t *push_n, *push_out;
  int64_t pcap;
  int64_t *task_pos;
  uint32_t *push_off;
  int32_t *push_wave, *pop_wave, *pop_cur, *pop_q;
  uint8_t *seen;
  int32_t *qidx;
  SweepQuery *dq;
  int32_t *plan;
  const int32_t *qidx_static;
  int nqd_static;
};

// Stops -> per-pop emission segment + canonical terms (run_deliver's on_batch):
// merged at m = stop: rounds 1..min(m, cur) are canonical (prefixes C, G, E),
// the pop's own rounds are stop+1 .. min(cur, top); unmerged sweeps reach
// rounds >= -1-stop only.
template <int NT>
__global__ __launch_bounds__(NT) void k_plan_emit(const int32_t *__restrict__ pop_cur,
                                                  const int32_t *__restrict__ pop_q,
                                                  const SweepQuery *__restrict__ dq,
                                                  const int32_t *__restrict__ stops, const u64 *__restrict__ Cc,
                                                  const u64 *__restrict__ Gc, const u64 *__restrict__ Ec,
                                                  const u64 *__restrict__ dedges, int rpb, int64_t rb_cap,
                                                  PopDesc *__restrict__ pd, int32_t *__restrict__ desc_of_pop,
                                                  u64 *__restrict__ extra_c, u64 *__restrict__ extra_g,
                                                  u64 *__restrict__ pedges, u64 *__restrict__ digest,
                                                  u64 *__restrict__ counts, int64_t *__restrict__ item_pref,
                                                  int32_t *__restrict__ plan) {
  __shared__ int64_t s[NT / 64];
  __shared__ int64_t c0, c1, c2;
  const int tid = threadIdx.x;
  const int64_t np = plan[PL_CAPERR] ? 0 : plan[PL_NPUSH];
  if (tid == 0) c0 = c1 = c2 = 0;
  __syncthreads();
  for (int64_t p0 = 0; p0 < np; p0 += NT) {
    const int64_t p = p0 + tid;
    int64_t has = 0, nr = 0, items = 0;
    int q = 0, first = 0, last = 0;
    u64 pos0 = 0;
    if (p < np) {
      q = pop_q[p];
      const int top = dq[q].top, stop = stops[q], cur = pop_cur[p];
      last = min(cur, top);
      u64 ec = 0, eg = 0, pe = dedges[q];
      if (stop >= 0) {
        const int cm = min(stop, cur);
        ec = Cc[cm];
        eg = Gc[cm];
        pos0 = ec;
        first = stop + 1;
        pe += Ec[stop];
      } else {
        first = max(1, -1 - stop);
      }
      extra_c[p] = ec;
      extra_g[p] = eg;
      pedges[p] = pe;
      digest[p] = 0;
      counts[p] = 0;  // k_emit_ids accumulates the pop's delivered-vertex count here
      has = first <= last ? 1 : 0;
      nr = has ? last - first + 1 : 0;
      items = has ? (nr + rpb - 1) / rpb : 0;
    }
    int64_t td, tr, ti;
    const int64_t di = block_scan_excl<NT>(has, s, td);
    const int64_t rb = block_scan_excl<NT>(nr, s, tr);
    const int64_t it = block_scan_excl<NT>(items, s, ti);
    if (p < np) desc_of_pop[p] = has ? (int32_t)(c0 + di) : -1;
    if (has) {
      PopDesc d{};
      d.mask_off = dq[q].mask_off;
      d.rbase_off = c1 + rb;
      d.pos0 = (int64_t)pos0;
      d.first = first;
      d.last = last;
      d.out = (int32_t)p;
      d.use_k = 0;
      pd[c0 + di] = d;
      item_pref[c0 + di] = c2 + it;
    }
    __syncthreads();
    if (tid == 0) { c0 += td; c1 += tr; c2 += ti; }
    __syncthreads();
  }
  if (tid == 0) {
    const bool over = c1 > rb_cap;  // planner bound violated: report, emit nothing
    item_pref[over ? 0 : c0] = over ? 0 : c2;
    plan[PL_NDESC] = over ? 0 : (int32_t)c0;
    if (over) plan[PL_CAPERR] = 2;
  }
  __syncthreads();
  // item -> segment map after the prefix (k_emit_ids looks its segment up in one load)
  const int nd = plan[PL_NDESC];
  for (int i = tid; i < nd; i += NT)
    for (int64_t it = item_pref[i]; it < item_pref[i + 1]; it++) item_pref[nd + 1 + it] = i;
}

// orderVertices planned on the device (dr_order_vertices, REF mode): per-pop
// count and digest = the canonical prefix terms + the pop's own rounds.
template <int NT>
__global__ __launch_bounds__(NT) void k_pop_final(const int32_t *__restrict__ plan,
                                                  const int32_t *__restrict__ desc_of_pop,
                                                  const u64 *__restrict__ extra_c, const u64 *__restrict__ extra_g,
                                                  const u64 *__restrict__ counts, const u64 *__restrict__ digest,
                                                  u64 *__restrict__ out_count, u64 *__restrict__ out_digest) {
  const int64_t np = plan[PL_NPUSH];
  for (int64_t p = (int64_t)blockIdx.x * NT + threadIdx.x; p < np; p += (int64_t)gridDim.x * NT) {
    out_count[p] = extra_c[p] + (desc_of_pop[p] >= 0 ? counts[p] : 0);
    out_digest[p] = extra_g[p] + digest[p];
  }
}

// Outputs -> pinned host memory (h_*, every workgroup a share), totals -> hdr (workgroup 0).
template <int NT>
__global__ __launch_bounds__(NT) void k_plan_final(int nw, const uint8_t *__restrict__ commit,
                                                   const int32_t *__restrict__ vcount,
                                                   const uint32_t *__restrict__ push_off,
                                                   const int32_t *__restrict__ push_wave,
                                                   const int32_t *__restrict__ desc_of_pop,
                                                   const u64 *__restrict__ extra_c, const u64 *__restrict__ extra_g,
                                                   const u64 *__restrict__ pedges, const u64 *__restrict__ counts,
                                                   const u64 *__restrict__ digest, const u64 *__restrict__ cedges,
                                                   const u64 *__restrict__ dstats, const int32_t *__restrict__ nseg,
                                                   const int32_t *__restrict__ plan, uint8_t *h_commit,
                                                   int32_t *h_vcount, uint32_t *h_push_off, int32_t *h_push_wave,
                                                   u64 *h_pc, u64 *h_pd, u64 *h_pe, u64 *h_hdr) {
  __shared__ u64 acc[8];
  const int tid = threadIdx.x;
  const int gt = blockIdx.x * NT + tid, gs = gridDim.x * NT;
  if (tid < 8) acc[tid] = 0;
  __syncthreads();
  const int caperr = plan[PL_CAPERR];
  const int64_t np = caperr ? 0 : plan[PL_NPUSH];
  const int nqc = plan[PL_NQC], nqd = plan[PL_NQD];
  for (int w = gt; w < nw; w += gs) {
    h_commit[w] = commit[w];
    h_vcount[w] = vcount[w];
  }
  if (!caperr)
    for (int w = gt; w <= nw; w += gs) h_push_off[w] = push_off[w];
  for (int64_t p = gt; p < np; p += gs) {
    const int di = desc_of_pop[p];
    h_push_wave[p] = push_wave[p];
    h_pc[p] = extra_c[p] + (di >= 0 ? counts[p] : 0);
    h_pd[p] = extra_g[p] + digest[p];
    h_pe[p] = pedges[p];
  }
  if (blockIdx.x != 0) return;  // totals: workgroup 0 (device-memory reads only)
  u64 de = 0, ce = 0, st[4] = {0, 0, 0, 0};
  for (int64_t p = tid; p < np; p += NT) de += pedges[p];
  for (int q = tid; q < nqc; q += NT) ce += cedges[q];
  for (int q = tid; q < nqd; q += NT)
#pragma unroll
    for (int k = 0; k < 4; k++) st[k] += dstats[4 * q + k];
  // one LDS atomic per wave and counter (256 same-address atomics serialise)
  de = wave_sum(de);
  ce = wave_sum(ce);
#pragma unroll
  for (int k = 0; k < 4; k++) st[k] = wave_sum(st[k]);
  if ((tid & 63) == 0) {
    atomicAdd(&acc[0], de);
    atomicAdd(&acc[1], ce);
#pragma unroll
    for (int k = 0; k < 4; k++) atomicAdd(&acc[2 + k], st[k]);
  }
  __syncthreads();
  if (tid == 0) {
    h_hdr[PH_NPUSH] = (u64)plan[PL_NPUSH];
    h_hdr[PH_CHAIN_E] = acc[1];
    h_hdr[PH_DELIVER_E] = acc[0];
    for (int k = 0; k < 4; k++) h_hdr[PH_PARTIAL + k] = acc[2 + k];
    h_hdr[PH_NQD] = (u64)nqd;
    h_hdr[PH_NSEG] = (u64)(int64_t)*nseg;
    h_hdr[PH_CAPERR] = (u64)caperr;
  }
}

// ---------------------------------------------------------------------------
// PAPER-mode delivery (DR_DELIVER_PAPER) on the memo path.  Pop p delivers
// cone(p) minus everything pops 0..p-1 delivered.  That set is downward closed,
// so the pruned sweep of the oracle delivers exactly cone(p) \ U_{p'<p} cone(p').
// Every vertex is delivered by the first pop whose cone holds it; only the first
// pop of each query (distinct leader) can deliver anything.  From the delivery
// sweeps' masks (SW_MERGE, no emission): query q's cone is K on rounds 1..cut_q
// (merged: cut = merge round + dmax - 1) and its own mask rows on lo_q..top_q.
// For round r the candidate owners are the first pop of the queries whose own
// range holds r, and first_K(r) = the smallest first pop among the merged
// queries with cut >= r (the first to hold K_r).
// ---------------------------------------------------------------------------

// One workgroup: first pops, cut / lo per query, first_K (a suffix minimum over
// rounds), and per round the queries whose own range holds it (CSR: qr_off,
// qr_list).  Scratch: qr_cnt [T+2].
template <int NT>
__global__ __launch_bounds__(NT) void k_paper_plan(int T, int dmax, const int32_t *__restrict__ plan,
                                                   const int32_t *__restrict__ pop_q, const SweepQuery *__restrict__ dq,
                                                   const int32_t *__restrict__ stops, int32_t *__restrict__ firstpop,
                                                   int32_t *__restrict__ qcut, int32_t *__restrict__ qlo,
                                                   uint32_t *__restrict__ firstK, uint32_t *__restrict__ qr_cnt,
                                                   uint32_t *__restrict__ qr_off, int32_t *__restrict__ qr_list) {
  __shared__ uint32_t s[NT / 64];
  const int tid = threadIdx.x;
  const int caperr = plan[PL_CAPERR];
  const int64_t np = caperr ? 0 : plan[PL_NPUSH];
  const int nq = caperr ? 0 : plan[PL_NQD];
  for (int q = tid; q < nq; q += NT) firstpop[q] = INT_MAX;
  for (int r = tid; r <= T + 1; r += NT) {
    firstK[r] = 0xffffffffu;
    qr_cnt[r] = 0;
  }
  __syncthreads();
  for (int64_t p = tid; p < np; p += NT) atomicMin(&firstpop[pop_q[p]], (int32_t)p);
  __syncthreads();
  for (int q = tid; q < nq; q += NT) {
    const int stop = stops[q], top = dq[q].top;
    const int cut = stop >= 0 ? min(stop + dmax - 1, top) : -1;
    const int lo = stop >= 0 ? cut + 1 : max(1, -1 - stop);
    qcut[q] = cut;
    qlo[q] = lo;
    const uint32_t fp = (uint32_t)__hip_atomic_load(&firstpop[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cut >= 1) atomicMin(&firstK[cut], fp);
    for (int r = lo; r <= top; r++) atomicAdd(&qr_cnt[r], 1u);
  }
  __syncthreads();
  // first_K(r) = min over c >= r of firstK[c]; qr_off = exclusive prefix of qr_cnt
  const int n = T + 2, per = (n + NT - 1) / NT;
  const int ra = tid * per, rb = min(n, ra + per);
  uint32_t mn = 0xffffffffu, cnt = 0;
  for (int r = ra; r < rb; r++) {
    mn = min(mn, __hip_atomic_load(&firstK[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    cnt += __hip_atomic_load(&qr_cnt[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  uint32_t tot;
  uint32_t run = block_scan_excl<NT>(cnt, s, tot);
  // suffix minimum: the minimum over the threads above (wave shuffles, then the waves above)
  __shared__ uint32_t smin[NT / 64];
  const int lane = tid & 63, wid = tid >> 6;
  uint32_t x = mn;  // inclusive suffix min within the wave
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_down(x, off);
    if (lane + off < 64) x = min(x, y);
  }
  if (lane == 0) smin[wid] = x;
  __syncthreads();
  uint32_t above = 0xffffffffu;  // waves above this one
  for (int i = wid + 1; i < NT / 64; i++) above = min(above, smin[i]);
  const uint32_t nxt = __shfl_down(x, 1);
  uint32_t suf = min(above, lane < 63 ? nxt : 0xffffffffu);
  for (int r = rb - 1; r >= ra; r--) {
    suf = min(suf, __hip_atomic_load(&firstK[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    firstK[r] = suf;
  }
  for (int r = ra; r < rb; r++) {
    const uint32_t c = __hip_atomic_load(&qr_cnt[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    qr_off[r] = run;
    run += c;
    qr_cnt[r] = 0;  // the fill counter below
  }
  if (tid == NT - 1) qr_off[n] = run;
  __syncthreads();
  for (int q = tid; q < nq; q += NT) {
    const int top = dq[q].top, lo = qlo[q];
    for (int r = lo; r <= top; r++) {
      const uint32_t at = __hip_atomic_load(&qr_off[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) +
                          atomicAdd(&qr_cnt[r], 1u);
      // (owner, mask row offset): k_paper_emit needs no further lookup
      const int64_t mo = dq[q].mask_off;
      qr_list[3 * (size_t)at] = __hip_atomic_load(&firstpop[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      qr_list[3 * (size_t)at + 1] = (int32_t)(uint32_t)mo;
      qr_list[3 * (size_t)at + 2] = (int32_t)(mo >> 32);
    }
  }
}

// One workgroup per query q (its first pop p delivers): rounds a..top, a = the
// first round with first_K = p (merged queries whose K range starts there) or
// lo_q.  Round r: the base set (K_r when r <= cut_q, else q's mask row) & P_r,
// minus the base sets of every candidate owner below p at r; positions from the
// counts of the rounds below (NT/64 rounds at a time, one per wave).
template <int WS, int NT>
__global__ __launch_bounds__(NT) void k_paper_emit(DagView g, const u64 *__restrict__ K, const u64 *__restrict__ masks,
                                                   const int32_t *__restrict__ plan, const SweepQuery *__restrict__ dq,
                                                   const int32_t *__restrict__ firstpop,
                                                   const int32_t *__restrict__ qcut, const int32_t *__restrict__ qlo,
                                                   const uint32_t *__restrict__ firstK,
                                                   const uint32_t *__restrict__ qr_off,
                                                   const int32_t *__restrict__ qr_list,
                                                   const uint32_t *__restrict__ slot_off,
                                                   const uint16_t *__restrict__ slot_src,
                                                   u64 *__restrict__ qcount, u64 *__restrict__ qdigest,
                                                   u64 *__restrict__ qedges) {
  constexpr int NWV = NT / 64;
  __shared__ u64 s_c[NWV], s_acc[2];
  __shared__ int s_a;
  const int q = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (q >= plan[PL_NQD] || plan[PL_CAPERR]) return;
  const int p = firstpop[q], cut = qcut[q], lo = qlo[q], top = dq[q].top;
  const int64_t moff = dq[q].mask_off;
  // first_K is non-decreasing in r: the first round l in 1..cut with first_K(l) >= p
  // (a = l when first_K(l) == p, else lo).  The NT rounds below cut are probed at once
  // (the boundary is usually a few rounds down); a binary search covers the rest.
  if (tid == 0) {
    s_acc[0] = s_acc[1] = 0;
    s_a = cut >= 1 ? 0 : lo;  // 0: not found yet
  }
  __syncthreads();
  if (cut >= 1) {
    const int r = cut - tid;
    if (r >= 1) {
      const bool ge = (int64_t)firstK[r] >= (int64_t)p;
      const bool below = r == 1 || (int64_t)firstK[r - 1] < (int64_t)p;
      if (ge && below) s_a = (int64_t)firstK[r] == (int64_t)p ? r : lo;  // the unique boundary
    }
    __syncthreads();
    if (tid == 0 && s_a == 0) {  // the boundary lies more than NT rounds below cut
      int l = 1, h = max(1, cut - NT + 1);
      while (l < h) {
        const int m = (l + h) >> 1;
        if ((int64_t)firstK[m] >= (int64_t)p) h = m; else l = m + 1;
      }
      s_a = (int64_t)firstK[l] == (int64_t)p ? l : lo;
    }
  }
  __syncthreads();
  const int a = s_a;
  u64 run = 0, dg = 0, ed = 0;
  for (int y0 = a; y0 <= top; y0 += NWV) {  // block-uniform
    const int r = y0 + wid;
    const bool on = r <= top;
    u64 mw = 0;
    if (on && lane < WS) {
      const u64 pw = g.present[(size_t)r * WS + lane];
      const uint32_t fk = firstK[r];
      const u64 kw = K[(size_t)r * WS + lane];
      u64 base = r <= cut ? kw : masks[moff + (int64_t)r * WS + lane];
      u64 ex = (int64_t)fk < (int64_t)p ? kw : 0ULL;  // K's owner comes first
      for (uint32_t i = qr_off[r]; i < qr_off[r + 1]; i++) {
        const int32_t *e = qr_list + 3 * (size_t)i;
        if (e[0] < p) {
          const int64_t mo = (int64_t)(((uint64_t)(uint32_t)e[2] << 32) | (uint32_t)e[1]);
          ex |= masks[mo + (int64_t)r * WS + lane];
        }
      }
      mw = base & ~ex & pw;
    }
    const u64 cnt = wave_sum((u64)popc64(mw));
    if (lane == 0) s_c[wid] = cnt;
    __syncthreads();
    u64 pos = run, tot = 0;
#pragma unroll
    for (int i = 0; i < NWV; i++) {
      const u64 c = s_c[i];
      pos += i < wid ? c : 0ULL;
      tot += c;
    }
    if (on && cnt)  // PAPER delivers an id once, at its first slot
      dg += wave_emit_round<WS, 8, true>(slot_off, slot_src, r, mw, pos, g.sdeg, g.wdeg, g.n, &ed, g.slot_rep, g.roff);
    run += tot;
    __syncthreads();
  }
  dg = wave_sum(dg);
  ed = wave_sum(ed);
  if (lane == 0) {
    if (dg) atomicAdd(&s_acc[0], dg);
    if (ed) atomicAdd(&s_acc[1], ed);
  }
  __syncthreads();
  if (tid == 0) {
    qcount[q] = run;
    qdigest[q] = s_acc[0];
    qedges[q] = s_acc[1];
  }
}

// One query's own-round emission (k_own_emit, or the delivery sweep's workgroup right after
// its sweep: dr::OwnEmit): rounds cut+1 .. top from its mask rows, positions from C_cut.
template <int WS, int NT>
__device__ __forceinline__ void own_emit_query(const DagView &g, const u64 *__restrict__ masks, int dmax, int q,
                                               int stop, int top, int64_t moff, const u64 *__restrict__ Cc,
                                               const uint32_t *__restrict__ slot_off,
                                               const uint16_t *__restrict__ slot_src, u64 *__restrict__ qcount,
                                               u64 *__restrict__ qdigest, int32_t *__restrict__ qcut) {
  constexpr int NWV = NT / 64;
  __shared__ u64 s_c[NWV], s_dg;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int cut = stop >= 0 ? min(stop + dmax - 1, top) : -1;
  const int first = stop >= 0 ? cut + 1 : max(1, -1 - stop);
  const u64 pos0 = cut >= 0 ? Cc[cut] : 0ULL;
  if (tid == 0) s_dg = 0;
  u64 run = pos0, dg = 0;
  for (int y0 = first; y0 <= top; y0 += NWV) {  // block-uniform
    const int r = y0 + wid;
    const bool on = r <= top;
    u64 mw = 0;
    uint32_t sa = 0, sb = 0;
    if (on) {  // the slot range loads beside the mask row
      sa = slot_off[r];
      sb = slot_off[r + 1];
      if (lane < WS) mw = masks[moff + (int64_t)r * WS + lane] & g.present[(size_t)r * WS + lane];
    }
    // REF delivers every slot of a reached id (process.go:418-429): repeated ones count too
    const u64 cnt = wave_sum((u64)popc64(mw)) + (on && g.dup_off ? (u64)dup_count<WS>(g, r, mw) : 0ULL);
    if (lane == 0) s_c[wid] = cnt;
    __syncthreads();
    u64 pos = run, tot = 0;
#pragma unroll
    for (int i = 0; i < NWV; i++) {
      const u64 c = s_c[i];
      pos += i < wid ? c : 0ULL;
      tot += c;
    }
    if (on && cnt) dg += wave_emit_slots<WS>(slot_src, r, sa, sb, mw, pos, nullptr, nullptr, 0, nullptr, nullptr, g.roff);
    run += tot;
    __syncthreads();
  }
  dg = wave_sum(dg);
  if (lane == 0 && dg) atomicAdd(&s_dg, dg);
  __syncthreads();
  if (tid == 0) {
    qcount[q] = run - pos0;
    qdigest[q] = s_dg;
    qcut[q] = cut;
  }
}

// REF delivery, own rounds (after the merging delivery sweeps, SW_MERGE): one
// workgroup per query, rounds cut+1 .. top (cut = merge round + dmax - 1: the
// merge run's rounds have the canonical positions too) or, for
// an unmerged sweep, every round it reached; positions from C_cut on.  NT/64
// rounds at a time, one per wave.  With Gc, the grid's last workgroup computes the
// canonical digest and edge prefixes G, E for k_replay_final (one pass of its
// threads: T + 1 <= 8 NT; a longer DAG's prefixes come from k_canon_prefix).
template <int WS, int NT>
__global__ __launch_bounds__(NT) void k_own_emit(DagView g, const u64 *__restrict__ masks, int dmax,
                                                 const int32_t *__restrict__ plan, const SweepQuery *__restrict__ dq,
                                                 const int32_t *__restrict__ stops, const u64 *__restrict__ Cc,
                                                 const uint32_t *__restrict__ slot_off,
                                                 const uint16_t *__restrict__ slot_src, u64 *__restrict__ qcount,
                                                 u64 *__restrict__ qdigest, int32_t *__restrict__ qcut, int T,
                                                 const u64 *__restrict__ RG, const u64 *__restrict__ CE,
                                                 u64 *__restrict__ Gc, u64 *__restrict__ Ec, const PopMark pm,
                                                 const PopPlanArgs pp, const int *__restrict__ lo_w) {
  // workgroup 0 (with Gc): the canonical prefixes G, E -- the longest workgroup, so it
  // starts first; the last (pp.active): the pop plan (plan_pops_body), which needs only the
  // chains' pushes (the launch before this one)
  const int pre = Gc ? 1 : 0;
  if (pre && blockIdx.x == 0) {  // (Gc null: k_canon_prefix computed them)
    if (lo_w) {  // the speculative prefixes are exact below the walk's lowest round: rescan from there
      const int lw = *lo_w;
      if (lw <= T)
        canon_prefix_gen<NT, 8>(
            lw, T, lw >= 1 ? Gc[lw - 1] : 0ULL, lw >= 1 ? Ec[lw - 1] : 0ULL, [&](int r) { return RG[r]; },
            [&](int r) { return CE[r]; }, Gc, Ec);
    } else {
      canon_prefix_regs<NT, 8>(T, RG, CE, Gc, Ec);
    }
    return;
  }
  if (pp.active && blockIdx.x == gridDim.x - 1) {
    plan_pops_body<NT>(pp.nw, pp.WS, pp.qflags, pp.lead, pp.task_wave, pp.task_q, pp.cq, pp.push_n, pp.push_out,
                       pp.pcap, pp.task_pos, pp.push_off, pp.push_wave, pp.pop_wave, pp.pop_cur, pp.pop_q, pp.seen,
                       pp.qidx, pp.dq, pp.plan, pp.qidx_static, pp.nqd_static);
    return;
  }
  const int q = (int)blockIdx.x - pre;
  // the query's fields load with the plan counts (the arena holds every slot below the grid bound)
  const int nq = plan[PL_NQD], caperr = plan[PL_CAPERR];
  const int stop = stops[q], top = dq[q].top;
  const int64_t moff = dq[q].mask_off;
  if (q >= nq || caperr) return;
  if (pm.commit && !pm.live(top)) return;  // a wave nobody pops: its sweep did not run
  own_emit_query<WS, NT>(g, masks, dmax, q, stop, top, moff, Cc, slot_off, slot_src, qcount, qdigest, qcut);
}


// Upward weak edges (App. A Q8: to the same or a later round) on the memo path
// (engine.hip dr_replay, up_verify).  The replay ran on the regular graph G_reg; an
// edge u -> v changes no cone C computed there when u in C implies v in C (C is then
// closed under the edge, so the least closed set holding the query is still C).  One
// thread per (edge, cone) pair -- the canonical cone K (q = -1) and every delivery
// query of the static table, whose cone is K at and below its cut and its own mask
// rows above (an unmerged query: its rows down to where it ended) -- counts the pairs
// where u is reached and v is not.  Any count sends dr_replay to the general sweep.
template <int WS>
__global__ __launch_bounds__(256) void k_verify_up(const u64 *__restrict__ K, const u64 *__restrict__ masks,
                                                   const SweepQuery *__restrict__ dq, int nq,
                                                   const int32_t *__restrict__ stops, const int32_t *__restrict__ qcut,
                                                   const int4 *__restrict__ up, int ne, int32_t *__restrict__ bad,
                                                   const PopMark pm) {
  const int64_t n = (int64_t)ne * (nq + 1);
  int cnt = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int e = (int)(i / (nq + 1)), q = (int)(i % (nq + 1)) - 1;
    const int4 E = up[e];  // (ru, su0, rv, tv0)
    auto bitK = [&](int r, int s) { return ((K[(size_t)r * WS + (s >> 6)] >> (s & 63)) & 1ULL) != 0; };
    bool in_u, in_v;
    if (q < 0) {
      in_u = bitK(E.x, E.y);
      in_v = bitK(E.z, E.w);
    } else {
      const SweepQuery Q = dq[q];
      if (pm.commit && !pm.live(Q.top)) continue;  // a wave nobody pops (its sweep did not run)
      const int stop = stops[q], cut = qcut[q], lo = stop >= 0 ? 0 : -1 - stop;
      auto in = [&](int r, int s) -> bool {
        if (r > Q.top || r < lo) return false;
        if (r <= cut) return bitK(r, s);
        return ((masks[Q.mask_off + (int64_t)r * WS + (s >> 6)] >> (s & 63)) & 1ULL) != 0;
      };
      in_u = in(E.x, E.y);
      in_v = in(E.z, E.w);
    }
    cnt += in_u && !in_v;
  }
  if (cnt) atomicAdd(bad, cnt);
}

// The canonical re-emission (per-round digests RG of rounds >= *rlo, positions from
// crbase: launch_canon's k_emit_ids) as the first nblk workgroups of the delivery sweeps'
// launch: it needs the canonical walk's K and positions, the sweeps need K alone, so the
// two run side by side instead of one launch after the other (C4: 6.6 us).  A workgroup
// takes round blocks of NT/64 rounds (a wave each) from the top down, nblk apart.
struct CanonEmit {
  int nblk;  // 0: none
  // the delivery queries grouped by XCD: blocks b and b + 8 share an XCD's L2 (round-robin
  // dispatch, MI355X_MICROARCH.md), so each XCD takes a contiguous run of the table --
  // adjacent waves' queries read the same rounds' words
  int xcd;
  int T;
  const uint32_t *slot_off;
  const uint16_t *slot_src;
  const u64 *K;
  const uint32_t *crbase;
  u64 *RG;
  const int *rlo;
};
template <int WS, int NT>
__device__ __forceinline__ void canon_emit_blocks(const DagView &g, const CanonEmit &ce, int b) {
  constexpr int RPB = NT / 64;
  __shared__ u64 s_dg;
  PopDesc d{};
  d.mask_off = 0;
  d.rbase_off = 1;  // crbase is indexed by round; rbase_off addresses round `first`
  d.pos0 = 0;
  d.first = 1;
  d.last = ce.T;
  d.out = 0;
  d.use_k = 1;
  const int lo = *ce.rlo;
  const int nb = (ce.T + RPB - 1) / RPB;
  const int blo = lo > 1 ? (lo - 1) / RPB : 0;  // the block holding round lo
  for (int blk = nb - 1 - b; blk >= blo; blk -= ce.nblk)  // (block-uniform)
    emit_block<WS, NT, RPB>(g, ce.slot_off, ce.slot_src, d, blk, nullptr, ce.K, ce.crbase, nullptr, nullptr, ce.RG,
                            nullptr, 0, &s_dg, nullptr, nullptr, lo);
}

// The own-round emission inside the delivery sweeps' launch (DR_OPT_FUSE bit 32): each query's
// workgroup emits its rounds above the cut as soon as its sweep stops, instead of a launch of
// its own after every sweep (k_own_emit)
struct OwnEmit {
  int on;
  const u64 *Cc;
  const uint32_t *slot_off;
  const uint16_t *slot_src;
  u64 *qcount, *qdigest;
  int32_t *qcut;
};
template <int WS, int NT, int MODE>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu((MODE & SW_MERGE) ? 3 : 1))) void k_sweep(
    DagView g, MemoView mv, const SweepQuery *__restrict__ qs, int nq, int seq, int depth_log2, u64 *__restrict__ masks,
    u64 *__restrict__ dlv, int32_t *__restrict__ push_out, int32_t *__restrict__ push_n, u64 *__restrict__ edges_out,
    u64 *__restrict__ wedges_out, uint8_t *__restrict__ hit_out, int32_t *__restrict__ stop_out,
    u64 *__restrict__ stats_out, const int *__restrict__ nq_dev, uint32_t *__restrict__ rcnt, const PopMark pm,
    const CanonEmit ce, const PopPlanArgs pp, const OwnEmit oe) {
  int bidx = (int)blockIdx.x;
  if constexpr ((MODE & SW_MERGE) != 0) {
    if (ce.nblk > 0) {  // (block-uniform) the first nblk workgroups re-emit canonical rounds
      if (bidx < ce.nblk) {
        canon_emit_blocks<WS, NT>(g, ce, bidx);
        return;
      }
      bidx -= ce.nblk;
    }
    if (ce.xcd && !seq && !nq_dev && bidx < nq) {  // (nblk is a multiple of 8: b % 8 still names the XCD)
      const int x = bidx & 7, k = bidx >> 3;
      bidx = x * (nq >> 3) + min(x, nq & 7) + k;
    }
    if (pp.active && (int)blockIdx.x == (int)gridDim.x - 1) {  // the last: the pop plan (plan_pops_body)
      plan_pops_body<NT>(pp.nw, pp.WS, pp.qflags, pp.lead, pp.task_wave, pp.task_q, pp.cq, pp.push_n, pp.push_out,
                         pp.pcap, pp.task_pos, pp.push_off, pp.push_wave, pp.pop_wave, pp.pop_cur, pp.pop_q, pp.seen,
                         pp.qidx, pp.dq, pp.plan, pp.qidx_static, pp.nqd_static);
      return;
    }
  }
  sweep_body<WS, NT, MODE>(bidx, g, mv, qs, nq, seq, depth_log2, masks, dlv, push_out, push_n, edges_out, wedges_out,
                           hit_out, stop_out, stats_out, nq_dev, rcnt, pm);
  if constexpr ((MODE & SW_MERGE) != 0) {
    if (oe.on && !seq && !nq_dev && bidx < nq) {  // (block-uniform)
      const SweepQuery q = qs[bidx];
      if (pm.commit && !pm.live(q.top)) return;  // a wave nobody pops: no sweep, no emission
      // (sweep_body ended with a barrier after thread 0 wrote the stop and the mask rows)
      own_emit_query<WS, NT>(g, masks, mv.dmax, bidx, stop_out[bidx], q.top, q.mask_off, oe.Cc, oe.slot_off,
                             oe.slot_src, oe.qcount, oe.qdigest, oe.qcut);
    }
  }
}

}  // namespace dr
