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

namespace dr {

// Committed waves -> tasks (wave, floor) -> leader-chain queries.  Persistent
// decidedWave: floor = the previous committed wave; literal: 0.  A task with
// wave - floor >= 2 walks rounds 4(w-1)+1 .. 4 floor + 1 and may push up to
// wave - floor - 1 leaders at out_off.
template <int NT>
__global__ __launch_bounds__(NT) void k_plan_chains(const uint8_t *__restrict__ commit, const uint16_t *__restrict__ lead,
                                                    int nw, int persistent, int qflags, int32_t *__restrict__ task_wave,
                                                    int32_t *__restrict__ task_q, SweepQuery *__restrict__ cq,
                                                    int32_t *__restrict__ plan) {
  __shared__ int64_t s[NT / 64];
  __shared__ int64_t c0, c1, c2;
  const int tid = threadIdx.x;
  if (tid == 0) c0 = c1 = c2 = 0;
  __syncthreads();
  for (int w0 = 0; w0 < nw; w0 += NT) {
    const int w = w0 + tid;
    const int64_t f = (w < nw && commit[w]) ? 1 : 0;
    int64_t tot;
    const int64_t ex = block_scan_excl<NT>(f, s, tot);
    if (f) task_wave[c0 + ex] = w + 1;
    __syncthreads();
    if (tid == 0) c0 += tot;
    __syncthreads();
  }
  const int ntask = (int)c0;
  for (int t0 = 0; t0 < ntask; t0 += NT) {
    const int t = t0 + tid;
    int w = 0, fl = 0;
    int64_t len = 0, has = 0;
    if (t < ntask) {
      w = task_wave[t];
      fl = (persistent && t > 0) ? task_wave[t - 1] : 0;
      len = w - fl - 1;
      has = len >= 1 ? 1 : 0;
    }
    int64_t tq, tl;
    const int64_t qi = block_scan_excl<NT>(has, s, tq);
    const int64_t off = block_scan_excl<NT>(has ? len : int64_t(0), s, tl);
    if (t < ntask) task_q[t] = has ? (int32_t)(c1 + qi) : -1;
    if (has) {
      SweepQuery q{};
      q.top = 4 * (w - 1) + 1;
      q.bottom = 4 * fl + 1;
      q.src0 = lead[w] - 1;
      q.flags = qflags;
      q.mask_off = 0;
      q.out_off = (int32_t)(c2 + off);
      q.tgt0 = -1;
      cq[c1 + qi] = q;
    }
    __syncthreads();
    if (tid == 0) { c1 += tq; c2 += tl; }
    __syncthreads();
  }
  if (tid == 0) {
    plan[PL_NTASK] = ntask;
    plan[PL_NQC] = (int32_t)c1;
    plan[PL_CAPERR] = 0;
    plan[PL_NQD] = 0;
    plan[PL_NDESC] = 0;
  }
}

// Pushes (task wave, then its chain's pushes in push order) -> pops in pop
// order (each task's pushes reversed, process.go:406-412), push_off per wave,
// and one delivery query per distinct leader, highest round first, with
// cumulative mask images (rounds 0..top).
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
                                                  SweepQuery *__restrict__ dq, int32_t *__restrict__ plan) {
  __shared__ int64_t s[NT / 64];
  __shared__ int64_t c0, c1;
  const int tid = threadIdx.x;
  const int ntask = plan[PL_NTASK];
  for (int i = tid; i <= nw; i += NT) seen[i] = 0;
  if (tid == 0) c0 = c1 = 0;
  __syncthreads();
  for (int t0 = 0; t0 < ntask; t0 += NT) {
    const int t = t0 + tid;
    int64_t cnt = 0;
    if (t < ntask) cnt = 1 + (task_q[t] >= 0 ? push_n[task_q[t]] : 0);
    int64_t tot;
    const int64_t ex = block_scan_excl<NT>(cnt, s, tot);
    if (t < ntask) task_pos[t] = c0 + ex;
    __syncthreads();
    if (tid == 0) c0 += tot;
    __syncthreads();
  }
  const int64_t np = c0;
  if (tid == 0) plan[PL_NPUSH] = (int32_t)np;
  if (np > pcap) {  // uniform; the host reports DR_E_CAPACITY with n_push = np
    if (tid == 0) plan[PL_CAPERR] = 1;
    return;
  }
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
  __syncthreads();
  for (int w = 1 + tid; w <= nw + 1; w += NT) {  // pushes before wave w
    int lo = 0, hi = ntask;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (task_wave[mid] >= w) hi = mid; else lo = mid + 1;
    }
    push_off[w - 1] = (uint32_t)(lo < ntask ? task_pos[lo] : np);
  }
  if (tid == 0) c0 = 0;
  __syncthreads();
  for (int i0 = 0; i0 < nw; i0 += NT) {
    const int i = i0 + tid, w = nw - i;
    const int64_t f = (i < nw && seen[w]) ? 1 : 0;
    const int top = 4 * (w - 1) + 1;
    int64_t tq, tm;
    const int64_t qi = block_scan_excl<NT>(f, s, tq);
    const int64_t mo = block_scan_excl<NT>(f ? (int64_t)(top + 1) * WS : int64_t(0), s, tm);
    if (f) {
      qidx[w] = (int32_t)(c0 + qi);
      SweepQuery q{};
      q.top = top;
      q.bottom = 0;
      q.src0 = lead[w] - 1;
      q.flags = qflags;
      q.mask_off = c1 + mo;
      q.tgt0 = -1;
      dq[c0 + qi] = q;
    }
    __syncthreads();
    if (tid == 0) { c0 += tq; c1 += tm; }
    __syncthreads();
  }
  if (tid == 0) plan[PL_NQD] = (int32_t)c0;
  for (int64_t p = tid; p < np; p += NT) pop_q[p] = qidx[pop_wave[p]];
}

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

}  // namespace dr
