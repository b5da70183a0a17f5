// shard_memo.hpp -- kernels of the memoized replay on the column-sharded DAG
// (dr_shard_replay, include/dagrider_shard.h).
//
// The single-GPU replay's memo carried over to column shards:
// the types both replay forms share (queries, their states, the kernel arguments)
// and the pieces both use:
//
//   k_ms_kcand     K^cand_r = U_{r+1} | OR_d WU_{r+d+2}[d] on the shard's columns
//                  (K^cand_T = P_T): RCCL mode's send buffer for the all-gather
//                  that gives every rank the full-width K.
//   next_bad       the next canonical segment's start (the highest bad round
//                  below a round).
//   ms_prefix_two  one workgroup's prefix sums of two arrays over the rounds.
//   k_ms_emit      per pop query: the canonical prefix at its cut plus its own
//                  rounds above the cut (counts, order-sensitive digest, edges).
//   k_ms_paper*    PAPER delivery (first-pop ownership of the REF cones).
//
// Query kinds: MQ_POP (orderVertices cone, strong + weak, merges with K), MQ_CHAIN
// (waveReady's leader chain, strong only, restarts), MQ_CANON (the canonical walk
// over the segments below bad rounds: K rows).  The fused form runs each query to
// its end in one workgroup (shard_fused.hpp), the stepped form one round per
// launch with an exchange between launches (shard_step.hpp).
//
// Semantics are dr_replay's (engine.hip): same commits, pushes, per-pop counts,
// digests and edge totals, bit for bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "wave_ops.hpp"

namespace drs {

using dr::u64;
using dr::shfl_xor64;
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

constexpr int MS_NT = 256;  // threads per workgroup (4 waves)
enum : int32_t { MQ_POP = 0, MQ_CHAIN = 1, MQ_CANON = 2 };

struct MQuery {
  int32_t type, top, bottom, src0;
  int64_t mask_off;   // MQ_POP: word offset of the mask row of round `top` (row j = round top - j)
  int32_t push_base;  // MQ_CHAIN: first slot of the query's pushes in push_out
  int32_t pad;
};

// Per-query state: the fused sweep's final state; the stepped form's state between
// launches (read and written in place by the query's workgroup).
struct MState {
  int32_t done, run, low, stop;  // stop: the round where the query merged / ended
  int32_t merged, npush;         // MQ_CANON: npush counts the segments walked
  int32_t cur, fresh;            // MQ_CANON: its current round; 1 = start the next segment below cur
  int32_t steps, pad;            // stepped form: launches the query was live in
  u64 edges;                     // MQ_CHAIN: strong degrees of the expanded vertices
};

struct MArgs {
  const u64 *strong;        // [max_rounds][nlocal][n][SP]: round-major over the local shards
  int64_t strong_stride;    // words between local shards' rows of one round (n * SP)
  int64_t strong_rstride;   // words per round (nlocal * n * SP)
  const uint32_t *wck;      // weak columns: key delta << 11 | local column
  const u64 *wcr;           // [column][W] sources with that weak edge
  const uint64_t *wcro;     // [nlocal][R+1] absolute column offsets per round
  const u64 *pres;          // [R][W]
  const uint16_t *sdeg;     // [R][n] strong degree
  const uint16_t *wdeg;     // [R][n] weak degree
  const u64 *sdr;           // [R] strong degree sum of a round
  const u64 *rdeg;          // [R] strong + weak degree sum of a round
  const uint16_t *lead;     // [nlead] chooseLeader(w), 1-based
  const u64 *U;             // [nlocal][R][SP]
  const u64 *WU;            // [nlocal][R][dd][SP]
  u64 *K;                   // [R][W] canonical cone, full width
  const MQuery *q;
  u64 *pend;                // stepped form: [nq][depth][nlocal * WSs] pending rings between launches
  u64 *masks;               // MQ_POP frontier rows
  int32_t *push_out;
  const uint8_t *good;       // [T+1] K^cand_r covers P_r (MQ_CANON: where segments start)
  const uint32_t *slot_off;  // [R+1] slot order (insertion order of every round)
  const uint16_t *slot_src;  // 1-based source per slot (0 = ghost)
  int32_t n, W, WSs, SP, G, shard0, nlocal, local, nq, depth, dd, dmax, summary, R, nlead, T;
};

// K^cand on the shard's columns, one wave per round (lane = column word).  Local
// mode writes the full-width K directly; RCCL mode writes ksend[r][WSs] for the
// all-gather (k_ms_kfin lays it out).
__global__ __launch_bounds__(MS_NT) void k_ms_kcand(MArgs a, int T, u64 *__restrict__ ksend) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), l = blockIdx.y, cw = threadIdx.x & 63;
  if (r > T || cw >= a.WSs) return;
  const int g = a.shard0 + l, w = g * a.WSs + cw;
  u64 v = 0;
  if (w < a.W) {
    if (r == T) {
      v = a.pres[(size_t)r * a.W + w];
    } else {
      const size_t ub = (size_t)l * a.R;
      v = a.U[(ub + r + 1) * a.SP + cw];
      for (int d = 0; d < a.dd && r + d + 2 <= T; d++) v |= a.WU[((ub + r + d + 2) * a.dd + d) * a.SP + cw];
    }
  }
  if (a.local) {
    if (w < a.W) a.K[(size_t)r * a.W + w] = v;
  } else {
    ksend[(size_t)r * a.WSs + cw] = v;
  }
}

// The highest bad round below `below` (-1: none), one wave (every lane gets it).
// The 0/1 flags are read 8 at a time (u64 words, a byte != 1 is a bad round), 16
// words per lane in flight: one pass covers 8192 rounds.
__device__ __forceinline__ int next_bad(const MArgs &a, int below) {
  constexpr int PL = 16;
  constexpr uint64_t ONES = 0x0101010101010101ULL;
  const int lane = threadIdx.x & 63;
  if (below <= 0) return -1;
  const uint64_t *g = reinterpret_cast<const uint64_t *>(a.good);
  const int wtop = (below - 1) >> 3, nb = below - 8 * wtop;  // rounds of word wtop below `below`: its low nb bytes
  const uint64_t topmask = nb >= 8 ? ~0ULL : (1ULL << (8 * nb)) - 1ULL;
  for (int top = wtop; top >= 0; top -= 64 * PL) {
    uint64_t v[PL];
#pragma unroll
    for (int k = 0; k < PL; k++) {
      const int x = top - PL * lane - k;
      v[k] = x >= 0 ? g[x] : ONES;
    }
    int best = -1;
#pragma unroll
    for (int k = PL - 1; k >= 0; k--) {
      const int x = top - PL * lane - k;
      uint64_t bad = v[k] ^ ONES;
      if (x == wtop) bad &= topmask;
      if (bad) best = 8 * x + (63 - __clzll(bad)) / 8;
    }
    for (int off = 32; off > 0; off >>= 1) best = max(best, __shfl_xor(best, off));
    if (best >= 0) return best;
  }
  return -1;
}

// inclusive prefixes of two arrays (a1 may be null) over 0..n-1 in one pass of one
// workgroup of NT threads: tiles of NT * CH elements, thread t owns CH consecutive
// elements (serial sums), one wave scan of the threads' totals for both arrays, one
// LDS hop for the waves' totals.  part: 2 * NT / 64 words of LDS.
template <int NT, int CH = 4>
__device__ __forceinline__ void ms_prefix_two(int n, const u64 *__restrict__ a0, u64 *__restrict__ b0,
                                              const u64 *__restrict__ a1, u64 *__restrict__ b1, u64 *part) {
  constexpr int NW = NT / 64, TILE = NT * CH;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  u64 cx = 0, cy = 0;  // carries from the tiles before
  for (int t0 = 0; t0 < n; t0 += TILE) {
    const int base = t0 + (int)threadIdx.x * CH;
    u64 x[CH], y[CH];
#pragma unroll
    for (int c = 0; c < CH; c++) {
      x[c] = base + c < n ? a0[base + c] : 0ULL;
      y[c] = (a1 && base + c < n) ? a1[base + c] : 0ULL;
    }
#pragma unroll
    for (int c = 1; c < CH; c++) {
      x[c] += x[c - 1];
      y[c] += y[c - 1];
    }
    const u64 sx = x[CH - 1], sy = y[CH - 1];
    u64 ix = sx, iy = sy;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const u64 tx = dr::shfl_up64(ix, off), ty = dr::shfl_up64(iy, off);
      if (lane >= off) {
        ix += tx;
        iy += ty;
      }
    }
    if (lane == 63) {
      part[wv] = ix;
      part[NW + wv] = iy;
    }
    __syncthreads();
    u64 ox = cx, oy = cy, tx = 0, ty = 0;
    for (int w = 0; w < NW; w++) {
      const u64 px = part[w], py = part[NW + w];
      if (w < wv) {
        ox += px;
        oy += py;
      }
      tx += px;
      ty += py;
    }
    __syncthreads();
    ox += ix - sx;
    oy += iy - sy;
#pragma unroll
    for (int c = 0; c < CH; c++)
      if (base + c < n) {
        b0[base + c] = ox + x[c];
        if (b1) b1[base + c] = oy + y[c];
      }
    cx += tx;
    cy += ty;
  }
}
// One wave emits round y's slots whose source bit is set in mw (lane w < W holds
// word w) in insertion order from position pos: digest terms and, with sdeg, the
// strong + weak degrees (this lane's shares).  Lane l takes SPT consecutive slots
// of each 64*SPT block: every slot and degree load of a block goes out at once
// (three memory latencies per round, not two per 64 slots), and an exclusive scan
// of the lanes' hit counts keeps the slot order.
template <int SPT = 16>
__device__ __forceinline__ void ms_wave_emit(const uint32_t *__restrict__ slot_off, const uint16_t *__restrict__ slot_src,
                                             int y, u64 mw, u64 pos, int W, const uint16_t *sdeg, const uint16_t *wdeg,
                                             int n, u64 &dg, u64 &ed) {
  const int lane = threadIdx.x & 63;
  const uint32_t s0 = slot_off[y], s1 = slot_off[y + 1];
  const uint32_t hi32 = (uint32_t)(mw >> 32), lo32 = (uint32_t)mw;
  for (uint32_t c0 = s0; c0 < s1; c0 += 64 * SPT) {
    const uint32_t i0 = c0 + (uint32_t)lane * SPT;
    int src[SPT];
#pragma unroll
    for (int q = 0; q < SPT; q++) src[q] = i0 + q < s1 ? (int)slot_src[i0 + q] : 0;
    uint32_t inm = 0;  // bit q: slot i0 + q is delivered
#pragma unroll
    for (int q = 0; q < SPT; q++) {
      const int sv = src[q];
      const int wd = sv > 0 ? (sv - 1) >> 6 : 0;
      const u64 word = ((u64)(uint32_t)__shfl((int)hi32, wd, 64) << 32) | (uint32_t)__shfl((int)lo32, wd, 64);
      inm |= (sv > 0 && ((word >> ((sv - 1) & 63)) & 1ULL)) ? 1u << q : 0u;
    }
    uint16_t d1[SPT], d2[SPT];
    if (sdeg) {
#pragma unroll
      for (int q = 0; q < SPT; q++) {
        const size_t at = (size_t)y * n + (src[q] > 0 ? src[q] - 1 : 0);
        d1[q] = (inm >> q) & 1u ? sdeg[at] : (uint16_t)0;
        d2[q] = (inm >> q) & 1u ? wdeg[at] : (uint16_t)0;
      }
    }
    const uint32_t cnt = (uint32_t)__popc(inm);
    uint32_t inc = cnt;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t t = __shfl_up(inc, off);
      if (lane >= off) inc += t;
    }
    u64 k = pos + (inc - cnt);
#pragma unroll
    for (int q = 0; q < SPT; q++)
      if ((inm >> q) & 1u) dg += dr::digest_term((uint32_t)y, (uint32_t)src[q], k++);
    if (sdeg) {
#pragma unroll
      for (int q = 0; q < SPT; q++) ed += (u64)d1[q] + d2[q];
    }
    pos += __shfl(inc, 63);
  }
  (void)W;
}

// REF emission of one pop query by one workgroup of NT threads (every thread
// calls it): the canonical prefix at the cut (C, G, E) plus the query's own
// rounds cut+1 .. top from its mask rows, 64 rounds at a time (counts, exclusive
// scan, digests and degrees).  The fused sweep calls it right after its own
// wave 0 wrote the mask rows: a workgroup barrier orders them (one CU, its L1
// writes through).
// SPT: slots per lane per block of ms_wave_emit (fewer: fewer registers, for a
// caller whose occupancy matters more than the emission's memory parallelism)
template <int NT = MS_NT, int SPT = 16>
__device__ __forceinline__ void ms_emit_query(const MArgs &a, const MQuery &Q, const MState &S,
                                              const uint32_t *__restrict__ slot_off,
                                              const uint16_t *__restrict__ slot_src, const u64 *__restrict__ Cc,
                                              const u64 *__restrict__ Gc, const u64 *__restrict__ Ec, int b,
                                              u64 *__restrict__ qcount, u64 *__restrict__ qdigest,
                                              u64 *__restrict__ qedges) {
  __shared__ uint32_t sCnt[64];
  __shared__ u64 sPos[64];
  __shared__ u64 sTot, sDg, sEd;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int top = Q.top;
  int cut, lo;
  if (S.merged) {
    cut = min(S.stop + a.dmax - 1, top);
    lo = cut + 1;
  } else {
    cut = 0;
    lo = max(1, S.stop);
  }
  if (tid == 0) {
    sDg = 0;
    sEd = 0;
  }
  auto mask_word = [&](int y) -> u64 {
    if (lane >= a.W) return 0ULL;
    return a.masks[Q.mask_off + (int64_t)(top - y) * a.W + lane] & a.pres[(size_t)y * a.W + lane];
  };
  u64 run = Cc[cut];
  for (int y0 = lo; y0 <= top; y0 += 64) {
    const int ny = min(64, top - y0 + 1);
    for (int i = wv; i < ny; i += NT / 64) {
      const u64 c = dr::wave_sum((u64)__popcll(mask_word(y0 + i)));
      if (lane == 0) sCnt[i] = (uint32_t)c;
    }
    __syncthreads();
    if (wv == 0) {
      u64 x = lane < ny ? sCnt[lane] : 0;
      const u64 v = x;
      for (int off = 1; off < 64; off <<= 1) {
        const u64 yv = __shfl_up(x, off);
        if (lane >= off) x += yv;
      }
      if (lane < ny) sPos[lane] = run + x - v;
      if (lane == 63) sTot = x;
    }
    __syncthreads();
    u64 dg = 0, ed = 0;
    for (int i = wv; i < ny; i += NT / 64) {
      const int y = y0 + i;
      ms_wave_emit<SPT>(slot_off, slot_src, y, mask_word(y), sPos[i], a.W, a.sdeg, a.wdeg, a.n, dg, ed);
    }
    dg = dr::wave_sum(dg);
    ed = dr::wave_sum(ed);
    if (lane == 0) {
      atomicAdd(&sDg, dg);
      atomicAdd(&sEd, ed);
    }
    run += sTot;
    __syncthreads();
  }
  if (tid == 0) {
    qcount[b] = run;
    qdigest[b] = sDg + Gc[cut];
    qedges[b] = sEd + Ec[cut];
  }
}

// REF emission, one workgroup per pop query (qidx; null: query b)
__global__ __launch_bounds__(MS_NT) void k_ms_emit(MArgs a, const int32_t *__restrict__ qidx, const MState *__restrict__ st,
                                                   const uint32_t *__restrict__ slot_off,
                                                   const uint16_t *__restrict__ slot_src, const u64 *__restrict__ Cc,
                                                   const u64 *__restrict__ Gc, const u64 *__restrict__ Ec,
                                                   u64 *__restrict__ qcount, u64 *__restrict__ qdigest,
                                                   u64 *__restrict__ qedges) {
  const int b = blockIdx.x, qi = qidx ? qidx[b] : b;
  ms_emit_query(a, a.q[qi], st[qi], slot_off, slot_src, Cc, Gc, Ec, b, qcount, qdigest, qedges);
}

// ---------------------------------------------------------------------------
// PAPER delivery (Alg. 3 line 54: a pop delivers its cone minus everything
// delivered before it).  The delivered set is downward closed, so every vertex
// goes to the FIRST pop whose cone holds it; only the first pop
// of each distinct leader delivers.  Per round r, one wave walks the distinct
// queries in first-pop order: base_q(r) = K_r for r <= cut_q, the query's own
// mask row for lo_q <= r <= top_q, else nothing; delivered = base & P & ~D,
// D |= base.  Pass 1 counts (and sums degrees), a per-query scan gives
// positions, pass 2 the order-sensitive digests.
// ---------------------------------------------------------------------------
struct MPaper {
  int32_t top, cut, lo, pad;
  int64_t mask_off;
};

__device__ __forceinline__ u64 paper_base(const MArgs &a, const MPaper &x, int r, u64 kr, int lane) {
  if (r <= x.cut) return kr;
  if (r < x.lo || r > x.top || lane >= a.W) return 0ULL;
  return a.masks[x.mask_off + (int64_t)(x.top - r) * a.W + lane];
}

template <bool DIGEST>
__global__ __launch_bounds__(MS_NT) void k_ms_paper(MArgs a, int rmax, const MPaper *__restrict__ qp, int m,
                                                    uint32_t *__restrict__ cnt, int rstride,
                                                    const uint32_t *__restrict__ slot_off,
                                                    const uint16_t *__restrict__ slot_src, u64 *__restrict__ qedges,
                                                    u64 *__restrict__ qdigest) {
  const int r = 1 + blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r > rmax) return;
  const u64 p = lane < a.W ? a.pres[(size_t)r * a.W + lane] : 0ULL;
  const u64 kr = lane < a.W ? a.K[(size_t)r * a.W + lane] : 0ULL;
  u64 D = 0;
  for (int i = 0; i < m; i++) {
    const MPaper x = qp[i];
    if (r > x.top) continue;  // wave-uniform
    const u64 base = paper_base(a, x, r, kr, lane) & p;
    const u64 dl = base & ~D;
    D |= base;
    if (__ballot(dl != 0ULL) == 0ULL) continue;
    if constexpr (!DIGEST) {
      const u64 c = dr::wave_sum((u64)__popcll(dl));
      u64 acc = 0;
      for (u64 y = dl; y; y &= y - 1) {
        const size_t at = (size_t)r * a.n + lane * 64 + __builtin_ctzll(y);
        acc += (u64)a.sdeg[at] + a.wdeg[at];
      }
      acc = dr::wave_sum(acc);
      if (lane == 0) {
        cnt[(size_t)i * rstride + r] = (uint32_t)c;
        atomicAdd(&qedges[i], acc);
      }
    } else {
      u64 dg = 0, ed = 0;
      ms_wave_emit(slot_off, slot_src, r, dl, cnt[(size_t)i * rstride + r], a.W, nullptr, nullptr, a.n, dg, ed);
      dg = dr::wave_sum(dg);
      if (lane == 0 && dg) atomicAdd(&qdigest[i], dg);
    }
  }
}

// per query: counts over rounds 1..rmax -> exclusive positions in place; total
__global__ __launch_bounds__(MS_NT) void k_ms_paper_scan(int rmax, uint32_t *__restrict__ cnt, int rstride,
                                                         u64 *__restrict__ qcount) {
  __shared__ u64 part[MS_NT];
  const int i = blockIdx.x, tid = threadIdx.x;
  uint32_t *c = cnt + (size_t)i * rstride;
  const int span = rmax, per = (span + MS_NT - 1) / MS_NT;
  const int a0 = 1 + tid * per, a1 = min(rmax + 1, a0 + per);
  u64 s = 0;
  for (int r = a0; r < a1; r++) s += c[r];
  part[tid] = s;
  __syncthreads();
  if (tid == 0) {
    u64 run = 0;
    for (int t = 0; t < MS_NT; t++) {
      const u64 v = part[t];
      part[t] = run;
      run += v;
    }
    qcount[i] = run;
  }
  __syncthreads();
  u64 run = part[tid];
  for (int r = a0; r < a1; r++) {
    const uint32_t v = c[r];
    c[r] = (uint32_t)run;
    run += v;
  }
}

}  // namespace drs
