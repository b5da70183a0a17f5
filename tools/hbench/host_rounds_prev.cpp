// host_rounds.cpp -- validation and host-state build of pre-packed rounds
// (dr_append_rounds_packed).  The weak-column build is a table lookup per weak
// edge (C4: ~31 K weak edges per round), so the work is split into (round,
// source chunk) tasks over the OpenMP threads -- a per-wave append of 4 rounds
// no longer leaves most cores idle -- and each round's chunk columns are merged
// by key afterwards.
#include "host_rounds.hpp"
namespace dr_host_old { using dr_host::PackedRounds; using dr_host::BuiltRounds; using dr_host::BuildScratch; using dr_host::HostRound; }

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>

#include <omp.h>

#include "dagrider_gpu.h"

namespace dr_host_old {
namespace {

int failf(std::string &err, int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  err = buf;
  return code;
}

// One source chunk [s_lo, s_hi) of a round (64-aligned, so its columns cover
// words [s_lo/64, s_hi/64) of every row): degrees, validation, weak columns.
struct Chunk {
  int rc = 0;
  std::string err;
  uint64_t deg = 0, nweak = 0;
  size_t nfar = 0;
  int dmax = 1, irr_tmax = 0;
  std::vector<uint32_t> key;   // this chunk's distinct near targets, in first-seen order
  std::vector<uint64_t> rows;  // [key][cw]: the chunk's words of each column
  std::vector<uint64_t> far;
  std::vector<uint64_t> irr;  // edges outside the round contract (general.hpp irr_pack)
};

// The slot pass of round i (insertion order, presence).  An id may repeat (the
// reference appends whatever uponDeliver / the buffer loop hands it,
// process.go:158-169, :229): every slot stays, the packed row is the id's one
// vertex as path()'s lookup sees it (its last slot, :112-116).
int build_slots(const PackedRounds &in, int i, BuiltRounds &out, std::string &err) {
  const int n = in.n, r = in.r0 + i;
  uint64_t *P = &out.pres[(size_t)i * in.WS];
  HostRound &h = out.rounds[i];
  h.slots.reserve(in.slot_off[i + 1] - in.slot_off[i]);
  for (uint32_t sl = in.slot_off[i]; sl < in.slot_off[i + 1]; sl++) {
    const int s = in.slot_src[sl];
    if (s > n) return failf(err, DR_E_CONTRACT, "round %d slot %u: source %d > n=%d", r, sl - in.slot_off[i], s, n);
    h.slots.push_back((uint16_t)s);
    if (s == 0) continue;  // ghost slot {0,0}
    P[(s - 1) >> 6] |= 1ULL << ((s - 1) & 63);
  }
  return 0;
}

// tab is this thread's (delta, t) -> local column table, all -1 on entry and exit
void build_chunk(const PackedRounds &in, int i, int s_lo, int s_hi, std::vector<int32_t> &tab, BuiltRounds &out,
                 Chunk &ck) {
  const int n = in.n, W = in.W, r = in.r0 + i;
  const int w_lo = s_lo >> 6, cw = (s_hi - s_lo + 63) >> 6;
  const uint64_t lastmask = (n % 64) ? ((1ULL << (n % 64)) - 1ULL) : ~0ULL;
  const uint64_t *P = &out.pres[(size_t)i * in.WS];
  std::vector<uint32_t> touched;
  int32_t *tb = tab.data();
  const uint32_t *wt = in.weak_tgt;
  int dm = ck.dmax;
  std::string &err = ck.err;
  for (int s0 = s_lo; s0 < s_hi; s0++) {
    const bool here = (P[s0 >> 6] >> (s0 & 63)) & 1ULL;
    const uint64_t *row = in.strong + ((size_t)i * n + s0) * W;
    uint64_t d = 0, any = 0;
    for (int w = 0; w < W; w++) { d += (uint64_t)__builtin_popcountll(row[w]); any |= row[w]; }
    if (any && !here) { ck.rc = failf(err, DR_E_CONTRACT, "round %d: strong edges on absent vertex (%d,%d)", r, r, s0 + 1); break; }
    if (any && r == 0) { ck.rc = failf(err, DR_E_CONTRACT, "round 0 vertex (0,%d) has strong edges", s0 + 1); break; }
    if (row[W - 1] & ~lastmask) {
      ck.rc = failf(err, DR_E_CONTRACT, "round %d vertex (%d,%d): strong target source > n", r, r, s0 + 1);
      break;
    }
    const uint32_t ea = in.weak_off[(size_t)i * n + s0], eb = in.weak_off[(size_t)i * n + s0 + 1];
    if (eb < ea) { ck.rc = failf(err, DR_E_INVAL, "weak_off not monotone at round %d", r); break; }
    if (eb > ea && !here) { ck.rc = failf(err, DR_E_CONTRACT, "round %d: weak edges on absent vertex (%d,%d)", r, r, s0 + 1); break; }
    const uint64_t mybit = 1ULL << (s0 & 63);
    const int myword = (s0 >> 6) - w_lo;
    uint64_t *rows = ck.rows.data();  // re-read after a new column grows it
    uint32_t nsx = 0;  // strong edges outside the row (bit 31)
    for (uint32_t e = ea; e < eb; e++) {
      const uint32_t t = wt[e];
      const bool sx = (t >> 31) != 0;
      const int tr = (int)((t >> 11) & 0xFFFFFu), ts = (int)(t & 2047u);
      if (ts >= n || tr >= in.max_rounds || (sx && tr == r - 1)) {
        ck.rc = ts >= n          ? failf(err, DR_E_CONTRACT, "edge (%d,%d)->(%d,%d): source > n", r, s0 + 1, tr, ts + 1)
                : !sx || tr != r - 1 ? failf(err, DR_E_CONTRACT, "edge (%d,%d)->(%d,%d): round >= max_rounds %d", r,
                                             s0 + 1, tr, ts + 1, in.max_rounds)
                                     : failf(err, DR_E_CONTRACT, "strong edge (%d,%d)->(%d,%d) belongs in the row", r,
                                             s0 + 1, tr, ts + 1);
        break;
      }
      if (sx || tr > r - 2) {  // outside the round contract (App. A Q8): kept for the general sweep / exception test
        ck.irr.push_back(((uint64_t)s0 << 32) | ((uint64_t)(sx ? 1u : 0u) << 31) | ((uint64_t)tr << 11) | (uint64_t)ts);
        ck.irr_tmax = tr > ck.irr_tmax ? tr : ck.irr_tmax;
        nsx += sx ? 1u : 0u;
        continue;
      }
      const int delta = r - tr;
      if (delta <= 1023) {
        const size_t at = (size_t)delta * n + ts;
        if (at >= tab.size()) {  // grow to this delta (+ slack); new entries -1 like the rest
          tab.resize(std::min<size_t>(1024, (size_t)delta + 9) * n, -1);
          tb = tab.data();
        }
        int32_t col = tb[at];
        if (col < 0) {
          col = tb[at] = (int32_t)ck.key.size();
          touched.push_back((uint32_t)at);
          ck.key.push_back(((uint32_t)delta << 11) | (uint32_t)ts);
          ck.rows.resize(ck.rows.size() + cw, 0ULL);
          rows = ck.rows.data();
        }
        rows[(size_t)col * cw + myword] |= mybit;
        dm = delta > dm ? delta : dm;
      } else {
        ck.far.push_back(((uint64_t)s0 << 32) | t);
        ck.nfar++;
      }
    }
    if (ck.rc) break;
    d += nsx;  // a vertex's strong degree counts every strong edge
    ck.deg += d;
    out.sdeg[(size_t)i * n + s0] = (uint16_t)std::min<uint64_t>(d, 65535u);
    out.wdeg[(size_t)i * n + s0] = (uint16_t)std::min<uint32_t>(eb - ea - nsx, 65535u);
    ck.nweak += eb - ea - nsx;
  }
  ck.dmax = dm;
  for (uint32_t at : touched) tab[at] = -1;
}

// Round i's columns: the union of its chunks' keys, sorted (wc_add's binary
// search relies on it), each row the chunks' words side by side.
void merge_round(const PackedRounds &in, int i, const Chunk *ck, int nch, int chunk, BuiltRounds &out) {
  const int WS = in.WS, n = in.n;
  HostRound &h = out.rounds[i];
  std::vector<uint32_t> keys;
  for (int c = 0; c < nch; c++) keys.insert(keys.end(), ck[c].key.begin(), ck[c].key.end());
  std::sort(keys.begin(), keys.end());
  keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
  h.wc_key = keys;
  h.wc_rows.assign(keys.size() * WS, 0ULL);
  for (int c = 0; c < nch; c++) {
    const Chunk &x = ck[c];
    const int s_lo = c * chunk, w_lo = s_lo >> 6, cw = (std::min(n, s_lo + chunk) - s_lo + 63) >> 6;
    for (size_t j = 0; j < x.key.size(); j++) {
      const size_t col = std::lower_bound(keys.begin(), keys.end(), x.key[j]) - keys.begin();
      std::memcpy(&h.wc_rows[col * WS + w_lo], &x.rows[j * cw], (size_t)cw * 8);
    }
    h.deg += x.deg;
    h.nweak += x.nweak;
    h.far.insert(h.far.end(), x.far.begin(), x.far.end());
    h.irr.insert(h.irr.end(), x.irr.begin(), x.irr.end());
  }
}

}  // namespace

int build_packed_rounds(const PackedRounds &in, int dmax0, BuiltRounds &out, std::string &err, BuildScratch &scr) {
  const int k = in.k, n = in.n;
  out.rounds.assign(k, HostRound{});
  out.pres.assign((size_t)k * in.WS, 0);
  out.sdeg.assign((size_t)k * n, 0);
  out.wdeg.assign((size_t)k * n, 0);
  const uint64_t nweak = in.weak_off[(size_t)k * n] - in.weak_off[0];
  const bool par = nweak >= 8192;  // thread start-up costs more than tiny appends
  const int nthr = par ? std::max(1, omp_get_max_threads()) : 1;
  // source chunks per round: enough (round, chunk) tasks for every thread, 64-aligned
  const int nwords = (n + 63) / 64;
  const int nch = std::max(1, std::min(nwords, (nthr + k - 1) / k));
  const int chunk = ((nwords + nch - 1) / nch) * 64;
  const int ntask = k * nch;
  std::vector<int> src(k, 0);
  std::vector<std::string> smsg(k);
  std::vector<Chunk> ck((size_t)ntask);
  for (auto &c : ck) c.dmax = dmax0;
  const int nth = std::max(1, std::min(ntask, nthr));  // no idle team members
  if ((int)scr.tab.size() < nth) scr.tab.resize(nth);
  for (auto &t : scr.tab)
    if (!t.empty() && t.size() % n) t.clear();  // sized for another n: start over
#pragma omp parallel num_threads(nth) if (par)
  {
    // this thread's table, kept across calls in the context (all -1 between uses)
    std::vector<int32_t> &tab = scr.tab[par ? omp_get_thread_num() : 0];
#pragma omp for schedule(static)
    for (int i = 0; i < k; i++) src[i] = build_slots(in, i, out, smsg[i]);  // presence before the chunks
#pragma omp for schedule(dynamic, 1)
    for (int t = 0; t < ntask; t++) {
      const int i = t / nch, c = t % nch;
      const int s_lo = c * chunk, s_hi = std::min(n, s_lo + chunk);
      if (src[i] == 0 && s_lo < s_hi) build_chunk(in, i, s_lo, s_hi, tab, out, ck[t]);
    }
#pragma omp for schedule(static)
    for (int i = 0; i < k; i++)
      if (src[i] == 0) merge_round(in, i, &ck[(size_t)i * nch], nch, chunk, out);
  }
  // errors as a sequential pass over the rounds reports them: a round's slot pass,
  // then its sources in order
  out.nfar = 0;
  out.dmax = dmax0;
  for (int i = 0; i < k; i++) {
    if (src[i]) {
      err = smsg[i];
      return src[i];
    }
    for (int c = 0; c < nch; c++) {
      const Chunk &x = ck[(size_t)i * nch + c];
      if (x.rc) {
        err = x.err;
        return x.rc;
      }
      out.nfar += x.nfar;
      out.nirr += x.irr.size();
      out.irr_tmax = std::max(out.irr_tmax, x.irr_tmax);
      out.dmax = std::max(out.dmax, x.dmax);
    }
  }
  return 0;
}

}  // namespace dr_host
