// host_rounds.cpp -- validation and host-state build of pre-packed rounds
// (dr_append_rounds_packed), one round per OpenMP thread.  The weak-column
// build is a table lookup per weak edge (C4: ~33 K weak edges per round), which
// a per-wave append of 4 rounds paid serially.
#include "host_rounds.hpp"

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>

#include <omp.h>

#include "dagrider_gpu.h"

namespace dr_host {
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

// one round; tab is this thread's (delta, t) -> column table, all -1 on entry and exit
int build_one(const PackedRounds &in, int i, std::vector<int32_t> &tab, BuiltRounds &out, size_t &nfar, int &dmax,
              std::string &err) {
  const int n = in.n, W = in.W, WS = in.WS, r = in.r0 + i;
  const uint64_t lastmask = (n % 64) ? ((1ULL << (n % 64)) - 1ULL) : ~0ULL;
  uint64_t *P = &out.pres[(size_t)i * WS];
  HostRound &h = out.rounds[i];
  for (uint32_t sl = in.slot_off[i]; sl < in.slot_off[i + 1]; sl++) {
    const int s = in.slot_src[sl];
    if (s > n) return failf(err, DR_E_CONTRACT, "round %d slot %u: source %d > n=%d", r, sl - in.slot_off[i], s, n);
    h.slots.push_back((uint16_t)s);
    if (s == 0) continue;  // ghost slot {0,0}
    uint64_t &wd = P[(s - 1) >> 6];
    const uint64_t bit = 1ULL << ((s - 1) & 63);
    if ((wd & bit) && r >= 1) return failf(err, DR_E_CONTRACT, "round %d: duplicate vertex id (%d,%d)", r, r, s);
    wd |= bit;
  }
  std::vector<uint32_t> touched;
  int rc = 0;
  for (int s0 = 0; s0 < n && !rc; s0++) {
    const bool here = (P[s0 >> 6] >> (s0 & 63)) & 1ULL;
    const uint64_t *row = in.strong + ((size_t)i * n + s0) * W;
    uint64_t d = 0, any = 0;
    for (int w = 0; w < W; w++) { d += (uint64_t)__builtin_popcountll(row[w]); any |= row[w]; }
    if (any && !here) { rc = failf(err, DR_E_CONTRACT, "round %d: strong edges on absent vertex (%d,%d)", r, r, s0 + 1); break; }
    if (any && r == 0) { rc = failf(err, DR_E_CONTRACT, "round 0 vertex (0,%d) has strong edges", s0 + 1); break; }
    if (row[W - 1] & ~lastmask) {
      rc = failf(err, DR_E_CONTRACT, "round %d vertex (%d,%d): strong target source > n", r, r, s0 + 1);
      break;
    }
    h.deg += d;
    out.sdeg[(size_t)i * n + s0] = (uint16_t)d;
    const uint32_t ea = in.weak_off[(size_t)i * n + s0], eb = in.weak_off[(size_t)i * n + s0 + 1];
    if (eb < ea) { rc = failf(err, DR_E_INVAL, "weak_off not monotone at round %d", r); break; }
    if (eb > ea && !here) { rc = failf(err, DR_E_CONTRACT, "round %d: weak edges on absent vertex (%d,%d)", r, r, s0 + 1); break; }
    out.wdeg[(size_t)i * n + s0] = (uint16_t)std::min<uint32_t>(eb - ea, 65535u);
    h.nweak += eb - ea;
    const uint64_t mybit = 1ULL << (s0 & 63);
    const int myword = s0 >> 6;
    const uint32_t *wt = in.weak_tgt;
    int32_t *tb = tab.data();
    uint64_t *rows = h.wc_rows.data();  // re-read after a new column grows it
    int dm = dmax;
    for (uint32_t e = ea; e < eb; e++) {
      const uint32_t t = wt[e];
      const int tr = (int)(t >> 11), ts = (int)(t & 2047u);
      if (ts >= n || tr > r - 2) {
        rc = ts >= n ? failf(err, DR_E_CONTRACT, "weak edge (%d,%d)->(%d,%d): source > n", r, s0 + 1, tr, ts + 1)
                     : failf(err, DR_E_CONTRACT, "weak edge (%d,%d)->(%d,%d) must target a round < r-1", r, s0 + 1, tr,
                             ts + 1);
        break;
      }
      const int delta = r - tr;
      if (delta <= 1023) {
        const size_t at = (size_t)delta * n + ts;
        int32_t col = tb[at];
        if (col < 0) {
          col = tb[at] = (int32_t)h.wc_key.size();
          touched.push_back((uint32_t)at);
          h.wc_key.push_back(((uint32_t)delta << 11) | (uint32_t)ts);
          h.wc_rows.resize(h.wc_rows.size() + WS, 0ULL);
          rows = h.wc_rows.data();
        }
        rows[(size_t)col * WS + myword] |= mybit;
        dm = delta > dm ? delta : dm;
      } else {
        h.far.push_back(((uint64_t)s0 << 32) | t);
        nfar++;
      }
    }
    dmax = dm;
  }
  for (uint32_t at : touched) tab[at] = -1;
  if (rc) return rc;
  // columns sorted by key (wc_add's binary search relies on it; no kernel does)
  const size_t nk = h.wc_key.size();
  bool sorted = true;
  for (size_t x = 1; x < nk && sorted; x++) sorted = h.wc_key[x - 1] < h.wc_key[x];
  if (!sorted) {
    std::vector<uint32_t> order(nk);
    for (size_t x = 0; x < nk; x++) order[x] = (uint32_t)x;
    std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return h.wc_key[a] < h.wc_key[b]; });
    std::vector<uint32_t> keys(nk);
    std::vector<uint64_t> rows(nk * WS);
    for (size_t x = 0; x < nk; x++) {
      keys[x] = h.wc_key[order[x]];
      std::memcpy(&rows[x * WS], &h.wc_rows[(size_t)order[x] * WS], (size_t)WS * 8);
    }
    h.wc_key.swap(keys);
    h.wc_rows.swap(rows);
  }
  return 0;
}

}  // namespace

int build_packed_rounds(const PackedRounds &in, int dmax0, BuiltRounds &out, std::string &err) {
  const int k = in.k, n = in.n;
  out.rounds.assign(k, HostRound{});
  out.pres.assign((size_t)k * in.WS, 0);
  out.sdeg.assign((size_t)k * n, 0);
  out.wdeg.assign((size_t)k * n, 0);
  std::vector<int> rc(k, 0), dm(k, dmax0);
  std::vector<size_t> nf(k, 0);
  std::vector<std::string> msg(k);
  const uint64_t nweak = in.weak_off[(size_t)k * n] - in.weak_off[0];
  const bool par = k > 1 && nweak >= 8192;  // thread start-up costs more than tiny rounds
  const int nth = std::max(1, std::min(k, omp_get_max_threads()));  // no idle team members
#pragma omp parallel num_threads(nth) if (par)
  {
    // per thread, kept across calls (all -1 between uses): (delta, t) -> column
    static thread_local std::vector<int32_t> tab;
    if (tab.size() < (size_t)1024 * n) tab.assign((size_t)1024 * n, -1);
#pragma omp for schedule(dynamic, 1)
    for (int i = 0; i < k; i++) rc[i] = build_one(in, i, tab, out, nf[i], dm[i], msg[i]);
  }
  out.nfar = 0;
  out.dmax = dmax0;
  for (int i = 0; i < k; i++) {
    if (rc[i]) {
      err = msg[i];
      return rc[i];
    }
    out.nfar += nf[i];
    out.dmax = std::max(out.dmax, dm[i]);
  }
  return 0;
}

}  // namespace dr_host
