// dag_gen.cpp -- synthetic DAG-Rider DAG generator (spec: include/dagrider_gen.h).
//
// Host code: runs once per workload, outside every timed region.  Parallel over
// vertices with OpenMP; each draw comes from a per-(round, source, purpose)
// splitmix64 stream, so the output does not depend on the thread count.
#include "dagrider_gen.h"

#include <omp.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

namespace {

inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

enum Stream : uint64_t { kPresent = 1, kTopup, kSlots, kLate, kStrongK, kStrong, kWeak };

struct Rng {
  uint64_t s;
  Rng(uint64_t seed, uint64_t r, uint64_t src, uint64_t stream)
      : s(mix64(seed ^ mix64((r << 24) ^ (src << 4) ^ stream))) {}
  uint64_t next() { s += 0x9E3779B97F4A7C15ULL; return mix64(s); }
  double u01() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
  bool bern(double p) { return u01() < p; }
};

}  // namespace

struct dr_gen_dag {
  int32_t n = 0, W = 0, nrounds = 0;
  std::vector<uint32_t> slot_off;
  std::vector<uint16_t> slot_src;
  std::vector<uint64_t> strong;
  std::vector<uint32_t> weak_off;
  std::vector<uint32_t> weak_tgt;
};

extern "C" int dr_gen_create(const dr_gen_params *prm, dr_gen_dag **out) {
  if (!prm || !out) return -1;
  const int n = prm->n, R = prm->last_round;
  if (n < 1 || n > 2048 || R < 0 || R >= (1 << 20) || prm->weak_depth < 0) return -1;
  if (prm->nthreads > 0) omp_set_num_threads(prm->nthreads);
  const int f = (n - 1) / 3, q = 2 * f + 1, W = (n + 63) / 64, NR = R + 1;
  dr_gen_dag *g = new (std::nothrow) dr_gen_dag();
  if (!g) return -1;
  g->n = n;
  g->W = W;
  g->nrounds = NR;
  const uint64_t seed = prm->seed;

  // Phase A (per round, cheap, parallel over rounds): presence, slot order, late set.
  std::vector<std::vector<uint16_t>> slots(NR);
  std::vector<std::vector<uint8_t>> late(NR, std::vector<uint8_t>(n, 0));
  std::vector<std::vector<uint16_t>> eligible(NR);  // present \ late, ascending
  std::vector<std::vector<uint16_t>> latelist(NR);  // late, ascending
#pragma omp parallel for schedule(static)
  for (int r = 0; r < NR; r++) {
    std::vector<uint8_t> pres(n, 0);
    if (r == 0) {
      std::fill(pres.begin(), pres.end(), 1);
      for (int s = 1; s <= n; s++) slots[r].push_back((uint16_t)s);
    } else {
      const bool leader_round = ((r - 1) & 3) == 0;
      bool leader_absent = false;
      int cnt = 0;
      for (int s = 1; s <= n; s++) {
        Rng rg(seed, r, s, kPresent);
        bool p;
        if (s == 1 && leader_round) { p = !rg.bern(prm->p_la); leader_absent = !p; }
        else p = rg.bern(prm->p_present);
        pres[s - 1] = p;
        cnt += p;
      }
      if (cnt < q) {
        Rng rg(seed, r, 0, kTopup);
        int o = (int)(rg.next() % (uint64_t)n);
        for (int i = 0; i < n && cnt < q; i++) {
          int s = 1 + (o + i) % n;
          if (pres[s - 1] || (s == 1 && leader_absent)) continue;
          pres[s - 1] = 1;
          cnt++;
        }
      }
      std::vector<uint16_t> v;
      for (int s = 1; s <= n; s++) if (pres[s - 1]) v.push_back((uint16_t)s);
      Rng rg(seed, r, 0, kSlots);
      for (int i = (int)v.size() - 1; i > 0; i--) {
        int j = (int)(rg.next() % (uint64_t)(i + 1));
        std::swap(v[i], v[j]);
      }
      slots[r] = std::move(v);
      // late set: never referenced by round r+1's strong edges
      int cap = std::min(f, cnt - q);
      int nl = 0;
      for (int s = 1; s <= n && nl < cap; s++) {
        if (!pres[s - 1]) continue;
        Rng lr(seed, r, s, kLate);
        if (lr.bern(prm->p_late)) { late[r][s - 1] = 1; nl++; }
      }
    }
    for (int s = 1; s <= n; s++) {
      if (!pres[s - 1]) continue;
      if (late[r][s - 1]) latelist[r].push_back((uint16_t)s);
      else eligible[r].push_back((uint16_t)s);
    }
  }
  g->slot_off.resize(NR + 1);
  g->slot_off[0] = 0;
  for (int r = 0; r < NR; r++) g->slot_off[r + 1] = g->slot_off[r] + (uint32_t)slots[r].size();
  g->slot_src.resize(g->slot_off[NR]);
  for (int r = 0; r < NR; r++)
    std::copy(slots[r].begin(), slots[r].end(), g->slot_src.begin() + g->slot_off[r]);

  // Phase B: strong rows (selection sampling) + weak degree, parallel over vertices.
  g->strong.assign((size_t)NR * n * W, 0);
  std::vector<uint32_t> wdeg((size_t)NR * n, 0);
  const int D = prm->weak_depth;
#pragma omp parallel for schedule(dynamic, 1)
  for (int r = 1; r < NR; r++) {
    const std::vector<uint16_t> &E = eligible[r - 1];
    const int m = (int)E.size();
    for (uint16_t s : slots[r]) {
      uint64_t *row = &g->strong[((size_t)r * n + (s - 1)) * W];
      Rng kr(seed, r, s, kStrongK);
      int lo = std::min(q, m);
      int k = lo + (int)(kr.next() % (uint64_t)(m - lo + 1));
      Rng sr(seed, r, s, kStrong);
      int chosen = 0;
      for (int i = 0; i < m && chosen < k; i++) {
        if (sr.u01() * (double)(m - i) < (double)(k - chosen)) {
          int t = E[i] - 1;
          row[t >> 6] |= 1ULL << (t & 63);
          chosen++;
        }
      }
      // weak degree
      uint32_t cnt = 0;
      Rng wr(seed, r, s, kWeak);
      for (int r2 = std::max(1, r - D); r2 <= r - 2; r2++)
        for (size_t i = 0; i < latelist[r2].size(); i++) cnt += wr.bern(prm->p_w);
      wdeg[(size_t)r * n + (s - 1)] = cnt;
    }
  }
  g->weak_off.resize((size_t)NR * n + 1);
  uint64_t acc = 0;
  for (size_t i = 0; i < (size_t)NR * n; i++) {
    g->weak_off[i] = (uint32_t)acc;
    acc += wdeg[i];
  }
  if (acc > 0xFFFFFFFFull) { delete g; return -1; }
  g->weak_off[(size_t)NR * n] = (uint32_t)acc;
  g->weak_tgt.resize(acc);
#pragma omp parallel for schedule(dynamic, 1)
  for (int r = 1; r < NR; r++) {
    for (uint16_t s : slots[r]) {
      uint32_t *dst = g->weak_tgt.data() + g->weak_off[(size_t)r * n + (s - 1)];
      Rng wr(seed, r, s, kWeak);
      for (int r2 = std::max(1, r - D); r2 <= r - 2; r2++)
        for (uint16_t u : latelist[r2])
          if (wr.bern(prm->p_w)) *dst++ = ((uint32_t)r2 << 11) | (uint32_t)(u - 1);
    }
  }
  *out = g;
  return 0;
}

extern "C" void dr_gen_free(dr_gen_dag *g) { delete g; }

extern "C" int dr_gen_info(const dr_gen_dag *g, int32_t *n, int32_t *W, int32_t *nrounds,
                           uint64_t *nslots, uint64_t *nweak) {
  if (!g) return -1;
  if (n) *n = g->n;
  if (W) *W = g->W;
  if (nrounds) *nrounds = g->nrounds;
  if (nslots) *nslots = g->slot_src.size();
  if (nweak) *nweak = g->weak_tgt.size();
  return 0;
}
extern "C" const uint32_t *dr_gen_slot_off(const dr_gen_dag *g) { return g->slot_off.data(); }
extern "C" const uint16_t *dr_gen_slot_src(const dr_gen_dag *g) { return g->slot_src.data(); }
extern "C" const uint64_t *dr_gen_strong(const dr_gen_dag *g) { return g->strong.data(); }
extern "C" const uint32_t *dr_gen_weak_off(const dr_gen_dag *g) { return g->weak_off.data(); }
extern "C" const uint32_t *dr_gen_weak_tgt(const dr_gen_dag *g) { return g->weak_tgt.data(); }
