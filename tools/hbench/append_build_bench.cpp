#ifndef DIR
#define DIR "/tmp/hbdata"
#endif
#include "host_rounds.hpp"
#include <chrono>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <omp.h>
template <class T> std::vector<T> rd(const char *p) {
  FILE *f = fopen(p, "rb"); fseek(f, 0, SEEK_END); long s = ftell(f); fseek(f, 0, SEEK_SET);
  std::vector<T> v(s / sizeof(T)); fread(v.data(), 1, s, f); fclose(f); return v; }
namespace dr_host_old { int build_packed_rounds(const dr_host::PackedRounds &in, int dmax0, dr_host::BuiltRounds &out, std::string &err, dr_host::BuildScratch &scr); }
int main(int argc, char **argv) {
  auto so = rd<uint32_t>(DIR "/slot_off.bin"); auto ss = rd<uint16_t>(DIR "/slot_src.bin");
  auto st = rd<uint64_t>(DIR "/strong.bin"); auto wo = rd<uint32_t>(DIR "/weak_off.bin");
  auto wt = rd<uint32_t>(DIR "/weak_tgt.bin");
  const int n = 1024, W = 16; dr_host::BuildScratch scr; unsigned long long cks = 0; std::vector<double> ts; int dmax = 1;
  int nw = argc > 1 ? atoi(argv[1]) : 300; bool old = argc > 2 && atoi(argv[2]); const int gap_us = argc > 3 ? atoi(argv[3]) : 0; const bool keep = argc > 4 && atoi(argv[4]); std::vector<dr_host::HostRound> kept;
  for (int w = 0; w <= nw; w++) {
    int r0 = w == 0 ? 0 : 4 * w - 3, r1 = w == 0 ? 1 : 4 * w + 1;
    dr_host::PackedRounds in; in.n = n; in.W = W; in.WS = W; in.r0 = r0; in.k = r1 - r0; in.max_rounds = 4001;
    std::vector<uint32_t> sof(so.begin() + r0, so.begin() + r1 + 1);
    std::vector<uint32_t> wof(wo.begin() + (size_t)r0 * n, wo.begin() + (size_t)r1 * n + 1);
    in.slot_off = sof.data(); in.slot_src = ss.data(); in.strong = st.data() + (size_t)r0 * n * W;
    in.weak_off = wof.data(); in.weak_tgt = wt.data();
    dr_host::BuiltRounds b; std::string err;
    auto t0 = std::chrono::steady_clock::now();
    int rc = old ? dr_host_old::build_packed_rounds(in, dmax, b, err, scr) : dr_host::build_packed_rounds(in, dmax, b, err, scr);
    auto t1 = std::chrono::steady_clock::now();
    if (rc) { printf("rc %d %s\n", rc, err.c_str()); return 1; }
    dmax = b.dmax; for (auto &hr : b.rounds) { for (auto k : hr.wc_key) cks = cks * 1000003u + k; for (auto x : hr.wc_rows) cks = cks * 1000003u + x; for (auto s2 : hr.slots) cks = cks*31u + s2; cks += hr.deg * 7 + hr.nweak; } for (auto x : b.pres) cks = cks * 1000003u + x; for (auto x : b.sdeg) cks = cks*31u + x; for (auto x : b.wdeg) cks = cks*31u+x;
    if (gap_us) { auto g0 = std::chrono::steady_clock::now(); while (std::chrono::steady_clock::now() - g0 < std::chrono::microseconds(gap_us)) {} }
    if (keep) for (auto &h : b.rounds) kept.push_back(std::move(h));
    if (w > 0) ts.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
  }
  std::sort(ts.begin(), ts.end());
  printf("cks %llx ", cks);
  printf("threads %d: p50 %.1f us p90 %.1f min %.1f\n", omp_get_max_threads(), ts[ts.size() / 2], ts[ts.size() * 9 / 10], ts[0]);
}
