// C++ port of the reference's hot-path tests, run against the GPU through the host
// mirror (dag_rider_amd/host/process.hpp):
//   TestPath   process/process_internal_test.go:8-84 (Figure-1 DAG, createDag :86-283)
//   TestStack  stack/stack_test.go:9-18
// plus the SURVEY.md s4 derived answers for waveReady(1) and orderVertices, the
// buffer pass, and an incremental mirror checked against a literal path().
// Exit status 0 iff every check passes.
#include <cstdio>
#include <deque>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "process.hpp"

using namespace dagrider;

static int failures = 0;
#define REQUIRE(cond, name)                                        \
  do {                                                             \
    bool ok_ = (cond);                                             \
    std::printf("%s %s\n", ok_ ? "PASS" : "FAIL", name);           \
    if (!ok_) failures++;                                          \
  } while (0)

static std::vector<vertexID> E(std::initializer_list<std::pair<int, int>> l) {
  std::vector<vertexID> v;
  for (auto &x : l) v.push_back(vertexID{x.first, x.second});
  return v;
}

// createDag: rounds 0..4, 5 slots each, slot 0 left zero-valued.
static std::vector<std::vector<vertex>> createDag(int rounds, int numprocs) {
  std::vector<std::vector<vertex>> dag(rounds);
  for (int r = 0; r <= 4; r++) {
    dag[r].resize(numprocs);
    for (int p = 1; p <= 4; p++) dag[r][p].id = vertexID{r, p};
  }
  for (int p = 1; p <= 4; p++) dag[1][p].strongEdges = E({{0, 1}, {0, 2}, {0, 3}});
  dag[2][1].strongEdges = E({{1, 1}, {1, 2}, {1, 4}});
  dag[2][2].strongEdges = E({{1, 1}, {1, 2}, {1, 4}});
  dag[2][3].strongEdges = E({{1, 1}, {1, 3}, {1, 4}});
  dag[2][4].strongEdges = E({{1, 1}, {1, 2}, {1, 4}});
  dag[3][1].strongEdges = E({{2, 1}, {2, 3}});
  dag[3][2].strongEdges = E({{2, 1}, {2, 2}, {2, 3}});
  dag[3][3].strongEdges = E({{2, 1}, {2, 2}, {2, 3}});
  dag[4][1].strongEdges = E({{3, 1}, {3, 2}, {3, 3}});
  dag[4][1].weakEdges = E({{2, 4}});
  return dag;
}

// literal path() (process.go:89-148): BFS with a visited set, last-match lookup
static bool ref_path(const Dag &dag, vertexID from, vertexID to, bool strong) {
  if (from == to) return true;
  std::set<std::pair<int, int>> visited{{from.round, from.source}};
  std::deque<vertexID> q{from};
  while (!q.empty()) {
    const vertexID id = q.front();
    q.pop_front();
    const vertex *v = nullptr;
    if (id.round >= 0 && id.round < (int)dag.size())
      for (const vertex &t : dag[id.round])
        if (t.id == id) v = &t;
    if (!v) continue;
    for (const auto *es : {&v->strongEdges, &v->weakEdges}) {
      if (es == &v->weakEdges && strong) break;
      for (const vertexID &e : *es) {
        if (!visited.insert({e.round, e.source}).second) continue;
        if (e == to) return true;
        q.push_back(e);
      }
    }
  }
  return false;
}

// Vertices arrive one at a time in a random causal order (late ones into old
// rounds, as the buffer loop admits them): process A mirrors p.dag
// incrementally (dr_append_vertices), B gets the whole DAG assigned before
// every check (full upload); both must agree with each other and with the
// literal path() on every query.
static void incremental_checks() {
  const int n = 8, f = 2, R = 14;
  uint64_t st = 0x9E3779B97F4A7C15ULL;
  auto rnd = [&]() { st = st * 6364136223846793005ULL + 1442695040888963407ULL; return (double)(st >> 11) / 9007199254740992.0; };
  Dag::Rounds full(R + 1);
  for (int s = 1; s <= n; s++) full[0].push_back(vertex{{0, s}, {}, {}, {}});
  for (int r = 1; r <= R; r++)
    for (int s = 1; s <= n; s++) {
      if (rnd() > 0.85) continue;
      vertex v{{r, s}, {}, {}, {}};
      for (const vertex &u : full[r - 1])
        if (rnd() < 0.6) v.strongEdges.push_back(u.id);
      for (int r2 = std::max(0, r - 6); r2 <= r - 2; r2++)
        for (const vertex &u : full[r2])
          if (rnd() < 0.08) v.weakEdges.push_back(u.id);
      full[r].push_back(v);
    }
  // causal arrival order
  std::vector<std::pair<int, int>> order, ready;
  std::map<std::pair<int, int>, int> need;
  std::map<std::pair<int, int>, std::vector<std::pair<int, int>>> users;
  for (int r = 0; r <= R; r++)
    for (size_t i = 0; i < full[r].size(); i++) {
      const vertex &v = full[r][i];
      int k = 0;
      for (const auto *es : {&v.strongEdges, &v.weakEdges})
        for (const vertexID &e : *es) {
          int slot = -1;
          for (size_t j = 0; j < full[e.round].size(); j++)
            if (full[e.round][j].id == e) slot = (int)j;
          if (slot < 0) continue;
          users[{e.round, slot}].push_back({r, (int)i});
          k++;
        }
      need[{r, (int)i}] = k;
      if (!k) ready.push_back({r, (int)i});
    }
  while (!ready.empty()) {
    const size_t at = (size_t)(rnd() * ready.size()) % ready.size();
    const auto x = ready[at];
    ready.erase(ready.begin() + (ptrdiff_t)at);
    order.push_back(x);
    for (const auto &u : users[x])
      if (--need[u] == 0) ready.push_back(u);
  }
  Transport ta, tb;
  std::vector<std::pair<int, int>> sa, sb;
  ta.Subscribe([&](const bcastMsg &m) { sa.push_back({m.round, m.sender}); });
  tb.Subscribe([&](const bcastMsg &m) { sb.push_back({m.round, m.sender}); });
  std::string err;
  auto A = Process::New(1, f, &ta, &err), B = Process::New(1, f, &tb, &err);
  A->dag = Dag::Rounds(1);
  bool paths_ok = true, waves_ok = true, order_ok = true;
  int checks = 0;
  for (size_t k = 0; k < order.size(); k++) {
    const auto x = order[k];
    if ((int)A->dag.size() <= x.first) A->dag.grow((size_t)x.first + 1 - A->dag.size());
    A->dag.append((size_t)x.first, full[x.first][x.second]);
    if (k % 4 != 3 && k + 1 != order.size()) continue;
    checks++;
    B->dag = A->dag.rounds();
    const int top = (int)A->dag.size() - 1;
    std::vector<vertexID> ids;
    for (int r = 0; r <= top; r++)
      for (size_t i = 0; i < A->dag[r].size(); i++) ids.push_back(A->dag[r][i].id);
    for (int q = 0; q < 24; q++) {
      const vertexID a = ids[(size_t)(rnd() * ids.size()) % ids.size()];
      const vertexID b{(int)(rnd() * (a.round + 1)), 1 + (int)(rnd() * n)};
      const bool s = rnd() < 0.5;
      const bool want = ref_path(A->dag, a, b, s);
      paths_ok &= A->path(a, b, s) == want && B->path(a, b, s) == want;
    }
    for (int w = 1; 4 * w <= top; w++) {
      for (Process *P : {A.get(), B.get()}) {
        P->decidedWave = 0;
        while (!P->leadersStack.IsEmpty()) P->leadersStack.Pop();
        P->waveReady(w);
      }
      bool same = A->lastVoteCount == B->lastVoteCount && A->decidedWave == B->decidedWave &&
                  A->leadersStack.items().size() == B->leadersStack.items().size();
      for (size_t i = 0; same && i < A->leadersStack.items().size(); i++)
        same = A->leadersStack.items()[i].id == B->leadersStack.items()[i].id;
      waves_ok &= same;
    }
    for (Process *P : {A.get(), B.get()}) {
      while (!P->leadersStack.IsEmpty()) P->leadersStack.Pop();
      P->round = top;
    }
    sa.clear();
    sb.clear();
    const vertexID lead = ids[(size_t)(rnd() * ids.size()) % ids.size()];
    if (lead.round >= 1) {
      for (Process *P : {A.get(), B.get()}) {
        for (const vertex &v : P->dag[lead.round])
          if (v.id == lead) P->leadersStack.Push(v);
        P->orderVertices();
      }
      std::vector<std::pair<int, int>> want;  // rounds 1..top, slot order, reachable from lead
      for (int r = 1; r <= top; r++)
        for (size_t i = 0; i < A->dag[r].size(); i++)
          if (ref_path(A->dag, lead, A->dag[r][i].id, false)) want.push_back({r, A->dag[r][i].id.source});
      order_ok &= sa == want && sb == want;
    }
  }
  std::printf("incremental: %zu arrivals, %d checkpoints\n", order.size(), checks);
  REQUIRE(paths_ok, "incremental/path-matches-literal-and-full-upload");
  REQUIRE(waves_ok, "incremental/waveReady-matches-full-upload");
  REQUIRE(order_ok, "incremental/orderVertices-matches-literal");
}

int main() {
  // TestStack
  {
    auto s = Stack<int>::New();
    REQUIRE(s.IsEmpty(), "TestStack/empty");
    s.Push(1);
    s.Push(2);
    REQUIRE(s.Pop() == 2, "TestStack/pop2");
    REQUIRE(s.Pop() == 1, "TestStack/pop1");
    REQUIRE(s.IsEmpty(), "TestStack/empty-again");
    bool panicked = false;
    try { s.Pop(); } catch (const panic_error &) { panicked = true; }
    REQUIRE(panicked, "TestStack/pop-empty-panics");
  }
  // New rejects index < 1 (process.go:38-40)
  {
    std::string err;
    auto p = Process::New(0, 1, nullptr, &err);
    REQUIRE(!err.empty(), "New/index-0-error");
  }
  const int index = 1, faulty = 1, rounds = 5, numprocs = 5;
  Transport tp;
  std::vector<bcastMsg> sunk;
  tp.Subscribe([&](const bcastMsg &m) { sunk.push_back(m); });
  std::string err;
  auto p = Process::New(index, faulty, &tp, &err);
  p->dag = createDag(rounds, numprocs);

  // TestPath
  REQUIRE(p->path({3, 1}, {2, 3}, true), "TestPath/strong path consecutive rounds");
  REQUIRE(p->path({3, 3}, {1, 4}, true), "TestPath/strong path separated by 2 rounds");
  REQUIRE(p->path({4, 1}, {2, 4}, false), "TestPath/weak path");
  REQUIRE(p->path({4, 1}, {1, 1}, false), "TestPath/hybrid path");
  REQUIRE(!p->path({3, 3}, {2, 4}, false), "TestPath/no path exists");

  // derived: waveReady(1) -> leader (1,1), vCount 1 < 2f+1, no commit
  p->waveReady(1);
  REQUIRE(p->lastVoteCount == 1 && p->leadersStack.IsEmpty() && p->decidedWave == 0, "waveReady(1)/no-commit");

  // derived: orderVertices with stack [(4,1)], p.round = 4 -> 12 vertices
  p->round = 4;
  p->leadersStack.Push(p->dag[4][1]);
  p->orderVertices();
  std::vector<std::pair<int, int>> want = {{1, 1}, {1, 2}, {1, 3}, {1, 4}, {2, 1}, {2, 2},
                                           {2, 3}, {2, 4}, {3, 1}, {3, 2}, {3, 3}, {4, 1}};
  bool same = sunk.size() == want.size();
  for (size_t i = 0; same && i < want.size(); i++)
    same = sunk[i].round == want[i].first && sunk[i].sender == want[i].second;
  REQUIRE(same && p->deliveredVertices.size() == 12 && p->leadersStack.IsEmpty(), "orderVertices/stack[(4,1)]");

  // buffer pass (process.go:200-234) at p.round = 4
  const size_t d4 = p->dag[4].size();
  p->buffer = {vertex{{4, 5}, {}, E({{3, 1}, {3, 2}}), {}},   // all present -> dag[4]
               vertex{{5, 1}, {}, E({{4, 1}}), {}},           // round 5 > p.round: stays
               vertex{{4, 3}, {}, E({{2, 1}}), E({{1, 9}})}};  // (1,9) absent: stays
  p->processBuffer();
  REQUIRE(p->dag[4].size() == d4 + 1 && p->buffer.size() == 2 && p->buffer[0].id == (vertexID{5, 1}),
          "processBuffer/admit-one");
  // at p.round = 5, (5,1) is admitted into p.dag[5], beyond the DAG: Go panics
  p->round = 5;
  bool panicked = false;
  try { p->processBuffer(); } catch (const panic_error &) { panicked = true; }
  REQUIRE(panicked, "processBuffer/dag-index-panics");
  p->round = 4;

  // panics: path from a round beyond the DAG; getWaveVertexLeader(0)
  panicked = false;
  try { p->path({7, 1}, {1, 1}, true); } catch (const panic_error &) { panicked = true; }
  REQUIRE(panicked, "path/out-of-range-panics");
  panicked = false;
  try { p->getWaveVertexLeader(0); } catch (const panic_error &) { panicked = true; }
  REQUIRE(panicked, "getWaveVertexLeader(0)/panics");

  // a re-delivered id is appended as Go appends it (process.go:229): p.dag[3] grows
  // by one slot and path() follows the id's LAST vertex (process.go:112-116)
  {
    p->round = 4;
    const size_t b0 = p->buffer.size(), d3 = p->dag[3].size();
    REQUIRE(p->path({3, 2}, {2, 2}, true), "processBuffer/before-redelivery");
    p->buffer.push_back(vertex{{3, 2}, {}, E({{2, 1}}), {}});  // (3,2) is already in p.dag[3]
    p->processBuffer();
    REQUIRE(p->buffer.size() == b0 && p->dag[3].size() == d3 + 1, "processBuffer/redelivered-appended");
    REQUIRE(!p->path({3, 2}, {2, 2}, true) && p->path({3, 2}, {2, 1}, true), "path/last-match-after-redelivery");
    REQUIRE(p->path({4, 1}, {2, 4}, false), "processBuffer/mirror-still-usable");
  }

  incremental_checks();

  std::printf("%s (%d failures)\n", failures ? "FAIL" : "OK", failures);
  return failures ? 1 : 0;
}
