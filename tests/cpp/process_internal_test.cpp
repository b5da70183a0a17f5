// C++ port of the reference's hot-path tests, run against the GPU through the host
// mirror (dag_rider_amd/host/process.hpp):
//   TestPath   process/process_internal_test.go:8-84 (Figure-1 DAG, createDag :86-283)
//   TestStack  stack/stack_test.go:9-18
// plus the SURVEY.md s4 derived answers for waveReady(1) and orderVertices.
// Exit status 0 iff every check passes.
#include <cstdio>
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

  std::printf("%s (%d failures)\n", failures ? "FAIL" : "OK", failures);
  return failures ? 1 : 0;
}
