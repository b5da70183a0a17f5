// process.hpp -- C++ host mirror of the reference's process.Process hot-path API
// over the C ABI (include/dagrider_gpu.h).
//
// Same names, argument meaning and error behaviour as xenowits/dag-rider:
//   vertexID / vertex / block          process/process.go:14-31
//   New / NewForT                      process/process.go:33-70 (index < 1 -> error)
//   Process::dag (assign, then query)  process/process.go:79, process_internal_test.go:18
//   dag.append(r, v)                   p.dag[r] = append(p.dag[r], v), process.go:229
//   path(from, to, strongPath)         process/process.go:87-148
//   waveReady(wave)                    process/process.go:312-354
//   getWaveVertexLeader(w)             process/process.go:356-371
//   orderVertices()                    process/process.go:404-443
//   buffer / processBuffer()           process/process.go:200-234 (one pass; present() :374-384)
//   chooseLeader / waveRound           process/process.go:386-402
//   Stack<T>                           stack/stack.go:3-28 (Pop on empty panics)
//   Transport / bcastMsg               process/transport.go:6-32 (delivery sink)
// Go panics (index out of range, empty Pop) become dagrider::panic_error.
// Differences, all documented in DESIGN.md s4: methods have pointer semantics
// (decidedWave / leadersStack / deliveredVertices persist; the reference's value
// receivers drop them); the DAG must satisfy the mirrored contract
// (dr_append_rounds_lists).  All reachability runs on the GPU.
// The device mirror follows p.dag incrementally: Dag records every append, and
// the next query streams the new vertices through dr_append_vertices (late
// vertices into old rounds included); only assigning a whole new DAG
// re-uploads it.
#pragma once
#include <algorithm>
#include <cstdint>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "dagrider_gpu.h"

namespace dagrider {

struct panic_error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

struct vertexID {
  int round = 0;
  int source = 0;
  bool operator==(const vertexID &o) const { return round == o.round && source == o.source; }
  bool operator!=(const vertexID &o) const { return !(*this == o); }
};

struct block {
  std::vector<uint8_t> data;
};

struct vertex {
  vertexID id;
  block blk;
  std::vector<vertexID> strongEdges;
  std::vector<vertexID> weakEdges;
};

template <class T>
class Stack {
 public:
  static Stack New() {
    Stack s;
    s.data_.reserve(16);
    return s;
  }
  bool IsEmpty() const { return data_.empty(); }
  void Push(T e) { data_.push_back(std::move(e)); }
  T Pop() {
    if (data_.empty()) throw panic_error("runtime error: index out of range [-1]");
    T e = std::move(data_.back());
    data_.pop_back();
    return e;
  }
  const std::vector<T> &items() const { return data_; }

 private:
  std::vector<T> data_;
};

struct bcastMsg {
  vertex v;
  int round = 0;
  int sender = 0;
};

class Transport {
 public:
  void Broadcast(const bcastMsg &m) {
    for (auto &c : subs_) c(m);
  }
  void Subscribe(std::function<void(const bcastMsg &)> c) { subs_.push_back(std::move(c)); }

 private:
  std::vector<std::function<void(const bcastMsg &)>> subs_;
};

// Process.dag (process.go:79): [][]vertex whose mutations are the reference's
// two -- assignment (p.dag = dag, process_internal_test.go:18) and append into
// a round (p.dag[r] = append(p.dag[r], v), process.go:229) -- plus growing by
// empty rounds.  Existing vertices are read-only, so the log of appends is the
// whole difference to the device mirror.
class Dag {
 public:
  using Rounds = std::vector<std::vector<vertex>>;
  Dag() = default;
  Dag(Rounds d) : r_(std::move(d)) {}
  Dag &operator=(Rounds d) {
    r_ = std::move(d);
    reset_ = true;
    log_.clear();
    return *this;
  }
  size_t size() const { return r_.size(); }
  bool empty() const { return r_.empty(); }
  const std::vector<vertex> &operator[](size_t r) const { return r_[r]; }
  const Rounds &rounds() const { return r_; }
  // p.dag[r] = append(p.dag[r], v)
  void append(size_t r, vertex v) {
    if (r >= r_.size()) throw panic_error("runtime error: index out of range");
    r_[r].push_back(std::move(v));
    log_.emplace_back((int)r, (int)r_[r].size() - 1);
  }
  // p.dag = append(p.dag, make([][]vertex, k)...): k more (empty) rounds
  void grow(size_t k = 1) { r_.resize(r_.size() + k); }

 private:
  friend class Process;
  Rounds r_;
  bool reset_ = true;                     // whole DAG replaced since the last mirror sync
  std::vector<std::pair<int, int>> log_;  // (round, slot) appended since then
};

inline int chooseLeader(int) { return 1; }
inline int waveRound(int w, int k) { return 4 * (w - 1) + k; }

class Process {
 public:
  // New (process.go:34-60): index must be >= 1.
  static std::unique_ptr<Process> New(int index, int faulty, Transport *tp, std::string *err,
                                      int device = 0) {
    if (index < 1) {
      if (err) *err = "process indexes should be 1-indexed";
      return std::unique_ptr<Process>(new Process());
    }
    std::unique_ptr<Process> p(new Process());
    p->index = index;
    p->faulty = faulty;
    p->tp = tp;
    p->device_ = device;
    // 2f+1 genesis vertices {0, index} (process.go:42-49)
    Dag::Rounds g(1);
    for (int i = 0; i < 2 * faulty + 1; i++) g[0].push_back(vertex{vertexID{0, index}, {}, {}, {}});
    p->dag = std::move(g);
    if (err) err->clear();
    return p;
  }

  ~Process() {
    if (ctx_) dr_destroy(ctx_);
  }

  Transport *tp = nullptr;
  int index = 0;
  int round = 0;
  int faulty = 0;
  Dag dag;
  int decidedWave = 0;
  std::vector<vertex> deliveredVertices;
  Stack<vertex> leadersStack = Stack<vertex>::New();

  // path (process.go:89-148)
  bool path(vertexID from, vertexID to, bool strongPath) {
    if (from == to) return true;
    sync();
    int32_t f[2] = {from.round, from.source}, t[2] = {to.round, to.source};
    uint8_t out = 0;
    check(dr_path_batch(ctx_, 1, f, t, strongPath ? 1 : 0, &out));
    return out != 0;
  }

  // The global coin behind chooseLeader (process.go:386-392): the reference's
  // constant 1 (DR_LEADER_CONST1, default), a seeded coin, or a caller's table
  // (dagrider_gpu.h dr_set_leader_coin); kept across mirror rebuilds.
  void setLeaderCoin(int mode, uint64_t seed = 0, std::vector<int32_t> table = {}) {
    coinMode_ = mode;
    coinSeed_ = seed;
    coinTable_ = std::move(table);
    if (ctx_) applyCoin();
  }

  // getWaveVertexLeader (process.go:357-371): FIRST slot with source == leader.
  std::pair<vertex, bool> getWaveVertexLeader(int w) {
    sync();
    const int leader = dr_wave_leader(ctx_, w);
    const int r = waveRound(w, 1);
    if (r < 0 || r >= (int)dag.size()) throw panic_error("runtime error: index out of range");
    for (const vertex &v : dag[r])
      if (v.id.source == leader) return {v, true};
    return {vertex{}, false};
  }

  // waveReady (process.go:314-354): commit rule + leader chain on the GPU.
  void waveReady(int wave) {
    sync();
    uint8_t commit = 0;
    int32_t vcount = 0;
    std::vector<int32_t> pushed((size_t)wave + 1);
    int np = 0;
    check(dr_wave_ready(ctx_, wave, decidedWave, &commit, &vcount, pushed.data(), (int)pushed.size(), &np));
    lastVoteCount = vcount;
    if (!commit) return;
    for (int i = 0; i < np; i++) leadersStack.Push(getWaveVertexLeader(pushed[i]).first);
    decidedWave = wave;
  }

  // orderVertices (process.go:404-443): pops every leader, delivers its causal
  // history (rounds 1..round) in (round, slot) order via tp->Broadcast.
  void orderVertices() {
    sync();
    std::vector<int32_t> st;
    for (const vertex &v : leadersStack.items()) { st.push_back(v.id.round); st.push_back(v.id.source); }
    const int ns = (int)st.size() / 2;
    if (ns == 0) return;
    size_t n = 0;
    std::vector<int32_t> ids(2 * 4096);
    int rc = dr_order_vertices(ctx_, st.data(), ns, round, DR_DELIVER_REF, ids.data(), ids.size() / 2, &n,
                               nullptr, nullptr);
    if (rc == DR_E_CAPACITY) {
      ids.resize(2 * n);
      rc = dr_order_vertices(ctx_, st.data(), ns, round, DR_DELIVER_REF, ids.data(), n, &n, nullptr, nullptr);
    }
    check(rc);
    while (!leadersStack.IsEmpty()) leadersStack.Pop();
    for (size_t i = 0; i < n; i++) {
      const vertex &v = lookup(vertexID{ids[2 * i], ids[2 * i + 1]});
      bcastMsg msg{v, v.id.round, v.id.source};
      if (tp) tp->Broadcast(msg);
      deliveredVertices.push_back(v);
    }
  }

  // One pass of the buffer loop (process.go:200-234): vertices of rounds <= round
  // whose predecessors are all present() (process.go:374-384) -- in the DAG or
  // appended earlier in this pass -- go to dag[v.id.round] in buffer order; the
  // rest stay buffered.  present() is a device presence-bitset test.
  void processBuffer() {
    if (buffer.empty()) return;
    int ms = 1;  // the mirror's n must cover the buffered ids' sources
    for (const vertex &v : buffer) ms = std::max(ms, v.id.source);
    sync(ms);
    std::vector<int32_t> ids, preds;
    std::vector<uint32_t> off{0};
    for (const vertex &v : buffer) {
      ids.push_back(v.id.round);
      ids.push_back(v.id.source);
      for (const auto *es : {&v.strongEdges, &v.weakEdges})
        for (const auto &e : *es) { preds.push_back(e.round); preds.push_back(e.source); }
      off.push_back((uint32_t)preds.size() / 2);
    }
    preds.push_back(0);
    std::vector<uint8_t> admit(buffer.size());
    check(dr_buffer_admit(ctx_, round, (int)buffer.size(), ids.data(), off.data(), preds.data(), admit.data()));
    // every admission's p.dag[r] must exist before anything moves (Go replaces
    // p.buffer only after the loop).  A vertex whose id is already in the round is
    // appended as Go does (path() then sees the last one, process.go:112-116).
    for (size_t i = 0; i < buffer.size(); i++)
      if (admit[i] && buffer[i].id.round >= (int)dag.size())
        throw panic_error("runtime error: index out of range");  // p.dag[r]
    std::vector<vertex> next;
    for (size_t i = 0; i < buffer.size(); i++) {
      if (admit[i]) dag.append(buffer[i].id.round, std::move(buffer[i]));
      else next.push_back(std::move(buffer[i]));
    }
    buffer = std::move(next);
  }

  std::vector<vertex> buffer;
  int lastVoteCount = -1;

 private:
  Process() = default;
  dr_ctx *ctx_ = nullptr;
  int device_ = 0;
  int n_ = 0;
  int cap_rounds_ = 0;
  int coinMode_ = DR_LEADER_CONST1;
  uint64_t coinSeed_ = 0;
  std::vector<int32_t> coinTable_;

  void applyCoin() {
    check(dr_set_leader_coin(ctx_, coinMode_, coinSeed_, (int)coinTable_.size(),
                             coinTable_.empty() ? nullptr : coinTable_.data()));
  }

  void check(int rc) {
    if (rc == DR_OK) return;
    std::string msg = dr_last_error(ctx_);
    if (rc == DR_E_INVAL) throw panic_error("runtime error: " + msg);
    throw std::runtime_error("dagrider: " + msg);
  }

  const vertex &lookup(vertexID id) const {
    const vertex *hit = nullptr;
    for (const vertex &v : dag[id.round])
      if (v.id == id) hit = &v;  // last match, as path() does (process.go:112-116)
    if (!hit) throw std::logic_error("delivered id not in DAG");
    return *hit;
  }

  static int max_source(const vertex &v) {
    int ms = v.id.source;
    for (const auto &e : v.strongEdges) ms = std::max(ms, e.source);
    for (const auto &e : v.weakEdges) ms = std::max(ms, e.source);
    return ms;
  }

  // Whole-DAG upload into a fresh context (p.dag was assigned, or the mirror
  // ran out of rounds or sources); room for growth is reserved.
  void rebuild(int need_n) {
    int ms = need_n;
    for (const auto &rnd : dag.r_)
      for (const vertex &v : rnd) ms = std::max(ms, max_source(v));
    if (ctx_) dr_destroy(ctx_);
    ctx_ = nullptr;
    n_ = std::max({ms, 3 * faulty + 1, 1});
    cap_rounds_ = std::max<int>(64, 2 * (int)dag.size());
    int rc = dr_create(n_, faulty, cap_rounds_, device_, &ctx_);
    if (rc != DR_OK) throw std::runtime_error(std::string("dagrider: ") + dr_last_error(nullptr));
    if (coinMode_ != DR_LEADER_CONST1) applyCoin();
    std::vector<uint32_t> so{0}, sto{0}, wo{0};
    std::vector<int32_t> sid, sti, wi;
    for (const auto &rnd : dag.r_) {
      for (const vertex &v : rnd) {
        sid.push_back(v.id.round);
        sid.push_back(v.id.source);
        for (const auto &e : v.strongEdges) { sti.push_back(e.round); sti.push_back(e.source); }
        for (const auto &e : v.weakEdges) { wi.push_back(e.round); wi.push_back(e.source); }
        sto.push_back((uint32_t)sti.size() / 2);
        wo.push_back((uint32_t)wi.size() / 2);
      }
      so.push_back((uint32_t)sid.size() / 2);
    }
    sti.push_back(0);
    wi.push_back(0);
    check(dr_append_rounds_lists(ctx_, 0, (int)dag.size(), so.data(), sid.data(), sto.data(), sti.data(),
                                 wo.data(), wi.data()));
    dag.reset_ = false;
    dag.log_.clear();
  }

  // Bring the device mirror up to p.dag: empty rounds opened since, then the
  // logged appends in order (dr_append_vertices, all or nothing).
  void sync(int need_n = 0) {
    bool full = !ctx_ || dag.reset_ || need_n > n_ || (int)dag.size() > cap_rounds_;
    for (size_t i = 0; !full && i < dag.log_.size(); i++)
      full = max_source(dag.r_[dag.log_[i].first][dag.log_[i].second]) > n_;
    if (full) return rebuild(need_n);
    const int have = dr_num_rounds(ctx_);
    if ((int)dag.size() > have) {
      const int k = (int)dag.size() - have;
      std::vector<uint32_t> so(k + 1, 0), off{0};
      int32_t zero = 0;
      check(dr_append_rounds_lists(ctx_, have, k, so.data(), &zero, off.data(), &zero, off.data(), &zero));
    }
    if (dag.log_.empty()) return;
    std::vector<int32_t> sr, sid, sti, wi;
    std::vector<uint32_t> sto{0}, wo{0};
    for (const auto &rs : dag.log_) {
      const vertex &v = dag.r_[rs.first][rs.second];
      sr.push_back(rs.first);
      sid.push_back(v.id.round);
      sid.push_back(v.id.source);
      for (const auto &e : v.strongEdges) { sti.push_back(e.round); sti.push_back(e.source); }
      for (const auto &e : v.weakEdges) { wi.push_back(e.round); wi.push_back(e.source); }
      sto.push_back((uint32_t)sti.size() / 2);
      wo.push_back((uint32_t)wi.size() / 2);
    }
    sti.push_back(0);
    wi.push_back(0);
    check(dr_append_vertices(ctx_, (int)sr.size(), sr.data(), sid.data(), sto.data(), sti.data(), wo.data(),
                             wi.data()));
    dag.log_.clear();
  }
};

}  // namespace dagrider
