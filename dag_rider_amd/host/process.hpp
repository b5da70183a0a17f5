// process.hpp -- C++ host mirror of the reference's process.Process hot-path API
// over the C ABI (include/dagrider_gpu.h).
//
// Same names, argument meaning and error behaviour as xenowits/dag-rider:
//   vertexID / vertex / block          process/process.go:14-31
//   New / NewForT                      process/process.go:33-70 (index < 1 -> error)
//   Process::dag (assign, then query)  process/process.go:79, process_internal_test.go:18
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
    p->dag.resize(1);
    for (int i = 0; i < 2 * faulty + 1; i++) p->dag[0].push_back(vertex{vertexID{0, index}, {}, {}, {}});
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
  std::vector<std::vector<vertex>> dag;
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

  // getWaveVertexLeader (process.go:357-371): FIRST slot with source == leader.
  std::pair<vertex, bool> getWaveVertexLeader(int w) {
    const int leader = chooseLeader(w);
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
    std::vector<vertex> next;
    for (size_t i = 0; i < buffer.size(); i++) {
      if (!admit[i]) { next.push_back(std::move(buffer[i])); continue; }
      const int r = buffer[i].id.round;
      if (r >= (int)dag.size()) throw panic_error("runtime error: index out of range");  // p.dag[r]
      dag[r].push_back(std::move(buffer[i]));
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
  uint64_t fp_ = 0;

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

  uint64_t fingerprint(int *maxsrc) const {
    uint64_t h = 1469598103934665603ULL;
    auto mix = [&](uint64_t x) { h = (h ^ x) * 1099511628211ULL; };
    int ms = 1;
    mix(dag.size());
    for (const auto &rnd : dag) {
      mix(rnd.size());
      for (const vertex &v : rnd) {
        mix((uint64_t)(uint32_t)v.id.round << 32 | (uint32_t)v.id.source);
        mix(v.strongEdges.size());
        mix(v.weakEdges.size());
        ms = std::max(ms, v.id.source);
        for (const auto &e : v.strongEdges) { mix((uint64_t)(uint32_t)e.round << 32 | (uint32_t)e.source); ms = std::max(ms, e.source); }
        for (const auto &e : v.weakEdges) { mix((uint64_t)(uint32_t)e.round << 32 | (uint32_t)e.source); ms = std::max(ms, e.source); }
      }
    }
    *maxsrc = ms;
    return h;
  }

  // Mirror p.dag onto the device when it changed (the reference mutates it in place).
  void sync(int need_n = 0) {
    int ms = 1;
    const uint64_t fp = fingerprint(&ms);
    if (ctx_ && fp == fp_ && need_n <= n_) return;
    if (ctx_) dr_destroy(ctx_);
    ctx_ = nullptr;
    n_ = std::max({ms, 3 * faulty + 1, need_n});
    int rc = dr_create(n_, faulty, (int)std::max<size_t>(dag.size(), 1), device_, &ctx_);
    if (rc != DR_OK) throw std::runtime_error(std::string("dagrider: ") + dr_last_error(nullptr));
    std::vector<uint32_t> so{0}, sto{0}, wo{0};
    std::vector<int32_t> sid, sti, wi;
    for (const auto &rnd : dag) {
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
    fp_ = fp;
  }
};

}  // namespace dagrider
