// host_rounds.hpp -- the host-side per-round state of a mirror and its builder
// for pre-packed rounds (dr_append_rounds_packed).  Host code only: compiled by
// g++ with OpenMP (host_rounds.cpp), used by engine.hip.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace dr_host {

// Host-side state of one mirrored round.  Everything variable-size per round lives
// here and is flattened to the device from the lowest changed round on
// (dr_ctx::upload_suffix), so a vertex appended to an old round
// (process.go:229) rewrites only the rounds from there to the top.
struct HostRound {
  std::vector<uint16_t> slots;   // source per slot, insertion order (0 = ghost {0,0})
  uint64_t deg = 0;              // total strong degree
  uint64_t nweak = 0;            // weak edges (near + far)
  std::vector<uint32_t> wc_key;  // weak columns: distinct near targets (delta << 11 | t-1), sorted
  std::vector<uint64_t> wc_rows; // [key][WS]: the round's sources with that weak edge
  std::vector<uint64_t> far;     // weak edges with delta > 1023: (own s-1) << 32 | (r' << 11 | t-1)
  std::vector<uint64_t> irr;     // edges outside the round contract (App. A Q8), general.hpp irr_pack
  uint32_t ndup = 0;             // slots repeating an id already in the round (engine.hip upload_suffix)
};

// k pre-packed rounds r0..r0+k-1 (the dr_append_rounds_packed arrays).
struct PackedRounds {
  int n = 0, W = 0, WS = 0, r0 = 0, k = 0, max_rounds = 0;
  const uint32_t *slot_off = nullptr;
  const uint16_t *slot_src = nullptr;
  const uint64_t *strong = nullptr;
  const uint32_t *weak_off = nullptr;
  const uint32_t *weak_tgt = nullptr;  // (r' << 11) | t-1; bit 31: a strong edge outside r-1 (App. A Q8)
  uint64_t *strong_stage = nullptr;    // optional: the rows are copied here too (each chunk task its own)
};

struct BuiltRounds {
  std::vector<HostRound> rounds;  // k
  std::vector<uint64_t> pres;     // k * WS presence words
  std::vector<uint16_t> sdeg, wdeg;  // k * n per-vertex strong / weak degrees
  size_t nfar = 0;
  size_t nirr = 0;                // edges outside the round contract (HostRound::irr)
  int irr_tmax = 0;               // the highest round one of them targets
  int dmax = 1;                   // largest near weak delta seen (>= the caller's)
};

// Per-context scratch of the builder: one (delta, t) -> column table per OpenMP
// thread, all -1 between uses, (largest delta seen + 1) * n entries each.  Owned
// by the mirror (dr_ctx), so it lives and dies with it.
struct BuildScratch {
  std::vector<std::vector<int32_t>> tab;
  std::vector<std::vector<uint64_t>> bm;    // merge_round's key bitmap, per thread
  std::vector<std::vector<uint32_t>> rank;  // and its running popcount per word
};

// Validate and build the host state of every round (rounds in parallel).
// Returns 0 or a DR_E_* code with `err` set to the message of the first failing
// round, exactly as a sequential pass over the rounds would report it.
int build_packed_rounds(const PackedRounds &in, int dmax0, BuiltRounds &out, std::string &err, BuildScratch &scr);

}  // namespace dr_host
