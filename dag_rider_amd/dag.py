"""DAG data model: the reference's vertex types and the two flat layouts the C ABI takes.

Mirrors ``vertexID`` / ``vertex`` (reference ``process/process.go:20-31``) and
``Process.dag [][]vertex`` (``process.go:79``).  ``flatten_lists`` turns a
``[][]vertex`` into the arrays ``dr_append_rounds_lists`` consumes (what a cgo
binding would build from the Go slice); ``PackedDag`` is the pre-packed layout
(``dr_append_rounds_packed``, ``include/dagrider_gen.h``).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Sequence

import numpy as np


@dataclass(frozen=True)
class VertexID:
    """vertexID (process.go:20-23): (round, source) identifies a vertex."""

    round: int = 0
    source: int = 0


@dataclass
class Vertex:
    """vertex (process.go:26-31). ``block`` is never read by the hot path."""

    id: VertexID = field(default_factory=VertexID)
    block: bytes = b""
    strong_edges: List[VertexID] = field(default_factory=list)
    weak_edges: List[VertexID] = field(default_factory=list)


Dag = List[List[Vertex]]


def flatten_lists(dag: Sequence[Sequence[Vertex]], r0: int = 0, r1: int | None = None):
    """Flatten rounds [r0, r1) of a [][]vertex into the list-form arrays."""
    r1 = len(dag) if r1 is None else r1
    slot_off = [0]
    slot_id: List[int] = []
    strong_off = [0]
    strong_ids: List[int] = []
    weak_off = [0]
    weak_ids: List[int] = []
    for r in range(r0, r1):
        for v in dag[r]:
            slot_id += [v.id.round, v.id.source]
            for e in v.strong_edges:
                strong_ids += [e.round, e.source]
            for e in v.weak_edges:
                weak_ids += [e.round, e.source]
            strong_off.append(len(strong_ids) // 2)
            weak_off.append(len(weak_ids) // 2)
        slot_off.append(len(slot_id) // 2)
    u32 = lambda a: np.asarray(a, dtype=np.uint32)
    i32 = lambda a: np.asarray(a if a else [0], dtype=np.int32)
    return (u32(slot_off), i32(slot_id), u32(strong_off), i32(strong_ids), u32(weak_off), i32(weak_ids))


@dataclass
class PackedDag:
    """Packed DAG: strong rows by (round, source-1), W=ceil(n/64) words; weak CSR by
    vertex index r*n+s-1, targets (round << 11) | (source-1), bit 31 set for a strong
    edge outside round r-1 (App. A Q8); slot_src 0 = ghost."""

    n: int
    nrounds: int
    slot_off: np.ndarray  # uint32 [nrounds+1]
    slot_src: np.ndarray  # uint16
    strong: np.ndarray  # uint64 [nrounds*n*W]
    weak_off: np.ndarray  # uint32 [nrounds*n+1]
    weak_tgt: np.ndarray  # uint32

    @property
    def W(self) -> int:
        return (self.n + 63) // 64

    @property
    def faulty(self) -> int:
        return (self.n - 1) // 3

    def prefix(self, nrounds: int) -> "PackedDag":
        nrounds = min(nrounds, self.nrounds)
        so = self.slot_off[: nrounds + 1]
        wo = self.weak_off[: nrounds * self.n + 1]
        return PackedDag(self.n, nrounds, so, self.slot_src[: so[-1]],
                         self.strong[: nrounds * self.n * self.W], wo, self.weak_tgt[: wo[-1]])

    def row(self, r: int, s: int) -> np.ndarray:
        o = (r * self.n + s - 1) * self.W
        return self.strong[o:o + self.W]

    def to_lists(self) -> Dag:
        """Expand into a [][]vertex (small DAGs only)."""
        dag: Dag = []
        for r in range(self.nrounds):
            rnd = []
            for sl in range(int(self.slot_off[r]), int(self.slot_off[r + 1])):
                s = int(self.slot_src[sl])
                if s == 0:
                    rnd.append(Vertex())
                    continue
                row = self.row(r, s)
                strong = [VertexID(r - 1, w * 64 + b + 1) for w in range(self.W) for b in range(64)
                          if (int(row[w]) >> b) & 1]
                g = r * self.n + s - 1
                ts = [int(t) for t in self.weak_tgt[self.weak_off[g]:self.weak_off[g + 1]]]
                # bit 31: a strong edge outside the row's round r-1 (App. A Q8)
                strong += [VertexID((t >> 11) & 0xFFFFF, (t & 2047) + 1) for t in ts if t >> 31]
                weak = [VertexID(t >> 11, (t & 2047) + 1) for t in ts if not t >> 31]
                rnd.append(Vertex(VertexID(r, s), b"", strong, weak))
            dag.append(rnd)
        return dag


def pack_lists(dag: Sequence[Sequence[Vertex]], n: int) -> PackedDag:
    """Pack a contract [][]vertex (ghost slots allowed) into a PackedDag.  An id that
    repeats in its round keeps every slot; its row and weak edges are its LAST slot's,
    the vertex path()'s lookup sees (process.go:112-116)."""
    W = (n + 63) // 64
    R = len(dag)
    slot_off = [0]
    slot_src: List[int] = []
    strong = np.zeros(R * n * W, dtype=np.uint64)
    weak_lists: List[List[int]] = [[] for _ in range(R * n)]
    for r, rnd in enumerate(dag):
        seen = set()
        for v in rnd:
            s = v.id.source
            if v.id == VertexID(0, 0):
                slot_src.append(0)
                continue
            slot_src.append(s)
            if s in seen:  # a later slot of the id replaces its edges
                strong[(r * n + s - 1) * W:(r * n + s) * W] = 0
                weak_lists[r * n + s - 1] = []
            seen.add(s)
            for e in v.strong_edges:
                o = (r * n + s - 1) * W + (e.source - 1) // 64
                strong[o] |= np.uint64(1 << ((e.source - 1) % 64))
            for e in v.weak_edges:
                weak_lists[r * n + s - 1].append((e.round << 11) | (e.source - 1))
        slot_off.append(len(slot_src))
    weak_off = np.zeros(R * n + 1, dtype=np.uint32)
    acc = 0
    for i, l in enumerate(weak_lists):
        weak_off[i] = acc
        acc += len(l)
    weak_off[-1] = acc
    weak_tgt = np.asarray([t for l in weak_lists for t in l], dtype=np.uint32)
    return PackedDag(n, R, np.asarray(slot_off, dtype=np.uint32), np.asarray(slot_src, dtype=np.uint16),
                     strong, weak_off, weak_tgt)
