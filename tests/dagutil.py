"""Test-side DAG builders.

``random_dag`` draws *unconstrained* contract DAGs (any strong-edge density, so
partial quorums, non-commits and leader-chain pushes are common; dangling strong
targets; ghost {0,0} slots; weak edges of any depth).  The product's generator
(dag_rider_amd.gen) only emits quorum-shaped DAGs, where every present leader
commits and chains are empty.
"""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np

from dag_rider_amd.dag import PackedDag, Vertex, VertexID

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def random_dag(rng: np.random.Generator, n: int, R: int, p_present=0.8, p_s=0.5, p_w=0.1, max_depth=6,
               dangling=0.05, ghosts=0.1, leader_p=0.85) -> PackedDag:
    W = (n + 63) // 64
    NR = R + 1
    slot_off = [0]
    slot_src = []
    strong = np.zeros(NR * n * W, dtype=np.uint64)
    pres = np.zeros((NR, n), dtype=bool)
    weak_lists = [[] for _ in range(NR * n)]
    for r in range(NR):
        if r == 0:
            p = np.ones(n, dtype=bool)
        else:
            p = rng.random(n) < p_present
            if (r - 1) % 4 == 0:
                p[0] = rng.random() < leader_p
        pres[r] = p
        srcs = [s + 1 for s in range(n) if p[s]]
        rng.shuffle(srcs)
        if ghosts and rng.random() < ghosts:
            srcs.insert(int(rng.integers(0, len(srcs) + 1)), 0)
        slot_src += srcs
        slot_off.append(len(slot_src))
        if r == 0:
            continue
        prev = pres[r - 1]
        for s in range(n):
            if not p[s]:
                continue
            u = rng.random(n)
            hit = np.where(prev, u < p_s, u < dangling)
            for t in np.nonzero(hit)[0]:
                o = (r * n + s) * W + t // 64
                strong[o] |= np.uint64(1 << (int(t) % 64))
            lo = max(0, r - max_depth)
            if r >= 2 and p_w > 0 and r - 1 > lo:
                cand = rng.random((r - 1 - lo, n)) < p_w / n * 2
                for r2, t in zip(*np.nonzero(cand)):
                    weak_lists[r * n + s].append(((lo + int(r2)) << 11) | int(t))
    weak_off = np.zeros(NR * n + 1, dtype=np.uint32)
    acc = 0
    for i, l in enumerate(weak_lists):
        weak_off[i] = acc
        acc += len(l)
    weak_off[-1] = acc
    weak_tgt = np.asarray([t for l in weak_lists for t in l], dtype=np.uint32)
    return PackedDag(n, NR, np.asarray(slot_off, np.uint32), np.asarray(slot_src, np.uint16), strong, weak_off,
                     weak_tgt)


def figure1():
    with open(os.path.join(GOLDEN, "figure1.json")) as f:
        g = json.load(f)
    dag = [[Vertex(VertexID(*v["id"]), b"", [VertexID(*e) for e in v["strong"]],
                   [VertexID(*e) for e in v["weak"]]) for v in rnd] for rnd in g["rounds"]]
    return g, dag


def dag_fingerprint(d: PackedDag) -> str:
    """Hash of a packed DAG's arrays: pins the generator's output across machines."""
    h = hashlib.blake2b(digest_size=16)
    h.update(np.asarray([d.n, d.nrounds], np.int64).tobytes())
    for a, t in ((d.slot_off, np.uint32), (d.slot_src, np.uint16), (d.strong, np.uint64), (d.weak_off, np.uint32),
                 (d.weak_tgt, np.uint32)):
        h.update(np.ascontiguousarray(a, dtype=t).tobytes())
    return h.hexdigest()


def replay_fingerprint(r) -> str:
    """Hash of every output of one replay (engine ReplayResult or oracle OracleReplay)."""
    h = hashlib.blake2b(digest_size=16)
    for a, t in ((r.commit, np.uint8), (r.vcount, np.int32), (r.push_off, np.uint32), (r.push_wave, np.int32),
                 (r.pop_count, np.uint64), (r.pop_digest, np.uint64), (r.pop_edges, np.uint64)):
        h.update(np.ascontiguousarray(a, dtype=t).tobytes())
    h.update(np.asarray([r.commit_edges, r.chain_edges, r.deliver_edges], np.uint64).tobytes())
    return h.hexdigest()


def load_large():
    import gzip

    with gzip.open(os.path.join(GOLDEN, "large_replay.json.gz"), "rt") as f:
        return json.load(f)


def with_repeated_ids(rng: np.random.Generator, dag, p_dup=0.3, max_extra=2):
    """A [][]vertex where some ids of rounds >= 1 repeat in their round, as the
    reference's uponDeliver / buffer loop append them (process/process.go:158-169,
    :229): each repeat is a separate slot at a random position, with its own random
    strong edges (to round r-1) and weak edges (below r-1).  path() follows an id's
    LAST slot (:112-116); vCount and REF delivery count every slot."""
    out = [list(r) for r in dag]
    for r in range(1, len(out)):
        ids = [v.id for v in out[r] if v.id != VertexID(0, 0)]
        if not ids:
            continue
        # distinct targets: an edge list naming one target twice is a multi-edge, which
        # the edge totals count once
        prev = sorted({v.id for v in out[r - 1] if v.id != VertexID(0, 0)}, key=lambda x: (x.round, x.source))
        below = sorted({v.id for rr in range(max(0, r - 6), r - 1) for v in out[rr] if v.id != VertexID(0, 0)},
                       key=lambda x: (x.round, x.source))
        for vid in ids:
            if rng.random() >= p_dup:
                continue
            for _ in range(int(rng.integers(1, max_extra + 1))):
                st = [u for u in prev if rng.random() < 0.6]
                wk = [u for u in below if rng.random() < 0.1]
                pos = int(rng.integers(0, len(out[r]) + 1))
                out[r].insert(pos, Vertex(vid, b"", st, wk))
    return out


def with_irregular_edges(rng: np.random.Generator, dag, p_irr=0.2, up=True):
    """A [][]vertex with edges outside the round contract, which
    uponDeliver admits (it checks only the strong-edge count, process/process.go:165)
    and path()'s BFS answers (:89-148): some vertices get strong edges to a round other
    than r-1 and weak edges to round r-1 or above; with `up`, also to the same round or
    later ones (cycles).  Targets are ids of mirrored rounds (present or not: a
    dangling target counts as reached), never one the vertex already names."""
    R = len(dag) - 1
    out = []
    for r, rnd in enumerate(dag):
        row = []
        for v in rnd:
            if v.id == VertexID(0, 0) or rng.random() >= p_irr:
                row.append(v)
                continue
            n_src = max(x.id.source for rr in dag for x in rr) or 1
            have = set(v.strong_edges) | set(v.weak_edges)
            st, wk = list(v.strong_edges), list(v.weak_edges)
            for _ in range(int(rng.integers(1, 4))):
                lo, hi = (0, R) if up else (0, max(0, r - 1))
                tr = int(rng.integers(lo, hi + 1))
                t = VertexID(tr, int(rng.integers(1, n_src + 1)))
                if t in have or t == v.id:
                    continue
                strong = rng.random() < 0.5
                if strong and tr == r - 1 or (not strong and tr <= r - 2):
                    strong = not strong  # keep it outside the contract
                if strong and tr == r - 1 or (not strong and tr <= r - 2):
                    continue
                (st if strong else wk).append(t)
                have.add(t)
            row.append(Vertex(v.id, v.block, st, wk))
        out.append(row)
    return out
