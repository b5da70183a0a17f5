"""setWeakEdges restated in pure Python -- TEST INFRASTRUCTURE ONLY (small DAGs).

Follows process/process.go:298-310 (the loop: r = round-2 down to 1, every slot of
dag[r] in order, u becomes a weak edge iff !path(v.id, u, false)) over a restatement
of path() at process.go:89-148 (self path; BFS with a visited map; vertex lookup =
the LAST slot of dag[id.round] with that id, a missing vertex has no edges; a
target is tested when first discovered).

Two modes, as dr_set_weak_edges:
  literal -- the code as written: v.id is still the zero id when setWeakEdges runs
             (createNewVertex assigns it later) and v is not
             in p.dag, so path() finds nothing;
  paper   -- Alg. 2 lines 29-31: v = (round, source) with its strong edges and the
             weak edges added so far, placed last in dag[round] so path() sees it.
"""
from __future__ import annotations

from collections import deque
from typing import List, Sequence, Tuple

LITERAL, PAPER = 0, 1

Id = Tuple[int, int]


def _edges(dag, vid: Id):
    """(strong, weak) of the last slot of dag[vid.round] with id vid (process.go:111-116)."""
    r = vid[0]
    if r < 0 or r >= len(dag):
        raise IndexError(f"p.dag[{r}]: index out of range (Go panic)")
    found = ([], [])
    for v in dag[r]:
        if v[0] == vid:
            found = (v[1], v[2])
    return found


def path(dag, frm: Id, to: Id, strong_only: bool) -> bool:
    """process.go:89-148."""
    if frm == to:
        return True
    visited = {frm}
    q = deque([frm])
    while q:
        vid = q.popleft()
        strong, weak = _edges(dag, vid)
        for lst in (strong, weak) if not strong_only else (strong,):
            for t in lst:
                if t not in visited:
                    if t == to:
                        return True
                    visited.add(t)
                    q.append(t)
    return False


def to_plain(lists) -> list:
    """dag_rider_amd.dag Vertex lists -> [[((r, s), strong ids, weak ids), ...], ...]."""
    return [[((v.id.round, v.id.source), [(e.round, e.source) for e in v.strong_edges],
              [(e.round, e.source) for e in v.weak_edges]) for v in rnd] for rnd in lists]


def set_weak_edges(dag, round_: int, source: int, strong: Sequence[Id], mode: int) -> List[Id]:
    """setWeakEdges(v, round) (process.go:298-310); dag in to_plain() form (not modified)."""
    dag = [list(rnd) for rnd in dag]
    weak: List[Id] = []
    if mode == LITERAL:
        vid = (0, 0)
    else:
        vid = (round_, source)
        v = (vid, list(strong), weak)  # weak grows as edges are added: path() sees them
        if round_ == len(dag):
            dag.append([v])
        else:
            dag[round_].append(v)
    for r in range(round_ - 2, 0, -1):
        for u in dag[r]:
            if not path(dag, vid, u[0], False):
                weak.append(u[0])
    return list(weak)
