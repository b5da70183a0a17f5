"""The buffer loop's admission pass restated in pure Python -- TEST INFRASTRUCTURE ONLY.

Follows process/process.go:200-234 (one pass over p.buffer: a vertex of a round
> p.round stays buffered (:203-206); otherwise it is appended to
p.dag[v.id.round] iff every strong edge (:210-216) and every weak edge (:217-223)
is present(), else it goes to the new buffer (:225-230)) over present() at
process.go:374-384 (a linear scan of p.dag[0..p.round] for a slot whose id
equals the predecessor id; ghost slots carry the zero id {0,0}).

Appending inside the pass is sequential, so a vertex admitted earlier in the pass
is present for the ones after it.  The reference wraps this pass in `for true`,
which never ends: dr_buffer_admit is one pass, and so is this.
Parity: no reference test covers this loop (it cannot terminate), so the
restatement is pinned only by reading the code -- "parity unpinned" against the
reference's own outputs.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

Id = Tuple[int, int]


class GoPanic(IndexError):
    """The reference panics here (runtime error: index out of range)."""


def present(dag, cur_round: int, vid: Id) -> bool:
    """process.go:374-384; dag in oracle.setweak.to_plain() form.  The scan runs over
    p.dag[0..p.round]; an id not found before len(p.dag) indexes past it (:376)."""
    for r in range(0, cur_round + 1):
        if r >= len(dag):
            raise GoPanic(f"present({vid}): p.dag[{r}] with len {len(dag)}")
        for v in dag[r]:
            if v[0] == vid:
                return True
    return False


def admit_pass(dag, cur_round: int, buffer: Sequence[Tuple[Id, Sequence[Id]]]) -> List[int]:
    """One pass of process.go:200-234; buffer = [(id, preds)], preds = strong + weak.
    Returns admit flags; dag is copied, not modified.  Raises GoPanic where Go panics:
    in present() (above) or at p.dag[v.id.round] for an admitted vertex past the DAG.
    all() stops at the first absent predecessor; Go evaluates strong edges to the
    first absent one, then weak edges to the first absent one -- either way the first
    absent predecessor evaluated is the one that panics."""
    dag = [list(rnd) for rnd in dag]
    out = []
    for vid, preds in buffer:
        if vid[0] > cur_round:
            out.append(0)
            continue
        if all(present(dag, cur_round, p) for p in preds):
            if vid[0] >= len(dag):
                raise GoPanic(f"p.dag[{vid[0]}] = append(...) with len {len(dag)}")
            dag[vid[0]].append((tuple(vid), [], []))
            out.append(1)
        else:
            out.append(0)
    return out
