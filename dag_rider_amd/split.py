"""Wave-range split of the all-waves commit sweep.

waveReady's commit decision for wave w (``process/process.go:326-339``) reads only
rounds 4w-3 .. 4w: the leader's round (``getWaveVertexLeader``, ``:357-371``) and the
three rounds whose strong edges carry the votes.  Waves are therefore independent
units: a contiguous wave range [w0, w1] needs rounds 4(w0-1) .. 4 w1 and nothing
else, so a GPU can hold only its range and decide its waves with no exchange.

``wave_slice`` cuts that window out of a packed DAG as a DAG of its own (round
4(w0-1) becomes round 0, keeping only its slots -- its rows point below the window
and are never read by the commit rule; weak edges are dropped: the rule follows
strong edges only).  Wave w of the full DAG is wave w - w0 + 1 of the slice, so a
non-constant leader coin (``chooseLeader``, ``:386-392``) is handed over shifted:
``slice_leaders``.

``split_commit`` decides every wave of a DAG rank by rank (one ``Engine`` per
range, as one process per GPU would) and concatenates the answers; the result is
``dr_wave_commit`` over the whole DAG, bit for bit.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np

from .dag import PackedDag


def wave_ranges(nwaves: int, world: int) -> List[Tuple[int, int]]:
    """Contiguous 1-based wave ranges [w0, w1], one per rank (sizes differ by <= 1)."""
    if world < 1 or nwaves < world:
        raise ValueError(f"cannot split {nwaves} waves over {world} ranks")
    return [(r * nwaves // world + 1, (r + 1) * nwaves // world) for r in range(world)]


def wave_slice(d: PackedDag, w0: int, w1: int) -> PackedDag:
    """Rounds 4(w0-1) .. 4 w1 of ``d`` shifted to 0 .. 4(w1-w0+1): everything the commit
    decisions of waves w0..w1 read (round 0 of the slice keeps its slots, no edges)."""
    n, W = d.n, d.W
    lo, hi = 4 * (w0 - 1), 4 * w1
    if w0 < 1 or w1 < w0 or hi >= d.nrounds:
        raise ValueError(f"waves [{w0}, {w1}] need rounds {lo}..{hi}, the DAG has 0..{d.nrounds - 1}")
    so = d.slot_off[lo:hi + 2].astype(np.int64)
    strong = d.strong[lo * n * W:(hi + 1) * n * W].copy()
    strong[:n * W] = 0
    k = hi - lo + 1
    return PackedDag(n, k, (so - so[0]).astype(np.uint32), d.slot_src[so[0]:so[-1]].copy(), strong,
                     np.zeros(k * n + 1, np.uint32), np.zeros(0, np.uint32))


def slice_leaders(leaders: Optional[Sequence[int]], w0: int, w1: int) -> Optional[List[int]]:
    """A leader table (leaders[w-1] = chooseLeader(w), 1 beyond its end) re-based to the
    slice's wave numbers; None stays None (the reference's constant coin)."""
    if leaders is None:
        return None
    return [int(leaders[w - 1]) if w - 1 < len(leaders) else 1 for w in range(w0, w1 + 1)]


def split_commit(d: PackedDag, faulty: int, nwaves: int, world: int, device: int = 0,
                 leaders: Optional[Sequence[int]] = None):
    """Every wave's commit decision, computed per wave range on its own mirror (one
    ``Engine`` per range, one after another on ``device``); returns (commit, vcount,
    ranges)."""
    from .engine import Engine
    from . import _lib as L

    commit, vcount = [], []
    ranges = wave_ranges(nwaves, world)
    for w0, w1 in ranges:
        sub = wave_slice(d, w0, w1)
        with Engine(d.n, faulty, sub.nrounds, device) as e:
            e.append_packed(sub)
            tab = slice_leaders(leaders, w0, w1)
            if tab is not None:
                e.set_leader_coin(L.DR_LEADER_TABLE, table=tab)
            cm, vc = e.wave_commit(1, w1 - w0 + 1)
        commit.append(cm.copy())
        vcount.append(vc.copy())
    return np.concatenate(commit), np.concatenate(vcount), ranges
