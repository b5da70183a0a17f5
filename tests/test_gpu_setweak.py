"""GPU parity of setWeakEdges (process.go:298-310) through dr_set_weak_edges.

Bar: the id list (order included) identical to the oracle's restatement
(oracle/setweak.py: the reference loop over a restatement of path()) in both modes,
on the Figure-1 fixture (pinned: (4,1)'s weak edge (2,4)), on unconstrained random
DAGs (ghost slots, dangling targets, deep weak edges) and on a vertex of the next,
not yet appended round.
"""
import numpy as np
import pytest

import oracle
from dag_rider_amd import _lib as L
from dag_rider_amd.engine import Engine
from dag_rider_amd.gen import generate, small_config
from dagutil import figure1, random_dag

pytestmark = pytest.mark.gpu
SW = oracle.setweak


def _check(e, plain, rnd, src, strong):
    for mode, omode in ((L.DR_WEAK_PAPER, SW.PAPER), (L.DR_WEAK_LITERAL, SW.LITERAL)):
        got = [tuple(x) for x in e.set_weak_edges(rnd, strong, mode).tolist()]
        want = SW.set_weak_edges(plain, rnd, src, strong, omode)
        assert got == want, (rnd, src, mode)


def test_setweak_figure1(gpu_device):
    g, dag = figure1()
    plain = SW.to_plain(dag)
    with Engine(g["n"], g["faulty"], 8, gpu_device) as e:
        e.append_lists(dag)
        got = [tuple(x) for x in e.set_weak_edges(4, [(3, 1), (3, 2), (3, 3)], L.DR_WEAK_PAPER).tolist()]
        assert [x for x in got if x != (0, 0)] == [(2, 4)]  # (4,1).weakEdges in the fixture
        for rnd in range(1, 6):
            for strong in ([], [(rnd - 1, 1)], [(rnd - 1, s) for s in (1, 2, 3)], [(rnd - 1, 4)]):
                _check(e, plain, rnd, 1, strong)


@pytest.mark.parametrize("seed,n,R", [(1, 6, 16), (2, 20, 14), (3, 70, 10)])
def test_setweak_random(gpu_device, seed, n, R):
    rng = np.random.default_rng(300 + seed)
    d = random_dag(rng, n, R, p_present=0.8, p_s=0.35, p_w=0.15, max_depth=6)
    plain = SW.to_plain(d.to_lists())
    with Engine(n, (n - 1) // 3, R + 2, gpu_device) as e:
        e.append_packed(d)
        for _ in range(8):
            rnd = int(rng.integers(1, R + 2))  # R + 1: the next round, not yet appended
            src = int(rng.integers(1, n + 1))
            k = int(rng.integers(0, n + 1))
            strong = sorted({(rnd - 1, int(t)) for t in rng.integers(1, n + 1, size=k)})
            _check(e, plain, rnd, src, strong)


def test_setweak_generated(gpu_device):
    """Generator DAG (late vertices, weak deltas 2..4): the late vertices a new vertex
    misses become its weak edges."""
    cfg = small_config(40, 24, 7)
    d = generate(cfg)
    plain = SW.to_plain(d.to_lists())
    rng = np.random.default_rng(8)
    with Engine(cfg.n, cfg.faulty, d.nrounds + 1, gpu_device) as e:
        e.append_packed(d)
        for rnd in (d.nrounds, d.nrounds - 1, 12, 5):
            present = [s for s in range(1, cfg.n + 1)
                       if any(int(x) == s for x in d.slot_src[d.slot_off[rnd - 1]:d.slot_off[rnd]])]
            strong = [(rnd - 1, s) for s in present if rng.random() < 0.7]
            _check(e, plain, rnd, 1, strong)


def test_setweak_errors(gpu_device):
    g, dag = figure1()
    with Engine(g["n"], g["faulty"], 8, gpu_device) as e:
        e.append_lists(dag)
        with pytest.raises(L.DrError) as ei:
            e.set_weak_edges(7, [], L.DR_WEAK_PAPER)  # beyond the next round
        assert ei.value.code == L.DR_E_INVAL
        with pytest.raises(L.DrError) as ei:
            e.set_weak_edges(4, [(2, 1)], L.DR_WEAK_PAPER)  # strong edge not to round-1
        assert ei.value.code == L.DR_E_CONTRACT
