"""GPU parity with exceptions to the regular graph on the memoized path.

An exception is an edge below its round that the regular graph G_reg (strong rows to
r-1, weak columns within the memo window) does not hold: a strong edge skipping rounds
or a weak edge to r-1 (uponDeliver admits them,
process/process.go:165), a weak edge past the window, a far weak edge.  The engine
tests each one once (engine.hip ensure_exceptions): when its target is already in its
source's G_reg cone it changes no cone and the memo (round summaries, canonical cone)
stays on; otherwise the queries run on the general sweep.  Either way every answer must
equal the bitset restatement's (oracle/ref_bitset.c takes these edges in weak_tgt,
bit 31 marking a strong one), itself cross-checked against the literal BFS in
tests/test_oracle.py.  Each test also checks the engine's verdict against the oracle's
own cone test on the DAG without the exceptions."""
import numpy as np
import pytest

import oracle
from dag_rider_amd import _lib as L
from dag_rider_amd.dag import PackedDag
from dag_rider_amd.engine import Engine
from dag_rider_amd.gen import CONFIGS, generate, with_extra_edges
from dagutil import random_dag

pytestmark = pytest.mark.gpu

MODES = [(cm, dm) for cm in (L.DR_CHAIN_LITERAL, L.DR_CHAIN_PERSISTENT) for dm in (L.DR_DELIVER_REF, L.DR_DELIVER_PAPER)]


def _same(got, want, ids=True):
    assert got.commit.tolist() == want.commit.tolist()
    assert got.vcount.tolist() == want.vcount.tolist()
    assert got.push_off.tolist() == want.push_off.tolist() and got.push_wave.tolist() == want.push_wave.tolist()
    assert got.pop_count.tolist() == want.pop_count.tolist()
    assert got.pop_digest.tolist() == want.pop_digest.tolist()
    assert got.pop_edges.tolist() == want.pop_edges.tolist()
    assert (got.commit_edges, got.chain_edges, got.deliver_edges) == \
        (want.commit_edges, want.chain_edges, want.deliver_edges)
    if ids:
        assert got.ids.tolist() == want.ids.tolist()


def _present(d: PackedDag, r: int):
    return sorted({int(x) for x in d.slot_src[d.slot_off[r]:d.slot_off[r + 1]] if x})


def _random_extras(rng, d: PackedDag, k: int, deep: int = 0):
    """k edges below their rounds: strong ones skipping >= 1 round, weak ones to r-1, and
    with deep > 0 weak ones `deep`.. rounds down (past the regular window)."""
    out = []
    while len(out) < k:
        r = int(rng.integers(3, d.nrounds))
        srcs = _present(d, r)
        if not srcs:
            continue
        s = int(rng.choice(srcs))
        kind = int(rng.integers(0, 3 if deep else 2))
        if kind == 0:
            tr, strong = int(rng.integers(max(0, r - 6), r - 1)), True
        elif kind == 1:
            tr, strong = r - 1, False
        else:
            if r - deep < 0:
                continue
            tr, strong = int(rng.integers(0, r - deep + 1)), False
        out.append((r, s, tr, int(rng.integers(1, d.n + 1)), strong))
    return tuple(out)


def _benign(base: PackedDag, extras) -> bool:
    """The engine's verdict, restated: every exception's target in its source's cone of
    the DAG without them (strong cone for a strong edge)."""
    p = oracle.PDag(base)
    return all(p.path((r, s), (tr, ts), strong) == 1 for r, s, tr, ts, strong in extras)


def _check_all(e, d, f, nw, rng, modes=MODES, ids=True):
    pd = oracle.PDag(d)
    cap = 1 << 18 if ids else 0
    for cm, dm in modes:
        want = pd.replay(f, nw, cm, dm, ids_cap=cap)
        assert want.rc == 0
        _same(e.replay(nw, cm, dm, ids_cap=cap), want, ids=ids)
    pairs = []
    for _ in range(120):
        fr = int(rng.integers(1, d.nrounds))
        pairs.append(((fr, int(rng.integers(1, d.n + 1))), (int(rng.integers(0, fr)), int(rng.integers(1, d.n + 1)))))
    for st in (True, False):
        got = e.path_batch(pairs, st).tolist()
        assert got == [pd.path(a, b, st) for a, b in pairs]


@pytest.mark.parametrize("seed", range(8))
def test_exceptions_random(gpu_device, seed):
    rng = np.random.default_rng(7300 + seed)
    n = int(rng.choice([4, 9, 33, 64, 100]))
    R = int(rng.integers(24, 60))
    base = random_dag(rng, n, R, p_present=rng.uniform(0.75, 1), p_s=rng.uniform(0.4, 0.95),
                      p_w=rng.uniform(0, 0.5), max_depth=int(rng.integers(2, 6)))
    extras = _random_extras(rng, base, int(rng.integers(1, 5)))
    d = with_extra_edges(base, extras)
    f = int(rng.integers(0, (n - 1) // 3 + 2))
    nw = (d.nrounds - 1) // 4
    with Engine(n, f, d.nrounds, gpu_device) as e:
        cut = int(rng.integers(1, d.nrounds))
        e.append_packed(d, 0, cut)
        if cut > 4:  # a query between the appends: its test covers the first part only
            e.wave_commit(1, (cut - 1) // 4)
        e.append_packed(d, cut, d.nrounds)
        _check_all(e, d, f, nw, rng)
        st = e.exception_stats()
        assert st["exceptions"] == len(extras) and st["upward"] == 0
        assert st["memo"] == int(_benign(base, extras)), (st, extras)


def test_exceptions_benign_keep_memo(gpu_device):
    """Full rounds (every vertex strong to every vertex of r-1): any edge below its
    round is benign, and one test sweep per exception is all it costs."""
    rng = np.random.default_rng(11)
    n, R = 16, 40
    base = random_dag(rng, n, R, p_present=1.0, p_s=1.0, p_w=0.2, max_depth=4, dangling=0.0, ghosts=0.0,
                      leader_p=1.0)
    extras = ((20, 3, 17, 5, True), (21, 4, 20, 9, False), (33, 1, 30, 2, True))
    d = with_extra_edges(base, extras)
    with Engine(n, 5, d.nrounds, gpu_device) as e:
        e.append_packed(d)
        _check_all(e, d, 5, (d.nrounds - 1) // 4, rng)
        st = e.exception_stats()
        assert st == dict(exceptions=3, changing=0, sweeps=3, regular_delta=st["regular_delta"], upward=0, memo=1)
        e.replay((d.nrounds - 1) // 4)
        assert e.exception_stats()["sweeps"] == 3  # tested once


def test_exceptions_changing_cone(gpu_device):
    """An exception whose target its source's cone misses: the queries leave the memo
    (general sweep) and still answer as the oracle does; appending rounds above it keeps
    the verdict without a new test."""
    rng = np.random.default_rng(12)
    n, R = 12, 44
    base = random_dag(rng, n, R, p_present=0.9, p_s=0.35, p_w=0.0, dangling=0.0, ghosts=0.0)
    p = oracle.PDag(base)
    ex = None
    for r in range(30, 10, -1):
        for s in _present(base, r):
            for t in range(1, n + 1):
                if p.path((r, s), (r - 3, t), True) == 0:
                    ex = (r, s, r - 3, t, True)
                    break
            if ex:
                break
        if ex:
            break
    assert ex is not None
    d = with_extra_edges(base, (ex,))
    with Engine(n, 3, d.nrounds, gpu_device) as e:
        e.append_packed(d, 0, 36)
        e.path_batch([((35, 1), (2, 1))], False)
        st = e.exception_stats()
        assert st["changing"] == 1 and st["memo"] == 0 and st["sweeps"] == 1
        e.append_packed(d, 36, d.nrounds)
        _check_all(e, d, 3, (d.nrounds - 1) // 4, rng)
        assert e.exception_stats()["sweeps"] == 1


def test_exceptions_far_and_deep(gpu_device):
    """Weak edges past the regular window (n <= 64: deltas > 255) and far ones (> 1023)
    on a long narrow DAG, beside edges skipping rounds."""
    rng = np.random.default_rng(13)
    n, R = 8, 1300
    base = random_dag(rng, n, R, p_present=0.95, p_s=0.8, p_w=0.3, max_depth=5, ghosts=0.0)
    extras = _random_extras(rng, base, 6, deep=300) + ((1200, _present(base, 1200)[0], 100, 3, False),)
    d = with_extra_edges(base, extras)
    with Engine(n, 2, d.nrounds, gpu_device) as e:
        e.append_packed(d)
        _check_all(e, d, 2, (d.nrounds - 1) // 4, rng, modes=[(L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF),
                                                           (L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_PAPER)], ids=False)
        st = e.exception_stats()
        assert st["exceptions"] == len(extras)
        assert st["memo"] == int(_benign(base, extras))


@pytest.mark.parametrize("name", ["c4-far", "c4-q8"])
def test_exceptions_c4_scale(gpu_device, name):
    """The bench lines' exceptions on a C4-width DAG (n = 1024) cut to 700 rounds: the
    Delta=600 weak edge and the strong edge to r-3, both benign -- the memo stays on."""
    cfg = CONFIGS[name]
    r, s, tr, ts, strong = cfg.extra[0]
    if name == "c4-far":
        r, tr = 650, 50
    else:
        r, tr = 601, 598
    import dataclasses
    small = dataclasses.replace(cfg, last_round=700, extra=((r, s, tr, ts, strong),))
    d = generate(small, nthreads=16)
    with Engine(small.n, small.faulty, d.nrounds, gpu_device) as e:
        e.append_packed(d)
        want = oracle.PDag(d).replay(small.faulty, small.nwaves, oracle.CHAIN_PERSISTENT, oracle.DELIVER_REF,
                                     nthreads=16)
        _same(e.replay(small.nwaves), want, ids=False)
        st = e.exception_stats()
        assert st["exceptions"] == 1 and st["changing"] == 0 and st["memo"] == 1
