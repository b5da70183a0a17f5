"""Buffer loop + present() (process.go:200-234, :374-384) through dr_buffer_admit.

CPU: the oracle restatement (oracle/buffer.py) on the Figure-1 DAG
(process_internal_test.go:86-283), including the in-pass dependency the sequential
append creates.  GPU: admit flags bit-exact against the oracle on Figure-1 and on
random DAGs with ghost slots, absent predecessors, vertices ahead of the current
round and chains of buffered vertices in both orders.  No reference test covers
this loop (it never terminates): parity unpinned beyond the restatement.
"""
import numpy as np
import pytest

import oracle
from dag_rider_amd import _lib as L
from dag_rider_amd.engine import Engine
from dagutil import figure1, random_dag

B = oracle.buffer


def test_oracle_figure1_pass():
    g, dag = figure1()
    plain = oracle.setweak.to_plain(dag)
    assert B.present(plain, 4, (4, 1)) and B.present(plain, 4, (0, 0))
    assert not B.present(plain, 3, (4, 1))  # present() scans rounds 0..p.round only
    assert not B.present(plain, 4, (2, 5))
    with pytest.raises(B.GoPanic):  # absent id with p.round >= len(p.dag): the scan runs off the end
        B.present(plain, 5, (2, 5))
    assert B.present(plain, 7, (4, 1))  # found before the end: no panic
    grown = plain + [[], [], []]  # p.dag with rounds 5..7 opened
    buf = [((5, 1), [(4, 1), (4, 2)]),          # present preds -> admitted
           ((6, 1), [(5, 1), (5, 2)]),          # (5,2) arrives later in the pass -> stays
           ((5, 2), [(4, 3), (0, 0)]),          # ghost id is present -> admitted
           ((6, 2), [(5, 1), (5, 2)]),          # both admitted earlier in this pass
           ((7, 1), []),                        # ahead of p.round -> stays
           ((5, 3), [(4, 9)])]                  # unknown predecessor -> stays
    assert B.admit_pass(grown, 6, buf) == [1, 0, 1, 1, 0, 0]
    assert B.admit_pass(grown, 5, buf) == [1, 0, 1, 0, 0, 0]  # round 6 > p.round
    assert B.admit_pass(plain, 4, buf) == [0, 0, 0, 0, 0, 0]
    for cur in (5, 6):  # (5,1) admitted into p.dag[5] of a 5-round DAG
        with pytest.raises(B.GoPanic):
            B.admit_pass(plain, cur, buf)
    with pytest.raises(B.GoPanic):  # (5,3)'s absent predecessor scanned past p.dag[7]
        B.admit_pass(grown, 8, buf)


def _random_buffer(rng, plain, n, R, q):
    """Buffered vertices of rounds around R with predecessors drawn from present ids,
    absent ids, the ghost id and other buffered vertices (earlier or later)."""
    ids = []
    for _ in range(q):
        ids.append((int(rng.integers(max(R - 3, 0), R + 2)), int(rng.integers(1, n + 1))))
    present = [v[0] for rnd in plain for v in rnd]
    buf = []
    for vid in ids:
        k = int(rng.integers(0, 6))
        preds = []
        for _ in range(k):
            u = rng.random()
            if u < 0.55 and present:
                preds.append(tuple(present[int(rng.integers(0, len(present)))]))
            elif u < 0.8:
                preds.append(ids[int(rng.integers(0, len(ids)))])
            elif u < 0.9:
                preds.append((0, 0))
            else:
                preds.append((int(rng.integers(-1, R + 3)), int(rng.integers(0, n + 2))))
        buf.append((vid, preds))
    return buf


def _expect(e, cur, buf, plain):
    """GPU admit flags == the oracle's, or DR_E_INVAL where the oracle panics."""
    try:
        want = B.admit_pass(plain, cur, buf)
    except B.GoPanic:
        with pytest.raises(L.DrError) as ei:
            e.buffer_admit(cur, buf)
        assert ei.value.code == L.DR_E_INVAL, cur
        return "panic"
    assert e.buffer_admit(cur, buf).tolist() == want, cur
    return want


@pytest.mark.gpu
def test_gpu_buffer_figure1(gpu_device):
    g, dag = figure1()
    plain = oracle.setweak.to_plain(dag)
    buf = [((5, 1), [(4, 1), (4, 2)]), ((6, 1), [(5, 1), (5, 2)]), ((5, 2), [(4, 3), (0, 0)]),
           ((6, 2), [(5, 1), (5, 2)]), ((7, 1), []), ((5, 3), [(4, 9)])]
    with Engine(g["n"], g["faulty"], 8, gpu_device) as e:
        e.append_lists(dag)
        got = {cur: _expect(e, cur, buf, plain) for cur in (3, 4, 5, 6, 7)}
        assert got[5] == got[6] == got[7] == "panic"
        assert e.buffer_admit(4, []).tolist() == []
        e.append_lists(dag + [[], [], []])  # open rounds 5..7 (p.dag grown)
        grown = plain + [[], [], []]
        got = {cur: _expect(e, cur, buf, grown) for cur in (3, 4, 5, 6, 7, 8)}
        assert got[6] == [1, 0, 1, 1, 0, 0] and got[8] == "panic"


@pytest.mark.gpu
@pytest.mark.parametrize("seed,n,R,q", [(1, 6, 12, 40), (2, 30, 10, 300), (3, 100, 8, 2000)])
def test_gpu_buffer_random(gpu_device, seed, n, R, q):
    rng = np.random.default_rng(500 + seed)
    d = random_dag(rng, n, R, p_present=0.8, p_s=0.35, p_w=0.15, max_depth=6)
    plain = oracle.setweak.to_plain(d.to_lists())
    grown = plain + [[], []]
    with Engine(n, (n - 1) // 3, R + 4, gpu_device) as e:
        e.append_packed(d)
        for _ in range(3):
            buf = _random_buffer(rng, plain, n, R, q)
            for cur in (R - 2, R - 1, R + 1):
                _expect(e, cur, buf, plain)
        e.append_lists(d.to_lists() + [[], []])  # rounds R+1, R+2 opened
        for _ in range(2):
            buf = _random_buffer(rng, plain, n, R, q)
            for cur in (R - 1, R + 1, R + 2, R + 3):
                _expect(e, cur, buf, grown)
