"""GPU parity on DAGs with repeated ids.

The reference appends a vertex whose id is already in its round when uponDeliver or
the buffer loop hands it one (process/process.go:158-169, :229).  path() then follows
the id's LAST slot (:112-116), waveReady's vCount counts every slot of round 4w (:332),
orderVertices delivers every slot in REF (the no-op filter, :418-429) and an id once
in PAPER.  The mirror accepts such DAGs through every append path and replays them on
the memo path (round summaries, canonical cone and emission count every slot of a
reached id; PAPER skips an id's later slots) and on the full sweeps; checked here
against the literal restatement (oracle/ref_literal.c),
which follows process.go line by line, on list-form DAGs whose repeated slots carry
their own edges."""
import numpy as np
import pytest

import oracle
from dag_rider_amd import _lib as L
from dag_rider_amd.dag import Vertex, VertexID, flatten_lists
from dag_rider_amd.engine import Engine, replay_batch
from dagutil import random_dag, with_repeated_ids

pytestmark = pytest.mark.gpu

MODES = [(cm, dm) for cm in (L.DR_CHAIN_LITERAL, L.DR_CHAIN_PERSISTENT) for dm in (L.DR_DELIVER_REF, L.DR_DELIVER_PAPER)]


def _same(got, want, ids=True):
    assert (got.commit == want.commit).all()
    assert (got.vcount == want.vcount).all()
    assert (got.push_off == want.push_off).all() and (got.push_wave == want.push_wave).all()
    assert (got.pop_count == want.pop_count).all()
    assert (got.pop_digest == want.pop_digest).all()
    assert (got.pop_edges == want.pop_edges).all()
    assert (got.commit_edges, got.deliver_edges) == (want.commit_edges, want.deliver_edges)
    if ids:
        assert got.ids.tolist() == want.ids.tolist()


@pytest.mark.parametrize("seed", range(10))
def test_repeated_ids_replay_path_order(gpu_device, seed):
    rng = np.random.default_rng(8800 + seed)
    n = int(rng.choice([3, 4, 7, 20, 64, 70]))
    R = int(rng.integers(8, 25))
    base = random_dag(rng, n, R, p_present=rng.uniform(0.6, 1), p_s=rng.uniform(0.2, 0.9),
                      p_w=rng.uniform(0, 0.8), max_depth=int(rng.integers(2, 9))).to_lists()
    dag = with_repeated_ids(rng, base, p_dup=float(rng.uniform(0.1, 0.5)))
    f = int(rng.integers(0, (n - 1) // 3 + 2))
    nw = R // 4
    ld = oracle.LDag(arrays=flatten_lists(dag))
    with Engine(n, f, R + 1, gpu_device) as e:
        cut = int(rng.integers(1, R + 1))
        e.append_lists(dag, 0, cut)
        e.append_lists(dag, cut, R + 1)
        for memo in (True, False):
            e.set_memo(memo)
            for plan in ((True, False) if memo else (True,)):
                e.set_device_plan(plan)
                for cm, dm in MODES:
                    want = ld.replay(f, nw, cm, dm, ids_cap=1 << 16)
                    assert want.rc == 0
                    _same(e.replay(nw, cm, dm, ids_cap=1 << 16), want)
                    got = e.replay(nw, cm, dm)
                    _same(got, want, ids=False)
                    assert (got.sweep["canon_segments"] >= 0) == memo  # the memo path ran
        e.set_memo(True)
        e.set_device_plan(True)
        # waveReady / orderVertices per call, path over a sample of pairs
        for w in range(1, nw + 1):
            rc, vc, st = ld.wave_ready(f, w, max(0, w - 2))
            cm_, vc_, pushed = e.wave_ready(w, max(0, w - 2))
            assert vc_ == vc and cm_ == (rc == 1)
        stack = [(int(rng.integers(0, R + 1)), int(rng.integers(1, n + 1))) for _ in range(3)]
        cur = int(rng.integers(0, R + 1))
        for mode in (L.DR_DELIVER_REF, L.DR_DELIVER_PAPER):
            ids_, cnt_, dg_ = e.order_vertices(stack, cur, mode)
            rc, want_ids, wc, wd = ld.order_vertices(stack, cur, mode)
            assert rc == 0
            assert ids_.tolist() == want_ids.tolist()
            assert cnt_.tolist() == wc.tolist() and dg_.tolist() == wd.tolist()
        allids = sorted({(v.id.round, v.id.source) for r in dag for v in r})
        samp = [allids[i] for i in rng.choice(len(allids), size=min(len(allids), 30), replace=False)]
        pairs = [(a, b) for a in samp for b in samp]
        for strong in (True, False):
            got = e.path_batch(pairs, strong)
            assert got.tolist() == [ld.path(a, b, strong) for a, b in pairs]


def test_repeated_ids_appended_one_by_one(gpu_device):
    """dr_append_vertices with ids already in old rounds (the buffer loop re-delivering
    a vertex): each repeat replaces the id's vertex for path(); checked after every
    append against the oracle on the same [][]vertex."""
    rng = np.random.default_rng(42)
    n, R = 8, 14
    dag = random_dag(rng, n, R, p_present=0.9, p_s=0.7, p_w=0.3, ghosts=0.0).to_lists()
    with Engine(n, 2, R + 4, gpu_device) as e:
        e.append_lists(dag)
        cur = [list(r) for r in dag]
        for step in range(12):
            r = int(rng.integers(1, R + 1))
            ids = [v.id for v in cur[r]]
            vid = ids[int(rng.integers(0, len(ids)))]
            prev = sorted({v.id for v in cur[r - 1]}, key=lambda x: (x.round, x.source))  # distinct targets
            below = sorted({v.id for rr in range(max(0, r - 5), r - 1) for v in cur[rr]},
                           key=lambda x: (x.round, x.source))
            v = Vertex(vid, b"", [u for u in prev if rng.random() < 0.5], [u for u in below if rng.random() < 0.15])
            e.append_vertices([v])
            cur[r].append(v)
            ld = oracle.LDag(arrays=flatten_lists(cur))
            nw = R // 4
            for cm, dm in MODES:
                _same(e.replay(nw, cm, dm, ids_cap=1 << 15), ld.replay(2, nw, cm, dm, ids_cap=1 << 15))
            pairs = [((R, s), (rr, t)) for s in range(1, n + 1) for rr in range(0, R) for t in range(1, n + 1)]
            assert e.path_batch(pairs, False).tolist() == [ld.path(a, b, False) for a, b in pairs]


def test_repeated_ids_in_a_batch(gpu_device):
    """dr_replay_batch with a context holding repeated ids: that context replays on its
    own (the fused small-DAG kernel counts per id), every result equal to dr_replay."""
    rng = np.random.default_rng(77)
    engines, want = [], []
    nw = 4
    for i in range(3):
        base = random_dag(rng, 16, 4 * nw, p_present=1.0, p_s=0.8, p_w=0.3, ghosts=0.0).to_lists()
        dag = with_repeated_ids(rng, base, p_dup=0.3) if i == 1 else base
        e = Engine(16, 5, 4 * nw + 1, gpu_device)
        e.append_lists(dag)
        engines.append(e)
        want.append(oracle.LDag(arrays=flatten_lists(dag)))
    try:
        for cm, dm in MODES:
            got = replay_batch(engines, nw, cm, dm)
            for g, ld in zip(got, want):
                _same(g, ld.replay(5, nw, cm, dm), ids=False)
    finally:
        for e in engines:
            e.close()


@pytest.mark.parametrize("seed", range(3))
def test_repeated_slots_generated_memo(gpu_device, seed):
    """Quorum-shaped DAGs (the C4 generator's spec) with repeated slots (gen.with_repeated_slots)
    on the memo path -- round summaries, canonical cone, device-planned and host-planned
    emission -- == the bitset oracle (oracle/ref_bitset.c, repeated ids: one row per id,
    vCount / REF count every slot, PAPER the first) in every mode; the memo path ran."""
    from dag_rider_amd.gen import generate, small_config

    rng = np.random.default_rng(9100 + seed)
    n = int(rng.choice([64, 130, 256, 1024]))
    cfg = small_config(n, int(rng.integers(40, 90)), 70 + seed, p_present=0.97, p_late=0.05, p_w=0.4,
                       weak_depth=int(rng.integers(2, 9)), p_la=0.1, p_dup=float(rng.uniform(0.02, 0.2)))
    d = generate(cfg)
    off = d.slot_off
    reps = sum(int((x := d.slot_src[off[r]:off[r + 1]])[x != 0].size - np.unique(x[x != 0]).size)
               for r in range(1, d.nrounds))
    assert reps > 0  # repeated ids present
    bs = oracle.PDag(d)
    nw = cfg.nwaves
    with Engine(n, cfg.faulty, d.nrounds, gpu_device) as e:
        e.append_packed(d)
        for plan in (True, False):
            e.set_device_plan(plan)
            for cm, dm in MODES:
                want = bs.replay(cfg.faulty, nw, cm, dm)
                assert want.rc == 0
                got = e.replay(nw, cm, dm)
                _same(got, want, ids=False)
                assert got.chain_edges == want.chain_edges
                assert got.sweep["canon_segments"] >= 0
