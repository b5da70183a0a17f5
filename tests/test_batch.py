"""GPU parity of dr_replay_batch: the fused one-wavefront-per-DAG
replay (dag_rider_amd/csrc/batch.hpp) against the oracle, against per-context
dr_replay, and against the C5 golden fingerprints (tests/golden/large_replay.json.gz).

random_dag draws unconstrained DAGs (partial quorums, failed commits, leader chains,
dangling targets, ghost slots), which the quorum-shaped generator never produces.
"""
import numpy as np
import pytest

import oracle
from dag_rider_amd import _lib as L
from dag_rider_amd.engine import Engine, ReplayBatch, replay_batch
from dag_rider_amd.gen import CONFIGS, c5_config, generate
from dagutil import dag_fingerprint, load_large, random_dag, replay_fingerprint

pytestmark = pytest.mark.gpu

MODES = [(cm, dm) for cm in (L.DR_CHAIN_LITERAL, L.DR_CHAIN_PERSISTENT) for dm in (L.DR_DELIVER_REF, L.DR_DELIVER_PAPER)]
# the fused kernel's two forms (batch.hpp: a workgroup per DAG, batch1w.hpp: a wavefront per DAG)
FORMS = [L.DR_BATCH_WORKGROUP, L.DR_BATCH_WAVE]


def _same(a, b):
    assert (a.commit == b.commit).all()
    assert (a.vcount == b.vcount).all()
    assert (a.push_off == b.push_off).all()
    assert (a.push_wave == b.push_wave).all()
    assert (a.pop_count == b.pop_count).all()
    assert (a.pop_digest == b.pop_digest).all()
    assert (a.pop_edges == b.pop_edges).all()
    assert (a.commit_edges, a.chain_edges, a.deliver_edges) == (b.commit_edges, b.chain_edges, b.deliver_edges)


def _random_batch(dev, seed, count, nw, ns=(1, 4, 7, 33, 64, 65, 100, 128), depth=(2, 12)):
    rng = np.random.default_rng(seed)
    items = []
    for _ in range(count):
        n = int(rng.choice(ns))
        R = 4 * nw + int(rng.integers(0, 6))
        d = random_dag(rng, n, R, p_present=rng.uniform(0.5, 1), p_s=rng.uniform(0.05, 0.9),
                       p_w=rng.uniform(0, 1), max_depth=int(rng.integers(*depth)))
        f = int(rng.integers(0, (n - 1) // 3 + 2))
        e = Engine(n, f, d.nrounds, dev)
        e.append_packed(d)
        items.append((d, f, e))
    return items


@pytest.mark.parametrize("form", FORMS)
@pytest.mark.parametrize("cm,dm", MODES)
def test_batch_random_vs_oracle(gpu_device, cm, dm, form):
    nw = 10
    items = _random_batch(gpu_device, 77 + 4 * cm + dm, 24, nw)
    items[0][2].set_batch_form(form)
    got = replay_batch([e for _, _, e in items], nw, cm, dm)
    for (d, f, e), g in zip(items, got):
        want = oracle.PDag(d).replay(f, nw, cm, dm)
        assert want.rc == 0
        _same(g, want)
        assert g.ms["deliver"] > 0  # the fused kernel ran
    for _, _, e in items:
        e.close()


@pytest.mark.parametrize("form", FORMS)
def test_batch_max_waves(gpu_device, form):
    """nw = 64 (the fused path's limit) at n = 128: long literal chains, up to 2080 pops."""
    nw = 64
    items = _random_batch(gpu_device, 5, 3, nw, ns=(128, 100, 64))
    items[0][2].set_batch_form(form)
    for cm, dm in MODES:
        got = replay_batch([e for _, _, e in items], nw, cm, dm)
        for (d, f, e), g in zip(items, got):
            _same(g, oracle.PDag(d).replay(f, nw, cm, dm))
    for _, _, e in items:
        e.close()


@pytest.mark.parametrize("form", FORMS)
def test_batch_matches_single_replay(gpu_device, form):
    """The fused batch and dr_replay context by context agree on everything."""
    nw = 12
    items = _random_batch(gpu_device, 9, 16, nw, depth=(2, 31))
    items[0][2].set_batch_form(form)
    for cm, dm in MODES:
        got = replay_batch([e for _, _, e in items], nw, cm, dm)
        for (_, _, e), g in zip(items, got):
            _same(g, e.replay(nw, cm, dm))
    for _, _, e in items:
        e.close()


def test_batch_general_shapes_fall_back(gpu_device):
    """n > 128 or weak deltas >= 32 in any context: the batch replays context by context."""
    nw = 6
    items = _random_batch(gpu_device, 11, 3, nw) + _random_batch(gpu_device, 12, 1, nw, ns=(200,)) + \
        _random_batch(gpu_device, 13, 1, nw, depth=(33, 40))
    for cm, dm in MODES:
        got = replay_batch([e for _, _, e in items], nw, cm, dm)
        for (d, f, e), g in zip(items, got):
            _same(g, oracle.PDag(d).replay(f, nw, cm, dm))
    for _, _, e in items:
        e.close()


def test_batch_errors(gpu_device):
    cfg = CONFIGS["c1"]  # 4 waves, commits (and so pushes) on every present leader
    d = generate(cfg)
    es = []
    for _ in range(2):
        es.append(Engine(cfg.n, cfg.faulty, d.nrounds, gpu_device))
        es[-1].append_packed(d)
    with pytest.raises(L.DrError) as ei:
        replay_batch([es[0], es[0]], 4)
    assert ei.value.code == L.DR_E_INVAL
    with pytest.raises(L.DrError) as ei:
        replay_batch(es, 50)  # rounds of wave 50 are not mirrored
    assert ei.value.code == L.DR_E_INVAL
    # capacity: a batch whose first context pushes more leaders than its buffers hold
    b = ReplayBatch(es, 4, L.DR_CHAIN_LITERAL)
    for i in range(len(es)):
        b._outs[i].push_cap = 0
    with pytest.raises(L.DrError) as ei:
        b.run()
    assert ei.value.code == L.DR_E_CAPACITY
    for e in es:
        e.close()


@pytest.mark.parametrize("form", FORMS)
def test_c5_batch_golden(gpu_device, form):
    """C5: 4096 independent n=128 x 128-round replays (seeds 5000+i) in one batch,
    bit-exact against the committed fingerprints (PERSISTENT/REF for all, LITERAL/REF and
    PERSISTENT/PAPER for the first 64), in both forms of the fused kernel."""
    g = load_large()["c5"]
    count = g["count"]
    engines = []
    try:
        for i in range(count):
            cfg = c5_config(i)
            d = generate(cfg)
            assert dag_fingerprint(d) == g["dag"][i], f"generator drift at C5 DAG {i}"
            e = Engine(cfg.n, cfg.faulty, d.nrounds, gpu_device)
            e.append_packed(d)
            engines.append(e)
        engines[0].set_batch_form(form)
        nw = c5_config(0).nwaves
        got = replay_batch(engines, nw, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF)
        bad = [i for i, r in enumerate(got) if replay_fingerprint(r) != g["persistent_ref"][i]]
        assert not bad, f"{len(bad)} C5 replays differ, first {bad[:8]}"
        detail = engines[:len(g["literal_ref"])]
        for key, cm, dm in (("literal_ref", L.DR_CHAIN_LITERAL, L.DR_DELIVER_REF),
                            ("persistent_paper", L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_PAPER)):
            got = replay_batch(detail, nw, cm, dm)
            assert [replay_fingerprint(r) for r in got] == g[key], key
    finally:
        for e in engines:
            e.close()


@pytest.mark.parametrize("form", FORMS)
def test_batch_plan_reuse(gpu_device, form):
    """A repeated batch (same contexts, modes and output buffers) reuses its plan: the
    checks, job table and output layout of the last call (engine.hip, BatchPlan). Any
    ABI call that can change a context in between -- appends, the leader coin, an
    option (the batch form), create/destroy -- and a changed output capacity or chain
    mode rebuild it."""
    nw = 8
    rng = np.random.default_rng(31)
    items = []
    for n in (4, 33, 64, 100, 128, 7):
        d = random_dag(rng, n, 4 * nw + 8, p_present=0.9, p_s=0.6, p_w=0.5, max_depth=8)
        f = (n - 1) // 3
        e = Engine(n, f, d.nrounds, gpu_device)
        e.append_packed(d, 0, 4 * nw + 1)  # rounds 0..4nw: the batch's waves and no more
        items.append((d, f, e))
    engines = [e for _, _, e in items]
    engines[0].set_batch_form(form)
    cm, dm = L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF
    want = [oracle.PDag(d).replay(f, nw, cm, dm) for d, f, _ in items]
    b = ReplayBatch(engines, nw, cm, dm)
    for _ in range(3):  # the first call builds the plan, the next ones reuse it
        for w, g in zip(want, b()):
            _same(g, w)
    for e, (d, _, _) in zip(engines[::2], items[::2]):  # appends in between: rebuilt
        e.append_packed(d)
    for _ in range(2):
        for w, g in zip(want, b()):
            _same(g, w)
    engines[2].set_leader_coin(L.DR_LEADER_SEEDED, 99)  # a different leader schedule
    got = b()
    for i, e in enumerate(engines):
        _same(got[i], e.replay(nw, cm, dm))
    engines[2].set_leader_coin()
    for w, g in zip(want, b()):
        _same(g, w)
    # a smaller output capacity in between (same buffers): rebuilt, and it must not fit
    np_max = max(len(w.push_wave) for w in want)
    i_max = max(range(len(want)), key=lambda i: len(want[i].push_wave))
    cap0 = b._outs[i_max].push_cap
    b._outs[i_max].push_cap = np_max - 1
    with pytest.raises(L.DrError) as ei:
        b.run()
    assert ei.value.code == L.DR_E_CAPACITY
    b._outs[i_max].push_cap = cap0
    for w, g in zip(want, b()):
        _same(g, w)
    # the other batch form on the first context (an option: rebuilt)
    engines[0].set_batch_form(L.DR_BATCH_WAVE if form != L.DR_BATCH_WAVE else L.DR_BATCH_WORKGROUP)
    for _ in range(2):
        for w, g in zip(want, b()):
            _same(g, w)
    engines[0].set_batch_form(form)
    # the other chain mode on the same output buffers: the mode is part of the plan's key
    bl = ReplayBatch(engines, nw, L.DR_CHAIN_LITERAL, dm)  # literal chains need the larger capacity
    want_lit = [oracle.PDag(d).replay(f, nw, L.DR_CHAIN_LITERAL, dm) for d, f, _ in items]
    for w, g in zip(want_lit, bl()):
        _same(g, w)
    bl.chain_mode = cm
    for _ in range(2):
        for w, g in zip(want, bl()):
            _same(g, w)
    bl.chain_mode = L.DR_CHAIN_LITERAL
    for w, g in zip(want_lit, bl()):
        _same(g, w)
    for e in engines:
        e.close()
    # new contexts (possibly at the old addresses) with new DAGs: rebuilt
    items = _random_batch(gpu_device, 32, 6, nw)
    items[0][2].set_batch_form(form)
    b = ReplayBatch([e for _, _, e in items], nw, cm, dm)
    for _ in range(2):
        for (d, f, _), g in zip(items, b()):
            _same(g, oracle.PDag(d).replay(f, nw, cm, dm))
    for _, _, e in items:
        e.close()


@pytest.mark.gpu
@pytest.mark.parametrize("form", [L.DR_BATCH_WORKGROUP, L.DR_BATCH_WAVE])
def test_batch_view_in_place(gpu_device, form):
    """dr_replay_batch_view: every context's results read in place from the batch's one
    copy back equal the oracle's and dr_replay_batch's, in all four chain x delivery
    modes, on repeated calls (the plan is reused) and across a rebuild (an append);
    a capacity below a context's pushes is DR_E_CAPACITY."""
    from dag_rider_amd.engine import ReplayBatchView

    nw = 6
    rng = np.random.default_rng(77)
    items = []
    for n in (4, 33, 64, 100, 128):
        d = random_dag(rng, n, 4 * nw + 6, p_present=0.9, p_s=0.6, p_w=0.5, max_depth=8)
        f = (n - 1) // 3
        e = Engine(n, f, d.nrounds, gpu_device)
        e.append_packed(d, 0, 4 * nw + 1)
        items.append((d, f, e))
    engines = [e for _, _, e in items]
    engines[0].set_batch_form(form)
    for cm in (L.DR_CHAIN_PERSISTENT, L.DR_CHAIN_LITERAL):
        for dm in (L.DR_DELIVER_REF, L.DR_DELIVER_PAPER):
            want = [oracle.PDag(d).replay(f, nw, cm, dm) for d, f, _ in items]
            bv = ReplayBatchView(engines, nw, cm, dm)
            for _ in range(2):
                bv.run()
                for w, g in zip(want, bv.results()):
                    _same(g, w)
            copied = ReplayBatch(engines, nw, cm, dm)()
            bv.run()
            for c, g in zip(copied, bv.results()):
                _same(g, c)
    items[1][2].append_packed(items[1][0])  # the rest of one DAG: the plan is rebuilt
    bv = ReplayBatchView(engines, nw)
    bv.run()
    for (d, f, _), g in zip(items, bv.results()):
        _same(g, oracle.PDag(d).replay(f, nw, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF))
    np_max = max(len(g.push_wave) for g in bv.results())
    small = ReplayBatchView(engines, nw, push_cap=np_max - 1)
    with pytest.raises(L.DrError) as ex:
        small.run()
    assert ex.value.code == L.DR_E_CAPACITY


@pytest.mark.parametrize("form", FORMS)
def test_batch_shared_stream(gpu_device, form):
    """DR_CREATE_SHARED_STREAM: contexts on the device's one shared stream (the C5 bench's
    batch members) replay alone and in a batch exactly as contexts with streams of their own,
    through appends in flight, destroys in any order and a new shared context after the
    last one went."""
    nw = 8
    rng = np.random.default_rng(515)
    dags = []
    for _ in range(6):
        n = int(rng.choice((7, 64, 100, 128)))
        d = random_dag(rng, n, 4 * nw + 2, p_present=0.9, p_s=0.5, p_w=0.5, max_depth=6)
        dags.append((d, int(rng.integers(0, (n - 1) // 3 + 1))))
    shared = []
    for d, f in dags:
        e = Engine(d.n, f, d.nrounds, gpu_device, shared_stream=True)
        e.append_packed(d)  # (the copies may still run when the next context appends)
        shared.append(e)
    shared[0].set_batch_form(form)
    for cm, dm in MODES:
        got = replay_batch(shared, nw, cm, dm)
        for (d, f), e, g in zip(dags, shared, got):
            want = oracle.PDag(d).replay(f, nw, cm, dm)
            _same(g, want)
            _same(e.replay(nw, cm, dm), want)
    for i in (3, 0, 5):  # destroy out of order; the others keep the stream
        shared[i].close()
    rest = [e for i, e in enumerate(shared) if i not in (3, 0, 5)]
    rest[0].set_batch_form(form)
    got = replay_batch(rest, nw, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF)
    for (d, f), g in zip([x for i, x in enumerate(dags) if i not in (3, 0, 5)], got):
        _same(g, oracle.PDag(d).replay(f, nw, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF))
    for e in rest:
        e.close()
    d, f = dags[1]
    with Engine(d.n, f, d.nrounds, gpu_device, shared_stream=True) as e:  # the stream is created again
        e.append_packed(d)
        _same(e.replay(nw, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF),
              oracle.PDag(d).replay(f, nw, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF))
