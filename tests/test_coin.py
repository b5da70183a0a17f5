"""chooseLeader (process.go:386-392) as a global coin: DR_LEADER_CONST1 (the
reference's constant 1, the default), DR_LEADER_SEEDED (a seeded coin every process
computes alike) and DR_LEADER_TABLE (the caller's coin output, e.g. a threshold
signature).  The reference has no coin to pin against: these tests pin the engine's
per-wave leader through the oracles, which take the same leader table, and the
seeded coin against its restatement (oracle.coin_leaders).  CONST1 leaves every
golden vector unchanged (tests/test_gpu_golden.py runs with the default)."""
import numpy as np
import pytest

import oracle
from dag_rider_amd import _lib as L
from dag_rider_amd.engine import Engine, replay_batch
from dag_rider_amd.gen import CONFIGS, c5_config, generate
from dagutil import random_dag

MODES = [(cm, dm) for cm in (L.DR_CHAIN_LITERAL, L.DR_CHAIN_PERSISTENT) for dm in (L.DR_DELIVER_REF, L.DR_DELIVER_PAPER)]


def _same(a, b, chain=True):
    """Every replay output; chain=False for the literal oracle, which does not count chain edges."""
    assert (a.commit == b.commit).all()
    assert (a.vcount == b.vcount).all()
    assert (a.push_off == b.push_off).all()
    assert (a.push_wave == b.push_wave).all()
    assert (a.pop_count == b.pop_count).all()
    assert (a.pop_digest == b.pop_digest).all()
    assert (a.pop_edges == b.pop_edges).all()
    assert (a.commit_edges, a.deliver_edges) == (b.commit_edges, b.deliver_edges)
    assert not chain or a.chain_edges == b.chain_edges


def test_seeded_coin_restated():
    """dr_coin_leader (a pure function: no device needed) == oracle.coin_leaders."""
    lib = L.lib()
    for seed, n in ((0, 4), (7, 64), (2**63 + 5, 1024), (12345, 2048)):
        want = oracle.coin_leaders(seed, n, 300)
        assert [lib.dr_coin_leader(seed, w, n) for w in range(1, 301)] == want
        assert all(1 <= x <= n for x in want) and len(set(want)) > 1


@pytest.mark.parametrize("seed", range(12))
def test_oracles_agree_with_coin(seed):
    rng = np.random.default_rng(700 + seed)
    n = int(rng.integers(2, 12))
    R = int(rng.integers(8, 30))
    d = random_dag(rng, n, R, p_present=rng.uniform(0.6, 1), p_s=rng.uniform(0.3, 0.9), p_w=rng.uniform(0, 0.6))
    f = (n - 1) // 3
    leaders = [int(x) for x in rng.integers(1, n + 1, size=R // 4 + 1)]
    lit, bs = oracle.LDag(packed=d, leaders=leaders), oracle.PDag(d, leaders=leaders)
    for cm, dm in MODES:
        a = lit.replay(f, R // 4, cm, dm, ids_cap=1 << 16)
        b = bs.replay(f, R // 4, cm, dm, ids_cap=1 << 16)
        assert a.rc == b.rc == 0
        _same(a, b, chain=False)
        assert (a.ids == b.ids).all()
    for w in range(1, R // 4 + 1):
        rc, v = lit.leader(w)
        assert rc < 0 or rc == 0 or v == (4 * w - 3, leaders[w - 1])


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(8))
def test_gpu_coin_random(gpu_device, seed):
    rng = np.random.default_rng(800 + seed)
    n = int(rng.choice([3, 7, 40, 64, 65, 130, 300]))
    R = int(rng.integers(12, 40))
    d = random_dag(rng, n, R, p_present=rng.uniform(0.6, 1), p_s=rng.uniform(0.2, 0.9), p_w=rng.uniform(0, 0.5),
                   max_depth=int(rng.integers(2, 10)))
    f = int(rng.integers(0, (n - 1) // 3 + 2))
    nw = R // 4
    with Engine(n, f, d.nrounds, gpu_device) as e:
        e.append_packed(d)
        for mode in (L.DR_LEADER_SEEDED, L.DR_LEADER_TABLE):
            if mode == L.DR_LEADER_SEEDED:
                coin = 1000 + seed
                e.set_leader_coin(mode, seed=coin)
                leaders = oracle.coin_leaders(coin, n, nw + 1)
            else:
                leaders = [int(x) for x in rng.integers(1, n + 1, size=nw + 1)]
                e.set_leader_coin(mode, table=leaders)
            assert [e.wave_leader(w) for w in range(1, nw + 2)] == leaders
            ld, bs = oracle.LDag(packed=d, leaders=leaders), oracle.PDag(d, leaders=leaders)
            for cm, dm in MODES:
                want = bs.replay(f, nw, cm, dm)
                for memo in (True, False):
                    for plan in (True, False):
                        e.set_memo(memo)
                        e.set_device_plan(plan)
                        _same(e.replay(nw, cm, dm), want)
            e.set_memo(True)
            for w in range(1, nw + 1):
                rc, vc, st = ld.wave_ready(f, w, max(0, w - 3))
                cm_, vc_, pushed = e.wave_ready(w, max(0, w - 3))
                assert vc_ == vc and cm_ == (len(st) > 0)
                assert [(4 * (x - 1) + 1, leaders[x - 1]) for x in pushed] == [tuple(s) for s in st]
        e.set_leader_coin(L.DR_LEADER_CONST1)
        _same(e.replay(nw), oracle.PDag(d).replay(f, nw))
        with pytest.raises(L.DrError):
            e.set_leader_coin(L.DR_LEADER_TABLE, table=[n + 1])


@pytest.mark.gpu
def test_gpu_coin_c2_and_c5(gpu_device):
    cfg = CONFIGS["c2"]
    d = generate(cfg)
    leaders = oracle.coin_leaders(99, cfg.n, cfg.nwaves)
    with Engine(cfg.n, cfg.faulty, d.nrounds, gpu_device) as e:
        e.append_packed(d)
        e.set_leader_coin(L.DR_LEADER_SEEDED, seed=99)
        for cm in (L.DR_CHAIN_LITERAL, L.DR_CHAIN_PERSISTENT):
            _same(e.replay(cfg.nwaves, cm), oracle.PDag(d, leaders=leaders).replay(cfg.faulty, cfg.nwaves, cm))
    # the fused small-DAG batch kernel takes each context's leaders
    engines, dags, tabs = [], [], []
    for i in range(24):
        c = c5_config(i)
        dd = generate(c)
        e = Engine(c.n, c.faulty, dd.nrounds, gpu_device)
        e.append_packed(dd)
        t = oracle.coin_leaders(i, c.n, c.nwaves)
        e.set_leader_coin(L.DR_LEADER_TABLE, table=t)
        engines.append(e)
        dags.append((c, dd))
        tabs.append(t)
    for cm, dm in MODES:
        got = replay_batch(engines, c5_config(0).nwaves, cm, dm)
        for (c, dd), t, g in zip(dags, tabs, got):
            _same(g, oracle.PDag(dd, leaders=t).replay(c.faulty, c.nwaves, cm, dm))
            assert g.ms["deliver"] > 0
    for e in engines:
        e.close()


@pytest.mark.gpu
def test_gpu_coin_figure1(gpu_device):
    """waveReady on the Figure-1 DAG (process_internal_test.go:86-283) under a table coin."""
    g_leaders = [3, 2, 4]
    from dagutil import figure1

    g, dag = figure1()
    with Engine(g["n"], g["faulty"], 8, gpu_device) as e:
        e.append_lists(dag)
        e.set_leader_coin(L.DR_LEADER_TABLE, table=g_leaders)
        ld = oracle.LDag(arrays=__import__("dag_rider_amd").flatten_lists(dag), leaders=g_leaders)
        rc, vc, st = ld.wave_ready(g["faulty"], 1, 0)
        cm, vc_, pushed = e.wave_ready(1, 0)
        assert (cm, vc_) == (rc == 1, vc)
