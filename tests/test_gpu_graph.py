"""DR_OPT_REPLAY_GRAPH: a repeated device-planned dr_replay is captured once as a hipGraph
and relaunched.  Every graph launch must give the oracle's replay (process.go:314-354
waveReady, :404-443 orderVertices), and any change of the DAG, the options, the wave count,
the modes or the push capacity must leave the graph for a fresh launch sequence."""
import numpy as np
import pytest

import oracle
from dag_rider_amd import _lib as L
from dag_rider_amd.engine import Engine
from dag_rider_amd.gen import CONFIGS, generate
from dagutil import dag_fingerprint, load_large, random_dag

pytestmark = pytest.mark.gpu


def _same(a, b):
    assert (a.commit == b.commit).all() and (a.vcount == b.vcount).all()
    assert (a.push_off == b.push_off).all() and (a.push_wave == b.push_wave).all()
    assert (a.pop_count == b.pop_count).all() and (a.pop_digest == b.pop_digest).all()
    assert (a.pop_edges == b.pop_edges).all()
    assert (a.commit_edges, a.chain_edges, a.deliver_edges) == (b.commit_edges, b.chain_edges, b.deliver_edges)


@pytest.mark.parametrize("timing", [0, 1])
@pytest.mark.parametrize("name", ["c2", "c5"])
def test_graph_replays_match_oracle(gpu_device, name, timing):
    cfg = CONFIGS[name]
    d = generate(cfg)
    bs = oracle.PDag(d)
    with Engine(cfg.n, cfg.faulty, d.nrounds, gpu_device) as e:
        e.append_packed(d)
        e.set_replay_graph(True)
        e.set_phase_timing(timing)
        for cm in (L.DR_CHAIN_PERSISTENT, L.DR_CHAIN_LITERAL):
            for dm in (L.DR_DELIVER_REF, L.DR_DELIVER_PAPER):
                want = bs.replay(cfg.faulty, cfg.nwaves, cm, dm)
                states = []
                for _ in range(4):
                    got = e.replay(cfg.nwaves, cm, dm)
                    states.append(e.replay_graph_state())
                    _same(got, want)
                    if timing:
                        assert got.ms["summary"] > 0  # the summary pass's events are graph nodes
                # first call with this configuration: kernel by kernel; second: captured
                assert states == [0, 1, 1, 1], states
        # a push capacity below the pushes: refused from the launch sequence, then again
        # from a graph of that configuration
        want = bs.replay(cfg.faulty, cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF)
        if len(want.push_wave) > 1:
            for _ in range(3):
                with pytest.raises(L.DrError) as ei:
                    e.replay(cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF, push_cap=len(want.push_wave) - 1)
                assert ei.value.code == L.DR_E_CAPACITY
        _same(e.replay(cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF), want)
        # option off (the default): kernel by kernel, same results
        e.set_replay_graph(False)
        for _ in range(2):
            _same(e.replay(cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF), want)
            assert e.replay_graph_state() == 0


@pytest.mark.parametrize("seed", range(6))
def test_graph_after_append_and_other_calls(gpu_device, seed):
    """Appending rounds (a new DAG version), per-call paths that rebuild the canonical cone
    (wave_ready, order_vertices: they swap K and Kprev) and a memo switch all sit between
    graph replays; every replay equals the oracle's on the DAG as it stands."""
    rng = np.random.default_rng(9100 + seed)
    n = int(rng.choice([16, 64, 100, 257]))
    R = 4 * int(rng.integers(8, 20)) + 1
    d = random_dag(rng, n, R, p_present=rng.uniform(0.7, 1), p_s=rng.uniform(0.1, 0.9), p_w=rng.uniform(0, 0.6),
                   max_depth=int(rng.integers(2, 8)))
    f = int(rng.integers(0, (n - 1) // 3 + 1))
    cut = R - 4
    nw = cut // 4
    with Engine(n, f, R + 1, gpu_device) as e:
        e.set_replay_graph(True)
        e.set_phase_timing(1)
        e.append_packed(d, 0, cut + 1)
        full = oracle.PDag(d)
        # waves 1..nw read rounds <= 4 nw only: the same replay on the prefix and the whole DAG
        want = full.replay(f, nw, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF)
        for _ in range(3):
            _same(e.replay(nw, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF), want)
        assert e.replay_graph_state() == 1
        e.append_packed(d, cut + 1, d.nrounds)
        # the same wave count over a longer DAG: a new version, never the old graph
        got = e.replay(nw, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF)
        assert e.replay_graph_state() == 0
        _same(got, want)
        for _ in range(2):
            _same(e.replay(nw, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF), want)
        assert e.replay_graph_state() == 1
        # per-call paths between graph replays
        cm, vc = e.wave_commit(1, nw)
        assert cm.tolist() == want.commit.tolist()
        stack = [(4 * w - 3, e.wave_leader(w)) for w in range(nw, 0, -1) if want.commit[w - 1]][:2]
        if stack:
            ids_, cnt_, dg_ = e.order_vertices(stack, R, L.DR_DELIVER_REF)
            _, wids, wc, wd = full.order_vertices(stack, R, L.DR_DELIVER_REF)
            assert ids_.tolist() == wids.tolist() and cnt_.tolist() == wc.tolist()
        for _ in range(3):
            _same(e.replay(nw, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF), want)
        # memo off (host-planned general path), then on again
        e.set_memo(False)
        _same(e.replay(nw, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF), want)
        e.set_memo(True)
        for _ in range(3):
            _same(e.replay(nw, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF), want)
        assert e.replay_graph_state() == 1


def test_graph_c4_golden(gpu_device):
    """The driver bench's configuration: graph launches of the full C4 replay against the
    committed golden, with the summary pass timed by graph event nodes."""
    g = load_large()["c4"]
    cfg = CONFIGS["c4"]
    d = generate(cfg, nthreads=16)
    assert dag_fingerprint(d) == g["dag"], "generator drift"
    want = g["persistent_ref"]
    with Engine(cfg.n, cfg.faulty, d.nrounds, gpu_device) as e:
        e.append_packed(d)
        e.set_replay_graph(True)
        e.set_phase_timing(1)
        for i in range(3):
            got = e.replay(cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF)
            assert e.replay_graph_state() == (1 if i else 0)
            assert "".join(str(int(x)) for x in got.commit) == want["commit"]
            assert got.push_wave.tolist() == want["push_wave"]
            for k in ("pop_count", "pop_digest", "pop_edges"):
                w = np.asarray([int(x) for x in want[k]], dtype=np.uint64)
                assert (getattr(got, k) == w).all(), k
            assert got.deliver_edges == int(want["deliver_edges"])
            assert got.ms["summary"] > 0
