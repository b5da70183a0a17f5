"""GPU parity: the HIP path (through the C ABI) against the oracle and the golden fixtures.

Bar: bit-exact for every output (commit bits, vote counts, pushed leaders, delivered
order via full id lists or count+digest, edges traversed, reach sets).
"""
import numpy as np
import pytest

import oracle
from dag_rider_amd import _lib as L
from dag_rider_amd.dag import flatten_lists, pack_lists
from dag_rider_amd.engine import Engine
from dag_rider_amd.gen import CONFIGS, generate
from dagutil import figure1, random_dag

pytestmark = pytest.mark.gpu


# --------------------------------------------------------------------------- Figure-1
def test_figure1_testpath(gpu_device):
    """TestPath (process_internal_test.go:8-84) through dr_append_rounds_lists + dr_path_batch."""
    g, dag = figure1()
    with Engine(g["n"], g["faulty"], 8, gpu_device) as e:
        e.append_lists(dag)
        for t in g["test_path"]:
            got = e.path_batch([(tuple(t["from"]), tuple(t["to"]))], t["strong"])[0]
            assert bool(got) == t["want"], t


def test_figure1_allpairs(gpu_device):
    g, dag = figure1()
    ids = [tuple(x) for x in g["allpairs_ids"]]
    pairs = [(a, b) for a in ids for b in ids]
    with Engine(g["n"], g["faulty"], 8, gpu_device) as e:
        e.append_lists(dag)
        for key, strong in (("strong", True), ("any", False)):
            got = e.path_batch(pairs, strong).reshape(len(ids), len(ids))
            assert (got == np.asarray(g["allpairs"][key], dtype=np.uint8)).all(), key


def test_figure1_wave_ready_and_order(gpu_device):
    g, dag = figure1()
    d = g["derived"]
    with Engine(g["n"], g["faulty"], 8, gpu_device) as e:
        e.append_lists(dag)
        commit, vcount, pushed = e.wave_ready(1, 0)
        assert (commit, vcount) == (d["wave_ready_1"]["commit"], d["wave_ready_1"]["vcount"])
        assert pushed == []
        for case in d["order_vertices"]:
            ids, cnt, dg = e.order_vertices([tuple(x) for x in case["stack"]], case["p_round"])
            assert ids.tolist() == case["want"]
            assert int(cnt[0]) == len(case["want"])
            assert int(dg[0]) == oracle.digest([tuple(x) for x in case["want"]])
        # strong reach set of (4,1) down to round 0
        (m,) = e.reach_sets([(4, 1)], [0], True)
        got = [[r, s] for r in range(5) for s in range(1, 5) if (int(m[r][0]) >> (s - 1)) & 1]
        assert got == d["strong_reach_4_1"]


def test_figure1_multi_pop_stack(gpu_device):
    """LIFO pops (stack/stack.go:23-28), ref (no dedup, Q2) vs paper (dedup) modes."""
    g, dag = figure1()
    ld = oracle.LDag(arrays=__import__("dag_rider_amd").flatten_lists(dag))
    stack = [(1, 1), (3, 3), (4, 1)]
    with Engine(g["n"], g["faulty"], 8, gpu_device) as e:
        e.append_lists(dag)
        for mode in (L.DR_DELIVER_REF, L.DR_DELIVER_PAPER):
            ids, cnt, dg = e.order_vertices(stack, 4, mode)
            rc, want, wc, wd = ld.order_vertices(stack, 4, mode)
            assert rc == 0
            assert ids.tolist() == want.tolist()
            assert cnt.tolist() == wc.tolist() and dg.tolist() == wd.tolist()


# --------------------------------------------------------------------------- random DAGs
def _compare_replay(a, b, ids=True):
    assert (a.commit == b.commit).all()
    assert (a.vcount == b.vcount).all()
    assert (a.push_off == b.push_off).all()
    assert (a.push_wave == b.push_wave).all()
    assert (a.pop_count == b.pop_count).all()
    assert (a.pop_digest == b.pop_digest).all()
    assert (a.pop_edges == b.pop_edges).all()
    assert a.commit_edges == b.commit_edges
    assert a.deliver_edges == b.deliver_edges
    if ids:
        assert (a.ids == b.ids).all()


@pytest.mark.parametrize("seed", range(48))
def test_random_dag_replay(gpu_device, seed):
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.choice([1, 3, 4, 7, 10, 63, 64, 65, 100, 130, 200, 257, 300, 513]))
    R = int(rng.integers(4, 41))
    # mostly shallow weak edges (round summaries apply), sometimes deep ones (they do not)
    depth = int(rng.integers(2, 12)) if seed % 4 else int(rng.integers(12, 40))
    d = random_dag(rng, n, R, p_present=rng.uniform(0.5, 1), p_s=rng.uniform(0.05, 0.9), p_w=rng.uniform(0, 1),
                   max_depth=depth)
    f = int(rng.integers(0, (n - 1) // 3 + 2))
    nw = R // 4
    bs = oracle.PDag(d)
    with Engine(n, f, R + 1, gpu_device) as e:
        if seed % 2:  # DR_OPT_FUSE: every launch grouping plus the fast merge (Q_FAST)
            e.set_fuse(63)
        # append in two chunks: exercises the append-only mirror
        cut = int(rng.integers(1, R + 1))
        e.append_packed(d, 0, cut)
        e.append_packed(d, cut, d.nrounds)
        for memo in (True, False):
            e.set_memo(memo)
            for cm in (L.DR_CHAIN_LITERAL, L.DR_CHAIN_PERSISTENT):
                for dm in (L.DR_DELIVER_REF, L.DR_DELIVER_PAPER):
                    want = bs.replay(f, nw, cm, dm, ids_cap=1 << 20)
                    assert want.rc == 0
                    got = e.replay(nw, cm, dm, ids_cap=1 << 20)
                    _compare_replay(got, want)
                    assert got.chain_edges == want.chain_edges
                    got2 = e.replay(nw, cm, dm)  # no ids: REF mode dedups identical leaders
                    _compare_replay(got2, want, ids=False)
            # orderVertices with arbitrary stacks and p.round below the leaders
            stack = [(int(rng.integers(0, R + 1)), int(rng.integers(1, n + 1))) for _ in range(3)]
            cur = int(rng.integers(0, R + 1))
            # literal BFS oracle (O(n^3 R^2)) for small n, the bitset oracle otherwise
            ov = oracle.LDag(packed=d) if n <= 16 else bs
            for mode in (L.DR_DELIVER_REF, L.DR_DELIVER_PAPER):
                ids_, cnt_, dg_ = e.order_vertices(stack, cur, mode)
                rc, want_ids, wc, wd = ov.order_vertices(stack, cur, mode)
                assert rc == 0
                assert ids_.tolist() == want_ids.tolist()
                assert cnt_.tolist() == wc.tolist() and dg_.tolist() == wd.tolist()
        e.set_memo(True)
        # path(): all pairs over a sample
        ids = [(r, s) for r in range(R + 1) for s in range(0, n + 1)]
        samp = [ids[i] for i in rng.choice(len(ids), size=min(len(ids), 40), replace=False)]
        pairs = [(a, b) for a in samp for b in samp]
        for strong in (True, False):
            got = e.path_batch(pairs, strong)
            want = np.asarray([bs.path(a, b, strong) for a, b in pairs], dtype=np.uint8)
            assert (got == want).all()
        # reach sets
        froms = [samp[i] for i in range(min(8, len(samp))) if samp[i][1] >= 1]
        if froms:
            bottoms = [int(rng.integers(0, fr[0] + 1)) for fr in froms]
            for strong in (True, False):
                got = e.reach_sets(froms, bottoms, strong)
                for fr, bt, m in zip(froms, bottoms, got):
                    want, _ = bs.cone(fr, bt, strong)
                    assert (m == want).all()


@pytest.mark.parametrize("seed", range(8))
def test_chains_long_gaps(gpu_device, seed):
    """Leader chains (process.go:341-350) over long runs of absent or unreachable leaders
    and frontiers that empty (random_dag with few leaders and sparse strong edges), every
    replay output against the oracle."""
    rng = np.random.default_rng(7000 + seed)
    n = int(rng.choice([4, 16, 64, 100]))
    R = 4 * int(rng.integers(20, 48)) + int(rng.integers(1, 4))
    d = random_dag(rng, n, R, p_present=rng.uniform(0.6, 1), p_s=rng.uniform(0.03, 0.7), p_w=rng.uniform(0, 0.5),
                   max_depth=int(rng.integers(2, 8)), leader_p=float(rng.choice([0.05, 0.2, 0.6])))
    f = int(rng.integers(0, (n - 1) // 3 + 2))
    nw = R // 4
    bs = oracle.PDag(d)
    with Engine(n, f, R + 1, gpu_device) as e:
        e.append_packed(d)
        for cm in (L.DR_CHAIN_LITERAL, L.DR_CHAIN_PERSISTENT):
            for dm in (L.DR_DELIVER_REF, L.DR_DELIVER_PAPER):
                want = bs.replay(f, nw, cm, dm)
                assert want.rc == 0
                got = e.replay(nw, cm, dm)
                _compare_replay(got, want, ids=False)
                assert got.chain_edges == want.chain_edges


def test_far_weak_edges(gpu_device):
    """Weak edges spanning > 1023 rounds use the far format and global frontier rows."""
    rng = np.random.default_rng(77)
    n, R = 5, 1200
    d = random_dag(rng, n, R, p_present=0.9, p_s=0.6, p_w=0.002, max_depth=1150, ghosts=0.0)
    assert any(((r := int(t) >> 11) < 200) for t in d.weak_tgt)
    bs = oracle.PDag(d)
    with Engine(n, 1, R + 1, gpu_device) as e:
        e.append_packed(d)
        for cm in (L.DR_CHAIN_LITERAL, L.DR_CHAIN_PERSISTENT):
            want = bs.replay(1, R // 4, cm, L.DR_DELIVER_REF)
            _compare_replay(e.replay(R // 4, cm, L.DR_DELIVER_REF), want, ids=False)
        pairs = [((R, s), (r, t)) for s in range(1, n + 1) for r in (0, 1, 5, 100, 600) for t in range(1, n + 1)]
        got = e.path_batch(pairs, False)
        assert (got == np.asarray([bs.path(a, b, False) for a, b in pairs], dtype=np.uint8)).all()


def test_memo_on_off_large_n(gpu_device):
    """n=2048 (row stride 32 words) and n=1024 with shallow weak edges: memo == full sweeps."""
    for n, R in ((2048, 24), (1024, 40)):
        rng = np.random.default_rng(n)
        d = random_dag(rng, n, R, p_present=0.97, p_s=0.7, p_w=0.02, max_depth=5, dangling=0.001, ghosts=0.0)
        f = (n - 1) // 3
        want = oracle.PDag(d).replay(f, R // 4, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF)
        with Engine(n, f, R + 1, gpu_device) as e:
            e.append_packed(d)
            for memo in (True, False):
                e.set_memo(memo)
                _compare_replay(e.replay(R // 4, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF), want, ids=False)


@pytest.mark.parametrize("n,depth", [(1024, 64), (1024, 66), (1024, 80), (1024, 255), (1024, 256),
                                     (1100, 66), (1100, 127), (1100, 128), (300, 150)])
def test_memo_window_boundary(gpu_device, n, depth):
    """Weak deltas across the regular window (engine.hip kMemoMaxDelta = 255 and the sweeps'
    LDS ring: 256 rounds at row stride 16 (n=1024), 128 at stride 32 (n=1100), so the
    summaries hold deltas up to 255 / 127; deeper weak edges are exceptions, tested once,
    and the memo stays on while every one is benign -- here, every one): every mode, memo
    and device plan on and off, == the bitset oracle, and the memo path really ran."""
    from dag_rider_amd.gen import small_config

    cfg = small_config(n, depth + 24, 40 + depth, p_present=0.97, p_late=0.02, p_w=0.05, weak_depth=depth,
                       p_la=0.1)
    d = generate(cfg)
    g = np.repeat(np.arange(d.nrounds * n, dtype=np.int64), np.diff(d.weak_off.astype(np.int64)))
    assert int((g // n - (d.weak_tgt.astype(np.int64) >> 11)).max()) == depth
    f, nw = cfg.faulty, cfg.nwaves
    bs = oracle.PDag(d)
    with Engine(n, f, d.nrounds, gpu_device) as e:
        e.append_packed(d)
        for memo in (True, False):
            e.set_memo(memo)
            for plan in ((True, False) if memo else (True,)):
                e.set_device_plan(plan)
                for cm in (L.DR_CHAIN_LITERAL, L.DR_CHAIN_PERSISTENT):
                    for dm in (L.DR_DELIVER_REF, L.DR_DELIVER_PAPER):
                        want = bs.replay(f, nw, cm, dm)
                        assert want.rc == 0
                        got = e.replay(nw, cm, dm)
                        _compare_replay(got, want, ids=False)
                        assert got.chain_edges == want.chain_edges
                        limit = 255 if n <= 1024 else 127
                        st = e.exception_stats()
                        assert (st["exceptions"] > 0) == (depth > limit) and st["regular_delta"] <= limit, st
                        assert st["changing"] == 0, st
                        assert (got.sweep["canon_segments"] >= 0) == memo, (got.sweep, st)
        e.set_memo(True)
        e.set_device_plan(True)
        stack = [(4 * w - 3, 1) for w in range(1, nw + 1)]
        for mode in (L.DR_DELIVER_REF, L.DR_DELIVER_PAPER):
            _, cnt_, dg_ = e.order_vertices(stack, d.nrounds - 1, mode, cap=0)
            rc, _, wc, wd = bs.order_vertices(stack, d.nrounds - 1, mode, cap=1)
            assert rc == 0 and cnt_.tolist() == wc.tolist() and dg_.tolist() == wd.tolist()


def test_list_and_packed_append_agree(gpu_device):
    rng = np.random.default_rng(7)
    d = random_dag(rng, 9, 20, ghosts=0.3)
    lists = d.to_lists()
    d2 = pack_lists(lists, 9)
    with Engine(9, 2, 21, gpu_device) as a, Engine(9, 2, 21, gpu_device) as b:
        a.append_packed(d)
        b.append_lists(lists)
        ra, rb = a.replay(5, ids_cap=1 << 16), b.replay(5, ids_cap=1 << 16)
        _compare_replay(ra, rb)
    assert (d2.strong == d.strong).all() and (d2.slot_src == d.slot_src).all()


# --------------------------------------------------------------------------- configs
@pytest.mark.parametrize("name,memo", [(c, m) for c in ("c1", "c2", "c5") for m in (True, False)])
def test_config_replay(gpu_device, name, memo):
    cfg = CONFIGS[name]
    d = generate(cfg)
    bs = oracle.PDag(d)
    with Engine(cfg.n, cfg.faulty, d.nrounds, gpu_device) as e:
        e.append_packed(d)
        e.set_memo(memo)
        for cm in (L.DR_CHAIN_LITERAL, L.DR_CHAIN_PERSISTENT):
            want = bs.replay(cfg.faulty, cfg.nwaves, cm, L.DR_DELIVER_REF)
            got = e.replay(cfg.nwaves, cm, L.DR_DELIVER_REF)
            _compare_replay(got, want, ids=False)
            assert got.chain_edges == want.chain_edges
        want = bs.replay(cfg.faulty, cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_PAPER)
        got = e.replay(cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_PAPER)
        _compare_replay(got, want, ids=False)


@pytest.mark.parametrize("name", ["c1", "c2", "c5"])
def test_device_planned_replay_matches_host_planned(gpu_device, name):
    """DR_OPT_DEVICE_PLAN on/off: the device planner restates run_chains/run_deliver exactly
    (pushes, pops, per-pop counts/digests/edges, sweep statistics, timings aside)."""
    cfg = CONFIGS[name]
    d = generate(cfg)
    with Engine(cfg.n, cfg.faulty, d.nrounds, gpu_device) as e:
        e.append_packed(d)
        for cm in (L.DR_CHAIN_LITERAL, L.DR_CHAIN_PERSISTENT):
            e.set_device_plan(True)
            a = e.replay(cfg.nwaves, cm, L.DR_DELIVER_REF)
            e.set_device_plan(False)
            b = e.replay(cfg.nwaves, cm, L.DR_DELIVER_REF)
            _compare_replay(a, b, ids=False)
            assert a.chain_edges == b.chain_edges
            assert a.sweep == b.sweep
            # twice in a row (arena reuse), then with a push capacity that is too small
            e.set_device_plan(True)
            _compare_replay(e.replay(cfg.nwaves, cm, L.DR_DELIVER_REF), b, ids=False)
            if len(b.push_wave) > 1:
                with pytest.raises(L.DrError) as ei:
                    e.replay(cfg.nwaves, cm, L.DR_DELIVER_REF, push_cap=len(b.push_wave) - 1)
                assert ei.value.code == L.DR_E_CAPACITY


@pytest.mark.parametrize("name", ["c1", "c2", "c5"])
def test_device_planned_paper_matches_host_planned(gpu_device, name):
    """PAPER delivery on the device-planned path (first-pop ownership of the merge sweeps'
    cones, replay_plan.hpp k_paper_*) against the host-planned pruned sweeps and the oracle."""
    cfg = CONFIGS[name]
    d = generate(cfg)
    bs = oracle.PDag(d)
    with Engine(cfg.n, cfg.faulty, d.nrounds, gpu_device) as e:
        e.append_packed(d)
        for cm in (L.DR_CHAIN_LITERAL, L.DR_CHAIN_PERSISTENT):
            e.set_device_plan(True)
            a = e.replay(cfg.nwaves, cm, L.DR_DELIVER_PAPER)
            e.set_device_plan(False)
            b = e.replay(cfg.nwaves, cm, L.DR_DELIVER_PAPER)
            _compare_replay(a, b, ids=False)
            _compare_replay(a, bs.replay(cfg.faulty, cfg.nwaves, cm, L.DR_DELIVER_PAPER), ids=False)
            e.set_device_plan(True)  # twice in a row: arena reuse, cone rebuilt after the PAPER replay
            _compare_replay(e.replay(cfg.nwaves, cm, L.DR_DELIVER_REF),
                            bs.replay(cfg.faulty, cfg.nwaves, cm, L.DR_DELIVER_REF), ids=False)
            _compare_replay(e.replay(cfg.nwaves, cm, L.DR_DELIVER_PAPER), b, ids=False)


def test_c1_literal_ids(gpu_device):
    """C1 seeded n=4: full delivered sequence against the literal restatement."""
    cfg = CONFIGS["c1"]
    d = generate(cfg)
    lit = oracle.LDag(packed=d)
    with Engine(cfg.n, cfg.faulty, d.nrounds, gpu_device) as e:
        e.append_packed(d)
        for cm in (L.DR_CHAIN_LITERAL, L.DR_CHAIN_PERSISTENT):
            for dm in (L.DR_DELIVER_REF, L.DR_DELIVER_PAPER):
                want = lit.replay(cfg.faulty, cfg.nwaves, cm, dm, ids_cap=1 << 16)
                got = e.replay(cfg.nwaves, cm, dm, ids_cap=1 << 16)
                _compare_replay(got, want)


# --------------------------------------------------------------------------- errors
def test_errors(gpu_device):
    g, dag = figure1()
    with Engine(4, 1, 8, gpu_device) as e:
        e.append_lists(dag)
        with pytest.raises(L.DrError) as ei:
            e.path_batch([((9, 1), (1, 1))], True)  # Go: index out of range
        assert ei.value.code == L.DR_E_INVAL
        assert e.path_batch([((9, 1), (9, 1))], True)[0] == 1  # self path returns before the lookup
        with pytest.raises(L.DrError):
            e.wave_commit(2, 2)  # round(2,1)=5 is not mirrored
        with pytest.raises(L.DrError) as ei:
            e.order_vertices([(4, 1)], 5)
        assert ei.value.code == L.DR_E_INVAL
    with Engine(4, 1, 8, gpu_device) as e:
        from dag_rider_amd.dag import Vertex, VertexID
        bad = [list(r) for r in dag]
        bad[3][1] = Vertex(VertexID(3, 1), b"", [VertexID(9, 1)])  # a target past max_rounds: no id the mirror holds
        with pytest.raises(L.DrError) as ei:
            e.append_lists(bad)
        assert ei.value.code == L.DR_E_CONTRACT
        ok = [list(r) for r in dag]
        ok[3][1] = Vertex(VertexID(3, 1), b"", [VertexID(1, 1)])  # a strong edge skipping a round (App. A Q8): kept
        e.append_lists(ok)
        ld = oracle.LDag(arrays=flatten_lists(ok))
        pairs = [((3, 1), (r, s)) for r in range(4) for s in range(1, 5)]
        assert e.path_batch(pairs, True).tolist() == [ld.path(a, b, True) for a, b in pairs]
