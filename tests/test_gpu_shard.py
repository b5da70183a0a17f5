"""GPU parity of the process-column sharded path (include/dagrider_shard.h).

The sharded sweep splits every strong row and the weak edges by target column
across G shards and exchanges the per-round frontier (local mode: shared buffer;
RCCL mode: ncclAllGather).  Bar: reach sets and path() answers bit-identical to the
oracle (oracle/ref_bitset.c cones, pinned to TestPath and the literal restatement)
and to the unsharded engine, for every shard count.
"""
import numpy as np
import pytest

import oracle
from dag_rider_amd import _lib as L
from dag_rider_amd.dag import pack_lists
from dag_rider_amd.engine import Engine
from dag_rider_amd.gen import CONFIGS, generate, small_config
from dag_rider_amd.shard import ShardEngine, shard_unique_id
from dagutil import dag_fingerprint, figure1, load_large, random_dag

pytestmark = pytest.mark.gpu


def _check_reach(se, bs, froms, bottoms):
    for strong in (True, False):
        got = se.reach_sets(froms, bottoms, strong)
        for fr, bt, m in zip(froms, bottoms, got):
            want, _ = bs.cone(fr, bt, strong)
            assert (m == want).all(), (fr, bt, strong)


def test_shard_figure1_testpath(gpu_device):
    """TestPath (process_internal_test.go:8-84) through the sharded path, G = 1..4."""
    g, dag = figure1()
    d = pack_lists(dag, g["n"])
    for G in (1, 2, 4):
        with ShardEngine(g["n"], g["faulty"], 8, gpu_device, nshards=G) as se:
            se.append_packed(d)
            for t in g["test_path"]:
                got = se.path_batch([(tuple(t["from"]), tuple(t["to"]))], t["strong"])[0]
                assert bool(got) == t["want"], (G, t)
            ids = [tuple(x) for x in g["allpairs_ids"]]
            pairs = [(a, b) for a in ids for b in ids]
            for key, strong in (("strong", True), ("any", False)):
                got = se.path_batch(pairs, strong).reshape(len(ids), len(ids))
                assert (got == np.asarray(g["allpairs"][key], dtype=np.uint8)).all(), (G, key)


@pytest.mark.parametrize("seed,n,R", [(1, 5, 24), (2, 70, 30), (3, 130, 20), (4, 300, 12)])
def test_shard_random_dags(gpu_device, seed, n, R):
    """Unconstrained random DAGs (dangling targets, ghosts, deep weak edges) at G = 1, 2, 3, 8."""
    rng = np.random.default_rng(1000 + seed)
    d = random_dag(rng, n, R, p_present=0.8, p_s=0.3, p_w=0.2, max_depth=7)
    bs = oracle.PDag(d)
    froms = [(int(rng.integers(1, R + 1)), int(rng.integers(1, n + 1))) for _ in range(70)]  # > one batch of 64
    bottoms = [int(rng.integers(0, fr[0] + 1)) for fr in froms]
    ids = [(r, s) for r in range(R + 1) for s in range(0, n + 1)]
    samp = [ids[i] for i in rng.choice(len(ids), size=min(len(ids), 24), replace=False)]
    pairs = [(a, b) for a in samp for b in samp]
    for G in (1, 2, 3, 8):
        with ShardEngine(n, (n - 1) // 3, R + 1, gpu_device, nshards=G) as se:
            se.append_packed(d)
            _check_reach(se, bs, froms, bottoms)
            for strong in (True, False):
                want = np.asarray([bs.path(a, b, strong) for a, b in pairs], dtype=np.uint8)
                assert (se.path_batch(pairs, strong) == want).all(), (G, strong)


def test_shard_incremental_append_and_edge_queries(gpu_device):
    """Round-by-round appends; bottom == top; absent/unknown sources agree with dr_reach_sets."""
    rng = np.random.default_rng(9)
    n, R = 90, 16
    d = random_dag(rng, n, R, p_present=0.7, p_s=0.4, p_w=0.3, max_depth=5)
    bs = oracle.PDag(d)
    with ShardEngine(n, 29, R + 1, gpu_device, nshards=2) as se, Engine(n, 29, R + 1, gpu_device) as e:
        for r in range(R + 1):
            se.append_packed(d, r, r + 1)
        e.append_packed(d)
        assert se.num_rounds == R + 1
        froms = [(R, 1), (R, n), (7, 3), (5, 5), (R, 0), (3, n)]
        bottoms = [R, 0, 7, 0, 2, 1]
        for strong in (True, False):
            got = se.reach_sets(froms, bottoms, strong)
            ref = e.reach_sets(froms, bottoms, strong)
            for a, b in zip(got, ref):
                assert (a == b).all()
        _check_reach(se, bs, [f for f in froms if f[1] >= 1], [b for f, b in zip(froms, bottoms) if f[1] >= 1])


def test_shard_generated_n1024(gpu_device):
    """C4 parameters (n=1024, weak delta 2..4) on 120 rounds: G = 1, 2, 4, 8 agree with the oracle."""
    cfg = small_config(1024, 120, 4, p_present=1.0, p_late=0.02, p_w=0.5, weak_depth=4)
    d = generate(cfg)
    bs = oracle.PDag(d)
    rng = np.random.default_rng(5)
    froms = [(120, 1), (117, 512)] + [(int(rng.integers(60, 121)), int(rng.integers(1, 1025))) for _ in range(10)]
    bottoms = [0, 30] + [int(rng.integers(0, 50)) for _ in range(10)]
    for G in (1, 2, 4, 8):
        with ShardEngine(1024, 341, 121, gpu_device, nshards=G) as se:
            se.append_packed(d)
            info = se.info()
            assert info["nshards"] == G and info["nlocal"] == G and (info["col0"], info["col1"]) == (1, 1025)
            _check_reach(se, bs, froms, bottoms)
            st = se.stats()
            assert st["rounds"] > 0 and st["exchange_bytes"] == 0  # local mode: no collective


def test_shard_rccl_single_rank(gpu_device):
    """RCCL mode with a one-rank communicator: the all-gather path runs and agrees."""
    rng = np.random.default_rng(11)
    n, R = 200, 20
    d = random_dag(rng, n, R, p_present=0.8, p_s=0.3, p_w=0.2, max_depth=6)
    bs = oracle.PDag(d)
    uid = shard_unique_id()
    with ShardEngine(n, 66, R + 1, gpu_device, nshards=1, rank=0, unique_id=uid) as se:
        se.append_packed(d)
        froms = [(R, s) for s in range(1, 40)]
        bottoms = [0] * len(froms)
        _check_reach(se, bs, froms, bottoms)
        st = se.stats()
        assert st["exchange_bytes"] > 0
        # the whole replay through the all-gathers (memo path: K^cand and every step)
        f, nw = 66, R // 4
        for cm, dm in MODES:  # one rank holds every column: the fused replay, nothing to exchange
            got = se.replay(nw, cm, dm)
            _same_replay(got, bs.replay(f, nw, cm, dm))
            assert got.sweep["canon_segments"] >= 0
        se.set_stepped(True)  # the stepped replay through the all-gathers (votes, K^cand, every step)
        for cm, dm in MODES:
            got = se.replay(nw, cm, dm)
            _same_replay(got, bs.replay(f, nw, cm, dm))
            assert got.sweep["canon_segments"] >= 0 and se.stats()["exchange_bytes"] > 0


def test_shard_errors(gpu_device):
    with pytest.raises(L.DrError):
        ShardEngine(10, 3, 8, gpu_device, nshards=0)
    with pytest.raises(L.DrError):
        ShardEngine(10, 3, 8, gpu_device, nshards=2, rank=1)  # local mode is rank 0
    g, dag = figure1()
    d = pack_lists(dag, g["n"])
    with ShardEngine(g["n"], g["faulty"], 8, gpu_device, nshards=2) as se:
        se.append_packed(d)
        with pytest.raises(L.DrError) as ei:
            se.reach_sets([(9, 1)], [0], True)
        assert ei.value.code == L.DR_E_INVAL
        with pytest.raises(L.DrError) as ei:
            se.append_packed(d, 2, 3)  # not contiguous
        assert ei.value.code == L.DR_E_STATE
    # a strong edge outside r-1 (bit 31 of weak_tgt) is named as unsupported, with its round
    from dag_rider_amd.gen import with_extra_edges
    d2 = with_extra_edges(d, [(4, 1, 1, 2, True)])
    with ShardEngine(g["n"], g["faulty"], 8, gpu_device, nshards=2) as se:
        with pytest.raises(L.DrError) as ei:
            se.append_packed(d2)
        assert ei.value.code == L.DR_E_CONTRACT
        assert "strong edge (4,1)->(1,2) outside r-1" in str(ei.value)


# --------------------------------------------------------------------------- commit + delivery
MODES = [(cm, dm) for cm in (L.DR_CHAIN_LITERAL, L.DR_CHAIN_PERSISTENT) for dm in (L.DR_DELIVER_REF, L.DR_DELIVER_PAPER)]


def _same_replay(a, b):
    assert (a.commit == b.commit).all()
    assert (a.vcount == b.vcount).all()
    assert (a.push_off == b.push_off).all()
    assert (a.push_wave == b.push_wave).all()
    for k in ("pop_count", "pop_digest", "pop_edges"):
        g, w = getattr(a, k), getattr(b, k)
        bad = np.nonzero(g != w)[0]
        assert len(bad) == 0, f"{k}: {len(bad)} pops differ, first at {bad[:5].tolist()}"
    assert (a.commit_edges, a.chain_edges, a.deliver_edges) == (b.commit_edges, b.chain_edges, b.deliver_edges)


@pytest.mark.parametrize("seed", range(12))
def test_shard_replay_random_dags(gpu_device, seed):
    """dr_shard_replay == the bitset oracle (every output, all four chain x deliver modes)
    on unconstrained random DAGs, at several shard counts, persistent and per-round launches."""
    rng = np.random.default_rng(3000 + seed)
    n = int(rng.choice([1, 4, 7, 64, 65, 130, 200, 300]))
    R = int(rng.integers(8, 41))
    d = random_dag(rng, n, R, p_present=rng.uniform(0.5, 1), p_s=rng.uniform(0.05, 0.9), p_w=rng.uniform(0, 1),
                   max_depth=int(rng.integers(2, 20)))
    f = int(rng.integers(0, (n - 1) // 3 + 2))
    nw = R // 4
    bs = oracle.PDag(d)
    for G in ((1, 2) if seed % 2 else (3, 8)):
        with ShardEngine(n, f, R + 1, gpu_device, nshards=G) as se:
            se.append_packed(d)
            for memo, persistent, stepped in ((True, True, False), (True, True, True), (False, True, False),
                                              (False, False, False)):
                se.set_memo(memo)
                se.set_persistent(persistent)
                se.set_stepped(stepped)
                for cm, dm in MODES:
                    want = bs.replay(f, nw, cm, dm)
                    assert want.rc == 0
                    _same_replay(se.replay(nw, cm, dm), want)


@pytest.mark.parametrize("seed", range(4))
def test_shard_memo_replay_generated(gpu_device, seed):
    """The memoized sharded replay (summaries per shard, canonical cone, pops and chains;
    fused, and stepped by relative round) == the bitset oracle on quorum-shaped DAGs with
    late vertices, weak edges up to 12 deep and absent leaders, at G = 1, 2, 3, 8, both
    chain modes, REF and PAPER delivery."""
    from dag_rider_amd.gen import small_config

    rng = np.random.default_rng(4400 + seed)
    n = int(rng.choice([64, 100, 256, 700, 1024]))
    cfg = small_config(n, int(rng.integers(40, 120)), 60 + seed, p_present=float(rng.uniform(0.9, 1)),
                       p_late=float(rng.uniform(0.02, 0.3)), p_w=float(rng.uniform(0.1, 0.6)),
                       weak_depth=int(rng.integers(2, 13)), p_la=0.1)
    d = generate(cfg)
    bs = oracle.PDag(d)
    nw = cfg.nwaves
    for G in (1, 2, 3, 8):
        with ShardEngine(n, cfg.faulty, d.nrounds, gpu_device, nshards=G) as se:
            se.append_packed(d)
            for stepped in (False, True):
                se.set_stepped(stepped)
                for cm, dm in MODES:
                    got = se.replay(nw, cm, dm)
                    _same_replay(got, bs.replay(cfg.faulty, nw, cm, dm))
                    assert got.sweep["canon_segments"] >= 0  # the memo path ran


def test_shard_commit_chain_order_calls(gpu_device):
    """The per-call entry points (wave_commit, wave_ready, order_vertices) == the engine's."""
    rng = np.random.default_rng(77)
    n, R = 100, 36
    d = random_dag(rng, n, R, p_present=0.9, p_s=0.7, p_w=0.4, max_depth=6)
    f = 20
    with ShardEngine(n, f, R + 1, gpu_device, nshards=4) as se, Engine(n, f, R + 1, gpu_device) as e:
        se.append_packed(d)
        e.append_packed(d)
        nw = R // 4
        a, b = se.wave_commit(1, nw), e.wave_commit(1, nw)
        assert (a[0] == b[0]).all() and (a[1] == b[1]).all()
        for w in range(1, nw + 1):
            for dec in (0, max(0, w - 3)):
                assert se.wave_ready(w, dec) == e.wave_ready(w, dec)
        for cur in (R, 20, 3, 0):
            stack = [(4 * w - 3, 1) for w in range(1, nw + 1)] + [(9, 5), (9, 5), (30, 17)]
            for mode in (L.DR_DELIVER_REF, L.DR_DELIVER_PAPER):
                tot, pc, pd = se.order_vertices(stack, cur, mode)
                _, pc2, pd2 = e.order_vertices(stack, cur, mode, cap=0)
                assert (pc == pc2).all() and (pd == pd2).all() and tot == int(pc2.sum()), (cur, mode)


def test_shard_stepped_steps_on_after_append(gpu_device):
    """The stepped replay launches as many steps as the last replay took; after an append
    (longer chains and cones) or a coin change it must step on until every query ends, and
    still equal the oracle.  Then a repeated replay waits on the host once."""
    from dag_rider_amd.gen import small_config

    cfg = small_config(130, 120, 71, p_present=0.95, p_late=0.2, p_w=0.4, weak_depth=6, p_la=0.3)
    d = generate(cfg)
    f = cfg.faulty
    rng = np.random.default_rng(5)
    for G in (1, 3):
        with ShardEngine(cfg.n, f, d.nrounds, gpu_device, nshards=G) as se:
            se.set_stepped(True)
            se.append_packed(d, 0, 41)
            bs = oracle.PDag(d)  # waves 1..10 read rounds <= 40 only
            for cm, dm in MODES:
                _same_replay(se.replay(10, cm, dm), bs.replay(f, 10, cm, dm))
            se.append_packed(d, 41, d.nrounds)
            for cm, dm in MODES:
                _same_replay(se.replay(cfg.nwaves, cm, dm), bs.replay(f, cfg.nwaves, cm, dm))
            _same_replay(se.replay(cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF),
                         bs.replay(f, cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF))
            assert se.stats()["host_syncs"] == 1
            leaders = [int(x) for x in rng.integers(1, cfg.n + 1, size=cfg.nwaves + 1)]
            se.set_leader_coin(L.DR_LEADER_TABLE, table=leaders)
            bl = oracle.PDag(d, leaders=leaders)
            for cm, dm in MODES:
                _same_replay(se.replay(cfg.nwaves, cm, dm), bl.replay(f, cfg.nwaves, cm, dm))


@pytest.mark.parametrize("seed", range(3))
def test_shard_stepped_canon_continuation(gpu_device, seed):
    """A canonical walk still live after the launched steps resumes after the batch steps
    ran (the walk and the batch shared their pending ring and frontier buffers).
    Step hints of 1 force the continuation on a first replay whose walk has several
    segments; every mode against the bitset oracle at G = 1 and 3."""
    rng = np.random.default_rng(6100 + seed)
    n, R = int(rng.choice([64, 130, 200])), 60
    # sparse strong edges: rounds their successors do not cover start canonical segments
    d = random_dag(rng, n, R, p_present=0.85, p_s=0.04, p_w=0.5, max_depth=8)
    f = (n - 1) // 3
    nw = R // 4
    bs = oracle.PDag(d)
    # (the stepped form does not count the walk's segments: the unsharded engine's walk of
    # the same DAG says there is one to continue through -- a segment spans at least dmax
    # rounds, so a step hint of 1 leaves the walk live after the first step)
    from dag_rider_amd.engine import Engine

    with Engine(n, f, R + 1, gpu_device) as e:
        e.append_packed(d)
        assert e.replay(nw, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF).sweep["canon_segments"] >= 1
    for G in (1, 3):
        for cm, dm in MODES:
            with ShardEngine(n, f, R + 1, gpu_device, nshards=G) as se:
                se.append_packed(d)
                se.set_stepped(True)
                se.set_step_hints(1)
                _same_replay(se.replay(nw, cm, dm), bs.replay(f, nw, cm, dm))


def test_shard_replay_leader_coin(gpu_device):
    """A caller's leader table (chooseLeader as a coin) through the sharded commit, chains and pops."""
    rng = np.random.default_rng(91)
    n, R = 40, 40
    d = random_dag(rng, n, R, p_present=0.9, p_s=0.8, p_w=0.3)
    leaders = [int(x) for x in rng.integers(1, n + 1, size=R // 4 + 1)]
    bs = oracle.PDag(d, leaders=leaders)
    with ShardEngine(n, 13, R + 1, gpu_device, nshards=2) as se:
        se.append_packed(d)
        se.set_leader_coin(L.DR_LEADER_TABLE, table=leaders)
        for stepped in (False, True):
            se.set_stepped(stepped)
            for cm, dm in MODES:
                _same_replay(se.replay(R // 4, cm, dm), bs.replay(13, R // 4, cm, dm))


def test_shard_replay_c4_full(gpu_device):
    """BASELINE config 4 (n=1024 x 4000 rounds) on the column-sharded DAG at G = 1, 2, 4, 8
    (local mode): the whole replay equals the committed golden vectors (ref and paper)."""
    g = load_large()["c4"]
    cfg = CONFIGS["c4"]
    d = generate(cfg, nthreads=16)
    assert dag_fingerprint(d) == g["dag"], "generator drift"
    for G in (1, 2, 4, 8):
        with ShardEngine(cfg.n, cfg.faulty, d.nrounds, gpu_device, nshards=G) as se:
            se.append_packed(d)
            got = se.replay(cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF)
            _check_golden(got, g["persistent_ref"])
            assert got.sweep["canon_segments"] >= 0 and se.stats()["rounds"] < 100  # memo: a few dozen steps
            _check_golden(se.replay(cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_PAPER), g["persistent_paper"])
            if G in (2, 8):  # the stepped form (what each rank of a G-rank group runs)
                se.set_stepped(True)
                _check_golden(se.replay(cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF), g["persistent_ref"])
                # again with the step counts the first replay took: every launch back to back, one host wait
                _check_golden(se.replay(cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF), g["persistent_ref"])
                assert se.stats()["host_syncs"] == 1
                se.set_stepped(False)
            if G in (1, 8):  # the batched full sweeps (DR_SHARD_OPT_MEMO 0), REF
                se.set_memo(False)
                _check_golden(se.replay(cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF), g["persistent_ref"])


def _check_golden(got, want):
    assert "".join(str(int(x)) for x in got.commit) == want["commit"]
    assert got.vcount.tolist() == want["vcount"]
    assert got.push_off.tolist() == want["push_off"]
    assert got.push_wave.tolist() == want["push_wave"]
    for k in ("pop_count", "pop_digest", "pop_edges"):
        w = np.asarray([int(x) for x in want[k]], dtype=np.uint64)
        bad = np.nonzero(getattr(got, k) != w)[0]
        assert len(bad) == 0, f"{k}: {len(bad)} pops differ, first at {bad[:5].tolist()}"
    assert (got.commit_edges, got.chain_edges, got.deliver_edges) == \
        (int(want["commit_edges"]), int(want["chain_edges"]), int(want["deliver_edges"]))
