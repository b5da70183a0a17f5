"""CPU tests of the oracle itself: pinned to the reference's known answers, then the
two restatements (literal BFS, packed bitset) cross-checked on seeded DAGs."""
import json
import os

import numpy as np
import pytest

import oracle
from dag_rider_amd.dag import flatten_lists, pack_lists
from dag_rider_amd.gen import CONFIGS, generate, small_config
from dagutil import GOLDEN, figure1, random_dag


def test_figure1_testpath_literal():
    """TestPath (process_internal_test.go:20-83) on the literal restatement."""
    g, dag = figure1()
    ld = oracle.LDag(arrays=flatten_lists(dag))
    for t in g["test_path"]:
        assert bool(ld.path(tuple(t["from"]), tuple(t["to"]), t["strong"])) == t["want"], t["ref"]


def test_figure1_testpath_bitset():
    g, dag = figure1()
    bs = oracle.PDag(pack_lists(dag, 4))
    for t in g["test_path"]:
        assert bool(bs.path(tuple(t["from"]), tuple(t["to"]), t["strong"])) == t["want"], t["ref"]


def test_figure1_derived_answers():
    g, dag = figure1()
    d = g["derived"]
    ld = oracle.LDag(arrays=flatten_lists(dag))
    rc, leader = ld.leader(1)
    assert rc == 1 and list(leader) == d["wave_ready_1"]["leader"]
    voters = [bool(ld.path((v.id.round, v.id.source), leader, True)) for v in dag[4]]
    assert voters == d["wave_ready_1"]["voters"]
    rc, vc, stack = ld.wave_ready(g["faulty"], 1, 0)
    assert (rc, vc, stack) == (int(d["wave_ready_1"]["commit"]), d["wave_ready_1"]["vcount"], [])
    for case in d["order_vertices"]:
        rc, ids, cnt, dg = ld.order_vertices([tuple(x) for x in case["stack"]], case["p_round"])
        assert rc == 0 and ids.tolist() == case["want"]
        assert int(dg[0]) == oracle.digest([tuple(x) for x in case["want"]])
    bs = oracle.PDag(pack_lists(dag, 4))
    m, _ = bs.cone((4, 1), 0, True)
    got = [[r, s] for r in range(5) for s in range(1, 5) if (int(m[r][0]) >> (s - 1)) & 1]
    assert got == d["strong_reach_4_1"]


def test_figure1_allpairs_regression():
    g, dag = figure1()
    ld = oracle.LDag(arrays=flatten_lists(dag))
    bs = oracle.PDag(pack_lists(dag, 4))
    ids = [tuple(x) for x in g["allpairs_ids"]]
    for key, strong in (("strong", True), ("any", False)):
        want = g["allpairs"][key]
        for i, a in enumerate(ids):
            for j, b in enumerate(ids):
                assert ld.path(a, b, strong) == want[i][j]
                assert bs.path(a, b, strong) == want[i][j], (a, b, strong)


def test_literal_panics_like_go():
    g, dag = figure1()
    ld = oracle.LDag(arrays=flatten_lists(dag))
    assert ld.path((7, 1), (1, 1), True) == oracle.PANIC  # p.dag[7] index out of range
    assert ld.path((7, 1), (7, 1), True) == 1  # from == to returns first
    assert ld.leader(0)[0] == oracle.PANIC  # waveRound(0,1) = -3


def test_stack_lifo_pop_order():
    """stack_test.go:9-18 semantics through orderVertices: pops run top first."""
    g, dag = figure1()
    ld = oracle.LDag(arrays=flatten_lists(dag))
    rc, ids, cnt, _ = ld.order_vertices([(1, 1), (4, 1)], 4)
    assert rc == 0 and cnt.tolist() == [12, 1]
    assert ids[:12].tolist()[-1] == [4, 1] and ids[12:].tolist() == [[1, 1]]


def _same(a, b):
    assert a.rc == 0 and b.rc == 0
    for k in ("commit", "vcount", "push_off", "push_wave", "pop_count", "pop_digest", "pop_edges"):
        assert (getattr(a, k) == getattr(b, k)).all(), k
    assert a.commit_edges == b.commit_edges and a.deliver_edges == b.deliver_edges
    if a.ids is not None:
        assert (a.ids == b.ids).all()


@pytest.mark.parametrize("seed", range(60))
def test_literal_vs_bitset_random(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 12))
    R = int(rng.integers(4, 25))
    d = random_dag(rng, n, R, p_present=rng.uniform(0.5, 1), p_s=rng.uniform(0.1, 0.9), p_w=rng.uniform(0, 1),
                   max_depth=int(rng.integers(2, 30)))
    f = int(rng.integers(0, (n - 1) // 3 + 2))
    lit, bs = oracle.LDag(packed=d), oracle.PDag(d)
    for cm in (oracle.CHAIN_LITERAL, oracle.CHAIN_PERSISTENT):
        for dm in (oracle.DELIVER_REF, oracle.DELIVER_PAPER):
            _same(lit.replay(f, R // 4, cm, dm, ids_cap=1 << 16), bs.replay(f, R // 4, cm, dm, ids_cap=1 << 16))
    stack = [(int(rng.integers(0, R + 1)), int(rng.integers(1, n + 1))) for _ in range(3)]
    cur = int(rng.integers(0, R + 1))
    for mode in (oracle.DELIVER_REF, oracle.DELIVER_PAPER):
        a, b = lit.order_vertices(stack, cur, mode), bs.order_vertices(stack, cur, mode)
        assert a[0] == b[0] == 0
        assert a[1].tolist() == b[1].tolist() and a[2].tolist() == b[2].tolist() and a[3].tolist() == b[3].tolist()
    ids = [(r, s) for r in range(R + 1) for s in range(0, n + 1)]
    for strong in (0, 1):
        for a in ids[::3]:
            for b in ids[::2]:
                assert lit.path(a, b, strong) == bs.path(a, b, strong)


@pytest.mark.parametrize("seed", range(16))
def test_literal_vs_bitset_extra_edges(seed):
    """Edges below their round outside the row/column shape (strong
    edges skipping rounds, weak edges to r-1; weak edges of any depth) ride in the packed
    weak_tgt, bit 31 marking a strong one: the bitset restatement answers as the literal
    BFS does on the same [][]vertex (or_ldag_from_packed)."""
    from dag_rider_amd.gen import with_extra_edges

    rng = np.random.default_rng(900 + seed)
    n = int(rng.integers(1, 40))
    R = int(rng.integers(6, 32))
    base = random_dag(rng, n, R, p_present=rng.uniform(0.6, 1), p_s=rng.uniform(0.2, 0.9), p_w=rng.uniform(0, 0.6),
                      max_depth=int(rng.integers(2, 10)))
    extra = []
    for _ in range(int(rng.integers(1, 8))):
        r = int(rng.integers(2, R + 1))
        srcs = [int(x) for x in base.slot_src[base.slot_off[r]:base.slot_off[r + 1]] if x]
        if not srcs:
            continue
        strong = bool(rng.random() < 0.5)
        tr = int(rng.integers(0, r - 1)) if strong else int(rng.integers(0, r))
        extra.append((r, int(rng.choice(srcs)), tr, int(rng.integers(1, n + 1)), strong))
    d = with_extra_edges(base, tuple(extra)) if extra else base
    f = int(rng.integers(0, (n - 1) // 3 + 2))
    lit, bs = oracle.LDag(packed=d), oracle.PDag(d)
    for cm in (oracle.CHAIN_LITERAL, oracle.CHAIN_PERSISTENT):
        for dm in (oracle.DELIVER_REF, oracle.DELIVER_PAPER):
            _same(lit.replay(f, R // 4, cm, dm, ids_cap=1 << 16), bs.replay(f, R // 4, cm, dm, ids_cap=1 << 16))
    ids = [(r, s) for r in range(R + 1) for s in range(1, n + 1)]
    for strong in (0, 1):
        for a in ids[::23]:
            for b in ids[::11]:
                assert lit.path(a, b, strong) == bs.path(a, b, strong)


@pytest.mark.parametrize("seed", range(20))
def test_literal_vs_bitset_generator(seed):
    rng = np.random.default_rng(100 + seed)
    cfg = small_config(int(rng.integers(1, 20)), int(rng.integers(4, 33)), seed,
                       p_present=float(rng.uniform(0.5, 1)), p_late=float(rng.uniform(0, 0.5)),
                       p_w=float(rng.uniform(0, 1)), weak_depth=int(rng.integers(2, 8)),
                       p_la=float(rng.uniform(0, 0.5)))
    d = generate(cfg)
    lit, bs = oracle.LDag(packed=d), oracle.PDag(d)
    for cm in (oracle.CHAIN_LITERAL, oracle.CHAIN_PERSISTENT):
        _same(lit.replay(cfg.faulty, cfg.nwaves, cm, oracle.DELIVER_REF, ids_cap=1 << 16),
              bs.replay(cfg.faulty, cfg.nwaves, cm, oracle.DELIVER_REF, ids_cap=1 << 16))


@pytest.mark.parametrize("seed", range(6))
def test_literal_multithreaded_identical(seed):
    """or_lit_replay_mt (the CPU baseline on every core) == the single-thread literal replay."""
    rng = np.random.default_rng(300 + seed)
    d = random_dag(rng, int(rng.integers(3, 12)), int(rng.integers(8, 25)), p_s=0.5, p_w=0.3)
    f = (d.n - 1) // 3
    lit = oracle.LDag(packed=d)
    for cm in (oracle.CHAIN_LITERAL, oracle.CHAIN_PERSISTENT):
        for dm in (oracle.DELIVER_REF, oracle.DELIVER_PAPER):
            _same(lit.replay(f, (d.nrounds - 1) // 4, cm, dm, ids_cap=1 << 16),
                  lit.replay(f, (d.nrounds - 1) // 4, cm, dm, ids_cap=1 << 16, nthreads=4))


def test_generator_deterministic_and_thread_independent():
    cfg = CONFIGS["c2"]
    a, b = generate(cfg, nthreads=1), generate(cfg, nthreads=4)
    for k in ("slot_off", "slot_src", "strong", "weak_off", "weak_tgt"):
        assert (getattr(a, k) == getattr(b, k)).all(), k


def test_generator_contract():
    d = generate(CONFIGS["c2"])
    n, W, f = d.n, d.W, d.faulty
    for r in range(1, d.nrounds):
        srcs = d.slot_src[d.slot_off[r]:d.slot_off[r + 1]]
        assert len(set(srcs.tolist())) == len(srcs) >= 2 * f + 1
        for s in srcs[:8]:
            row = d.row(r, int(s))
            k = sum(bin(int(x)).count("1") for x in row)
            assert k >= 2 * f + 1
        g0, g1 = d.weak_off[r * n], d.weak_off[(r + 1) * n]
        assert all((int(t) >> 11) <= r - 2 for t in d.weak_tgt[g0:g1])


def test_golden_c2_replay():
    """C2 replay outputs (tests/golden/c2_replay.json) -- regression vectors of the
    cross-checked oracle; the GPU is compared against the same numbers."""
    with open(os.path.join(GOLDEN, "c2_replay.json")) as f:
        g = json.load(f)
    cfg = CONFIGS["c2"]
    d = generate(cfg)
    r = oracle.PDag(d).replay(cfg.faulty, cfg.nwaves, oracle.CHAIN_PERSISTENT, oracle.DELIVER_REF)
    assert r.commit.tolist() == g["commit"] and r.vcount.tolist() == g["vcount"]
    assert r.push_wave.tolist() == g["push_wave"]
    assert [str(x) for x in r.pop_count] == g["pop_count"] and [str(x) for x in r.pop_digest] == g["pop_digest"]
    assert str(r.deliver_edges) == g["deliver_edges"] and str(r.commit_edges) == g["commit_edges"]
    # the literal restatement agrees on the first waves
    k = g["literal_prefix_waves"]
    lit = oracle.LDag(packed=d, nrounds=4 * k + 1).replay(cfg.faulty, k, oracle.CHAIN_PERSISTENT,
                                                          oracle.DELIVER_REF)
    npop = int(lit.push_off[k])
    assert lit.pop_digest.tolist() == r.pop_digest[:npop].tolist()


def test_large_golden_pins_generator_and_oracle():
    """The committed C3/C4/C5 golden vectors: the generator reproduces the C5 DAGs (and the
    C3/C4 configs they were made from), and the oracle reproduces the first C5 replays in
    every recorded mode (the full C3/C4 replays take a minute each; the GPU tests compare them)."""
    from dag_rider_amd.gen import CONFIGS, c5_config, generate
    from dagutil import dag_fingerprint, load_large, replay_fingerprint

    g = load_large()
    for name in ("c3", "c4"):
        cfg = dict(CONFIGS[name].__dict__)
        assert cfg.pop("p_dup") == 0.0 and cfg.pop("extra") == ()  # (fields added after the vectors were written)
        assert g[name]["config"] == cfg
        assert len(g[name]["persistent_ref"]["pop_digest"]) == len(g[name]["persistent_ref"]["push_wave"])
    c5 = g["c5"]
    assert c5["count"] == 4096 and len(c5["persistent_ref"]) == 4096
    for i in range(6):
        cfg = c5_config(i)
        d = generate(cfg)
        assert dag_fingerprint(d) == c5["dag"][i]
        bs = oracle.PDag(d)
        for key, cm, dm in (("persistent_ref", oracle.CHAIN_PERSISTENT, oracle.DELIVER_REF),
                            ("literal_ref", oracle.CHAIN_LITERAL, oracle.DELIVER_REF),
                            ("persistent_paper", oracle.CHAIN_PERSISTENT, oracle.DELIVER_PAPER)):
            assert replay_fingerprint(bs.replay(cfg.faulty, cfg.nwaves, cm, dm, nthreads=1)) == c5[key][i]


def test_large_golden_pins():
    """The committed full-size vectors carry the literal-restatement prefix checks made
    when they were written (8 C3 waves, 4 C4 waves) and the literal-chain fingerprints."""
    from dagutil import load_large

    g = load_large()
    assert g["c3"]["literal_prefix_waves"] >= 8 and g["c4"]["literal_prefix_waves"] >= 4
    for name in ("c3", "c4"):
        lit = g[name]["literal_ref"]
        assert len(lit["fingerprint"]) == 32 and lit["n_push"] > len(g[name]["persistent_ref"]["push_wave"])


@pytest.mark.parametrize("seed", range(12))
def test_paper_delivery_is_first_cone_owner(seed):
    """The identity the device PAPER path rests on (replay_plan.hpp k_paper_*): the
    delivered set is downward closed, so the oracle's pruned sweep delivers exactly
    cone(p) minus the cones of the pops before p, in (round, slot) order -- every vertex
    to the first pop whose REF cone holds it."""
    rng = np.random.default_rng(4000 + seed)
    n, R = int(rng.integers(4, 24)), int(rng.integers(8, 48))
    depth = int(rng.integers(2, 12)) if seed % 3 else int(rng.integers(12, 30))
    d = random_dag(rng, n, R, p_present=rng.uniform(0.5, 1), p_s=rng.uniform(0.05, 0.9), p_w=rng.uniform(0, 1),
                   max_depth=depth)
    f = int(rng.integers(0, (n - 1) // 3 + 2))
    bs = oracle.PDag(d)
    for cm in (oracle.CHAIN_LITERAL, oracle.CHAIN_PERSISTENT):
        ref = bs.replay(f, R // 4, cm, oracle.DELIVER_REF, ids_cap=1 << 20)
        pap = bs.replay(f, R // 4, cm, oracle.DELIVER_PAPER, ids_cap=1 << 20)
        assert ref.rc == 0 and pap.rc == 0
        assert (ref.push_wave == pap.push_wave).all()
        ro = np.concatenate([[0], np.cumsum(ref.pop_count.astype(np.int64))])
        po = np.concatenate([[0], np.cumsum(pap.pop_count.astype(np.int64))])
        seen = set()
        for p in range(len(ref.pop_count)):
            cone = [tuple(v) for v in ref.ids[ro[p]:ro[p + 1]].tolist()]
            want = [v for v in cone if v not in seen]
            assert [tuple(v) for v in pap.ids[po[p]:po[p + 1]].tolist()] == want
            assert int(pap.pop_digest[p]) == oracle.digest(want)
            seen.update(cone)
