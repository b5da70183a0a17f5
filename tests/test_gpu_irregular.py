"""GPU parity on mirrors holding edges outside the round contract.

uponDeliver admits a vertex whose strong edges do not all target r-1, or whose weak
edges do not all lie below r-1 (it checks only the strong-edge count,
process/process.go:165), and path()'s BFS with a visited set answers for any graph
(:89-148), cycles included.  The mirror keeps such edges beside the packed rows and
answers every query with the general sweep (dag_rider_amd/csrc/general.hpp); checked
against the literal restatement (oracle/ref_literal.c), which runs the reference's BFS
on the same [][]vertex.  Nothing here is refused with DR_E_CONTRACT."""
import numpy as np
import pytest

import oracle
from dag_rider_amd import _lib as L
from dag_rider_amd.dag import Vertex, VertexID, flatten_lists
from dag_rider_amd.engine import Engine
from dagutil import random_dag, with_irregular_edges, with_repeated_ids

pytestmark = pytest.mark.gpu

MODES = [(cm, dm) for cm in (L.DR_CHAIN_LITERAL, L.DR_CHAIN_PERSISTENT) for dm in (L.DR_DELIVER_REF, L.DR_DELIVER_PAPER)]


def _same(got, want, ids=True):
    assert got.commit.tolist() == want.commit.tolist()
    assert got.vcount.tolist() == want.vcount.tolist()
    assert got.push_off.tolist() == want.push_off.tolist() and got.push_wave.tolist() == want.push_wave.tolist()
    assert got.pop_count.tolist() == want.pop_count.tolist()
    assert got.pop_digest.tolist() == want.pop_digest.tolist()
    assert got.pop_edges.tolist() == want.pop_edges.tolist()
    assert (got.commit_edges, got.deliver_edges) == (want.commit_edges, want.deliver_edges)
    if ids:
        assert got.ids.tolist() == want.ids.tolist()


@pytest.mark.parametrize("seed", range(10))
def test_irregular_edges_replay_path_order(gpu_device, seed):
    rng = np.random.default_rng(5100 + seed)
    n = int(rng.choice([4, 7, 12, 20, 70]))
    R = int(rng.integers(8, 21))
    base = random_dag(rng, n, R, p_present=rng.uniform(0.7, 1), p_s=rng.uniform(0.3, 0.9),
                      p_w=rng.uniform(0, 0.6), max_depth=int(rng.integers(2, 7))).to_lists()
    dag = with_irregular_edges(rng, base, p_irr=float(rng.uniform(0.05, 0.3)), up=bool(seed % 3))
    if seed % 4 == 1:
        dag = with_repeated_ids(rng, dag, p_dup=0.2)
    f = int(rng.integers(0, (n - 1) // 3 + 2))
    nw = R // 4
    ld = oracle.LDag(arrays=flatten_lists(dag))
    with Engine(n, f, R + 1, gpu_device) as e:
        cut = int(rng.integers(1, R + 1))
        e.append_lists(dag, 0, cut)
        e.append_lists(dag, cut, R + 1)
        for cm, dm in MODES:
            want = ld.replay(f, nw, cm, dm, ids_cap=1 << 16)
            assert want.rc == 0
            _same(e.replay(nw, cm, dm, ids_cap=1 << 16), want)
            _same(e.replay(nw, cm, dm), want, ids=False)
        for w in range(1, nw + 1):
            for dec in (0, max(0, w - 2)):
                rc, vc, stack = ld.wave_ready(f, w, dec)
                cm_, vc_, pushed = e.wave_ready(w, dec)
                assert vc_ == vc and cm_ == (rc == 1)
                if cm_:  # the pushed leaders, as waves
                    assert pushed == [(r - 1) // 4 + 1 for r, _ in stack]
        stack = [(int(rng.integers(0, R + 1)), int(rng.integers(1, n + 1))) for _ in range(3)]
        for cur in (R, int(rng.integers(0, R + 1))):
            for mode in (L.DR_DELIVER_REF, L.DR_DELIVER_PAPER):
                ids_, cnt_, dg_ = e.order_vertices(stack, cur, mode)
                rc, want_ids, wc, wd = ld.order_vertices(stack, cur, mode)
                assert rc == 0
                assert ids_.tolist() == want_ids.tolist()
                assert cnt_.tolist() == wc.tolist() and dg_.tolist() == wd.tolist()
        allids = sorted({(v.id.round, v.id.source) for r in dag for v in r if v.id != VertexID(0, 0)})
        samp = [allids[i] for i in rng.choice(len(allids), size=min(len(allids), 24), replace=False)]
        pairs = [(a, b) for a in samp for b in samp]
        for strong in (True, False):
            got = e.path_batch(pairs, strong)
            assert got.tolist() == [ld.path(a, b, strong) for a, b in pairs]
        # reach sets: the bits of every id of rounds bottom..from
        froms = samp[:5]
        bottoms = [int(rng.integers(0, fr[0] + 1)) for fr in froms]
        for strong in (True, False):
            sets = e.reach_sets(froms, bottoms, strong)
            for fr, bt, m in zip(froms, bottoms, sets):
                m = np.asarray(m).reshape(-1)
                for r in range(bt, fr[0] + 1):
                    for s in range(1, n + 1):
                        bit = int((int(m[(r - bt) * ((n + 63) // 64) + (s - 1) // 64]) >> ((s - 1) % 64)) & 1)
                        assert bit == (1 if (r, s) == fr else ld.path(fr, (r, s), strong)), (fr, r, s, strong)


def test_irregular_cycle_and_self_round(gpu_device):
    """A two-vertex cycle across rounds and a same-round edge: path() follows them both
    ways (the BFS's visited set ends the cycle), waveReady counts a voter that reaches
    the leader only through an upward edge."""
    g = [[Vertex(VertexID(0, s)) for s in (1, 2, 3, 4)]]
    for r in range(1, 9):
        g.append([Vertex(VertexID(r, s), b"", [VertexID(r - 1, t) for t in (1, 2, 3)], []) for s in (1, 2, 3, 4)])
    # (4,4) --strong--> (6,2) (upward), (6,2) --weak--> (4,4): a cycle; (5,3) --strong--> (5,1) (same round)
    g[4][3] = Vertex(VertexID(4, 4), b"", [VertexID(3, 1), VertexID(3, 2), VertexID(3, 3), VertexID(6, 2)], [])
    g[6][1] = Vertex(VertexID(6, 2), b"", [VertexID(5, 1), VertexID(5, 2), VertexID(5, 3)], [VertexID(4, 4)])
    g[5][2] = Vertex(VertexID(5, 3), b"", [VertexID(4, 1), VertexID(5, 1)], [])
    ld = oracle.LDag(arrays=flatten_lists(g))
    with Engine(4, 1, 9, gpu_device) as e:
        e.append_lists(g)
        ids = [(r, s) for r in range(9) for s in range(1, 5)]
        pairs = [(a, b) for a in ids for b in ids]
        for strong in (True, False):
            assert e.path_batch(pairs, strong).tolist() == [ld.path(a, b, strong) for a, b in pairs]
        for cm, dm in MODES:
            _same(e.replay(2, cm, dm, ids_cap=1 << 12), ld.replay(1, 2, cm, dm, ids_cap=1 << 12))


def test_irregular_vertex_through_buffer_admit(gpu_device):
    """The buffer loop (process.go:200-234): a vertex whose strong edges skip a round is
    admitted once its predecessors are present (dr_buffer_admit) and appended
    (dr_append_vertices); every query then answers as the oracle does."""
    rng = np.random.default_rng(17)
    n, R = 6, 12
    dag = random_dag(rng, n, R, p_present=1.0, p_s=0.8, p_w=0.3, ghosts=0.0).to_lists()
    with Engine(n, 1, R + 4, gpu_device) as e:
        e.append_lists(dag)
        v1 = Vertex(VertexID(R + 1, 1), b"", [VertexID(R, t) for t in (1, 2, 3)], [])
        e.append_vertices([v1])  # round R+1 opens (p.dag has a slot for it)
        v = Vertex(VertexID(R + 1, 2), b"", [VertexID(R, 1), VertexID(R, 2), VertexID(R - 2, 3)],
                   [VertexID(R, 4), VertexID(R - 5, 1)])
        preds = [(u.round, u.source) for u in v.strong_edges + v.weak_edges]
        admit = e.buffer_admit(R + 1, [((R + 1, 2), preds)])
        assert admit.tolist() == [1]
        e.append_vertices([v])  # not refused: the strong edge to R-2 and the weak one to R are kept
        dag2 = [list(r) for r in dag] + [[v1, v]]
        ld = oracle.LDag(arrays=flatten_lists(dag2))
        ids = [(r, s) for r in range(R + 2) for s in range(1, n + 1)]
        pairs = [((R + 1, 2), b) for b in ids]
        for strong in (True, False):
            assert e.path_batch(pairs, strong).tolist() == [ld.path(a, b, strong) for a, b in pairs]
        for mode in (L.DR_DELIVER_REF, L.DR_DELIVER_PAPER):
            ids_, cnt_, dg_ = e.order_vertices([(R + 1, 2), (R - 3, 1)], R + 1, mode)
            rc, want_ids, wc, wd = ld.order_vertices([(R + 1, 2), (R - 3, 1)], R + 1, mode)
            assert rc == 0 and ids_.tolist() == want_ids.tolist() and dg_.tolist() == wd.tolist()


@pytest.mark.parametrize("seed", range(4))
def test_upward_weak_edges_verified_memo(gpu_device, seed):
    """Weak edges to the same or a later round on quorum-shaped DAGs:
    dr_replay (REF, no ids) runs the memo replay on the regular graph and checks every
    such edge against every cone it computed (k_verify_up).  Edges inside the canonical
    regime change no cone -> the memo path answers (dr_last_replay_path 1); an edge from a
    low vertex up to a late one nobody reaches does -> the general sweep (2).  Both equal
    the general sweep (memo off, itself checked against the literal restatement above), and
    on the small instances (seeds 0, 1) the literal restatement's BFS, in both chain modes.
    (The literal REF replay runs one BFS per delivery candidate and pop: at n = 64 x 60
    rounds it takes minutes.)"""
    from dag_rider_amd.gen import generate, small_config, with_extra_edges

    rng = np.random.default_rng(5600 + seed)
    literal = seed < 2
    n = 16 if literal else int(rng.choice([64, 130]))
    cfg = small_config(n, 4 * (int(rng.integers(6, 9)) if literal else int(rng.integers(10, 25))), 5600 + seed,
                       p_present=1.0, p_late=0.05, p_w=0.4, weak_depth=4)
    d = generate(cfg)
    R = d.nrounds - 1
    present = lambda r: [int(s) for s in d.slot_src[d.slot_off[r]:d.slot_off[r + 1]] if s]  # noqa: E731
    benign = []
    for _ in range(3):  # same-round and one-round-up edges in the middle (full canonical rounds)
        r = int(rng.integers(R // 3, 2 * R // 3))
        a, b = rng.choice(present(r), size=2, replace=False)
        benign.append((r, int(a), r, int(b), False))
        up = present(r + 1)
        benign.append((r, int(a), r + 1, int(up[int(rng.integers(0, len(up)))]), False))
    # from a round-2 vertex up to the top round: the top round's vertices are reached by no
    # lower pop, so the cones holding the round-2 vertex grow
    bad = [(2, present(2)[0], R, present(R)[-1], False)]
    for extra, want_path in ((benign, 1), (benign + bad, 2)):
        dx = with_extra_edges(d, extra)
        ld = oracle.LDag(packed=dx) if literal else None
        with Engine(n, cfg.faulty, dx.nrounds, gpu_device) as e, \
                Engine(n, cfg.faulty, dx.nrounds, gpu_device) as eg:
            e.append_packed(dx)
            eg.append_packed(dx)
            eg.set_memo(False)  # every query on the general sweep
            assert e.exception_stats()["upward"] == len(extra)
            for cm in (L.DR_CHAIN_PERSISTENT, L.DR_CHAIN_LITERAL):
                got = e.replay(cfg.nwaves, cm, L.DR_DELIVER_REF)
                _same(got, eg.replay(cfg.nwaves, cm, L.DR_DELIVER_REF), ids=False)
                # (at n <= 130 a pop's cone is partial for several rounds below its top, so a
                # middle round's edge may well change one: the check may send even the "benign"
                # set to the general sweep -- test_upward_edge_memo_path_at_n1024 pins path 1)
                path = e.last_replay_path()
                assert path == want_path or path == 2, (cm, path)
                if ld is not None:
                    want = ld.replay(cfg.faulty, cfg.nwaves, cm, L.DR_DELIVER_REF)
                    assert want.rc == 0
                    _same(got, want, ids=False)


def test_upward_edge_memo_path_at_n1024(gpu_device):
    """A same-round and a next-round weak edge in the middle of a C4-shaped DAG (n = 1024,
    quorum strong edges): every cone that reaches their source is full there, so the verified
    memo replay keeps the memo path (dr_last_replay_path 1, the c4-up bench line's case) and
    equals the general sweep."""
    from dag_rider_amd.gen import generate, small_config, with_extra_edges

    cfg = small_config(1024, 48, 5700, p_present=1.0, p_late=0.02, p_w=0.5, weak_depth=4)
    d = generate(cfg)
    present = lambda r: [int(s) for s in d.slot_src[d.slot_off[r]:d.slot_off[r + 1]] if s]  # noqa: E731
    extra = [(26, present(26)[3], 26, present(26)[9], False), (26, present(26)[5], 27, present(27)[11], False)]
    dx = with_extra_edges(d, extra)
    with Engine(cfg.n, cfg.faulty, dx.nrounds, gpu_device) as e, \
            Engine(cfg.n, cfg.faulty, dx.nrounds, gpu_device) as eg:
        e.append_packed(dx)
        eg.append_packed(dx)
        eg.set_memo(False)
        assert e.exception_stats()["upward"] == 2
        for cm in (L.DR_CHAIN_PERSISTENT, L.DR_CHAIN_LITERAL):
            got = e.replay(cfg.nwaves, cm, L.DR_DELIVER_REF)
            assert e.last_replay_path() == 1
            _same(got, eg.replay(cfg.nwaves, cm, L.DR_DELIVER_REF), ids=False)
