"""Repeated ids on the CPU oracle (literal restatement, oracle/ref_literal.c): the
reference appends whatever uponDeliver / the buffer loop hand it (process.go:158-169,
:229), so an id can repeat in a round.  path() follows the id's LAST slot (:112-116);
vCount counts every slot (:332); REF delivery delivers every slot (:418-429); PAPER
(Alg. 3 line 54) skips an id already delivered.  The GPU side: tests/test_gpu_dups.py."""
import numpy as np

import oracle
from dag_rider_amd.dag import Vertex, VertexID, flatten_lists
from dagutil import figure1, random_dag, with_repeated_ids


def test_last_match_lookup_and_slot_counts():
    g, dag = figure1()
    d2 = [list(r) for r in dag]
    # (3,2) re-delivered with a single strong edge: path() now sees only that one
    d2[3].append(Vertex(VertexID(3, 2), b"", [VertexID(2, 1)], []))
    lo, ld = oracle.LDag(arrays=flatten_lists(dag)), oracle.LDag(arrays=flatten_lists(d2))
    assert lo.path((3, 2), (2, 2), True) == 1 and ld.path((3, 2), (2, 2), True) == 0
    assert ld.path((3, 2), (2, 1), True) == 1
    # a round-4 slot pair votes twice
    d3 = [list(r) for r in dag]
    d3[4].append(Vertex(VertexID(4, 1), b"", [VertexID(3, 1), VertexID(3, 2), VertexID(3, 3)], [VertexID(2, 4)]))
    rc0, vc0, _ = oracle.LDag(arrays=flatten_lists(dag)).wave_ready(g["faulty"], 1, 0)
    rc1, vc1, _ = oracle.LDag(arrays=flatten_lists(d3)).wave_ready(g["faulty"], 1, 0)
    assert rc0 >= 0 and rc1 >= 0 and vc1 == vc0 + 1


def test_ref_delivers_every_slot_paper_once():
    rng = np.random.default_rng(5)
    base = random_dag(rng, 6, 12, p_present=1.0, p_s=0.8, p_w=0.3, ghosts=0.0).to_lists()
    dag = with_repeated_ids(rng, base, p_dup=0.4)
    ld = oracle.LDag(arrays=flatten_lists(dag))
    stack = [(9, 1)]
    _, ids_ref, cr, _ = ld.order_vertices(stack, 11, oracle.DELIVER_REF)
    _, ids_pap, cp, _ = ld.order_vertices(stack, 11, oracle.DELIVER_PAPER)
    ref = [tuple(x) for x in ids_ref.tolist()]
    pap = [tuple(x) for x in ids_pap.tolist()]
    assert len(set(ref)) < len(ref)          # repeated ids delivered once per slot
    assert len(set(pap)) == len(pap)         # PAPER: once per id
    assert sorted(set(ref)) == sorted(pap)   # the same ids
    # REF order: rounds ascending, slots in insertion order
    assert [r for r, _ in ref] == sorted(r for r, _ in ref)


def test_bitset_oracle_agrees_with_literal_on_repeated_ids():
    """The bitset restatement (oracle/ref_bitset.c: one packed row per id, the last
    slot's) == the literal one (every slot with its own edges, last-match lookup) on
    DAGs with repeated ids: every replay output in all four modes, and orderVertices."""
    from dag_rider_amd.dag import pack_lists

    for seed in range(12):
        rng = np.random.default_rng(6600 + seed)
        n = int(rng.choice([3, 5, 8, 20, 70]))
        R = int(rng.integers(8, 21))
        base = random_dag(rng, n, R, p_present=rng.uniform(0.6, 1), p_s=rng.uniform(0.2, 0.9),
                          p_w=rng.uniform(0, 0.8), max_depth=int(rng.integers(2, 8))).to_lists()
        dag = with_repeated_ids(rng, base, p_dup=float(rng.uniform(0.1, 0.5)))
        f = int(rng.integers(0, (n - 1) // 3 + 2))
        nw = R // 4
        ld, bs = oracle.LDag(arrays=flatten_lists(dag)), oracle.PDag(pack_lists(dag, n))
        for cm in (oracle.CHAIN_LITERAL, oracle.CHAIN_PERSISTENT):
            for dm in (oracle.DELIVER_REF, oracle.DELIVER_PAPER):
                a = ld.replay(f, nw, cm, dm, ids_cap=1 << 16)
                b = bs.replay(f, nw, cm, dm, ids_cap=1 << 16)
                assert a.rc == 0 and b.rc == 0
                for k in ("commit", "vcount", "push_off", "push_wave", "pop_count", "pop_digest", "pop_edges", "ids"):
                    assert getattr(a, k).tolist() == getattr(b, k).tolist(), (seed, cm, dm, k)
                # (chain edges: the literal restatement does not count them; the GPU tests pin them on the bitset one)
                assert (a.commit_edges, a.deliver_edges) == (b.commit_edges, b.deliver_edges), (seed, cm, dm)
        stack = [(int(rng.integers(0, R + 1)), int(rng.integers(1, n + 1))) for _ in range(3)]
        cur = int(rng.integers(0, R + 1))
        for mode in (oracle.DELIVER_REF, oracle.DELIVER_PAPER):
            ra, ia, ca, da = ld.order_vertices(stack, cur, mode)
            rb, ib, cb, db = bs.order_vertices(stack, cur, mode)
            assert ra == rb == 0 and ia.tolist() == ib.tolist() and ca.tolist() == cb.tolist()
            assert da.tolist() == db.tolist()
