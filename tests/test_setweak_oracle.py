"""setWeakEdges (process.go:298-310) oracle, pinned on the reference's Figure-1 DAG
(process_internal_test.go:86-283): a new round-4 vertex with (4,1)'s strong edges gets
exactly (4,1)'s weak edge (2,4) in paper mode, and every non-ghost slot of rounds 2..1
in literal mode (v.id is still {0,0})."""
import oracle
from dagutil import figure1


def test_figure1_pins():
    g, dag = figure1()
    plain = oracle.setweak.to_plain(dag)
    strong41 = [(3, 1), (3, 2), (3, 3)]
    paper = oracle.setweak.set_weak_edges(plain, 4, 1, strong41, oracle.setweak.PAPER)
    # ghost slots {0,0} (slot 0 of every round in the fixture) are never reached
    assert [x for x in paper if x != (0, 0)] == [(2, 4)]  # = (4,1).weakEdges in the fixture
    v41 = [v for v in dag[4] if (v.id.round, v.id.source) == (4, 1)][0]
    assert [(e.round, e.source) for e in v41.weak_edges] == [(2, 4)]
    # the first ghost becomes a weak edge; after that path(v, {0,0}) holds (weak edge)
    assert paper == [(0, 0), (2, 4)]
    lit = oracle.setweak.set_weak_edges(plain, 4, 1, strong41, oracle.setweak.LITERAL)
    assert lit == [(2, 1), (2, 2), (2, 3), (2, 4), (1, 1), (1, 2), (1, 3), (1, 4)]


def test_path_restatement_matches_testpath():
    """The Python path() used by the setWeakEdges oracle answers TestPath (T,T,T,T,F)."""
    g, dag = figure1()
    plain = oracle.setweak.to_plain(dag)
    for t in g["test_path"]:
        assert oracle.setweak.path(plain, tuple(t["from"]), tuple(t["to"]), t["strong"]) == t["want"]


def test_paper_mode_against_bitset_cones():
    """Paper mode = present vertices outside the cone of v's edges (weak ones included),
    cross-checked against the C bitset oracle's cones on a seeded DAG."""
    from dag_rider_amd.gen import generate, small_config

    d = generate(small_config(13, 14, 3))
    plain = oracle.setweak.to_plain(d.to_lists())
    bs = oracle.PDag(d)
    for rnd, src in [(14, 2), (10, 5), (6, 1)]:
        strong = [(rnd - 1, s) for s in range(1, 14) if (s * 7 + rnd) % 3]
        got = oracle.setweak.set_weak_edges(plain, rnd, src, strong, oracle.setweak.PAPER)
        # every added u is outside the union of the strong targets' cones
        for (r, s) in got:
            for t in strong:
                m, _ = bs.cone(t, r, False)
                assert not (int(m[0][(s - 1) // 64]) >> ((s - 1) % 64)) & 1
        assert got  # the seeded DAG has late vertices
