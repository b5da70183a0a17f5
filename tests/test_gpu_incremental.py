"""Vertex-granular append (dr_append_vertices): the device mirror follows p.dag as
the buffer loop grows it, one vertex at a time and into old rounds
(p.dag[v.id.round] = append(...), process.go:229).

Vertices of seeded random DAGs arrive in a random causal order (every vertex after
its predecessors, the order the buffer loop admits them in), so late vertices land
in rounds far below the top.  After every few arrivals the HIP path answers path(),
waveReady() and orderVertices() on the DAG as it stands and must match the literal
oracle on the same list DAG, with round summaries kept incrementally (memo) and
without them.  The mirror is all-or-nothing: a rejected append leaves it unchanged.
"""
import numpy as np
import pytest

import oracle
from dag_rider_amd import _lib as L
from dag_rider_amd.dag import Vertex, VertexID, flatten_lists
from dag_rider_amd.engine import Engine
from dagutil import random_dag


def causal_order(dag, rng):
    """(round, slot) of every vertex in a random order in which each vertex follows
    all of its predecessors that exist in the DAG (dangling targets never arrive)."""
    ids = {}
    for r, rnd in enumerate(dag):
        for i, v in enumerate(rnd):
            if v.id != VertexID(0, 0):
                ids[(v.id.round, v.id.source)] = (r, i)
    need = {}
    users = {}
    for r, rnd in enumerate(dag):
        for i, v in enumerate(rnd):
            deps = {(e.round, e.source) for e in v.strong_edges + v.weak_edges} & ids.keys()
            need[(r, i)] = len(deps)
            for d in deps:
                users.setdefault(ids[d], []).append((r, i))
    ready = [k for k, c in need.items() if c == 0]
    out = []
    while ready:
        k = ready.pop(int(rng.integers(0, len(ready))))
        out.append(k)
        for u in users.get(k, []):
            need[u] -= 1
            if need[u] == 0:
                ready.append(u)
    assert len(out) == len(need)
    return out


def _check(engines, cur, n, faulty, rng, nq=40):
    """Every engine against the literal oracle on the current list DAG."""
    ld = oracle.LDag(arrays=flatten_lists(cur))
    nr = len(cur)
    present = [(v.id.round, v.id.source) for rnd in cur for v in rnd if v.id != VertexID(0, 0)]
    if not present:
        return
    pairs = []
    for _ in range(nq):
        a = present[int(rng.integers(0, len(present)))]
        b = (int(rng.integers(0, a[0] + 1)), int(rng.integers(1, n + 1)))
        pairs.append((a, b))
    for strong in (True, False):
        want = [ld.path(a, b, strong) for a, b in pairs]
        for e in engines:
            assert e.path_batch(pairs, strong).tolist() == want, strong
    for w in range(1, (nr - 1) // 4 + 1):
        for decided in (0, max(0, w - 2)):
            rc, vc, st = ld.wave_ready(faulty, w, decided)
            for e in engines:
                if rc == oracle.PANIC:
                    with pytest.raises(L.DrError):
                        e.wave_ready(w, decided)
                    continue
                commit, vcount, pushed = e.wave_ready(w, decided)
                assert vcount == vc
                assert commit == (len(st) > 0)
                assert [(4 * (x - 1) + 1, 1) for x in pushed] == [tuple(s) for s in st]
    top = nr - 1
    leaders = [(r, s) for (r, s) in present if r >= 1]
    stack = [leaders[int(rng.integers(0, len(leaders)))] for _ in range(3)] if leaders else []
    for mode in (L.DR_DELIVER_REF, L.DR_DELIVER_PAPER):
        rc, want, wc, wd = ld.order_vertices(stack, top, mode)
        assert rc == 0
        for e in engines:
            ids, cnt, dg = e.order_vertices(stack, top, mode)
            assert ids.tolist() == want.tolist()
            assert cnt.tolist() == wc.tolist() and dg.tolist() == wd.tolist()
            # counts + digests only: REF mode takes the device-planned path on fresh summaries
            _, cnt, dg = e.order_vertices(stack, top, mode, cap=0)
            assert cnt.tolist() == wc.tolist() and dg.tolist() == wd.tolist()


@pytest.mark.gpu
@pytest.mark.parametrize("seed,n,R,step", [(1, 4, 13, 1), (2, 8, 17, 3), (3, 40, 13, 9), (4, 70, 9, 25)])
def test_gpu_append_vertices_causal(gpu_device, seed, n, R, step):
    rng = np.random.default_rng(9000 + seed)
    full = random_dag(rng, n, R, p_present=0.85, p_s=0.6, p_w=0.3, max_depth=6, ghosts=0.0).to_lists()
    faulty = (n - 1) // 3
    order = causal_order(full, rng)
    engines = [Engine(n, faulty, R + 2, gpu_device), Engine(n, faulty, R + 2, gpu_device)]
    engines[1].set_memo(False)
    cur = []
    try:
        for i0 in range(0, len(order), step):
            batch = order[i0:i0 + step]
            verts = []
            for (r, i) in batch:
                v = full[r][i]
                while len(cur) <= r:
                    cur.append([])
                cur[r].append(v)
                verts.append(v)
            # p.dag grows as needed: empty rounds below the batch's top round first
            # (dr_append_rounds_lists with no slots), the top one by its first vertex
            for e in engines:
                if e.num_rounds < len(cur) - 1:
                    e.append_lists([[]] * (len(cur) - 1), e.num_rounds, len(cur) - 1)
                e.append_vertices(verts)
            assert all(e.num_rounds == len(cur) for e in engines)
            _check(engines, cur, n, faulty, rng)
    finally:
        for e in engines:
            e.close()


@pytest.mark.gpu
def test_gpu_append_vertices_all_or_nothing(gpu_device):
    rng = np.random.default_rng(77)
    full = random_dag(rng, 6, 8, p_present=1.0, p_s=0.7, p_w=0.2, ghosts=0.0).to_lists()
    with Engine(6, 1, 12, gpu_device) as e:
        e.append_lists(full[:6])
        good = full[6][:2]
        before = e.path_batch([((5, s), (4, t)) for s in range(1, 7) for t in range(1, 7)], False).tolist()
        # (a strong edge not to r-1 or a weak edge not below r-1 is accepted: App. A Q8,
        # tests/test_gpu_irregular.py)
        bad_cases = [
            good + [Vertex(VertexID(6, 9), b"", [], [])],                      # source > n
            good + [Vertex(VertexID(6, 3), b"", [VertexID(12, 1)], [])],      # target round >= max_rounds
            good + [Vertex(VertexID(6, 3), b"", [], [VertexID(5, 7)])],       # target source > n
            good + [Vertex(VertexID(0, 0), b"", [VertexID(4, 1)], [])],       # ghost with edges
        ]
        for verts in bad_cases:
            with pytest.raises(L.DrError) as ei:
                e.append_vertices(verts)
            assert ei.value.code == L.DR_E_CONTRACT
            assert e.num_rounds == 6
        with pytest.raises(L.DrError) as ei:  # p.dag[8] with 7 rounds after opening 6: Go index out of range
            e.append_vertices(good + [Vertex(VertexID(8, 1), b"", [], [])])
        assert ei.value.code == L.DR_E_INVAL and e.num_rounds == 6
        after = e.path_batch([((5, s), (4, t)) for s in range(1, 7) for t in range(1, 7)], False).tolist()
        assert after == before
        e.append_vertices(full[6] + full[7])  # opens rounds 6 and 7
        assert e.num_rounds == 8
        ld = oracle.LDag(arrays=flatten_lists(full[:8]))
        pairs = [((7, s), (r, t)) for s in range(1, 7) for r in range(0, 7) for t in range(1, 7)]
        assert e.path_batch(pairs, False).tolist() == [ld.path(a, b, False) for a, b in pairs]


@pytest.mark.gpu
def test_gpu_append_vertices_ghost_and_round0(gpu_device):
    """Ghost slots {0,0} go to any p.dag[r] (slot_round); round 0 may repeat ids (genesis)."""
    with Engine(4, 1, 8, gpu_device) as e:
        e.append_vertices([Vertex(VertexID(0, 1)), Vertex(VertexID(0, 1)), Vertex(VertexID(0, 2)),
                           Vertex(VertexID(0, 3))])
        e.append_vertices([Vertex(VertexID(1, s), b"", [VertexID(0, 1), VertexID(0, 2), VertexID(0, 3)])
                           for s in (2, 1)] + [Vertex()], rounds=[1, 1, 1])
        e.append_vertices([Vertex(VertexID(2, 1), b"", [VertexID(1, 1), VertexID(1, 2)])])
        cur = [[Vertex(VertexID(0, 1)), Vertex(VertexID(0, 1)), Vertex(VertexID(0, 2)), Vertex(VertexID(0, 3))],
               [Vertex(VertexID(1, 2), b"", [VertexID(0, 1), VertexID(0, 2), VertexID(0, 3)]),
                Vertex(VertexID(1, 1), b"", [VertexID(0, 1), VertexID(0, 2), VertexID(0, 3)]), Vertex()],
               [Vertex(VertexID(2, 1), b"", [VertexID(1, 1), VertexID(1, 2)])]]
        ld = oracle.LDag(arrays=flatten_lists(cur))
        for stack in ([(2, 1)], [(1, 1), (2, 1)]):
            for mode in (L.DR_DELIVER_REF, L.DR_DELIVER_PAPER):
                ids, cnt, dg = e.order_vertices(stack, 2, mode)
                rc, want, wc, wd = ld.order_vertices(stack, 2, mode)
                assert ids.tolist() == want.tolist() and dg.tolist() == wd.tolist()


@pytest.mark.gpu
@pytest.mark.parametrize("cfg_name", ["c2", "c4-small"])
def test_gpu_wave_loop_matches_replay(gpu_device, cfg_name):
    """The drop-in loop (append 4 rounds -> waveReady -> orderVertices, counts and
    digests) equals one full dr_replay on every wave: the canonical cone is
    rebuilt incrementally between calls (only rounds from the lowest changed one
    are re-emitted) and pops are planned on the device."""
    from dag_rider_amd.gen import CONFIGS, GenConfig, generate

    cfg = CONFIGS["c2"] if cfg_name == "c2" else GenConfig("c4-small", 1024, 240, 4, 1.0, 0.02, 0.5, 4, 0.0)
    d = generate(cfg, nthreads=8)
    nw = (d.nrounds - 1) // 4
    with Engine(cfg.n, cfg.faulty, d.nrounds, gpu_device) as e:
        e.append_packed(d, 0, 1)
        decided, commit, pushes, pc, pdg = 0, [], [], [], []
        for w in range(1, nw + 1):
            e.append_packed(d, 4 * w - 3, 4 * w + 1)
            cm, vc, pushed = e.wave_ready(w, decided)
            commit.append(cm)
            if cm:
                pushes += pushed
                _, cnt, dg = e.order_vertices([(4 * (x - 1) + 1, e.wave_leader(x)) for x in pushed], 4 * w,
                                              L.DR_DELIVER_REF, cap=0)
                pc += cnt.tolist()
                pdg += dg.tolist()
                decided = w
        ref = e.replay(nw, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF)
    assert commit == ref.commit.astype(bool).tolist()
    assert pushes == ref.push_wave.tolist()
    assert pc == ref.pop_count.tolist() and pdg == ref.pop_digest.tolist()


@pytest.mark.gpu
def test_staged_packed_append_then_queries(gpu_device):
    """A per-round packed append returns before its copies run: the next call
    on the context -- path, waveReady, orderVertices, or destroy -- runs behind them on the
    same stream.  Appends of 4 rounds at a time, each followed at once by queries against
    the literal oracle on the prefix; the last append is followed by destroy alone."""
    from dag_rider_amd.gen import generate, small_config

    cfg = small_config(100, 48, 77, p_present=0.95, p_late=0.2, p_w=0.4, weak_depth=6)
    d = generate(cfg)
    rng = np.random.default_rng(13)
    with Engine(cfg.n, cfg.faulty, d.nrounds, gpu_device) as e:
        e.append_packed(d, 0, 1)
        r1 = 1
        while r1 + 4 <= d.nrounds - 4:
            e.append_packed(d, r1, r1 + 4)
            r1 += 4
            ld = oracle.LDag(packed=d, nrounds=r1)
            pairs = []
            for _ in range(16):
                ra = int(rng.integers(1, r1))
                srcs = d.slot_src[d.slot_off[ra]:d.slot_off[ra + 1]]
                srcs = srcs[srcs != 0]
                if len(srcs):
                    a = (ra, int(srcs[int(rng.integers(0, len(srcs)))]))
                    pairs.append((a, (int(rng.integers(0, ra + 1)), int(rng.integers(1, cfg.n + 1)))))
            assert e.path_batch(pairs, False).tolist() == [ld.path(a, b, False) for a, b in pairs]
            w = (r1 - 1) // 4
            if w >= 1:
                rc, vc, st = ld.wave_ready(cfg.faulty, w, 0)
                assert rc in (0, 1)  # (1: committed; a panic is negative)
                commit, vcount, pushed = e.wave_ready(w, 0)
                assert vcount == vc and commit == (rc == 1)
                if commit:
                    assert [(4 * (x - 1) + 1, e.wave_leader(x)) for x in pushed] == list(st)
        e.append_packed(d, r1, d.nrounds)  # then destroy with the copies possibly in flight


@pytest.mark.gpu
def test_gpu_wave_loop_call_overlap_interleaved(gpu_device):
    """DR_OPT_CALL_OVERLAP: after a REF orderVertices, waveReady launches the canonical cone of
    the new top once a commit is known (1) or on a second stream while the commit rule runs (2).  The loop below skips
    orderVertices on some commits, answers others in PAPER mode (with ids) or REF mode (ids,
    or counts + digests on the device-planned path), and asks path() between calls; every
    answer equals a context with the overlap off doing the same calls."""
    from dag_rider_amd.gen import GenConfig, generate

    cfg = GenConfig("c4-small", 1024, 160, 4, 1.0, 0.02, 0.5, 4, 0.0)
    d = generate(cfg, nthreads=8)
    nw = (d.nrounds - 1) // 4
    rng = np.random.default_rng(31)
    engines = [Engine(cfg.n, cfg.faulty, d.nrounds, gpu_device) for _ in range(3)]
    for e, ov in zip(engines, (1, 2, 0)):
        e.set_call_overlap(ov)
    try:
        for e in engines:
            e.append_packed(d, 0, 1)
        decided = 0
        for w in range(1, nw + 1):
            out = []
            for e in engines:
                e.append_packed(d, 4 * w - 3, 4 * w + 1)
                out.append(e.wave_ready(w, decided))
            assert out[0] == out[1] == out[2]
            cm, _, pushed = out[0]
            pairs = [((4 * w, int(rng.integers(1, cfg.n + 1))), (int(rng.integers(0, 4 * w)),
                                                                  int(rng.integers(1, cfg.n + 1))))
                     for _ in range(8)]
            want = engines[2].path_batch(pairs, False).tolist()
            assert all(e.path_batch(pairs, False).tolist() == want for e in engines[:2])
            if not cm:
                continue
            stack = [(4 * (x - 1) + 1, engines[0].wave_leader(x)) for x in pushed]
            k = w % 4
            if k == 1:
                continue  # committed, not delivered: the next waveReady forks again
            mode = L.DR_DELIVER_PAPER if k == 2 else L.DR_DELIVER_REF
            cap = 0 if k == 3 else None
            res = [e.order_vertices(stack, 4 * w, mode, cap=cap) if cap is not None
                   else e.order_vertices(stack, 4 * w, mode) for e in engines]
            for r in res[:2]:
                for a, b in zip(r, res[2]):
                    assert np.asarray(a).tolist() == np.asarray(b).tolist()
            decided = w
    finally:
        for e in engines:
            e.close()
