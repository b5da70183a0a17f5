"""DRW1 capture format (dag_rider_amd/wire.py): lossless round
trips of the Figure-1 DAG (ghost slots, process_internal_test.go:86-283) and of random
DAGs, the replay arrays equal flatten_lists() of the original, corrupt captures are
rejected, and (GPU) a decoded capture gives the same reach sets as the original."""
import numpy as np
import pytest

from dag_rider_amd import wire
from dag_rider_amd.dag import Vertex, VertexID, flatten_lists
from dagutil import figure1, random_dag


def _same(a, b):
    assert len(a) == len(b)
    for ra, rb in zip(a, b):
        assert [(v.id, v.block, v.strong_edges, v.weak_edges) for v in ra] == \
               [(v.id, v.block, v.strong_edges, v.weak_edges) for v in rb]


def test_figure1_round_trip():
    _, dag = figure1()
    dag[2][1].block = b"tx-batch"
    buf = wire.encode(dag)
    _same(wire.decode(buf), dag)
    for x, y in zip(wire.arrays(buf), flatten_lists(dag)):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_round_trip(seed):
    rng = np.random.default_rng(700 + seed)
    dag = random_dag(rng, 20, 12, p_w=0.2).to_lists()
    _same(wire.decode(wire.encode(dag)), dag)


def test_empty_and_corrupt():
    assert wire.decode(wire.encode([])) == []
    assert wire.decode(wire.encode([[], []])) == [[], []]
    one = [[Vertex(VertexID(0, 1))]]
    buf = wire.encode(one)
    _same(wire.decode(buf), one)
    with pytest.raises(ValueError):
        wire.decode(b"XXXX" + buf[4:])
    with pytest.raises(ValueError):
        wire.decode(buf + b"\0")


@pytest.mark.gpu
def test_gpu_replay_from_capture(gpu_device):
    from dag_rider_amd.engine import Engine

    rng = np.random.default_rng(777)
    dag = random_dag(rng, 30, 10).to_lists()
    back = wire.decode(wire.encode(dag))
    qs = [((r, s), (b, t)) for r in range(2, 10) for s in (1, 7, 30) for b, t in ((0, 1), (r - 2, 5))]
    res = []
    for d in (dag, back):
        with Engine(30, 9, 12, gpu_device) as e:
            e.append_lists(d)
            res.append([e.path_batch(qs, strong).tolist() for strong in (False, True)])
    assert res[0] == res[1]
