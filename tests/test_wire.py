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


def _mangle(buf: bytes, which: int, fn) -> bytes:
    """Apply fn to array `which` (0..5 in flatten_lists order) of a capture, in place."""
    import struct

    pos = 12
    b = bytearray(buf)
    for i in range(6):
        (k,) = struct.unpack_from("<Q", b, pos)
        pos += 8
        if i == which:
            a = np.frombuffer(b, dtype=np.uint32 if i in (0, 2, 4) else np.int32, count=k, offset=pos).copy()
            fn(a)
            b[pos:pos + 4 * k] = a.tobytes()
        pos += 4 * k
    return bytes(b)


@pytest.mark.parametrize("which,fn", [
    (0, lambda a: a.__setitem__(-1, a[-1] + 1)),      # slot_off does not end at nslots
    (0, lambda a: a.__setitem__(1, a[2] + 5)),        # slot_off decreasing
    (2, lambda a: a.__setitem__(0, 1)),               # strong_off not 0-based
    (2, lambda a: a.__setitem__(3, a[-1] + 100)),     # strong_off past strong_ids
    (4, lambda a: a.__setitem__(-1, a[-1] + 2)),      # weak_off past weak_ids
    (4, lambda a: a.__setitem__(2, 2**31)),           # weak_off jumps
])
def test_corrupt_offsets_rejected(which, fn):
    """Offsets that dr_append_rounds_lists would trust as raw pointers are checked."""
    rng = np.random.default_rng(5)
    dag = random_dag(rng, 6, 6, p_w=0.5).to_lists()
    buf = wire.encode(dag)
    with pytest.raises(ValueError):
        wire.arrays(_mangle(buf, which, fn))
    for cut in (5, 13, len(buf) // 2, len(buf) - 1):  # truncation anywhere
        with pytest.raises(ValueError):
            wire.decode(buf[:cut])


def test_c_reader_agrees():
    """The C reader (dr_wire_check, include/dagrider_wire.h: host-only) accepts what
    wire.py writes, reports the same counts and blocks, and rejects what wire.py rejects."""
    import ctypes as C

    from dag_rider_amd import _lib as L

    lib = L.lib()
    rng = np.random.default_rng(9)
    dag = random_dag(rng, 9, 7, p_w=0.4).to_lists()
    dag[3][0].block = b"payload-3-0"
    buf = wire.encode(dag)
    nr, ns = L.i32(), L.i32()
    assert lib.dr_wire_check(buf, len(buf), C.byref(nr), C.byref(ns)) == 0
    assert (nr.value, ns.value) == (len(dag), sum(len(r) for r in dag))
    data, n = C.c_void_p(), C.c_size_t()
    k = sum(len(r) for r in dag[:3])
    assert lib.dr_wire_block(buf, len(buf), k, C.byref(data), C.byref(n)) == 0
    assert C.string_at(data, n.value) == b"payload-3-0"
    bad = [buf[:-1], buf + b"\0", b"XXXX" + buf[4:], _mangle(buf, 2, lambda a: a.__setitem__(0, 1)),
           _mangle(buf, 4, lambda a: a.__setitem__(-1, a[-1] + 2)), _mangle(buf, 0, lambda a: a.__setitem__(1, 10**6))]
    for b in bad:
        assert lib.dr_wire_check(b, len(b), None, None) == L.DR_E_INVAL
    for cut in range(0, len(buf), max(1, len(buf) // 97)):
        assert lib.dr_wire_check(buf[:cut], cut, None, None) == L.DR_E_INVAL


@pytest.mark.gpu
def test_gpu_c_reader_replay(gpu_device):
    """A capture replayed through the C reader == the original through dr_append_rounds_lists."""
    from dag_rider_amd.engine import Engine

    rng = np.random.default_rng(778)
    dag = random_dag(rng, 30, 10).to_lists()
    buf = wire.encode(dag)
    qs = [((r, s), (b, t)) for r in range(2, 10) for s in (1, 7, 30) for b, t in ((0, 1), (r - 2, 5))]
    with Engine(30, 9, 12, gpu_device) as a, Engine(30, 9, 12, gpu_device) as b:
        a.append_lists(dag)
        b.append_capture(buf)
        assert b.num_rounds == len(dag)
        for strong in (False, True):
            assert a.path_batch(qs, strong).tolist() == b.path_batch(qs, strong).tolist()
        ra, rb = a.replay(2), b.replay(2)
        assert (ra.pop_digest == rb.pop_digest).all() and (ra.commit == rb.commit).all()


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


def test_go_fixture_current():
    """tests/golden/figure1.drw1 (read by go/dagridergpu's tests, which re-encode it byte
    for byte) is what wire.py writes for the fixture DAG."""
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_wire_fixture import fixture_dag

    with open(os.path.join(os.path.dirname(__file__), "golden", "figure1.drw1"), "rb") as f:
        assert f.read() == wire.encode(fixture_dag())
