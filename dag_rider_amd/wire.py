"""Binary capture/replay format for a DAG.

The reference ships vertices between processes as Go values over channels
(``bcastMsg`` ``process/transport.go:13-17`` carrying ``vertex``
``process/process.go:26-31``) and has no on-disk form.  This format stores a
``[][]vertex`` as the flat arrays ``dr_append_rounds_lists`` consumes, so a
captured run is replayed into the device mirror straight from the file
(``arrays()`` returns zero-copy views), plus each vertex's ``block`` bytes.

Layout (little-endian):
  magic b"DRW1", u32 nrounds, u32 nslots
  six arrays in flatten_lists() order -- slot_off u32[nrounds+1], slot_id i32[2*nslots],
  strong_off u32[nslots+1], strong_ids i32[2*E_s], weak_off u32[nslots+1],
  weak_ids i32[2*E_w] -- each preceded by its u64 element count
  block_off u64[nslots+1], block bytes
"""
from __future__ import annotations

import struct
from typing import Sequence, Tuple

import numpy as np

from .dag import Dag, Vertex, VertexID, flatten_lists

MAGIC = b"DRW1"
_DT = (np.uint32, np.int32, np.uint32, np.int32, np.uint32, np.int32)


def encode(dag: Sequence[Sequence[Vertex]]) -> bytes:
    arrs = list(flatten_lists(dag))
    nslots = int(arrs[0][-1])
    # flatten_lists pads empty id arrays with one zero; store the true lengths
    arrs[1] = arrs[1][:2 * nslots]
    arrs[3] = arrs[3][:2 * int(arrs[2][-1])]
    arrs[5] = arrs[5][:2 * int(arrs[4][-1])]
    out = [MAGIC, struct.pack("<II", len(dag), nslots)]
    for a, dt in zip(arrs, _DT):
        a = np.ascontiguousarray(a, dtype=dt)
        out += [struct.pack("<Q", a.size), a.tobytes()]
    blocks = [v.block for rnd in dag for v in rnd]
    boff = np.zeros(nslots + 1, np.uint64)
    if blocks:
        boff[1:] = np.cumsum([len(b) for b in blocks])
    out += [boff.tobytes(), b"".join(blocks)]
    return b"".join(out)


def _offsets(name: str, off: np.ndarray, n: int, total: int):
    """An offset array: n+1 entries, starting at 0, non-decreasing, ending at total."""
    if off.size != n + 1:
        raise ValueError(f"corrupt DRW1 capture: {name} has {off.size} entries, want {n + 1}")
    if int(off[0]) != 0 or int(off[-1]) != total or (off.size > 1 and (np.diff(off.astype(np.int64)) < 0).any()):
        raise ValueError(f"corrupt DRW1 capture: {name} is not a 0-based non-decreasing prefix ending at {total}")


def _parse(buf: bytes):
    """Header and arrays of a capture, every size and offset checked: arrays() feeds
    dr_append_rounds_lists, which trusts them as raw pointers and lengths."""
    if len(buf) < 12 or buf[:4] != MAGIC:
        raise ValueError("not a DRW1 DAG capture")
    nrounds, nslots = struct.unpack_from("<II", buf, 4)
    pos = 12
    arrs = []
    for dt in _DT:
        if pos + 8 > len(buf):
            raise ValueError("corrupt DRW1 capture: truncated array header")
        (k,) = struct.unpack_from("<Q", buf, pos)
        pos += 8
        if k > (len(buf) - pos) // 4:
            raise ValueError("corrupt DRW1 capture: array runs past the end")
        a = np.frombuffer(buf, dtype=dt, count=k, offset=pos)
        pos += 4 * k
        arrs.append(a)
    so, sid, sto, sti, wo, wi = arrs
    if sid.size != 2 * nslots:
        raise ValueError("corrupt DRW1 capture: round/slot counts disagree")
    _offsets("slot_off", so, nrounds, nslots)
    if sti.size % 2 or wi.size % 2:
        raise ValueError("corrupt DRW1 capture: odd id array")
    _offsets("strong_off", sto, nslots, sti.size // 2)
    _offsets("weak_off", wo, nslots, wi.size // 2)
    if pos + 8 * (nslots + 1) > len(buf):
        raise ValueError("corrupt DRW1 capture: block offsets truncated")
    boff = np.frombuffer(buf, dtype=np.uint64, count=nslots + 1, offset=pos)
    pos += 8 * (nslots + 1)
    if int(boff[0]) != 0 or (boff.size > 1 and (boff[1:] < boff[:-1]).any()):
        raise ValueError("corrupt DRW1 capture: block offsets not a 0-based non-decreasing prefix")
    if pos + int(boff[-1]) != len(buf):
        raise ValueError("corrupt DRW1 capture: block bytes truncated or trailing data")
    return nrounds, arrs, boff, pos


def arrays(buf: bytes) -> Tuple[np.ndarray, ...]:
    """The dr_append_rounds_lists arrays of a capture (views into buf; empty id
    arrays padded to one element as flatten_lists does)."""
    _, arrs, _, _ = _parse(buf)
    return tuple(a if a.size else np.zeros(1, a.dtype) for a in arrs)


def decode(buf: bytes) -> Dag:
    nrounds, (so, sid, sto, sti, wo, wi), boff, pos = _parse(buf)
    dag: Dag = []
    k = 0
    for r in range(nrounds):
        rnd = []
        for _ in range(int(so[r + 1] - so[r])):
            st = [VertexID(int(sti[2 * e]), int(sti[2 * e + 1])) for e in range(int(sto[k]), int(sto[k + 1]))]
            wk = [VertexID(int(wi[2 * e]), int(wi[2 * e + 1])) for e in range(int(wo[k]), int(wo[k + 1]))]
            blk = bytes(buf[pos + int(boff[k]):pos + int(boff[k + 1])])
            rnd.append(Vertex(VertexID(int(sid[2 * k]), int(sid[2 * k + 1])), blk, st, wk))
            k += 1
        dag.append(rnd)
    return dag
