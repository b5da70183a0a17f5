"""Python handle on a process-column sharded DAG mirror (include/dagrider_shard.h).

SURVEY.md s8(e): a DAG split by target column across the GPUs of one node, one
process per GPU, with one RCCL all-gather of the frontier per round inside the
library.  Reach sets and path(), waveReady's commit and chain, orderVertices and
the whole replay all run on the sharded DAG.  ``ShardEngine.from_process_group`` builds the RCCL group from the
``torch.distributed`` default group (rank 0 makes the unique id, a broadcast hands it
to every rank).  ``ShardEngine(..., nshards=G)`` without an id is local mode: all G
column shards in one context on one device (same kernels, same split).

All compute happens in the HIP library; there is no CPU implementation here.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L
from .dag import PackedDag
from .engine import ReplayResult, _replay_out, _replay_result


def shard_unique_id() -> bytes:
    """dr_shard_unique_id: a fresh RCCL unique id (needs a HIP device)."""
    buf = (C.c_uint8 * L.DR_SHARD_ID_BYTES)()
    lib = L.lib()
    rc = lib.dr_shard_unique_id(buf)
    if rc != L.DR_OK:
        raise L.DrError(rc, lib.dr_shard_last_error(None).decode())
    return bytes(buf)


def exchange_unique_id(dist, make_id=shard_unique_id, group=None) -> bytes:
    """Rank 0 makes the id, every rank of `group` receives it (torch.distributed
    broadcast_object_list: works over gloo or nccl)."""
    box = [make_id() if dist.get_rank(group) == 0 else None]
    dist.broadcast_object_list(box, src=0, group=group)
    uid = box[0]
    if not isinstance(uid, (bytes, bytearray)) or len(uid) != L.DR_SHARD_ID_BYTES:
        raise RuntimeError("malformed shard unique id")
    return bytes(uid)


class ShardEngine:
    """One column-sharded Process.dag mirror (dr_shard_create ... dr_shard_destroy)."""

    def __init__(self, n: int, faulty: int, max_rounds: int, device: int = 0, nshards: int = 1, rank: int = 0,
                 unique_id: Optional[bytes] = None):
        self._L = L.lib()
        h = L.P()
        idp = None
        if unique_id is not None:
            self._id = (C.c_uint8 * L.DR_SHARD_ID_BYTES).from_buffer_copy(unique_id)
            idp = C.cast(self._id, L.P)
        rc = self._L.dr_shard_create(n, faulty, max_rounds, device, nshards, rank, idp, C.byref(h))
        if rc != L.DR_OK:
            raise L.DrError(rc, self._L.dr_shard_last_error(None).decode())
        self._h = h
        self.n, self.faulty, self.max_rounds, self.device = n, faulty, max_rounds, device
        self.nshards, self.rank = nshards, rank

    @classmethod
    def from_process_group(cls, dist, n: int, faulty: int, max_rounds: int, device: int) -> "ShardEngine":
        """One shard per rank of the torch.distributed default group (RCCL mode)."""
        uid = exchange_unique_id(dist)
        return cls(n, faulty, max_rounds, device, dist.get_world_size(), dist.get_rank(), uid)

    def close(self):
        if getattr(self, "_h", None):
            self._L.dr_shard_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc: int):
        if rc != L.DR_OK:
            raise L.DrError(rc, self._L.dr_shard_last_error(self._h).decode())

    @property
    def num_rounds(self) -> int:
        return self._L.dr_shard_num_rounds(self._h)

    def info(self) -> dict:
        v = [C.c_int() for _ in range(5)]
        self._check(self._L.dr_shard_info(self._h, *[C.byref(x) for x in v]))
        return dict(zip(("nshards", "shard0", "nlocal", "col0", "col1"), [x.value for x in v]))

    def stats(self) -> dict:
        ms, rounds, xb = L.f32(), L.u64(), L.u64()
        self._check(self._L.dr_shard_stats(self._h, C.byref(ms), C.byref(rounds), C.byref(xb)))
        sy = L.u64()
        self._check(self._L.dr_shard_host_syncs(self._h, C.byref(sy)))
        return dict(ms=ms.value, rounds=rounds.value, exchange_bytes=xb.value, host_syncs=sy.value)

    def append_packed(self, d: PackedDag, r0: Optional[int] = None, r1: Optional[int] = None):
        r0 = self.num_rounds if r0 is None else r0
        r1 = d.nrounds if r1 is None else r1
        n, W = d.n, d.W
        so = np.ascontiguousarray(d.slot_off[r0:r1 + 1])
        st = np.ascontiguousarray(d.strong[r0 * n * W:r1 * n * W])
        wo = np.ascontiguousarray(d.weak_off[r0 * n:r1 * n + 1])
        wt = d.weak_tgt if len(d.weak_tgt) else np.zeros(1, np.uint32)
        self._check(self._L.dr_shard_append_rounds_packed(self._h, r0, r1 - r0, L.ptr(so), L.ptr(d.slot_src),
                                                          L.ptr(st), L.ptr(wo), L.ptr(wt)))

    def reach_sets(self, froms: Sequence[Tuple[int, int]], bottoms: Sequence[int], strong_only: bool) -> List[np.ndarray]:
        q = len(froms)
        fr = np.asarray(froms if q else [(0, 0)], dtype=np.int32).reshape(-1)
        bt = np.asarray(bottoms if q else [0], dtype=np.int32)
        W = (self.n + 63) // 64
        need = sum((f[0] - b + 1) * W for f, b in zip(froms, bottoms))
        out = np.zeros(max(need, 1), dtype=np.uint64)
        nw = C.c_size_t()
        self._check(self._L.dr_shard_reach_sets(self._h, q, L.ptr(fr), L.ptr(bt), int(strong_only), L.ptr(out), need,
                                                C.byref(nw)))
        res, o = [], 0
        for f, b in zip(froms, bottoms):
            k = (f[0] - b + 1) * W
            res.append(out[o:o + k].reshape(-1, W))
            o += k
        return res

    def path_batch(self, pairs: Sequence[Tuple[Tuple[int, int], Tuple[int, int]]], strong_only: bool) -> np.ndarray:
        q = len(pairs)
        fr = np.asarray([p[0] for p in pairs] if q else [(0, 0)], dtype=np.int32).reshape(-1)
        to = np.asarray([p[1] for p in pairs] if q else [(0, 0)], dtype=np.int32).reshape(-1)
        out = np.zeros(max(q, 1), dtype=np.uint8)
        self._check(self._L.dr_shard_path_batch(self._h, q, L.ptr(fr), L.ptr(to), int(strong_only), L.ptr(out)))
        return out[:q]

    def set_persistent(self, on: bool):
        """DR_SHARD_OPT_PERSISTENT: one cooperative launch per sweep batch (local mode)."""
        self._check(self._L.dr_shard_set_option(self._h, L.DR_SHARD_OPT_PERSISTENT, int(on)))

    def set_memo(self, on: bool):
        """DR_SHARD_OPT_MEMO: memoized REF replay (summaries, canonical cone, relative-round steps)."""
        self._check(self._L.dr_shard_set_option(self._h, L.DR_SHARD_OPT_MEMO, int(on)))

    def set_stepped(self, on: bool):
        """DR_SHARD_OPT_STEPPED: the memo replay's stepped form (one round per launch, columns
        exchanged between launches) even when this context holds every column."""
        self._check(self._L.dr_shard_set_option(self._h, L.DR_SHARD_OPT_STEPPED, int(on)))

    def set_phase_timing(self, on: bool):
        """DR_SHARD_OPT_PHASE_TIMING: per-phase device times in the replay's ms_* (default on)."""
        self._check(self._L.dr_shard_set_option(self._h, L.DR_SHARD_OPT_PHASE_TIMING, int(on)))

    def set_step_hints(self, steps: int):
        """DR_SHARD_OPT_STEP_HINTS: the stepped form's initial step counts (1 forces every
        continuation of a live canonical walk or query)."""
        self._check(self._L.dr_shard_set_option(self._h, L.DR_SHARD_OPT_STEP_HINTS, int(steps)))

    def set_leader_coin(self, mode: int = L.DR_LEADER_CONST1, seed: int = 0,
                        table: Optional[Sequence[int]] = None):
        """chooseLeader (process.go:386-392), as Engine.set_leader_coin."""
        t = np.asarray(table if table is not None else [1], dtype=np.int32)
        k = len(table) if table is not None else 0
        self._check(self._L.dr_shard_set_leader_coin(self._h, mode, seed, k, L.ptr(t)))

    def wave_commit(self, w0: int, w1: int):
        nw = w1 - w0 + 1
        cm = np.zeros(max(nw, 1), np.uint8)
        vc = np.zeros(max(nw, 1), np.int32)
        self._check(self._L.dr_shard_wave_commit(self._h, w0, w1, L.ptr(cm), L.ptr(vc)))
        return cm[:nw], vc[:nw]

    def wave_ready(self, wave: int, decided_wave: int):
        cm = np.zeros(1, np.uint8)
        vc = np.zeros(1, np.int32)
        cap = max(wave + 1, 1)
        pw = np.zeros(cap, np.int32)
        npush = C.c_int()
        self._check(self._L.dr_shard_wave_ready(self._h, wave, decided_wave, L.ptr(cm), L.ptr(vc), L.ptr(pw), cap,
                                                C.byref(npush)))
        return bool(cm[0]), int(vc[0]), [int(x) for x in pw[:npush.value]]

    def order_vertices(self, stack: Sequence[Tuple[int, int]], cur_round: int, mode: int = L.DR_DELIVER_REF):
        """Per-pop delivered counts and digests (and the total) of orderVertices."""
        ns = len(stack)
        st = np.asarray(stack if ns else [(0, 0)], dtype=np.int32).reshape(-1)
        out_n = C.c_size_t()
        pc = np.zeros(max(ns, 1), np.uint64)
        pd = np.zeros(max(ns, 1), np.uint64)
        self._check(self._L.dr_shard_order_vertices(self._h, L.ptr(st), ns, cur_round, mode, C.byref(out_n),
                                                    L.ptr(pc), L.ptr(pd)))
        return out_n.value, pc[:ns], pd[:ns]

    def replay(self, nwaves: int, chain_mode: int = L.DR_CHAIN_PERSISTENT, deliver_mode: int = L.DR_DELIVER_REF,
               push_cap: Optional[int] = None) -> ReplayResult:
        """dr_shard_replay: the whole replay (commit, chains, delivery) on the sharded DAG."""
        o, keep = _replay_out(nwaves, chain_mode, 0, push_cap)
        self._check(self._L.dr_shard_replay(self._h, nwaves, chain_mode, deliver_mode, C.byref(o)))
        return _replay_result(o, keep, 0)


class ShardReplayer:
    """dr_shard_replay into output buffers allocated once (the bench's timed steps);
    result() returns views of those buffers, overwritten by the next call."""

    def __init__(self, se: ShardEngine, nwaves: int, chain_mode: int = L.DR_CHAIN_PERSISTENT,
                 deliver_mode: int = L.DR_DELIVER_REF):
        self._se = se
        self._o, self._keep = _replay_out(nwaves, chain_mode, 0)
        self._fn, self._args = se._L.dr_shard_replay, (se._h, nwaves, chain_mode, deliver_mode, C.byref(self._o))

    def __call__(self) -> None:
        rc = self._fn(*self._args)
        if rc != L.DR_OK:
            self._se._check(rc)

    def result(self) -> ReplayResult:
        return _replay_result(self._o, self._keep, 0)
