"""ctypes binding of oracle/liboracle.so (oracle.h).  TEST INFRASTRUCTURE ONLY."""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")

CHAIN_LITERAL, CHAIN_PERSISTENT = 0, 1
DELIVER_REF, DELIVER_PAPER = 0, 1
PANIC = -1

P = C.c_void_p


class Vid(C.Structure):
    _fields_ = [("round", C.c_int32), ("source", C.c_int32)]


class LDagS(C.Structure):
    _fields_ = [("nrounds", C.c_int32), ("slot_off", P), ("slot_id", P), ("strong_off", P), ("strong_ids", P),
                ("weak_off", P), ("weak_ids", P), ("leader", P), ("nleader", C.c_int32)]


class PDagS(C.Structure):
    _fields_ = [("n", C.c_int32), ("W", C.c_int32), ("nrounds", C.c_int32), ("slot_off", P), ("slot_src", P),
                ("strong", P), ("weak_off", P), ("weak_tgt", P), ("leader", P), ("nleader", C.c_int32)]


class ReplayOutS(C.Structure):
    _fields_ = [("commit", P), ("vcount", P), ("push_off", P), ("push_wave", P), ("push_cap", C.c_int64),
                ("pop_count", P), ("pop_digest", P), ("pop_edges", P), ("ids", P), ("ids_cap", C.c_int64),
                ("n_push", C.c_int64), ("n_ids", C.c_int64), ("commit_edges", C.c_uint64),
                ("chain_edges", C.c_uint64), ("deliver_edges", C.c_uint64)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `make oracle`")
        L = C.CDLL(LIB_PATH)
        sig = {
            "or_digest_term": (C.c_uint64, [C.c_int32, C.c_int32, C.c_uint64]),
            "or_lit_path": (C.c_int, [C.POINTER(LDagS), Vid, Vid, C.c_int]),
            "or_lit_leader": (C.c_int, [C.POINTER(LDagS), C.c_int, C.POINTER(Vid)]),
            "or_lit_wave_ready": (C.c_int, [C.POINTER(LDagS), C.c_int, C.c_int, C.c_int, P, C.POINTER(C.c_int),
                                            C.c_int, C.POINTER(C.c_int)]),
            "or_lit_order_vertices": (C.c_int, [C.POINTER(LDagS), P, C.c_int, C.c_int, C.c_int, P, P, C.c_int64,
                                                C.POINTER(C.c_int64), P, P]),
            "or_lit_replay": (C.c_int, [C.POINTER(LDagS), C.c_int, C.c_int, C.c_int, C.c_int,
                                        C.POINTER(ReplayOutS)]),
            "or_lit_replay_mt": (C.c_int, [C.POINTER(LDagS), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                           C.POINTER(ReplayOutS)]),
            "or_ldag_from_packed": (C.c_int, [C.POINTER(PDagS), C.c_int, C.POINTER(LDagS)]),
            "or_ldag_free": (None, [C.POINTER(LDagS)]),
            "or_bs_path": (C.c_int, [C.POINTER(PDagS), Vid, Vid, C.c_int]),
            "or_bs_cone": (C.c_int, [C.POINTER(PDagS), Vid, C.c_int, C.c_int, P, P]),
            "or_bs_commit_sweep": (C.c_int, [C.POINTER(PDagS), C.c_int, C.c_int, C.c_int, P, P, P]),
            "or_bs_order_vertices": (C.c_int, [C.POINTER(PDagS), P, C.c_int, C.c_int, C.c_int, P, C.c_int64,
                                               C.POINTER(C.c_int64), P, P]),
            "or_bs_replay": (C.c_int, [C.POINTER(PDagS), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                       C.POINTER(ReplayOutS)]),
        }
        for k, (r, a) in sig.items():
            f = getattr(L, k)
            f.restype, f.argtypes = r, a
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(P)


def digest_term(r: int, s: int, k: int) -> int:
    return lib().or_digest_term(r, s, k)


def digest(seq: Sequence[Tuple[int, int]]) -> int:
    return sum(digest_term(r, s, k) for k, (r, s) in enumerate(seq)) & ((1 << 64) - 1)


def coin_leaders(seed: int, n: int, nwaves: int):
    """The engine's seeded coin (DR_LEADER_SEEDED) restated: leader(w) = 1 +
    splitmix64(seed + w * 0x9E3779B97F4A7C15) mod n, for w = 1..nwaves."""
    M = (1 << 64) - 1
    out = []
    for w in range(1, nwaves + 1):
        z = (seed + w * 0x9E3779B97F4A7C15) & M
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        z ^= z >> 31
        out.append(1 + z % n)
    return out


def _set_leaders(obj, leaders):
    """chooseLeader(w) = leaders[w-1] (None: the reference's constant 1)."""
    if leaders is None:
        obj.s.leader, obj.s.nleader = None, 0
        return
    obj._lead = np.ascontiguousarray(np.asarray(leaders, np.int32))
    obj.s.leader, obj.s.nleader = _p(obj._lead), len(obj._lead)


class LDag:
    """List-form DAG (the literal [][]vertex), from flatten_lists-style arrays or a packed prefix."""

    def __init__(self, arrays=None, packed=None, nrounds: Optional[int] = None, leaders=None):
        self._owned = False
        self.s = LDagS()
        if arrays is not None:
            so, sid, sto, sti, wo, wi = [np.ascontiguousarray(a) for a in arrays]
            self._keep = (so, sid, sto, sti, wo, wi)
            self.s.nrounds = len(so) - 1
            self.s.slot_off, self.s.slot_id, self.s.strong_off = _p(so), _p(sid), _p(sto)
            self.s.strong_ids, self.s.weak_off, self.s.weak_ids = _p(sti), _p(wo), _p(wi)
        else:
            pd = PDag(packed)
            self._pd = pd
            rc = lib().or_ldag_from_packed(C.byref(pd.s), nrounds if nrounds is not None else packed.nrounds,
                                           C.byref(self.s))
            assert rc == 0
            self._owned = True
        _set_leaders(self, leaders)

    def __del__(self):
        if getattr(self, "_owned", False):
            lib().or_ldag_free(C.byref(self.s))
            self._owned = False

    def path(self, fr, to, strong: bool) -> int:
        return lib().or_lit_path(C.byref(self.s), Vid(*fr), Vid(*to), int(strong))

    def leader(self, w: int):
        v = Vid()
        rc = lib().or_lit_leader(C.byref(self.s), w, C.byref(v))
        return rc, (v.round, v.source)

    def wave_ready(self, faulty: int, wave: int, decided: int):
        st = np.zeros(2 * (wave + 2), np.int32)
        sl = C.c_int(0)
        vc = C.c_int(0)
        rc = lib().or_lit_wave_ready(C.byref(self.s), faulty, wave, decided, _p(st), C.byref(sl), wave + 2,
                                     C.byref(vc))
        return rc, vc.value, [tuple(int(x) for x in st[2 * i:2 * i + 2]) for i in range(sl.value)]

    def order_vertices(self, stack, cur_round: int, mode: int = DELIVER_REF, cap: int = 1 << 20):
        ns = len(stack)
        st = np.asarray(stack if ns else [(0, 0)], np.int32).reshape(-1)
        out = np.zeros(2 * cap, np.int32)
        on = C.c_int64(0)
        pc = np.zeros(max(ns, 1), np.uint64)
        pd = np.zeros(max(ns, 1), np.uint64)
        rc = lib().or_lit_order_vertices(C.byref(self.s), _p(st), ns, cur_round, mode, None, _p(out), cap,
                                         C.byref(on), _p(pc), _p(pd))
        return rc, out[:2 * min(on.value, cap)].reshape(-1, 2), pc[:ns], pd[:ns]

    def replay(self, faulty: int, nwaves: int, chain_mode=CHAIN_PERSISTENT, deliver_mode=DELIVER_REF,
               ids_cap: int = 0, nthreads: int = 1):
        return _replay(lambda o: lib().or_lit_replay_mt(C.byref(self.s), faulty, nwaves, chain_mode, deliver_mode,
                                                        nthreads, C.byref(o)), nwaves, chain_mode, ids_cap)


class PDag:
    """Packed DAG view (dag_rider_amd.dag.PackedDag duck type)."""

    def __init__(self, d, leaders=None):
        self.d = d
        self._keep = [np.ascontiguousarray(x) for x in (d.slot_off, d.slot_src, d.strong, d.weak_off,
                                                         d.weak_tgt if len(d.weak_tgt) else np.zeros(1, np.uint32))]
        self.s = PDagS(d.n, (d.n + 63) // 64, d.nrounds, *[_p(x) for x in self._keep], None, 0)
        _set_leaders(self, leaders)

    def path(self, fr, to, strong: bool) -> int:
        return lib().or_bs_path(C.byref(self.s), Vid(*fr), Vid(*to), int(strong))

    def cone(self, fr, bottom: int, strong: bool):
        W = (self.d.n + 63) // 64
        m = np.zeros((fr[0] - bottom + 1) * W, np.uint64)
        e = C.c_uint64(0)
        rc = lib().or_bs_cone(C.byref(self.s), Vid(*fr), bottom, int(strong), _p(m), C.byref(e))
        assert rc == 0
        return m.reshape(-1, W), e.value

    def order_vertices(self, stack, cur_round: int, mode: int = DELIVER_REF, cap: int = 1 << 20):
        ns = len(stack)
        st = np.asarray(stack if ns else [(0, 0)], np.int32).reshape(-1)
        out = np.zeros(2 * cap, np.int32)
        on = C.c_int64(0)
        pc = np.zeros(max(ns, 1), np.uint64)
        pd = np.zeros(max(ns, 1), np.uint64)
        rc = lib().or_bs_order_vertices(C.byref(self.s), _p(st), ns, cur_round, mode, _p(out), cap, C.byref(on),
                                        _p(pc), _p(pd))
        return rc, out[:2 * min(on.value, cap)].reshape(-1, 2), pc[:ns], pd[:ns]

    def commit_sweep(self, faulty: int, w0: int, w1: int):
        nw = w1 - w0 + 1
        cm = np.zeros(nw, np.uint8)
        vc = np.zeros(nw, np.int32)
        e = C.c_uint64(0)
        rc = lib().or_bs_commit_sweep(C.byref(self.s), faulty, w0, w1, _p(cm), _p(vc), C.byref(e))
        assert rc == 0
        return cm, vc, e.value

    def replay(self, faulty: int, nwaves: int, chain_mode=CHAIN_PERSISTENT, deliver_mode=DELIVER_REF,
               ids_cap: int = 0, nthreads: int = 0):
        return _replay(lambda o: lib().or_bs_replay(C.byref(self.s), faulty, nwaves, chain_mode, deliver_mode,
                                                    nthreads, C.byref(o)), nwaves, chain_mode, ids_cap)


@dataclass
class OracleReplay:
    rc: int
    commit: np.ndarray
    vcount: np.ndarray
    push_off: np.ndarray
    push_wave: np.ndarray
    pop_count: np.ndarray
    pop_digest: np.ndarray
    pop_edges: np.ndarray
    ids: Optional[np.ndarray]
    commit_edges: int
    chain_edges: int
    deliver_edges: int


def _replay(call, nwaves, chain_mode, ids_cap):
    cap = nwaves * (nwaves + 1) // 2 + 1 if chain_mode == CHAIN_LITERAL else 2 * nwaves + 1
    cm = np.zeros(nwaves, np.uint8)
    vc = np.zeros(nwaves, np.int32)
    po = np.zeros(nwaves + 1, np.uint32)
    pw = np.zeros(cap, np.int32)
    pc = np.zeros(cap, np.uint64)
    pdg = np.zeros(cap, np.uint64)
    pe = np.zeros(cap, np.uint64)
    ids = np.zeros(2 * ids_cap, np.int32) if ids_cap else None
    o = ReplayOutS()
    o.commit, o.vcount, o.push_off, o.push_wave, o.push_cap = _p(cm), _p(vc), _p(po), _p(pw), cap
    o.pop_count, o.pop_digest, o.pop_edges, o.ids, o.ids_cap = _p(pc), _p(pdg), _p(pe), _p(ids), ids_cap
    rc = call(o)
    k = o.n_push
    return OracleReplay(rc, cm, vc, po, pw[:k], pc[:k], pdg[:k], pe[:k],
                        None if ids is None else ids[:2 * min(o.n_ids, ids_cap)].reshape(-1, 2),
                        o.commit_edges, o.chain_edges, o.deliver_edges)
