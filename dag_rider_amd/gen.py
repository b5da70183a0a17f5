"""Synthetic DAG workloads (generator spec: include/dagrider_gen.h) and the five configs.

CONFIGS pins SURVEY.md s8(d)'s proposed parameters.  The generator is host C++
(deterministic splitmix64 streams), so the same DAG is produced here and on the
GPU box without shipping data.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib as L
from .dag import PackedDag


@dataclass(frozen=True)
class GenConfig:
    name: str
    n: int
    last_round: int  # R: rounds 0..R
    seed: int
    p_present: float
    p_late: float
    p_w: float
    weak_depth: int
    p_la: float = 0.0
    # repeated ids: every id of a round >= 1 gets one more slot
    # w.p. p_dup, at a random position of its round (uponDeliver / the buffer loop
    # appending a vertex already in the round, process.go:158-169, :229)
    p_dup: float = 0.0
    # single edges added after generation, (round, source, target round, target source,
    # strong): a weak edge past the memo window or a strong edge skipping rounds (App. A
    # Q8) -- exceptions to the regular graph (engine.hip ensure_exceptions)
    extra: tuple = ()

    @property
    def faulty(self) -> int:
        return (self.n - 1) // 3

    @property
    def nwaves(self) -> int:
        return self.last_round // 4


CONFIGS = {
    # C1: seeded n=4 companion of the Figure-1 fixture (4 waves)
    "c1": GenConfig("c1", 4, 16, 1, 1.0, 0.25, 1.0, 4, 0.0),
    "c2": GenConfig("c2", 64, 1000, 2, 0.95, 0.05, 0.5, 8, 0.05),
    "c3": GenConfig("c3", 256, 10000, 3, 1.0, 0.3, 0.25, 4, 0.0),
    "c4": GenConfig("c4", 1024, 4000, 4, 1.0, 0.02, 0.5, 4, 0.0),
    # C4 with weak edges up to 80 rounds deep, past the memo window (weak deltas <= 65,
    # engine.hip memo_ok): every pop sweeps its whole cone (bench.py --config c4-deep)
    "c4-deep": GenConfig("c4-deep", 1024, 4000, 4, 1.0, 0.02, 0.03, 80, 0.0),
    # C4 with weak edges up to 64 rounds deep, the memo window's far end (--config c4-deep64)
    "c4-deep64": GenConfig("c4-deep64", 1024, 4000, 4, 1.0, 0.02, 0.04, 64, 0.0),
    # C4 with repeated ids: ~1 % of each round's ids delivered twice (--config c4-dups)
    "c4-dups": GenConfig("c4-dups", 1024, 4000, 4, 1.0, 0.02, 0.5, 4, 0.0, 0.01),
    # C4 + one weak edge 600 rounds deep (past the regular window): an exception whose
    # target is in its source's regular cone, so the memo stays on (--config c4-far)
    "c4-far": GenConfig("c4-far", 1024, 4000, 4, 1.0, 0.02, 0.5, 4, 0.0, extra=((2002, 17, 1402, 5, False),)),
    # C4 + one strong edge to round r-3 (--config c4-q8)
    "c4-q8": GenConfig("c4-q8", 1024, 4000, 4, 1.0, 0.02, 0.5, 4, 0.0, extra=((2001, 17, 1998, 5, True),)),
    # C4 + one weak edge to its own round (App. A Q8, not below the source: no exception
    # test applies): every query takes the general sweep (--config c4-up, k_gsweep at scale)
    "c4-up": GenConfig("c4-up", 1024, 4000, 4, 1.0, 0.02, 0.5, 4, 0.0, extra=((2002, 17, 2002, 5, False),)),
    # C5: one of the 4096 independent n=128 replays (seed 5000+i)
    "c5": GenConfig("c5", 128, 128, 5000, 0.9, 0.1, 0.5, 4, 0.05),
}


def generate(cfg: GenConfig, nthreads: int = 0) -> PackedDag:
    lib = L.lib()
    p = L.GenParams(cfg.n, cfg.last_round, cfg.seed, cfg.p_present, cfg.p_late, cfg.p_w, cfg.p_la,
                    cfg.weak_depth, nthreads)
    h = L.P()
    rc = lib.dr_gen_create(C.byref(p), C.byref(h))
    if rc != 0:
        raise ValueError(f"generator rejected {cfg}")
    try:
        n, W, nr = L.i32(), L.i32(), L.i32()
        ns, nw = L.u64(), L.u64()
        lib.dr_gen_info(h, C.byref(n), C.byref(W), C.byref(nr), C.byref(ns), C.byref(nw))
        n, W, nr, ns, nw = n.value, W.value, nr.value, ns.value, nw.value

        def view(fn, dtype, count):
            if count == 0:
                return np.zeros(0, dtype)
            addr = fn(h)
            buf = (C.c_char * (count * np.dtype(dtype).itemsize)).from_address(addr)
            return np.frombuffer(buf, dtype=dtype, count=count).copy()

        d = PackedDag(n, nr,
                      view(lib.dr_gen_slot_off, np.uint32, nr + 1),
                      view(lib.dr_gen_slot_src, np.uint16, ns),
                      view(lib.dr_gen_strong, np.uint64, nr * n * W),
                      view(lib.dr_gen_weak_off, np.uint32, nr * n + 1),
                      view(lib.dr_gen_weak_tgt, np.uint32, nw))
    finally:
        lib.dr_gen_free(h)
    if cfg.p_dup > 0:
        d = with_repeated_slots(d, cfg.p_dup, cfg.seed)
    return with_extra_edges(d, cfg.extra) if cfg.extra else d


def with_extra_edges(d: PackedDag, extra) -> PackedDag:
    """Append single edges to their vertices' weak_tgt lists: (r, s, tr, ts, strong) adds
    (r, s) -> (tr, ts), a strong one with bit 31 set (include/dagrider_gpu.h,
    dr_append_rounds_packed).  Each source must be present in its round."""
    n = d.n
    off = d.weak_off.astype(np.int64)
    tgt = d.weak_tgt
    at, val = [], []
    for r, s, tr, ts, strong in sorted(extra):
        g = r * n + s - 1
        at.append(off[g + 1])
        val.append((tr << 11) | (ts - 1) | ((1 << 31) if strong else 0))
    tgt = np.insert(tgt, at, np.asarray(val, np.uint32)).astype(np.uint32)
    add = np.zeros(len(off), np.int64)
    for r, s, *_ in extra:
        add[r * n + s:] += 1  # every offset after the vertex's own list start
    return PackedDag(n, d.nrounds, d.slot_off, d.slot_src, d.strong, (off + add).astype(np.uint32), tgt)


def with_repeated_slots(d: PackedDag, p_dup: float, seed: int) -> PackedDag:
    """Every id of a round >= 1 gets one more slot w.p. p_dup, at a random position of
    its round.  The packed row is per id (its last slot's, path()'s lookup,
    process.go:112-116), so only the slot lists change; vCount and REF delivery count
    the extra slots, PAPER delivers an id at its first."""
    rng = np.random.default_rng(np.random.SeedSequence([seed, 0x5107]))
    off = d.slot_off.astype(np.int64)
    parts, new_off = [], [0]
    for r in range(d.nrounds):
        s = d.slot_src[off[r]:off[r + 1]]
        if r >= 1:
            ids = s[s != 0]
            pick = ids[rng.random(len(ids)) < p_dup]
            if len(pick):
                s = np.insert(s, np.sort(rng.integers(0, len(s) + 1, size=len(pick))), pick)
        parts.append(s)
        new_off.append(new_off[-1] + len(s))
    return PackedDag(d.n, d.nrounds, np.asarray(new_off, np.uint32), np.concatenate(parts).astype(np.uint16),
                     d.strong, d.weak_off, d.weak_tgt)


def c5_config(i: int) -> GenConfig:
    """DAG i of C5's batch of 4096 independent n=128 replays (seed 5000+i)."""
    import dataclasses

    return dataclasses.replace(CONFIGS["c5"], name=f"c5-{i}", seed=CONFIGS["c5"].seed + i)


def small_config(n: int, last_round: int, seed: int, **kw) -> GenConfig:
    """Seeded small DAGs for cross-checks (parameters randomised per seed by the caller)."""
    base = dict(p_present=0.9, p_late=0.2, p_w=0.5, weak_depth=4, p_la=0.1)
    base.update(kw)
    return GenConfig(f"small-{n}-{last_round}-{seed}", n, last_round, seed, **base)
