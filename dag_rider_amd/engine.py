"""Python handle on one device mirror (dr_ctx) -- a thin veneer over the C ABI.

Each method names the reference function it stands in for; semantics are those of
``include/dagrider_gpu.h``.  All compute happens in the HIP library: there is no
Python or CPU implementation of any query here.
"""
from __future__ import annotations

import ctypes as C
import functools
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L
from .dag import PackedDag, Vertex, flatten_lists


@dataclass
class ReplayResult:
    commit: np.ndarray  # uint8 [nwaves]
    vcount: np.ndarray  # int32 [nwaves]
    push_off: np.ndarray  # uint32 [nwaves+1]
    push_wave: np.ndarray  # int32 [n_push]
    pop_count: np.ndarray  # uint64 [n_push]
    pop_digest: np.ndarray  # uint64 [n_push]
    pop_edges: np.ndarray  # uint64 [n_push]
    ids: Optional[np.ndarray]  # int32 [n_ids, 2]
    commit_edges: int
    chain_edges: int
    deliver_edges: int
    ms: dict
    sweep: dict

    @property
    def total_edges(self) -> int:
        return self.commit_edges + self.chain_edges + self.deliver_edges


class Engine:
    """One Process.dag mirror on a GPU (dr_create ... dr_destroy)."""

    def __init__(self, n: int, faulty: int, max_rounds: int, device: int = 0, shared_stream: bool = False):
        self._L = L.lib()
        h = L.P()
        # shared_stream: DR_CREATE_SHARED_STREAM (one stream for every such context of the
        # device: the members of a large dr_replay_batch)
        rc = self._L.dr_create_ex(n, faulty, max_rounds, device, L.DR_CREATE_SHARED_STREAM if shared_stream else 0,
                                  C.byref(h))
        if rc != L.DR_OK:
            raise L.DrError(rc, self._L.dr_last_error(None).decode())
        self._h = h
        self.n, self.faulty, self.max_rounds, self.device = n, faulty, max_rounds, device

    def close(self):
        if getattr(self, "_h", None):
            self._L.dr_destroy(self._h)
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
            raise L.DrError(rc, self._L.dr_last_error(self._h).decode())

    def set_memo(self, on: bool):
        """DR_OPT_MEMO: round summaries + canonical cone (identical results either way)."""
        self._check(self._L.dr_set_option(self._h, L.DR_OPT_MEMO, int(on)))

    def set_leader_coin(self, mode: int = L.DR_LEADER_CONST1, seed: int = 0,
                        table: Optional[Sequence[int]] = None):
        """chooseLeader (process.go:386-392): constant 1 (the reference), a seeded coin, or a table."""
        t = np.asarray(table if table is not None else [1], np.int32)
        k = len(table) if table is not None else 0
        self._check(self._L.dr_set_leader_coin(self._h, mode, seed, k, L.ptr(t)))

    def wave_leader(self, wave: int) -> int:
        """chooseLeader(wave) under the current coin (1-based source)."""
        return int(self._L.dr_wave_leader(self._h, wave))

    def set_phase_timing(self, level: int):
        """DR_OPT_PHASE_TIMING: 2 = every replay phase timed, 1 = summary pass only, 0 = none."""
        self._check(self._L.dr_set_option(self._h, L.DR_OPT_PHASE_TIMING, int(level)))

    def set_device_plan(self, on: bool):
        """DR_OPT_DEVICE_PLAN: plan dr_replay's phases on the device (identical results either way)."""
        self._check(self._L.dr_set_option(self._h, L.DR_OPT_DEVICE_PLAN, int(on)))

    def set_commit_split(self, mode: int):
        """DR_OPT_COMMIT_SPLIT: several workgroups per wave for short wave ranges (1: every range
        shorter than the CU count, 2: ranges of at most 4 waves, the default; 0 = one workgroup
        per wave; identical results)."""
        self._check(self._L.dr_set_option(self._h, L.DR_OPT_COMMIT_SPLIT, int(mode)))

    def set_replay_graph(self, on: bool):
        """DR_OPT_REPLAY_GRAPH: replay a repeated device-planned dr_replay as one captured
        hipGraph (default off; identical results)."""
        self._check(self._L.dr_set_option(self._h, L.DR_OPT_REPLAY_GRAPH, int(on)))

    def replay_graph_state(self) -> int:
        """The last replay's form: 1 graph launch, 0 kernel by kernel, -1 after a failed capture."""
        return int(self._L.dr_replay_graph_state(self._h))

    def set_fuse(self, mask: int):
        """DR_OPT_FUSE: which independent replay phases share a launch (7 = all, 0 = none)."""
        self._check(self._L.dr_set_option(self._h, L.DR_OPT_FUSE, int(mask)))

    def set_call_overlap(self, mode: int):
        """DR_OPT_CALL_OVERLAP: after a REF orderVertices, waveReady launches the canonical cone of
        the new top without waiting for it (1, the default: behind the commit rule when no leader
        chain can follow, else once it knows of a commit; 2: on a second stream beside the commit
        rule); 0 = orderVertices computes it.  Identical results."""
        self._check(self._L.dr_set_option(self._h, L.DR_OPT_CALL_OVERLAP, int(mode)))

    def set_batch_form(self, form: int):
        """DR_OPT_BATCH_FORM (read from a batch's first engine): DR_BATCH_AUTO, DR_BATCH_WORKGROUP
        (four wavefronts per DAG) or DR_BATCH_WAVE (one wavefront per DAG); identical results."""
        self._check(self._L.dr_set_option(self._h, L.DR_OPT_BATCH_FORM, int(form)))

    def profile_kernel(self, kernel: int, variant: int = 0, iters: int = 20) -> float:
        """dr_profile_kernel: average device ms of one kernel variant (tuning hook of the
        profiling build: DR_LIB_VARIANT=timing, include/dagrider_tuning.h)."""
        ms = L.f32()
        self._check(self._L.dr_profile_kernel(self._h, kernel, variant, iters, C.byref(ms)))
        return ms.value

    def last_kernel_ms(self) -> float:
        """dr_last_kernel_ms: device time of the last commit-rule launch (HIP events)."""
        ms = L.f32()
        self._check(self._L.dr_last_kernel_ms(self._h, C.byref(ms)))
        return ms.value

    def append_phases(self) -> dict:
        """dr_last_append_phases: host ms of the last packed append by phase."""
        ms = (C.c_float * 4)()
        self._check(self._L.dr_last_append_phases(self._h, ms))
        return dict(build=ms[0], stage_rows=ms[1], stage_rounds=ms[2], copy_wait=ms[3])

    def exception_stats(self) -> dict:
        """dr_exception_stats: the exceptions to the regular graph and the test's verdict
        (include/dagrider_gpu.h)."""
        out = np.zeros(6, np.int64)
        self._check(self._L.dr_exception_stats(self._h, out.ctypes.data))
        keys = ("exceptions", "changing", "sweeps", "regular_delta", "upward", "memo")
        return {k: int(v) for k, v in zip(keys, out)}

    def mirror_stats(self) -> dict:
        """dr_mirror_stats: rounds, slots, weak-column entries and weak edges of the mirror."""
        out = np.zeros(4, np.int64)
        self._check(self._L.dr_mirror_stats(self._h, out.ctypes.data, 4))
        return {k: int(v) for k, v in zip(("rounds", "slots", "weak_columns", "weak_edges"), out)}

    def set_slice(self, round_offset: int = 0, pos_base: int = 0, seeded_top: int = 0, own_w0: int = 0,
                  probes: Sequence[int] = (), clear: bool = False):
        """dr_set_slice: this mirror is global rounds [round_offset, ...) of a bigger DAG
        (dag_rider_amd/split.py, include/dagrider_gpu.h); clear=True drops it."""
        if clear:
            self._check(self._L.dr_set_slice(self._h, None))
            return
        if len(probes) > 8:
            raise ValueError("at most 8 probe rounds")
        cfg = L.SliceCfg(round_offset, seeded_top, pos_base, own_w0, len(probes))
        for i, r in enumerate(probes):
            cfg.probe[i] = int(r)
        self._check(self._L.dr_set_slice(self._h, C.byref(cfg)))

    def last_replay_path(self) -> int:
        """dr_last_replay_path: 0 memo, 1 memo with the upward edges verified, 2 general after a
        failed check, 3 general."""
        return int(self._L.dr_last_replay_path(self._h))

    def slice_result(self) -> dict:
        """dr_slice_result: C, G, E at the probes, the owned pops' lowest merge round and the
        owned commits' chain edges from the last dr_replay."""
        o = L.SliceOut()
        self._check(self._L.dr_slice_result(self._h, C.byref(o)))
        return dict(C=[int(x) for x in o.C], G=[int(x) for x in o.G], E=[int(x) for x in o.E],
                    min_stop=int(o.min_stop), own_chain_edges=int(o.own_chain_edges))

    @property
    def num_rounds(self) -> int:
        return self._L.dr_num_rounds(self._h)

    # ---- p.dag[r] = append(...)  (process.go:229) ----
    def append_lists(self, dag: Sequence[Sequence[Vertex]], r0: Optional[int] = None, r1: Optional[int] = None):
        r0 = self.num_rounds if r0 is None else r0
        r1 = len(dag) if r1 is None else r1
        a = flatten_lists(dag, r0, r1)
        self._check(self._L.dr_append_rounds_lists(self._h, r0, r1 - r0, *[L.ptr(x) for x in a]))

    def append_packed(self, d: PackedDag, r0: Optional[int] = None, r1: Optional[int] = None):
        r0 = self.num_rounds if r0 is None else r0
        r1 = d.nrounds if r1 is None else r1
        n, W = d.n, d.W
        so = np.ascontiguousarray(d.slot_off[r0:r1 + 1])
        st = np.ascontiguousarray(d.strong[r0 * n * W:r1 * n * W])
        wo = np.ascontiguousarray(d.weak_off[r0 * n:r1 * n + 1])
        self._check(self._L.dr_append_rounds_packed(self._h, r0, r1 - r0, L.ptr(so), L.ptr(d.slot_src), L.ptr(st),
                                                    L.ptr(wo), L.ptr(d.weak_tgt if len(d.weak_tgt) else
                                                                     np.zeros(1, np.uint32))))

    def append_vertices(self, verts: Sequence[Vertex], rounds: Optional[Sequence[int]] = None):
        """p.dag[v.id.round] = append(p.dag[v.id.round], v) (process.go:229) per vertex, in
        order; rounds[i] (default v.id.round) is the dag index, == num_rounds opens it."""
        k = len(verts)
        if k == 0:
            return
        ids = np.asarray([(v.id.round, v.id.source) for v in verts], np.int32).reshape(-1)
        so = np.zeros(k + 1, np.uint32)
        wo = np.zeros(k + 1, np.uint32)
        st: List[int] = []
        wk: List[int] = []
        for i, v in enumerate(verts):
            for e in v.strong_edges:
                st += [e.round, e.source]
            for e in v.weak_edges:
                wk += [e.round, e.source]
            so[i + 1] = len(st) // 2
            wo[i + 1] = len(wk) // 2
        sti = np.asarray(st if st else [0], np.int32)
        wki = np.asarray(wk if wk else [0], np.int32)
        rr = None if rounds is None else np.asarray(rounds, np.int32)
        self._check(self._L.dr_append_vertices(self._h, k, L.ptr(rr), L.ptr(ids), L.ptr(so), L.ptr(sti), L.ptr(wo),
                                               L.ptr(wki)))

    def append_capture(self, buf: bytes):
        """Replay a DRW1 capture (dag_rider_amd/wire.py) through the C reader (dr_wire_append)."""
        b = C.create_string_buffer(bytes(buf), len(buf))
        self._check(self._L.dr_wire_append(self._h, b, len(buf)))

    # ---- path(from, to, strongPath)  (process.go:89-148), batched ----
    def path_batch(self, pairs: Sequence[Tuple[Tuple[int, int], Tuple[int, int]]], strong_only: bool) -> np.ndarray:
        q = len(pairs)
        fr = np.asarray([p[0] for p in pairs], dtype=np.int32).reshape(-1)
        to = np.asarray([p[1] for p in pairs], dtype=np.int32).reshape(-1)
        out = np.zeros(max(q, 1), dtype=np.uint8)
        self._check(self._L.dr_path_batch(self._h, q, L.ptr(fr), L.ptr(to), int(strong_only), L.ptr(out)))
        return out[:q]

    def reach_sets(self, froms: Sequence[Tuple[int, int]], bottoms: Sequence[int], strong_only: bool) -> List[np.ndarray]:
        q = len(froms)
        fr = np.asarray(froms, dtype=np.int32).reshape(-1)
        bt = np.asarray(bottoms, dtype=np.int32)
        W = (self.n + 63) // 64
        need = sum((f[0] - b + 1) * W for f, b in zip(froms, bottoms))
        out = np.zeros(max(need, 1), dtype=np.uint64)
        nw = C.c_size_t()
        self._check(self._L.dr_reach_sets(self._h, q, L.ptr(fr), L.ptr(bt), int(strong_only), L.ptr(out), need,
                                          C.byref(nw)))
        res, o = [], 0
        for f, b in zip(froms, bottoms):
            k = (f[0] - b + 1) * W
            res.append(out[o:o + k].reshape(-1, W))
            o += k
        return res

    # ---- setWeakEdges (process.go:298-310) ----
    def set_weak_edges(self, round_: int, strong: Sequence[Tuple[int, int]], mode: int = L.DR_WEAK_PAPER,
                       cap: Optional[int] = None) -> np.ndarray:
        """The weak edges of a vertex of round `round_` with these strong edges, in the
        reference's order (rounds round-2 .. 1, slot order); ids as an [k, 2] int32 array."""
        ns = len(strong)
        st = np.asarray(strong if ns else [(0, 0)], dtype=np.int32).reshape(-1)
        out_n = C.c_size_t()
        self._check(self._L.dr_set_weak_edges(self._h, round_, ns, L.ptr(st), mode, None, 0, C.byref(out_n)))
        k = out_n.value
        ids = np.zeros(max(k, 1) * 2, np.int32)
        self._check(self._L.dr_set_weak_edges(self._h, round_, ns, L.ptr(st), mode, L.ptr(ids), k, C.byref(out_n)))
        return ids[:2 * k].reshape(-1, 2)

    # ---- buffer loop + present() (process.go:200-234, :374-384) ----
    def buffer_admit(self, cur_round: int, buffer: Sequence[Tuple[Tuple[int, int], Sequence[Tuple[int, int]]]]
                     ) -> np.ndarray:
        """One pass of the buffer loop: buffer = [(id, predecessors)] in buffer order.
        Returns admit[i] (uint8): 1 where the reference appends vertex i to the DAG."""
        q = len(buffer)
        ids = np.asarray([v for v, _ in buffer] if q else [(0, 0)], dtype=np.int32).reshape(-1)
        off = np.zeros(q + 1, np.uint32)
        flat = []
        for i, (_, pr) in enumerate(buffer):
            flat.extend(pr)
            off[i + 1] = len(flat)
        preds = np.asarray(flat if flat else [(0, 0)], dtype=np.int32).reshape(-1)
        admit = np.zeros(max(q, 1), np.uint8)
        self._check(self._L.dr_buffer_admit(self._h, cur_round, q, L.ptr(ids), L.ptr(off), L.ptr(preds),
                                            L.ptr(admit)))
        return admit[:q]

    # ---- waveReady (process.go:314-354) ----
    def wave_commit(self, w0: int, w1: int):
        nw = w1 - w0 + 1
        cm = np.zeros(max(nw, 1), np.uint8)
        vc = np.zeros(max(nw, 1), np.int32)
        self._check(self._L.dr_wave_commit(self._h, w0, w1, L.ptr(cm), L.ptr(vc)))
        return cm[:nw], vc[:nw]

    def wave_ready(self, wave: int, decided_wave: int):
        cm = np.zeros(1, np.uint8)
        vc = np.zeros(1, np.int32)
        cap = max(wave + 1, 1)
        pw = np.zeros(cap, np.int32)
        npush = C.c_int()
        self._check(self._L.dr_wave_ready(self._h, wave, decided_wave, L.ptr(cm), L.ptr(vc), L.ptr(pw), cap,
                                          C.byref(npush)))
        return bool(cm[0]), int(vc[0]), [int(x) for x in pw[:npush.value]]

    # ---- orderVertices (process.go:404-443) ----
    def order_vertices(self, stack: Sequence[Tuple[int, int]], cur_round: int, mode: int = L.DR_DELIVER_REF,
                       cap: int = 1 << 20):
        """Delivered ids [k, 2] (None with cap=0: counts and digests only), per-pop counts, digests."""
        ns = len(stack)
        st = np.asarray(stack if ns else [(0, 0)], dtype=np.int32).reshape(-1)
        ids = np.zeros(max(cap, 1) * 2, np.int32) if cap else None
        out_n = C.c_size_t()
        pc = np.zeros(max(ns, 1), np.uint64)
        pd = np.zeros(max(ns, 1), np.uint64)
        self._check(self._L.dr_order_vertices(self._h, L.ptr(st), ns, cur_round, mode, L.ptr(ids), cap,
                                              C.byref(out_n), L.ptr(pc), L.ptr(pd)))
        k = out_n.value
        return (ids[:2 * k].reshape(-1, 2) if cap else None), pc[:ns], pd[:ns]

    # ---- whole replay ----
    def replay(self, nwaves: int, chain_mode: int = L.DR_CHAIN_PERSISTENT, deliver_mode: int = L.DR_DELIVER_REF,
               ids_cap: int = 0, push_cap: Optional[int] = None) -> ReplayResult:
        """The Alg. 3 wiring the reference lacks: waveReady(w) for w = 1..nwaves, orderVertices on commit."""
        o, keep = _replay_out(nwaves, chain_mode, ids_cap, push_cap)
        self._check(self._L.dr_replay(self._h, nwaves, chain_mode, deliver_mode, C.byref(o)))
        return _replay_result(o, keep, ids_cap)


@functools.lru_cache(maxsize=64)
def _out_layout(nwaves: int, push_cap: int, ids_cap: int):
    """(name, dtype, byte offset, byte size) of every dr_replay output inside one buffer,
    ordered so each array is aligned to its itemsize."""
    pc = max(push_cap, 1)
    spec = (("pc", np.uint64, pc), ("pdg", np.uint64, pc), ("pe", np.uint64, pc), ("vc", np.int32, nwaves),
            ("po", np.uint32, nwaves + 1), ("pw", np.int32, pc), ("ids", np.int32, 2 * ids_cap),
            ("cm", np.uint8, nwaves))
    out, off = [], 0
    for name, t, k in spec:
        nb = np.dtype(t).itemsize * k
        out.append((name, t, off, nb))
        off += nb
    return tuple(out), off + 8


def _replay_out(nwaves: int, chain_mode: int, ids_cap: int = 0, push_cap: Optional[int] = None, buf=None):
    """Output arrays of one dr_replay, carved from a single allocation: a C4 step is
    ~0.25 ms on the GPU, and nine separate arrays plus nine ctypes pointer conversions
    cost ~45 us of Python per call.  buf: carve from the caller's buffer instead (at
    least _replay_out_bytes long)."""
    push_cap = push_cap if push_cap is not None else _default_push_cap(nwaves, chain_mode)
    layout, total = _out_layout(nwaves, push_cap, ids_cap)
    if buf is None:
        buf = np.zeros(total, np.uint8)
    base = buf.ctypes.data
    keep, a = {"_buf": buf}, {}
    for name, t, off, nb in layout:
        keep[name] = buf[off:off + nb].view(t)
        a[name] = base + off
    if not ids_cap:
        keep["ids"], a["ids"] = None, None
    o = L.ReplayOut(a["cm"], a["vc"], a["po"], a["pw"], push_cap, a["pc"], a["pdg"], a["pe"], a["ids"], ids_cap)
    return o, keep


def _default_push_cap(nwaves: int, chain_mode: int) -> int:
    return nwaves * (nwaves + 1) // 2 if chain_mode == L.DR_CHAIN_LITERAL else 2 * nwaves + 1


def _replay_out_bytes(nwaves: int, chain_mode: int, ids_cap: int = 0) -> int:
    return _out_layout(nwaves, _default_push_cap(nwaves, chain_mode), ids_cap)[1]


def _replay_result(o, keep, ids_cap: int = 0) -> ReplayResult:
    k = o.n_push
    ids = keep["ids"]
    return ReplayResult(keep["cm"], keep["vc"], keep["po"], keep["pw"][:k], keep["pc"][:k], keep["pdg"][:k],
                        keep["pe"][:k], None if ids is None else ids[:2 * min(o.n_ids, ids_cap)].reshape(-1, 2),
                        o.commit_edges, o.chain_edges, o.deliver_edges,
                        dict(commit=o.ms_commit, chain=o.ms_chain, deliver=o.ms_deliver, emit=o.ms_emit,
                             summary=o.ms_summary),
                        dict(count=o.sweep_count, partial=o.sweep_partial, row_bytes=o.sweep_row_bytes,
                             weak_scanned=o.sweep_weak_scanned, shortcut=o.sweep_shortcut,
                             canon_segments=o.canon_segments))


class Replayer:
    """dr_replay of one engine into output buffers allocated once (Engine.replay allocates
    per call, ~20-45 us of Python that a 0.25 ms C4 step cannot hide).  result() returns
    views of those buffers: the next call overwrites them."""

    def __init__(self, eng: "Engine", nwaves: int, chain_mode: int = L.DR_CHAIN_PERSISTENT,
                 deliver_mode: int = L.DR_DELIVER_REF, ids_cap: int = 0):
        self._eng, self._ids_cap = eng, ids_cap
        self._o, self._keep = _replay_out(nwaves, chain_mode, ids_cap)
        self._fn, self._args = eng._L.dr_replay, (eng._h, nwaves, chain_mode, deliver_mode, C.byref(self._o))

    def __call__(self) -> None:
        rc = self._fn(*self._args)
        if rc != L.DR_OK:
            self._eng._check(rc)

    @property
    def ms_summary(self) -> float:
        return self._o.ms_summary

    def result(self) -> ReplayResult:
        return _replay_result(self._o, self._keep, self._ids_cap)


class ReplayBatch:
    """dr_replay_batch over a fixed list of engines: output buffers are allocated once and
    reused by every call (the C5 bench replays the same batch many times)."""

    def __init__(self, engines: Sequence["Engine"], nwaves: int, chain_mode: int = L.DR_CHAIN_PERSISTENT,
                 deliver_mode: int = L.DR_DELIVER_REF):
        self.engines = list(engines)
        self.nwaves, self.chain_mode, self.deliver_mode = nwaves, chain_mode, deliver_mode
        n = len(self.engines)
        self._ctxs = (L.P * n)(*[e._h for e in self.engines])
        self._outs = (L.ReplayOut * n)()
        self._keep = []
        # every context's outputs in one allocation, in context order: dr_replay_batch
        # unpacks thousands of small result arrays per call (C5: 4096), and contiguous
        # destinations keep that a sequential write
        stride = (_replay_out_bytes(nwaves, chain_mode) + 63) // 64 * 64
        self._buf = np.zeros(max(1, n) * stride, np.uint8)
        for i in range(n):
            o, keep = _replay_out(nwaves, chain_mode, buf=self._buf[i * stride:(i + 1) * stride])
            self._outs[i] = o
            self._keep.append(keep)

    def run(self) -> None:
        L0 = L.lib()
        rc = L0.dr_replay_batch(self._ctxs, len(self.engines), self.nwaves, self.chain_mode, self.deliver_mode,
                                self._outs)
        if rc != L.DR_OK:
            raise L.DrError(rc, L0.dr_last_error(self.engines[0]._h).decode())

    def results(self) -> List[ReplayResult]:
        return [_replay_result(self._outs[i], self._keep[i]) for i in range(len(self.engines))]

    def __call__(self) -> List[ReplayResult]:
        self.run()
        return self.results()

    def host_phases(self) -> dict:
        """dr_last_batch_phases of the last run: host prep, launch -> host, copy back, unpack (ms)."""
        ms = (C.c_float * 4)()
        L.lib().dr_last_batch_phases(self.engines[0]._h, ms)
        return dict(host_prep=ms[0], launch_to_host=ms[1], copy_back=ms[2], unpack=ms[3])

    def form(self) -> str:
        """dr_last_batch_form of the last run: the fused kernel that ran ("" when none did)."""
        f = L.lib().dr_last_batch_form(self.engines[0]._h)
        return {L.DR_BATCH_WORKGROUP: "k_replay_small", L.DR_BATCH_WAVE: "k_replay_small_1w"}.get(f, "")


class ReplayBatchView:
    """dr_replay_batch_view over a fixed list of engines: each call leaves every context's
    results where the batch's single copy back put them (no per-context copies);
    results() wraps them as numpy views, valid until the next call."""

    def __init__(self, engines: Sequence["Engine"], nwaves: int, chain_mode: int = L.DR_CHAIN_PERSISTENT,
                 deliver_mode: int = L.DR_DELIVER_REF, push_cap: Optional[int] = None):
        self.engines = list(engines)
        self.nwaves, self.chain_mode, self.deliver_mode = nwaves, chain_mode, deliver_mode
        n = len(self.engines)
        self._ctxs = (L.P * n)(*[e._h for e in self.engines])
        self._views = (L.ReplayView * n)()
        if push_cap is None:
            push_cap = nwaves if chain_mode == L.DR_CHAIN_PERSISTENT else nwaves * (nwaves + 1) // 2
        self.push_cap = push_cap

    def run(self) -> None:
        L0 = L.lib()
        rc = L0.dr_replay_batch_view(self._ctxs, len(self.engines), self.nwaves, self.chain_mode,
                                     self.deliver_mode, self.push_cap, self._views)
        if rc != L.DR_OK:
            raise L.DrError(rc, L0.dr_last_error(self.engines[0]._h).decode())

    def results(self) -> List[ReplayResult]:
        nw, out = self.nwaves, []
        for v in self._views:
            k = int(v.n_push)

            def arr(p, dt, m):
                return np.ctypeslib.as_array(C.cast(p, C.POINTER(dt)), shape=(max(m, 1),))[:m]
            out.append(ReplayResult(arr(v.commit, C.c_uint8, nw), arr(v.vcount, C.c_int32, nw),
                                    arr(v.push_off, C.c_uint32, nw + 1), arr(v.push_wave, C.c_int32, k),
                                    arr(v.pop_count, C.c_uint64, k), arr(v.pop_digest, C.c_uint64, k),
                                    arr(v.pop_edges, C.c_uint64, k), None, v.commit_edges, v.chain_edges,
                                    v.deliver_edges, dict(commit=0.0, chain=0.0, deliver=v.ms_deliver, emit=0.0,
                                                          summary=0.0),
                                    {}))
        return out

    def host_phases(self) -> dict:
        """dr_last_batch_phases of the last run: host prep, launch -> host, copy back, unpack (ms)."""
        ms = (C.c_float * 4)()
        L.lib().dr_last_batch_phases(self.engines[0]._h, ms)
        return dict(host_prep=ms[0], launch_to_host=ms[1], copy_back=ms[2], unpack=ms[3])

    def form(self) -> str:
        """dr_last_batch_form of the last run: the fused kernel that ran ("" when none did)."""
        f = L.lib().dr_last_batch_form(self.engines[0]._h)
        return {L.DR_BATCH_WORKGROUP: "k_replay_small", L.DR_BATCH_WAVE: "k_replay_small_1w"}.get(f, "")


def replay_batch(engines: Sequence["Engine"], nwaves: int, chain_mode: int = L.DR_CHAIN_PERSISTENT,
                 deliver_mode: int = L.DR_DELIVER_REF) -> List[ReplayResult]:
    """dr_replay_batch: every engine's dr_replay, as one fused launch when the DAGs are small."""
    return ReplayBatch(engines, nwaves, chain_mode, deliver_mode)()
