"""Wave-range split of the all-waves commit sweep.

waveReady's commit decision for wave w (``process/process.go:326-339``) reads only
rounds 4w-3 .. 4w: the leader's round (``getWaveVertexLeader``, ``:357-371``) and the
three rounds whose strong edges carry the votes.  Waves are therefore independent
units: a contiguous wave range [w0, w1] needs rounds 4(w0-1) .. 4 w1 and nothing
else, so a GPU can hold only its range and decide its waves with no exchange.

``wave_slice`` cuts that window out of a packed DAG as a DAG of its own (round
4(w0-1) becomes round 0, keeping only its slots -- its rows point below the window
and are never read by the commit rule; weak edges are dropped: the rule follows
strong edges only).  Wave w of the full DAG is wave w - w0 + 1 of the slice, so a
non-constant leader coin (``chooseLeader``, ``:386-392``) is handed over shifted:
``slice_leaders``.

``split_commit`` decides every wave of a DAG rank by rank (one ``Engine`` per
range, as one process per GPU would) and concatenates the answers; the result is
``dr_wave_commit`` over the whole DAG, bit for bit.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np

from .dag import PackedDag


def wave_ranges(nwaves: int, world: int) -> List[Tuple[int, int]]:
    """Contiguous 1-based wave ranges [w0, w1], one per rank (sizes differ by <= 1)."""
    if world < 1 or nwaves < world:
        raise ValueError(f"cannot split {nwaves} waves over {world} ranks")
    return [(r * nwaves // world + 1, (r + 1) * nwaves // world) for r in range(world)]


def wave_slice(d: PackedDag, w0: int, w1: int) -> PackedDag:
    """Rounds 4(w0-1) .. 4 w1 of ``d`` shifted to 0 .. 4(w1-w0+1): everything the commit
    decisions of waves w0..w1 read (round 0 of the slice keeps its slots, no edges)."""
    n, W = d.n, d.W
    lo, hi = 4 * (w0 - 1), 4 * w1
    if w0 < 1 or w1 < w0 or hi >= d.nrounds:
        raise ValueError(f"waves [{w0}, {w1}] need rounds {lo}..{hi}, the DAG has 0..{d.nrounds - 1}")
    so = d.slot_off[lo:hi + 2].astype(np.int64)
    strong = d.strong[lo * n * W:(hi + 1) * n * W].copy()
    strong[:n * W] = 0
    k = hi - lo + 1
    return PackedDag(n, k, (so - so[0]).astype(np.uint32), d.slot_src[so[0]:so[-1]].copy(), strong,
                     np.zeros(k * n + 1, np.uint32), np.zeros(0, np.uint32))


def slice_leaders(leaders: Optional[Sequence[int]], w0: int, w1: int) -> Optional[List[int]]:
    """A leader table (leaders[w-1] = chooseLeader(w), 1 beyond its end) re-based to the
    slice's wave numbers; None stays None (the reference's constant coin)."""
    if leaders is None:
        return None
    return [int(leaders[w - 1]) if w - 1 < len(leaders) else 1 for w in range(w0, w1 + 1)]


def split_commit(d: PackedDag, faulty: int, nwaves: int, world: int, device: int = 0,
                 leaders: Optional[Sequence[int]] = None):
    """Every wave's commit decision, computed per wave range on its own mirror (one
    ``Engine`` per range, one after another on ``device``); returns (commit, vcount,
    ranges)."""
    from .engine import Engine
    from . import _lib as L

    commit, vcount = [], []
    ranges = wave_ranges(nwaves, world)
    for w0, w1 in ranges:
        sub = wave_slice(d, w0, w1)
        with Engine(d.n, faulty, sub.nrounds, device) as e:
            e.append_packed(sub)
            tab = slice_leaders(leaders, w0, w1)
            if tab is not None:
                e.set_leader_coin(L.DR_LEADER_TABLE, table=tab)
            cm, vc = e.wave_commit(1, w1 - w0 + 1)
        commit.append(cm.copy())
        vcount.append(vc.copy())
    return np.concatenate(commit), np.concatenate(vcount), ranges


# ---------------------------------------------------------------------------
# The whole replay split into wave ranges (SURVEY.md s8(e) row 1
# widened from the commit sweep to waveReady + orderVertices, process.go:314-354,
# :404-443).  Rank k of N owns waves [w0, w1] and mirrors the global rounds
# [off, top] as a DAG of its own (``replay_slice_dag``):
#
#   - below: ``halo`` whole waves under w0 (rank 0: none), so every owned commit's leader
#     chain (persistent decidedWave: down to the previous commit) and every pop sweep of
#     an owned commit (down to its merge with the canonical cone K) stay inside; weak
#     edges of the lowest rounds that point below ``off`` are dropped -- the lowest
#     ``dmax`` slice rounds are a landing zone whose edge counts are never used (checked:
#     every owned pop merges at or above slice round dmax);
#   - above: ``dmax`` rounds past 4 w1 (the top rank: up to the DAG's top), whose strong
#     rows and weak columns feed K^cand of the owned rounds.  They are "seeded" full
#     (dr_set_slice seeded_top: K covers every present vertex there), which is exact when
#     the rank above finds K full on its own lowest dmax rounds -- the rounds that feed
#     the owned ones (the window check below).  Two canonical cones whose reach sets
#     cover the present vertices of the same dmax consecutive rounds agree on every
#     round below (every contribution to round m-1 comes from rounds m .. m+dmax-1,
#     DESIGN.md s3.2).
#
# The device replay of a slice (dr_replay with dr_set_slice) gives digests keyed by
# global rounds and positions counted from pos_base = the global canonical count of
# rounds 1..off (guessed as the presence prefix, checked after the exchange), so its
# pop counts are global and its digests / edges are global up to one additive offset
# per rank.  One all-gather of 13 words per rank (``SliceSummary``) supplies the
# offsets and every rank's checks:
#
#   Coff_k = sum_{j<k} C_own_j        (C_own: canonical count over the owned rounds)
#   Goff_k = sum_{j<k} G_own_j - G_k(lo_k - 1)   (G_k: the slice's digest prefix)
#   Eoff_k = sum_{j<k} E_own_j - E_k(lo_k - 1)
#   pos_base_k must equal Coff_k - (C_k(lo_k - 1) - pos_base_k)   (else: one re-run)
#
# and ``combine_slices`` concatenates the owned waves' outputs: the whole replay, bit
# for bit.
# ---------------------------------------------------------------------------
import dataclasses


class SliceError(RuntimeError):
    """A slice whose halo does not hold what its owned waves need (a chain or pop
    reaching below it, a canonical cone not full at a rank boundary): the split does not
    apply to this DAG with these halos."""


@dataclasses.dataclass(frozen=True)
class SlicePlan:
    rank: int
    world: int
    w0: int          # owned global waves [w0, w1]
    w1: int
    wf: int          # the slice's first wave (global): slice wave 1
    off: int         # global round of slice round 0 (= 4 (wf - 1))
    top: int         # global top round of the slice
    dmax: int        # the DAG's largest weak delta (the canonical window)

    @property
    def nrounds(self) -> int:
        return self.top - self.off + 1

    @property
    def nwaves(self) -> int:  # slice waves replayed: 1 .. own top
        return self.w1 - self.wf + 1

    @property
    def own_w0(self) -> int:  # first owned slice wave
        return self.w0 - self.wf + 1

    @property
    def lo(self) -> int:  # first owned global round
        return 4 * (self.w0 - 1) + 1

    @property
    def hi(self) -> int:  # last owned global round
        return 4 * self.w1

    @property
    def seeded(self) -> int:  # rounds above the owned ones taken as full (not the top rank)
        return 0 if self.rank == self.world - 1 else self.top - self.hi

    def probes(self):
        """Slice rounds whose C, G, E the replay reports: lo-1, hi, lo+dmax-1 (the owned
        rounds' bounds and the bottom window the rank below was seeded with)."""
        return [self.lo - 1 - self.off, self.hi - self.off, min(self.lo + self.dmax - 1, self.hi) - self.off]


def weak_dmax(d: PackedDag) -> int:
    """Largest weak delta r - r' of the DAG (1: no weak edge)."""
    if len(d.weak_tgt) == 0:
        return 1
    n = d.n
    cnt = np.diff(d.weak_off.astype(np.int64))
    vr = np.repeat(np.arange(d.nrounds * n, dtype=np.int64) // n, cnt)
    tr = (d.weak_tgt.astype(np.int64) >> 11) & 0xFFFFF
    return max(1, int((vr - tr).max()))


def slice_plans(d: PackedDag, nwaves: int, world: int, halo: int = 8, dmax: Optional[int] = None) -> List[SlicePlan]:
    """Every rank's slice of an nwaves replay of d: owned wave ranges as wave_ranges,
    ``halo`` waves below each (rank 0: from wave 1) and dmax rounds above (the top rank:
    the DAG's top)."""
    if np.any(d.weak_tgt >> 31):
        raise SliceError("strong edges outside r-1 (App. A Q8): the wave split takes regular DAGs only")
    dm = weak_dmax(d) if dmax is None else dmax
    T = d.nrounds - 1
    out = []
    for k, (w0, w1) in enumerate(wave_ranges(nwaves, world)):
        wf = max(1, w0 - halo)
        top = T if k == world - 1 else min(T, 4 * w1 + dm)
        out.append(SlicePlan(k, world, w0, w1, wf, 4 * (wf - 1), top, dm))
    return out


def replay_slice_dag(d: PackedDag, p: SlicePlan) -> PackedDag:
    """Global rounds [p.off, p.top] of d as a DAG of their own: rounds shifted by -off,
    round 0's rows cleared, weak edges that point below off dropped."""
    n, W = d.n, d.W
    lo, hi = p.off, p.top
    so = d.slot_off[lo:hi + 2].astype(np.int64)
    strong = d.strong[lo * n * W:(hi + 1) * n * W].copy()
    strong[:n * W] = 0
    k = hi - lo + 1
    wo = d.weak_off[lo * n:(hi + 1) * n + 1].astype(np.int64)
    tg = d.weak_tgt[wo[0]:wo[-1]].astype(np.int64)
    tr = (tg >> 11) & 0xFFFFF
    keep = tr >= lo
    cnt = np.diff(wo)
    owner = np.repeat(np.arange(k * n), cnt)
    new_cnt = np.bincount(owner[keep], minlength=k * n)
    new_off = np.zeros(k * n + 1, np.int64)
    np.cumsum(new_cnt, out=new_off[1:])
    tgt = (((tr[keep] - lo) << 11) | (tg[keep] & 2047)).astype(np.uint32)
    return PackedDag(n, k, (so - so[0]).astype(np.uint32), d.slot_src[so[0]:so[-1]].copy(), strong,
                     new_off.astype(np.uint32), tgt)


def presence_prefix(d: PackedDag) -> np.ndarray:
    """[round] present (non-ghost) slots of rounds 1..r, the engine's ppref."""
    nz = np.add.reduceat((d.slot_src != 0).astype(np.int64), d.slot_off[:-1].astype(np.int64)) \
        if len(d.slot_src) else np.zeros(d.nrounds, np.int64)
    nz = np.where(np.diff(d.slot_off.astype(np.int64)) > 0, nz, 0)
    nz[0] = 0
    return np.cumsum(nz)


def round_strong_degrees(d: PackedDag, r0: int, r1: int) -> np.ndarray:
    """Strong degree sum of each round in [r0, r1] (popcount of the rows)."""
    n, W = d.n, d.W
    rows = d.strong[r0 * n * W:(r1 + 1) * n * W].reshape(r1 - r0 + 1, n * W)
    return np.bitwise_count(rows).sum(axis=1, dtype=np.int64)


# per-rank words of the exchange (one all-gather)
SUMMARY_FIELDS = ("C_own", "G_own", "E_own", "C_lo1", "G_lo1", "E_lo1", "pos_base", "window_full", "min_stop",
                  "chain_ok", "own_chain_edges", "n_pops", "commit_edges")


def slice_summary(p: SlicePlan, sd: PackedDag, res, sres: dict, pos_base: int) -> np.ndarray:
    """This rank's exchange words (SUMMARY_FIELDS, uint64) from its slice replay."""
    C, G, E = sres["C"], sres["G"], sres["E"]
    m = 2**64
    pp = presence_prefix(sd)
    a, b, c = p.probes()
    # the owned rounds' lowest dmax rounds hold every present vertex in K (the rank
    # below was seeded with them): C over them equals the presence count
    window_full = int(C[2] - C[0] == pp[c] - pp[a])
    own = p.own_w0
    cm = np.asarray(res.commit)
    owned_commits = np.nonzero(cm[own - 1:])[0]
    chain_ok = 1
    if p.off > 0 and len(owned_commits):
        first = own + int(owned_commits[0])  # slice wave
        chain_ok = int(bool(cm[:first - 1].any()))  # its persistent floor lies inside the slice
    n_pops = int(res.push_off[p.nwaves]) - int(res.push_off[own - 1])
    vc = np.asarray(res.vcount)
    deg = round_strong_degrees(sd, 4 * (own - 1) + 1, 4 * p.nwaves)
    ce = 0
    for w in range(own, p.nwaves + 1):
        if vc[w - 1] >= 0:
            base = 4 * (w - 1) + 1 - 4 * (own - 1) - 1
            ce += int(deg[base + 1] + deg[base + 2] + deg[base + 3])
    vals = [(C[1] - C[0]) % m, (G[1] - G[0]) % m, (E[1] - E[0]) % m, C[0], G[0], E[0], pos_base, window_full,
            sres["min_stop"] % m, chain_ok, sres["own_chain_edges"], n_pops, ce]
    return np.asarray([int(v) % m for v in vals], dtype=np.uint64)


def check_and_offsets(plans: Sequence[SlicePlan], summaries: np.ndarray):
    """From every rank's exchange words ([world][13] uint64): the per-rank (Goff, Eoff)
    and the ranks whose pos_base guess was wrong, with the right base; raises SliceError
    when a halo assumption fails."""
    S = {f: summaries[:, i] for i, f in enumerate(SUMMARY_FIELDS)}
    m = 2**64
    offs, redo = [], {}
    cC = cG = cE = 0
    for k, p in enumerate(plans):
        if k + 1 < len(plans) and not int(S["window_full"][k + 1]):
            raise SliceError(f"rank {k + 1}: the canonical cone is not full on its lowest {p.dmax} rounds "
                             f"(rank {k}'s seeded top)")
        ms = int(summaries[:, SUMMARY_FIELDS.index("min_stop")].view(np.int64)[k])  # (two's complement)
        if p.off > 0 and ms < p.dmax:  # (rank 0's slice starts at the DAG's round 0: nothing below)
            raise SliceError(f"rank {k}: a pop of an owned commit merges at slice round {ms} < {p.dmax} "
                             f"(more halo waves needed)")
        if not int(S["chain_ok"][k]):
            raise SliceError(f"rank {k}: no commit in the halo below its first owned commit (its leader chain "
                             f"floor lies below the slice)")
        want = (cC - int(S["C_lo1"][k]) + int(S["pos_base"][k])) % m
        if want != int(S["pos_base"][k]):
            redo[k] = want
        offs.append(((cG - int(S["G_lo1"][k])) % m, (cE - int(S["E_lo1"][k])) % m))
        cC, cG, cE = (cC + int(S["C_own"][k])) % m, (cG + int(S["G_own"][k])) % m, (cE + int(S["E_own"][k])) % m
    return offs, redo


def owned_part(p: SlicePlan, res, goff: int, eoff: int) -> dict:
    """The owned waves' outputs of a slice replay, in global numbering, offsets applied."""
    own, nw = p.own_w0, p.nwaves
    a, b = int(res.push_off[own - 1]), int(res.push_off[nw])
    m = np.uint64(0xFFFFFFFFFFFFFFFF)
    return dict(
        commit=np.asarray(res.commit[own - 1:nw]).copy(),
        vcount=np.asarray(res.vcount[own - 1:nw]).copy(),
        push_len=np.diff(np.asarray(res.push_off[own - 1:nw + 1], np.int64)),
        push_wave=(np.asarray(res.push_wave[a:b], np.int64) + (p.wf - 1)).astype(np.int32),
        pop_count=np.asarray(res.pop_count[a:b], np.uint64).copy(),
        pop_digest=(np.asarray(res.pop_digest[a:b], np.uint64) + np.uint64(goff)) & m,
        pop_edges=(np.asarray(res.pop_edges[a:b], np.uint64) + np.uint64(eoff)) & m,
    )


def combine_slices(parts: Sequence[dict], summaries: np.ndarray):
    """Concatenate every rank's owned part (owned_part) into the whole replay's outputs:
    a ReplayResult-like namespace (commit, vcount, push_off, push_wave, pop_count,
    pop_digest, pop_edges, commit_edges, chain_edges, deliver_edges)."""
    from types import SimpleNamespace

    S = {f: summaries[:, i] for i, f in enumerate(SUMMARY_FIELDS)}
    cat = lambda k: np.concatenate([pt[k] for pt in parts])  # noqa: E731
    push_len = cat("push_len")
    push_off = np.zeros(len(push_len) + 1, np.uint32)
    np.cumsum(push_len, out=push_off[1:])
    pe = cat("pop_edges")
    with np.errstate(over="ignore"):
        de = int(pe.sum(dtype=np.uint64))
    return SimpleNamespace(commit=cat("commit"), vcount=cat("vcount"), push_off=push_off, push_wave=cat("push_wave"),
                           pop_count=cat("pop_count"), pop_digest=cat("pop_digest"), pop_edges=pe,
                           commit_edges=int(S["commit_edges"].sum(dtype=np.uint64)),
                           chain_edges=int(S["own_chain_edges"].sum(dtype=np.uint64)), deliver_edges=de)


class SliceRank:
    """One rank's slice engine: the mirror of its rounds, configured once; replay()
    returns (ReplayResult, slice_result).  guess_base: pos_base from the global presence
    prefix (the exchange checks it; rebase() re-runs with the right one)."""

    def __init__(self, d: PackedDag, p: SlicePlan, faulty: int, device: int = 0,
                 leaders: Optional[Sequence[int]] = None, global_ppref: Optional[np.ndarray] = None):
        from .engine import Engine, Replayer
        from . import _lib as L

        self.p = p
        self.sd = replay_slice_dag(d, p)
        self.eng = Engine(d.n, faulty, self.sd.nrounds, device)
        self.eng.append_packed(self.sd)
        tab = slice_leaders(leaders, p.wf, p.w1 + (p.top - p.hi + 3) // 4 + 1)
        if tab is not None:
            self.eng.set_leader_coin(L.DR_LEADER_TABLE, table=tab)
        gp = presence_prefix(d) if global_ppref is None else global_ppref
        self.pos_base = int(gp[p.off]) if p.off > 0 else 0
        self._configure()
        self.step = Replayer(self.eng, p.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF)

    def _configure(self):
        p = self.p
        self.eng.set_slice(round_offset=p.off, pos_base=self.pos_base, seeded_top=p.seeded, own_w0=p.own_w0,
                           probes=p.probes())

    def rebase(self, pos_base: int):
        self.pos_base = int(pos_base)
        self._configure()

    def replay(self):
        self.step()
        return self.step.result(), self.eng.slice_result()

    def summary(self, res, sres) -> np.ndarray:
        return slice_summary(self.p, self.sd, res, sres, self.pos_base)

    def close(self):
        self.eng.close()


def split_replay(d: PackedDag, faulty: int, nwaves: int, world: int, device: int = 0, halo: int = 8,
                 leaders: Optional[Sequence[int]] = None):
    """The whole replay (persistent chains, REF delivery) rank by rank on one device, as N
    processes would run it (one slice engine each), with the exchange done in memory:
    returns (combined result, plans, per-rank summaries)."""
    plans = slice_plans(d, nwaves, world, halo)
    gp = presence_prefix(d)
    ranks = [SliceRank(d, p, faulty, device, leaders, gp) for p in plans]
    try:
        outs = [r.replay() for r in ranks]
        summ = np.stack([r.summary(*o) for r, o in zip(ranks, outs)])
        offs, redo = check_and_offsets(plans, summ)
        if redo:  # a wrong position-base guess (a rank below had a non-full canonical round): re-run those
            for k, base in redo.items():
                ranks[k].rebase(base)
                outs[k] = ranks[k].replay()
                summ[k] = ranks[k].summary(*outs[k])
            offs, redo = check_and_offsets(plans, summ)
            assert not redo
        parts = [owned_part(p, o[0], *off) for p, o, off in zip(plans, outs, offs)]
        return combine_slices(parts, summ), plans, summ
    finally:
        for r in ranks:
            r.close()


# ---------------------------------------------------------------------------
# The exchange between processes (one rank per GPU): one all-gather of the 13
# summary words, each rank's offsets applied on that rank, one all-gather of the
# owned parts (padded to the longest; rank 0 keeps them).  dist: torch.distributed
# (nccl = RCCL on GPU tensors, gloo on CPU tensors), dev: the tensors' device.
# ---------------------------------------------------------------------------
def dist_exchange(dist, summary: np.ndarray, world: int, dev) -> np.ndarray:
    import torch

    mine = torch.from_numpy(summary.view(np.int64).copy()).to(dev)
    out = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(out, mine)
    return np.stack([t.cpu().numpy() for t in out]).view(np.uint64)


def _pack_part(part: dict) -> np.ndarray:
    return np.concatenate([part["commit"].astype(np.int64), part["vcount"].astype(np.int64),
                           part["push_len"].astype(np.int64), part["push_wave"].astype(np.int64),
                           part["pop_count"].view(np.int64), part["pop_digest"].view(np.int64),
                           part["pop_edges"].view(np.int64)])


def _unpack_part(buf: np.ndarray, nwo: int, npop: int) -> dict:
    o = [0]

    def take(k):
        x = buf[o[0]:o[0] + k]
        o[0] += k
        return x

    return dict(commit=take(nwo).astype(np.uint8), vcount=take(nwo).astype(np.int32), push_len=take(nwo).copy(),
                push_wave=take(npop).astype(np.int32), pop_count=take(npop).view(np.uint64).copy(),
                pop_digest=take(npop).view(np.uint64).copy(), pop_edges=take(npop).view(np.uint64).copy())


def dist_gather_parts(dist, part: dict, plans: Sequence[SlicePlan], summaries: np.ndarray, rank: int, dev):
    """Every rank's owned part on rank 0 (None elsewhere): one all-gather of the packed
    parts, padded to the longest (the lengths come from the exchange words)."""
    import torch

    npops = summaries[:, SUMMARY_FIELDS.index("n_pops")].astype(np.int64)
    nwos = np.asarray([p.w1 - p.w0 + 1 for p in plans], np.int64)
    L = int((3 * nwos + 4 * npops).max())
    buf = np.zeros(L, np.int64)
    pk = _pack_part(part)
    buf[:len(pk)] = pk
    mine = torch.from_numpy(buf).to(dev)
    out = [torch.empty_like(mine) for _ in plans]
    dist.all_gather(out, mine)
    if rank != 0:
        return None
    return [_unpack_part(t.cpu().numpy(), int(nw), int(npop)) for t, nw, npop in zip(out, nwos, npops)]


def dist_split_step(dist, sr: "SliceRank", plans: Sequence[SlicePlan], dev, outs=None):
    """One wave-split replay across the ranks of dist: this rank's slice replay (or the
    given outs), the exchange, a re-run of this rank if its position base was wrong, its
    offsets, and the gather.  Returns (combined result on rank 0 else None, summaries)."""
    world = len(plans)
    res, sres = outs if outs is not None else sr.replay()
    summ = dist_exchange(dist, sr.summary(res, sres), world, dev)
    offs, redo = check_and_offsets(plans, summ)
    if redo:  # every rank takes part in the second exchange
        if sr.p.rank in redo:
            sr.rebase(redo[sr.p.rank])
            res, sres = sr.replay()
        summ = dist_exchange(dist, sr.summary(res, sres), world, dev)
        offs, redo = check_and_offsets(plans, summ)
        if redo:
            raise SliceError(f"position bases still wrong after one re-run: ranks {sorted(redo)}")
    part = owned_part(sr.p, res, *offs[sr.p.rank])
    parts = dist_gather_parts(dist, part, plans, summ, sr.p.rank, dev)
    return (combine_slices(parts, summ) if parts is not None else None), summ
