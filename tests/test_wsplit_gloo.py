"""The wave-split replay's reassembly across processes (dag_rider_amd/split.py
dist_split_step) on CPU: world_size 2 over gloo.

Each rank holds the outputs a slice replay would give for its waves -- here made from
the bitset oracle's whole replay of a small generated DAG, with the digests and edge
counts shifted by per-rank offsets that only the exchange words reveal (what a slice's
device replay leaves: global up to one additive offset) -- and one rank starts with a
wrong position-base guess.  The exchange, that rank's re-run, the offsets and the gather
must give rank 0 the whole replay bit for bit."""
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
M = 2**64


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _dag_and_want():
    import oracle
    from dag_rider_amd.gen import generate, small_config

    cfg = small_config(64, 160, 8200, p_present=1.0, p_late=0.05, p_w=0.4, weak_depth=4)
    d = generate(cfg)
    want = oracle.PDag(d).replay(cfg.faulty, cfg.nwaves, oracle.CHAIN_PERSISTENT, oracle.DELIVER_REF)
    return cfg, d, want


class _FakeSlice:
    """A slice rank whose device replay is simulated from the whole replay (the
    arithmetic of dr_set_slice's outputs, not its kernels)."""

    def __init__(self, p, plans, want, rng_seed, wrong_base):
        from dag_rider_amd.split import SUMMARY_FIELDS

        self.p = p
        rng = np.random.default_rng(rng_seed)  # every rank draws every rank's values alike
        world = len(plans)
        self.vals = [dict(C_own=int(rng.integers(1, 1 << 40)), G_own=int(rng.integers(0, 1 << 63)),
                          E_own=int(rng.integers(0, 1 << 40)), X=int(rng.integers(0, 1 << 20)),
                          G_lo1=int(rng.integers(0, 1 << 63)), E_lo1=int(rng.integers(0, 1 << 40)))
                     for _ in range(world)]
        k = p.rank
        self.true_base = (sum(v["C_own"] for v in self.vals[:k]) - self.vals[k]["X"]) % M
        self.pos_base = (self.true_base + 5) % M if wrong_base else self.true_base
        self.goff = (sum(v["G_own"] for v in self.vals[:k]) - self.vals[k]["G_lo1"]) % M
        self.eoff = (sum(v["E_own"] for v in self.vals[:k]) - self.vals[k]["E_lo1"]) % M
        self.want, self.fields = want, SUMMARY_FIELDS
        self.replays = 0

    def replay(self):
        from types import SimpleNamespace

        self.replays += 1
        p, w = self.p, self.want
        po = np.asarray(w.push_off, np.int64)
        a, b = po[p.wf - 1], po[p.w1]
        sub = lambda x, o: ((np.asarray(x, np.uint64)[a:b].astype(object) - o) % M).astype(np.uint64)  # noqa: E731
        res = SimpleNamespace(commit=np.asarray(w.commit)[p.wf - 1:p.w1], vcount=np.asarray(w.vcount)[p.wf - 1:p.w1],
                              push_off=(po[p.wf - 1:p.w1 + 1] - a).astype(np.uint32),
                              push_wave=np.asarray(w.push_wave, np.int64)[a:b] - (p.wf - 1),
                              pop_count=np.asarray(w.pop_count, np.uint64)[a:b],
                              pop_digest=sub(w.pop_digest, self.goff), pop_edges=sub(w.pop_edges, self.eoff))
        return res, None

    def rebase(self, base):
        self.pos_base = int(base)

    def summary(self, res, sres):
        v, k, p = self.vals[self.p.rank], self.p.rank, self.p
        po = np.asarray(self.want.push_off, np.int64)
        n_pops = int(po[p.w1] - po[p.w0 - 1])
        world = len(self.vals)
        share = lambda tot: tot // world + (tot % world if k == world - 1 else 0)  # noqa: E731
        d = dict(C_own=v["C_own"], G_own=v["G_own"], E_own=v["E_own"], C_lo1=(self.pos_base + v["X"]) % M,
                 G_lo1=v["G_lo1"], E_lo1=v["E_lo1"], pos_base=self.pos_base, window_full=1, min_stop=1 << 20,
                 chain_ok=1, own_chain_edges=share(int(self.want.chain_edges)), n_pops=n_pops,
                 commit_edges=share(int(self.want.commit_edges)))
        return np.asarray([d[f] for f in self.fields], np.uint64)


def _worker(rank, world, port, out):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist

    from dag_rider_amd.split import dist_split_step, slice_plans

    dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)
    try:
        cfg, d, want = _dag_and_want()
        plans = slice_plans(d, cfg.nwaves, world, halo=4)
        sr = _FakeSlice(plans[rank], plans, want, 99, wrong_base=(rank == 1))
        got, summ = dist_split_step(dist, sr, plans, "cpu")
        out[rank] = dict(replays=sr.replays, base_ok=sr.pos_base == sr.true_base)
        if rank == 0:
            ok = all([(np.asarray(got.commit) == np.asarray(want.commit)).all(),
                      (np.asarray(got.vcount) == np.asarray(want.vcount)).all(),
                      (np.asarray(got.push_off) == np.asarray(want.push_off)).all(),
                      (np.asarray(got.push_wave) == np.asarray(want.push_wave)).all(),
                      (got.pop_count == np.asarray(want.pop_count, np.uint64)).all(),
                      (got.pop_digest == np.asarray(want.pop_digest, np.uint64)).all(),
                      (got.pop_edges == np.asarray(want.pop_edges, np.uint64)).all(),
                      got.chain_edges == int(want.chain_edges), got.commit_edges == int(want.commit_edges),
                      got.deliver_edges == int(want.deliver_edges)])
            out["ok"] = bool(ok)
    finally:
        dist.destroy_process_group()


def test_wave_split_reassembly_two_ranks_gloo():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    assert out["ok"]
    assert out[0]["replays"] == 1 and out[1]["replays"] == 2  # rank 1 re-ran with the exchanged base
    assert out[0]["base_ok"] and out[1]["base_ok"]


def test_slice_plans_and_dag():
    """Slice geometry on the CPU: owned ranges tile the waves, halos below, dmax rounds
    above (the top rank: the DAG's top), and the slice DAG keeps its rounds' slots, rows
    and the weak edges that stay inside it."""
    sys.path.insert(0, ROOT)
    from dag_rider_amd.split import presence_prefix, replay_slice_dag, slice_plans, weak_dmax

    cfg, d, _ = _dag_and_want()
    dm = weak_dmax(d)
    plans = slice_plans(d, cfg.nwaves, 3, halo=4)
    assert [p.w0 for p in plans][0] == 1 and plans[-1].w1 == cfg.nwaves
    assert all(plans[i].w1 + 1 == plans[i + 1].w0 for i in range(2))
    for p in plans:
        assert p.off == 4 * (p.wf - 1) and p.wf == max(1, p.w0 - 4)
        assert p.top == (d.nrounds - 1 if p.rank == 2 else min(d.nrounds - 1, 4 * p.w1 + dm))
        sd = replay_slice_dag(d, p)
        assert sd.nrounds == p.top - p.off + 1
        n, W = d.n, d.W
        assert not sd.strong[:n * W].any()
        r = p.off + 5
        assert (sd.strong[5 * n * W:6 * n * W] == d.strong[r * n * W:(r + 1) * n * W]).all()
        tr = (sd.weak_tgt.astype(np.int64) >> 11) & 0xFFFFF
        assert (tr >= 0).all() and len(sd.weak_tgt) == int(sd.weak_off[-1])
        pp, gp = presence_prefix(sd), presence_prefix(d)
        assert pp[-1] == gp[p.top] - gp[p.off]
