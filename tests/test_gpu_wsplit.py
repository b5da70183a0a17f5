"""GPU parity of the whole replay split into wave ranges (SURVEY.md
s8(e) row 1 widened to waveReady + orderVertices, process.go:314-354, :404-443).

Every rank's slice (dag_rider_amd/split.py: its waves, a halo of waves below, the dmax
rounds above it seeded full) replays on a mirror holding only those rounds, one mirror
per rank in one process (what N GPUs do side by side); the exchange words are combined
in memory.  The reassembled replay must equal the whole DAG's -- the committed C4 golden
vectors at N = 2, 4, 8, and the bitset oracle on generated DAGs -- or the split must
refuse with SliceError, never answer wrongly."""
import numpy as np
import pytest

import oracle
from dag_rider_amd import _lib as L
from dag_rider_amd.engine import Engine
from dag_rider_amd.gen import CONFIGS, generate, small_config
from dag_rider_amd.split import SliceError, split_replay
from dagutil import dag_fingerprint, load_large

pytestmark = pytest.mark.gpu


def _same(got, want):
    assert (np.asarray(got.commit) == np.asarray(want.commit)).all()
    assert (np.asarray(got.vcount) == np.asarray(want.vcount)).all()
    assert (np.asarray(got.push_off) == np.asarray(want.push_off)).all()
    assert (np.asarray(got.push_wave) == np.asarray(want.push_wave)).all()
    for k in ("pop_count", "pop_digest", "pop_edges"):
        g, w = np.asarray(getattr(got, k), np.uint64), np.asarray(getattr(want, k), np.uint64)
        bad = np.nonzero(g != w)[0]
        assert len(bad) == 0, f"{k}: {len(bad)} pops differ, first at {bad[:5].tolist()}"
    assert (got.commit_edges, got.chain_edges, got.deliver_edges) == \
        (want.commit_edges, want.chain_edges, want.deliver_edges)


def test_wsplit_c4_golden(gpu_device):
    """C4 (n=1024 x 4000 rounds) split over 2, 4 and 8 ranks == the golden replay."""
    g = load_large()["c4"]["persistent_ref"]
    cfg = CONFIGS["c4"]
    d = generate(cfg, nthreads=16)
    assert dag_fingerprint(d) == load_large()["c4"]["dag"], "generator drift"
    from types import SimpleNamespace

    want = SimpleNamespace(commit=np.asarray([int(c) for c in g["commit"]], np.uint8),
                           vcount=np.asarray(g["vcount"], np.int32), push_off=np.asarray(g["push_off"], np.uint32),
                           push_wave=np.asarray(g["push_wave"], np.int32),
                           pop_count=np.asarray([int(x) for x in g["pop_count"]], np.uint64),
                           pop_digest=np.asarray([int(x) for x in g["pop_digest"]], np.uint64),
                           pop_edges=np.asarray([int(x) for x in g["pop_edges"]], np.uint64),
                           commit_edges=int(g["commit_edges"]), chain_edges=int(g["chain_edges"]),
                           deliver_edges=int(g["deliver_edges"]))
    for world in (2, 4, 8):
        got, plans, _ = split_replay(d, cfg.faulty, cfg.nwaves, world, gpu_device)
        assert len(plans) == world
        _same(got, want)


@pytest.mark.parametrize("seed", range(6))
def test_wsplit_generated(gpu_device, seed):
    """Quorum-shaped DAGs (late vertices, weak edges up to 8 deep, a few absent
    leaders) split over 2, 3 and 5 ranks == the bitset oracle; a split whose halo is too
    short for the DAG raises SliceError instead of answering."""
    rng = np.random.default_rng(7100 + seed)
    n = int(rng.choice([64, 100, 256]))
    cfg = small_config(n, 4 * int(rng.integers(40, 70)), 7100 + seed, p_present=float(rng.uniform(0.95, 1)),
                       p_late=float(rng.uniform(0.0, 0.1)), p_w=float(rng.uniform(0.1, 0.6)),
                       weak_depth=int(rng.integers(2, 9)), p_la=0.02)
    d = generate(cfg)
    want = oracle.PDag(d).replay(cfg.faulty, cfg.nwaves, oracle.CHAIN_PERSISTENT, oracle.DELIVER_REF)
    ran = 0
    for world in (2, 3, 5):
        try:
            got, _, _ = split_replay(d, cfg.faulty, cfg.nwaves, world, gpu_device, halo=6)
        except SliceError:
            continue
        _same(got, want)
        ran += 1
    assert ran >= 1


def test_wsplit_rebase_and_refusals(gpu_device):
    """A DAG whose canonical cone misses vertices in its middle (late vertices nobody
    references): the ranks above guess the position base from the presence prefix, the
    exchange finds the right one and they re-run; the result equals the oracle.  A halo
    of one wave is refused (a chain or pop needs more), never answered wrongly."""
    cfg = small_config(64, 240, 7300, p_present=0.9, p_late=0.3, p_w=0.3, weak_depth=6, p_la=0.1)
    d = generate(cfg)
    want = oracle.PDag(d).replay(cfg.faulty, cfg.nwaves, oracle.CHAIN_PERSISTENT, oracle.DELIVER_REF)
    with Engine(cfg.n, cfg.faulty, d.nrounds, gpu_device) as e:
        e.append_packed(d)
        full = e.replay(cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF)
    _same(full, want)
    outcomes = []
    for world, halo in ((2, 12), (4, 12), (4, 1)):
        try:
            got, _, summ = split_replay(d, cfg.faulty, cfg.nwaves, world, gpu_device, halo=halo)
        except SliceError as ex:
            outcomes.append(("refused", str(ex)))
            continue
        _same(got, want)
        outcomes.append(("ok", None))
    assert any(o[0] == "ok" for o in outcomes), outcomes


def test_wsplit_slice_contract(gpu_device):
    """dr_set_slice: a sliced context answers dr_replay only (REF, persistent chains)."""
    cfg = CONFIGS["c2"]
    d = generate(cfg)
    with Engine(cfg.n, cfg.faulty, d.nrounds, gpu_device) as e:
        e.append_packed(d)
        e.set_slice(round_offset=0, pos_base=0, own_w0=1, probes=[0, 4])
        with pytest.raises(L.DrError) as ei:
            e.path_batch([((8, 1), (7, 1))], True)
        assert ei.value.code == L.DR_E_STATE
        with pytest.raises(L.DrError) as ei:
            e.replay(cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_PAPER)
        assert ei.value.code == L.DR_E_STATE
        # a slice of the whole DAG (offset 0, base 0, nothing seeded) is the whole replay
        got = e.replay(cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF)
        sres = e.slice_result()
        e.set_slice(clear=True)
        want = e.replay(cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF)
        _same(got, want)
        assert sres["own_chain_edges"] == want.chain_edges
        assert sres["C"][0] == 0
