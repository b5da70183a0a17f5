"""GPU parity of the wave-range commit split (process.go:314-339).

Every rank's slice (dag_rider_amd/split.py) is decided by dr_wave_commit on a mirror
that holds only that slice's rounds, one mirror per rank in one process (what N GPUs
do side by side); the concatenated commit bits and vote counts must equal the whole
DAG's -- the full engine, the full replay, and the committed C4 golden vectors."""
import numpy as np
import pytest

from dag_rider_amd import _lib as L
from dag_rider_amd.engine import Engine
from dag_rider_amd.gen import CONFIGS, generate
from dag_rider_amd.split import split_commit
from dagutil import dag_fingerprint, load_large, random_dag

pytestmark = pytest.mark.gpu


def test_split_c2(gpu_device):
    cfg = CONFIGS["c2"]
    d = generate(cfg)
    with Engine(cfg.n, cfg.faulty, d.nrounds, gpu_device) as e:
        e.append_packed(d)
        full = e.wave_commit(1, cfg.nwaves)
        rep = e.replay(cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF)
    assert (full[0] == rep.commit).all() and (full[1] == rep.vcount).all()
    for world in (2, 4, 8):
        cm, vc, _ = split_commit(d, cfg.faulty, cfg.nwaves, world, gpu_device)
        assert (cm == full[0]).all() and (vc == full[1]).all(), world


def test_split_c4_golden(gpu_device):
    """C4 (n=1024 x 4000 rounds): 2, 4 and 8 wave ranges == the golden commit/vcount vectors."""
    g = load_large()["c4"]["persistent_ref"]
    cfg = CONFIGS["c4"]
    d = generate(cfg, nthreads=16)
    assert dag_fingerprint(d) == load_large()["c4"]["dag"], "generator drift"
    want_c = np.asarray([int(ch) for ch in g["commit"]], np.uint8)
    want_v = np.asarray(g["vcount"], np.int32)
    for world in (2, 4, 8):
        cm, vc, ranges = split_commit(d, cfg.faulty, cfg.nwaves, world, gpu_device)
        assert len(ranges) == world
        assert (cm == want_c).all() and (vc == want_v).all(), world


@pytest.mark.parametrize("seed", range(4))
def test_split_random_with_coin(gpu_device, seed):
    """Unconstrained DAGs and a caller's leader table: the slices take the table re-based."""
    rng = np.random.default_rng(900 + seed)
    n = int(rng.choice([7, 64, 130]))
    R = 4 * int(rng.integers(6, 14))
    d = random_dag(rng, n, R, p_present=0.85, p_s=rng.uniform(0.2, 0.9), p_w=0.3)
    f = (n - 1) // 3
    nw = R // 4
    leaders = [int(x) for x in rng.integers(1, n + 1, size=nw)]
    with Engine(n, f, R + 1, gpu_device) as e:
        e.append_packed(d)
        e.set_leader_coin(L.DR_LEADER_TABLE, table=leaders)
        full = e.wave_commit(1, nw)
    for world in (2, 3, 5):
        cm, vc, _ = split_commit(d, f, nw, world, gpu_device, leaders)
        assert (cm == full[0]).all() and (vc == full[1]).all(), (seed, world)


@pytest.mark.parametrize("n", [64, 128, 300, 700, 1024, 2048])
def test_commit_split_kernel(gpu_device, n):
    """dr_wave_commit on short wave ranges runs each wave's vote on several workgroups
    (k_commit_split, DR_OPT_COMMIT_SPLIT): the same commits and vCounts as one workgroup
    per wave (k_commit) and as the whole-DAG commit rule, for every range length, with
    quorum-shaped DAGs (late vertices, absent leaders) and a seeded leader coin."""
    from dag_rider_amd.gen import small_config

    cfg = small_config(n, 120, 900 + n, p_present=0.95, p_late=0.1, p_w=0.3, weak_depth=4, p_la=0.1)
    d = generate(cfg)
    nw = cfg.nwaves
    for coin in (False, True):
        with Engine(n, cfg.faulty, d.nrounds, gpu_device) as e:
            e.append_packed(d)
            if coin:
                e.set_leader_coin(L.DR_LEADER_SEEDED, 5 + n)
            e.set_commit_split(0)
            want_c, want_v = e.wave_commit(1, nw)
            want1 = [e.wave_commit(w, w) for w in range(1, nw + 1)]
            for mode in (1, 2):  # several workgroups per wave: every short range / ranges of <= 4 waves
                e.set_commit_split(mode)
                for w0, w1 in ((1, nw), (1, 1), (3, 9), (nw - 4, nw), (2, nw - 1)):
                    for _ in range(2):  # the kernel leaves its arrival counters zero for the next launch
                        cm, vc = e.wave_commit(w0, w1)
                        assert (cm == want_c[w0 - 1:w1]).all() and (vc == want_v[w0 - 1:w1]).all(), (mode, w0, w1)
                for w in range(1, nw + 1):
                    cm, vc = e.wave_commit(w, w)
                    assert cm[0] == want1[w - 1][0][0] and vc[0] == want1[w - 1][1][0], (mode, w)
                    assert e.wave_ready(w, max(0, w - 3))[:2] == (bool(cm[0]), int(vc[0]))
