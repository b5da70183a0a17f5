"""Wave-range split of the commit sweep (dag_rider_amd/split.py)
checked on the CPU oracle: the commit decisions of every wave range, each decided on its
own slice of rounds, concatenate to the decisions on the whole DAG.  The slice is the
whole input a rank's GPU holds; the GPU side of the same check is tests/test_gpu_split.py."""
import numpy as np
import pytest

import oracle
from dag_rider_amd.gen import CONFIGS, generate
from dag_rider_amd.split import slice_leaders, wave_ranges, wave_slice
from dagutil import random_dag


def _split_oracle(d, f, nw, world, leaders=None):
    cm, vc, ce = [], [], 0
    for w0, w1 in wave_ranges(nw, world):
        sub = wave_slice(d, w0, w1)
        assert sub.nrounds == 4 * (w1 - w0 + 1) + 1
        c, v, e = oracle.PDag(sub, leaders=slice_leaders(leaders, w0, w1)).commit_sweep(f, 1, w1 - w0 + 1)
        cm.append(c)
        vc.append(v)
        ce += e
    return np.concatenate(cm), np.concatenate(vc), ce


def test_wave_ranges():
    for nw in (8, 9, 125, 1000):
        for world in (1, 2, 3, 4, 8):
            rs = wave_ranges(nw, world)
            assert rs[0][0] == 1 and rs[-1][1] == nw and len(rs) == world
            assert all(b[0] == a[1] + 1 for a, b in zip(rs, rs[1:]))
            sizes = [b - a + 1 for a, b in rs]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        wave_ranges(3, 4)


def test_split_c2_matches_full():
    cfg = CONFIGS["c2"]
    d = generate(cfg)
    full = oracle.PDag(d).commit_sweep(cfg.faulty, 1, cfg.nwaves)
    for world in (2, 4, 8):
        cm, vc, ce = _split_oracle(d, cfg.faulty, cfg.nwaves, world)
        assert (cm == full[0]).all() and (vc == full[1]).all() and ce == full[2], world


@pytest.mark.parametrize("seed", range(6))
def test_split_random_dags_with_coin(seed):
    """Unconstrained DAGs (partial quorums, absent leaders, ghosts) and a leader table."""
    rng = np.random.default_rng(700 + seed)
    n = int(rng.choice([4, 7, 40, 70]))
    R = 4 * int(rng.integers(4, 12))
    d = random_dag(rng, n, R, p_present=0.85, p_s=rng.uniform(0.2, 0.9), p_w=0.3)
    f = (n - 1) // 3
    nw = R // 4
    leaders = [int(x) for x in rng.integers(1, n + 1, size=nw)] if seed % 2 else None
    full = oracle.PDag(d, leaders=leaders).commit_sweep(f, 1, nw)
    for world in (2, 3, 4):
        if world > nw:
            continue
        cm, vc, ce = _split_oracle(d, f, nw, world, leaders)
        assert (cm == full[0]).all() and (vc == full[1]).all() and ce == full[2], (seed, world)


def test_wave_slice_bounds():
    d = generate(CONFIGS["c1"])
    with pytest.raises(ValueError):
        wave_slice(d, 0, 1)
    with pytest.raises(ValueError):
        wave_slice(d, 2, 5)  # rounds past the DAG
    s = wave_slice(d, 2, 3)
    assert s.nrounds == 9 and not s.strong[:d.n * d.W].any() and len(s.weak_tgt) == 0
