"""Full-size GPU parity for C3 (n=256 x 10k rounds, weak-heavy) and C4 (n=1024 x 4k
rounds) against the committed golden replays (tests/golden/large_replay.json.gz, made by
the bitset oracle after the literal restatement agreed on a prefix).  The DAGs are
regenerated on the GPU box by the product's seeded generator; its output is pinned by a
fingerprint first."""
import numpy as np
import pytest

from dag_rider_amd import _lib as L
from dag_rider_amd.engine import Engine
from dag_rider_amd.gen import CONFIGS, generate
from dagutil import dag_fingerprint, load_large, replay_fingerprint

pytestmark = pytest.mark.gpu


def _check(got, want):
    assert "".join(str(int(x)) for x in got.commit) == want["commit"]
    assert got.vcount.tolist() == want["vcount"]
    assert got.push_off.tolist() == want["push_off"]
    assert got.push_wave.tolist() == want["push_wave"]
    for k in ("pop_count", "pop_digest", "pop_edges"):
        w = np.asarray([int(x) for x in want[k]], dtype=np.uint64)
        g = getattr(got, k)
        bad = np.nonzero(g != w)[0]
        assert len(bad) == 0, f"{k}: {len(bad)} pops differ, first at {bad[:5].tolist()}"
    assert (got.commit_edges, got.chain_edges, got.deliver_edges) == \
        (int(want["commit_edges"]), int(want["chain_edges"]), int(want["deliver_edges"]))


@pytest.mark.parametrize("name", ["c3", "c4"])
def test_large_config_golden(gpu_device, name):
    g = load_large()[name]
    cfg = CONFIGS[name]
    d = generate(cfg, nthreads=16)
    assert dag_fingerprint(d) == g["dag"], "generator drift"
    with Engine(cfg.n, cfg.faulty, d.nrounds, gpu_device) as e:
        e.append_packed(d)
        _check(e.replay(cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF), g["persistent_ref"])
        for mask in (0, 1, 2, 4, 7, 15, 23, 31, 39, 55, 63):  # DR_OPT_FUSE: the launch groupings give the same replay
            e.set_fuse(mask)
            _check(e.replay(cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF), g["persistent_ref"])
        e.set_device_plan(False)  # the host-planned phases give the same replay
        _check(e.replay(cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF), g["persistent_ref"])
        e.set_device_plan(True)
        _check(e.replay(cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_PAPER), g["persistent_paper"])


@pytest.mark.parametrize("name", ["c3", "c4"])
def test_large_config_golden_literal_chain(gpu_device, name):
    """DR_CHAIN_LITERAL (the reference's Q1: decidedWave never advances, every commit
    chains down to wave 1, O(w^2) pops) on the full C3 / C4 DAG: replay fingerprint,
    push count and edge totals equal the bitset oracle's."""
    g = load_large()[name]
    cfg = CONFIGS[name]
    d = generate(cfg, nthreads=16)
    assert dag_fingerprint(d) == g["dag"], "generator drift"
    want = g["literal_ref"]
    with Engine(cfg.n, cfg.faulty, d.nrounds, gpu_device) as e:
        e.append_packed(d)
        got = e.replay(cfg.nwaves, L.DR_CHAIN_LITERAL, L.DR_DELIVER_REF)
    assert len(got.push_wave) == want["n_push"]
    assert (got.commit_edges, got.chain_edges, got.deliver_edges) == \
        (int(want["commit_edges"]), int(want["chain_edges"]), int(want["deliver_edges"]))
    assert replay_fingerprint(got) == want["fingerprint"]
