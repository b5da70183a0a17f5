"""bench.py's multi-rank path (one process per GPU, weak scaling) on CPU: world_size 2
over gloo.  Each rank derives its own workload (distinct seed, same shape), the job's
time is the slowest rank's and its edge total the sum over ranks."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist

    import bench
    from dag_rider_amd.gen import CONFIGS, generate, small_config

    dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)
    try:
        cfg = bench.rank_config(CONFIGS["c4"], rank, world)
        small = bench.rank_config(small_config(16, 12, 5), rank, world)
        d = generate(small)
        edges = int(d.weak_off[-1]) + 1000 * (rank + 1)  # any per-rank count
        dt, tot = bench.reduce_over_ranks(dist, 0.5 + rank, edges, "cpu")
        out[rank] = (cfg.seed, cfg.n, cfg.last_round, small.seed, int(d.strong.sum() % (1 << 32)), edges, dt, tot)
    finally:
        dist.destroy_process_group()


def test_weak_scaling_two_ranks_gloo():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    r0, r1 = out[0], out[1]
    # same shape, independent units
    assert r0[1:3] == r1[1:3] and r0[0] != r1[0] and r0[3] != r1[3]
    # max time, summed edges, identical on every rank
    assert r0[6] == r1[6] == 1.5
    assert r0[7] == r1[7] == float(r0[5] + r1[5])


def test_single_rank_passthrough():
    sys.path.insert(0, ROOT)
    import bench
    from dag_rider_amd.gen import CONFIGS

    assert bench.rank_config(CONFIGS["c4"], 0, 1) == CONFIGS["c4"]
    assert bench.reduce_over_ranks(None, 2.0, 7, "cpu") == (2.0, 7.0)


def test_bench_gpus_spawns_ranks():
    """bench.py --gpus 2 outside torchrun really starts 2 ranks (torch.distributed.run)
    and rank 0 prints one line reduced over both: max time, summed work."""
    import json
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-selftest"],
                       capture_output=True, text=True, timeout=240, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert sorted(r["rank"] for r in out["ranks"]) == [0, 1]
    assert len({r["pid"] for r in out["ranks"]}) == 2
    assert out["selftest_ms_per_step"] == 500.0 and out["selftest_value"] == 3000 / 0.5
    # the C4 N > 1 line (bench.c4_multi_line): the column-sharded replay of one DAG,
    # slowest rank (0.5 ms), strong scaling, replicas in detail
    assert out["config"]["parallelism"] == "colshard2" and out["scaling"] == "strong"
    assert out["ms_per_step"] == 0.5 and out["value"] == 1e9 / 0.5e-3
    assert out["detail"]["replicas"]["parallelism"] == "replicas2"
    assert out["detail"]["verify_vs_unsharded"] is True


def test_bench_gpus_colshard_failure_is_labelled():
    """A rank whose sharded run fails: the line carries the replicas number, says so."""
    import json
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-selftest",
                        "--selftest-fail"], capture_output=True, text=True, timeout=240, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][0])
    assert out["config"]["parallelism"] == "replicas2" and out["scaling"] == "weak"
    assert "FAILED" in out["config"]["workload"] and out["detail"]["colshard_errors"][1] == "selftest failure"
    assert out["value"] == 3000 / 0.5


def test_bench_gpus_colshard_wrong_result_not_published():
    """Rank 0's check of the sharded replay against the unsharded engine fails: the sharded
    number is not the line's value; the line carries the replicas number and says why."""
    import json
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-selftest",
                        "--selftest-wrong"], capture_output=True, text=True, timeout=240, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][0])
    assert out["config"]["parallelism"] == "replicas2" and out["scaling"] == "weak"
    assert out["detail"]["colshard_errors"][0] == "verify_vs_unsharded failed"
    assert out["value"] == 3000 / 0.5


def test_bench_world_mismatch_refused():
    """Under torchrun a WORLD_SIZE that disagrees with --gpus exits non-zero, prints nothing."""
    import subprocess

    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-selftest"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 2 and not p.stdout.strip()


def _id_worker(rank, world, port, out):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from dag_rider_amd.shard import exchange_unique_id

    dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)
    try:
        made = []

        def make():  # stands in for ncclGetUniqueId, which needs a GPU
            made.append(rank)
            return bytes((7 * i + 3) % 256 for i in range(128))

        out[rank] = (exchange_unique_id(dist, make), tuple(made))
    finally:
        dist.destroy_process_group()


def test_shard_unique_id_exchange_gloo():
    """The column-sharded path's RCCL bootstrap: rank 0 makes the unique id, every rank gets it."""
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_id_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    assert out[0][0] == out[1][0] and len(out[0][0]) == 128
    assert out[0][1] == (0,) and out[1][1] == ()


def test_shard_no_cpu_fallback():
    """dr_shard_create fails loudly without a HIP device."""
    sys.path.insert(0, ROOT)
    try:
        import torch

        if torch.cuda.is_available():
            pytest.skip("a GPU is visible")
    except Exception:
        pass
    from dag_rider_amd import _lib as L
    from dag_rider_amd.shard import ShardEngine

    with pytest.raises(L.DrError) as ei:
        ShardEngine(16, 5, 8, 0, nshards=2)
    assert ei.value.code == L.DR_E_HIP
