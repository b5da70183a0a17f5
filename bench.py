"""Benchmark: DAG edges traversed/sec (commit + delivery) on MI355X.

Workload (BASELINE.json configs[3], the metric's n=1024 case; fits one GPU): the
synthetic C4 DAG, n=1024 processes x 4000 rounds, replayed end to end through the
C ABI: waveReady for all 1000 waves (commit sweep + leader chains,
decidedWave persistent) and orderVertices for every committed leader
(DR_DELIVER_REF: each pop delivers its full causal history, as the reference's
no-op dedup does).  One step = one dr_replay of the resident DAG.  Edges are
counted by SURVEY.md s8(d)'s formula (the same numbers the CPU oracle reports).

N>1 (torchrun, one rank per GPU): each rank replays its own independent C4 DAG
(seed 4+rank): independent units, no data-path collective ("scaling": "weak").
After the timed region, N>1 also runs the process-column sharded sweep of one C4
DAG across all ranks (RCCL all-gather of the frontier per round; detail.colshard).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# HBM bytes per launch measured by rocprofv3 PMC passes (FETCH_SIZE x2 + WRITE_SIZE, gfx950
# correction of MI355X_MICROARCH.md) on this bench: tools/pmc_traffic.py output
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "r01", "traffic.json")
# replay phase -> the kernels it launches (names as rocprofv3 reports them)
PHASE_KERNELS = {"summary": ["dr::k_summary_commit<16, 512, 1>"],
                 "sweep": ["dr::k_sweep<16, 256, 9>"],
                 "batch": ["dr::k_replay_small<8, false, true>"]}


def measured_traffic(phase):
    """PMC-measured HBM bytes per launch of a phase's kernels, or None if not profiled."""
    try:
        with open(TRAFFIC_FILE) as f:
            t = json.load(f)
        return sum(t[k]["traffic_bytes"] for k in PHASE_KERNELS[phase])
    except (OSError, KeyError, ValueError):
        return None


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(cfg, d, budget_s: float):
    """Time the oracle's literal restatement of process.go (the reference algorithm:
    BFS + hash-set visited + linear id scans, one BFS per delivery candidate) on a
    bounded sample: a full replay of the first k waves, k grown until the budget."""
    import oracle

    best = None
    k = 1
    while k <= cfg.nwaves:
        ld = oracle.LDag(packed=d, nrounds=4 * k + 1)
        t0 = time.perf_counter()
        r = ld.replay(cfg.faulty, k, oracle.CHAIN_PERSISTENT, oracle.DELIVER_REF)
        dt = time.perf_counter() - t0
        assert r.rc == 0
        edges = r.commit_edges + r.deliver_edges  # literal restatement does not count chain edges
        best = dict(value=edges / dt, unit="edges/s", cores=1, kind="port",
                    sample=f"C4 waves 1..{k} (rounds 0..{4 * k}) literal replay: {edges} edges in {dt:.2f} s, "
                           f"single thread, oracle/ref_literal.c")
        if dt * 6 > budget_s:  # the next wave costs several times more (cone grows)
            break
        k += 1
    return best


def cpu_bitset(cfg, d, nthreads: int, budget_s: float):
    """The optimized CPU restatement (packed bitsets, OpenMP) on a bounded sample of pops."""
    import oracle

    bs = oracle.PDag(d)
    k = max(1, cfg.nwaves // 16)
    t0 = time.perf_counter()
    r = bs.replay(cfg.faulty, k, oracle.CHAIN_PERSISTENT, oracle.DELIVER_REF, nthreads=nthreads)
    dt = time.perf_counter() - t0
    assert r.rc == 0
    e = r.commit_edges + r.chain_edges + r.deliver_edges
    return dict(value=e / dt, unit="edges/s", cores=nthreads, kind="port",
                sample=f"C4 waves 1..{k} bitset replay (oracle/ref_bitset.c, OpenMP): {e} edges in {dt:.2f} s")


def kernel_bytes(cfg, d, res):
    """Algorithmic bytes per launch of each replay phase."""
    n, W, T = cfg.n, (cfg.n + 63) // 64, d.nrounds - 1
    leaders = int((res.vcount >= 0).sum())
    dd = max(0, weak_depth(d) - 1)
    sw = res.sweep
    out = {
        # k_summary_commit: every strong row of rounds 1..T read once; U and SD written
        # (the weak-column keys -> WU pass, k_weak_union, runs after it, ~4 us, untimed here)
        "summary": dict(kernel="k_summary_commit (rows -> U, SD + waveReady commit rule)", ms=res.ms["summary"],
                        bytes=T * n * W * 8 + T * W * 8 + T * 8),
        # round 4w-2: the word holding the leader bit; rounds 4w-1, 4w: whole rows
        "commit": dict(kernel="k_commit (waveReady commit rule)", ms=res.ms["commit"],
                       bytes=leaders * (n * 8 + 2 * n * W * 8)),
        # partial rounds: rows of the frontier + the round's weak columns (key + row); summary
        # rounds: U + WU; every round: presence, K and the reach mask written
        "sweep": dict(kernel="k_sweep (orderVertices cones, merge with canonical)", ms=res.ms["deliver"],
                      bytes=sw["row_bytes"] + sw["weak_scanned"] * (W * 8 + 4) + sw["shortcut"] * (1 + dd) * W * 8
                      + (sw["partial"] + sw["shortcut"]) * 3 * W * 8),
    }
    return out


def weak_columns(d):
    """weak-column entries of the device mirror: distinct (round, delta, target) over
    the near weak edges (delta <= 1023), kernels.hpp DagView::wc_*."""
    import numpy as np

    n = d.n
    g = np.repeat(np.arange(d.nrounds * n, dtype=np.int64), np.diff(d.weak_off.astype(np.int64)))
    if len(g) == 0:
        return 0
    r = g // n
    t = d.weak_tgt.astype(np.int64)
    delta = r - (t >> 11)
    near = delta <= 1023
    return int(len(np.unique((r[near] << 22) | (delta[near] << 11) | (t[near] & 2047))))


def weak_depth(d):
    """largest weak-edge delta of the DAG (the summary window)."""
    import numpy as np

    n = d.n
    g = np.repeat(np.arange(d.nrounds * n, dtype=np.int64), np.diff(d.weak_off.astype(np.int64)))
    if len(g) == 0:
        return 1
    return int((g // n - (d.weak_tgt.astype(np.int64) >> 11)).max())


def rank_config(cfg, rank: int, world: int):
    """Weak scaling: rank r replays its own independent DAG of the same shape (seed + r)."""
    import dataclasses

    return dataclasses.replace(cfg, seed=cfg.seed + rank) if world > 1 else cfg


def reduce_over_ranks(dist, dt: float, edges: int, device: str):
    """Whole-job numbers: the slowest rank's time (MAX) and all ranks' edges (SUM).
    device is "cuda" under RCCL ("nccl"), "cpu" under gloo (tests/test_dist_gloo.py)."""
    import torch

    if dist is None:
        return dt, float(edges)
    t = torch.tensor([dt], device=device, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    e = torch.tensor([float(edges)], device=device, dtype=torch.float64)
    dist.all_reduce(e)
    return float(t.item()), float(e.item())


def colshard_child(args):
    """One rank of the process-column sharded sweep: every rank
    holds 1/N of the target columns; the frontier is all-gathered over RCCL each round.
    Workload: the full causal-history reach sets (strong + weak, rounds 0..leader) of
    the 64 newest wave leaders of the C4 DAG -- the sets orderVertices delivers."""
    import numpy as np

    from dag_rider_amd.gen import CONFIGS, generate
    from dag_rider_amd.shard import ShardEngine

    cfg = CONFIGS["c4"]
    d = generate(cfg, nthreads=16)
    se = ShardEngine(cfg.n, cfg.faulty, d.nrounds, args.cs_device, args.cs_world, args.cs_rank,
                     bytes.fromhex(args.cs_uid))
    se.append_packed(d)
    froms = [(4 * w - 3, 1) for w in range(cfg.nwaves, cfg.nwaves - 64, -1)]
    bottoms = [0] * len(froms)
    got = se.reach_sets(froms, bottoms, False)  # warm-up
    runs = []
    for _ in range(3):
        got = se.reach_sets(froms, bottoms, False)
        runs.append(se.stats())
    st = min(runs, key=lambda x: x["ms"])
    out = dict(st, nshards=args.cs_world, queries=len(froms), info=se.info())
    se.close()
    if args.cs_rank == 0:
        from dag_rider_amd.engine import Engine

        with Engine(cfg.n, cfg.faulty, d.nrounds, args.cs_device) as e:
            e.append_packed(d)
            ref = e.reach_sets(froms, bottoms, False)
        out["verify_vs_unsharded"] = bool(all((a == b).all() for a, b in zip(got, ref)))
        out["reach_bits"] = int(sum(int(np.unpackbits(a.view(np.uint8)).sum()) for a in got))
    print(json.dumps(out), flush=True)


def colshard_check(dist, rank: int, world: int, local: int, timeout_s: float = 240.0):
    """Run colshard_child in one child process per rank (a hung collective can then be
    killed without losing the headline line); returns rank 0's result + max time."""
    import subprocess

    from dag_rider_amd.shard import exchange_unique_id

    if dist is not None:
        uid = exchange_unique_id(dist)
    else:
        from dag_rider_amd.shard import shard_unique_id

        uid = shard_unique_id()
    cmd = [sys.executable, os.path.abspath(__file__), "--colshard-child", "--cs-uid", uid.hex(),
           "--cs-rank", str(rank), "--cs-world", str(world), "--cs-device", str(local)]
    res = None
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s)
        lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
        res = json.loads(lines[-1]) if p.returncode == 0 and lines else dict(error=(p.stderr or "")[-400:])
    except subprocess.TimeoutExpired:
        res = dict(error=f"timed out after {timeout_s} s")
    if dist is not None:
        allr = [None] * world
        dist.all_gather_object(allr, res)
    else:
        allr = [res]
    ms = [r.get("ms") for r in allr if r and "ms" in r]
    if rank == 0 and res is not None:
        res["ms_max_over_ranks"] = max(ms) if len(ms) == world else None
        res["errors"] = [r.get("error") for r in allr if r and "error" in r] or None
    return res


def run_c5(args, rank: int, world: int, local: int, dist):
    """C5 (BASELINE.json configs[4]): the fixed batch of 4096 independent n=128 x 128-round
    replays (seeds 5000+i), split across ranks (strong scaling); each rank replays its
    DAGs as one fused dr_replay_batch launch (one wavefront per DAG, batch.hpp)."""
    import torch

    from dag_rider_amd import _lib as L
    from dag_rider_amd.engine import Engine, ReplayBatch
    from dag_rider_amd.gen import c5_config, generate

    total = 4096
    lo, hi = rank * total // world, (rank + 1) * total // world
    t0 = time.perf_counter()
    engines, dag_bytes = [], 0
    for i in range(lo, hi):
        cfg = c5_config(i)
        d = generate(cfg)
        e = Engine(cfg.n, cfg.faulty, d.nrounds, local)
        e.append_packed(d)
        engines.append(e)
        dag_bytes += d.nrounds * cfg.n * d.W * 8 + weak_columns(d) * (4 + d.W * 8)
    log(f"[rank {rank}] C5 DAGs {lo}..{hi - 1} loaded in {time.perf_counter() - t0:.1f} s")
    nw = c5_config(0).nwaves
    b = ReplayBatch(engines, nw, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF)
    for _ in range(args.warmup):
        b.run()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        b.run()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    res = b.results()
    edges = sum(r.total_edges for r in res)
    kms = max(r.ms["deliver"] for r in res)  # the fused launch's device time (HIP events)
    dt, total_edges = reduce_over_ranks(dist, time.perf_counter() - t0, edges, "cuda")
    if rank != 0:
        return None
    ach = dag_bytes / (kms / 1e3) / 1e9 if kms > 0 else 0.0
    return {
        "metric": "DAG edges traversed/sec (commit+delivery)",
        "value": total_edges * args.steps / dt,
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (seeded generator, SURVEY.md s8(d) C5 parameters, seeds 5000+i)",
        "config": {"workload": "C5: 4096 independent n=128 x 128-round replays (waveReady + orderVertices ref, "
                               "persistent decidedWave), split across ranks",
                   "dags": total, "dags_per_rank": hi - lo, "n": 128, "rounds": 128, "waves": nw,
                   "parallelism": f"dp{world}" if world > 1 else "single"},
        "roofline": {"bound": "latency", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": ach / HBM_PEAK_GBS, "traffic": measured_traffic("batch"),
                     "kernel": "k_replay_small (one wavefront per DAG)",
                     "bytes_per_launch": dag_bytes, "ms_per_launch": kms,
                     "note": "unique DAG bytes (strong rows + weak columns) once per launch"},
        "cpu_baseline": None,
        "detail": {"edges_per_step": edges, "commits": int(sum(int(r.commit.sum()) for r in res)),
                   "pops": int(sum(len(r.pop_count) for r in res))},
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c4")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--verify", action="store_true", help="check the replay against the bitset oracle")
    ap.add_argument("--colshard", action="store_true",
                    help="also run the process-column sharded C4 sweep (default on when N>1)")
    ap.add_argument("--no-colshard", action="store_true")
    ap.add_argument("--colshard-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cs-uid", default="", help=argparse.SUPPRESS)
    ap.add_argument("--cs-rank", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--cs-world", type=int, default=1, help=argparse.SUPPRESS)
    ap.add_argument("--cs-device", type=int, default=0, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.colshard_child:
        return colshard_child(args)

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))

    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", init_method="env://")
    torch.cuda.set_device(local)

    from dag_rider_amd import _lib as L
    from dag_rider_amd.engine import Engine
    from dag_rider_amd.gen import CONFIGS, generate

    if args.config == "c5":
        out = run_c5(args, rank, world, local, dist)
        if out is not None:
            print(json.dumps(out), flush=True)
        if dist:
            dist.destroy_process_group()
        return

    cfg = rank_config(CONFIGS[args.config], rank, world)
    t0 = time.perf_counter()
    d = generate(cfg, nthreads=16)
    log(f"[rank {rank}] generated {cfg} in {time.perf_counter() - t0:.1f} s")
    eng = Engine(cfg.n, cfg.faulty, d.nrounds, local)
    t0 = time.perf_counter()
    eng.append_packed(d)
    log(f"[rank {rank}] loaded DAG into HBM in {time.perf_counter() - t0:.1f} s")

    def step():
        return eng.replay(cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF)

    # timed steps: HIP events around the summary pass only (the dominant kernel);
    # every other phase is timed by one extra, untimed-by-the-clock replay below
    eng.set_phase_timing(1)
    for _ in range(args.warmup):
        res = step()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ms_summary = 0.0
    for _ in range(args.steps):
        res = step()
        ms_summary += res.ms["summary"]
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt, total_edges = reduce_over_ranks(dist, time.perf_counter() - t0, res.total_edges, "cuda")
    eng.set_phase_timing(2)
    prof = step()  # per-phase HIP event times (same work, outside the timed region)
    res.ms = dict(prof.ms, summary=ms_summary / args.steps)

    verify = None
    if args.verify and rank == 0:
        import oracle

        want = oracle.PDag(d).replay(cfg.faulty, cfg.nwaves, oracle.CHAIN_PERSISTENT, oracle.DELIVER_REF,
                                     nthreads=16)
        verify = bool((want.commit == res.commit).all() and (want.pop_digest == res.pop_digest).all()
                      and (want.pop_count == res.pop_count).all() and want.deliver_edges == res.deliver_edges
                      and want.chain_edges == res.chain_edges and want.commit_edges == res.commit_edges)

    colshard = None
    if (world > 1 or args.colshard) and not args.no_colshard:
        colshard = colshard_check(dist, rank, world, local)
        if rank == 0:
            log(f"[colshard] {colshard}")

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    W = (cfg.n + 63) // 64
    kb = kernel_bytes(cfg, d, res)
    # dominant kernel = the phase with the largest device time (HIP events)
    dom = max(kb, key=lambda k: kb[k]["ms"])
    ach = kb[dom]["bytes"] / (kb[dom]["ms"] / 1e3) / 1e9 if kb[dom]["ms"] > 0 else 0.0
    cpu = None
    cpu2 = None
    if not args.no_cpu and world == 1:
        cpu = cpu_baseline(cfg, d, args.cpu_budget)
        cpu2 = cpu_bitset(cfg, d, 16, args.cpu_budget)

    ms_per_step = dt / args.steps * 1e3
    out = {
        "metric": "DAG edges traversed/sec (commit+delivery)",
        "value": total_edges * args.steps / dt,
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (seeded generator, SURVEY.md s8(d) C4 parameters)",
        "config": {"workload": f"C4 full replay: n={cfg.n} x {cfg.last_round} rounds, {cfg.nwaves} waves, "
                               "waveReady (persistent decidedWave) + orderVertices (ref, full cones) per commit",
                   "n": cfg.n, "rounds": cfg.last_round, "waves": cfg.nwaves,
                   "parallelism": f"replicas{world}" if world > 1 else "single"},
        "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": ach / HBM_PEAK_GBS, "traffic": measured_traffic(dom),
                     "traffic_unit": "bytes/launch (rocprofv3 PMC, profiles/r01/traffic.json)",
                     "kernel": kb[dom]["kernel"], "bytes_per_launch": kb[dom]["bytes"],
                     "ms_per_launch": kb[dom]["ms"]},
        "cpu_baseline": cpu,
        "cpu_bitset": cpu2,
        "detail": {"edges_per_step": res.total_edges, "commit_edges": res.commit_edges,
                   "chain_edges": res.chain_edges, "deliver_edges": res.deliver_edges,
                   "commits": int(res.commit.sum()), "pops": int(len(res.pop_count)),
                   "ms": res.ms, "ms_note": "summary: mean over the timed steps; other phases: one "
                   "profiling replay after them (DR_OPT_PHASE_TIMING=2)",
                   "sweep": res.sweep, "verify_vs_oracle": verify,
                   "colshard": colshard,
                   "kernels": {k: dict(v, GBps=(v["bytes"] / (v["ms"] / 1e3) / 1e9 if v["ms"] > 0 else None))
                               for k, v in kb.items()}},
    }
    print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
