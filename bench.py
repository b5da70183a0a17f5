"""Benchmark: DAG edges traversed/sec (commit+delivery) on MI355X.

Default workload (BASELINE.json configs[3], the metric's n=1024 case; fits one GPU):
the synthetic C4 DAG, n=1024 processes x 4000 rounds, replayed end to end through
the C ABI: waveReady for all 1000 waves (commit sweep + leader chains, decidedWave
persistent) and orderVertices for every committed leader (DR_DELIVER_REF: each pop
delivers its full causal history, as the reference's no-op dedup does).  One step =
one dr_replay of the resident DAG.  Edges are counted by SURVEY.md s8(d)'s formula
(the same numbers the CPU oracle reports).

Other lines (--config): c3 (n=256 x 10k rounds, weak-heavy: the metric's other
half), c2, c5 (4096 independent n=128 replays, split across ranks), c4-deep (weak
edges 80 rounds deep, past the memo window of 65: every pop sweeps its cone),
c4-deep64 (weak edges 64 deep: memoized at the window's far end), c4-loop (the drop-in call
pattern: per wave append 4 rounds -> dr_wave_ready -> dr_order_vertices, per-wave
latency), c4-far / c4-q8 (C4 + one weak edge 600 rounds deep / one strong edge to round
r-3: exceptions to the regular graph, tested once and found benign, so the memo stays on),
c4-up (C4 + one weak edge to its own round: the general sweep serves every query; no oracle
takes such an edge at this size, the general sweep's parity is tests/test_gpu_irregular.py's),
--deliver paper (dedup across pops).

--gpus N without torchrun: spawns N ranks (torch.distributed.run) before anything
touches a GPU; under torchrun WORLD_SIZE must equal N.  For C4 at N > 1 the line
is BASELINE.json configs[3] as named: ONE C4 DAG (seed 4) with its process columns
sharded across the N GPUs, the memoized replay with the frontier all-gathered over
RCCL ("parallelism": "colshardN", "scaling": "strong": the same edges per step at
every N), timed in one child process per rank (a hung collective is killed, not
waited for) and checked on rank 0 against the unsharded engine.  detail.replicas
holds every rank replaying its own unsharded C4 DAG (seed 4+rank, weak scaling),
detail.commit_split the all-waves commit sweep of the DAG split into wave ranges.
C5 at N > 1 splits its 4096 DAGs across the ranks.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# HBM bytes per launch measured by rocprofv3 PMC passes (FETCH_SIZE x2 + WRITE_SIZE, gfx950
# correction of MI355X_MICROARCH.md) on this bench: tools/pmc_traffic.py output
TRAFFIC_FILES = [os.path.join(ROOT, "profiles", r, "traffic.json") for r in ("r06", "r05", "r04", "r03")]


def fuse_mask() -> int:
    """The engine's DR_OPT_FUSE mask for this process (DR_FUSE overrides the default 23)."""
    return int(os.environ.get("DR_FUSE", "23"))


def phase_kernels(phase: str, W: int = 16):
    """Replay phase -> candidate lists of the kernels it launches at row stride W, named as
    rocprofv3 reports them (engine.hip's launch geometry: launch_sc_shipped, sweep_block_m,
    launch_own_emit_t, the batch forms of DR_OPT_BATCH_FORM).  The first list whose every
    kernel is in the traffic file is summed."""
    blk = {1: 64, 2: 128, 4: 256, 8: 512}.get(W, 1024)
    if phase == "summary":
        return [[f"dr::k_summary_commit<{W}, 1024, 2, false>" if W == 16 else f"dr::k_summary_commit<{W}, {blk}, 8, false>"]]
    if phase == "sweep":  # merging pop sweeps (SW_WEAK | SW_MERGE = 9), own-round emission, final pass
        nt = 192 if W == 16 else min(blk, 512)
        return [[f"dr::k_sweep<{W}, {nt}, 9>", f"dr::k_own_emit<{W}, 256>",
                 "dr::k_replay_final<1024>"]]
    if phase == "batch_k_replay_small_1w":  # the wave-per-DAG form (many DAGs per CU)
        return [["dr::k_replay_small_1w<false, true>"]]
    if phase == "batch_k_replay_small":  # the workgroup form (a ring depth per launch)
        return [[f"dr::k_replay_small<{d}, false, true>"] for d in (4, 8, 16, 32)]
    return []
CPU_THREADS = 16  # the GPU box's host share for one GPU (OMP_NUM_THREADS there)


def cpu_threads() -> int:
    """Host threads the CPU baselines use: this GPU's share of the box.  The GPU box
    exports OMP_NUM_THREADS=16 per GPU; os.sched_getaffinity there lists every thread
    of the (shared) host, which the box's rules forbid one GPU's job to take over."""
    try:
        share = int(os.environ.get("OMP_NUM_THREADS", CPU_THREADS))
    except ValueError:
        share = CPU_THREADS
    return max(1, min(share, cpu_info()["affinity"] or 1))


def measured_traffic(phase, W: int = 16, config: str = "c4"):
    """PMC-measured HBM bytes per launch of a phase's kernels (the newest traffic file that
    profiled them on this config), with the file it came from; (None, None) if none did."""
    for path in TRAFFIC_FILES:
        try:
            with open(path) as f:
                t = json.load(f)
        except (OSError, ValueError):
            continue
        # per config since round 4 ({config: {kernel: ...}}); round 3's file is C4's kernels
        t = t.get(config, {}) if any(isinstance(v, dict) and "traffic_bytes" not in v for v in t.values()) else (
            t if config == "c4" else {})
        for names in phase_kernels(phase, W):
            if all(k in t for k in names):
                return sum(t[k]["traffic_bytes"] for k in names), os.path.relpath(path, ROOT)
    return None, None


def emit_line(out: dict) -> None:
    """Print a bench line with the library's provenance (dr_build_id next to this tree's
    source hash: a prebuilt library must match the sources it is reported against)."""
    from dag_rider_amd import _lib as L

    out.setdefault("provenance", L.provenance())
    print(json.dumps(out), flush=True)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_info():
    """Host CPU model and the cores this process may use (recorded with every baseline)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count()
    return dict(model=model, nproc=os.cpu_count(), affinity=aff, omp_num_threads=os.environ.get("OMP_NUM_THREADS"))


def _median_runs(fn, runs):
    ts, out = [], None
    for _ in range(runs):
        t0 = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts), ts, out


def cpu_literal(cfg, d, budget_s: float, full_edges: int, deliver_mode: int):
    """The oracle's literal restatement of process.go (the reference's algorithm: BFS +
    hash-set visited + linear id scans, one BFS per voter and per orderVertices
    candidate) on a bounded sample: a replay of waves 1..k.  Single thread (the
    reference is one goroutine) and one thread per core of this GPU's host share
    (the independent BFSs of the voter loop and of a pop's candidates in parallel);
    median of 5 runs each.  The full replay is extrapolated per edge at the sample's
    rate (a lower bound) and by the per-wave cost model of literal_wave_model."""
    import oracle

    nt = cpu_threads()
    k, cum = 0, []
    while k < min(cfg.nwaves, 6):
        k += 1
        ld = oracle.LDag(packed=d, nrounds=4 * k + 1)
        t0 = time.perf_counter()
        r = ld.replay(cfg.faulty, k, oracle.CHAIN_PERSISTENT, deliver_mode, nthreads=nt)
        cum.append(time.perf_counter() - t0)
        assert r.rc == 0
        if cum[-1] * 4 > budget_s / 4:
            break
    ld = oracle.LDag(packed=d, nrounds=4 * k + 1)
    mt_med, mt_ts, r = _median_runs(
        lambda: ld.replay(cfg.faulty, k, oracle.CHAIN_PERSISTENT, deliver_mode, nthreads=nt), 5)
    edges = r.commit_edges + r.deliver_edges  # the literal restatement does not count chain edges
    ld1 = oracle.LDag(packed=d, nrounds=5)
    st_med, st_ts, r1 = _median_runs(lambda: ld1.replay(cfg.faulty, 1, oracle.CHAIN_PERSISTENT, deliver_mode), 5)
    e1 = r1.commit_edges + r1.deliver_edges
    model = literal_wave_model(cfg, d, nt) if cfg.n * cfg.last_round >= 64 * 1000 else None
    return dict(value=e1 / st_med, unit="edges/s", cores=1, kind="port",
                sample=f"{cfg.name} waves 1..1 (rounds 0..4) literal replay (oracle/ref_literal.c, the reference's "
                       f"algorithm), single thread: {e1} edges, median {st_med:.2f} s of 5 runs",
                runs_s=st_ts,
                all_cores=dict(value=edges / mt_med, cores=nt, waves=k, edges=edges, median_s=mt_med, runs_s=mt_ts,
                               cum_s=cum),
                extrapolated_full_s_per_edge=full_edges / (e1 / st_med),
                wave_model=model, host=cpu_info())


def literal_wave_model(cfg, d, nt: int, waves=(2, 3, 4, 6, 8, 12, 16), per_wave: int = 64, seed: int = 1):
    """Per-wave cost of the literal replay, measured on samples and fitted with a free
    intercept.  orderVertices of wave w's leader runs one path() BFS per slot of rounds
    1..4w (process.go:414-431); a BFS costs ~ the part of the leader's cone it explores
    (the whole cone when the slot is unreachable), so its mean time grows ~ linearly in w
    and the pop costs N_cand(w) x mean(w) ~ w^2.  For each sampled wave: per_wave slots,
    one in each of per_wave evenly spaced rounds of 1..4w (stratified by round), each
    BFS timed on its own thread's CPU clock (thread_time, on nt threads).  Fit mean(w) = a + b w (least squares, free intercept,
    residuals reported); full replay = sum over all waves of the voter time (mean of the
    samples) + N_cand(w) x (a + b w), single thread.  The voters of waveReady(w)
    (process.go:330-335) are sampled the same way: per_wave/4 slots of round 4w per wave."""
    from concurrent.futures import ThreadPoolExecutor

    import numpy as np

    import oracle

    waves = [w for w in waves if w <= cfg.nwaves]
    top = 4 * max(waves) + 1
    ld = oracle.LDag(packed=d, nrounds=top)
    rng = np.random.default_rng(seed)
    so = d.slot_off.astype(np.int64)
    jobs = []
    for w in waves:
        rounds = np.unique(np.linspace(1, 4 * w, per_wave).round().astype(np.int64))
        rounds = np.resize(rounds, per_wave)
        for r in rounds:
            if so[r + 1] > so[r]:
                s = int(d.slot_src[int(rng.integers(so[r], so[r + 1]))])
                jobs.append(("pop", w, (4 * w - 3, 1), (int(r), s) if s else (0, 0), False))
        # voters: slots of round 4w, path(v, leader, strong) (process.go:330-335)
        for i in rng.integers(so[4 * w], so[4 * w + 1], size=per_wave // 4):
            s = int(d.slot_src[int(i)])
            jobs.append(("vote", w, (4 * w, s) if s else (0, 0), (4 * w - 3, 1), True))

    def one(job):
        kind, w, fr, to, strong = job
        t0 = time.thread_time()
        ld.path(fr, to, strong)
        return kind, w, time.thread_time() - t0

    t0 = time.perf_counter()
    with ThreadPoolExecutor(nt) as ex:
        res = list(ex.map(one, jobs))
    wall = time.perf_counter() - t0
    mean = {w: float(np.mean([t for k, ww, t in res if k == "pop" and ww == w])) for w in waves}
    vmean = float(np.mean([t for k, _, t in res if k == "vote"]))
    x = np.asarray(waves, np.float64)
    y = np.asarray([mean[w] for w in waves])
    (a, b), *_ = np.linalg.lstsq(np.stack([np.ones_like(x), x], 1), y, rcond=None)
    pred = a + b * x
    ncand = lambda w: int(so[min(4 * w, d.nrounds - 1) + 1] - so[1])
    nvote = lambda w: int(so[4 * w + 1] - so[4 * w])
    full = sum(nvote(w) * vmean + ncand(w) * max(a + b * w, 0.0) for w in range(1, cfg.nwaves + 1))
    return dict(model="wave(w) = N_vote(w) x v + N_cand(w) x (a + b w); N_cand(w) = slots of rounds 1..4w, "
                      "N_vote(w) = slots of round 4w, v = mean voter BFS",
                waves=waves, bfs_samples_per_wave=per_wave, bfs_mean_s={str(w): mean[w] for w in waves},
                voter_bfs_mean_s=vmean, voter_samples=len([j for j in jobs if j[0] == "vote"]), a=float(a), b=float(b),
                residual_rel={str(w): float((yy - pp) / yy) for w, yy, pp in zip(waves, y, pred)},
                r2=float(1 - ((y - pred) ** 2).sum() / max(((y - y.mean()) ** 2).sum(), 1e-30)),
                sample_wall_s=wall, threads=nt, extrapolated_full_s_single_thread=full,
                extrapolated_full_s_all_threads=full / nt)


def cpu_bitset(cfg, d, nthreads: int, full_runs: int, deliver_mode: int):
    """The optimized CPU restatement (packed bitsets, OpenMP): the full replay, median of runs."""
    import oracle

    bs = oracle.PDag(d)
    med, ts, r = _median_runs(lambda: bs.replay(cfg.faulty, cfg.nwaves, oracle.CHAIN_PERSISTENT, deliver_mode,
                                                nthreads=nthreads), full_runs)
    assert r.rc == 0
    e = r.commit_edges + r.chain_edges + r.deliver_edges
    return dict(value=e / med, unit="edges/s", cores=nthreads, kind="port",
                sample=f"{cfg.name} full replay ({cfg.nwaves} waves) bitset restatement (oracle/ref_bitset.c, "
                       f"OpenMP {nthreads} threads): {e} edges, median {med:.3f} s of {full_runs} runs",
                runs_s=ts), r


def same_replay(a, b) -> bool:
    """Every replay output equal (tests/test_coin.py _same): commits, vote counts, push
    offsets and pushed waves, per-pop count / digest / edges, and every edge total."""
    import numpy as np

    arr = ("commit", "vcount", "push_off", "push_wave", "pop_count", "pop_digest", "pop_edges")
    return bool(all(np.array_equal(np.asarray(getattr(a, k)), np.asarray(getattr(b, k))) for k in arr)
                and (a.commit_edges, a.chain_edges, a.deliver_edges) == (b.commit_edges, b.chain_edges,
                                                                         b.deliver_edges))


def kernel_bytes(cfg, d, res, dreg=None, mstat=None, wu_fused=True):
    """Algorithmic bytes per launch of each replay phase.  dreg: the engine's
    regular weak window (the summaries' depth; deeper weak edges are exceptions, s3.5).
    mstat (Engine.mirror_stats) with wu_fused: the row pass's launch also carries the weak
    unions and speculative digests (DR_OPT_FUSE bit 1): the weak-column keys (4 B each), the
    slot sources (2 B each), slot offsets, column offsets and presence prefixes (16 B per round)
    read, WU and RG written."""
    n, W, T = cfg.n, (cfg.n + 63) // 64, d.nrounds - 1
    leaders = int((res.vcount >= 0).sum())
    dd = max(0, (dreg if dreg else weak_depth(d)) - 1)
    sw = res.sweep
    wu = (4 * mstat["weak_columns"] + 2 * mstat["slots"] + 16 * T + T * dd * W * 8 + 8 * T) if (mstat and wu_fused) \
        else 0
    return {
        # k_summary_commit: every strong row of rounds 1..T read once; U and SD written; with
        # the weak unions in the same launch, their bytes too
        "summary": dict(kernel="k_summary_commit (rows -> U, SD + waveReady commit rule"
                               + (" + weak unions, speculative digests)" if wu else ")"), ms=res.ms["summary"],
                        bytes=T * n * W * 8 + T * W * 8 + T * 8 + wu),
        # round 4w-2: the word holding the leader bit; rounds 4w-1, 4w: whole rows
        "commit": dict(kernel="k_commit (waveReady commit rule)", ms=res.ms["commit"],
                       bytes=leaders * (n * 8 + 2 * n * W * 8)),
        # partial rounds: rows of the frontier + the round's weak columns (key + row); summary
        # rounds: U + WU; every round: presence, K and the reach mask written
        "sweep": dict(kernel="k_sweep (orderVertices cones, merge with canonical)", ms=res.ms["deliver"],
                      bytes=sw["row_bytes"] + sw["weak_scanned"] * (W * 8 + 4) + sw["shortcut"] * (1 + dd) * W * 8
                      + (sw["partial"] + sw["shortcut"]) * 3 * W * 8),
    }


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
    delta = r - ((t >> 11) & 0xFFFFF)
    near = (delta >= 2) & (delta <= 1023) & ((t >> 31) == 0)  # (bit 31 / delta < 2: App. A Q8 edges, no column)
    return int(len(np.unique((r[near] << 22) | (delta[near] << 11) | (t[near] & 2047))))


def weak_depth(d):
    """largest weak-edge delta of the DAG (the summary window)."""
    import numpy as np

    n = d.n
    g = np.repeat(np.arange(d.nrounds * n, dtype=np.int64), np.diff(d.weak_off.astype(np.int64)))
    if len(g) == 0:
        return 1
    t = d.weak_tgt.astype(np.int64)
    weak = (t >> 31) == 0  # (bit 31: a strong edge outside the rows)
    return int((g[weak] // n - (t[weak] >> 11)).max()) if weak.any() else 1


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


def commit_split(dist, rank: int, world: int, local: int, want_commit=None, want_vcount=None, iters: int = 20):
    """the all-waves commit sweep of ONE C4 DAG (seed 4), waves
    split into contiguous ranges, one per GPU, each GPU holding only its rounds
    (dag_rider_amd/split.py); no exchange.  Returns rank 0's view: max time over
    ranks, bit-exact check of the gathered commits against the full replay on rank 0."""
    import numpy as np

    from dag_rider_amd.gen import CONFIGS, generate

    cfg = CONFIGS["c4"]
    d = generate(cfg, nthreads=CPU_THREADS)
    mine = rank_share(cfg, d, rank, world, local, iters, dist)
    allr = [None] * world
    if dist:
        dist.all_gather_object(allr, mine)
    else:
        allr = [mine]
    if rank != 0:
        return None
    cmt = np.concatenate([np.asarray(r["commit"], np.uint8) for r in allr])
    vct = np.concatenate([np.asarray(r["vcount"], np.int32) for r in allr])
    ok = None
    if want_commit is not None:
        ok = bool((cmt == want_commit).all() and (vct == want_vcount).all())
    ms = max(r["ms"] for r in allr)
    kms = max(r["kernel_ms"] for r in allr)
    alg = sum(r["bytes"] for r in allr)
    return dict(waves=cfg.nwaves, ranges=[(r["w0"], r["w1"]) for r in allr], ms_max_over_ranks=ms,
                kernel_ms_max_over_ranks=kms, waves_per_s=cfg.nwaves / (ms / 1e3), algorithmic_bytes=alg,
                per_rank=[{k: r[k] for k in ("rank", "w0", "w1", "ms", "kernel_ms", "bytes", "GBps_kernel")}
                          for r in allr],
                verify_vs_full_replay=ok, note="dr_wave_commit (k_commit) per rank: ms = wall clock incl. D2H, "
                "kernel_ms = HIP events (dr_last_kernel_ms)")


def commit_bytes(n: int, W: int, leaders: int) -> int:
    """k_commit's algorithmic bytes: per wave with a leader, the leader's 16-B chunk of
    each row of round 4w-2 and rounds 4w-1, 4w whole (bench kernel_bytes 'commit')."""
    return leaders * (n * 16 + 2 * n * W * 8)


def rank_share(cfg, d, rank: int, world: int, local: int, iters: int, dist=None):
    """One rank's share of the wave-range commit split: its slice of rounds on its own
    mirror, dr_wave_commit over its waves, timed (wall clock and HIP events)."""
    import numpy as np
    import torch

    from dag_rider_amd.engine import Engine
    from dag_rider_amd.split import wave_ranges, wave_slice

    w0, w1 = wave_ranges(cfg.nwaves, world)[rank]
    sub = wave_slice(d, w0, w1)
    with Engine(cfg.n, cfg.faulty, sub.nrounds, local) as e:
        e.append_packed(sub)
        if os.environ.get("DR_BENCH_COMMIT_SPLIT"):  # tuning: 1 = k_commit_split (default 0, k_commit)
            e.set_commit_split(int(os.environ["DR_BENCH_COMMIT_SPLIT"]))
        cm, vc = e.wave_commit(1, w1 - w0 + 1)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        kms = []
        t0 = time.perf_counter()
        for _ in range(iters):
            cm, vc = e.wave_commit(1, w1 - w0 + 1)
            kms.append(e.last_kernel_ms())
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / iters
    km = float(np.median(kms))
    nb = commit_bytes(cfg.n, (cfg.n + 63) // 64, int((vc >= 0).sum()))
    return dict(rank=rank, w0=w0, w1=w1, commit=cm.tolist(), vcount=vc.tolist(), ms=dt * 1e3, kernel_ms=km,
                bytes=nb, GBps_kernel=nb / (km / 1e3) / 1e9 if km > 0 else None)


def run_rank_share(args, local: int):
    """--rank-share N on one GPU: every rank's share of the wave-range commit split of
    the C4 DAG, decided one after another on this GPU (what each of N GPUs does on its
    own), checked against the full DAG's decisions; the line reports the slowest share."""
    import numpy as np

    from dag_rider_amd.engine import Engine
    from dag_rider_amd.gen import CONFIGS, generate

    cfg = CONFIGS["c4"]
    d = generate(cfg, nthreads=CPU_THREADS)
    N = args.rank_share
    shares = [rank_share(cfg, d, r, N, local, max(args.steps, 1)) for r in range(N)]
    with Engine(cfg.n, cfg.faulty, d.nrounds, local) as e:
        e.append_packed(d)
        fc, fv = e.wave_commit(1, cfg.nwaves)
        e.wave_commit(1, cfg.nwaves)
        full_kms = e.last_kernel_ms()
    cm = np.concatenate([np.asarray(s["commit"], np.uint8) for s in shares])
    vc = np.concatenate([np.asarray(s["vcount"], np.int32) for s in shares])
    ok = bool((cm == fc).all() and (vc == fv).all())
    slow = max(shares, key=lambda s: s["ms"])
    # commit edges of the slowest share: strong degrees of rounds 4w-2..4w of its waves
    deg = np.asarray([int(np.unpackbits(d.strong[r * cfg.n * d.W:(r + 1) * cfg.n * d.W].view(np.uint8)).sum())
                      for r in range(4 * (slow["w0"] - 1), 4 * slow["w1"] + 1)], np.int64)
    base = 4 * (slow["w0"] - 1)
    edges = sum(int(deg[4 * w - 2 - base] + deg[4 * w - 1 - base] + deg[4 * w - base])
                for w in range(slow["w0"], slow["w1"] + 1) if vc[w - 1] >= 0)
    km = slow["kernel_ms"]
    return {
        "metric": "DAG edges traversed/sec (commit sweep, one rank's wave range)",
        "value": edges / (slow["ms"] / 1e3),
        "unit": "edges/s",
        "n_gpus": 1,
        "steps": max(args.steps, 1),
        "warmup": 1,
        "ms_per_step": slow["ms"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (seeded generator, SURVEY.md s8(d) C4 parameters)",
        "config": {"workload": f"C4 all-waves commit sweep split into {N} wave ranges (SURVEY.md s8(e) row 1): "
                               f"each share on its own mirror of its rounds, dr_wave_commit; line = slowest share",
                   "n": cfg.n, "rounds": cfg.last_round, "waves": cfg.nwaves, "parallelism": f"waves{N}"},
        "roofline": {"bound": "hbm", "achieved": slow["bytes"] / (km / 1e3) / 1e9 if km > 0 else None,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": slow["bytes"] / (km / 1e3) / 1e9 / HBM_PEAK_GBS if km > 0 else None,
                     "traffic": None, "kernel": "k_commit (waveReady commit rule)",
                     "bytes_per_launch": slow["bytes"], "ms_per_launch": km},
        "cpu_baseline": None,
        "detail": {"shares": [{k: s[k] for k in ("rank", "w0", "w1", "ms", "kernel_ms", "bytes", "GBps_kernel")}
                              for s in shares],
                   "full_dag_kernel_ms": full_kms, "verify_vs_full_dag": ok, "commit_edges_slowest": edges},
    }


def wsplit_share_bytes(p, n: int, W: int) -> int:
    """Algorithmic bytes of one slice's row pass (k_summary_commit): every strong row of
    slice rounds 1..top once, plus U and SD (bench kernel_bytes 'summary')."""
    T = p.nrounds - 1
    return T * n * W * 8 + T * W * 8 + 8 * T


def run_wave_split_shares(args, local: int):
    """--wave-split N on one GPU: the whole C4 replay split into N wave ranges
    (dag_rider_amd/split.py), every rank's slice on its own mirror, timed one after another
    on this GPU (what each of N GPUs runs), combined with the exchange done in memory and
    checked against the unsharded replay; the line reports the slowest share."""
    import numpy as np
    import torch

    from dag_rider_amd import _lib as L
    from dag_rider_amd.engine import Engine
    from dag_rider_amd.gen import CONFIGS, generate
    from dag_rider_amd.split import (SliceRank, check_and_offsets, combine_slices, owned_part, presence_prefix,
                                     slice_plans)

    cfg = CONFIGS["c4"]
    d = generate(cfg, nthreads=CPU_THREADS)
    N = args.wave_split
    plans = slice_plans(d, cfg.nwaves, N, halo=args.halo)
    gp = presence_prefix(d)
    ranks = [SliceRank(d, p, cfg.faulty, local, None, gp) for p in plans]
    shares, outs = [], []
    steps = max(args.steps, 1)
    for sr in ranks:
        sr.eng.set_phase_timing(1)
        for _ in range(max(args.warmup, 1)):
            sr.step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ms_sum = 0.0
        for _ in range(steps):
            sr.step()
            ms_sum += sr.step.ms_summary
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        res, sres = sr.step.result(), sr.eng.slice_result()
        res = dataclasses.replace(res, **{k: getattr(res, k).copy() for k in
                                          ("commit", "vcount", "push_off", "push_wave", "pop_count", "pop_digest",
                                           "pop_edges")})
        outs.append((res, sres))
        p = sr.p
        nb = wsplit_share_bytes(p, cfg.n, d.W)
        km = ms_sum / steps
        shares.append(dict(rank=p.rank, w0=p.w0, w1=p.w1, wf=p.wf, rounds=[p.off, p.top], seeded=p.seeded,
                           ms=dt * 1e3, summary_kernel_ms=km, row_bytes=nb,
                           GBps_summary=nb / (km / 1e3) / 1e9 if km > 0 else None,
                           pops_own=int(res.push_off[p.nwaves]) - int(res.push_off[p.own_w0 - 1])))
    summ = np.stack([sr.summary(*o) for sr, o in zip(ranks, outs)])
    offs, redo = check_and_offsets(plans, summ)
    for k, base in redo.items():  # (C4: never -- its canonical cone is full below the top)
        ranks[k].rebase(base)
        ranks[k].step()
        outs[k] = (ranks[k].step.result(), ranks[k].eng.slice_result())
        summ[k] = ranks[k].summary(*outs[k])
    if redo:
        offs, _ = check_and_offsets(plans, summ)
    got = combine_slices([owned_part(p, o[0], *off) for p, o, off in zip(plans, outs, offs)], summ)
    for sr in ranks:
        sr.close()
    with Engine(cfg.n, cfg.faulty, d.nrounds, local) as e:
        e.append_packed(d)
        want = e.replay(cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF)
    ok = same_replay(got, want)
    slow = max(shares, key=lambda x: x["ms"])
    # the slowest share's edges: its owned commits, chains and pops
    k = slow["rank"]
    S = summ[k]
    from dag_rider_amd.split import SUMMARY_FIELDS as F

    pa, pb = int(got.push_off[plans[k].w0 - 1]), int(got.push_off[plans[k].w1])
    share_edges = int(S[F.index("commit_edges")]) + int(S[F.index("own_chain_edges")]) + \
        int(np.asarray(got.pop_edges[pa:pb], np.uint64).sum(dtype=np.uint64))
    km = slow["summary_kernel_ms"]
    return {
        "metric": "DAG edges traversed/sec (commit+delivery, one rank's wave range of the whole replay)",
        "value": share_edges / (slow["ms"] / 1e3),
        "unit": "edges/s",
        "n_gpus": 1,
        "steps": steps,
        "warmup": max(args.warmup, 1),
        "ms_per_step": slow["ms"],
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (seeded generator, SURVEY.md s8(d) C4 parameters)",
        "config": {"workload": f"C4 full replay (waveReady persistent + orderVertices REF) split into {N} wave "
                               f"ranges (dag_rider_amd/split.py): each share on its own mirror of its rounds "
                               f"({args.halo}-wave halo below, dmax rounds above, seeded full); line = slowest "
                               f"share, exchange excluded (one all-gather of 13 words + the gather of the pops "
                               f"per replay in the N-GPU line)",
                   "n": cfg.n, "rounds": cfg.last_round, "waves": cfg.nwaves, "parallelism": f"wavesplit{N}"},
        "roofline": {"bound": "hbm", "achieved": slow["row_bytes"] / (km / 1e3) / 1e9 if km > 0 else None,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": slow["row_bytes"] / (km / 1e3) / 1e9 / HBM_PEAK_GBS if km > 0 else None,
                     "traffic": None, "kernel": "k_summary_commit over the slowest share's slice",
                     "bytes_per_launch": slow["row_bytes"], "ms_per_launch": km},
        "cpu_baseline": None,
        "detail": {"shares": shares, "verify_vs_unsharded": ok, "share_edges_slowest": share_edges,
                   "whole_replay_edges": int(got.commit_edges + got.chain_edges + got.deliver_edges),
                   "rebased_ranks": sorted(redo), "ms_max_over_shares": slow["ms"]},
    }


def wsplit_run(dist, rank: int, world: int, local: int, steps: int, warmup: int, halo: int):
    """The N-GPU wave-split replay of the ONE seed-4 C4 DAG: this rank's slice mirror,
    warm-up steps, a barrier, then exactly `steps` timed steps of dist_split_step (the
    slice replay, the 13-word all-gather over RCCL, offsets, the gather of the owned
    pops); rank 0 checks the combined replay against the unsharded engine.  Returns
    rank 0's view (None elsewhere); errors are reported, not raised."""
    import torch

    from dag_rider_amd import _lib as L
    from dag_rider_amd.gen import CONFIGS, generate
    from dag_rider_amd.split import SliceError, SliceRank, dist_split_step, presence_prefix, slice_plans

    cfg = CONFIGS["c4"]
    d = generate(cfg, nthreads=CPU_THREADS)
    dev = torch.device("cuda", local)
    err = None
    try:
        plans = slice_plans(d, cfg.nwaves, world, halo=halo)
        sr = SliceRank(d, plans[rank], cfg.faulty, local, None, presence_prefix(d))
        sr.eng.set_phase_timing(0)
        for _ in range(max(warmup, 1)):
            got, summ = dist_split_step(dist, sr, plans, dev)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            got, summ = dist_split_step(dist, sr, plans, dev)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        sr.close()
    except SliceError as ex:
        err, dt = f"SliceError: {ex}", 0.0
    t = torch.tensor([dt], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank != 0:
        return None
    if err:
        return dict(error=err)
    from dag_rider_amd.engine import Engine

    with Engine(cfg.n, cfg.faulty, d.nrounds, local) as e:
        e.append_packed(d)
        want = e.replay(cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF)
    ms = float(t.item()) / steps * 1e3
    edges = int(got.commit_edges + got.chain_edges + got.deliver_edges)
    return dict(ms=ms, edges=edges, verify_vs_unsharded=same_replay(got, want), world=world, halo=halo,
                ranges=[(p.w0, p.w1) for p in plans])


def colshard_child(args):
    """One rank of the process-column sharded C4 replay (BASELINE.json configs[3],
    SURVEY.md s8(e)): every rank holds 1/N of the target columns of the ONE seed-4 C4
    DAG; dr_shard_replay runs the memoized replay with the frontier all-gathered over
    RCCL (shard_memo.hpp).  Warm-up replays, a collective as the start barrier, then
    exactly --steps timed replays (each returns with its results in host memory).
    Rank 0 then checks every output against the unsharded engine's dr_replay."""
    from dag_rider_amd import _lib as L
    from dag_rider_amd.gen import CONFIGS, generate
    from dag_rider_amd.shard import ShardEngine, ShardReplayer

    cfg = CONFIGS["c4"]
    d = generate(cfg, nthreads=CPU_THREADS)
    se = ShardEngine(cfg.n, cfg.faulty, d.nrounds, args.cs_device, args.cs_world, args.cs_rank,
                     bytes.fromhex(args.cs_uid))
    se.append_packed(d)
    step = ShardReplayer(se, cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF)
    for _ in range(max(args.warmup, 1)):
        step()
    se.wave_commit(1, 1)  # a collective: every rank has finished its warm-up
    se.set_phase_timing(False)  # the timed replays record no phase events
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    dt = time.perf_counter() - t0
    se.set_phase_timing(True)
    step()  # one more replay (every rank) for the per-phase device times
    rep = step.result()
    st = se.stats()
    info = se.info()
    out = dict(rank=args.cs_rank, ms=dt / args.steps * 1e3, steps=args.steps, phases_ms=rep.ms,
               sweep_steps=st["rounds"], exchange_bytes=st["exchange_bytes"], edges=rep.total_edges,
               commits=int(rep.commit.sum()), pops=len(rep.pop_count), canon_segments=rep.sweep["canon_segments"],
               cols=(info["col0"], info["col1"]), row_bytes=(d.nrounds - 1) * cfg.n * 8 *
               ((cfg.n + 63) // 64 + args.cs_world - 1) // args.cs_world)
    se.close()
    if args.cs_rank == 0:
        from dag_rider_amd.engine import Engine

        with Engine(cfg.n, cfg.faulty, d.nrounds, args.cs_device) as e:
            e.append_packed(d)
            rr = e.replay(cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF)
        out["verify_vs_unsharded"] = same_replay(rep, rr)
    print(json.dumps(out), flush=True)


def colshard_run(dist, rank: int, world: int, local: int, steps: int, warmup: int, timeout_s: float = 300.0):
    """Run colshard_child in one child process per rank (a hung collective is killed
    by the time limit instead of hanging the job); returns every rank's result (or
    error) on every rank."""
    import subprocess

    from dag_rider_amd.shard import exchange_unique_id

    uid = exchange_unique_id(dist)
    cmd = [sys.executable, os.path.abspath(__file__), "--colshard-child", "--cs-uid", uid.hex(),
           "--cs-rank", str(rank), "--cs-world", str(world), "--cs-device", str(local),
           "--steps", str(steps), "--warmup", str(warmup)]
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s)
        lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
        res = json.loads(lines[-1]) if p.returncode == 0 and lines else dict(
            rank=rank, error=f"exit {p.returncode}: " + (p.stderr or "")[-400:])
    except subprocess.TimeoutExpired:
        res = dict(rank=rank, error=f"timed out after {timeout_s} s")
    allr = [None] * world
    dist.all_gather_object(allr, res)
    return allr


def c4_multi_line(args, world: int, cs_all, replicas, split, wsplit=None):
    """The N > 1 line of the C4 config: the column-sharded replay of ONE C4 DAG
    (strong scaling: the same 1.75e12 edges per step whatever N; BASELINE.json
    configs[3] "process-column sharded across 2/4/8 GPUs with RCCL frontier
    all-gather"), its slowest rank's time per replay.  The independent-replicas
    number (every rank its own C4 DAG) goes to detail.replicas.  If any rank's
    sharded run failed, the line says so and carries the replicas number instead,
    labelled as such ("parallelism": "replicasN").  A sharded replay that rank 0 found
    different from the unsharded engine's counts as failed the same way: its number is
    never published."""
    ok = all(r is not None and "error" not in r for r in cs_all)
    verified = ok and bool(cs_all[0].get("verify_vs_unsharded"))
    if ok and not verified:
        cs_all = [dict(r, error="verify_vs_unsharded failed") if r.get("rank") == 0 else r for r in cs_all]
        ok = False
    base = {
        "metric": "DAG edges traversed/sec (commit+delivery)",
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "higher_is_better": True,
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (seeded generator, SURVEY.md s8(d) C4 parameters)",
        "cpu_baseline": None,
    }
    rep_detail = dict(replicas, parallelism=f"replicas{world}", scaling="weak",
                      note="every rank replays its own C4 DAG (seed 4 + rank), unsharded; value = summed edges / "
                           "slowest rank")
    cs_detail = dict(ok=ok and verified, ranks=cs_all,
                     ms=max(r["ms"] for r in cs_all) if ok and verified else None)
    if wsplit is not None and "error" not in wsplit and wsplit.get("verify_vs_unsharded"):
        ms = wsplit["ms"]
        return dict(base, **{
            "value": wsplit["edges"] / (ms / 1e3),
            "ms_per_step": ms,
            "scaling": "strong",
            "config": {"workload": "C4 full replay of ONE DAG (n=1024 x 4000 rounds, seed 4) split into "
                                   f"{world} wave ranges, one per GPU (dag_rider_amd/split.py): each GPU mirrors "
                                   f"its waves' rounds plus a {wsplit['halo']}-wave halo below and the dmax rounds "
                                   "above, replays waveReady (persistent decidedWave) + orderVertices (ref) for its "
                                   "waves, then one RCCL all-gather of 13 words per rank (canonical prefixes, "
                                   "checks) and one of the owned pops; value = the whole replay's edges / the "
                                   "slowest rank's time per step",
                       "n": 1024, "rounds": 4000, "waves": 1000, "parallelism": f"wavesplit{world}"},
            "roofline": replicas.get("roofline"),
            "detail": {"verify_vs_unsharded": True, "wsplit": wsplit, "colshard": cs_detail, "replicas": rep_detail,
                       "commit_split": split,
                       "roofline_note": "roofline: rank 0's unsharded replica replay (same kernels, whole DAG)"},
        })
    if ok and verified:
        ms = max(r["ms"] for r in cs_all)
        edges = cs_all[0]["edges"]
        r0 = cs_all[0]
        summ = r0["phases_ms"].get("summary", 0.0)
        rb = r0["row_bytes"]
        return dict(base, **{
            "value": edges / (ms / 1e3),
            "ms_per_step": ms,
            "scaling": "strong",
            "config": {"workload": "C4 full replay of ONE DAG (n=1024 x 4000 rounds, seed 4), process columns sharded "
                                   f"across {world} GPUs (1/{world} of every strong row and the weak edges targeting "
                                   "its columns per GPU), frontier all-gathered over RCCL: waveReady (persistent "
                                   "decidedWave) + orderVertices (ref, full cones), memoized (shard_memo.hpp)",
                       "n": 1024, "rounds": 4000, "waves": 1000, "parallelism": f"colshard{world}"},
            "roofline": {"bound": "hbm", "achieved": rb / (summ / 1e3) / 1e9 if summ > 0 else None,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": rb / (summ / 1e3) / 1e9 / HBM_PEAK_GBS if summ > 0 else None, "traffic": None,
                         "kernel": "summary phase per rank (k_ms_summary over the rank's columns + K^cand exchange "
                                   "+ canonical segment), rank 0", "bytes_per_launch": rb, "ms_per_launch": summ},
            "detail": {"verify_vs_unsharded": verified, "ranks": cs_all, "replicas": rep_detail,
                       "commit_split": split, "wsplit": wsplit},
        })
    errs = [r.get("error") if r else "no result" for r in cs_all]
    return dict(base, **{
        "value": replicas["value"],
        "ms_per_step": replicas["ms_per_step"],
        "scaling": "weak",
        "config": {"workload": f"C4 full replay, independent replicas (seed 4 + rank) -- the column-sharded run "
                               f"FAILED on this node: {errs}", "n": 1024, "rounds": 4000, "waves": 1000,
                   "parallelism": f"replicas{world}"},
        "roofline": replicas.get("roofline"),
        "detail": {"colshard_errors": errs, "ranks": cs_all, "replicas": rep_detail, "commit_split": split,
                   "wsplit": wsplit},
    })


def run_c5(args, rank: int, world: int, local: int, dist):
    """C5 (BASELINE.json configs[4]): the fixed batch of 4096 independent n=128 x 128-round
    replays (seeds 5000+i), split across ranks (strong scaling); each rank replays its
    DAGs as one fused dr_replay_batch launch (batch.hpp)."""
    import torch

    from dag_rider_amd import _lib as L
    from dag_rider_amd.engine import Engine, ReplayBatchView
    from dag_rider_amd.gen import c5_config, generate

    total = 4096
    lo, hi = rank * total // world, (rank + 1) * total // world
    if args.dags:  # one GPU's share at N = 4096 / dags (e.g. 512 = one rank's share at N = 8)
        if world > 1:
            raise SystemExit("--dags is a single-GPU option")
        lo, hi = 0, min(args.dags, total)
    t0 = time.perf_counter()
    engines, dags, dag_bytes = [], [], 0
    for i in range(lo, hi):
        cfg = c5_config(i)
        d = generate(cfg)
        e = Engine(cfg.n, cfg.faulty, d.nrounds, local, shared_stream=True)  # one HIP stream for the batch
        e.append_packed(d)
        engines.append(e)
        dags.append(d)
        dag_bytes += d.nrounds * cfg.n * d.W * 8 + weak_columns(d) * (4 + d.W * 8)
    log(f"[rank {rank}] C5 DAGs {lo}..{hi - 1} loaded in {time.perf_counter() - t0:.1f} s")
    nw = c5_config(0).nwaves
    # results in place (dr_replay_batch_view): the step ends with every DAG's results in host
    # memory, without 4096 per-context copies
    b = ReplayBatchView(engines, nw, L.DR_CHAIN_PERSISTENT, args.deliver_mode)
    for _ in range(args.warmup):
        b.run()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step_ends = []
    for _ in range(args.steps):
        b.run()  # synchronous: the step ends with every DAG's results on the host
        step_ends.append(time.perf_counter())
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    wall = time.perf_counter() - t0  # the timed region ends here: reading the results back is not a step
    step_ms = [(b1 - b0) * 1e3 for b0, b1 in zip([t0] + step_ends[:-1], step_ends)]
    res = b.results()
    edges = sum(r.total_edges for r in res)
    kms = max(r.ms["deliver"] for r in res)  # the fused launch's device time (HIP events)
    dt, total_edges = reduce_over_ranks(dist, wall, edges, "cuda")
    if rank != 0:
        return None
    cpu = None
    if not args.no_cpu and world == 1:
        cpu = cpu_c5(dags, args.deliver_mode, res) if not args.dags else None
    ach = dag_bytes / (kms / 1e3) / 1e9 if kms > 0 else 0.0
    form = b.form()  # the fused kernel that ran (AUTO: the wave form above 6 DAGs per CU)
    # PMC traffic of this form at this batch size, when the traffic file holds it; the bound
    # from the measured bytes' rate: >= 25 % of peak reads as HBM-bound, else latency-bound
    tr_bytes = tr_file = None
    if not args.dags or args.dags >= total:
        tr_bytes, tr_file = measured_traffic("batch_" + form, 2, "c5")
    tr_rate = tr_bytes / (kms / 1e3) / 1e9 if tr_bytes and kms > 0 else None
    bound = "hbm" if max(ach, tr_rate or 0.0) >= 0.25 * HBM_PEAK_GBS else "latency"
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
        "config": {"workload": f"C5: {total if not args.dags else hi - lo} independent n=128 x 128-round replays "
                               "(waveReady + orderVertices "
                               f"{'paper' if args.deliver_mode else 'ref'}, persistent decidedWave), split across ranks",
                   "dags": total if not args.dags else hi - lo, "dags_per_rank": hi - lo, "n": 128, "rounds": 128, "waves": nw,
                   "parallelism": f"dp{world}" if world > 1 else "single"},
        "roofline": {"bound": bound, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": ach / HBM_PEAK_GBS, "traffic": tr_bytes,
                     "traffic_unit": f"bytes/launch (rocprofv3 PMC, {tr_file})",
                     "traffic_rate_GBps": tr_rate,
                     "kernel": f"{form} ({'batch1w.hpp' if form.endswith('1w') else 'batch.hpp'})",
                     "bytes_per_launch": dag_bytes, "ms_per_launch": kms,
                     "note": "unique DAG bytes (strong rows + weak columns) once per launch; bound from the "
                             "larger of the algorithmic and the measured rate"},
        "cpu_baseline": cpu,
        "detail": {"edges_per_step": edges, "commits": int(sum(int(r.commit.sum()) for r in res)),
                   "pops": int(sum(len(r.pop_count) for r in res)),
                   # the last step's phases (dr_replay_batch, first output): host prep before the
                   # launch, launch -> results on the host, the copy back (device), the unpack
                   "step_phases_ms": dict(b.host_phases(), kernel=kms),
                   "step_ms": step_ms},
    }


def cpu_c5(dags, deliver_mode, gpu_res, lit_dags: int = 16, lit_waves: int = 4):
    """C5 on the host, one DAG per thread (independent replays on every core): the
    bitset restatement on all 4096 DAGs (checked against the GPU's per-DAG outputs)
    and the literal restatement (the reference's algorithm) on a bounded sample,
    waves 1..lit_waves of the first lit_dags DAGs (a whole literal C5 replay takes
    minutes per DAG: its cost grows ~ w^2 per wave).  Median of 5 runs each."""
    from concurrent.futures import ThreadPoolExecutor

    import oracle

    nt = cpu_threads()
    f = (dags[0].n - 1) // 3
    nw = (dags[0].nrounds - 1) // 4

    def lit(i):
        return oracle.LDag(packed=dags[i], nrounds=4 * lit_waves + 1).replay(f, lit_waves, oracle.CHAIN_PERSISTENT,
                                                                             deliver_mode)

    def bit(i):
        return oracle.PDag(dags[i]).replay(f, nw, oracle.CHAIN_PERSISTENT, deliver_mode, nthreads=1)

    out = {}
    for name, fn, k in (("literal", lit, min(lit_dags, len(dags))), ("bitset", bit, len(dags))):
        ts = []
        for i in range(5):
            t0 = time.perf_counter()
            with ThreadPoolExecutor(nt) as ex:
                rs = list(ex.map(fn, range(k)))
            ts.append(time.perf_counter() - t0)
            log(f"[cpu c5] {name} run {i}: {ts[-1]:.2f} s")
        med = statistics.median(ts)
        e = sum(r.commit_edges + (r.chain_edges if name == "bitset" else 0) + r.deliver_edges for r in rs)
        out[name] = dict(value=e / med, unit="edges/s", cores=nt, kind="port", dags=k, median_s=med, runs_s=ts)
        if name == "bitset":
            out[name]["matches_gpu"] = bool(all((r.pop_digest == g.pop_digest).all() and (r.commit == g.commit).all()
                                                for r, g in zip(rs, gpu_res)))
    lt = out["literal"]
    return dict(value=lt["value"], unit="edges/s", cores=nt, kind="port",
                sample=f"C5 DAGs 0..{lt['dags'] - 1}, waves 1..{lit_waves} each, literal replay "
                       f"(oracle/ref_literal.c), one DAG per thread on {nt} threads, median of 5 runs",
                literal=lt, bitset_all_dags=out["bitset"], host=cpu_info())


def run_loop(args, local: int):
    """The drop-in call pattern on C4 (the reference's Start loop wired as Alg. 3): for
    each wave w the 4 new rounds are appended (dr_append_rounds_packed), waveReady(w)
    runs (dr_wave_ready: incremental round summaries, commit rule, leader chain) and
    on commit orderVertices delivers the pushed leaders (dr_order_vertices: the
    canonical cone of the new top, per-pop counts and digests).  Per-wave latency;
    outputs checked against one dr_replay of the whole DAG."""
    import numpy as np
    import torch

    from dag_rider_amd import _lib as L
    from dag_rider_amd.engine import Engine
    from dag_rider_amd.gen import CONFIGS, generate

    cfg = CONFIGS["c4"]
    d = generate(cfg, nthreads=CPU_THREADS)
    nw = cfg.nwaves if args.loop_waves <= 0 else min(args.loop_waves, cfg.nwaves)

    def one_pass(e):
        e.append_packed(d, 0, 1)
        decided = 0
        lat = {"append": [], "wave_ready": [], "order_vertices": [], "wave": []}
        aph = {k: [] for k in ("build", "stage_rows", "stage_rounds", "copy_wait")}
        commit, vcount, pushes, pc, pdg = [], [], [], [], []
        torch.cuda.synchronize()
        t_start = time.perf_counter()
        for w in range(1, nw + 1):
            t0 = time.perf_counter()
            e.append_packed(d, 4 * w - 3, 4 * w + 1)
            t1 = time.perf_counter()
            for k, v in e.append_phases().items():
                aph[k].append(v * 1e-3)
            cm, vc, pushed = e.wave_ready(w, decided)
            t2 = time.perf_counter()
            commit.append(cm)
            vcount.append(vc)
            if cm:
                pushes += pushed
                _, cnt, dg = e.order_vertices([(4 * (x - 1) + 1, 1) for x in pushed], 4 * w, L.DR_DELIVER_REF,
                                              cap=0)
                pc += cnt.tolist()
                pdg += dg.tolist()
                decided = w
            t3 = time.perf_counter()
            lat["append"].append(t1 - t0)
            lat["wave_ready"].append(t2 - t1)
            lat["order_vertices"].append(t3 - t2)
            lat["wave"].append(t3 - t0)
        total = time.perf_counter() - t_start
        lat.update({"append." + k: v for k, v in aph.items()})
        return total, lat, (np.asarray(commit, np.uint8), np.asarray(vcount, np.int32), pushes, pc, pdg)

    # warm-up pass (first-call costs), then the measured pass on a fresh mirror
    with Engine(cfg.n, cfg.faulty, 4 * nw + 1, local) as e:
        one_pass(e)
    with Engine(cfg.n, cfg.faulty, 4 * nw + 1, local) as e:
        total, lat, (cm, vc, pushes, pc, pdg) = one_pass(e)
        ref = e.replay(nw, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF)
    ok = bool((cm == ref.commit).all() and (vc == ref.vcount).all() and pushes == ref.push_wave.tolist()
              and pc == ref.pop_count.tolist() and pdg == ref.pop_digest.tolist())

    def pct(x):
        a = np.asarray(x) * 1e6
        return dict(p50=float(np.percentile(a, 50)), p90=float(np.percentile(a, 90)),
                    p99=float(np.percentile(a, 99)), mean=float(a.mean()), max=float(a.max()))

    edges = ref.total_edges
    return {
        "metric": "DAG edges traversed/sec (commit+delivery)",
        "value": edges / total,
        "unit": "edges/s",
        "n_gpus": 1,
        "steps": 1,
        "warmup": 1,
        "ms_per_step": total * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (seeded generator, SURVEY.md s8(d) C4 parameters)",
        "config": {"workload": f"C4 per-wave drop-in loop, waves 1..{nw}: append 4 rounds -> dr_wave_ready -> "
                               "dr_order_vertices (ref, counts + digests), host wall clock per call",
                   "n": cfg.n, "rounds": 4 * nw, "waves": nw, "parallelism": "single"},
        "roofline": None,
        "cpu_baseline": None,
        "detail": {"latency_us": {k: pct(v) for k, v in lat.items()}, "verify_vs_replay": ok,
                   "edges": edges, "commits": int(cm.sum()), "pops": len(pc)},
    }


def spawn_ranks(args) -> int:
    """bench.py --gpus N outside torchrun: N ranks via torch.distributed.run, started
    before this process touches a GPU; their exit status is ours."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    log(f"[bench] spawning {args.gpus} ranks: {' '.join(cmd)}")
    return subprocess.call(cmd)


def dist_selftest(rank: int, world: int, local: int, args=None) -> int:
    """The multi-rank plumbing without a GPU (gloo): every rank reports in, the job's
    numbers are reduced exactly as the GPU path reduces them, and the C4 N > 1 line is
    built by the same code (c4_multi_line) from every rank's sharded-replay result
    (synthetic here: rank r took 0.25 (r+1) ms; --selftest-fail makes rank 1 fail,
    --selftest-wrong makes rank 0's check against the unsharded engine fail)
    (tests/test_dist_gloo.py)."""
    import torch.distributed as dist

    dist.init_process_group("gloo", init_method="env://")
    try:
        dt, tot = reduce_over_ranks(dist, 0.25 * (rank + 1), 1000 * (rank + 1), "cpu")
        ranks = [None] * world
        dist.all_gather_object(ranks, dict(rank=rank, local_rank=local, pid=os.getpid()))
        fail = args is not None and args.selftest_fail and rank == 1
        wrong = args is not None and args.selftest_wrong  # rank 0's check against the unsharded engine fails
        mine = dict(rank=rank, error="selftest failure") if fail else dict(
            rank=rank, ms=0.25 * (rank + 1), edges=10 ** 9, verify_vs_unsharded=not wrong, phases_ms={"summary": 0.1},
            row_bytes=1000)
        cs_all = [None] * world
        dist.all_gather_object(cs_all, mine)
        if rank == 0:
            a = argparse.Namespace(steps=3, warmup=1)
            reps = dict(value=tot / dt, ms_per_step=dt * 1e3, roofline=None)
            line = c4_multi_line(a, world, cs_all, reps, None)
            line.update(metric_selftest="dist selftest", selftest_value=tot / dt, ranks=ranks,
                        selftest_ms_per_step=dt * 1e3)
            print(json.dumps(line), flush=True)
    finally:
        dist.destroy_process_group()
    return 0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c4", choices=["c1", "c2", "c3", "c4", "c4-deep", "c4-deep64", "c4-dups", "c5",
                                                       "c4-loop", "c4-far", "c4-q8", "c4-up"])
    ap.add_argument("--graph", action="store_true",
                    help="replay the captured hipGraph of the launch sequence (DR_OPT_REPLAY_GRAPH)")
    ap.add_argument("--no-memo", action="store_true",
                    help="DR_OPT_MEMO 0: every cone swept whole (the general full-cone sweep line)")
    ap.add_argument("--deliver", default="ref", choices=["ref", "paper"])
    ap.add_argument("--cpu-budget", type=float, default=40.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--phase-timing", type=int, default=1, help=argparse.SUPPRESS)  # 0: no events (experiment)
    ap.add_argument("--event-every", type=int, default=4,
                    help="bracket the summary pass with HIP events on every k-th timed step (each event "
                         "record costs the stream ~4 us: tools/experiments/launch_probe.hip)")
    ap.add_argument("--loop-waves", type=int, default=0, help="c4-loop: waves to run (0 = all)")
    ap.add_argument("--dags", type=int, default=0, help="c5 on one GPU: replay only the first N DAGs")
    ap.add_argument("--rank-share", type=int, default=0,
                    help="one GPU: time every rank's share of the C4 wave-range commit split for N ranks")
    ap.add_argument("--wave-split", type=int, default=0,
                    help="one GPU: time every rank's share of the C4 replay split into N wave ranges")
    ap.add_argument("--halo", type=int, default=8, help="wave split: waves below each rank's range it mirrors")
    ap.add_argument("--no-wsplit", action="store_true", help="N>1: skip the wave-split replay")
    ap.add_argument("--verify", action="store_true", help="check the replay against the bitset oracle")
    ap.add_argument("--verify-general", action="store_true",
                    help="check the replay against the general sweep's (memo off) on the GPU (c4-up: no CPU oracle "
                         "takes edges to the same round at this size)")
    ap.add_argument("--colshard", action="store_true",
                    help="also run the process-column sharded C4 sweep (default on when N>1)")
    ap.add_argument("--no-colshard", action="store_true")
    ap.add_argument("--dist-selftest", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--selftest-fail", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--selftest-wrong", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--colshard-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cs-uid", default="", help=argparse.SUPPRESS)
    ap.add_argument("--cs-rank", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--cs-world", type=int, default=1, help=argparse.SUPPRESS)
    ap.add_argument("--cs-device", type=int, default=0, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.colshard_child:
        colshard_child(args)
        return 0
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn_ranks(args)
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:
        log(f"[bench] WORLD_SIZE={world} but --gpus {args.gpus}: refusing to report a mislabelled line")
        return 2
    if args.dist_selftest:
        return dist_selftest(rank, world, local, args)

    from dag_rider_amd import _lib as L

    args.deliver_mode = L.DR_DELIVER_PAPER if args.deliver == "paper" else L.DR_DELIVER_REF
    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", init_method="env://")
    torch.cuda.set_device(local)

    from dag_rider_amd.engine import Engine, Replayer
    from dag_rider_amd.gen import CONFIGS, generate

    if args.config == "c5":
        out = run_c5(args, rank, world, local, dist)
        if out is not None:
            emit_line(out)
        if dist:
            dist.destroy_process_group()
        return 0
    if args.rank_share:
        if world > 1 or args.config != "c4":
            log("[bench] --rank-share is a single-GPU line of the C4 commit split")
            return 2
        emit_line(run_rank_share(args, local))
        return 0
    if args.wave_split:
        if world > 1 or args.config != "c4":
            log("[bench] --wave-split is a single-GPU line of the C4 replay's wave split")
            return 2
        emit_line(run_wave_split_shares(args, local))
        return 0
    if args.config == "c4-loop":
        if world > 1:
            log("[bench] c4-loop is a single-GPU latency line")
            return 2
        emit_line(run_loop(args, local))
        return 0

    cfg = rank_config(CONFIGS[args.config], rank, world)
    t0 = time.perf_counter()
    d = generate(cfg, nthreads=CPU_THREADS)
    log(f"[rank {rank}] generated {cfg} in {time.perf_counter() - t0:.1f} s")
    eng = Engine(cfg.n, cfg.faulty, d.nrounds, local)
    if args.no_memo:
        eng.set_memo(False)
    if args.graph:
        eng.set_replay_graph(True)
    t0 = time.perf_counter()
    eng.append_packed(d)
    log(f"[rank {rank}] loaded DAG into HBM in {time.perf_counter() - t0:.1f} s")

    # one step = one dr_replay of every wave into output buffers allocated once
    step = Replayer(eng, cfg.nwaves, L.DR_CHAIN_PERSISTENT, args.deliver_mode)

    # timed steps: HIP events around the summary pass only (the dominant kernel);
    # every other phase is timed by one extra, untimed-by-the-clock replay below
    eng.set_phase_timing(args.phase_timing)
    for _ in range(args.warmup):
        step()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ms_summary, n_ev = 0.0, 0
    every = max(1, args.event_every) if args.phase_timing == 1 else 1
    for i in range(args.steps):
        if every > 1:  # (a host-side option: no device work)
            eng.set_phase_timing(1 if i % every == 0 else 0)
        step()
        if i % every == 0:
            ms_summary += step.ms_summary
            n_ev += 1
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    wall = time.perf_counter() - t0  # the timed region ends here
    graph_state = eng.replay_graph_state()  # 1: the timed steps launched the captured hipGraph
    res = step.result()
    res = dataclasses.replace(res, **{k: getattr(res, k).copy() for k in
                                      ("commit", "vcount", "push_off", "push_wave", "pop_count", "pop_digest",
                                       "pop_edges")})
    dt, total_edges = reduce_over_ranks(dist, wall, res.total_edges, "cuda")
    eng.set_phase_timing(2)
    prof = eng.replay(cfg.nwaves, L.DR_CHAIN_PERSISTENT, args.deliver_mode)  # per-phase HIP event times
    res.ms = dict(prof.ms, summary=ms_summary / max(n_ev, 1))

    verify = None
    cpu = cpu2 = None
    if rank == 0 and world == 1 and not args.no_cpu:
        runs = 5 if cfg.n * cfg.last_round <= 1024 * 4000 else 3
        cpu2, want = cpu_bitset(cfg, d, CPU_THREADS, runs, args.deliver_mode)
        verify = same_replay(res, want)
        cpu = cpu_literal(cfg, d, args.cpu_budget, res.total_edges, args.deliver_mode)
    elif args.verify_general and rank == 0:
        with Engine(cfg.n, cfg.faulty, d.nrounds, local) as eg:
            eg.append_packed(d)
            eg.set_memo(False)
            t0 = time.perf_counter()
            wantg = eg.replay(cfg.nwaves, L.DR_CHAIN_PERSISTENT, args.deliver_mode)
            log(f"[rank 0] general-sweep replay (memo off) in {time.perf_counter() - t0:.1f} s, path "
                f"{eg.last_replay_path()}")
        verify = same_replay(res, wantg)
    elif args.verify and rank == 0:
        import oracle

        want = oracle.PDag(d).replay(cfg.faulty, cfg.nwaves, oracle.CHAIN_PERSISTENT, args.deliver_mode,
                                     nthreads=CPU_THREADS)
        verify = same_replay(res, want)

    split = colshard = None
    multi = world > 1 and args.config == "c4" and not args.no_colshard
    if world > 1 and args.config == "c4":
        split = commit_split(dist, rank, world, local, res.commit if rank == 0 else None,
                             res.vcount if rank == 0 else None)
    if multi or (args.colshard and args.config == "c4"):
        if dist is None:  # one-rank RCCL group (--colshard at N=1): gloo-free id exchange
            class _One:
                @staticmethod
                def get_rank(group=None):
                    return 0

                @staticmethod
                def broadcast_object_list(box, src=0, group=None):
                    return None

                @staticmethod
                def all_gather_object(out, obj):
                    out[0] = obj

            colshard = colshard_run(_One, rank, 1, local, args.steps, args.warmup)
        else:
            colshard = colshard_run(dist, rank, world, local, args.steps, args.warmup)
    if rank == 0 and colshard is not None:
        log(f"[colshard] {colshard}")
    wsplit = None
    if world > 1 and args.config == "c4" and not args.no_wsplit:
        wsplit = wsplit_run(dist, rank, world, local, args.steps, args.warmup, args.halo)
        if rank == 0:
            log(f"[wsplit] {wsplit}")

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return 0

    exc = eng.exception_stats()
    kb = kernel_bytes(cfg, d, res, exc["regular_delta"], eng.mirror_stats(), (fuse_mask() & 1) != 0)
    # dominant kernel = the phase with the largest device time (HIP events)
    dom = max(kb, key=lambda k: kb[k]["ms"])
    ach = kb[dom]["bytes"] / (kb[dom]["ms"] / 1e3) / 1e9 if kb[dom]["ms"] > 0 else 0.0
    # PMC traffic of the dominant phase's kernels for this row stride (REF delivery: the
    # profiled launch sequence); lines whose dominant kernel moves < 1 % of peak in its time
    # are latency-bound and say so
    tr_bytes, tr_file = (measured_traffic(dom, (cfg.n + 63) // 64, cfg.name) if args.deliver == "ref" and not args.no_memo
                         else (None, None))
    bound = "hbm" if ach >= 0.01 * HBM_PEAK_GBS else "latency"
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
        "data": f"synthetic (seeded generator, SURVEY.md s8(d) {cfg.name.upper()} parameters)",
        "replay_form": {1: "hipGraph", 0: "launches", -1: "launches (capture failed)"}[graph_state],
        "config": {"workload": f"{cfg.name.upper()} full replay: n={cfg.n} x {cfg.last_round} rounds, {cfg.nwaves} "
                               f"waves, waveReady (persistent decidedWave) + orderVertices ({args.deliver}"
                               f"{', full cones' if args.deliver == 'ref' else ', dedup'}) per commit"
                               + (" -- memo off (DR_OPT_MEMO 0): every cone swept whole" if args.no_memo else ""),
                   "n": cfg.n, "rounds": cfg.last_round, "waves": cfg.nwaves,
                   "parallelism": f"replicas{world}" if world > 1 else "single"},
        "roofline": {"bound": bound, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": ach / HBM_PEAK_GBS,
                     "traffic": tr_bytes, "traffic_unit": f"bytes/launch (rocprofv3 PMC, {tr_file})",
                     "kernel": kb[dom]["kernel"], "bytes_per_launch": kb[dom]["bytes"],
                     "ms_per_launch": kb[dom]["ms"]},
        "cpu_baseline": cpu,
        "cpu_bitset": cpu2,
        "detail": {"edges_per_step": res.total_edges, "commit_edges": res.commit_edges,
                   "chain_edges": res.chain_edges, "deliver_edges": res.deliver_edges,
                   "commits": int(res.commit.sum()), "pops": int(len(res.pop_count)),
                   "ms": res.ms, "ms_note": f"summary: mean over the {n_ev} timed steps whose summary pass HIP events "
                   f"bracket (every {every}th: each record costs the stream ~4 us); other phases: one "
                   "profiling replay after them (DR_OPT_PHASE_TIMING=2)",
                   "sweep": res.sweep, "verify_vs_oracle": verify, "exceptions": exc,
                   "replay_path": {0: "memo", 1: "memo, upward weak edges verified (k_verify_up)",
                                   2: "general sweep (an upward edge changes a cone)", 3: "general sweep",
                                   -1: "none"}.get(eng.last_replay_path(), "?"),
                   "commit_split": split, "colshard": colshard[0] if colshard else None,
                   "kernels": {k: dict(v, GBps=(v["bytes"] / (v["ms"] / 1e3) / 1e9 if v["ms"] > 0 else None))
                               for k, v in kb.items()}},
    }
    if multi:
        out = c4_multi_line(args, world, colshard, dict(value=out["value"], ms_per_step=ms_per_step,
                                                        roofline=out["roofline"], edges_per_step=res.total_edges,
                                                        verify_vs_oracle=verify), split, wsplit)
    emit_line(out)
    if dist:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
