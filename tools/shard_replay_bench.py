"""Time the memoized column-sharded replay (dr_shard_replay, shard_memo.hpp) on one GPU:
C4 (or the config named by --config), local mode with G column shards in one context
(the same kernels and column split as RCCL mode; the exchange is the shared frontier
buffer).  Each line: G, wall ms per replay (median of --runs), per-phase device ms,
steps, and the check against the unsharded engine's dr_replay."""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from dag_rider_amd import _lib as L
    from dag_rider_amd.engine import Engine
    from dag_rider_amd.gen import CONFIGS, generate
    from dag_rider_amd.shard import ShardEngine, ShardReplayer

    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--runs", type=int, default=20)
    ap.add_argument("--shards", default="1,2,4,8")
    ap.add_argument("--stepped", default="0,1", help="replay forms: 0 fused, 1 stepped (DR_SHARD_OPT_STEPPED)")
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    d = generate(cfg, nthreads=16)
    with Engine(cfg.n, cfg.faulty, d.nrounds, 0) as e:
        e.append_packed(d)
        rref = e.replay(cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF)
    for G, stepped in [(int(g), int(s)) for g in args.shards.split(",") for s in args.stepped.split(",")]:
        with ShardEngine(cfg.n, cfg.faulty, d.nrounds, 0, nshards=G) as se:
            se.append_packed(d)
            se.set_stepped(bool(stepped))
            rp = ShardReplayer(se, cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF)  # outputs allocated once
            rp()  # warm-up
            se.set_phase_timing(False)  # timed replays: no phase events
            walls = []
            for _ in range(args.runs):
                t0 = time.perf_counter()
                rp()
                walls.append((time.perf_counter() - t0) * 1e3)
            se.set_phase_timing(True)
            rp()  # one more replay for the per-phase device times
            r = rp.result()
            st = se.stats()
            ok = bool((r.commit == rref.commit).all() and (r.vcount == rref.vcount).all()
                      and (r.push_off == rref.push_off).all() and (r.push_wave == rref.push_wave).all()
                      and (r.pop_count == rref.pop_count).all() and (r.pop_digest == rref.pop_digest).all()
                      and (r.pop_edges == rref.pop_edges).all()
                      and (r.commit_edges, r.chain_edges, r.deliver_edges)
                      == (rref.commit_edges, rref.chain_edges, rref.deliver_edges))
            print(json.dumps(dict(config=cfg.name, G=G, memo=True, form="stepped" if stepped else "fused", replay_ok=ok, ms_wall_median=statistics.median(walls),
                                  ms_wall_min=min(walls), runs=walls, phases_ms=r.ms, device_ms=sum(r.ms.values()), steps=st["rounds"], host_syncs=st["host_syncs"],
                                  canon_segments=r.sweep["canon_segments"], cones=r.sweep["count"],
                                  edges=r.total_edges)), flush=True)


if __name__ == "__main__":
    main()
