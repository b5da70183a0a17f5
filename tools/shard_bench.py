"""Time the column-sharded path on one GPU, C4 DAG, local mode with G = 1, 2, 4, 8
column shards in one context (same kernels and column split as RCCL mode, the
exchange being the shared frontier buffer), with the persistent cooperative sweep
and with one launch per round:
  - reach sets (strong + weak, rounds 0..leader) of the 64 newest wave leaders;
  - the whole replay (dr_shard_replay: commit votes, chains, delivery cones and
    emission), checked against the unsharded engine's dr_replay.
Prints one JSON line per (G, launch mode)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from dag_rider_amd import _lib as L
    from dag_rider_amd.engine import Engine
    from dag_rider_amd.gen import CONFIGS, generate
    from dag_rider_amd.shard import ShardEngine

    cfg = CONFIGS["c4"]
    d = generate(cfg, nthreads=16)
    froms = [(4 * w - 3, 1) for w in range(cfg.nwaves, cfg.nwaves - 64, -1)]
    bottoms = [0] * len(froms)
    with Engine(cfg.n, cfg.faulty, d.nrounds, 0) as e:
        e.append_packed(d)
        ref = e.reach_sets(froms, bottoms, False)
        rref = e.replay(cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF)
    for G in [int(x) for x in (sys.argv[1:] or ["1", "2", "4", "8"])]:
        with ShardEngine(cfg.n, cfg.faulty, d.nrounds, 0, nshards=G) as se:
            se.append_packed(d)
            for persistent in (True, False):
                se.set_persistent(persistent)
                got = se.reach_sets(froms, bottoms, False)
                runs = []
                for _ in range(3):
                    se.reach_sets(froms, bottoms, False)
                    runs.append(se.stats())
                st = min(runs, key=lambda x: x["ms"])
                ok = all((a == b).all() for a, b in zip(got, ref))
                reps = []
                for _ in range(2):
                    t0 = time.perf_counter()
                    r = se.replay(cfg.nwaves, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF)
                    reps.append((time.perf_counter() - t0, r, se.stats()))
                wall, r, rst = min(reps, key=lambda x: x[0])
                rok = bool((r.commit == rref.commit).all() and (r.vcount == rref.vcount).all()
                           and (r.push_wave == rref.push_wave).all() and (r.pop_count == rref.pop_count).all()
                           and (r.pop_digest == rref.pop_digest).all() and (r.pop_edges == rref.pop_edges).all()
                           and r.total_edges == rref.total_edges)
                print(json.dumps(dict(G=G, persistent=persistent, reach_ok=bool(ok),
                                      reach_us_per_round=1e3 * st["ms"] / st["rounds"], reach=st,
                                      replay_ok=rok, replay_ms_wall=wall * 1e3, replay_ms=r.ms,
                                      replay_sweep_rounds=rst["rounds"],
                                      replay_sweep_us_per_round=1e3 * (r.ms["chain"] + r.ms["deliver"]) /
                                      max(1, rst["rounds"]))), flush=True)


if __name__ == "__main__":
    main()
