"""Time the column-sharded sweep on one GPU: the C4 DAG, reach sets (strong + weak,
rounds 0..leader) of the 64 newest wave leaders, local mode with G = 1, 2, 4, 8
column shards in one context (same kernels and column split as RCCL mode, the
exchange being the shared frontier buffer), checked against the unsharded engine.
Prints one JSON line per G."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
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
    for G in [int(x) for x in (sys.argv[1:] or ["1", "2", "4", "8"])]:
        with ShardEngine(cfg.n, cfg.faulty, d.nrounds, 0, nshards=G) as se:
            se.append_packed(d)
            got = se.reach_sets(froms, bottoms, False)
            runs = []
            for _ in range(3):
                se.reach_sets(froms, bottoms, False)
                runs.append(se.stats())
            st = min(runs, key=lambda x: x["ms"])
            ok = all((a == b).all() for a, b in zip(got, ref))
            print(json.dumps(dict(G=G, ok=bool(ok), us_per_round=1e3 * st["ms"] / st["rounds"], **st)), flush=True)


if __name__ == "__main__":
    main()
