"""Column-sharded reachability across RCCL ranks (one process per rank): every rank
builds its shard of a seeded n=1024 DAG, runs the same reach-set batch, and rank 0
checks the gathered result against the unsharded engine.

    python tools/shard_rccl_check.py --ranks 2 [--same-gpu]

--same-gpu puts every rank on device 0 (a 1-GPU box); otherwise rank i uses device i.
Prints one JSON line per rank 0 run.
"""
import argparse
import json
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def worker(rank, world, port, same_gpu, rounds, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import numpy as np
    import torch.distributed as dist

    from dag_rider_amd.engine import Engine
    from dag_rider_amd.gen import generate, small_config
    from dag_rider_amd.shard import ShardEngine

    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = 0 if same_gpu else rank
    cfg = small_config(1024, rounds, 4, p_present=1.0, p_late=0.02, p_w=0.5, weak_depth=4)
    d = generate(cfg)
    froms = [(rounds - (i % 8), 1 + 97 * i % 1024) for i in range(64)]
    bottoms = [0] * 64
    se = ShardEngine.from_process_group(dist, 1024, 341, rounds + 1, dev)
    se.append_packed(d)
    for strong in (True, False):
        got = se.reach_sets(froms, bottoms, strong)
        st = se.stats()
        if rank == 0:
            with Engine(1024, 341, rounds + 1, dev) as e:
                e.append_packed(d)
                ref = e.reach_sets(froms, bottoms, strong)
            ok = all((a == b).all() for a, b in zip(got, ref))
            out.append(dict(strong=strong, ok=bool(ok), ranks=world, **se.info(), **st))
    se.close()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=200)
    ap.add_argument("--same-gpu", action="store_true")
    a = ap.parse_args()
    import torch.multiprocessing as mp

    mgr = mp.Manager()
    out = mgr.list()
    mp.spawn(worker, args=(a.ranks, _port(), a.same_gpu, a.rounds, out), nprocs=a.ranks, join=True)
    for r in out:
        print(json.dumps(r), flush=True)
    sys.exit(0 if out and all(r["ok"] for r in out) else 1)


if __name__ == "__main__":
    main()
