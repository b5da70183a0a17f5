"""The general sweep (k_gsweep, general.hpp) at C4 scale: the c4-up DAG (C4 + one weak
edge to its own round, App. A Q8) takes it for every query.  Times path() batches and
one wave's waveReady vote (one general sweep per present voter of round 4w), the units a
whole c4-up replay is made of (1000 waves x 1024 voters + 977 pops: minutes).

usage: python tools/gsweep_bench.py [queries]     -> one JSON line per measurement
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dag_rider_amd.engine import Engine  # noqa: E402
from dag_rider_amd.gen import CONFIGS, generate  # noqa: E402


def main():
    nq = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    cfg = CONFIGS["c4-up"]
    d = generate(cfg, nthreads=16)
    rng = np.random.default_rng(1)
    with Engine(cfg.n, cfg.faulty, d.nrounds, 0) as e:
        e.append_packed(d)
        print(json.dumps({"config": "c4-up", "exceptions": e.exception_stats()}), flush=True)
        for strong in (True, False):
            pairs = []
            for _ in range(nq):
                fr = int(rng.integers(2, d.nrounds))
                pairs.append(((fr, int(rng.integers(1, cfg.n + 1))), (int(rng.integers(0, fr)), int(rng.integers(1, cfg.n + 1)))))
            e.path_batch(pairs[:8], strong)  # first-call costs
            t0 = time.perf_counter()
            e.path_batch(pairs, strong)
            dt = time.perf_counter() - t0
            print(json.dumps({"what": "path_batch", "strong": strong, "queries": nq, "ms": dt * 1e3,
                              "us_per_query": dt * 1e6 / nq}), flush=True)
        for w in (10, 500):
            t0 = time.perf_counter()
            cm, vc = e.wave_commit(w, w)
            dt = time.perf_counter() - t0
            print(json.dumps({"what": "wave_commit (one general sweep per voter)", "wave": w, "ms": dt * 1e3,
                              "commit": int(cm[0]), "vcount": int(vc[0])}), flush=True)


if __name__ == "__main__":
    main()
