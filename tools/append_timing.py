"""Per-wave append latency on C4 (the c4-loop's append step alone): the ctypes call to
dr_append_rounds_packed with its arguments prepared beforehand, and the Engine method
around it.  usage: python tools/append_timing.py [waves] [--torch]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if "--torch" in sys.argv:
    import torch  # noqa: F401  (the bench process has torch and its OpenMP runtime loaded)

from dag_rider_amd import _lib as L  # noqa: E402
from dag_rider_amd.engine import Engine  # noqa: E402
from dag_rider_amd.gen import CONFIGS, generate  # noqa: E402


def main():
    nw = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 300
    cfg = CONFIGS["c4"]
    d = generate(cfg)
    n, W = d.n, d.W
    res = {}
    modes = ("loop",) if "--loop" in sys.argv else ("call", "method")
    for mode in modes:
        with Engine(cfg.n, cfg.faulty, 4 * nw + 1, 0) as e:
            e.append_packed(d, 0, 1)
            args = []
            for w in range(1, nw + 1):
                r0, r1 = 4 * w - 3, 4 * w + 1
                so = np.ascontiguousarray(d.slot_off[r0:r1 + 1])
                st = d.strong[r0 * n * W:r1 * n * W]
                wo = np.ascontiguousarray(d.weak_off[r0 * n:r1 * n + 1])
                args.append((r0, r1 - r0, L.ptr(so), L.ptr(d.slot_src), L.ptr(st), L.ptr(wo), L.ptr(d.weak_tgt), so,
                             st, wo))
            ts = []
            decided = 0
            for w in range(1, nw + 1):
                t0 = time.perf_counter()
                if mode == "loop":
                    e.append_packed(d, 4 * w - 3, 4 * w + 1)
                    ts.append(time.perf_counter() - t0)
                    cm, vc, pushed = e.wave_ready(w, decided)
                    if cm:
                        e.order_vertices([(4 * (x - 1) + 1, 1) for x in pushed], 4 * w, L.DR_DELIVER_REF, cap=0)
                        decided = w
                    continue
                if mode == "call":
                    a = args[w - 1]
                    rc = e._L.dr_append_rounds_packed(e._h, *a[:7])
                    assert rc == 0, e._L.dr_last_error(e._h)
                else:
                    e.append_packed(d, 4 * w - 3, 4 * w + 1)
                ts.append(time.perf_counter() - t0)
        a = np.asarray(ts[10:]) * 1e6
        dec = np.array_split(np.asarray(ts) * 1e6, 10)
        res[mode + "_by_decile_mean"] = [float(x.mean()) for x in dec]
        res[mode] = dict(p50=float(np.percentile(a, 50)), p90=float(np.percentile(a, 90)), mean=float(a.mean()))
    print(json.dumps(dict(waves=nw, torch="--torch" in sys.argv, omp=os.environ.get("OMP_NUM_THREADS"),
                          us=res)), flush=True)


if __name__ == "__main__":
    main()
