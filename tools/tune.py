"""Kernel tuning: times dr_profile_kernel variants on the C4 DAG (interleaved, one process)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dag_rider_amd.engine import Engine  # noqa: E402
from dag_rider_amd.gen import CONFIGS, generate  # noqa: E402

cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c4"]
d = generate(cfg, nthreads=16)
e = Engine(cfg.n, cfg.faulty, d.nrounds, 0)
e.append_packed(d)
rows_b = d.nrounds * cfg.n * ((cfg.n + 63) // 64) * 8
weak_b = int(d.weak_off[-1]) * 4
cases = [("summary_commit shipped", 0, 0, rows_b + weak_b), ("rows only", 0, 1, rows_b), ("weak only", 0, 2, weak_b),
         ("weak unroll 8", 0, 3, rows_b + weak_b), ("stream rows", 1, 0, rows_b), ("stream rows+weak", 1, 1, rows_b + weak_b),
         ("stream rows blocked", 1, 2, rows_b), ("summary_commit NT=512", 0, 4, rows_b + weak_b),
         ("summary_commit NT=256", 0, 5, rows_b + weak_b),
         ("split 2 streams", 0, 6, rows_b + weak_b), ("split 1 stream", 0, 7, rows_b + weak_b),
         ("weak_union alone", 0, 8, weak_b), ("rows only NT=256", 0, 9, rows_b), ("rows only NT=1024", 0, 10, rows_b),
         ("rows GRP16", 0, 13, rows_b), ("rows temporal loads", 0, 14, rows_b), ("rows GRP16 NT=1024", 0, 15, rows_b), ("summary phase (all)", 2, 0, rows_b + weak_b)]
res = {name: [] for name, *_ in cases}
for rep in range(5):
    for name, k, v, b in cases:
        res[name].append(e.profile_kernel(k, v, 10))
out = {}
for name, k, v, b in cases:
    ms = sorted(res[name])
    out[name] = dict(ms_med=ms[len(ms) // 2], ms_min=ms[0], GBps=b / (ms[len(ms) // 2] / 1e3) / 1e9, bytes=b)
    print(f"{name:24s} {ms[len(ms)//2]*1e3:8.1f} us  {out[name]['GBps']:8.1f} GB/s", flush=True)
print(json.dumps(out))
