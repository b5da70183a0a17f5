"""Kernel tuning: times dr_profile_kernel variants on the C4 DAG (interleaved, one process).

k_summary_commit geometries (engine.hip launch_sv_t, WS = 16): block size, 16-B
chunks in flight per thread, and software pipelining across the round barriers;
beside them the bare streaming reads of the same rows (the practical ceiling)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("DR_LIB_VARIANT", "timing")  # dr_profile_kernel lives in the profiling build only
from dag_rider_amd.engine import Engine  # noqa: E402
from dag_rider_amd.gen import CONFIGS, generate  # noqa: E402

cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c4"]
d = generate(cfg, nthreads=16)
e = Engine(cfg.n, cfg.faulty, d.nrounds, 0)
e.append_packed(d)
W = (cfg.n + 63) // 64
T = d.nrounds - 1
rows_b = T * cfg.n * W * 8 + T * W * 8 + T * 8  # rows read + U + SD written (bench.py kernel_bytes)
cases = [("shipped", 0, 0), ("NT512 GRP8", 0, 1), ("NT512 GRP8 pipe", 0, 2), ("NT512 GRP4 pipe", 0, 3),
         ("NT1024 GRP4 pipe", 0, 4), ("NT1024 GRP8", 0, 5), ("NT256 GRP8 pipe", 0, 6), ("NT1024 GRP2 pipe", 0, 7),
         ("NT512 GRP16", 0, 8), ("NT256 GRP16", 0, 9), ("NT512 GRP2 pipe", 0, 10), ("NT1024 GRP1 pipe", 0, 11),
         ("NT256 GRP4 pipe", 0, 12), ("NT1024 GRP4", 0, 13), ("NT1024 GRP2", 0, 14), ("NT1024 GRP1", 0, 15),
         ("NT512 GRP2", 0, 16), ("NT512 GRP4", 0, 17), ("NT256 GRP2", 0, 18), ("NT256 GRP4", 0, 19),
         ("stream rows", 1, 0), ("stream rows blocked", 1, 2)]
res = {name: [] for name, *_ in cases}
for rep in range(5):
    for name, k, v in cases:
        res[name].append(e.profile_kernel(k, v, 10))
out = {}
for name, k, v in cases:
    ms = sorted(res[name])
    out[name] = dict(ms_med=ms[len(ms) // 2], ms_min=ms[0], GBps=rows_b / (ms[len(ms) // 2] / 1e3) / 1e9)
    print(f"{name:24s} {ms[len(ms)//2]*1e3:8.1f} us  {out[name]['GBps']:8.1f} GB/s", flush=True)
print(json.dumps(out))
