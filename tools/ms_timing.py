"""Where the fused sharded replay's sweep time goes: per-query ticks of
k_ms_sweep_full from the profiling build (libdagrider_gpu_timing.so,
shard_fused.hpp DR_SWEEP_TIMING) on C4 at the given shard counts.

usage: python tools/ms_timing.py [config] [G,...]
"""
import ctypes as C
import json
import os
import sys

os.environ["DR_LIB_VARIANT"] = "timing"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from dag_rider_amd import _lib as L  # noqa: E402
from dag_rider_amd.gen import CONFIGS, generate  # noqa: E402
from dag_rider_amd.shard import ShardEngine  # noqa: E402

cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c4"]
shards = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,8").split(",")]
d = generate(cfg, nthreads=16)
lib = L.lib()
lib.dr_debug_ms_timing.restype = C.c_int
lib.dr_debug_ms_timing.argtypes = [C.c_void_p, C.c_int]
tick_us = 0.01  # wall_clock64 runs at 100 MHz on gfx950
for G in shards:
    with ShardEngine(cfg.n, cfg.faulty, d.nrounds, 0, nshards=G) as se:
        se.append_packed(d)
        for _ in range(3):
            r = se.replay(cfg.nwaves)
        nq = int(r.sweep["count"]) + cfg.nwaves
        buf = np.zeros(8 * nq, np.uint64)
        assert lib.dr_debug_ms_timing(L.ptr(buf), nq) == 0
    t = buf.reshape(nq, 8)
    live = t[:, 1] > 0
    t = t[live].astype(np.int64)
    t0 = t[:, 0].min()
    start = (t[:, 0] - t0) * tick_us
    end = (t[:, 1] - t0) * tick_us
    dur = end - start
    out = dict(G=G, queries=int(live.sum()), span_us=float(end.max()),
               start_p50=float(np.median(start)), start_max=float(start.max()))
    for typ, name in ((0, "pop"), (1, "chain")):
        m = t[:, 5] == typ
        if not m.any():
            continue
        out[name] = dict(n=int(m.sum()), dur_p50=float(np.median(dur[m])), dur_max=float(dur[m].max()),
                         end_max=float(end[m].max()),
                         w0_rounds_mean=float(t[m, 2].mean()), wg_rounds_mean=float(t[m, 3].mean()),
                         wg_rounds_max=int(t[m, 3].max()), wg_us_mean=float((t[m, 4] * tick_us).mean()),
                         walk_mean=float((t[m, 6] - t[m, 7]).mean()), walk_max=int((t[m, 6] - t[m, 7]).max()))
    slow = np.argsort(-dur)[:5]
    out["slowest"] = [dict(type=int(t[i, 5]), top=int(t[i, 6]), stop=int(t[i, 7]), start=float(start[i]),
                           dur=float(dur[i]), w0=int(t[i, 2]), wg=int(t[i, 3]), wg_us=float(t[i, 4] * tick_us))
                      for i in slow]
    print(json.dumps(out), flush=True)
