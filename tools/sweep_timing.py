"""Where a delivery sweep's time goes: per-query phase timings from the profiling
build (libdagrider_gpu_timing.so, kernels.hpp DR_SWEEP_TIMING) of one C4 replay.

usage: DR_LIB_VARIANT=timing python tools/sweep_timing.py [config]
"""
import ctypes as C
import json
import os
import sys

os.environ["DR_LIB_VARIANT"] = "timing"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from dag_rider_amd import _lib as L  # noqa: E402
from dag_rider_amd.engine import Engine  # noqa: E402
from dag_rider_amd.gen import CONFIGS, generate  # noqa: E402

cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c4"]
d = generate(cfg, nthreads=16)
lib = L.lib()
lib.dr_debug_sweep_timing.restype = C.c_int
lib.dr_debug_sweep_timing.argtypes = [C.c_void_p, C.c_int]
with Engine(cfg.n, cfg.faulty, d.nrounds, 0) as e:
    e.append_packed(d)
    for _ in range(3):
        res = e.replay(cfg.nwaves)
    nq = int(res.sweep["count"])
    buf = np.zeros(16 * nq, np.uint64)
    assert lib.dr_debug_sweep_timing(L.ptr(buf), nq) == 0
t = buf.reshape(nq, 16).astype(np.float64)
t = t[t[:, 3] > 0]  # (a static-table query nobody popped records nothing)
tick_us = 0.01  # wall_clock64 runs at 100 MHz on gfx950
out = {}
for k, name in enumerate(["prologue", "phaseA", "expansion", "total"]):
    v = t[:, k] * tick_us
    out[name + "_us"] = dict(mean=float(v.mean()), p50=float(np.median(v)), max=float(v.max()))
for k, name in ((8, "exp_issue"), (9, "exp_rows"), (10, "exp_fold"), (11, "exp_weak"), (12, "results")):
    v = t[:, k] * tick_us
    out[name + "_us"] = dict(mean=float(v.mean()), p50=float(np.median(v)), max=float(v.max()))
v = t[:, 15] * tick_us
out["emit_us"] = dict(mean=float(v.mean()), p50=float(np.median(v)), max=float(v.max()))
st = (t[:, 13] - t[:, 13].min()) * tick_us  # workgroup start offsets within the launch
en = (t[:, 14] - t[:, 13].min()) * tick_us
out["start_offset_us"] = dict(p50=float(np.median(st)), p90=float(np.percentile(st, 90)), max=float(st.max()))
out["end_offset_us"] = dict(p50=float(np.median(en)), p90=float(np.percentile(en, 90)), max=float(en.max()))
out["summary_rounds"] = float(t[:, 4].mean())
out["partial_rounds"] = float(t[:, 5].mean())
out["queries"] = nq
out["swept"] = int(len(t))
print(json.dumps(out, indent=1))
