"""Where the fused C5 replay's time goes: per-DAG phase timings of k_replay_small
(batch.hpp) from the profiling build (libdagrider_gpu_timing.so, DR_SWEEP_TIMING).

usage: python tools/batch_timing.py [dags ...]   (default: 512 1024 2048 4096); both kernel forms
One JSON line per batch size: the kernel's HIP-event time and, per phase, the mean /
p50 / max duration over the DAGs (wall_clock64 ticks, 100 MHz on gfx950).
"""
import ctypes as C
import json
import os
import sys
import time

os.environ["DR_LIB_VARIANT"] = "timing"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from dag_rider_amd import _lib as L  # noqa: E402
from dag_rider_amd.engine import Engine, ReplayBatch  # noqa: E402
from dag_rider_amd.gen import c5_config, generate  # noqa: E402

sizes = [int(x) for x in sys.argv[1:]] or [512, 1024, 2048, 4096]
lib = L.lib()
lib.dr_debug_sweep_timing.restype = C.c_int
lib.dr_debug_sweep_timing.argtypes = [C.c_void_p, C.c_int]
t0 = time.perf_counter()
engines = []
for i in range(max(sizes)):
    cfg = c5_config(i)
    d = generate(cfg)
    e = Engine(cfg.n, cfg.faulty, d.nrounds, 0)
    e.append_packed(d)
    engines.append(e)
print(f"loaded {len(engines)} DAGs in {time.perf_counter() - t0:.1f} s", file=sys.stderr)
nw = c5_config(0).nwaves
names = ["pass_F", "pass_G_tail", "chains", "emission", "outputs"]
names_w = ["leaders", "cone_pass", "chains", "emission", "outputs"]  # the wave form's phases
for nd, form in [(nd, f) for nd in sizes for f in (L.DR_BATCH_WORKGROUP, L.DR_BATCH_WAVE)]:
    engines[0].set_batch_form(form)
    b = ReplayBatch(engines[:nd], nw, L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF)
    for _ in range(3):
        b.run()
    res = b.results()
    wave = form == L.DR_BATCH_WAVE
    buf = np.zeros(16 * nd, np.uint64)
    assert lib.dr_debug_sweep_timing(L.ptr(buf), nd) == 0
    t = buf.reshape(nd, 16)[:, :6].astype(np.float64) * 0.01  # us
    out = {"dags": nd, "form": "wave" if wave else "workgroup", "kernel_ms": max(r.ms["deliver"] for r in res)}
    for k, name in enumerate(names_w if wave else names):
        v = t[:, k + 1] - t[:, k]
        out[name + "_us"] = dict(mean=round(float(v.mean()), 2), p50=round(float(np.median(v)), 2),
                                 max=round(float(v.max()), 2))
    cyc = buf.reshape(nd, 16)[:, 8:14].astype(np.float64)  # cone-pass cycle counters (s_memtime)
    parts = (["loop_and_loads", "commit_rule", "ring_seed_stores_ballots", "weak_columns", "expand_K", "expand_solo"]
             if wave else ["wait_loop", "ring_seed_ballots", "weak_columns", "K_weak_spread", "expand_K", "expand_solo"])
    out["cone_pass_cycles_mean"] = {k: round(float(cyc[:, i].mean())) for i, k in enumerate(parts)}
    tot = t[:, 5] - t[:, 0]
    out["dag_total_us"] = dict(mean=round(float(tot.mean()), 2), max=round(float(tot.max()), 2))
    st = t[:, 0] - t[:, 0].min()
    out["start_offset_us"] = dict(p50=round(float(np.median(st)), 2), max=round(float(st.max()), 2))
    print(json.dumps(out), flush=True)
for e in engines:
    e.close()
