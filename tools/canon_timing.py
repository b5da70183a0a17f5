"""Where k_canon's time goes (one workgroup walking the canonical cone): wall-clock
stamps from the profiling build (libdagrider_gpu_timing.so, kernels.hpp
g_canon_timing) of one replay per config.

usage: python tools/canon_timing.py [config ...]   (default: c4 c3)
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

lib = L.lib()
lib.dr_debug_canon_timing.restype = C.c_int
lib.dr_debug_canon_timing.argtypes = [C.c_void_p]
for name in sys.argv[1:] or ["c4", "c3"]:
    cfg = CONFIGS[name]
    d = generate(cfg, nthreads=16)
    with Engine(cfg.n, cfg.faulty, d.nrounds, 0) as e:
        e.append_packed(d)
        for _ in range(3):
            e.replay(cfg.nwaves)
        buf = np.zeros(8, np.uint64)
        assert lib.dr_debug_canon_timing(L.ptr(buf)) == 0
    t = buf.astype(np.float64)
    print(json.dumps({"config": name, "segments_us": (t[1] - t[0]) * 0.01, "positions_us": (t[2] - t[1]) * 0.01,
                      "segments": int(buf[3]), "rounds_walked": int(buf[4]),
                      "segment_init_us": float(t[5]) * 0.01}), flush=True)
