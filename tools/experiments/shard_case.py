"""Replay one random-DAG case of tests/test_gpu_shard.py::test_shard_replay_random_dags on
every (G, memo, persistent, stepped, chain, deliver) combination and report which differ."""
import os
import sys
import traceback

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from dag_rider_amd import _lib as L  # noqa: E402
from dag_rider_amd.shard import ShardEngine  # noqa: E402
from dagutil import random_dag  # noqa: E402
import oracle  # noqa: E402

seed = int(sys.argv[1]) if len(sys.argv) > 1 else 0
rng = np.random.default_rng(3000 + seed)
n = int(rng.choice([1, 4, 7, 64, 65, 130, 200, 300]))
R = int(rng.integers(8, 41))
d = random_dag(rng, n, R, p_present=rng.uniform(0.5, 1), p_s=rng.uniform(0.05, 0.9), p_w=rng.uniform(0, 1),
               max_depth=int(rng.integers(2, 20)))
f = int(rng.integers(0, (n - 1) // 3 + 2))
nw = R // 4
print("n", n, "R", R, "f", f, "nw", nw)
bs = oracle.PDag(d)
MODES = [(L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_REF), (L.DR_CHAIN_PERSISTENT, L.DR_DELIVER_PAPER),
         (L.DR_CHAIN_LITERAL, L.DR_DELIVER_REF), (L.DR_CHAIN_LITERAL, L.DR_DELIVER_PAPER)]
for G in (1, 2, 3, 8):
    with ShardEngine(n, f, R + 1, 0, nshards=G) as se:
        se.append_packed(d)
        for memo, persistent, stepped in ((True, True, False), (True, True, True)):
            se.set_memo(memo)
            se.set_persistent(persistent)
            se.set_stepped(stepped)
            for cm, dm in MODES:
                want = bs.replay(f, nw, cm, dm)
                tag = f"G={G} memo={memo} pers={persistent} stepped={stepped} cm={cm} dm={dm}"
                try:
                    got = se.replay(nw, cm, dm)
                except Exception as e:  # noqa: BLE001
                    print(tag, "ERROR", e, "want push_wave", list(want.push_wave), "commit", list(want.commit))
                    continue
                bad = [k for k in ("commit", "vcount", "push_off", "push_wave", "pop_count", "pop_digest", "pop_edges")
                       if not np.array_equal(getattr(got, k), getattr(want, k))]
                for k in ("commit_edges", "chain_edges", "deliver_edges"):
                    if getattr(got, k) != getattr(want, k):
                        bad.append(k)
                print(tag, "OK" if not bad else "DIFF " + ",".join(bad))
                if bad:
                    print("  got push", list(got.push_wave), "want", list(want.push_wave),
                          "chain_edges", got.chain_edges, want.chain_edges)

if os.environ.get("DR_DBG"):
    import ctypes as C
    lib = L.lib()
    with ShardEngine(n, f, R + 1, 0, nshards=1) as se:
        se.append_packed(d)
        buf = np.zeros(64 * 64 * 4, np.int32)
        lib.dr_debug_dbg(buf.ctypes.data_as(C.c_void_p))
        buf[:] = -7
        # upload sentinel not possible: read after one failing replay
        se.set_persistent(True)
        try:
            se.replay(nw, L.DR_CHAIN_LITERAL, L.DR_DELIVER_REF)
        except Exception as e:  # noqa: BLE001
            print("err", e)
        lib.dr_debug_dbg(buf.ctypes.data_as(C.c_void_p))
        b = buf.reshape(64, 64, 4)
        for q in range(64):
            rows = [tuple(b[q, k]) for k in range(64) if b[q, k, 0] != 0 or b[q, k, 1] != 0]
            if rows:
                print("q", q, rows[:12])
