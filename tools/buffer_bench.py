"""Time dr_buffer_admit (the buffer pass, process.go:200-234) on a generated DAG.

The buffer holds one full next round: n vertices of round R+1, each with the 2f+1
strong edges of round R the generator would give it plus a few weak edges, and a
second copy of the round one round further ahead that depends on the first (so the
pass needs a second sweep).  Reports the wall time of one call (H2D of the buffer
included) and the present() comparisons the reference's linear scan
(process.go:374-384) would make for the same pass.

    python tools/buffer_bench.py [--n 1024] [--rounds 400] [--iters 20]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dag_rider_amd import _lib as L  # noqa: E402
from dag_rider_amd.engine import Engine  # noqa: E402
from dag_rider_amd.gen import generate, small_config  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=400)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    n, R = a.n, a.rounds
    f = (n - 1) // 3
    d = generate(small_config(n, R, 11))
    rng = np.random.default_rng(5)
    buf = []
    def srcs(r):  # sources present in round r (the buffer's own round R+1 is complete)
        if r > R:
            return np.arange(1, n + 1)
        a = d.slot_src[d.slot_off[r]:d.slot_off[r + 1]].astype(np.int64)
        return a[a > 0]

    for r in (R + 1, R + 2):
        for s in range(1, n + 1):
            strong = [(r - 1, int(t)) for t in np.sort(rng.choice(srcs(r - 1), 2 * f + 1, replace=False))]
            weak = []
            for _ in range(3):
                wr = int(rng.integers(max(r - 6, 0), r - 1))
                weak.append((wr, int(rng.choice(srcs(wr)))))
            buf.append(((r, s), strong + weak))
    npred = sum(len(p) for _, p in buf)
    ids = np.asarray([v for v, _ in buf], np.int32).reshape(-1)
    off = np.zeros(len(buf) + 1, np.uint32)
    off[1:] = np.cumsum([len(p) for _, p in buf])
    preds = np.asarray([x for _, p in buf for x in p], np.int32).reshape(-1)
    adm = np.zeros(len(buf), np.uint8)
    with Engine(n, f, R + 4, 0) as e:
        e.append_packed(d)
        ref = e.buffer_admit(R + 2, buf)  # warm-up through the Python veneer

        def call():
            e._check(e._L.dr_buffer_admit(e._h, R + 2, len(buf), L.ptr(ids), L.ptr(off), L.ptr(preds), L.ptr(adm)))

        call()
        assert np.array_equal(adm, ref)
        t0 = time.perf_counter()
        for _ in range(a.iters):
            call()
        dt = (time.perf_counter() - t0) / a.iters
    slots = int(d.slot_off[-1])
    print(json.dumps({"what": "dr_buffer_admit one pass", "n": n, "dag_rounds": R + 1, "buffered": len(buf),
                      "predecessors": npred, "admitted": int(adm.sum()), "ms_per_pass": dt * 1e3,
                      "preds_per_s": npred / dt,
                      "reference_scan_comparisons_upper": npred * slots}))


if __name__ == "__main__":
    main()
