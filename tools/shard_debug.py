"""Debug helper: one random-DAG sharded replay vs the oracle, per-pop detail."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle  # noqa: E402
from dag_rider_amd import _lib as L  # noqa: E402
from dag_rider_amd.shard import ShardEngine  # noqa: E402
from dagutil import random_dag  # noqa: E402

seed = int(sys.argv[1]) if len(sys.argv) > 1 else 0
rng = np.random.default_rng(3000 + seed)
n = int(rng.choice([1, 4, 7, 64, 65, 130, 200, 300]))
R = int(rng.integers(8, 41))
d = random_dag(rng, n, R, p_present=rng.uniform(0.5, 1), p_s=rng.uniform(0.05, 0.9), p_w=rng.uniform(0, 1),
               max_depth=int(rng.integers(2, 20)))
f = int(rng.integers(0, (n - 1) // 3 + 2))
nw = R // 4
bs = oracle.PDag(d)
print("n", n, "R", R, "f", f)
for G in (1, 2, 3, 8):
    with ShardEngine(n, f, R + 1, 0, nshards=G) as se:
        se.append_packed(d)
        for persistent in (True, False):
            se.set_persistent(persistent)
            for cm in (0, 1):
                for dm in (0, 1):
                    want = bs.replay(f, nw, cm, dm)
                    got = se.replay(nw, cm, dm)
                    bad = np.nonzero(got.pop_count != want.pop_count)[0]
                    print(f"G={G} pers={persistent} cm={cm} dm={dm}: pops {len(want.pop_count)} bad {bad.tolist()[:8]}",
                          "edges", got.deliver_edges == want.deliver_edges)
                    if len(bad):
                        # pop leader rounds: reconstruct from push lists
                        pops = []
                        for w in range(1, nw + 1):
                            pw = got.push_wave[got.push_off[w - 1]:got.push_off[w]].tolist()
                            pops += [(x, 4 * w) for x in reversed(pw)]
                        for i in bad[:4]:
                            lw, cur = pops[i]
                            top = 4 * lw - 3
                            (cone,) = se.reach_sets([(top, 1)], [1], False)
                            wc, _ = bs.cone((top, 1), 1, False)
                            print("  pop", i, "leader wave", lw, "cur", cur, "got", got.pop_count[i], "want",
                                  want.pop_count[i], "reach ok", bool((cone == wc).all()))
                            cnt, pc, pd = se.order_vertices([(top, 1)], cur, dm)
                            print("   order_vertices alone:", pc.tolist())
