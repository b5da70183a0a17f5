"""Fill BASELINE.md's round-3 results table from the final bench lines.

usage: python tools/fill_baseline.py <dir with bench.json bench_c1.json bench_c2.json
       bench_c3.json bench_c5.json bench_c5_512.json>
Each file's last line is one bench.py JSON line; placeholders (C4_MS, ...) are replaced.
"""
import json
import os
import sys

d = sys.argv[1]


def line(name):
    p = os.path.join(d, name)
    if not os.path.exists(p):
        return None
    txt = open(p).read().strip().splitlines()
    return json.loads(txt[-1]) if txt else None


def e(x):
    if x is None:
        return "—"
    m, ex = f"{x:.2e}".split("e")
    return f"{m}·10^{int(ex)}"


rep = {}
for key, f in (("C1", "bench_c1.json"), ("C2", "bench_c2.json"), ("C3", "bench_c3.json"), ("C4", "bench.json"),
               ("C5", "bench_c5.json"), ("C5S", "bench_c5_512.json")):
    b = line(f)
    if b is None:
        continue
    rep[key + "_MS"] = f"{b['ms_per_step']:.3f}"
    rep[key + "_EPS"] = e(b["value"])
    rf = b.get("roofline") or {}
    rep[key + "_FRAC"] = f"{rf.get('frac', 0):.2f} ({rf.get('kernel', '')})" if rf else "—"
    cb = b.get("cpu_baseline") or {}
    if key == "C5":
        lit = cb.get("literal") or {}
        bit = cb.get("bitset_all_dags") or {}
        rep[key + "_LIT"] = f"— / {e(lit.get('value'))} (waves 1-4 of 16 DAGs)"
        rep[key + "_BIT"] = e(bit.get("value"))
    elif cb:
        ac = cb.get("all_cores") or {}
        rep[key + "_LIT"] = f"{e(cb.get('value'))} / {e(ac.get('value'))}"
        rep[key + "_BIT"] = e((b.get("cpu_bitset") or {}).get("value"))
p = "BASELINE.md"
s = open(p).read()
for k in sorted(rep, key=len, reverse=True):
    s = s.replace(k, rep[k])
open(p, "w").write(s)
print(json.dumps(rep, indent=1))
