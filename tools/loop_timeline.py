"""One wave of the per-call loop (bench.py --config c4-loop under rocprofv3 --kernel-trace
--hip-trace): host API calls (indented, launch-sized ones and waits) and kernels in time
order, from the append of wave k of the measured pass to the next append.

usage: python tools/loop_timeline.py <rocprofv3 output dir> [k]
"""
import csv
import glob
import os
import sys

d = sys.argv[1]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 40
K, A = [], []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    K += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + r["Kernel_Name"][:64]) for r in csv.DictReader(open(f))]
for f in glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True):
    A += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "A " + r["Function"]) for r in csv.DictReader(open(f))]
K.sort()
A.sort()
rs = [x for x in K if "k_round_summary" in x[2]]
half = len(rs) // 2  # the warm-up pass, then the measured pass
t0, t1 = rs[half + k][0], rs[half + k + 1][0]
skip = {"hipGetLastError", "__hipPushCallConfiguration", "__hipPopCallConfiguration", "hipEventQuery", "hipSetDevice"}
ev = sorted(e for e in K + A if t0 - 40000 <= e[0] < t1 - 40000 and not (e[2][0] == "A" and e[2][2:] in skip))
base = ev[0][0]
busy = sum(e - s for s, e, n in ev if n[0] == "K")
for s, e, n in ev:
    print(f"{(s - base) / 1e3:8.1f} us {(e - s) / 1e3:6.1f}  {'      ' if n[0] == 'A' else ''}{n}")
print(f"wave span {(t1 - t0) / 1e3:.1f} us (traced), kernels busy {busy / 1e3:.1f} us")
