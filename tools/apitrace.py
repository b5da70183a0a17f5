"""Interleave HIP API calls and kernels of the last replay step (rocprofv3 --hip-trace --kernel-trace CSVs).

usage: python tools/apitrace.py DIR [ANCHOR_KERNEL [NTH_FROM_END [SPAN_US]]]
(default: from the last k_summary_commit to the end of the trace)"""
import csv
import glob
import os
import sys

d = sys.argv[1]
ev = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + r["Kernel_Name"][:60]))
for f in glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "A " + r["Function"]))
ev.sort()
starts = [i for i, e in enumerate(ev) if e[2].startswith("A") and "hipLaunchKernel" in e[2]]
anchor = sys.argv[2] if len(sys.argv) > 2 else "k_summary_commit"
nth = int(sys.argv[3]) if len(sys.argv) > 3 else 1
span = float(sys.argv[4]) if len(sys.argv) > 4 else float("inf")
ks = [i for i, e in enumerate(ev) if e[2].startswith("K") and anchor in e[2]]
i0 = ks[-nth]
# back up to the API launch of that kernel
while i0 > 0 and not (ev[i0][2].startswith("A") and "Launch" in ev[i0][2]):
    i0 -= 1
t0 = ev[i0][0]
prev_api_end = None
for s, e, name in ev[i0:]:
    if (s - t0) / 1e3 > span:
        break
    gap = ""
    if name.startswith("A"):
        if prev_api_end is not None:
            gap = f"host {(s - prev_api_end) / 1e3:6.1f}"
        prev_api_end = e
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f}  {gap:12s} {name}")
