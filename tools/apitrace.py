"""Interleave HIP API calls and kernels of the last replay step (rocprofv3 --hip-trace --kernel-trace CSVs)."""
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
ks = [i for i, e in enumerate(ev) if "k_summary_commit" in e[2]]
i0 = ks[-1]
# back up to the API launch of that kernel
while i0 > 0 and not (ev[i0][2].startswith("A") and "Launch" in ev[i0][2]):
    i0 -= 1
t0 = ev[i0][0]
prev_api_end = None
for s, e, name in ev[i0:]:
    gap = ""
    if name.startswith("A"):
        if prev_api_end is not None:
            gap = f"host {(s - prev_api_end) / 1e3:6.1f}"
        prev_api_end = e
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f}  {gap:12s} {name}")
