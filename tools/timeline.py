"""Print the last replay step's kernel/copy timeline (with gaps) from rocprofv3 CSVs.

usage: python tools/timeline.py <dir containing *_kernel_trace.csv [*_memory_copy_trace.csv]>
"""
import csv
import glob
import os
import sys

d = sys.argv[1]
ev = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + r["Kernel_Name"][:70]))
for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C " + r.get("Direction", "") + " " + r.get("Size", r.get("Bytes", ""))))
ev.sort()
# the last step starts at the last k_summary_commit launch
starts = [i for i, e in enumerate(ev) if "k_summary_commit" in e[2]]
i0 = starts[-1] if starts else max(0, len(ev) - 60)
prev = None
t0 = ev[i0][0]
busy = 0
for s, e, name in ev[i0:]:
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    busy += e - s
    print(f"{(s - t0) / 1e3:9.1f} us  gap {gap:7.1f}  dur {(e - s) / 1e3:7.1f}  {name}")
    prev = e
print(f"span {(ev[-1][1] - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us")
