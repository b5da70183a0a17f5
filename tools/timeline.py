"""Print the last replay step's kernel/copy timeline (with gaps) from rocprofv3 CSVs.

usage: python tools/timeline.py <dir containing *_kernel_trace.csv [*_memory_copy_trace.csv]>
       [--last] [--start KERNEL_SUBSTRING]   (default start marker: k_summary_commit)
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
# bench.py's last replay is a profiling one (every phase bracketed by HIP events);
# the last TIMED step starts at the second-to-last k_summary_commit (--last: the last)
mark = sys.argv[sys.argv.index("--start") + 1] if "--start" in sys.argv else "k_summary_commit"
starts = [i for i, e in enumerate(ev) if mark in e[2]]
pick = -1 if "--last" in sys.argv or len(starts) < 2 else -2
i0 = starts[pick] if starts else max(0, len(ev) - 60)
i1 = starts[pick + 1] if pick == -2 else len(ev)
prev = None
t0 = ev[i0][0]
busy = 0
for s, e, name in ev[i0:i1]:
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    busy += e - s
    print(f"{(s - t0) / 1e3:9.1f} us  gap {gap:7.1f}  dur {(e - s) / 1e3:7.1f}  {name}")
    prev = e
print(f"span {(ev[i1 - 1][1] - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us")
