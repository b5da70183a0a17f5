"""Timeline of one sharded replay from a rocprofv3 kernel (+ memory copy) trace: the
replay that starts at the k-th k_ms_wu launch (default: the third, a timed replay of the
first configuration), with gaps and durations.

usage: python tools/shard_timeline.py <rocprof dir> [k]   (k may be negative: from the end)
"""
import csv
import glob
import os
import sys

d = sys.argv[1]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
ev = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:72]))
for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY " + r.get("Direction", "")))
ev.sort()
starts = [i for i, e in enumerate(ev) if "k_ms_wu" in e[2]]
i0 = starts[k]
i1 = starts[k + 1] if k + 1 < len(starts) and k != -1 else len(ev)
t0, prev, busy = ev[i0][0], None, 0
for s, e, n in ev[i0:i1]:
    busy += e - s
    print(f"{(s - t0) / 1e3:8.1f} us  gap {((s - prev) / 1e3 if prev else 0):6.1f}  dur {(e - s) / 1e3:6.1f}  {n}")
    prev = e
print(f"span {(ev[i1 - 1][1] - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us")
