"""Per-kernel medians from a rocprofv3 kernel-trace database (run_results.db), split
into segments at each occurrence of a marker kernel (e.g. one segment per shard count)."""
import collections
import sqlite3
import sys


def main():
    db = sys.argv[1]
    markers = [m for m in sys.argv[2].split(",") if m] if len(sys.argv) > 2 else []
    c = sqlite3.connect(db)
    seg, acc = "all", collections.defaultdict(lambda: collections.defaultdict(list))
    for name, s, e in c.execute("select name,start,end from kernels order by start"):
        for m in markers:
            if m in name:
                seg = m
        acc[seg][name.split("(")[0].replace("void ", "")].append((e - s) / 1000)
    for g, d in acc.items():
        tot = 0.0
        print(g)
        for k, v in sorted(d.items(), key=lambda x: -sum(x[1])):
            v2 = sorted(v)
            med = v2[len(v2) // 2]
            print("  %-50s n=%-4d med_us=%.2f" % (k[:50], len(v), med))


if __name__ == "__main__":
    main()
