#!/usr/bin/env python3
"""Print a rocprofv3 --stats kernel table (a run directory or its *kernel_stats.csv):
calls, average and total time per kernel, short names.  usage: kstats.py DIR|CSV [N]"""
import csv
import glob
import os
import sys


def short(name: str) -> str:
    name = name.split("(")[0]
    return name.replace("void ", "").replace("ptype::", "")[:90]


def main():
    p = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    if os.path.isdir(p):
        hits = glob.glob(os.path.join(p, "**", "*kernel_stats.csv"), recursive=True)
        if not hits:
            sys.exit(f"no kernel_stats.csv under {p}")
        p = hits[0]
    rows = list(csv.DictReader(open(p)))
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"{'kernel':90s} {'calls':>6s} {'avg_us':>9s} {'total_ms':>9s} {'pct':>6s}")
    for r in rows[:n]:
        print(f"{short(r['Name']):90s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.2f} "
              f"{float(r['TotalDurationNs']) / 1e6:9.3f} {float(r['Percentage']):6.2f}")
    print(f"total kernel time {total / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
