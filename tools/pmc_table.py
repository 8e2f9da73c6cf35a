#!/usr/bin/env python3
"""Per-kernel PMC table from rocprofv3 --pmc runs (csv output): every counter of
every run directory averaged per call, joined with kernel durations; FETCH_SIZE
and WRITE_SIZE (KB) also give the achieved HBM bandwidth.

usage: python tools/pmc_table.py [--filter ptype] <run_dir> [<run_dir> ...]
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--filter", default="ptype")
    args = ap.parse_args()
    vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [per dispatch]
    durs = defaultdict(list)
    for d in args.dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                name = r.get("Kernel_Name", "")
                if args.filter not in name:
                    continue
                vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
                if r.get("End_Timestamp") and r.get("Start_Timestamp"):
                    durs[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    counters = sorted({c for k in vals.values() for c in k})
    short = [c.replace("SQ_", "").replace("_SIZE", "")[:12] for c in counters]
    print(f"{'kernel':52s} {'us':>8s} " + " ".join(f"{s:>12s}" for s in short) + f" {'TB/s':>6s}")
    for name in sorted(vals, key=lambda n: -sum(durs[n]) if durs[n] else 0):
        us = sum(durs[name]) / len(durs[name]) if durs[name] else float("nan")
        row = []
        for c in counters:
            v = vals[name].get(c)
            row.append(f"{sum(v) / len(v):12.4g}" if v else f"{'-':>12s}")
        f, w = vals[name].get("FETCH_SIZE"), vals[name].get("WRITE_SIZE")
        bw = ""
        if f and w and us == us:
            bw = f"{(sum(f) / len(f) + sum(w) / len(w)) * 1024 / (us * 1e-6) / 1e12:6.2f}"
        print(f"{name[:52]:52s} {us:8.1f} " + " ".join(row) + f" {bw:>6s}")


if __name__ == "__main__":
    main()
