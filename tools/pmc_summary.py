#!/usr/bin/env python3
"""Per-kernel HBM traffic from rocprofv3 --pmc runs (FETCH_SIZE / WRITE_SIZE, KB)
joined with kernel durations -> achieved bandwidth per ptype kernel.

usage: python tools/pmc_summary.py <fetch_run_dir> <write_run_dir>
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        if r.get("Counter_Name") != counter:
            continue
        name = r.get("Kernel_Name", "")
        dur = None
        if r.get("End_Timestamp") and r.get("Start_Timestamp"):
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        per[name].append((float(r["Counter_Value"]), dur))
    return per


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    print(f"{'kernel':58s} {'calls':>5s} {'read MB':>9s} {'write MB':>9s} {'us':>8s} {'TB/s':>6s}")
    for name in sorted(fetch, key=lambda n: -sum(v for v, _ in fetch[n])):
        if "ptype" not in name:
            continue
        fr, wr = fetch[name], write.get(name, [])
        n = len(fr)
        rd = sum(v for v, _ in fr) / n / 1024  # KB -> MB per call
        wb = sum(v for v, _ in wr) / max(len(wr), 1) / 1024
        durs = [d for _, d in fr if d] + [d for _, d in wr if d]
        us = (sum(durs) / len(durs) * 1e6) if durs else float("nan")
        bw = (rd + wb) / 1e6 / (us * 1e-6) if durs else float("nan")
        print(f"{name[:58]:58s} {n:5d} {rd:9.1f} {wb:9.1f} {us:8.1f} {bw:6.2f}")


if __name__ == "__main__":
    main()
