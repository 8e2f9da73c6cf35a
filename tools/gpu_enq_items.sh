#!/bin/bash
# Arrival-sharded mailbox enqueue: items per thread (PTYPE_ENQ_ITEMS) at 1 Mi and
# 8 Mi messages per step, mailbox delivery step times + kernel averages.
# usage (under gpurun, repo root): tools/gpu_enq_items.sh TAG
set -o pipefail
TAG=${1:-ei}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for M in 1048576 8388608; do
  for K in 1 2 4 0; do
    PTYPE_ENQ_ITEMS=$K timeout -k 10 120 python bench.py --msgs-per-gpu $M --delivery mailbox --steps 16 --warmup 8 --steps-per-graph 8 --no-secondary --rtt-calls 0 > gpurun_out/ei.json 2> gpurun_out/ei.err || { echo "M=$M K=$K FAILED"; tail -5 gpurun_out/ei.err; exit 1; }
    PTYPE_ENQ_ITEMS=$K timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/eiprof_${M}_$K -o run --output-format csv -- python bench.py --msgs-per-gpu $M --delivery mailbox --steps 16 --warmup 8 --steps-per-graph 8 --no-secondary --rtt-calls 0 > gpurun_out/eiprof.log 2>&1 || { echo "PROF M=$M K=$K FAILED"; exit 1; }
    python - $M $K <<'PY'
import csv, glob, json, sys
M, K = sys.argv[1:3]
d = json.loads(open("gpurun_out/ei.json").read().strip().splitlines()[-1])
f = glob.glob(f"gpurun_out/eiprof_{M}_{K}/**/run_kernel_stats.csv", recursive=True)[0]
ks = {r["Name"].split("(")[0].replace("void ptype::", "").replace("ptype::", "")[:22]: float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(f))}
print(f"M={M} items={K}(0=auto): {d['ms_per_step']:.4f} ms/step {d['value']/1e9:.1f} G msg/s  " + "  ".join(f"{k}={v:.1f}us" for k, v in ks.items() if k.startswith(("mailbox", "gen"))))
PY
  done
done
