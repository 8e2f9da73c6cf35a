#!/bin/bash
# Compute side of an R-rank step on one GPU (bench --loopback R), R = 1, 2, 4, 8,
# plus a kernel trace of the R = 8 step.  usage: tools/gpu_loopback.sh TAG
set -o pipefail
TAG=${1:-lb}
mkdir -p gpurun_out
for R in 2 4 8; do
  timeout -k 10 200 python bench.py --loopback $R --steps 20 --warmup 3 --rtt-calls 0 > gpurun_out/lb_${TAG}_$R.json 2> gpurun_out/lb_${TAG}_$R.err || { echo "LOOPBACK $R FAILED"; tail -20 gpurun_out/lb_${TAG}_$R.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'ms/step %.4f' % d['ms_per_step'], 'G msg/s/GPU %.1f' % (d['value']/1e9), d['config']['wire'], d['config']['record_bytes'])" gpurun_out/lb_${TAG}_$R.json $R
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lbprof_$TAG -o run --output-format csv -- python bench.py --loopback 8 --steps 5 --warmup 2 --rtt-calls 0 > gpurun_out/lbprof_$TAG.log 2>&1 || { echo "PROFILE FAILED"; exit 1; }
python tools/timeline.py gpurun_out/lbprof_$TAG/run_kernel_trace.csv > gpurun_out/lb_timeline_$TAG.txt 2>&1 || true
python - "$TAG" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(f"gpurun_out/lbprof_{sys.argv[1]}/run_kernel_stats.csv")))
for r in rows[:14]:
    print(r["Name"][:60].ljust(60), r["Calls"].rjust(4), ("%.1f" % (float(r["AverageNs"]) / 1e3)).rjust(9), "us", r["Percentage"][:5], "%")
PY
