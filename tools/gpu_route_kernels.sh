#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for R in 1 8; do
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/rk_$R -o run --output-format csv -- python tools/packed_route_bench.py 2097152 $R > gpurun_out/rk_$R.log 2>&1 || { echo "PROF FAILED"; tail -5 gpurun_out/rk_$R.log; exit 1; }
python - $R <<'PY'
import csv, sys
rows = list(csv.DictReader(open(f"gpurun_out/rk_{sys.argv[1]}/run_kernel_stats.csv")))
print("R =", sys.argv[1])
for r in rows[:7]:
    print("  ", r["Name"][:60].ljust(60), r["Calls"].rjust(4), ("%.1f" % (float(r["AverageNs"]) / 1e3)).rjust(7), "us")
PY
done
