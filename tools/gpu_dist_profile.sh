#!/bin/bash
# RCCL path on one GPU (--force-dist): wire v3 vs v2 step time + kernel profile of v3.
# usage (under gpurun): bash tools/gpu_dist_profile.sh TAG
set -o pipefail
TAG=${1:-dist}
mkdir -p gpurun_out
for W in v3 v2; do
  PTYPE_WIRE=$W timeout -k 10 300 python bench.py --force-dist --steps 20 --warmup 5 --rtt-calls 0 > gpurun_out/dist_${TAG}_$W.json 2> gpurun_out/dist_${TAG}_$W.err || { echo "DIST $W FAILED"; tail -20 gpurun_out/dist_${TAG}_$W.err; exit 1; }
  cat gpurun_out/dist_${TAG}_$W.json
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python bench.py --force-dist --steps 10 --warmup 2 --rtt-calls 0 > gpurun_out/prof_${TAG}.log 2>&1 || { echo "PROFILE FAILED"; tail -20 gpurun_out/prof_${TAG}.log; exit 1; }
python - "$TAG" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(f"gpurun_out/prof_{sys.argv[1]}/run_kernel_stats.csv")))
for r in rows[:16]:
    print(r["Name"][:70].ljust(70), r["Calls"].rjust(4), ("%.1f" % (float(r["AverageNs"]) / 1e3)).rjust(9), "us", r["Percentage"][:5], "%")
PY
