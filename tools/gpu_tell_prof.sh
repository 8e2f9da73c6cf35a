#!/bin/bash
# Token-ring tells (bench_suite tell): wall time per epoch vs kernel time per epoch.
# usage (under gpurun, repo root): tools/gpu_tell_prof.sh TAG
set -o pipefail
TAG=${1:-tell}
mkdir -p gpurun_out
timeout -k 10 200 python tools/bench_suite.py tell > gpurun_out/tell_$TAG.jsonl 2> gpurun_out/tell_$TAG.err || { echo "TELL FAILED"; tail -20 gpurun_out/tell_$TAG.err; exit 1; }
cat gpurun_out/tell_$TAG.jsonl
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/tellprof_$TAG -o run --output-format csv -- python tools/bench_suite.py tell > gpurun_out/tellprof_$TAG.log 2>&1 || { echo "PROFILE FAILED"; tail -20 gpurun_out/tellprof_$TAG.log; exit 1; }
python - "$TAG" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/tellprof_{sys.argv[1]}/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:12]:
    print(r["Name"][:60].ljust(60), r["Calls"].rjust(5), ("%.1f" % (float(r["AverageNs"]) / 1e3)).rjust(9), "us", r["Percentage"][:5], "%")
PY
