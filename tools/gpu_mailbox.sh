#!/bin/bash
# HBM mailboxes on the GPU: tests, bench (direct headline + mailbox secondary),
# and a kernel-trace profile of the mailbox-delivery step.
# usage (under gpurun, repo root): tools/gpu_mailbox.sh TAG [extra pytest files]
set -o pipefail
TAG=${1:-mb}
shift
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mailbox_gpu.py "$@" -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/mbtest_$TAG.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/mbtest_$TAG.log; exit 1; }
tail -3 gpurun_out/mbtest_$TAG.log
timeout -k 10 300 python bench.py --rtt-calls 500 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "BENCH FAILED"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --rtt-calls 0 --no-secondary --delivery mailbox > gpurun_out/prof_$TAG.log 2>&1 || { echo "PROFILE FAILED"; tail -20 gpurun_out/prof_$TAG.log; exit 1; }
python - "$TAG" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/prof_{sys.argv[1]}/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:12]:
    print(r["Name"][:70].ljust(70), r["Calls"].rjust(4), ("%.1f" % (float(r["AverageNs"]) / 1e3)).rjust(9), "us", r["Percentage"][:5], "%")
PY
