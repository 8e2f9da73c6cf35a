#!/bin/bash
# GPU validation + bench + kernel profile (run under gpurun from the repo root).
# usage: tools/gpu_check.sh TAG [pytest-target]
set -o pipefail
TAG=${1:-run}
TARGET=${2:-tests}
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "SMOKE FAILED"; tail -30 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 700 python -u -m pytest $TARGET -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/test_$TAG.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/test_$TAG.log; exit 1; }
tail -1 gpurun_out/test_$TAG.log
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "BENCH FAILED"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
# the RCCL collective path on one rank (all-to-alls + barrier + all_reduce)
timeout -k 10 300 python bench.py --force-dist --steps 10 --warmup 3 --rtt-calls 0 > gpurun_out/bench_dist_$TAG.json 2> gpurun_out/bench_dist_$TAG.err || { echo "DIST BENCH FAILED"; tail -20 gpurun_out/bench_dist_$TAG.err; exit 1; }
cat gpurun_out/bench_dist_$TAG.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --rtt-calls 0 --no-secondary > gpurun_out/prof_$TAG.log 2>&1 || { echo "PROFILE FAILED"; exit 1; }
python - "$TAG" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/prof_{sys.argv[1]}/**/run_kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in rows[:12]:
    print(r["Name"][:60].ljust(60), r["Calls"].rjust(4), ("%.1f" % (float(r["AverageNs"]) / 1e3)).rjust(9), "us", r["Percentage"][:5], "%")
PY
