#!/bin/bash
# route_prep variants (items per thread x pipelined id loads): correctness test, timing, per-kernel stats.
# usage (under gpurun, repo root): tools/gpu_prep_sweep.sh TAG
set -o pipefail
TAG=${1:-ps}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_device_kernels.py -m gpu -x -q -k route_directory --timeout 120 --timeout-method thread > gpurun_out/ps_test_$TAG.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/ps_test_$TAG.log; exit 1; }
tail -1 gpurun_out/ps_test_$TAG.log
timeout -k 10 300 python tools/prep_sweep.py > gpurun_out/ps_$TAG.jsonl 2> gpurun_out/ps_$TAG.err || { echo "SWEEP FAILED"; tail -20 gpurun_out/ps_$TAG.err; exit 1; }
cat gpurun_out/ps_$TAG.jsonl
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/psprof_$TAG -o run --output-format csv -- python tools/prep_sweep.py 4194304 8 > gpurun_out/psprof_$TAG.log 2>&1 || { echo "PROFILE FAILED"; tail -20 gpurun_out/psprof_$TAG.log; exit 1; }
python - "$TAG" <<'PY'
import csv, glob, sys, collections
f = glob.glob(f"gpurun_out/psprof_{sys.argv[1]}/**/run_kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "route_prep" in r["Kernel_Name"]]
by = collections.defaultdict(list)
for r in rows:
    by[r["Kernel_Name"][:70]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in by.items():
    v = sorted(v)
    print(k.ljust(70), len(v), "median %.1f us" % v[len(v) // 2])
PY
