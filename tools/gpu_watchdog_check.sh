#!/bin/bash
# The bench's hang watchdog fires, dumps the engine's hand-off state and exits 3
# (forced with a 1 s limit on a run that takes longer), then the full GPU suite.
# usage (under gpurun, repo root): tools/gpu_watchdog_check.sh TAG
set -o pipefail
TAG=${1:-wd}
mkdir -p gpurun_out
PTYPE_HANG_DIAG=2 timeout -k 10 120 python bench.py --force-dist --steps 20000 --warmup 2 --rtt-calls 0 --no-secondary > gpurun_out/wd_$TAG.out 2> gpurun_out/wd_$TAG.err
rc=$?
echo "watchdog run exit: $rc"; grep -E "HANG|signalled|drained" gpurun_out/wd_$TAG.err | head -12
[ $rc -eq 3 ] || { echo "WATCHDOG DID NOT FIRE AS EXPECTED"; tail -20 gpurun_out/wd_$TAG.err; exit 1; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/test_$TAG.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/test_$TAG.log; exit 1; }
tail -1 gpurun_out/test_$TAG.log
