#!/bin/bash
# Cross-process single call (X3): the GPU test (device and host request ring),
# then the calculator xproc bench with the ring on the device and in host shm.
# usage (under gpurun, repo root): tools/gpu_xproc.sh TAG
set -o pipefail
TAG=${1:-xproc}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_shm_rpc_gpu.py -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/xproc_test_$TAG.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/xproc_test_$TAG.log; exit 1; }
grep -E "p50 RTT|passed|failed" gpurun_out/xproc_test_$TAG.log
OUT=gpurun_out/xproc_$TAG.jsonl
: > $OUT
timeout -k 10 200 python tools/bench_suite.py xproc --calls 20000 >> $OUT 2> gpurun_out/xproc_$TAG.err || { echo "XPROC DEVICE FAILED"; tail -20 gpurun_out/xproc_$TAG.err; exit 1; }
PTYPE_XPROC_RING=host timeout -k 10 200 python tools/bench_suite.py xproc --calls 20000 >> $OUT 2>> gpurun_out/xproc_$TAG.err || { echo "XPROC HOST FAILED"; tail -20 gpurun_out/xproc_$TAG.err; exit 1; }
grep '^{' $OUT
