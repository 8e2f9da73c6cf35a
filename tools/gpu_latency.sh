#!/bin/bash
# single-call latency: probe (trace breakdown) + bench p50, plus the device-runtime tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/latency_probe.py > gpurun_out/latency.json 2> gpurun_out/latency.err || { echo "PROBE FAILED"; tail -5 gpurun_out/latency.err; exit 1; }
cat gpurun_out/latency.json
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --rtt-calls 5000 > gpurun_out/lat_bench.json 2> gpurun_out/lat_bench.err || { echo "BENCH FAILED"; tail -5 gpurun_out/lat_bench.err; exit 1; }
grep -o '"p50_rtt_us": [0-9.]*' gpurun_out/lat_bench.json
timeout -k 10 300 python -u -m pytest tests/test_runtime_gpu.py tests/test_shm_rpc_gpu.py tests/test_observability.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/lat_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/lat_tests.log; exit 1; }
tail -1 gpurun_out/lat_tests.log
