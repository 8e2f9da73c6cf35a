#!/bin/bash
# the driver's round-end entry points on one GPU: smoke() and a short bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 200 python bench.py --steps 3 --warmup 1 > gpurun_out/short_bench.json 2> gpurun_out/short_bench.err || { echo "BENCH FAILED"; tail -20 gpurun_out/short_bench.err; exit 1; }
grep -o '"value": [0-9.e+]*, "unit": "msg/s"' gpurun_out/short_bench.json
