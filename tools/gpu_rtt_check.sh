#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --force-dist --steps 10 --warmup 3 --rtt-calls 2000 > gpurun_out/rtt_dist.json 2> gpurun_out/rtt_dist.err || { echo "RTT DIST FAILED"; tail -20 gpurun_out/rtt_dist.err; exit 1; }
grep '"value"' gpurun_out/rtt_dist.json
timeout -k 10 300 python -u -m pytest tests/test_engine_multirank_gpu.py tests/test_packed_wire.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/rtt_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/rtt_tests.log; exit 1; }
tail -1 gpurun_out/rtt_tests.log
