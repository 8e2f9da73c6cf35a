#!/bin/bash
# Latency path A/B: request ring in device memory (default) vs pinned host memory,
# then the dispatcher's GPU tests.
set -o pipefail
TAG=${1:-ring}
mkdir -p gpurun_out
for rm in device host device host; do
  PTYPE_RING_MEM=$rm timeout -k 10 120 python bench.py --steps 2 --warmup 1 --rtt-calls 20000 > gpurun_out/ring_${TAG}_$rm.json 2> gpurun_out/ring_${TAG}_$rm.err || { echo "BENCH $rm FAILED"; tail -20 gpurun_out/ring_${TAG}_$rm.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2].ljust(7), 'p50 %.3f us' % d['p50_rtt_us'], d.get('rtt_request_ring'))" gpurun_out/ring_${TAG}_$rm.json $rm
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_runtime_gpu.py tests/test_shm_rpc_gpu.py tests/test_observability.py tests/test_models.py tests/test_examples.py > gpurun_out/ring_${TAG}_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/ring_${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/ring_${TAG}_tests.log
