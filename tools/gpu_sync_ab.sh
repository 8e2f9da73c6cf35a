#!/bin/bash
# A/B of the engine's cross-stream hand-offs (stream wait-value words vs events):
# loopback R = 8 and the forced single-rank RCCL path, then the engine GPU tests.
set -o pipefail
TAG=${1:-ab}
mkdir -p gpurun_out
for mode in values events; do
  for R in 8; do
    PTYPE_STREAM_SYNC=$mode timeout -k 10 200 python bench.py --loopback $R --steps 20 --warmup 3 --rtt-calls 0 > gpurun_out/ab_${TAG}_${mode}_$R.json 2> gpurun_out/ab_${TAG}_${mode}_$R.err || { echo "LOOPBACK $mode $R FAILED"; tail -20 gpurun_out/ab_${TAG}_${mode}_$R.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'loopback', sys.argv[3], 'ms/step %.4f' % d['ms_per_step'])" gpurun_out/ab_${TAG}_${mode}_$R.json $mode $R
  done
  PTYPE_STREAM_SYNC=$mode timeout -k 10 200 python bench.py --force-dist --steps 20 --warmup 3 --rtt-calls 0 > gpurun_out/ab_${TAG}_${mode}_rccl.json 2> gpurun_out/ab_${TAG}_${mode}_rccl.err || { echo "RCCL $mode FAILED"; tail -20 gpurun_out/ab_${TAG}_${mode}_rccl.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'rccl-forced ms/step %.4f' % d['ms_per_step'])" gpurun_out/ab_${TAG}_${mode}_rccl.json $mode
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_engine_gpu.py tests/test_engine_multirank_gpu.py tests/test_packed_wire.py > gpurun_out/ab_${TAG}_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/ab_${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/ab_${TAG}_tests.log
