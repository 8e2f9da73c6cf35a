#!/bin/bash
# A/B of engine knobs on the multi-rank path: loopback R (compute side of an
# R-rank step) and the forced single-rank RCCL path, one line per variant, then
# the engine GPU tests.  usage: tools/gpu_ab.sh TAG "name:ENV=V ..." ["name2:ENV=V"] ...
set -o pipefail
TAG=$1; shift
R=${LOOPBACK_R:-8}
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  for mode in loopback rccl; do
    if [ $mode = loopback ]; then args="--loopback $R ${LOOPBACK_EXTRA}"; else args="--force-dist"; fi
    out=gpurun_out/ab_${TAG}_${name}_$mode
    env $envs timeout -k 10 200 python bench.py $args ${BENCH_EXTRA} --steps 30 --warmup 3 --rtt-calls 0 > $out.json 2> $out.err || { echo "$name $mode FAILED"; tail -20 $out.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2].ljust(14), sys.argv[3].ljust(9), 'ms/step %.4f' % d['ms_per_step'])" $out.json $name $mode
  done
done
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_engine_gpu.py tests/test_engine_multirank_gpu.py tests/test_packed_wire.py > gpurun_out/ab_${TAG}_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/ab_${TAG}_tests.log; exit 1; }
  tail -1 gpurun_out/ab_${TAG}_tests.log
fi
