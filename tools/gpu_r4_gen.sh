#!/bin/bash
# Round-4: the request generator, scalar vs 4-per-thread (PTYPE_GEN_VEC), bit-exact vs the
# CPU reference, and its time in the bench step at 1 Mi and 8 Mi.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4gen}
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  "tests/test_device_kernels.py::test_gpu_route_dispatch_complete" > gpurun_out/${TAG}_tests.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_tests.log
for V in 1 0; do
  for MQ in 1048576 8388608; do
    rm -rf gpurun_out/${TAG}_v${V}_$MQ
    PTYPE_GEN_VEC=$V timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_v${V}_$MQ -o prof -- \
      python3 bench.py --msgs-per-gpu $MQ --steps 16 --warmup 4 --no-secondary > gpurun_out/${TAG}_v${V}_$MQ.log 2>&1 || exit 2
    PTYPE_GEN_VEC=$V timeout -k 10 200 python3 bench.py --msgs-per-gpu $MQ --steps 40 --warmup 8 --no-secondary > gpurun_out/${TAG}_b_v${V}_$MQ.json 2>/dev/null || exit 3
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e9,2), 'G msg/s', round(d['ms_per_step']*1e3,1), 'us/step')" gpurun_out/${TAG}_b_v${V}_$MQ.json v${V}_$MQ
  done
done
