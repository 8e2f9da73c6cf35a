#!/bin/bash
# quick iteration: engine/packed GPU tests, then the RCCL-path profile
set -o pipefail
TAG=${1:-it}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_packed_wire.py tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/iter_$TAG.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/iter_$TAG.log; exit 1; }
tail -2 gpurun_out/iter_$TAG.log
bash tools/gpu_dist_profile.sh $TAG
