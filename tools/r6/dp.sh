#!/bin/bash
# Round 6: the compiled-DataPlane paths on one GPU (RCCL at world 1, IpcComm across
# processes, the bench's N > 1 line over IpcComm) and the FIFO / overflow tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6dp}
timeout -k 10 1500 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread \
  tests/test_elastic_gpu.py tests/test_elastic_ipc_gpu.py tests/test_ipc_comm_gpu.py tests/test_bench.py \
  tests/test_sorted_exchange_gpu.py tests/test_packed_wire.py tests/test_engine_gpu.py \
  -k "not multi_gpu" > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed|Error" gpurun_out/${TAG}_tests.log | tail -60
exit $rc
