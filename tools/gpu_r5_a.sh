#!/bin/bash
# Round-5 session A: loopback-8 kernel stats before / after the rank byte table +
# ordered-drain gate, the sorted-exchange and IpcComm GPU tests, the 1 Mi step's
# kernel stats and the N=1 bench.  Every GPU step under its own limit; the first
# failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5a}
PTYPE_SX_RANK_TABLE=0 PTYPE_SX_SHARD_GATE=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_l8old -o prof -- \
  python3 bench.py --loopback 8 --steps 8 --warmup 4 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_l8old.log 2>&1 || exit 2
echo l8old; tail -1 gpurun_out/${TAG}_l8old.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_l8 -o prof -- \
  python3 bench.py --loopback 8 --steps 8 --warmup 4 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_l8.log 2>&1 || exit 3
echo l8; tail -1 gpurun_out/${TAG}_l8.log
timeout -k 10 200 python3 bench.py --loopback 8 --steps 20 --warmup 5 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_l8b.json 2>gpurun_out/${TAG}_l8b.err || exit 4
echo l8b; cat gpurun_out/${TAG}_l8b.json
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_sorted_exchange_gpu.py tests/test_ipc_comm_gpu.py tests/test_xcall_gpu.py tests/test_shm_rpc_gpu.py \
  > gpurun_out/${TAG}_tests.log 2>&1 || exit 5
tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_1m -o prof -- \
  python3 bench.py --msgs-per-gpu 1048576 --steps 8 --warmup 4 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_1m.log 2>&1 || exit 6
echo 1m; tail -1 gpurun_out/${TAG}_1m.log
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_b1.json 2> gpurun_out/${TAG}_b1.err || exit 7
cat gpurun_out/${TAG}_b1.json
timeout -k 10 200 python3 bench.py --pipeline on --no-secondary > gpurun_out/${TAG}_pipe8m.json 2> gpurun_out/${TAG}_pipe8m.err || exit 8
cat gpurun_out/${TAG}_pipe8m.json
timeout -k 10 200 python3 bench.py --pipeline on --no-secondary --msgs-per-gpu 1048576 > gpurun_out/${TAG}_pipe1m.json 2> gpurun_out/${TAG}_pipe1m.err || exit 9
cat gpurun_out/${TAG}_pipe1m.json
