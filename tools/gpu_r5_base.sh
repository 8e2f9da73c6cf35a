#!/bin/bash
# Round-5 baseline: loopback-8 kernel stats, the 1 Mi (config 2) step's kernel stats,
# and the N=1 bench with secondaries.  Every GPU step under its own limit; the first
# failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5base}
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_l8 -o prof -- \
  python3 bench.py --loopback 8 --steps 8 --warmup 4 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_l8.log 2>&1 || exit 2
echo l8 done; tail -1 gpurun_out/${TAG}_l8.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_1m -o prof -- \
  python3 bench.py --msgs-per-gpu 1048576 --steps 8 --warmup 4 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_1m.log 2>&1 || exit 3
echo 1m done; tail -1 gpurun_out/${TAG}_1m.log
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_b1.json 2> gpurun_out/${TAG}_b1.err || exit 4
cat gpurun_out/${TAG}_b1.json
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  "tests/test_ipc_comm_gpu.py::test_killed_rank_is_a_peer_failure_within_the_timeout" > gpurun_out/${TAG}_kill.log 2>&1 || exit 5
tail -3 gpurun_out/${TAG}_kill.log
