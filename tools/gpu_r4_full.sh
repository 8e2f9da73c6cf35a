#!/bin/bash
# Round-4 closing tiers on one MI355X: every GPU test, smoke(), the N=1 bench, then the
# N=4 bench as four processes on this GPU over IpcComm (host time per Send at R=4).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4full}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -rP --timeout 240 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed|skipped" gpurun_out/${TAG}_gpu_tests.log | tail -15
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/${TAG}_smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; head -c 600 gpurun_out/${TAG}_bench.json; echo
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 4 --comm ipc --msgs-per-gpu 1048576 --actors-per-gpu 32768 --steps 10 --warmup 5 --rtt-calls 100 --no-secondary \
  > gpurun_out/${TAG}_ipc4.json 2> gpurun_out/${TAG}_ipc4.err
rc=$?; echo "ipc4 rc=$rc"; tail -c 1500 gpurun_out/${TAG}_ipc4.json; echo
