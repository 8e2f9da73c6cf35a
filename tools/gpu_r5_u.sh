#!/bin/bash
# Round-5 session U: all four sorted-exchange events at device scope (out = only compute -> comm) -- the sorted
# exchange's GPU tests (RCCL at world 1, in-process ranks, IpcComm processes) and
# the --loopback 8 / --force-dist lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5t}
val() { python3 -c "import json; d=[json.loads(x) for x in open('$1') if x.startswith('{')][-1]; print(round(d['value']/1e9,3), round(d['ms_per_step'],4))"; }
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_sorted_exchange_gpu.py tests/test_ipc_comm_gpu.py tests/test_elastic_ipc_gpu.py \
  > gpurun_out/${TAG}_tests.txt 2>&1 || { tail -30 gpurun_out/${TAG}_tests.txt; exit 3; }
tail -2 gpurun_out/${TAG}_tests.txt
L8="python3 bench.py --loopback 8 --steps 20 --warmup 5 --rtt-calls 0 --no-secondary"
for V in new out new out; do
  F="gpurun_out/${TAG}_l8_${V}_$RANDOM.json"
  case $V in
    new) timeout -k 10 200 $L8 > $F 2>$F.err || exit 3 ;;
    out) PTYPE_SX_EVENT_FENCE=out timeout -k 10 200 $L8 > $F 2>$F.err || exit 3 ;;
  esac
  echo "l8 $V $(val $F)"
done
F="gpurun_out/${TAG}_fd_$RANDOM.json"
timeout -k 10 200 python3 bench.py --force-dist --steps 20 --warmup 5 --rtt-calls 0 --no-secondary > $F 2>$F.err || exit 3
echo "force-dist $(val $F)"
