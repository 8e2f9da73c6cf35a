#!/bin/bash
# Round-5 session S: loopback-8 hand-off costs.  The next Send's agreement vector is
# cleared by this Send's first completion launch instead of a fill launch at the
# start of the step (PTYPE_SX_META_ZERO=0: the old fill); the compute -> comm
# events without their system-scope fence (PTYPE_SX_EVENT_FENCE=device).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5s}
val() { python3 -c "import json; d=[json.loads(x) for x in open('$1') if x.startswith('{')][-1]; print(round(d['value']/1e9,3), round(d['ms_per_step'],4))"; }
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_sorted_exchange_gpu.py tests/test_ipc_comm_gpu.py > gpurun_out/${TAG}_tests.txt 2>&1 || { tail -30 gpurun_out/${TAG}_tests.txt; exit 3; }
tail -2 gpurun_out/${TAG}_tests.txt
L8="python3 bench.py --loopback 8 --steps 20 --warmup 5 --rtt-calls 0 --no-secondary"
for V in new old fence new old fence; do
  F="gpurun_out/${TAG}_l8_${V}_$RANDOM.json"
  case $V in
    new) timeout -k 10 200 $L8 > $F 2>$F.err || exit 3 ;;
    old) PTYPE_SX_META_ZERO=0 timeout -k 10 200 $L8 > $F 2>$F.err || exit 3 ;;
    fence) PTYPE_SX_EVENT_FENCE=device timeout -k 10 200 $L8 > $F 2>$F.err || exit 3 ;;
  esac
  echo "l8 $V $(val $F)"
done
