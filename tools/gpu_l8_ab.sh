#!/bin/bash
# Loopback-8 A/B over environments: sorted-exchange GPU tests, then 3 rounds of
# bench --loopback 8 under each environment given.  usage: TAG ENV1 [ENV2 ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
timeout -k 10 400 python -u -m pytest tests/test_sorted_exchange_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for E in "$@"; do
    env $E timeout -k 10 200 python3 bench.py --loopback 8 --steps 10 --warmup 4 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_l8.json 2> gpurun_out/${TAG}_l8.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'loop8', round(d['ms_per_step'],4), 'ms/step')" gpurun_out/${TAG}_l8.json "$E"
  done
done
