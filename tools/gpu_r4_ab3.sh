#!/bin/bash
# Round-4 mailbox A/B: the mailbox GPU tests, then VAR in {1, 0} x fused sort + drain
# (PTYPE_MBOX_FUSED) -- per-kernel stats of the 8 Mi Send and the bench headline
# for each.  usage: gpu_r4_ab3.sh TAG VAR (e.g. PTYPE_MBOX_REC8)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4ab3}
VAR=${2:-PTYPE_MBOX_REC8}
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_mailbox_gpu.py \
  > gpurun_out/${TAG}_tests.log 2>&1 || exit 1
tail -2 gpurun_out/${TAG}_tests.log
for R in 1 0; do
  for F in 1 0; do
    V=${TAG}_v${R}f${F}
    rm -rf gpurun_out/${V}_prof
    env $VAR=$R PTYPE_MBOX_FUSED=$F timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${V}_prof -o prof -- \
      python3 tools/mb_variant.py actor 10 > gpurun_out/${V}_prof.log 2>&1 || exit 2
    env $VAR=$R PTYPE_MBOX_FUSED=$F timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 \
      > gpurun_out/${V}_bench.json 2> gpurun_out/${V}_bench.err || exit 3
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e9,2), 'G msg/s', round(d['ms_per_step'],4), 'ms', 'c2', round(d.get('secondaries',{}).get('config2_1m',{}).get('value',0)/1e9,2))" gpurun_out/${V}_bench.json $V
  done
done
