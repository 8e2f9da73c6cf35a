#!/bin/bash
# Round-4 mailbox A/B on one MI355X: fused sort + drain (PTYPE_MBOX_FUSED) x
# group look-back (PTYPE_LB_GROUP), per-kernel stats of the 8 Mi actor-sharded
# Send (tools/mb_variant.py) and the bench headline for each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4ab}
for F in 1 0; do
  for G in 1 0; do
    V=${TAG}_f${F}g${G}
    rm -rf gpurun_out/${V}_prof
    PTYPE_MBOX_FUSED=$F PTYPE_LB_GROUP=$G timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${V}_prof -o prof -- \
      python3 tools/mb_variant.py actor 10 > gpurun_out/${V}_prof.log 2>&1 || exit 1
    PTYPE_MBOX_FUSED=$F PTYPE_LB_GROUP=$G timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-secondary \
      > gpurun_out/${V}_bench.json 2> gpurun_out/${V}_bench.err || exit 2
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e9,2), 'G msg/s', round(d['ms_per_step'],4), 'ms')" gpurun_out/${V}_bench.json $V
  done
done
