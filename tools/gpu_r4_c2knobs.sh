#!/bin/bash
# 1 Mi bench step (config 2 size) by stateless view shard count, two repetitions.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
TAG=${1:-r4c2k}
for rep in 1 2; do
  for SH in 4 8 16; do
    PTYPE_MBOX_STATELESS_SHARDS=$SH timeout -k 10 200 python3 bench.py --msgs-per-gpu 1048576 --steps 40 --warmup 8 --no-secondary > gpurun_out/${TAG}.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('shards', sys.argv[2], round(d['value']/1e9,2), 'G msg/s', round(d['ms_per_step']*1e3,1), 'us')" gpurun_out/${TAG}.json $SH
  done
done
