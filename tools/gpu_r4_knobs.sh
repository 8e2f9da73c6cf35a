#!/bin/bash
# Headline knobs A/B, two repetitions each (same box): default, non-temporal directory gathers,
# a 4-shard stateless view, both.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
TAG=${1:-r4kn}
for rep in 1 2; do
  for V in "X=0" "PTYPE_DIR_NT=1" "PTYPE_MBOX_STATELESS_SHARDS=4" "PTYPE_MBOX_STATELESS_SHARDS=8"; do
    env $V timeout -k 10 200 python3 bench.py --steps 30 --warmup 5 --no-secondary > gpurun_out/${TAG}.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e9,2), 'G msg/s', round(d['ms_per_step']*1e3,1), 'us')" gpurun_out/${TAG}.json "$V"
  done
done
