#!/bin/bash
# Steps per graph replay (bench --steps-per-graph) at 8 Mi and 1 Mi, two repetitions.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
TAG=${1:-r4spg}
for rep in 1 2; do
  for MQ in 8388608 1048576; do
    for U in 4 10 20; do
      timeout -k 10 200 python3 bench.py --msgs-per-gpu $MQ --steps 20 --warmup 5 --steps-per-graph $U --no-secondary > gpurun_out/${TAG}.json 2>/dev/null || exit 1
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'U', sys.argv[3], round(d['value']/1e9,2), 'G msg/s', round(d['ms_per_step']*1e3,1), 'us')" gpurun_out/${TAG}.json $MQ $U
    done
  done
done
