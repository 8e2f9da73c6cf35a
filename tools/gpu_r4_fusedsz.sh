#!/bin/bash
# Fused sort + drain vs two kernels by batch size (bench step, generator included).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
TAG=${1:-r4fz}
for MQ in 524288 1048576 2097152 4194304; do
  for F in 1 0; do
    PTYPE_MBOX_FUSED=$F timeout -k 10 200 python3 bench.py --msgs-per-gpu $MQ --steps 40 --warmup 8 --no-secondary > gpurun_out/${TAG}_${MQ}_$F.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'fused', sys.argv[3], round(d['value']/1e9,2), 'G msg/s', round(d['ms_per_step']*1e3,1), 'us')" gpurun_out/${TAG}_${MQ}_$F.json $MQ $F
  done
done
