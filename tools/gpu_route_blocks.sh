#!/bin/bash
# route grid A/B: blocks per route pass (PTYPE_ROUTE_BLOCKS) on the N=1 bench and the RCCL path
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/route_blocks.jsonl
for NB in 512 2048 4096; do
  for MODE in "" "--force-dist"; do
    PTYPE_ROUTE_BLOCKS=$NB timeout -k 10 300 python bench.py $MODE --steps 30 --warmup 5 --rtt-calls 0 > gpurun_out/rb.json 2> gpurun_out/rb.err || { echo "FAILED $NB $MODE"; tail -5 gpurun_out/rb.err; exit 1; }
    echo "{\"blocks\": $NB, \"mode\": \"$MODE\", \"bench\": $(grep '"value"' gpurun_out/rb.json)}" >> gpurun_out/route_blocks.jsonl
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/route_blocks.jsonl"):
    d = json.loads(l)
    print(d["blocks"], d["mode"] or "n1", round(d["bench"]["ms_per_step"], 4), round(d["bench"]["value"] / 1e9, 2))
PY
