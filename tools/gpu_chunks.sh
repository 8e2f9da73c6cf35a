#!/bin/bash
# chunk count A/B on the RCCL path (--force-dist)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/chunks.jsonl
for CH in 2 4 6 8; do
  timeout -k 10 300 python bench.py --force-dist --chunks $CH --steps 30 --warmup 5 --rtt-calls 0 > gpurun_out/ch.json 2> gpurun_out/ch.err || { echo "FAILED $CH"; tail -5 gpurun_out/ch.err; exit 1; }
  echo "{\"chunks\": $CH, \"bench\": $(grep '"value"' gpurun_out/ch.json)}" >> gpurun_out/chunks.jsonl
done
python - <<'PY'
import json
for l in open("gpurun_out/chunks.jsonl"):
    d = json.loads(l)
    print(d["chunks"], round(d["bench"]["ms_per_step"], 4), round(d["bench"]["value"] / 1e9, 2))
PY
