#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for SC in system device; do
  PTYPE_EVENT_SCOPE=$SC timeout -k 10 300 python bench.py --force-dist --steps 30 --warmup 5 --rtt-calls 0 > gpurun_out/evscope_$SC.json 2> gpurun_out/evscope_$SC.err || { echo "FAILED $SC"; tail -5 gpurun_out/evscope_$SC.err; exit 1; }
  echo $SC $(python -c "import json;d=json.load(open('gpurun_out/evscope_$SC.json'));print(d['ms_per_step'])")
done
