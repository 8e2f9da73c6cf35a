#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for NB in 256 512 1024 2048 4096; do
  PTYPE_META_BLOCKS=$NB timeout -k 10 120 python tools/meta_bench.py >> gpurun_out/meta_sweep.jsonl 2> gpurun_out/meta_sweep.err || { echo "FAILED $NB"; tail -5 gpurun_out/meta_sweep.err; exit 1; }
done
cat gpurun_out/meta_sweep.jsonl
