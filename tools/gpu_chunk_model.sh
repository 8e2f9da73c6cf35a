#!/bin/bash
# Chunk-count choice under a modelled interconnect: bench --loopback R with the
# all-to-all held for off-rank bytes / (R - 1) links x LINK GB/s.  usage: TAG [LINK]
set -o pipefail
TAG=${1:-cm}; LINK=${2:-60}
mkdir -p gpurun_out
out=gpurun_out/chunk_model_$TAG.jsonl; : > $out
for R in 2 4 8; do
  bw=$(python -c "print($LINK * ($R - 1))")
  for C in 1 2 4 8; do
    timeout -k 10 120 python bench.py --loopback $R --link-gbps $bw --chunks $C --steps 20 --warmup 3 --rtt-calls 0 --no-secondary > gpurun_out/cm.json 2> gpurun_out/cm.err || { echo "R=$R chunks=$C FAILED"; tail -5 gpurun_out/cm.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/cm.json').read().strip().splitlines()[-1]); r={'R': $R, 'link_gbps_per_rank': $bw, 'chunks': $C, 'ms_per_step': d['ms_per_step'], 'G_msg_s_node_est': $R * 8388608 / d['ms_per_step'] / 1e6}; print(json.dumps(r))" | tee -a $out
  done
done
