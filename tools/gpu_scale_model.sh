#!/bin/bash
# Modelled node scaling with the current multi-rank pipeline: bench --loopback R
# (rank 0 of a symmetric R-rank node, default chunks) with the all-to-alls held
# for the off-rank bytes at LINK GB/s per link x (R - 1) links.  usage: TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-sm}
mkdir -p gpurun_out
out=gpurun_out/scale_model_$TAG.jsonl; : > $out
for LINK in 0 60 100; do
  for R in 2 4 8; do
    bw=$(python3 -c "print($LINK * ($R - 1))")
    timeout -k 10 150 python3 bench.py --loopback $R --link-gbps $bw --steps 20 --warmup 4 --rtt-calls 0 --no-secondary > gpurun_out/sm.json 2> gpurun_out/sm.err || { echo "R=$R link=$LINK FAILED"; tail -5 gpurun_out/sm.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/sm.json').read().strip().splitlines()[-1]); r={'R': $R, 'link_gbps_per_link': $LINK, 'ms_per_step': round(d['ms_per_step'], 4), 'G_msg_s_node_est': round($R * 8388608 / d['ms_per_step'] / 1e6, 1), 'wire_bytes_per_msg': d['config'].get('wire_bytes_per_msg')}; print(json.dumps(r))" | tee -a $out
  done
done
