#!/bin/bash
# Round-5 session R: loopback-8 chunk counts (a chunk of 4 Mi is 1024 sender tiles, 1.33
# rounds of the 768 resident blocks; 3 chunks of 2.67 Mi fit one round each).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5r}
val() { python3 -c "import json; d=[json.loads(x) for x in open('$1') if x.startswith('{')][-1]; print(round(d['value']/1e9,3), round(d['ms_per_step'],4), d['config'].get('chunks'))"; }
L8="python3 bench.py --loopback 8 --steps 20 --warmup 5 --rtt-calls 0 --no-secondary"
for C in 2 1 3 4 6 2 3; do
  F="gpurun_out/${TAG}_l8_c${C}_$RANDOM.json"
  timeout -k 10 200 $L8 --chunks $C > $F 2>$F.err || exit 3
  echo "l8 chunks=$C $(val $F)"
done
