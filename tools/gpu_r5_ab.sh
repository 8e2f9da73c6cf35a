#!/bin/bash
# Round-5 session AB: loopback-8 with the completion's messages per thread per trip
# (PTYPE_COMP_U 2 / 4 (default) / 8) and the parallel drain's blocks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5ab}
val() { python3 -c "import json; d=[json.loads(x) for x in open('$1') if x.startswith('{')][-1]; print(round(d['value']/1e9,3), round(d['ms_per_step'],4))"; }
L8="python3 bench.py --loopback 8 --steps 20 --warmup 5 --rtt-calls 0 --no-secondary"
for K in ${KS:-"X=0" "PTYPE_COMP_U=8" "PTYPE_COMP_U=2" "PTYPE_SX_DRAIN_BLOCKS=4096" "PTYPE_SX_DRAIN_BLOCKS=1024" "X=0" "PTYPE_COMP_U=8"}; do
  F="gpurun_out/${TAG}_$(echo $K | tr ' =' '__')_$RANDOM.json"
  env $K timeout -k 10 200 $L8 > $F 2>$F.err || exit 3
  echo "l8 [$K] $(val $F)"
done
