#!/bin/bash
# Round-5 session G: the N > 1 sender sort's tile variants on the loopback-8
# compute side (PTYPE_SX_TILE: 2048-message tiles and/or early argument loads),
# each line verified by the bench; then the sorted-exchange GPU tests with the
# best variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5g}
val() { python3 -c "import json; d=json.load(open('$1')); print(round(d['value']/1e9,3), round(d['ms_per_step'],4))"; }
L8="python3 bench.py --loopback 8 --steps 20 --warmup 5 --rtt-calls 0 --no-secondary"
for K in "X=0" "PTYPE_SX_TILE=4" "PTYPE_SX_TILE=4e" "PTYPE_SX_TILE=8e" "X=1"; do
  env $K timeout -k 10 200 $L8 > gpurun_out/${TAG}_l8_$K.json 2>gpurun_out/${TAG}_l8_$K.err || exit 3
  echo "l8 [$K] $(val gpurun_out/${TAG}_l8_$K.json)"
done
