#!/bin/bash
# Round-5 session P: quick A/Bs -- the stateless ring view (4 / 2 shards), the generator's
# grid, and the loopback-8 sender with early argument loads (re-measured twice).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5p}
val() { python3 -c "import json; d=[json.loads(x) for x in open('$1') if x.startswith('{')][-1]; print(round(d['value']/1e9,3), round(d['ms_per_step'],4))"; }
for K in "X=0" "PTYPE_MBOX_STATELESS_SHARDS=4" "PTYPE_MBOX_STATELESS_SHARDS=2" "PTYPE_GEN_BLOCKS=4096" "PTYPE_GEN_BLOCKS=16384" "X=1"; do
  F="gpurun_out/${TAG}_8m_$(echo $K | tr ' =' '__').json"
  env $K timeout -k 10 200 python3 bench.py --no-secondary --rtt-calls 0 > $F 2>$F.err || exit 3
  echo "8m [$K] $(val $F)"
done
L8="python3 bench.py --loopback 8 --steps 20 --warmup 5 --rtt-calls 0 --no-secondary"
for K in "X=0" "PTYPE_SX_TILE=4e" "X=1" "PTYPE_SX_TILE=4e"; do
  F="gpurun_out/${TAG}_l8_$(echo $K | tr ' =' '__')_$RANDOM.json"
  env $K timeout -k 10 200 $L8 > $F 2>$F.err || exit 4
  echo "l8 [$K] $(val $F)"
done
