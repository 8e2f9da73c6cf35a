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
# the ordered (SeqFold) Send's sort: one pass with look-back (default) vs count + scan + scatter
for K in "X=0" "PTYPE_MBOX_SORT=twopass" "PTYPE_MBOX_SORT=ldscount"; do
  env $K timeout -k 10 200 python3 bench.py --no-secondary --rtt-calls 0 --method seqfold > gpurun_out/${TAG}_seq_$K.json 2>gpurun_out/${TAG}_seq_$K.err || exit 4
  echo "seqfold [$K] $(val gpurun_out/${TAG}_seq_$K.json)"
done
# the headline 8 Mi step: 4096- vs 2048-message tiles for the unfused sort + ring drain
for K in "X=0" "PTYPE_MBOX_SK=4"; do
  env $K timeout -k 10 200 python3 bench.py --no-secondary --rtt-calls 0 > gpurun_out/${TAG}_8m_$K.json 2>gpurun_out/${TAG}_8m_$K.err || exit 5
  echo "8m [$K] $(val gpurun_out/${TAG}_8m_$K.json)"
done
# the N > 1 path at world 1 with the RCCL collectives forced on: eager vs one hipGraph per step
for K in "--graph off" "--graph on"; do
  timeout -k 10 200 python3 bench.py --force-dist --no-secondary --rtt-calls 0 $K > "gpurun_out/${TAG}_fd_${K#--graph }.json" 2>"gpurun_out/${TAG}_fd_${K#--graph }.err" || exit 6
  echo "force-dist [$K] $(val "gpurun_out/${TAG}_fd_${K#--graph }.json")"
done
