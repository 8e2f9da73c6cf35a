#!/bin/bash
# Round-5 session I: the one-argument SeqFold batch (no a1 column: the windowed
# ordered drain's smaller LDS) with 2048- vs 4096-record windows and the binned
# form, then counter passes over the SeqFold step and the 1 Mi step (kernel trace
# only, each pass under its own kill limit).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5i}
val() { python3 -c "import json; d=json.load(open('$1')); print(round(d['value']/1e9,3), round(d['ms_per_step'],4))"; }
for K in "X=0" "PTYPE_ORD_WIN=4096" "PTYPE_ORD_DRAIN=bin PTYPE_ORD_BIN_ROUNDS=1"; do
  F="gpurun_out/${TAG}_seq_$(echo $K | tr ' =' '__').json"
  env $K timeout -k 10 200 python3 bench.py --no-secondary --rtt-calls 0 --method seqfold > $F 2>$F.err || exit 3
  echo "seqfold [$K] $(val $F)"
done
for W in seq 1m; do
  if [ $W = seq ]; then A="--method seqfold"; else A="--msgs-per-gpu 1048576"; fi
  P=0
  for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA"; do
    P=$((P+1))
    rm -rf gpurun_out/${TAG}_${W}_pmc_$P
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/${TAG}_${W}_pmc_$P -o pmc --output-format csv -- \
      python3 bench.py $A --steps 4 --warmup 3 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_${W}_pmc_$P.log 2>&1
    rc=$?; echo "$W pmc pass $P rc=$rc"
    [ $rc -eq 0 ] || break
  done
  python3 tools/pmc_table.py gpurun_out/${TAG}_${W}_pmc_* > gpurun_out/${TAG}_${W}_pmc.txt
  sed -n 1,12p gpurun_out/${TAG}_${W}_pmc.txt
done
