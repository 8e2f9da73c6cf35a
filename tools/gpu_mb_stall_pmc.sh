#!/bin/bash
# Stall counters of the N=1 mailbox Send (per-actor rings): where do the scatter
# and drain waves wait?  Two passes, kernel trace only.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${1:-actor}
P=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD" "SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_BUSY_CYCLES TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES"; do
  P=$((P+1))
  rm -rf gpurun_out/stall_${V}_$P
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/stall_${V}_$P -o pmc --output-format csv -- python3 tools/mb_variant.py $V 3 > gpurun_out/stall_${V}_$P.log 2>&1
  rc=$?; echo "pass $P rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_table.py gpurun_out/stall_${V}_1 gpurun_out/stall_${V}_2 > gpurun_out/stall_${V}.txt
cat gpurun_out/stall_${V}.txt
