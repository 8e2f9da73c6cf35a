#!/bin/bash
# PMC of the N=1 mailbox Send (tools/mb_variant.py actor): stall counters (two
# passes) and HBM bytes (FETCH_SIZE, WRITE_SIZE: one pass each).  Kernel trace
# only, each pass under its own kill timer.  Env passes through (e.g. PTYPE_MBOX_FUSED).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4pmc}
P=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD" \
         "SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  P=$((P+1))
  rm -rf gpurun_out/${TAG}_$P
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/${TAG}_$P -o pmc --output-format csv -- \
    python3 tools/mb_variant.py actor 3 > gpurun_out/${TAG}_$P.log 2>&1
  rc=$?; echo "pass $P rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_table.py gpurun_out/${TAG}_1 gpurun_out/${TAG}_2 gpurun_out/${TAG}_3 gpurun_out/${TAG}_4 > gpurun_out/${TAG}.txt
cat gpurun_out/${TAG}.txt
