#!/bin/bash
# Loopback-8 PMC (round 4): HBM bytes (FETCH_SIZE, WRITE_SIZE: one pass each) and the stall
# counters (two passes) of the R = 8 pipeline's kernels; kernel trace only, each pass killed
# at its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4l8pmc}
P=0
for C in "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD" \
         "SQ_WAVES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES"; do
  P=$((P+1))
  rm -rf gpurun_out/${TAG}_$P
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/${TAG}_$P -o pmc --output-format csv -- \
    python3 bench.py --loopback 8 --steps 4 --warmup 3 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_$P.log 2>&1
  rc=$?; echo "pass $P rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_table.py gpurun_out/${TAG}_1 gpurun_out/${TAG}_2 gpurun_out/${TAG}_3 gpurun_out/${TAG}_4 > gpurun_out/${TAG}.txt
cat gpurun_out/${TAG}.txt
