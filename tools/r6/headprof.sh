#!/bin/bash
# Round 6: kernel stats + counter passes of the headline step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6hp}
rm -rf gpurun_out/${TAG}_k
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_k -o k --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}.json 2>&1 || exit 1
python3 -c "
import csv,glob
f=glob.glob('gpurun_out/${TAG}_k/*kernel_stats.csv')[0]
for r in list(csv.DictReader(open(f)))[:5]: print('%-60s %5s %8.1f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))"
P=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD" \
         "SQ_WAVES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES" "FETCH_SIZE" "WRITE_SIZE"; do
  P=$((P+1)); rm -rf gpurun_out/${TAG}_pmc_$P
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/${TAG}_pmc_$P -o pmc --output-format csv -- \
    python3 bench.py --steps 4 --warmup 3 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_pmc_$P.log 2>&1 || exit 2
done
python3 tools/pmc_table.py gpurun_out/${TAG}_pmc_* > gpurun_out/${TAG}_pmc.txt
head -5 gpurun_out/${TAG}_pmc.txt | cut -c1-60,200-420
