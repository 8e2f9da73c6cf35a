#!/bin/bash
# Round 6 rehearsal: smoke, every GPU test, the N = 1 bench line (driver arguments), the
# loopback-8 line, kernel stats of the headline / SeqFold / 1 Mi steps, and counter passes
# over the headline, loopback-8 and 1 Mi steps.  Usage: final.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6f}
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 2400 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/${TAG}_tests.log | head; exit 2; }
grep -E "passed|failed" gpurun_out/${TAG}_tests.log | tail -1
timeout -k 10 600 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 3; }
timeout -k 10 300 python3 bench.py --loopback 8 --steps 20 --warmup 5 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_l8.json 2> gpurun_out/${TAG}_l8.err || exit 4
python3 tools/r6/summ.py gpurun_out/${TAG}_bench.json gpurun_out/${TAG}_l8.json
bash tools/r6/kst.sh ${TAG}k > gpurun_out/${TAG}_kst.txt 2>&1 || { tail gpurun_out/${TAG}_kst.txt; exit 5; }
for W in head l8 c2; do
  case $W in head) A="";; l8) A="--loopback 8";; c2) A="--msgs-per-gpu 1048576";; esac
  P=0
  for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE"; do
    P=$((P+1))
    rm -rf gpurun_out/${TAG}_${W}_pmc_$P
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/${TAG}_${W}_pmc_$P -o pmc --output-format csv -- \
      python3 bench.py $A --steps 4 --warmup 3 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_${W}_pmc_$P.log 2>&1
    rc=$?; echo "$W pmc pass $P rc=$rc"
    [ $rc -eq 0 ] || exit 6
  done
  python3 tools/pmc_table.py gpurun_out/${TAG}_${W}_pmc_* > gpurun_out/${TAG}_${W}_pmc.txt
done
echo done
