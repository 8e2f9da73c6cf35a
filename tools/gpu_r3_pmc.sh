#!/bin/bash
# Round-3 perf session: mailbox + sorted-exchange GPU tests, N=1 bench, loopback-8,
# then PMC passes (kernel trace only, one counter group per run) over both.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-p}
timeout -k 10 420 python -u -m pytest tests/test_mailbox_gpu.py tests/test_sorted_exchange_gpu.py -v --timeout 150 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/${TAG}_tests.log | tail -15
[ $rc -le 1 ] || exit $rc
timeout -k 10 240 python bench.py --steps 20 --warmup 8 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; head -c 3000 gpurun_out/${TAG}_bench.json; echo
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python bench.py --loopback 8 --steps 10 --warmup 4 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_loop8.json 2> gpurun_out/${TAG}_loop8.err
rc=$?; echo "loop8 rc=$rc"; head -c 300 gpurun_out/${TAG}_loop8.json; echo
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
P=0
for C in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS"; do
  P=$((P+1))
  for MODE in n1 l8; do
    if [ $MODE = n1 ]; then A="--steps 3 --warmup 1"; else A="--loopback 8 --steps 3 --warmup 1"; fi
    timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/${TAG}_pmc_${MODE}_$P -o pmc --output-format csv -- python3 bench.py $A --rtt-calls 0 --graph off --no-secondary > gpurun_out/${TAG}_pmc_${MODE}_$P.log 2>&1
    rc=$?; echo "pmc $MODE pass $P rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
for MODE in n1 l8; do
  python3 tools/pmc_table.py gpurun_out/${TAG}_pmc_${MODE}_1 gpurun_out/${TAG}_pmc_${MODE}_2 gpurun_out/${TAG}_pmc_${MODE}_3 > gpurun_out/${TAG}_pmc_${MODE}.txt
  cat gpurun_out/${TAG}_pmc_${MODE}.txt
done
