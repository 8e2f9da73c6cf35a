#!/bin/bash
# Loopback-8 PMC: FETCH_SIZE / WRITE_SIZE passes (kernel trace only, one counter per run)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-l8pmc}
for C in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/${TAG}_$C
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/${TAG}_$C -o pmc --output-format csv -- python3 bench.py --loopback 8 --steps 4 --warmup 3 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_$C.log 2>&1 || { echo "pmc $C failed"; tail -5 gpurun_out/${TAG}_$C.log; exit 1; }
done
python3 tools/pmc_table.py --filter "" gpurun_out/${TAG}_FETCH_SIZE gpurun_out/${TAG}_WRITE_SIZE > gpurun_out/${TAG}.txt 2>&1; cat gpurun_out/${TAG}.txt
