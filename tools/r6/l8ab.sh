#!/bin/bash
# Round 6: sorted-exchange GPU tests, then the loopback-8 line three times (and its kernel stats).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6l8}
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_sorted_exchange_gpu.py \
  tests/test_ipc_comm_gpu.py tests/test_engine_multirank_gpu.py -m gpu > gpurun_out/${TAG}_tests.log 2>&1 \
  || { grep -E "FAILED|Error" gpurun_out/${TAG}_tests.log | head; exit 1; }
grep -E "passed|failed" gpurun_out/${TAG}_tests.log | tail -1
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --loopback 8 --steps 20 --warmup 5 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_$r.json 2> gpurun_out/${TAG}_$r.err || exit 2
done
python3 tools/r6/summ.py gpurun_out/${TAG}_1.json gpurun_out/${TAG}_2.json gpurun_out/${TAG}_3.json
rm -rf gpurun_out/${TAG}_k
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_k -o k --output-format csv -- \
  python3 bench.py --loopback 8 --steps 20 --warmup 5 --rtt-calls 0 --no-secondary > /dev/null 2>&1 || exit 3
python3 -c "
import csv,glob
f=glob.glob('gpurun_out/${TAG}_k/*kernel_stats.csv')[0]
for r in list(csv.DictReader(open(f)))[:7]: print('%-60s %5s %8.1f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))"
