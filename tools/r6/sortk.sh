#!/bin/bash
# Round 6: the headline sort's kernel time (kernel stats) and two bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6sk}
rm -rf gpurun_out/${TAG}_k
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_k -o k --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_0.json 2>&1 || exit 1
python3 -c "
import csv,glob
f=glob.glob('gpurun_out/${TAG}_k/*kernel_stats.csv')[0]
for r in list(csv.DictReader(open(f)))[:4]: print('%-60s %5s %8.1f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))"
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_$r.json 2>/dev/null || exit 2
done
python3 tools/r6/summ.py gpurun_out/${TAG}_1.json gpurun_out/${TAG}_2.json
