#!/bin/bash
# Round 6: kernel stats (rocprofv3 --kernel-trace --stats) of the N = 1 bench lines:
# headline 8 Mi, SeqFold 8 Mi, config 2 at 1 Mi, wide args.  Usage: kst.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6k}
run() {  # name, bench args...
  local n=$1; shift
  rm -rf gpurun_out/${TAG}_$n
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_$n -o k --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --rtt-calls 0 --no-secondary "$@" > gpurun_out/${TAG}_$n.json 2> gpurun_out/${TAG}_$n.err
}
run head && run seq --method seqfold && run c2 --msgs-per-gpu 1048576 || exit 1
python3 tools/r6/summ.py gpurun_out/${TAG}_head.json gpurun_out/${TAG}_seq.json gpurun_out/${TAG}_c2.json
for n in head seq c2; do echo "== $n"; f=$(find gpurun_out/${TAG}_$n -name '*kernel_stats.csv'); python3 -c "
import csv,sys
for r in list(csv.DictReader(open('$f')))[:8]: print('%-70s %5s %9.1f us avg' % (r['Name'][:70], r['Calls'], float(r['AverageNs'])/1e3))"; done
