#!/bin/bash
# Round 6: smoke(), every GPU test (one pytest process, per-test limit), the N=1 bench,
# the loopback-8 line.  Usage: tools/r6/full.sh TAG [pytest -k expr]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6full}
K=${2:-}
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 2400 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${K:+-k "$K"} > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/${TAG}_tests.log | tail -8
[ $rc -eq 0 ] || exit 2
timeout -k 10 600 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 3; }
timeout -k 10 300 python3 bench.py --loopback 8 --steps 20 --warmup 5 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_l8.json 2> gpurun_out/${TAG}_l8.err || { tail -20 gpurun_out/${TAG}_l8.err; exit 4; }
python3 tools/r6/summ.py gpurun_out/${TAG}_bench.json gpurun_out/${TAG}_l8.json
