#!/bin/bash
# Round 6 last check of the committed tree: smoke, every GPU test, the N = 1 bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
TAG=${1:-r6z}
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/${TAG}_tests.log | head; exit 2; }
grep -E "passed|failed" gpurun_out/${TAG}_tests.log | tail -1
timeout -k 10 600 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 3; }
python3 tools/r6/summ.py gpurun_out/${TAG}_bench.json
