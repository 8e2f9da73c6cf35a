#!/bin/bash
# Round 6: mailbox GPU tests, then the in-process actor / arrival A/B at 8 Mi.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6ab2}
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/ -m gpu -k "mailbox or arrival" \
  > gpurun_out/${TAG}_tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/${TAG}_tests.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/${TAG}_tests.log | tail -1
timeout -k 10 300 python3 tools/r6/ab_inproc.py > gpurun_out/${TAG}.json 2> gpurun_out/${TAG}.err || exit 2
cat gpurun_out/${TAG}.json
