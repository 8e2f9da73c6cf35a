#!/bin/bash
# Round-5 session D: the compiled data plane's GPU tests first (native lifecycle,
# Join runtime re-formation), then the whole GPU suite.  Every GPU step under its
# own limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5d}
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_elastic_gpu.py \
  > gpurun_out/${TAG}_elastic.log 2>&1; rc=$?
echo "elastic rc=$rc"; tail -5 gpurun_out/${TAG}_elastic.log
[ $rc -eq 0 ] || exit 2
timeout -k 10 1000 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/ \
  > gpurun_out/${TAG}_suite.log 2>&1; rc=$?
echo "suite rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/${TAG}_suite.log | tail -8
exit $rc
