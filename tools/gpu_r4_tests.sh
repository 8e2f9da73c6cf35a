#!/bin/bash
# Every GPU test (one pytest process, per-test timeout), then smoke().
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4t}
timeout -k 10 1100 python -u -m pytest tests -m gpu -v -rP --timeout 240 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed|skipped" gpurun_out/${TAG}_gpu_tests.log | tail -15
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/${TAG}_smoke.log
