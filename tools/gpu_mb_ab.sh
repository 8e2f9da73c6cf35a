#!/bin/bash
# Mailbox A/B: the mailbox + sorted-exchange GPU tests, then `mb_variant.py VARIANT`
# under each environment given (e.g. "PTYPE_OS_LATE=0" "PTYPE_OS_LATE=1"), 3 runs each.
# usage: bash tools/gpu_mb_ab.sh TAG VARIANT ENV1 [ENV2 ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; V=$2; shift 2
timeout -k 10 500 python -u -m pytest tests/test_mailbox_gpu.py tests/test_sorted_exchange_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for E in "$@"; do
    echo -n "$E: "; env $E timeout -k 10 120 python3 tools/mb_variant.py $V 20 || exit $?
  done
done
