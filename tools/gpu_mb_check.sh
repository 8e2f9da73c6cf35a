#!/bin/bash
# mailbox GPU tests, then the three mailbox variants' Send time (tools/mb_variant.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mailbox_gpu.py tests/test_sorted_exchange_gpu.py > gpurun_out/mbt.log 2>&1 || { tail -30 gpurun_out/mbt.log; exit 1; }
tail -2 gpurun_out/mbt.log
for V in ${@:-actor arrival seqfold}; do
  timeout -k 10 120 python3 tools/mb_variant.py $V 20 || exit $?
done
