#!/bin/bash
# Mailbox iteration on one GPU: the mailbox GPU tests, then each Send variant's
# time (+ the message-order drain A/B) and a per-kernel profile.
# usage (under gpurun): bash tools/gpu_mb_iter.sh TAG [pytest -k expr]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-mbiter}
K=${2:-}
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 400 python -u -m pytest tests/test_mailbox_gpu.py -x -q --timeout 120 --timeout-method thread "${KARG[@]}" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for V in actor arrival seqfold; do
  timeout -k 10 120 python3 tools/mb_variant.py $V 20 || exit $?
done
PTYPE_MBOX_DRAIN=msg timeout -k 10 120 python3 tools/mb_variant.py actor 20 || exit $?
MB_M=1048576 timeout -k 10 120 python3 tools/mb_variant.py actor 50 || exit $?
MB_M=1048576 timeout -k 10 120 python3 tools/mb_variant.py arrival 50 || exit $?
for V in actor arrival seqfold; do
  rm -rf gpurun_out/${TAG}_prof_$V
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_$V -o prof -- python3 tools/mb_variant.py $V 5 > gpurun_out/${TAG}_prof_$V.log 2>&1 || exit $?
done
