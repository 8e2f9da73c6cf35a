#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for V in actor; do
  MB_M=1048576 timeout -k 10 120 python3 tools/mb_variant.py $V 20 || exit $?
  rm -rf gpurun_out/v1m_$V
  MB_M=1048576 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/v1m_$V -o prof -- python3 tools/mb_variant.py $V 10 > gpurun_out/v1m_$V.log 2>&1 || exit $?
done
