#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for V in actor arrival seqfold; do
  timeout -k 10 120 python3 tools/mb_variant.py $V 10 || exit $?
  rm -rf gpurun_out/vprof_$V
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/vprof_$V -o prof -- python3 tools/mb_variant.py $V 5 > gpurun_out/vprof_$V.log 2>&1 || exit $?
done
