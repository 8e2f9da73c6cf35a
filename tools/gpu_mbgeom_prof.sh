#!/bin/bash
# Per-kernel times of the N=1 mailbox step at several shard counts.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for S in ${SHARDS:-64 256 512}; do
  rm -rf gpurun_out/gprof_$S
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/gprof_$S -o prof -- python3 bench.py --steps 10 --warmup 4 --rtt-calls 0 --no-secondary --graph off --mailbox-shards $S $EXTRA > gpurun_out/gprof_$S.log 2>&1
  rc=$?; echo "S=$S rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
