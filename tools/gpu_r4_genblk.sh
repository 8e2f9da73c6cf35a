#!/bin/bash
# Generator grid sweep (PTYPE_GEN_BLOCKS) at 1 Mi and 8 Mi: kernel time from a trace of the bench step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4gb}
for MQ in 1048576 8388608; do
  for GB in 512 1024 2048 4096 8192; do
    D=gpurun_out/${TAG}_${MQ}_$GB
    rm -rf $D
    PTYPE_GEN_VEC=0 PTYPE_GEN_BLOCKS=$GB timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D -o prof -- \
      python3 bench.py --msgs-per-gpu $MQ --steps 8 --warmup 4 --no-secondary > $D.log 2>&1 || exit 1
    echo -n "$MQ $GB: "; python3 tools/rocpd_summary.py $D/prof_results.db | grep gen_requests | awk '{print $4}'
  done
done
