#!/bin/bash
# Sorted exchange receiver drain grid sweep (PTYPE_SX_DRAIN_BLOCKS) on the loopback-8 step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4db}
for B in 2048 1024 4096 8192; do
  rm -rf gpurun_out/${TAG}_$B
  PTYPE_SX_DRAIN_BLOCKS=$B timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_$B -o prof -- \
    python3 bench.py --loopback 8 --steps 6 --warmup 4 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_$B.log 2>&1 || exit 1
  echo -n "blocks $B drain_par<2>: "; python3 tools/rocpd_summary.py gpurun_out/${TAG}_$B/prof_results.db | grep "sx_drain_par_kernelILi2" | awk '{print $4}'
done
