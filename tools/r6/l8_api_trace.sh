#!/bin/bash
# Round 6: loopback-8 step with the HIP API trace (host cost per call) + kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6_l8rt}
rm -rf gpurun_out/$TAG
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --stats -d gpurun_out/$TAG -o rt --output-format csv -- \
  python3 bench.py --loopback 8 --steps 20 --warmup 5 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}.json 2> gpurun_out/${TAG}.err || exit 1
find gpurun_out/$TAG -name '*stats.csv' | head
