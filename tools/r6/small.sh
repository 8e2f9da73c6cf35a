#!/bin/bash
# Round 6: loopback-8 at 256 Ki messages per rank -- kernel, memory-copy and HIP API
# traces of the eager sorted-exchange Send (where a small step's time goes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6s}
for c in 0 1; do
  rm -rf gpurun_out/${TAG}_$c
  PTYPE_TUNE=sx_comm_cs=$c timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace -d gpurun_out/${TAG}_$c \
    -o t --output-format csv -- python3 bench.py --loopback 8 --msgs-per-gpu 262144 --steps 20 --warmup 5 --rtt-calls 0 \
    --no-secondary > gpurun_out/${TAG}_$c.json 2> gpurun_out/${TAG}_$c.err || exit 1
done
ls -R gpurun_out/${TAG}_0 | head
