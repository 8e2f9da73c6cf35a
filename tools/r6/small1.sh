#!/bin/bash
# Round 6: kernel trace of the N = 1 mailbox step at 256 Ki and 1 Mi messages (actor / arrival).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6k1}
for m in 262144 1048576; do
  for sh in actor arrival; do
    rm -rf gpurun_out/${TAG}_${m}_$sh
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_${m}_$sh -o k --output-format csv -- \
      python3 bench.py --msgs-per-gpu $m --sharding $sh --steps 20 --warmup 5 --rtt-calls 0 --no-secondary \
      > gpurun_out/${TAG}_${m}_$sh.json 2> gpurun_out/${TAG}_${m}_$sh.err || exit 1
  done
done
