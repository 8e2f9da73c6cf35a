#!/bin/bash
# Round-5 session V: one-step kernel timelines (gaps included) of the N = 1 lines:
# the headline (8 Mi), config 2 (1 Mi) and SeqFold, from rocprofv3 kernel traces.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5v}
B="bench.py --steps 12 --warmup 4 --rtt-calls 0 --no-secondary"
run() {  # name, extra args
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_$1 -o tr -- python3 $B ${@:2} \
    > gpurun_out/${TAG}_$1.log 2>&1 || { tail -20 gpurun_out/${TAG}_$1.log; exit 3; }
  F=$(ls gpurun_out/${TAG}_$1/*/tr_kernel_trace.csv 2>/dev/null || ls gpurun_out/${TAG}_$1/tr_kernel_trace.csv)
  echo "== $1"
  python3 tools/timeline.py $F gen_requests all > gpurun_out/${TAG}_$1_timeline.txt && cat gpurun_out/${TAG}_$1_timeline.txt
}
run head && run c2 --msgs-per-gpu 1048576 && run seq --method seqfold --mailbox-shards 256
