#!/bin/bash
# Round-5 session X: device-scope atomic throughput with the blocks spread over
# counter sets (tools/atomic_contention_probe.hip).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
TAG=${1:-r5x}
timeout -k 10 60 ./tools/atomic_contention_probe.bin > gpurun_out/${TAG}_atomics.jsonl || exit 3
cat gpurun_out/${TAG}_atomics.jsonl
