#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/packed_route_bench.py > gpurun_out/packed_route.jsonl 2> gpurun_out/packed_route.err || { echo "FAILED"; tail -10 gpurun_out/packed_route.err; exit 1; }
cat gpurun_out/packed_route.jsonl
