#!/bin/bash
# Kernel breakdown of the optimus fan-out: 1 GPU and the 8-rank loopback step.
# usage (under gpurun, repo root): tools/gpu_optimus_prof.sh TAG
set -o pipefail
TAG=${1:-op}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for L in 0 8; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/opprof_${TAG}_$L -o run --output-format csv -- python tools/bench_suite.py optimus --loopback $L --steps 5 > gpurun_out/opprof_${TAG}_$L.log 2>&1 || { echo "PROF $L FAILED"; tail -20 gpurun_out/opprof_${TAG}_$L.log; exit 1; }
  echo "== loopback $L"; tail -1 gpurun_out/opprof_${TAG}_$L.log | cut -c1-300
  python tools/kstats.py gpurun_out/opprof_${TAG}_$L 2>&1 | head -14
done
