#!/bin/bash
# DRAM bytes per kernel on the RCCL path (--force-dist, wire v3), one counter per pass.
# Event hand-offs: with the default stream wait-value hand-offs a --pmc pass hung silently
# (observed); with PTYPE_STREAM_SYNC=events it completes in seconds.
# usage (under gpurun): bash tools/gpu_pmc_dist.sh TAG
set -o pipefail
TAG=${1:-pmcd}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for C in FETCH_SIZE WRITE_SIZE; do
  PTYPE_STREAM_SYNC=events timeout -k 10 150 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmcd_${TAG}_$C -o pmc --output-format csv -- python bench.py --force-dist --steps 3 --warmup 1 --rtt-calls 0 > gpurun_out/pmcd_${TAG}_$C.log 2>&1 || { echo "PMC dist $C FAILED"; tail -5 gpurun_out/pmcd_${TAG}_$C.log; exit 1; }
done
python tools/pmc_summary.py gpurun_out/pmcd_${TAG}_FETCH_SIZE gpurun_out/pmcd_${TAG}_WRITE_SIZE | tee gpurun_out/pmcd_${TAG}_summary.txt
