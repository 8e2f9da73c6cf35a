#!/bin/bash
# Round-4: where the bench's 1 Mi mailbox step goes -- kernel trace of the bench at
# --msgs-per-gpu 1 Mi (graph replays, generator included), and the fused kernel at 1 Mi.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4c2}
rm -rf gpurun_out/${TAG}_bench1m
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_bench1m -o prof -- \
  python3 bench.py --msgs-per-gpu 1048576 --steps 16 --warmup 4 --no-secondary > gpurun_out/${TAG}_bench1m.log 2>&1 || exit 1
timeout -k 10 200 python3 bench.py --msgs-per-gpu 1048576 --steps 40 --warmup 8 --no-secondary > gpurun_out/${TAG}_b1m.json 2>/dev/null || exit 2
PTYPE_MBOX_FUSED=1 timeout -k 10 200 python3 bench.py --msgs-per-gpu 1048576 --steps 40 --warmup 8 --no-secondary > gpurun_out/${TAG}_b1m_fused.json 2>/dev/null || exit 3
timeout -k 10 200 python3 bench.py --msgs-per-gpu 1048576 --steps 40 --warmup 8 --no-secondary --graph off > gpurun_out/${TAG}_b1m_eager.json 2>/dev/null || exit 4
for f in b1m b1m_fused b1m_eager; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e9,2), 'G msg/s', round(d['ms_per_step']*1e3,1), 'us/step', d['config'].get('hip_graph'), d['config'].get('steps_per_graph'))" gpurun_out/${TAG}_$f.json $f; done
