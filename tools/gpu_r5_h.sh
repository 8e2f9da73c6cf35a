#!/bin/bash
# Round-5 session H: the binned ordered drain's super-window (PTYPE_ORD_BIN_ROUNDS) against
# the windowed default, the 1 Mi arrival-sharded step's kernels.  Output to files (no pipes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5h}
val() { python3 -c "import json; d=json.load(open('$1')); print(round(d['value']/1e9,3), round(d['ms_per_step'],4))"; }
for K in "X=0" "PTYPE_ORD_DRAIN=bin PTYPE_ORD_BIN_ROUNDS=1" "PTYPE_ORD_DRAIN=bin PTYPE_ORD_BIN_ROUNDS=2" "PTYPE_ORD_DRAIN=bin PTYPE_ORD_BIN_ROUNDS=4"; do
  F="gpurun_out/${TAG}_seq_$(echo $K | tr ' =' '__').json"
  env $K timeout -k 10 200 python3 bench.py --no-secondary --rtt-calls 0 --method seqfold > $F 2>$F.err || exit 3
  echo "seqfold [$K] $(val $F)"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_arr -o prof -- \
  python3 bench.py --msgs-per-gpu 1048576 --sharding arrival --steps 8 --warmup 4 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_arr.log 2>&1 || exit 4
python3 tools/kstats.py gpurun_out/${TAG}_arr/prof_kernel_stats.csv > gpurun_out/${TAG}_arr.txt && sed -n 1,6p gpurun_out/${TAG}_arr.txt
