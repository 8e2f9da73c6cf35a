#!/bin/bash
# Round-5 session Q: the persistent prefetching mailbox sort at 8 Mi (bench-verified replies).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5q}
val() { python3 -c "import json; d=[json.loads(x) for x in open('$1') if x.startswith('{')][-1]; print(round(d['value']/1e9,3), round(d['ms_per_step'],4))"; }
for K in "X=0" "PTYPE_MBOX_PERSIST=1" "PTYPE_MBOX_PERSIST=2" "X=1" "PTYPE_MBOX_PERSIST=1"; do
  F="gpurun_out/${TAG}_8m_$(echo $K | tr ' =' '__')_$RANDOM.json"
  env $K timeout -k 10 200 python3 bench.py --no-secondary --rtt-calls 0 > $F 2>$F.err || exit 3
  echo "8m [$K] $(val $F)"
done
PTYPE_MBOX_PERSIST=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_p -o prof -- \
  python3 bench.py --steps 8 --warmup 4 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_p.log 2>&1 || exit 4
python3 tools/kstats.py gpurun_out/${TAG}_p/prof_kernel_stats.csv > gpurun_out/${TAG}_p.txt && sed -n 1,5p gpurun_out/${TAG}_p.txt
