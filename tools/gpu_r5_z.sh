#!/bin/bash
# Round-5 session Z: rank byte gathers (route mode 3) in the N = 1 stateless mailbox
# Send -- mailbox tests, then the headline (8 Mi) and config 2 (1 Mi) lines with
# and without (PTYPE_MBOX_RANK_TABLE=0), and kernel stats of the new default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5z}
val() { python3 -c "import json; d=[json.loads(x) for x in open('$1') if x.startswith('{')][-1]; print(round(d['value']/1e9,3), round(d['ms_per_step'],4), d['config'].get('registry_lookup', '')[:24])"; }
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mailbox_gpu.py \
  > gpurun_out/${TAG}_tests.txt 2>&1 || { tail -30 gpurun_out/${TAG}_tests.txt; exit 3; }
tail -1 gpurun_out/${TAG}_tests.txt
H="python3 bench.py --steps 50 --warmup 10 --rtt-calls 0 --no-secondary"
C="python3 bench.py --msgs-per-gpu 1048576 --delivery mailbox --sharding actor --steps 200 --warmup 20 --rtt-calls 0 --no-secondary"
for V in 1 0 1 0; do
  F="gpurun_out/${TAG}_head_rt${V}_$RANDOM.json"
  PTYPE_MBOX_RANK_TABLE=$V timeout -k 10 200 $H > $F 2>$F.err || exit 3
  echo "8Mi rank_table=$V $(val $F)"
done
for V in 1 0 1 0; do
  F="gpurun_out/${TAG}_c2_rt${V}_$RANDOM.json"
  PTYPE_MBOX_RANK_TABLE=$V timeout -k 10 200 $C > $F 2>$F.err || exit 3
  echo "1Mi rank_table=$V $(val $F)"
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o rt -- \
  $H > gpurun_out/${TAG}_prof.log 2>&1 || exit 3
F=$(find gpurun_out/${TAG}_prof -name 'rt_kernel_stats.csv' | head -1)
cp $F gpurun_out/${TAG}_head_kernel_stats.csv
cut -d, -f1-4 $F | sed -n 1,5p
