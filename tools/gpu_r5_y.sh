#!/bin/bash
# Round-5 session Y: grouped run reservations in the one-pass mailbox sort (tile t
# reserves on group t % 8's counters, in its 1/8 segment of each shard's room;
# PTYPE_MBOX_RESV_GROUPS=1: one counter per shard).  Mailbox tests both ways, then
# the headline (8 Mi) and config 2 (1 Mi) lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5y}
val() { python3 -c "import json; d=[json.loads(x) for x in open('$1') if x.startswith('{')][-1]; print(round(d['value']/1e9,3), round(d['ms_per_step'],4))"; }
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mailbox_gpu.py \
  > gpurun_out/${TAG}_tests_g8.txt 2>&1 || { tail -30 gpurun_out/${TAG}_tests_g8.txt; exit 3; }
tail -1 gpurun_out/${TAG}_tests_g8.txt
H="python3 bench.py --steps 50 --warmup 10 --rtt-calls 0 --no-secondary"
C="python3 bench.py --msgs-per-gpu 1048576 --delivery mailbox --sharding actor --steps 200 --warmup 20 --rtt-calls 0 --no-secondary"
for V in 8 1 8 1; do
  F="gpurun_out/${TAG}_head_g${V}_$RANDOM.json"
  PTYPE_MBOX_RESV_GROUPS=$V timeout -k 10 200 $H > $F 2>$F.err || exit 3
  echo "8Mi groups=$V $(val $F)"
done
for V in 8 1 8 1; do
  F="gpurun_out/${TAG}_c2_g${V}_$RANDOM.json"
  PTYPE_MBOX_RESV_GROUPS=$V timeout -k 10 200 $C > $F 2>$F.err || exit 3
  echo "1Mi groups=$V $(val $F)"
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o g8 -- \
  $H > gpurun_out/${TAG}_prof.log 2>&1 || exit 3
F=$(find gpurun_out/${TAG}_prof -name 'g8_kernel_stats.csv' | head -1)
cut -d, -f1-4 $F | sed -n 1,5p
