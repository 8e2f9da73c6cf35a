#!/bin/bash
# Round-5 session W: config 2 (1 Mi messages) fused sort + drain with 2048-message
# tiles (PTYPE_MBOX_SK=4: 512 blocks, 2 per CU, 90 VGPRs) vs 4096 (default) and
# 1024 (SK=2); kernel stats of the SK=4 form.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5w}
val() { python3 -c "import json; d=[json.loads(x) for x in open('$1') if x.startswith('{')][-1]; print(round(d['value']/1e9,3), round(d['ms_per_step'],4))"; }
B="python3 bench.py --msgs-per-gpu 1048576 --delivery mailbox --sharding actor --steps 200 --warmup 20 --rtt-calls 0 --no-secondary"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mailbox_gpu.py \
  > gpurun_out/${TAG}_tests_default.txt 2>&1 || { tail -30 gpurun_out/${TAG}_tests_default.txt; exit 3; }
PTYPE_MBOX_SK=4 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_mailbox_gpu.py \
  > gpurun_out/${TAG}_tests_sk4.txt 2>&1 || { tail -30 gpurun_out/${TAG}_tests_sk4.txt; exit 3; }
tail -1 gpurun_out/${TAG}_tests_default.txt gpurun_out/${TAG}_tests_sk4.txt
for V in 8 4 2 8 4 2; do
  F="gpurun_out/${TAG}_c2_sk${V}_$RANDOM.json"
  PTYPE_MBOX_SK=$V timeout -k 10 200 $B > $F 2>$F.err || exit 3
  echo "1Mi sk=$V $(val $F)"
done
PTYPE_MBOX_SK=4 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o sk4 -- \
  $B > gpurun_out/${TAG}_prof.log 2>&1 || exit 3
F=$(find gpurun_out/${TAG}_prof -name 'sk4_kernel_stats.csv' | head -1)
cut -d, -f1-4 $F | sed -n 1,5p
# device-scope atomic throughput on the hot reservation counters
timeout -k 10 60 ./tools/atomic_contention_probe.bin > gpurun_out/${TAG}_atomics.jsonl || exit 3
cat gpurun_out/${TAG}_atomics.jsonl
