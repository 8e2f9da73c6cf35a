#!/bin/bash
# Dispatcher polling knobs with the request ring in device memory: p50 RTT per setting.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/poll_sweep.jsonl; : > $out
for cfg in "64 0 1" "64 1 1" "64 0 0" "64 1 0" "16 0 1" "64 0 1" "64 1 1"; do
  set -- $cfg
  PTYPE_POLL_LANES=$1 PTYPE_POLL_FULL=$2 PTYPE_POLL_SLEEP=$3 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --rtt-calls 20000 > gpurun_out/ps.json 2> gpurun_out/ps.err || { echo "FAILED $cfg"; tail -10 gpurun_out/ps.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/ps.json').read().strip().splitlines()[-1]); print(json.dumps({'lanes': $1, 'full': $2, 'sleep': $3, 'ring': d.get('rtt_request_ring'), 'p50_us': round(d['p50_rtt_us'], 3)}))" | tee -a $out
done
