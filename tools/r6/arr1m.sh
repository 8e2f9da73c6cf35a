#!/bin/bash
# Round 6: mailbox GPU tests, then the 1 Mi / 256 Ki stateless Send: fused arrival (default),
# two-kernel arrival (tune mbox_fused=0) and the actor-sharded fused sort (auto_arrival=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6a1}
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/ -m gpu -k "mailbox or arrival" \
  > gpurun_out/${TAG}_tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/${TAG}_tests.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/${TAG}_tests.log | tail -1
run() {  # label, tune, bench args
  local lab=$1 tn=$2; shift 2
  PTYPE_TUNE=$tn timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --rtt-calls 0 --no-secondary "$@" \
    > gpurun_out/${TAG}_$lab.json 2> gpurun_out/${TAG}_$lab.err || { tail -5 gpurun_out/${TAG}_$lab.err; exit 1; }
  python3 - "$lab" gpurun_out/${TAG}_$lab.json <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[2]) if x.startswith("{")][-1])
print("%-18s %.4f ms/step %6.2f G msg/s" % (sys.argv[1], d["ms_per_step"], d["value"] / 1e9))
PY
}
for rep in 1 2; do
  for m in 1048576 262144; do
    run ${m}_fused_$rep "" --msgs-per-gpu $m
    run ${m}_twok_$rep mbox_fused=0 --msgs-per-gpu $m --sharding arrival
    run ${m}_actor_$rep auto_arrival=0 --msgs-per-gpu $m
  done
done
