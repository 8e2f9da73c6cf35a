#!/bin/bash
# Round 6: mailbox GPU tests, then the fused arrival Send with 16-B vs 8-B records (tune
# mbox_rec8=0 / 1) at 1 Mi and 8 Mi, alternated, two rounds; and the actor sort at 8 Mi.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6a8c}
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
  run 1m_rec16_$rep mbox_rec8=0 --msgs-per-gpu 1048576
  run 1m_rec8_$rep mbox_rec8=1 --msgs-per-gpu 1048576
  run 8m_arr16_$rep mbox_rec8=0 --sharding arrival
  run 8m_arr8_$rep mbox_rec8=1 --sharding arrival
  run 8m_actor_$rep "" --sharding actor
done
