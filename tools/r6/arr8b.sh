#!/bin/bash
# Round 6: mailbox GPU tests, then the stateless Send by size: actor-sharded sort vs arrival
# rings in one launch (per-wave 8-B records), alternated, two rounds at 8 Mi.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6a8b}
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/ -m gpu -k "mailbox or arrival" \
  > gpurun_out/${TAG}_tests.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/${TAG}_tests.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/${TAG}_tests.log | tail -1
for m in 1048576 8388608 8388608; do
  for sh in actor arrival; do
    PTYPE_TUNE=auto_arrival=0 timeout -k 10 200 python3 bench.py --msgs-per-gpu $m --sharding $sh --steps 20 --warmup 5 \
      --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_${m}_$sh.json 2> gpurun_out/${TAG}_${m}_$sh.err || { tail -5 gpurun_out/${TAG}_${m}_$sh.err; exit 1; }
    python3 - "$m" "$sh" gpurun_out/${TAG}_${m}_$sh.json <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[3]) if x.startswith("{")][-1])
print("M=%8s %-8s %.4f ms/step %6.2f G msg/s" % (sys.argv[1], sys.argv[2], d["ms_per_step"], d["value"] / 1e9))
PY
  done
done
