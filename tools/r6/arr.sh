#!/bin/bash
# Round 6: N = 1 mailbox Send, actor-sharded (sort) vs arrival-sharded rings, by batch size.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6ar}
for m in 262144 1048576 2097152 4194304; do
  for sh in actor arrival; do
    timeout -k 10 200 python3 bench.py --msgs-per-gpu $m --sharding $sh --steps 20 --warmup 5 --rtt-calls 0 --no-secondary \
      > gpurun_out/${TAG}_${m}_$sh.json 2> gpurun_out/${TAG}_${m}_$sh.err || { tail -5 gpurun_out/${TAG}_${m}_$sh.err; exit 1; }
    python3 - "$m" "$sh" gpurun_out/${TAG}_${m}_$sh.json <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[3]) if x.startswith("{")][-1])
print("M=%8s %-8s %.4f ms/step %6.2f G msg/s" % (sys.argv[1], sys.argv[2], d["ms_per_step"], d["value"] / 1e9))
PY
  done
done
