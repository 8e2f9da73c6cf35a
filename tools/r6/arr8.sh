#!/bin/bash
# Round 6: 8 Mi stateless mailbox Send -- actor-sharded sort vs arrival rings (two kernels)
# vs arrival rings in one launch (tune mbox_fused=1), alternated, two rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6a8}
for rep in 1 2; do
  for v in actor arrival arrivalfused; do
    sh=actor; tn=""
    [ $v = arrival ] && sh=arrival
    [ $v = arrivalfused ] && sh=arrival && tn="mbox_fused=1"
    PTYPE_TUNE=$tn timeout -k 10 200 python3 bench.py --sharding $sh --steps 20 --warmup 5 --rtt-calls 0 --no-secondary \
      > gpurun_out/${TAG}_${v}_$rep.json 2> gpurun_out/${TAG}_${v}_$rep.err || { tail -5 gpurun_out/${TAG}_${v}_$rep.err; exit 1; }
    python3 - "$v" gpurun_out/${TAG}_${v}_$rep.json <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[2]) if x.startswith("{")][-1])
print("%-13s %.4f ms/step %6.2f G msg/s" % (sys.argv[1], d["ms_per_step"], d["value"] / 1e9))
PY
  done
done
