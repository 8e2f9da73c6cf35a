#!/bin/bash
# Round 6: loopback-8 step vs batch size with the sorted exchange's collectives on the
# engine's comm stream (events between the streams) or on the caller's stream (tune
# sx_comm_cs=1: no cross-stream hand-offs, copies serialised with the compute).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6cs}
for m in 262144 1048576 2097152 4194304 8388608; do
  for c in 0 1; do
    PTYPE_TUNE=sx_comm_cs=$c timeout -k 10 200 python3 bench.py --loopback 8 --msgs-per-gpu $m --steps 20 --warmup 5 \
      --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_${m}_$c.json 2> gpurun_out/${TAG}_${m}_$c.err || { tail -5 gpurun_out/${TAG}_${m}_$c.err; exit 1; }
    python3 - "$m" "$c" gpurun_out/${TAG}_${m}_$c.json <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[3]) if x.startswith("{")][-1])
h = d["config"].get("host_split") or {}
print("M=%8s cs=%s  %.4f ms/step  %6.2f G msg/s  enqueue %6.1f us  wait %6.1f us" % (sys.argv[1], sys.argv[2], d["ms_per_step"], d["value"] / 1e9, h.get("enqueue_us_per_send", -1), h.get("agreement_wait_us_per_send", -1)))
PY
  done
done
