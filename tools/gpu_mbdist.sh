#!/bin/bash
# Mailbox delivery on receipt: GPU tests + the RCCL path (--force-dist) with
# direct vs mailbox delivery, and the R = 8 loopback pipeline both ways.
set -o pipefail
TAG=${1:-mbd}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mailbox_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/mbd_$TAG.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/mbd_$TAG.log; exit 1; }
tail -2 gpurun_out/mbd_$TAG.log
OUT=gpurun_out/mbd_$TAG.jsonl
: > $OUT
for D in direct mailbox; do
  timeout -k 10 200 python bench.py --force-dist --steps 10 --warmup 3 --rtt-calls 0 --no-secondary --delivery $D >> $OUT 2> gpurun_out/mbd_${TAG}_$D.err || { echo "FORCE-DIST $D FAILED"; tail -20 gpurun_out/mbd_${TAG}_$D.err; exit 1; }
  timeout -k 10 200 python bench.py --loopback 8 --link-gbps 120 --steps 10 --warmup 3 --rtt-calls 0 --no-secondary --delivery $D >> $OUT 2>> gpurun_out/mbd_${TAG}_$D.err || { echo "LOOPBACK $D FAILED"; tail -20 gpurun_out/mbd_${TAG}_$D.err; exit 1; }
done
python - "$OUT" <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    if not ln.startswith("{"):
        continue  # RCCL's version banner goes to stdout
    d = json.loads(ln); c = d["config"]
    print(c["parallelism"][:60], c.get("loopback_ranks"), c["delivery"], c["wire"], "ms/step %.3f" % d["ms_per_step"], "G msg/s %.1f" % (d["value"] / 1e9))
PY
