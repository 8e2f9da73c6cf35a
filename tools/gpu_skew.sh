#!/bin/bash
# Skew + snapshot round: engine / mailbox / kernel GPU tests, then
#   * the R = 8 pipeline on one GPU (FakeComm loopback, xGMI-like link model):
#     uniform vs Zipf(1.1) load, both pre-generated, adaptive slot capacity on,
#     and Zipf with the static capacity (PTYPE_ADAPTIVE_C=0) for the re-send rounds;
#   * the headline N=1 bench; the 1M-actor registry stress with the snapshot.
# usage (under gpurun, repo root): tools/gpu_skew.sh TAG
set -o pipefail
TAG=${1:-skew}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_engine_multirank_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/skewtest_$TAG.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/skewtest_$TAG.log; exit 1; }
tail -2 gpurun_out/skewtest_$TAG.log
OUT=gpurun_out/skew_$TAG.jsonl
: > $OUT
COMMON="--loopback 8 --link-gbps 120 --steps 10 --warmup 3 --rtt-calls 0 --no-secondary"
timeout -k 10 200 python bench.py $COMMON --pregen >> $OUT 2> gpurun_out/skew_$TAG.err || { echo "UNIFORM FAILED"; tail -20 gpurun_out/skew_$TAG.err; exit 1; }
timeout -k 10 200 python bench.py $COMMON --zipf 1.1 >> $OUT 2>> gpurun_out/skew_$TAG.err || { echo "ZIPF FAILED"; tail -20 gpurun_out/skew_$TAG.err; exit 1; }
PTYPE_ADAPTIVE_C=0 timeout -k 10 200 python bench.py $COMMON --zipf 1.1 >> $OUT 2>> gpurun_out/skew_$TAG.err || { echo "ZIPF STATIC FAILED"; tail -20 gpurun_out/skew_$TAG.err; exit 1; }
PTYPE_ADAPTIVE_C=0 timeout -k 10 200 python bench.py $COMMON --pregen >> $OUT 2>> gpurun_out/skew_$TAG.err || { echo "UNIFORM STATIC FAILED"; tail -20 gpurun_out/skew_$TAG.err; exit 1; }
python - "$OUT" <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    if not ln.startswith("{"):
        continue
    d = json.loads(ln); c = d["config"]
    print(c.get("load"), "C", c.get("slot_capacity"), "/", c.get("slot_capacity_alloc"), "static", c.get("slot_capacity_static"),
          "resends", c.get("resend_rounds"), "ms/step %.3f" % d["ms_per_step"], "G msg/s %.1f" % (d["value"] / 1e9))
PY
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "BENCH FAILED"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 300 python tools/bench_suite.py registry --actors 1048576 > gpurun_out/registry_$TAG.json 2> gpurun_out/registry_$TAG.err || { echo "REGISTRY FAILED"; tail -20 gpurun_out/registry_$TAG.err; exit 1; }
cat gpurun_out/registry_$TAG.json
