#!/bin/bash
# Exact-size exchange (counts all-to-all + grouped send/recv) vs padded all-to-all:
# wire-format / multi-rank GPU tests, then the R = 8 loopback step uniform and Zipf,
# with and without the link model, each exchange mode.
# usage (under gpurun, repo root): tools/gpu_exact.sh TAG
set -o pipefail
TAG=${1:-ex}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_packed_wire.py tests/test_engine_multirank_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ex_test_$TAG.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/ex_test_$TAG.log; exit 1; }
tail -1 gpurun_out/ex_test_$TAG.log
OUT=gpurun_out/ex_$TAG.jsonl
: > $OUT
for mode in exact padded; do
  for load in "--pregen" "--zipf 1.1"; do
    for link in 0 120; do
      PTYPE_EXCHANGE=$mode timeout -k 10 200 python bench.py --loopback 8 --steps 10 --warmup 3 --rtt-calls 0 --no-secondary --link-gbps $link $load >> $OUT 2>> gpurun_out/ex_$TAG.err || { echo "BENCH $mode $load $link FAILED"; tail -20 gpurun_out/ex_$TAG.err; exit 1; }
    done
  done
done
PTYPE_ADAPTIVE_C=force timeout -k 10 200 python bench.py --force-dist --steps 10 --warmup 3 --rtt-calls 0 >> $OUT 2>> gpurun_out/ex_$TAG.err || { echo "FORCE-DIST FAILED"; tail -20 gpurun_out/ex_$TAG.err; exit 1; }
python3 - "$OUT" <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    if ln.startswith("{"):
        d = json.loads(ln); c = d["config"]
        print(c.get("exchange"), c.get("load"), "link", c.get("link_gbps"), "ms/step %.3f" % d["ms_per_step"],
              "wire B/msg %.2f" % c.get("wire_bytes_per_msg", -1), c.get("parallelism"))
PY
