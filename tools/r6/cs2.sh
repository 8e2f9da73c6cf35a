#!/bin/bash
# Round 6: small Sends on the caller's stream -- the N > 1 GPU tests, then loopback-8 at
# 256 Ki .. 8 Mi messages per rank (default policy) and the 8 Mi / 1 Mi lines again.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6c2}
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_sorted_exchange_gpu.py \
  tests/test_ipc_comm_gpu.py tests/test_elastic_gpu.py tests/test_elastic_ipc_gpu.py tests/test_engine_multirank_gpu.py \
  tests/test_bench.py -m gpu -k "not multi_gpu" > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
grep -E "passed|failed|FAILED" gpurun_out/${TAG}_tests.log | tail -5
[ $rc -eq 0 ] || exit 2
for m in 262144 1048576 2097152 8388608; do
  timeout -k 10 200 python3 bench.py --loopback 8 --msgs-per-gpu $m --steps 20 --warmup 5 --rtt-calls 0 --no-secondary \
    > gpurun_out/${TAG}_$m.json 2> gpurun_out/${TAG}_$m.err || { tail -5 gpurun_out/${TAG}_$m.err; exit 3; }
  python3 - "$m" gpurun_out/${TAG}_$m.json <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[2]) if x.startswith("{")][-1])
h = d["config"].get("host_split") or {}
print("M=%8s %.4f ms/step %6.2f G msg/s enqueue %6.1f us wait %6.1f us" % (sys.argv[1], d["ms_per_step"], d["value"] / 1e9, h.get("enqueue_us_per_send", -1), h.get("agreement_wait_us_per_send", -1)))
PY
done
