#!/bin/bash
# Sorted exchange GPU tests, then loopback-8 uniform and Zipf(1.1) with the link model:
# the exchange form each takes and its step time.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4l8c}
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_sorted_exchange_gpu.py > gpurun_out/${TAG}_tests.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_tests.log
for Z in 0 1.1; do
  timeout -k 10 300 python3 bench.py --loopback 8 --zipf $Z --link-gbps 120 --steps 10 --warmup 5 --rtt-calls 0 --no-secondary \
    > gpurun_out/${TAG}_z$Z.json 2>/dev/null || exit 2
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print('loop8 zipf', sys.argv[2], round(d['ms_per_step'],4), 'ms/step', c['exchange'], round(c['wire_bytes_per_msg'],2), 'B/msg', c.get('resend_rounds'))" gpurun_out/${TAG}_z$Z.json $Z
done
