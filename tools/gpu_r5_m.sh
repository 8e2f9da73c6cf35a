#!/bin/bash
# Round-5 session M: the relay / peer-lane tests with their measurements printed
# (-s), then the N = 1 bench line with every secondary and the loopback-8 line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5m}
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 280 --timeout-method thread tests/test_xcall_gpu.py \
  > gpurun_out/${TAG}_xcall.log 2>&1; rc=$?
echo "xcall rc=$rc"; grep -E "passed|failed|FAILED|^relay|^duplex|^coord|p50" gpurun_out/${TAG}_xcall.log | cut -c1-400 | tail -12
[ $rc -eq 0 ] || exit 2
timeout -k 10 600 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 3
python3 - <<'PY'
import json
l = [x for x in open("gpurun_out/r5m_bench.json") if x.startswith("{")][-1]
d = json.loads(l)
print("headline", round(d["value"] / 1e9, 2), "G", round(d["ms_per_step"], 4), "ms")
for k, v in d.get("secondaries", {}).items():
    if isinstance(v, dict) and "value" in v:
        print(" ", k, round(v["value"] / 1e9, 2), round(v.get("ms_per_step", 0), 4))
PY
timeout -k 10 200 python3 bench.py --loopback 8 --steps 20 --warmup 5 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_l8.json 2>gpurun_out/${TAG}_l8.err || exit 4
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_l8.json')); print('l8', round(d['value']/1e9,2), round(d['ms_per_step'],4), d['config'].get('host_split'))"
