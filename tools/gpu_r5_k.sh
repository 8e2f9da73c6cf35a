#!/bin/bash
# Round-5 session K (round-end rehearsal): smoke(), the whole GPU suite, then the
# driver's default bench line with every secondary.  Every step under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5k}
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/${TAG}_smoke.log
[ $rc -eq 0 ] || exit 2
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/${TAG}_suite.log 2>&1; rc=$?
echo "suite rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/${TAG}_suite.log | tail -5
[ $rc -le 1 ] || exit 3
timeout -k 10 600 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err; rc=$?
echo "bench rc=$rc"
TAG=$TAG python3 - <<'PY'
import json, os, sys
l = [x for x in open(f"gpurun_out/{os.environ['TAG']}_bench.json") if x.startswith("{")][-1]
d = json.loads(l)
print("headline", round(d["value"] / 1e9, 2), "G", round(d["ms_per_step"], 4), "ms")
for k, v in d.get("secondaries", {}).items():
    if isinstance(v, dict):
        print(" ", k, {kk: (round(vv / 1e9, 2) if kk == "value" else vv) for kk, vv in v.items()
                        if kk in ("value", "ms_per_step", "error")})
PY
