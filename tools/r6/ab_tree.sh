#!/bin/bash
# In-box A/B of the working tree against a copy of the previous build in ./abold
# (bench.py + the package with its built modules): alternated headline runs.
# Usage: ab_tree.sh TAG [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
TAG=$1; shift
for rep in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then B=abold/bench.py; else B=bench.py; fi
    timeout -k 10 200 python3 $B --no-secondary --rtt-calls 0 "$@" > gpurun_out/${TAG}_${v}_$rep.json 2> gpurun_out/${TAG}_${v}_$rep.err || { tail -5 gpurun_out/${TAG}_${v}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.loads([x for x in open('gpurun_out/${TAG}_${v}_$rep.json') if x.startswith('{')][-1]); print('$v', round(d['ms_per_step'],4), round(d['value']/1e9,2))"
  done
done
