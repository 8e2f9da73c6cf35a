#!/bin/bash
# In-box A/B/C: ./abold (previous build), ./abnt1 (a second saved build) and the working
# tree, alternated.  Usage: ab3.sh TAG [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
TAG=$1; shift
for rep in 1 2 3; do
  for v in old nt1 new; do
    case $v in old) B=abold/bench.py;; nt1) B=abnt1/bench.py;; new) B=bench.py;; esac
    timeout -k 10 200 python3 $B --no-secondary --rtt-calls 0 "$@" > gpurun_out/${TAG}_${v}_$rep.json 2> gpurun_out/${TAG}_${v}_$rep.err || { tail -5 gpurun_out/${TAG}_${v}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.loads([x for x in open('gpurun_out/${TAG}_${v}_$rep.json') if x.startswith('{')][-1]); print('$v', round(d['ms_per_step'],4), round(d['value']/1e9,2))"
  done
done
