#!/bin/bash
# complete_packed items per thread (PTYPE_COMP_U) on the loopback-8 step: step time + kernel time.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4cu}
for U in 4 8 2; do
  rm -rf gpurun_out/${TAG}_$U
  PTYPE_COMP_U=$U timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_$U -o prof -- \
    python3 bench.py --loopback 8 --steps 6 --warmup 4 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_$U.log 2>&1 || exit 1
  echo -n "U=$U complete: "; python3 tools/rocpd_summary.py gpurun_out/${TAG}_$U/prof_results.db | grep complete_packed | awk '{print $4}'
  PTYPE_COMP_U=$U timeout -k 10 200 python3 bench.py --loopback 8 --steps 10 --warmup 5 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_b$U.json 2>/dev/null || exit 2
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('   step', round(d['ms_per_step'],4), 'ms')" gpurun_out/${TAG}_b$U.json
done
