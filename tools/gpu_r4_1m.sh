#!/bin/bash
# Round-4: the 1 Mi mailbox Send (BASELINE config 2 size) by sort kernel, per-kernel
# stats; the headline bench with the defaults; the loopback-8 compute side (sorted
# exchange) uniform and Zipf(1.1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4m}
for E in onepass twopass; do
  rm -rf gpurun_out/${TAG}_1m_$E
  MB_M=1048576 PTYPE_MBOX_SORT=$E timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_1m_$E -o prof -- \
    python3 tools/mb_variant.py actor 20 > gpurun_out/${TAG}_1m_$E.log 2>&1 || exit 1
  echo -n "1Mi $E: "; MB_M=1048576 PTYPE_MBOX_SORT=$E timeout -k 10 100 python3 tools/mb_variant.py actor 50 || exit 2
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 3
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', round(d['value']/1e9,2), 'G msg/s', round(d['ms_per_step'],4), 'ms', {k: round(v.get('value',0)/1e9,2) for k,v in d.get('secondaries',{}).items() if isinstance(v, dict) and 'value' in v})" gpurun_out/${TAG}_bench.json
for Z in 0 1.1; do
  timeout -k 10 300 python3 bench.py --loopback 8 --zipf $Z --link-gbps 120 --steps 10 --warmup 5 --rtt-calls 0 --no-secondary \
    > gpurun_out/${TAG}_loop8_z$Z.json 2> gpurun_out/${TAG}_loop8_z$Z.err || exit 4
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('loop8 zipf', sys.argv[2], round(d['ms_per_step'],4), 'ms/step', d.get('wire', d.get('config',{}).get('wire')))" gpurun_out/${TAG}_loop8_z$Z.json $Z
done
