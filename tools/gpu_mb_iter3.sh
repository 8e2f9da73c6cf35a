#!/bin/bash
# One-pass (look-back) sort: mailbox tests, variants, two-pass A/B, headline bench, profiles.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-mbiter}
timeout -k 10 300 python -u -m pytest tests/test_mailbox_gpu.py -x -q --timeout 60 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -5 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for V in actor seqfold; do
  timeout -k 10 120 python3 tools/mb_variant.py $V 20 || exit $?
  PTYPE_MBOX_SORT=twopass timeout -k 10 120 python3 tools/mb_variant.py $V 20 || exit $?
done
MB_M=1048576 timeout -k 10 120 python3 tools/mb_variant.py actor 50 || exit $?
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --rtt-calls 0 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); print('bench', round(d['value']/1e9,2), 'G msg/s', round(d['ms_per_step'],4), 'ms')
for k,v in d['secondaries'].items(): print('  ', k, round(v['value']/1e9,2), round(v['ms_per_step'],4))" gpurun_out/${TAG}_bench.json
for V in actor seqfold; do
  rm -rf gpurun_out/${TAG}_prof_$V
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_$V -o prof -- python3 tools/mb_variant.py $V 5 > gpurun_out/${TAG}_prof_$V.log 2>&1 || exit $?
done
