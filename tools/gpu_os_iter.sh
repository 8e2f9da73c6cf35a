#!/bin/bash
# One-pass look-back sorts (mailbox + sorted exchange): GPU tests, A/B against the
# two-pass kernels, N=1 bench, loopback-8, per-kernel profiles.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-os}
timeout -k 10 400 python -u -m pytest tests/test_mailbox_gpu.py tests/test_sorted_exchange_gpu.py -x -q --timeout 60 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -5 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for V in actor seqfold; do
  timeout -k 10 120 python3 tools/mb_variant.py $V 20 || exit $?
  PTYPE_MBOX_SORT=twopass timeout -k 10 120 python3 tools/mb_variant.py $V 20 || exit $?
done
MB_M=1048576 timeout -k 10 120 python3 tools/mb_variant.py actor 50 || exit $?
for E in onepass twopass; do
  PTYPE_SX_SORT=$E timeout -k 10 200 python3 bench.py --loopback 8 --steps 10 --warmup 4 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_loop8_$E.json 2> gpurun_out/${TAG}_loop8_$E.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('loop8', sys.argv[2], round(d['ms_per_step'],4), 'ms/step')" gpurun_out/${TAG}_loop8_$E.json $E
done
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --rtt-calls 0 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); print('bench', round(d['value']/1e9,2), 'G msg/s', round(d['ms_per_step'],4), 'ms')
for k,v in d['secondaries'].items(): print('  ', k, round(v['value']/1e9,2), round(v['ms_per_step'],4))" gpurun_out/${TAG}_bench.json
for V in actor seqfold; do
  rm -rf gpurun_out/${TAG}_prof_$V
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_$V -o prof -- python3 tools/mb_variant.py $V 5 > gpurun_out/${TAG}_prof_$V.log 2>&1 || exit $?
done
for E in onepass twopass; do
  rm -rf gpurun_out/${TAG}_prof_loop8_$E
  PTYPE_SX_SORT=$E timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_loop8_$E -o prof -- python3 bench.py --loopback 8 --steps 6 --warmup 4 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_prof_loop8_$E.log 2>&1 || exit $?
done
