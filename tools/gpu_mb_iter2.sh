#!/bin/bash
# Mailbox iteration, short form: the mailbox tests, the Send variants, and the
# N=1 headline at two warm-up lengths (first-measurement effects).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-mbiter}
timeout -k 10 400 python -u -m pytest tests/test_mailbox_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for V in actor arrival seqfold; do
  timeout -k 10 120 python3 tools/mb_variant.py $V 20 || exit $?
done
MB_M=1048576 timeout -k 10 120 python3 tools/mb_variant.py actor 50 || exit $?
MB_M=1048576 timeout -k 10 120 python3 tools/mb_variant.py arrival 50 || exit $?
for W in 5 40; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup $W --no-secondary --rtt-calls 0 > gpurun_out/${TAG}_bench_w$W.json 2> gpurun_out/${TAG}_bench_w$W.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench warmup', sys.argv[2], round(d['value']/1e9,2), 'G msg/s', round(d['ms_per_step'],4), 'ms')" gpurun_out/${TAG}_bench_w$W.json $W
done
rm -rf gpurun_out/${TAG}_prof_arrival
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_arrival -o prof -- python3 tools/mb_variant.py arrival 5 > gpurun_out/${TAG}_prof_arrival.log 2>&1 || exit $?
