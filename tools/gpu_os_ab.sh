#!/bin/bash
# One-pass sorts A/B (group look-back): tests, mailbox one/two-pass, loopback-8 one/two-pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-osab}
timeout -k 10 500 python -u -m pytest tests/test_mailbox_gpu.py tests/test_sorted_exchange_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for E in PTYPE_MBOX_SORT=onepass PTYPE_MBOX_SORT=twopass; do
    echo -n "$E: "; env $E timeout -k 10 120 python3 tools/mb_variant.py actor 20 || exit $?
  done
  for E in twopass onepass; do
    PTYPE_SX_SORT=$E timeout -k 10 200 python3 bench.py --loopback 8 --steps 10 --warmup 4 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_loop8_$E.json 2> gpurun_out/${TAG}_loop8_$E.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('loop8', sys.argv[2], round(d['ms_per_step'],4), 'ms/step')" gpurun_out/${TAG}_loop8_$E.json $E
  done
done
rm -rf gpurun_out/${TAG}_prof_loop8
PTYPE_SX_SORT=onepass timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_loop8 -o prof -- python3 bench.py --loopback 8 --steps 6 --warmup 4 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_prof_loop8.log 2>&1 || exit $?
timeout -k 10 120 python3 tools/send_host_time.py > gpurun_out/${TAG}_send_host_time.json 2>&1 || exit $?
head -c 300 gpurun_out/${TAG}_send_host_time.json; echo
rm -rf gpurun_out/${TAG}_prof_actor
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_actor -o prof -- python3 tools/mb_variant.py actor 5 > gpurun_out/${TAG}_prof_actor.log 2>&1 || exit $?
