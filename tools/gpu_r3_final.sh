#!/bin/bash
# Round-3 closing session on one MI355X: every GPU test, smoke(), the N=1 bench
# (driver arguments), mailbox A/Bs, loopback-8, kernel stats and PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-fin}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/${TAG}_gpu_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/${TAG}_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); print('bench', round(d['value']/1e9,2), 'G msg/s', round(d['ms_per_step'],4), 'ms, p50', d['p50_rtt_us'])
for k,v in d['secondaries'].items(): print('  ', k, round(v['value']/1e9,2), round(v['ms_per_step'],4))" gpurun_out/${TAG}_bench.json
for E in PTYPE_MBOX_SORT=onepass PTYPE_MBOX_SORT=twopass; do
  echo -n "$E: "; env $E timeout -k 10 120 python3 tools/mb_variant.py actor 20 || exit $?
done
timeout -k 10 200 python3 bench.py --loopback 8 --steps 10 --warmup 4 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_loop8.json 2> gpurun_out/${TAG}_loop8.err || exit $?
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('loop8', round(d['ms_per_step'],4), 'ms/step')" gpurun_out/${TAG}_loop8.json
rm -rf gpurun_out/${TAG}_prof
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o prof -- python3 bench.py --steps 10 --warmup 2 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
for V in arrival seqfold; do
  rm -rf gpurun_out/${TAG}_prof_$V
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_$V -o prof -- python3 tools/mb_variant.py $V 5 > gpurun_out/${TAG}_prof_$V.log 2>&1 || exit $?
done
for C in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/${TAG}_pmc_$C
  timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/${TAG}_pmc_$C -o pmc --output-format csv -- python3 tools/mb_variant.py actor 3 > gpurun_out/${TAG}_pmc_$C.log 2>&1 || exit $?
done
python3 tools/pmc_table.py gpurun_out/${TAG}_pmc_FETCH_SIZE gpurun_out/${TAG}_pmc_WRITE_SIZE > gpurun_out/${TAG}_pmc.txt 2>&1; cat gpurun_out/${TAG}_pmc.txt
