#!/bin/bash
# Round-5 session B: the GPU tests touched this round (one pytest process), a
# loopback-8 knob sweep (bench lines only), the N=1 bench with and without the
# pipelined generator, and kernel-stats CSVs.  Each GPU step under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5b}
timeout -k 10 900 python -u -m pytest -v --timeout 240 --timeout-method thread \
  tests/test_ipc_comm_gpu.py tests/test_xcall_gpu.py tests/test_shm_rpc_gpu.py tests/test_elastic_ipc_gpu.py \
  > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/${TAG}_tests.log | tail -30
[ $rc -le 1 ] || exit $rc
L8="python3 bench.py --loopback 8 --steps 20 --warmup 5 --rtt-calls 0 --no-secondary"
i=0
for K in "" "PTYPE_SX_OCC8=1" "PTYPE_COMP_U=2" "PTYPE_SX_DRAIN_BLOCKS=4096" "PTYPE_SX_DRAIN_PER=512" "CHUNKS1"; do
  i=$((i+1))
  if [ "$K" = "CHUNKS1" ]; then
    timeout -k 10 200 $L8 --chunks 1 > gpurun_out/${TAG}_l8_$i.json 2>gpurun_out/${TAG}_l8_$i.err || exit 3
  else
    env $K timeout -k 10 200 $L8 > gpurun_out/${TAG}_l8_$i.json 2>gpurun_out/${TAG}_l8_$i.err || exit 3
  fi
  echo "l8 [$K] $(python3 -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_l8_$i.json')); print(round(d['ms_per_step'],4))")"
done
timeout -k 10 200 python3 bench.py --pipeline on --no-secondary --rtt-calls 0 > gpurun_out/${TAG}_pipe8m.json 2> gpurun_out/${TAG}_pipe8m.err || exit 4
timeout -k 10 200 python3 bench.py --pipeline off --no-secondary --rtt-calls 0 > gpurun_out/${TAG}_nopipe8m.json 2> gpurun_out/${TAG}_nopipe8m.err || exit 5
timeout -k 10 200 python3 bench.py --pipeline on --no-secondary --rtt-calls 0 --msgs-per-gpu 1048576 > gpurun_out/${TAG}_pipe1m.json 2> gpurun_out/${TAG}_pipe1m.err || exit 6
timeout -k 10 200 python3 bench.py --pipeline off --no-secondary --rtt-calls 0 --msgs-per-gpu 1048576 > gpurun_out/${TAG}_nopipe1m.json 2> gpurun_out/${TAG}_nopipe1m.err || exit 7
for f in pipe8m nopipe8m pipe1m nopipe1m; do
  echo "$f $(python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_$f.json')); print(round(d['value']/1e9,2), round(d['ms_per_step'],4))")"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_l8prof -o prof -- \
  python3 bench.py --loopback 8 --steps 8 --warmup 4 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_l8prof.log 2>&1 || exit 8
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_1mprof -o prof -- \
  python3 bench.py --msgs-per-gpu 1048576 --steps 8 --warmup 4 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_1mprof.log 2>&1 || exit 9
timeout -k 10 500 python3 bench.py > gpurun_out/${TAG}_b1.json 2> gpurun_out/${TAG}_b1.err || exit 10
cat gpurun_out/${TAG}_b1.json
