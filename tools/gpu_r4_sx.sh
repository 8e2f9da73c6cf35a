#!/bin/bash
# Round-4 sorted exchange: GPU tests (FakeComm ranks, IpcComm processes), then the
# loopback-8 compute side with the reserving one-pass sender sort vs count + scan +
# scatter, kernel stats of each, and the Zipf case.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4sx}
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_sorted_exchange_gpu.py \
  "tests/test_ipc_comm_gpu.py::test_sorted_exchange_across_processes_calculator_exact" \
  "tests/test_ipc_comm_gpu.py::test_sorted_exchange_across_processes_seqfold_exactly_once_fifo" \
  "tests/test_engine_multirank_gpu.py::test_gpu_replicated_prime_over_fakecomm_r4" > gpurun_out/${TAG}_tests.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_tests.log
for E in reserve twopass; do
  V=""; [ $E = twopass ] && V=twopass
  rm -rf gpurun_out/${TAG}_l8_$E
  PTYPE_SX_SORT=$V timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_l8_$E -o prof -- \
    python3 bench.py --loopback 8 --steps 6 --warmup 4 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_l8_$E.log 2>&1 || exit 2
  PTYPE_SX_SORT=$V timeout -k 10 200 python3 bench.py --loopback 8 --steps 10 --warmup 5 --rtt-calls 0 --no-secondary \
    > gpurun_out/${TAG}_l8_$E.json 2>/dev/null || exit 3
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('loop8', sys.argv[2], round(d['ms_per_step'],4), 'ms/step')" gpurun_out/${TAG}_l8_$E.json $E
done
timeout -k 10 200 python3 bench.py --loopback 8 --zipf 1.1 --link-gbps 120 --steps 10 --warmup 5 --rtt-calls 0 --no-secondary \
  > gpurun_out/${TAG}_l8_zipf.json 2>/dev/null || exit 4
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print('loop8 zipf', round(d['ms_per_step'],4), 'ms/step', c['exchange'], round(c['wire_bytes_per_msg'],2), 'B/msg resends', c['resend_rounds'])" gpurun_out/${TAG}_l8_zipf.json
