#!/bin/bash
# Round-5 session F: the binned ordered drain -- mailbox / ordered GPU tests, then
# the SeqFold line binned vs windowed (PTYPE_ORD_DRAIN=win) and its kernel stats, the
# 1 Mi step with 1024- vs 4096-message fused tiles (PTYPE_MBOX_SK=8) and its kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5f}
val() { python3 -c "import json; d=json.load(open('$1')); print(round(d['value']/1e9,3), round(d['ms_per_step'],4))"; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_mailbox_gpu.py \
  tests/test_sorted_exchange_gpu.py "tests/test_ipc_comm_gpu.py::test_sorted_exchange_across_processes_seqfold_exactly_once_fifo" \
  "tests/test_xcall_gpu.py::test_actor_handler_decides_its_remote_call_and_continues_on_the_reply" \
  > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/${TAG}_tests.log | tail -5
[ $rc -eq 0 ] || exit 2
for K in "X=0" "PTYPE_ORD_DRAIN=win"; do
  env $K timeout -k 10 200 python3 bench.py --no-secondary --rtt-calls 0 --method seqfold > gpurun_out/${TAG}_seq_$K.json 2>gpurun_out/${TAG}_seq_$K.err || exit 3
  echo "seqfold [$K] $(val gpurun_out/${TAG}_seq_$K.json)"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_seqp -o prof -- \
  python3 bench.py --method seqfold --steps 8 --warmup 4 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_seqp.log 2>&1 || exit 4
python3 tools/kstats.py gpurun_out/${TAG}_seqp/prof_kernel_stats.csv > gpurun_out/${TAG}_seqp.txt && sed -n 1,8p gpurun_out/${TAG}_seqp.txt
for K in "X=0" "PTYPE_MBOX_SK=8"; do
  env $K timeout -k 10 200 python3 bench.py --no-secondary --rtt-calls 0 --msgs-per-gpu 1048576 > gpurun_out/${TAG}_1m_$K.json 2>gpurun_out/${TAG}_1m_$K.err || exit 5
  echo "1m [$K] $(val gpurun_out/${TAG}_1m_$K.json)"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_1mp -o prof -- \
  python3 bench.py --msgs-per-gpu 1048576 --steps 8 --warmup 4 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_1mp.log 2>&1 || exit 6
python3 tools/kstats.py gpurun_out/${TAG}_1mp/prof_kernel_stats.csv > gpurun_out/${TAG}_1mp.txt && sed -n 1,6p gpurun_out/${TAG}_1mp.txt
