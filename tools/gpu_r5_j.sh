#!/bin/bash
# Round-5 session J: the ordered drain's register fold for uniform SeqFold batches and
# 4096-record windows -- the ordered / mailbox GPU tests first, then the SeqFold line
# A/B and its kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5j}
val() { python3 -c "import json; d=json.load(open('$1')); print(round(d['value']/1e9,3), round(d['ms_per_step'],4))"; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_mailbox_gpu.py \
  "tests/test_ipc_comm_gpu.py::test_sorted_exchange_across_processes_seqfold_exactly_once_fifo" \
  > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/${TAG}_tests.log | tail -5
[ $rc -eq 0 ] || exit 2
for K in "X=0" "PTYPE_ORD_FIXED=0" "PTYPE_ORD_WIN=2048" "PTYPE_ORD_WIN=2048 PTYPE_ORD_FIXED=0"; do
  F="gpurun_out/${TAG}_seq_$(echo $K | tr ' =' '__').json"
  env $K timeout -k 10 200 python3 bench.py --no-secondary --rtt-calls 0 --method seqfold > $F 2>$F.err || exit 3
  echo "seqfold [$K] $(val $F)"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_seqp -o prof -- \
  python3 bench.py --method seqfold --steps 8 --warmup 4 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_seqp.log 2>&1 || exit 4
python3 tools/kstats.py gpurun_out/${TAG}_seqp/prof_kernel_stats.csv > gpurun_out/${TAG}_seqp.txt && sed -n 1,6p gpurun_out/${TAG}_seqp.txt
