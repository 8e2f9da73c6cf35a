#!/bin/bash
# Round-5 session L: the ordered paths after the register folds -- the ordered GPU
# tests (mailbox, sorted exchange, IpcComm FIFO), then SeqFold with the drain's
# window prefetch and with the sender's late argument loads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5l}
val() { python3 -c "import json; d=json.load(open('$1')); print(round(d['value']/1e9,3), round(d['ms_per_step'],4))"; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_mailbox_gpu.py \
  tests/test_sorted_exchange_gpu.py "tests/test_ipc_comm_gpu.py::test_sorted_exchange_across_processes_seqfold_exactly_once_fifo" \
  > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/${TAG}_tests.log | tail -5
[ $rc -eq 0 ] || exit 2
for K in "X=0" "PTYPE_ORD_PREFETCH=1" "PTYPE_OS_LATE=1" "PTYPE_ORD_PREFETCH=1 PTYPE_OS_LATE=1"; do
  F="gpurun_out/${TAG}_seq_$(echo $K | tr ' =' '__').json"
  env $K timeout -k 10 200 python3 bench.py --no-secondary --rtt-calls 0 --method seqfold > $F 2>$F.err || exit 3
  echo "seqfold [$K] $(val $F)"
done
