#!/bin/bash
# Round-5 session N: ordered Sends in 8-B records -- the mailbox GPU tests with
# PTYPE_ORD_REC8=1 (SeqFold exactly-once / FIFO audits included), then SeqFold A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5n}
val() { python3 -c "import json; d=json.load(open('$1')); print(round(d['value']/1e9,3), round(d['ms_per_step'],4))"; }
PTYPE_ORD_REC8=1 PTYPE_MBOX_REC8=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_mailbox_gpu.py \
  > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
echo "tests (ORD_REC8) rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/${TAG}_tests.log | tail -5
[ $rc -eq 0 ] || exit 2
for K in "X=0" "PTYPE_ORD_REC8=1"; do
  F="gpurun_out/${TAG}_seq_$(echo $K | tr ' =' '__').json"
  env $K timeout -k 10 200 python3 bench.py --no-secondary --rtt-calls 0 --method seqfold > $F 2>$F.err || exit 3
  echo "seqfold [$K] $(val $F)"
done
