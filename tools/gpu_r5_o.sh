#!/bin/bash
# Round-5 session O: the ordered 8-B-record test and the duplex relay test (numbers printed).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5o}
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 280 --timeout-method thread \
  tests/test_mailbox_gpu.py::test_mailbox_seqfold_in_8b_records_exactly_once_fifo \
  tests/test_xcall_gpu.py::test_duplex_relays_do_not_block_the_dispatchers > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|FAILED|^duplex|Error|assert" gpurun_out/${TAG}_tests.log | cut -c1-700 | tail -8
exit $rc
