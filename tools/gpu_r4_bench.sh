#!/bin/bash
# Round-4 bench session: the N=1 bench with its secondaries, an A/B without the
# fused sort + drain kernel, a kernel-stats profile, then the tests that SIGKILL
# a rank.  Every GPU step under its own time limit; the first failure ends it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4}
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_b1.json 2> gpurun_out/${TAG}_b1.err || exit 2
PTYPE_MBOX_FUSED=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-secondary \
  > gpurun_out/${TAG}_b1_nofused.json 2> gpurun_out/${TAG}_b1_nofused.err || exit 3
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o prof -- \
  python bench.py --steps 8 --warmup 4 --no-secondary > gpurun_out/${TAG}_prof.log 2>&1 || exit 4
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_ipc_comm_gpu.py::test_killed_rank_is_a_peer_failure_within_the_timeout" \
  tests/test_elastic_ipc_gpu.py > gpurun_out/${TAG}_t2.log 2>&1 || exit 5
