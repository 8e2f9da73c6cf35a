#!/bin/bash
# Round-4 GPU session: the mailbox kernels (fused sort + drain, group look-back,
# tag wrap), GPU peer calls and relays, the IpcComm process tests; then the bench
# with its secondaries, an A/B without the fused kernel and a kernel-stats
# profile; the tests that SIGKILL a rank run last.  Every GPU step under its own
# time limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PYT tests/test_mailbox_gpu.py tests/test_sorted_exchange_gpu.py tests/test_xcall_gpu.py \
  tests/test_device_kernels.py::test_prime_gather_kernel_matches_reference \
  "tests/test_ipc_comm_gpu.py::test_ipc_comm_collectives_exact" \
  "tests/test_ipc_comm_gpu.py::test_sorted_exchange_across_processes_calculator_exact" \
  "tests/test_ipc_comm_gpu.py::test_sorted_exchange_across_processes_seqfold_exactly_once_fifo" \
  "tests/test_ipc_comm_gpu.py::test_epoch_engine_across_processes_exact_size_exchange" \
  > gpurun_out/r4_t1.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4_b1.json 2> gpurun_out/r4_b1.err || exit 2
PTYPE_MBOX_FUSED=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-secondary \
  > gpurun_out/r4_b1_nofused.json 2> gpurun_out/r4_b1_nofused.err || exit 3
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4_prof -o r4 -- \
  python bench.py --steps 8 --warmup 4 --no-secondary > gpurun_out/r4_prof.log 2>&1 || exit 4
timeout -k 10 400 $PYT "tests/test_ipc_comm_gpu.py::test_killed_rank_is_a_peer_failure_within_the_timeout" \
  tests/test_elastic_ipc_gpu.py > gpurun_out/r4_t2.log 2>&1 || exit 5
