# GPU session: sorted mailbox + sorted exchange tests, the N=1 bench, the
# loopback-8 compute side, and rocprofv3 kernel stats of both.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests/test_mailbox_gpu.py tests/test_sorted_exchange_gpu.py -v --timeout 150 --timeout-method thread > gpurun_out/r3_mb_tests.log 2>&1
rc=$?; echo "tests rc=$rc"
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r3_mb_tests.log | tail -40
[ $rc -le 1 ] || exit $rc  # a crash / time limit: nothing more on the GPU
timeout -k 10 240 python bench.py --steps 20 --warmup 8 > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err
rc=$?; echo "bench rc=$rc"; head -c 4000 gpurun_out/r3_bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python bench.py --loopback 8 --steps 10 --warmup 4 --rtt-calls 0 --no-secondary > gpurun_out/r3_loop8.json 2> gpurun_out/r3_loop8.err
rc=$?; echo "loop8 rc=$rc"; head -c 2500 gpurun_out/r3_loop8.json
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r3prof" -o prof -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 8 --warmup 4 --rtt-calls 0 --no-secondary > "$GRAFT_REPO_ROOT/gpurun_out/r3_prof_bench.log" 2>&1
echo "prof rc=$?"
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r3prof_l8" -o prof -- python3 "$GRAFT_REPO_ROOT/bench.py" --loopback 8 --steps 6 --warmup 4 --rtt-calls 0 --no-secondary > "$GRAFT_REPO_ROOT/gpurun_out/r3_prof_l8.log" 2>&1
echo "prof l8 rc=$?"
