set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests/test_mailbox_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/r3_mb_tests.log 2>&1
echo "tests rc=$?"
tail -5 gpurun_out/r3_mb_tests.log
timeout -k 10 240 python bench.py --steps 20 --warmup 8 > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/r3_bench.json | head -c 3000
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r3prof" -o prof -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 8 --warmup 4 --rtt-calls 100 --no-secondary > "$GRAFT_REPO_ROOT/gpurun_out/r3_prof_bench.log" 2>&1
echo "prof rc=$?"
