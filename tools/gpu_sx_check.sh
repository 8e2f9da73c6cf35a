set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_sorted_exchange_gpu.py > gpurun_out/sxt.log 2>&1 || { tail -30 gpurun_out/sxt.log; exit 1; }
tail -2 gpurun_out/sxt.log
bash tools/gpu_loopprof.sh rw 8
