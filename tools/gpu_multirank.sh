set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_engine_multirank_gpu.py -m gpu -x -v --timeout 280 --timeout-method thread > gpurun_out/multirank.log 2>&1 || { echo "MULTIRANK FAILED"; tail -60 gpurun_out/multirank.log; exit 1; }
tail -12 gpurun_out/multirank.log
