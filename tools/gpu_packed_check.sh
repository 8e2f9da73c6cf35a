set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_packed_wire.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/packed_tests.log 2>&1 || { echo "PACKED TESTS FAILED"; tail -40 gpurun_out/packed_tests.log; exit 1; }
tail -3 gpurun_out/packed_tests.log
bash tools/gpu_check.sh s2b
