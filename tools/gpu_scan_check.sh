set -o pipefail
bash tools/gpu_route_kernels.sh && timeout -k 10 400 python -u -m pytest tests/test_device_kernels.py tests/test_packed_wire.py tests/test_engine_multirank_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/scan_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/scan_tests.log; exit 1; }
tail -1 gpurun_out/scan_tests.log
