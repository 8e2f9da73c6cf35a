timeout -k 10 800 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_bench.py -k "api_send_secondary_at_n2 or force_dist" > gpurun_out/r6dp2.log 2>&1 && \
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_sorted_exchange_gpu.py tests/test_packed_wire.py tests/test_engine_gpu.py -m gpu > gpurun_out/r6dp3.log 2>&1
rc=$?; grep -hE "passed|failed|FAILED" gpurun_out/r6dp2.log gpurun_out/r6dp3.log | tail; exit $rc
