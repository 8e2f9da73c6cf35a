#!/bin/bash
# Mailbox path: GPU tests, the bench's mailbox figure, and FETCH/WRITE PMC of the
# enqueue + drain kernels (separate counter passes, kernel trace only).
# usage (under gpurun, repo root): tools/gpu_mbpmc.sh TAG
set -o pipefail
TAG=${1:-mbp}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_mailbox_gpu.py tests/test_persistent_streams_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/mbp_test_$TAG.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/mbp_test_$TAG.log; exit 1; }
tail -1 gpurun_out/mbp_test_$TAG.log
timeout -k 10 300 python bench.py --delivery mailbox --rtt-calls 0 > gpurun_out/bench_mb_$TAG.json 2> gpurun_out/bench_mb_$TAG.err || { echo "BENCH FAILED"; tail -20 gpurun_out/bench_mb_$TAG.err; exit 1; }
python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print('mailbox headline ms/step %.4f G msg/s %.1f; direct secondary %s' % (d['ms_per_step'], d['value']/1e9, d.get('secondary_delivery')))" gpurun_out/bench_mb_$TAG.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 200 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/mbpmc_${TAG}_$C -o pmc --output-format csv -- python bench.py --delivery mailbox --steps 3 --warmup 1 --rtt-calls 0 --graph off --no-secondary > gpurun_out/mbpmc_${TAG}_$C.log 2>&1 || { echo "PMC $C FAILED"; tail -5 gpurun_out/mbpmc_${TAG}_$C.log; exit 1; }
done
python tools/pmc_summary.py gpurun_out/mbpmc_${TAG}_FETCH_SIZE gpurun_out/mbpmc_${TAG}_WRITE_SIZE | tee gpurun_out/mbpmc_${TAG}_summary.txt
