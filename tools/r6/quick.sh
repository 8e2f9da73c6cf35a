# quick GPU check: selected tests (-k "$1") + one bench run (all secondaries) -> gpurun_out/$2*
set -o pipefail
tag=${2:-q}
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/ -m gpu -k "$1" > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/${tag}_tests.log | tail -2
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 8 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -20 gpurun_out/${tag}_bench.err; exit 1; }
python3 tools/r6/summ.py gpurun_out/${tag}_bench.json || true
