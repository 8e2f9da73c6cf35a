#!/bin/bash
# Pipelined packed scatter (next tile's loads across this tile's barriers) vs one tile at a time:
# v3 wire GPU tests, then R = 8 loopback steps and per-kernel stats, each way.
# usage (under gpurun, repo root): tools/gpu_scatter_pipe.sh TAG
set -o pipefail
TAG=${1:-sp}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_packed_wire.py tests/test_engine_multirank_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sp_test_$TAG.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/sp_test_$TAG.log; exit 1; }
tail -1 gpurun_out/sp_test_$TAG.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for P in 1 0 1 0; do
  PTYPE_SCATTER_PIPE=$P timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/sp_${TAG}_$P -o run --output-format csv -- python bench.py --loopback 8 --steps 20 --warmup 3 --rtt-calls 0 --no-secondary --pregen > gpurun_out/sp_${TAG}_$P.log 2>&1 || { echo "RUN $P FAILED"; tail -20 gpurun_out/sp_${TAG}_$P.log; exit 1; }
  python - "$TAG" "$P" <<'PY'
import csv, glob, sys, json
tag, p = sys.argv[1], sys.argv[2]
f = glob.glob(f"gpurun_out/sp_{tag}_{p}/**/run_kernel_stats.csv", recursive=True)[0]
rows = {r["Name"].split("(")[0]: float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(f))}
line = [l for l in open(f"gpurun_out/sp_{tag}_{p}.log") if l.startswith("{")]
ms = json.loads(line[-1])["ms_per_step"] if line else None
print("pipe", p, "scatter %.1f us" % next(v for k, v in rows.items() if "route_scatter_packed" in k), "step ms", ms)
PY
done
