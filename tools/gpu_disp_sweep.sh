#!/bin/bash
# dispatch_packed grid sweep on the R = 8 loopback step (PTYPE_DISPATCH_BLOCKS), per-kernel stats.
# usage (under gpurun, repo root): tools/gpu_disp_sweep.sh TAG
set -o pipefail
TAG=${1:-ds}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for B in 2048 4096 8192 16384; do
  PTYPE_DISPATCH_BLOCKS=$B timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ds_${TAG}_$B -o run --output-format csv -- python bench.py --loopback 8 --steps 10 --warmup 3 --rtt-calls 0 --no-secondary --pregen > gpurun_out/ds_${TAG}_$B.log 2>&1 || { echo "RUN $B FAILED"; tail -20 gpurun_out/ds_${TAG}_$B.log; exit 1; }
  python - "$TAG" "$B" <<'PY'
import csv, glob, sys, json
tag, b = sys.argv[1], sys.argv[2]
f = glob.glob(f"gpurun_out/ds_{tag}_{b}/**/run_kernel_stats.csv", recursive=True)[0]
rows = {r["Name"].split("(")[0]: float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(f))}
line = [l for l in open(f"gpurun_out/ds_{tag}_{b}.log") if l.startswith("{")]
ms = json.loads(line[-1])["ms_per_step"] if line else None
print(b, "dispatch %.1f us" % next(v for k, v in rows.items() if "dispatch_packed" in k),
      "complete %.1f us" % next(v for k, v in rows.items() if "complete_packed" in k), "step ms", ms)
PY
done
