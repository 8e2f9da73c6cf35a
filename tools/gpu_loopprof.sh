#!/bin/bash
# Kernel-time breakdown of the R-rank pipeline on one GPU (FakeComm loopback):
# the bench step with no link model (pure kernels + local copies), uniform load,
# then the same under rocprofv3 --kernel-trace --stats.
# usage (under gpurun, repo root): tools/gpu_loopprof.sh TAG [R]
set -o pipefail
TAG=${1:-lp}
R=${2:-8}
mkdir -p gpurun_out
OUT=gpurun_out/loop_$TAG.jsonl
: > $OUT
COMMON="--loopback $R --steps 10 --warmup 3 --rtt-calls 0 --no-secondary --pregen"
timeout -k 10 200 python bench.py $COMMON --link-gbps 0 >> $OUT 2> gpurun_out/loop_$TAG.err || { echo "NOLINK FAILED"; tail -20 gpurun_out/loop_$TAG.err; exit 1; }
timeout -k 10 200 python bench.py $COMMON --link-gbps 120 >> $OUT 2>> gpurun_out/loop_$TAG.err || { echo "LINK FAILED"; tail -20 gpurun_out/loop_$TAG.err; exit 1; }
python - "$OUT" <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    if ln.startswith("{"):
        d = json.loads(ln); c = d["config"]
        print("link", c.get("link_gbps"), "ms/step %.3f" % d["ms_per_step"], "G msg/s %.2f" % (d["value"] / 1e9), c.get("wire"), c.get("record_bytes"), c.get("reply_bytes"))
PY
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/loopprof_$TAG -o run --output-format csv -- python bench.py $COMMON --link-gbps 0 > gpurun_out/loopprof_$TAG.log 2>&1 || { echo "PROF FAILED"; tail -20 gpurun_out/loopprof_$TAG.log; exit 1; }
python tools/kstats.py gpurun_out/loopprof_$TAG 2>&1 | head -30
