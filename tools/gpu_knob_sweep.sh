#!/bin/bash
# A/B of one env knob on the R-rank loopback step: bench line + per-kernel times
# under rocprofv3 --kernel-trace --stats for each value.
# usage (under gpurun, repo root): tools/gpu_knob_sweep.sh TAG VAR "v1 v2 ..." [R]
set -o pipefail
TAG=$1; VAR=$2; VALS=$3; R=${4:-8}
mkdir -p gpurun_out
OUT=gpurun_out/knob_$TAG.txt
: > $OUT
COMMON="--loopback $R --steps 10 --warmup 3 --rtt-calls 0 --no-secondary --pregen --link-gbps 0"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in $VALS; do
  export $VAR=$v
  timeout -k 10 200 python bench.py $COMMON > gpurun_out/knob_${TAG}_$v.json 2> gpurun_out/knob_${TAG}_$v.err || { echo "BENCH $v FAILED"; tail -20 gpurun_out/knob_${TAG}_$v.err; exit 1; }
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/knobprof_${TAG}_$v -o run --output-format csv -- python bench.py $COMMON > gpurun_out/knobprof_${TAG}_$v.log 2>&1 || { echo "PROF $v FAILED"; tail -20 gpurun_out/knobprof_${TAG}_$v.log; exit 1; }
  python - "$TAG" "$v" "$VAR" >> $OUT <<'PY'
import csv, glob, json, sys
tag, v, var = sys.argv[1:4]
d = json.load(open(f"gpurun_out/knob_{tag}_{v}.json"))
f = glob.glob(f"gpurun_out/knobprof_{tag}_{v}/**/run_kernel_stats.csv", recursive=True)[0]
ks = "  ".join("%s=%.1fus" % (r["Name"].split("(")[0].replace("void ", "").replace("ptype::", "")[:34], float(r["AverageNs"]) / 1e3)
               for r in list(csv.DictReader(open(f)))[:7])
print(f"{var}={v}: {d['ms_per_step']:.4f} ms/step  {ks}")
PY
done
cat $OUT
