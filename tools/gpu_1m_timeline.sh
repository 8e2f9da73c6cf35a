#!/bin/bash
# 1 Mi messages per step (BASELINE config 2 size), 8 steps per graph replay: kernel durations and the gaps between them.
# usage (under gpurun, repo root): tools/gpu_1m_timeline.sh TAG [extra bench args]
set -o pipefail
TAG=${1:-t1m}
shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/t1m_$TAG -o run --output-format csv -- python bench.py --msgs-per-gpu 1048576 --steps 64 --warmup 8 --steps-per-graph 8 --rtt-calls 0 --no-secondary "$@" > gpurun_out/t1m_$TAG.log 2>&1 || { echo "RUN FAILED"; tail -20 gpurun_out/t1m_$TAG.log; exit 1; }
grep '^{' gpurun_out/t1m_$TAG.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', round(d['value']/1e9,2), 'G msg/s, ms/step', round(d['ms_per_step'],4))"
python - "$TAG" <<'PY'
import csv, glob, sys, collections
f = glob.glob(f"gpurun_out/t1m_{sys.argv[1]}/**/run_kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
rows = rows[len(rows) // 2:]  # steady state
dur = collections.defaultdict(list)
gaps = []
prev = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    dur[r["Kernel_Name"].split("(")[0][:50]].append((e - s) / 1e3)
    if prev is not None:
        gaps.append((s - prev) / 1e3)
    prev = e
for k, v in dur.items():
    v.sort()
    print(k.ljust(52), len(v), "median %.1f us" % v[len(v) // 2])
gaps.sort()
print("gaps: n", len(gaps), "median %.1f us" % gaps[len(gaps) // 2], "p90 %.1f us" % gaps[int(len(gaps) * 0.9)])
PY
