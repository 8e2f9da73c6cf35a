#!/bin/bash
# SQ instruction / wait counters of the R = 8 pipeline's kernels (bench --loopback 8),
# one counter pass (kernel trace only), summarised per kernel.
# usage (under gpurun, repo root): tools/gpu_loop_sq.sh TAG
set -o pipefail
TAG=${1:-sq}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES --kernel-trace -d gpurun_out/lsq_$TAG -o pmc --output-format csv -- python bench.py --loopback 8 --steps 3 --warmup 1 --rtt-calls 0 --no-secondary --pregen --link-gbps 0 > gpurun_out/lsq_$TAG.log 2>&1 || { echo "PMC FAILED"; tail -5 gpurun_out/lsq_$TAG.log; exit 1; }
python3 - "$TAG" <<'PY'
import csv, collections, sys
rows = list(csv.DictReader(open(f"gpurun_out/lsq_{sys.argv[1]}/pmc_counter_collection.csv")))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
calls = collections.Counter()
seen = set()
for r in rows:
    k = r["Kernel_Name"]
    if "ptype" not in k:
        continue
    name = k.split("(")[0].replace("void ", "").replace("ptype::", "")[:34]
    agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
    key = (name, r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    if key not in seen:
        seen.add(key); calls[name] += 1
cols = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_WAIT_INST_LDS", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES"]
print("%-34s %5s " % ("kernel (per call, M)", "calls") + " ".join("%10s" % c.replace("SQ_", "").replace("INSTS_", "I_")[:10] for c in cols))
for k, d in sorted(agg.items(), key=lambda kv: -kv[1]["SQ_WAVE_CYCLES"]):
    n = max(calls[k], 1)
    print("%-34s %5d " % (k, n) + " ".join("%10.2f" % (d[c] / n / 1e6) for c in cols))
PY
