#!/bin/bash
# SQ counters of the packed route kernels at R=1 vs R=8 (one counter pass each)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for R in 1 8; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES --kernel-trace -d gpurun_out/spmc_$R -o pmc --output-format csv -- python tools/packed_route_bench.py 2097152 $R > gpurun_out/spmc_$R.log 2>&1 || { echo "PMC $R FAILED"; tail -5 gpurun_out/spmc_$R.log; exit 1; }
done
python - <<'PY'
import csv, collections
for R in (1, 8):
    rows = list(csv.DictReader(open(f"gpurun_out/spmc_{R}/pmc_counter_collection.csv")))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.Counter()
    for r in rows:
        k = r["Kernel_Name"]
        if "scatter" not in k and "route_prep" not in k and "dispatch_packed" not in k:
            continue
        agg[k[:40]][r["Counter_Name"]] += float(r["Counter_Value"])
    print("R =", R)
    for k, d in agg.items():
        print("  ", k, {c: "%.3g" % v for c, v in sorted(d.items())})
PY
