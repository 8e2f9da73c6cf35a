#!/bin/bash
# Stateless view shard count sweep (PTYPE_MBOX_STATELESS_SHARDS) with the reserving one-pass
# sort and 8-B records: the 8 Mi Send alone (mb_variant) and the bench headline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4sh}
for SH in 4 8 16 32 64; do
  echo -n "shards $SH: "; PTYPE_MBOX_STATELESS_SHARDS=$SH timeout -k 10 100 python3 tools/mb_variant.py actor 30 || exit 1
  PTYPE_MBOX_STATELESS_SHARDS=$SH timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-secondary > gpurun_out/${TAG}_$SH.json 2>/dev/null || exit 2
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('   bench', round(d['value']/1e9,2), 'G msg/s', round(d['ms_per_step']*1e3,1), 'us/step')" gpurun_out/${TAG}_$SH.json
done
