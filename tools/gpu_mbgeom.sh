#!/bin/bash
# Mailbox geometry sweep on the N=1 headline step: shards x slots (ms/step).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for S in 64 128 256 512; do
  for Q in 0 65536; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 8 --rtt-calls 0 --no-secondary --mailbox-shards $S --mailbox-slots $Q > gpurun_out/geom_${S}_${Q}.json 2>/dev/null
    rc=$?
    [ $rc -eq 0 ] || { echo "S=$S Q=$Q rc=$rc"; exit $rc; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('S=%s Q=%s ms/step %.4f  %.1f G msg/s' % (sys.argv[2], sys.argv[3], d['ms_per_step'], d['value']/1e9))" gpurun_out/geom_${S}_${Q}.json $S $Q
  done
done
