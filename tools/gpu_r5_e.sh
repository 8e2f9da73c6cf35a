#!/bin/bash
# Round-5 session E: where the small (1 Mi, config 2) step and the ordered SeqFold
# step spend their time -- kernel stats of each, then shard-count sweeps.  Every
# GPU step under its own limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5e}
val() { python3 -c "import json; d=json.load(open('$1')); print(round(d['value']/1e9,3), round(d['ms_per_step'],4))"; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_seqp -o prof -- \
  python3 bench.py --method seqfold --steps 8 --warmup 4 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_seqp.log 2>&1 || exit 2
echo seqp; tail -1 gpurun_out/${TAG}_seqp.log | cut -c1-200
for SH in 32 64 128 512; do
  timeout -k 10 200 python3 bench.py --no-secondary --rtt-calls 0 --msgs-per-gpu 1048576 --mailbox-shards $SH > gpurun_out/${TAG}_1m_$SH.json 2>gpurun_out/${TAG}_1m_$SH.err || exit 3
  echo "1m shards=$SH $(val gpurun_out/${TAG}_1m_$SH.json)"
done
for K in "PTYPE_MBOX_FUSED=0" "ARR"; do
  if [ "$K" = ARR ]; then A="--sharding arrival"; E="X=0"; else A=""; E=$K; fi
  env $E timeout -k 10 200 python3 bench.py --no-secondary --rtt-calls 0 --msgs-per-gpu 1048576 $A > gpurun_out/${TAG}_1m_$K.json 2>gpurun_out/${TAG}_1m_$K.err || exit 4
  echo "1m [$K] $(val gpurun_out/${TAG}_1m_$K.json)"
done
for SH in 64 128; do
  timeout -k 10 200 python3 bench.py --no-secondary --rtt-calls 0 --mailbox-shards $SH --method seqfold > gpurun_out/${TAG}_seq_$SH.json 2>gpurun_out/${TAG}_seq_$SH.err || exit 5
  echo "seqfold shards=$SH $(val gpurun_out/${TAG}_seq_$SH.json)"
done
