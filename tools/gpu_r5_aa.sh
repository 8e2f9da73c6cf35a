#!/bin/bash
# Round-5 session AA: counter passes over the headline step (rank byte gathers) and
# the loopback-8 step (after the hand-off changes); kernel trace only, each pass
# under its own kill limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5aa}
for W in head l8; do
  if [ $W = head ]; then A=""; else A="--loopback 8"; fi
  P=0
  for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD" \
           "SQ_WAVES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE"; do
    P=$((P+1))
    rm -rf gpurun_out/${TAG}_${W}_pmc_$P
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/${TAG}_${W}_pmc_$P -o pmc --output-format csv -- \
      python3 bench.py $A --steps 4 --warmup 3 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_${W}_pmc_$P.log 2>&1
    rc=$?; echo "$W pmc pass $P rc=$rc"
    [ $rc -eq 0 ] || exit 3
  done
  python3 tools/pmc_table.py gpurun_out/${TAG}_${W}_pmc_* > gpurun_out/${TAG}_${W}_pmc.txt
  sed -n 1,10p gpurun_out/${TAG}_${W}_pmc.txt | cut -c1-60,280-400
done
# replies stored non-temporal (PTYPE_REPLY_NT=1) on the headline and SeqFold lines
val() { python3 -c "import json; d=[json.loads(x) for x in open('$1') if x.startswith('{')][-1]; print(round(d['value']/1e9,3), round(d['ms_per_step'],4))"; }
for V in 1 0 1 0; do
  F="gpurun_out/${TAG}_nt${V}_$RANDOM.json"
  PTYPE_REPLY_NT=$V timeout -k 10 200 python3 bench.py --steps 50 --warmup 10 --rtt-calls 0 --no-secondary > $F 2>$F.err || exit 3
  G="gpurun_out/${TAG}_seqnt${V}_$RANDOM.json"
  PTYPE_REPLY_NT=$V timeout -k 10 200 python3 bench.py --steps 30 --warmup 10 --rtt-calls 0 --no-secondary --method seqfold > $G 2>$G.err || exit 3
  echo "reply_nt=$V head $(val $F) seqfold $(val $G)"
done
