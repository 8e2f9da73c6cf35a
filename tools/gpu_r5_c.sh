#!/bin/bash
# Round-5 session C: the relay tests, NT-store A/Bs (loopback-8 and N=1), the
# ordered SeqFold line with 256 / 512 / 1024 shards, then the loopback-8 PMC
# passes (kernel trace only, each pass under its own kill limit).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5c}
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread \
  "tests/test_xcall_gpu.py::test_duplex_relays_do_not_block_the_dispatchers" \
  "tests/test_xcall_gpu.py::test_relay_target_killed_mid_relay" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|passed|failed|duplex|relay target" gpurun_out/${TAG}_tests.log | tail -8
[ $rc -le 1 ] || exit $rc
val() { python3 -c "import json; d=json.load(open('$1')); print(round(d['value']/1e9,3), round(d['ms_per_step'],4))"; }
L8="python3 bench.py --loopback 8 --steps 20 --warmup 5 --rtt-calls 0 --no-secondary"
for K in "X=0" "PTYPE_COMP_NT=1" "PTYPE_GEN_NT=1"; do
  env $K timeout -k 10 200 $L8 > gpurun_out/${TAG}_l8_$K.json 2>gpurun_out/${TAG}_l8_$K.err || exit 3
  echo "l8 [$K] $(val gpurun_out/${TAG}_l8_$K.json)"
done
for K in "X=0" "PTYPE_GEN_NT=1"; do
  for MM in 8388608 1048576; do
    env $K timeout -k 10 200 python3 bench.py --no-secondary --rtt-calls 0 --msgs-per-gpu $MM > gpurun_out/${TAG}_n1_${K}_$MM.json 2>gpurun_out/${TAG}_n1.err || exit 4
    echo "n1 $MM [$K] $(val gpurun_out/${TAG}_n1_${K}_$MM.json)"
  done
done
for SH in 256 512 1024; do
  timeout -k 10 200 python3 bench.py --no-secondary --rtt-calls 0 --mailbox-shards $SH --method seqfold > gpurun_out/${TAG}_seq_$SH.json 2>gpurun_out/${TAG}_seq_$SH.err || exit 6
  echo "seqfold shards=$SH $(val gpurun_out/${TAG}_seq_$SH.json)"
done
P=0
for C in "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD" \
         "SQ_WAVES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES"; do
  P=$((P+1))
  rm -rf gpurun_out/${TAG}_pmc_$P
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/${TAG}_pmc_$P -o pmc --output-format csv -- \
    python3 bench.py --loopback 8 --steps 4 --warmup 3 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}_pmc_$P.log 2>&1
  rc=$?; echo "pmc pass $P rc=$rc"
  [ $rc -eq 0 ] || exit 7
done
python3 tools/pmc_table.py gpurun_out/${TAG}_pmc_1 gpurun_out/${TAG}_pmc_2 gpurun_out/${TAG}_pmc_3 gpurun_out/${TAG}_pmc_4 > gpurun_out/${TAG}_pmc.txt
head -20 gpurun_out/${TAG}_pmc.txt
