#!/bin/bash
# BASELINE configs 1/2/4/5 (+ tells, cross-process calls, K4 gob) on one GPU + hardware counters for the Send kernels.
# usage (under gpurun): bash tools/gpu_suite.sh TAG
set -o pipefail
TAG=${1:-suite}
mkdir -p gpurun_out
OUT=gpurun_out/suite_$TAG.jsonl
: > $OUT
timeout -k 10 300 python tools/bench_suite.py host-rpc >> $OUT 2> gpurun_out/suite_$TAG.err || { echo "host-rpc FAILED"; tail -5 gpurun_out/suite_$TAG.err; exit 1; }
timeout -k 10 300 python tools/bench_suite.py gpu-1m >> $OUT 2>> gpurun_out/suite_$TAG.err || { echo "gpu-1m FAILED"; tail -5 gpurun_out/suite_$TAG.err; exit 1; }
timeout -k 10 300 python tools/bench_suite.py optimus >> $OUT 2>> gpurun_out/suite_$TAG.err || { echo "optimus FAILED"; tail -5 gpurun_out/suite_$TAG.err; exit 1; }
# config 4's 8-GPU step on one GPU: rank 0 of an 8-rank node (FakeComm loopback), links unmodelled / at 120 GB/s
timeout -k 10 300 python tools/bench_suite.py optimus --loopback 8 >> $OUT 2>> gpurun_out/suite_$TAG.err || { echo "optimus loopback FAILED"; tail -5 gpurun_out/suite_$TAG.err; exit 1; }
timeout -k 10 300 python tools/bench_suite.py optimus --loopback 8 --link-gbps 120 >> $OUT 2>> gpurun_out/suite_$TAG.err || { echo "optimus loopback link FAILED"; tail -5 gpurun_out/suite_$TAG.err; exit 1; }
timeout -k 10 300 python tools/bench_suite.py tell >> $OUT 2>> gpurun_out/suite_$TAG.err || { echo "tell FAILED"; tail -5 gpurun_out/suite_$TAG.err; exit 1; }
timeout -k 10 300 python tools/bench_suite.py xproc >> $OUT 2>> gpurun_out/suite_$TAG.err || { echo "xproc FAILED"; tail -5 gpurun_out/suite_$TAG.err; exit 1; }
timeout -k 10 300 python tools/bench_suite.py registry >> $OUT 2>> gpurun_out/suite_$TAG.err || { echo "registry FAILED"; tail -5 gpurun_out/suite_$TAG.err; exit 1; }
timeout -k 10 300 python tools/bench_suite.py gob >> $OUT 2>> gpurun_out/suite_$TAG.err || { echo "gob FAILED"; tail -5 gpurun_out/suite_$TAG.err; exit 1; }
cat $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmc_${TAG}_$C -o pmc --output-format csv -- python bench.py --steps 3 --warmup 1 --rtt-calls 0 --graph off > gpurun_out/pmc_${TAG}_$C.log 2>&1 || { echo "PMC $C FAILED"; tail -5 gpurun_out/pmc_${TAG}_$C.log; exit 1; }
done
python tools/pmc_summary.py gpurun_out/pmc_${TAG}_FETCH_SIZE gpurun_out/pmc_${TAG}_WRITE_SIZE | tee gpurun_out/pmc_${TAG}_summary.txt
# the RCCL path (wire v3) with collectives forced on at world 1.  Counter passes use
# event hand-offs: counter collection serialises dispatches device-wide, which deadlocks
# a cross-queue wait-value hand-off (root cause in profiles/README.md).
for C in FETCH_SIZE WRITE_SIZE; do
  PTYPE_STREAM_SYNC=events timeout -k 10 150 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmcd_${TAG}_$C -o pmc --output-format csv -- python bench.py --force-dist --steps 3 --warmup 1 --rtt-calls 0 > gpurun_out/pmcd_${TAG}_$C.log 2>&1 || { echo "PMC dist $C FAILED"; tail -5 gpurun_out/pmcd_${TAG}_$C.log; exit 1; }
done
python tools/pmc_summary.py gpurun_out/pmcd_${TAG}_FETCH_SIZE gpurun_out/pmcd_${TAG}_WRITE_SIZE | tee gpurun_out/pmcd_${TAG}_summary.txt
