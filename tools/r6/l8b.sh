#!/bin/bash
# Round 6: loopback-8 host cost per HIP call (runtime trace + kernel stats), and the
# graph cache at 1 Mi messages per rank (host-bound sizes) vs eager.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6l}
rm -rf gpurun_out/$TAG
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --stats -d gpurun_out/$TAG -o rt --output-format csv -- \
  python3 bench.py --loopback 8 --steps 20 --warmup 5 --rtt-calls 0 --no-secondary > gpurun_out/${TAG}.json 2> gpurun_out/${TAG}.err || exit 1
for g in 1 0; do
  PTYPE_TUNE=sx_graph=$g timeout -k 10 300 python3 bench.py --loopback 8 --msgs-per-gpu 1048576 --steps 20 --warmup 5 --rtt-calls 0 \
    --no-secondary > gpurun_out/${TAG}_1m_g$g.json 2> gpurun_out/${TAG}_1m_g$g.err || { tail -20 gpurun_out/${TAG}_1m_g$g.err; exit 4; }
done
python3 tools/r6/summ.py gpurun_out/${TAG}.json gpurun_out/${TAG}_1m_g1.json gpurun_out/${TAG}_1m_g0.json
find gpurun_out/$TAG -name '*stats.csv'
