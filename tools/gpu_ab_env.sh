#!/bin/bash
# A/B of an environment knob on the mailbox variants: tools/gpu_ab_env.sh VAR VALUE [variants]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
VAR=$1; VAL=$2; shift 2
for V in ${@:-actor seqfold}; do
  timeout -k 10 120 python3 tools/mb_variant.py $V 10 | sed "s/^/A  /" || exit $?
  env $VAR=$VAL timeout -k 10 120 python3 tools/mb_variant.py $V 10 | sed "s/^/B $VAR=$VAL  /" || exit $?
done
