#!/bin/bash
# Alternate bench runs with an environment switch: VAR=SN_FUSE_SPLITK A=0 B=1 MODELS="caffenet googlenet" bash scripts/env_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for i in 1 2; do
  for m in ${MODELS:-caffenet}; do
    for v in $A $B; do
      env $VAR=$v timeout -k 10 300 python bench.py --model $m --steps ${STEPS:-30} --warmup 5 $ARGS 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m $VAR=$v', d['value'], d['ms_per_step'])" || exit 1
    done
  done
done
