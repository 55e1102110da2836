#!/bin/bash
# Sequential (1 stream) vs branch-stream graphs: CaffeNet (no branches) and GoogLeNet.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for r in 1 2; do
  for m in caffenet googlenet; do
    for st in 4 1 2; do
      timeout -k 10 300 python bench.py --model $m --steps 30 --warmup 5 --streams $st 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m streams $st', d['value'], d['ms_per_step'], flush=True)" || exit 1
    done
  done
done
