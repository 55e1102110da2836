#!/bin/bash
# Feed group A/B under the default host run-ahead bound (driver-shaped CaffeNet bench).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for r in ${REPS:-1 2}; do
  for g in ${GROUPS_AB:-2 1 4 3}; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --feed-group $g 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('feed-group $g', d['value'], d['ms_per_step'], flush=True)" || exit 1
  done
done
