#!/bin/bash
# Host run-ahead bound A/B (SN_MAX_AHEAD): driver-shaped CaffeNet bench and the in-stream
# 10-step slices of scripts/stability.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for d in 0 1 2 3 4; do
    SN_MAX_AHEAD=$d timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('max_ahead $d bench 20/5', d['value'], d['ms_per_step'], flush=True)" || exit 1
  done
done
for d in 0 2 3; do
  SN_MAX_AHEAD=$d timeout -k 10 300 python scripts/stability.py 2>&1 | grep -E "in-stream|chunks" | sed "s/^/max_ahead $d /" || exit 1
done
