#!/bin/bash
# Weight gradients (or only the bandwidth-bound fused InnerProduct update) on a side stream
# inside the captured graph, under the run-ahead bound: driver-shaped CaffeNet bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for r in 1 2; do
  for v in "SN_WGRAD_STREAM=0" "SN_WGRAD_STREAM=1 SN_WGRAD_KINDS=fcsgd" "SN_WGRAD_STREAM=1 SN_WGRAD_KINDS=fc,fcsgd" "SN_WGRAD_STREAM=1"; do
    env $v timeout -k 10 300 python bench.py --steps 30 --warmup 5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], flush=True)" || exit 1
  done
done
