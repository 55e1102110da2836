#!/bin/bash
# Run-ahead bound default (2) vs unbounded, interleaved: CaffeNet driver-shaped bench x3,
# GoogLeNet and cifar10_quick once each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for r in 1 2 3; do
  for d in 2 0; do
    SN_MAX_AHEAD=$d timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('caffenet max_ahead $d', d['value'], d['ms_per_step'], flush=True)" || exit 1
  done
done
for m in googlenet cifar10_quick; do
  for d in 2 0; do
    SN_MAX_AHEAD=$d timeout -k 10 300 python bench.py --model $m --steps 40 --warmup 5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m max_ahead $d', d['value'], d['ms_per_step'], flush=True)" || exit 1
  done
done
