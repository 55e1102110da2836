#!/bin/bash
# Second grouped-feeder A/B: driver-shaped bench (20 timed / 5 warmup) interleaved over groups.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for g in 1 2 3 4 8 2 3 4 8 1 2 4; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 --feed-group $g > gpurun_out/b2_g$g.json 2> gpurun_out/b2_g$g.err || { echo "bench g$g failed"; tail -20 gpurun_out/b2_g$g.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/b2_g$g.json')); print('feed-group $g', d['value'], d['ms_per_step'], flush=True)"
done
timeout -k 10 240 python bench.py --steps 50 --warmup 10 --feed-group 2 > gpurun_out/b2_long.json 2>/dev/null && python -c "import json; d=json.load(open('gpurun_out/b2_long.json')); print('feed-group 2 50 steps', d['value'], d['ms_per_step'])"
