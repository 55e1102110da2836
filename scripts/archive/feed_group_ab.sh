#!/bin/bash
# Grouped H2D feeder A/B: stability probe at GROUP=1/4, then the driver-shaped bench at --feed-group 1/2/4.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for g in 1 4; do
  GROUP=$g timeout -k 10 240 python -u scripts/stability.py > gpurun_out/stab_g$g.txt 2>&1 || { echo "stability g$g failed"; tail -20 gpurun_out/stab_g$g.txt; exit 1; }
  echo "== GROUP=$g"; cat gpurun_out/stab_g$g.txt
done
for g in 1 2 4 1 4; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 --feed-group $g > gpurun_out/bench_g$g.json 2> gpurun_out/bench_g$g.err || { echo "bench g$g failed"; tail -20 gpurun_out/bench_g$g.err; exit 1; }
  echo "== feed-group $g"; python -c "import json,sys; d=json.load(open('gpurun_out/bench_g$g.json')); print(d['value'], d['ms_per_step'])"
done
