#!/bin/bash
# Quick box-variance check: driver-shaped CaffeNet bench at feed group 1 / 2, twice each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for g in 2 1 2 1; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 --feed-group $g > gpurun_out/bc_g$g.json 2> gpurun_out/bc_g$g.err || { echo "bench g$g failed"; tail -20 gpurun_out/bc_g$g.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bc_g$g.json')); print('feed-group $g', d['value'], d['ms_per_step'], flush=True)"
done
timeout -k 10 120 rocm-smi --showclocks --showpower --showtemp > gpurun_out/bc_smi.txt 2>&1; cat gpurun_out/bc_smi.txt | grep -i "sclk\|mclk\|power\|temp" | head -12
