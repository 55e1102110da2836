#!/bin/bash
# Box-variance probe: driver-shaped bench twice, then the in-process stability probe with and
# without the per-step H2D minibatch copy (NOFEED=1 is a timing-only diagnostic).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench 20/5', d['value'], d['ms_per_step'], flush=True)" || exit 1
done
timeout -k 10 300 python scripts/stability.py > gpurun_out/stab_feed.txt 2>&1 || { tail -5 gpurun_out/stab_feed.txt; exit 1; }
echo "== feed"; cat gpurun_out/stab_feed.txt | grep -v amdgpu.ids
NOFEED=1 timeout -k 10 300 python scripts/stability.py > gpurun_out/stab_nofeed.txt 2>&1 || { tail -5 gpurun_out/stab_nofeed.txt; exit 1; }
echo "== nofeed"; cat gpurun_out/stab_nofeed.txt | grep -v amdgpu.ids
timeout -k 10 60 rocm-smi --showclocks --showpower --showtemp 2>&1 | grep -iE "sclk|mclk|fclk|power|temp" | head -10 || true
