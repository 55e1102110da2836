#!/bin/bash
# Per-step GPU times of repeated driver-shaped CaffeNet benches (find what a slow run loses).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for r in ${REPS:-1 2 3 4 5 6 7 8}; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --step-times $ARGS 2> gpurun_out/st.err | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('run $r', d['value'], d['ms_per_step'], flush=True)" || exit 1
  grep "step ms" gpurun_out/st.err
done
