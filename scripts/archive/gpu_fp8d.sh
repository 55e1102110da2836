#!/bin/bash
# fidelity-setting sweep: chaos floor (bf16 vs bf16alt) vs fp8 at several learning rates, tiles pinned (gpurun)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
out=gpurun_out/fp8_lr.txt; : > $out
for lr in ${LRS:-0.001 0.002 0.005}; do
  echo "== lr $lr" >> $out
  SN_GEMM_AUTOTUNE=0 timeout -k 10 300 python -u scripts/fp8_trajectory.py --steps 200 --lr $lr --modes bf16,bf16alt,fp8dgw,fp8dg5w >> $out 2>&1 || exit 3
done
grep -E "^==|max \||first" $out
