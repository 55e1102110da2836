#!/bin/bash
# cifar10_quick stability sweep: learning rate x split-K order of conv1's weight gradient x seed
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
: > gpurun_out/cifar_sweep.txt
for lr in 0.001 0.0005 0.00025; do
  for cfg in "" "cfg=32x201x102400:10:229" "cfg=32x201x102400:10:128" "cfg=32x201x102400:10:300"; do
    for seed in 5 7; do
      timeout -k 10 120 python -u scripts/dbg_thin.py graph only=NONE lr=$lr seed=$seed $cfg > gpurun_out/dbg_thin_run.log 2>&1 || { tail -20 gpurun_out/dbg_thin_run.log; exit 4; }
      grep -E "^graph" gpurun_out/dbg_thin_run.log | cut -c1-250 | tee -a gpurun_out/cifar_sweep.txt
    done
  done
done
