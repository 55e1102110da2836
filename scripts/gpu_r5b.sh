#!/bin/bash
# thin-tile root cause: repeat-launch stress of the suspect product, then summation-order / seed trajectories
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
: > gpurun_out/dbg_thin_b.log
for ts in "22 229" "10 178" "22 178" "10 229" "21 229"; do
  timeout -k 10 120 python -u scripts/dbg_thin_stress.py $ts 200 >> gpurun_out/dbg_thin_b.log 2>&1 || { tail -20 gpurun_out/dbg_thin_b.log; exit 3; }
done
grep -v amdgpu gpurun_out/dbg_thin_b.log | grep -v "^rep" | tail -12
for a in "only=NONE" "only=NONE seed=1" "only=NONE seed=2" "cfg=32x201x102400:10:229" "cfg=32x201x102400:22:178" "cfg=32x201x102400:0:229" "seed=1" "seed=2"; do
  timeout -k 10 120 python -u scripts/dbg_thin.py graph $a > gpurun_out/dbg_thin_run.log 2>&1 || { tail -20 gpurun_out/dbg_thin_run.log; exit 4; }
  grep -E "^graph|forced" gpurun_out/dbg_thin_run.log | cut -c1-250
done
