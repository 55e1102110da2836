# round 6: fp8 one-step update gate + long trajectories (bf16 convergence) at lr 0.002 / 0.005
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread tests/test_fp8_update_gate_gpu.py > gpurun_out/r6_fp8_gate.log 2>&1; rc=$?; echo gate rc $rc
case $rc in 0|1) ;; *) exit $rc;; esac
for lr in 0.002 0.005; do
  timeout -k 10 400 python -u scripts/fp8_trajectory.py --steps ${STEPS:-1000} --lr $lr --modes bf16,bf16alt,fp8dgw > gpurun_out/r6_fp8_traj_$lr.txt 2>&1 || { echo traj $lr failed; exit 1; }
  tail -4 gpurun_out/r6_fp8_traj_$lr.txt
done
