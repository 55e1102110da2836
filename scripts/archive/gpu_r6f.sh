# round 6: fp8 gates (one-step update, convergence) then the wgrad retune of the small models
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_fp8_update_gate_gpu.py tests/test_fp8_fidelity_gpu.py > gpurun_out/r6f_fp8.log 2>&1; rc=$?; echo "fp8 tests rc $rc"
grep -E "passed|failed|PASSED|FAILED|mean GPU|plateau left|last-100" gpurun_out/r6f_fp8.log | tail -12
case $rc in 0|1) ;; *) exit $rc;; esac
env STRIP=1 MODELS="caffenet|alexnet|cifar10_quick|cifar10_full" bash scripts/gpu_retune.sh
