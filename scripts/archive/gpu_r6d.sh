# round 6: pool+LRN backward forms, fp8 one-step gate, long fp8 trajectories
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pool_lrn_gpu.py > gpurun_out/r6d_plrn_tests.log 2>&1 || { tail -30 gpurun_out/r6d_plrn_tests.log; exit 1; }
tail -2 gpurun_out/r6d_plrn_tests.log
timeout -k 10 200 python -u scripts/plrn_probe.py > gpurun_out/r6d_plrn_probe.txt 2>&1 || { cat gpurun_out/r6d_plrn_probe.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r6d_plrn_probe.txt
bash scripts/archive/gpu_r6_fp8.sh
