#!/bin/bash
# fp8 round-4 checks (gpurun): MC fp8 numerics, trajectories (amax history), VGG-16 b2048 A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_fp8_mc_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/fp8_mc_tests.log 2>&1
rc=$?; tail -3 gpurun_out/fp8_mc_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u scripts/fp8_trajectory.py --steps 200 --modes ${TRAJ_MODES:-bf16,bf16alt,fp8dg,fp8dgw} > gpurun_out/fp8_traj.txt 2>&1 || { tail -20 gpurun_out/fp8_traj.txt; exit 3; }
cat gpurun_out/fp8_traj.txt
for mode in "--dtype fp8" "--dtype fp8 --no-fp8-wgrad" "--dtype bf16"; do
  timeout -k 10 300 python -u bench.py --model vgg16 --steps ${VGG_STEPS:-8} --warmup 3 $mode >> gpurun_out/vgg_ab.jsonl 2>> gpurun_out/vgg_ab.err || { echo "vgg $mode failed"; tail -20 gpurun_out/vgg_ab.err; exit 4; }
  tail -1 gpurun_out/vgg_ab.jsonl | cut -c1-300
done
