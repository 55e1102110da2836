#!/bin/bash
# fp8 GPU tests, 200-step VGG-16 loss trajectories (bf16 / fp8 fwd / + e4m3 dgrad / + e5m2
# dgrad), then VGG-16 batch-2048 bench with e4m3 vs e5m2 data gradients.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_gpu.py -k "fp8" \
  tests/test_net_gpu.py::test_fp8_forward_training > gpurun_out/fp8_dgrad_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/fp8_dgrad_tests.log; exit 1; }
tail -3 gpurun_out/fp8_dgrad_tests.log
timeout -k 10 500 python -u scripts/fp8_trajectory.py > gpurun_out/fp8_trajectory.txt 2>gpurun_out/fp8_trajectory.err || { echo "trajectory failed"; tail -20 gpurun_out/fp8_trajectory.err; exit 1; }
cat gpurun_out/fp8_trajectory.txt
: > gpurun_out/fp8_dgrad_fmt.jsonl
for spec in "--dtype fp8 --fp8-dgrad-format e5m2" "--dtype fp8"; do
  timeout -k 10 400 python bench.py --model vgg16 --steps 8 --warmup 3 $spec >> gpurun_out/fp8_dgrad_fmt.jsonl 2> gpurun_out/fp8_dgrad_fmt.err || { echo "bench $spec failed"; tail -20 gpurun_out/fp8_dgrad_fmt.err; exit 1; }
  tail -1 gpurun_out/fp8_dgrad_fmt.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$spec', d['value'], d['ms_per_step'], 'fp8', d['config']['fp8_layers'], 'loss', d['config']['final_loss'], flush=True)"
done
