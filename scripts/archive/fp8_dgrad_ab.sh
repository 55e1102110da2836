#!/bin/bash
# fp8 data-gradient GPU tests, then VGG-16 (default per-GPU batch 2048) bf16 vs fp8 forward
# vs fp8 forward + data gradients, interleaved on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_gpu.py -k "fp8" \
  tests/test_net_gpu.py::test_fp8_forward_training > gpurun_out/fp8_dgrad_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/fp8_dgrad_tests.log; exit 1; }
tail -3 gpurun_out/fp8_dgrad_tests.log
: > gpurun_out/fp8_dgrad_ab.jsonl
for spec in "--dtype fp8" "--dtype fp8 --no-fp8-dgrad" "--dtype bf16" ${EXTRA_SPECS}; do
  timeout -k 10 400 python bench.py --model vgg16 --steps ${STEPS:-8} --warmup 3 $spec >> gpurun_out/fp8_dgrad_ab.jsonl 2> gpurun_out/fp8_dgrad_ab.err || { echo "bench $spec failed"; tail -20 gpurun_out/fp8_dgrad_ab.err; exit 1; }
  tail -1 gpurun_out/fp8_dgrad_ab.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$spec', d['value'], d['ms_per_step'], 'fp8', d['config']['fp8_layers'], 'loss', d['config']['final_loss'], flush=True)"
done
