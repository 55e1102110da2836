#!/bin/bash
# fp8 GPU tests (incl. the fused-quantisation bitwise test), then VGG-16 b2048 fp8 with and
# without the fused side outputs, and bf16.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_gpu.py -k "fp8" \
  tests/test_net_gpu.py tests/test_layers_gpu.py tests/test_kernels_gpu.py -k "fp8 or pool" > gpurun_out/fp8_fused_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/fp8_fused_tests.log; exit 1; }
tail -3 gpurun_out/fp8_fused_tests.log

: > gpurun_out/fp8_fused_ab.jsonl
for spec in "--dtype fp8" "SN_FP8_FUSED_QUANT=0 --dtype fp8" "--dtype fp8" "SN_FP8_FUSED_QUANT=0 --dtype fp8"; do
  envs=""; args="$spec"
  if [[ "$spec" == SN_* ]]; then envs="${spec%% *}"; args="${spec#* }"; fi
  env $envs timeout -k 10 400 python bench.py --model vgg16 --steps 8 --warmup 3 $args >> gpurun_out/fp8_fused_ab.jsonl 2> gpurun_out/fp8_fused_ab.err || { echo "bench $spec failed"; tail -20 gpurun_out/fp8_fused_ab.err; exit 1; }
  tail -1 gpurun_out/fp8_fused_ab.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$spec', d['value'], d['ms_per_step'], 'fp8', d['config']['fp8_layers'], 'loss', d['config']['final_loss'], flush=True)"
done
