#!/bin/bash
# after the register-spill fix: GEMM / split-K / fixup tests, then CaffeNet, GoogLeNet and VGG-16 (bf16 + fp8) benches
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_gpu.py tests/test_splitk_fixup_gpu.py tests/test_fused_splitk_gpu.py tests/test_layers_gpu.py -m gpu > gpurun_out/spill_tests.log 2>&1 || { tail -30 gpurun_out/spill_tests.log; exit 3; }
tail -1 gpurun_out/spill_tests.log
: > gpurun_out/spill_bench.jsonl
for m in caffenet googlenet caffenet googlenet; do
  timeout -k 10 300 python -u bench.py --model $m >> gpurun_out/spill_bench.jsonl 2> gpurun_out/spill_bench.err || { tail -20 gpurun_out/spill_bench.err; exit 5; }
  echo "$m: $(tail -1 gpurun_out/spill_bench.jsonl | cut -c1-110)"
done
for dt in fp8 bf16; do
  timeout -k 10 500 python -u bench.py --model vgg16 --dtype $dt --steps 6 --warmup 3 >> gpurun_out/spill_bench.jsonl 2> gpurun_out/spill_bench.err || { tail -20 gpurun_out/spill_bench.err; exit 5; }
  echo "vgg16 $dt: $(tail -1 gpurun_out/spill_bench.jsonl | cut -c1-75)"
done
