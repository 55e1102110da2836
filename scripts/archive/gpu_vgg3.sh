#!/bin/bash
# VGG-16 b2048: fp8 (default: direct e4m3 conv1_2) and bf16 back-to-back, twice; fp8 / release / direct tests (gpurun)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
: > gpurun_out/vgg_ab3.jsonl
for dt in fp8 bf16 fp8 bf16; do
  timeout -k 10 300 python -u bench.py --model vgg16 --steps 8 --warmup 3 --dtype $dt >> gpurun_out/vgg_ab3.jsonl 2> gpurun_out/vgg_ab3.err || { echo "vgg $dt failed"; tail -5 gpurun_out/vgg_ab3.err; exit 4; }
  echo "$dt $(tail -1 gpurun_out/vgg_ab3.jsonl | cut -c1-140)"
done
timeout -k 10 600 python -u -m pytest tests/test_fp8_fidelity_gpu.py tests/test_conv3x3_fp8_gpu.py tests/test_net_gpu.py -q -rf -s --timeout 300 --timeout-method thread > gpurun_out/vgg3_tests.log 2>&1
rc=$?; grep -E "chaos floor|^bf16|^fp8|passed|failed" gpurun_out/vgg3_tests.log | tail -8; exit $rc
