#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv3x3_fp8_gpu.py tests/test_kernels_gpu.py -q -x -k "conv3x3 or direct or packed" --timeout 120 --timeout-method thread > gpurun_out/dh_tests.log 2>&1 || { tail -30 gpurun_out/dh_tests.log; exit 3; }
tail -1 gpurun_out/dh_tests.log
timeout -k 10 200 python3 scripts/direct8_probe.py > gpurun_out/dh_probe.txt 2>&1 || { tail -5 gpurun_out/dh_probe.txt; exit 4; }
grep -v amdgpu gpurun_out/dh_probe.txt | tail -8
for dt in fp8 bf16 fp8 bf16; do
  timeout -k 10 300 python -u bench.py --model vgg16 --steps 8 --warmup 3 --dtype $dt 2>/dev/null | grep -o '"value": [0-9.]*' | sed "s/^/vgg $dt /"
done
