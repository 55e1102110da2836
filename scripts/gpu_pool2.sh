#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "pool" --timeout 120 --timeout-method thread > gpurun_out/pool2_tests.log 2>&1 || { tail -30 gpurun_out/pool2_tests.log; exit 3; }
tail -2 gpurun_out/pool2_tests.log
timeout -k 10 180 python3 scripts/pool2_probe.py > gpurun_out/pool2_probe.txt 2>&1 || { cat gpurun_out/pool2_probe.txt; exit 4; }
grep -v amdgpu gpurun_out/pool2_probe.txt
: > gpurun_out/vgg_pool2.jsonl
for v in 1 0 1 0; do
  SN_POOL_K2S2=$v timeout -k 10 300 python -u bench.py --model vgg16 --steps 8 --warmup 3 --dtype fp8 >> gpurun_out/vgg_pool2.jsonl 2> gpurun_out/vgg_pool2.err || { tail -5 gpurun_out/vgg_pool2.err; exit 5; }
  echo "k2s2=$v $(tail -1 gpurun_out/vgg_pool2.jsonl | grep -o '"value": [0-9.]*')"
done
: > gpurun_out/gn_pool3.jsonl
for v in 1 0 1 0; do
  SN_POOL_K3S1=$v timeout -k 10 300 python -u bench.py --model googlenet >> gpurun_out/gn_pool3.jsonl 2> gpurun_out/gn_pool3.err || { tail -5 gpurun_out/gn_pool3.err; exit 6; }
  echo "k3s1=$v $(tail -1 gpurun_out/gn_pool3.jsonl | grep -o '"value": [0-9.]*')"
done
