#!/bin/bash
# GoogLeNet conv2/3x3 as two 96-output direct launches: kernel tests, probe, GoogLeNet A/B, GoogLeNet net tests
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "conv" > gpurun_out/ba_tests.log 2>&1 || { tail -40 gpurun_out/ba_tests.log; exit 3; }
tail -1 gpurun_out/ba_tests.log
timeout -k 10 200 python -u scripts/direct96_probe.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_net_gpu.py -m gpu -k "googlenet or GoogLeNet" > gpurun_out/ba_net.log 2>&1 || { tail -40 gpurun_out/ba_net.log; exit 4; }
tail -1 gpurun_out/ba_net.log
: > gpurun_out/ba_ab.jsonl
for i in 1 2 3; do
  for v in 1 0; do
    SN_CONV_DIRECT96=$v timeout -k 10 300 python -u bench.py --model googlenet >> gpurun_out/ba_ab.jsonl 2> gpurun_out/ba_ab.err || { tail -20 gpurun_out/ba_ab.err; exit 5; }
    echo "googlenet direct96=$v: $(tail -1 gpurun_out/ba_ab.jsonl | grep -o '"value": [0-9.]*')"
  done
done
