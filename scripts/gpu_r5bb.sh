#!/bin/bash
# packed <1, 64> direct conv for GoogLeNet conv2/3x3_reduce: tests, probe, GoogLeNet A/B
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "packed11 or direct96" > gpurun_out/bb_tests.log 2>&1 || { tail -40 gpurun_out/bb_tests.log; exit 3; }
tail -1 gpurun_out/bb_tests.log
timeout -k 10 200 python -u scripts/direct96_probe.py 2>&1 | grep -v amdgpu.ids
: > gpurun_out/bb_ab.jsonl
for i in 1 2 3; do
  for v in 1 0; do
    SN_CONV_PACKED11=$v timeout -k 10 300 python -u bench.py --model googlenet >> gpurun_out/bb_ab.jsonl 2> gpurun_out/bb_ab.err || { tail -20 gpurun_out/bb_ab.err; exit 5; }
    echo "googlenet packed11=$v: $(tail -1 gpurun_out/bb_ab.jsonl | grep -o '"value": [0-9.]*')"
  done
done
