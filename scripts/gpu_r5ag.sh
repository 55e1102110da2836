#!/bin/bash
# packed 4x4 direct conv (GoogLeNet conv1): kernel tests, then GoogLeNet bench A/B
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "packed" > gpurun_out/p44_tests.log 2>&1 || { tail -40 gpurun_out/p44_tests.log; exit 3; }
tail -1 gpurun_out/p44_tests.log
: > gpurun_out/p44_ab.jsonl
for i in 1 2 3; do
  for v in 1 0; do
    SN_CONV_PACKED44=$v timeout -k 10 300 python -u bench.py --model googlenet >> gpurun_out/p44_ab.jsonl 2> gpurun_out/p44_ab.err || { tail -20 gpurun_out/p44_ab.err; exit 5; }
    echo "googlenet packed44=$v: $(tail -1 gpurun_out/p44_ab.jsonl | cut -c45-75)"
  done
done
