#!/bin/bash
# in-launch split-K combine: its tests, the GEMM / layer / training suites with it on, and
# CaffeNet + GoogLeNet bench A/B (SN_GEMM_FIXUP 0 / 1)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_splitk_fixup_gpu.py -m gpu > gpurun_out/fix_tests.log 2>&1 || { tail -40 gpurun_out/fix_tests.log; exit 3; }
tail -1 gpurun_out/fix_tests.log
SN_GEMM_FIXUP=1 timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_gpu.py tests/test_layers_gpu.py tests/test_fused_splitk_gpu.py tests/test_net_gpu.py -m gpu > gpurun_out/fix_suite.log 2>&1 || { tail -40 gpurun_out/fix_suite.log; exit 4; }
tail -1 gpurun_out/fix_suite.log
: > gpurun_out/fix_ab.jsonl
for i in 1 2; do
  for fx in 0 1; do
    SN_GEMM_FIXUP=$fx timeout -k 10 300 python -u bench.py >> gpurun_out/fix_ab.jsonl 2> gpurun_out/fix_ab.err || { tail -20 gpurun_out/fix_ab.err; exit 5; }
    echo "caffenet fixup=$fx: $(tail -1 gpurun_out/fix_ab.jsonl | cut -c70-130)"
  done
done
for i in 1 2; do
  for fx in 0 1; do
    SN_GEMM_FIXUP=$fx timeout -k 10 300 python -u bench.py --model googlenet >> gpurun_out/fix_ab.jsonl 2> gpurun_out/fix_ab.err || { tail -20 gpurun_out/fix_ab.err; exit 5; }
    echo "googlenet fixup=$fx: $(tail -1 gpurun_out/fix_ab.jsonl | cut -c1-60)"
  done
done
