#!/bin/bash
# MC im2col row table: GEMM / conv / layer GPU tests, CaffeNet + GoogLeNet bench A/B (row table
# vs per-instruction walk)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_gpu.py tests/test_gemm_pk_gpu.py tests/test_layers_gpu.py tests/test_kernels_gpu.py tests/test_fused_splitk_gpu.py -m gpu > gpurun_out/rt_tests.log 2>&1 || { tail -30 gpurun_out/rt_tests.log; exit 3; }
tail -2 gpurun_out/rt_tests.log
: > gpurun_out/rt_ab.jsonl
for i in 1 2; do
  for lg in 0 2; do
    SN_GEMM_LEGACY_ADDR=$lg timeout -k 10 300 python -u bench.py >> gpurun_out/rt_ab.jsonl 2> gpurun_out/rt_ab.err || { tail -20 gpurun_out/rt_ab.err; exit 5; }
    echo "caffenet legacy=$lg: $(tail -1 gpurun_out/rt_ab.jsonl | cut -c70-130)"
  done
done
for lg in 0 2; do
  SN_GEMM_LEGACY_ADDR=$lg timeout -k 10 300 python -u bench.py --model googlenet >> gpurun_out/rt_ab.jsonl 2> gpurun_out/rt_ab.err || { tail -20 gpurun_out/rt_ab.err; exit 5; }
  echo "googlenet legacy=$lg: $(tail -1 gpurun_out/rt_ab.jsonl | cut -c70-130)"
done

