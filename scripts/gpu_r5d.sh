#!/bin/bash
# 32x32x16 MFMA twins + N-d conv: numerics, then CaffeNet per-product census (tuned vs 32x32 twins), dense A/B
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_conv_nd_gpu.py tests/test_pool_lrn_gpu.py -x -q -rf --timeout 120 --timeout-method thread -k "gemm256 or thin or tile64 or nd_layers or eligibility" > gpurun_out/mf32_tests.log 2>&1
rc=$?; tail -5 gpurun_out/mf32_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/pk_probe.py --model caffenet --tiles 23,24,25,26,27,28 > gpurun_out/mf32_census.txt 2>&1 || { tail -20 gpurun_out/mf32_census.txt; exit 3; }
grep -v amdgpu gpurun_out/mf32_census.txt
timeout -k 10 300 python -u scripts/pk_probe.py --dense --tiles 0,23,13,26,16,25,11,28 > gpurun_out/mf32_dense.txt 2>&1 || { tail -20 gpurun_out/mf32_dense.txt; exit 4; }
grep -v amdgpu gpurun_out/mf32_dense.txt
