#!/bin/bash
# CaffeNet per-product census: tiles 10 / 20 (3-stage weight-gradient forms) x row table on / off
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gemm_gpu.py -m gpu -k "mc or wgrad or im2col or tile" > gpurun_out/t20_tests.log 2>&1 || { tail -30 gpurun_out/t20_tests.log; exit 3; }
tail -1 gpurun_out/t20_tests.log
for lg in 0 2; do
  SN_GEMM_LEGACY_ADDR=$lg timeout -k 10 400 python -u scripts/pk_probe.py --model caffenet --tiles 10,20 > gpurun_out/census_t20_l$lg.txt 2>&1 || { tail -20 gpurun_out/census_t20_l$lg.txt; exit 4; }
  grep -E "bwd|total" gpurun_out/census_t20_l$lg.txt | cut -c1-160
done
