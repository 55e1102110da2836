#!/bin/bash
# pk GEMM tiles: numerics tests, then dense + CaffeNet A/B probes (gpurun).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_fp8_mc_gpu.py tests/test_gemm_pk_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/pk_tests.log 2>&1
rc=$?
tail -5 gpurun_out/pk_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc, stopping"; exit $rc; fi
timeout -k 10 400 python -u scripts/pk_probe.py --dense > gpurun_out/pk_dense.txt 2>&1 || { echo "dense probe failed"; tail -20 gpurun_out/pk_dense.txt; exit 3; }
cat gpurun_out/pk_dense.txt
timeout -k 10 400 python -u scripts/pk_probe.py --model ${MODEL:-caffenet} > gpurun_out/pk_model.txt 2>&1 || { echo "model probe failed"; tail -20 gpurun_out/pk_model.txt; exit 4; }
cat gpurun_out/pk_model.txt
