#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/gemm_tests.log 2>&1; rc=$?
tail -15 gpurun_out/gemm_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python scripts/tile_probe.py ${TILES:-0 6 7} > gpurun_out/tile_probe.txt 2>&1 || { tail gpurun_out/tile_probe.txt; exit 1; }
cat gpurun_out/tile_probe.txt
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2>/dev/null && cat gpurun_out/bench.json
