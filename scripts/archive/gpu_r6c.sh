#!/bin/bash
# r6: lean MC im2col stager + pruned GEMM library + fp32 device mode — numerics, wgrad probe, bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_gemm_gpu.py tests/test_gemm_fp8_mc_gpu.py tests/test_conv_nd_gpu.py tests/test_kernels_gpu.py tests/test_layers_gpu.py tests/test_fused_splitk_gpu.py tests/test_bench_fidelity_gpu.py tests/test_fp32_device_gpu.py > gpurun_out/r6c_tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/r6c_tests.log; exit 1; }
tail -2 gpurun_out/r6c_tests.log
timeout -k 10 400 python -u scripts/wgrad_probe.py --case conv3,conv4,conv5,conv2 --tiles 0,10,13 --splits 4,6,8,12,16,24 --forms implicit > gpurun_out/r6c_wgrad.txt 2>&1 || exit 1
grep "BEST\|tuned" gpurun_out/r6c_wgrad.txt
for i in 1 2; do timeout -k 10 240 python bench.py > gpurun_out/r6c_bench$i.json 2>/dev/null || exit 1; cut -c1-150 gpurun_out/r6c_bench$i.json; done
timeout -k 10 300 python bench.py --dtype fp32 --steps 10 --warmup 2 > gpurun_out/r6c_bench_fp32.json 2> gpurun_out/r6c_bench_fp32.err || { tail -20 gpurun_out/r6c_bench_fp32.err; exit 1; }
cut -c1-200 gpurun_out/r6c_bench_fp32.json
