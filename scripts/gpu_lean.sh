#!/bin/bash
# lean DMA-issue GEMM mainloop + 8-phase 256x256 tiles (40/41) + e4m3 direct conv: numerics, dense
# shapes, CaffeNet bench + GEMM census, VGG-16 b2048 fp8 (direct on / off) vs bf16 (gpurun)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_conv3x3_fp8_gpu.py tests/test_pool_lrn_gpu.py tests/test_kernels_gpu.py tests/test_gemm_gpu.py tests/test_gemm_fp8_mc_gpu.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/lean_tests.log 2>&1
rc=$?; tail -8 gpurun_out/lean_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/pk_probe.py --dense --tiles 0,6,11,13,16,40,41 > gpurun_out/lean_dense.txt 2>&1 || { tail -20 gpurun_out/lean_dense.txt; exit 4; }
cat gpurun_out/lean_dense.txt
timeout -k 10 300 python -u bench.py > gpurun_out/lean_bench.json 2> gpurun_out/lean_bench.err || { tail -20 gpurun_out/lean_bench.err; exit 5; }
cut -c1-200 gpurun_out/lean_bench.json
timeout -k 10 400 python -u scripts/pk_probe.py --model caffenet --tiles 40,41 > gpurun_out/lean_census.txt 2>&1 || { tail -20 gpurun_out/lean_census.txt; exit 3; }
tail -2 gpurun_out/lean_census.txt
: > gpurun_out/vgg_ab.jsonl
for mode in "--dtype fp8" "--dtype fp8 DIRECT0" "--dtype bf16"; do
  if [ "${mode#*DIRECT0}" != "$mode" ]; then env_d=0; args="--dtype fp8"; else env_d=1; args="$mode"; fi
  SN_CONV_DIRECT_FP8=$env_d timeout -k 10 300 python -u bench.py --model vgg16 --steps ${VGG_STEPS:-8} --warmup 3 $args >> gpurun_out/vgg_ab.jsonl 2>> gpurun_out/vgg_ab.err || { echo "vgg $mode failed"; tail -20 gpurun_out/vgg_ab.err; exit 4; }
  echo "$mode direct=$env_d"; tail -1 gpurun_out/vgg_ab.jsonl | cut -c1-160
done
