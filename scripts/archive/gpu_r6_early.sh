# round 6: gemm_kernel A/B (numerics, conv probe, benches)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_gpu.py tests/test_bench_fidelity_gpu.py > gpurun_out/early_tests.log 2>&1 || { tail -30 gpurun_out/early_tests.log; exit 1; }
tail -2 gpurun_out/early_tests.log
timeout -k 10 300 python -u scripts/conv_probe.py --case cn_conv2g,cn_conv3,cn_conv5g,vgg_conv4_2 --tiles=-1,0,10,16 > gpurun_out/early_conv.txt 2>&1 || exit 1
grep -v amdgpu gpurun_out/early_conv.txt
: > gpurun_out/early_bench.jsonl
b() { timeout -k 10 300 python bench.py "$@" >> gpurun_out/early_bench.jsonl 2>> gpurun_out/early_bench.err || { echo "bench $* failed"; tail -5 gpurun_out/early_bench.err; exit 1; }; tail -1 gpurun_out/early_bench.jsonl | cut -c1-150; }
b && b && b --model googlenet && b --model vgg16 && b --model vgg16 --dtype fp8
