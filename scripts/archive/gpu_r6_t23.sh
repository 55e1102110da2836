# round 6: the 4-wave 256x256 tile (128x128 per wave): numerics, then dense / conv timing vs the other tiles and hipBLASLt
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -k "gemm256 and 23" > gpurun_out/t23_tests.log 2>&1 || { tail -30 gpurun_out/t23_tests.log; exit 1; }
tail -2 gpurun_out/t23_tests.log
timeout -k 10 400 python -u scripts/gemm_vs_blas.py > gpurun_out/t23_blas.txt 2>&1 || { tail -20 gpurun_out/t23_blas.txt; exit 1; }
grep -v amdgpu gpurun_out/t23_blas.txt
timeout -k 10 300 python -u scripts/conv_probe.py --case cn_conv2g,cn_conv3,vgg_conv3_2,vgg_conv4_2 --tiles=-1,0,11,13,23 > gpurun_out/t23_conv.txt 2>&1 || { tail -20 gpurun_out/t23_conv.txt; exit 1; }
grep -v amdgpu gpurun_out/t23_conv.txt
